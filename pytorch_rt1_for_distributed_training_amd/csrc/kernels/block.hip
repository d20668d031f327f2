// Per-frame reductions and the MBConv block tail, channels-last bf16.
//
//  frame_pool     : pool[n,c]  = sum_hw act(y*scale+shift) [* G]     (SE squeeze fwd, SE gate grad)
//  block_tail     : out = (bn3(y3) * keep[n] + skip) * film_mult[n,c] + film_add[n,c]
//                   (project BN, stochastic depth, residual and FiLM in ONE pass;
//                    FiLM follows every MBConv block)
//  tail_bwd_reduce: per (n,c): dmult = sum_hw dout*h, dadd = sum_hw dout   (FiLM grads)
//                   per-frame partial rows of sum dz3, sum dz3*xhat3 with
//                   dz3 = dout*film_mult*keep (project-BN backward)
//
// Work layouts: see FrameGeo (workgroup-per-frame for large maps, wave-per-frame for small ones).
#include <cstdlib>

#include "common.h"

using namespace rt1;

namespace {

constexpr int BLOCK = 256;

// Two work layouts for the per-(frame, channel) reductions:
//  block mode (large maps): one workgroup = frame n x <=8 channel vectors, 256 threads = (vector,
//    pixel lane), optional pixel splits (gridDim.z) as separate partial blocks, LDS reduction;
//  wave mode (HW <= WAVE_HW, C >= 64): one WAVE = frame n x 8 channel vectors, 8 pixel lanes, reduced
//    with 3 cross-lane shuffles -- no LDS, no barrier.  On 10x10 / 19x19 maps a workgroup-per-frame
//    layout spends most of its time in the LDS reduction of 32 pixel lanes for ~3-12 pixels each.
constexpr int WAVE_HW = 1500;

// channel vectors per workgroup in block mode: 8, or the whole row when 8 does not divide it (C = 144: 18 vectors as
// one group of 18 instead of 8 + 8 + 2, whose last workgroup idled 3/4 of its lanes on 128-B row pieces)
__host__ __device__ inline int frame_cv(int nv) { return (nv <= 8 || (nv % 8 != 0 && nv <= 32)) ? nv : 8; }

template <bool WAVE>
struct FrameGeo {
    int n, nv, cv, ncv, v0, lane_cv, pl, PL, p0, p1;
    bool valid;
    __device__ FrameGeo(int C, int HW, int N) {
        nv = C >> 3;
        if constexpr (WAVE) {
            const int chunks = (nv + 7) >> 3;
            const int item = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
            valid = item < N * chunks;
            n = valid ? item / chunks : 0;
            v0 = (item - n * chunks) * 8;
            cv = 8;
            ncv = valid ? min(8, nv - v0) : 0;
            lane_cv = threadIdx.x & 7;
            pl = (threadIdx.x & 63) >> 3;
            PL = 8;
            p0 = 0;
            p1 = HW;
        } else {
            n = blockIdx.x;
            cv = frame_cv(nv);
            v0 = blockIdx.y * cv;
            ncv = min(cv, nv - v0);
            lane_cv = threadIdx.x % cv;
            pl = threadIdx.x / cv;
            PL = BLOCK / cv;
            const int per = (HW + gridDim.z - 1) / gridDim.z;
            p0 = blockIdx.z * per;
            p1 = min(HW, p0 + per);
            valid = true;
        }
    }
    __device__ bool active() const { return valid && lane_cv < ncv && pl < PL; }
};

// Reduce NACC accumulators of 8 channels over the pixel lanes, then call put(k, c, value) once per
// (accumulator, channel) of the frame chunk (c = absolute channel).
template <bool WAVE, int NACC, typename Put>
__device__ void reduce_put(float (&a)[NACC][8], const FrameGeo<WAVE>& f, float* red, Put put) {
    if constexpr (WAVE) {
#pragma unroll
        for (int k = 0; k < NACC; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = a[k][j];
                v += __shfl_xor(v, 8, 64);
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
                a[k][j] = v;
            }
        if (f.valid && f.pl == 0 && f.lane_cv < f.ncv) {
#pragma unroll
            for (int k = 0; k < NACC; ++k)
#pragma unroll
                for (int j = 0; j < 8; ++j) put(k, (f.v0 + f.lane_cv) * 8 + j, a[k][j]);
        }
    } else {
        const int C8 = f.cv * 8;
        __syncthreads();
        if (f.pl < f.PL) {
#pragma unroll
            for (int k = 0; k < NACC; ++k)
#pragma unroll
                for (int j = 0; j < 8; ++j) red[(k * f.PL + f.pl) * C8 + f.lane_cv * 8 + j] = a[k][j];
        }
        __syncthreads();
        // all 256 threads share the (accumulator, channel) outputs; each sums PL partials
        for (int o = threadIdx.x; o < NACC * C8; o += BLOCK) {
            const int k = o / C8, cc = o - k * C8;
            if (cc >= f.ncv * 8) continue;
            float s = 0.f;
            for (int p = 0; p < f.PL; ++p) s += red[(k * f.PL + p) * C8 + cc];
            put(k, f.v0 * 8 + cc, s);
        }
    }
}

template <bool WAVE, int FP_U = 4>
__global__ __launch_bounds__(BLOCK) void frame_pool_kernel(const bf16_t* __restrict__ y, const bf16_t* __restrict__ G,
                                                           int N, int HW, int C, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int act,
                                                           float* __restrict__ pool) {
    __shared__ float red[WAVE ? 1 : BLOCK * 8];
    const FrameGeo<WAVE> f(C, HW, N);
    const int n = f.n;
    float a[1][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[0][j] = 0.f;
    if (f.active()) {
        const int c0 = (f.v0 + f.lane_cv) * 8;
        float sc[8], sh[8];
        if (scale) {
            load8f(scale + c0, sc);
            load8f(shift + c0, sh);
        }
        // FP_U pixels' loads issued before any of them is used; the per-lane sum order stays pixel order
        int p = f.p0 + f.pl;
        for (; p + (FP_U - 1) * f.PL < f.p1; p += FP_U * f.PL) {
            uint4 uy[FP_U], ug[FP_U];
#pragma unroll
            for (int u = 0; u < FP_U; ++u) {
                const int64_t off = ((int64_t)n * HW + p + u * f.PL) * C + c0;
                uy[u] = *reinterpret_cast<const uint4*>(y + off);
                if (G) ug[u] = *reinterpret_cast<const uint4*>(G + off);
            }
#pragma unroll
            for (int u = 0; u < FP_U; ++u) {
                float v[8];
                unpack8(uy[u], v);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = scale ? act_fwd(fmaf(v[j], sc[j], sh[j]), act) : v[j];
                if (G) {
                    float gv[8];
                    unpack8(ug[u], gv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] *= gv[j];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) a[0][j] += v[j];
            }
        }
        for (; p < f.p1; p += f.PL) {
            const int64_t off = ((int64_t)n * HW + p) * C + c0;
            float v[8];
            load8(y + off, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = scale ? act_fwd(fmaf(v[j], sc[j], sh[j]), act) : v[j];
            if (G) {
                float gv[8];
                load8(G + off, gv);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] *= gv[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) a[0][j] += v[j];
        }
    }
    // pixel split z writes its own [N, C] partial block (summed in a fixed order by the caller)
    const int64_t zoff = WAVE ? 0 : (int64_t)blockIdx.z * N * C;
    reduce_put<WAVE, 1>(a, f, red, [&](int, int c, float v) { pool[zoff + (int64_t)n * C + c] = v; });
}

template <int VPT>
__global__ __launch_bounds__(BLOCK) void block_tail_kernel(const bf16_t* __restrict__ y3, int64_t M, int HW, int C,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ keep,
                                                           const bf16_t* __restrict__ skip,
                                                           const float* __restrict__ fmul,
                                                           const float* __restrict__ fadd,
                                                           bf16_t* __restrict__ out) {
    const RowGeo g(C, BLOCK);
    if (!g.active) return;
    float sc[VPT][8], sh[VPT][8];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int v = min(g.vec0 + k * BLOCK, g.nv - 1);
        load8f(scale + v * 8, sc[k]);
        load8f(shift + v * 8, sh[k]);
    }
    for (int64_t r = (int64_t)blockIdx.x * g.slots + g.slot; r < M; r += (int64_t)gridDim.x * g.slots) {
        const int64_t n = (int64_t)((uint32_t)r / (uint32_t)HW);
        const float kp = keep ? keep[n] : 1.f;
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
            const int v = g.vec0 + k * BLOCK;
            if (v >= g.nv) continue;
            const int c0 = v * 8;
            float f[8];
            load8(y3 + r * C + c0, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], sc[k][j], sh[k][j]) * kp;
            if (skip) {
                float q[8];
                load8(skip + r * C + c0, q);
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] += q[j];
            }
            if (fmul) {
                float a[8], b[8];
                load8f(fmul + n * C + c0, a);
                load8f(fadd + n * C + c0, b);
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], a[j], b[j]);
            }
            store8(out + r * C + c0, f);
        }
    }
}

// Outputs per (n,c): dmul, dadd; per-frame partial rows pdz/pdzx [N, C].
// pixels' loads in flight per lane in the multi-block frame reductions below (one pixel at a time: 2.3-2.7 TB/s,
// profiles/r4_pmc_bytes.md).  The wave-per-frame variants keep one: their short-lived waves lost occupancy to the
// extra registers (frame_pool 8 vs 4 in flight and se_bn_bwd_reduce 4 vs 1 were 11-14 % slower, r4_frame_unroll_ab.md)
constexpr int RD_U = 4;

template <bool WAVE>
__global__ __launch_bounds__(BLOCK) void tail_bwd_reduce_kernel(const bf16_t* __restrict__ dout,
                                                                const bf16_t* __restrict__ y3, int N, int HW, int C,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ keep,
                                                                const bf16_t* __restrict__ skip,
                                                                const float* __restrict__ fmul,
                                                                float* __restrict__ dmul, float* __restrict__ dadd,
                                                                float* __restrict__ pdz, float* __restrict__ pdzx) {
    __shared__ float red[WAVE ? 1 : 4 * BLOCK * 8];
    const FrameGeo<WAVE> f(C, HW, N);
    const int n = f.n;
    float a[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[k][j] = 0.f;
    const float kp = keep ? keep[n] : 1.f;
    if (f.active()) {
        const int c0 = (f.v0 + f.lane_cv) * 8;
        float sc[8], sh[8], mu[8], rr[8], fm[8];
        load8f(scale + c0, sc);
        load8f(shift + c0, sh);
        load8f(mean + c0, mu);
        load8f(rstd + c0, rr);
        if (fmul) load8f(fmul + (int64_t)n * C + c0, fm);
        else {
#pragma unroll
            for (int j = 0; j < 8; ++j) fm[j] = 1.f;
        }
        auto step = [&](const uint4 ud, const uint4 uy, const uint4 us) {
            float d[8], yv[8], s[8];
            unpack8(ud, d);
            unpack8(uy, yv);
            unpack8(us, s);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float h = fmaf(yv[j], sc[j], sh[j]) * kp + (skip ? s[j] : 0.f);
                a[0][j] = fmaf(d[j], h, a[0][j]);
                a[1][j] += d[j];
                const float dz = d[j] * fm[j] * kp;
                a[2][j] += dz;
                a[3][j] = fmaf(dz, (yv[j] - mu[j]) * rr[j], a[3][j]);
            }
        };
        int p = f.p0 + f.pl;
        if constexpr (WAVE) {
            // the next pixel's loads are issued before the current one is consumed
            if (p < f.p1) {
                int64_t off = ((int64_t)n * HW + p) * C + c0;
                uint4 d0 = *reinterpret_cast<const uint4*>(dout + off), y0 = *reinterpret_cast<const uint4*>(y3 + off);
                uint4 s0 = skip ? *reinterpret_cast<const uint4*>(skip + off) : make_uint4(0, 0, 0, 0);
                for (p += f.PL; p < f.p1; p += f.PL) {
                    off = ((int64_t)n * HW + p) * C + c0;
                    const uint4 d1 = *reinterpret_cast<const uint4*>(dout + off);
                    const uint4 y1 = *reinterpret_cast<const uint4*>(y3 + off);
                    const uint4 s1 = skip ? *reinterpret_cast<const uint4*>(skip + off) : make_uint4(0, 0, 0, 0);
                    step(d0, y0, s0);
                    d0 = d1;
                    y0 = y1;
                    s0 = s1;
                }
                step(d0, y0, s0);
            }
        } else {
            // RD_U pixels' loads in flight per lane, consumed in pixel order (the per-lane sum order is unchanged)
            constexpr int U = RD_U;
            for (; p + (U - 1) * f.PL < f.p1; p += U * f.PL) {
                uint4 ud[U], uy[U], us[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t off = ((int64_t)n * HW + p + u * f.PL) * C + c0;
                    ud[u] = *reinterpret_cast<const uint4*>(dout + off);
                    uy[u] = *reinterpret_cast<const uint4*>(y3 + off);
                    us[u] = skip ? *reinterpret_cast<const uint4*>(skip + off) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) step(ud[u], uy[u], us[u]);
            }
            for (; p < f.p1; p += f.PL) {
                const int64_t off = ((int64_t)n * HW + p) * C + c0;
                step(*reinterpret_cast<const uint4*>(dout + off), *reinterpret_cast<const uint4*>(y3 + off),
                     skip ? *reinterpret_cast<const uint4*>(skip + off) : make_uint4(0, 0, 0, 0));
            }
        }
    }
    const int64_t zoff = WAVE ? 0 : (int64_t)blockIdx.z * 4 * N * C;   // split z: its own [4, N, C] block
    reduce_put<WAVE, 4>(a, f, red, [&](int k, int c, float v) {
        const int64_t o = (int64_t)n * C + c;
        float* dst = k == 0 ? dmul : k == 1 ? dadd : k == 2 ? pdz : pdzx;
        if (!dst) return;
        dst[zoff + o] = v;
    });
}

// SE-gate + BN backward statistics in ONE pass over (dA, y) per frame:
//   z = y*scale+shift, a = silu(z), sg = silu'(z), xh = (y-mean)*rstd
//   out[0] = sum_hw dA*a      (SE gate gradient)      out[1] = sum_hw dA*sg
//   out[2] = sum_hw sg        out[3] = sum_hw dA*sg*xh      out[4] = sum_hw sg*xh
// With the gate s[n,c] and the pool gradient rb[n,c] known afterwards, the BN
// backward sums are  sum dz = sum_n s*out1 + rb*out2,  sum dz*xh = sum_n s*out3 + rb*out4.
template <bool WAVE>
__global__ __launch_bounds__(BLOCK) void se_bn_bwd_reduce_kernel(const bf16_t* __restrict__ G,
                                                                 const bf16_t* __restrict__ y, int N, int HW, int C,
                                                                 const float* __restrict__ scale,
                                                                 const float* __restrict__ shift,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd,
                                                                 float* __restrict__ out) {
    __shared__ float red[WAVE ? 1 : 5 * BLOCK * 8];
    const FrameGeo<WAVE> f(C, HW, N);
    const int n = f.n;
    float a[5][8];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[k][j] = 0.f;
    if (f.active()) {
        const int c0 = (f.v0 + f.lane_cv) * 8;
        float sc[8], sh[8], mu[8], rr[8];
        load8f(scale + c0, sc);
        load8f(shift + c0, sh);
        load8f(mean + c0, mu);
        load8f(rstd + c0, rr);
        auto step = [&](const uint4 ug, const uint4 uy) {
            float gv[8], yv[8];
            unpack8(ug, gv);
            unpack8(uy, yv);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float z = fmaf(yv[j], sc[j], sh[j]);
                const float sgm = sigmoidf_(z);
                const float act = z * sgm;
                const float sg = sgm * (1.f + z * (1.f - sgm));
                const float xh = (yv[j] - mu[j]) * rr[j];
                a[0][j] = fmaf(gv[j], act, a[0][j]);
                const float gs = gv[j] * sg;
                a[1][j] += gs;
                a[2][j] += sg;
                a[3][j] = fmaf(gs, xh, a[3][j]);
                a[4][j] = fmaf(sg, xh, a[4][j]);
            }
        };
        if constexpr (WAVE) {
            // the next pixel's loads are issued before the current one is consumed
            int p = f.p0 + f.pl;
            if (p < f.p1) {
                int64_t off = ((int64_t)n * HW + p) * C + c0;
                uint4 g0 = *reinterpret_cast<const uint4*>(G + off), y0 = *reinterpret_cast<const uint4*>(y + off);
                for (p += f.PL; p < f.p1; p += f.PL) {
                    off = ((int64_t)n * HW + p) * C + c0;
                    const uint4 g1 = *reinterpret_cast<const uint4*>(G + off);
                    const uint4 y1 = *reinterpret_cast<const uint4*>(y + off);
                    step(g0, y0);
                    g0 = g1;
                    y0 = y1;
                }
                step(g0, y0);
            }
        } else {
            // RD_U pixels' loads in flight per lane, consumed in pixel order (the per-lane sum order is unchanged)
            int p = f.p0 + f.pl;
            for (; p + (RD_U - 1) * f.PL < f.p1; p += RD_U * f.PL) {
                uint4 ug[RD_U], uy[RD_U];
#pragma unroll
                for (int u = 0; u < RD_U; ++u) {
                    const int64_t off = ((int64_t)n * HW + p + u * f.PL) * C + c0;
                    ug[u] = *reinterpret_cast<const uint4*>(G + off);
                    uy[u] = *reinterpret_cast<const uint4*>(y + off);
                }
#pragma unroll
                for (int u = 0; u < RD_U; ++u) step(ug[u], uy[u]);
            }
            for (; p < f.p1; p += f.PL) {
                const int64_t off = ((int64_t)n * HW + p) * C + c0;
                step(*reinterpret_cast<const uint4*>(G + off), *reinterpret_cast<const uint4*>(y + off));
            }
        }
    }
    const int64_t NC = (int64_t)N * C;
    const int64_t zoff = WAVE ? 0 : (int64_t)blockIdx.z * 5 * NC;      // split z: its own [5, N, C] block
    reduce_put<WAVE, 5>(a, f, red, [&](int k, int c, float v) { out[zoff + k * NC + (int64_t)n * C + c] = v; });
}

// residual-branch gradient: x[m, c] += y[m, c] * s[m / HW, c]   (in place; skip grad through FiLM)
__global__ __launch_bounds__(BLOCK) void add_scaled_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                           const float* __restrict__ sc, int64_t M, int HW, int C) {
    const RowGeo g(C, BLOCK);
    if (!g.active) return;
    for (int64_t r = (int64_t)blockIdx.x * g.slots + g.slot; r < M; r += (int64_t)gridDim.x * g.slots) {
        const int64_t n = (int64_t)((uint32_t)r / (uint32_t)HW);
        for (int v = g.vec0; v < g.nv; v += BLOCK) {
            const int c0 = v * 8;
            float a[8], b[8], f[8];
            load8(x + r * C + c0, a);
            load8(y + r * C + c0, b);
            load8f(sc + n * C + c0, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = fmaf(b[j], f[j], a[j]);
            store8(x + r * C + c0, a);
        }
    }
}

// Flat-vector versions of the two elementwise passes (same layout as bn.hip's flat apply kernels): the
// [M, C] tensor is a run of M*C/8 16-byte vectors, lane i takes vectors base + u*BLOCK (all loads of a
// round issued first), per-channel BN constants staged once per workgroup in LDS.  Every lane is busy at
// every width (the row layout idles 6-10 % of them at C = 40/232/384) and FLAT_U vectors are in flight.
constexpr int FLAT_U = 4;

__global__ __launch_bounds__(BLOCK) void block_tail_flat_kernel(const bf16_t* __restrict__ y3, uint32_t total,
                                                                FastDiv by_nv, FastDiv by_hw, int C,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift,
                                                                const float* __restrict__ keep,
                                                                const bf16_t* __restrict__ skip,
                                                                const float* __restrict__ fmul,
                                                                const float* __restrict__ fadd,
                                                                bf16_t* __restrict__ out) {
    extern __shared__ float4 lds_raw[];
    float* L = reinterpret_cast<float*>(lds_raw);     // [2][C]: scale, shift
    for (int c = threadIdx.x; c < C; c += BLOCK) {
        L[c] = scale[c];
        L[C + c] = shift[c];
    }
    __syncthreads();
    const uint32_t nv = (uint32_t)(C >> 3);
    const uint32_t step = gridDim.x * BLOCK * FLAT_U;
    for (uint32_t base = blockIdx.x * BLOCK * FLAT_U + threadIdx.x; base < total; base += step) {
        // branch-free body (tail vectors clamped to the last one, only their stores masked), so the per-frame FiLM /
        // keep loads of all FLAT_U vectors can be issued together instead of one L2 round trip per vector
        uint4 ry[FLAT_U], rk[FLAT_U];
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t i = min(base + u * BLOCK, total - 1);
            ry[u] = *reinterpret_cast<const uint4*>(y3 + (size_t)i * 8);
            if (skip) rk[u] = *reinterpret_cast<const uint4*>(skip + (size_t)i * 8);
        }
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t iu = base + u * BLOCK, i = min(iu, total - 1);
            const uint32_t r = by_nv.div(i), c0 = (i - r * nv) * 8, n = by_hw.div(r);
            const float kp = keep ? keep[n] : 1.f;
            float f[8], sc[8], sh[8];
            unpack8(ry[u], f);
            load8f(L + c0, sc);
            load8f(L + C + c0, sh);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], sc[j], sh[j]) * kp;
            if (skip) {
                float q[8];
                unpack8(rk[u], q);
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] += q[j];
            }
            if (fmul) {
                float a[8], b[8];
                load8f(fmul + (size_t)n * C + c0, a);
                load8f(fadd + (size_t)n * C + c0, b);
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], a[j], b[j]);
            }
            if (iu < total) store8(out + (size_t)i * 8, f);
        }
    }
}

__global__ __launch_bounds__(BLOCK) void add_scaled_flat_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                                const float* __restrict__ sc, uint32_t total,
                                                                uint32_t HW, int C) {
    const uint32_t nv = (uint32_t)(C >> 3);
    const uint32_t step = gridDim.x * BLOCK * FLAT_U;
    for (uint32_t base = blockIdx.x * BLOCK * FLAT_U + threadIdx.x; base < total; base += step) {
        uint4 rx[FLAT_U], ry[FLAT_U];
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t i = base + u * BLOCK;
            if (i < total) {
                rx[u] = *reinterpret_cast<const uint4*>(x + (size_t)i * 8);
                ry[u] = *reinterpret_cast<const uint4*>(y + (size_t)i * 8);
            }
        }
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t i = base + u * BLOCK;
            if (i >= total) break;
            const uint32_t r = i / nv, c0 = (i - r * nv) * 8;
            float a[8], b[8], f[8];
            unpack8(rx[u], a);
            unpack8(ry[u], b);
            load8f(sc + (size_t)(r / HW) * C + c0, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = fmaf(b[j], f[j], a[j]);
            store8(x + (size_t)i * 8, a);
        }
    }
}

inline bool flat_ok(int64_t M, int C) { return M * (int64_t)(C >> 3) < (int64_t)0xF0000000LL && C <= 8192; }

inline unsigned flat_grid(int64_t total) {
    int64_t b = (total + BLOCK * FLAT_U - 1) / (BLOCK * FLAT_U);
    if (b > 4096) b = 4096;
    return (unsigned)(b < 1 ? 1 : b);
}

bool use_wave(int HW, int C) { return HW <= WAVE_HW && C >= 64; }
unsigned wave_grid(int N, int C) { return (unsigned)(((int64_t)N * ((C / 8 + 7) / 8) + 3) / 4); }

}  // namespace

extern "C" {

// pixel splits: enough workgroups to fill the chip (>= 8 per CU) while every
// workgroup still streams >= 128 pixels; each split writes its own partial block (deterministic sums)
int rt1_frame_splits(int N, int HW, int C) {
    if (use_wave(HW, C)) return 1;
    const int nv = C / 8, cv = frame_cv(nv);
    const int64_t base = (int64_t)N * ((nv + cv - 1) / cv);
    int64_t z = (2048 + base - 1) / base;
    const int64_t zmax = HW / 128 > 1 ? HW / 128 : 1;
    if (z > zmax) z = zmax;
    return (int)(z < 1 ? 1 : z);
}

int rt1_frame_pool(const bf16_t* y, const bf16_t* G, int N, int HW, int C, const float* scale, const float* shift,
                   int act, int splits, float* pool, hipStream_t st) {
    const int nv = C / 8, cv = frame_cv(nv);
    if (use_wave(HW, C))
        hipLaunchKernelGGL(frame_pool_kernel<true>, dim3(wave_grid(N, C)), dim3(BLOCK), 0, st, y, G, N, HW, C, scale,
                           shift, act, pool);
    else   // 8 pixels' loads in flight per lane (4: -0.2 % step, profiles/r3_frame_pool_u8_ab.log)
        hipLaunchKernelGGL((frame_pool_kernel<false, 8>), dim3(N, (nv + cv - 1) / cv, splits), dim3(BLOCK), 0, st, y, G,
                           N, HW, C, scale, shift, act, pool);
    return (int)hipGetLastError();
}

int rt1_se_bn_bwd_reduce(const bf16_t* G, const bf16_t* y, int N, int HW, int C, const float* scale,
                         const float* shift, const float* mean, const float* rstd, int splits, float* out,
                         hipStream_t st) {
    const int nv = C / 8, cv = frame_cv(nv);
    if (use_wave(HW, C))
        hipLaunchKernelGGL(se_bn_bwd_reduce_kernel<true>, dim3(wave_grid(N, C)), dim3(BLOCK), 0, st, G, y, N, HW, C,
                           scale, shift, mean, rstd, out);
    else
        hipLaunchKernelGGL(se_bn_bwd_reduce_kernel<false>, dim3(N, (nv + cv - 1) / cv, splits), dim3(BLOCK), 0, st, G,
                           y, N, HW, C, scale, shift, mean, rstd, out);
    return (int)hipGetLastError();
}

int rt1_block_tail(const bf16_t* y3, int64_t M, int HW, int C, const float* scale, const float* shift,
                   const float* keep, const bf16_t* skip, const float* fmul, const float* fadd, bf16_t* out,
                   hipStream_t st) {
    if (M <= 0 || C <= 0) return 0;   // empty tensor: nothing to launch
    if (flat_ok(M, C)) {
        const int64_t total = M * (C >> 3);
        hipLaunchKernelGGL(block_tail_flat_kernel, dim3(flat_grid(total)), dim3(BLOCK), 2 * C * sizeof(float), st, y3,
                           (uint32_t)total, FastDiv((uint32_t)(C >> 3)), FastDiv((uint32_t)HW), C, scale, shift, keep,
                           skip, fmul, fadd, out);
        return (int)hipGetLastError();
    }
    const int nv = C >> 3;
    const int slots = nv <= BLOCK ? BLOCK / nv : 1;
    int64_t blocks = (M + slots - 1) / slots;
    if (blocks > 8192) blocks = 8192;
    if (nv > BLOCK)
        hipLaunchKernelGGL(block_tail_kernel<2>, dim3((unsigned)blocks), dim3(BLOCK), 0, st, y3, M, HW, C, scale, shift,
                           keep, skip, fmul, fadd, out);
    else
        hipLaunchKernelGGL(block_tail_kernel<1>, dim3((unsigned)blocks), dim3(BLOCK), 0, st, y3, M, HW, C, scale, shift,
                           keep, skip, fmul, fadd, out);
    return (int)hipGetLastError();
}

int rt1_add_scaled(bf16_t* x, const bf16_t* y, const float* sc, int64_t M, int HW, int C, hipStream_t st) {
    if (flat_ok(M, C)) {
        const int64_t total = M * (C >> 3);
        hipLaunchKernelGGL(add_scaled_flat_kernel, dim3(flat_grid(total)), dim3(BLOCK), 0, st, x, y, sc,
                           (uint32_t)total, (uint32_t)HW, C);
        return (int)hipGetLastError();
    }
    const int nv = C >> 3;
    const int slots = nv <= BLOCK ? BLOCK / nv : 1;
    int64_t blocks = (M + slots - 1) / slots;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(add_scaled_kernel, dim3((unsigned)blocks), dim3(BLOCK), 0, st, x, y, sc, M, HW, C);
    return (int)hipGetLastError();
}

int rt1_tail_bwd_reduce(const bf16_t* dout, const bf16_t* y3, int N, int HW, int C, const float* scale,
                        const float* shift, const float* mean, const float* rstd, const float* keep,
                        const bf16_t* skip, const float* fmul, int splits, float* dmul, float* dadd, float* pdz,
                        float* pdzx, hipStream_t st) {
    const int nv = C / 8, cv = frame_cv(nv);
    if (use_wave(HW, C))
        hipLaunchKernelGGL(tail_bwd_reduce_kernel<true>, dim3(wave_grid(N, C)), dim3(BLOCK), 0, st, dout, y3, N, HW, C,
                           scale, shift, mean, rstd, keep, skip, fmul, dmul, dadd, pdz, pdzx);
    else
        hipLaunchKernelGGL(tail_bwd_reduce_kernel<false>, dim3(N, (nv + cv - 1) / cv, splits), dim3(BLOCK), 0, st, dout,
                           y3, N, HW, C, scale, shift, mean, rstd, keep, skip, fmul, dmul, dadd, pdz, pdzx);
    return (int)hipGetLastError();
}

}  // extern "C"
