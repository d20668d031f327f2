// Train-mode BatchNorm building blocks on channels-last bf16 activations.
//
// RT-1's image tokenizer has 78 BatchNorm2d layers.  In train
// mode each needs a global per-channel reduction between its producer and its
// consumer, so BN is split into:
//   * a statistics pass that writes one partial row (sum, sum of squares) per
//     workgroup — never a global atomic, so thousands of workgroups do not
//     contend on C addresses (MI355X_MICROARCH 'Global float atomics':
//     same-row contention is ~14x slower);
//   * bn_finalize: fp64 reduction of the partial rows -> per-channel
//     scale/shift, saved mean/rstd, running-stat update (momentum 0.1,
//     unbiased running var, as torch);
//   * the normalise+activation is applied in the CONSUMER's prologue (dwconv,
//     SE pool, project-operand build) or by bn_apply when a materialised
//     tensor is needed.
// Backward mirrors it: bn_bwd_reduce (partials of sum dz and sum dz*xhat) ->
// bn_bwd_finalize (dgamma, dbeta, the two means) -> bn_bwd_apply.  The upstream
// gradient may be given as  g = G[m,c] * rs[n,c] + rb[n,c]  (n = m / HW) so the
// squeeze-excitation gate and pool gradients never need their own pass.
//
// Layout: x is [M, C] row-major (M = N*H*W), C % 8 == 0; every lane moves 8
// channels (16 B).  A workgroup of 256 threads covers `slots` rows at once
// (slots = 256 / (C/8)); C/8 > 256 uses VPT=2 vectors per thread.
#include <cstdlib>

#include "common.h"

using namespace rt1;

namespace {

constexpr int BLOCK = 256;
constexpr int BN_STATS_RU = 4;   // rows per load round in bn_stats (A/B: 1 = one load in flight per lane)

struct Geo {
    int nv, vpt, slots;
    __device__ Geo(int C) {
        nv = C >> 3;
        vpt = (nv + BLOCK - 1) / BLOCK;
        slots = vpt == 1 ? BLOCK / nv : 1;
    }
};

// reduce (s, q)[vpt][8] over the block's row slots and write one partial row
template <int VPT>
__device__ void reduce_write(float (&s)[VPT][8], float (&q)[VPT][8], const Geo& g, int slot, int vec0, bool active,
                             float* lds, float* __restrict__ prow_s, float* __restrict__ prow_q) {
    if (g.slots == 1) {
        if (active) {
#pragma unroll
            for (int k = 0; k < VPT; ++k) {
                const int v = vec0 + k * BLOCK;
                if (v < g.nv) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        prow_s[v * 8 + j] = s[k][j];
                        prow_q[v * 8 + j] = q[k][j];
                    }
                }
            }
        }
        return;
    }
    // VPT == 1 here
    const int C = g.nv * 8;
    if (active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            lds[slot * C + vec0 * 8 + j] = s[0][j];
            lds[g.slots * C + slot * C + vec0 * 8 + j] = q[0][j];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += BLOCK) {
        float a = 0.f, b = 0.f;
        for (int sl = 0; sl < g.slots; ++sl) {
            a += lds[sl * C + c];
            b += lds[g.slots * C + sl * C + c];
        }
        prow_s[c] = a;
        prow_q[c] = b;
    }
}

template <int VPT>
__global__ __launch_bounds__(BLOCK) void bn_stats_kernel(const bf16_t* __restrict__ x, int64_t M, int C,
                                                         int64_t rows_per_block, float* __restrict__ psum,
                                                         float* __restrict__ psq) {
    __shared__ float lds[2 * BLOCK * 8];
    const Geo g(C);
    const int t = threadIdx.x;
    const int slot = g.slots == 1 ? 0 : t / g.nv;
    const int vec0 = g.slots == 1 ? t : t % g.nv;
    const bool active = slot < g.slots;
    float s[VPT][8], q[VPT][8];
#pragma unroll
    for (int k = 0; k < VPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[k][j] = q[k][j] = 0.f;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(M, r0 + rows_per_block);
    if (active) {
        // RU rows per round with every load issued before the first add: one 16-B load in flight per lane
        // left the reduction at ~3.5 TB/s on the wide low-resolution layers
        constexpr int RU = BN_STATS_RU;
        int64_t r = r0 + slot;
        for (; r + (RU - 1) * g.slots < r1; r += RU * g.slots) {
            uint4 raw[RU][VPT];
#pragma unroll
            for (int u = 0; u < RU; ++u)
#pragma unroll
                for (int k = 0; k < VPT; ++k) {
                    const int v = min(vec0 + k * BLOCK, g.nv - 1);
                    raw[u][k] = *reinterpret_cast<const uint4*>(x + (r + u * g.slots) * C + v * 8);
                }
#pragma unroll
            for (int u = 0; u < RU; ++u)
#pragma unroll
                for (int k = 0; k < VPT; ++k) {
                    if (vec0 + k * BLOCK >= g.nv) continue;
                    float f[8];
                    unpack8(raw[u][k], f);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        s[k][j] += f[j];
                        q[k][j] = fmaf(f[j], f[j], q[k][j]);
                    }
                }
        }
        for (; r < r1; r += g.slots) {
            const bf16_t* row = x + r * C;
#pragma unroll
            for (int k = 0; k < VPT; ++k) {
                const int v = vec0 + k * BLOCK;
                if (v < g.nv) {
                    float f[8];
                    load8(row + v * 8, f);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        s[k][j] += f[j];
                        q[k][j] = fmaf(f[j], f[j], q[k][j]);
                    }
                }
            }
        }
    }
    reduce_write<VPT>(s, q, g, slot, vec0, active, lds, psum + (int64_t)blockIdx.x * C, psq + (int64_t)blockIdx.x * C);
}

// Finalize reductions over the P partial rows of the producing kernels (P = their grid: up to 2048-4096 rows).
// A workgroup owns 16 channels x 16 row groups, so every load instruction reads 64-B runs
// of 16 channels from 4 rows (the one-wave-per-channel layout touched 64 rows, 4 B each, per instruction), 4 rows
// in flight per lane; the 16 row-group partials combine in LDS in a fixed order (deterministic).
constexpr int FIN_CH = 16, FIN_RG = 16;
// CH channels x (256 / CH) row groups per workgroup.  CH = 16 reads 64-B runs; with many partial rows and few
// channels (P ~ 2048 rows, C <= 1024: a few workgroups that each walk 128 rows per thread, ~11 us, latency-bound)
// CH = 4 gives 4x the workgroups and a quarter of the dependent row walk per thread.
template <int CH>
__device__ __forceinline__ bool fin_colsum_t(const float* __restrict__ pa, const float* __restrict__ pb, int P, int C,
                                             double& a, double& b) {
    constexpr int RG = 256 / CH;
    __shared__ double red[2][RG][CH];
    const int cl = threadIdx.x % CH, rg = threadIdx.x / CH;
    const int c = blockIdx.x * CH + cl;
    double x = 0.0, y = 0.0;
    if (c < C) {
        int p = rg;
        for (; p + 3 * RG < P; p += 4 * RG) {
            float u[4], v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u[k] = pa[(int64_t)(p + k * RG) * C + c];
                v[k] = pb[(int64_t)(p + k * RG) * C + c];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x += (double)u[k];
                y += (double)v[k];
            }
        }
        for (; p < P; p += RG) {
            x += (double)pa[(int64_t)p * C + c];
            y += (double)pb[(int64_t)p * C + c];
        }
    }
    red[0][rg][cl] = x;
    red[1][rg][cl] = y;
    __syncthreads();
    if (rg != 0 || c >= C) return false;
    a = 0.0;
    b = 0.0;
    for (int r = 0; r < RG; ++r) {
        a += red[0][r][cl];
        b += red[1][r][cl];
    }
    return true;
}
__device__ __forceinline__ bool fin_colsum(const float* __restrict__ pa, const float* __restrict__ pb, int P, int C,
                                           double& a, double& b) {
    return fin_colsum_t<FIN_CH>(pa, pb, P, C, a, b);
}
int fin_ch(int P, int C) { return (P >= 128 && C <= 1024) ? 4 : FIN_CH; }
int fin_grid(int C, int ch = FIN_CH) { return (C + ch - 1) / ch; }

// fp64 sums over P partial rows (fin_colsum_t)
template <int CH>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ psum, const float* __restrict__ psq,
                                                          int P, int C, double count, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, float momentum,
                                                          float* __restrict__ running_mean,
                                                          float* __restrict__ running_var, float* __restrict__ scale,
                                                          float* __restrict__ shift, float* __restrict__ save_mean,
                                                          float* __restrict__ save_rstd) {
    double a = 0.0, b = 0.0;
    const int c = blockIdx.x * CH + (int)(threadIdx.x % CH);
    const bool lead = fin_colsum_t<CH>(psum, psq, P, C, a, b);
    if (lead) {
        const double mean = a / count;
        double var = b / count - mean * mean;
        var = var < 0.0 ? 0.0 : var;
        const float rstd = (float)(1.0 / sqrt(var + (double)eps));
        const float gm = gamma ? gamma[c] : 1.f;
        const float bt = beta ? beta[c] : 0.f;
        scale[c] = gm * rstd;
        shift[c] = bt - (float)mean * gm * rstd;
        save_mean[c] = (float)mean;
        save_rstd[c] = rstd;
        if (running_mean) {
            const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
            running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
            running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
        }
    }
}

// out = act(y*scale + shift) [* rs[n, c]]   (bf16 -> bf16)
template <int VPT>
__global__ __launch_bounds__(BLOCK) void bn_apply_kernel(const bf16_t* __restrict__ y, int64_t M, int C,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int act,
                                                         const float* __restrict__ rs, int64_t HW,
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
    const uint32_t hw = (uint32_t)(HW > 0 ? HW : 1);
    for (int64_t r = (int64_t)blockIdx.x * g.slots + g.slot; r < M; r += (int64_t)gridDim.x * g.slots) {
        const int64_t n = rs ? (int64_t)((uint32_t)r / hw) : 0;
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
            const int v = g.vec0 + k * BLOCK;
            if (v >= g.nv) continue;
            const int c0 = v * 8;
            float f[8];
            load8(y + r * C + c0, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = act_fwd(fmaf(f[j], sc[k][j], sh[k][j]), act);
            if (rs) {
                float q[8];
                load8f(rs + n * C + c0, q);
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] *= q[j];
            }
            store8(out + r * C + c0, f);
        }
    }
}

template <int VPT>
__global__ __launch_bounds__(BLOCK) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ G,
                                                              const float* __restrict__ rs,
                                                              const float* __restrict__ rb, int64_t HW,
                                                              const bf16_t* __restrict__ y, int64_t M, int C,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd, int act,
                                                              int64_t rows_per_block, float* __restrict__ pdz,
                                                              float* __restrict__ pdzx) {
    __shared__ float lds[2 * BLOCK * 8];
    const Geo g(C);
    const int t = threadIdx.x;
    const int slot = g.slots == 1 ? 0 : t / g.nv;
    const int vec0 = g.slots == 1 ? t : t % g.nv;
    const bool active = slot < g.slots;
    float s[VPT][8], q[VPT][8], sc[VPT][8], sh[VPT][8], mu[VPT][8], rr[VPT][8];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int v = min(vec0 + k * BLOCK, g.nv - 1);
        load8f(scale + v * 8, sc[k]);
        load8f(shift + v * 8, sh[k]);
        load8f(mean + v * 8, mu[k]);
        load8f(rstd + v * 8, rr[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[k][j] = q[k][j] = 0.f;
    }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(M, r0 + rows_per_block);
    const uint32_t hw = (uint32_t)(HW > 0 ? HW : 1);
    if (active && !rs && !rb) {
        // plain gradient (the top conv's BN): RU rows per round with all 2 x RU loads issued before the math.  One row
        // at a time per lane kept a single load pair in flight and ran the [76800, 1536] top at 1.4 TB/s (337 us)
        constexpr int RU = BN_STATS_RU;
        int64_t r = r0 + slot;
        for (; r + (RU - 1) * g.slots < r1; r += RU * g.slots) {
            uint4 rg[RU][VPT], ry[RU][VPT];
#pragma unroll
            for (int u = 0; u < RU; ++u)
#pragma unroll
                for (int k = 0; k < VPT; ++k) {
                    const int v = min(vec0 + k * BLOCK, g.nv - 1);
                    rg[u][k] = *reinterpret_cast<const uint4*>(G + (r + u * g.slots) * C + v * 8);
                    ry[u][k] = *reinterpret_cast<const uint4*>(y + (r + u * g.slots) * C + v * 8);
                }
#pragma unroll
            for (int u = 0; u < RU; ++u)
#pragma unroll
                for (int k = 0; k < VPT; ++k) {
                    if (vec0 + k * BLOCK >= g.nv) continue;
                    float gv[8], yv[8];
                    unpack8(rg[u][k], gv);
                    unpack8(ry[u][k], yv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float dz = gv[j];
                        if (act == ACT_SILU) dz *= silu_grad(fmaf(yv[j], sc[k][j], sh[k][j]));
                        const float xh = (yv[j] - mu[k][j]) * rr[k][j];
                        s[k][j] += dz;
                        q[k][j] = fmaf(dz, xh, q[k][j]);
                    }
                }
        }
        for (; r < r1; r += g.slots) {
#pragma unroll
            for (int k = 0; k < VPT; ++k) {
                const int v = vec0 + k * BLOCK;
                if (v < g.nv) {
                    float gv[8], yv[8];
                    load8(G + r * C + v * 8, gv);
                    load8(y + r * C + v * 8, yv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float dz = gv[j];
                        if (act == ACT_SILU) dz *= silu_grad(fmaf(yv[j], sc[k][j], sh[k][j]));
                        const float xh = (yv[j] - mu[k][j]) * rr[k][j];
                        s[k][j] += dz;
                        q[k][j] = fmaf(dz, xh, q[k][j]);
                    }
                }
            }
        }
    } else if (active) {
        for (int64_t r = r0 + slot; r < r1; r += g.slots) {
            const int64_t n = (rs || rb) ? (int64_t)((uint32_t)r / hw) : 0;
#pragma unroll
            for (int k = 0; k < VPT; ++k) {
                const int v = vec0 + k * BLOCK;
                if (v < g.nv) {
                    const int c0 = v * 8;
                    float gv[8], yv[8];
                    load8(G + r * C + c0, gv);
                    if (rs) {
                        float w[8];
                        load8f(rs + n * C + c0, w);
#pragma unroll
                        for (int j = 0; j < 8; ++j) gv[j] *= w[j];
                    }
                    if (rb) {
                        float w[8];
                        load8f(rb + n * C + c0, w);
#pragma unroll
                        for (int j = 0; j < 8; ++j) gv[j] += w[j];
                    }
                    load8(y + r * C + c0, yv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float dz = gv[j];
                        if (act == ACT_SILU) dz *= silu_grad(fmaf(yv[j], sc[k][j], sh[k][j]));
                        const float xh = (yv[j] - mu[k][j]) * rr[k][j];
                        s[k][j] += dz;
                        q[k][j] = fmaf(dz, xh, q[k][j]);
                    }
                }
            }
        }
    }
    reduce_write<VPT>(s, q, g, slot, vec0, active, lds, pdz + (int64_t)blockIdx.x * C, pdzx + (int64_t)blockIdx.x * C);
}

// sums -> dbeta (+=), dgamma (+=), and the two per-channel coefficients of the apply pass
struct PwBwdConsts {   // optional [5, C] output of bn_bwd_finalize for the fused expand backward
    const float *scale, *shift, *gamma, *mean, *rstd;
    float* out;
};

template <int CH>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ pdz,
                                                              const float* __restrict__ pdzx, int P, int C,
                                                              double count, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, float* __restrict__ mdz,
                                                              float* __restrict__ mdzx, int accumulate,
                                                              PwBwdConsts k) {
    double a = 0.0, b = 0.0;
    const int c = blockIdx.x * CH + (int)(threadIdx.x % CH);
    const bool lead = fin_colsum_t<CH>(pdz, pdzx, P, C, a, b);
    if (lead) {
        if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)a : (float)a;
        if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)b : (float)b;
        const float mz = (float)(a / count), mx = (float)(b / count);
        mdz[c] = mz;
        mdzx[c] = mx;
        if (k.out) {
            // the expand-backward kernel's constants (pwbwd.hip): [scale, shift, k1, -k1 rstd mdzx, -k1 (mdz - mean rstd mdzx)]
            const float rr = k.rstd[c], k1 = k.gamma[c] * rr;
            k.out[c] = k.scale[c];
            k.out[C + c] = k.shift[c];
            k.out[2 * C + c] = k1;
            k.out[3 * C + c] = -k1 * rr * mx;
            k.out[4 * C + c] = -k1 * (mz - k.mean[c] * rr * mx);
        }
    }
}

// dy = gamma*rstd * (dz - mean(dz) - xhat * mean(dz*xhat))   -> bf16
template <int VPT>
__global__ __launch_bounds__(BLOCK) void bn_bwd_apply_kernel(const bf16_t* __restrict__ G,
                                                             const float* __restrict__ rs,
                                                             const float* __restrict__ rb, int64_t HW,
                                                             const bf16_t* __restrict__ y, int64_t M, int C,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma, int act,
                                                             const float* __restrict__ mdz,
                                                             const float* __restrict__ mdzx,
                                                             bf16_t* __restrict__ dy,
                                                             const float* __restrict__ keep) {
    const RowGeo g(C, BLOCK);
    if (!g.active) return;
    // per-channel: dy = k1*dz + k0 + k2*y   with  k1 = gamma*rstd, k2 = -k1*rstd*mdzx, k0 = -k1*(mdz - mu*rstd*mdzx)
    float k0[VPT][8], k1[VPT][8], k2[VPT][8], sc[VPT][8], sh[VPT][8];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int v = min(g.vec0 + k * BLOCK, g.nv - 1);
        float mu[8], rr[8], a[8], b[8];
        load8f(mean + v * 8, mu);
        load8f(rstd + v * 8, rr);
        load8f(mdz + v * 8, a);
        load8f(mdzx + v * 8, b);
        load8f(scale + v * 8, sc[k]);
        load8f(shift + v * 8, sh[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float gm = gamma ? gamma[v * 8 + j] : 1.f;
            k1[k][j] = gm * rr[j];
            k2[k][j] = -k1[k][j] * rr[j] * b[j];
            k0[k][j] = -k1[k][j] * (a[j] - mu[j] * rr[j] * b[j]);
        }
    }
    const uint32_t hw = (uint32_t)(HW > 0 ? HW : 1);
    for (int64_t r = (int64_t)blockIdx.x * g.slots + g.slot; r < M; r += (int64_t)gridDim.x * g.slots) {
        const int64_t n = (rs || rb) ? (int64_t)((uint32_t)r / hw) : 0;
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
            const int v = g.vec0 + k * BLOCK;
            if (v >= g.nv) continue;
            const int c0 = v * 8;
            float gv[8], yv[8];
            load8(G + r * C + c0, gv);
            if (rs) {
                float q[8];
                load8f(rs + n * C + c0, q);
                const float kp = keep ? keep[n] : 1.f;     // rs * keep[frame] rounded first, as (fmul * keep) was
#pragma unroll
                for (int j = 0; j < 8; ++j) gv[j] *= keep ? q[j] * kp : q[j];
            }
            if (rb) {
                float q[8];
                load8f(rb + n * C + c0, q);
#pragma unroll
                for (int j = 0; j < 8; ++j) gv[j] += q[j];
            }
            load8(y + r * C + c0, yv);
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float dz = gv[j];
                if (act == ACT_SILU) dz *= silu_grad(fmaf(yv[j], sc[k][j], sh[k][j]));
                o[j] = fmaf(k1[k][j], dz, fmaf(k2[k][j], yv[j], k0[k][j]));
            }
            store8(dy + r * C + c0, o);
        }
    }
}

// ---- flat layout for the apply passes -------------------------------------------------------------
// The row layout above leaves lanes idle whenever 256 is not a multiple of C/8 (C = 816: 80 % busy,
// 1392: 68 %, 2304: 56 % with VPT = 2) and keeps only one 16-B load per operand in flight per lane.
// Here the [M, C] tensor is a flat run of M*C/8 16-byte vectors: lane i of a workgroup takes vectors
// base + u*BLOCK (u < FLAT_U, all loads issued before any math), and the per-channel constants are staged
// once per workgroup in LDS, so every lane is busy at every width and FLAT_U*2 loads are in flight.
constexpr int FLAT_U = 4;

__device__ __forceinline__ void lds8(const float* p, float (&o)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// out = act(y*scale + shift) [* rs[n, c]]
template <bool SILU>
__global__ __launch_bounds__(BLOCK) void bn_apply_flat_kernel(const bf16_t* __restrict__ y, uint32_t total, int C,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const float* __restrict__ rs, FastDiv by_nv,
                                                              FastDiv by_hw, bf16_t* __restrict__ out) {
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
        // branch-free body (tail vectors clamped to the last one, only their stores masked): the per-frame gate loads
        // of all FLAT_U vectors can be issued together
        uint4 raw[FLAT_U];
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t i = min(base + u * BLOCK, total - 1);
            raw[u] = *reinterpret_cast<const uint4*>(y + (size_t)i * 8);
        }
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t iu = base + u * BLOCK, i = min(iu, total - 1);
            const uint32_t r = by_nv.div(i), c0 = (i - r * nv) * 8;
            float f[8], sc[8], sh[8];
            f[0] = __uint_as_float(raw[u].x << 16); f[1] = __uint_as_float(raw[u].x & 0xffff0000u);
            f[2] = __uint_as_float(raw[u].y << 16); f[3] = __uint_as_float(raw[u].y & 0xffff0000u);
            f[4] = __uint_as_float(raw[u].z << 16); f[5] = __uint_as_float(raw[u].z & 0xffff0000u);
            f[6] = __uint_as_float(raw[u].w << 16); f[7] = __uint_as_float(raw[u].w & 0xffff0000u);
            lds8(L + c0, sc);
            lds8(L + C + c0, sh);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float t = fmaf(f[j], sc[j], sh[j]);
                f[j] = SILU ? silu(t) : t;
            }
            if (rs) {
                float q[8];
                load8f(rs + (size_t)by_hw.div(r) * C + c0, q);
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] *= q[j];
            }
            if (iu < total) store8(out + (size_t)i * 8, f);
        }
    }
}

// dy = k1*dz + k2*y + k0 with dz = (G*rs + rb) [* silu'(y*scale + shift)]   (constants as in the row kernel)
template <bool SILU>
__global__ __launch_bounds__(BLOCK) void bn_bwd_apply_flat_kernel(const bf16_t* __restrict__ G,
                                                                  const float* __restrict__ rs,
                                                                  const float* __restrict__ rb, FastDiv by_hw,
                                                                  const bf16_t* __restrict__ y, uint32_t total, int C,
                                                                  FastDiv by_nv,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ shift,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd,
                                                                  const float* __restrict__ gamma,
                                                                  const float* __restrict__ mdz,
                                                                  const float* __restrict__ mdzx,
                                                                  bf16_t* __restrict__ dy,
                                                                  const float* __restrict__ keep) {
    extern __shared__ float4 lds_raw[];
    float* L = reinterpret_cast<float*>(lds_raw);     // [5][C]: k0, k1, k2, scale, shift
    for (int c = threadIdx.x; c < C; c += BLOCK) {
        const float rr = rstd[c], b = mdzx[c];
        const float k1 = (gamma ? gamma[c] : 1.f) * rr;
        L[c] = -k1 * (mdz[c] - mean[c] * rr * b);
        L[C + c] = k1;
        L[2 * C + c] = -k1 * rr * b;
        L[3 * C + c] = scale[c];
        L[4 * C + c] = shift[c];
    }
    __syncthreads();
    const uint32_t nv = (uint32_t)(C >> 3);
    const uint32_t step = gridDim.x * BLOCK * FLAT_U;
    for (uint32_t base = blockIdx.x * BLOCK * FLAT_U + threadIdx.x; base < total; base += step) {
        // branch-free body (tail vectors clamped to the last one, only their stores masked): the per-frame rs / rb /
        // keep loads of all FLAT_U vectors can be issued together
        uint4 rg[FLAT_U], ry[FLAT_U];
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t i = min(base + u * BLOCK, total - 1);
            rg[u] = *reinterpret_cast<const uint4*>(G + (size_t)i * 8);
            ry[u] = *reinterpret_cast<const uint4*>(y + (size_t)i * 8);
        }
#pragma unroll
        for (int u = 0; u < FLAT_U; ++u) {
            const uint32_t iu = base + u * BLOCK, i = min(iu, total - 1);
            const uint32_t r = by_nv.div(i), c0 = (i - r * nv) * 8;
            float gv[8], yv[8];
            const uint32_t gw[4] = {rg[u].x, rg[u].y, rg[u].z, rg[u].w};
            const uint32_t yw[4] = {ry[u].x, ry[u].y, ry[u].z, ry[u].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                gv[2 * j] = __uint_as_float(gw[j] << 16); gv[2 * j + 1] = __uint_as_float(gw[j] & 0xffff0000u);
                yv[2 * j] = __uint_as_float(yw[j] << 16); yv[2 * j + 1] = __uint_as_float(yw[j] & 0xffff0000u);
            }
            if (rs || rb) {
                const uint32_t n = by_hw.div(r);
                const size_t off = (size_t)n * C + c0;
                if (rs) {
                    float q[8];
                    load8f(rs + off, q);
                    const float kp = keep ? keep[n] : 1.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) gv[j] *= keep ? q[j] * kp : q[j];
                }
                if (rb) {
                    float q[8];
                    load8f(rb + off, q);
#pragma unroll
                    for (int j = 0; j < 8; ++j) gv[j] += q[j];
                }
            }
            float k0[8], k1[8], k2[8], o[8];
            lds8(L + c0, k0);
            lds8(L + C + c0, k1);
            lds8(L + 2 * C + c0, k2);
            if (SILU) {
                float sc[8], sh[8];
                lds8(L + 3 * C + c0, sc);
                lds8(L + 4 * C + c0, sh);
#pragma unroll
                for (int j = 0; j < 8; ++j) gv[j] *= silu_grad(fmaf(yv[j], sc[j], sh[j]));
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = fmaf(k1[j], gv[j], fmaf(k2[j], yv[j], k0[j]));
            if (iu < total) store8(dy + (size_t)i * 8, o);
        }
    }
}

// flat kernels: they need the vector count to fit 32 bits
// the per-thread kernels cover at most VPT=2 vectors of 8 channels per lane: C must be a multiple of 8, <= 4096
inline bool bn_channels_ok(int C) { return C > 0 && (C & 7) == 0 && (C >> 3) <= 2 * BLOCK; }

inline bool use_flat(int64_t M, int C) {
    return M * (int64_t)(C >> 3) < (int64_t)0xF0000000LL && C <= 3072;   // 5*C floats of LDS <= 60 KB
}

inline int flat_grid(int64_t total) {
    int64_t b = (total + BLOCK * FLAT_U - 1) / (BLOCK * FLAT_U);
    if (b > 4096) b = 4096;
    return (int)(b < 1 ? 1 : b);
}

inline int row_grid(int64_t M, int C) {
    const int nv = C >> 3;
    const int slots = nv <= BLOCK ? BLOCK / nv : 1;
    int64_t b = (M + slots - 1) / slots;
    if (b > 8192) b = 8192;
    return (int)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" {

int rt1_bn_partials_rows(int64_t M, int C, int P) {
    (void)C;
    return (int)((M + P - 1) / P);
}

int rt1_bn_stats(const bf16_t* x, int64_t M, int C, int P, float* psum, float* psq, hipStream_t st) {
    if (!bn_channels_ok(C)) return (int)hipErrorInvalidValue;
    const int64_t rpb = (M + P - 1) / P;
    if ((C >> 3) > BLOCK)
        hipLaunchKernelGGL(bn_stats_kernel<2>, dim3(P), dim3(BLOCK), 0, st, x, M, C, rpb, psum, psq);
    else
        hipLaunchKernelGGL(bn_stats_kernel<1>, dim3(P), dim3(BLOCK), 0, st, x, M, C, rpb, psum, psq);
    return (int)hipGetLastError();
}

int rt1_bn_finalize(const float* psum, const float* psq, int P, int C, double count, const float* gamma,
                    const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                    float* scale, float* shift, float* save_mean, float* save_rstd, hipStream_t st) {
    if (fin_ch(P, C) == 4)
        hipLaunchKernelGGL(bn_finalize_kernel<4>, dim3(fin_grid(C, 4)), dim3(256), 0, st, psum, psq, P, C, count, gamma,
                           beta, eps, momentum, running_mean, running_var, scale, shift, save_mean, save_rstd);
    else
        hipLaunchKernelGGL(bn_finalize_kernel<FIN_CH>, dim3(fin_grid(C)), dim3(256), 0, st, psum, psq, P, C, count,
                           gamma, beta, eps, momentum, running_mean, running_var, scale, shift, save_mean, save_rstd);
    return (int)hipGetLastError();
}

int rt1_bn_apply(const bf16_t* y, int64_t M, int C, const float* scale, const float* shift, int act,
                 const float* rs, int64_t HW, bf16_t* out, hipStream_t st) {
    if (!bn_channels_ok(C)) return (int)hipErrorInvalidValue;
    if (use_flat(M, C)) {
        const uint32_t total = (uint32_t)(M * (C >> 3));
        const FastDiv hw((uint32_t)(HW > 0 ? HW : 1)), nv((uint32_t)(C >> 3));
        const size_t lds = 2 * C * sizeof(float);
        if (act == ACT_SILU)
            hipLaunchKernelGGL(bn_apply_flat_kernel<true>, dim3(flat_grid(total)), dim3(BLOCK), lds, st, y, total, C,
                               scale, shift, rs, nv, hw, out);
        else
            hipLaunchKernelGGL(bn_apply_flat_kernel<false>, dim3(flat_grid(total)), dim3(BLOCK), lds, st, y, total, C,
                               scale, shift, rs, nv, hw, out);
        return (int)hipGetLastError();
    }
    if ((C >> 3) > BLOCK)
        hipLaunchKernelGGL(bn_apply_kernel<2>, dim3(row_grid(M, C)), dim3(BLOCK), 0, st, y, M, C, scale, shift, act, rs,
                           HW, out);
    else
        hipLaunchKernelGGL(bn_apply_kernel<1>, dim3(row_grid(M, C)), dim3(BLOCK), 0, st, y, M, C, scale, shift, act, rs,
                           HW, out);
    return (int)hipGetLastError();
}

int rt1_bn_bwd_reduce(const bf16_t* G, const float* rs, const float* rb, int64_t HW, const bf16_t* y, int64_t M,
                      int C, const float* scale, const float* shift, const float* mean, const float* rstd, int act,
                      int P, float* pdz, float* pdzx, hipStream_t st) {
    if (!bn_channels_ok(C)) return (int)hipErrorInvalidValue;
    const int64_t rpb = (M + P - 1) / P;
    if ((C >> 3) > BLOCK)
        hipLaunchKernelGGL(bn_bwd_reduce_kernel<2>, dim3(P), dim3(BLOCK), 0, st, G, rs, rb, HW, y, M, C, scale, shift,
                           mean, rstd, act, rpb, pdz, pdzx);
    else
        hipLaunchKernelGGL(bn_bwd_reduce_kernel<1>, dim3(P), dim3(BLOCK), 0, st, G, rs, rb, HW, y, M, C, scale, shift,
                           mean, rstd, act, rpb, pdz, pdzx);
    return (int)hipGetLastError();
}

int rt1_bn_bwd_finalize(const float* pdz, const float* pdzx, int P, int C, double count, float* dgamma, float* dbeta,
                        float* mdz, float* mdzx, hipStream_t st, int accumulate) {
    const PwBwdConsts k{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (fin_ch(P, C) == 4)
        hipLaunchKernelGGL(bn_bwd_finalize_kernel<4>, dim3(fin_grid(C, 4)), dim3(256), 0, st, pdz, pdzx, P, C, count,
                           dgamma, dbeta, mdz, mdzx, accumulate, k);
    else
        hipLaunchKernelGGL(bn_bwd_finalize_kernel<FIN_CH>, dim3(fin_grid(C)), dim3(256), 0, st, pdz, pdzx, P, C, count,
                           dgamma, dbeta, mdz, mdzx, accumulate, k);
    return (int)hipGetLastError();
}

int rt1_bn_bwd_finalize_consts(const float* pdz, const float* pdzx, int P, int C, double count, float* dgamma,
                               float* dbeta, float* mdz, float* mdzx, const float* scale, const float* shift,
                               const float* gamma, const float* mean, const float* rstd, float* consts,
                               hipStream_t st) {
    const PwBwdConsts k{scale, shift, gamma, mean, rstd, consts};
    if (fin_ch(P, C) == 4)
        hipLaunchKernelGGL(bn_bwd_finalize_kernel<4>, dim3(fin_grid(C, 4)), dim3(256), 0, st, pdz, pdzx, P, C, count,
                           dgamma, dbeta, mdz, mdzx, 0, k);
    else
        hipLaunchKernelGGL(bn_bwd_finalize_kernel<FIN_CH>, dim3(fin_grid(C)), dim3(256), 0, st, pdz, pdzx, P, C, count,
                           dgamma, dbeta, mdz, mdzx, 0, k);
    return (int)hipGetLastError();
}

int rt1_bn_bwd_apply(const bf16_t* G, const float* rs, const float* rb, int64_t HW, const bf16_t* y, int64_t M, int C,
                     const float* scale, const float* shift, const float* mean, const float* rstd, const float* gamma,
                     int act, const float* mdz, const float* mdzx, bf16_t* dy, hipStream_t st, const float* keep) {
    if (!bn_channels_ok(C)) return (int)hipErrorInvalidValue;
    if (keep && !rs) return (int)hipErrorInvalidValue;     // keep scales the per-frame row multiplier rs
    if (use_flat(M, C)) {
        const uint32_t total = (uint32_t)(M * (C >> 3));
        const FastDiv hw((uint32_t)(HW > 0 ? HW : 1)), nv((uint32_t)(C >> 3));
        const size_t lds = 5 * C * sizeof(float);
        if (act == ACT_SILU)
            hipLaunchKernelGGL(bn_bwd_apply_flat_kernel<true>, dim3(flat_grid(total)), dim3(BLOCK), lds, st, G, rs, rb,
                               hw, y, total, C, nv, scale, shift, mean, rstd, gamma, mdz, mdzx, dy, keep);
        else
            hipLaunchKernelGGL(bn_bwd_apply_flat_kernel<false>, dim3(flat_grid(total)), dim3(BLOCK), lds, st, G, rs,
                               rb, hw, y, total, C, nv, scale, shift, mean, rstd, gamma, mdz, mdzx, dy, keep);
        return (int)hipGetLastError();
    }
    if ((C >> 3) > BLOCK)
        hipLaunchKernelGGL(bn_bwd_apply_kernel<2>, dim3(row_grid(M, C)), dim3(BLOCK), 0, st, G, rs, rb, HW, y, M, C,
                           scale, shift, mean, rstd, gamma, act, mdz, mdzx, dy, keep);
    else
        hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, dim3(row_grid(M, C)), dim3(BLOCK), 0, st, G, rs, rb, HW, y, M, C,
                           scale, shift, mean, rstd, gamma, act, mdz, mdzx, dy, keep);
    return (int)hipGetLastError();
}

}  // extern "C"
