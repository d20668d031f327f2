// Squeeze-excitation backward glue of an MBConv block, fused.
//
// Between its four small GEMMs (dz^T hs, dz f2, dh^T pool, dh f1 -- hipBLASLt), the SE + BN2 backward is a
// chain of [N, C] / [N, se] elementwise maps and column sums over the N frames.  As separate torch ops that is
// ~20 launches per block (x 26 blocks per step, each a few microseconds of GPU time for a few MB); here it is
// three kernels (64 columns x 16 frame groups per workgroup, coalesced across the columns), fp64 column sums in
// a fixed order (bit-reproducible, like the rest of the step):
//   se_bwd_dz     dz = dsum * g * (1 - g)                                  ; db_fc2 = sum_n dz
//   se_bwd_dh     dh = dzf2 * silu'(h)                                     ; db_fc1 = sum_n dh
//   se_bwd_bnsum  rb = rbraw / HW ; sdz = sum_n g*S1 + rb*S2 ; sdzx = sum_n g*S3 + rb*S4 ; mdz, mdzx = / M
// (S1..S4 are the per-frame partial sums of se_bn_bwd_reduce; BN2's dbeta = sdz, dgamma = sdzx.)
#include <algorithm>
#include <cstdlib>

#include "common.h"

using namespace rt1;

namespace {

// a workgroup = CO columns x RG row groups (1024 threads): each thread walks every RG-th frame of its column, the RG
// partial sums of a column are then added in row-group order through LDS (deterministic).  CO = 64 for the wide
// layers; CO = 16 (64 row groups), where 64-column workgroups left few CUs walking 48 frames per thread (the launches
// were 13-24 us of latency for a few hundred KB).
constexpr int COLS = 64, RG = 16, BLOCK = COLS * RG;
constexpr int CO_NARROW = 16;
#ifndef SE_NARROW_MAX
#define SE_NARROW_MAX 4096      // widest C on the 16-column layout (A/B: 256 keeps the 64-column one for C > 256)
#endif
__host__ __device__ constexpr int rg_of(int co) { return BLOCK / co; }

template <int NACC, int CO = COLS>
__device__ __forceinline__ void column_reduce(double (&acc)[NACC], double (*sh)[BLOCK / CO][CO]) {
    constexpr int RGN = BLOCK / CO;
    const int cl = threadIdx.x % CO, rg = threadIdx.x / CO;
#pragma unroll
    for (int a = 0; a < NACC; ++a) sh[a][rg][cl] = acc[a];
    __syncthreads();
    if (rg == 0) {
#pragma unroll
        for (int a = 0; a < NACC; ++a) {
            double t = 0.0;
            for (int r = 0; r < RGN; ++r) t += sh[a][r][cl];
            acc[a] = t;
        }
    }
}

template <int CO>
__global__ __launch_bounds__(BLOCK) void se_bwd_dz_kernel(const float* __restrict__ dsum, const float* __restrict__ gate,
                                                          int N, int C, float* __restrict__ dz,
                                                          float* __restrict__ db) {
    constexpr int RGN = BLOCK / CO;
    __shared__ double sh[1][RGN][CO];
    const int c = blockIdx.x * CO + threadIdx.x % CO, rg = threadIdx.x / CO;
    double acc[1] = {0.0};
    if (c < C) {
#pragma unroll 4
        for (int n = rg; n < N; n += RGN) {
            const int64_t i = (int64_t)n * C + c;
            const float g = gate[i];
            const float d = dsum[i] * g * (1.f - g);
            dz[i] = d;
            acc[0] += (double)d;
        }
    }
    column_reduce<1, CO>(acc, sh);
    if (rg == 0 && c < C) db[c] = (float)acc[0];
}

template <int CO>
__global__ __launch_bounds__(BLOCK) void se_bwd_dh_kernel(const float* __restrict__ dzf2, const float* __restrict__ h,
                                                          int N, int S, float* __restrict__ dh,
                                                          float* __restrict__ db) {
    constexpr int RGN = BLOCK / CO;
    __shared__ double sh[1][RGN][CO];
    const int s = blockIdx.x * CO + threadIdx.x % CO, rg = threadIdx.x / CO;
    double acc[1] = {0.0};
    if (s < S) {
#pragma unroll 4
        for (int n = rg; n < N; n += RGN) {
            const int64_t i = (int64_t)n * S + s;
            const float x = h[i];
            const float sg = 1.f / (1.f + __expf(-x));
            const float d = dzf2[i] * (sg * (1.f + x * (1.f - sg)));
            dh[i] = d;
            acc[0] += (double)d;
        }
    }
    column_reduce<1, CO>(acc, sh);
    if (rg == 0 && s < S) db[s] = (float)acc[0];
}

// red: [5, N, C] (S0 unused here), gate [N, C], rbraw [N, C] -> rb [N, C], sdz / sdzx / mdz / mdzx [C]
template <int CO>
__global__ __launch_bounds__(BLOCK) void se_bwd_bnsum_kernel(const float* __restrict__ red,
                                                             const float* __restrict__ gate,
                                                             const float* __restrict__ rbraw, float inv_hw, int N,
                                                             int C, double count, float* __restrict__ rb,
                                                             float* __restrict__ sdz, float* __restrict__ sdzx,
                                                             float* __restrict__ mdz, float* __restrict__ mdzx) {
    constexpr int RGN = BLOCK / CO;
    __shared__ double sh[2][RGN][CO];
    const int c = blockIdx.x * CO + threadIdx.x % CO, rg = threadIdx.x / CO;
    const int64_t NC = (int64_t)N * C;
    double acc[2] = {0.0, 0.0};
    if (c < C) {
#pragma unroll 4
        for (int n = rg; n < N; n += RGN) {
            const int64_t i = (int64_t)n * C + c;
            const float g = gate[i];
            const float r = rbraw[i] * inv_hw;
            rb[i] = r;
            acc[0] += (double)(g * red[NC + i] + r * red[2 * NC + i]);
            acc[1] += (double)(g * red[3 * NC + i] + r * red[4 * NC + i]);
        }
    }
    column_reduce<2, CO>(acc, sh);
    if (rg == 0 && c < C) {
        sdz[c] = (float)acc[0];
        sdzx[c] = (float)acc[1];
        mdz[c] = (float)(acc[0] / count);
        mdzx[c] = (float)(acc[1] / count);
    }
}


// ---------------------------------------------------------------- whole SE MLP: 2 forward + 4 backward kernels
// The squeeze-excitation MLP of every MBConv block is [N, C] x [C, S] x [S, C] with N = 768 frames, C <= 2304,
// S <= 96 (~0.7 GFLOP at the widest block).  As torch ops it is 4-5 forward and 7 backward launches per block
// (hipBLASLt fp32 GEMMs on 16x16 .. 32x32 macro tiles plus silu / sigmoid / glue maps).  Here, all fp32 FMAs with
// fixed summation orders (bit-reproducible), weights read in their parameter layouts (fc1 [S, C], fc2 [C, S]):
//   se_rowdot   part[ks][n][j] = sum_{c in slice ks} X[n][c] W[j][c]      fc1 (X = pool sum) / bwd (X = dz, W = fc2^T)
//   se_rowmat   out[n][c] = epi(sum_j Y[n][j] V[c][j])   Y = act(sum_ks part + b): fwd gate = sigmoid(. + b2) from
//               hs = silu(h); bwd rb = (.) / HW from dh = (.) silu'(h)
//   se_wsum_part / se_wsum_fin   the reductions over frames (fc weight / bias gradients, BN2 sums in fp64), split
//               over NS frame slices then combined in slice order
// Every launch has 100-900 workgroups of register-blocked tiles (LDS-staged operands, 4-16 FMAs per LDS read).  A
// first version ran one workgroup per 8 frames with a pair of lanes per output and every frame chain serial in one
// workgroup for the weight sums: 35-470 us per call (profiles/r3_gemm_step_ab.md).
constexpr int SE_BLOCK = 256;
constexpr int RD_FT = 32, RD_JT = 32, RD_KC = 64, RD_LD = RD_KC + 4;
constexpr int RM_CT = 128;
constexpr int WS_CT = 64, WS_JT = 32, WS_FC = 32, WS_NS = 8;

// thread (fr, ur) = 2 frames x 2 units; the K slice [kb, ke) is walked in LDS chunks of RD_KC, float4 along K
template <bool BWD>
__global__ NO_PACKED_FP32 __launch_bounds__(SE_BLOCK) void se_rowdot_kernel(const float* __restrict__ X, const float* __restrict__ gate,
                                                             const float* __restrict__ W, int N, int C, int S,
                                                             int kslice, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float xs[RD_FT][RD_LD];
    __shared__ __attribute__((aligned(16))) float ws[RD_JT][RD_LD];
    const int t = threadIdx.x;
    const int n0 = blockIdx.x * RD_FT, j0 = blockIdx.y * RD_JT, ks = blockIdx.z;
    const int kb = ks * kslice, ke = min(C, kb + kslice);
    const int fr = (t >> 4) * 2, ur = (t & 15) * 2;
    float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    for (int c0 = kb; c0 < ke; c0 += RD_KC) {
        __syncthreads();
        for (int i = t; i < RD_FT * RD_KC / 4; i += SE_BLOCK) {
            const int r = i / (RD_KC / 4), q = (i % (RD_KC / 4)) * 4, n = n0 + r, c = c0 + q;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n < N && c < ke) {
                const int64_t o = (int64_t)n * C + c;
                v = *reinterpret_cast<const float4*>(X + o);
                if constexpr (BWD) {     // dz = dsum * g (1 - g)
                    const float4 g = *reinterpret_cast<const float4*>(gate + o);
                    v.x *= g.x * (1.f - g.x); v.y *= g.y * (1.f - g.y);
                    v.z *= g.z * (1.f - g.z); v.w *= g.w * (1.f - g.w);
                }
            }
            *reinterpret_cast<float4*>(&xs[r][q]) = v;
        }
        if constexpr (!BWD) {            // fc1 [S, C]: rows along K
            for (int i = t; i < RD_JT * RD_KC / 4; i += SE_BLOCK) {
                const int r = i / (RD_KC / 4), q = (i % (RD_KC / 4)) * 4, j = j0 + r, c = c0 + q;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (j < S && c < ke) v = *reinterpret_cast<const float4*>(W + (int64_t)j * C + c);
                *reinterpret_cast<float4*>(&ws[r][q]) = v;
            }
        } else {                         // fc2 [C, S]: read along S (coalesced rows), stored transposed
            for (int i = t; i < RD_JT * RD_KC; i += SE_BLOCK) {
                const int q = i / RD_JT, r = i % RD_JT, j = j0 + r, c = c0 + q;
                ws[r][q] = (j < S && c < ke) ? W[(int64_t)c * S + j] : 0.f;
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int k = 0; k < RD_KC; k += 4) {
            const float4 x0 = *reinterpret_cast<const float4*>(&xs[fr][k]);
            const float4 x1 = *reinterpret_cast<const float4*>(&xs[fr + 1][k]);
            const float4 w0 = *reinterpret_cast<const float4*>(&ws[ur][k]);
            const float4 w1 = *reinterpret_cast<const float4*>(&ws[ur + 1][k]);
            acc[0][0] = fmaf(x0.w, w0.w, fmaf(x0.z, w0.z, fmaf(x0.y, w0.y, fmaf(x0.x, w0.x, acc[0][0]))));
            acc[0][1] = fmaf(x0.w, w1.w, fmaf(x0.z, w1.z, fmaf(x0.y, w1.y, fmaf(x0.x, w1.x, acc[0][1]))));
            acc[1][0] = fmaf(x1.w, w0.w, fmaf(x1.z, w0.z, fmaf(x1.y, w0.y, fmaf(x1.x, w0.x, acc[1][0]))));
            acc[1][1] = fmaf(x1.w, w1.w, fmaf(x1.z, w1.z, fmaf(x1.y, w1.y, fmaf(x1.x, w1.x, acc[1][1]))));
        }
    }
    float* pp = part + (int64_t)ks * N * S;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int n = n0 + fr + a, j = j0 + ur + b;
            if (n < N && j < S) pp[(int64_t)n * S + j] = acc[a][b];
        }
}

// Y rows of this workgroup's FT frames from the K-slice partials, times the (S x RM_CT) tile of V, over K = S
// fwd: h = sum part * inv_hw + b1 (stored by channel tile 0), Y = silu(h), out = gate = sigmoid(Y . fc2^T + b2)
// bwd: dh = sum part * silu'(h)  (stored by channel tile 0), Y = dh,      out = rb   = (Y . fc1) * inv_hw
// FT = 16 where 32-frame tiles leave the chip under-filled (24 x ceil(C / 128) workgroups at N = 768: 24-264 for all
// but the widest block).  The V tile is loaded into registers first and written to LDS after the partial sums: its
// loads are independent of them, so their latency hides under the partial reduction instead of following it.
__host__ __device__ constexpr int rm_fwd_stride(int S) { return S | 1; }

template <bool BWD, int FT>
__global__ NO_PACKED_FP32 __launch_bounds__(SE_BLOCK) void se_rowmat_kernel(const float* __restrict__ part, int KS,
                                                             const float* __restrict__ b1, const float* __restrict__ hin,
                                                             float* __restrict__ yout, const float* __restrict__ V,
                                                             const float* __restrict__ b2, float inv_hw, int N, int C,
                                                             int S, float* __restrict__ out) {
    constexpr int FPT = FT / 16;                     // frames per thread in the product
    constexpr int NVB = 128 * RM_CT / SE_BLOCK;      // V values per thread at the largest S (128)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    // fwd: fc2 rows as loaded, [RM_CT][SP] with an odd row stride SP: the staging stores (consecutive lanes along j)
    // and the product's reads (16 lane groups 4 rows apart, same j) are both bank-conflict free.  (The [S][RM_CT]
    // transpose it replaces had every lane of a store on one bank: 6.6 conflict cycles per LDS cycle, SQ counters.)
    // bwd: fc1 [S][RM_CT], as loaded, float4 reads along the channels
    const int SP = rm_fwd_stride(S);
    float* ys = sm;                                  // [FT][S]
    float* vt = sm + FT * S;
    const int t = threadIdx.x, n0 = blockIdx.x * FT, c0 = blockIdx.y * RM_CT;
    const int64_t NS_ = (int64_t)N * S;
    const int nv = S * RM_CT;
    // fwd: element i = (cl, j) = divmod(i, S) of the contiguous [RM_CT][S] block of fc2 rows, stepped by SE_BLOCK
    // without a division per element (64 integer divisions per thread, twice, were the bulk of the forward's time)
    const int dq = SE_BLOCK / S, dr = SE_BLOCK - dq * S, cl0 = t / S, j0 = t - cl0 * S;
    float v[NVB];
    const int vend = min(nv, (C - c0) * S);          // fwd: the rows c < C of the block
#pragma unroll
    for (int u = 0; u < NVB; ++u) {
        const int i = u * SE_BLOCK + t;
        v[u] = 0.f;
        if constexpr (!BWD) {            // fc2 [C, S]: rows c0 .. c0 + RM_CT are one contiguous block
            if (i < vend) v[u] = V[(int64_t)c0 * S + i];
        } else if (i < nv) {             // fc1 [S, C]: row j contiguous in c
            const int jj = i / RM_CT, c = c0 + i - jj * RM_CT;
            if (c < C) v[u] = V[(int64_t)jj * C + c];
        }
    }
    for (int base = 0; base < FT * S; base += 4 * SE_BLOCK) {
        // the K-slice partials of 4 outputs: slice-outer so each round has 4 x 4 independent loads in flight (an
        // output-outer loop issued one dependent L2 load per partial); per output the sum order is still k = 0 ..
        float sum[4];
        int64_t o[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = base + u * SE_BLOCK + t, r = i / S, n = n0 + r;
            sum[u] = 0.f;
            ok[u] = i < FT * S && n < N;
            o[u] = ok[u] ? (int64_t)n * S + (i - r * S) : 0;
        }
#pragma unroll 4
        for (int k = 0; k < KS; ++k) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (ok[u]) sum[u] += part[k * NS_ + o[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = base + u * SE_BLOCK + t;
            if (i >= FT * S) break;
            const int r = i / S, j = i - r * S, n = n0 + r;
            float y = 0.f;
            if (n < N) {
                const int64_t o = (int64_t)n * S + j;
                if constexpr (!BWD) {
                    const float hv = sum[u] * inv_hw + b1[j];
                    if (blockIdx.y == 0) yout[o] = hv;
                    y = silu(hv);
                } else {
                    const float x = hin[o];
                    const float sg = sigmoidf_(x);
                    y = sum[u] * (sg * (1.f + x * (1.f - sg)));
                    if (blockIdx.y == 0) yout[o] = y;
                }
            }
            ys[i] = y;
        }
    }
    {
        int cl = cl0, j = j0;
#pragma unroll
        for (int u = 0; u < NVB; ++u) {
            const int i = u * SE_BLOCK + t;
            if (i >= nv) break;
            if constexpr (!BWD) vt[cl * SP + j] = v[u];
            else vt[i] = v[u];
            j += dr;
            cl += dq;
            if (j >= S) { j -= S; ++cl; }
        }
    }
    __syncthreads();
    // thread = FPT frames x 8 channels (two float4 column groups 64 apart: conflict-free LDS reads)
    const int f = (t >> 4) * FPT, cq = (t & 15) * 4;
    float acc[FPT][8];
#pragma unroll
    for (int a = 0; a < FPT; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = 0.f;
    for (int j = 0; j < S; ++j) {
        float vv[8];
        if constexpr (!BWD) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                vv[b] = vt[(cq + b) * SP + j];
                vv[4 + b] = vt[(64 + cq + b) * SP + j];
            }
        } else {
            const float4 v4 = *reinterpret_cast<const float4*>(vt + j * RM_CT + cq);
            const float4 u4 = *reinterpret_cast<const float4*>(vt + j * RM_CT + 64 + cq);
            vv[0] = v4.x; vv[1] = v4.y; vv[2] = v4.z; vv[3] = v4.w;
            vv[4] = u4.x; vv[5] = u4.y; vv[6] = u4.z; vv[7] = u4.w;
        }
#pragma unroll
        for (int a = 0; a < FPT; ++a) {
            const float y = ys[(f + a) * S + j];
#pragma unroll
            for (int b = 0; b < 8; ++b) acc[a][b] = fmaf(y, vv[b], acc[a][b]);
        }
    }
#pragma unroll
    for (int a = 0; a < FPT; ++a) {
        const int n = n0 + f + a;
        if (n >= N) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = c0 + cq + h * 64;          // C % 4 == 0: a float4 group is all in or all out
            if (c >= C) continue;
            float r[4];
#pragma unroll
            for (int b = 0; b < 4; ++b)
                r[b] = BWD ? acc[a][h * 4 + b] * inv_hw : sigmoidf_(acc[a][h * 4 + b] + b2[c + b]);
            *reinterpret_cast<float4*>(out + (int64_t)n * C + c) = make_float4(r[0], r[1], r[2], r[3]);
        }
    }
}

// weight / bias / BN2 sums over one frame slice (blockIdx.z) of a (64-channel x 32-unit) tile; thread (cq, jp) = 4
// channels x 2 units of both products:  dw2[c][j] += dz hs,  dw1[j][c] += dh pool.  Channel tile 0 also sums db1
// (threads cq = 0), unit tile 0 the per-channel db2 / BN2 sums in fp64 while staging.
__global__ NO_PACKED_FP32 __launch_bounds__(SE_BLOCK) void se_wsum_part_kernel(const float* __restrict__ red,
                                                                const float* __restrict__ gate,
                                                                const float* __restrict__ h,
                                                                const float* __restrict__ dh,
                                                                const float* __restrict__ pool,
                                                                const float* __restrict__ rb, int N, int C, int S,
                                                                int nslice, float* __restrict__ pw2,
                                                                float* __restrict__ pw1, double* __restrict__ pc,
                                                                double* __restrict__ pj) {
    __shared__ __attribute__((aligned(16))) float zs[WS_FC][WS_CT];
    __shared__ __attribute__((aligned(16))) float ps[WS_FC][WS_CT];
    __shared__ __attribute__((aligned(16))) float hs[WS_FC][WS_JT];
    __shared__ __attribute__((aligned(16))) float ds[WS_FC][WS_JT];
    const int t = threadIdx.x;
    const int c0 = blockIdx.x * WS_CT, j0 = blockIdx.y * WS_JT, sl = blockIdx.z;
    const int nb = sl * nslice, ne = min(N, nb + nslice);
    const int cq = (t & 15) * 4, jp = (t >> 4) * 2;
    const int64_t NC = (int64_t)N * C;
    float a2[4][2], a1[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a) a2[a][0] = a2[a][1] = a1[a][0] = a1[a][1] = 0.f;
    // per-channel sums (unit tile 0 only): every thread accumulates the channel quad it stages (q = t % 16) over its
    // staging rows (t / 16, t / 16 + 16 of each chunk); the 16 row groups are combined in order at the end
    double cz[4] = {0.0, 0.0, 0.0, 0.0}, c1[4] = {0.0, 0.0, 0.0, 0.0}, c2[4] = {0.0, 0.0, 0.0, 0.0};
    double jd[2] = {0.0, 0.0};
    const bool csum = blockIdx.y == 0, jsum = blockIdx.x == 0 && cq == 0;
    for (int f0 = nb; f0 < ne; f0 += WS_FC) {
        __syncthreads();
        for (int i = t; i < WS_FC * WS_CT / 4; i += SE_BLOCK) {
            const int r = i / (WS_CT / 4), q = (i % (WS_CT / 4)) * 4, n = f0 + r, c = c0 + q;
            float4 z = make_float4(0.f, 0.f, 0.f, 0.f), p = z;
            if (n < ne && c < C) {
                const int64_t o = (int64_t)n * C + c;
                const float4 d = *reinterpret_cast<const float4*>(red + o);
                const float4 g = *reinterpret_cast<const float4*>(gate + o);
                z = make_float4(d.x * g.x * (1.f - g.x), d.y * g.y * (1.f - g.y), d.z * g.z * (1.f - g.z),
                                d.w * g.w * (1.f - g.w));
                p = *reinterpret_cast<const float4*>(pool + o);
                if (csum) {
                    const float4 rr = *reinterpret_cast<const float4*>(rb + o);
                    const float4 r1 = *reinterpret_cast<const float4*>(red + NC + o);
                    const float4 r2 = *reinterpret_cast<const float4*>(red + 2 * NC + o);
                    const float4 r3 = *reinterpret_cast<const float4*>(red + 3 * NC + o);
                    const float4 r4 = *reinterpret_cast<const float4*>(red + 4 * NC + o);
                    const float gg[4] = {g.x, g.y, g.z, g.w}, rv[4] = {rr.x, rr.y, rr.z, rr.w};
                    const float v1[4] = {r1.x, r1.y, r1.z, r1.w}, v2[4] = {r2.x, r2.y, r2.z, r2.w};
                    const float v3[4] = {r3.x, r3.y, r3.z, r3.w}, v4[4] = {r4.x, r4.y, r4.z, r4.w};
                    const float zz[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
                    for (int a = 0; a < 4; ++a) {
                        cz[a] += (double)zz[a];
                        c1[a] += (double)(gg[a] * v1[a] + rv[a] * v2[a]);
                        c2[a] += (double)(gg[a] * v3[a] + rv[a] * v4[a]);
                    }
                }
            }
            *reinterpret_cast<float4*>(&zs[r][q]) = z;
            *reinterpret_cast<float4*>(&ps[r][q]) = p;
        }
        for (int i = t; i < WS_FC * WS_JT; i += SE_BLOCK) {
            const int r = i / WS_JT, q = i % WS_JT, n = f0 + r, j = j0 + q;
            float hv = 0.f, dv = 0.f;
            if (n < ne && j < S) {
                const float x = h[(int64_t)n * S + j];
                hv = x * sigmoidf_(x);
                dv = dh[(int64_t)n * S + j];
            }
            hs[r][q] = hv;
            ds[r][q] = dv;
        }
        __syncthreads();
        const int fe = min(WS_FC, ne - f0);
        for (int r = 0; r < fe; ++r) {
            const float4 z = *reinterpret_cast<const float4*>(&zs[r][cq]);
            const float4 p = *reinterpret_cast<const float4*>(&ps[r][cq]);
            const float2 hv = *reinterpret_cast<const float2*>(&hs[r][jp]);
            const float2 dv = *reinterpret_cast<const float2*>(&ds[r][jp]);
            const float zz[4] = {z.x, z.y, z.z, z.w}, pp[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                a2[a][0] = fmaf(zz[a], hv.x, a2[a][0]);
                a2[a][1] = fmaf(zz[a], hv.y, a2[a][1]);
                a1[a][0] = fmaf(dv.x, pp[a], a1[a][0]);
                a1[a][1] = fmaf(dv.y, pp[a], a1[a][1]);
            }
            if (jsum) {
                jd[0] += (double)dv.x;
                jd[1] += (double)dv.y;
            }
        }
    }
    if (csum) {              // combine the 16 staging row groups of each channel quad in row-group order
        __shared__ double cred[3][16][WS_CT];
        __syncthreads();
        const int q = (t & 15) * 4, g = t >> 4;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            cred[0][g][q + a] = cz[a];
            cred[1][g][q + a] = c1[a];
            cred[2][g][q + a] = c2[a];
        }
        __syncthreads();
        if (t < WS_CT) {
            double x0 = 0.0, x1 = 0.0, x2 = 0.0;
            for (int r = 0; r < 16; ++r) {
                x0 += cred[0][r][t];
                x1 += cred[1][r][t];
                x2 += cred[2][r][t];
            }
            const int c = c0 + t;
            if (c < C) {
                pc[((int64_t)sl * 3 + 0) * C + c] = x0;
                pc[((int64_t)sl * 3 + 1) * C + c] = x1;
                pc[((int64_t)sl * 3 + 2) * C + c] = x2;
            }
        }
    }
    const int64_t CS = (int64_t)C * S;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int c = c0 + cq + a;
        if (c >= C) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int j = j0 + jp + b;
            if (j >= S) continue;
            pw2[sl * CS + (int64_t)c * S + j] = a2[a][b];
            pw1[sl * CS + (int64_t)j * C + c] = a1[a][b];
        }
    }
    if (jsum) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
            if (j0 + jp + b < S) pj[(int64_t)sl * S + j0 + jp + b] = jd[b];
    }
}

// slice partials -> dw2 [C, S], dw1 [S, C] (x inv_hw: pool holds frame SUMS), db2, BN2 sums / means, db1
__global__ __launch_bounds__(SE_BLOCK) void se_wsum_fin_kernel(const float* __restrict__ pw2,
                                                               const float* __restrict__ pw1,
                                                               const double* __restrict__ pc,
                                                               const double* __restrict__ pj, int NSL, int C, int S,
                                                               float inv_hw, double count, float* __restrict__ dw2,
                                                               float* __restrict__ dw1, float* __restrict__ db2,
                                                               float* __restrict__ db1, float* __restrict__ sdz,
                                                               float* __restrict__ sdzx, float* __restrict__ mdz,
                                                               float* __restrict__ mdzx) {
    const int64_t CS = (int64_t)C * S;
    const int64_t total = 2 * CS + C + S;
    for (int64_t i = (int64_t)blockIdx.x * SE_BLOCK + threadIdx.x; i < total; i += (int64_t)gridDim.x * SE_BLOCK) {
        if (i < CS) {
            float a = 0.f;
#pragma unroll 8
            for (int k = 0; k < NSL; ++k) a += pw2[k * CS + i];
            dw2[i] = a;
        } else if (i < 2 * CS) {
            const int64_t o = i - CS;
            float a = 0.f;
#pragma unroll 8
            for (int k = 0; k < NSL; ++k) a += pw1[k * CS + o];
            dw1[o] = a * inv_hw;
        } else if (i < 2 * CS + C) {
            const int c = (int)(i - 2 * CS);
            double z = 0.0, x = 0.0, y = 0.0;
#pragma unroll 8
            for (int k = 0; k < NSL; ++k) {
                z += pc[((int64_t)k * 3 + 0) * C + c];
                x += pc[((int64_t)k * 3 + 1) * C + c];
                y += pc[((int64_t)k * 3 + 2) * C + c];
            }
            db2[c] = (float)z;
            sdz[c] = (float)x;
            sdzx[c] = (float)y;
            mdz[c] = (float)(x / count);
            mdzx[c] = (float)(y / count);
        } else {
            const int j = (int)(i - 2 * CS - C);
            double a = 0.0;
#pragma unroll 8
            for (int k = 0; k < NSL; ++k) a += pj[(int64_t)k * S + j];
            db1[j] = (float)a;
        }
    }
}

constexpr int RD_TARGET_WG = 512;   // se_rowdot workgroups the K split aims for

int rd_splits(int N, int C, int S) {
    const int base = ((N + RD_FT - 1) / RD_FT) * ((S + RD_JT - 1) / RD_JT);
    const int chunks = (C + RD_KC - 1) / RD_KC;
    int ks = (RD_TARGET_WG + base - 1) / base;    // ~512 workgroups: few K chunks each, few partials for se_rowmat
    return ks < 1 ? 1 : (ks > chunks ? chunks : ks);
}

// 32-frame se_rowmat tiles once they give this many workgroups (N = 768: C = 1392 -> 264, C = 2304 -> 432 tiles of 32
// frames).  Same-box A/Bs (profiles/r6_se_ab*.log): the forward is faster on 32-frame tiles from C = 1392 up (16-frame
// tiles: 44.4 vs 36.2 us there), the backward on 16-frame tiles at C = 1392 (74 vs 84 us) and on 32-frame ones at
// C = 2304 (864 workgroups of 16 frames at 2 per CU are two waves of workgroups: 208 vs 160 us)
#ifndef SE_RM_WIDE_WG_FWD
#define SE_RM_WIDE_WG_FWD 200
#endif
#ifndef SE_RM_WIDE_WG_BWD
#define SE_RM_WIDE_WG_BWD 300
#endif
template <bool BWD>
void launch_rowmat(const float* part, int KS, const float* b1, const float* hin, float* yout, const float* V,
                   const float* b2, float inv_hw, int N, int C, int S, float* out, hipStream_t st) {
    const int ct = (C + RM_CT - 1) / RM_CT;
    if (((N + 31) / 32) * ct >= (BWD ? SE_RM_WIDE_WG_BWD : SE_RM_WIDE_WG_FWD))
        hipLaunchKernelGGL((se_rowmat_kernel<BWD, 32>), dim3((N + 31) / 32, ct), dim3(SE_BLOCK),
                           (size_t)(32 * S + RM_CT * (BWD ? S : rm_fwd_stride(S))) * sizeof(float), st, part, KS, b1, hin, yout, V, b2, inv_hw, N,
                           C, S, out);
    else
        hipLaunchKernelGGL((se_rowmat_kernel<BWD, 16>), dim3((N + 15) / 16, ct), dim3(SE_BLOCK),
                           (size_t)(16 * S + RM_CT * (BWD ? S : rm_fwd_stride(S))) * sizeof(float), st, part, KS, b1, hin, yout, V, b2, inv_hw, N,
                           C, S, out);
}

// frame slices of se_wsum_part: WS_NS, more (up to WS_NS_MAX) where the (channel x unit) tiles alone give few
// workgroups -- 3-72 tiles on the narrow blocks (C <= 576), i.e. 24-576 workgroups walking 96 frames each at N = 768
// with 8 slices, most of them latency-bound on one CU.  A pure function of the shape: the summation order (slice
// partials, then slices in order in se_wsum_fin) stays fixed per shape, so the sums stay bit-reproducible.
constexpr int WS_NS_MAX = 32, WS_TARGET_WG = 512;
int ws_splits(int N, int C, int S) {
    const int base = ((C + WS_CT - 1) / WS_CT) * ((S + WS_JT - 1) / WS_JT);
    int ns = (WS_TARGET_WG + base - 1) / base;
    ns = ns < WS_NS ? WS_NS : (ns > WS_NS_MAX ? WS_NS_MAX : ns);
    return ns > N ? (N < 1 ? 1 : N) : ns;
}

}  // namespace

extern "C" {

int rt1_se_bwd_dz(const float* dsum, const float* gate, int N, int C, float* dz, float* db, hipStream_t st) {
    if (N <= 0 || C <= 0) return (int)hipErrorInvalidValue;
    if (C <= SE_NARROW_MAX)
        hipLaunchKernelGGL(se_bwd_dz_kernel<CO_NARROW>, dim3((C + CO_NARROW - 1) / CO_NARROW), dim3(BLOCK), 0, st, dsum,
                           gate, N, C, dz, db);
    else
        hipLaunchKernelGGL(se_bwd_dz_kernel<COLS>, dim3((C + COLS - 1) / COLS), dim3(BLOCK), 0, st, dsum, gate, N, C, dz,
                           db);
    return (int)hipGetLastError();
}

int rt1_se_bwd_dh(const float* dzf2, const float* h, int N, int S, float* dh, float* db, hipStream_t st) {
    if (N <= 0 || S <= 0) return (int)hipErrorInvalidValue;
    if (S <= SE_NARROW_MAX)
        hipLaunchKernelGGL(se_bwd_dh_kernel<CO_NARROW>, dim3((S + CO_NARROW - 1) / CO_NARROW), dim3(BLOCK), 0, st, dzf2,
                           h, N, S, dh, db);
    else
        hipLaunchKernelGGL(se_bwd_dh_kernel<COLS>, dim3((S + COLS - 1) / COLS), dim3(BLOCK), 0, st, dzf2, h, N, S, dh,
                           db);
    return (int)hipGetLastError();
}

int rt1_se_bwd_bnsum(const float* red, const float* gate, const float* rbraw, float inv_hw, int N, int C, double count,
                     float* rb, float* sdz, float* sdzx, float* mdz, float* mdzx, hipStream_t st) {
    if (N <= 0 || C <= 0 || count <= 0) return (int)hipErrorInvalidValue;
    if (C <= SE_NARROW_MAX)
        hipLaunchKernelGGL(se_bwd_bnsum_kernel<CO_NARROW>, dim3((C + CO_NARROW - 1) / CO_NARROW), dim3(BLOCK), 0, st, red,
                           gate, rbraw, inv_hw, N, C, count, rb, sdz, sdzx, mdz, mdzx);
    else
        hipLaunchKernelGGL(se_bwd_bnsum_kernel<COLS>, dim3((C + COLS - 1) / COLS), dim3(BLOCK), 0, st, red, gate, rbraw,
                           inv_hw, N, C, count, rb, sdz, sdzx, mdz, mdzx);
    return (int)hipGetLastError();
}


int rt1_se_part_size(int N, int C, int S) { return rd_splits(N, C, S) * N * S; }

// pool_sum [N, C] (frame_pool) -> h = fc1 pre-activation [N, S], gate [N, C]; part: rt1_se_part_size floats
int rt1_se_fwd(const float* pool_sum, float inv_hw, int N, int C, int S, const float* w1, const float* b1,
               const float* w2, const float* b2, float* part, float* h, float* gate, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || S > 128 || C % 4) return (int)hipErrorInvalidValue;
    const int ks = rd_splits(N, C, S);
    const int kslice = ((C + ks - 1) / ks + RD_KC - 1) / RD_KC * RD_KC;
    const int ksn = (C + kslice - 1) / kslice;
    hipLaunchKernelGGL(se_rowdot_kernel<false>, dim3((N + RD_FT - 1) / RD_FT, (S + RD_JT - 1) / RD_JT, ksn),
                       dim3(SE_BLOCK), 0, st, pool_sum, nullptr, w1, N, C, S, kslice, part);
    launch_rowmat<false>(part, ksn, b1, nullptr, h, w2, b2, inv_hw, N, C, S, gate, st);
    return (int)hipGetLastError();
}

// dsum = red row 0 [N, C], gate [N, C], h [N, S] -> dh [N, S], rb [N, C]
int rt1_se_bwd_frame(const float* dsum, const float* gate, const float* h, float inv_hw, int N, int C, int S,
                     const float* w1, const float* w2, float* part, float* dh, float* rb, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || S > 128 || C % 4) return (int)hipErrorInvalidValue;
    const int ks = rd_splits(N, C, S);
    const int kslice = ((C + ks - 1) / ks + RD_KC - 1) / RD_KC * RD_KC;
    const int ksn = (C + kslice - 1) / kslice;
    hipLaunchKernelGGL(se_rowdot_kernel<true>, dim3((N + RD_FT - 1) / RD_FT, (S + RD_JT - 1) / RD_JT, ksn),
                       dim3(SE_BLOCK), 0, st, dsum, gate, w2, N, C, S, kslice, part);
    launch_rowmat<true>(part, ksn, nullptr, h, dh, w1, nullptr, inv_hw, N, C, S, rb, st);
    return (int)hipGetLastError();
}

// workspace floats for rt1_se_bwd_wsum: 2 * NS * C * S floats + (3 * NS * C + NS * S) doubles
size_t rt1_se_wsum_ws_bytes(int N, int C, int S) {
    const int ns = ws_splits(N, C, S);
    return (size_t)2 * ns * C * S * sizeof(float) + ((size_t)3 * ns * C + (size_t)ns * S) * sizeof(double);
}

int rt1_se_bwd_wsum(const float* red, const float* gate, const float* h, const float* dh, const float* pool,
                    const float* rb, int N, int C, int S, float inv_hw, double count, void* ws, float* dw2,
                    float* dw1, float* db2, float* db1, float* sdz, float* sdzx, float* mdz, float* mdzx,
                    hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || count <= 0 || C % 4) return (int)hipErrorInvalidValue;
    const int ns = ws_splits(N, C, S);
    const int nslice = (N + ns - 1) / ns;
    const int nsl = (N + nslice - 1) / nslice;
    double* pc = reinterpret_cast<double*>(ws);                       // [NS][3][C]
    double* pj = pc + (size_t)3 * ns * C;                             // [NS][S]
    float* pw2 = reinterpret_cast<float*>(pj + (size_t)ns * S);       // [NS][C][S]
    float* pw1 = pw2 + (size_t)ns * C * S;                            // [NS][S][C]
    hipLaunchKernelGGL(se_wsum_part_kernel, dim3((C + WS_CT - 1) / WS_CT, (S + WS_JT - 1) / WS_JT, nsl),
                       dim3(SE_BLOCK), 0, st, red, gate, h, dh, pool, rb, N, C, S, nslice, pw2, pw1, pc, pj);
    const int64_t total = 2 * (int64_t)C * S + C + S;
    const int grid = (int)std::min<int64_t>(1024, (total + SE_BLOCK - 1) / SE_BLOCK);
    hipLaunchKernelGGL(se_wsum_fin_kernel, dim3(grid), dim3(SE_BLOCK), 0, st, pw2, pw1, pc, pj, nsl, C, S, inv_hw, count,
                       dw2, dw1, db2, db1, sdz, sdzx, mdz, mdzx);
    return (int)hipGetLastError();
}

}  // extern "C"
