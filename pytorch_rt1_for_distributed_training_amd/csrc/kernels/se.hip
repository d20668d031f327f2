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


// ---------------------------------------------------------------- whole SE MLP in four / three kernels
// The squeeze-excitation MLP of every MBConv block is [N, C] x [C, S] x [S, C] with N = 768 frames, C <= 2304,
// S <= 96: ~0.7 GFLOP at the widest block, but as torch ops it was 6 forward and 8 backward launches of
// few-microsecond kernels (hipBLASLt GEMMs on 16x16 .. 32x32 macro tiles, silu / sigmoid / divide maps) per block,
// ~340 launches per step.  Here the forward is two kernels and the backward three, all fp32 FMAs with fixed
// summation orders (bit-reproducible), weights read in their parameter layouts (fc1 [S, C], fc2 [C, S]):
//   se_fc1    h = pool . fc1^T + b1                  grid (frame groups x unit groups), C streamed through LDS
//   se_fc2    gate = sigmoid(silu(h) . fc2^T + b2)   grid (frame groups x channel groups), fc2 chunks through LDS
//   se_bwd_a  dz = dsum g (1 - g);  dh = (dz . fc2) silu'(h)   (frame groups x unit groups)
//   se_bwd_b  rb = (dh . fc1) / HW                   (frame groups x channel groups)
//   se_bwd_wsum  the reductions over the frames (fc weight / bias gradients, BN2 sums)
// A first version ran each per-frame chain in ONE workgroup per 8 frames (96 workgroups for 768 frames, every
// workgroup walking all C channels and all S units: long dependent FMA chains on a third of the CUs) and measured
// 2.5-5x slower than the launches it replaced (profiles/r2_se_fused_ab.log).  Splitting the unit / channel
// dimension over the grid gives 200-900 workgroups per launch.
constexpr int SE_FR = 8;        // frames per workgroup
constexpr int SE_BLOCK = 256;
constexpr int SE_SU = 16;       // fc1 / dz.fc2 output units per workgroup
constexpr int SE_CH = 256;      // channels per LDS chunk
constexpr int SE_JC = 32;       // fc2 columns per LDS chunk (se_fc2)

// thread layout of the unit-group kernels: pair p = t / 2 = (frame f = p / SE_SU, unit u = p % SE_SU), half = t & 1
// sums the even / odd channels of each chunk; the halves are added with one xor shuffle (fixed order)
__global__ __launch_bounds__(SE_BLOCK) void se_fc1_kernel(const float* __restrict__ pool_sum, float inv_hw, int N,
                                                          int C, int S, const float* __restrict__ w1,
                                                          const float* __restrict__ b1, float* __restrict__ pool,
                                                          float* __restrict__ h) {
    __shared__ float pl[SE_FR][SE_CH + 1];
    __shared__ float wl[SE_SU][SE_CH + 1];
    const int t = threadIdx.x, p = t >> 1, half = t & 1, f = p / SE_SU, u = p % SE_SU;
    const int n0 = blockIdx.x * SE_FR, j0 = blockIdx.y * SE_SU;
    float acc = 0.f;
    for (int c0 = 0; c0 < C; c0 += SE_CH) {
        __syncthreads();
        for (int i = t; i < SE_FR * SE_CH; i += SE_BLOCK) {
            const int ff = i / SE_CH, cc = i - ff * SE_CH, n = n0 + ff, c = c0 + cc;
            float v = 0.f;
            if (n < N && c < C) {
                v = pool_sum[(int64_t)n * C + c] * inv_hw;
                if (blockIdx.y == 0) pool[(int64_t)n * C + c] = v;
            }
            pl[ff][cc] = v;
        }
        for (int i = t; i < SE_SU * SE_CH; i += SE_BLOCK) {
            const int uu = i / SE_CH, cc = i - uu * SE_CH, j = j0 + uu, c = c0 + cc;
            wl[uu][cc] = (j < S && c < C) ? w1[(int64_t)j * C + c] : 0.f;
        }
        __syncthreads();
#pragma unroll 8
        for (int cc = half; cc < SE_CH; cc += 2) acc = fmaf(pl[f][cc], wl[u][cc], acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    const int n = n0 + f, j = j0 + u;
    if (half == 0 && n < N && j < S) h[(int64_t)n * S + j] = acc + b1[j];
}

// thread = output channel c (of this workgroup's SE_BLOCK), SE_FR frames; silu(h) rows in LDS, fc2 [c][j] chunks
// staged transposed-coalesced ([SE_BLOCK][SE_JC + 1])
__global__ __launch_bounds__(SE_BLOCK) void se_fc2_kernel(const float* __restrict__ h, int N, int C, int S,
                                                          const float* __restrict__ w2, const float* __restrict__ b2,
                                                          float* __restrict__ gate) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* hs = sm;                                   // [SE_FR][S]
    float* wl = hs + SE_FR * S;                       // [SE_BLOCK][SE_JC + 1]
    const int t = threadIdx.x, n0 = blockIdx.x * SE_FR, c0 = blockIdx.y * SE_BLOCK, c = c0 + t;
    for (int i = t; i < SE_FR * S; i += SE_BLOCK) {
        const int ff = i / S, j = i - ff * S, n = n0 + ff;
        hs[i] = n < N ? silu(h[(int64_t)n * S + j]) : 0.f;
    }
    float acc[SE_FR];
    const float bv = c < C ? b2[c] : 0.f;
#pragma unroll
    for (int ff = 0; ff < SE_FR; ++ff) acc[ff] = bv;
    for (int jb = 0; jb < S; jb += SE_JC) {
        const int jn = min(SE_JC, S - jb);
        __syncthreads();
        for (int i = t; i < SE_BLOCK * SE_JC; i += SE_BLOCK) {
            const int r = i / SE_JC, q = i - r * SE_JC;
            wl[r * (SE_JC + 1) + q] = (c0 + r < C && q < jn) ? w2[(int64_t)(c0 + r) * S + jb + q] : 0.f;
        }
        __syncthreads();
        for (int q = 0; q < jn; ++q) {
            const float w = wl[t * (SE_JC + 1) + q];
#pragma unroll
            for (int ff = 0; ff < SE_FR; ++ff) acc[ff] = fmaf(w, hs[ff * S + jb + q], acc[ff]);
        }
    }
    if (c < C) {
#pragma unroll
        for (int ff = 0; ff < SE_FR; ++ff)
            if (n0 + ff < N) gate[(int64_t)(n0 + ff) * C + c] = sigmoidf_(acc[ff]);
    }
}

// dsum = sum_hw dA * a2 (se_bn_bwd_reduce row 0):  dz = dsum g (1 - g) (written by unit group 0);
// dh = (dz . fc2) * silu'(h), hs = silu(h) (for se_bwd_wsum)
__global__ __launch_bounds__(SE_BLOCK) void se_bwd_a_kernel(const float* __restrict__ dsum,
                                                            const float* __restrict__ gate,
                                                            const float* __restrict__ h, int N, int C, int S,
                                                            const float* __restrict__ w2, float* __restrict__ dz,
                                                            float* __restrict__ dh, float* __restrict__ hsout) {
    __shared__ float zl[SE_FR][SE_CH + 1];
    __shared__ float wl[SE_SU][SE_CH + 1];
    const int t = threadIdx.x, p = t >> 1, half = t & 1, f = p / SE_SU, u = p % SE_SU;
    const int n0 = blockIdx.x * SE_FR, j0 = blockIdx.y * SE_SU;
    float acc = 0.f;
    for (int c0 = 0; c0 < C; c0 += SE_CH) {
        __syncthreads();
        for (int i = t; i < SE_FR * SE_CH; i += SE_BLOCK) {
            const int ff = i / SE_CH, cc = i - ff * SE_CH, n = n0 + ff, c = c0 + cc;
            float v = 0.f;
            if (n < N && c < C) {
                const int64_t k = (int64_t)n * C + c;
                const float g = gate[k];
                v = dsum[k] * g * (1.f - g);
                if (blockIdx.y == 0) dz[k] = v;
            }
            zl[ff][cc] = v;
        }
        // fc2 [c][j0 .. j0 + SE_SU): consecutive threads walk the 16 units of one row
        for (int i = t; i < SE_SU * SE_CH; i += SE_BLOCK) {
            const int cc = i / SE_SU, uu = i - cc * SE_SU, j = j0 + uu, c = c0 + cc;
            wl[uu][cc] = (j < S && c < C) ? w2[(int64_t)c * S + j] : 0.f;
        }
        __syncthreads();
#pragma unroll 8
        for (int cc = half; cc < SE_CH; cc += 2) acc = fmaf(zl[f][cc], wl[u][cc], acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    const int n = n0 + f, j = j0 + u;
    if (half == 0 && n < N && j < S) {
        const int64_t k = (int64_t)n * S + j;
        const float x = h[k];
        const float sg = sigmoidf_(x);
        dh[k] = acc * (sg * (1.f + x * (1.f - sg)));
        hsout[k] = x * sg;
    }
}

// rb[n][c] = inv_hw * sum_j dh[n][j] fc1[j][c]  (thread = channel: fc1 rows coalesced across threads)
__global__ __launch_bounds__(SE_BLOCK) void se_bwd_b_kernel(const float* __restrict__ dh, float inv_hw, int N, int C,
                                                            int S, const float* __restrict__ w1,
                                                            float* __restrict__ rb) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* dl = sm;                                   // [SE_FR][S]
    const int t = threadIdx.x, n0 = blockIdx.x * SE_FR, c = blockIdx.y * SE_BLOCK + t;
    for (int i = t; i < SE_FR * S; i += SE_BLOCK) {
        const int ff = i / S, j = i - ff * S, n = n0 + ff;
        dl[i] = n < N ? dh[(int64_t)n * S + j] : 0.f;
    }
    __syncthreads();
    if (c >= C) return;
    float r[SE_FR];
#pragma unroll
    for (int ff = 0; ff < SE_FR; ++ff) r[ff] = 0.f;
    for (int j = 0; j < S; ++j) {
        const float w = w1[(int64_t)j * C + c];
#pragma unroll
        for (int ff = 0; ff < SE_FR; ++ff) r[ff] = fmaf(dl[ff * S + j], w, r[ff]);
    }
#pragma unroll
    for (int ff = 0; ff < SE_FR; ++ff)
        if (n0 + ff < N) rb[(int64_t)(n0 + ff) * C + c] = r[ff] * inv_hw;
}

// reductions over the N frames, grid (ceil(C / 64), ceil(S / 16)); thread = (column c, frame group rg of 4):
//   dw2[c][j] = sum_n dz[n][c] hs[n][j]     dw1[j][c] = sum_n dh[n][j] pool[n][c]       (j in this y-chunk)
//   y-chunk 0 also: db2[c] = sum_n dz, and the BN2 sums of se_bwd_bnsum (fp64); x-block 0: db1[j] = sum_n dh
constexpr int WS_J = 16, WS_RG = 4, WS_COLS = 64;
__global__ __launch_bounds__(SE_BLOCK) void se_bwd_wsum_kernel(const float* __restrict__ dz,
                                                               const float* __restrict__ dh,
                                                               const float* __restrict__ hs,
                                                               const float* __restrict__ pool,
                                                               const float* __restrict__ red,
                                                               const float* __restrict__ gate,
                                                               const float* __restrict__ rb, int N, int C, int S,
                                                               double count, float* __restrict__ dw2,
                                                               float* __restrict__ dw1, float* __restrict__ db2,
                                                               float* __restrict__ db1, float* __restrict__ sdz,
                                                               float* __restrict__ sdzx, float* __restrict__ mdz,
                                                               float* __restrict__ mdzx) {
    __shared__ float shf[2][WS_J][WS_RG][WS_COLS];
    __shared__ double shd[3][WS_RG][WS_COLS];
    const int t = threadIdx.x, cl = t % WS_COLS, rg = t / WS_COLS;
    const int c = blockIdx.x * WS_COLS + cl, j0 = blockIdx.y * WS_J;
    const int jn = min(WS_J, S - j0);
    const bool first = blockIdx.y == 0;
    const int64_t NC = (int64_t)N * C;
    float a2[WS_J], a1[WS_J];
#pragma unroll
    for (int q = 0; q < WS_J; ++q) a2[q] = a1[q] = 0.f;
    double bz = 0.0, s0 = 0.0, s1 = 0.0;
    if (c < C) {
        for (int n = rg; n < N; n += WS_RG) {
            const int64_t k = (int64_t)n * C + c;
            const float zv = dz[k], pv = pool[k];
            const float* hr = hs + (int64_t)n * S + j0;
            const float* dr = dh + (int64_t)n * S + j0;
#pragma unroll
            for (int q = 0; q < WS_J; ++q) {
                if (q < jn) {
                    a2[q] = fmaf(zv, hr[q], a2[q]);
                    a1[q] = fmaf(dr[q], pv, a1[q]);
                }
            }
            if (first) {
                const float g = gate[k], r = rb[k];
                bz += (double)zv;
                s0 += (double)(g * red[NC + k] + r * red[2 * NC + k]);
                s1 += (double)(g * red[3 * NC + k] + r * red[4 * NC + k]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < WS_J; ++q) {
        shf[0][q][rg][cl] = a2[q];
        shf[1][q][rg][cl] = a1[q];
    }
    shd[0][rg][cl] = bz;
    shd[1][rg][cl] = s0;
    shd[2][rg][cl] = s1;
    __syncthreads();
    // rg-ordered combine: thread (q = rg .. step 4, column cl)
    if (c < C) {
        for (int q = rg; q < jn; q += WS_RG) {
            float x2 = 0.f, x1 = 0.f;
            for (int r = 0; r < WS_RG; ++r) {
                x2 += shf[0][q][r][cl];
                x1 += shf[1][q][r][cl];
            }
            dw2[(int64_t)c * S + j0 + q] = x2;
            dw1[(int64_t)(j0 + q) * C + c] = x1;
        }
        if (first && rg == 0) {
            double x = 0.0, y = 0.0, z = 0.0;
            for (int r = 0; r < WS_RG; ++r) {
                x += shd[0][r][cl];
                y += shd[1][r][cl];
                z += shd[2][r][cl];
            }
            db2[c] = (float)x;
            sdz[c] = (float)y;
            sdzx[c] = (float)z;
            mdz[c] = (float)(y / count);
            mdzx[c] = (float)(z / count);
        }
    }
    if (blockIdx.x == 0 && t < jn) {
        double x = 0.0;
        for (int n = 0; n < N; ++n) x += (double)dh[(int64_t)n * S + j0 + t];
        db1[j0 + t] = (float)x;
    }
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


int rt1_se_fwd(const float* pool_sum, float inv_hw, int N, int C, int S, const float* w1, const float* b1,
               const float* w2, const float* b2, float* pool, float* h, float* gate, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || S > 1024) return (int)hipErrorInvalidValue;
    const unsigned fg = (unsigned)((N + SE_FR - 1) / SE_FR);
    hipLaunchKernelGGL(se_fc1_kernel, dim3(fg, (S + SE_SU - 1) / SE_SU), dim3(SE_BLOCK), 0, st, pool_sum, inv_hw, N, C,
                       S, w1, b1, pool, h);
    const size_t lds = (size_t)(SE_FR * S + SE_BLOCK * (SE_JC + 1)) * sizeof(float);
    hipLaunchKernelGGL(se_fc2_kernel, dim3(fg, (C + SE_BLOCK - 1) / SE_BLOCK), dim3(SE_BLOCK), lds, st, h, N, C, S, w2,
                       b2, gate);
    return (int)hipGetLastError();
}

int rt1_se_bwd_frame(const float* dsum, const float* gate, const float* h, float inv_hw, int N, int C, int S,
                     const float* w1, const float* w2, float* dz, float* dh, float* hs, float* rb, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || S > 1024) return (int)hipErrorInvalidValue;
    const unsigned fg = (unsigned)((N + SE_FR - 1) / SE_FR);
    hipLaunchKernelGGL(se_bwd_a_kernel, dim3(fg, (S + SE_SU - 1) / SE_SU), dim3(SE_BLOCK), 0, st, dsum, gate, h, N, C,
                       S, w2, dz, dh, hs);
    hipLaunchKernelGGL(se_bwd_b_kernel, dim3(fg, (C + SE_BLOCK - 1) / SE_BLOCK), dim3(SE_BLOCK),
                       (size_t)SE_FR * S * sizeof(float), st, dh, inv_hw, N, C, S, w1, rb);
    return (int)hipGetLastError();
}

int rt1_se_bwd_wsum(const float* dz, const float* dh, const float* hs, const float* pool, const float* red,
                    const float* gate, const float* rb, int N, int C, int S, double count, float* dw2, float* dw1,
                    float* db2, float* db1, float* sdz, float* sdzx, float* mdz, float* mdzx, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || count <= 0) return (int)hipErrorInvalidValue;
    dim3 grid((C + WS_COLS - 1) / WS_COLS, (S + WS_J - 1) / WS_J);
    hipLaunchKernelGGL(se_bwd_wsum_kernel, grid, dim3(SE_BLOCK), 0, st, dz, dh, hs, pool, red, gate, rb, N, C, S,
                       count, dw2, dw1, db2, db1, sdz, sdzx, mdz, mdzx);
    return (int)hipGetLastError();
}

}  // extern "C"
