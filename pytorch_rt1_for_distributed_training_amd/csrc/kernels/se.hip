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


// ---------------------------------------------------------------- whole SE MLP in two / three kernels
// The squeeze-excitation MLP of every MBConv block is [N, C] x [C, S] x [S, C] with N = 768 frames, C <= 2304,
// S <= 96: ~0.7 GFLOP at the widest block, but as torch ops it was 6 forward and 8 backward launches of
// few-microsecond kernels (hipBLASLt GEMMs on 16x16 .. 32x32 macro tiles, silu / sigmoid / divide maps) per block,
// ~340 launches per step.  Here: se_fwd (pool mean -> fc1 -> SiLU -> fc2 -> sigmoid), se_bwd_frame (the per-frame
// chain dz -> dh -> rb) and se_bwd_wsum (the reductions over frames: fc weight / bias gradients and the BN2 sums),
// all in fp32 FMAs with fixed summation orders (bit-reproducible), weights read in their parameter layouts
// (fc1 [S, C], fc2 [C, S]).
constexpr int SE_FR = 8;       // frames per workgroup (per-frame kernels)
constexpr int SE_BLOCK = 256;
constexpr int SE_CCH = 64;     // fc2 rows staged per LDS chunk

// stage fc2 rows [c0, c0 + SE_CCH) x S into LDS with row stride S + 1 (odd: the per-lane row reads are conflict-free)
__device__ __forceinline__ void stage_fc2(float* w2l, const float* __restrict__ w2, int c0, int C, int S) {
    const int n = min(SE_CCH, C - c0) * S;
    for (int i = threadIdx.x; i < n; i += SE_BLOCK) {
        const int r = i / S, j = i - r * S;
        w2l[r * (S + 1) + j] = w2[(int64_t)c0 * S + i];
    }
}

// pool_sum [N, C] (sum over the frame's pixels) -> pool [N, C] (mean), h [N, S] (fc1 pre-activation), gate [N, C]
__global__ __launch_bounds__(SE_BLOCK) void se_fwd_kernel(const float* __restrict__ pool_sum, float inv_hw, int N,
                                                          int C, int S, const float* __restrict__ w1,
                                                          const float* __restrict__ b1, const float* __restrict__ w2,
                                                          const float* __restrict__ b2, float* __restrict__ pool,
                                                          float* __restrict__ h, float* __restrict__ gate) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* pl = sm;                               // [SE_FR][C]
    float* hs = pl + SE_FR * C;                   // [SE_FR][S]
    float* w2l = hs + SE_FR * S;                  // [SE_CCH][S + 1]
    const int n0 = blockIdx.x * SE_FR, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    for (int i = t; i < SE_FR * C; i += SE_BLOCK) {
        const int f = i / C, c = i - f * C, n = n0 + f;
        float v = 0.f;
        if (n < N) {
            v = pool_sum[(int64_t)n * C + c] * inv_hw;
            pool[(int64_t)n * C + c] = v;
        }
        pl[i] = v;
    }
    __syncthreads();
    // fc1: one wave per output unit j, lanes over the C inputs (w1 row j read coalesced), SE_FR frames at once
    for (int j = wave; j < S; j += SE_BLOCK / 64) {
        float acc[SE_FR];
#pragma unroll
        for (int f = 0; f < SE_FR; ++f) acc[f] = 0.f;
        for (int c = lane; c < C; c += 64) {
            const float w = w1[(int64_t)j * C + c];
#pragma unroll
            for (int f = 0; f < SE_FR; ++f) acc[f] = fmaf(w, pl[f * C + c], acc[f]);
        }
#pragma unroll
        for (int f = 0; f < SE_FR; ++f) {
            const float v = wave_sum(acc[f]) + b1[j];
            if (lane == 0) {
                hs[f * S + j] = silu(v);
                if (n0 + f < N) h[(int64_t)(n0 + f) * S + j] = v;
            }
        }
    }
    // fc2 + sigmoid: chunks of SE_CCH output channels staged in LDS; thread = (channel, frame group of 2)
    const int cl = t % SE_CCH, fg = t / SE_CCH;   // 4 frame groups x 2 frames
    for (int c0 = 0; c0 < C; c0 += SE_CCH) {
        __syncthreads();
        stage_fc2(w2l, w2, c0, C, S);
        __syncthreads();
        const int c = c0 + cl;
        if (c >= C) continue;
        float a0 = b2[c], a1 = a0;
        const float* wr = w2l + cl * (S + 1);
        const float *h0 = hs + (2 * fg) * S, *h1 = h0 + S;
        for (int j = 0; j < S; ++j) {
            const float w = wr[j];
            a0 = fmaf(w, h0[j], a0);
            a1 = fmaf(w, h1[j], a1);
        }
        const int na = n0 + 2 * fg;
        if (na < N) gate[(int64_t)na * C + c] = sigmoidf_(a0);
        if (na + 1 < N) gate[(int64_t)(na + 1) * C + c] = sigmoidf_(a1);
    }
}

// per-frame backward chain.  dsum = sum_hw dA * a2 (se_bn_bwd_reduce row 0):
//   dz = dsum * g (1 - g) ;  dh = (dz . fc2) * silu'(h) ;  rb = (dh . fc1) / HW ;  hs = silu(h) (for se_bwd_wsum)
__global__ __launch_bounds__(SE_BLOCK) void se_bwd_frame_kernel(const float* __restrict__ dsum,
                                                                const float* __restrict__ gate,
                                                                const float* __restrict__ h, float inv_hw, int N,
                                                                int C, int S, const float* __restrict__ w1,
                                                                const float* __restrict__ w2, float* __restrict__ dz,
                                                                float* __restrict__ dh, float* __restrict__ hsout,
                                                                float* __restrict__ rb) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* dzl = sm;                              // [SE_FR][C]
    float* dhl = dzl + SE_FR * C;                 // [SE_FR][S]
    float* w2l = dhl + SE_FR * S;                 // [SE_CCH][S + 1]
    const int n0 = blockIdx.x * SE_FR, t = threadIdx.x;
    for (int i = t; i < SE_FR * C; i += SE_BLOCK) {
        const int f = i / C, c = i - f * C, n = n0 + f;
        float v = 0.f;
        if (n < N) {
            const int64_t k = (int64_t)n * C + c;
            const float g = gate[k];
            v = dsum[k] * g * (1.f - g);
            dz[k] = v;
        }
        dzl[i] = v;
    }
    // dhs[f][j] = sum_c dz[f][c] fc2[c][j]: thread = (unit j, frame) pairs, fc2 rows through LDS in chunks
    constexpr int MAXP = 4;                        // (j, f) pairs per thread: S * SE_FR <= 4 * 256
    float acc[MAXP];
#pragma unroll
    for (int q = 0; q < MAXP; ++q) acc[q] = 0.f;
    for (int c0 = 0; c0 < C; c0 += SE_CCH) {
        __syncthreads();
        stage_fc2(w2l, w2, c0, C, S);
        __syncthreads();
        const int cn = min(SE_CCH, C - c0);
#pragma unroll
        for (int q = 0; q < MAXP; ++q) {
            const int p = t + q * SE_BLOCK, j = p % S, f = p / S;
            if (f >= SE_FR) continue;
            float a = acc[q];
            const float* dzr = dzl + f * C + c0;
            for (int cc = 0; cc < cn; ++cc) a = fmaf(dzr[cc], w2l[cc * (S + 1) + j], a);
            acc[q] = a;
        }
    }
#pragma unroll
    for (int q = 0; q < MAXP; ++q) {
        const int p = t + q * SE_BLOCK, j = p % S, f = p / S, n = n0 + f;
        if (f >= SE_FR) continue;
        float d = 0.f;
        if (n < N) {
            const float x = h[(int64_t)n * S + j];
            const float sg = sigmoidf_(x);
            d = acc[q] * (sg * (1.f + x * (1.f - sg)));
            dh[(int64_t)n * S + j] = d;
            hsout[(int64_t)n * S + j] = x * sg;
        }
        dhl[f * S + j] = d;
    }
    __syncthreads();
    // rb[f][c] = inv_hw * sum_j dh[f][j] fc1[j][c]  (fc1 columns coalesced across threads)
    for (int c = t; c < C; c += SE_BLOCK) {
        float r[SE_FR];
#pragma unroll
        for (int f = 0; f < SE_FR; ++f) r[f] = 0.f;
        for (int j = 0; j < S; ++j) {
            const float w = w1[(int64_t)j * C + c];
#pragma unroll
            for (int f = 0; f < SE_FR; ++f) r[f] = fmaf(dhl[f * S + j], w, r[f]);
        }
#pragma unroll
        for (int f = 0; f < SE_FR; ++f)
            if (n0 + f < N) rb[(int64_t)(n0 + f) * C + c] = r[f] * inv_hw;
    }
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


size_t se_lds(int C, int S) { return (size_t)(SE_FR * C + SE_FR * S + SE_CCH * (S + 1)) * sizeof(float); }

int rt1_se_fwd(const float* pool_sum, float inv_hw, int N, int C, int S, const float* w1, const float* b1,
               const float* w2, const float* b2, float* pool, float* h, float* gate, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || se_lds(C, S) > 160 * 1024) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(se_fwd_kernel, dim3((N + SE_FR - 1) / SE_FR), dim3(SE_BLOCK), se_lds(C, S), st, pool_sum,
                       inv_hw, N, C, S, w1, b1, w2, b2, pool, h, gate);
    return (int)hipGetLastError();
}

int rt1_se_bwd_frame(const float* dsum, const float* gate, const float* h, float inv_hw, int N, int C, int S,
                     const float* w1, const float* w2, float* dz, float* dh, float* hs, float* rb, hipStream_t st) {
    if (N <= 0 || C <= 0 || S <= 0 || S * SE_FR > 4 * SE_BLOCK || se_lds(C, S) > 160 * 1024)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(se_bwd_frame_kernel, dim3((N + SE_FR - 1) / SE_FR), dim3(SE_BLOCK), se_lds(C, S), st, dsum,
                       gate, h, inv_hw, N, C, S, w1, w2, dz, dh, hs, rb);
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
