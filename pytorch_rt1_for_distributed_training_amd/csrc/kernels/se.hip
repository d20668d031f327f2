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

// a workgroup = 64 columns x 16 row groups (1024 threads): each thread walks every 16th frame of its column,
// the 16 partial sums of a column are then added in row-group order through LDS (deterministic)
constexpr int COLS = 64, RG = 16, BLOCK = COLS * RG;

template <int NACC>
__device__ __forceinline__ void column_reduce(double (&acc)[NACC], double (*sh)[RG][COLS]) {
    const int cl = threadIdx.x % COLS, rg = threadIdx.x / COLS;
#pragma unroll
    for (int a = 0; a < NACC; ++a) sh[a][rg][cl] = acc[a];
    __syncthreads();
    if (rg == 0) {
#pragma unroll
        for (int a = 0; a < NACC; ++a) {
            double t = 0.0;
            for (int r = 0; r < RG; ++r) t += sh[a][r][cl];
            acc[a] = t;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void se_bwd_dz_kernel(const float* __restrict__ dsum, const float* __restrict__ gate,
                                                          int N, int C, float* __restrict__ dz,
                                                          float* __restrict__ db) {
    __shared__ double sh[1][RG][COLS];
    const int c = blockIdx.x * COLS + threadIdx.x % COLS, rg = threadIdx.x / COLS;
    double acc[1] = {0.0};
    if (c < C) {
#pragma unroll 4
        for (int n = rg; n < N; n += RG) {
            const int64_t i = (int64_t)n * C + c;
            const float g = gate[i];
            const float d = dsum[i] * g * (1.f - g);
            dz[i] = d;
            acc[0] += (double)d;
        }
    }
    column_reduce(acc, sh);
    if (rg == 0 && c < C) db[c] = (float)acc[0];
}

__global__ __launch_bounds__(BLOCK) void se_bwd_dh_kernel(const float* __restrict__ dzf2, const float* __restrict__ h,
                                                          int N, int S, float* __restrict__ dh,
                                                          float* __restrict__ db) {
    __shared__ double sh[1][RG][COLS];
    const int s = blockIdx.x * COLS + threadIdx.x % COLS, rg = threadIdx.x / COLS;
    double acc[1] = {0.0};
    if (s < S) {
#pragma unroll 4
        for (int n = rg; n < N; n += RG) {
            const int64_t i = (int64_t)n * S + s;
            const float x = h[i];
            const float sg = 1.f / (1.f + __expf(-x));
            const float d = dzf2[i] * (sg * (1.f + x * (1.f - sg)));
            dh[i] = d;
            acc[0] += (double)d;
        }
    }
    column_reduce(acc, sh);
    if (rg == 0 && s < S) db[s] = (float)acc[0];
}

// red: [5, N, C] (S0 unused here), gate [N, C], rbraw [N, C] -> rb [N, C], sdz / sdzx / mdz / mdzx [C]
__global__ __launch_bounds__(BLOCK) void se_bwd_bnsum_kernel(const float* __restrict__ red,
                                                             const float* __restrict__ gate,
                                                             const float* __restrict__ rbraw, float inv_hw, int N,
                                                             int C, double count, float* __restrict__ rb,
                                                             float* __restrict__ sdz, float* __restrict__ sdzx,
                                                             float* __restrict__ mdz, float* __restrict__ mdzx) {
    __shared__ double sh[2][RG][COLS];
    const int c = blockIdx.x * COLS + threadIdx.x % COLS, rg = threadIdx.x / COLS;
    const int64_t NC = (int64_t)N * C;
    double acc[2] = {0.0, 0.0};
    if (c < C) {
#pragma unroll 4
        for (int n = rg; n < N; n += RG) {
            const int64_t i = (int64_t)n * C + c;
            const float g = gate[i];
            const float r = rbraw[i] * inv_hw;
            rb[i] = r;
            acc[0] += (double)(g * red[NC + i] + r * red[2 * NC + i]);
            acc[1] += (double)(g * red[3 * NC + i] + r * red[4 * NC + i]);
        }
    }
    column_reduce(acc, sh);
    if (rg == 0 && c < C) {
        sdz[c] = (float)acc[0];
        sdzx[c] = (float)acc[1];
        mdz[c] = (float)(acc[0] / count);
        mdzx[c] = (float)(acc[1] / count);
    }
}

}  // namespace

extern "C" {

int rt1_se_bwd_dz(const float* dsum, const float* gate, int N, int C, float* dz, float* db, hipStream_t st) {
    if (N <= 0 || C <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(se_bwd_dz_kernel, dim3((C + COLS - 1) / COLS), dim3(BLOCK), 0, st, dsum, gate, N, C, dz, db);
    return (int)hipGetLastError();
}

int rt1_se_bwd_dh(const float* dzf2, const float* h, int N, int S, float* dh, float* db, hipStream_t st) {
    if (N <= 0 || S <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(se_bwd_dh_kernel, dim3((S + COLS - 1) / COLS), dim3(BLOCK), 0, st, dzf2, h, N, S, dh, db);
    return (int)hipGetLastError();
}

int rt1_se_bwd_bnsum(const float* red, const float* gate, const float* rbraw, float inv_hw, int N, int C, double count,
                     float* rb, float* sdz, float* sdzx, float* mdz, float* mdzx, hipStream_t st) {
    if (N <= 0 || C <= 0 || count <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(se_bwd_bnsum_kernel, dim3((C + COLS - 1) / COLS), dim3(BLOCK), 0, st, red, gate, rbraw, inv_hw,
                       N, C, count, rb, sdz, sdzx, mdz, mdzx);
    return (int)hipGetLastError();
}

}  // extern "C"
