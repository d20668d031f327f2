// BatchNorm statistics of an expand conv's output computed from its INPUT (the y1-free expand blocks, "x-mode").
//
// For y1 = x @ We^T (x [M, Cin], We [Ce, Cin]) the batch statistics of output channel c are linear / quadratic
// forms of the first two moments of x:
//     sum_m y1[m, c]    = w_c . sx            sx = sum_m x[m, :]            (Cin)
//     sum_m y1[m, c]^2  = w_c^T G w_c         G  = x^T x                    (Cin x Cin)
// so BN1 (film_efficientnet_encoder.py:185-195, train mode) never needs y1 itself: the depthwise kernels recompute
// it per tile on MFMA (dwconv.hip stage_xmfma) and this kernel turns (G, sx) into BN1's constants with the same
// finalisation as bn_finalize (bn.hip): biased variance for the normalisation, the unbiased one for the running
// estimate, momentum update in place.  Everything after G is fp64: the quadratic form subtracts mean^2 from E[y^2].
//
// One wave per output channel: lanes stride over the Cin^2 terms, fixed-order wave reduction (deterministic).
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BLOCK = 256;
constexpr int XG_ROWS = 128;          // rows per staged chunk: one 32-row MFMA k-step per wave

__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* base0, const bf16_t* base1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// Partial moments of x [M, Cin] (Cin <= 16 * NT, Cin % 8 == 0) over a contiguous row range per workgroup:
//     part[b][i * Cin + j] = sum_m x[m, i] x[m, j]      part[b][Cin^2 + j] = sum_m x[m, j]
// 128-row chunks are staged row-major into LDS (the next chunk's 16-B loads in flight during the MFMAs); each wave
// reads its 32 rows k-major with ds_read_b64_tr_b16 as both MFMA operands (G = x^T x) and against a ones fragment
// (the column sums).  fp32 per workgroup, reduced in fp64 by gram_reduce_kernel.  One pass over x at HBM rate: the
// MFMA work is NT^2 + NT instructions per 32 rows per wave.
template <int NT>
__global__ __launch_bounds__(BLOCK) void xgram_kernel(const bf16_t* __restrict__ x, int64_t M, int cin,
                                                      int64_t rows_per_wg, float* __restrict__ part) {
    constexpr int CP = NT * 16, LDX = CP + 8;
    constexpr int NV = (XG_ROWS * CP / 8 + BLOCK - 1) / BLOCK;   // 16-B vectors per thread per chunk (upper bound)
    __shared__ __attribute__((aligned(16))) bf16_t xl[XG_ROWS * LDX];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int lr = lane & 15, lh = lane >> 4;
    const int av = cin / 8;                                     // 16-B vectors per row
    const int64_t m_begin = (int64_t)blockIdx.x * rows_per_wg;
    const int64_t m_end = m_begin + rows_per_wg < M ? m_begin + rows_per_wg : M;
    // the padding columns [cin, CP) stay zero for the whole kernel
    for (int i = t; i < XG_ROWS * (LDX - cin) ; i += BLOCK) {
        const int r = i / (LDX - cin), c = cin + i % (LDX - cin);
        xl[r * LDX + c] = 0;
    }
    f32x4 acc[NT][NT], accs[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        accs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const short one = 0x3f80;                                   // bf16 1.0
    const bf16x8 ones = bf16x8{one, one, one, one, one, one, one, one};
    uint4 rv[NV];
    auto issue = [&](int64_t m0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int v = t + k * BLOCK, r = v / av;
            rv[k] = make_uint4(0, 0, 0, 0);
            if (r < XG_ROWS && m0 + r < m_end)
                rv[k] = *reinterpret_cast<const uint4*>(x + (m0 + r) * cin + (v - r * av) * 8);
        }
    };
    if (m_begin < m_end) issue(m_begin);
    for (int64_t m0 = m_begin; m0 < m_end; m0 += XG_ROWS) {
        __syncthreads();                                        // previous chunk's reads are done
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int v = t + k * BLOCK, r = v / av;
            if (r < XG_ROWS) *reinterpret_cast<uint4*>(xl + r * LDX + (v - r * av) * 8) = rv[k];
        }
        __syncthreads();
        if (m0 + XG_ROWS < m_end) issue(m0 + XG_ROWS);
        const int q = lr >> 2, p = lr & 3;
        const int r0 = wave * 32 + lh * 8 + q;
        bf16x8 f[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) f[j] = tr_read8(xl + r0 * LDX + j * 16 + p * 4, xl + (r0 + 4) * LDX + j * 16 + p * 4);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[i], f[j], acc[i][j], 0, 0, 0);
            accs[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, f[i], accs[i], 0, 0, 0);
        }
    }
    // fixed-order sum of the 4 waves through LDS (wave 0 writes, waves 1-3 add in turn), then the partial row
    __syncthreads();
    float* red = reinterpret_cast<float*>(xl);                  // [CP * CP + CP]
    constexpr int L = CP * CP + CP;
    static_assert(L * 4 <= XG_ROWS * LDX * 2, "reduction scratch fits the chunk buffer");
    for (int w = 0; w < 4; ++w) {
        if (wave == w) {
#pragma unroll
            for (int i = 0; i < NT; ++i) {
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float* r = red + (i * 16 + lh * 4 + e) * CP + j * 16 + lr;
                        *r = w == 0 ? acc[i][j][e] : *r + acc[i][j][e];
                    }
                if (lh == 0) {
                    float* r = red + CP * CP + i * 16 + lr;
                    *r = w == 0 ? accs[i][0] : *r + accs[i][0];
                }
            }
        }
        __syncthreads();
    }
    float* o = part + (int64_t)blockIdx.x * (cin * cin + cin);
    for (int i = t; i < cin * cin + cin; i += BLOCK)
        o[i] = red[i < cin * cin ? (i / cin) * CP + i % cin : CP * CP + (i - cin * cin)];
}

// out[c] = sum_b part[b][c] in fp64, fixed order (deterministic): 64 columns x 4 row groups per workgroup, 8 loads in
// flight per thread, the 4 group sums combined in order through LDS
__global__ __launch_bounds__(BLOCK) void gram_reduce_kernel(const float* __restrict__ part, int P, int L,
                                                            double* __restrict__ out) {
    __shared__ double red[4][64];
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s = 0.0;
    if (c < L) {
        int b = rg;
        for (; b + 28 < P; b += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(b + 4 * u) * L + c];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
        for (; b < P; b += 4) s += (double)part[(int64_t)b * L + c];
    }
    red[rg][cl] = s;
    __syncthreads();
    if (rg == 0 && c < L) out[c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void bn_from_gram_kernel(const double* __restrict__ G, const double* __restrict__ sx,
                                                           const bf16_t* __restrict__ we, int cin, int C, double count,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps, float momentum,
                                                           float* __restrict__ running_mean,
                                                           float* __restrict__ running_var, float* __restrict__ scale,
                                                           float* __restrict__ shift, float* __restrict__ save_mean,
                                                           float* __restrict__ save_rstd) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= C) return;
    const bf16_t* wc = we + (int64_t)c * cin;
    double s1 = 0.0, s2 = 0.0;
    for (int i = lane; i < cin * cin; i += 64) {
        const int a = i / cin, b = i - a * cin;
        s2 += (double)bf2f(wc[a]) * (double)bf2f(wc[b]) * G[i];
    }
    for (int a = lane; a < cin; a += 64) s1 += (double)bf2f(wc[a]) * sx[a];
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if (lane != 0) return;
    const double mean = s1 / count;
    double var = s2 / count - mean * mean;
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

// The same constants from WG = we @ G (fp32 [C, cin], one library GEMM) and sx: E[y_c^2] = WG[c] . w_c / M,
// mean_c = w_c . sx / M, per channel one wave of coalesced row reads with fp64 sums.  For the wide expand convs
// (cin 96-232), where a per-channel quadratic form over G (cin^2 reads per channel) took 140 us per layer.
__global__ __launch_bounds__(256) void bn_from_wg_kernel(const float* __restrict__ WG, const float* __restrict__ sx,
                                                         const bf16_t* __restrict__ we, int cin, int C, double count,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps, float momentum,
                                                         float* __restrict__ running_mean,
                                                         float* __restrict__ running_var, float* __restrict__ scale,
                                                         float* __restrict__ shift, float* __restrict__ save_mean,
                                                         float* __restrict__ save_rstd) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= C) return;
    const bf16_t* wc = we + (int64_t)c * cin;
    const float* tc = WG + (int64_t)c * cin;
    double s1 = 0.0, s2 = 0.0;
    for (int a = lane; a < cin; a += 64) {
        const double w = (double)bf2f(wc[a]);
        s2 += w * (double)tc[a];
        s1 += w * (double)sx[a];
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if (lane != 0) return;
    const double mean = s1 / count;
    double var = s2 / count - mean * mean;
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

}  // namespace

// Gram moments of x [M, cin] in fp64: work = [grid][cin^2 + cin] fp32 partials (grid from rt1_xgram_grid), out =
// [cin^2 + cin] fp64 (G row-major, then sum x)
extern "C" int rt1_xgram_grid(int64_t M, int cin) {
    (void)cin;
    const int64_t g = (M + 8 * XG_ROWS - 1) / (8 * XG_ROWS);      // >= 8 chunks per workgroup
    return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

extern "C" int rt1_xgram(const bf16_t* x, int64_t M, int cin, int grid, float* work, double* out, hipStream_t st) {
    if (M <= 0 || cin <= 0 || cin % 8 || cin > 64 || grid < 1) return (int)hipErrorInvalidValue;
    const int64_t rows = ((M + grid - 1) / grid + XG_ROWS - 1) / XG_ROWS * XG_ROWS;
    if (cin <= 32) hipLaunchKernelGGL((xgram_kernel<2>), dim3(grid), dim3(BLOCK), 0, st, x, M, cin, rows, work);
    else if (cin <= 48) hipLaunchKernelGGL((xgram_kernel<3>), dim3(grid), dim3(BLOCK), 0, st, x, M, cin, rows, work);
    else hipLaunchKernelGGL((xgram_kernel<4>), dim3(grid), dim3(BLOCK), 0, st, x, M, cin, rows, work);
    const int L = cin * cin + cin;
    hipLaunchKernelGGL(gram_reduce_kernel, dim3((L + 63) / 64), dim3(BLOCK), 0, st, work, grid, L, out);
    return (int)hipGetLastError();
}

// G: [cin, cin] fp64, sx: [cin] fp64 (rt1_xgram's out)
extern "C" int rt1_bn_from_gram(const double* G, const double* sx, const bf16_t* we, int cin, int C, double count,
                                const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                                float* running_var, float* scale, float* shift, float* save_mean, float* save_rstd,
                                hipStream_t st) {
    if (cin <= 0 || C <= 0 || count <= 0.0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_from_gram_kernel, dim3((C + 3) / 4), dim3(256), 0, st, G, sx, we, cin, C, count, gamma, beta,
                       eps, momentum, running_mean, running_var, scale, shift, save_mean, save_rstd);
    return (int)hipGetLastError();
}

// WG = we @ G [C, cin] fp32 and sx [cin] fp32 (G = wgrad(x, x), sx = colsum(x) of the dz-mode expand backward)
extern "C" int rt1_bn_from_wg(const float* WG, const float* sx, const bf16_t* we, int cin, int C, double count,
                              const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                              float* running_var, float* scale, float* shift, float* save_mean, float* save_rstd,
                              hipStream_t st) {
    if (cin <= 0 || C <= 0 || count <= 0.0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_from_wg_kernel, dim3((C + 3) / 4), dim3(256), 0, st, WG, sx, we, cin, C, count, gamma, beta,
                       eps, momentum, running_mean, running_var, scale, shift, save_mean, save_rstd);
    return (int)hipGetLastError();
}
