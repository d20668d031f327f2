// EfficientNet stem: 3x3 stride-2 conv (3 -> COUT) on the raw frames with the
// RT-1 random-shift augmentation and the uint8 -> [0,1] conversion fused into
// the input read (SURVEY K1+K2: the reference pads, fancy-indexes and /255s the
// whole batch before the conv; here no shifted copy is ever materialised).
//
//   p[ci, y, x] = img[ci, y+dy, x+dx] / 255 (uint8) or img[...] (float), 0 outside
//   out[n, ho, wo, co] = sum_{ci,kh,kw} W[co,ci,kh,kw] * p[ci, 2ho-1+kh, 2wo-1+kw]
//
// (dy, dx) are read from DEVICE memory so a captured hipGraph replays with a
// fresh shift each step.  Output is channels-last bf16 plus per-workgroup BN
// partial rows.  Backward needs only dW (frames have no gradient).
#include "common.h"

using namespace rt1;

namespace {

constexpr int BLOCK = 256;

template <typename TIn>
__device__ __forceinline__ float pix(const TIn* __restrict__ img, int64_t base, int y, int x, int H, int W) {
    if (y < 0 || y >= H || x < 0 || x >= W) return 0.f;
    if constexpr (sizeof(TIn) == 1) return (float)img[base + (int64_t)y * W + x] * (1.f / 255.f);
    else return (float)img[base + (int64_t)y * W + x];
}

template <typename TIn>
__device__ __forceinline__ void load_patch(const TIn* __restrict__ img, int n, int ho, int wo, int H, int W,
                                           int dy, int dx, float (&p)[27]) {
    const int y0 = 2 * ho - 1 + dy, x0 = 2 * wo - 1 + dx;
    // the shifted image is zero where (y - dy) or (x - dx) falls outside [0, H) x [0, W)
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
        const int64_t base = ((int64_t)n * 3 + ci) * H * W;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int yy = y0 + kh;          // source row in the unshifted image
            const int ys = yy - dy;          // row in the shifted (output) frame
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int xx = x0 + kw, xs = xx - dx;
                const bool inside = ys >= 0 && ys < H && xs >= 0 && xs < W;
                p[ci * 9 + kh * 3 + kw] = inside ? pix(img, base, yy, xx, H, W) : 0.f;
            }
        }
    }
}

// thread role = output channel vector (8 channels); COUT/8 roles per pixel, pixel lanes stride the pixels
template <typename TIn, int COUT>
__global__ __launch_bounds__(BLOCK) void stem_fwd_kernel(const TIn* __restrict__ img, const int* __restrict__ shift,
                                                         const float* __restrict__ w, int N, int H, int W, int Ho,
                                                         int Wo, bf16_t* __restrict__ out, float* __restrict__ psum,
                                                         float* __restrict__ psq) {
    constexpr int NCV = COUT / 8;
    constexpr int PLN = BLOCK / NCV;
    __shared__ float wl[27 * COUT];
    __shared__ float red[2 * COUT];
    for (int i = threadIdx.x; i < COUT * 27; i += BLOCK) {
        const int co = i / 27, k = i % 27;
        wl[k * COUT + co] = w[i];  // [tap][co]
    }
    for (int i = threadIdx.x; i < 2 * COUT; i += BLOCK) red[i] = 0.f;
    __syncthreads();
    const int cvec = threadIdx.x % NCV, pl = threadIdx.x / NCV;
    const int dy = shift ? shift[0] : 0, dx = shift ? shift[1] : 0;
    float s[8], q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
    if (pl < PLN) {
        const int64_t total = (int64_t)N * Ho * Wo;
        for (int64_t i = (int64_t)blockIdx.x * PLN + pl; i < total; i += (int64_t)gridDim.x * PLN) {
            const int n = (int)(i / ((int64_t)Ho * Wo));
            const int r = (int)(i - (int64_t)n * Ho * Wo);
            const int ho = r / Wo, wo = r % Wo;
            float p[27];
            load_patch(img, n, ho, wo, H, W, dy, dx, p);
            float acc[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = 0.f;
            // opaque per-iteration offset: keeps the 27x8 weights in LDS instead of 216 hoisted VGPRs
            int wofs = cvec * 8;
            asm volatile("" : "+v"(wofs));
#pragma unroll
            for (int k = 0; k < 27; ++k) {
                float wv[8];
                load8f(wl + k * COUT + wofs, wv);
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = fmaf(p[k], wv[j], acc[j]);
            }
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                f[j] = bf2f(f2bf(acc[j]));
                s[j] += f[j];
                q[j] = fmaf(f[j], f[j], q[j]);
            }
            store8(out + i * COUT + cvec * 8, f);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            atomicAdd(&red[cvec * 8 + j], s[j]);
            atomicAdd(&red[COUT + cvec * 8 + j], q[j]);
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < COUT; c += BLOCK) {
        psum[(int64_t)blockIdx.x * COUT + c] = red[c];
        psq[(int64_t)blockIdx.x * COUT + c] = red[COUT + c];
    }
}

// dW partials: thread role = (output channel vector cvec, input channel ci); pixel lanes stride the pixels.
template <typename TIn, int COUT>
__global__ __launch_bounds__(BLOCK) void stem_bwd_weight_kernel(const TIn* __restrict__ img,
                                                                const int* __restrict__ shift,
                                                                const bf16_t* __restrict__ dyv, int N, int H, int W,
                                                                int Ho, int Wo, float* __restrict__ dwp) {
    constexpr int NCV = COUT / 8;
    constexpr int ROLES = NCV * 3;
    constexpr int PLN = BLOCK / ROLES;
    __shared__ float red[COUT * 27];
    for (int i = threadIdx.x; i < COUT * 27; i += BLOCK) red[i] = 0.f;
    __syncthreads();
    const int role = threadIdx.x % ROLES, pl = threadIdx.x / ROLES;
    const int cvec = role / 3, ci = role % 3;
    const int dy = shift ? shift[0] : 0, dx = shift ? shift[1] : 0;
    float acc[8][9];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[j][k] = 0.f;
    if (pl < PLN) {
        const int64_t total = (int64_t)N * Ho * Wo;
        for (int64_t i = (int64_t)blockIdx.x * PLN + pl; i < total; i += (int64_t)gridDim.x * PLN) {
            const int n = (int)(i / ((int64_t)Ho * Wo));
            const int r = (int)(i - (int64_t)n * Ho * Wo);
            const int ho = r / Wo, wo = r % Wo;
            float g[8];
            load8(dyv + i * COUT + cvec * 8, g);
            const int64_t base = ((int64_t)n * 3 + ci) * H * W;
            const int y0 = 2 * ho - 1 + dy, x0 = 2 * wo - 1 + dx;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const int yy = y0 + kh, xx = x0 + kw;
                    const int ys = yy - dy, xs = xx - dx;
                    const float v = (ys >= 0 && ys < H && xs >= 0 && xs < W) ? pix(img, base, yy, xx, H, W) : 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[j][kh * 3 + kw] = fmaf(g[j], v, acc[j][kh * 3 + kw]);
                }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int k = 0; k < 9; ++k) atomicAdd(&red[(cvec * 8 + j) * 27 + ci * 9 + k], acc[j][k]);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < COUT * 27; i += BLOCK) dwp[(int64_t)blockIdx.x * COUT * 27 + i] = red[i];
}

}  // namespace

extern "C" {

int rt1_stem_fwd(const void* img, int img_is_u8, const int* shift, const float* w, int N, int H, int W, int Cout,
                 int grid, bf16_t* out, float* psum, float* psq, hipStream_t st) {
    if (Cout != 40) return (int)hipErrorInvalidValue;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    if (img_is_u8)
        hipLaunchKernelGGL((stem_fwd_kernel<uint8_t, 40>), dim3(grid), dim3(BLOCK), 0, st, (const uint8_t*)img, shift, w,
                           N, H, W, Ho, Wo, out, psum, psq);
    else
        hipLaunchKernelGGL((stem_fwd_kernel<float, 40>), dim3(grid), dim3(BLOCK), 0, st, (const float*)img, shift, w, N,
                           H, W, Ho, Wo, out, psum, psq);
    return (int)hipGetLastError();
}

int rt1_stem_bwd_weight(const void* img, int img_is_u8, const int* shift, const bf16_t* dy, int N, int H, int W,
                        int Cout, int grid, float* dwp, hipStream_t st) {
    if (Cout != 40) return (int)hipErrorInvalidValue;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    if (img_is_u8)
        hipLaunchKernelGGL((stem_bwd_weight_kernel<uint8_t, 40>), dim3(grid), dim3(BLOCK), 0, st, (const uint8_t*)img,
                           shift, dy, N, H, W, Ho, Wo, dwp);
    else
        hipLaunchKernelGGL((stem_bwd_weight_kernel<float, 40>), dim3(grid), dim3(BLOCK), 0, st, (const float*)img, shift,
                           dy, N, H, W, Ho, Wo, dwp);
    return (int)hipGetLastError();
}

}  // extern "C"
