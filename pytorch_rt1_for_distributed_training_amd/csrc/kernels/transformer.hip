// Elementwise / normalisation kernels of the RT-1 decoder layer (SURVEY K12 LayerNorm, K15/K16 residual,
// dropout), E = 512 channels: one wave per token row, 8 channels (16 B bf16 / 32 B fp32) per lane.
// The residual stream stays fp32; GEMM operands are bf16.
//
//   ln_fwd          y = (x - mu) * rstd * g + b            x fp32 -> y bf16, saves mu / rstd
//   ln_bwd          dx = dres + rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat));  dg, db partials
//   resid_add       out = x + a + bias                      (attention out-projection residual)
//   drop_resid_add  out = x + dropout(h + bias)             (FF residual; counter-hash mask)
//                   both optionally followed by the NEXT LayerNorm of out on the same row (xn bf16, mu, rstd): the
//                   residual rows are never re-read by a separate ln_fwd (LN2 after the out-projection, the next
//                   layer's LN1 after the FF)
//   ln_bwd          optionally also stores bf16(dx) with its column sums (the next GEMM's operand and bias gradient:
//                   no drop_bwd pass for the out-projection)
//   drop_bwd        dh = dout * keep / (1 - p)              (same hash -> same mask), bf16
#include "common.h"

using namespace rt1;

namespace {

constexpr int E = 512;
constexpr int ROWS_PER_BLOCK = 4;   // 4 waves

__device__ __forceinline__ uint32_t mix32(uint32_t seed, uint32_t a, uint32_t b) {
    uint32_t x = seed ^ (a * 0x9E3779B1u) ^ (b * 0x85EBCA77u) ^ 0x27d4eb2fu;
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ bool dropped(uint32_t seed, int row, int col, float p) {
    return (float)(mix32(seed, (uint32_t)row, (uint32_t)col) >> 8) * (1.0f / 16777216.0f) < p;
}

__device__ __forceinline__ void load8x(const float* __restrict__ p, float (&o)[8]) { load8f(p, o); }
__device__ __forceinline__ void store8f(float* __restrict__ p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                     const float* __restrict__ b, int T, float eps,
                                                     bf16_t* __restrict__ y, float* __restrict__ mu,
                                                     float* __restrict__ rs) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= T) return;
    const int c0 = lane * 8;
    float v[8], gg[8], bb[8];
    load8x(x + (int64_t)row * E + c0, v);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    const float m = wave_sum(s) * (1.f / E);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        v[j] -= m;
        q = fmaf(v[j], v[j], q);
    }
    const float r = rsqrtf(wave_sum(q) * (1.f / E) + eps);
    load8f(g + c0, gg);
    load8f(b + c0, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j] * r, gg[j], bb[j]);
    store8(y + (int64_t)row * E + c0, v);
    if (lane == 0) {
        mu[row] = m;
        rs[row] = r;
    }
}

// dg/db: per-block partial rows [gridDim.x][E] (summed on the host side)
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ mu, const float* __restrict__ rs,
                                                     const float* __restrict__ g, const float* __restrict__ dres,
                                                     int T, float* __restrict__ dx, float* __restrict__ dgp,
                                                     float* __restrict__ dbp, bf16_t* __restrict__ dxb,
                                                     float* __restrict__ dsp) {
    __shared__ float red[ROWS_PER_BLOCK][3][E];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = lane * 8;
    float gg[8], ag[8], ab[8], as[8];
    load8f(g + c0, gg);
#pragma unroll
    for (int j = 0; j < 8; ++j) ag[j] = ab[j] = as[j] = 0.f;
    for (int row = blockIdx.x * ROWS_PER_BLOCK + w; row < T; row += gridDim.x * ROWS_PER_BLOCK) {
        float d[8], xv[8];
        load8(dy + (int64_t)row * E + c0, d);
        load8x(x + (int64_t)row * E + c0, xv);
        const float m = mu[row], r = rs[row];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            xv[j] = (xv[j] - m) * r;           // xhat
            ag[j] = fmaf(d[j], xv[j], ag[j]);
            ab[j] += d[j];
            const float gd = d[j] * gg[j];
            s1 += gd;
            s2 = fmaf(gd, xv[j], s2);
        }
        s1 = wave_sum(s1) * (1.f / E);
        s2 = wave_sum(s2) * (1.f / E);
        float o[8];
        if (dres) load8x(dres + (int64_t)row * E + c0, o);
        else {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += r * (d[j] * gg[j] - s1 - xv[j] * s2);
        store8f(dx + (int64_t)row * E + c0, o);
        if (dxb) {
            store8(dxb + (int64_t)row * E + c0, o);
#pragma unroll
            for (int j = 0; j < 8; ++j) as[j] += o[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[w][0][c0 + j] = ag[j];
        red[w][1][c0 + j] = ab[j];
        red[w][2][c0 + j] = as[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < E; c += 256) {
        float a = 0.f, bsum = 0.f, ssum = 0.f;
#pragma unroll
        for (int k = 0; k < ROWS_PER_BLOCK; ++k) {
            a += red[k][0][c];
            bsum += red[k][1][c];
            ssum += red[k][2][c];
        }
        dgp[(int64_t)blockIdx.x * E + c] = a;
        dbp[(int64_t)blockIdx.x * E + c] = bsum;
        if (dxb) dsp[(int64_t)blockIdx.x * E + c] = ssum;
    }
}

// out = x + (a + bias) [dropout on (a + bias) when p > 0]
__global__ __launch_bounds__(256) void resid_kernel(const float* __restrict__ x, const bf16_t* __restrict__ a,
                                                    const float* __restrict__ bias, int T, float p, uint32_t salt,
                                                    const uint32_t* __restrict__ seed_dev, float* __restrict__ out,
                                                    const float* __restrict__ lg, const float* __restrict__ lb,
                                                    float eps, bf16_t* __restrict__ xn, float* __restrict__ mu,
                                                    float* __restrict__ rs) {
    const uint32_t seed = dev_seed(salt, seed_dev);
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= T) return;
    const int c0 = lane * 8;
    float xv[8], av[8], bb[8];
    load8x(x + (int64_t)row * E + c0, xv);
    load8(a + (int64_t)row * E + c0, av);
    load8f(bias + c0, bb);
    const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float h = av[j] + bb[j];
        if (p > 0.f) h = dropped(seed, row, c0 + j, p) ? 0.f : h * ik;
        xv[j] += h;
    }
    store8f(out + (int64_t)row * E + c0, xv);
    if (lg) {
        // the next LayerNorm of the row just formed, with ln_fwd_kernel's arithmetic (bit-identical to running it)
        float v[8], s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            v[j] = xv[j];
            s += v[j];
        }
        const float m = wave_sum(s) * (1.f / E);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            v[j] -= m;
            q = fmaf(v[j], v[j], q);
        }
        const float r = rsqrtf(wave_sum(q) * (1.f / E) + eps);
        float gg[8], bl[8];
        load8f(lg + c0, gg);
        load8f(lb + c0, bl);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j] * r, gg[j], bl[j]);
        store8(xn + (int64_t)row * E + c0, v);
        if (lane == 0) {
            mu[row] = m;
            rs[row] = r;
        }
    }
}

// dh = dout * keep/(1-p) as bf16 (the GEMM operand), plus the fp32 per-block column sums (bias grad)
__global__ __launch_bounds__(256) void drop_bwd_kernel(const float* __restrict__ dout, int T, float p, uint32_t salt,
                                                       const uint32_t* __restrict__ seed_dev, bf16_t* __restrict__ dh,
                                                       float* __restrict__ dbp) {
    const uint32_t seed = dev_seed(salt, seed_dev);
    __shared__ float red[ROWS_PER_BLOCK][E];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = lane * 8;
    const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int row = blockIdx.x * ROWS_PER_BLOCK + w; row < T; row += gridDim.x * ROWS_PER_BLOCK) {
        float d[8];
        load8x(dout + (int64_t)row * E + c0, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (p > 0.f) d[j] = dropped(seed, row, c0 + j, p) ? 0.f : d[j] * ik;
            acc[j] += d[j];
        }
        store8(dh + (int64_t)row * E + c0, d);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w][c0 + j] = acc[j];
    __syncthreads();
    for (int c = threadIdx.x; c < E; c += 256) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < ROWS_PER_BLOCK; ++k) a += red[k][c];
        dbp[(int64_t)blockIdx.x * E + c] = a;
    }
}

}  // namespace

extern "C" {

int rt1_tf_grid(int T) {
    const int g = (T + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
    return g < 512 ? g : 512;
}

int rt1_ln_fwd(const float* x, const float* g, const float* b, int T, float eps, bf16_t* y, float* mu, float* rs,
               hipStream_t st) {
    hipLaunchKernelGGL(ln_fwd_kernel, dim3((T + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK), dim3(256), 0, st, x, g, b, T,
                       eps, y, mu, rs);
    return (int)hipGetLastError();
}

int rt1_ln_bwd(const bf16_t* dy, const float* x, const float* mu, const float* rs, const float* g, const float* dres,
               int T, float* dx, float* dgp, float* dbp, bf16_t* dxb, float* dsp, int grid, hipStream_t st) {
    if (dxb && !dsp) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(ln_bwd_kernel, dim3(grid), dim3(256), 0, st, dy, x, mu, rs, g, dres, T, dx, dgp, dbp, dxb, dsp);
    return (int)hipGetLastError();
}

int rt1_resid(const float* x, const bf16_t* a, const float* bias, int T, float p, uint32_t seed,
              const uint32_t* seed_dev, float* out, const float* lg, const float* lb, float eps, bf16_t* xn, float* mu,
              float* rs, hipStream_t st) {
    if (lg && (!lb || !xn || !mu || !rs)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(resid_kernel, dim3((T + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK), dim3(256), 0, st, x, a, bias, T,
                       p, seed, seed_dev, out, lg, lb, eps, xn, mu, rs);
    return (int)hipGetLastError();
}

int rt1_drop_bwd(const float* dout, int T, float p, uint32_t seed, const uint32_t* seed_dev, bf16_t* dh, float* dbp,
                 int grid, hipStream_t st) {
    hipLaunchKernelGGL(drop_bwd_kernel, dim3(grid), dim3(256), 0, st, dout, T, p, seed, seed_dev, dh, dbp);
    return (int)hipGetLastError();
}

}  // extern "C"
