// Fused Adam / AdamW over the flat fp32 parameter buffer (gfx950).
//
// Replaces torch.optim.Adam's per-tensor foreach launches (reference
// distribute_train.py:100): ONE launch updates every trainable
// parameter.  Memory-bound: per element it reads p, g, m, v and writes p, m, v
// (28 B/elem -> 35.2M params = 0.99 GB, ~0.16 ms at 6.3 TB/s).  Loads and
// stores are float4 (16 B/lane), the grid is capped at 8 waves x 256 CUs and
// grid-strides the rest (CDNA guide G11/G13).
//
// The data-parallel 1/world average (grad_scale) and the bias corrections are
// folded in; with weight_decay > 0 the decay is decoupled (AdamW).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct AdamArgs {
    float lr, beta1, beta2, eps, weight_decay;
    float step_size;      // lr / (1 - beta1^t)
    float inv_sqrt_bc2;   // 1 / sqrt(1 - beta2^t)
    float grad_scale;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamArgs& a) {
    g *= a.grad_scale;
    if (a.weight_decay != 0.f) p *= (1.f - a.lr * a.weight_decay);
    m = fmaf(a.beta1, m, (1.f - a.beta1) * g);
    v = fmaf(a.beta2, v, (1.f - a.beta2) * g * g);
    const float denom = sqrtf(v) * a.inv_sqrt_bc2 + a.eps;
    p -= a.step_size * (m / denom);
}

__global__ __launch_bounds__(256) void flat_adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        int64_t n4, int64_t n, AdamArgs a,
                                                        const float* __restrict__ state) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    if (state) {   // {step, lr} on the device (captured-graph replays)
        const float t = state[0], lr = state[1];
        a.lr = lr;
        a.step_size = lr / -expm1f(t * logf(a.beta1));          // 1 - beta^t without cancellation
        a.inv_sqrt_bc2 = rsqrtf(-expm1f(t * logf(a.beta2)));
    }
    for (; i < n4; i += stride) {
        float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
        adam_elem(pp.x, gg.x, mm.x, vv.x, a);
        adam_elem(pp.y, gg.y, mm.y, vv.y, a);
        adam_elem(pp.z, gg.z, mm.z, vv.z, a);
        adam_elem(pp.w, gg.w, mm.w, vv.w, a);
        p4[i] = pp; m4[i] = mm; v4[i] = vv;
    }
    // scalar tail (flat buffers are 64-element aligned, so normally empty)
    for (int64_t j = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        float pp = p[j], mm = m[j], vv = v[j];
        adam_elem(pp, g[j], mm, vv, a);
        p[j] = pp; m[j] = mm; v[j] = vv;
    }
}

}  // namespace

extern "C" int rt1_flat_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                             float beta2, float eps, float weight_decay, float step_size, float inv_sqrt_bc2,
                             float grad_scale, hipStream_t stream) {
    AdamArgs a{lr, beta1, beta2, eps, weight_decay, step_size, inv_sqrt_bc2, grad_scale};
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(flat_adam_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p, g, m, v, n4, n, a,
                       (const float*)nullptr);
    return (int)hipGetLastError();
}

extern "C" int rt1_flat_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* state,
                                 float beta1, float beta2, float eps, float weight_decay, float grad_scale,
                                 hipStream_t stream) {
    AdamArgs a{0.f, beta1, beta2, eps, weight_decay, 0.f, 1.f, grad_scale};
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(flat_adam_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p, g, m, v, n4, n, a, state);
    return (int)hipGetLastError();
}
