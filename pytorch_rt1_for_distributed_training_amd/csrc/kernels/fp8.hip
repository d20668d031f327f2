// fp8 (OCP e4m3fn, gfx950) activation quantisation with delayed per-tensor scaling (BASELINE config 5).
//
// out = sat_448(x / scale), scale = amax_prev / 448, where amax_prev is the running amax recorded by the
// previous call at this GEMM site; the same pass records max|x| of THIS call into amax_next (integer
// atomicMax on the float bits of |x|: order-independent, so bitwise reproducible).  One read of x (bf16),
// one write of the fp8 copy -- the operand of the hipBLASLt fp8 GEMM (v_mfma ... fp8 on CDNA4).
#include "common.h"

using namespace rt1;

namespace {

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
    a = __builtin_amdgcn_fmed3f(a, 448.f, -448.f);
    b = __builtin_amdgcn_fmed3f(b, 448.f, -448.f);
    c = __builtin_amdgcn_fmed3f(c, 448.f, -448.f);
    d = __builtin_amdgcn_fmed3f(d, 448.f, -448.f);
    uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);   // bytes 0,1
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);              // bytes 2,3
    return w;
}

__global__ __launch_bounds__(256) void fp8_quant_kernel(const bf16_t* __restrict__ x, int64_t n8,
                                                        const float* __restrict__ amax_prev,
                                                        float* __restrict__ scale_out, uint2* __restrict__ out,
                                                        unsigned int* __restrict__ amax_next) {
    const float amax = fmaxf(amax_prev[0], 1e-12f);
    const float scale = amax * (1.f / 448.f);
    const float inv = 448.f / amax;
    if (blockIdx.x == 0 && threadIdx.x == 0) scale_out[0] = scale;
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        float v[8];
        load8(x + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
        uint2 o;
        o.x = pack4_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
        o.y = pack4_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
        out[i] = o;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(amax_next, __float_as_uint(m));
}

}  // namespace

extern "C" int rt1_fp8_quant(const bf16_t* x, int64_t n, const float* amax_prev, float* scale_out, uint8_t* out,
                             unsigned int* amax_next, hipStream_t st) {
    if (n % 8) return (int)hipErrorInvalidValue;
    const int64_t n8 = n / 8;
    int64_t blocks = (n8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(fp8_quant_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n8, amax_prev, scale_out,
                       reinterpret_cast<uint2*>(out), amax_next);
    return (int)hipGetLastError();
}
