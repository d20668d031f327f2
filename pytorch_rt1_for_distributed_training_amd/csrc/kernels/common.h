// Shared device helpers for the RT-1 kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace rt1 {

typedef uint16_t bf16_t;  // raw bf16 storage

constexpr int kWave = 64;

// Kernels whose fp32 FMAs the compiler packs as v_pk_fma_f32 with a low lane that selects the HIGH source element
// (op_sel:[0,1,0] / [1,0,0], a broadcast of an odd element) are built without packed fp32.  With two processes
// sharing the GPU, such an instruction in se_wsum_part lost its low-lane product for the 16 lanes of one row group:
// dw1 = correct - exactly one frame's term (profiles/r4_se_dp_rootcause.md).  tests/test_isa_audit.py fails on any
// such instruction in the built objects.
#define NO_PACKED_FP32 __attribute__((target("no-packed-fp32-ops")))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
    // plain cast: hipcc -O3 emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
    __hip_bfloat16 h = __float2bfloat16(f);
    return *reinterpret_cast<bf16_t*>(&h);
}

// 8 x bf16 <-> 8 x f32 through one 16-byte access
__device__ __forceinline__ void load8(const bf16_t* __restrict__ p, float (&o)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xffff0000u);
    o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xffff0000u);
    o[4] = __uint_as_float(u.z << 16); o[5] = __uint_as_float(u.z & 0xffff0000u);
    o[6] = __uint_as_float(u.w << 16); o[7] = __uint_as_float(u.w & 0xffff0000u);
}

// the same from a 16-byte value already in registers
__device__ __forceinline__ void unpack8(const uint4 u, float (&f)[8]) {
    f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
    f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
    f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}

// one v_cvt_pk_bf16_f32 (RNE) for the pair; two scalar casts OR'ed together cost two converts plus a v_or_b32_sdwa
typedef float pk_f2_t __attribute__((ext_vector_type(2)));
typedef __bf16 pk_bf2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((pk_f2_t){a, b}, pk_bf2_t));
}

__device__ __forceinline__ void store8(bf16_t* __restrict__ p, const float (&v)[8]) {
    uint4 u;
    u.x = pack2(v[0], v[1]); u.y = pack2(v[2], v[3]); u.z = pack2(v[4], v[5]); u.w = pack2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = u;
}

__device__ __forceinline__ void load8f(const float* __restrict__ p, float (&o)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// v_exp_f32 + v_rcp_f32 (1 ulp): avoids the IEEE division sequence in every SiLU of the memory-bound kernels
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float silu(float x) { return x * sigmoidf_(x); }
// d/dx silu(x) = s + x s (1 - s)
__device__ __forceinline__ float silu_grad(float x) {
    const float s = sigmoidf_(x);
    return s * (1.f + x * (1.f - s));
}

// Row-vector work layout for [M, C] channels-last tensors: a 256-thread block
// covers `slots` rows at once, each thread owns fixed channel vector(s)
// (8 channels, 16 B) so per-channel constants live in registers and no
// per-element index division is needed.  C/8 > 256 uses VPT = 2.
struct RowGeo {
    int nv, vpt, slots, slot, vec0;
    bool active;
    __device__ RowGeo(int C, int block = 256) {
        nv = C >> 3;
        vpt = (nv + block - 1) / block;
        slots = vpt == 1 ? block / nv : 1;
        slot = slots == 1 ? 0 : (int)threadIdx.x / nv;
        vec0 = slots == 1 ? (int)threadIdx.x : (int)threadIdx.x % nv;
        active = slot < slots;
    }
};

// n / d for any 32-bit n and a divisor fixed per launch (1 <= d < 2^31): one mul_hi, an add and two shifts instead
// of the ~40-instruction integer division (Granlund-Montgomery round-up multiplier, built on the host)
struct FastDiv {
    uint32_t m = 1;
    int s1 = 0, s2 = 0;
    FastDiv() = default;
    __host__ explicit FastDiv(uint32_t d) {
        if (d == 0) d = 1;   // a zero divisor only arises with an empty launch: no trap on the host, no element divided
        int l = 0;
        while ((1ull << l) < d) ++l;
        m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
        s1 = l > 0 ? 1 : 0;
        s2 = l > 0 ? l - 1 : 0;
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const {
        const uint32_t t = __umulhi(m, n);
        return (t + ((n - t) >> s1)) >> s2;
    }
};

enum Act : int { ACT_NONE = 0, ACT_SILU = 1 };

__device__ __forceinline__ float act_fwd(float x, int act) { return act == ACT_SILU ? silu(x) : x; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Dropout seed = host salt (per call site) + a device-resident step counter, so a captured hipGraph draws a
// fresh mask on every replay (the counter is advanced by a device op inside the graph).
__device__ __forceinline__ uint32_t dev_seed(uint32_t salt, const uint32_t* __restrict__ counter) {
    return salt + (counter ? counter[0] * 0x9E3779B1u : 0u);
}

}  // namespace rt1
