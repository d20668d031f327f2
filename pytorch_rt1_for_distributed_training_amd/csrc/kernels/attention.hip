// RT-1 masked self-attention on MFMA (gfx950, wave64), one workgroup per (batch, head).
//
// Spec (reference transformer.py:82-109, mask transformer_network.py:156-192):
//   S = Q K^T / sqrt(D), masked (j > i, or i and j both action tokens) -> softmax
//   -> dropout(p) -> @ V.   Sequence = T steps x (K image + A action) tokens (66 at T=6).
// The mask is evaluated arithmetically (never loaded): allowed(i,j) =
//   j <= i  &&  !(act(i) && act(j)),   act(p) = (p % L) >= K_img.
//
// Layout: qkv is the fused projection output [B, S, 3, H, D] bf16 (D = 128);
// out is [B, S, H, D] bf16 so the out-projection GEMM reads it as [B*S, H*D].
// Per workgroup (4 waves): K and V^T are staged in LDS (zero-padded to S_pad,
// a multiple of 32), each wave takes 16-query row blocks:
//   QK^T : mfma_f32_16x16x32_bf16, A = Q rows straight from global (16 B / lane),
//          B = K rows from LDS; only key blocks <= the row block (causal).
//   softmax in registers (row = 4 regs x 16 lanes, shuffle reductions), the
//          per-row log-sum-exp is written for the backward pass;
//   dropout: counter-based hash of (seed, b, h, i, j) -> identical mask in backward;
//   P V  : P goes through a per-wave LDS tile to become the A operand,
//          B = V^T rows from LDS.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 128;
constexpr int WAVES = 4;

__device__ __forceinline__ bool attn_allowed(int i, int j, int S, int L, int Kimg) {
    if (j > i || j >= S) return false;
    const bool ai = (i % L) >= Kimg, aj = (j % L) >= Kimg;
    return !(ai && aj);
}

// 32-bit mix (splitmix-style); uniform in [0, 1)
__device__ __forceinline__ float hash_uniform(uint32_t seed, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t x = seed ^ (a * 0x9E3779B1u) ^ (b * 0x85EBCA77u) ^ (c * 0xC2B2AE3Du);
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}

__global__ __launch_bounds__(256) void rt1_attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                           float* __restrict__ lse, int B, int S, int H, int L,
                                                           int Kimg, float scale, float drop_p, uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Sp = (S + 31) & ~31;
    bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);            // [Sp][D]
    bf16_t* Vt = Ks + Sp * D;                                 // [D][Sp]
    bf16_t* Pw = Vt + D * Sp;                                 // [WAVES][16][Sp]
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh % H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t row_stride = 3LL * H * D;                   // between consecutive tokens
    const bf16_t* qbase = qkv + (int64_t)b * S * row_stride + (int64_t)h * D;
    const bf16_t* kbase = qbase + (int64_t)H * D;
    const bf16_t* vbase = kbase + (int64_t)H * D;

    // ---- stage K rows and V^T (zero padded)
    for (int i = tid; i < Sp * (D / 8); i += 256) {
        const int r = i / (D / 8), c = (i % (D / 8)) * 8;
        uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
        if (r < S) {
            kv = *reinterpret_cast<const uint4*>(kbase + (int64_t)r * row_stride + c);
            vv = *reinterpret_cast<const uint4*>(vbase + (int64_t)r * row_stride + c);
        }
        *reinterpret_cast<uint4*>(Ks + r * D + c) = kv;
        const bf16_t* vp = reinterpret_cast<const bf16_t*>(&vv);
#pragma unroll
        for (int j = 0; j < 8; ++j) Vt[(c + j) * Sp + r] = vp[j];
    }
    __syncthreads();

    const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
    const int nrb = (S + 15) / 16;
    bf16_t* P = Pw + wave * 16 * Sp;
    const int lr = lane & 15, lg = lane >> 4;                  // MFMA lane row / group
    for (int rb = wave; rb < nrb; rb += WAVES) {
        const int q0 = rb * 16;
        // Q fragments (A operand): lane holds Q[q0 + lr][32*ks + 8*lg + j]
        bf16x8 qf[D / 32];
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
            const int q = q0 + lr;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (q < S) u = *reinterpret_cast<const uint4*>(qbase + (int64_t)q * row_stride + 32 * ks + 8 * lg);
            qf[ks] = *reinterpret_cast<bf16x8*>(&u);
        }
        const int nkb = rb + 1;                                 // causal: key blocks 0..rb
        constexpr int MAXKB = 16;                               // supports S <= 256 (max_seq_len)
        f32x4 sacc[MAXKB];
#pragma unroll
        for (int kb = 0; kb < MAXKB; ++kb) {
            sacc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (kb < nkb) {
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) {
                    const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (kb * 16 + lr) * D + 32 * ks + 8 * lg);
                    sacc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, sacc[kb], 0, 0, 0);
                }
            }
        }
        // C layout: sacc[kb][r] = S[q0 + 4*lg + r][kb*16 + lr]
        float mx[4], sm[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) mx[r] = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < MAXKB; ++kb) {
            if (kb >= nkb) break;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = q0 + 4 * lg + r, j = kb * 16 + lr;
                const float v = attn_allowed(i, j, S, L, Kimg) ? sacc[kb][r] * scale : -INFINITY;
                sacc[kb][r] = v;
                mx[r] = fmaxf(mx[r], v);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
            sm[r] = 0.f;
        }
#pragma unroll
        for (int kb = 0; kb < MAXKB; ++kb) {
            if (kb >= nkb) break;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = (mx[r] == -INFINITY) ? 0.f : __expf(sacc[kb][r] - mx[r]);
                sacc[kb][r] = e;
                sm[r] += e;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) sm[r] += __shfl_xor(sm[r], o, 64);
        }
        if (lr == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = q0 + 4 * lg + r;
                if (i < S) lse[(int64_t)bh * S + i] = (sm[r] > 0.f) ? mx[r] + __logf(sm[r]) : -INFINITY;
            }
        }
        // normalise, dropout, write P (bf16) to this wave's LDS tile (zero beyond nkb*16 up to the 32-key step)
        const int kend = ((nkb * 16) + 31) & ~31;
#pragma unroll
        for (int kb = 0; kb < MAXKB; ++kb) {
            if (kb * 16 >= kend) break;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = q0 + 4 * lg + r, j = kb * 16 + lr;
                float p = 0.f;
                if (kb < nkb && sm[r] > 0.f) {
                    p = sacc[kb][r] / sm[r];
                    if (drop_p > 0.f)
                        p = hash_uniform(seed, (uint32_t)bh, (uint32_t)i, (uint32_t)j) < drop_p ? 0.f : p * inv_keep;
                }
                P[(4 * lg + r) * Sp + j] = f2bf(p);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's P writes landed
        __builtin_amdgcn_wave_barrier();
        // O = P V : A = P[q][key] (LDS row), B = V^T[d][key] (LDS row)
        f32x4 oacc[D / 16];
#pragma unroll
        for (int db = 0; db < D / 16; ++db) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < kend; k0 += 32) {
            const bf16x8 pf = *reinterpret_cast<const bf16x8*>(P + lr * Sp + k0 + 8 * lg);
#pragma unroll
            for (int db = 0; db < D / 16; ++db) {
                const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vt + (db * 16 + lr) * Sp + k0 + 8 * lg);
                oacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, oacc[db], 0, 0, 0);
            }
        }
        // C layout: oacc[db][r] = O[q0 + 4*lg + r][db*16 + lr]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int q = q0 + 4 * lg + r;
            if (q < S) {
                bf16_t* orow = out + (((int64_t)b * S + q) * H + h) * D;
#pragma unroll
                for (int db = 0; db < D / 16; ++db) orow[db * 16 + lr] = f2bf(oacc[db][r]);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// keep-mask of the forward's dropout (1 = kept), [B*H, S, S] uint8, same hash
__global__ __launch_bounds__(256) void rt1_attn_keepmask_kernel(uint8_t* __restrict__ keep, int BH, int S,
                                                                float drop_p, uint32_t seed) {
    const int64_t total = (int64_t)BH * S * S;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int j = (int)(t % S);
        const int i = (int)((t / S) % S);
        const int bh = (int)(t / ((int64_t)S * S));
        keep[t] = hash_uniform(seed, (uint32_t)bh, (uint32_t)i, (uint32_t)j) < drop_p ? 0 : 1;
    }
}

}  // namespace

extern "C" {

int rt1_attn_keepmask(uint8_t* keep, int BH, int S, float drop_p, uint32_t seed, hipStream_t st) {
    int64_t blocks = ((int64_t)BH * S * S + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(rt1_attn_keepmask_kernel, dim3((unsigned)blocks), dim3(256), 0, st, keep, BH, S, drop_p, seed);
    return (int)hipGetLastError();
}

int rt1_attn_fwd(const bf16_t* qkv, bf16_t* out, float* lse, int B, int S, int H, int L, int Kimg, float scale,
                 float drop_p, uint32_t seed, hipStream_t st) {
    if (S > 256 || S < 1) return (int)hipErrorInvalidValue;
    const int Sp = (S + 31) & ~31;
    const size_t lds = (size_t)(Sp * D * 2 + WAVES * 16 * Sp) * sizeof(bf16_t);
    hipLaunchKernelGGL(rt1_attn_fwd_kernel, dim3(B * H), dim3(256), lds, st, qkv, out, lse, B, S, H, L, Kimg, scale,
                       drop_p, seed);
    return (int)hipGetLastError();
}

}  // extern "C"
