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
// The backward (rt1_attn_bwd_kernel, below) regenerates P and the dropout mask and produces dQ, dK, dV
// in one kernel per (batch, head).
#include <cstdlib>

#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 128;

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

// MAXKB = Sp / 16 key blocks (compile-time, so the score accumulators stay in registers)
template <int MAXKB, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void rt1_attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                           float* __restrict__ lse, int B, int S, int H, int L,
                                                           int Kimg, float scale, float drop_p, uint32_t salt,
    const uint32_t* __restrict__ seed_dev) {
    const uint32_t seed = dev_seed(salt, seed_dev);
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
    for (int i = tid; i < Sp * (D / 8); i += WAVES * 64) {
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
                                                                float drop_p, uint32_t salt,
    const uint32_t* __restrict__ seed_dev) {
    const uint32_t seed = dev_seed(salt, seed_dev);
    const int64_t total = (int64_t)BH * S * S;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int j = (int)(t % S);
        const int i = (int)((t / S) % S);
        const int bh = (int)(t / ((int64_t)S * S));
        keep[t] = hash_uniform(seed, (uint32_t)bh, (uint32_t)i, (uint32_t)j) < drop_p ? 0 : 1;
    }
}


// ------------------------------------------------------------------ backward
// One workgroup per (batch, head), S <= 96 (RT-1 T <= 8).  With P recomputed from Q, K and the saved
// log-sum-exp, and the forward's dropout mask regenerated from the same hash:
//   Pd = P * keep/(1-p),  dPd = dO V^T,  delta_i = dO_i . O_i,  dS = P * (dPd * keep/(1-p) - delta) * scale
//   dQ = dS K,  dK = dS^T Q,  dV = Pd^T dO
// Phase 1 (query row blocks per wave): S, P, dPd in registers -> Pd, dS rows into LDS; dQ from dS rows
//   and K (MFMA B operand read k-major with ds_read_b64_tr_b16).
// Phase 2 (key row blocks per wave): dV and dK as MFMAs over the query index, both operands read
//   transposed from the LDS images (Pd/dS and dO/Q) with ds_read_b64_tr_b16.
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BWD_MAX_S = 96;
constexpr int LDQ = D + 16;          // Q / K / dO image row stride (bf16)

__device__ __forceinline__ bf16x8 tr8(const bf16_t* a0, const bf16_t* a1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void rt1_attn_bwd_kernel(const bf16_t* __restrict__ qkv,
                                                           const bf16_t* __restrict__ out,
                                                           const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse,
                                                           bf16_t* __restrict__ dqkv, int B, int S, int H, int L,
                                                           int Kimg, float scale, float drop_p, uint32_t salt,
    const uint32_t* __restrict__ seed_dev) {
    const uint32_t seed = dev_seed(salt, seed_dev);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Sp = (S + 31) & ~31;
    const int LDP = Sp + 16;
    bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);             // [Sp][LDQ]
    bf16_t* Ks = Qs + Sp * LDQ;
    bf16_t* dOs = Ks + Sp * LDQ;
    bf16_t* Pds = dOs + Sp * LDQ;                              // [Sp][LDP]  Pd[i][j]
    bf16_t* dSs = Pds + Sp * LDP;                              // [Sp][LDP]  dS[i][j]
    float* delta = reinterpret_cast<float*>(dSs + Sp * LDP);   // [Sp]
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh % H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 15, lg = lane >> 4;
    const int64_t rs3 = 3LL * H * D, rs1 = (int64_t)H * D;
    const bf16_t* qbase = qkv + (int64_t)b * S * rs3 + (int64_t)h * D;
    const bf16_t* kbase = qbase + rs1;
    const bf16_t* vbase = kbase + rs1;
    const bf16_t* obase = out + (int64_t)b * S * rs1 + (int64_t)h * D;
    const bf16_t* dobase = dout + (int64_t)b * S * rs1 + (int64_t)h * D;
    bf16_t* dqbase = dqkv + (int64_t)b * S * rs3 + (int64_t)h * D;

    // ---- stage Q, K, dO rows (zero padded) and delta_i = dO_i . O_i
    for (int i = tid; i < Sp * (D / 8); i += NW * 64) {
        const int r = i / (D / 8), c = (i % (D / 8)) * 8;
        uint4 qv = make_uint4(0, 0, 0, 0), kv = qv, dv = qv;
        if (r < S) {
            qv = *reinterpret_cast<const uint4*>(qbase + (int64_t)r * rs3 + c);
            kv = *reinterpret_cast<const uint4*>(kbase + (int64_t)r * rs3 + c);
            dv = *reinterpret_cast<const uint4*>(dobase + (int64_t)r * rs1 + c);
        }
        *reinterpret_cast<uint4*>(Qs + r * LDQ + c) = qv;
        *reinterpret_cast<uint4*>(Ks + r * LDQ + c) = kv;
        *reinterpret_cast<uint4*>(dOs + r * LDQ + c) = dv;
    }
    for (int r = wave; r < Sp; r += NW) {
        float acc = 0.f;
        if (r < S) {
            const uint32_t o2 = *reinterpret_cast<const uint32_t*>(obase + (int64_t)r * rs1 + 2 * lane);
            const uint32_t d2 = *reinterpret_cast<const uint32_t*>(dobase + (int64_t)r * rs1 + 2 * lane);
            acc = __uint_as_float(o2 << 16) * __uint_as_float(d2 << 16) +
                  __uint_as_float(o2 & 0xffff0000u) * __uint_as_float(d2 & 0xffff0000u);
        }
        acc = wave_sum(acc);
        if (lane == 0) delta[r] = acc;
    }
    __syncthreads();

    const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
    const int nrb = Sp / 16;
    constexpr int MAXKB = BWD_MAX_S / 16;
    // ---------------- phase 1: query row blocks
    for (int rb = wave; rb < nrb; rb += NW) {
        const int q0 = rb * 16;
        const int nkb = rb + 1;                                     // causal key blocks
        bf16x8 qf[D / 32], df[D / 32];
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
            qf[ks] = *reinterpret_cast<const bf16x8*>(Qs + (q0 + lr) * LDQ + 32 * ks + 8 * lg);
            df[ks] = *reinterpret_cast<const bf16x8*>(dOs + (q0 + lr) * LDQ + 32 * ks + 8 * lg);
        }
        f32x4 sacc[MAXKB], pacc[MAXKB];
#pragma unroll
        for (int kb = 0; kb < MAXKB; ++kb) {
            sacc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
            pacc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (kb < nkb) {
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) {
                    const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (kb * 16 + lr) * LDQ + 32 * ks + 8 * lg);
                    sacc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, sacc[kb], 0, 0, 0);
                    // dPd = dO V^T: B[k = d][col = j] = V[j][d], read straight from global (L2)
                    const int j = kb * 16 + lr;
                    uint4 vu = make_uint4(0, 0, 0, 0);
                    if (j < S) vu = *reinterpret_cast<const uint4*>(vbase + (int64_t)j * rs3 + 32 * ks + 8 * lg);
                    pacc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(df[ks], *reinterpret_cast<bf16x8*>(&vu),
                                                                        pacc[kb], 0, 0, 0);
                }
            }
        }
        // C layout: [kb][r] -> (i = q0 + 4*lg + r, j = kb*16 + lr)
        float lrow[4], drow[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = q0 + 4 * lg + r;
            lrow[r] = i < S ? lse[(int64_t)bh * S + i] : 0.f;
            drow[r] = delta[i];
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int kb = 0; kb < MAXKB; ++kb) {
            if (kb * 16 >= Sp) break;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = q0 + 4 * lg + r, j = kb * 16 + lr;
                float pd = 0.f, ds = 0.f;
                if (kb < nkb && i < S && attn_allowed(i, j, S, L, Kimg)) {
                    const float p = __expf(sacc[kb][r] * scale - lrow[r]);
                    float keep = 1.f;
                    if (drop_p > 0.f)
                        keep = hash_uniform(seed, (uint32_t)bh, (uint32_t)i, (uint32_t)j) < drop_p ? 0.f : inv_keep;
                    pd = p * keep;
                    ds = p * (pacc[kb][r] * keep - drow[r]) * scale;
                }
                Pds[(q0 + 4 * lg + r) * LDP + j] = f2bf(pd);
                dSs[(q0 + 4 * lg + r) * LDP + j] = f2bf(ds);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's dS rows are in LDS
        __builtin_amdgcn_wave_barrier();
        // dQ = dS K over j < kend (A = dS rows, B[k = j][col = d] = K[j][d] via transposed reads)
        const int kend = ((nkb * 16) + 31) & ~31;
        f32x4 qacc[D / 16];
#pragma unroll
        for (int db = 0; db < D / 16; ++db) qacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int tq = (lane & 15) >> 2, tp = lane & 3;
        for (int k0 = 0; k0 < kend; k0 += 32) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(dSs + (q0 + lr) * LDP + k0 + 8 * lg);
            const int jr = k0 + 8 * lg + tq;
#pragma unroll
            for (int db = 0; db < D / 16; ++db) {
                const bf16x8 kt = tr8(Ks + jr * LDQ + db * 16 + 4 * tp, Ks + (jr + 4) * LDQ + db * 16 + 4 * tp);
                qacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, kt, qacc[db], 0, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = q0 + 4 * lg + r;
            if (i < S) {
                bf16_t* row = dqbase + (int64_t)i * rs3;
#pragma unroll
                for (int db = 0; db < D / 16; ++db) row[db * 16 + lr] = f2bf(qacc[db][r]);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // ---------------- phase 2: key row blocks: dV = Pd^T dO, dK = dS^T Q  (k = query index i >= j)
    const int tq = (lane & 15) >> 2, tp = lane & 3;
    for (int jb = wave; jb < nrb; jb += NW) {
        const int j0 = jb * 16;
        f32x4 vacc[D / 16], kacc[D / 16];
#pragma unroll
        for (int db = 0; db < D / 16; ++db) vacc[db] = kacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int i0 = j0 & ~31; i0 < Sp; i0 += 32) {
            const int ir = i0 + 8 * lg + tq;
            // A[row = j][k = i] = Pd[i][j]  /  dS[i][j]
            const bf16x8 pa = tr8(Pds + ir * LDP + j0 + 4 * tp, Pds + (ir + 4) * LDP + j0 + 4 * tp);
            const bf16x8 sa = tr8(dSs + ir * LDP + j0 + 4 * tp, dSs + (ir + 4) * LDP + j0 + 4 * tp);
#pragma unroll
            for (int db = 0; db < D / 16; ++db) {
                const bf16x8 ob = tr8(dOs + ir * LDQ + db * 16 + 4 * tp, dOs + (ir + 4) * LDQ + db * 16 + 4 * tp);
                const bf16x8 qb = tr8(Qs + ir * LDQ + db * 16 + 4 * tp, Qs + (ir + 4) * LDQ + db * 16 + 4 * tp);
                vacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ob, vacc[db], 0, 0, 0);
                kacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, qb, kacc[db], 0, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = j0 + 4 * lg + r;
            if (j < S) {
                bf16_t* krow = dqbase + (int64_t)j * rs3 + rs1;
                bf16_t* vrow = krow + rs1;
#pragma unroll
                for (int db = 0; db < D / 16; ++db) {
                    krow[db * 16 + lr] = f2bf(kacc[db][r]);
                    vrow[db * 16 + lr] = f2bf(vacc[db][r]);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ backward, long histories (S <= 256)
// The S <= 96 kernel keeps whole S x S Pd / dS images in LDS; at T = 15 (S = 165) that is > 160 KB.  Here the
// backward is split into two kernels that stream 32-row chunks through LDS instead, so LDS is O(chunk * D):
//   dkdv: each wave owns a 16-key block j and accumulates dV_j = sum_i Pd[i, j] dO_i and dK_j = sum_i dS[i, j] Q_i
//         over the 32-query chunks i >= j (the 4 waves of a round share each staged Q / dO chunk);
//   dq:   each wave owns a 16-query block i and accumulates dQ_i = sum_j dS[i, j] K_j over 32-key chunks j <= i.
// Both recompute S, P (from the saved LSE) and dP = dO V^T with MFMAs, regenerate the dropout mask from the
// forward's hash, and transpose the 16 x 32 Pd^T / dS tiles through a per-wave LDS tile into MFMA A operands.
// No atomics: every output row is owned by exactly one wave (bitwise deterministic).
constexpr int LDT = 40;              // per-wave 16 x 32 tile stride (bf16)

__device__ __forceinline__ void stage_rows32(bf16_t* dst, const bf16_t* base, int64_t stride, int r0, int S) {
    // 32 rows x 128 bf16 -> dst[32][LDQ], zero beyond S; 256 threads x 2 16-byte vectors
    for (int v = threadIdx.x; v < 32 * (D / 8); v += 256) {
        const int r = v / (D / 8), c = (v % (D / 8)) * 8;
        uint4 u = make_uint4(0, 0, 0, 0);
        if (r0 + r < S) u = *reinterpret_cast<const uint4*>(base + (int64_t)(r0 + r) * stride + c);
        *reinterpret_cast<uint4*>(dst + r * LDQ + c) = u;
    }
}

// delta_i = dO_i . O_i for all rows, into LDS
__device__ __forceinline__ void stage_delta(float* delta, const bf16_t* obase, const bf16_t* dobase, int64_t rs1, int S,
                                            int Sp) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int r = wave; r < Sp; r += 4) {
        float acc = 0.f;
        if (r < S) {
            const uint32_t o2 = *reinterpret_cast<const uint32_t*>(obase + (int64_t)r * rs1 + 2 * lane);
            const uint32_t d2 = *reinterpret_cast<const uint32_t*>(dobase + (int64_t)r * rs1 + 2 * lane);
            acc = __uint_as_float(o2 << 16) * __uint_as_float(d2 << 16) +
                  __uint_as_float(o2 & 0xffff0000u) * __uint_as_float(d2 & 0xffff0000u);
        }
        acc = wave_sum(acc);
        if (lane == 0) delta[r] = acc;
    }
}

__global__ __launch_bounds__(256) void rt1_attn_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv,
                                                                const bf16_t* __restrict__ out,
                                                                const bf16_t* __restrict__ dout,
                                                                const float* __restrict__ lse,
                                                                bf16_t* __restrict__ dqkv, int S, int H, int L,
                                                                int Kimg, float scale, float drop_p, uint32_t salt,
                                                                const uint32_t* __restrict__ seed_dev) {
    const uint32_t seed = dev_seed(salt, seed_dev);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Sp = (S + 31) & ~31;
    bf16_t* Qc = reinterpret_cast<bf16_t*>(smem);            // [32][LDQ]
    bf16_t* dOc = Qc + 32 * LDQ;                              // [32][LDQ]
    bf16_t* Tw = dOc + 32 * LDQ;                              // [4 waves][2][16][LDT]  Pd^T, dS^T tiles
    float* delta = reinterpret_cast<float*>(Tw + 4 * 2 * 16 * LDT);   // [Sp]
    float* lsel = delta + Sp;                                 // [Sp]
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh % H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 15, lg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
    const int64_t rs3 = 3LL * H * D, rs1 = (int64_t)H * D;
    const bf16_t* qbase = qkv + (int64_t)b * S * rs3 + (int64_t)h * D;
    const bf16_t* kbase = qbase + rs1;
    const bf16_t* vbase = kbase + rs1;
    const bf16_t* obase = out + (int64_t)b * S * rs1 + (int64_t)h * D;
    const bf16_t* dobase = dout + (int64_t)b * S * rs1 + (int64_t)h * D;
    bf16_t* dbase = dqkv + (int64_t)b * S * rs3 + (int64_t)h * D;
    stage_delta(delta, obase, dobase, rs1, S, Sp);
    for (int r = tid; r < Sp; r += 256) lsel[r] = r < S ? lse[(int64_t)bh * S + r] : 0.f;
    bf16_t* Tp = Tw + wave * 2 * 16 * LDT;                    // Pd^T tile [16 j][32 i]
    bf16_t* Ts = Tp + 16 * LDT;                               // dS^T tile
    const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
    const int nkb = (S + 15) / 16;
    for (int round = 0; round * 4 < nkb; ++round) {
        const int jb = round * 4 + wave;
        const int j0 = jb * 16;
        const bool active = jb < nkb;
        // K_j and V_j rows as A operands (lane: row j0 + lr, k = 32 ks + 8 lg ..)
        bf16x8 kf[D / 32], vf[D / 32];
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
            uint4 ku = make_uint4(0, 0, 0, 0), vu = ku;
            if (active && j0 + lr < S) {
                ku = *reinterpret_cast<const uint4*>(kbase + (int64_t)(j0 + lr) * rs3 + 32 * ks + 8 * lg);
                vu = *reinterpret_cast<const uint4*>(vbase + (int64_t)(j0 + lr) * rs3 + 32 * ks + 8 * lg);
            }
            kf[ks] = *reinterpret_cast<bf16x8*>(&ku);
            vf[ks] = *reinterpret_cast<bf16x8*>(&vu);
        }
        f32x4 vacc[D / 16], kacc[D / 16];
#pragma unroll
        for (int db = 0; db < D / 16; ++db) vacc[db] = kacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int i0 = (round * 64) & ~31; i0 < Sp; i0 += 32) {
            __syncthreads();                                   // previous chunk fully consumed
            stage_rows32(Qc, qbase, rs3, i0, S);
            stage_rows32(dOc, dobase, rs1, i0, S);
            __syncthreads();
            if (!active || i0 + 31 < j0) continue;             // chunk entirely before this key block (causal)
#pragma unroll
            for (int ih = 0; ih < 2; ++ih) {
                f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dpt = st;
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) {
                    const bf16x8 qb = *reinterpret_cast<const bf16x8*>(Qc + (16 * ih + lr) * LDQ + 32 * ks + 8 * lg);
                    const bf16x8 ob = *reinterpret_cast<const bf16x8*>(dOc + (16 * ih + lr) * LDQ + 32 * ks + 8 * lg);
                    st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qb, st, 0, 0, 0);
                    dpt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[ks], ob, dpt, 0, 0, 0);
                }
                // C layout: [r] -> (j = j0 + 4 lg + r, i = i0 + 16 ih + lr)
                const int i = i0 + 16 * ih + lr;
                const float li = lsel[i], di = delta[i];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = j0 + 4 * lg + r;
                    float pd = 0.f, ds = 0.f;
                    if (i < S && attn_allowed(i, j, S, L, Kimg)) {
                        const float p = __expf(st[r] * scale - li);
                        float keep = 1.f;
                        if (drop_p > 0.f)
                            keep = hash_uniform(seed, (uint32_t)bh, (uint32_t)i, (uint32_t)j) < drop_p ? 0.f : inv_keep;
                        pd = p * keep;
                        ds = p * (dpt[r] * keep - di) * scale;
                    }
                    Tp[(4 * lg + r) * LDT + 16 * ih + lr] = f2bf(pd);
                    Ts[(4 * lg + r) * LDT + 16 * ih + lr] = f2bf(ds);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);                // lgkmcnt(0): this wave's tiles are in LDS
            __builtin_amdgcn_wave_barrier();
            const bf16x8 pa = *reinterpret_cast<const bf16x8*>(Tp + lr * LDT + 8 * lg);
            const bf16x8 sa = *reinterpret_cast<const bf16x8*>(Ts + lr * LDT + 8 * lg);
            const int ir = 8 * lg + tq;
#pragma unroll
            for (int db = 0; db < D / 16; ++db) {
                const bf16x8 ob = tr8(dOc + ir * LDQ + db * 16 + 4 * tp, dOc + (ir + 4) * LDQ + db * 16 + 4 * tp);
                const bf16x8 qb = tr8(Qc + ir * LDQ + db * 16 + 4 * tp, Qc + (ir + 4) * LDQ + db * 16 + 4 * tp);
                vacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ob, vacc[db], 0, 0, 0);
                kacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, qb, kacc[db], 0, 0, 0);
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (active) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = j0 + 4 * lg + r;
                if (j < S) {
                    bf16_t* krow = dbase + (int64_t)j * rs3 + rs1;
                    bf16_t* vrow = krow + rs1;
#pragma unroll
                    for (int db = 0; db < D / 16; ++db) {
                        krow[db * 16 + lr] = f2bf(kacc[db][r]);
                        vrow[db * 16 + lr] = f2bf(vacc[db][r]);
                    }
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void rt1_attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv,
                                                              const bf16_t* __restrict__ out,
                                                              const bf16_t* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              bf16_t* __restrict__ dqkv, int S, int H, int L,
                                                              int Kimg, float scale, float drop_p, uint32_t salt,
                                                              const uint32_t* __restrict__ seed_dev) {
    const uint32_t seed = dev_seed(salt, seed_dev);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Sp = (S + 31) & ~31;
    bf16_t* Kc = reinterpret_cast<bf16_t*>(smem);            // [32][LDQ]
    bf16_t* Vc = Kc + 32 * LDQ;                               // [32][LDQ]
    bf16_t* Tw = Vc + 32 * LDQ;                               // [4 waves][16][LDT]  dS tiles
    float* delta = reinterpret_cast<float*>(Tw + 4 * 16 * LDT);
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh % H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 15, lg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
    const int64_t rs3 = 3LL * H * D, rs1 = (int64_t)H * D;
    const bf16_t* qbase = qkv + (int64_t)b * S * rs3 + (int64_t)h * D;
    const bf16_t* kbase = qbase + rs1;
    const bf16_t* vbase = kbase + rs1;
    const bf16_t* obase = out + (int64_t)b * S * rs1 + (int64_t)h * D;
    const bf16_t* dobase = dout + (int64_t)b * S * rs1 + (int64_t)h * D;
    bf16_t* dbase = dqkv + (int64_t)b * S * rs3 + (int64_t)h * D;
    stage_delta(delta, obase, dobase, rs1, S, Sp);
    __syncthreads();
    bf16_t* Ts = Tw + wave * 16 * LDT;
    const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
    const int nqb = (S + 15) / 16;
    for (int round = 0; round * 4 < nqb; ++round) {
        const int qb = round * 4 + wave;
        const int q0 = qb * 16;
        const bool active = qb < nqb;
        bf16x8 qf[D / 32], df[D / 32];
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
            uint4 qu = make_uint4(0, 0, 0, 0), du = qu;
            if (active && q0 + lr < S) {
                qu = *reinterpret_cast<const uint4*>(qbase + (int64_t)(q0 + lr) * rs3 + 32 * ks + 8 * lg);
                du = *reinterpret_cast<const uint4*>(dobase + (int64_t)(q0 + lr) * rs1 + 32 * ks + 8 * lg);
            }
            qf[ks] = *reinterpret_cast<bf16x8*>(&qu);
            df[ks] = *reinterpret_cast<bf16x8*>(&du);
        }
        float lrow[4], drow[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = q0 + 4 * lg + r;
            lrow[r] = (active && i < S) ? lse[(int64_t)bh * S + i] : 0.f;
            drow[r] = (active && i < Sp) ? delta[i] : 0.f;
        }
        f32x4 qacc[D / 16];
#pragma unroll
        for (int db = 0; db < D / 16; ++db) qacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int jend = min(Sp, ((round * 4 + 3) * 16 + 16 + 31) & ~31);   // keys <= last query of the round
        for (int j0 = 0; j0 < jend; j0 += 32) {
            __syncthreads();
            stage_rows32(Kc, kbase, rs3, j0, S);
            stage_rows32(Vc, vbase, rs3, j0, S);
            __syncthreads();
            if (!active || j0 > q0 + 15) continue;              // chunk entirely after this query block
#pragma unroll
            for (int jh = 0; jh < 2; ++jh) {
                f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = s;
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) {
                    const bf16x8 kb = *reinterpret_cast<const bf16x8*>(Kc + (16 * jh + lr) * LDQ + 32 * ks + 8 * lg);
                    const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vc + (16 * jh + lr) * LDQ + 32 * ks + 8 * lg);
                    s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kb, s, 0, 0, 0);
                    dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(df[ks], vb, dp, 0, 0, 0);
                }
                // C layout: [r] -> (i = q0 + 4 lg + r, j = j0 + 16 jh + lr)
                const int j = j0 + 16 * jh + lr;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = q0 + 4 * lg + r;
                    float ds = 0.f;
                    if (i < S && attn_allowed(i, j, S, L, Kimg)) {
                        const float p = __expf(s[r] * scale - lrow[r]);
                        float keep = 1.f;
                        if (drop_p > 0.f)
                            keep = hash_uniform(seed, (uint32_t)bh, (uint32_t)i, (uint32_t)j) < drop_p ? 0.f : inv_keep;
                        ds = p * (dp[r] * keep - drow[r]) * scale;
                    }
                    Ts[(4 * lg + r) * LDT + 16 * jh + lr] = f2bf(ds);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const bf16x8 sa = *reinterpret_cast<const bf16x8*>(Ts + lr * LDT + 8 * lg);
            const int jr = 8 * lg + tq;
#pragma unroll
            for (int db = 0; db < D / 16; ++db) {
                const bf16x8 kt = tr8(Kc + jr * LDQ + db * 16 + 4 * tp, Kc + (jr + 4) * LDQ + db * 16 + 4 * tp);
                qacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, kt, qacc[db], 0, 0, 0);
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (active) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = q0 + 4 * lg + r;
                if (i < S) {
                    bf16_t* row = dbase + (int64_t)i * rs3;
#pragma unroll
                    for (int db = 0; db < D / 16; ++db) row[db * 16 + lr] = f2bf(qacc[db][r]);
                }
            }
        }
    }
}

}  // namespace

extern "C" {

int rt1_attn_keepmask(uint8_t* keep, int BH, int S, float drop_p, uint32_t seed, const uint32_t* seed_dev,
                      hipStream_t st) {
    int64_t blocks = ((int64_t)BH * S * S + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(rt1_attn_keepmask_kernel, dim3((unsigned)blocks), dim3(256), 0, st, keep, BH, S, drop_p, seed,
                       seed_dev);
    return (int)hipGetLastError();
}

int rt1_attn_fwd(const bf16_t* qkv, bf16_t* out, float* lse, int B, int S, int H, int L, int Kimg, float scale,
                 float drop_p, uint32_t seed, const uint32_t* seed_dev, hipStream_t st) {
    if (S > 256 || S < 1) return (int)hipErrorInvalidValue;
    const int Sp = (S + 31) & ~31;
    // 8 waves per (batch, head) (2 workgroups / CU by LDS): the causal row blocks spread over twice the waves, and the
    // K / V^T staging runs on 512 threads (+0.1 % step, profiles/r5_attn_fwd_8w_ab.log); 4 waves where the 8 P tiles
    // overflow the 160 KB
    const size_t lds8 = (size_t)(Sp * D * 2 + 8 * 16 * Sp) * sizeof(bf16_t);
    const int nw = lds8 > 160 * 1024 ? 4 : 8;
    const size_t lds = (size_t)(Sp * D * 2 + nw * 16 * Sp) * sizeof(bf16_t);
#define LAUNCH(NKB)                                                                                                  \
    do {                                                                                                             \
        if (nw == 4)                                                                                                 \
            hipLaunchKernelGGL((rt1_attn_fwd_kernel<NKB, 4>), dim3(B * H), dim3(256), lds, st, qkv, out, lse, B, S, \
                               H, L, Kimg, scale, drop_p, seed, seed_dev);                                           \
        else                                                                                                         \
            hipLaunchKernelGGL((rt1_attn_fwd_kernel<NKB, 8>), dim3(B * H), dim3(512), lds, st, qkv, out, lse, B, S, \
                               H, L, Kimg, scale, drop_p, seed, seed_dev);                                           \
    } while (0)
    switch (Sp / 16) {
        case 2: LAUNCH(2); break;
        case 4: LAUNCH(4); break;
        case 6: LAUNCH(6); break;
        case 8: LAUNCH(8); break;
        case 10: LAUNCH(10); break;
        case 12: LAUNCH(12); break;
        case 14: LAUNCH(14); break;
        default: LAUNCH(16); break;
    }
#undef LAUNCH
    return (int)hipGetLastError();
}

size_t rt1_attn_bwd_lds(int S) {
    const int Sp = (S + 31) & ~31;
    return (size_t)(3 * Sp * LDQ + 2 * Sp * (Sp + 16)) * sizeof(bf16_t) + (size_t)Sp * sizeof(float);
}

int rt1_attn_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* dout, const float* lse, bf16_t* dqkv, int B,
                 int S, int H, int L, int Kimg, float scale, float drop_p, uint32_t seed, const uint32_t* seed_dev,
                 hipStream_t st) {
    if (S > BWD_MAX_S || S < 1) return (int)hipErrorInvalidValue;
    // 8 waves per (batch, head): the ~126 KB of LDS images allow one workgroup per CU, so the waves of that one
    // workgroup are the CU's whole occupancy; with 4 the causal row / key blocks ran 2 per wave (-0.35 % step,
    // profiles/r5_attn_bwd_8w_ab.log)
    hipLaunchKernelGGL(rt1_attn_bwd_kernel<8>, dim3(B * H), dim3(512), rt1_attn_bwd_lds(S), st, qkv, out, dout, lse,
                       dqkv, B, S, H, L, Kimg, scale, drop_p, seed, seed_dev);
    return (int)hipGetLastError();
}

// streamed two-kernel backward for any S <= 256 (used for S > 96, e.g. the T = 15 long-history config)
int rt1_attn_bwd_long(const bf16_t* qkv, const bf16_t* out, const bf16_t* dout, const float* lse, bf16_t* dqkv, int B,
                      int S, int H, int L, int Kimg, float scale, float drop_p, uint32_t seed,
                      const uint32_t* seed_dev, hipStream_t st) {
    if (S > 256 || S < 1) return (int)hipErrorInvalidValue;
    const int Sp = (S + 31) & ~31;
    const size_t lds_kv = (size_t)(2 * 32 * LDQ + 4 * 2 * 16 * LDT) * sizeof(bf16_t) + 2 * (size_t)Sp * sizeof(float);
    const size_t lds_q = (size_t)(2 * 32 * LDQ + 4 * 16 * LDT) * sizeof(bf16_t) + (size_t)Sp * sizeof(float);
    hipLaunchKernelGGL(rt1_attn_bwd_dkdv_kernel, dim3(B * H), dim3(256), lds_kv, st, qkv, out, dout, lse, dqkv, S, H,
                       L, Kimg, scale, drop_p, seed, seed_dev);
    hipLaunchKernelGGL(rt1_attn_bwd_dq_kernel, dim3(B * H), dim3(256), lds_q, st, qkv, out, dout, lse, dqkv, S, H, L,
                       Kimg, scale, drop_p, seed, seed_dev);
    return (int)hipGetLastError();
}

}  // extern "C"
