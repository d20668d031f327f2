// TokenLearner, one workgroup per frame, forward and backward.
//
// Spec (tokenizers/token_learner.py:64-95): x [P, C=512] (P = h*w feature positions of one frame)
//   xn = LayerNorm_C(x);  z1 = xn W1^T + b1 (C -> 64);  h = GELU_tanh(z1);  a = h W2^T + b2 (64 -> T=8)
//   s[t, :] = softmax_P(a[:, t]);  out[t, c] = sum_p s[t, p] x[p, c]        (pooling of the UN-normalised x)
//
// Forward (tl_fwd_kernel): LN statistics (wave per row, centred two-pass in registers) -> z1 on MFMA
// (mfma_f32_16x16x32_bf16, LN applied to the A operand as it is loaded, W1 streamed from L2) -> h in LDS ->
// the 8 logits per position on the VALU -> softmax over P (wave per token) -> pooling (thread per channel
// pair, x rows read once, coalesced).  Saved for backward: mu, rstd [P], z1 (bf16) [P, 64], s [T, P].
//
// Backward (tl_bwd_kernel), given dO [T, C]:
//   dS[t, p] = dO_t . x_p  (wave per row, dO held in registers)      da = s * (dS - sum_p s dS)   (softmax)
//   dW2 / db2 per-frame partials;  dz1 = (da^T W2) * gelu'(z1)  (-> LDS + global, for dW1 on hipBLASLt)
//   dxn = dz1 W1 on MFMA, 16 rows x 512 columns per wave (128 accumulator registers), then LayerNorm
//   backward from the row sums of dxn*gamma and dxn*gamma*xhat, plus the pooling path s^T dO:
//   dx = rstd (g - mean g - xhat mean(g xhat)) + sum_t s[t, p] dO[t, c];  dgamma / dbeta per-frame partials;
//   xn (bf16) for dW1 = dz1^T xn.
// Per-frame partials are summed on the host in a fixed order: no atomics, bitwise reproducible.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int C = 512;       // RT-1 token embedding
constexpr int H1 = 64;       // bottleneck
constexpr int T = 8;         // tokens
constexpr int PMAX = 256;    // positions per frame (10x10 / 8x15 / 15x15 maps)
constexpr int LDZ = H1 + 8;  // LDS row stride of z1 / dz1 tiles (bf16)

__device__ __forceinline__ float gelu_tanh(float z) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (z + k1 * z * z * z);
    return 0.5f * z * (1.f + tanhf(u));
}

__global__ __launch_bounds__(256) void tl_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     const bf16_t* __restrict__ W1, const float* __restrict__ b1,
                                                     const float* __restrict__ W2, const float* __restrict__ b2, int P,
                                                     bf16_t* __restrict__ out, float* __restrict__ mu_o,
                                                     float* __restrict__ rs_o, bf16_t* __restrict__ z1_o,
                                                     float* __restrict__ s_o) {
    __shared__ float mu[PMAX], rs[PMAX];
    __shared__ __attribute__((aligned(16))) float gam[C], bet[C];
    __shared__ float Hs[PMAX][H1 + 1];
    __shared__ float Sl[T][PMAX];
    const int n = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bf16_t* xf = x + (int64_t)n * P * C;
    for (int c = tid; c < C; c += 256) { gam[c] = gamma[c]; bet[c] = beta[c]; }
    // ---- LayerNorm statistics: wave per row, 8 channels per lane
    for (int p = wave; p < P; p += 4) {
        float v[8];
        load8(xf + (int64_t)p * C + 8 * lane, v);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
        const float m = wave_sum(s) * (1.f / C);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) q += (v[j] - m) * (v[j] - m);
        const float var = wave_sum(q) * (1.f / C);
        if (lane == 0) {
            mu[p] = m;
            rs[p] = rsqrtf(var + eps);
        }
    }
    __syncthreads();
    for (int p = tid; p < P; p += 256) {
        mu_o[(int64_t)n * P + p] = mu[p];
        rs_o[(int64_t)n * P + p] = rs[p];
    }
    // ---- z1 = LN(x) W1^T + b1 on MFMA; h = gelu(z1) -> LDS
    const int lr = lane & 15, lg = lane >> 4;
    const int nrb = (P + 15) / 16;
    for (int rb = wave; rb < nrb; rb += 4) {
        const int p0 = rb * 16;
        const int pa = p0 + lr;
        f32x4 acc[H1 / 16];
#pragma unroll
        for (int nt = 0; nt < H1 / 16; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float m = pa < P ? mu[pa] : 0.f, r = pa < P ? rs[pa] : 0.f;
#pragma unroll 2
        for (int ks = 0; ks < C / 32; ++ks) {
            const int c0 = 32 * ks + 8 * lg;
            float v[8];
            if (pa < P) {
                load8(xf + (int64_t)pa * C + c0, v);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (v[j] - m) * r * gam[c0 + j] + bet[c0 + j];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = 0.f;
            }
            bf16_t ab[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) ab[j] = f2bf(v[j]);
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(ab);
#pragma unroll
            for (int nt = 0; nt < H1 / 16; ++nt) {
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(W1 + (int64_t)(16 * nt + lr) * C + c0);
                acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[nt], 0, 0, 0);
            }
        }
        // C layout: acc[nt][i] = z1[p0 + 4 lg + i][16 nt + lr]
#pragma unroll
        for (int nt = 0; nt < H1 / 16; ++nt) {
            const int j = 16 * nt + lr;
            const float bj = b1[j];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int p = p0 + 4 * lg + i;
                if (p < P) {
                    const bf16_t zb = f2bf(acc[nt][i] + bj);
                    z1_o[((int64_t)n * P + p) * H1 + j] = zb;
                    Hs[p][j] = gelu_tanh(bf2f(zb));      // from the stored bf16 z1: the backward recomputes it
                }
            }
        }
    }
    __syncthreads();
    // ---- logits a[t, p] = h_p . W2_t + b2_t
    for (int idx = tid; idx < P * T; idx += 256) {
        const int t = idx % T, p = idx / T;
        const float* w = W2 + t * H1;
        float s = b2[t];
#pragma unroll 8
        for (int j = 0; j < H1; ++j) s = fmaf(Hs[p][j], w[j], s);
        Sl[t][p] = s;
    }
    __syncthreads();
    // ---- softmax over positions, wave per token
    for (int t = wave; t < T; t += 4) {
        float m = -INFINITY;
        for (int p = lane; p < P; p += 64) m = fmaxf(m, Sl[t][p]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float s = 0.f;
        for (int p = lane; p < P; p += 64) {
            const float e = __expf(Sl[t][p] - m);
            Sl[t][p] = e;
            s += e;
        }
        const float inv = 1.f / wave_sum(s);
        for (int p = lane; p < P; p += 64) {
            const float v = Sl[t][p] * inv;
            Sl[t][p] = v;
            s_o[((int64_t)n * T + t) * P + p] = v;
        }
    }
    __syncthreads();
    // ---- pooling: thread = channel pair, all 8 tokens
    const int c = 2 * tid;
    float acc0[T], acc1[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc0[t] = acc1[t] = 0.f;
    for (int p = 0; p < P; ++p) {
        const uint32_t u = *reinterpret_cast<const uint32_t*>(xf + (int64_t)p * C + c);
        const float x0 = __uint_as_float(u << 16), x1 = __uint_as_float(u & 0xffff0000u);
#pragma unroll
        for (int t = 0; t < T; ++t) {
            acc0[t] = fmaf(Sl[t][p], x0, acc0[t]);
            acc1[t] = fmaf(Sl[t][p], x1, acc1[t]);
        }
    }
#pragma unroll
    for (int t = 0; t < T; ++t)
        *reinterpret_cast<uint32_t*>(out + ((int64_t)n * T + t) * C + c) = pack2(acc0[t], acc1[t]);
}

// PM: positions the LDS tiles are sized for (128 covers the 10x10 map of 300x300 frames: 58 KB of LDS, two
// workgroups per CU; 256 for the larger maps).  The dxn MFMA tile is produced in two 256-column halves (64 accumulator
// registers instead of 128) and recomputed for the output pass: one wave holding all 512 columns spilled 528 B/lane
// and ran at one wave per SIMD.
template <int PM>
__global__ __launch_bounds__(256, 2) void tl_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dO,
                                                     const float* __restrict__ S, const bf16_t* __restrict__ z1,
                                                     const float* __restrict__ mu, const float* __restrict__ rs,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     const bf16_t* __restrict__ W1T, const float* __restrict__ W2,
                                                     int P, bf16_t* __restrict__ dx, bf16_t* __restrict__ dz1_o,
                                                     bf16_t* __restrict__ xn_o, float* __restrict__ pw2,
                                                     float* __restrict__ pg) {
    __shared__ float dOs[T][C];
    __shared__ float Ss[T][PM];
    __shared__ float dSs[T][PM];
    __shared__ __attribute__((aligned(16))) bf16_t Dz[PM * LDZ];
    __shared__ float red[4][2][C];
    __shared__ __attribute__((aligned(16))) float gbs[2][C];     // LayerNorm gamma / beta
    __shared__ float pwr[4][T][H1];                                 // dW2 partials of the 4 position groups
    const int n = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bf16_t* xf = x + (int64_t)n * P * C;
    for (int i = tid; i < T * C; i += 256) dOs[i / C][i % C] = bf2f(dO[(int64_t)n * T * C + i]);
    for (int i = tid; i < T * P; i += 256) Ss[i / P][i % P] = S[(int64_t)n * T * P + i];
    for (int i = tid; i < 4 * 2 * C; i += 256) (&red[0][0][0])[i] = 0.f;
    for (int i = tid; i < C; i += 256) {
        gbs[0][i] = gamma[i];
        gbs[1][i] = beta[i];
    }
    __syncthreads();
    // ---- dS[t, p] = dO_t . x_p on MFMA: 16-position blocks per wave, A = the dO rows (tokens; zero from T to 16),
    // B = the x rows; lane (lr, lg) ends with dS[4 lg + r][p0 + lr].  (It was a wave per position with 8 wave-wide
    // shuffle reductions per row.)
    {
        const int lr = lane & 15, lg = lane >> 4;
        const bf16_t* dof = dO + (int64_t)n * T * C;
        const bf16x8 zero8 = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        for (int rb = wave; rb < (P + 15) / 16; rb += 4) {
            const int p0 = rb * 16;
            const bool pok = p0 + lr < P;
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
            for (int ks = 0; ks < C / 32; ++ks) {
                const bf16x8 av = lr < T ? *reinterpret_cast<const bf16x8*>(dof + lr * C + 32 * ks + 8 * lg) : zero8;
                const bf16x8 bv = pok ? *reinterpret_cast<const bf16x8*>(xf + (int64_t)(p0 + lr) * C + 32 * ks + 8 * lg)
                                      : zero8;
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
            }
            if (lg < T / 4 && pok) {
#pragma unroll
                for (int r = 0; r < 4; ++r) dSs[4 * lg + r][p0 + lr] = acc[r];
            }
        }
    }
    __syncthreads();
    // ---- softmax backward, wave per token: da = s (dS - <s, dS>)
    for (int t = wave; t < T; t += 4) {
        float d = 0.f;
        for (int p = lane; p < P; p += 64) d = fmaf(Ss[t][p], dSs[t][p], d);
        d = wave_sum(d);
        for (int p = lane; p < P; p += 64) dSs[t][p] = Ss[t][p] * (dSs[t][p] - d);
    }
    __syncthreads();
    const bf16_t* zf = z1 + (int64_t)n * P * H1;
    // ---- dW2 / db2 partials and dz1 = (da^T W2) * gelu'(z1) in ONE pass over z1: thread = (column j, position
    // group pg), one tanh per (p, j) for both gelu(z1) and gelu'(z1) (the dW2 loop had recomputed gelu for every
    // token pair: 4 tanh per element, plus one more in the dz1 loop); the 4 position groups' dW2 partials combine
    // through LDS in a fixed order
    {
        const int j = tid & 63, pg = tid >> 6;
        const float k0 = 0.7978845608028654f, k1 = 0.044715f;
        float w2[T], aw[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            w2[t] = W2[t * H1 + j];
            aw[t] = 0.f;
        }
        for (int p = pg; p < P; p += 4) {
            const float z = bf2f(zf[(int64_t)p * H1 + j]);
            const float th = tanhf(k0 * (z + k1 * z * z * z));
            const float hz = 0.5f * z * (1.f + th);
            const float gd = 0.5f * (1.f + th) + 0.5f * z * (1.f - th * th) * k0 * (1.f + 3.f * k1 * z * z);
            float dh = 0.f;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const float ds = dSs[t][p];
                aw[t] = fmaf(ds, hz, aw[t]);
                dh = fmaf(ds, w2[t], dh);
            }
            const bf16_t d = f2bf(dh * gd);
            Dz[p * LDZ + j] = d;
            dz1_o[((int64_t)n * P + p) * H1 + j] = d;
        }
#pragma unroll
        for (int t = 0; t < T; ++t) pwr[pg][t][j] = aw[t];
        __syncthreads();
        for (int i = tid; i < T * H1; i += 256) {
            const int t = i / H1, jj = i - t * H1;
            pw2[((int64_t)n * T + t) * (H1 + 1) + jj] = ((pwr[0][t][jj] + pwr[1][t][jj]) + pwr[2][t][jj]) + pwr[3][t][jj];
        }
        if (tid < T) {
            float s = 0.f;
            for (int p = 0; p < P; ++p) s += dSs[tid][p];
            pw2[((int64_t)n * T + tid) * (H1 + 1) + H1] = s;
        }
    }
    __syncthreads();
    // ---- dxn = dz1 W1 (MFMA, 16 rows x 256 columns per wave and pass) -> LayerNorm backward + pooling path
    // The product is formed transposed (W1 rows as the MFMA's first operand), so a lane holds 4 CONSECUTIVE columns
    // of one row: x is read and dx / xn are written as 8-byte vectors (they were 2-byte loads and stores of one
    // element per lane and row: the kernel waited on memory 76 % of its cycles, profiles/r6_sq_step.txt).
    const int lr = lane & 15, lg = lane >> 4;
    const int nrb = (P + 15) / 16;
    constexpr int HC = C / 2;                    // columns per half
    auto dxn_half = [&](int p0, int half, f32x4 (&acc)[HC / 16]) {
#pragma unroll
        for (int ct = 0; ct < HC / 16; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < H1 / 32; ++ks) {
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(Dz + (p0 + lr) * LDZ + 32 * ks + 8 * lg);
#pragma unroll
            for (int ct = 0; ct < HC / 16; ++ct) {
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(W1T + (int64_t)(half * HC + 16 * ct + lr) * H1 +
                                                                  32 * ks + 8 * lg);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[ct], 0, 0, 0);
            }
        }
    };
    for (int rb = wave; rb < nrb; rb += 4) {
        const int p0 = rb * 16;
        const int p = p0 + lr;                   // this lane's row
        const bool ok = p < P;
        const float m = ok ? mu[(int64_t)n * P + p] : 0.f;
        const float r = ok ? rs[(int64_t)n * P + p] : 0.f;
        const bf16_t* xrow = xf + (int64_t)(ok ? p : 0) * C;
        f32x4 acc[HC / 16];
        // C layout: acc[ct][i] = dxn[p0 + lr][half * 256 + 16 ct + 4 lg + i].  Pass 1: row sums of g and g * xhat.
        float sg = 0.f, sgx = 0.f;
        for (int half = 0; half < 2; ++half) {
            dxn_half(p0, half, acc);
            // fully unrolled: a partially unrolled ct loop indexes acc[] at run time, which puts the MFMA results
            // in scratch memory
#pragma unroll
            for (int ct = 0; ct < HC / 16; ++ct) {
                const int c = half * HC + 16 * ct + 4 * lg;
                const float4 gm = *reinterpret_cast<const float4*>(&gbs[0][c]);
                const uint2 xu = ok ? *reinterpret_cast<const uint2*>(xrow + c) : make_uint2(0u, 0u);
                const float xv[4] = {__uint_as_float(xu.x << 16), __uint_as_float(xu.x & 0xffff0000u),
                                     __uint_as_float(xu.y << 16), __uint_as_float(xu.y & 0xffff0000u)};
                const float gv[4] = {gm.x, gm.y, gm.z, gm.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float xh = (xv[i] - m) * r;
                    const float g = acc[ct][i] * gv[i];
                    sg += g;
                    sgx = fmaf(g, xh, sgx);
                }
            }
        }
        // the row's 512 columns are spread over the 4 lane groups of its lr
        sg += __shfl_xor(sg, 16, 64);
        sg += __shfl_xor(sg, 32, 64);
        sgx += __shfl_xor(sgx, 16, 64);
        sgx += __shfl_xor(sgx, 32, 64);
        sg *= (1.f / C);
        sgx *= (1.f / C);
        float st[T];
#pragma unroll
        for (int t = 0; t < T; ++t) st[t] = ok ? Ss[t][p] : 0.f;
        // Pass 2 (dxn recomputed per half): dx, xn, dgamma / dbeta column partials
        for (int half = 0; half < 2; ++half) {
            dxn_half(p0, half, acc);
#pragma unroll
            for (int ct = 0; ct < HC / 16; ++ct) {
                const int c = half * HC + 16 * ct + 4 * lg;
                const float4 gm4 = *reinterpret_cast<const float4*>(&gbs[0][c]);
                const float4 bt4 = *reinterpret_cast<const float4*>(&gbs[1][c]);
                const uint2 xu = ok ? *reinterpret_cast<const uint2*>(xrow + c) : make_uint2(0u, 0u);
                const float xv[4] = {__uint_as_float(xu.x << 16), __uint_as_float(xu.x & 0xffff0000u),
                                     __uint_as_float(xu.y << 16), __uint_as_float(xu.y & 0xffff0000u)};
                const float gv[4] = {gm4.x, gm4.y, gm4.z, gm4.w}, bv[4] = {bt4.x, bt4.y, bt4.z, bt4.w};
                float pool[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const float4 d4 = *reinterpret_cast<const float4*>(&dOs[t][c]);
                    pool[0] = fmaf(st[t], d4.x, pool[0]);
                    pool[1] = fmaf(st[t], d4.y, pool[1]);
                    pool[2] = fmaf(st[t], d4.z, pool[2]);
                    pool[3] = fmaf(st[t], d4.w, pool[3]);
                }
                float dxv[4], xnv[4], dgs[4], dbs[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float xh = (xv[i] - m) * r;
                    const float d = ok ? acc[ct][i] : 0.f;
                    dxv[i] = r * (d * gv[i] - sg - xh * sgx) + pool[i];
                    xnv[i] = xh * gv[i] + bv[i];
                    dgs[i] = d * xh;
                    dbs[i] = d;
                }
                if (ok) {
                    const int64_t off = ((int64_t)n * P + p) * C + c;
                    *reinterpret_cast<uint2*>(dx + off) = make_uint2(pack2(dxv[0], dxv[1]), pack2(dxv[2], dxv[3]));
                    *reinterpret_cast<uint2*>(xn_o + off) = make_uint2(pack2(xnv[0], xnv[1]), pack2(xnv[2], xnv[3]));
                }
                // column sums over the 16 rows of the block (the lr lanes of this lane group), fixed xor order
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) {
                        dgs[i] += __shfl_xor(dgs[i], o, 64);
                        dbs[i] += __shfl_xor(dbs[i], o, 64);
                    }
                }
                if (lr == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        red[wave][0][c + i] += dgs[i];
                        red[wave][1][c + i] += dbs[i];
                    }
                }
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < 2 * C; i += 256) {
        const int k = i / C, c = i % C;
        pg[((int64_t)n * 2 + k) * C + c] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    }
}

}  // namespace

extern "C" {

int rt1_tl_supported(int P, int Cc, int h1, int t) { return (P >= 1 && P <= PMAX && Cc == C && h1 == H1 && t == T) ? 1 : 0; }

int rt1_tl_fwd(const bf16_t* x, const float* gamma, const float* beta, float eps, const bf16_t* W1, const float* b1,
               const float* W2, const float* b2, int N, int P, bf16_t* out, float* mu, float* rs, bf16_t* z1,
               float* s, hipStream_t st) {
    if (N <= 0 || P < 1 || P > PMAX) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(tl_fwd_kernel, dim3(N), dim3(256), 0, st, x, gamma, beta, eps, W1, b1, W2, b2, P, out, mu, rs,
                       z1, s);
    return (int)hipGetLastError();
}

int rt1_tl_bwd(const bf16_t* x, const bf16_t* dO, const float* s, const bf16_t* z1, const float* mu, const float* rs,
               const float* gamma, const float* beta, const bf16_t* W1T, const float* W2, int N, int P, bf16_t* dx,
               bf16_t* dz1, bf16_t* xn, float* pw2, float* pg, hipStream_t st) {
    if (N <= 0 || P < 1 || P > PMAX) return (int)hipErrorInvalidValue;
if (P <= 128)
        hipLaunchKernelGGL(tl_bwd_kernel<128>, dim3(N), dim3(256), 0, st, x, dO, s, z1, mu, rs, gamma, beta, W1T, W2, P, dx,
                       dz1, xn, pw2, pg);
    else
        hipLaunchKernelGGL(tl_bwd_kernel<PMAX>, dim3(N), dim3(256), 0, st, x, dO, s, z1, mu, rs, gamma, beta, W1T, W2, P, dx,
                       dz1, xn, pw2, pg);
    return (int)hipGetLastError();
}

}  // extern "C"
