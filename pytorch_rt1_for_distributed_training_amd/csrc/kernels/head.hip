// Fused RT-1 action head: gather -> logits GEMM (MFMA) -> log-softmax -> CE -> argmax.
//
// Reference semantics (transformer.py:197, transformer_network.py:304-322): logits = Linear(512 -> V) over all
// T*L positions, then the T*A positions that predict action tokens are gathered and scored with
// cross_entropy(reduction='none').  Here the gather comes FIRST (18 of 66 rows at T=6), so the GEMM only
// touches the rows that are scored, and everything after the GEMM stays on chip:
//
//   rows  r = b*P + p  (P = T*A predicted positions), h_r = hidden[b, pos[p], :]  (fp32 residual stream)
//   z_r   = h_r W^T + bias                       (16 x V tile per workgroup, mfma_f32_16x16x32_bf16)
//   ce_r  = logsumexp(z_r) - z_r[target_r]       (fp32)
//   pred_r = argmax z_r                          (first maximum, like torch.argmax)
//   G_r   = softmax(z_r) - onehot(target_r)      (bf16, d ce_r / d z_r; the backward scales it by dce_r)
//   hb_r  = bf16(h_r)                            (the dW operand of the backward)
//
// Workgroup = 4 waves = 16 rows x V columns (V = 64 * NT): wave w owns columns [w*V/4, (w+1)*V/4).
// The 16 A rows are staged once in LDS as bf16; W (V x 512 bf16, L2-resident) is read straight from
// global as the B operand (16 B per lane, contiguous along K).  Row max / argmax / sum-exp are reduced
// with 16-lane shuffles inside a wave and through LDS across the 4 waves (fixed order: deterministic).
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int E = 512;          // token embedding (RT-1 d_model)
constexpr int LDA = E + 8;      // LDS row stride (bf16): shifts consecutive rows by 4 banks

template <int NT>               // 16-column MFMA tiles per wave: V = 4 waves * NT * 16
__global__ __launch_bounds__(256) void head_ce_fwd_kernel(const float* __restrict__ hidden, const int* __restrict__ pos,
                                                          const bf16_t* __restrict__ W, const float* __restrict__ bias,
                                                          const int* __restrict__ target, int R, int P, int S,
                                                          float* __restrict__ ce, int* __restrict__ pred,
                                                          bf16_t* __restrict__ G, bf16_t* __restrict__ hb) {
    constexpr int V = 64 * NT;
    __shared__ __attribute__((aligned(16))) bf16_t As[16 * LDA];
    __shared__ float red_m[4][16];
    __shared__ int red_i[4][16];
    __shared__ float red_s[4][16];
    __shared__ float tl[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r0 = blockIdx.x * 16;

    // ---- gather 16 rows (fp32) -> bf16 LDS tile + hb; 16 threads per row, 32 floats each
    {
        const int rr = tid >> 4, c0 = (tid & 15) * 32;
        const int r = r0 + rr;
        float v[32];
        if (r < R) {
            const int b = r / P, p = r - b * P;
            const int sp = min(max(pos[p], 0), S - 1);            // device-side guard: never read out of [0, S)
            const float* src = hidden + ((int64_t)b * S + sp) * E + c0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float t8[8];
                load8f(src + 8 * i, t8);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[8 * i + j] = t8[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float t8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) t8[j] = v[8 * i + j];
            store8(As + rr * LDA + c0 + 8 * i, t8);
            if (r < R) store8(hb + (int64_t)r * E + c0 + 8 * i, t8);
        }
    }
    if (tid < 16) tl[tid] = 0.f;
    __syncthreads();

    // ---- logits tile: acc[nt][i] = z[4*lg + i][col0 + 16*nt + lr]
    const int lr = lane & 15, lg = lane >> 4;
    const int col0 = wave * (V / 4);
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int ks = 0; ks < E / 32; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(As + lr * LDA + 32 * ks + 8 * lg);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const bf16x8 bw = *reinterpret_cast<const bf16x8*>(W + (int64_t)(col0 + 16 * nt + lr) * E + 32 * ks + 8 * lg);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw, acc[nt], 0, 0, 0);
        }
    }
    int tgt[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = r0 + 4 * lg + i;
        tgt[i] = r < R ? target[r] : -1;
    }
    float mx[4];
    int ix[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { mx[i] = -INFINITY; ix[i] = 0x7fffffff; }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = col0 + 16 * nt + lr;
        const float bc = bias[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float z = acc[nt][i] + bc;
            acc[nt][i] = z;
            if (z > mx[i]) { mx[i] = z; ix[i] = col; }     // columns increase with nt: strict > keeps the first
            if (col == tgt[i]) tl[4 * lg + i] = z;          // exactly one lane in the block owns the target
        }
    }
    // 16-lane (same lg) max/argmax
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const float om = __shfl_xor(mx[i], o, 64);
            const int oi = __shfl_xor(ix[i], o, 64);
            if (om > mx[i] || (om == mx[i] && oi < ix[i])) { mx[i] = om; ix[i] = oi; }
        }
    }
    if (lr == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) { red_m[wave][4 * lg + i] = mx[i]; red_i[wave][4 * lg + i] = ix[i]; }
    }
    __syncthreads();
    float gm[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 4 * lg + i;
        float m = red_m[0][row];
        int id = red_i[0][row];
#pragma unroll
        for (int w = 1; w < 4; ++w)
            if (red_m[w][row] > m) { m = red_m[w][row]; id = red_i[w][row]; }   // waves in column order
        gm[i] = m;
        ix[i] = id;
    }
    float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm[i] += __expf(acc[nt][i] - gm[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) sm[i] += __shfl_xor(sm[i], o, 64);
    if (lr == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) red_s[wave][4 * lg + i] = sm[i];
    }
    __syncthreads();
    float lse[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 4 * lg + i;
        const float s = red_s[0][row] + red_s[1][row] + red_s[2][row] + red_s[3][row];   // fixed order
        lse[i] = gm[i] + __logf(s);
    }
    if (wave == 0 && lr == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = r0 + 4 * lg + i;
            if (r < R) {
                ce[r] = lse[i] - tl[4 * lg + i];
                pred[r] = ix[i];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = r0 + 4 * lg + i;
        if (r >= R) continue;
        bf16_t* grow = G + (int64_t)r * V;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int col = col0 + 16 * nt + lr;
            const float g = __expf(acc[nt][i] - lse[i]) - (col == tgt[i] ? 1.f : 0.f);
            grow[col] = f2bf(g);
        }
    }
}

// dZ = G * dce[row] (bf16), the operand of both backward GEMMs
__global__ __launch_bounds__(256) void head_ce_scale_kernel(const bf16_t* __restrict__ G, const float* __restrict__ dce,
                                                            int R, int V, bf16_t* __restrict__ dz) {
    const int64_t n8 = (int64_t)R * V / 8;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        const int r = (int)((i * 8) / V);
        float v[8];
        load8(G + i * 8, v);
        const float s = dce[r];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= s;
        store8(dz + i * 8, v);
    }
}

// ---- action tokenization (reference tokenizers/action_tokenizer.py:105-128) in one launch: every
// (row, token) of the concatenated action tokens from its component -- Box: clamp to [low, high], normalise, scale by
// vocab - 1 and truncate (fp32, the reference's operation order); Discrete: the value itself.  Writes the int64 labels
// (aux / checkpoint-compatible) and the int32 copy the fused CE head reads.
struct TokArgs {
    const void* p[8];
    int kind[8];     // 0: Box fp32 [rows, dim], 1: Discrete int64 [rows], 2: Discrete int32 [rows]
    int dim[8];
    int off[8];      // first token of the component
    int n;
    float low[32], high[32];
};

__global__ __launch_bounds__(256) void action_tokenize_kernel(TokArgs a, int rows, int A, int V,
                                                              int64_t* __restrict__ out64, int* __restrict__ out32) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= rows * A) return;
    const int r = idx / A, j = idx - r * A;
    int c = 0;
    for (int i = 1; i < a.n; ++i)
        if (j >= a.off[i]) c = i;
    int tok;
    if (a.kind[c] == 0) {
        const int d = a.dim[c];
        float x = reinterpret_cast<const float*>(a.p[c])[(int64_t)r * d + (j - a.off[c])];
        const float lo = a.low[j], hi = a.high[j];
        x = fminf(fmaxf(x, lo), hi);
        tok = (int)((x - lo) / (hi - lo) * (float)(V - 1));
    } else if (a.kind[c] == 1) {
        tok = (int)reinterpret_cast<const int64_t*>(a.p[c])[r];
    } else {
        tok = reinterpret_cast<const int*>(a.p[c])[r];
    }
    out64[idx] = tok;
    out32[idx] = tok;
}

}  // namespace

extern "C" {

// comps: kind / dim per component as in TokArgs; low / high per token (Box tokens; ignored for Discrete)
int rt1_action_tokenize(const void* const* comps, const int* kind, const int* dim, int n, const float* low,
                        const float* high, int rows, int V, int64_t* out64, int* out32, hipStream_t st) {
    if (n < 1 || n > 8 || rows < 1 || V < 2) return (int)hipErrorInvalidValue;
    TokArgs a{};
    int A = 0;
    for (int i = 0; i < n; ++i) {
        a.p[i] = comps[i];
        a.kind[i] = kind[i];
        a.dim[i] = kind[i] == 0 ? dim[i] : 1;
        a.off[i] = A;
        A += a.dim[i];
    }
    if (A > 32) return (int)hipErrorInvalidValue;
    a.n = n;
    for (int j = 0; j < A; ++j) { a.low[j] = low[j]; a.high[j] = high[j]; }
    const int total = rows * A;
    hipLaunchKernelGGL(action_tokenize_kernel, dim3((total + 255) / 256), dim3(256), 0, st, a, rows, A, V, out64, out32);
    return (int)hipGetLastError();
}

int rt1_head_ce_supported(int V, int E_) { return E_ == E && (V == 256 || V == 512 || V == 1024) ? 1 : 0; }

int rt1_head_ce_fwd(const float* hidden, const int* pos, const bf16_t* W, const float* bias, const int* target, int R,
                    int P, int S, int V, float* ce, int* pred, bf16_t* G, bf16_t* hb, hipStream_t st) {
    if (R <= 0 || P <= 0 || S <= 0) return (int)hipErrorInvalidValue;
    const dim3 grid((R + 15) / 16), block(256);
    switch (V) {
        case 256: hipLaunchKernelGGL(head_ce_fwd_kernel<4>, grid, block, 0, st, hidden, pos, W, bias, target, R, P, S,
                                     ce, pred, G, hb); break;
        case 512: hipLaunchKernelGGL(head_ce_fwd_kernel<8>, grid, block, 0, st, hidden, pos, W, bias, target, R, P, S,
                                     ce, pred, G, hb); break;
        case 1024: hipLaunchKernelGGL(head_ce_fwd_kernel<16>, grid, block, 0, st, hidden, pos, W, bias, target, R, P,
                                      S, ce, pred, G, hb); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int rt1_head_ce_scale(const bf16_t* G, const float* dce, int R, int V, bf16_t* dz, hipStream_t st) {
    if (V % 8) return (int)hipErrorInvalidValue;
    int64_t blocks = ((int64_t)R * V / 8 + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(head_ce_scale_kernel, dim3((unsigned)blocks), dim3(256), 0, st, G, dce, R, V, dz);
    return (int)hipGetLastError();
}

}  // extern "C"
