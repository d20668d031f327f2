// Tall-skinny pointwise GEMM on MFMA: C[M, N] = A[M, K] @ W[N, K]^T for the mid/low-resolution 1x1 convs of
// FiLM-EfficientNet-B3 where the reduction is WIDE and the output NARROW: project convs (K = 576..2304 ->
// N = 96..384) and the data-gradient of the expand convs (K = Ce -> N = Cin).  
//
// Every shape is HBM-bound on A (e.g. 277k x 816 bf16 = 452 MB against a 136-column output); hipBLASLt's macro
// tiles reach 37-42 % of the HBM roofline here because N = 96 / 136 / 232 is far from its 128 / 256-wide tiles.
//
// Design (CDNA4, wave64, mfma_f32_16x16x32_bf16):
//   * A workgroup owns BM = 4 waves x RB x 16 rows and ALL N columns (padded to NT x 16) for N <= 144, so A is
//     read from HBM exactly once; wider outputs are cut into 128-column slices whose workgroups run on one
//     XCD together and share A through its L2.  Each wave keeps RB x NT accumulators (<= 128 VGPRs).
//   * W streams through LDS in 32-wide K chunks, double-buffered: the next chunk's W pieces and the next A
//     fragments are loaded into registers while the current chunk's MFMAs run, one barrier per chunk.
//     W (<= 1.8 MB) stays L2-resident; each workgroup reads it once per BM rows.
//   * The product is computed transposed, C^T = W . A^T (MFMA-A = W rows from LDS, MFMA-B = A rows straight
//     from HBM in operand layout), so each accumulator holds 4 consecutive output channels of one pixel and a
//     lane stores 8 contiguous bytes.
//   * K and N tails (K = 816 = 25.5 x 32, N = 136 / 232) are zero-filled at load time; no padding in memory.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int LDW = 40;   // LDS row stride of a W chunk (bf16): 32 + 8 -> rows land 16 B apart in the banks
constexpr int PRO_KMAX = 2304;   // widest K the operand prologue stages its per-channel constants for

// Project-conv operand prologue (PRO): A is the depthwise output y2 and the GEMM consumes
//     a = silu(y2 * scale[k] + shift[k]) * gate[row / hw, k]
// rebuilt in registers as each A fragment arrives (same formula and rounding as bn_apply, so bit-identical);
// aout (optional) also stores a for the weight gradient.  Replaces the bn_apply pass (read y2, write a) + the GEMM's
// read of a with one read of y2 (+ the a store).
struct TallPro {
    const float *scale, *shift, *gate;
    int hw;
    bf16_t* aout;
};

// Second reduction segment (TAIL, y-free expand backward of the wide blocks): C = A @ W^T + A2 @ W2^T + bias2 with
// A2 [M, K2], W2 [N, K2] bf16; the K loop runs over both segments' 32-wide chunks (the segment of a chunk only
// switches the wave-uniform base pointers and row strides, so the loads keep the plain kernel's registers).
struct TallTail {
    const bf16_t* A2;
    const bf16_t* W2;
    const float* bias;
    int K2;
    const bf16_t* res;   // optional residual: C += res[m, n] * rmul[m / rhw, n] (the block's skip-path gradient)
    const float* rmul;
    int rhw;
};

// EPI 0: C bf16.  EPI 1 (transformer token embedding): Cf fp32 = acc + bias[n] + pos[(m % S), n].
template <int NT, int RB, int EPI, bool PRO, bool TAIL = false>
__global__ __launch_bounds__(256, 2) void pw_tall_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                         int M, int K, int N, bf16_t* __restrict__ C,
                                                         const float* __restrict__ bias, const float* __restrict__ pos,
                                                         int S, float* __restrict__ Cf, TallPro pro, TallTail tl) {
    constexpr int NP = NT * 16;
    constexpr int PIECES = NP * 4;                    // 16-byte pieces of one [NP x 32] W chunk
    constexpr int PPT = (PIECES + 255) / 256;
    __shared__ __attribute__((aligned(16))) bf16_t Ws[2][NP * LDW];
    __shared__ __attribute__((aligned(16))) float prc[PRO ? 2 * PRO_KMAX : 1];   // scale | shift
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 15, lg = lane >> 4;
    // XCD-aware tile order: workgroup b runs on XCD b % 8; the ns N-slices of one row tile get ids 8 apart so
    // they share an XCD (and its L2) and are dispatched together -> A is fetched from HBM once per row tile
    const int ns = (N + NP - 1) / NP;
    const int b = blockIdx.x, grp = b / (8 * ns), rem = b % (8 * ns);
    const int tile = grp * 8 + (rem & 7);
    const int nb = (rem >> 3) * NP;                   // first output channel of this workgroup's N slice
    if ((int64_t)tile * (4 * RB * 16) >= M) return;  // whole workgroup: tile-count padding to a multiple of 8
    const int64_t m0 = (int64_t)tile * (4 * RB * 16) + wave * RB * 16;
    const int nk1 = (K + 31) / 32;
    const int nk = nk1 + (TAIL ? (tl.K2 + 31) / 32 : 0);
    // PRO: per-channel constants in LDS (read by the barrier below); this lane's RB gate rows (frame of each row)
    int64_t grow[PRO ? RB : 1];
    if constexpr (PRO) {
        for (int i = tid; i < K; i += 256) {
            prc[i] = pro.scale[i];
            prc[PRO_KMAX + i] = pro.shift[i];
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int64_t row = m0 + 16 * r + lr;
            grow[r] = (row < M ? row / pro.hw : 0) * (int64_t)K;
        }
    }

    uint4 wreg[PPT];
    auto load_w = [&](int kc) {
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int v = tid + 256 * i;
            const bool t2 = TAIL && kc >= nk1;
            const bf16_t* Wb = t2 ? tl.W2 : W;
            const int KK = t2 ? tl.K2 : K;
            const int row = nb + (v >> 2), k = (t2 ? kc - nk1 : kc) * 32 + (v & 3) * 8;
            wreg[i] = make_uint4(0, 0, 0, 0);
            if (v < PIECES && row < N && k < KK) wreg[i] = *reinterpret_cast<const uint4*>(Wb + (int64_t)row * KK + k);
        }
    };
    auto store_w = [&](int buf) {
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int v = tid + 256 * i;
            if (v < PIECES) *reinterpret_cast<uint4*>(&Ws[buf][(v >> 2) * LDW + (v & 3) * 8]) = wreg[i];
        }
    };
    float4 gv[PRO ? RB : 1][2];                       // PRO: gate values of the fragments in flight
    auto load_a = [&](int kc, bf16x8 (&dst)[RB]) {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int64_t row = m0 + 16 * r + lr;
            const bool t2 = TAIL && kc >= nk1;
            const bf16_t* Ab = t2 ? tl.A2 : A;
            const int KK = t2 ? tl.K2 : K;
            const int k = (t2 ? kc - nk1 : kc) * 32 + 8 * lg;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (row < M && k < KK) u = *reinterpret_cast<const uint4*>(Ab + row * KK + k);
            dst[r] = *reinterpret_cast<bf16x8*>(&u);
            if constexpr (PRO) {
                gv[r][0] = gv[r][1] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (row < M && k < K) {
                    gv[r][0] = *reinterpret_cast<const float4*>(pro.gate + grow[r] + k);
                    gv[r][1] = *reinterpret_cast<const float4*>(pro.gate + grow[r] + k + 4);
                }
            }
        }
    };
    // PRO: a = silu(y * scale + shift) * gate on the fragments of chunk kc (and their store for the weight gradient)
    auto prologue = [&](int kc, bf16x8 (&frag)[RB]) {
        if constexpr (PRO) {
            const int k = kc * 32 + 8 * lg;
            if (k >= K) return;
            float sc[8], sh[8];
            load8f(prc + k, sc);
            load8f(prc + PRO_KMAX + k, sh);
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int64_t row = m0 + 16 * r + lr;
                float x[8];
                unpack8(__builtin_bit_cast(uint4, frag[r]), x);
                const float g[8] = {gv[r][0].x, gv[r][0].y, gv[r][0].z, gv[r][0].w,
                                    gv[r][1].x, gv[r][1].y, gv[r][1].z, gv[r][1].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = silu(fmaf(x[j], sc[j], sh[j])) * g[j];
                uint4 u;
                u.x = pack2(x[0], x[1]); u.y = pack2(x[2], x[3]); u.z = pack2(x[4], x[5]); u.w = pack2(x[6], x[7]);
                if (row >= M) u = make_uint4(0, 0, 0, 0);
                frag[r] = __builtin_bit_cast(bf16x8, u);
                // one N slice stores the operand (the others rebuild the same rows)
                if (pro.aout && nb == 0 && row < M) *reinterpret_cast<uint4*>(pro.aout + row * K + k) = u;
            }
        }
    };

    f32x4 acc[RB][NT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 af[RB], an[RB];
    load_w(0);
    store_w(0);
    load_a(0, af);
    __syncthreads();                                   // also publishes the PRO constants
    prologue(0, af);
    for (int kc = 0; kc < nk; ++kc) {
        const int buf = kc & 1;
        const bool more = kc + 1 < nk;
        if (more) {
            load_w(kc + 1);
            load_a(kc + 1, an);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const bf16x8 wf = *reinterpret_cast<const bf16x8*>(&Ws[buf][(16 * t + lr) * LDW + 8 * lg]);
#pragma unroll
            for (int r = 0; r < RB; ++r) acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, af[r], acc[r][t], 0, 0, 0);
        }
        if (more) {
            store_w(buf ^ 1);                  // buf ^ 1 was last read before the previous barrier
            prologue(kc + 1, an);
#pragma unroll
            for (int r = 0; r < RB; ++r) af[r] = an[r];
        }
        __syncthreads();
    }
    // acc[r][t][i] = C[m0 + 16 r + lr][nb + 16 t + 4 lg + i]
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int64_t m = m0 + 16 * r + lr;
        if (m >= M) continue;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int n = nb + 16 * t + 4 * lg;
            if (n < N) {
                if constexpr (EPI == 0) {
                    if constexpr (TAIL) {
                        const float4 b = *reinterpret_cast<const float4*>(tl.bias + n);
                        acc[r][t][0] += b.x; acc[r][t][1] += b.y; acc[r][t][2] += b.z; acc[r][t][3] += b.w;
                        if (tl.res) {
                            const uint2 d = *reinterpret_cast<const uint2*>(tl.res + m * N + n);
                            const float4 f = *reinterpret_cast<const float4*>(tl.rmul + (m / tl.rhw) * N + n);
                            acc[r][t][0] = fmaf(__uint_as_float(d.x << 16), f.x, acc[r][t][0]);
                            acc[r][t][1] = fmaf(__uint_as_float(d.x & 0xffff0000u), f.y, acc[r][t][1]);
                            acc[r][t][2] = fmaf(__uint_as_float(d.y << 16), f.z, acc[r][t][2]);
                            acc[r][t][3] = fmaf(__uint_as_float(d.y & 0xffff0000u), f.w, acc[r][t][3]);
                        }
                    }
                    uint2 o;
                    o.x = pack2(acc[r][t][0], acc[r][t][1]);
                    o.y = pack2(acc[r][t][2], acc[r][t][3]);
                    *reinterpret_cast<uint2*>(C + m * N + n) = o;
                } else {
                    const float4 b = *reinterpret_cast<const float4*>(bias + n);
                    const float4 q = *reinterpret_cast<const float4*>(pos + (int64_t)(m % S) * N + n);
                    float4 o;
                    o.x = acc[r][t][0] + b.x + q.x;
                    o.y = acc[r][t][1] + b.y + q.y;
                    o.z = acc[r][t][2] + b.z + q.z;
                    o.w = acc[r][t][3] + b.w + q.w;
                    *reinterpret_cast<float4*>(Cf + m * N + n) = o;
                }
            }
        }
    }
}

template <int NT, int RB, int EPI = 0>
int launch_tall(const bf16_t* A, const bf16_t* W, int M, int K, int N, bf16_t* C, hipStream_t st,
                const float* bias = nullptr, const float* pos = nullptr, int S = 1, float* Cf = nullptr,
                TallPro pro = TallPro{nullptr, nullptr, nullptr, 1, nullptr},
                TallTail tl = TallTail{nullptr, nullptr, nullptr, 0, nullptr, nullptr, 1}) {
    const int bm = 4 * RB * 16;
    const int tiles = ((M + bm - 1) / bm + 7) / 8 * 8, ns = (N + NT * 16 - 1) / (NT * 16);
    const dim3 grid(tiles * ns);
    if (pro.scale)
        hipLaunchKernelGGL((pw_tall_kernel<NT, RB, EPI, true>), grid, dim3(256), 0, st, A, W, M, K, N, C, bias, pos, S,
                           Cf, pro, tl);
    else if (tl.A2)
        hipLaunchKernelGGL((pw_tall_kernel<NT, RB, EPI, false, true>), grid, dim3(256), 0, st, A, W, M, K, N, C, bias,
                           pos, S, Cf, pro, tl);
    else
        hipLaunchKernelGGL((pw_tall_kernel<NT, RB, EPI, false>), grid, dim3(256), 0, st, A, W, M, K, N, C, bias, pos,
                           S, Cf, pro, tl);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// wide reduction, narrow output: K >= 256, K > N, N <= 384 (multiples of 8)
int rt1_pw_tall_supported(int K, int N) {
    return (K % 8 == 0 && N % 8 == 0 && K >= 256 && N >= 16 && N <= 384 && K > N) ? 1 : 0;
}

// shapes where this kernel beats hipBLASLt on MI355X (tools/debug/tall_sweep.py: 1.1-2.3x for N <= 136 at
// 61-85 % of the HBM roofline; the 128-column-slice path for N = 232 / 384 runs at 0.55-0.8x of hipBLASLt)
int rt1_pw_tall_preferred(int K, int N) { return (rt1_pw_tall_supported(K, N) && N <= 144) ? 1 : 0; }

// scale != nullptr: the operand prologue (TallPro) with gate [M / hw, K] fp32; aout optional [M, K] bf16
int rt1_pw_tall(const bf16_t* A, const bf16_t* W, int M, int K, int N, bf16_t* C, const float* scale,
                const float* shift, const float* gate, int hw, bf16_t* aout, hipStream_t st) {
    if (!rt1_pw_tall_supported(K, N) || M <= 0) return (int)hipErrorInvalidValue;
    if (scale && (!shift || !gate || hw <= 0 || M % hw || K > PRO_KMAX)) return (int)hipErrorInvalidValue;
    const TallPro pro{scale, shift, gate, hw > 0 ? hw : 1, aout};
    if (N <= 96) return launch_tall<6, 4>(A, W, M, K, N, C, st, nullptr, nullptr, 1, nullptr, pro);
    if (N <= 144) return launch_tall<9, 3>(A, W, M, K, N, C, st, nullptr, nullptr, 1, nullptr, pro);
    // wider outputs: 128-column slices (XCD-grouped, see the kernel), so every W fragment read from LDS feeds RB MFMAs
    // (a single-slice RB = 1 / 2 tile is LDS-read bound: one 1 KB ds_read per MFMA)
    if (M >= 65536) return launch_tall<8, 4>(A, W, M, K, N, C, st, nullptr, nullptr, 1, nullptr, pro);
    return launch_tall<8, 2>(A, W, M, K, N, C, st, nullptr, nullptr, 1, nullptr, pro);
}

// token embedding of the RT-1 transformer: out[m, :] = A[m, :] @ W^T + bias + pos[m % S, :]   (fp32 out)
// K % 8 == 0, N % 16 == 0 (N = 512 in RT-1), 128-column slices, RB = 2 (M = B * S is a few thousand rows)
int rt1_embed_fwd(const bf16_t* A, const bf16_t* W, const float* bias, const float* pos, int M, int K, int N, int S,
                  float* out, hipStream_t st) {
    if (K % 8 != 0 || N % 16 != 0 || M <= 0 || S <= 0 || K < 8) return (int)hipErrorInvalidValue;
    return launch_tall<8, 2, 1>(A, W, M, K, N, nullptr, st, bias, pos, S, out);
}

// C = A @ W^T + A2 @ W2^T + bias [+ res * rmul[m / rhw]] (A2 [M, K2], W2 [N, K2] bf16, bias [N] fp32; K2 % 8 == 0):
// the y-free wide expand dgrad dz @ (diag(k1) We) + x @ Mk + r0 (+ the residual path's gradient) in one pass
int rt1_pw_tall_tail(const bf16_t* A, const bf16_t* W, int M, int K, int N, const bf16_t* A2, const bf16_t* W2, int K2,
                     const float* bias, const bf16_t* res, const float* rmul, int rhw, bf16_t* C, hipStream_t st) {
    if (!rt1_pw_tall_preferred(K, N) || M <= 0 || K2 <= 0 || K2 % 8 || !A2 || !W2 || !bias)
        return (int)hipErrorInvalidValue;
    if (res && (!rmul || rhw <= 0 || M % rhw)) return (int)hipErrorInvalidValue;
    const TallPro pro{nullptr, nullptr, nullptr, 1, nullptr};
    const TallTail tl{A2, W2, bias, K2, res, rmul, rhw > 0 ? rhw : 1};
    if (N <= 96) return launch_tall<6, 4>(A, W, M, K, N, C, st, nullptr, nullptr, 1, nullptr, pro, tl);
    return launch_tall<9, 3>(A, W, M, K, N, C, st, nullptr, nullptr, 1, nullptr, pro, tl);
}

}  // extern "C"
