// General tiled MFMA GEMM for the mid-size products of the step, with the surrounding elementwise work fused:
//
//     C[M, N] = pro(A)[M, K] . op(B)  (+ bias[N])        A bf16 row-major; C bf16 or fp32
//     op(B) = B^T for B [N, K] (NT: a Linear / 1x1-conv weight, the forward)
//           = B   for B [K, N] (NN: the same weight in a data-gradient dY @ W)
//     pro(A) = silu(A * scale[k] + shift[k]) * gate[m / hw][k]   (optional: the project conv's operand rebuilt from
//              the depthwise output y2 -- BN2 + SiLU + squeeze-excitation gate -- instead of a bn_apply pass)
//     STATS: per-column partial sum / sum of squares of the STORED bf16 C per M tile (the consumer BatchNorm's
//            batch statistics, reduced by bn_finalize) -- no separate bn_stats pass over C
//     TAIL:  C = A . B^T + A2 . B2^T + bias + res * rmul[m / rhw]  (NT; a second K segment, then a residual epilogue):
//            the dz-mode expand data-gradient of the deep blocks, dx = dz . (diag(k1) We) + x . Mk + r0 + dout * fmul
//            (see backbone.expand_bwd_z_gemm) in one pass -- no bn_bwd_apply over the Ce-wide dA1 / y1, no add_scaled_
//
// Sites (SURVEY K8, K13, K15, K16 and the deep K3/K6 convs): the transformer Q/K/V, out and FF projections and their
// data gradients (T = 8448 token rows at b128), the deep project convs (M = 76,800 pixel rows, K = 816..2304,
// N = 232/384), top 384 -> 1536 and conv1x1 1536 -> 512 and their data gradients.  hipBLASLt ran them at 11-47 % of
// their roofline (profiles/r2_gemm_census.log) and needed the separate BN passes around them.
//
// Tiling (CDNA4, wave64): a 256-thread workgroup owns a BM x BN tile of C, 4 waves in WM x (4 / WM), each wave a
// (BM / WM) x (BN * WM / 4) sub-tile of v_mfma_f32_16x16x32_bf16 accumulators (fp32).  K advances 64 at a time:
// the next k-slab is loaded global -> registers (16-B vectors) while the current one multiplies out of LDS, then the
// registers are written to LDS (prologue applied on the way).  Both operands are read from LDS in MFMA operand layout:
// K-contiguous rows with ds_read_b128 (A, and B in NT), the [K][N] slab of NN with ds_read_b64_tr_b16 (the gfx950
// LDS transpose).  The product is formed as C^T = op(B)^T . A^T, so each lane's accumulator is 4 CONSECUTIVE output
// columns of one row (8- / 16-byte stores).  Workgroup -> tile mapping is XCD-aware: consecutive tiles of one M row
// block (which share the A rows) go to the same XCD, whose L2 then serves the A slab to all of them.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BLOCK = 256;
constexpr int BK = 64;
constexpr int LDK = BK + 8;     // LDS row stride (bf16) of K-contiguous slabs: +16 B against bank aliasing

__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* base0, const bf16_t* base1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

struct GemmArgs {
    const bf16_t* A;
    const bf16_t* B;
    void* C;
    int M, N, K;
    const float* bias;                        // [N] or nullptr
    const float *scale, *shift, *gate;        // prologue (PRO): [K], [K], [M / hw, K]
    int hw;
    float *ps, *pq;                           // STATS: [tiles_m, N]
    bf16_t* aout;                             // PRO: optional [M, K] store of the rebuilt operand (weight gradient)
    const bf16_t *A2, *B2;                    // TAIL: second K segment, A2 [M, K2], B2 [N, K2]
    int K2;
    const bf16_t* res;                        // TAIL: residual [M, N] bf16 (or nullptr) times rmul [M / rhw, N] fp32
    const float* rmul;
    int rhw;
    int lda;                                  // A row stride (elements; K unless a caller pads A's rows)
    const int4* cmap;                         // OUT_F32: per 4-column group {base, row stride, +add bits, -} or nullptr
};

constexpr int GEMM_LDS_STORE = 1;   // plain bf16 products: LDS-staged 16-byte row stores (0: stores from the MFMA layout)

template <int BM, int BN, int WM, bool NN>
struct GShape {
    static constexpr int WN = 4 / WM;
    static constexpr int WTM = BM / WM, WTN = BN / WN;          // wave sub-tile
    static constexpr int MT = WTM / 16, NT = WTN / 16;           // 16 x 16 accumulators per wave
    static constexpr int LDN = BN + 8;                           // NN: [BK][BN] slab row stride
    static constexpr int A_ELEMS = BM * LDK;
    static constexpr int B_ELEMS = NN ? BK * LDN : BN * LDK;
    static constexpr int PA = BM * BK / 8 / BLOCK;               // 16-B vectors per thread per slab
    static constexpr int PB = BN * BK / 8 / BLOCK;
    static constexpr size_t buf = (size_t)(A_ELEMS + B_ELEMS) * 2;
    // one slab buffer: occupancy (3 workgroups / CU at 36 KB) hides the HBM latency better than a double buffer
    // at 72 KB (2 / CU), which measured 5-50 % slower over the step's shapes
    static constexpr size_t lds = buf;
    static_assert(WTM % 16 == 0 && WTN % 16 == 0 && PA * BLOCK * 8 == BM * BK && PB * BLOCK * 8 == BN * BK,
                  "tile / thread split");
};

template <int BM, int BN, int WM, bool NN, bool PRO, bool OUT_F32, bool STATS, bool TAIL = false>
__global__ __launch_bounds__(BLOCK, 2) void gemm_kernel(GemmArgs g) {
    static_assert(!TAIL || (!NN && !PRO && !OUT_F32 && !STATS), "TAIL: plain NT bf16 product");
    using S = GShape<BM, BN, WM, NN>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int lr = lane & 15, lh = lane >> 4;
    const int wm = wave % WM, wn = wave / WM;
    const int M = g.M, N = g.N, K = g.K;

    // XCD-aware tile order: blockIdx b runs on XCD b % 8; each XCD takes a contiguous range of the M-major tile list
    const int tiles_n = (N + BN - 1) / BN;
    const int T = gridDim.x;
    const int b = blockIdx.x, xcd = b & 7, per = T >> 3, extra = T & 7;
    const int tile = xcd * per + min(xcd, extra) + (b >> 3);
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;

    // global -> register slabs: A rows r = v / 8 (8 vectors of 8 k per row), B likewise (NT) or k rows of BN (NN)
    struct Regs {
        uint4 ra[S::PA], rb[S::PB];
        float gt[PRO ? S::PA : 1][PRO ? 8 : 1];       // PRO: gate values of the thread's A rows for the slab
    };
    const int acol = (t & 7) * 8;                     // this thread's fixed k offset inside an A / NT-B slab row
    // slab s: k0 = s * BK of (A, B, K), or with TAIL past the first segment's ns1 slabs, of (A2, B2, K2)
    const int ns1 = (K + BK - 1) / BK;
    auto issue = [&](Regs& R, int s) {
        auto& ra = R.ra;
        auto& rb = R.rb;
        auto& gt = R.gt;
        const bool seg2 = TAIL && s >= ns1;
        const bf16_t* Ap = seg2 ? g.A2 : g.A;
        const bf16_t* Bp = seg2 ? g.B2 : g.B;
        const int Ks = seg2 ? g.K2 : K;
        const int k0 = (seg2 ? s - ns1 : s) * BK;
#pragma unroll
        for (int i = 0; i < S::PA; ++i) {
            const int r = (t >> 3) + i * (BLOCK / 8);
            const int64_t m = m0 + r;
            const int k = k0 + acol;
            ra[i] = make_uint4(0, 0, 0, 0);
            if (m < M && k < Ks) ra[i] = *reinterpret_cast<const uint4*>(Ap + m * (seg2 ? Ks : g.lda) + k);
            if constexpr (PRO) {
                if (m < M && k < K) {
                    const float* gp = g.gate + (m / g.hw) * K + k;
                    const float4 x0 = *reinterpret_cast<const float4*>(gp);
                    const float4 x1 = *reinterpret_cast<const float4*>(gp + 4);
                    gt[i][0] = x0.x; gt[i][1] = x0.y; gt[i][2] = x0.z; gt[i][3] = x0.w;
                    gt[i][4] = x1.x; gt[i][5] = x1.y; gt[i][6] = x1.z; gt[i][7] = x1.w;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < S::PB; ++i) {
            rb[i] = make_uint4(0, 0, 0, 0);
            if constexpr (NN) {
                const int v = t + i * BLOCK, kr = v / (BN / 8), c = (v - kr * (BN / 8)) * 8;
                if (k0 + kr < K && n0 + c < N)
                    rb[i] = *reinterpret_cast<const uint4*>(g.B + (int64_t)(k0 + kr) * N + n0 + c);
            } else {
                const int r = (t >> 3) + i * (BLOCK / 8), k = k0 + acol;
                if (n0 + r < N && k < Ks) rb[i] = *reinterpret_cast<const uint4*>(Bp + (int64_t)(n0 + r) * Ks + k);
            }
        }
    };
    auto stage = [&](const Regs& R, int k0, int bsel) {
        const auto& ra = R.ra;
        const auto& rb = R.rb;
        const auto& gt = R.gt;
        bf16_t* Al = reinterpret_cast<bf16_t*>(smem + bsel * S::buf);
        bf16_t* Bl = Al + S::A_ELEMS;
        float sc[8], sh[8];
        if constexpr (PRO) {
            const int k = k0 + acol;
            if (k < K) {
                load8f(g.scale + k, sc);
                load8f(g.shift + k, sh);
            }
        }
#pragma unroll
        for (int i = 0; i < S::PA; ++i) {
            const int r = (t >> 3) + i * (BLOCK / 8);
            uint4 u = ra[i];
            if constexpr (PRO) {
                if (m0 + r < M && k0 + acol < K) {
                    float f[8];
                    unpack8(u, f);
#pragma unroll
                    for (int j = 0; j < 8; ++j) f[j] = silu(fmaf(f[j], sc[j], sh[j])) * gt[i][j];
                    u.x = pack2(f[0], f[1]); u.y = pack2(f[2], f[3]); u.z = pack2(f[4], f[5]); u.w = pack2(f[6], f[7]);
                    // the first N tile of each row block also stores the operand (each A row block is staged once
                    // per N tile)
                    if (g.aout && tn == 0) *reinterpret_cast<uint4*>(g.aout + (m0 + r) * K + k0 + acol) = u;
                }
            }
            *reinterpret_cast<uint4*>(Al + r * LDK + acol) = u;
        }
#pragma unroll
        for (int i = 0; i < S::PB; ++i) {
            if constexpr (NN) {
                const int v = t + i * BLOCK, kr = v / (BN / 8), c = (v - kr * (BN / 8)) * 8;
                *reinterpret_cast<uint4*>(Bl + kr * S::LDN + c) = rb[i];
            } else {
                const int r = (t >> 3) + i * (BLOCK / 8);
                *reinterpret_cast<uint4*>(Bl + r * LDK + acol) = rb[i];
            }
        }
    };

    f32x4 acc[S::NT][S::MT];
    const int q4 = lr >> 2, p4 = lr & 3;
    auto compute = [&](int bsel) {
        const bf16_t* Al = reinterpret_cast<const bf16_t*>(smem + bsel * S::buf);
        const bf16_t* Bl = Al + S::A_ELEMS;
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
            bf16x8 fa[S::MT];
#pragma unroll
            for (int j = 0; j < S::MT; ++j)
                fa[j] = *reinterpret_cast<const bf16x8*>(Al + (wm * S::WTM + j * 16 + lr) * LDK + ks * 32 + lh * 8);
#pragma unroll
            for (int i = 0; i < S::NT; ++i) {
                bf16x8 fb;
                if constexpr (NN) {
                    const int r0 = ks * 32 + lh * 8 + q4, cb = wn * S::WTN + i * 16 + p4 * 4;
                    fb = tr_read8(Bl + r0 * S::LDN + cb, Bl + (r0 + 4) * S::LDN + cb);
                } else {
                    fb = *reinterpret_cast<const bf16x8*>(Bl + (wn * S::WTN + i * 16 + lr) * LDK + ks * 32 + lh * 8);
                }
#pragma unroll
                for (int j = 0; j < S::MT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    // the next slab is loaded into registers while the current one multiplies out of LDS
    const int ns = ns1 + (TAIL ? (g.K2 + BK - 1) / BK : 0);
    auto mainloop = [&]() {
#pragma unroll
        for (int i = 0; i < S::NT; ++i)
#pragma unroll
            for (int j = 0; j < S::MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        Regs R;
        issue(R, 0);
        for (int s = 0; s < ns; ++s) {
            __syncthreads();                          // the previous slab's operand reads are done
            stage(R, s * BK, 0);
            __syncthreads();
            if (s + 1 < ns) issue(R, s + 1);
            compute(0);
        }
    };

    mainloop();

    if constexpr (!OUT_F32 && !STATS && !TAIL && !PRO && GEMM_LDS_STORE) {
        if (g.bias == nullptr) {
            // plain bf16 product (the wide project data gradients): the tile goes through LDS so each thread
            // stores 16-byte pieces of full tile rows (the MFMA layout leaves 8-byte pieces of 16 rows per store)
            constexpr int TL = BN + 8, C8 = BN / 8;
            bf16_t* T = reinterpret_cast<bf16_t*>(smem);
            __syncthreads();                          // operand reads of the last slab are done
#pragma unroll
            for (int i = 0; i < S::NT; ++i)
#pragma unroll
                for (int j = 0; j < S::MT; ++j) {
                    uint2 u;
                    u.x = pack2(acc[i][j][0], acc[i][j][1]);
                    u.y = pack2(acc[i][j][2], acc[i][j][3]);
                    *reinterpret_cast<uint2*>(T + (wm * S::WTM + j * 16 + lr) * TL + wn * S::WTN + i * 16 + lh * 4) = u;
                }
            __syncthreads();
            bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
            for (int o = t; o < BM * C8; o += BLOCK) {
                const int r = o / C8, c = (o - r * C8) * 8;
                if (m0 + r < M && n0 + c < N)
                    *reinterpret_cast<uint4*>(C + (m0 + r) * N + n0 + c) = *reinterpret_cast<const uint4*>(T + r * TL + c);
            }
            return;
        }
    }

    // epilogue: lane holds C[m][n .. n+3], m = m0 + wm*WTM + j*16 + lr, n = n0 + wn*WTN + i*16 + lh*4
    float ssum[S::NT][4], ssq[S::NT][4];
#pragma unroll
    for (int i = 0; i < S::NT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) ssum[i][e] = ssq[i][e] = 0.f;
#pragma unroll
    for (int i = 0; i < S::NT; ++i) {
        const int n = n0 + wn * S::WTN + i * 16 + lh * 4;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (g.bias && n < N) {
            const float4 b4 = *reinterpret_cast<const float4*>(g.bias + n);
            bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
        }
#pragma unroll
        for (int j = 0; j < S::MT; ++j) {
            const int64_t m = m0 + wm * S::WTM + j * 16 + lr;
            if (m >= M || n >= N) continue;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
            if constexpr (TAIL) {
                if (g.res) {
                    const uint2 r2 = *reinterpret_cast<const uint2*>(g.res + m * N + n);
                    const float4 f4 = *reinterpret_cast<const float4*>(g.rmul + (m / g.rhw) * N + n);
                    v[0] += __uint_as_float(r2.x << 16) * f4.x;
                    v[1] += __uint_as_float(r2.x & 0xffff0000u) * f4.y;
                    v[2] += __uint_as_float(r2.y << 16) * f4.z;
                    v[3] += __uint_as_float(r2.y & 0xffff0000u) * f4.w;
                }
            }
            if constexpr (OUT_F32) {
                float* cp = reinterpret_cast<float*>(g.C) + m * N + n;
                if (g.cmap) {
                    // scattered column groups (the FiLM projections: each block's [M, C] slice contiguous)
                    const int4 cm = g.cmap[n >> 2];
                    cp = reinterpret_cast<float*>(g.C) + cm.x + m * cm.y;
                    const float add = __int_as_float(cm.z);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += add;
                }
                *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
                uint2 u;
                u.x = pack2(v[0], v[1]);
                u.y = pack2(v[2], v[3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(g.C) + m * N + n) = u;
                if constexpr (STATS) {
                    // statistics describe the stored bf16 tensor
                    const float s0 = __uint_as_float(u.x << 16), s1 = __uint_as_float(u.x & 0xffff0000u);
                    const float s2 = __uint_as_float(u.y << 16), s3 = __uint_as_float(u.y & 0xffff0000u);
                    ssum[i][0] += s0; ssq[i][0] = fmaf(s0, s0, ssq[i][0]);
                    ssum[i][1] += s1; ssq[i][1] = fmaf(s1, s1, ssq[i][1]);
                    ssum[i][2] += s2; ssq[i][2] = fmaf(s2, s2, ssq[i][2]);
                    ssum[i][3] += s3; ssq[i][3] = fmaf(s3, s3, ssq[i][3]);
                }
            }
        }
    }
    if constexpr (STATS) {
        // over the 16 row lanes (lr) of each lane group, fixed xor order; then over the WM row waves through LDS
#pragma unroll
        for (int i = 0; i < S::NT; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    ssum[i][e] += __shfl_xor(ssum[i][e], o, 64);
                    ssq[i][e] += __shfl_xor(ssq[i][e], o, 64);
                }
            }
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);   // [WM][2][BN]
        if (lr == 0) {
#pragma unroll
            for (int i = 0; i < S::NT; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int c = wn * S::WTN + i * 16 + lh * 4 + e;
                    red[(wm * 2) * BN + c] = ssum[i][e];
                    red[(wm * 2 + 1) * BN + c] = ssq[i][e];
                }
        }
        __syncthreads();
        for (int c = t; c < BN; c += BLOCK) {
            float a = 0.f, q = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                a += red[(w * 2) * BN + c];
                q += red[(w * 2 + 1) * BN + c];
            }
            if (n0 + c < N) {
                g.ps[(int64_t)tm * N + n0 + c] = a;
                g.pq[(int64_t)tm * N + n0 + c] = q;
            }
        }
    }
}

// tile configurations: 0 = 128 x 128 (2 x 2 waves), 1 = 64 x 256 (1 x 4: wide N, few rows), 2 = 256 x 64 (4 x 1),
// 3 = 64 x 64 and 4 = 128 x 64 (2 x 2: short-K products of a few thousand rows, where occupancy hides the slab loads)
struct Cfg { int bm, bn; };
constexpr Cfg CFGS[] = {{128, 128}, {64, 256}, {256, 64}, {64, 64}, {128, 64}};
constexpr int NCFG = 5;

int pick_cfg(int M, int N, int K, int cfg) {
    if (cfg >= 0 && cfg < NCFG) return cfg;
    (void)K;
    if (N <= 64) return 2;
    if (M <= 16384 && N >= 1024) return 1;
    return 0;
}

template <int BM, int BN, int WM, bool NN>
int launch_cfg(const GemmArgs& a, bool pro, bool f32, bool stats, hipStream_t st) {
    using S = GShape<BM, BN, WM, NN>;
    static_assert(BM * (BN + 8) * 2 <= S::lds, "LDS-staged store tile fits");
    const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const dim3 grid(tiles);
    if constexpr (!NN) {
        if (a.A2) {
            if (pro || f32 || stats) return (int)hipErrorInvalidValue;
            hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, false, false, false, false, true>), grid, dim3(BLOCK), S::lds,
                               st, a);
            return (int)hipGetLastError();
        }
    } else {
        if (a.A2) return (int)hipErrorInvalidValue;
    }
    // STATS reuses the operand LDS for its [WM][2][BN] reduction
    static_assert(WM * 2 * BN * 4 <= S::lds, "stats scratch fits");
#define G(P, F, ST) hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, NN, P, F, ST>), grid, dim3(BLOCK), S::lds, st, a)
    if (pro) {
        if (f32) return (int)hipErrorInvalidValue;
        if (stats) G(true, false, true); else G(true, false, false);
    } else if (f32) {
        if (stats) return (int)hipErrorInvalidValue;
        G(false, true, false);
    } else {
        if (stats) G(false, false, true); else G(false, false, false);
    }
#undef G
    return (int)hipGetLastError();
}

template <bool NN>
int launch_any(int cfg, const GemmArgs& a, bool pro, bool f32, bool stats, hipStream_t st) {
    switch (cfg) {
        case 0: return launch_cfg<128, 128, 2, NN>(a, pro, f32, stats, st);
        case 1: return launch_cfg<64, 256, 1, NN>(a, pro, f32, stats, st);
        case 2: return launch_cfg<256, 64, 4, NN>(a, pro, f32, stats, st);
        case 3: return launch_cfg<64, 64, 2, NN>(a, pro, f32, stats, st);
        default: return launch_cfg<128, 64, 2, NN>(a, pro, f32, stats, st);
    }
}

}  // namespace

extern "C" {

int rt1_gemm_tiles_m(int M, int N, int K, int cfg) {
    const Cfg c = CFGS[pick_cfg(M, N, K, cfg)];
    return (M + c.bm - 1) / c.bm;
}

// C = pro(A) . op(B) (+ bias); nn: B is [K, N] (else [N, K]); out_f32: C fp32 (else bf16); ps/pq: stats partials
// [rt1_gemm_tiles_m(...), N] (bf16 output only); scale/shift/gate/hw: the A prologue (bf16 output only)
int rt1_gemm(const bf16_t* A, const bf16_t* B, void* C, int M, int N, int K, int nn, const float* bias,
             const float* scale, const float* shift, const float* gate, int hw, int out_f32, float* ps, float* pq,
             int cfg, bf16_t* aout, hipStream_t st) {
    if (M <= 0 || N <= 0 || K <= 0 || (N % 8) || (K % 8)) return (int)hipErrorInvalidValue;
    const bool pro = scale != nullptr;
    if (pro && (!shift || !gate || hw <= 0 || M % hw)) return (int)hipErrorInvalidValue;
    if ((ps != nullptr) != (pq != nullptr) || (aout && !pro)) return (int)hipErrorInvalidValue;
    GemmArgs a{A, B, C, M, N, K, bias, scale, shift, gate, hw, ps, pq, aout, nullptr, nullptr, 0, nullptr, nullptr, 1, K,
               nullptr};
    const bool stats = ps != nullptr;
    const int c = pick_cfg(M, N, K, cfg);
    return nn ? launch_any<true>(c, a, pro, out_f32, stats, st) : launch_any<false>(c, a, pro, out_f32, stats, st);
}

// C = A . B^T + A2 . B2^T + bias + res * rmul[m / rhw] (bf16 C, NT operands; res / rmul optional)
int rt1_gemm_tail(const bf16_t* A, const bf16_t* B, int M, int N, int K, const bf16_t* A2, const bf16_t* B2, int K2,
                  const float* bias, const bf16_t* res, const float* rmul, int rhw, bf16_t* C, int cfg,
                  hipStream_t st) {
    if (M <= 0 || N <= 0 || K <= 0 || K2 <= 0 || (N % 8) || (K % 8) || (K2 % 8) || !A2 || !B2)
        return (int)hipErrorInvalidValue;
    if (res && (!rmul || rhw <= 0 || M % rhw)) return (int)hipErrorInvalidValue;
    GemmArgs a{A, B, C, M, N, K, bias, nullptr, nullptr, nullptr, 1, nullptr, nullptr, nullptr, A2, B2, K2, res, rmul,
               rhw > 0 ? rhw : 1, K, nullptr};
    return launch_any<false>(pick_cfg(M, N, K, cfg), a, false, false, false, st);
}

// FiLM projections: C = A . B^T + bias (+ cmap add) in fp32 with A [M, K] bf16 at row stride lda and
// B [N, K] bf16; cmap[n / 4] = {base, row stride, float bits of an add, 0} scatters each 4-column group to
// C[base + m * stride .. + 3], so every block's (1 + gamma) / beta slice comes out as its own contiguous [M, C] array
int rt1_gemm_cmap(const bf16_t* A, int lda, const bf16_t* B, float* C, int M, int N, int K, const float* bias,
                  const int* cmap, int cfg, hipStream_t st) {
    if (M <= 0 || N <= 0 || K <= 0 || (N % 8) || (K % 8) || lda < K || (lda % 8) || !cmap)
        return (int)hipErrorInvalidValue;
    GemmArgs a{A, B, C, M, N, K, bias, nullptr, nullptr, nullptr, 1, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
               nullptr, nullptr, 1, lda, reinterpret_cast<const int4*>(cmap)};
    return launch_any<false>(pick_cfg(M, N, K, cfg), a, false, true, false, st);
}

}  // extern "C"
