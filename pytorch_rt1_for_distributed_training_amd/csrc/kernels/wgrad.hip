// Weight gradient of a 1x1 convolution / linear layer on MFMA, streaming the pixel dimension:
//
//     dW[co, ci] = sum_m dy[m, co] * a[m, ci]        dy: [M, Co] bf16, a: [M, Ci] bf16, dW fp32
//
// with an optional PROLOGUE on `a`, so the project convolution's input A = silu(bn2(y2)) * gate[n] can be
// rebuilt from y2 inside the kernel instead of being materialised (a[m, ci] = act(y2[m, ci] * scale[ci] +
// shift[ci]) * gate[m / hw, ci]).
//
// Replaces the split-K torch.bmm (hipBLASLt, fp32 partial tiles) + sum of the previous revision for every
// 1x1-conv weight gradient of the encoder (SURVEY K3/K6 backward, film_efficientnet_encoder.py:185-224).
//
// Shape of the computation: M (frames x pixels, up to 17 M rows) is the MFMA k dimension.  A workgroup owns
// one TCO x TCI output tile and a contiguous range of rows (split-K over grid.y); it streams 64-row chunks:
//   * global -> registers (16-byte vectors; the next chunk is issued before the current chunk's MFMAs, so
//     HBM latency hides behind them), prologue applied on the way, registers -> LDS row-major;
//   * both operands are read k-major with ds_read_b64_tr_b16 (the gfx950 LDS transpose: 4 rows x 16 columns
//     per 16-lane group), feeding v_mfma_f32_16x16x32_bf16; 4 waves split the tile WR x (4 / WR);
//   * at the end each workgroup writes its fp32 partial tile; a fixed-order column sum (reduce.hip) combines
//     the splits, so the result is bitwise reproducible (no atomics).
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BLOCK = 256;
constexpr int ROWS = 64;

// LDS-only barrier: the chunk loop never needs the global-memory fence a __syncthreads implies
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

struct Prologue {
    const float* scale;   // [Ci] or nullptr (no prologue)
    const float* shift;   // [Ci]
    const float* gate;    // [M / hw, Ci] or nullptr
    int act;              // ACT_NONE / ACT_SILU
    int hw;               // rows per frame (gate row = m / hw)
};

__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* base0, const bf16_t* base1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int TCO, int TCI, int WR>
struct WShape {
    static constexpr int WC = 4 / WR;
    static constexpr int NCO = TCO / 16 / WR;      // 16-row co tiles per wave
    static constexpr int NCI = TCI / 16 / WC;      // 16-col ci tiles per wave
    static constexpr int LDA = TCO + 8;            // LDS row strides (bf16), multiples of 8
    static constexpr int LDB = TCI + 8;
    static constexpr int VA = ROWS * TCO / 8;      // 16-B vectors per chunk
    static constexpr int VB = ROWS * TCI / 8;
    static constexpr int PA = (VA + BLOCK - 1) / BLOCK;   // per thread
    static constexpr int PB = (VB + BLOCK - 1) / BLOCK;
    static constexpr size_t stage_bytes = (size_t)ROWS * (LDA + LDB) * 2;
    static constexpr size_t lds = stage_bytes;   // one chunk buffer (two: 1.25x slower, profiles/r2_wgrad_db_ab.log)
    static_assert(TCO % (16 * WR) == 0 && TCI % (16 * WC) == 0, "tile / wave split");
    static_assert((TCI / 8) <= BLOCK && BLOCK % (TCI / 8) == 0, "a column vectors fixed per thread");
};

// PRO: 0 = a as is, 1 = a*scale + shift, 2 = silu(a*scale + shift); times gate[m / hw] when pro.gate is set.
// The gate rows of the <= 2 frames a 64-row chunk touches (hw >= 64) are fetched with the chunk's data.
// Workgroup -> (output tile, row split).  grouped (splits % 8 == 0): 1-D grid, workgroup b runs on XCD b % 8 and
// the T output tiles of one split are consecutive slots on ONE XCD, so the split's dy / a rows come from HBM once
// and the other T-1 tiles re-read them from that XCD's L2 (tile-major order spread every split's tiles over all 8
// XCDs: each XCD fetched its own copy of the rows, ~T/2 x the compulsory bytes on the 136 x 816 / 232 x 1392 deep
// shapes).  Otherwise: blockIdx.x = tile, blockIdx.y = split.
// DYF: dy is fp32 and column-mapped -- dy[m, co] = dyf[map[co / 4].x + m * map[co / 4].y + co % 4] (the FiLM
// projections' per-block [M, C] gradient slices, csrc/kernels/gemm.hip rt1_gemm_cmap); rounded to bf16 at staging.
// With DYF the first ci tile's workgroups also sum their fp32 dy rows per column: dbout[split][co] (the bias
// gradient, fixed order: per-thread row sums, then the 32 row threads of a column through LDS).
// DBS: the same column sums of a bf16 dy (the Gram matrix G = x^T x with dy = a = x: sx = sum_m x comes with G).
// pstride: elements per split of out; dbout[split * dbstride + co].
struct DyMap {
    const float* dyf;
    const int4* map;
    float* dbout;
    int64_t dbstride;
};

template <int TCO, int TCI, int WR, int PRO, bool DYF = false, bool DBS = false>
__global__ __launch_bounds__(BLOCK, 2) void wgrad_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ a,
                                                         int64_t M, int Co, int Ci, int tiles_ci,
                                                         int64_t rows_per_split, Prologue pro,
                                                         float* __restrict__ out, int grouped_tiles, int64_t pstride,
                                                         DyMap dmap = DyMap{nullptr, nullptr, nullptr, 0}) {
    using S = WShape<TCO, TCI, WR>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* al_dy = reinterpret_cast<bf16_t*>(smem);
    bf16_t* al_a = al_dy + ROWS * S::LDA;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int lr = lane & 15, lh = lane >> 4;
    int tile, split;
    if (grouped_tiles > 0) {
        const int b = blockIdx.x, slot = b >> 3;
        tile = slot % grouped_tiles;
        split = (slot / grouped_tiles) * 8 + (b & 7);
    } else {
        tile = blockIdx.x;
        split = blockIdx.y;
    }
    const int co0 = (tile / tiles_ci) * TCO, ci0 = (tile % tiles_ci) * TCI;
    const int64_t m_begin = (int64_t)split * rows_per_split;
    const int64_t m_end = m_begin + rows_per_split < M ? m_begin + rows_per_split : M;
    const int wr = wave % WR, wc = wave / WR;

    // this thread's fixed column vector of the a tile (TCI / 8 vectors per row): prologue constants in registers
    constexpr int AV = TCI / 8;
    const int acol = (t % AV) * 8;
    const bool acol_ok = ci0 + acol < Ci;
    float sc[8], sh[8], g0[8], g1[8];
    if constexpr (PRO != 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sc[j] = acol_ok ? pro.scale[ci0 + acol + j] : 0.f;
            sh[j] = acol_ok ? pro.shift[ci0 + acol + j] : 0.f;
            g0[j] = g1[j] = 1.f;
        }
    }
    const bool has_gate = PRO != 0 && pro.gate != nullptr;
    const uint32_t nframes = has_gate ? (uint32_t)(M / pro.hw) : 0;

    f32x4 acc[S::NCO][S::NCI];
#pragma unroll
    for (int i = 0; i < S::NCO; ++i)
#pragma unroll
        for (int j = 0; j < S::NCI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 ra[S::PA], rb[S::PB];
    float4 rf[DYF ? S::PA : 1][2];
    constexpr bool SUMS = DYF || DBS;
    float dbacc[SUMS ? 8 : 1];
    if constexpr (SUMS) {
        static_assert(BLOCK % (TCO / 8) == 0, "fixed dy column group per thread");
#pragma unroll
        for (int j = 0; j < 8; ++j) dbacc[j] = 0.f;
    }
    auto issue = [&](int64_t m0) {
#pragma unroll
        for (int k = 0; k < S::PA; ++k) {
            const int v = t + k * BLOCK;
            const int r = v / (TCO / 8), c = (v % (TCO / 8)) * 8;
            if constexpr (DYF) {
                rf[k][0] = rf[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (v < S::VA && m0 + r < m_end && co0 + c < Co) {
                    const int4 c0 = dmap.map[(co0 + c) >> 2], c1 = dmap.map[((co0 + c) >> 2) + 1];
                    rf[k][0] = *reinterpret_cast<const float4*>(dmap.dyf + c0.x + (m0 + r) * c0.y);
                    rf[k][1] = *reinterpret_cast<const float4*>(dmap.dyf + c1.x + (m0 + r) * c1.y);
                }
            } else {
                ra[k] = make_uint4(0, 0, 0, 0);
                if (v < S::VA && m0 + r < m_end && co0 + c < Co)
                    ra[k] = *reinterpret_cast<const uint4*>(dy + (m0 + r) * Co + co0 + c);
            }
        }
#pragma unroll
        for (int k = 0; k < S::PB; ++k) {
            const int v = t + k * BLOCK;
            const int r = v / AV;
            rb[k] = make_uint4(0, 0, 0, 0);
            if (v < S::VB && m0 + r < m_end && acol_ok)
                rb[k] = *reinterpret_cast<const uint4*>(a + (m0 + r) * Ci + ci0 + acol);
        }
        if (has_gate && acol_ok) {
            const uint32_t f0 = (uint32_t)m0 / (uint32_t)pro.hw;
            load8f(pro.gate + (int64_t)f0 * Ci + ci0 + acol, g0);
            if (f0 + 1 < nframes) load8f(pro.gate + (int64_t)(f0 + 1) * Ci + ci0 + acol, g1);
        }
    };
    auto stage = [&](int64_t m0, bf16_t* al_dy, bf16_t* al_a) {
#pragma unroll
        for (int k = 0; k < S::PA; ++k) {
            const int v = t + k * BLOCK;
            if (v < S::VA) {
                const int r = v / (TCO / 8), c = (v % (TCO / 8)) * 8;
                if constexpr (DYF) {
                    dbacc[0] += rf[k][0].x; dbacc[1] += rf[k][0].y; dbacc[2] += rf[k][0].z; dbacc[3] += rf[k][0].w;
                    dbacc[4] += rf[k][1].x; dbacc[5] += rf[k][1].y; dbacc[6] += rf[k][1].z; dbacc[7] += rf[k][1].w;
                    ra[k].x = pack2(rf[k][0].x, rf[k][0].y); ra[k].y = pack2(rf[k][0].z, rf[k][0].w);
                    ra[k].z = pack2(rf[k][1].x, rf[k][1].y); ra[k].w = pack2(rf[k][1].z, rf[k][1].w);
                } else if constexpr (DBS) {
                    if (ci0 == 0) {
                        float f[8];
                        unpack8(ra[k], f);
#pragma unroll
                        for (int j = 0; j < 8; ++j) dbacc[j] += f[j];
                    }
                }
                *reinterpret_cast<uint4*>(al_dy + r * S::LDA + c) = ra[k];
            }
        }
        const int64_t fb = has_gate ? ((int64_t)((uint32_t)m0 / (uint32_t)pro.hw) + 1) * pro.hw : 0;
#pragma unroll
        for (int k = 0; k < S::PB; ++k) {
            const int v = t + k * BLOCK;
            if (v < S::VB) {
                const int r = v / AV;
                uint4 u = rb[k];
                if (PRO != 0 && acol_ok && m0 + r < m_end) {
                    float f[8];
                    unpack8(u, f);
                    const bool second = m0 + r >= fb;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float y = fmaf(f[j], sc[j], sh[j]);
                        if constexpr (PRO == 2) y = silu(y);
                        f[j] = has_gate ? y * (second ? g1[j] : g0[j]) : y;
                    }
                    u.x = pack2(f[0], f[1]); u.y = pack2(f[2], f[3]); u.z = pack2(f[4], f[5]); u.w = pack2(f[6], f[7]);
                }
                *reinterpret_cast<uint4*>(al_a + r * S::LDB + acol) = u;
            }
        }
    };

    auto mfma_chunk = [&](const bf16_t* al_dy, const bf16_t* al_a) {
        const int q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
        for (int ks = 0; ks < ROWS / 32; ++ks) {
            const int r0 = ks * 32 + lh * 8 + q;
            bf16x8 fb[S::NCI];
#pragma unroll
            for (int j = 0; j < S::NCI; ++j) {
                const int cb = (wc * S::NCI + j) * 16 + p * 4;
                fb[j] = tr_read8(al_a + r0 * S::LDB + cb, al_a + (r0 + 4) * S::LDB + cb);
            }
#pragma unroll
            for (int i = 0; i < S::NCO; ++i) {
                const int cb = (wr * S::NCO + i) * 16 + p * 4;
                const bf16x8 fa = tr_read8(al_dy + r0 * S::LDA + cb, al_dy + (r0 + 4) * S::LDA + cb);
#pragma unroll
                for (int j = 0; j < S::NCI; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    if (m_begin < m_end) issue(m_begin);
    for (int64_t m0 = m_begin; m0 < m_end; m0 += ROWS) {
        __syncthreads();                       // previous chunk's MFMA reads are done
        stage(m0, al_dy, al_a);
        __syncthreads();
        if (m0 + ROWS < m_end) issue(m0 + ROWS);   // next chunk in flight during the MFMAs
        mfma_chunk(al_dy, al_a);
    }
    if constexpr (SUMS) {
        if (ci0 == 0) {
            constexpr int CG = TCO / 8, RT = BLOCK / CG;        // column groups, row threads per group
            float* red = reinterpret_cast<float*>(smem);        // [RT][TCO]
            __syncthreads();                                    // the last chunk's operand reads are done
#pragma unroll
            for (int j = 0; j < 8; ++j) red[(t / CG) * TCO + (t % CG) * 8 + j] = dbacc[j];
            __syncthreads();
            if (t < TCO && co0 + t < Co) {
                float v = 0.f;
                for (int r = 0; r < RT; ++r) v += red[r * TCO + t];
                dmap.dbout[(int64_t)split * dmap.dbstride + co0 + t] = v;
            }
        }
    }
    // partial tile: out[split][co][ci]; D rows = co (lh*4 + e), cols = ci (lr)
    float* o = out + (int64_t)split * pstride;
#pragma unroll
    for (int i = 0; i < S::NCO; ++i)
#pragma unroll
        for (int j = 0; j < S::NCI; ++j) {
            const int ci = ci0 + (wc * S::NCI + j) * 16 + lr;
            if (ci >= Ci) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int co = co0 + (wr * S::NCO + i) * 16 + lh * 4 + e;
                if (co < Co) o[(int64_t)co * Ci + ci] = acc[i][j][e];
            }
        }
}

struct Variant { int tco, tci, wr; };

// tile variants: skinny Co (24..48), mid, square, and the wide 128 x 256 tile for the deep layers
constexpr Variant VARIANTS[] = {{32, 256, 1}, {64, 128, 1}, {128, 128, 2}, {64, 256, 2}, {128, 64, 4}, {128, 256, 2}};
constexpr int NVAR = sizeof(VARIANTS) / sizeof(VARIANTS[0]);

Variant pick(int Co, int Ci, int variant = -1) {
    if (variant >= 0 && variant < NVAR) return VARIANTS[variant];
    // least padded MAC work; ties -> bigger tile (fewer partial writes)
    Variant best = VARIANTS[0];
    double best_cost = 1e300;
    for (const Variant& v : VARIANTS) {
        const double tiles = (double)((Co + v.tco - 1) / v.tco) * ((Ci + v.tci - 1) / v.tci);
        const double cost = tiles * v.tco * v.tci * 1.0 + tiles * 4096.0;   // + per-tile fixed cost
        if (cost < best_cost * 0.999) { best_cost = cost; best = v; }
    }
    return best;
}

template <int TCO, int TCI, int WR>
int launch(const bf16_t* dy, const bf16_t* a, int64_t M, int Co, int Ci, int splits, int64_t rows, Prologue pro,
           float* out, bool sums, hipStream_t st) {
    using S = WShape<TCO, TCI, WR>;
    const int tci = (Ci + TCI - 1) / TCI, tco = (Co + TCO - 1) / TCO;
    const bool grouped = splits % 8 == 0;
    const dim3 grid = grouped ? dim3(tco * tci * splits) : dim3(tco * tci, splits);
    const int gt = grouped ? tco * tci : 0;
    const int64_t ps = (int64_t)Co * Ci + (sums ? Co : 0);
#define K(P) hipLaunchKernelGGL((wgrad_kernel<TCO, TCI, WR, P>), grid, dim3(BLOCK), S::lds, st, dy, a, M, Co, Ci, tci, \
                                rows, pro, out, gt, ps)
    if (sums)
        hipLaunchKernelGGL((wgrad_kernel<TCO, TCI, WR, 0, false, true>), grid, dim3(BLOCK), S::lds, st, dy, a, M, Co,
                           Ci, tci, rows, pro, out, gt, ps, DyMap{nullptr, nullptr, out + (int64_t)Co * Ci, ps});
    else if (!pro.scale) K(0);
    else if (pro.act == ACT_SILU) K(2);
    else K(1);
#undef K
    return (int)hipGetLastError();
}

template <int TCO, int TCI, int WR>
int launch_dymap(const float* dyf, const int* map, const bf16_t* a, int64_t M, int Co, int Ci, int splits, float* out,
                 float* dbout, hipStream_t st) {
    using S = WShape<TCO, TCI, WR>;
    const int64_t rows = ((M + splits - 1) / splits + ROWS - 1) / ROWS * ROWS;
    const int tci = (Ci + TCI - 1) / TCI, tco = (Co + TCO - 1) / TCO;
    Prologue pro{nullptr, nullptr, nullptr, 0, 1};
    hipLaunchKernelGGL((wgrad_kernel<TCO, TCI, WR, 0, true>), dim3(tco * tci, splits), dim3(BLOCK), S::lds, st, nullptr,
                       a, M, Co, Ci, tci, rows, pro, out, 0, (int64_t)Co * Ci,
                       DyMap{dyf, reinterpret_cast<const int4*>(map), dbout, Co});
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// Split count for the pixel dimension: enough workgroups (~2 per CU over the output tiles) with >= 2 chunks each;
// rounded to a multiple of 8 from 8 splits up (XCD-grouped launch, see the kernel).  variant < 0: pick().
int rt1_wgrad_splits(int64_t M, int Co, int Ci, int variant) {
    const Variant v = pick(Co, Ci, variant);
    const int64_t tiles = (int64_t)((Co + v.tco - 1) / v.tco) * ((Ci + v.tci - 1) / v.tci);
    int64_t want = (512 + tiles - 1) / tiles;
    const int64_t max_by_rows = (M + 2 * ROWS - 1) / (2 * ROWS);
    if (want > max_by_rows) want = max_by_rows;
    if (want > 2048) want = 2048;
    if (want >= 8) want = want / 8 * 8;
    return (int)(want < 1 ? 1 : want);
}

// out: [splits, Co, Ci] fp32 (splits from rt1_wgrad_splits with the same variant); scale/shift/gate optional.
// sums (no prologue): out is [splits, Co * Ci + Co], each split's dW partial followed by its column sums of dy.
int rt1_wgrad_run(const bf16_t* dy, const bf16_t* a, int64_t M, int Co, int Ci, const float* scale,
                  const float* shift, const float* gate, int act, int hw, int splits, float* out, int variant,
                  int sums, hipStream_t st) {
    if (M <= 0 || Co <= 0 || Ci <= 0 || (Co % 8) || (Ci % 8) || splits < 1 || variant >= NVAR || (sums && scale))
        return (int)hipErrorInvalidValue;
    // the gate needs >= 64-row frames (a chunk spans <= 2) and 32-bit row indices
    if (scale && (!shift || (gate && (hw < ROWS || M % hw || M >= ((int64_t)1 << 31)))))
        return (int)hipErrorInvalidValue;
    Prologue pro{scale, shift, gate, act, hw > 0 ? hw : 1};
    const int64_t rows = ((M + splits - 1) / splits + ROWS - 1) / ROWS * ROWS;
    const Variant v = pick(Co, Ci, variant);
#define L(A, B, C) if (v.tco == A && v.tci == B && v.wr == C) return launch<A, B, C>(dy, a, M, Co, Ci, splits, rows, pro, out, sums != 0, st);
    L(32, 256, 1) L(64, 128, 1) L(128, 128, 2) L(64, 256, 2) L(128, 64, 4) L(128, 256, 2)
#undef L
    return (int)hipErrorInvalidValue;
}

// FiLM weight and bias gradients: out [splits, Co, Ci] fp32 partials of dW = dy^T a with dy fp32 column-mapped
// (DyMap), a [M, Ci] bf16, and dbout [splits, Co] the column sums of dy; 64 x 128 tiles
// tile 0: 64 x 128 (the fp32 dy slab is re-read once per 128 ci), 1: 64 x 256 (half the dy re-reads, half the tiles)
int rt1_wgrad_dymap(const float* dyf, const int* map, const bf16_t* a, int64_t M, int Co, int Ci, int splits,
                    float* out, float* dbout, int tile, hipStream_t st) {
    if (M <= 0 || Co <= 0 || Ci <= 0 || (Co % 8) || (Ci % 8) || splits < 1 || !dyf || !map || !dbout)
        return (int)hipErrorInvalidValue;
    if (tile == 1) return launch_dymap<64, 256, 2>(dyf, map, a, M, Co, Ci, splits, out, dbout, st);
    return launch_dymap<64, 128, 1>(dyf, map, a, M, Co, Ci, splits, out, dbout, st);
}

}  // extern "C"
