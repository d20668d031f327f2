// Large-tile MFMA GEMM for the deep / wide 1x1 convolutions and their data gradients:
//
//     C[M, N] = pro(A)[M, K] . op(B)  (+ bias[N])                 A bf16 row-major, C bf16
//     op(B) = B^T for B [N, K] (NT: the forward of a 1x1 conv / Linear)
//           = B   for B [K, N] (NN: dY . W, the data gradient of the same weight)
//     pro(A) = silu(A * scale[k] + shift[k]) * gate[m / hw][k]     (PRO, NT only: the project conv's operand rebuilt
//              from the depthwise output y2 -- BN2 + SiLU + squeeze-excitation gate -- no bn_apply pass; the rebuilt
//              operand can also be stored for the weight gradient, `aout`)
//     STATS: per-column partial sum / sum of squares of the STORED bf16 C per 256-row tile (the consumer BatchNorm's
//            batch statistics, reduced by bn_finalize): no bn_stats pass over C
//
// Why a second GEMM next to gemm.hip / pwgemm.hip: at M = 76,800 pixel rows the wide-N expand / top convs (K = 384 ->
// N = 1536 / 2304) write a 6x wider C than they read; the 64..128-row tiles of the existing kernels re-read the weight
// slab from L2 per 128 rows and need a separate bn_stats pass over C (profiles/r5_trace1: pw_wide 384 -> 2304 at
// 1.4 TB/s + bn_stats 94 us).
//
// Design (CDNA4 rules from the MI355X HIP guide, §5 'glds vs register staging' row 1):
//   * 256 x BN tile, 8 waves = 512 threads as 2 (M) x 4 (N); each wave owns 128 x BN/4 of C in
//     v_mfma_f32_16x16x32_bf16 accumulators.  bn = 256: 256 x 256 tiles, K slabs of 64, one workgroup per CU;
//     bn = 128: 256 x 128 tiles, K slabs of 32, two workgroups per CU (one's DMA waits / epilogue overlap the other's
//     MFMAs).
//   * K slabs go through TWO LDS stages filled by global_load_lds_dwordx4 (LDS-DMA, no VGPR staging): the next slab's
//     DMA is issued before the current slab's MFMAs and waited for (vmcnt(0) + one barrier) at the next step.
//   * LDS images are lane-linear (the DMA writes base + 16 * lane); bank-conflict-free reads come from permuting the
//     per-lane SOURCE address (rule 21): K-contiguous [rows][BK] slabs (A, NT-B) store 16-B chunk c of row r at
//     kswz(r, c) (c ^ (r & 7) for 128-B rows, c ^ P[(r >> 2) & 3] for 64-B rows), conflict-free for the 16x16x32
//     operand's ds_read_b128; the NN B slab [BK k][BN n] (read with ds_read_b64_tr_b16, the gfx950 LDS transpose)
//     stores chunk c of k-row r at c ^ s(r), s(r) = ((r & 3) << 1) | (((r >> 3) & 1) << 3), conflict-free for the
//     transposed reads' 8 rows x 2 chunks (all four checked exhaustively against the lane-group bank rules).
//   * Out-of-range rows / K tails: the lane's DMA source is a 16-B zero block in global memory, so partial tiles and
//     K % BK != 0 need no masking in the MFMA loop.
//   * The product is formed as C^T = op(B)^T . A^T (MFMA-A = B rows), so a lane's accumulator holds 4 consecutive
//     columns of one row; the bf16 tile is staged through LDS and leaves as 16-B pieces of whole rows.
//   * XCD-aware bijective tile order: each XCD takes a contiguous range of the M-major tile list, so the N tiles of
//     one 256-row block run on one XCD together and its L2 serves the A rows to all of them.
//
// Measured (tools/bench_gemm256.py, profiles/r5_gemm256_bench.log): ahead of hipBLASLt / gemm.hip / pw_wide on the
// top and block-25 expand convs (1.06-1.10x) and the transformer QKV forward; 0.4-0.95x on the narrow-K / NN
// shapes, which stay where they are.  A persistent 4-stage variant (counted vmcnt, raw barriers, C stores in flight
// across tiles) measured slower on every shape (per-slab cost unchanged at ~1.8 us per 64-deep slab of a 256 x 256
// tile, i.e. ~48 % of the MFMA rate; profiles/r5_gemm256_persistent.log) and was not kept.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int NTHR = 512;
constexpr int BM = 256;

__device__ __attribute__((aligned(16))) uint4 g256_zero[1];   // zero source of out-of-range DMA lanes

struct G256Args {
    const bf16_t* A;
    const bf16_t* B;
    bf16_t* C;
    int M, N, K;
    const float* bias;                     // [N] or nullptr
    const float *scale, *shift, *gate;     // PRO: [K], [K], [M / hw, K]
    int hw;
    bf16_t* aout;                          // PRO: optional [M, K] store of the rebuilt operand
    float *ps, *pq;                        // STATS: [tiles_m, N]
};

constexpr int g256_occ(int bn) { return bn == 128 ? 2 : 1; }

template <int BN, int BK, bool NN>
struct G256 {
    static constexpr int A_BYTES = BM * BK * 2;                 // 32 / 16 KB
    static constexpr int B_BYTES = BN * BK * 2;
    static constexpr int STAGE = A_BYTES + B_BYTES;
    static constexpr int ROWB = BK * 2;                         // K-contiguous slab row bytes (128 or 64)
    static constexpr int WTM = BM / 2, WTN = BN / 4;            // wave sub-tile (2 x 4 waves)
    static constexpr int MT = WTM / 16, NTL = WTN / 16;         // 16 x 16 accumulators per wave
    static constexpr int TLD = BN + 8;                          // epilogue tile row pitch (bf16)
    static constexpr int TILE_BYTES = BM * TLD * 2;
    static constexpr int RED_BYTES = 2 * 2 * BN * 4;            // STATS: [2 row waves][sum, sq][BN]
    static constexpr int LDS = (2 * STAGE > TILE_BYTES ? 2 * STAGE : TILE_BYTES) + RED_BYTES;
    // DMA wave-instructions (1 KB each) per slab and per wave
    static constexpr int A_INS = A_BYTES / 1024 / 8;
    static constexpr int B_INS = B_BYTES / 1024 / 8;
    static constexpr int NN_ROWB = BN * 2;                      // NN B slab row bytes
    // workgroups per CU: the 256 x 128 tile (64 accumulator VGPRs) runs two, so one workgroup's DMA waits and
    // store-bound epilogue overlap the other's MFMAs; the 256 x 256 tile (128 accumulator VGPRs) runs one
    static constexpr int OCC = g256_occ(BN);
    static_assert(A_INS >= 1 && B_INS >= 1 && OCC * LDS <= 160 * 1024, "tile / LDS split");
};

// physical 16-B chunk of logical chunk c in row r of a K-contiguous slab: 128-B rows (BK = 64) c ^ (r & 7); 64-B rows
// (BK = 32) c ^ P[(r >> 2) & 3] with P = {0, 2, 3, 1} -- both conflict-free for the 16x16x32 operand's ds_read_b128
template <int BK>
__device__ __forceinline__ int kswz(int r, int c) {
    if constexpr (BK == 64) return c ^ (r & 7);
    else return c ^ ((0x78 >> (((r >> 2) & 3) * 2)) & 3);   // P packed 2 bits each: 0b01_11_10_00
}

// workgroup barrier for LDS hand-offs only: a __syncthreads() would also wait for this wave's outstanding global
// stores and DMAs (the previous tile's C stores and the next slabs must stay in flight across it)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int nn_swz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ bf16x8 tr_read8(const char* p0, const char* p1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int BN, int BK, bool NN, bool PRO, bool STATS, bool BIAS>
__global__ __launch_bounds__(NTHR, g256_occ(BN)) __attribute__((amdgpu_waves_per_eu(2 * g256_occ(BN), 2 * g256_occ(BN)))) void g256_kernel(G256Args g) {
    using S = G256<BN, BK, NN>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int lr = lane & 15, lh = lane >> 4;
    const int M = g.M, N = g.N, K = g.K;

    // XCD-aware bijective remap: the blocks b = x, x + 8, ... of XCD x take tiles [start(x), start(x) + count(x)), so
    // the N tiles of a 256-row block run on one XCD at the same time and its L2 serves them the A rows
    const int T = gridDim.x, b = blockIdx.x, x = b & 7, q = T >> 3, rr = T & 7;
    const int tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
    const int tiles_n = (N + BN - 1) / BN;
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;

    // ---- LDS-DMA of one K slab into stage `st`
    auto issue = [&](int s, int st) {
        const int k0 = s * BK;
        char* As = smem + st * S::STAGE;
        char* Bs = As + S::A_BYTES;
#pragma unroll
        for (int i = 0; i < S::A_INS; ++i) {
            constexpr int RPI = 1024 / S::ROWB, CPR = S::ROWB / 16;   // rows / chunks per wave-instruction
            const int j = wave * S::A_INS + i;
            const int r = j * RPI + lane / CPR;
            const int c = kswz<BK>(r, lane % CPR);
            const int64_t m = m0 + r;
            const int k = k0 + c * 8;
            const void* src = (m < M && k < K) ? (const void*)(g.A + m * K + k) : (const void*)g256_zero;
            dma16(src, As + j * 1024);
        }
#pragma unroll
        for (int i = 0; i < S::B_INS; ++i) {
            const int j = wave * S::B_INS + i;
            if constexpr (NN) {
                constexpr int RPI = 1024 / S::NN_ROWB;          // k rows per wave-instruction (2 or 4)
                constexpr int CPR = S::NN_ROWB / 16;            // 16-B chunks per row (32 or 16)
                const int r = j * RPI + lane / CPR;
                const int c = (lane % CPR) ^ nn_swz(r);
                const int k = k0 + r, n = n0 + c * 8;
                const void* src = (k < K && n < N) ? (const void*)(g.B + (int64_t)k * N + n) : (const void*)g256_zero;
                dma16(src, Bs + j * 1024);
            } else {
                constexpr int RPI = 1024 / S::ROWB, CPR = S::ROWB / 16;
                const int r = j * RPI + lane / CPR;
                const int c = kswz<BK>(r, lane % CPR);
                const int n = n0 + r, k = k0 + c * 8;
                const void* src = (n < N && k < K) ? (const void*)(g.B + (int64_t)n * K + k) : (const void*)g256_zero;
                dma16(src, Bs + j * 1024);
            }
        }
    };

    // ---- PRO: rebuild the A slab in place, each 16-B chunk once (4 per thread), zero chunks left as they are
    auto transform = [&](int s, int st) {
        const int k0 = s * BK;
        char* As = smem + st * S::STAGE;
        constexpr int CPR = S::ROWB / 16;
        // the physical chunk pc of row r holds logical chunk kswz(r, pc) (the swizzle is an involution); one chunk at
        // a time: the accumulators are live here
#pragma unroll 1
        for (int u = 0; u < BM * CPR / NTHR; ++u) {
            const int id = t + u * NTHR, r = id / CPR, pc = id % CPR, c = kswz<BK>(r, pc);
            const int64_t m = m0 + r;
            const int k = k0 + c * 8;
            if (m < M && k < K) {
                uint4* p = reinterpret_cast<uint4*>(As + r * S::ROWB + pc * 16);
                uint4 v = *p;
                float f[8], sc[8], sh[8], gt[8];
                unpack8(v, f);
                load8f(g.scale + k, sc);
                load8f(g.shift + k, sh);
                load8f(g.gate + (int64_t)((uint32_t)m / (uint32_t)g.hw) * K + k, gt);   // 32-bit divide (M < 2^31)
#pragma unroll
                for (int e = 0; e < 8; ++e) f[e] = silu(fmaf(f[e], sc[e], sh[e])) * gt[e];
                v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]); v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
                *p = v;
                if (g.aout && tn == 0) *reinterpret_cast<uint4*>(g.aout + m * K + k) = v;
            }
        }
    };

    f32x4 acc[S::NTL][S::MT];

    auto compute = [&](int st) {
        const char* As = smem + st * S::STAGE;
        const char* Bs = As + S::A_BYTES;
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
            const int ch = ks * 4 + lh;                         // this lane's logical 16-B chunk of a 32-k step
            // the NTL B fragments stay in registers; the A fragments stream through (one live at a time keeps the
            // 256 x 128 variants within the 128 VGPRs of two workgroups per CU)
            bf16x8 fb[S::NTL];
#pragma unroll
            for (int i = 0; i < S::NTL; ++i) {
                if constexpr (NN) {
                    // rows k = ks*32 + 8*lh + q (+4), columns n = nb + 4p: lane 4q + p of each 16-lane group
                    const int q4 = lr >> 2, p4 = lr & 3;
                    const int nb = wn * S::WTN + i * 16;
                    const int r0 = ks * 32 + lh * 8 + q4, r1 = r0 + 4;
                    const int cc = (nb >> 3) + (p4 >> 1), off = (p4 & 1) * 8;
                    fb[i] = tr_read8(Bs + r0 * S::NN_ROWB + ((cc ^ nn_swz(r0)) << 4) + off,
                                     Bs + r1 * S::NN_ROWB + ((cc ^ nn_swz(r1)) << 4) + off);
                } else {
                    const int r = wn * S::WTN + i * 16 + lr;
                    fb[i] = *reinterpret_cast<const bf16x8*>(Bs + r * S::ROWB + (kswz<BK>(r, ch) << 4));
                }
            }
#pragma unroll
            for (int j = 0; j < S::MT; ++j) {
                const int r = wm * S::WTM + j * 16 + lr;
                const bf16x8 fa = *reinterpret_cast<const bf16x8*>(As + r * S::ROWB + (kswz<BK>(r, ch) << 4));
#pragma unroll
                for (int i = 0; i < S::NTL; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa, acc[i][j], 0, 0, 0);
            }
        }
    };

    const int ns = (K + BK - 1) / BK;
#pragma unroll
    for (int i = 0; i < S::NTL; ++i)
#pragma unroll
        for (int j = 0; j < S::MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue(0, 0);
    for (int s = 0; s < ns; ++s) {
        // slab s has landed (this wave's DMA) and every wave is past its reads of the other stage (step s - 1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if constexpr (PRO) {
            transform(s, s & 1);
            __syncthreads();
        }
        if (s + 1 < ns) issue(s + 1, (s + 1) & 1);
        compute(s & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                            // operand reads done: the LDS becomes the C tile

    // ---- epilogue: lane holds C[m][n .. n+3], m = wm*128 + j*16 + lr, n = wn*WTN + i*16 + lh*4 (tile-local)
    bf16_t* Tl = reinterpret_cast<bf16_t*>(smem);
    float* red = reinterpret_cast<float*>(smem + (S::LDS - S::RED_BYTES));
#pragma unroll
    for (int i = 0; i < S::NTL; ++i) {
        const int nl = wn * S::WTN + i * 16 + lh * 4;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (BIAS) {
            if (n0 + nl < N) {
                const float4 b4 = *reinterpret_cast<const float4*>(g.bias + n0 + nl);
                bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
            }
        }
        float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < S::MT; ++j) {
            const int ml = wm * S::WTM + j * 16 + lr;
            uint2 u;
            u.x = pack2(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1]);
            u.y = pack2(acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]);
            *reinterpret_cast<uint2*>(Tl + ml * S::TLD + nl) = u;
            if constexpr (STATS) {
                if (m0 + ml < M) {                              // statistics describe the stored bf16 rows
                    const float s0 = __uint_as_float(u.x << 16), s1 = __uint_as_float(u.x & 0xffff0000u);
                    const float s2 = __uint_as_float(u.y << 16), s3 = __uint_as_float(u.y & 0xffff0000u);
                    ssum[0] += s0; ssq[0] = fmaf(s0, s0, ssq[0]);
                    ssum[1] += s1; ssq[1] = fmaf(s1, s1, ssq[1]);
                    ssum[2] += s2; ssq[2] = fmaf(s2, s2, ssq[2]);
                    ssum[3] += s3; ssq[3] = fmaf(s3, s3, ssq[3]);
                }
            }
        }
        if constexpr (STATS) {
            // over the 16 row lanes of each lane group (fixed xor order); the 2 row waves combine through LDS below
#pragma unroll
            for (int e = 0; e < 4; ++e) {
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    ssum[e] += __shfl_xor(ssum[e], o, 64);
                    ssq[e] += __shfl_xor(ssq[e], o, 64);
                }
                if (lr == 0) {
                    red[(wm * 2) * BN + nl + e] = ssum[e];
                    red[(wm * 2 + 1) * BN + nl + e] = ssq[e];
                }
            }
        }
    }
    lds_barrier();
    if constexpr (STATS) {
        for (int c = t; c < BN; c += NTHR) {
            if (n0 + c < N) {
                g.ps[(int64_t)tm * N + n0 + c] = red[c] + red[2 * BN + c];
                g.pq[(int64_t)tm * N + n0 + c] = red[BN + c] + red[3 * BN + c];
            }
        }
    }
    // 16-B pieces of whole tile rows (N % 8 == 0)
    constexpr int C8 = BN / 8;
    for (int o = t; o < BM * C8; o += NTHR) {
        const int r = o / C8, c = (o - r * C8) * 8;
        if (m0 + r < M && n0 + c < N)
            *reinterpret_cast<uint4*>(g.C + (m0 + r) * N + n0 + c) = *reinterpret_cast<const uint4*>(Tl + r * S::TLD + c);
    }
}

template <int BN, int BK, bool NN, bool PRO, bool STATS, bool BIAS>
int launch(const G256Args& a, hipStream_t st) {
    using S = G256<BN, BK, NN>;
    auto kern = g256_kernel<BN, BK, NN, PRO, STATS, BIAS>;
    static const hipError_t attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       S::LDS);
    if (attr != hipSuccess) return (int)attr;
    const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(NTHR), S::LDS, st, a);
    return (int)hipGetLastError();
}

template <int BN, int BK>
int dispatch(const G256Args& a, bool nn, bool pro, bool stats, bool bias, hipStream_t st) {
    if (nn) {
        if (pro || stats || bias) return (int)hipErrorInvalidValue;
        return launch<BN, BK, true, false, false, false>(a, st);
    }
    if (pro) {
        if (bias) return (int)hipErrorInvalidValue;
        return stats ? launch<BN, BK, false, true, true, false>(a, st) : launch<BN, BK, false, true, false, false>(a, st);
    }
    if (stats) return bias ? (int)hipErrorInvalidValue : launch<BN, BK, false, false, true, false>(a, st);
    return bias ? launch<BN, BK, false, false, false, true>(a, st) : launch<BN, BK, false, false, false, false>(a, st);
}

}  // namespace

extern "C" {

int rt1_g256_tiles_m(int M) { return (M + BM - 1) / BM; }

// C = pro(A) . op(B) (+ bias): nn = 1: B [K, N] (else [N, K]); bn = 256 or 128 (N tile); ps / pq: STATS partials
// [rt1_g256_tiles_m(M), N]; scale / shift / gate / hw / aout: the PRO operand rebuild (NT only)
int rt1_g256(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int nn, const float* bias,
             const float* scale, const float* shift, const float* gate, int hw, bf16_t* aout, float* ps, float* pq,
             int bn, hipStream_t st) {
    if (M <= 0 || N <= 0 || K <= 0 || (N % 8) || (K % 8)) return (int)hipErrorInvalidValue;
    const bool pro = scale != nullptr;
    if (pro && (!shift || !gate || hw <= 0 || M % hw)) return (int)hipErrorInvalidValue;
    if ((ps != nullptr) != (pq != nullptr) || (aout && !pro)) return (int)hipErrorInvalidValue;
    G256Args a{A, B, C, M, N, K, bias, scale, shift, gate, hw, aout, ps, pq};
    // bn = 128: 256 x 128 tiles, K slabs of 32, two workgroups per CU; bn = 256: 256 x 256, slabs of 64, one per CU
    if (bn == 128) return dispatch<128, 32>(a, nn != 0, pro, ps != nullptr, bias != nullptr, st);
    if (bn == 256) return dispatch<256, 64>(a, nn != 0, pro, ps != nullptr, bias != nullptr, st);
    return (int)hipErrorInvalidValue;
}

}  // extern "C"
