// Persistent, LDS-DMA-pipelined MFMA GEMM for the large plain products of the step (gemm.hip v2):
//
//     C[M, N] = A[M, K] . B[N, K]^T  (+ bias[N])  [ -> dropout -> + R ]       A, B bf16 (K contiguous, "NT")
//
// epilogues: bf16 C with optional per-(M half-tile) column partial sums / sums of squares of the STORED values (the
// consumer BatchNorm's statistics, reduced by bn_finalize -- no bn_stats pass), or fp32 C = R + dropout(acc + bias)
// with R an fp32 residual stream (the transformer's out-projection / FF residual, SURVEY K15 / K16: no tf_resid
// pass; the dropout hash is transformer.hip's, so its backward regenerates the same mask).
//
// Sites (SURVEY K3/K6 blocks 24-25, K8 top + conv1x1, K13/K15/K16 and their data gradients, which take the weight
// transposed so every product is NT): hipBLASLt runs them at 20-60 % of their roofline and v1 (gemm.hip, register-
// staged single LDS buffer) loses to it on the N >= 384 shapes (profiles/r3_gemm_bench.log).  What v1 lacks there:
//
// * Staging: global -> LDS straight through LDS-DMA (`global_load_lds_dwordx4`, 16 B per lane, no VGPR round trip,
//   no ds_write pass) into a 3-stage ring, issued two K-slabs ahead: slab g+2 streams in while slab g multiplies.
//   One wave-instruction fills 1 KiB = 8 rows x 128 B of a [rows][64] bf16 slab image; the image is lane-linear, so
//   its bank swizzle is applied on the SOURCE address: 16-B chunk c of row r lands at position c ^ ((r >> 1) & 7),
//   which makes the 16-row fragment reads (ds_read_b128) conflict-free.  Waits are counted (`s_waitcnt vmcnt(8)`:
//   one slab of 8 DMAs per wave left in flight) before a raw `s_barrier`; no `__syncthreads()` (its vmcnt(0) would
//   drain the ring) and a single `extern __shared__` array (a second one makes hipcc wait vmcnt(0) per k-step).
// * Persistence: one workgroup per CU walks its tiles as ONE flat slab sequence, so the next tile's first slabs are
//   already in flight while the current tile's epilogue stores (short-K shapes: top K = 384 is 6 slabs per tile).
//   Tiles are dealt XCD-major (bijective): the workgroups of one XCD take consecutive tiles of the same M row block,
//   whose A slab its L2 then serves to all of them.
// * Tile 128 x 128 x 64, 4 waves of 64 x 64 (4 x 4 accumulators of v_mfma_f32_16x16x32_bf16).  The product is formed
//   as C^T = B . A^T, so a lane's accumulator is 4 consecutive columns of one row (8- / 16-byte stores).
//
// Rows past M / N and K chunks past K read a 16-byte zero line instead of the operand (no branches in the DMA issue,
// no out-of-range reads); K and N must be multiples of 8, and a bias vector padded to whole 128-column tiles is
// always passed (zeros for none).
#include "common.h"

#include <algorithm>

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BLOCK = 256;
constexpr int BM = 128, BN = 128;
// pipeline variants (BK, STAGES, workgroups / CU): the slab depth, the ring depth (prefetch distance STAGES - 1) and
// the occupancy the register / LDS budget targets
template <int BK_, int STAGES_, int OCC_>
struct G2Cfg {
    static constexpr int BK = BK_, STAGES = STAGES_, OCC = OCC_;
    static constexpr int ROWB = BK * 2;                             // bytes per slab row
    static constexpr int CPR = ROWB / 16;                           // 16-B chunks per row (8 or 4)
    static constexpr int SLAB_BYTES = BM * BK * 2;                  // one operand's slab image
    static constexpr int STAGE_BYTES = 2 * SLAB_BYTES;              // A + B
    static constexpr int LDS_BYTES = STAGES * STAGE_BYTES;
    static constexpr int DMA_PER_SLAB = SLAB_BYTES / 1024 / 4;      // wave-instructions per operand slab per wave
    // 16-B chunk c of row r sits at position c ^ swz(r): the 16 rows of a fragment read hit distinct 16-B bank slots
    static __device__ __forceinline__ int swz(int r) { return CPR == 8 ? (r >> 1) & 7 : (r >> 2) & 3; }
};

__device__ __attribute__((aligned(16))) uint4 g_zero16 = {0u, 0u, 0u, 0u};

struct G2Args {
    const bf16_t* A;
    const bf16_t* B;
    void* C;
    int M, N, K;
    const float* bias;            // [ceil(N / 128) * 128] (zeros past N, and all zeros for none: loaded unconditionally)
    float *ps, *pq;               // bf16 C + stats: [2 * tiles_m, N] partials
    const float* R;               // fp32 C: residual [M, N] (nullptr: none)
    float p;                      // fp32 C: dropout probability on acc + bias (0: off)
    uint32_t salt;
    const uint32_t* seed_dev;
};

__device__ __forceinline__ uint32_t mix32(uint32_t seed, uint32_t a, uint32_t b) {   // transformer.hip's hash
    uint32_t x = seed ^ (a * 0x9E3779B1u) ^ (b * 0x85EBCA77u) ^ 0x27d4eb2fu;
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}


// One LDS-DMA wave-instruction: 16 B per lane from `src` into LDS at the wave-uniform `dst` + lane * 16.  Issued as
// inline asm so hipcc's waitcnt pass does not see an LDS write in flight: through the builtin it drains the whole
// ring (`s_waitcnt vmcnt(0)`) before the next ds_read of ANY stage.  The ring's waits are the explicit counted
// vmcnt(8) / vmcnt(0) of the main loop; the compiler's own waits for its loads stay correct (vmcnt counts in
// order, so an extra DMA in flight only makes them more conservative).
__device__ __forceinline__ void dma16(const void* src, const char* dst) {
    const uint32_t lds = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)dst);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
                 : "memory");
}

// raw workgroup barrier that is also a compiler fence: no LDS read may move above it (an LDS read hoisted between
// this wave's counted vmcnt and the barrier would see another wave's DMA half-landed)
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }

template <class CF, bool OUT_F32, bool STATS>
__global__ __launch_bounds__(BLOCK, CF::OCC) void gemm2_kernel(G2Args g) {
    constexpr int BK = CF::BK, STAGES = CF::STAGES, SLAB_BYTES = CF::SLAB_BYTES, STAGE_BYTES = CF::STAGE_BYTES;
    constexpr int DMA_PER_SLAB = CF::DMA_PER_SLAB, CPR = CF::CPR, ROWB = CF::ROWB;
    constexpr int INFLIGHT = 2 * DMA_PER_SLAB * (STAGES - 2);       // DMAs per wave that may stay in flight
    extern __shared__ __attribute__((aligned(1024))) char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int lr = lane & 15, lh = lane >> 4;
    const int wm = wave & 1, wn = wave >> 1;
    const int M = g.M, N = g.N, K = g.K;
    const int KS = (K + BK - 1) / BK;
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    const int T = tiles_m * tiles_n;

    // XCD-major bijective deal: workgroup b runs on XCD b % 8; XCD x owns tiles [lo, hi); its workgroups stride it
    const int P = gridDim.x, b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const int pw = (P >> 3) + ((P & 7) > xcd ? 1 : 0);          // workgroups on this XCD
    const int q = T >> 3, rr = T & 7;
    const int lo = xcd * q + min(xcd, rr), hi = lo + q + (xcd < rr ? 1 : 0);
    const int nloc = slot < hi - lo ? (hi - lo - slot + pw - 1) / pw : 0;
    const int G = nloc * KS;

    // LDS-DMA of slab gi: operand rows [row0, row0 + 128) of A (M) and B (N), k chunk [k0, k0 + 64)
    auto issue = [&](int gi) {
        const int i = gi / KS, ks = gi - i * KS;
        const int tile = lo + slot + i * pw;
        const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
        const int k0 = ks * BK;
        char* st = smem + (gi % STAGES) * STAGE_BYTES;
#pragma unroll
        for (int u = 0; u < DMA_PER_SLAB; ++u) {
            const int qi = (wave * DMA_PER_SLAB + u) * 64 + lane;     // 16-B position in the slab image
            const int r = qi / CPR, c = (qi % CPR) ^ CF::swz(r);      // row, source chunk
            const int k = k0 + c * 8;
            const int64_t ma = (int64_t)tm * BM + r, nb = (int64_t)tn * BN + r;
            const void* sa = (ma < M && k < K) ? (const void*)(g.A + ma * K + k) : (const void*)&g_zero16;
            const void* sb = (nb < N && k < K) ? (const void*)(g.B + nb * K + k) : (const void*)&g_zero16;
            const int ofs = (wave * DMA_PER_SLAB + u) * 1024;
            dma16(sa, st + ofs);
            dma16(sb, st + SLAB_BYTES + ofs);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
        if (s0 < G) issue(s0);
    for (int gi = 0; gi < G; ++gi) {
        // slab gi has landed once at most INFLIGHT VMEM operations of this wave are outstanding: the next STAGES - 2
        // slabs' DMAs were issued after slab gi's and loads complete in order, so a DMA of slab gi still in flight
        // would mean more (epilogue stores only add to the count: more conservative).  Near the end, drain.
        if (gi + STAGES - 2 >= G) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(INFLIGHT) : "memory");
        barrier_raw();
        // into the stage read by slab gi - 1, which every wave has finished (it passed this barrier after them)
        if (gi + STAGES - 1 < G) issue(gi + STAGES - 1);
        const char* st = smem + (gi % STAGES) * STAGE_BYTES;
        const char* Al = st;
        const char* Bl = st + SLAB_BYTES;
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
            const int c = ks * 4 + lh;
            bf16x8 fa[4], fb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = wm * 64 + j * 16 + lr;
                fa[j] = *reinterpret_cast<const bf16x8*>(Al + r * ROWB + ((c ^ CF::swz(r)) << 4));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wn * 64 + i * 16 + lr;
                fb[i] = *reinterpret_cast<const bf16x8*>(Bl + r * ROWB + ((c ^ CF::swz(r)) << 4));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
        }
        const int i_t = gi / KS;
        if (gi - i_t * KS != KS - 1) continue;

        // ---- epilogue of tile i_t: lane holds C[m][n .. n+3], m = m0 + wm*64 + j*16 + lr, n = n0 + wn*64 + i*16 + lh*4
        const int tile = lo + slot + i_t * pw;
        const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
        const int64_t m0 = (int64_t)tm * BM + wm * 64;
        const int n0 = tn * BN + wn * 64;
        uint32_t seed = 0;
        if constexpr (OUT_F32) seed = g.p > 0.f ? dev_seed(g.salt, g.seed_dev) : 0u;
        const float ik = (OUT_F32 && g.p > 0.f) ? 1.f / (1.f - g.p) : 1.f;
        const __attribute__((address_space(4))) float* bias_c =
            (const __attribute__((address_space(4))) float*)(uintptr_t)g.bias;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = n0 + i * 16 + lh * 4;
            // the bias through SCALAR loads (padded to whole 128-column tiles: in range): a vector load here would
            // make hipcc wait vmcnt(0) at its use -- draining the DMA ring once per tile -- since the DMAs are
            // invisible to its count; the lane then picks its 4 of the wave's 16 values of this column block
            float bv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int cb = n0 + i * 16 + e;
                const float c0 = bias_c[cb], c1 = bias_c[cb + 4], c2 = bias_c[cb + 8], c3 = bias_c[cb + 12];
                bv[e] = lh == 0 ? c0 : (lh == 1 ? c1 : (lh == 2 ? c2 : c3));
            }
            float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t m = m0 + j * 16 + lr;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
                acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (m >= M || n >= N) continue;
                if constexpr (OUT_F32) {
                    if (g.p > 0.f) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const bool drop = (float)(mix32(seed, (uint32_t)m, (uint32_t)(n + e)) >> 8) *
                                              (1.0f / 16777216.0f) < g.p;
                            v[e] = drop ? 0.f : v[e] * ik;
                        }
                    }
                    if (g.R) {
                        const float4 r4 = *reinterpret_cast<const float4*>(g.R + m * N + n);
                        v[0] += r4.x; v[1] += r4.y; v[2] += r4.z; v[3] += r4.w;
                    }
                    *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + m * N + n) =
                        make_float4(v[0], v[1], v[2], v[3]);
                } else {
                    uint2 u;
                    u.x = pack2(v[0], v[1]);
                    u.y = pack2(v[2], v[3]);
                    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(g.C) + m * N + n) = u;
                    if constexpr (STATS) {      // statistics describe the stored bf16 tensor
                        const float s[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                            __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            ssum[e] += s[e];
                            ssq[e] = fmaf(s[e], s[e], ssq[e]);
                        }
                    }
                }
            }
            if constexpr (STATS) {
                // over the 16 row lanes of each column group (fixed xor order); one partial row per (tile, wm)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) {
                        ssum[e] += __shfl_xor(ssum[e], o, 64);
                        ssq[e] += __shfl_xor(ssq[e], o, 64);
                    }
                }
                if (lr == 0 && n < N) {
                    const int64_t prow = (int64_t)(tm * 2 + wm) * N + n;
                    *reinterpret_cast<float4*>(g.ps + prow) = make_float4(ssum[0], ssum[1], ssum[2], ssum[3]);
                    *reinterpret_cast<float4*>(g.pq + prow) = make_float4(ssq[0], ssq[1], ssq[2], ssq[3]);
                }
            }
        }
    }
}

// pipeline variants: 0 = BK 64 x 3 stages, 1 WG/CU (96 KiB); 1 = BK 32 x 4 stages, 2 WGs/CU (64 KiB each);
// 2 = BK 32 x 8 stages, 1 WG/CU (128 KiB); 3 = BK 64 x 2 stages, 2 WGs/CU (64 KiB each)
typedef G2Cfg<64, 3, 1> V0;
typedef G2Cfg<32, 4, 2> V1;
typedef G2Cfg<32, 8, 1> V2;
typedef G2Cfg<64, 2, 2> V3;

template <class CF>
int launch_v(const G2Args& a, bool out_f32, bool stats, int grid, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)gemm2_kernel<CF, false, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, CF::LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)gemm2_kernel<CF, false, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, CF::LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)gemm2_kernel<CF, true, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, CF::LDS_BYTES);
        attr = true;
    }
    const int g = grid * CF::OCC;
    if (out_f32)
        hipLaunchKernelGGL((gemm2_kernel<CF, true, false>), dim3(g), dim3(BLOCK), CF::LDS_BYTES, st, a);
    else if (stats)
        hipLaunchKernelGGL((gemm2_kernel<CF, false, true>), dim3(g), dim3(BLOCK), CF::LDS_BYTES, st, a);
    else
        hipLaunchKernelGGL((gemm2_kernel<CF, false, false>), dim3(g), dim3(BLOCK), CF::LDS_BYTES, st, a);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// partial rows of the stats epilogue
int rt1_gemm2_stat_rows(int M) { return 2 * ((M + BM - 1) / BM); }

// workgroups of a launch: one per CU (1 workgroup / CU: 96 KiB of LDS), never more than the tiles
int rt1_gemm2_grid(int M, int N, int cus) {
    const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    return T < cus ? T : cus;
}

int rt1_gemm2(const bf16_t* A, const bf16_t* B, void* C, int M, int N, int K, const float* bias, int out_f32,
              float* ps, float* pq, const float* R, float p, uint32_t salt, const uint32_t* seed_dev, int grid,
              hipStream_t st, int variant) {
    if (M <= 0 || N <= 0 || K <= 0 || (N % 8) || (K % 8) || grid <= 0 || !bias) return (int)hipErrorInvalidValue;
    if ((ps != nullptr) != (pq != nullptr) || (out_f32 && ps) || (!out_f32 && (R || p > 0.f)))
        return (int)hipErrorInvalidValue;
    G2Args a{A, B, C, M, N, K, bias, ps, pq, R, p, salt, seed_dev};
    const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    switch (variant) {
        case 1: return launch_v<V1>(a, out_f32, ps != nullptr, std::min(grid, (T + 1) / 2), st);
        case 2: return launch_v<V2>(a, out_f32, ps != nullptr, grid, st);
        case 3: return launch_v<V3>(a, out_f32, ps != nullptr, std::min(grid, (T + 1) / 2), st);
        default: return launch_v<V0>(a, out_f32, ps != nullptr, grid, st);
    }
}

}  // extern "C"
