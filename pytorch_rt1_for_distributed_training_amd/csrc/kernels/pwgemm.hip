// Skinny pointwise-convolution GEMM on MFMA: C[M, N] = A[M, K] @ B[N, K]^T, bf16 in / fp32 accumulate /
// bf16 out, for the EfficientNet-B3 1x1 convolutions where M (frames x pixels) is 10^6..10^7 and K, N
// are small (24..288).  (expand / project convs of the 26 MBConv blocks.)
//
// Why not hipBLASLt: with N = 24..48 its smallest macro tile (64x256 / 32x256) is mostly padding, and
// every one of these shapes is HBM-bound (arithmetic intensity K*N/(K+N) < 40 flop/B, far below the
// ~420 flop/B balance point of MI355X), so the whole game is streaming A once at full bandwidth.
//
// Design (CDNA4, wave64, mfma_f32_16x16x32_bf16):
//   * B (the weight, <= 288x288) is staged once per workgroup into LDS, zero-padded to [NT*16][KC*32].
//   * Each wave owns strips of R x 16 rows of A and computes ALL N columns for them: the A fragments
//     are loaded straight from HBM in MFMA operand layout (16 B per lane, lanes 16 rows x 64 B), so A
//     is read exactly once and never touches LDS; the next strip's fragments are prefetched into a
//     second register set while the current strip's MFMAs run.
//   * The product is computed transposed, C^T = B . A^T: MFMA-A = weight rows (from LDS), MFMA-B = A rows,
//     so the accumulator's 4 registers are 4 CONSECUTIVE output channels of one pixel and each lane
//     stores 8 contiguous bytes (the natural orientation would scatter 2-byte stores down a column).
//   * R (strips per wave-iteration) is sized so accumulators + two A fragment sets stay ~128 VGPRs.
//   * PRO (project convs): the operand is rebuilt in registers as A = silu(y*scale + shift) * gate[frame] from the
//     depthwise output y, so the block never writes (and the GEMM never reads) a separate A tensor.  scale/shift
//     sit in LDS; each wave stages the gate rows of the <= 2 frames its strip touches (prefetched one strip ahead
//     with the A fragments).  Same formula and rounding as bn_apply, so the product is bit-identical.
//   * BNB (project data gradients of blocks 0-7): the operand is the BN3-backward output
//     dy3 = k1 * (dout * fmul[frame] * keep[frame]) + k2 * y3 + k0, rebuilt from (dout, y3) with bn_bwd_apply's
//     formula and rounding and stored once (aout) for the project weight-gradient / projbwd pass: the separate
//     bn_bwd_apply launch and the GEMM's read of dy3 disappear.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BLOCK = 256;

template <int KC, int N, bool BNB = false>
struct PwShape {
    static constexpr int NT = (N + 15) / 16;
    // fragment sets held per strip row: A (+ its prefetch), and y3 (+ prefetch) for the BN-backward prologue
    static constexpr int r0 = 128 / (4 * (NT + (BNB ? 4 : 2) * KC));
    static constexpr int R = r0 < 1 ? 1 : (r0 > 8 ? 8 : r0);
    static constexpr int LDB = KC * 32 + 8;        // weight image row stride (bf16): +16 B against bank aliasing
    static constexpr int LDC = N + 8;              // output staging row stride (bf16): +16 B, rows 16-B aligned
    static constexpr size_t b_bytes = (size_t)NT * 16 * LDB * 2;
    static constexpr size_t c_bytes = (size_t)R * 16 * LDC * 2;   // per wave
    static constexpr size_t red_bytes = 4 * 64 * 16 * 4;           // BN-stat partials, aliases the C images
    static constexpr size_t lds = b_bytes + (4 * c_bytes > red_bytes ? 4 * c_bytes : red_bytes);
    static constexpr int KCP = KC * 32;
    static constexpr size_t pro_bytes = (size_t)(3 + 4 * 2) * KCP * 4;   // 2-3 channel vectors + 4 waves x 2 frame rows
};

struct PwPro {
    const float *scale, *shift, *gate;   // [K], [K], [M / hw, K]
    int hw;
    bf16_t* aout;                        // optional [M, K]: the rebuilt operand, for consumers that need it stored
};

// BN-backward operand prologue: A (the kernel's operand input) is dout; pro.gate = fmul rows, pro.hw, pro.aout = dy3
struct PwBnb {
    const bf16_t* y;                                   // [M, K] BN input (y3)
    const float *gamma, *mean, *rstd, *mdz, *mdzx;     // [K] (gamma may be nullptr)
    const float* keep;                                 // [M / hw] drop-path mask or nullptr
};


template <int KC, int R>
__device__ __forceinline__ void load_a(bf16x8 (&af)[R][KC], const bf16_t* __restrict__ A, int64_t m0, int M, int K,
                                       int lr, int lh) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t row = m0 + r * 16 + lr;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            const int col = kc * 32 + lh * 8;
            if (row < M && col < K)
                af[r][kc] = *reinterpret_cast<const bf16x8*>(A + row * K + col);
            else
                af[r][kc] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// STATS: per-workgroup partial (sum, sum of squares) of every output channel of the STORED bf16 C,
// written to ps/pq[blockIdx.x][N] for the consumer BatchNorm (bn_finalize reduces the rows).
// this lane's share (KC floats) of the gate rows of the <= 2 frames strip [m0, m0 + 16R) touches
template <int KC, int R>
__device__ __forceinline__ void load_gate(float (&gv)[KC], const PwPro& p, int64_t m0, int M, int K, int lane,
                                          const float* __restrict__ keep = nullptr) {
    constexpr int KCP = KC * 32;
    const int f0 = (int)(m0 / p.hw);
    const int64_t last = (m0 + 16 * R < M ? m0 + 16 * R : M) - 1;
    const int fl = (int)(last / p.hw);
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const int i = lane + j * 64, slot = i >= KCP ? 1 : 0, c = i - slot * KCP;
        float v = (c < K && f0 + slot <= fl) ? p.gate[(int64_t)(f0 + slot) * K + c] : 0.f;
        if (keep && f0 + slot <= fl) v *= keep[f0 + slot];      // fmul * keep, rounded as the torch product was
        gv[j] = v;
    }
}

template <int KC, int N, bool STATS, bool PRO, bool BNB = false>
__global__ __launch_bounds__(BLOCK) void pw_gemm_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                        int M, int K, bf16_t* __restrict__ C, float* __restrict__ ps,
                                                        float* __restrict__ pq, PwPro pro, PwBnb bnb) {
    using S = PwShape<KC, N, BNB>;
    constexpr bool ROWS = PRO || BNB;           // per-frame rows staged per wave (gate / fmul)
    constexpr int R = S::R, LDB = S::LDB, LDC = S::LDC, NT = S::NT, KCP = S::KCP;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* bl = reinterpret_cast<bf16_t*>(smem);
    for (int i = threadIdx.x; i < NT * 16 * KC * 4; i += BLOCK) {   // 16-B chunks, KC*4 per row
        const int n = i / (KC * 4), c = (i - n * (KC * 4)) * 8;
        uint4 u = make_uint4(0, 0, 0, 0);
        if (n < N && c < K) u = *reinterpret_cast<const uint4*>(B + (int64_t)n * K + c);
        *reinterpret_cast<uint4*>(bl + n * LDB + c) = u;
    }
    float* psc = reinterpret_cast<float*>(smem + S::lds);
    float* psh = psc + KCP;
    float* pk2 = psh + KCP;
    if constexpr (PRO) {
        for (int i = threadIdx.x; i < KCP; i += BLOCK) {
            psc[i] = i < K ? pro.scale[i] : 0.f;
            psh[i] = i < K ? pro.shift[i] : 0.f;
        }
    }
    if constexpr (BNB) {
        // bn_bwd_apply's constants: k0 (psc), k1 (psh), k2 (pk2); zero past K so the padding columns stay zero
        for (int i = threadIdx.x; i < KCP; i += BLOCK) {
            float k0 = 0.f, k1 = 0.f, k2 = 0.f;
            if (i < K) {
                const float rr = bnb.rstd[i], b = bnb.mdzx[i];
                k1 = (bnb.gamma ? bnb.gamma[i] : 1.f) * rr;
                k0 = -k1 * (bnb.mdz[i] - bnb.mean[i] * rr * b);
                k2 = -k1 * rr * b;
            }
            psc[i] = k0;
            psh[i] = k1;
            pk2[i] = k2;
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float* gwl = psc + 3 * KCP + wave * 2 * KCP;     // PRO / BNB: this wave's two frame rows
    const int lr = lane & 15, lh = lane >> 4;
    bf16_t* cl = reinterpret_cast<bf16_t*>(smem + S::b_bytes + wave * S::c_bytes);
    const int64_t strips = ((int64_t)M + 16 * R - 1) / (16 * R);
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t s = (int64_t)blockIdx.x * 4 + wave;
    // statistics lane map: lane owns channel chunk sc8 (8 channels) of rows srow0, srow0+RG, ...
    constexpr int CPR = N / 8, RG = 64 / CPR;
    const int sc8 = lane % CPR, srow0 = lane / CPR;
    float sacc[8], qacc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sacc[j] = qacc[j] = 0.f;

    bf16x8 af[R][KC], an[R][KC];
    bf16x8 ay[BNB ? R : 1][BNB ? KC : 1], ayn[BNB ? R : 1][BNB ? KC : 1];
    float gc[ROWS ? KC : 1], gn[ROWS ? KC : 1];
    const float* keep = BNB ? bnb.keep : nullptr;
    if (s < strips) {
        load_a<KC, R>(af, A, s * 16 * R, M, K, lr, lh);
        if constexpr (BNB) load_a<KC, R>(ay, bnb.y, s * 16 * R, M, K, lr, lh);
        if constexpr (ROWS) load_gate<KC, R>(gc, pro, s * 16 * R, M, K, lane, keep);
    }
    for (; s < strips; s += stride) {
        const int64_t m0 = s * 16 * R;
        if (s + stride < strips) {
            load_a<KC, R>(an, A, (s + stride) * 16 * R, M, K, lr, lh);
            if constexpr (BNB) load_a<KC, R>(ayn, bnb.y, (s + stride) * 16 * R, M, K, lr, lh);
            if constexpr (ROWS) load_gate<KC, R>(gn, pro, (s + stride) * 16 * R, M, K, lane, keep);
        }
        if constexpr (ROWS) {
#pragma unroll
            for (int j = 0; j < KC; ++j) gwl[lane + j * 64] = gc[j];
            wave_sync_lds();
        }
        const int64_t fb = ROWS ? (m0 / pro.hw + 1) * pro.hw : 0;    // first row of the strip's second frame
        f32x4 acc[R][NT];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[r][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            if constexpr (PRO) {
                // rebuild this k-chunk of the operand right before its MFMAs (keeps the live set to one chunk)
                const int col = kc * 32 + lh * 8;
                float sc[8], sh[8];
                load8f(psc + col, sc);
                load8f(psh + col, sh);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float x[8], gv[8];
                    unpack8(__builtin_bit_cast(uint4, af[r][kc]), x);
                    load8f(gwl + (m0 + r * 16 + lr >= fb ? KCP : 0) + col, gv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) x[j] = silu(fmaf(x[j], sc[j], sh[j])) * gv[j];
                    uint4 u;
                    u.x = pack2(x[0], x[1]); u.y = pack2(x[2], x[3]); u.z = pack2(x[4], x[5]); u.w = pack2(x[6], x[7]);
                    af[r][kc] = __builtin_bit_cast(bf16x8, u);
                    if (pro.aout) {
                        const int64_t row = m0 + r * 16 + lr;
                        if (row < M && col < K) *reinterpret_cast<uint4*>(pro.aout + row * K + col) = u;
                    }
                }
            }
            if constexpr (BNB) {
                // dy3 = k1 * (dout * rs[frame]) + k2 * y3 + k0 (bn_bwd_apply_flat_kernel, ACT_NONE), rounded to bf16
                const int col = kc * 32 + lh * 8;
                float k0[8], k1[8], k2[8];
                load8f(psc + col, k0);
                load8f(psh + col, k1);
                load8f(pk2 + col, k2);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float g[8], yv[8], q[8], o[8];
                    unpack8(__builtin_bit_cast(uint4, af[r][kc]), g);
                    unpack8(__builtin_bit_cast(uint4, ay[r][kc]), yv);
                    load8f(gwl + (m0 + r * 16 + lr >= fb ? KCP : 0) + col, q);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        g[j] *= q[j];
                        o[j] = fmaf(k1[j], g[j], fmaf(k2[j], yv[j], k0[j]));
                    }
                    uint4 u;
                    u.x = pack2(o[0], o[1]); u.y = pack2(o[2], o[3]); u.z = pack2(o[4], o[5]); u.w = pack2(o[6], o[7]);
                    af[r][kc] = __builtin_bit_cast(bf16x8, u);
                    const int64_t row = m0 + r * 16 + lr;
                    if (row < M && col < K) *reinterpret_cast<uint4*>(pro.aout + row * K + col) = u;
                }
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const bf16x8 bf = *reinterpret_cast<const bf16x8*>(bl + (nt * 16 + lr) * LDB + kc * 32 + lh * 8);
#pragma unroll
                for (int r = 0; r < R; ++r)
                    acc[r][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af[r][kc], acc[r][nt], 0, 0, 0);
            }
        }
        // accumulators -> bf16 strip image [16R][N] in this wave's LDS slice (8 B per lane: 4 channels of a pixel)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int n = nt * 16 + lh * 4;
                if (n < N) {
                    uint2 u;
                    u.x = pack2(acc[r][nt][0], acc[r][nt][1]);
                    u.y = pack2(acc[r][nt][2], acc[r][nt][3]);
                    *reinterpret_cast<uint2*>(cl + (r * 16 + lr) * LDC + n) = u;
                }
            }
        wave_sync_lds();
        // the strip is one contiguous [rows][N] block of C: store it with linear 16-B lanes
        const int64_t rem = (int64_t)M - m0;
        const int rows = rem < 16 * R ? (int)rem : 16 * R;
        bf16_t* cdst = C + m0 * N;
        for (int g = lane; g < rows * CPR; g += 64) {
            const int row = g / CPR, c = g - row * CPR;
            uint4 v = *reinterpret_cast<const uint4*>(cl + row * LDC + c * 8);
            *reinterpret_cast<uint4*>(cdst + (int64_t)g * 8) = v;
        }
        if constexpr (STATS) {
            if (srow0 < RG) {
                for (int row = srow0; row < rows; row += RG) {
                    float v[8];
                    load8(cl + row * LDC + sc8 * 8, v);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        sacc[j] += v[j];
                        qacc[j] = fmaf(v[j], v[j], qacc[j]);
                    }
                }
            }
        }
        wave_sync_lds();
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) af[r][kc] = an[r][kc];
        if constexpr (BNB) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int kc = 0; kc < KC; ++kc) ay[r][kc] = ayn[r][kc];
        }
        if constexpr (ROWS) {
#pragma unroll
            for (int j = 0; j < KC; ++j) gc[j] = gn[j];
        }
    }
    if constexpr (STATS) {
        float* red = reinterpret_cast<float*>(smem + S::b_bytes);     // [4 waves][64 lanes][s 8 | q 8]
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[(wave * 64 + lane) * 16 + j] = sacc[j];
            red[(wave * 64 + lane) * 16 + 8 + j] = qacc[j];
        }
        __syncthreads();
        for (int n = threadIdx.x; n < N; n += BLOCK) {
            const int c8 = n >> 3, j = n & 7;
            float a = 0.f, b = 0.f;
            for (int w = 0; w < 4; ++w)
                for (int g = 0; g < RG; ++g) {
                    const int l = g * CPR + c8;
                    a += red[(w * 64 + l) * 16 + j];
                    b += red[(w * 64 + l) * 16 + 8 + j];
                }
            ps[(int64_t)blockIdx.x * N + n] = a;
            pq[(int64_t)blockIdx.x * N + n] = b;
        }
    }
}


// (K, N) pairs of the B3 backbone's high-resolution 1x1 convs, forward and backward-data orientations
// (KC = ceil(K/32) specialises the k-loop; N is exact)
#define PW_SHAPES(X)                                                                                            \
    X(2, 24) X(1, 40) X(1, 24) X(1, 144) X(5, 24) X(5, 32) X(1, 192) X(6, 32) X(6, 48) X(2, 192)       \
    X(2, 288) X(9, 48)

template <int KC, int N, bool BNB = false>
int grid_for(int M, int max_blocks) {
    using S = PwShape<KC, N, BNB>;
    const int64_t strips = ((int64_t)M + 16 * S::R - 1) / (16 * S::R);
    int64_t g = (strips + 3) / 4;
    if (g > max_blocks) g = max_blocks;
    return (int)(g < 1 ? 1 : g);
}

template <int KC, int N>
int launch(const bf16_t* A, const bf16_t* B, int M, int K, bf16_t* C, float* ps, float* pq, int max_blocks,
           const PwPro& pro, hipStream_t st) {
    using S = PwShape<KC, N>;
    const int g = grid_for<KC, N>(M, max_blocks);
    if (pro.scale) {
        if (pro.hw < 16 * S::R || M % pro.hw) return (int)hipErrorInvalidValue;   // a strip spans <= 2 frames
        const size_t lds = S::lds + S::pro_bytes;
        if (ps)
            hipLaunchKernelGGL((pw_gemm_kernel<KC, N, true, true>), dim3(g), dim3(BLOCK), lds, st, A, B, M, K, C, ps,
                               pq, pro, PwBnb{});
        else
            hipLaunchKernelGGL((pw_gemm_kernel<KC, N, false, true>), dim3(g), dim3(BLOCK), lds, st, A, B, M, K, C, ps,
                               pq, pro, PwBnb{});
    } else if (ps) {
        hipLaunchKernelGGL((pw_gemm_kernel<KC, N, true, false>), dim3(g), dim3(BLOCK), S::lds, st, A, B, M, K, C, ps,
                           pq, pro, PwBnb{});
    } else {
        hipLaunchKernelGGL((pw_gemm_kernel<KC, N, false, false>), dim3(g), dim3(BLOCK), S::lds, st, A, B, M, K, C, ps,
                           pq, pro, PwBnb{});
    }
    return (int)hipGetLastError();
}

template <int KC, int N>
int launch_bnb(const bf16_t* A, const bf16_t* B, int M, int K, bf16_t* C, int max_blocks, const PwPro& pro,
               const PwBnb& bnb, hipStream_t st) {
    using S = PwShape<KC, N, true>;
    if (pro.hw < 16 * S::R || M % pro.hw || !pro.aout || !pro.gate || !bnb.y) return (int)hipErrorInvalidValue;
    const int g = grid_for<KC, N, true>(M, max_blocks);
    hipLaunchKernelGGL((pw_gemm_kernel<KC, N, false, false, true>), dim3(g), dim3(BLOCK), S::lds + S::pro_bytes, st, A,
                       B, M, K, C, nullptr, nullptr, pro, bnb);
    return (int)hipGetLastError();
}

// the project data-gradient shapes of blocks 0-7 (K = Cout, N = Ce)
#define PW_BNB_SHAPES(X) X(1, 40) X(1, 24) X(1, 144) X(1, 192) X(2, 192) X(2, 288)


// ------------------------------------------------------------------ wide-N variant
// Mid-resolution 1x1 convs (blocks 9-25, top): K <= 512 but N = 576..2304, M = 77K..277K.  The weight no
// longer fits in LDS, so a workgroup keeps its 4 x R x 16 rows of A in registers (read from HBM once) and
// walks N in 64-column chunks: each chunk of B (64 x K) is staged into LDS by the whole workgroup (an L2
// read shared by 4 waves), every wave runs its R x 4 x KC MFMAs, and the 64-column C chunk leaves through
// a per-wave LDS transpose as 128-B row segments.
template <int KC, int R>
struct WideShape {
    static constexpr int WNC = KC <= 5 ? 64 : 32;                  // output columns per chunk
    static constexpr int LDB = KC * 32 + 8;
    static constexpr int LDC = WNC + 8;
    static constexpr size_t b_bytes = (size_t)WNC * LDB * 2;       // one B chunk buffer (two are used)
    static constexpr size_t c_bytes = (size_t)R * 16 * LDC * 2;    // per wave
    static constexpr size_t lds = 2 * b_bytes + 4 * c_bytes;
    static constexpr int CH = KC * 4;                              // 16-B pieces per staged B row
    static constexpr int PER = (WNC * CH + BLOCK - 1) / BLOCK;     // pieces per thread per chunk
};

template <int KC, int R, int P>
__device__ __forceinline__ void wide_fetch(uint4 (&u)[P], const bf16_t* __restrict__ B, int n0, int K, int N) {
    using S = WideShape<KC, R>;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int i = threadIdx.x + k * BLOCK;
        const int n = i / S::CH, c = (i - n * S::CH) * 8;
        u[k] = make_uint4(0, 0, 0, 0);
        if (i < S::WNC * S::CH && n0 + n < N && c < K)
            u[k] = *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + n) * K + c);
    }
}

template <int KC, int R, int P>
__device__ __forceinline__ void wide_put(const uint4 (&u)[P], bf16_t* bl) {
    using S = WideShape<KC, R>;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int i = threadIdx.x + k * BLOCK;
        const int n = i / S::CH, c = (i - n * S::CH) * 8;
        if (i < S::WNC * S::CH) *reinterpret_cast<uint4*>(bl + n * S::LDB + c) = u[k];
    }
}

// LDS-only barrier: s_barrier after the LDS counter drains.  A __syncthreads would also fence global
// memory, i.e. wait for every C store of the chunk (vmcnt(0)) before the next chunk could start.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// B chunks are double-buffered in LDS: the next chunk's loads go out before this chunk's MFMAs and are
// written to the other buffer after them; one LDS-only barrier per chunk.
constexpr int WIDE_PF = 1;   // pw_wide (K <= 160): next strip's A rows prefetched during the current strip
template <int KC, int R>
__global__ __launch_bounds__(BLOCK) void pw_wide_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                        int M, int K, int N, bf16_t* __restrict__ C) {
    using S = WideShape<KC, R>;
    constexpr int LDB = S::LDB, LDC = S::LDC, WNC = S::WNC;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* buf0 = reinterpret_cast<bf16_t*>(smem);
    bf16_t* buf1 = reinterpret_cast<bf16_t*>(smem + S::b_bytes);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lh = lane >> 4;
    bf16_t* cl = reinterpret_cast<bf16_t*>(smem + 2 * S::b_bytes + wave * S::c_bytes);
    const int64_t rows_wg = 4 * R * 16;
    const int64_t strips = ((int64_t)M + rows_wg - 1) / rows_wg;
    const int nch = (N + WNC - 1) / WNC;
    // PF (narrow K): the next strip's A rows are loaded during this strip's first N chunk, after its B-chunk fetch,
    // so they stay in flight behind the MFMAs instead of being waited for at the top of the next strip
    constexpr bool PF = WIDE_PF && KC <= 5 && R <= 2;   // (the R = 4 form would drop to one wave per SIMD)
    bf16x8 af[R][KC], an[PF ? R : 1][PF ? KC : 1];
    if (PF && (int64_t)blockIdx.x < strips)
        load_a<KC, R>(af, A, (int64_t)blockIdx.x * rows_wg + (int64_t)wave * R * 16, M, K, lr, lh);
    for (int64_t s = blockIdx.x; s < strips; s += gridDim.x) {
        const int64_t m0 = s * rows_wg + (int64_t)wave * R * 16;
        if constexpr (!PF) load_a<KC, R>(af, A, m0, M, K, lr, lh);
        const int64_t rem = (int64_t)M - m0;
        const int rows = rem <= 0 ? 0 : (rem < 16 * R ? (int)rem : 16 * R);
        uint4 u[S::PER];
        // retire the A loads here, visibly to the compiler's wait-count pass: otherwise it re-waits
        // vmcnt(0) at their first use inside the chunk loop, draining the next chunk's loads every chunk
        __builtin_amdgcn_s_waitcnt(0x0F70);    // vmcnt(0) expcnt(7) lgkmcnt(15)
        lds_barrier();                         // the previous strip's readers of both buffers are done
        wide_fetch<KC, R, S::PER>(u, B, 0, K, N);
        wide_put<KC, R, S::PER>(u, buf0);
        lds_barrier();
        for (int j = 0; j < nch; ++j) {
            const int n0 = j * WNC;
            if (j + 1 < nch) wide_fetch<KC, R, S::PER>(u, B, n0 + WNC, K, N);
            if constexpr (PF) {
                if (j == 0 && s + gridDim.x < strips)
                    load_a<KC, R>(an, A, (s + gridDim.x) * rows_wg + (int64_t)wave * R * 16, M, K, lr, lh);
            }
            const bf16_t* bl = (j & 1) ? buf1 : buf0;
            f32x4 acc[R][WNC / 16];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int nt = 0; nt < WNC / 16; ++nt) acc[r][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
#pragma unroll
                for (int nt = 0; nt < WNC / 16; ++nt) {
                    const bf16x8 bf = *reinterpret_cast<const bf16x8*>(bl + (nt * 16 + lr) * LDB + kc * 32 + lh * 8);
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        acc[r][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af[r][kc], acc[r][nt], 0, 0, 0);
                }
            }
            if (j + 1 < nch) wide_put<KC, R, S::PER>(u, (j & 1) ? buf0 : buf1);
            if (rows > 0) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int nt = 0; nt < WNC / 16; ++nt) {
                        uint2 v;
                        v.x = pack2(acc[r][nt][0], acc[r][nt][1]);
                        v.y = pack2(acc[r][nt][2], acc[r][nt][3]);
                        *reinterpret_cast<uint2*>(cl + (r * 16 + lr) * LDC + nt * 16 + lh * 4) = v;
                    }
                wave_sync_lds();
                const int cols = N - n0 < WNC ? N - n0 : WNC;          // multiple of 8
                const int cpr = cols / 8;
                for (int g = lane; g < rows * cpr; g += 64) {
                    const int row = g / cpr, c = g - row * cpr;
                    *reinterpret_cast<uint4*>(C + (m0 + row) * N + n0 + c * 8) =
                        *reinterpret_cast<const uint4*>(cl + row * LDC + c * 8);
                }
                wave_sync_lds();
            }
            lds_barrier();                     // next buffer written; this buffer's readers are done
        }
        if constexpr (PF) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int kc = 0; kc < KC; ++kc) af[r][kc] = an[r][kc];
        }
    }
}

template <int KC, int R>
int launch_wide(const bf16_t* A, const bf16_t* B, int M, int K, int N, bf16_t* C, int max_blocks, hipStream_t st) {
    using S = WideShape<KC, R>;
    const int64_t strips = ((int64_t)M + 64 * R - 1) / (64 * R);
    int64_t g = strips < max_blocks ? strips : max_blocks;
    if (g < 1) g = 1;
    hipLaunchKernelGGL((pw_wide_kernel<KC, R>), dim3((unsigned)g), dim3(BLOCK), S::lds, st, A, B, M, K, N, C);
    return (int)hipGetLastError();
}

// KC -> rows per wave (R x 16) so the register-resident A fragments stay <= ~96 VGPRs
#define WIDE_KC_SHAPES(X) X(3, 4) X(5, 2) X(8, 2) X(12, 2)

}  // namespace

extern "C" {

// 1 if a specialisation exists for this (K, N)
int rt1_pw_gemm_supported(int K, int N) {
    if (K % 8 || N % 8 || K <= 0 || N <= 0) return 0;
    const int kc = (K + 31) / 32;
#define X(KC, NN) if (kc == KC && N == NN) return 1;
    PW_SHAPES(X)
#undef X
    return 0;
}

int rt1_pw_gemm_grid(int M, int K, int N, int max_blocks) {
    const int kc = (K + 31) / 32;
#define X(KC, NN) if (kc == KC && N == NN) return grid_for<KC, NN>(M, max_blocks);
    PW_SHAPES(X)
#undef X
    return 0;
}

// ps/pq: nullptr, or [rt1_pw_gemm_grid(...)][N] fp32 BN-stat partials of C.  scale != nullptr: A is the
// depthwise output y and the GEMM consumes silu(y*scale + shift) * gate[row / hw] (gate [M / hw, K] fp32);
// aout != nullptr also stores that operand ([M, K] bf16)
int rt1_pw_gemm(const bf16_t* A, const bf16_t* B, int M, int K, int N, bf16_t* C, float* ps, float* pq,
                int max_blocks, const float* scale, const float* shift, const float* gate, int hw, bf16_t* aout,
                hipStream_t st) {
    const int kc = (K + 31) / 32;
    const PwPro pro{scale, shift, gate, hw, aout};
#define X(KC, NN) if (kc == KC && N == NN) return launch<KC, NN>(A, B, M, K, C, ps, pq, max_blocks, pro, st);
    PW_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}


// dA = dy3 @ W^T with dy3 = BN3-backward(dout, y3) built in the operand prologue and stored to dy_out:
// rs = fmul [M / hw, K] (times keep [M / hw] when given), constants from gamma / mean / rstd / mdz / mdzx [K]
int rt1_pw_gemm_bnbwd_supported(int K, int N) {
    const int kc = (K + 31) / 32;
    if (K % 8 || N % 8) return 0;
#define X(KC, NN) if (kc == KC && N == NN) return 1;
    PW_BNB_SHAPES(X)
#undef X
    return 0;
}

int rt1_pw_gemm_bnbwd(const bf16_t* dout, const bf16_t* B, int M, int K, int N, bf16_t* C, int max_blocks,
                      const bf16_t* y, const float* fmul, const float* keep, int hw, const float* gamma,
                      const float* mean, const float* rstd, const float* mdz, const float* mdzx, bf16_t* dy_out,
                      hipStream_t st) {
    const int kc = (K + 31) / 32;
    const PwPro pro{nullptr, nullptr, fmul, hw, dy_out};
    const PwBnb bnb{y, gamma, mean, rstd, mdz, mdzx, keep};
#define X(KC, NN) if (kc == KC && N == NN) return launch_bnb<KC, NN>(dout, B, M, K, C, max_blocks, pro, bnb, st);
    PW_BNB_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

// wide-N GEMM: K <= 512 (K % 8 == 0), N % 16 == 0 and N >= 256
int rt1_pw_wide_supported(int K, int N) {
    if (K % 8 || K <= 0 || N % 16 || N < 256) return 0;
    const int kc = (K + 31) / 32;
#define X(KC, R) if (kc == KC) return 1;
    WIDE_KC_SHAPES(X)
#undef X
    return 0;
}

int rt1_pw_wide(const bf16_t* A, const bf16_t* B, int M, int K, int N, bf16_t* C, int max_blocks, hipStream_t st) {
    const int kc = (K + 31) / 32;
#define X(KC, R) if (kc == KC) return launch_wide<KC, R>(A, B, M, K, N, C, max_blocks, st);
    WIDE_KC_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

}  // extern "C"
