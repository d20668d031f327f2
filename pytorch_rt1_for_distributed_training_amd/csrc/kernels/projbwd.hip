// Project-conv backward statistics of the skinny MBConv blocks (0-7), per frame, from (dy3, y2) in ONE pass.
//
// The block's backward needs, per frame n and expanded channel c (SURVEY K5/K6/K10 backward,
// film_efficientnet_encoder.py:185-244):
//   S0 = sum_hw dA * act      (SE gate gradient)          act = silu(z), z = y2*scale + shift (BN2)
//   S1 = sum_hw dA * sg       S2 = sum_hw sg               sg  = silu'(z)
//   S3 = sum_hw dA * sg * xh  S4 = sum_hw sg * xh          xh  = (y2 - mean) * rstd
// and the project weight gradient dWp = sum_p dy3[p]^T (act[p] * gate[n(p)]).  dA = dy3 @ Wp is linear in dy3, so
// with the per-frame products
//   G_q[n] = dy3[n]^T X_q[n]   (Cout x Ce),   X_0 = act, X_1 = sg, X_2 = sg * xh
// every dA-weighted sum is a contraction with Wp:  S0[n,c] = sum_o Wp[o,c] G_0[n][o,c]  (S1, S3 likewise), and
// dWp[o,c] = sum_n gate[n,c] G_0[n][o,c].
//
// The previous dataflow materialised A = act*gate in the forward (one Ce-wide write), re-read it for dWp (one read)
// and re-read dA next to y2 in se_bn_bwd_reduce (two reads); here one kernel reads y2 and the narrow dy3 once, so
// three Ce-wide activation passes per block disappear (blocks 0-7 carry ~8.5 GB of Ce-wide tensors per pass).
//
// Kernel 1 (proj_bwd_frame_kernel): workgroup = (frame n, 32/64-channel tile, row split fs).  64-row chunks of dy3 and
// y2 are staged into LDS (the BN2/SiLU prologue builds X_0..X_2 once per element, S2/S4 accumulate in registers);
// the three products run on v_mfma_f32_16x16x32_bf16 with pixels as the reduction axis, operands read k-major with
// ds_read_b64_tr_b16 (the gfx950 LDS transpose).  Wave w owns the 16-channel slice w of the tile for all three
// products, so each B fragment is read once and feeds Cout/16 MFMAs.
// The contractions with Wp run in the epilogue (lane sums + two xor shuffles); only G_0 leaves the kernel, for
// dWp.  Kernels 2/3: the row-split sum and dWp, fixed-order (deterministic, bit-reproducible like the rest of the
// step).
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BLOCK = 256;
constexpr int ROWS = 64;                 // pixels per staged chunk (2 MFMA k-steps)
constexpr int PB_DEPTH = 1;             // chunks in flight ahead of the one being staged (2: no gain, removed)
constexpr int PB_OCC = 3;               // __launch_bounds__ workgroups per CU
// (a hi + lo bf16 pair for act, one extra MFMA per k-step, did not move the SE fc1 gradient's parity:
// profiles/r3_parity_pb_hilo.log)
constexpr int NQ = 3;                   // MFMA operand images: act, sg, sg*xh

__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* base0, const bf16_t* base1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// KO: Cout padded to 16 * KO (Cout = 24 / 32 / 48 -> KO = 2 / 2 / 3); TC: channels per workgroup tile (32 for the
// 24-channel block, else 64), one 16-channel slice per wave
template <int KO, int TC>
__global__ __launch_bounds__(BLOCK, PB_OCC) void proj_bwd_frame_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, int N, int HW, int Cout, int Ce, int tiles_c,
    int fsplit, int rows_per_split, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ rstd, const bf16_t* __restrict__ Wp,
    float* __restrict__ G, float* __restrict__ R) {
    constexpr int CO = 16 * KO, LDD = CO + 8, LDX = TC + 8;
    constexpr int VD = CO / 8;                       // 16-B vectors of a staged dy3 row
    constexpr int DV = (ROWS * VD + BLOCK - 1) / BLOCK;
    constexpr int VX = TC / 8;                       // 16-B vectors of a staged y2 row
    constexpr int RG = BLOCK / VX;                   // rows per staging pass (row groups of a column vector)
    constexpr int YP = ROWS / RG;                    // staging passes per chunk
    constexpr size_t D_ELEMS = (size_t)ROWS * LDD, X_ELEMS = (size_t)ROWS * LDX;
    static_assert(2 * RG * TC * 4 <= (D_ELEMS + NQ * X_ELEMS) * 2, "S2/S4 reduction must fit the staging images");
    __shared__ __attribute__((aligned(16))) bf16_t sm[D_ELEMS + NQ * X_ELEMS];
    bf16_t* Dl = sm;
    bf16_t* Xl = sm + D_ELEMS;

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int lr = lane & 15, lh = lane >> 4;
    const int ct = blockIdx.x % tiles_c;
    const int rest = blockIdx.x / tiles_c;
    const int fs = rest % fsplit, n = rest / fsplit;
    const int c0 = ct * TC;
    const int64_t frame0 = (int64_t)n * HW;
    const int64_t m_begin = frame0 + (int64_t)fs * rows_per_split;
    const int64_t m_end = min(m_begin + rows_per_split, frame0 + HW);

    // y2 staging map: a fixed 8-channel column vector per thread, rows r0 + RG * k of a chunk
    const int acol = (t % VX) * 8, r0 = t / VX;
    const bool cok = c0 + acol < Ce;
    float sc[8], sh[8], mu[8], rr[8], s2[8], s4[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        sc[j] = cok ? scale[c0 + acol + j] : 0.f;
        sh[j] = cok ? shift[c0 + acol + j] : 0.f;
        mu[j] = cok ? mean[c0 + acol + j] : 0.f;
        rr[j] = cok ? rstd[c0 + acol + j] : 0.f;
        s2[j] = s4[j] = 0.f;
    }
    f32x4 acc[NQ][KO];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int i = 0; i < KO; ++i) acc[q][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool mma = wave * 16 < TC && c0 + wave * 16 < Ce;   // this wave's 16-channel slice holds real channels

    // PB_DEPTH register sets: the next chunk(s) are in flight while chunk i is staged and multiplied
    uint4 ry[PB_DEPTH][YP], rd[PB_DEPTH][DV];
    auto issue = [&](int set, int64_t m0) {
#pragma unroll
        for (int k = 0; k < YP; ++k) {
            const int64_t row = m0 + r0 + RG * k;
            ry[set][k] = make_uint4(0, 0, 0, 0);
            if (cok && row < m_end) ry[set][k] = *reinterpret_cast<const uint4*>(y + row * Ce + c0 + acol);
        }
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            const int v = t + k * BLOCK;
            const int row = v / VD, col = (v - row * VD) * 8;
            rd[set][k] = make_uint4(0, 0, 0, 0);
            if (v < ROWS * VD && col < Cout && m0 + row < m_end)
                rd[set][k] = *reinterpret_cast<const uint4*>(dy + (m0 + row) * Cout + col);
        }
    };
    auto stage = [&](int set, int64_t m0) {
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            const int v = t + k * BLOCK;
            if (v < ROWS * VD) {
                const int row = v / VD, col = (v - row * VD) * 8;
                *reinterpret_cast<uint4*>(Dl + row * LDD + col) = rd[set][k];
            }
        }
#pragma unroll
        for (int k = 0; k < YP; ++k) {
            const int row = r0 + RG * k;
            uint4 o0 = make_uint4(0, 0, 0, 0), o1 = o0, o2 = o0;
            if (cok && m0 + row < m_end) {
                float f[8], a[8], g[8], gx[8];
                unpack8(ry[set][k], f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float z = fmaf(f[j], sc[j], sh[j]);
                    const float sgm = sigmoidf_(z);
                    a[j] = z * sgm;
                    g[j] = sgm * (1.f + z * (1.f - sgm));
                    gx[j] = g[j] * ((f[j] - mu[j]) * rr[j]);
                    s2[j] += g[j];
                    s4[j] += gx[j];
                }
                o0 = make_uint4(pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(a[4], a[5]), pack2(a[6], a[7]));
                o1 = make_uint4(pack2(g[0], g[1]), pack2(g[2], g[3]), pack2(g[4], g[5]), pack2(g[6], g[7]));
                o2 = make_uint4(pack2(gx[0], gx[1]), pack2(gx[2], gx[3]), pack2(gx[4], gx[5]), pack2(gx[6], gx[7]));
            }
            *reinterpret_cast<uint4*>(Xl + row * LDX + acol) = o0;
            *reinterpret_cast<uint4*>(Xl + X_ELEMS + row * LDX + acol) = o1;
            *reinterpret_cast<uint4*>(Xl + 2 * X_ELEMS + row * LDX + acol) = o2;
        }
    };
    auto mfma_chunk = [&]() {
        if (!mma) return;
        const int q4 = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
        for (int ks = 0; ks < ROWS / 32; ++ks) {
            const int rk = ks * 32 + lh * 8 + q4;
            const int cb = wave * 16 + p * 4;
            bf16x8 fb[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                fb[q] = tr_read8(Xl + q * X_ELEMS + rk * LDX + cb, Xl + q * X_ELEMS + (rk + 4) * LDX + cb);
#pragma unroll
            for (int i = 0; i < KO; ++i) {
                const int ob = i * 16 + p * 4;
                const bf16x8 fa = tr_read8(Dl + rk * LDD + ob, Dl + (rk + 4) * LDD + ob);
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    acc[q][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[q], acc[q][i], 0, 0, 0);
            }
        }
    };

    if (m_begin < m_end) issue(0, m_begin);
    for (int64_t m0 = m_begin; m0 < m_end; m0 += ROWS) {
        __syncthreads();                             // the previous chunk's MFMA reads are done
        stage(0, m0);
        __syncthreads();
        if (m0 + ROWS < m_end) issue(0, m0 + ROWS);   // next chunk in flight during the MFMAs
        mfma_chunk();
    }
    // accumulator D rows = o (i*16 + lh*4 + e), cols = c (lr).  G_0 -> G[fs][n][o][c] (for dWp); the three
    // dA-weighted sums are contracted with Wp right here: sum over the lane's (i, e), then over the 4 lane groups
    // (lanes lr, lr+16, lr+32, lr+48) with two xor shuffles in a fixed order
    const int64_t NC = (int64_t)N * Ce;
    float* Rf = R + (int64_t)fs * 5 * NC;
    if (mma) {
        const int c = c0 + wave * 16 + lr;
        const bool cin = c < Ce;
        float* g = G + ((int64_t)fs * N + n) * (int64_t)Cout * Ce;
        float v[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < KO; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = i * 16 + lh * 4 + e;
                if (o < Cout && cin) {
                    const float w = bf2f(Wp[(int64_t)o * Ce + c]);
                    const float g0 = acc[0][i][e];
                    g[(int64_t)o * Ce + c] = g0;
                    v[0] = fmaf(w, g0, v[0]);
#pragma unroll
                    for (int q = 1; q < 3; ++q) v[q] = fmaf(w, acc[q][i][e], v[q]);
                }
            }
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            v[q] += __shfl_xor(v[q], 16);
            v[q] += __shfl_xor(v[q], 32);
        }
        if (lh == 0 && cin) {
            Rf[(int64_t)n * Ce + c] = v[0];              // S0
            Rf[NC + (int64_t)n * Ce + c] = v[1];         // S1
            Rf[3 * NC + (int64_t)n * Ce + c] = v[2];     // S3
        }
    }
    // S2 / S4: the RG row groups of each column vector, added in row-group order through LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);       // [2][RG][TC] floats (the staging images are done)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * TC + acol + j] = s2[j];
        red[RG * TC + r0 * TC + acol + j] = s4[j];
    }
    __syncthreads();
    if (t < 2 * TC) {
        const int which = t / TC, cc = t % TC;
        float a = 0.f;
        for (int r = 0; r < RG; ++r) a += red[which * RG * TC + r * TC + cc];
        if (c0 + cc < Ce) Rf[(2 + 2 * which) * NC + (int64_t)n * Ce + c0 + cc] = a;   // S2, S4
    }
}

// red = sum over the row splits of R [fs][5][N][Ce] (fixed order); only launched when fsplit > 1
__global__ __launch_bounds__(BLOCK) void proj_bwd_red_kernel(const float* __restrict__ R, int64_t n5, int fsplit,
                                                             float* __restrict__ red) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n5) return;
    float a = 0.f;
    for (int f = 0; f < fsplit; ++f) a += R[(int64_t)f * n5 + i];
    red[i] = a;
}

// dWp[o][c] = sum_n gate[n][c] * sum_fs G_0[fs][n][o][c]: a workgroup = 64 (o, c) columns x 16 frame groups, every
// thread walks every 16th frame, the 16 partials of a column are added in group order (fixed order, fp64)
constexpr int DW_COLS = 64, DW_RG = 16;
__global__ __launch_bounds__(DW_COLS * DW_RG) void proj_bwd_dw_kernel(const float* __restrict__ G,
                                                                      const float* __restrict__ gate, int N, int Cout,
                                                                      int Ce, int fsplit, float* __restrict__ dW) {
    __shared__ double sh[DW_RG][DW_COLS];
    const int64_t OC = (int64_t)Cout * Ce;
    const int64_t col = (int64_t)blockIdx.x * DW_COLS + threadIdx.x % DW_COLS;
    const int rg = threadIdx.x / DW_COLS;
    double a = 0.0;
    if (col < OC) {
        const int c = (int)(col % Ce);
#pragma unroll 4
        for (int n = rg; n < N; n += DW_RG) {
            float g = 0.f;
            for (int fs = 0; fs < fsplit; ++fs) g += G[((int64_t)fs * N + n) * OC + col];
            a += (double)(g * gate[(int64_t)n * Ce + c]);
        }
    }
    sh[rg][threadIdx.x % DW_COLS] = a;
    __syncthreads();
    if (rg == 0 && col < OC) {
        double s = 0.0;
        for (int r = 0; r < DW_RG; ++r) s += sh[r][threadIdx.x];
        dW[col] = (float)s;
    }
}

}  // namespace

extern "C" {

int rt1_proj_bwd_supported(int Cout, int Ce) { return (Cout % 8 == 0 && Cout <= 48 && Ce % 8 == 0) ? 1 : 0; }

// row splits per frame: enough workgroups to cover the chip ~3 times, >= 8 chunks per split
inline int proj_tc(int Ce) { return Ce <= 32 ? 32 : 64; }

int rt1_proj_bwd_fsplit(int N, int HW, int Ce) {
    const int tiles = (Ce + proj_tc(Ce) - 1) / proj_tc(Ce);
    const int64_t wgs = (int64_t)N * tiles;
    int fs = (int)((1536 + wgs - 1) / wgs);
    const int max_fs = HW / (8 * ROWS);
    if (fs > max_fs) fs = max_fs;
    return fs < 1 ? 1 : fs;
}

// G: [fsplit, N, Cout, Ce] fp32 (the per-frame dy3^T act products), R: [fsplit, 5, N, Ce] fp32 (the five sums per
// row split); every entry written
int rt1_proj_bwd_frame(const bf16_t* dy, const bf16_t* y, int N, int HW, int Cout, int Ce, const float* scale,
                       const float* shift, const float* mean, const float* rstd, const bf16_t* Wp, int fsplit,
                       float* G, float* R, hipStream_t st) {
    if (!rt1_proj_bwd_supported(Cout, Ce) || N <= 0 || HW <= 0 || fsplit < 1) return (int)hipErrorInvalidValue;
    const int tc = proj_tc(Ce), tiles = (Ce + tc - 1) / tc;
    const int rows = ((HW + fsplit - 1) / fsplit + ROWS - 1) / ROWS * ROWS;
    const dim3 grid((unsigned)((int64_t)N * fsplit * tiles));
#define L(KO, TCC) hipLaunchKernelGGL((proj_bwd_frame_kernel<KO, TCC>), grid, dim3(BLOCK), 0, st, dy, y, N, HW, Cout, \
                                      Ce, tiles, fsplit, rows, scale, shift, mean, rstd, Wp, G, R)
    if (Cout <= 32 && tc == 32) L(2, 32);
    else if (Cout <= 32) L(2, 64);
    else if (tc == 32) L(3, 32);
    else L(3, 64);
#undef L
    return (int)hipGetLastError();
}

// red: [5, N, Ce] fp32 (fsplit > 1: the sum of R over the splits; fsplit == 1: R itself, nothing launched);
// dW: [Cout, Ce] fp32
int rt1_proj_bwd_finalize(const float* G, const float* R, const float* gate, int N, int Cout, int Ce, int fsplit,
                          float* red, float* dW, hipStream_t st) {
    const int64_t n5 = (int64_t)5 * N * Ce, OC = (int64_t)Cout * Ce;
    if (fsplit > 1)
        hipLaunchKernelGGL(proj_bwd_red_kernel, dim3((unsigned)((n5 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, R, n5,
                           fsplit, red);
    hipLaunchKernelGGL(proj_bwd_dw_kernel, dim3((unsigned)((OC + DW_COLS - 1) / DW_COLS)), dim3(DW_COLS * DW_RG), 0, st,
                       G, gate, N, Cout, Ce, fsplit, dW);
    return (int)hipGetLastError();
}

}  // extern "C"
