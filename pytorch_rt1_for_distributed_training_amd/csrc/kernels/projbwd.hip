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
// Kernel 1 (proj_bwd_frame_kernel): workgroup = (frame n, 64-channel tile, row split fs).  64-row chunks of dy3 and
// y2 are staged into LDS (the BN2/SiLU prologue builds X_0..X_2 once per element, S2/S4 accumulate in registers);
// the three products run on v_mfma_f32_16x16x32_bf16 with pixels as the reduction axis, operands read k-major with
// ds_read_b64_tr_b16 (the gfx950 LDS transpose).  Wave w owns the 16-channel slice w of the tile for all three
// products, so each B fragment is read once and feeds Cout/16 MFMAs.
// Kernels 2/3: fixed-order contractions (deterministic, bit-reproducible like the rest of the step).
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BLOCK = 256;
constexpr int ROWS = 64;                 // pixels per staged chunk (2 MFMA k-steps)
constexpr int TC = 64;                   // channels per workgroup tile (4 waves x 16)
constexpr int LDX = TC + 8;              // LDS row stride of an X image (bf16)

__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* base0, const bf16_t* base1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// KO: Cout padded to 16 * KO (Cout = 24 / 32 / 48 -> KO = 2 / 2 / 3)
template <int KO>
__global__ __launch_bounds__(BLOCK, 2) void proj_bwd_frame_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, int N, int HW, int Cout, int Ce, int tiles_c,
    int fsplit, int rows_per_split, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ G, float* __restrict__ S) {
    constexpr int CO = 16 * KO, LDD = CO + 8;
    constexpr int VD = CO / 8;                       // 16-B vectors of a staged dy3 row
    constexpr int DV = (ROWS * VD + BLOCK - 1) / BLOCK;
    constexpr size_t D_ELEMS = (size_t)ROWS * LDD, X_ELEMS = (size_t)ROWS * LDX;
    __shared__ __attribute__((aligned(16))) bf16_t sm[D_ELEMS + 3 * X_ELEMS];
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

    // y2 staging map: a fixed 8-channel column vector per thread, rows r0 and r0 + 32 of a chunk
    const int acol = (t & 7) * 8, r0 = t >> 3;
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
    f32x4 acc[3][KO];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int i = 0; i < KO; ++i) acc[q][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool mma = c0 + wave * 16 < Ce;            // this wave's 16-channel slice holds real channels

    uint4 ry[2], rd[DV];
    auto issue = [&](int64_t m0) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int64_t row = m0 + r0 + 32 * k;
            ry[k] = make_uint4(0, 0, 0, 0);
            if (cok && row < m_end) ry[k] = *reinterpret_cast<const uint4*>(y + row * Ce + c0 + acol);
        }
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            const int v = t + k * BLOCK;
            const int row = v / VD, col = (v - row * VD) * 8;
            rd[k] = make_uint4(0, 0, 0, 0);
            if (v < ROWS * VD && col < Cout && m0 + row < m_end)
                rd[k] = *reinterpret_cast<const uint4*>(dy + (m0 + row) * Cout + col);
        }
    };
    auto stage = [&](int64_t m0) {
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            const int v = t + k * BLOCK;
            if (v < ROWS * VD) {
                const int row = v / VD, col = (v - row * VD) * 8;
                *reinterpret_cast<uint4*>(Dl + row * LDD + col) = rd[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int row = r0 + 32 * k;
            uint4 o0 = make_uint4(0, 0, 0, 0), o1 = o0, o2 = o0;
            if (cok && m0 + row < m_end) {
                float f[8], a[8], g[8], gx[8];
                unpack8(ry[k], f);
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

    if (m_begin < m_end) issue(m_begin);
    for (int64_t m0 = m_begin; m0 < m_end; m0 += ROWS) {
        __syncthreads();                             // the previous chunk's MFMA reads are done
        stage(m0);
        __syncthreads();
        if (m0 + ROWS < m_end) issue(m0 + ROWS);      // next chunk in flight during the MFMAs
        if (mma) {
            const int q4 = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
            for (int ks = 0; ks < ROWS / 32; ++ks) {
                const int rk = ks * 32 + lh * 8 + q4;
                const int cb = wave * 16 + p * 4;
                bf16x8 fb[3];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    fb[q] = tr_read8(Xl + q * X_ELEMS + rk * LDX + cb, Xl + q * X_ELEMS + (rk + 4) * LDX + cb);
#pragma unroll
                for (int i = 0; i < KO; ++i) {
                    const int ob = i * 16 + p * 4;
                    const bf16x8 fa = tr_read8(Dl + rk * LDD + ob, Dl + (rk + 4) * LDD + ob);
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        acc[q][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[q], acc[q][i], 0, 0, 0);
                }
            }
        }
    }
    // G[fs][q][n][o][c]: D rows = o (lh*4 + e), cols = c (lr)
    if (mma) {
        const int c = c0 + wave * 16 + lr;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            float* g = G + (((int64_t)fs * 3 + q) * N + n) * (int64_t)Cout * Ce;
#pragma unroll
            for (int i = 0; i < KO; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int o = i * 16 + lh * 4 + e;
                    if (o < Cout && c < Ce) g[(int64_t)o * Ce + c] = acc[q][i][e];
                }
        }
    }
    // S2 / S4: the 32 row groups of each column vector, added in row-group order through LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);       // [2][32][64] floats = 16 KB (the staging images are done)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * TC + acol + j] = s2[j];
        red[32 * TC + r0 * TC + acol + j] = s4[j];
    }
    __syncthreads();
    if (t < 2 * TC) {
        const int which = t / TC, cc = t % TC;
        float a = 0.f;
        for (int r = 0; r < 32; ++r) a += red[which * 32 * TC + r * TC + cc];
        if (c0 + cc < Ce) S[(((int64_t)fs * 2 + which) * N + n) * Ce + c0 + cc] = a;
    }
}

// red[k][n][c] (k = 0..4, the se_bn_bwd_reduce layout) from G / S and the bf16 project weight Wp [Cout][Ce]
__global__ __launch_bounds__(BLOCK) void proj_bwd_red_kernel(const float* __restrict__ G, const float* __restrict__ S,
                                                             const bf16_t* __restrict__ Wp, int N, int Cout, int Ce,
                                                             int fsplit, float* __restrict__ red) {
    const int64_t NC = (int64_t)N * Ce;
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= NC) return;
    const int n = (int)(i / Ce), c = (int)(i - (int64_t)n * Ce);
    const int64_t OC = (int64_t)Cout * Ce;
    float r0 = 0.f, r1 = 0.f, r3 = 0.f;
    for (int o = 0; o < Cout; ++o) {
        const float w = bf2f(Wp[(int64_t)o * Ce + c]);
        float g0 = 0.f, g1 = 0.f, g2 = 0.f;
        for (int fs = 0; fs < fsplit; ++fs) {
            const int64_t base = ((int64_t)fs * 3 * N + n) * OC + (int64_t)o * Ce + c;
            g0 += G[base];
            g1 += G[base + (int64_t)N * OC];
            g2 += G[base + 2 * (int64_t)N * OC];
        }
        r0 = fmaf(w, g0, r0);
        r1 = fmaf(w, g1, r1);
        r3 = fmaf(w, g2, r3);
    }
    float r2 = 0.f, r4 = 0.f;
    for (int fs = 0; fs < fsplit; ++fs) {
        r2 += S[((int64_t)fs * 2 * N + n) * Ce + c];
        r4 += S[((int64_t)fs * 2 * N + N + n) * Ce + c];
    }
    red[i] = r0;
    red[NC + i] = r1;
    red[2 * NC + i] = r2;
    red[3 * NC + i] = r3;
    red[4 * NC + i] = r4;
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
            for (int fs = 0; fs < fsplit; ++fs) g += G[((int64_t)fs * 3 * N + n) * OC + col];
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
int rt1_proj_bwd_fsplit(int N, int HW, int Ce) {
    const int tiles = (Ce + TC - 1) / TC;
    const int64_t wgs = (int64_t)N * tiles;
    int fs = (int)((1536 + wgs - 1) / wgs);
    const int max_fs = HW / (8 * ROWS);
    if (fs > max_fs) fs = max_fs;
    return fs < 1 ? 1 : fs;
}

// G: [fsplit, 3, N, Cout, Ce] fp32, S: [fsplit, 2, N, Ce] fp32 (every entry written)
int rt1_proj_bwd_frame(const bf16_t* dy, const bf16_t* y, int N, int HW, int Cout, int Ce, const float* scale,
                       const float* shift, const float* mean, const float* rstd, int fsplit, float* G, float* S,
                       hipStream_t st) {
    if (!rt1_proj_bwd_supported(Cout, Ce) || N <= 0 || HW <= 0 || fsplit < 1) return (int)hipErrorInvalidValue;
    const int tiles = (Ce + TC - 1) / TC;
    const int rows = ((HW + fsplit - 1) / fsplit + ROWS - 1) / ROWS * ROWS;
    const dim3 grid((unsigned)((int64_t)N * fsplit * tiles));
    if (Cout <= 32)
        hipLaunchKernelGGL(proj_bwd_frame_kernel<2>, grid, dim3(BLOCK), 0, st, dy, y, N, HW, Cout, Ce, tiles, fsplit,
                           rows, scale, shift, mean, rstd, G, S);
    else
        hipLaunchKernelGGL(proj_bwd_frame_kernel<3>, grid, dim3(BLOCK), 0, st, dy, y, N, HW, Cout, Ce, tiles, fsplit,
                           rows, scale, shift, mean, rstd, G, S);
    return (int)hipGetLastError();
}

// red: [5, N, Ce] fp32; dW: [Cout, Ce] fp32
int rt1_proj_bwd_finalize(const float* G, const float* S, const bf16_t* Wp, const float* gate, int N, int Cout,
                          int Ce, int fsplit, float* red, float* dW, hipStream_t st) {
    const int64_t NC = (int64_t)N * Ce, OC = (int64_t)Cout * Ce;
    hipLaunchKernelGGL(proj_bwd_red_kernel, dim3((unsigned)((NC + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, G, S, Wp,
                       N, Cout, Ce, fsplit, red);
    hipLaunchKernelGGL(proj_bwd_dw_kernel, dim3((unsigned)((OC + DW_COLS - 1) / DW_COLS)), dim3(DW_COLS * DW_RG), 0, st,
                       G, gate, N, Cout, Ce, fsplit, dW);
    return (int)hipGetLastError();
}

}  // extern "C"
