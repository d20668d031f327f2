// Fused backward of an MBConv expand stage (1x1 conv Cin->Ce, BatchNorm, SiLU) for the high-resolution
// blocks (SURVEY K3 backward + K10 backward), ONE pass over the Ce-wide tensors:
//
//   dz  = dA1 * silu'(y1*sc + sh)                       (SiLU backward)
//   dy1 = k1*dz + k2*y1 + k0                            (BatchNorm backward apply, per-channel k*)
//   dx  = dy1 @ We            [M, Cin]                  (data gradient, MFMA)        (+ dout*fmul: residual)
//   dWe = dy1^T @ x           [Ce, Cin]                 (weight gradient, MFMA, per-workgroup partials)
//
// The unfused chain (bn_bwd_apply -> dgrad GEMM -> split-K wgrad GEMM) reads or writes the Ce-wide dy1
// three more times; at block 2 (M = 17.3 M pixels, Ce = 144) each pass is ~5 GB of HBM traffic.
//
// Per workgroup iteration = 64 rows (4 waves x 16):
//   * each wave loads its dA1 / y1 rows in MFMA-B layout (16 B per lane), forms dy1 in registers,
//     runs the dgrad MFMAs against the We^T image in LDS (C^T = We^T . dy1^T: the 4 accumulator registers
//     are 4 consecutive input channels of one pixel -> 8-byte stores of dx), and writes its dy1 rows to LDS;
//   * the x rows of the strip are staged into LDS;
//   * after a barrier the wgrad MFMAs read BOTH operands m-major with ds_read_b64_tr_b16 (gfx950 hardware
//     transpose: 4 rows x 16 columns per 16-lane group, delivered column-major), so the sum over pixels
//     is the MFMA k dimension; each wave owns every 4th 16-channel Ce tile x all Cin tiles.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int BLOCK = 256;
constexpr int ROWS = 64;   // rows per workgroup iteration

template <int CE, int CIN>
struct BwdShape {
    static constexpr int KC = (CE + 31) / 32;          // 32-channel k-chunks of the dgrad
    static constexpr int CEP = KC * 32;
    static constexpr int NTI = (CIN + 15) / 16;        // 16-channel tiles of Cin
    static constexpr int CINP = NTI * 16;
    static constexpr int NTE = (CE + 15) / 16;         // 16-channel tiles of Ce (real ones)
    static constexpr int TPW = (NTE + 3) / 4;          // Ce tiles per wave in the wgrad
    static constexpr int LDW = CEP + 8;                // We^T image row stride (bf16)
    static constexpr int LDY = CEP + 8;                // dy1 tile row stride (bf16), multiple of 8
    static constexpr int LDX = CINP + 8;               // x tile row stride (bf16)
    static constexpr size_t w_off = 0;
    static constexpr size_t c_off = w_off + (size_t)CINP * LDW * 2;
    static constexpr size_t y_off = c_off + (size_t)5 * CEP * 4;
    static constexpr size_t x_off = y_off + (size_t)ROWS * LDY * 2;
    static constexpr size_t lds = x_off + (size_t)ROWS * LDX * 2;
};

__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* base0, const bf16_t* base1) {
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base0);
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)base1);
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int CE, int CIN, bool SKIP>
__global__ __launch_bounds__(BLOCK) void pw_bwd_kernel(const bf16_t* __restrict__ dA, const bf16_t* __restrict__ y,
                                                       const bf16_t* __restrict__ x, const bf16_t* __restrict__ We,
                                                       const float* __restrict__ consts, int M,
                                                       bf16_t* __restrict__ dx, const bf16_t* __restrict__ dout,
                                                       const float* __restrict__ fmul, int HW,
                                                       float* __restrict__ dwp) {
    using S = BwdShape<CE, CIN>;
    constexpr int KC = S::KC, CEP = S::CEP, NTI = S::NTI, CINP = S::CINP, NTE = S::NTE, TPW = S::TPW;
    constexpr int LDW = S::LDW, LDY = S::LDY, LDX = S::LDX;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* wl = reinterpret_cast<bf16_t*>(smem + S::w_off);
    float* cl = reinterpret_cast<float*>(smem + S::c_off);
    bf16_t* yl = reinterpret_cast<bf16_t*>(smem + S::y_off);
    bf16_t* xl = reinterpret_cast<bf16_t*>(smem + S::x_off);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int lr = lane & 15, lh = lane >> 4;

    // We^T image [CINP][CEP] (zero padded) and the per-channel constants [5][CEP]
    for (int i = t; i < CINP * CEP; i += BLOCK) {
        const int ci = i / CEP, ce = i - ci * CEP;
        wl[ci * LDW + ce] = (ci < CIN && ce < CE) ? We[ce * CIN + ci] : (bf16_t)0;
    }
    for (int i = t; i < 5 * CEP; i += BLOCK) {
        const int k = i / CEP, ce = i - k * CEP;
        cl[i] = ce < CE ? consts[k * CE + ce] : 0.f;
    }
    // zero the x tile's pad columns once (the strips only write [0, CIN))
    if constexpr (CINP > CIN) {
        for (int i = t; i < ROWS * (CINP - CIN); i += BLOCK) {
            const int r = i / (CINP - CIN), c = CIN + (i - r * (CINP - CIN));
            xl[r * LDX + c] = 0;
        }
    }

    f32x4 accw[TPW][NTI];
#pragma unroll
    for (int a = 0; a < TPW; ++a)
#pragma unroll
        for (int b = 0; b < NTI; ++b) accw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int strips = (M + ROWS - 1) / ROWS;
    for (int s = blockIdx.x; s < strips; s += gridDim.x) {
        const int m0 = s * ROWS;
        __syncthreads();   // previous iteration's wgrad reads of yl / xl are done (and the images above written)
        // ---- x rows of the strip -> LDS (16-B chunks, zero beyond M)
        constexpr int XCH = CIN / 8;
        for (int i = t; i < ROWS * XCH; i += BLOCK) {
            const int r = i / XCH, c = (i - r * XCH) * 8;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (m0 + r < M) u = *reinterpret_cast<const uint4*>(x + (int64_t)(m0 + r) * CIN + c);
            *reinterpret_cast<uint4*>(xl + r * LDX + c) = u;
        }
        // ---- this wave's 16 rows: dy1 in registers -> dgrad MFMAs, dy1 -> LDS
        const int row = m0 + wave * 16 + lr;
        const bool rok = row < M;
        f32x4 accd[NTI];
#pragma unroll
        for (int b = 0; b < NTI; ++b) accd[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            const int c0 = kc * 32 + lh * 8;
            float dv[8];
            if (rok && c0 < CE) {
                float av[8], yv[8], sc[8], sh[8], k1[8], k2[8], k0[8];
                load8(dA + (int64_t)row * CE + c0, av);
                load8(y + (int64_t)row * CE + c0, yv);
                load8f(cl + c0, sc);
                load8f(cl + CEP + c0, sh);
                load8f(cl + 2 * CEP + c0, k1);
                load8f(cl + 3 * CEP + c0, k2);
                load8f(cl + 4 * CEP + c0, k0);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float dz = av[j] * silu_grad(fmaf(yv[j], sc[j], sh[j]));
                    dv[j] = fmaf(k1[j], dz, fmaf(k2[j], yv[j], k0[j]));
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) dv[j] = 0.f;
            }
            uint4 u;
            u.x = pack2(dv[0], dv[1]); u.y = pack2(dv[2], dv[3]); u.z = pack2(dv[4], dv[5]); u.w = pack2(dv[6], dv[7]);
            *reinterpret_cast<uint4*>(yl + (wave * 16 + lr) * LDY + c0) = u;
            bf16x8 df;
            __builtin_memcpy(&df, &u, 16);
#pragma unroll
            for (int b = 0; b < NTI; ++b) {
                const bf16x8 wf = *reinterpret_cast<const bf16x8*>(wl + (b * 16 + lr) * LDW + kc * 32 + lh * 8);
                accd[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, df, accd[b], 0, 0, 0);
            }
        }
        // ---- dx epilogue: lane holds dx[row][b*16 + lh*4 + 0..3]
        if (rok) {
            const int64_t n = SKIP ? (int64_t)((uint32_t)row / (uint32_t)HW) : 0;
#pragma unroll
            for (int b = 0; b < NTI; ++b) {
                const int ci = b * 16 + lh * 4;
                if (ci < CIN) {
                    float o[4] = {accd[b][0], accd[b][1], accd[b][2], accd[b][3]};
                    if constexpr (SKIP) {
                        const uint2 d = *reinterpret_cast<const uint2*>(dout + (int64_t)row * CIN + ci);
                        const float4 f = *reinterpret_cast<const float4*>(fmul + n * CIN + ci);
                        o[0] = fmaf(__uint_as_float(d.x << 16), f.x, o[0]);
                        o[1] = fmaf(__uint_as_float(d.x & 0xffff0000u), f.y, o[1]);
                        o[2] = fmaf(__uint_as_float(d.y << 16), f.z, o[2]);
                        o[3] = fmaf(__uint_as_float(d.y & 0xffff0000u), f.w, o[3]);
                    }
                    uint2 u;
                    u.x = pack2(o[0], o[1]);
                    u.y = pack2(o[2], o[3]);
                    *reinterpret_cast<uint2*>(dx + (int64_t)row * CIN + ci) = u;
                }
            }
        }
        __syncthreads();
        // ---- wgrad: dWe[ce][ci] += sum_m dy1[m][ce] * x[m][ci]   (k = m, 2 steps of 32 rows)
#pragma unroll
        for (int ks = 0; ks < ROWS / 32; ++ks) {
            // tr-read addressing: lane 4q+p of a 16-lane group -> row q (of 4), columns 4p..4p+3
            const int q = (lane & 15) >> 2, p = lane & 3;
            const int r0 = ks * 32 + lh * 8 + q;          // rows r0 and r0+4 feed elements 0..3 / 4..7
            bf16x8 xb[NTI];
#pragma unroll
            for (int b = 0; b < NTI; ++b)
                xb[b] = tr_read8(xl + r0 * LDX + b * 16 + p * 4, xl + (r0 + 4) * LDX + b * 16 + p * 4);
#pragma unroll
            for (int a = 0; a < TPW; ++a) {
                const int et = wave + 4 * a;
                if (et < NTE) {
                    const bf16x8 ya = tr_read8(yl + r0 * LDY + et * 16 + p * 4, yl + (r0 + 4) * LDY + et * 16 + p * 4);
#pragma unroll
                    for (int b = 0; b < NTI; ++b)
                        accw[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ya, xb[b], accw[a][b], 0, 0, 0);
                }
            }
        }
    }
    // ---- per-workgroup weight-gradient partials: dwp[blockIdx.x][ce][ci]   (D: col = ci, rows = ce)
#pragma unroll
    for (int a = 0; a < TPW; ++a) {
        const int et = wave + 4 * a;
        if (et >= NTE) continue;
#pragma unroll
        for (int b = 0; b < NTI; ++b) {
            const int ci = b * 16 + lr;
            if (ci >= CIN) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ce = et * 16 + lh * 4 + i;
                if (ce < CE) dwp[((int64_t)blockIdx.x * CE + ce) * CIN + ci] = accw[a][b][i];
            }
        }
    }
}

#define RT1_PWBWD_SHAPES(X) X(144, 24) X(192, 32) X(288, 48)

template <int CE, int CIN>
int launch(const bf16_t* dA, const bf16_t* y, const bf16_t* x, const bf16_t* We, const float* consts, int M,
           bf16_t* dx, const bf16_t* dout, const float* fmul, int HW, float* dwp, int grid, hipStream_t st) {
    using S = BwdShape<CE, CIN>;
    if (dout)
        hipLaunchKernelGGL((pw_bwd_kernel<CE, CIN, true>), dim3(grid), dim3(BLOCK), S::lds, st, dA, y, x, We, consts,
                           M, dx, dout, fmul, HW, dwp);
    else
        hipLaunchKernelGGL((pw_bwd_kernel<CE, CIN, false>), dim3(grid), dim3(BLOCK), S::lds, st, dA, y, x, We, consts,
                           M, dx, dout, fmul, HW, dwp);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int rt1_pw_bwd_supported(int CE, int CIN) {
#define X(A, B) if (CE == A && CIN == B) return 1;
    RT1_PWBWD_SHAPES(X)
#undef X
    return 0;
}

int rt1_pw_bwd_grid(int M, int max_blocks) {
    const int strips = (M + ROWS - 1) / ROWS;
    const int g = strips < max_blocks ? strips : max_blocks;
    return g < 1 ? 1 : g;
}

// dwp: [grid][CE][CIN] fp32 partials (grid = rt1_pw_bwd_grid); consts: [5][CE] = sc, sh, k1, k2, k0
int rt1_pw_bwd(const bf16_t* dA, const bf16_t* y, const bf16_t* x, const bf16_t* We, const float* consts, int M,
               int CE, int CIN, bf16_t* dx, const bf16_t* dout, const float* fmul, int HW, float* dwp, int grid,
               hipStream_t st) {
#define X(A, B) if (CE == A && CIN == B) return launch<A, B>(dA, y, x, We, consts, M, dx, dout, fmul, HW, dwp, grid, st);
    RT1_PWBWD_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

}  // extern "C"
