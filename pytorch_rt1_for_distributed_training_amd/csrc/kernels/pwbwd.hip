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
constexpr int PWZ_PF = 1;       // pw_bwd_z: next strip's dz pieces in registers during the weight-gradient MFMAs
constexpr int PWZ_PF_KC = 6;    // ... all of them for KC <= this many 32-channel chunks (Ce = 288, KC 9, would drop a wave
                     // per SIMD) ...
constexpr int PWZ_PF_PART = 0;  // ... and the first this many beyond that (5 at Ce = 288 keeps 2 waves: step-neutral, r4_pwz_part_ab.log)

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

// ------------------------------------------------------------------ y-free variant (pw_bwd_z)
// The BN1 backward apply dy1 = k1*dz + k2*y1 + k0 is the only reason the kernel above reads the Ce-wide y1 (the
// largest tensor of the block: 5 GB at block 2).  y1 = x @ We^T is linear in the block input, so both products can
// be rewritten over the Cin-wide x instead (k* are per-Ce-channel constants, We is [Ce, Cin]):
//
//   dx  = dy1 @ We   = (k1*dz) @ We  +  x @ Mk  +  r0           Mk = We^T diag(k2) We  [Cin, Cin],  r0 = k0 @ We
//   dWe = dy1^T @ x  = diag(k1) (dz^T x)  +  diag(k2) We G  +  k0 (x) sx            G = x^T x,  sx = sum_m x
//
// The depthwise backward stores dz = dA1 * silu'(bn1(y1)) directly (its BN1 epilogue already forms it), so this
// kernel reads dz and x only: dy1's operand is k1*dz, the x @ Mk correction is two more MFMAs per output tile against
// a hi/lo bf16 split of Mk (x is exact bf16, so the correction keeps ~fp32 accuracy), and G / sx come out of the wgrad
// loop's x fragments (sx as an MFMA against a ones fragment).  pw_bwd_prep_kernel builds Mk / r0 once per call,
// pw_bwd_finish_kernel adds the G / sx terms to the fixed-order sum of the per-workgroup partials.
template <int CE, int CIN>
struct ZShape {
    using S = BwdShape<CE, CIN>;
    static constexpr int KCI = (CIN + 31) / 32;        // 32-channel k-chunks of the x @ Mk correction
    static constexpr int KCP = KCI * 32;               // Mk image row length (bf16, zero padded; global, L1-resident)
    static constexpr int NG = S::NTI * S::NTI;         // G tiles
    static constexpr int TPG = (NG + 3) / 4;           // G tiles per wave
    static constexpr size_t w_off = 0;
    static constexpr size_t k_off = w_off + (size_t)S::CINP * S::LDW * 2;        // k1 [CEP]
    static constexpr size_t r_off = k_off + (size_t)S::CEP * 4;                  // r0 [CINP]
    static constexpr size_t y_off = r_off + (size_t)S::CINP * 4;
    static constexpr size_t x_off = y_off + (size_t)ROWS * S::LDY * 2;
    static constexpr size_t lds = x_off + (size_t)ROWS * S::LDX * 2;
    static constexpr int PW = CE * CIN + CIN * CIN + CIN;                      // partial row: dWe | G | sx
};

template <int CE, int CIN, bool SKIP>
__global__ __launch_bounds__(BLOCK) void pw_bwd_z_kernel(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ x,
                                                         const bf16_t* __restrict__ We,
                                                         const float* __restrict__ consts,
                                                         const bf16_t* __restrict__ mk, const float* __restrict__ r0,
                                                         int M, bf16_t* __restrict__ dx,
                                                         const bf16_t* __restrict__ dout,
                                                         const float* __restrict__ fmul, int HW,
                                                         float* __restrict__ part) {
    using S = BwdShape<CE, CIN>;
    using Z = ZShape<CE, CIN>;
    constexpr int KC = S::KC, CEP = S::CEP, NTI = S::NTI, CINP = S::CINP, NTE = S::NTE, TPW = S::TPW;
    constexpr int LDW = S::LDW, LDY = S::LDY, LDX = S::LDX, KCI = Z::KCI, KCP = Z::KCP, NG = Z::NG, TPG = Z::TPG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* wl = reinterpret_cast<bf16_t*>(smem + Z::w_off);
    float* k1l = reinterpret_cast<float*>(smem + Z::k_off);
    float* r0l = reinterpret_cast<float*>(smem + Z::r_off);
    bf16_t* yl = reinterpret_cast<bf16_t*>(smem + Z::y_off);
    bf16_t* xl = reinterpret_cast<bf16_t*>(smem + Z::x_off);
    // wave index in a scalar register: the G / sx tile selection below branches on it per wave, with compile-time
    // register indices (a lane-varying index into xb[] compiled to ~1800 v_cndmask selects)
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int lr = lane & 15, lh = lane >> 4;

    for (int i = t; i < CINP * CEP; i += BLOCK) {
        const int ci = i / CEP, ce = i - ci * CEP;
        wl[ci * LDW + ce] = (ci < CIN && ce < CE) ? We[ce * CIN + ci] : (bf16_t)0;
    }
    for (int i = t; i < CEP; i += BLOCK) k1l[i] = i < CE ? consts[2 * CE + i] : 0.f;
    for (int i = t; i < CINP; i += BLOCK) r0l[i] = i < CIN ? r0[i] : 0.f;
    if constexpr (CINP > CIN) {
        for (int i = t; i < ROWS * (CINP - CIN); i += BLOCK) {
            const int r = i / (CINP - CIN), c = CIN + (i - r * (CINP - CIN));
            xl[r * LDX + c] = 0;
        }
    }

    f32x4 accw[TPW][NTI], accg[TPG], accs;
#pragma unroll
    for (int a = 0; a < TPW; ++a)
#pragma unroll
        for (int b = 0; b < NTI; ++b) accw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < TPG; ++a) accg[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    accs = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (short)0x3f80;

    const int strips = (M + ROWS - 1) / ROWS;
    // this lane's dz pieces of the NEXT strip, loaded after the current strip's data-gradient stores so they are in
    // flight during its weight-gradient MFMAs (PWZ_PF)
    constexpr int PN = !PWZ_PF ? 0 : KC <= PWZ_PF_KC ? KC : (PWZ_PF_PART < KC ? PWZ_PF_PART : KC);
    constexpr bool PFZ = PN > 0;
    uint4 dzr[PFZ ? PN : 1];
    auto load_dz = [&](int ss) {
        const int rr = ss * ROWS + wave * 16 + lr;
#pragma unroll
        for (int kc = 0; kc < PN; ++kc) {
            const int c0 = kc * 32 + lh * 8;
            dzr[kc] = (rr < M && c0 < CE) ? *reinterpret_cast<const uint4*>(dz + (int64_t)rr * CE + c0)
                                           : make_uint4(0, 0, 0, 0);
        }
    };
    if (PFZ && (int)blockIdx.x < strips) load_dz(blockIdx.x);
    for (int s = blockIdx.x; s < strips; s += gridDim.x) {
        const int m0 = s * ROWS;
        uint4 dzc[PFZ ? PN : 1];
        if constexpr (PFZ) {
#pragma unroll
            for (int kc = 0; kc < PN; ++kc) dzc[kc] = dzr[kc];
        }
        __syncthreads();
        constexpr int XCH = CIN / 8;
        for (int i = t; i < ROWS * XCH; i += BLOCK) {
            const int r = i / XCH, c = (i - r * XCH) * 8;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (m0 + r < M) u = *reinterpret_cast<const uint4*>(x + (int64_t)(m0 + r) * CIN + c);
            *reinterpret_cast<uint4*>(xl + r * LDX + c) = u;
        }
        const int row = m0 + wave * 16 + lr;
        const bool rok = row < M;
        f32x4 accd[NTI];
#pragma unroll
        for (int b = 0; b < NTI; ++b) accd[b] = f32x4{0.f, 0.f, 0.f, 0.f};
        // ---- (k1 * dz) @ We
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            const int c0 = kc * 32 + lh * 8;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (rok && c0 < CE) {
                float zv[8], k1[8];
                if (kc < PN) unpack8(dzc[kc < PN ? kc : 0], zv);
                else load8(dz + (int64_t)row * CE + c0, zv);
                load8f(k1l + c0, k1);
                u.x = pack2(k1[0] * zv[0], k1[1] * zv[1]); u.y = pack2(k1[2] * zv[2], k1[3] * zv[3]);
                u.z = pack2(k1[4] * zv[4], k1[5] * zv[5]); u.w = pack2(k1[6] * zv[6], k1[7] * zv[7]);
            }
            *reinterpret_cast<uint4*>(yl + (wave * 16 + lr) * LDY + c0) = u;
            bf16x8 df;
            __builtin_memcpy(&df, &u, 16);
#pragma unroll
            for (int b = 0; b < NTI; ++b) {
                const bf16x8 wf = *reinterpret_cast<const bf16x8*>(wl + (b * 16 + lr) * LDW + kc * 32 + lh * 8);
                accd[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, df, accd[b], 0, 0, 0);
            }
        }
        // ---- + x @ Mk (hi + lo)
#pragma unroll
        for (int kk = 0; kk < KCI; ++kk) {
            const int c0 = kk * 32 + lh * 8;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (rok && c0 < CIN) u = *reinterpret_cast<const uint4*>(x + (int64_t)row * CIN + c0);
            bf16x8 xf;
            __builtin_memcpy(&xf, &u, 16);
#pragma unroll
            for (int b = 0; b < NTI; ++b) {
                const bf16x8 mh = *reinterpret_cast<const bf16x8*>(mk + (b * 16 + lr) * KCP + c0);
                const bf16x8 mlo = *reinterpret_cast<const bf16x8*>(mk + (CINP + b * 16 + lr) * KCP + c0);
                accd[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mh, xf, accd[b], 0, 0, 0);
                accd[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mlo, xf, accd[b], 0, 0, 0);
            }
        }
        if (rok) {
            const int64_t n = SKIP ? (int64_t)((uint32_t)row / (uint32_t)HW) : 0;
#pragma unroll
            for (int b = 0; b < NTI; ++b) {
                const int ci = b * 16 + lh * 4;
                if (ci < CIN) {
                    const float4 rv = *reinterpret_cast<const float4*>(r0l + ci);
                    float o[4] = {accd[b][0] + rv.x, accd[b][1] + rv.y, accd[b][2] + rv.z, accd[b][3] + rv.w};
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
        if (PFZ && s + (int)gridDim.x < strips) load_dz(s + gridDim.x);
        __syncthreads();
        // ---- wgrad (k1*dz)^T x, G = x^T x, sx = x^T 1
#pragma unroll
        for (int ks = 0; ks < ROWS / 32; ++ks) {
            const int q = (lane & 15) >> 2, p = lane & 3;
            const int r0w = ks * 32 + lh * 8 + q;
            bf16x8 xb[NTI];
#pragma unroll
            for (int b = 0; b < NTI; ++b)
                xb[b] = tr_read8(xl + r0w * LDX + b * 16 + p * 4, xl + (r0w + 4) * LDX + b * 16 + p * 4);
#pragma unroll
            for (int a = 0; a < TPW; ++a) {
                const int et = wave + 4 * a;
                if (et < NTE) {
                    const bf16x8 ya = tr_read8(yl + r0w * LDY + et * 16 + p * 4, yl + (r0w + 4) * LDY + et * 16 + p * 4);
#pragma unroll
                    for (int b = 0; b < NTI; ++b)
                        accw[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ya, xb[b], accw[a][b], 0, 0, 0);
                }
            }
#pragma unroll
            for (int gi = 0; gi < NG; ++gi)
                if ((gi & 3) == wave)
                    accg[gi >> 2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[gi / NTI], xb[gi % NTI], accg[gi >> 2],
                                                                            0, 0, 0);
#pragma unroll
            for (int b = 0; b < NTI; ++b)
                if (b == wave) accs = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[b], ones, accs, 0, 0, 0);
        }
    }
    float* pr = part + (int64_t)blockIdx.x * Z::PW;
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
                if (ce < CE) pr[ce * CIN + ci] = accw[a][b][i];
            }
        }
    }
#pragma unroll
    for (int a = 0; a < TPG; ++a) {
        const int gt = wave + 4 * a;
        if (gt >= NG) continue;
        const int cj = (gt % NTI) * 16 + lr;
        if (cj >= CIN) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ci = (gt / NTI) * 16 + lh * 4 + i;
            if (ci < CIN) pr[CE * CIN + ci * CIN + cj] = accg[a][i];
        }
    }
    if (wave < NTI && lr == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ci = wave * 16 + lh * 4 + i;
            if (ci < CIN) pr[CE * CIN + CIN * CIN + ci] = accs[i];
        }
    }
}

// Mk = We^T diag(k2) We as a hi / lo bf16 pair of zero-padded MFMA A images [2][CINP][KCP] (KCP = Cin rounded up to
// 32), r0 = k0 @ We [CIN] (k2, k0 = consts rows 3, 4)
// (We, k2, k0 staged in LDS first: the per-thread dot products read strided columns of We)
__global__ __launch_bounds__(256) void pw_bwd_prep_kernel(const bf16_t* __restrict__ We,
                                                          const float* __restrict__ consts, int CE, int CIN, int CINP,
                                                          int KCP, bf16_t* __restrict__ mk, float* __restrict__ r0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* k2l = reinterpret_cast<float*>(smem);
    float* k0l = k2l + CE;
    bf16_t* wl = reinterpret_cast<bf16_t*>(k0l + CE);
    for (int j = threadIdx.x; j < CE; j += 256) {
        k2l[j] = consts[3 * CE + j];
        k0l[j] = consts[4 * CE + j];
    }
    for (int j = threadIdx.x; j < CE * CIN; j += 256) wl[j] = We[j];
    __syncthreads();
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < CINP * KCP) {
        const int ci = i / KCP, cj = i - ci * KCP;
        float a = 0.f;
        if (ci < CIN && cj < CIN)
            for (int ce = 0; ce < CE; ++ce) a = fmaf(bf2f(wl[ce * CIN + ci]) * k2l[ce], bf2f(wl[ce * CIN + cj]), a);
        const bf16_t hi = f2bf(a);
        mk[i] = hi;
        mk[CINP * KCP + i] = f2bf(a - bf2f(hi));
    } else if (i < CINP * KCP + CIN) {
        const int ci = i - CINP * KCP;
        float a = 0.f;
        for (int ce = 0; ce < CE; ++ce) a = fmaf(k0l[ce], bf2f(wl[ce * CIN + ci]), a);
        r0[ci] = a;
    }
}

// dWe[ce][ci] = S[ce][ci] + k2[ce] * sum_cj We[ce][cj] G[cj][ci] + k0[ce] * sx[ci]   (S = summed partial rows)
__global__ __launch_bounds__(256) void pw_bwd_finish_kernel(const float* __restrict__ S, const bf16_t* __restrict__ We,
                                                            const float* __restrict__ consts, int CE, int CIN,
                                                            float* __restrict__ dWe) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= CE * CIN) return;
    const int ce = i / CIN, ci = i - ce * CIN;
    const float* G = S + CE * CIN;
    const float* sx = G + CIN * CIN;
    float a = 0.f;
    for (int cj = 0; cj < CIN; ++cj) a = fmaf(bf2f(We[ce * CIN + cj]), G[cj * CIN + ci], a);
    dWe[i] = S[i] + consts[3 * CE + ce] * a + consts[4 * CE + ce] * sx[ci];
}

// ---- the same algebra for the wide expand convs (blocks 9-17, Cin 96 / 136):
//   dx = dz @ (diag(k1) We) + x @ Mk + r0   (pwtall.hip pw_tall_tail / gemm.hip TAIL: both products in one K loop)
//   dWe = diag(k1) (dz^T x) + diag(k2) We G + k0 (x) sx            (wgrad.hip for dz^T x and G, then pw_z_finish)
// pw_z_prep_kernel, ONE launch for the three small operands:
//   * workgroups [0, n_mk): Mk = We^T diag(k2) We (bf16 [CIN, CIN]) and r0 = k0^T We (fp32 [CIN]) as 32 x 32 tiles of
//     the [CIN + 1, CIN] product (row CIN = r0); 16 waves split the CE reduction (wave w takes ce = w, w + 16, ...),
//     each lane a 4 x 4 block of the tile in fp32 FMAs from L2-resident We rows, the 16 slices summed in a fixed
//     order through LDS (deterministic).  It was a pw_z_prep launch + a hipBLASLt GEMM (MT16x16 / MT32x32 tiles,
//     6-10 us) + a bf16 conversion of Mk: three dependent launches per wide block.
//   * workgroups [n_mk, ...): the transposed scaled weights Wt[ci][ce] = k1[ce] We[ce][ci] (the dgrad's [N, K]
//     operand) through a 32 x 32 LDS tile of We (coalesced reads of We rows and writes of Wt rows).
// (Per-thread dot products down the We columns, one output per thread, ran 45-110 us per call: latency-bound.)
constexpr int ZP_THREADS = 1024, ZP_SLICES = ZP_THREADS / 64, ZP_CH = 64;

__device__ __forceinline__ void zp_load4(const bf16_t* __restrict__ row, int c0, int CIN, bool vec, float (&o)[4]) {
    if (vec && c0 + 3 < CIN) {
        const uint2 u = *reinterpret_cast<const uint2*>(row + c0);
        o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xffff0000u);
        o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xffff0000u);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = c0 + k < CIN ? bf2f(row[c0 + k]) : 0.f;
    }
}

__global__ __launch_bounds__(ZP_THREADS) void pw_z_prep_kernel(const bf16_t* __restrict__ We,
                                                               const float* __restrict__ consts, int CE, int CIN,
                                                               int n_mk, int tj_n, bf16_t* __restrict__ wt,
                                                               bf16_t* __restrict__ mk, float* __restrict__ r0) {
    __shared__ float red[ZP_SLICES][32 * 32];
    const int t = threadIdx.x;
    const float* k1 = consts + 2 * CE;
    const float* k2 = consts + 3 * CE;
    const float* k0 = consts + 4 * CE;
    if ((int)blockIdx.x >= n_mk) {
        // Wt tile: 32 ce x 32 ci
        float(*tile)[33] = reinterpret_cast<float(*)[33]>(&red[0][0]);
        const int b = blockIdx.x - n_mk;
        const int tiles_ce = (CE + 31) / 32;
        const int ce0 = (b % tiles_ce) * 32, ci0 = (b / tiles_ce) * 32;
        const int tx = t & 31, ty = t >> 5;                    // 32 x 32
        const int ce = ce0 + ty, ci = ci0 + tx;
        tile[ty][tx] = (ce < CE && ci < CIN) ? bf2f(We[(int64_t)ce * CIN + ci]) : 0.f;
        __syncthreads();
        const int ce2 = ce0 + tx, ci2 = ci0 + ty;
        if (ce2 < CE && ci2 < CIN) wt[(int64_t)ci2 * CE + ce2] = f2bf(k1[ce2] * tile[tx][ty]);
        return;
    }
    const int ti = blockIdx.x / tj_n, tj = blockIdx.x - ti * tj_n;
    const int lane = t & 63, w = t >> 6;
    const int ri = (lane >> 3) * 4, cj = (lane & 7) * 4;
    const int i0 = ti * 32 + ri;
    float acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
    // We's two 32-column slices (rows ti, columns tj of the product) go through LDS in chunks of ZP_CH rows: every
    // thread loads 4 bf16 of one chunk row (threads [0, 512) the i slice, [512, 1024) the j slice), the next chunk's
    // loads in flight while the 16 waves run the current one (wave w takes chunk rows 4w .. 4w + 3).  Loaded row by row
    // straight from L2 each wave waited ~CE / 64 full L2 round trips; this is CE / ZP_CH + 1 of them per workgroup.
    uint2* wl = reinterpret_cast<uint2*>(&red[0][0]);           // [2][2][ZP_CH][8] uint2, aliases the slice buffer
    const int lrow = (t & 511) >> 3, lc4 = (t & 7) * 4, lsel = t >> 9;
    const int lcol = (lsel ? tj : ti) * 32 + lc4;
    auto load_chunk = [&](int ce0) -> uint2 {
        const int ce = ce0 + lrow;
        if (ce >= CE || lcol >= CIN) return make_uint2(0, 0);
        const bf16_t* row = We + (int64_t)ce * CIN;
        if ((CIN & 3) == 0) return *reinterpret_cast<const uint2*>(row + lcol);
        uint32_t h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = lcol + k < CIN ? (uint32_t)row[lcol + k] : 0u;
        return make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    };
    const int nch = (CE + ZP_CH - 1) / ZP_CH;
    uint2 nxt = load_chunk(0);
    for (int k = 0; k < nch; ++k) {
        const int buf = k & 1;
        wl[((buf * 2 + lsel) * ZP_CH + lrow) * 8 + (lc4 >> 2)] = nxt;
        __syncthreads();
        if (k + 1 < nch) nxt = load_chunk((k + 1) * ZP_CH);
#pragma unroll
        for (int q = 0; q < ZP_CH / ZP_SLICES; ++q) {
            const int cl = w * (ZP_CH / ZP_SLICES) + q, ce = k * ZP_CH + cl;
            if (ce >= CE) break;
            const uint2 ua = wl[((buf * 2 + 0) * ZP_CH + cl) * 8 + (ri >> 2)];
            const uint2 ub = wl[((buf * 2 + 1) * ZP_CH + cl) * 8 + (cj >> 2)];
            float a[4] = {__uint_as_float(ua.x << 16), __uint_as_float(ua.x & 0xffff0000u), __uint_as_float(ua.y << 16),
                          __uint_as_float(ua.y & 0xffff0000u)};
            const float b[4] = {__uint_as_float(ub.x << 16), __uint_as_float(ub.x & 0xffff0000u),
                                __uint_as_float(ub.y << 16), __uint_as_float(ub.y & 0xffff0000u)};
            const float s2 = k2[ce], s0 = k0[ce];
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = i0 + r < CIN ? a[r] * s2 : (i0 + r == CIN ? s0 : 0.f);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(a[r], b[c], acc[r][c]);
        }
        // the chunk two iterations ahead overwrites this buffer only after the next barrier
    }
    __syncthreads();                                              // the slice buffer is reused for the partial tiles
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) red[w][(ri + r) * 32 + cj + c] = acc[r][c];
    __syncthreads();
    // one output per thread, the 16 slices summed in slice order
    const int oi = t >> 5, oj = t & 31;
    const int i = ti * 32 + oi, j = tj * 32 + oj;
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < ZP_SLICES; ++s) sum += red[s][t];
    if (j < CIN) {
        if (i < CIN) mk[(int64_t)i * CIN + j] = f2bf(sum);
        else if (i == CIN) r0[j] = sum;
    }
}

// dWe[ce][ci] = k1[ce] S[ce][ci] + k2[ce] sum_cj We[ce][cj] G[cj][ci] + k0[ce] sx[ci]
// S: the wgrad kernel's row-split partials [splits, CE, CIN] of dz^T x, summed here in split order (no separate
// colsum launch)
__global__ __launch_bounds__(256) void pw_z_finish_kernel(const float* __restrict__ S, int splits,
                                                          const float* __restrict__ G,
                                                          const float* __restrict__ sx, const bf16_t* __restrict__ We,
                                                          const float* __restrict__ consts, int CE, int CIN,
                                                          float* __restrict__ dWe) {
    const int64_t n = (int64_t)CE * CIN;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int ce = (int)(i / CIN), ci = (int)(i - (int64_t)ce * CIN);
    float s = S[i];
    for (int k = 1; k < splits; ++k) s += S[k * n + i];
    float a = 0.f;
#pragma unroll 8
    for (int cj = 0; cj < CIN; ++cj) a = fmaf(bf2f(We[(int64_t)ce * CIN + cj]), G[(int64_t)cj * CIN + ci], a);
    dWe[i] = consts[2 * CE + ce] * s + consts[3 * CE + ce] * a + consts[4 * CE + ce] * sx[ci];
}

#define PWBWD_SHAPES(X) X(144, 24) X(192, 32) X(288, 48)

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

template <int CE, int CIN>
int launch_z(const bf16_t* dz, const bf16_t* x, const bf16_t* We, const float* consts, const bf16_t* mk,
             const float* r0, int M, bf16_t* dx, const bf16_t* dout, const float* fmul, int HW, float* part, int grid,
             hipStream_t st) {
    using Z = ZShape<CE, CIN>;
    if (dout)
        hipLaunchKernelGGL((pw_bwd_z_kernel<CE, CIN, true>), dim3(grid), dim3(BLOCK), Z::lds, st, dz, x, We, consts, mk,
                           r0, M, dx, dout, fmul, HW, part);
    else
        hipLaunchKernelGGL((pw_bwd_z_kernel<CE, CIN, false>), dim3(grid), dim3(BLOCK), Z::lds, st, dz, x, We, consts,
                           mk, r0, M, dx, dout, fmul, HW, part);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int rt1_pw_bwd_supported(int CE, int CIN) {
#define X(A, B) if (CE == A && CIN == B) return 1;
    PWBWD_SHAPES(X)
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
    PWBWD_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

// y-free expand backward.  part: [grid][CE*CIN + CIN*CIN + CIN] fp32 partials (rt1_pw_bwd_z_width); mk:
// rt1_pw_bwd_z_mk_elems bf16 and r0 [CIN] fp32 scratch written by the prep launch; consts [5][CE] as rt1_pw_bwd
int rt1_pw_bwd_z_width(int CE, int CIN) { return CE * CIN + CIN * CIN + CIN; }
int rt1_pw_bwd_z_mk_elems(int CIN) { return 2 * ((CIN + 15) / 16 * 16) * ((CIN + 31) / 32 * 32); }

int rt1_pw_bwd_z(const bf16_t* dz, const bf16_t* x, const bf16_t* We, const float* consts, int M, int CE, int CIN,
                 bf16_t* mk, float* r0, bf16_t* dx, const bf16_t* dout, const float* fmul, int HW, float* part,
                 int grid, hipStream_t st) {
    if (!rt1_pw_bwd_supported(CE, CIN) || M <= 0 || grid <= 0) return (int)hipErrorInvalidValue;
    const int CINP = (CIN + 15) / 16 * 16, KCP = (CIN + 31) / 32 * 32;
    hipLaunchKernelGGL(pw_bwd_prep_kernel, dim3((CINP * KCP + CIN + 255) / 256), dim3(256),
                       (size_t)CE * 8 + (size_t)CE * CIN * 2, st, We, consts, CE, CIN, CINP, KCP, mk, r0);
#define X(A, B) if (CE == A && CIN == B) return launch_z<A, B>(dz, x, We, consts, mk, r0, M, dx, dout, fmul, HW, part, grid, st);
    PWBWD_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

int rt1_pw_bwd_z_finish(const float* S, const bf16_t* We, const float* consts, int CE, int CIN, float* dWe,
                        hipStream_t st) {
    hipLaunchKernelGGL(pw_bwd_finish_kernel, dim3((CE * CIN + 255) / 256), dim3(256), 0, st, S, We, consts, CE, CIN,
                       dWe);
    return (int)hipGetLastError();
}

int rt1_pw_z_prep(const bf16_t* We, const float* consts, int CE, int CIN, bf16_t* wt, bf16_t* mk, float* r0,
                  hipStream_t st) {
    if (CIN <= 0 || CE <= 0) return (int)hipErrorInvalidValue;
    const int tj_n = (CIN + 31) / 32, ti_n = (CIN + 1 + 31) / 32;
    const int n_mk = ti_n * tj_n, n_wt = ((CE + 31) / 32) * tj_n;
    hipLaunchKernelGGL(pw_z_prep_kernel, dim3((unsigned)(n_mk + n_wt)), dim3(ZP_THREADS), 0, st, We, consts, CE, CIN,
                       n_mk, tj_n, wt, mk, r0);
    return (int)hipGetLastError();
}

int rt1_pw_z_finish(const float* S, int splits, const float* G, const float* sx, const bf16_t* We,
                    const float* consts, int CE, int CIN, float* dWe, hipStream_t st) {
    const int64_t n = (int64_t)CE * CIN;
    if (splits < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(pw_z_finish_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, S, splits, G, sx, We,
                       consts, CE, CIN, dWe);
    return (int)hipGetLastError();
}

}  // extern "C"
