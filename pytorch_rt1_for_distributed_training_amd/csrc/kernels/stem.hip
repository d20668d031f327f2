// EfficientNet stem: 3x3 stride-2 conv (3 -> COUT) on the raw frames with the
// RT-1 random-shift augmentation and the uint8 -> [0,1] conversion fused into
// the input read (SURVEY K1+K2: the reference pads, fancy-indexes and /255s the
// whole batch before the conv; here no shifted copy is ever materialised).
//
//   p[ci, y, x] = img[ci, y+dy, x+dx] / 255 (uint8) or img[...] (float), 0 outside
//   out[n, ho, wo, co] = sum_{ci,kh,kw} W[co,ci,kh,kw] * p[ci, 2ho-1+kh, 2wo-1+kw]
//
// (dy, dx) are read from DEVICE memory so a captured hipGraph replays with a
// fresh shift each step.  Output is channels-last bf16 plus per-workgroup BN
// partial rows.  Backward needs only dW (frames have no gradient).
#include "common.h"

using namespace rt1;

namespace {

constexpr int BLOCK = 256;
constexpr int COUT = 40, NCV = COUT / 8;
constexpr int TOH = 12, TOW = 32;                    // output tile (rows x cols)
constexpr int IH = 2 * TOH + 1, IW = 2 * TOW + 1;    // input window of the tile (stride 2, pad 1)
constexpr int SR = 4;                                // outputs per thread strip (along W)
constexpr int STRIPS = TOH * TOW / SR;               // 96
constexpr int STEM_PIPE = 1;                              // forward: next tile's window loads in flight during the products

template <typename TIn>
__device__ __forceinline__ float to_unit(TIn v) {
    if constexpr (sizeof(TIn) == 1) return (float)v * (1.f / 255.f);
    else return (float)v;
}

// Stage the tile's input window p[ci][r][c] = shifted frame at (y0 + r, x0 + c), zero outside:
//   p(y, x) = img[y + dy][x + dx] if (y, x) and (y + dy, x + dx) are both inside the frame.
// Consecutive threads read consecutive columns of one image row (coalesced).
template <typename TIn>
__device__ __forceinline__ void stage_input(float* in, const TIn* __restrict__ img, int n, int H, int W, int y0,
                                            int x0, int dy, int dx) {
    for (int e = threadIdx.x; e < 3 * IH * IW; e += BLOCK) {
        const int ci = e / (IH * IW);
        const int rem = e - ci * IH * IW;
        const int r = rem / IW, c = rem - r * IW;
        const int y = y0 + r, x = x0 + c, ys = y + dy, xs = x + dx;
        float v = 0.f;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W && (unsigned)ys < (unsigned)H &&
            (unsigned)xs < (unsigned)W)
            v = to_unit(img[(((int64_t)n * 3 + ci) * H + ys) * W + xs]);
        in[e] = v;
    }
}

__device__ __forceinline__ void tile_of(int64_t t, int tiles_h, int tiles_w, int& n, int& oh0, int& ow0) {
    n = (int)(t / (tiles_h * tiles_w));
    const int r = (int)(t - (int64_t)n * tiles_h * tiles_w);
    oh0 = (r / tiles_w) * TOH;
    ow0 = (r % tiles_w) * TOW;
}

// LDS ordering between the lanes of one wave (a staging buffer written, then read by other lanes of the same wave)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The MFMA kernels' bf16 input window in LDS: rows of IWP = 68 (IW = 65 padded to 4-column groups).  uint8 frames
// with W % 4 == 0 and a 4-byte aligned base (vec) are staged 4 columns at a time from two aligned dword loads per row
// group (v_alignbyte-style funnel shift): one load pair + one 8-byte LDS store per 4 pixels instead of 4 byte loads
// and 4 two-byte stores.  Zero outside the frame for both the shifted and the unshifted coordinate; the same
// x / 255 and RNE bf16 rounding as the element-wise path.
constexpr int IWP = 68;
// The vector staging split in two for software pipelining: win_load issues the (<= WIN_K per thread) aligned dword
// pairs of a tile's window into registers, win_store funnel-shifts / converts them into LDS -- the next tile's loads
// are in flight while the current tile multiplies.
constexpr int WIN_G = (IW + 3) / 4, WIN_K = (3 * IH * WIN_G + BLOCK - 1) / BLOCK;
struct WinRegs {
    uint32_t lo[WIN_K], hi[WIN_K];
};
__device__ __forceinline__ void win_load(WinRegs& w, const uint8_t* __restrict__ img, int n, int H, int W, int y0,
                                         int x0, int dy, int dx) {
#pragma unroll
    for (int k = 0; k < WIN_K; ++k) {
        const int e = threadIdx.x + k * BLOCK;
        w.lo[k] = w.hi[k] = 0u;
        if (e >= 3 * IH * WIN_G) continue;
        const int rowi = e / WIN_G, g = e - rowi * WIN_G;
        const int ci = rowi / IH, r = rowi - ci * IH;
        const int y = y0 + r, ys = y + dy;
        if ((unsigned)y < (unsigned)H && (unsigned)ys < (unsigned)H) {
            const uint8_t* rowp = img + (((int64_t)n * 3 + ci) * H + ys) * W;
            const int xs = x0 + 4 * g + dx;
            const int a = xs >= 0 ? (xs & ~3) : -((3 - xs) & ~3);
            if (a >= 0 && a < W) w.lo[k] = *reinterpret_cast<const uint32_t*>(rowp + a);
            if (a + 4 >= 0 && a + 4 < W) w.hi[k] = *reinterpret_cast<const uint32_t*>(rowp + a + 4);
        }
    }
}
__device__ __forceinline__ void win_store(bf16_t* __restrict__ inb, const WinRegs& w, int W, int x0, int dx) {
#pragma unroll
    for (int k = 0; k < WIN_K; ++k) {
        const int e = threadIdx.x + k * BLOCK;
        if (e >= 3 * IH * WIN_G) continue;
        const int rowi = e / WIN_G, g = e - rowi * WIN_G;
        const int xc = x0 + 4 * g, xs = xc + dx;
        const int a = xs >= 0 ? (xs & ~3) : -((3 - xs) & ~3);
        const uint32_t b = (uint32_t)((((uint64_t)w.hi[k] << 32) | w.lo[k]) >> (8 * (xs - a)));
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            v[j] = (unsigned)(xc + j) < (unsigned)W ? (float)((b >> (8 * j)) & 255u) * (1.f / 255.f) : 0.f;
        *reinterpret_cast<uint2*>(inb + rowi * IWP + 4 * g) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
}

template <typename TIn>
__device__ __forceinline__ void stage_window_bf16(bf16_t* __restrict__ inb, const TIn* __restrict__ img, int n, int H,
                                                  int W, int y0, int x0, int dy, int dx, bool vec) {
    if constexpr (sizeof(TIn) == 1) {
        if (vec) {
            constexpr int G = (IW + 3) / 4;           // 17 four-column groups per window row
            for (int e = threadIdx.x; e < 3 * IH * G; e += BLOCK) {
                const int rowi = e / G, g = e - rowi * G;          // rowi = ci * IH + r
                const int ci = rowi / IH, r = rowi - ci * IH;
                const int y = y0 + r, ys = y + dy;
                const int xc = x0 + 4 * g, xs = xc + dx;
                uint32_t b = 0u;
                if ((unsigned)y < (unsigned)H && (unsigned)ys < (unsigned)H) {
                    const uint8_t* rowp = reinterpret_cast<const uint8_t*>(img) + (((int64_t)n * 3 + ci) * H + ys) * W;
                    const int a = xs >= 0 ? (xs & ~3) : -((3 - xs) & ~3);   // floor to a multiple of 4
                    // W % 4 == 0: an aligned dword is all inside the row or all outside
                    const uint32_t lo = (a >= 0 && a < W) ? *reinterpret_cast<const uint32_t*>(rowp + a) : 0u;
                    const uint32_t hi = (a + 4 >= 0 && a + 4 < W) ? *reinterpret_cast<const uint32_t*>(rowp + a + 4) : 0u;
                    b = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (xs - a)));
                }
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    v[j] = (unsigned)(xc + j) < (unsigned)W ? (float)((b >> (8 * j)) & 255u) * (1.f / 255.f) : 0.f;
                *reinterpret_cast<uint2*>(inb + rowi * IWP + 4 * g) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
            }
            return;
        }
    }
    for (int e = threadIdx.x; e < 3 * IH * IW; e += BLOCK) {
        const int rowi = e / IW, c = e - rowi * IW;
        const int ci = rowi / IH, r = rowi - ci * IH;
        const int y = y0 + r, x = x0 + c, ys = y + dy, xs = x + dx;
        float v = 0.f;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W && (unsigned)ys < (unsigned)H &&
            (unsigned)xs < (unsigned)W)
            v = to_unit(img[(((int64_t)n * 3 + ci) * H + ys) * W + xs]);
        inb[rowi * IWP + c] = f2bf(v);
    }
}

// dW on the matrix cores: per tile, dW[co][tap] += sum_px dy[px][co] * P[px][tap] as 16x16x32 bf16 MFMAs with
// the PIXELS as the reduction axis (3 co-blocks x 2 tap-blocks of 16 = 48 x 32 >= 40 x 27).  The dy tile is
// staged as [px][co] with 16-byte stores and read back with the gfx950 LDS transpose (ds_read_b64_tr_b16: the
// [co][px] layout with 2-byte stores was slower); B fragments (8 pixels of one tap) are
// gathered from the fp32 input window and rounded to bf16 (the bf16 operands autocast would use).  The 4 waves
// split the tile's 12 pixel steps; their accumulators are summed in wave order at the end (deterministic).
constexpr int TPX = TOH * TOW;            // 384 pixels per tile
constexpr int LDY = 48;                   // natural [px][co] dy tile row (40 channels + 8 zero, bf16)
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// The stem BN's backward applied while the dy tile is staged (block 0 carries the stem BN, StemPreFn): dyv then
// holds g = dL/d silu(bn(x)) and dy = k1 * g * silu'(x*scale + shift) + k2 * x + k0 is rebuilt per element, with
// exactly the operations and bf16 rounding of bn_bwd_apply (bn.hip), so the [N, Ho, Wo, 40] dy never reaches HBM.
struct StemBnBwd {
    const bf16_t* x;
    const float *scale, *shift, *mean, *rstd, *gamma, *mdz, *mdzx;
};

template <typename TIn, bool BN>
__global__ __launch_bounds__(BLOCK) void stem_wgrad_mfma_kernel(const TIn* __restrict__ img,
                                                                const int* __restrict__ shift,
                                                                const bf16_t* __restrict__ dyv, int N, int H, int W,
                                                                int Ho, int Wo, float* __restrict__ dwp, StemBnBwd bn,
                                                                int vec) {
    __shared__ __attribute__((aligned(16))) bf16_t inb[3 * IH * IWP];  // input window, already bf16
    __shared__ __attribute__((aligned(16))) bf16_t gtT[TPX * LDY];
    __shared__ float kc[BN ? 5 * COUT : 1];                            // k0, k1, k2, scale, shift
    if constexpr (BN) {
        for (int c = threadIdx.x; c < COUT; c += BLOCK) {
            const float rr = bn.rstd[c], b = bn.mdzx[c];
            const float k1 = (bn.gamma ? bn.gamma[c] : 1.f) * rr;
            kc[c] = -k1 * (bn.mdz[c] - bn.mean[c] * rr * b);
            kc[COUT + c] = k1;
            kc[2 * COUT + c] = -k1 * rr * b;
            kc[3 * COUT + c] = bn.scale[c];
            kc[4 * COUT + c] = bn.shift[c];
        }
    }
    const int dy = shift ? shift[0] : 0, dx = shift ? shift[1] : 0;
    const int tiles_h = (Ho + TOH - 1) / TOH, tiles_w = (Wo + TOW - 1) / TOW;
    const int64_t ntiles = (int64_t)N * tiles_h * tiles_w;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lg = lane >> 4;
    // rows 40..47 of the transposed tile stay zero (the third co-block's padding)
    for (int i = threadIdx.x; i < TPX; i += BLOCK)                    // channels 40..47 of every pixel row stay zero
        *reinterpret_cast<uint4*>(gtT + i * LDY + 40) = make_uint4(0, 0, 0, 0);
    // this lane's two B-fragment taps: tap = tb * 16 + lr -> (ci, kh, kw), or none past 27
    int toff[2];
    bool tval[2];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
        const int tap = tb * 16 + lr;
        tval[tb] = tap < 27;
        const int ci = tap / 9, kk = tap % 9;
        toff[tb] = tval[tb] ? (ci * IH + kk / 3) * IWP + kk % 3 : 0;
    }
    f32x4_t acc[3][2];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // uint8 vector path: the next tile's window and dy (/ x) pieces are loaded into registers while this tile
    // multiplies (same staging math as below, applied when they are written to LDS)
    constexpr bool U8 = sizeof(TIn) == 1;
    constexpr int DYK = (TPX * NCV + BLOCK - 1) / BLOCK;
    const bool pipe = U8 && vec != 0 && STEM_PIPE;
    WinRegs wr;
    uint4 gq[DYK], xq[BN ? DYK : 1];
    auto dy_load = [&](int64_t tt) {
        int n1, a1, b1;
        tile_of(tt, tiles_h, tiles_w, n1, a1, b1);
        if constexpr (U8) win_load(wr, img, n1, H, W, 2 * a1 - 1, 2 * b1 - 1, dy, dx);
#pragma unroll
        for (int k = 0; k < DYK; ++k) {
            const int e = threadIdx.x + k * BLOCK;
            gq[k] = make_uint4(0, 0, 0, 0);
            if constexpr (BN) xq[k] = make_uint4(0, 0, 0, 0);
            if (e >= TPX * NCV) continue;
            const int px = e / NCV, v = e - px * NCV;
            const int oh = a1 + px / TOW, ow = b1 + px % TOW;
            if (oh < Ho && ow < Wo) {
                const int64_t off = (((int64_t)n1 * Ho + oh) * Wo + ow) * COUT + v * 8;
                gq[k] = *reinterpret_cast<const uint4*>(dyv + off);
                if constexpr (BN) xq[k] = *reinterpret_cast<const uint4*>(bn.x + off);
            }
        }
    };
    auto dy_store = [&](int oh0, int ow0) {
#pragma unroll
        for (int k = 0; k < DYK; ++k) {
            const int e = threadIdx.x + k * BLOCK;
            if (e >= TPX * NCV) continue;
            const int px = e / NCV, v = e - px * NCV;
            uint4 u = gq[k];
            if constexpr (BN) {
                const int oh = oh0 + px / TOW, ow = ow0 + px % TOW;
                if (oh < Ho && ow < Wo) {
                    const uint4 ux = xq[k];
                    const uint32_t gw[4] = {u.x, u.y, u.z, u.w}, xw[4] = {ux.x, ux.y, ux.z, ux.w};
                    float o[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float g = __uint_as_float(j & 1 ? gw[j >> 1] & 0xffff0000u : gw[j >> 1] << 16);
                        const float xv = __uint_as_float(j & 1 ? xw[j >> 1] & 0xffff0000u : xw[j >> 1] << 16);
                        const int c = v * 8 + j;
                        const float dz = g * silu_grad(fmaf(xv, kc[3 * COUT + c], kc[4 * COUT + c]));
                        o[j] = fmaf(kc[COUT + c], dz, fmaf(kc[2 * COUT + c], xv, kc[c]));
                    }
                    u = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
                }
            }
            *reinterpret_cast<uint4*>(gtT + px * LDY + v * 8) = u;
        }
    };
    if (pipe && (int64_t)blockIdx.x < ntiles) {
        if constexpr (BN) __syncthreads();        // kc (the BN constants) is read by dy_store
        dy_load(blockIdx.x);
    }
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        int n, oh0, ow0;
        tile_of(t, tiles_h, tiles_w, n, oh0, ow0);
        __syncthreads();
        if (pipe) {
            win_store(inb, wr, W, 2 * ow0 - 1, dx);
            dy_store(oh0, ow0);
            if (t + gridDim.x < ntiles) dy_load(t + gridDim.x);
            __syncthreads();
        } else {
        stage_window_bf16(inb, img, n, H, W, 2 * oh0 - 1, 2 * ow0 - 1, dy, dx, vec != 0);   // shifted window
        for (int e = threadIdx.x; e < TPX * NCV; e += BLOCK) {          // dy tile -> [co][px], zero outside
            const int px = e / NCV, v = e - px * NCV;
            const int oh = oh0 + px / TOW, ow = ow0 + px % TOW;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (oh < Ho && ow < Wo) {
                const int64_t off = (((int64_t)n * Ho + oh) * Wo + ow) * COUT + v * 8;
                u = *reinterpret_cast<const uint4*>(dyv + off);
                if constexpr (BN) {
                    const uint4 ux = *reinterpret_cast<const uint4*>(bn.x + off);
                    const uint32_t gw[4] = {u.x, u.y, u.z, u.w}, xw[4] = {ux.x, ux.y, ux.z, ux.w};
                    float o[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float g = __uint_as_float(j & 1 ? gw[j >> 1] & 0xffff0000u : gw[j >> 1] << 16);
                        const float xv = __uint_as_float(j & 1 ? xw[j >> 1] & 0xffff0000u : xw[j >> 1] << 16);
                        const int c = v * 8 + j;
                        const float dz = g * silu_grad(fmaf(xv, kc[3 * COUT + c], kc[4 * COUT + c]));
                        o[j] = fmaf(kc[COUT + c], dz, fmaf(kc[2 * COUT + c], xv, kc[c]));
                    }
                    u = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
                }
            }
            *reinterpret_cast<uint4*>(gtT + px * LDY + v * 8) = u;
        }
        __syncthreads();
        }
        for (int ks = wave; ks < TPX / 32; ks += 4) {
            const int px0 = ks * 32 + 8 * lg;                           // this lane's 8 pixels (one output row)
            const int oy = px0 / TOW, ox0 = px0 % TOW;
            bf16x8_t bfr[2];
#pragma unroll
            for (int tb = 0; tb < 2; ++tb) {
                const bf16_t* row = inb + toff[tb] + 2 * oy * IWP + 2 * ox0;
                bf16x8_t f;
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = tval[tb] ? (short)row[2 * j] : (short)0;
                bfr[tb] = f;
            }
#pragma unroll
            for (int cb = 0; cb < 3; ++cb) {
                // MFMA-A = dy^T: lane (lr, lg) needs pixels px0 .. px0+7 of channel cb*16 + lr; the transposing
                // read assembles them from rows px0 + q4 / + 4 + q4 of the [px][co] tile (as gemm.hip's NN operand)
                const int q4 = lr >> 2, p4 = lr & 3;
                const bf16_t* b0 = gtT + (px0 + q4) * LDY + cb * 16 + p4 * 4;
                const bf16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)b0);
                const bf16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(b0 + 4 * LDY));
                const bf16x8_t afr = bf16x8_t{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
                for (int tb = 0; tb < 2; ++tb)
                    acc[cb][tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[tb], acc[cb][tb], 0, 0, 0);
            }
        }
    }
    // acc[cb][tb][i] = dW[co = cb*16 + 4*lg + i][tap = tb*16 + lr]; sum the 4 waves in order via LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(gtT);                         // 4 x 48 x 32 floats (reuses the dy tile)
    static_assert(TPX * LDY * 2 >= 4 * 48 * 32 * 4, "reduction buffer");
#pragma unroll
    for (int cb = 0; cb < 3; ++cb)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                red[(wave * 48 + cb * 16 + 4 * lg + i) * 32 + tb * 16 + lr] = acc[cb][tb][i];
    __syncthreads();
    for (int i = threadIdx.x; i < COUT * 27; i += BLOCK) {
        const int co = i / 27, tap = i % 27;
        float a = 0.f;
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) a += red[(wv * 48 + co) * 32 + tap];
        dwp[(int64_t)blockIdx.x * COUT * 27 + i] = a;
    }
}

// Forward on the matrix cores: out^T[co][px] = W[co][tap] . P^T[tap][px] per 16-pixel block, one 16x16x32 bf16
// MFMA per 16 output channels (taps 27 -> 32, channels 40 -> 48).  W stays in registers as the A operand; the B
// operand (8 taps of one pixel) is gathered from the bf16 input window in LDS; the accumulator holds 4
// consecutive channels of one pixel (8-byte stores).  BN partial sums of the stored bf16 values are reduced
// over the 16 pixel lanes, the 4 waves and the workgroup's tiles in a fixed order.
template <typename TIn>
__global__ __launch_bounds__(BLOCK) void stem_fwd_mfma_kernel(const TIn* __restrict__ img,
                                                              const int* __restrict__ shift,
                                                              const float* __restrict__ w, int N, int H, int W,
                                                              int Ho, int Wo, bf16_t* __restrict__ out,
                                                              float* __restrict__ psum, float* __restrict__ psq, int vec) {
    __shared__ __attribute__((aligned(16))) bf16_t inb[3 * IH * IWP];
    __shared__ float red[4 * 2 * 48 * 16];
    // per wave: the 16-pixel block's 40 channels, contiguous in the channels-last output (1280 B), written back as
    // 16-byte pieces instead of 8-byte pieces of 16 separate pixel rows
    __shared__ __attribute__((aligned(16))) bf16_t ost[4][16 * COUT];
    const int dy = shift ? shift[0] : 0, dx = shift ? shift[1] : 0;
    const int tiles_h = (Ho + TOH - 1) / TOH, tiles_w = (Wo + TOW - 1) / TOW;
    const int64_t ntiles = (int64_t)N * tiles_h * tiles_w;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lg = lane >> 4;
    // A operand: W[co = nb*16 + lr][tap = 8*lg + j] (zero past 40 channels / 27 taps)
    bf16x8_t wa[3];
    int toff[8];
    bool tval[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int tap = 8 * lg + j;
        tval[j] = tap < 27;
        const int ci = tap / 9, kk = tap % 9;
        toff[j] = tval[j] ? (ci * IH + kk / 3) * IWP + kk % 3 : 0;
    }
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) {
        const int co = nb * 16 + lr;
#pragma unroll
        for (int j = 0; j < 8; ++j) wa[nb][j] = (short)((co < COUT && tval[j]) ? f2bf(w[co * 27 + 8 * lg + j]) : 0);
    }
    float s[3][4], q[3][4];
#pragma unroll
    for (int nb = 0; nb < 3; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[nb][i] = q[nb][i] = 0.f;
    // uint8 vector path: the next tile's window loads are issued before this tile's products (WinRegs)
    constexpr bool U8 = sizeof(TIn) == 1;
    const bool pipe = U8 && vec != 0 && STEM_PIPE;
    WinRegs wr;
    if (pipe && (int64_t)blockIdx.x < ntiles) {
        int n1, a1, b1;
        tile_of(blockIdx.x, tiles_h, tiles_w, n1, a1, b1);
        if constexpr (U8) win_load(wr, img, n1, H, W, 2 * a1 - 1, 2 * b1 - 1, dy, dx);
    }
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        int n, oh0, ow0;
        tile_of(t, tiles_h, tiles_w, n, oh0, ow0);
        __syncthreads();
        if (pipe) {
            win_store(inb, wr, W, 2 * ow0 - 1, dx);
            if (t + gridDim.x < ntiles) {
                int n1, a1, b1;
                tile_of(t + gridDim.x, tiles_h, tiles_w, n1, a1, b1);
                if constexpr (U8) win_load(wr, img, n1, H, W, 2 * a1 - 1, 2 * b1 - 1, dy, dx);
            }
        } else {
            stage_window_bf16(inb, img, n, H, W, 2 * oh0 - 1, 2 * ow0 - 1, dy, dx, vec != 0);
        }
        __syncthreads();
        for (int pb = wave; pb < TPX / 16; pb += 4) {
            const int px = pb * 16 + lr;                                // this lane's pixel of the block
            const int oy = px / TOW, ox = px % TOW;
            const bf16_t* base = inb + 2 * oy * IWP + 2 * ox;
            bf16x8_t bfr;
#pragma unroll
            for (int j = 0; j < 8; ++j) bfr[j] = tval[j] ? (short)base[toff[j]] : (short)0;
            const int oh = oh0 + oy, ow = ow0 + ox;
            const bool live = oh < Ho && ow < Wo;
#pragma unroll
            for (int nb = 0; nb < 3; ++nb) {
                f32x4_t acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb], bfr, f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                const int co0 = nb * 16 + 4 * lg;                       // acc[i] = out[pixel][co0 + i]
                if (co0 < COUT) {
                    uint2 u;
                    u.x = pack2(acc[0], acc[1]);
                    u.y = pack2(acc[2], acc[3]);
                    *reinterpret_cast<uint2*>(&ost[wave][lr * COUT + co0]) = u;
                    if (live) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float f = bf2f(f2bf(acc[i]));
                            s[nb][i] += f;
                            q[nb][i] = fmaf(f, f, q[nb][i]);
                        }
                    }
                }
            }
            wave_lds_sync();
            // the block's 16 pixels are consecutive in one output row: 80 16-byte pieces, pixel = piece / 5
            const int ox0 = (pb * 16) % TOW;
            bf16_t* dst = out + (((int64_t)n * Ho + oh) * Wo + ow0 + ox0) * COUT;
            for (int pc = lane; pc < 16 * COUT / 8; pc += 64) {
                if (oh < Ho && ow0 + ox0 + pc / (COUT / 8) < Wo)
                    *reinterpret_cast<uint4*>(dst + pc * 8) = *reinterpret_cast<const uint4*>(&ost[wave][pc * 8]);
            }
            wave_lds_sync();
        }
    }
    // partials: [wave][s|q][channel 48][pixel lane 16] -> fixed-order sums
#pragma unroll
    for (int nb = 0; nb < 3; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = nb * 16 + 4 * lg + i;
            red[((wave * 2 + 0) * 48 + co) * 16 + lr] = s[nb][i];
            red[((wave * 2 + 1) * 48 + co) * 16 + lr] = q[nb][i];
        }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * COUT; c += BLOCK) {
        const int co = c % COUT, sq = c / COUT;
        float a = 0.f;
        for (int wv = 0; wv < 4; ++wv)
            for (int l = 0; l < 16; ++l) a += red[((wv * 2 + sq) * 48 + co) * 16 + l];
        (sq ? psq : psum)[(int64_t)blockIdx.x * COUT + co] = a;
    }
}

}  // namespace

extern "C" {

// the 4-column uint8 window staging: 4-byte aligned frames of a width divisible by 4
static int vec_ok(const void* img, int W) { return ((reinterpret_cast<uintptr_t>(img) & 3) == 0 && W % 4 == 0) ? 1 : 0; }

// workgroups for a frame batch: one per 12x32 output tile, capped
int rt1_stem_grid(int N, int H, int W, int max_blocks) {
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const int64_t tiles = (int64_t)N * ((Ho + TOH - 1) / TOH) * ((Wo + TOW - 1) / TOW);
    const int64_t g = tiles < max_blocks ? tiles : max_blocks;
    return (int)(g < 1 ? 1 : g);
}

int rt1_stem_fwd(const void* img, int img_is_u8, const int* shift, const float* w, int N, int H, int W, int Cout,
                 int grid, bf16_t* out, float* psum, float* psq, hipStream_t st) {
    if (Cout != 40) return (int)hipErrorInvalidValue;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    if (img_is_u8)
        hipLaunchKernelGGL((stem_fwd_mfma_kernel<uint8_t>), dim3(grid), dim3(BLOCK), 0, st, (const uint8_t*)img, shift,
                           w, N, H, W, Ho, Wo, out, psum, psq, vec_ok(img, W));
    else
        hipLaunchKernelGGL((stem_fwd_mfma_kernel<float>), dim3(grid), dim3(BLOCK), 0, st, (const float*)img, shift, w,
                           N, H, W, Ho, Wo, out, psum, psq, 0);
    return (int)hipGetLastError();
}

int rt1_stem_bwd_weight(const void* img, int img_is_u8, const int* shift, const bf16_t* dy, int N, int H, int W,
                        int Cout, int grid, float* dwp, hipStream_t st, const bf16_t* bn_x, const float* bn_scale,
                        const float* bn_shift, const float* bn_mean, const float* bn_rstd, const float* bn_gamma,
                        const float* bn_mdz, const float* bn_mdzx) {
    if (Cout != 40) return (int)hipErrorInvalidValue;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const StemBnBwd bn{bn_x, bn_scale, bn_shift, bn_mean, bn_rstd, bn_gamma, bn_mdz, bn_mdzx};
    if (bn_x) {   // the BN-backward prologue lives in the MFMA kernel only
        if (!bn_scale || !bn_shift || !bn_mean || !bn_rstd || !bn_mdz || !bn_mdzx) return (int)hipErrorInvalidValue;
        if (img_is_u8)
            hipLaunchKernelGGL((stem_wgrad_mfma_kernel<uint8_t, true>), dim3(grid), dim3(BLOCK), 0, st,
                               (const uint8_t*)img, shift, dy, N, H, W, Ho, Wo, dwp, bn, vec_ok(img, W));
        else
            hipLaunchKernelGGL((stem_wgrad_mfma_kernel<float, true>), dim3(grid), dim3(BLOCK), 0, st,
                               (const float*)img, shift, dy, N, H, W, Ho, Wo, dwp, bn, 0);
        return (int)hipGetLastError();
    }
    if (img_is_u8)
        hipLaunchKernelGGL((stem_wgrad_mfma_kernel<uint8_t, false>), dim3(grid), dim3(BLOCK), 0, st, (const uint8_t*)img,
                           shift, dy, N, H, W, Ho, Wo, dwp, bn, vec_ok(img, W));
    else
        hipLaunchKernelGGL((stem_wgrad_mfma_kernel<float, false>), dim3(grid), dim3(BLOCK), 0, st, (const float*)img,
                           shift, dy, N, H, W, Ho, Wo, dwp, bn, 0);
    return (int)hipGetLastError();
}

}  // extern "C"
