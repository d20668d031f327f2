// Depthwise k x k convolution (k in {3,5}, stride in {1,2}, pad (k-1)/2) on
// channels-last bf16 activations, with the surrounding BatchNorm work fused
// (26 depthwise convs of the FiLM-EfficientNet-B3; memory-bound,
// vector ALU, not MFMA work).
//
// forward:   out = dwconv( act(x*scale + shift) )       (prologue optional)
//            + per-workgroup partial (sum, sumsq) of out for the next BN
// bwd data:  dx = dwconv^T(dy)                           (-> grad wrt the activated input)
//            + optional epilogue: dz = dx * silu'(y_in*scale+shift) partials
//              (sum dz, sum dz*xhat) for the producer BN's backward
// bwd weight: dw[c, tap] = sum dy * act(x*scale+shift)   (per-workgroup partials)
//
// Tiling (CDNA4): a 256-thread workgroup owns CV<=8 channel vectors (8 bf16 =
// 16 B each, so one pixel's chunk is a 128-B contiguous line) x a spatial tile.
// The input tile + halo is staged ONCE into LDS with the BN+SiLU prologue
// already applied (so each input element pays one exp, not k*k), then every
// thread computes R consecutive outputs along W for 8 channels from LDS.
// Workgroups loop over tiles (grid = min(tiles, ~8/CU)) so the BN partial rows
// stay few (one per workgroup) and are reduced by bn_finalize.
#include "common.h"

using namespace rt1;

namespace {

constexpr int BLOCK = 256;

struct DwGeo {
    int N, H, W, C, Ho, Wo, k, s, pad;
    int nv;      // C / 8
    int cv;      // channel vectors per workgroup chunk
    int chunks;  // ceil(nv / cv)
};

// ------------------------------------------------------------------ forward
template <int K, int S, int R>
__global__ __launch_bounds__(BLOCK) void dw_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int act, DwGeo g, int TH,
                                                       int TW, bf16_t* __restrict__ out, float* __restrict__ psum,
                                                       float* __restrict__ psq) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int IH = (TH - 1) * S + K, IW = (TW - 1) * S + K;
    const int cv = g.cv;
    // LDS: input tile [IH*IW][cv] x uint4 (8 bf16), weights [K*K][cv*8] f32, reduce scratch
    uint4* tile = reinterpret_cast<uint4*>(smem);
    float* wl = reinterpret_cast<float*>(smem + (size_t)IH * IW * cv * 16);
    float* red = reinterpret_cast<float*>(smem);  // aliases the tile after the last tile is consumed

    const int chunk = blockIdx.y;
    const int v0 = chunk * cv;                       // first channel vector of this chunk
    const int ncv = min(cv, g.nv - v0);              // vectors valid in this chunk
    const int t = threadIdx.x;
    const int lane_cv = t % cv;
    const int pl = t / cv;                           // pixel lane
    const int PL = BLOCK / cv;
    const int groups_w = TW / R;
    const int ngroups = TH * groups_w;

    // stage weights (f32, [tap][c]) once per workgroup
    for (int i = t; i < K * K * cv * 8; i += BLOCK) {
        const int tap = i / (cv * 8), cc = i % (cv * 8);
        const int c = v0 * 8 + cc;
        wl[i] = (cc < ncv * 8) ? w[(int64_t)c * K * K + tap] : 0.f;
    }

    const int tiles_h = (g.Ho + TH - 1) / TH, tiles_w = (g.Wo + TW - 1) / TW;
    const int64_t ntiles = (int64_t)g.N * tiles_h * tiles_w;

    float s_acc[8], q_acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s_acc[j] = q_acc[j] = 0.f;

    for (int64_t tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
        const int n = (int)(tile_id / (tiles_h * tiles_w));
        const int rem = (int)(tile_id - (int64_t)n * tiles_h * tiles_w);
        const int oh0 = (rem / tiles_w) * TH, ow0 = (rem % tiles_w) * TW;
        const int ih0 = oh0 * S - g.pad, iw0 = ow0 * S - g.pad;
        __syncthreads();  // previous tile fully consumed (and weights staged on the first pass)
        // ---- stage input tile with prologue
        for (int i = t; i < IH * IW * cv; i += BLOCK) {
            const int p = i / cv, vv = i % cv;
            const int ih = ih0 + p / IW, iw = iw0 + p % IW;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (vv < ncv && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) {
                const int c0 = (v0 + vv) * 8;
                const bf16_t* src = x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c0;
                if (scale) {
                    float f[8], sc[8], sh[8];
                    load8(src, f);
                    load8f(scale + c0, sc);
                    load8f(shift + c0, sh);
#pragma unroll
                    for (int j = 0; j < 8; ++j) f[j] = act_fwd(fmaf(f[j], sc[j], sh[j]), act);
                    u.x = pack2(f[0], f[1]); u.y = pack2(f[2], f[3]); u.z = pack2(f[4], f[5]); u.w = pack2(f[6], f[7]);
                } else {
                    u = *reinterpret_cast<const uint4*>(src);
                }
            }
            tile[i] = u;
        }
        __syncthreads();
        // ---- compute R outputs along W per group
        if (lane_cv < ncv) {
            for (int grp = pl; grp < ngroups; grp += PL) {
                const int ty = grp / groups_w, tx = (grp % groups_w) * R;
                const int oh = oh0 + ty;
                if (oh >= g.Ho) continue;
                float acc[R][8];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[r][j] = 0.f;
#pragma unroll 1
                for (int kh = 0; kh < K; ++kh) {
                    const int row = ty * S + kh;
                    constexpr int NIN = (R - 1) * S + K;
                    float wrow[K][8];
#pragma unroll
                    for (int kw = 0; kw < K; ++kw) load8f(wl + (kh * K + kw) * cv * 8 + lane_cv * 8, wrow[kw]);
                    // stream the NIN input vectors of this row; each feeds every (r, kw) with r*S + kw == q
#pragma unroll
                    for (int q = 0; q < NIN; ++q) {
                        const uint4 u = tile[(row * IW + tx * S + q) * cv + lane_cv];
                        float in[8];
                        in[0] = __uint_as_float(u.x << 16); in[1] = __uint_as_float(u.x & 0xffff0000u);
                        in[2] = __uint_as_float(u.y << 16); in[3] = __uint_as_float(u.y & 0xffff0000u);
                        in[4] = __uint_as_float(u.z << 16); in[5] = __uint_as_float(u.z & 0xffff0000u);
                        in[6] = __uint_as_float(u.w << 16); in[7] = __uint_as_float(u.w & 0xffff0000u);
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const int kw = q - r * S;
                            if (kw >= 0 && kw < K) {
#pragma unroll
                                for (int j = 0; j < 8; ++j) acc[r][j] = fmaf(in[j], wrow[kw][j], acc[r][j]);
                            }
                        }
                    }
                }
                const int c0 = (v0 + lane_cv) * 8;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int ow = ow0 + tx + r;
                    if (ow < g.Wo) {
                        // round to bf16 first so the statistics describe the stored tensor
                        float o[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            o[j] = bf2f(f2bf(acc[r][j]));
                            s_acc[j] += o[j];
                            q_acc[j] = fmaf(o[j], o[j], q_acc[j]);
                        }
                        store8(out + (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c0, o);
                    }
                }
            }
        }
    }
    // ---- per-workgroup channel partials
    if (psum) {
        __syncthreads();
        const int C8 = cv * 8;
        for (int i = t; i < PL * C8 * 2; i += BLOCK) red[i] = 0.f;
        __syncthreads();
        if (pl < PL) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                red[pl * C8 + lane_cv * 8 + j] = s_acc[j];
                red[PL * C8 + pl * C8 + lane_cv * 8 + j] = q_acc[j];
            }
        }
        __syncthreads();
        for (int cc = t; cc < ncv * 8; cc += BLOCK) {
            float a = 0.f, b = 0.f;
            for (int p = 0; p < PL; ++p) {
                a += red[p * C8 + cc];
                b += red[PL * C8 + p * C8 + cc];
            }
            psum[(int64_t)blockIdx.x * g.C + v0 * 8 + cc] = a;
            psq[(int64_t)blockIdx.x * g.C + v0 * 8 + cc] = b;
        }
    }
}

// ------------------------------------------------------------------ backward data
// dx[n, ih, iw, c] = sum_{kh,kw: (ih+pad-kh)%S==0, ...} w[c,kh,kw] * dy[n, (ih+pad-kh)/S, (iw+pad-kw)/S, c]
// epilogue (optional, y_in != nullptr): dz = dx * silu'(y_in*scale+shift);  partials of dz and dz*xhat
template <int K, int S>
__global__ __launch_bounds__(BLOCK) void dw_bwd_data_kernel(const bf16_t* __restrict__ dy, const float* __restrict__ w,
                                                            DwGeo g, int TH, int TW, bf16_t* __restrict__ dx,
                                                            const bf16_t* __restrict__ y_in,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            float* __restrict__ pdz, float* __restrict__ pdzx) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // dy rows needed for input rows [ih0, ih0+TH): ho in [ceil((ih0+pad-K+1)/S), floor((ih0+TH-1+pad)/S)]
    const int DH = (TH - 1 + K - 1) / S + 2, DW = (TW - 1 + K - 1) / S + 2;
    const int cv = g.cv;
    uint4* tile = reinterpret_cast<uint4*>(smem);
    float* wl = reinterpret_cast<float*>(smem + (size_t)DH * DW * cv * 16);
    float* red = reinterpret_cast<float*>(smem);  // aliases the tile after the last tile is consumed

    const int chunk = blockIdx.y;
    const int v0 = chunk * cv;
    const int ncv = min(cv, g.nv - v0);
    const int t = threadIdx.x;
    const int lane_cv = t % cv;
    const int pl = t / cv;
    const int PL = BLOCK / cv;

    for (int i = t; i < K * K * cv * 8; i += BLOCK) {
        const int tap = i / (cv * 8), cc = i % (cv * 8);
        wl[i] = (cc < ncv * 8) ? w[(int64_t)(v0 * 8 + cc) * K * K + tap] : 0.f;
    }
    const int tiles_h = (g.H + TH - 1) / TH, tiles_w = (g.W + TW - 1) / TW;
    const int64_t ntiles = (int64_t)g.N * tiles_h * tiles_w;
    float s_acc[8], q_acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s_acc[j] = q_acc[j] = 0.f;

    for (int64_t tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
        const int n = (int)(tile_id / (tiles_h * tiles_w));
        const int rem = (int)(tile_id - (int64_t)n * tiles_h * tiles_w);
        const int ih0 = (rem / tiles_w) * TH, iw0 = (rem % tiles_w) * TW;
        // first dy row/col that can touch this tile (floor division of possibly negative numbers)
        const int a_h = ih0 + g.pad - (K - 1), a_w = iw0 + g.pad - (K - 1);
        const int oh_lo = a_h >= 0 ? (a_h + S - 1) / S : -((-a_h) / S);
        const int ow_lo = a_w >= 0 ? (a_w + S - 1) / S : -((-a_w) / S);
        __syncthreads();
        for (int i = t; i < DH * DW * cv; i += BLOCK) {
            const int p = i / cv, vv = i % cv;
            const int oh = oh_lo + p / DW, ow = ow_lo + p % DW;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (vv < ncv && oh >= 0 && oh < g.Ho && ow >= 0 && ow < g.Wo)
                u = *reinterpret_cast<const uint4*>(dy + (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + (v0 + vv) * 8);
            tile[i] = u;
        }
        __syncthreads();
        if (lane_cv < ncv) {
            for (int pix = pl; pix < TH * TW; pix += PL) {
                const int ih = ih0 + pix / TW, iw = iw0 + pix % TW;
                if (ih >= g.H || iw >= g.W) continue;
                float acc[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
                for (int kh = 0; kh < K; ++kh) {
                    const int nh = ih + g.pad - kh;
                    if (nh < 0 || (S == 2 && (nh & 1))) continue;
                    const int oh = nh / S;
                    if (oh >= g.Ho) continue;
#pragma unroll
                    for (int kw = 0; kw < K; ++kw) {
                        const int nw = iw + g.pad - kw;
                        if (nw < 0 || (S == 2 && (nw & 1))) continue;
                        const int ow = nw / S;
                        if (ow >= g.Wo) continue;
                        const uint4 u = tile[((oh - oh_lo) * DW + (ow - ow_lo)) * cv + lane_cv];
                        float wv[8];
                        load8f(wl + (kh * K + kw) * cv * 8 + lane_cv * 8, wv);
                        acc[0] = fmaf(__uint_as_float(u.x << 16), wv[0], acc[0]);
                        acc[1] = fmaf(__uint_as_float(u.x & 0xffff0000u), wv[1], acc[1]);
                        acc[2] = fmaf(__uint_as_float(u.y << 16), wv[2], acc[2]);
                        acc[3] = fmaf(__uint_as_float(u.y & 0xffff0000u), wv[3], acc[3]);
                        acc[4] = fmaf(__uint_as_float(u.z << 16), wv[4], acc[4]);
                        acc[5] = fmaf(__uint_as_float(u.z & 0xffff0000u), wv[5], acc[5]);
                        acc[6] = fmaf(__uint_as_float(u.w << 16), wv[6], acc[6]);
                        acc[7] = fmaf(__uint_as_float(u.w & 0xffff0000u), wv[7], acc[7]);
                    }
                }
                const int c0 = (v0 + lane_cv) * 8;
                const int64_t off = (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c0;
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(acc[j]));
                store8(dx + off, o);
                if (y_in) {
                    float yv[8], sc[8], sh[8], mu[8], rr[8];
                    load8(y_in + off, yv);
                    load8f(scale + c0, sc);
                    load8f(shift + c0, sh);
                    load8f(mean + c0, mu);
                    load8f(rstd + c0, rr);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float dz = o[j] * silu_grad(fmaf(yv[j], sc[j], sh[j]));
                        s_acc[j] += dz;
                        q_acc[j] = fmaf(dz, (yv[j] - mu[j]) * rr[j], q_acc[j]);
                    }
                }
            }
        }
    }
    if (pdz) {
        __syncthreads();
        const int C8 = cv * 8;
        for (int i = t; i < PL * C8 * 2; i += BLOCK) red[i] = 0.f;
        __syncthreads();
        if (pl < PL) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                red[pl * C8 + lane_cv * 8 + j] = s_acc[j];
                red[PL * C8 + pl * C8 + lane_cv * 8 + j] = q_acc[j];
            }
        }
        __syncthreads();
        for (int cc = t; cc < ncv * 8; cc += BLOCK) {
            float a = 0.f, b = 0.f;
            for (int p = 0; p < PL; ++p) {
                a += red[p * C8 + cc];
                b += red[PL * C8 + p * C8 + cc];
            }
            pdz[(int64_t)blockIdx.x * g.C + v0 * 8 + cc] = a;
            pdzx[(int64_t)blockIdx.x * g.C + v0 * 8 + cc] = b;
        }
    }
}

// ------------------------------------------------------------------ backward weight
// Threads are laid out as (channel vector, kernel row kh, pixel lane); each
// keeps K x 8 accumulators (one kernel row for 8 channels) over all output
// pixels of all tiles it visits.  Partials: dwp[blockIdx.x][c][tap].
template <int K, int S>
__global__ __launch_bounds__(BLOCK) void dw_bwd_weight_kernel(const bf16_t* __restrict__ dy,
                                                              const bf16_t* __restrict__ x,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, int act, DwGeo g,
                                                              int TH, int TW, float* __restrict__ dwp) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int IH = (TH - 1) * S + K, IW = (TW - 1) * S + K;
    const int cv = g.cv;
    uint4* xt = reinterpret_cast<uint4*>(smem);
    uint4* dt = xt + IH * IW * cv;
    float* red = reinterpret_cast<float*>(smem);  // aliases the tiles after the last tile is consumed

    const int chunk = blockIdx.y;
    const int v0 = chunk * cv;
    const int ncv = min(cv, g.nv - v0);
    const int t = threadIdx.x;
    const int per = cv * K;                  // threads per pixel lane
    const int lane_cv = t % cv;
    const int kh = (t / cv) % K;
    const int pl = t / per;
    const int PL = BLOCK / per;

    const int tiles_h = (g.Ho + TH - 1) / TH, tiles_w = (g.Wo + TW - 1) / TW;
    const int64_t ntiles = (int64_t)g.N * tiles_h * tiles_w;
    float acc[K][8];
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;

    for (int64_t tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
        const int n = (int)(tile_id / (tiles_h * tiles_w));
        const int rem = (int)(tile_id - (int64_t)n * tiles_h * tiles_w);
        const int oh0 = (rem / tiles_w) * TH, ow0 = (rem % tiles_w) * TW;
        const int ih0 = oh0 * S - g.pad, iw0 = ow0 * S - g.pad;
        __syncthreads();
        for (int i = t; i < IH * IW * cv; i += BLOCK) {
            const int p = i / cv, vv = i % cv;
            const int ih = ih0 + p / IW, iw = iw0 + p % IW;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (vv < ncv && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) {
                const int c0 = (v0 + vv) * 8;
                const bf16_t* src = x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c0;
                if (scale) {
                    float f[8], sc[8], sh[8];
                    load8(src, f);
                    load8f(scale + c0, sc);
                    load8f(shift + c0, sh);
#pragma unroll
                    for (int j = 0; j < 8; ++j) f[j] = act_fwd(fmaf(f[j], sc[j], sh[j]), act);
                    u.x = pack2(f[0], f[1]); u.y = pack2(f[2], f[3]); u.z = pack2(f[4], f[5]); u.w = pack2(f[6], f[7]);
                } else {
                    u = *reinterpret_cast<const uint4*>(src);
                }
            }
            xt[i] = u;
        }
        for (int i = t; i < TH * TW * cv; i += BLOCK) {
            const int p = i / cv, vv = i % cv;
            const int oh = oh0 + p / TW, ow = ow0 + p % TW;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (vv < ncv && oh < g.Ho && ow < g.Wo)
                u = *reinterpret_cast<const uint4*>(dy + (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + (v0 + vv) * 8);
            dt[i] = u;
        }
        __syncthreads();
        if (pl < PL && lane_cv < ncv) {
            for (int pix = pl; pix < TH * TW; pix += PL) {
                const int ty = pix / TW, tx = pix % TW;
                const uint4 du = dt[pix * cv + lane_cv];
                float d[8];
                d[0] = __uint_as_float(du.x << 16); d[1] = __uint_as_float(du.x & 0xffff0000u);
                d[2] = __uint_as_float(du.y << 16); d[3] = __uint_as_float(du.y & 0xffff0000u);
                d[4] = __uint_as_float(du.z << 16); d[5] = __uint_as_float(du.z & 0xffff0000u);
                d[6] = __uint_as_float(du.w << 16); d[7] = __uint_as_float(du.w & 0xffff0000u);
                const int row = ty * S + kh;
#pragma unroll
                for (int kw = 0; kw < K; ++kw) {
                    const uint4 u = xt[(row * IW + tx * S + kw) * cv + lane_cv];
                    acc[kw][0] = fmaf(d[0], __uint_as_float(u.x << 16), acc[kw][0]);
                    acc[kw][1] = fmaf(d[1], __uint_as_float(u.x & 0xffff0000u), acc[kw][1]);
                    acc[kw][2] = fmaf(d[2], __uint_as_float(u.y << 16), acc[kw][2]);
                    acc[kw][3] = fmaf(d[3], __uint_as_float(u.y & 0xffff0000u), acc[kw][3]);
                    acc[kw][4] = fmaf(d[4], __uint_as_float(u.z << 16), acc[kw][4]);
                    acc[kw][5] = fmaf(d[5], __uint_as_float(u.z & 0xffff0000u), acc[kw][5]);
                    acc[kw][6] = fmaf(d[6], __uint_as_float(u.w << 16), acc[kw][6]);
                    acc[kw][7] = fmaf(d[7], __uint_as_float(u.w & 0xffff0000u), acc[kw][7]);
                }
            }
        }
    }
    // reduce over pixel lanes: red[pl][c][tap]
    __syncthreads();
    const int C8 = cv * 8;
    const int KK = K * K;
    for (int i = t; i < PL * C8 * KK; i += BLOCK) red[i] = 0.f;
    __syncthreads();
    if (pl < PL && lane_cv < ncv) {
#pragma unroll
        for (int kw = 0; kw < K; ++kw)
#pragma unroll
            for (int j = 0; j < 8; ++j) red[(pl * C8 + lane_cv * 8 + j) * KK + kh * K + kw] = acc[kw][j];
    }
    __syncthreads();
    for (int i = t; i < ncv * 8 * KK; i += BLOCK) {
        float a = 0.f;
        for (int p = 0; p < PL; ++p) a += red[p * C8 * KK + i];
        dwp[(int64_t)blockIdx.x * g.C * KK + (int64_t)v0 * 8 * KK + i] = a;
    }
}

// sum partial rows: out[j] (+)= sum_p part[p][j]
__global__ __launch_bounds__(256) void sum_rows_kernel(const float* __restrict__ part, int P, int L,
                                                       float* __restrict__ out, int accumulate) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= L) return;
    float a = 0.f;
    for (int p = 0; p < P; ++p) a += part[(int64_t)p * L + j];
    out[j] = accumulate ? out[j] + a : a;
}

DwGeo make_geo(int N, int H, int W, int C, int k, int s) {
    DwGeo g;
    g.N = N; g.H = H; g.W = W; g.C = C; g.k = k; g.s = s; g.pad = (k - 1) / 2;
    g.Ho = (H + 2 * g.pad - k) / s + 1;
    g.Wo = (W + 2 * g.pad - k) / s + 1;
    g.nv = C / 8;
    g.cv = g.nv < 8 ? g.nv : 8;
    g.chunks = (g.nv + g.cv - 1) / g.cv;
    return g;
}

}  // namespace

extern "C" {

// tile geometry shared by launcher and the host-side partial-buffer sizing
void rt1_dw_tiles(int k, int s, int cv, int* TH, int* TW, int* R) {
    (void)k;
    const int rm = cv >= 8 ? 1 : (8 / cv);
    if (s == 1) { *TH = 8 * rm; *TW = 16; *R = 4; }
    else { *TH = 4 * rm; *TW = 16; *R = 2; }
}

int rt1_dw_grid(int N, int H, int W, int C, int k, int s, int max_blocks_x) {
    DwGeo g = make_geo(N, H, W, C, k, s);
    int TH, TW, R;
    rt1_dw_tiles(k, s, g.cv, &TH, &TW, &R);
    const int64_t tiles = (int64_t)N * ((g.Ho + TH - 1) / TH) * ((g.Wo + TW - 1) / TW);
    int64_t gx = tiles < max_blocks_x ? tiles : max_blocks_x;
    return (int)(gx < 1 ? 1 : gx);
}

int rt1_dw_fwd(const bf16_t* x, const float* w, const float* scale, const float* shift, int act, int N, int H, int W,
               int C, int k, int s, int grid_x, bf16_t* out, float* psum, float* psq, hipStream_t st) {
    DwGeo g = make_geo(N, H, W, C, k, s);
    int TH, TW, R;
    rt1_dw_tiles(k, s, g.cv, &TH, &TW, &R);
    const int IH = (TH - 1) * s + k, IW = (TW - 1) * s + k;
    const int PL = BLOCK / g.cv;
    size_t lds = (size_t)IH * IW * g.cv * 16 + (size_t)k * k * g.cv * 8 * 4;
    const size_t red = (size_t)PL * g.cv * 8 * 2 * 4;
    lds = lds > red ? lds : red;
    dim3 grid(grid_x, g.chunks);
#define L(KK, SS, RR)                                                                                           \
    hipLaunchKernelGGL((dw_fwd_kernel<KK, SS, RR>), grid, dim3(BLOCK), lds, st, x, w, scale, shift, act, g, TH, \
                       TW, out, psum, psq)
    if (k == 3 && s == 1) L(3, 1, 4);
    else if (k == 3 && s == 2) L(3, 2, 2);
    else if (k == 5 && s == 1) L(5, 1, 4);
    else if (k == 5 && s == 2) L(5, 2, 2);
    else return (int)hipErrorInvalidValue;
#undef L
    return (int)hipGetLastError();
}

int rt1_dw_bwd_data(const bf16_t* dy, const float* w, int N, int H, int W, int C, int k, int s, int grid_x, bf16_t* dx,
                    const bf16_t* y_in, const float* scale, const float* shift, const float* mean, const float* rstd,
                    float* pdz, float* pdzx, hipStream_t st) {
    DwGeo g = make_geo(N, H, W, C, k, s);
    const int TH = 8 * (g.cv >= 8 ? 1 : 8 / g.cv), TW = 16;
    const int DH = (TH - 1 + k - 1) / s + 2, DW = (TW - 1 + k - 1) / s + 2;
    const int PL = BLOCK / g.cv;
    size_t lds = (size_t)DH * DW * g.cv * 16 + (size_t)k * k * g.cv * 8 * 4;
    const size_t red = (size_t)PL * g.cv * 8 * 2 * 4;
    lds = lds > red ? lds : red;
    dim3 grid(grid_x, g.chunks);
#define L(KK, SS)                                                                                                  \
    hipLaunchKernelGGL((dw_bwd_data_kernel<KK, SS>), grid, dim3(BLOCK), lds, st, dy, w, g, TH, TW, dx, y_in, scale, \
                       shift, mean, rstd, pdz, pdzx)
    if (k == 3 && s == 1) L(3, 1);
    else if (k == 3 && s == 2) L(3, 2);
    else if (k == 5 && s == 1) L(5, 1);
    else if (k == 5 && s == 2) L(5, 2);
    else return (int)hipErrorInvalidValue;
#undef L
    return (int)hipGetLastError();
}

int rt1_dw_bwd_grid(int N, int H, int W, int C, int k, int s, int max_blocks_x) {
    DwGeo g = make_geo(N, H, W, C, k, s);
    const int TH = 8 * (g.cv >= 8 ? 1 : 8 / g.cv), TW = 16;
    const int64_t tiles = (int64_t)N * ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
    int64_t gx = tiles < max_blocks_x ? tiles : max_blocks_x;
    return (int)(gx < 1 ? 1 : gx);
}

int rt1_dw_bwd_weight(const bf16_t* dy, const bf16_t* x, const float* scale, const float* shift, int act, int N, int H,
                      int W, int C, int k, int s, int grid_x, float* dwp, hipStream_t st) {
    DwGeo g = make_geo(N, H, W, C, k, s);
    int TH, TW, R;
    rt1_dw_tiles(k, s, g.cv, &TH, &TW, &R);
    const int IH = (TH - 1) * s + k, IW = (TW - 1) * s + k;
    const int PL = BLOCK / (g.cv * k);
    size_t lds = (size_t)IH * IW * g.cv * 16 + (size_t)TH * TW * g.cv * 16;
    const size_t red = (size_t)PL * g.cv * 8 * k * k * 4;
    lds = lds > red ? lds : red;
    dim3 grid(grid_x, g.chunks);
#define L(KK, SS)                                                                                                  \
    hipLaunchKernelGGL((dw_bwd_weight_kernel<KK, SS>), grid, dim3(BLOCK), lds, st, dy, x, scale, shift, act, g, TH, \
                       TW, dwp)
    if (k == 3 && s == 1) L(3, 1);
    else if (k == 3 && s == 2) L(3, 2);
    else if (k == 5 && s == 1) L(5, 1);
    else if (k == 5 && s == 2) L(5, 2);
    else return (int)hipErrorInvalidValue;
#undef L
    return (int)hipGetLastError();
}

int rt1_sum_rows(const float* part, int P, int L, float* out, int accumulate, hipStream_t st) {
    hipLaunchKernelGGL(sum_rows_kernel, dim3((L + 255) / 256), dim3(256), 0, st, part, P, L, out, accumulate);
    return (int)hipGetLastError();
}

}  // extern "C"
