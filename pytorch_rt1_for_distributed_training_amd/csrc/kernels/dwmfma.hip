// Depthwise k x k stride-1 convolution on MFMA (low-resolution layers: maps up to 40 x 40).
//
//     out[n, h, w, c] = sum_{kh, kw} W[c, kh, kw] * act(x[n, h + kh - P, w + kw - P, c])
//     act = identity | silu(x * scale[c] + shift[c]) (BN1 + SiLU of the expand conv, applied while staging)
//     STATS: per-workgroup partial sum / sum of squares of the STORED bf16 out (BN2's batch statistics)
//
// STATUS: opt-in (RT1_DW_MFMA=1; ext.dw_fwd_mfma always): measured slower than the vector-ALU forward of dwconv.hip on
// every layer it covers (profiles/r3_dw_mfma_ab.md).  Kept as the tested MFMA formulation of the depthwise taps.
//
// Why MFMA for a depthwise conv (film_efficientnet_encoder.py:198-208).  A depthwise conv has no
// contraction over channels, so the vector-ALU kernels in dwconv.hip spend ~25 packed FMAs per output element on a
// k5 layer plus the bf16 unpacks of every tap: the 19x19 / 10x10 k5 layers ran at 1.7-2.0 TB/s, issue bound
// (profiles/r2_dw_kbench.log).  Per channel, though, the conv over a 4 x 4 output patch is a matrix product: its 8 x 8
// input window (k5; 6 x 6 of it for k3), flattened to 64 = (window row, window column), times a 16 x 64 Toeplitz
// matrix T_c[(dh, dw)][(r, u)] = W[c, r - dh, u - dw] (zero off the kernel support).  So with the PATCHES as the
// MFMA's N dimension,
//
//     D[16 outputs of a patch][16 patches] = T_c[16][64] . B_c[64][16 patches]        (2 x mfma_f32_16x16x32_bf16)
//
// T_c is built once per channel per workgroup and stays in registers (it is the same for every patch of every frame
// the workgroup visits); 20 % of the MFMA's MACs are useful for k5 (25 of 128 per output), but the matrix cores
// have ~16x the vector FMA rate, so the taps cost ~1/3 of a k5 vector FMA loop and take no VALU issue slots.  What
// remains on the VALU is the staging prologue (BN + SiLU, once per input element) and the data movement.
//
// Layout and work split.  A 512-thread workgroup owns a 64-channel chunk (every pixel's 128-byte line) and walks
// units (frame, band of BPH patch rows) of its frame slot.  Per unit the band's input window is staged into a
// CHANNEL-MAJOR LDS image [64][4 BPH + 4][4 Wp + 4] (window (r, u) of patch (ph, pw) at row 4 ph + r, column 4 pw + u):
// 8 consecutive threads load one pixel pair's 2 x 128 B (fully coalesced), apply the prologue and write per-channel
// pixel pairs.  The loads of the NEXT unit are issued right after, so they fly while this unit multiplies out.  Only
// in-frame pixels (and the partial pairs at the edges) are written per unit, so the zero halo is cleared once (a
// frame cut into several bands re-zeroes its out-of-frame rows).  Wave w takes the chunk's 8-channel vector w: a
// lane's B fragment (8 window columns of one window row) is two aligned 8-byte LDS reads, and the accumulator of lane l
// holds outputs (row l/16, columns 0..3) of patch l%16.  Those are rounded to bf16 and written back into the SAME
// image at their own pixels' positions (the interior, which the wave's MFMAs have consumed and the next staging
// rewrites; the halo stays zero), and the workgroup then reads the interior back channels-last (8 threads per pixel,
// 16-byte coalesced stores) with the BN statistics of the stored values.
#include "common.h"

using namespace rt1;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int BLOCK = 512, CC = 64;

struct MGeo {
    int N, H, W, C;
    int Hp, Wp;        // 4 x 4 output patches per frame
    int BPH, nb;       // patch rows per band, bands per frame
    int IC, IRB;       // image columns (4 Wp + 4) and rows (4 BPH + 4)
    int IMG;           // elements per channel image
    int jlo, jhi;      // pixel pairs (image columns 2j, 2j+1) holding in-frame pixels
    int chunks, FS;    // 64-channel chunks, frame slots (partial-statistics rows)
};

__device__ __forceinline__ short bfs(float f) { return (short)f2bf(f); }

// silu(x * sc + sh) of a pixel pair of one channel in packed f32 math, times the pair's in-frame mask (the conv pads
// act(x) with zeros)
__device__ __forceinline__ f2 silu_pair(f2 x, float sc, float sh, f2 mask) {
    const f2 z = x * f2{sc, sc} + f2{sh, sh};
    const f2 nz = z * f2{-1.4426950408889634f, -1.4426950408889634f};
    const f2 den = f2{__builtin_amdgcn_exp2f(nz.x), __builtin_amdgcn_exp2f(nz.y)} + f2{1.f, 1.f};
    return z * f2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)} * mask;
}

// MAXG: groups of 16 patches per unit; MAXR: staging items per thread per unit (host-checked bounds); D: units whose
// loads are in flight (a ring of register sets: HBM latency under load is several microseconds, one unit ahead
// left the kernel latency bound at ~1.5 TB/s)
template <int K, int MAXG, int MAXR, int D>
__global__ __launch_bounds__(BLOCK, 1) void dw_fwd_mfma_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, MGeo g,
                                                               bf16_t* __restrict__ out, float* __restrict__ psum,
                                                               float* __restrict__ psq) {
    constexpr int KK = K * K, P = (K - 1) / 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* im = reinterpret_cast<bf16_t*>(smem);                   // [64][IMG]
    float* scl = reinterpret_cast<float*>(im + CC * g.IMG);         // [2][64] prologue constants
    float* red = scl + 2 * CC;                                      // [8 waves][8 vectors][16] statistics
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int fs = blockIdx.x, chunk = blockIdx.y;
    const int c0 = chunk * CC, ncv = min(8, g.C / 8 - chunk * 8);
    const bool silu_pro = scale != nullptr, stats = psum != nullptr;

    // weights of the chunk through LDS (aliasing the image, cleared below), then the Toeplitz fragments of wave wv's
    // vector: lane (m = l%16 -> output (dh, dw) = (m/4, m%4), kg = l/16) holds T[m][32 s + 8 kg + e] = W[4 s + kg - dh][e - dw]
    float* wl = reinterpret_cast<float*>(im);
    for (int i = t; i < CC * KK; i += BLOCK) wl[i] = (i / KK < ncv * 8) ? w[(int64_t)c0 * KK + i] : 0.f;
    for (int i = t; i < 2 * CC; i += BLOCK) {
        const int c = i & (CC - 1);
        scl[i] = (silu_pro && c < ncv * 8) ? (i < CC ? scale : shift)[c0 + c] : 0.f;
    }
    __syncthreads();
    const int m = lane & 15, kg = lane >> 4, dh = m >> 2, dw = m & 3;
    bf16x8 afr[8][2];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int r = 4 * s + kg - dh;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int u = e - dw;
                const bool ok = r >= 0 && r < K && u >= 0 && u < K;
                afr[j][s][e] = bfs(ok ? wl[(wv * 8 + j) * KK + (ok ? r * K + u : 0)] : 0.f);
            }
        }
    __syncthreads();
    for (int i = t; i < CC * g.IMG / 2; i += BLOCK) reinterpret_cast<uint32_t*>(im)[i] = 0u;   // zero halo

    // ---- per-thread geometry (divisions once; the loops step it incrementally)
    // staging item it = t + 512 i: vector sv = t % 8 (fixed), pixel pair pr = t / 8 + 64 i -> row rlo + pr / NJ,
    // pair jlo + pr % NJ
    const int NJ = g.jhi - g.jlo;
    const int rlo = g.nb == 1 ? P : 0;                              // one band per frame never dirties the halo rows
    const int npairs = (g.nb == 1 ? 4 * g.Hp : g.IRB) * NJ;
    const int sv = t & 7, pr0 = t >> 3;
    const int sd_r = 64 / NJ, sd_j = 64 - sd_r * NJ;
    const int s_r0 = pr0 / NJ, s_j0 = pr0 - s_r0 * NJ;
    const bool sv_ok = sv < ncv;
    float sc[8], sh[8];
    load8f(scl + sv * 8, sc);
    load8f(scl + CC + sv * 8, sh);
    // taps: patch pidx = 16 gi + m of the band -> (ph, pw)
    const int gd_r = 16 / g.Wp, gd_c = 16 - gd_r * g.Wp;
    const int m_r = m / g.Wp, m_c = m - m_r * g.Wp;
    // read-back: pixel px = t / 8 + 64 i of the band's output rows -> (row, column)
    const int rd_r = 64 / g.W, rd_c = 64 - rd_r * g.W;
    const int b_r0 = pr0 / g.W, b_c0 = pr0 - b_r0 * g.W;

    f2 s_acc[4], q_acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s_acc[j] = q_acc[j] = f2{0.f, 0.f};
    const int units = g.N * g.nb;
    auto issue = [&](int un, uint4 (&pf)[MAXR][2]) {
        const int n = un / g.nb, band = un - n * g.nb;
        const int h0 = 4 * band * g.BPH - P + rlo;                  // input row of staged row rlo
        const bf16_t* xf = x + (int64_t)n * g.H * g.W * g.C + c0 + sv * 8;
        int rr = s_r0, jj = s_j0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
            const int h = h0 + rr, wq = 2 * (g.jlo + jj) - P;
            const bool hok = sv_ok && pr0 + 64 * i < npairs && (unsigned)h < (unsigned)g.H;
            const bool ok0 = hok && (unsigned)wq < (unsigned)g.W, ok1 = hok && (unsigned)(wq + 1) < (unsigned)g.W;
            const bf16_t* src = xf + ((int64_t)h * g.W + wq) * g.C;
            pf[i][0] = ok0 ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
            pf[i][1] = ok1 ? *reinterpret_cast<const uint4*>(src + g.C) : make_uint4(0, 0, 0, 0);
            rr += sd_r; jj += sd_j;
            if (jj >= NJ) { jj -= NJ; ++rr; }
        }
    };
    auto body = [&](int un, uint4 (&pf)[MAXR][2]) {
        const int n = un / g.nb, band = un - n * g.nb;
        const int ph0 = band * g.BPH, nph = min(g.BPH, g.Hp - ph0);
        const int h0 = 4 * ph0 - P + rlo;
        const int orows = min(4 * nph, g.H - 4 * ph0);
        __syncthreads();   // the previous unit's read-back is done (and, first time, the halo is cleared)
        // ---- stage: prologue + transposed pair writes (8 per-channel 32-bit words per item)
        {
            int rr = s_r0, jj = s_j0;
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {
#ifdef RT1_DWM_T_NOSTAGE   // timing-only build: the loads are consumed, no prologue / transposed writes
                if (pr0 + 64 * i < npairs)
                    reinterpret_cast<uint32_t*>(im)[t] = pf[i][0].x ^ pf[i][1].y;
                if (false) {
#else
                if (pr0 + 64 * i < npairs) {
#endif
                    const int h = h0 + rr, wq = 2 * (g.jlo + jj) - P;
                    const bool hok = (unsigned)h < (unsigned)g.H;
                    const f2 mask = {(hok && (unsigned)wq < (unsigned)g.W) ? 1.f : 0.f,
                                     (hok && (unsigned)(wq + 1) < (unsigned)g.W) ? 1.f : 0.f};
                    float a0[8], a1[8];
                    unpack8(pf[i][0], a0);
                    unpack8(pf[i][1], a1);
                    uint32_t* dst = reinterpret_cast<uint32_t*>(im + sv * 8 * g.IMG + (rlo + rr) * g.IC + 2 * (g.jlo + jj));
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        f2 pv = {a0[e], a1[e]};
                        if (silu_pro) pv = silu_pair(pv, sc[e], sh[e], mask);
                        dst[e * (g.IMG / 2)] = pack2(pv.x, pv.y);
                    }
                }
                rr += sd_r; jj += sd_j;
                if (jj >= NJ) { jj -= NJ; ++rr; }
            }
        }
        // the next unit's loads fly while this one multiplies out and is written back
        if (un + D * g.FS < units) issue(un + D * g.FS, pf);
        __syncthreads();
        // ---- taps on MFMA (wave wv: vector wv, channel by channel); bf16 outputs into the consumed interior
#ifdef RT1_DWM_T_NOCOMP   // timing-only build: no taps
        if (false) {
#else
        if (wv < ncv) {
#endif
            const int np = nph * g.Wp, ngrp = (np + 15) >> 4;
            int boff[MAXG], ooff[MAXG];
            int ph = m_r, pw = m_c;
#pragma unroll
            for (int gi = 0; gi < MAXG; ++gi) {
                const bool in = 16 * gi + m < np;
                const int phc = in ? ph : nph - 1, pwc = in ? pw : g.Wp - 1;   // pad, don't mask
                boff[gi] = (4 * phc + kg) * g.IC + 4 * pwc;
                // every lane writes its 4 outputs (a padded lane duplicates its patch's): the columns / rows past the
                // frame land on image cells the staging rewrites every unit
                ooff[gi] = (4 * phc + kg + P) * g.IC + 4 * pwc + P;
                ph += gd_r; pw += gd_c;
                if (pw >= g.Wp) { pw -= g.Wp; ++ph; }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bf16_t* ci = im + (wv * 8 + j) * g.IMG;
                f32x4 acc[MAXG];
#pragma unroll
                for (int gi = 0; gi < MAXG; ++gi) {
                    acc[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (gi >= ngrp) continue;
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const bf16_t* bp = ci + boff[gi] + 4 * s * g.IC;
                        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(bp);
                        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(bp + 4);
                        const bf16x8 bb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                        acc[gi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j][s], bb, acc[gi], 0, 0, 0);
                    }
                }
                // all of this channel's window reads precede its output writes (in-order DS ops of one wave)
#pragma unroll
                for (int gi = 0; gi < MAXG; ++gi) {
                    if (gi >= ngrp) continue;
                    const uint32_t lo2 = pack2(acc[gi][0], acc[gi][1]), hi2 = pack2(acc[gi][2], acc[gi][3]);
                    bf16_t* op = ci + ooff[gi];
                    if constexpr (P == 2) {                         // 4-byte aligned output runs
                        reinterpret_cast<uint32_t*>(op)[0] = lo2;
                        reinterpret_cast<uint32_t*>(op)[1] = hi2;
                    } else {
                        op[0] = (bf16_t)lo2;
                        op[1] = (bf16_t)(lo2 >> 16);
                        op[2] = (bf16_t)hi2;
                        op[3] = (bf16_t)(hi2 >> 16);
                    }
                }
            }
        }
        __syncthreads();
        // ---- read back channels-last: 8 threads per pixel (one 8-channel vector each), statistics on the way
        {
            const int npx = orows * g.W;
            bf16_t* of = out + ((int64_t)n * g.H + 4 * ph0) * g.W * g.C + c0 + sv * 8;
            const bf16_t* src0 = im + sv * 8 * g.IMG + P * g.IC + P;
            int fr = b_r0, fc = b_c0;
#ifdef RT1_DWM_T_NORB   // timing-only build: no read-back
            for (int px = pr0; px < 0; px += 64) {
#else
            for (int px = pr0; px < npx; px += 64) {
#endif
                if (sv_ok) {
                    const bf16_t* sp = src0 + fr * g.IC + fc;
                    uint32_t uw[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        uw[e] = (uint32_t)sp[(2 * e) * g.IMG] | ((uint32_t)sp[(2 * e + 1) * g.IMG] << 16);
                    *reinterpret_cast<uint4*>(of + ((int64_t)fr * g.W + fc) * g.C) = make_uint4(uw[0], uw[1], uw[2], uw[3]);
                    if (stats) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const f2 vv = {__uint_as_float(uw[e] << 16), __uint_as_float(uw[e] & 0xffff0000u)};
                            s_acc[e] += vv;
                            q_acc[e] = vv * vv + q_acc[e];
                        }
                    }
                }
                fr += rd_r; fc += rd_c;
                if (fc >= g.W) { fc -= g.W; ++fr; }
            }
        }
    };
    uint4 pf[D][MAXR][2];
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (fs + d * g.FS < units) issue(fs + d * g.FS, pf[d]);
    for (int un = fs; un < units; un += D * g.FS) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (un + d * g.FS >= units) break;                      // workgroup-uniform
            body(un + d * g.FS, pf[d]);
        }
    }
    if (stats) {
        // threads of one vector: lanes sv, sv + 8, ... of every wave -> shuffle over lane / 8, then over the waves
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int o = 8; o < 64; o <<= 1) {
                s_acc[e].x += __shfl_xor(s_acc[e].x, o, 64);
                s_acc[e].y += __shfl_xor(s_acc[e].y, o, 64);
                q_acc[e].x += __shfl_xor(q_acc[e].x, o, 64);
                q_acc[e].y += __shfl_xor(q_acc[e].y, o, 64);
            }
        if (lane < 8) {
            float* rp = red + (wv * 8 + lane) * 16;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                rp[2 * e] = s_acc[e].x; rp[2 * e + 1] = s_acc[e].y;
                rp[8 + 2 * e] = q_acc[e].x; rp[8 + 2 * e + 1] = q_acc[e].y;
            }
        }
        __syncthreads();
        if (t < 2 * CC) {
            const int c = t & (CC - 1), q = t >> 6;                // q: 0 sum, 1 sum of squares
            if (c < ncv * 8) {
                float a = 0.f;
                for (int ww = 0; ww < 8; ++ww) a += red[(ww * 8 + c / 8) * 16 + 8 * q + c % 8];
                (q ? psq : psum)[(int64_t)fs * g.C + c0 + c] = a;
            }
        }
    }
}

#ifndef RT1_DWM_WG_TARGET
#define RT1_DWM_WG_TARGET 1024   // 512-thread workgroups over the whole layer (each walks several units)
#endif
#ifndef RT1_DWM_LDS_KB
#define RT1_DWM_LDS_KB 76
#endif

inline int cdivm(int a, int b) { return (a + b - 1) / b; }

size_t mfma_lds(const MGeo& g) { return (size_t)CC * g.IMG * 2 + (size_t)(2 * CC + 64 * 16) * 4; }

// staging items per thread per unit
int mfma_rounds(const MGeo& g) {
    const int rows = g.nb == 1 ? 4 * g.Hp : g.IRB;
    return cdivm(rows * (g.jhi - g.jlo), 64);
}

// the largest band (patch rows per unit) whose image fits the LDS budget, at most 4 groups of 16 patches
MGeo mgeo(int N, int H, int W, int C, int k) {
    MGeo g;
    g.N = N; g.H = H; g.W = W; g.C = C;
    g.Hp = cdivm(H, 4); g.Wp = cdivm(W, 4);
    g.IC = 4 * g.Wp + 4;
    if (g.IC % 8 == 0) g.IC += 4;                              // rows 2 mod 4 dwords apart (LDS banks)
    const int P = (k - 1) / 2;
    g.jlo = P / 2;
    g.jhi = cdivm(4 * g.Wp + P, 2);                            // up to the last output cell (re-zeroed per unit)
    g.chunks = cdivm(C, CC);
    for (int bph = g.Hp; bph >= 1; --bph) {
        g.BPH = bph;
        g.IRB = 4 * bph + 4;
        const int img = g.IRB * g.IC;
        g.IMG = img + (img % 16 == 0 ? 4 : 0);               // channel images not 32-B aligned to each other
        g.nb = cdivm(g.Hp, bph);
        if (cdivm(bph * g.Wp, 16) <= 4 && mfma_rounds(g) <= 4 && mfma_lds(g) <= (size_t)RT1_DWM_LDS_KB * 1024) break;
    }
    g.FS = 1;
    return g;
}

// opt-in (RT1_DW_MFMA=1): measured slower than the vector-ALU forward in dwconv.hip (profiles/r3_dw_mfma_ab.md)
bool mfma_env_on() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("RT1_DW_MFMA");
        on = (e && e[0] == '1') ? 1 : 0;
    }
    return on == 1;
}

}  // namespace

extern "C" {

// The MFMA path covers stride-1 k3 / k5 layers with maps <= 40 x 40, channel counts that are multiples of 8, and
// the copy / BN+SiLU prologues.  ext.dw_fwd takes it only with RT1_DW_MFMA=1 (force = 0); ext.dw_fwd_mfma always.
int rt1_dw_mfma_ok(int H, int W, int C, int k, int s, int act, int force) {
    if (!force && !mfma_env_on()) return 0;
    if (s != 1 || (k != 3 && k != 5) || C % 8 || H > 40 || W > 40 || H < 1 || W < 1) return 0;
    if (act != 0 && act != 1) return 0;
    const MGeo g = mgeo(1, H, W, C, k);
    return (cdivm(g.BPH * g.Wp, 16) <= 4 && mfma_rounds(g) <= 4 && mfma_lds(g) <= (size_t)RT1_DWM_LDS_KB * 1024)
               ? 1 : 0;
}

// frame slots = rows of the partial-statistics buffers
int rt1_dw_mfma_grid(int N, int H, int W, int C, int max_blocks_x) {
    const MGeo g = mgeo(N, H, W, C, 5);
    int fs = cdivm(RT1_DWM_WG_TARGET, g.chunks);
    const int units = N * g.nb;
    if (fs > units) fs = units;
    if (fs > max_blocks_x) fs = max_blocks_x;
    return fs < 1 ? 1 : fs;
}

int rt1_dw_mfma_fwd(const bf16_t* x, const float* w, const float* scale, const float* shift, int act, int N, int H,
                    int W, int C, int k, int grid_x, bf16_t* out, float* psum, float* psq, hipStream_t st) {
    MGeo g = mgeo(N, H, W, C, k);
    if (g.nb != mgeo(N, H, W, C, 5).nb) return (int)hipErrorInvalidValue;   // rows were sized with the k5 bands
    g.FS = grid_x;
    if (scale != nullptr && act != 1) return (int)hipErrorInvalidValue;    // the prologue is BN + SiLU or nothing
    const int maxg = cdivm(g.BPH * g.Wp, 16), maxr = mfma_rounds(g);
    const size_t lds = mfma_lds(g);
    dim3 grid(g.FS, g.chunks);
#define LM(KK, MG, MR, DD)                                                                                         \
    hipLaunchKernelGGL((dw_fwd_mfma_kernel<KK, MG, MR, DD>), grid, dim3(BLOCK), lds, st, x, w, scale, shift, g, out, \
                       psum, psq)
    // the model's shapes: 10x10 (1 group, 2 rounds), 19x19 and the 38x38 bands (2, 4); anything else the generic (4, 4)
#define LC(KK)                                                                                                      \
    do {                                                                                                           \
        if (maxg <= 1 && maxr <= 2) LM(KK, 1, 2, 2);                                                               \
        else if (maxg <= 2) LM(KK, 2, 4, 1);                                                                       \
        else LM(KK, 4, 4, 1);                                                                                      \
    } while (0)
    if (k == 5) LC(5);
    else LC(3);
#undef LC
#undef LM
    return (int)hipGetLastError();
}

}  // extern "C"
