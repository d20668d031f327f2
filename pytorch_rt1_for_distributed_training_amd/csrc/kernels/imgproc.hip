// Random-resized-crop of raw uint8 frames on the GPU (reference D2 ``DecodeAndRandomResizedCrop``,
// /root/reference/load_np_dataset.py:8-39: PIL ``crop(box).resize((W, H), BILINEAR)``).
//
// The training input pipeline ships raw HWC uint8 frames + one integer crop box per frame to HBM and runs this
// kernel on the prefetch stream, instead of 6 PIL resizes per sample on the CPU.  It reproduces Pillow's
// resampler bit for bit: the antialiased bilinear ("triangle") filter with support scaled by the downscale
// factor, coefficients normalised in double then rounded to 22-bit fixed point, a horizontal pass rounded to
// uint8, then the vertical pass (Pillow's two-pass order, Resample.c ImagingResampleInner).
//
// Banded kernel (crop_resize_band_kernel, the training path): a workgroup owns BAND output rows of one frame.  It
// computes the frame's column taps and its rows' taps once in double (into LDS), stages the source rows the band
// needs with 16-byte loads, runs the horizontal pass into a uint8 [row][channel][W] image in LDS, then the vertical
// pass for 4 output pixels per thread with 32-bit LDS reads and stores.  The first version -- one thread per output
// pixel recomputing both tap sets in double and reading the window with byte loads from global -- took 1.27 ms per
// b128 batch (profiles/r4_resident_decode.log) on the prefetch stream, i.e. on top of the training step; it remains
// the general fallback (frames whose row bytes are not 16-B multiples, W % 4 != 0, downscales beyond 3x).
// Output is planar [N, 3, H, W] uint8, the layout the stem kernel reads.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int PREC = 22;            // Pillow PRECISION_BITS = 32 - 8 - 2
constexpr int MAXK = 16;            // taps per axis: supports downscale factors up to ~7.5x

template <int K = MAXK>
struct Taps {
    int lo, n;
    int k[K];
};

// Pillow precompute_coeffs + normalize_coeffs_8bpc for output index `o` (crop = [0, in_size), box = full crop)
template <int K>
__device__ __forceinline__ void taps_for(int o, int in_size, int out_size, Taps<K>& t) {
    constexpr int MAXK = K;
    const double scale = (double)in_size / (double)out_size;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = fs;                 // bilinear filter support 1.0
    const double center = (o + 0.5) * scale;
    const double ss = 1.0 / fs;
    int lo = (int)(center - support + 0.5);
    if (lo < 0) lo = 0;
    int hi = (int)(center + support + 0.5);
    if (hi > in_size) hi = in_size;
    int n = hi - lo;
    if (n > MAXK) n = MAXK;
    double w[MAXK];
    double ww = 0.0;
    for (int i = 0; i < n; ++i) {
        double x = (i + lo - center + 0.5) * ss;
        x = x < 0.0 ? -x : x;
        w[i] = x < 1.0 ? 1.0 - x : 0.0;
        ww += w[i];
    }
    for (int i = 0; i < n; ++i) {
        const double v = ww != 0.0 ? w[i] / ww : w[i];
        t.k[i] = v < 0 ? (int)(-0.5 + v * (double)(1 << PREC)) : (int)(0.5 + v * (double)(1 << PREC));
    }
    t.lo = lo;
    t.n = n;
}

// taps_for with FK taps, fully unrolled (predicated on i < n: the same sums in the same order, no scratch arrays);
// weights past n are 0, so callers may run all FK taps branch-free
constexpr int FK = 8;        // taps per axis in the banded kernel: n <= 2 * max(scale, 1) + 2, so downscales <= 3x
__device__ __forceinline__ void taps_fk(int o, int in_size, int out_size, int& lo_out, int& n_out, int (&k)[FK]) {
    const double scale = (double)in_size / (double)out_size;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = fs;
    const double center = (o + 0.5) * scale;
    const double ss = 1.0 / fs;
    int lo = (int)(center - support + 0.5);
    if (lo < 0) lo = 0;
    int hi = (int)(center + support + 0.5);
    if (hi > in_size) hi = in_size;
    int n = hi - lo;
    if (n > FK) n = FK;
    double w[FK];
    double ww = 0.0;
#pragma unroll
    for (int i = 0; i < FK; ++i) {
        double x = (i + lo - center + 0.5) * ss;
        x = x < 0.0 ? -x : x;
        w[i] = (i < n && x < 1.0) ? 1.0 - x : 0.0;
        if (i < n) ww += w[i];
    }
#pragma unroll
    for (int i = 0; i < FK; ++i) {
        const double v = ww != 0.0 ? w[i] / ww : w[i];
        k[i] = i >= n ? 0 : (v < 0 ? (int)(-0.5 + v * (double)(1 << PREC)) : (int)(0.5 + v * (double)(1 << PREC)));
    }
    lo_out = lo;
    n_out = n;
}

__device__ __forceinline__ int clip8(int v) {
    v >>= PREC;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// clip8 for values packed 4 to a 32-bit word.  The opaque copy keeps the compiler from fusing two clip8 + byte packs
// into v_ashr_pk_u8_i32: it treated that instruction's result as zero-extended to 32 bits, but the high half of the
// destination register kept its old contents, and OR-ing the upper bytes in then corrupted byte 2 (channels 1 and 2
// at every 4th column were off by up to 204, tools/debug/imgproc_diff.py).  tests/test_isa_audit.py bans the op.
__device__ __forceinline__ uint32_t clip8_opaque(int v) {
    int r = clip8(v);
    asm volatile("" : "+v"(r));
    return (uint32_t)r;
}

// raw: [F, h, w, 3] uint8; rows: [N] int64 frame indices into raw (nullptr: frame n = raw[n], F = N) -- the
// HBM-resident input path (data/resident.py) gathers the batch's frames from the resident episode range here, so no
// frame crosses PCIe per step; boxes: [N, 4] int32 (x0, y0, x1, y1), the crop [x0, x1) x [y0, y1) inside the frame;
// out: [N, 3, H, W] uint8
__global__ __launch_bounds__(256) void crop_resize_kernel(const uint8_t* __restrict__ raw,
                                                          const int64_t* __restrict__ rows, int64_t F,
                                                          const int* __restrict__ boxes, int N, int h, int w,
                                                          int H, int W, uint8_t* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)N * H * W;
    if (idx >= total) return;
    const int n = (int)(idx / ((int64_t)H * W));
    const int rem = (int)(idx - (int64_t)n * H * W);
    const int oy = rem / W, ox = rem - oy * W;
    // boxes are validated by the loader; clamp anyway so a bad box can never read outside the frame
    int x0 = boxes[n * 4 + 0], y0 = boxes[n * 4 + 1], x1 = boxes[n * 4 + 2], y1 = boxes[n * 4 + 3];
    x0 = x0 < 0 ? 0 : (x0 > w - 1 ? w - 1 : x0);
    y0 = y0 < 0 ? 0 : (y0 > h - 1 ? h - 1 : y0);
    x1 = x1 <= x0 ? x0 + 1 : (x1 > w ? w : x1);
    y1 = y1 <= y0 ? y0 + 1 : (y1 > h ? h : y1);
    const int cw = x1 - x0, ch = y1 - y0;
    Taps<> tx, ty;
    taps_for(ox, cw, W, tx);
    taps_for(oy, ch, H, ty);
    int64_t fr = rows ? rows[n] : n;
    fr = fr < 0 ? 0 : (fr >= F ? F - 1 : fr);      // rows are validated by the loader; never read outside raw
    const uint8_t* frame = raw + fr * h * w * 3;
    int acc[3] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
    for (int j = 0; j < ty.n; ++j) {
        const uint8_t* row = frame + ((int64_t)(y0 + ty.lo + j) * w + x0 + tx.lo) * 3;
        int hs[3] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
        for (int i = 0; i < tx.n; ++i) {
            const int k = tx.k[i];
            hs[0] += (int)row[i * 3 + 0] * k;
            hs[1] += (int)row[i * 3 + 1] * k;
            hs[2] += (int)row[i * 3 + 2] * k;
        }
        const int k = ty.k[j];
        acc[0] += clip8(hs[0]) * k;          // horizontal pass result is stored as uint8 before the vertical one
        acc[1] += clip8(hs[1]) * k;
        acc[2] += clip8(hs[2]) * k;
    }
    const int64_t plane = (int64_t)H * W;
    uint8_t* o = out + (int64_t)n * 3 * plane + rem;
    o[0] = (uint8_t)clip8(acc[0]);
    o[plane] = (uint8_t)clip8(acc[1]);
    o[2 * plane] = (uint8_t)clip8(acc[2]);
}

constexpr int BAND = 8;      // output rows per workgroup (~50 KB of LDS: 3 workgroups / CU; 10 rows: 2, -11 %)
#ifndef RT1_IMG_TIMING
#define RT1_IMG_TIMING 0     // timing-only builds (values wrong): 1 no tap math, 2 no staging, 4 no horizontal, 8 no vertical
#endif

__device__ __forceinline__ void clamp_box(const int* boxes, int n, int h, int w, int& x0, int& y0, int& x1, int& y1) {
    // boxes are validated by the loader; clamp anyway so a bad box can never read outside the frame
    x0 = boxes[n * 4 + 0], y0 = boxes[n * 4 + 1], x1 = boxes[n * 4 + 2], y1 = boxes[n * 4 + 3];
    x0 = x0 < 0 ? 0 : (x0 > w - 1 ? w - 1 : x0);
    y0 = y0 < 0 ? 0 : (y0 > h - 1 ? h - 1 : y0);
    x1 = x1 <= x0 ? x0 + 1 : (x1 > w ? w : x1);
    y1 = y1 <= y0 ? y0 + 1 : (y1 > h ? h : y1);
}

// LDS: column taps xk [FK][W] + xlo / xn [W], the band's row taps yk [BAND][FK] + ylo / yn, then (16-B aligned) the
// staged source rows [rmax][sb] and the horizontal-pass image [rmax][3][W]
__global__ __launch_bounds__(256) void crop_resize_band_kernel(const uint8_t* __restrict__ raw,
                                                               const int64_t* __restrict__ rows, int64_t F,
                                                               const int* __restrict__ boxes, int h, int w, int H,
                                                               int W, int rmax, int sb, uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) int smi[];
    int* xk = smi;
    int* xlo = xk + FK * W;
    int* xn = xlo + W;
    int* yk = xn + W;
    int* ylo = yk + BAND * FK;
    int* yn = ylo + BAND;
    uint8_t* src = reinterpret_cast<uint8_t*>(smi) + (((size_t)(3 * W + (FK + 2) * BAND + FK * W) * 4 + 15) & ~(size_t)15);
    uint8_t* mid = src + (size_t)rmax * sb;
    const int n = blockIdx.y, t = threadIdx.x;
    const int oy0 = blockIdx.x * BAND;
    const int nb = H - oy0 < BAND ? H - oy0 : BAND;
    int x0, y0, x1, y1;
    clamp_box(boxes, n, h, w, x0, y0, x1, y1);
    const int cw = x1 - x0, ch = y1 - y0;
    for (int ox = t; ox < W; ox += 256) {
        int k[FK];
#if RT1_IMG_TIMING & 1
        xlo[ox] = ox; xn[ox] = 4;
#pragma unroll
        for (int i = 0; i < FK; ++i) k[i] = i;
#else
        taps_fk(ox, cw, W, xlo[ox], xn[ox], k);
#endif
#pragma unroll
        for (int i = 0; i < FK; ++i) xk[i * W + ox] = k[i];
    }
    if (t < nb) {
        int k[FK];
        taps_fk(oy0 + t, ch, H, ylo[t], yn[t], k);
#pragma unroll
        for (int i = 0; i < FK; ++i) yk[t * FK + i] = k[i];
    }
    __syncthreads();
    // the band's source rows [r0, r1) of the crop (lo and hi are monotone in the output row)
    const int r0 = ylo[0];
    int r1 = r0;
    for (int i = 0; i < nb; ++i) r1 = ylo[i] + yn[i] > r1 ? ylo[i] + yn[i] : r1;
    const int nr = r1 - r0 < rmax ? r1 - r0 : rmax;            // the host bound makes the clamp a no-op
    int64_t fr = rows ? rows[n] : n;
    fr = fr < 0 ? 0 : (fr >= F ? F - 1 : fr);                  // rows are validated by the loader; never read outside raw
    const uint8_t* frame = raw + fr * h * w * 3;
    const int xs = (3 * x0) & ~15;
    int xe = (3 * x1 + 15) & ~15;
    xe = xe > 3 * w ? 3 * w : xe;                               // 3 w is a multiple of 16 on this path
    const int nv = (xe - xs) >> 4;
    // SU 16-B loads in flight per thread before any LDS store (one load per iteration left every load's HBM
    // latency exposed: ~8 round trips per workgroup)
    constexpr int SU = 8;
    const int nvec = nr * nv;
    for (int i0 = t; i0 < ((RT1_IMG_TIMING & 2) ? 0 : nvec); i0 += 256 * SU) {
        uint4 v[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            const int i = i0 + u * 256;
            if (i < nvec) {
                const int r = i / nv, c = i - r * nv;
                v[u] = *reinterpret_cast<const uint4*>(frame + ((int64_t)(y0 + r0 + r) * w) * 3 + xs + 16 * c);
            }
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            const int i = i0 + u * 256;
            if (i < nvec) {
                const int r = i / nv, c = i - r * nv;
                *reinterpret_cast<uint4*>(src + r * sb + 16 * c) = v[u];
            }
        }
    }
    __syncthreads();
    // horizontal pass (rounded to uint8, as Pillow stores it between the passes): one output column per lane, so the
    // lanes' source bytes sit ~3.4 bytes apart (the 4-columns-per-lane form strided them 14 bytes apart: 7-way LDS
    // bank conflicts on the byte reads, 8-way on the tap table)
    for (int i = t; i < ((RT1_IMG_TIMING & 4) ? 0 : nr * W); i += 256) {
        const int r = i / W, ox = i - r * W;
        // all FK taps, branch-free: the weights past n are 0 and the bytes they read stay inside the LDS allocation
        // (the row slot has 16 spare bytes, the last row is followed by mid), so every load issues at once
        const uint8_t* p = src + r * sb + 3 * (x0 + xlo[ox]) - xs;
        int h0 = 1 << (PREC - 1), h1 = h0, h2 = h0;
#pragma unroll
        for (int k = 0; k < FK; ++k) {
            // 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate): bytes x weights < 2^23, all >= 0
            const unsigned kk = (unsigned)xk[k * W + ox];
            h0 += (int)__umul24(p[3 * k + 0], kk);
            h1 += (int)__umul24(p[3 * k + 1], kk);
            h2 += (int)__umul24(p[3 * k + 2], kk);
        }
        uint8_t* m = mid + (size_t)r * 3 * W + ox;
        m[0] = (uint8_t)clip8(h0);
        m[W] = (uint8_t)clip8(h1);
        m[2 * W] = (uint8_t)clip8(h2);
    }
    __syncthreads();
    // vertical pass: 4 consecutive output pixels per thread (W % 4 == 0), one 32-bit store per channel
    const int W4 = W >> 2;
    const int64_t plane = (int64_t)H * W;
    for (int i = t; i < ((RT1_IMG_TIMING & 8) ? 0 : nb * W4); i += 256) {
        const int ol = i / W4, ox = (i - ol * W4) * 4;
        const int lo = ylo[ol] - r0;
        int a[3][4];
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) a[c][j] = 1 << (PREC - 1);
#pragma unroll
        for (int k = 0; k < FK; ++k) {                          // branch-free as above; rows past the band clamp
            const unsigned kk = (unsigned)yk[ol * FK + k];
            const int rr = lo + k < nr ? lo + k : nr - 1;
            const uint8_t* m = mid + (size_t)rr * 3 * W + ox;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const uint32_t q = *reinterpret_cast<const uint32_t*>(m + c * W);
#pragma unroll
                for (int j = 0; j < 4; ++j) a[c][j] += (int)__umul24(__builtin_amdgcn_ubfe(q, 8 * j, 8), kk);
            }
        }
        uint8_t* o = out + (int64_t)n * 3 * plane + (int64_t)(oy0 + ol) * W + ox;
#pragma unroll
        for (int c = 0; c < 3; ++c)
            *reinterpret_cast<uint32_t*>(o + c * plane) = clip8_opaque(a[c][0]) | (clip8_opaque(a[c][1]) << 8) |
                                                         (clip8_opaque(a[c][2]) << 16) | (clip8_opaque(a[c][3]) << 24);
    }
}

}  // namespace

extern "C" {

int rt1_crop_resize_gather_u8(const uint8_t* raw, int64_t F, const int64_t* rows, const int* boxes, int N, int h,
                              int w, int H, int W, uint8_t* out, hipStream_t st) {
    if (N <= 0 || H <= 0 || W <= 0 || F <= 0) return (int)hipErrorInvalidValue;
    // banded kernel: 16-B source rows, 4-pixel output groups, <= FK taps per axis (downscale <= 3x), LDS fits
    const double sy = (double)h / H, sx = (double)w / W;
    const int rmax = (int)((BAND - 1) * sy + 2.0 * (sy > 1.0 ? sy : 1.0)) + 3;
    const int sb = 3 * w + 16;
    const size_t lds = (((size_t)(3 * W + (FK + 2) * BAND + FK * W) * 4 + 15) & ~(size_t)15) + (size_t)rmax * sb +
                       (size_t)rmax * 3 * W;
    if ((3 * w) % 16 == 0 && ((uintptr_t)raw & 15) == 0 && W % 4 == 0 && sy <= 3.0 && sx <= 3.0 &&
        lds <= 96 * 1024) {
        hipLaunchKernelGGL(crop_resize_band_kernel, dim3((H + BAND - 1) / BAND, N), dim3(256), lds, st, raw, rows, F,
                           boxes, h, w, H, W, rmax, sb, out);
        return (int)hipGetLastError();
    }
    const int64_t total = (int64_t)N * H * W;
    const int grid = (int)((total + 255) / 256);
    hipLaunchKernelGGL(crop_resize_kernel, dim3(grid), dim3(256), 0, st, raw, rows, F, boxes, N, h, w, H, W, out);
    return (int)hipGetLastError();
}

int rt1_crop_resize_u8(const uint8_t* raw, const int* boxes, int N, int h, int w, int H, int W, uint8_t* out,
                       hipStream_t st) {
    return rt1_crop_resize_gather_u8(raw, N, nullptr, boxes, N, h, w, H, W, out, st);
}

}  // extern "C"
