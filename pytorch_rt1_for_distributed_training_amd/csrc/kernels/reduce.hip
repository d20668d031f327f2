// Deterministic column sums: out[b][c] = sum_r in[b][r][c], fp32 accumulation in a FIXED order.
//
// Every weight gradient of the encoder is produced as per-workgroup partial rows (dwconv, pw_bwd, stem,
// frame pools, split-K GEMMs) that must be summed.  ATen's generic reduction for tall [R, C] inputs splits R
// over several workgroups and finishes with a global-memory semaphore + "last block" combine; under hipGraph
// replay on gfx950 that path produced sporadically wrong sums (tools/scratch/dp_graph_debug.py: block 2's
// depthwise/expand weight gradients off by 1e3x, different on every replay).  This kernel never synchronises
// across workgroups: pass 1 reduces fixed row chunks into [chunks][C], pass 2 (a second launch) reduces the
// chunks, and within a workgroup the 4 row groups combine in LDS as ((r0 + r1) + r2) + r3.  Same inputs ->
// same bits, eager or replayed.
//
// Layout: one workgroup = 64 lanes x 4 row groups; a lane owns V consecutive columns (V = 4 when C % 4 == 0,
// 16-B fp32 / 8-B bf16 loads), a row group walks rows rg, rg + 4, ... of its chunk with 4 independent loads
// in flight per lane.
#include "common.h"

using namespace rt1;

namespace {

constexpr int CS_THREADS = 256;

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <typename T, int V>
__device__ __forceinline__ void ldv(const T* p, float (&o)[V]) {
    if constexpr (V == 4 && sizeof(T) == 4) {
        const float4 u = *reinterpret_cast<const float4*>(p);
        o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w;
    } else if constexpr (V == 4 && sizeof(T) == 2) {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xffff0000u);
        o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xffff0000u);
    } else {
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = ld1<T>(p + j);
    }
}

// RGS row groups of 64 lanes: 4 (256 threads) normally, 16 (1024 threads) when the launch has few workgroups (narrow
// inputs of a few hundred rows ran on one or two workgroups for 12-18 us)
template <typename T, int V, int RGS = 4>
__global__ __launch_bounds__(64 * RGS) void colsum_kernel(const T* __restrict__ in, int64_t R, int C,
                                                          int64_t batch_stride, int64_t rows_per_chunk,
                                                          float* __restrict__ out, int64_t out_batch_stride) {
    __shared__ float red[RGS][64 * V];
    const int t = threadIdx.x, lane = t & 63, rg = t >> 6;
    const int c0 = (blockIdx.x * 64 + lane) * V;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < R ? r0 + rows_per_chunk : R;
    const T* base = in + (int64_t)blockIdx.z * batch_stride;
    float a[V];
#pragma unroll
    for (int j = 0; j < V; ++j) a[j] = 0.f;
    if (c0 < C) {
        int64_t r = r0 + rg;
        for (; r + 3 * RGS < r1; r += 4 * RGS) {
            float v0[V], v1[V], v2[V], v3[V];
            ldv<T, V>(base + r * C + c0, v0);
            ldv<T, V>(base + (r + RGS) * C + c0, v1);
            ldv<T, V>(base + (r + 2 * RGS) * C + c0, v2);
            ldv<T, V>(base + (r + 3 * RGS) * C + c0, v3);
#pragma unroll
            for (int j = 0; j < V; ++j) a[j] = (((a[j] + v0[j]) + v1[j]) + v2[j]) + v3[j];
        }
        for (; r < r1; r += RGS) {
            float v0[V];
            ldv<T, V>(base + r * C + c0, v0);
#pragma unroll
            for (int j = 0; j < V; ++j) a[j] += v0[j];
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) red[rg][lane * V + j] = a[j];
    __syncthreads();
    if (rg == 0 && c0 < C) {
        float* o = out + (int64_t)blockIdx.z * out_batch_stride + (int64_t)blockIdx.y * C + c0;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int k = lane * V + j;
            float x = red[0][k];
#pragma unroll
            for (int g = 1; g < RGS; ++g) x += red[g][k];
            o[j] = x;
        }
    }
}

template <typename T>
int launch_pass(const T* in, int64_t R, int C, int B, int64_t bstride, int64_t chunk_rows, int chunks, float* out,
                int64_t obstride, hipStream_t st) {
    const bool v4 = (C % 4) == 0;
    const int V = v4 ? 4 : 1;
    const int cb = (C + 64 * V - 1) / (64 * V);
    dim3 grid(cb, chunks, B);
    const bool wide = (int64_t)cb * chunks * B < 64 && chunk_rows >= 64;    // few workgroups: 16 row groups each
    if (wide) {
        if (v4) hipLaunchKernelGGL((colsum_kernel<T, 4, 16>), grid, dim3(1024), 0, st, in, R, C, bstride, chunk_rows,
                                   out, obstride);
        else hipLaunchKernelGGL((colsum_kernel<T, 1, 16>), grid, dim3(1024), 0, st, in, R, C, bstride, chunk_rows,
                                out, obstride);
    } else if (v4) {
        hipLaunchKernelGGL((colsum_kernel<T, 4>), grid, dim3(CS_THREADS), 0, st, in, R, C, bstride, chunk_rows, out,
                           obstride);
    } else {
        hipLaunchKernelGGL((colsum_kernel<T, 1>), grid, dim3(CS_THREADS), 0, st, in, R, C, bstride, chunk_rows, out,
                           obstride);
    }
    return (int)hipGetLastError();
}

// Gradient gather: up to MC_MAX copies of 4-byte words (src -> dst, n words each) in ONE launch, grid.y = copy index.
// Replaces the per-tensor D2D blits of torch._foreach_copy_ (one copyBuffer dispatch per stolen gradient,
// ~270 per RT-1 step) when the flat gradient buffer collects the tensors autograd produced; also packs the
// transformer's Q/K/V weight shadows once per step.  128 entries = 3 KB of kernel arguments.
constexpr int MC_MAX = 128;
struct CopyList {
    const float* src[MC_MAX];
    float* dst[MC_MAX];
    int64_t n[MC_MAX];
};

__global__ __launch_bounds__(256) void multi_copy_kernel(CopyList L) {
    const int i = blockIdx.y;
    const float* __restrict__ s = L.src[i];
    float* __restrict__ d = L.dst[i];
    const int64_t n = L.n[i];
    const int64_t stride = (int64_t)gridDim.x * 256;
    const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
    int64_t head = 0;
    if (vec) {
        const int64_t nv = n / 4;
        for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += stride)
            reinterpret_cast<float4*>(d)[v] = reinterpret_cast<const float4*>(s)[v];
        head = nv * 4;
    }
    for (int64_t e = head + (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) d[e] = s[e];
}

// Gradient gather with the split-K sums folded in: dst[e] = sum_{k < splits} src[k * sstride + e], k in order (a
// copy for splits == 1).  The weight-gradient kernels leave their row-split partials [splits, Co, Ci] unsummed at
// the sites that produce a final parameter gradient (parallel/flat.py defer_partials); this one launch per bucket
// replaces a colsum launch per weight gradient.
struct ReduceList {
    const float* src[MC_MAX];
    float* dst[MC_MAX];
    int64_t n[MC_MAX];
    int64_t sstride[MC_MAX];
    int splits[MC_MAX];
    int groups[MC_MAX];         // split groups per workgroup (1..16, a power of two): 256 / groups float4 columns each
};

// A workgroup owns 256 / G consecutive float4 columns of one entry; thread group g (of G) sums splits g, g + G, ...
// in order (4 loads in flight), then the G group sums combine in LDS as ((s0 + s1) + s2) + ...  Entries with many
// splits and few elements (the deep layers' split-K partials: 64-256 splits of a few thousand weights) get G = 16,
// so their sums are not one long dependent chain per thread.  Fixed order throughout: same inputs, same bits.
__global__ __launch_bounds__(256) void multi_reduce_copy_kernel(ReduceList L) {
    __shared__ float4 red[256];
    const int i = blockIdx.y;
    const float* __restrict__ s = L.src[i];
    float* __restrict__ d = L.dst[i];
    const int64_t n = L.n[i], ss = L.sstride[i];
    const int S = L.splits[i], G = L.groups[i];
    const int CW = 256 / G;                                        // float4 columns per workgroup
    const int t = threadIdx.x, g = t / CW, c = t - g * CW;
    const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0 && (ss & 3) == 0;
    if (vec) {
        const int64_t nv = n / 4, sv = ss >> 2;
        for (int64_t v0 = (int64_t)blockIdx.x * CW; v0 < nv; v0 += (int64_t)gridDim.x * CW) {   // uniform per WG
            const int64_t v = v0 + c;
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            if (v < nv && g < S) {
                const float4* p = reinterpret_cast<const float4*>(s) + v;
                a = p[g * sv];
                int k = g + G;
                for (; k + 3 * G < S; k += 4 * G) {
                    const float4 b0 = p[k * sv], b1 = p[(k + G) * sv], b2 = p[(k + 2 * G) * sv], b3 = p[(k + 3 * G) * sv];
                    a.x = (((a.x + b0.x) + b1.x) + b2.x) + b3.x;
                    a.y = (((a.y + b0.y) + b1.y) + b2.y) + b3.y;
                    a.z = (((a.z + b0.z) + b1.z) + b2.z) + b3.z;
                    a.w = (((a.w + b0.w) + b1.w) + b2.w) + b3.w;
                }
                for (; k < S; k += G) {
                    const float4 b = p[k * sv];
                    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
                }
            }
            if (G == 1) {
                if (v < nv) reinterpret_cast<float4*>(d)[v] = a;
                continue;
            }
            __syncthreads();                                       // previous round's LDS reads are done
            red[t] = a;
            __syncthreads();
            if (g == 0 && v < nv) {
                for (int h = 1; h < G; ++h) {
                    const float4 b = red[h * CW + c];
                    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
                }
                reinterpret_cast<float4*>(d)[v] = a;
            }
        }
        if (blockIdx.x == 0 && t < (int)(n - nv * 4)) {           // tail elements (n % 4)
            const int64_t e = nv * 4 + t;
            float x = s[e];
            for (int k = 1; k < S; ++k) x += s[k * ss + e];
            d[e] = x;
        }
        return;
    }
    for (int64_t e = (int64_t)blockIdx.x * 256 + t; e < n; e += (int64_t)gridDim.x * 256) {
        float x = s[e];
        for (int k = 1; k < S; ++k) x += s[k * ss + e];
        d[e] = x;
    }
}

}  // namespace

extern "C" {

// Number of row chunks of pass 1 (1 = single pass straight into out): enough workgroups to spread a tall input
// over the chip (~1024 in flight), each chunk >= 256 rows so pass 2 stays small.
int rt1_colsum_chunks(int64_t R, int C, int B) {
    if (R <= 512) return 1;
    const int V = (C % 4) == 0 ? 4 : 1;
    const int64_t cb = ((int64_t)C + 64 * V - 1) / (64 * V) * (B > 0 ? B : 1);
    int64_t chunks = (R + 255) / 256;
    const int64_t want = cb >= 1024 ? 1 : (1024 + cb - 1) / cb;
    if (chunks > want) chunks = want;
    if (chunks > 4096) chunks = 4096;
    return (int)(chunks < 1 ? 1 : chunks);
}

// in: B x [R, C] (batch stride R*C) fp32 or bf16; out: B x [C] fp32; tmp: B x [chunks, C] fp32 when chunks > 1
int rt1_colsum(const void* in, int in_is_bf16, int64_t R, int C, int B, float* out, float* tmp, int chunks,
               hipStream_t st) {
    if (R <= 0 || C <= 0 || B <= 0) return (int)hipErrorInvalidValue;
    const int64_t bstride = R * (int64_t)C;
    if (chunks <= 1) {
        return in_is_bf16 ? launch_pass<bf16_t>((const bf16_t*)in, R, C, B, bstride, R, 1, out, C, st)
                          : launch_pass<float>((const float*)in, R, C, B, bstride, R, 1, out, C, st);
    }
    const int64_t rows = (R + chunks - 1) / chunks;
    int e = in_is_bf16 ? launch_pass<bf16_t>((const bf16_t*)in, R, C, B, bstride, rows, chunks, tmp,
                                             (int64_t)chunks * C, st)
                       : launch_pass<float>((const float*)in, R, C, B, bstride, rows, chunks, tmp,
                                            (int64_t)chunks * C, st);
    if (e) return e;
    return launch_pass<float>(tmp, chunks, C, B, (int64_t)chunks * C, chunks, 1, out, C, st);
}

// count <= 32 fp32 copies in one launch (grid.x sized by the largest)
int rt1_multi_copy(const float* const* src, float* const* dst, const int64_t* n, int count, hipStream_t st) {
    if (count <= 0) return 0;
    if (count > MC_MAX) return (int)hipErrorInvalidValue;
    CopyList L;
    int64_t mx = 0;
    for (int i = 0; i < count; ++i) {
        L.src[i] = src[i];
        L.dst[i] = dst[i];
        L.n[i] = n[i];
        if (n[i] > mx) mx = n[i];
    }
    int64_t gx = (mx / 4 + 255) / 256;
    if (gx > 64) gx = 64;
    if (gx < 1) gx = 1;
    hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)gx, count), dim3(256), 0, st, L);
    return (int)hipGetLastError();
}

// count <= MC_MAX reduce-copies in one launch: dst[i][e] = sum_k src[i][k * sstride[i] + e] (k < splits[i])
int rt1_multi_reduce_copy(const float* const* src, float* const* dst, const int64_t* n, const int64_t* sstride,
                          const int* splits, int count, hipStream_t st) {
    if (count <= 0) return 0;
    if (count > MC_MAX) return (int)hipErrorInvalidValue;
    ReduceList L;
    int64_t gx = 1;
    for (int i = 0; i < count; ++i) {
        if (splits[i] < 1) return (int)hipErrorInvalidValue;
        L.src[i] = src[i];
        L.dst[i] = dst[i];
        L.n[i] = n[i];
        L.sstride[i] = sstride[i];
        L.splits[i] = splits[i];
        int G = 1;                                   // ~8+ splits per group, at most 16 groups
        while (G < 16 && splits[i] >= 16 * G) G *= 2;
        L.groups[i] = G;
        const int64_t wg = (n[i] / 4 + 256 / G - 1) / (256 / G);
        if (wg > gx) gx = wg;
    }
    if (gx > 256) gx = 256;
    hipLaunchKernelGGL(multi_reduce_copy_kernel, dim3((unsigned)gx, count), dim3(256), 0, st, L);
    return (int)hipGetLastError();
}

}  // extern "C"
