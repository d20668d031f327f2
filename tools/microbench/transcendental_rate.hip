// Throughput of the gfx950 VALU instruction classes the BN + SiLU staging uses: full-rate fp32 FMA, packed fp32 FMA,
// v_exp_f32 and v_rcp_f32 (transcendental).  Each lane runs 8 independent chains (enough ILP to saturate a SIMD with
// 8+ waves); the grid fills every CU several times over.  Prints wave-instructions per CU per cycle.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/transcendental_rate.hip -o /tmp/trate && /tmp/trate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void kern(float* out, float seed) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = seed + threadIdx.x * 1e-6f + j * 1e-3f;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (OP == 0) v[j] = fmaf(v[j], 0.999f, 1e-7f);
            else if constexpr (OP == 1) v[j] = __builtin_amdgcn_exp2f(v[j] * -0.001f);
            else if constexpr (OP == 2) v[j] = __builtin_amdgcn_rcpf(v[j] + 1.0f);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * sizeof(float));
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double ghz = p.clockRate / 1e6;
    const int blocks = cus * 8;
    const char* names[3] = {"v_fma_f32", "v_exp_f32", "v_rcp_f32"};
    for (int op = 0; op < 3; ++op) {
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (op == 0) hipLaunchKernelGGL(kern<0>, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
            if (op == 1) hipLaunchKernelGGL(kern<1>, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
            if (op == 2) hipLaunchKernelGGL(kern<2>, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double wave_insts = (double)blocks * 4 * ITERS * 8;     // waves x instructions (the main op)
        const double cycles = ms * 1e-3 * ghz * 1e9;
        printf("%-10s %8.3f ms  %6.3f wave-instructions / CU / cycle (clock %.2f GHz, %d CUs)\n", names[op], ms,
               wave_insts / cus / cycles, ghz, cus);
    }
    return 0;
}
