// extern "C" launchers of the RT-1 HIP kernels (csrc/kernels/*.hip).
// All take raw device pointers and the stream to launch on; they return the
// hipError_t of the launch (0 = success) and never synchronise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

int rt1_flat_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, float weight_decay, float step_size, float inv_sqrt_bc2, float grad_scale,
                  hipStream_t stream);

}  // extern "C"
