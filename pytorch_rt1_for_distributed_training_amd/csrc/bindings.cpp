// Python bindings for the RT-1 HIP kernels (module _rt1_hip).
//
// Kernels live in csrc/kernels/*.hip as plain HIP translation units exposing
// extern "C" launchers (raw pointers + hipStream_t); this file is the only one
// that sees torch headers.  Every binding validates shapes/dtypes/devices on
// the host BEFORE launching (a mis-shaped launch on a GPU box can fault the
// whole node) and launches on PyTorch's current HIP stream, so the ops compose
// with torch streams and hipGraph capture.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "rt1_kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_launch(int err, const char* what) {
    TORCH_CHECK(err == 0, what, ": HIP launch failed: ", hipGetErrorString((hipError_t)err));
}

void check_dev(const at::Tensor& t, const char* name, at::ScalarType dt) {
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void flat_adam(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, double lr, double beta1, double beta2,
               double eps, double weight_decay, double step_size, double inv_sqrt_bc2, double grad_scale) {
    check_dev(p, "param", at::kFloat);
    check_dev(g, "grad", at::kFloat);
    check_dev(m, "exp_avg", at::kFloat);
    check_dev(v, "exp_avg_sq", at::kFloat);
    const int64_t n = p.numel();
    TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "flat_adam: size mismatch");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(p.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(m.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(v.data_ptr()) % 16 == 0,
                "flat_adam: buffers must be 16-byte aligned");
    check_launch(rt1_flat_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), n,
                               (float)lr, (float)beta1, (float)beta2, (float)eps, (float)weight_decay,
                               (float)step_size, (float)inv_sqrt_bc2, (float)grad_scale, cur_stream()),
                 "flat_adam");
}

}  // namespace

PYBIND11_MODULE(_rt1_hip, m) {
    m.doc() = "RT-1 HIP/CDNA4 kernels (gfx950)";
    m.def("flat_adam", &flat_adam, "fused Adam/AdamW over flat fp32 buffers");
}
