// Python bindings for the RT-1 HIP kernels (module _rt1_hip).
//
// Kernels live in csrc/kernels/*.hip as plain HIP translation units exposing
// extern "C" launchers (raw pointers + hipStream_t); this file is the only one
// that sees torch headers.  Every binding validates shapes/dtypes/devices on
// the host BEFORE launching (a mis-shaped launch on a GPU box can fault the
// whole node) and launches on PyTorch's current HIP stream, so the ops compose
// with torch streams and hipGraph capture.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "rt1_kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// RT1_SYNC_CHECK=1: synchronise after every launch so an asynchronous fault is attributed to the op that
// launched it (the HIP_LAUNCH_BLOCKING-style debug mode; skipped while a hipGraph is being captured)
bool sync_check() {
    static const bool on = [] {
        const char* e = std::getenv("RT1_SYNC_CHECK");
        return e != nullptr && *e != '\0' && *e != '0';
    }();
    return on;
}

void check_launch(int err, const char* what) {
    TORCH_CHECK(err == 0, what, ": HIP launch failed: ", hipGetErrorString((hipError_t)err));
    if (sync_check()) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        hipStreamIsCapturing(c10::hip::getCurrentHIPStream().stream(), &cs);
        if (cs == hipStreamCaptureStatusNone) {
            const hipError_t e = hipDeviceSynchronize();
            TORCH_CHECK(e == hipSuccess, what, ": kernel failed (RT1_SYNC_CHECK): ", hipGetErrorString(e));
        }
    }
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


using OptT = c10::optional<at::Tensor>;
using Bf = uint16_t;

// optional device-resident dropout step counter (int32[1]); nullptr = host seed only
const uint32_t* seed_ptr(const OptT& t) {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "seed_dev must be a GPU int32 tensor");
    return reinterpret_cast<const uint32_t*>(t->data_ptr());
}

void flat_adam_dev(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor state, double beta1,
                   double beta2, double eps, double weight_decay, double grad_scale) {
    check_dev(p, "param", at::kFloat);
    check_dev(g, "grad", at::kFloat);
    check_dev(m, "exp_avg", at::kFloat);
    check_dev(v, "exp_avg_sq", at::kFloat);
    check_dev(state, "state", at::kFloat);
    const int64_t n = p.numel();
    TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && state.numel() >= 2, "flat_adam_dev: sizes");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(p.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(m.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(v.data_ptr()) % 16 == 0,
                "flat_adam_dev: buffers must be 16-byte aligned");
    check_launch(rt1_flat_adam_dev(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                                   n, state.data_ptr<float>(), (float)beta1, (float)beta2, (float)eps,
                                   (float)weight_decay, (float)grad_scale, cur_stream()),
                 "flat_adam_dev");
}

// Deterministic fixed-order sum over the rows of B x [R, C] (fp32 or bf16, contiguous) -> B x [C] fp32
// (csrc/kernels/reduce.hip).  Replaces ATen's tall-reduction path, whose cross-workgroup semaphore combine gave
// wrong weight gradients under hipGraph replay.
at::Tensor colsum3(const at::Tensor& x, int64_t B, int64_t R, int64_t C) {
    TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "colsum: contiguous GPU tensor required");
    TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "colsum: fp32 or bf16");
    TORCH_CHECK(B * R * C == x.numel() && C > 0 && C < (int64_t)1 << 31 && R > 0, "colsum: bad shape");
    if (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 != 0) return colsum3(x.clone(), B, R, C);   // vector loads
    auto out = at::empty({B, C}, x.options().dtype(at::kFloat));
    const int chunks = rt1_colsum_chunks(R, (int)C, (int)B);
    at::Tensor tmp;
    if (chunks > 1) tmp = at::empty({B, chunks, C}, out.options());
    check_launch(rt1_colsum(x.data_ptr(), x.scalar_type() == at::kBFloat16, R, (int)C, (int)B, out.data_ptr<float>(),
                            chunks > 1 ? tmp.data_ptr<float>() : nullptr, chunks, cur_stream()), "colsum");
    return out;
}
// sum over dim 0 of any contiguous tensor -> fp32 tensor of shape x.shape[1:]
at::Tensor sum0(const at::Tensor& x) {
    TORCH_CHECK(x.dim() >= 2, "sum0: need >= 2 dims");
    const int64_t R = x.size(0);
    const int64_t C = x.numel() / R;
    return colsum3(x, 1, R, C).view(x.sizes().slice(1));
}
at::Tensor colsum_py(at::Tensor x) { return sum0(x.contiguous()); }

// dst[i].copy_(src[i]) for contiguous GPU tensors of one dtype and equal numel whose sizes are whole 4-byte words,
// 128 copies per launch (the flat-gradient gather, the per-step Q/K/V weight packing)
void multi_copy_(std::vector<at::Tensor> dst, std::vector<at::Tensor> src) {
    TORCH_CHECK(dst.size() == src.size(), "multi_copy_: list lengths differ");
    std::vector<const float*> sp;
    std::vector<float*> dp;
    std::vector<int64_t> np;
    for (size_t i = 0; i < dst.size(); ++i) {
        const auto& d = dst[i];
        const auto& s = src[i];
        const int64_t nb = d.numel() * (int64_t)d.element_size();
        TORCH_CHECK(d.is_cuda() && s.is_cuda() && d.scalar_type() == s.scalar_type() && d.is_contiguous() &&
                    s.is_contiguous() && d.numel() == s.numel() && nb % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(d.data_ptr()) | reinterpret_cast<uintptr_t>(s.data_ptr())) & 3) == 0,
                    "multi_copy_: contiguous GPU tensors of one dtype, equal size, whole aligned 4-byte words (entry ",
                    i, ")");
        if (d.numel() == 0) continue;
        sp.push_back(reinterpret_cast<const float*>(s.data_ptr()));
        dp.push_back(reinterpret_cast<float*>(d.data_ptr()));
        np.push_back(nb / 4);
    }
    for (size_t o = 0; o < sp.size(); o += 128) {
        const int cnt = (int)std::min<size_t>(128, sp.size() - o);
        check_launch(rt1_multi_copy(sp.data() + o, dp.data() + o, np.data() + o, cnt, cur_stream()), "multi_copy_");
    }
}

// dst[i] = sum_k src[i].flat[k * sstride[i] : k * sstride[i] + dst[i].numel()] for k < splits[i] (fp32; src[i] is
// the first split's [..] view of a contiguous [splits, ..] partial tensor, splits 1 = a copy), MC_MAX per launch
void multi_reduce_copy_(std::vector<at::Tensor> dst, std::vector<at::Tensor> src, std::vector<int64_t> splits,
                        std::vector<int64_t> sstride) {
    TORCH_CHECK(dst.size() == src.size() && dst.size() == splits.size() && dst.size() == sstride.size(),
                "multi_reduce_copy_: list lengths differ");
    std::vector<const float*> sp;
    std::vector<float*> dp;
    std::vector<int64_t> np, ssp;
    std::vector<int> kp;
    for (size_t i = 0; i < dst.size(); ++i) {
        const auto& d = dst[i];
        const auto& s = src[i];
        TORCH_CHECK(d.is_cuda() && s.is_cuda() && d.scalar_type() == at::kFloat && s.scalar_type() == at::kFloat &&
                    d.is_contiguous() && s.is_contiguous() && d.numel() == s.numel() && splits[i] >= 1 &&
                    (splits[i] == 1 || sstride[i] >= s.numel()),
                    "multi_reduce_copy_: contiguous fp32 GPU tensors of equal size, splits >= 1 (entry ", i, ")");
        if (d.numel() == 0) continue;
        sp.push_back(s.data_ptr<float>());
        dp.push_back(d.data_ptr<float>());
        np.push_back(d.numel());
        ssp.push_back(sstride[i]);
        kp.push_back((int)splits[i]);
    }
    for (size_t o = 0; o < sp.size(); o += 128) {
        const int cnt = (int)std::min<size_t>(128, sp.size() - o);
        check_launch(rt1_multi_reduce_copy(sp.data() + o, dp.data() + o, np.data() + o, ssp.data() + o, kp.data() + o,
                                           cnt, cur_stream()), "multi_reduce_copy_");
    }
}

// raw [N, h, w, 3] uint8 frames + boxes [N, 4] int32 (x0, y0, x1, y1) -> [N, 3, H, W] uint8 (Pillow bilinear)
at::Tensor crop_resize_u8(at::Tensor raw, at::Tensor boxes, int64_t H, int64_t W) {
    TORCH_CHECK(raw.is_cuda() && raw.is_contiguous() && raw.scalar_type() == at::kByte && raw.dim() == 4 &&
                raw.size(3) == 3, "raw must be a contiguous [N, h, w, 3] uint8 GPU tensor");
    TORCH_CHECK(boxes.is_cuda() && boxes.is_contiguous() && boxes.scalar_type() == at::kInt && boxes.dim() == 2 &&
                boxes.size(0) == raw.size(0) && boxes.size(1) == 4, "boxes must be [N, 4] int32 on the GPU");
    TORCH_CHECK(H > 0 && W > 0 && raw.size(0) * H * W < ((int64_t)1 << 40), "bad output size");
    // the kernel keeps <= 16 Pillow filter taps per axis; a crop is at most the frame, so bound the worst case here
    auto taps = [](double src, double dst) { return (int)std::ceil(2.0 * std::max(src / dst, 1.0)) + 1; };
    TORCH_CHECK(taps((double)raw.size(1), (double)H) <= 16 && taps((double)raw.size(2), (double)W) <= 16,
                "crop_resize_u8: downscale from ", raw.size(1), "x", raw.size(2), " to ", H, "x", W,
                " needs more than 16 filter taps per axis; use the Pillow path (data.shards.gpu_crop_supported)");
    auto out = at::empty({raw.size(0), 3, H, W}, raw.options());
    if (raw.size(0) == 0) return out;
    check_launch(rt1_crop_resize_u8(raw.data_ptr<uint8_t>(), boxes.data_ptr<int>(), (int)raw.size(0),
                                    (int)raw.size(1), (int)raw.size(2), (int)H, (int)W, out.data_ptr<uint8_t>(),
                                    cur_stream()), "crop_resize_u8");
    return out;
}

// the same with the frames gathered by index from an HBM-resident frame table: raw [F, h, w, 3], rows [N] int64
// (data/resident.py: the batch's frames never cross PCIe)
at::Tensor crop_resize_gather_u8(at::Tensor raw, at::Tensor rows, at::Tensor boxes, int64_t H, int64_t W) {
    TORCH_CHECK(raw.is_cuda() && raw.is_contiguous() && raw.scalar_type() == at::kByte && raw.dim() == 4 &&
                raw.size(3) == 3 && raw.size(0) > 0, "raw must be a non-empty contiguous [F, h, w, 3] uint8 GPU tensor");
    TORCH_CHECK(rows.is_cuda() && rows.is_contiguous() && rows.scalar_type() == at::kLong && rows.dim() == 1,
                "rows must be a contiguous [N] int64 GPU tensor");
    TORCH_CHECK(boxes.is_cuda() && boxes.is_contiguous() && boxes.scalar_type() == at::kInt && boxes.dim() == 2 &&
                boxes.size(0) == rows.size(0) && boxes.size(1) == 4, "boxes must be [N, 4] int32 on the GPU");
    TORCH_CHECK(H > 0 && W > 0 && rows.size(0) * H * W < ((int64_t)1 << 40), "bad output size");
    auto taps = [](double src, double dst) { return (int)std::ceil(2.0 * std::max(src / dst, 1.0)) + 1; };
    TORCH_CHECK(taps((double)raw.size(1), (double)H) <= 16 && taps((double)raw.size(2), (double)W) <= 16,
                "crop_resize_gather_u8: downscale needs more than 16 filter taps per axis");
    auto out = at::empty({rows.size(0), 3, H, W}, raw.options());
    if (rows.size(0) == 0) return out;
    check_launch(rt1_crop_resize_gather_u8(raw.data_ptr<uint8_t>(), raw.size(0), rows.data_ptr<int64_t>(),
                                           boxes.data_ptr<int>(), (int)rows.size(0), (int)raw.size(1),
                                           (int)raw.size(2), (int)H, (int)W, out.data_ptr<uint8_t>(), cur_stream()),
                 "crop_resize_gather_u8");
    return out;
}

Bf* bp(const at::Tensor& t) { return reinterpret_cast<Bf*>(t.data_ptr()); }
const Bf* bpo(const OptT& t) { return t.has_value() && t->defined() ? reinterpret_cast<const Bf*>(t->data_ptr()) : nullptr; }
const float* fpo(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }
float* fpo_mut(OptT& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

void check_bf(const at::Tensor& t, const char* name) { check_dev(t, name, at::kBFloat16); }
void check_f(const at::Tensor& t, const char* name, int64_t numel) {
    check_dev(t, name, at::kFloat);
    TORCH_CHECK(numel < 0 || t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
}
void check_opt_f(const OptT& t, const char* name, int64_t numel) {
    if (t.has_value() && t->defined()) check_f(*t, name, numel);
}
void check_opt_bf(const OptT& t, const char* name, int64_t numel) {
    if (t.has_value() && t->defined()) {
        check_bf(*t, name);
        TORCH_CHECK(t->numel() == numel, name, " has ", t->numel(), " elements, expected ", numel);
    }
}
// [M, C] view of a channels-last activation (any leading dims), C % 8 == 0
std::pair<int64_t, int> rows_cols(const at::Tensor& t) {
    TORCH_CHECK(t.dim() >= 2, "activation must have >= 2 dims");
    const int C = (int)t.size(-1);
    TORCH_CHECK(C % 8 == 0, "channel count ", C, " must be a multiple of 8");
    return {t.numel() / C, C};
}
at::TensorOptions f32(const at::Tensor& like) { return like.options().dtype(at::kFloat); }

std::vector<at::Tensor> bn_stats(at::Tensor x, int64_t P) {
    check_bf(x, "x");
    auto [M, C] = rows_cols(x);
    TORCH_CHECK(P >= 1 && P <= 65535, "P out of range");
    auto ps = at::empty({P, C}, f32(x)), pq = at::empty({P, C}, f32(x));
    check_launch(rt1_bn_stats(bp(x), M, C, (int)P, ps.data_ptr<float>(), pq.data_ptr<float>(), cur_stream()), "bn_stats");
    return {ps, pq};
}

std::vector<at::Tensor> bn_finalize(at::Tensor ps, at::Tensor pq, double count, OptT gamma, OptT beta, double eps,
                                    double momentum, OptT rmean, OptT rvar) {
    check_f(ps, "psum", -1);
    check_f(pq, "psq", ps.numel());
    TORCH_CHECK(ps.dim() == 2, "partials must be [P, C]");
    const int P = (int)ps.size(0), C = (int)ps.size(1);
    check_opt_f(gamma, "gamma", C); check_opt_f(beta, "beta", C);
    check_opt_f(rmean, "running_mean", C); check_opt_f(rvar, "running_var", C);
    auto o = at::empty({4, C}, f32(ps));
    float* b = o.data_ptr<float>();
    check_launch(rt1_bn_finalize(ps.data_ptr<float>(), pq.data_ptr<float>(), P, C, count, fpo(gamma), fpo(beta),
                                 (float)eps, (float)momentum, fpo_mut(rmean), fpo_mut(rvar), b, b + C, b + 2 * C,
                                 b + 3 * C, cur_stream()), "bn_finalize");
    return {o[0], o[1], o[2], o[3]};
}

at::Tensor bn_apply(at::Tensor y, at::Tensor scale, at::Tensor shift, int64_t act, OptT rs, int64_t HW) {
    check_bf(y, "y");
    auto [M, C] = rows_cols(y);
    check_f(scale, "scale", C); check_f(shift, "shift", C);
    if (rs.has_value() && rs->defined()) {
        TORCH_CHECK(HW > 0 && M % HW == 0, "HW must divide the row count");
        check_f(*rs, "rs", (M / HW) * C);
    }
    auto out = at::empty_like(y);
    check_launch(rt1_bn_apply(bp(y), M, C, scale.data_ptr<float>(), shift.data_ptr<float>(), (int)act, fpo(rs), HW,
                              bp(out), cur_stream()), "bn_apply");
    return out;
}

void check_grad_mods(const OptT& rs, const OptT& rb, int64_t M, int C, int64_t HW) {
    if ((rs.has_value() && rs->defined()) || (rb.has_value() && rb->defined()))
        TORCH_CHECK(HW > 0 && M % HW == 0, "HW must divide the row count");
    check_opt_f(rs, "rs", HW > 0 ? (M / HW) * C : -1);
    check_opt_f(rb, "rb", HW > 0 ? (M / HW) * C : -1);
}

std::vector<at::Tensor> bn_bwd_reduce(at::Tensor G, OptT rs, OptT rb, int64_t HW, at::Tensor y, at::Tensor scale,
                                      at::Tensor shift, at::Tensor mean, at::Tensor rstd, int64_t act, int64_t P) {
    check_bf(G, "G"); check_bf(y, "y");
    auto [M, C] = rows_cols(y);
    TORCH_CHECK(G.numel() == y.numel(), "G/y size mismatch");
    check_grad_mods(rs, rb, M, C, HW);
    check_f(scale, "scale", C); check_f(shift, "shift", C); check_f(mean, "mean", C); check_f(rstd, "rstd", C);
    TORCH_CHECK(P >= 1 && P <= 65535, "P out of range");
    auto pa = at::empty({P, C}, f32(y)), pb = at::empty({P, C}, f32(y));
    check_launch(rt1_bn_bwd_reduce(bp(G), fpo(rs), fpo(rb), HW, bp(y), M, C, scale.data_ptr<float>(),
                                   shift.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)act,
                                   (int)P, pa.data_ptr<float>(), pb.data_ptr<float>(), cur_stream()), "bn_bwd_reduce");
    return {pa, pb};
}

std::vector<at::Tensor> bn_bwd_finalize(at::Tensor pa, at::Tensor pb, double count, OptT dgamma, OptT dbeta) {
    check_f(pa, "pdz", -1); check_f(pb, "pdzx", pa.numel());
    TORCH_CHECK(pa.dim() == 2, "partials must be [P, C]");
    const int P = (int)pa.size(0), C = (int)pa.size(1);
    check_opt_f(dgamma, "dgamma", C); check_opt_f(dbeta, "dbeta", C);
    auto o = at::empty({2, C}, f32(pa));
    check_launch(rt1_bn_bwd_finalize(pa.data_ptr<float>(), pb.data_ptr<float>(), P, C, count, fpo_mut(dgamma),
                                     fpo_mut(dbeta), o.data_ptr<float>(), o.data_ptr<float>() + C, cur_stream(), 1),
                 "bn_bwd_finalize");
    return {o[0], o[1]};
}

// same reduction, fresh outputs (no zero-filled accumulators): -> mdz, mdzx, dgamma, dbeta  (views of one [4, C])
std::vector<at::Tensor> bn_bwd_finalize_new(at::Tensor pa, at::Tensor pb, double count) {
    check_f(pa, "pdz", -1); check_f(pb, "pdzx", pa.numel());
    TORCH_CHECK(pa.dim() == 2, "partials must be [P, C]");
    const int P = (int)pa.size(0), C = (int)pa.size(1);
    auto o = at::empty({4, C}, f32(pa));
    float* b = o.data_ptr<float>();
    check_launch(rt1_bn_bwd_finalize(pa.data_ptr<float>(), pb.data_ptr<float>(), P, C, count, b + 2 * C, b + 3 * C, b,
                                     b + C, cur_stream(), 0),
                 "bn_bwd_finalize_new");
    return {o[0], o[1], o[2], o[3]};
}

// bn_bwd_finalize_new + the [5, C] constants of the fused expand backward (pwbwd.hip) in the same launch:
// {mdz, mdzx, dgamma, dbeta, consts = [scale, shift, gamma*rstd, -k1 rstd mdzx, -k1 (mdz - mean rstd mdzx)]}
std::vector<at::Tensor> bn_bwd_finalize_pw(at::Tensor pa, at::Tensor pb, double count, at::Tensor scale,
                                           at::Tensor shift, at::Tensor gamma, at::Tensor mean, at::Tensor rstd) {
    check_f(pa, "pdz", -1); check_f(pb, "pdzx", pa.numel());
    TORCH_CHECK(pa.dim() == 2, "partials must be [P, C]");
    const int P = (int)pa.size(0), C = (int)pa.size(1);
    check_f(scale, "scale", C); check_f(shift, "shift", C); check_f(gamma, "gamma", C); check_f(mean, "mean", C);
    check_f(rstd, "rstd", C);
    auto o = at::empty({4, C}, f32(pa));
    auto k = at::empty({5, C}, f32(pa));
    float* b = o.data_ptr<float>();
    check_launch(rt1_bn_bwd_finalize_consts(pa.data_ptr<float>(), pb.data_ptr<float>(), P, C, count, b + 2 * C,
                                            b + 3 * C, b, b + C, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                            gamma.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                            k.data_ptr<float>(), cur_stream()),
                 "bn_bwd_finalize_pw");
    return {o[0], o[1], o[2], o[3], k};
}

at::Tensor bn_bwd_apply(at::Tensor G, OptT rs, OptT rb, int64_t HW, at::Tensor y, at::Tensor scale, at::Tensor shift,
                        at::Tensor mean, at::Tensor rstd, OptT gamma, int64_t act, at::Tensor mdz, at::Tensor mdzx,
                        OptT keep) {
    check_bf(G, "G"); check_bf(y, "y");
    auto [M, C] = rows_cols(y);
    TORCH_CHECK(G.numel() == y.numel(), "G/y size mismatch");
    check_grad_mods(rs, rb, M, C, HW);
    check_f(scale, "scale", C); check_f(shift, "shift", C); check_f(mean, "mean", C); check_f(rstd, "rstd", C);
    check_opt_f(gamma, "gamma", C); check_f(mdz, "mdz", C); check_f(mdzx, "mdzx", C);
    const bool has_keep = keep.has_value() && keep->defined();
    if (has_keep) {
        TORCH_CHECK(rs.has_value() && rs->defined() && HW > 0, "bn_bwd_apply: keep scales rs (needs rs and HW)");
        check_f(*keep, "keep", M / HW);
    }
    auto dy = at::empty_like(y);
    check_launch(rt1_bn_bwd_apply(bp(G), fpo(rs), fpo(rb), HW, bp(y), M, C, scale.data_ptr<float>(),
                                  shift.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), fpo(gamma),
                                  (int)act, mdz.data_ptr<float>(), mdzx.data_ptr<float>(), bp(dy), cur_stream(),
                                  has_keep ? keep->data_ptr<float>() : nullptr),
                 "bn_bwd_apply");
    return dy;
}

void check_nhwc(const at::Tensor& x, const char* name) {
    check_bf(x, name);
    TORCH_CHECK(x.dim() == 4, name, " must be [N, H, W, C]");
    TORCH_CHECK(x.size(3) % 8 == 0, name, " channels must be a multiple of 8");
}

std::vector<at::Tensor> dw_fwd(at::Tensor x, at::Tensor w, OptT scale, OptT shift, int64_t act, int64_t k, int64_t s,
                               int64_t max_blocks) {
    check_nhwc(x, "x");
    TORCH_CHECK((k == 3 || k == 5) && (s == 1 || s == 2), "dwconv supports k in {3,5}, s in {1,2}");
    const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3);
    check_f(w, "w", (int64_t)C * k * k);
    check_opt_f(scale, "scale", C); check_opt_f(shift, "shift", C);
    TORCH_CHECK(scale.has_value() == shift.has_value(), "scale/shift must be given together");
    const int p = (int)(k - 1) / 2;
    const int Ho = (H + 2 * p - (int)k) / (int)s + 1, Wo = (W + 2 * p - (int)k) / (int)s + 1;
    const bool pro = scale.has_value() && scale->defined();
    const int gx = rt1_dw_grid(N, H, W, C, (int)k, (int)s, (int)max_blocks, pro, 0);
    auto out = at::empty({N, Ho, Wo, C}, x.options());
    auto ps = at::empty({gx, C}, f32(x)), pq = at::empty({gx, C}, f32(x));
    check_launch(rt1_dw_fwd(bp(x), w.data_ptr<float>(), fpo(scale), fpo(shift), (int)act, N, H, W, C, (int)k, (int)s,
                            gx, bp(out), ps.data_ptr<float>(), pq.data_ptr<float>(), cur_stream()),
                 "dw_fwd");
    return {out, ps, pq};
}

std::vector<at::Tensor> dw_bwd_data(at::Tensor dy, at::Tensor w, int64_t H, int64_t W, int64_t k, int64_t s, OptT y_in,
                                    OptT scale, OptT shift, OptT mean, OptT rstd, int64_t max_blocks) {
    check_nhwc(dy, "dy");
    TORCH_CHECK((k == 3 || k == 5) && (s == 1 || s == 2), "dwconv supports k in {3,5}, s in {1,2}");
    const int N = (int)dy.size(0), C = (int)dy.size(3);
    const int p = (int)(k - 1) / 2;
    TORCH_CHECK(dy.size(1) == (H + 2 * p - k) / s + 1 && dy.size(2) == (W + 2 * p - k) / s + 1, "dy spatial mismatch");
    check_f(w, "w", (int64_t)C * k * k);
    const bool epi = y_in.has_value() && y_in->defined();
    if (epi) {
        check_opt_bf(y_in, "y_in", (int64_t)N * H * W * C);
        check_f(*scale, "scale", C); check_f(*shift, "shift", C); check_f(*mean, "mean", C); check_f(*rstd, "rstd", C);
    }
    const int gx = rt1_dw_bwd_grid(N, (int)H, (int)W, C, (int)k, (int)s, (int)max_blocks, epi ? 1 : 0);
    auto dx = at::empty({N, H, W, C}, dy.options());
    at::Tensor pa, pb;
    if (epi) { pa = at::empty({gx, C}, f32(dy)); pb = at::empty({gx, C}, f32(dy)); }
    auto wflip = w.view({C, k * k}).flip({1}).contiguous();
    check_launch(rt1_dw_bwd_data(bp(dy), w.data_ptr<float>(), wflip.data_ptr<float>(), N, (int)H, (int)W, C, (int)k,
                                 (int)s, gx, bp(dx), bpo(y_in),
                                 epi ? scale->data_ptr<float>() : nullptr, epi ? shift->data_ptr<float>() : nullptr,
                                 epi ? mean->data_ptr<float>() : nullptr, epi ? rstd->data_ptr<float>() : nullptr,
                                 epi ? pa.data_ptr<float>() : nullptr, epi ? pb.data_ptr<float>() : nullptr,
                                 cur_stream()), "dw_bwd_data");
    if (epi) return {dx, pa, pb};
    return {dx};
}

at::Tensor dw_bwd_weight(at::Tensor dy, at::Tensor x, OptT scale, OptT shift, int64_t act, int64_t k, int64_t s,
                         int64_t max_blocks) {
    check_nhwc(dy, "dy"); check_nhwc(x, "x");
    TORCH_CHECK((k == 3 || k == 5) && (s == 1 || s == 2), "dwconv supports k in {3,5}, s in {1,2}");
    const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3);
    const int p = (int)(k - 1) / 2;
    TORCH_CHECK(dy.size(0) == N && dy.size(3) == C && dy.size(1) == (H + 2 * p - k) / s + 1 &&
                dy.size(2) == (W + 2 * p - k) / s + 1, "dy/x shape mismatch");
    check_opt_f(scale, "scale", C); check_opt_f(shift, "shift", C);
    const int gx = rt1_dw_wgrad_grid(N, H, W, C, (int)k, (int)s, (int)max_blocks, scale.has_value() && scale->defined());
    auto part = at::empty({gx, (int64_t)C * k * k}, f32(x));
    check_launch(rt1_dw_bwd_weight(bp(dy), bp(x), fpo(scale), fpo(shift), (int)act, N, H, W, C, (int)k, (int)s, gx,
                                   part.data_ptr<float>(), cur_stream()), "dw_bwd_weight");
    return sum0(part).view({C, k * k});
}

// Whole stride-1 depthwise backward in one pass (dwconv.hip dw_bwd_fused_kernel): dy = BN2-backward-apply(dA, y2)
// is rebuilt in the staging prologue (gate / rb [N, C]; BN2 scale, shift, mean, rstd, gamma, mdz, mdzx [C]) and
// feeds both dx = dwconv^T(dy) and dW = sum dy (x) act(x1*scale1+shift1).  mean1/rstd1 select the BN1 epilogue
// (expand blocks, x1 = y1): returns {dx, dW [C, k*k], pdz, pdzx}; otherwise {dx, dW}.
std::vector<at::Tensor> dw_bwd_fused(at::Tensor dA, at::Tensor y2, at::Tensor gate, at::Tensor rb, at::Tensor sc2,
                                     at::Tensor sh2, at::Tensor mu2, at::Tensor rs2, at::Tensor g2, at::Tensor mdz2,
                                     at::Tensor mdzx2, at::Tensor w, int64_t k, at::Tensor x1, OptT sc1, OptT sh1,
                                     int64_t act1, OptT mu1, OptT rs1, int64_t max_blocks,
                                     int64_t variant, bool zout, OptT res, OptT rmul) {
    check_nhwc(dA, "dA"); check_nhwc(y2, "y2"); check_nhwc(x1, "x1");
    const Bf* y2p = bp(y2);
    TORCH_CHECK(k == 3 || k == 5, "dw_bwd_fused: k in {3,5}");
    const int N = (int)x1.size(0), H = (int)x1.size(1), W = (int)x1.size(2), C = (int)x1.size(3);
    const int p = (int)(k - 1) / 2;
    // stride from the shapes: dA / y2 at the input resolution (s = 1) or at the stride-2 output resolution
    const bool s2 = dA.size(1) != H || dA.size(2) != W;
    if (s2) {
        TORCH_CHECK(dA.size(0) == N && dA.size(3) == C && dA.size(1) == (H + 2 * p - k) / 2 + 1 &&
                    dA.size(2) == (W + 2 * p - k) / 2 + 1 && y2.sizes() == dA.sizes(),
                    "dw_bwd_fused: dA, y2 must be [N, H, W, C] (stride 1) or the stride-2 output of x1");
    } else {
        TORCH_CHECK(dA.sizes() == x1.sizes() && y2.sizes() == x1.sizes(),
                    "dw_bwd_fused: dA, y2, x1 must share [N, H, W, C]");
    }
    check_f(gate, "gate", (int64_t)N * C); check_f(rb, "rb", (int64_t)N * C);
    check_f(sc2, "sc2", C); check_f(sh2, "sh2", C); check_f(mu2, "mu2", C); check_f(rs2, "rs2", C);
    check_f(g2, "g2", C); check_f(mdz2, "mdz2", C); check_f(mdzx2, "mdzx2", C);
    check_f(w, "w", (int64_t)C * k * k);
    check_opt_f(sc1, "sc1", C); check_opt_f(sh1, "sh1", C);
    const bool pro = sc1.has_value() && sc1->defined();
    TORCH_CHECK(!pro || (sh1.has_value() && sh1->defined()), "dw_bwd_fused: sh1 needed with sc1");
    const bool epi = mu1.has_value() && mu1->defined();
    if (epi) {
        TORCH_CHECK(pro, "dw_bwd_fused: the BN1 epilogue needs sc1/sh1");
        check_f(*mu1, "mu1", C); check_f(*rs1, "rs1", C);
    }
    if (s2) TORCH_CHECK(pro == epi, "dw_bwd_fused (stride 2): the BN1+SiLU operand and the BN1 epilogue go together");
    TORCH_CHECK(!zout || epi, "dw_bwd_fused: zout (store dz) needs the BN1 epilogue");
    const bool has_res = res.has_value() && res->defined();
    if (has_res) {
        // dx += res * rmul[n, c] in the unified stride-1 kernel's plain store (non-expand residual blocks)
        TORCH_CHECK(!s2 && !epi && !pro && rt1_dw_bwd_uses_uni((int)variant, 0, 0),
                    "dw_bwd_fused: the residual epilogue is for the unified stride-1 kernel without BN1");
        check_nhwc(*res, "res");
        TORCH_CHECK(res->sizes() == x1.sizes(), "dw_bwd_fused: res must be [N, H, W, C]");
        TORCH_CHECK(rmul.has_value() && rmul->defined(), "dw_bwd_fused: res needs rmul");
        check_f(*rmul, "rmul", (int64_t)N * C);
    }
    const int gx = s2 ? rt1_dw_bwd_fused_s2_grid(N, H, W, C, (int)k, (int)max_blocks, epi ? 1 : 0, 0)
                      : rt1_dw_bwd_fused_grid(N, H, W, C, (int)k, (int)max_blocks, pro ? 1 : 0, epi ? 1 : 0, (int)variant,
                                              0);
    auto dx = at::empty({N, H, W, C}, x1.options());
    auto part = at::empty({gx, (int64_t)C * k * k}, f32(x1));
    at::Tensor pa, pb;
    if (epi) { pa = at::empty({gx, C}, f32(x1)); pb = at::empty({gx, C}, f32(x1)); }
    if (s2) {
        TORCH_CHECK(!epi || act1 == 1, "dw_bwd_fused (stride 2): the operand prologue is BN + SiLU");
        check_launch(rt1_dw_bwd_fused_s2(bp(dA), y2p, gate.data_ptr<float>(), rb.data_ptr<float>(),
                                         sc2.data_ptr<float>(), sh2.data_ptr<float>(), mu2.data_ptr<float>(),
                                         rs2.data_ptr<float>(), g2.data_ptr<float>(), mdz2.data_ptr<float>(),
                                         mdzx2.data_ptr<float>(), w.data_ptr<float>(), bp(x1), fpo(sc1), fpo(sh1),
                                         epi ? mu1->data_ptr<float>() : nullptr, epi ? rs1->data_ptr<float>() : nullptr,
                                         N, H, W, C, (int)k, gx, bp(dx), epi ? pa.data_ptr<float>() : nullptr,
                                         epi ? pb.data_ptr<float>() : nullptr, part.data_ptr<float>(), cur_stream(),
                                         zout ? 1 : 0, nullptr, nullptr, 0),
                     "dw_bwd_fused_s2");
        auto dw = sum0(part).view({C, k * k});
        if (epi) return {dx, dw, pa, pb};
        return {dx, dw};
    }
    // the unified kernel flips the taps itself; only the two-pass kernel takes a flipped copy
    at::Tensor wflip;
    if (!rt1_dw_bwd_uses_uni((int)variant, pro ? 1 : 0, epi ? 1 : 0)) wflip = w.view({C, k * k}).flip({1}).contiguous();
    check_launch(rt1_dw_bwd_fused(bp(dA), y2p, gate.data_ptr<float>(), rb.data_ptr<float>(), sc2.data_ptr<float>(),
                                  sh2.data_ptr<float>(), mu2.data_ptr<float>(), rs2.data_ptr<float>(),
                                  g2.data_ptr<float>(), mdz2.data_ptr<float>(), mdzx2.data_ptr<float>(),
                                  w.data_ptr<float>(), wflip.defined() ? wflip.data_ptr<float>() : nullptr, bp(x1), fpo(sc1), fpo(sh1), (int)act1,
                                  epi ? mu1->data_ptr<float>() : nullptr, epi ? rs1->data_ptr<float>() : nullptr, N, H,
                                  W, C, (int)k, gx, bp(dx), epi ? pa.data_ptr<float>() : nullptr,
                                  epi ? pb.data_ptr<float>() : nullptr, part.data_ptr<float>(), cur_stream(), (int)variant,
                                  zout ? 1 : 0, nullptr, nullptr, 0, has_res ? bp(*res) : nullptr,
                                  has_res ? rmul->data_ptr<float>() : nullptr),
                 "dw_bwd_fused");
    auto dw = sum0(part).view({C, k * k});
    if (epi) return {dx, dw, pa, pb};
    return {dx, dw};
}

// ---- y1-free expand blocks (x-mode): the depthwise kernels recompute y1 = x @ we^T on MFMA per staged tile
// the depthwise tile a layer gets: which = 0 forward, 1 unified backward; cin > 0 = x-mode -> [TH, TW, LDS bytes, sb]
std::vector<int64_t> dw_tile_info(int64_t which, int64_t H, int64_t W, int64_t C, int64_t k, int64_t s, int64_t cin) {
    int out[4] = {0, 0, 0, 0};
    TORCH_CHECK(rt1_dw_tile_info((int)which, (int)H, (int)W, (int)C, (int)k, (int)s, (int)cin, out) == 0,
                "dw_tile_info: no tile for this layer");
    return {out[0], out[1], out[2], out[3]};
}

bool dw_x_supported(int64_t cin, int64_t C, int64_t k, int64_t s) {
    return rt1_dw_x_supported((int)cin, (int)C, (int)k, (int)s) != 0;
}

void check_xexp(const at::Tensor& x, const at::Tensor& we, int64_t C) {
    check_nhwc(x, "x");
    check_bf(we, "we");
    TORCH_CHECK(we.dim() == 2 && we.size(0) == C && we.size(1) == x.size(3), "we must be [Ce, Cin] matching x");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(we.data_ptr()) % 16 == 0,
                "x / we must be 16-byte aligned");
}

// out = dwconv(silu(bn1(x @ we^T))) (BN1 constants sc1 / sh1), BN2 partial statistics -> {out, ps, pq}
std::vector<at::Tensor> dw_fwd_x(at::Tensor x, at::Tensor we, at::Tensor w, at::Tensor sc1, at::Tensor sh1, int64_t k,
                                 int64_t s, int64_t max_blocks) {
    const int C = (int)we.size(0);
    check_xexp(x, we, C);
    const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), cin = (int)x.size(3);
    TORCH_CHECK(rt1_dw_x_supported(cin, C, (int)k, (int)s), "dw_fwd_x: no x-mode specialisation for Cin=", cin,
                " C=", C, " k=", k, " s=", s);
    check_f(w, "w", (int64_t)C * k * k); check_f(sc1, "sc1", C); check_f(sh1, "sh1", C);
    const int p = (int)(k - 1) / 2;
    const int Ho = (H + 2 * p - (int)k) / (int)s + 1, Wo = (W + 2 * p - (int)k) / (int)s + 1;
    const int gx = rt1_dw_grid_x(N, H, W, C, (int)k, (int)s, cin, (int)max_blocks);
    auto out = at::empty({N, Ho, Wo, C}, x.options());
    auto ps = at::empty({gx, C}, f32(x)), pq = at::empty({gx, C}, f32(x));
    check_launch(rt1_dw_fwd_x(bp(x), cin, bp(we), w.data_ptr<float>(), sc1.data_ptr<float>(), sh1.data_ptr<float>(), N,
                              H, W, C, (int)k, (int)s, gx, bp(out), ps.data_ptr<float>(), pq.data_ptr<float>(),
                              cur_stream()), "dw_fwd_x");
    return {out, ps, pq};
}

// dw_bwd_fused of an x-mode expand block: the strip centres' y1 is recomputed from (x, we) instead of read; always
// the unified kernel with the BN1 epilogue -> {dx or dz (zout), dW, pdz, pdzx}
std::vector<at::Tensor> dw_bwd_fused_x(at::Tensor dA, at::Tensor y2, at::Tensor gate, at::Tensor rb, at::Tensor sc2,
                                       at::Tensor sh2, at::Tensor mu2, at::Tensor rs2, at::Tensor g2, at::Tensor mdz2,
                                       at::Tensor mdzx2, at::Tensor w, int64_t k, at::Tensor x, at::Tensor we,
                                       at::Tensor sc1, at::Tensor sh1, at::Tensor mu1, at::Tensor rs1,
                                       int64_t max_blocks, bool zout) {
    const int C = (int)we.size(0);
    check_xexp(x, we, C);
    check_nhwc(dA, "dA"); check_nhwc(y2, "y2");
    const Bf* y2p = bp(y2);
    TORCH_CHECK(k == 3 || k == 5, "dw_bwd_fused_x: k in {3,5}");
    const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), cin = (int)x.size(3);
    const int p = (int)(k - 1) / 2;
    const bool s2 = dA.size(1) != H || dA.size(2) != W;
    const int s = s2 ? 2 : 1;
    TORCH_CHECK(dA.size(0) == N && dA.size(3) == C && dA.size(1) == (H + 2 * p - k) / s + 1 &&
                dA.size(2) == (W + 2 * p - k) / s + 1 && y2.sizes() == dA.sizes(),
                "dw_bwd_fused_x: dA, y2 must be the depthwise output of x's map with C channels");
    TORCH_CHECK(rt1_dw_x_supported(cin, C, (int)k, s), "dw_bwd_fused_x: no x-mode specialisation for Cin=", cin,
                " C=", C, " k=", k, " s=", s);
    check_f(gate, "gate", (int64_t)N * C); check_f(rb, "rb", (int64_t)N * C);
    check_f(sc2, "sc2", C); check_f(sh2, "sh2", C); check_f(mu2, "mu2", C); check_f(rs2, "rs2", C);
    check_f(g2, "g2", C); check_f(mdz2, "mdz2", C); check_f(mdzx2, "mdzx2", C);
    check_f(w, "w", (int64_t)C * k * k);
    check_f(sc1, "sc1", C); check_f(sh1, "sh1", C); check_f(mu1, "mu1", C); check_f(rs1, "rs1", C);
    const int gx = s2 ? rt1_dw_bwd_fused_s2_grid(N, H, W, C, (int)k, (int)max_blocks, 1, cin)
                      : rt1_dw_bwd_fused_grid(N, H, W, C, (int)k, (int)max_blocks, 1, 1, 1, cin);
    auto dx = at::empty({N, H, W, C}, x.options());
    auto part = at::empty({gx, (int64_t)C * k * k}, f32(x));
    auto pa = at::empty({gx, C}, f32(x)), pb = at::empty({gx, C}, f32(x));
    if (s2) {
        check_launch(rt1_dw_bwd_fused_s2(bp(dA), y2p, gate.data_ptr<float>(), rb.data_ptr<float>(),
                                         sc2.data_ptr<float>(), sh2.data_ptr<float>(), mu2.data_ptr<float>(),
                                         rs2.data_ptr<float>(), g2.data_ptr<float>(), mdz2.data_ptr<float>(),
                                         mdzx2.data_ptr<float>(), w.data_ptr<float>(), nullptr, sc1.data_ptr<float>(),
                                         sh1.data_ptr<float>(), mu1.data_ptr<float>(), rs1.data_ptr<float>(), N, H, W, C,
                                         (int)k, gx, bp(dx), pa.data_ptr<float>(), pb.data_ptr<float>(),
                                         part.data_ptr<float>(), cur_stream(), zout ? 1 : 0, bp(x), bp(we), cin),
                     "dw_bwd_fused_x (stride 2)");
    } else {
        check_launch(rt1_dw_bwd_fused(bp(dA), y2p, gate.data_ptr<float>(), rb.data_ptr<float>(), sc2.data_ptr<float>(),
                                      sh2.data_ptr<float>(), mu2.data_ptr<float>(), rs2.data_ptr<float>(),
                                      g2.data_ptr<float>(), mdz2.data_ptr<float>(), mdzx2.data_ptr<float>(),
                                      w.data_ptr<float>(), nullptr, nullptr, sc1.data_ptr<float>(), sh1.data_ptr<float>(),
                                      1, mu1.data_ptr<float>(), rs1.data_ptr<float>(), N, H, W, C, (int)k, gx, bp(dx),
                                      pa.data_ptr<float>(), pb.data_ptr<float>(), part.data_ptr<float>(), cur_stream(), 1,
                                      zout ? 1 : 0, bp(x), bp(we), cin),
                     "dw_bwd_fused_x");
    }
    return {dx, sum0(part).view({C, k * k}), pa, pb};
}

// C = pro(A) . op(B) (+ bias) on the tiled MFMA GEMM (gemm.hip).  A [M, K] bf16; B bf16 [N, K] (nn = false: a
// weight, C = A W^T) or [K, N] (nn = true: C = A B).  pro = (scale [K], shift [K], gate [M / hw, K], hw) rebuilds
// A as silu(A * scale + shift) * gate in the operand load.  stats: also the per-M-tile column sum / sum of squares
// of the stored bf16 C -> {C, ps, pq}; else {C}; store_a appends the rebuilt operand A [M, K] (prologue only).
std::vector<at::Tensor> gemm(at::Tensor A, at::Tensor B, bool nn, OptT bias, OptT scale, OptT shift, OptT gate,
                             int64_t hw, bool out_f32, bool stats, int64_t cfg, bool store_a) {
    check_bf(A, "A"); check_bf(B, "B");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "gemm: 2-D operands");
    const int64_t M = A.size(0), K = A.size(1);
    const int64_t N = nn ? B.size(1) : B.size(0);
    TORCH_CHECK((nn ? B.size(0) : B.size(1)) == K, "gemm: inner dimensions differ");
    TORCH_CHECK(M > 0 && N % 8 == 0 && K % 8 == 0 && N > 0 && K > 0, "gemm: N and K must be multiples of 8");
    TORCH_CHECK(M < ((int64_t)1 << 31) && N * K < ((int64_t)1 << 31), "gemm: too large");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
                "gemm: operands must be 16-byte aligned");
    check_opt_f(bias, "bias", N);
    const bool pro = scale.has_value() && scale->defined();
    if (pro) {
        check_f(*scale, "scale", K); check_f(*shift, "shift", K);
        TORCH_CHECK(hw > 0 && M % hw == 0, "gemm: hw must divide M");
        check_f(*gate, "gate", (M / hw) * K);
        TORCH_CHECK(!out_f32, "gemm: the prologue path writes bf16");
    }
    TORCH_CHECK(!(stats && out_f32), "gemm: statistics describe a bf16 output");
    TORCH_CHECK(!store_a || pro, "gemm: store_a stores the prologue's rebuilt operand");
    auto C = at::empty({M, N}, A.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
    at::Tensor aout;
    if (store_a) aout = at::empty_like(A);
    at::Tensor ps, pq;
    if (stats) {
        const int tm = rt1_gemm_tiles_m((int)M, (int)N, (int)K, (int)cfg);
        ps = at::empty({tm, N}, f32(A));
        pq = at::empty({tm, N}, f32(A));
    }
    check_launch(rt1_gemm(bp(A), bp(B), C.data_ptr(), (int)M, (int)N, (int)K, nn ? 1 : 0, fpo(bias), fpo(scale),
                          fpo(shift), fpo(gate), (int)hw, out_f32 ? 1 : 0, stats ? ps.data_ptr<float>() : nullptr,
                          stats ? pq.data_ptr<float>() : nullptr, (int)cfg, store_a ? bp(aout) : nullptr,
                          cur_stream()), "gemm");
    std::vector<at::Tensor> out{C};
    if (stats) { out.push_back(ps); out.push_back(pq); }
    if (store_a) out.push_back(aout);
    return out;
}

// FiLM projections of every block at once: xe [M, lda] bf16 (the context embedding, cast once per step),
// w [N, K] bf16 (the packed projection weights, K <= lda), bias [N] fp32, cmap [N / 4, 4] int32 (rt1_gemm_cmap) ->
// flat fp32 [total] with each block's slice laid out as its own contiguous [M, C] array
at::Tensor film_fwd(at::Tensor xe, int64_t K, at::Tensor w, at::Tensor bias, at::Tensor cmap, int64_t total,
                    int64_t cfg) {
    check_bf(xe, "xe"); check_bf(w, "w");
    TORCH_CHECK(xe.dim() == 2 && w.dim() == 2 && w.size(1) == K && K <= xe.size(1), "film_fwd: xe [M, >= K], w [N, K]");
    const int64_t M = xe.size(0), N = w.size(0);
    TORCH_CHECK(M > 0 && N % 8 == 0 && K % 8 == 0 && xe.size(1) % 8 == 0, "film_fwd: N, K, lda multiples of 8");
    check_f(bias, "bias", N);
    TORCH_CHECK(cmap.is_cuda() && cmap.is_contiguous() && cmap.scalar_type() == at::kInt && cmap.numel() == N,
                "film_fwd: cmap must be an int32 [N / 4, 4] GPU tensor");
    TORCH_CHECK(total == M * N, "film_fwd: total must be M * N");
    auto out = at::empty({total}, f32(xe));
    check_launch(rt1_gemm_cmap(bp(xe), (int)xe.size(1), bp(w), out.data_ptr<float>(), (int)M, (int)N, (int)K,
                               bias.data_ptr<float>(), cmap.data_ptr<int>(), (int)cfg, cur_stream()), "film_fwd");
    return out;
}

// ... and its weight / bias gradients: dflat fp32 [M * N] in the cmap layout, xe [M, >= K] bf16 -> {dW [N, K], db [N]}
std::vector<at::Tensor> film_wgrad(at::Tensor dflat, at::Tensor cmap, at::Tensor xe, int64_t K, int64_t splits,
                                   int64_t tile) {
    check_bf(xe, "xe");
    TORCH_CHECK(xe.dim() == 2 && K <= xe.size(1), "film_wgrad: xe [M, >= K]");
    const int64_t M = xe.size(0), N = cmap.numel();
    check_f(dflat, "dflat", M * N);
    TORCH_CHECK(cmap.is_cuda() && cmap.is_contiguous() && cmap.scalar_type() == at::kInt && N % 8 == 0 && K % 8 == 0,
                "film_wgrad: cmap int32 [N / 4, 4], N and K multiples of 8");
    auto a = xe.size(1) == K ? xe : xe.narrow(1, 0, K).contiguous();
    const int s = (int)std::max<int64_t>(1, std::min<int64_t>(splits, (M + 63) / 64));
    auto part = at::empty({s, N, K}, f32(xe));
    auto dbp = at::empty({s, N}, f32(xe));
    check_launch(rt1_wgrad_dymap(dflat.data_ptr<float>(), cmap.data_ptr<int>(), bp(a), M, (int)N, (int)K, s,
                                 part.data_ptr<float>(), dbp.data_ptr<float>(), (int)tile, cur_stream()),
                 "film_wgrad");
    if (s == 1) return {part[0], dbp[0]};
    return {sum0(part), sum0(dbp)};
}

// C = pro(A) @ op(B) (+ bias) on gemm256.hip (256-row tiles, LDS-DMA, 8 waves): A [M, K] bf16, B [N, K] (nn = false)
// or [K, N] (nn = true) bf16 -> [C] (+ [ps, pq] BN-stat partials [tiles_m, N]) (+ [aout] the rebuilt PRO operand)
std::vector<at::Tensor> gemm256(at::Tensor A, at::Tensor B, bool nn, OptT bias, OptT scale, OptT shift, OptT gate,
                                int64_t hw, bool stats, bool store_a, int64_t bn) {
    check_bf(A, "A"); check_bf(B, "B");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "gemm256: 2-D operands");
    const int64_t M = A.size(0), K = A.size(1);
    const int64_t N = nn ? B.size(1) : B.size(0);
    TORCH_CHECK((nn ? B.size(0) : B.size(1)) == K, "gemm256: inner dimensions differ");
    TORCH_CHECK(M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0, "gemm256: N and K must be multiples of 8");
    TORCH_CHECK(M < ((int64_t)1 << 31) && M * K < ((int64_t)1 << 40), "gemm256: too large");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
                "gemm256: operands must be 16-byte aligned");
    TORCH_CHECK(bn == 128 || bn == 256, "gemm256: bn must be 128 or 256");
    check_opt_f(bias, "bias", N);
    const bool pro = scale.has_value() && scale->defined();
    if (pro) {
        TORCH_CHECK(!nn, "gemm256: the operand prologue is an NT path");
        check_f(*scale, "scale", K); check_f(*shift, "shift", K);
        TORCH_CHECK(hw > 0 && M % hw == 0, "gemm256: hw must divide M");
        check_f(*gate, "gate", (M / hw) * K);
    }
    TORCH_CHECK(!store_a || pro, "gemm256: store_a stores the prologue's rebuilt operand");
    TORCH_CHECK(!(nn && (stats || (bias.has_value() && bias->defined()))), "gemm256: NN is a plain product");
    auto C = at::empty({M, N}, A.options().dtype(at::kBFloat16));
    at::Tensor aout, ps, pq;
    if (store_a) aout = at::empty_like(A);
    if (stats) {
        const int tm = rt1_g256_tiles_m((int)M);
        ps = at::empty({tm, N}, f32(A));
        pq = at::empty({tm, N}, f32(A));
    }
    check_launch(rt1_g256(bp(A), bp(B), bp(C), (int)M, (int)N, (int)K, nn ? 1 : 0, fpo(bias), fpo(scale), fpo(shift),
                          fpo(gate), (int)hw, store_a ? bp(aout) : nullptr, stats ? ps.data_ptr<float>() : nullptr,
                          stats ? pq.data_ptr<float>() : nullptr, (int)bn, cur_stream()), "gemm256");
    std::vector<at::Tensor> out{C};
    if (stats) { out.push_back(ps); out.push_back(pq); }
    if (store_a) out.push_back(aout);
    return out;
}

// C = A @ B^T + A2 @ B2^T + bias (+ res * rmul[m / rhw]) on gemm.hip (A [M, K], B [N, K], A2 [M, K2], B2 [N, K2] bf16,
// bias [N] fp32, res [M, N] bf16, rmul [M / rhw, N] fp32) -> C [M, N] bf16
at::Tensor gemm_tail(at::Tensor A, at::Tensor B, at::Tensor A2, at::Tensor B2, OptT bias, OptT res, OptT rmul,
                     int64_t rhw, int64_t cfg) {
    check_bf(A, "A"); check_bf(B, "B"); check_bf(A2, "A2"); check_bf(B2, "B2");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A2.dim() == 2 && B2.dim() == 2, "gemm_tail: 2-D operands");
    const int64_t M = A.size(0), K = A.size(1), N = B.size(0), K2 = A2.size(1);
    TORCH_CHECK(B.size(1) == K && A2.size(0) == M && B2.size(0) == N && B2.size(1) == K2, "gemm_tail: shapes");
    TORCH_CHECK(N % 8 == 0 && K % 8 == 0 && K2 % 8 == 0, "gemm_tail: N, K, K2 must be multiples of 8");
    TORCH_CHECK(M < ((int64_t)1 << 31), "gemm_tail: too large");
    for (const at::Tensor* t : {&A, &B, &A2, &B2})
        TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_tail: operands must be 16-byte aligned");
    check_opt_f(bias, "bias", N);
    const bool has_res = res.has_value() && res->defined();
    if (has_res) {
        check_opt_bf(res, "res", M * N);
        TORCH_CHECK(rmul.has_value() && rmul->defined() && rhw > 0 && M % rhw == 0, "gemm_tail: residual needs rmul");
        check_f(*rmul, "rmul", (M / rhw) * N);
    }
    auto C = at::empty({M, N}, A.options());
    check_launch(rt1_gemm_tail(bp(A), bp(B), (int)M, (int)N, (int)K, bp(A2), bp(B2), (int)K2, fpo(bias),
                               has_res ? bp(*res) : nullptr, has_res ? rmul->data_ptr<float>() : nullptr,
                               has_res ? (int)rhw : 1, bp(C), (int)cfg, cur_stream()), "gemm_tail");
    return C;
}


// G = x^T x and sum x of x [M, Cin] bf16 in one pass (xexpand.hip) -> [Cin^2 + Cin] fp64
at::Tensor xgram(at::Tensor x) {
    check_bf(x, "x");
    auto [M, cin] = rows_cols(x);
    TORCH_CHECK(cin <= 64, "xgram: Cin <= 64");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "xgram: x must be 16-byte aligned");
    const int grid = rt1_xgram_grid(M, cin);
    auto work = at::empty({grid, (int64_t)cin * cin + cin}, f32(x));
    auto out = at::empty({(int64_t)cin * cin + cin}, x.options().dtype(at::kDouble));
    check_launch(rt1_xgram(bp(x), M, cin, grid, work.data_ptr<float>(), out.data_ptr<double>(), cur_stream()), "xgram");
    return out;
}

// Train-mode BN1 constants of y1 = x @ we^T from x alone (xgram + the fp64 quadratic forms), running stats updated in
// place -> {scale, shift, mean, rstd}
std::vector<at::Tensor> x_bn_stats(at::Tensor x, at::Tensor we, OptT gamma, OptT beta, double eps, double momentum,
                                   OptT rmean, OptT rvar) {
    check_bf(we, "we");
    auto [M, cin] = rows_cols(x);
    TORCH_CHECK(we.dim() == 2 && we.size(1) == cin, "we must be [Ce, Cin] matching x");
    const int C = (int)we.size(0);
    check_opt_f(gamma, "gamma", C); check_opt_f(beta, "beta", C);
    check_opt_f(rmean, "running_mean", C); check_opt_f(rvar, "running_var", C);
    auto g = xgram(x);
    const double* gp = g.data_ptr<double>();
    auto o = at::empty({4, C}, f32(x));
    float* b = o.data_ptr<float>();
    check_launch(rt1_bn_from_gram(gp, gp + (int64_t)cin * cin, bp(we), cin, C, (double)M, fpo(gamma), fpo(beta),
                                  (float)eps, (float)momentum, fpo_mut(rmean), fpo_mut(rvar), b, b + C, b + 2 * C,
                                  b + 3 * C, cur_stream()), "bn_from_gram");
    return {o[0], o[1], o[2], o[3]};
}

// BN constants of y = x @ we^T from G = x^T x [cin, cin] and sx = sum_rows x [cin] (fp32, e.g. wgrad(x, x) and
// colsum(x)) over `count` rows: {scale, shift, mean, rstd} [C]; running stats updated in place (training)
std::vector<at::Tensor> bn_from_gram(at::Tensor G, at::Tensor sx, at::Tensor we, double count, OptT gamma, OptT beta,
                                     double eps, double momentum, OptT rmean, OptT rvar) {
    check_bf(we, "we");
    TORCH_CHECK(we.dim() == 2, "we must be [C, cin]");
    const int C = (int)we.size(0), cin = (int)we.size(1);
    check_f(G, "G", (int64_t)cin * cin);
    check_f(sx, "sx", cin);
    check_opt_f(gamma, "gamma", C); check_opt_f(beta, "beta", C);
    check_opt_f(rmean, "running_mean", C); check_opt_f(rvar, "running_var", C);
    auto WG = at::mm(we.to(at::kFloat), G);            // [C, cin] fp32, one library GEMM
    auto o = at::empty({4, C}, f32(G));
    float* b = o.data_ptr<float>();
    check_launch(rt1_bn_from_wg(WG.data_ptr<float>(), sx.data_ptr<float>(), bp(we), cin, C, count, fpo(gamma),
                                      fpo(beta), (float)eps, (float)momentum, fpo_mut(rmean), fpo_mut(rvar), b, b + C,
                                      b + 2 * C, b + 3 * C, cur_stream()), "bn_from_gram");
    return {o[0], o[1], o[2], o[3]};
}

// dW [Co, Ci] fp32 = dy^T a for dy [M, Co], a [M, Ci] bf16 (csrc/kernels/wgrad.hip); optional prologue on a:
// a' = act(a * scale + shift) * gate[m / hw]  (scale/shift [Ci] fp32, gate [M / hw, Ci] fp32)
at::Tensor wgrad(at::Tensor dy, at::Tensor a, OptT scale, OptT shift, OptT gate, int64_t act, int64_t hw,
                 int64_t variant, int64_t splits_req, bool partials, bool sums) {
    check_bf(dy, "dy"); check_bf(a, "a");
    TORCH_CHECK(dy.dim() == 2 && a.dim() == 2 && dy.size(0) == a.size(0), "wgrad: dy [M, Co], a [M, Ci]");
    const int64_t M = dy.size(0), Co = dy.size(1), Ci = a.size(1);
    TORCH_CHECK(M > 0 && Co % 8 == 0 && Ci % 8 == 0, "wgrad: M > 0, Co % 8 == 0, Ci % 8 == 0");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0,
                "wgrad: operands must be 16-byte aligned");
    const bool pro = scale.has_value() && scale->defined();
    if (pro) {
        check_f(*scale, "scale", Ci);
        TORCH_CHECK(shift.has_value() && shift->defined(), "wgrad: shift needed with scale");
        check_f(*shift, "shift", Ci);
    }
    const bool has_gate = gate.has_value() && gate->defined();
    if (has_gate) {
        TORCH_CHECK(pro && hw > 0 && M % hw == 0, "wgrad: gate needs scale/shift and hw dividing M");
        check_f(*gate, "gate", (M / hw) * Ci);
    }
    TORCH_CHECK(variant < 6, "wgrad: variant must be < 6 (-1 = automatic)");
    // splits_req > 0: the row-split count (sweeps, short-M shapes); else the automatic one
    const int splits = splits_req > 0 ? (int)std::min<int64_t>(splits_req, (M + 63) / 64)
                                      : rt1_wgrad_splits(M, (int)Co, (int)Ci, (int)variant);
    TORCH_CHECK(!(sums && pro), "wgrad: sums without a prologue only");
    // sums: [splits, Co * Ci + Co], each split's dW partial followed by its column sums of dy (the bias gradient)
    auto part = sums ? at::empty({splits, Co * Ci + Co}, f32(dy)) : at::empty({splits, Co, Ci}, f32(dy));
    check_launch(rt1_wgrad_run(bp(dy), bp(a), M, (int)Co, (int)Ci, pro ? scale->data_ptr<float>() : nullptr,
                               pro ? shift->data_ptr<float>() : nullptr, has_gate ? gate->data_ptr<float>() : nullptr,
                               (int)act, (int)hw, splits, part.data_ptr<float>(), (int)variant, sums ? 1 : 0,
                               cur_stream()), "wgrad");
    if (partials) return part;                  // [splits, Co, Ci]: the caller sums (parallel/flat.py defer_partials)
    return splits > 1 ? sum0(part) : part[0];
}

// Gram moments of x [M, C] bf16: {G = x^T x [C, C], sx = sum_m x [C]} fp32 from one pass of the MFMA wgrad kernel
// (the first ci tile's workgroups sum their staged rows, csrc/kernels/wgrad.hip DBS) and ONE fixed-order sum of the
// [splits, C * C + C] partials -- instead of the wgrad + a colsum launch re-reading x
std::vector<at::Tensor> gram(at::Tensor x, int64_t variant, int64_t splits_req) {
    check_bf(x, "x");
    TORCH_CHECK(x.dim() == 2 && x.size(0) > 0 && x.size(1) % 8 == 0, "gram: x [M, C], C % 8 == 0");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "gram: x must be 16-byte aligned");
    TORCH_CHECK(variant < 6, "gram: variant must be < 6 (-1 = automatic)");
    const int64_t M = x.size(0), C = x.size(1);
    const int splits = splits_req > 0 ? (int)std::min<int64_t>(splits_req, (M + 63) / 64)
                                      : rt1_wgrad_splits(M, (int)C, (int)C, (int)variant);
    auto part = at::empty({splits, C * C + C}, f32(x));
    check_launch(rt1_wgrad_run(bp(x), bp(x), M, (int)C, (int)C, nullptr, nullptr, nullptr, 0, 1, splits,
                               part.data_ptr<float>(), (int)variant, 1, cur_stream()), "gram");
    auto s = splits > 1 ? sum0(part) : part[0];
    return {s.narrow(0, 0, C * C).view({C, C}), s.narrow(0, C * C, C)};
}

at::Tensor frame_pool(at::Tensor y, OptT G, OptT scale, OptT shift, int64_t act) {
    check_bf(y, "y");
    TORCH_CHECK(y.dim() == 3, "y must be [N, HW, C]");
    const int N = (int)y.size(0), HW = (int)y.size(1), C = (int)y.size(2);
    TORCH_CHECK(C % 8 == 0, "C % 8");
    check_opt_bf(G, "G", y.numel());
    check_opt_f(scale, "scale", C); check_opt_f(shift, "shift", C);
    const int splits = rt1_frame_splits(N, HW, C);
    auto pool = at::empty({splits, N, C}, f32(y));
    check_launch(rt1_frame_pool(bp(y), bpo(G), N, HW, C, fpo(scale), fpo(shift), (int)act, splits,
                                pool.data_ptr<float>(), cur_stream()), "frame_pool");
    return splits > 1 ? sum0(pool) : pool[0];
}

at::Tensor block_tail(at::Tensor y3, at::Tensor scale, at::Tensor shift, OptT keep, OptT skip, OptT fmul, OptT fadd) {
    check_bf(y3, "y3");
    TORCH_CHECK(y3.dim() == 3, "y3 must be [N, HW, C]");
    const int N = (int)y3.size(0), HW = (int)y3.size(1), C = (int)y3.size(2);
    TORCH_CHECK(C % 8 == 0, "C % 8");
    check_f(scale, "scale", C); check_f(shift, "shift", C);
    check_opt_f(keep, "keep", N); check_opt_bf(skip, "skip", y3.numel());
    check_opt_f(fmul, "fmul", (int64_t)N * C); check_opt_f(fadd, "fadd", (int64_t)N * C);
    TORCH_CHECK(fmul.has_value() == fadd.has_value(), "fmul/fadd together");
    auto out = at::empty_like(y3);
    check_launch(rt1_block_tail(bp(y3), (int64_t)N * HW, HW, C, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                fpo(keep), bpo(skip), fpo(fmul), fpo(fadd), bp(out), cur_stream()), "block_tail");
    return out;
}

// x[n, p, c] += y[n, p, c] * s[n, c]  (in place)
void add_scaled_(at::Tensor x, at::Tensor y, at::Tensor s) {
    check_bf(x, "x"); check_bf(y, "y");
    TORCH_CHECK(x.dim() == 3 && y.sizes() == x.sizes(), "x/y must be [N, HW, C]");
    const int N = (int)x.size(0), HW = (int)x.size(1), C = (int)x.size(2);
    TORCH_CHECK(C % 8 == 0, "C % 8");
    check_f(s, "s", (int64_t)N * C);
    check_launch(rt1_add_scaled(bp(x), bp(y), s.data_ptr<float>(), (int64_t)N * HW, HW, C, cur_stream()), "add_scaled_");
}

std::vector<at::Tensor> tail_bwd_reduce(at::Tensor dout, at::Tensor y3, at::Tensor scale, at::Tensor shift,
                                        at::Tensor mean, at::Tensor rstd, OptT keep, OptT skip, OptT fmul) {
    check_bf(dout, "dout"); check_bf(y3, "y3");
    TORCH_CHECK(y3.dim() == 3 && dout.sizes() == y3.sizes(), "dout/y3 must be [N, HW, C]");
    const int N = (int)y3.size(0), HW = (int)y3.size(1), C = (int)y3.size(2);
    TORCH_CHECK(C % 8 == 0, "C % 8");
    check_f(scale, "scale", C); check_f(shift, "shift", C); check_f(mean, "mean", C); check_f(rstd, "rstd", C);
    check_opt_f(keep, "keep", N); check_opt_bf(skip, "skip", y3.numel()); check_opt_f(fmul, "fmul", (int64_t)N * C);
    const int splits = rt1_frame_splits(N, HW, C);
    auto parts = at::empty({splits, 4, N, C}, f32(y3));
    float* b = parts.data_ptr<float>();
    const int64_t NC = (int64_t)N * C;
    check_launch(rt1_tail_bwd_reduce(bp(dout), bp(y3), N, HW, C, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                     mean.data_ptr<float>(), rstd.data_ptr<float>(), fpo(keep), bpo(skip), fpo(fmul),
                                     splits, b, b + NC, b + 2 * NC, b + 3 * NC, cur_stream()), "tail_bwd_reduce");
    auto o = splits > 1 ? sum0(parts) : parts[0];
    return {o[0], o[1], o[2], o[3]};
}

std::vector<at::Tensor> stem_fwd(at::Tensor img, OptT shift, at::Tensor w, int64_t max_blocks) {
    TORCH_CHECK(img.is_cuda() && img.is_contiguous() && img.dim() == 4 && img.size(1) == 3, "img must be [N,3,H,W]");
    const bool u8 = img.scalar_type() == at::kByte;
    TORCH_CHECK(u8 || img.scalar_type() == at::kFloat, "img must be uint8 or float32");
    check_f(w, "w", 40 * 27);
    if (shift.has_value() && shift->defined()) {
        TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kInt && shift->numel() == 2, "shift: int32[2] on GPU");
    }
    const int N = (int)img.size(0), H = (int)img.size(2), W = (int)img.size(3);
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const int64_t g = rt1_stem_grid(N, H, W, (int)max_blocks);
    auto out = at::empty({N, Ho, Wo, 40}, img.options().dtype(at::kBFloat16));
    auto ps = at::empty({g, 40}, f32(w)), pq = at::empty({g, 40}, f32(w));
    const int* sp = (shift.has_value() && shift->defined()) ? shift->data_ptr<int>() : nullptr;
    check_launch(rt1_stem_fwd(img.data_ptr(), u8, sp, w.data_ptr<float>(), N, H, W, 40, (int)g, bp(out),
                              ps.data_ptr<float>(), pq.data_ptr<float>(), cur_stream()), "stem_fwd");
    return {out, ps, pq};
}

at::Tensor stem_bwd_weight(at::Tensor img, OptT shift, at::Tensor dy, int64_t max_blocks, OptT bn_x, OptT sc, OptT sh,
                           OptT mean, OptT rstd, OptT gamma, OptT mdz, OptT mdzx) {
    TORCH_CHECK(img.is_cuda() && img.is_contiguous() && img.dim() == 4 && img.size(1) == 3, "img must be [N,3,H,W]");
    const bool u8 = img.scalar_type() == at::kByte;
    TORCH_CHECK(u8 || img.scalar_type() == at::kFloat, "img must be uint8 or float32");
    const int N = (int)img.size(0), H = (int)img.size(2), W = (int)img.size(3);
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    check_bf(dy, "dy");
    TORCH_CHECK(dy.numel() == (int64_t)N * Ho * Wo * 40, "dy must be [N, Ho, Wo, 40]");
    if (shift.has_value() && shift->defined()) {
        TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kInt && shift->numel() == 2, "shift: int32[2] on GPU");
    }
    const bool bn = bn_x.has_value() && bn_x->defined();
    if (bn) {
        // dy = gradient of silu(bn(bn_x)); the stem BN backward runs in the kernel's staging
        check_bf(*bn_x, "bn_x");
        TORCH_CHECK(bn_x->numel() == dy.numel(), "bn_x must be [N, Ho, Wo, 40]");
        check_f(*sc, "scale", 40); check_f(*sh, "shift", 40); check_f(*mean, "mean", 40); check_f(*rstd, "rstd", 40);
        check_f(*mdz, "mdz", 40); check_f(*mdzx, "mdzx", 40);
        check_opt_f(gamma, "gamma", 40);
    }
    const int64_t g = rt1_stem_grid(N, H, W, (int)max_blocks);
    auto part = at::empty({g, 40 * 27}, f32(dy));
    const int* sp = (shift.has_value() && shift->defined()) ? shift->data_ptr<int>() : nullptr;
    check_launch(rt1_stem_bwd_weight(img.data_ptr(), u8, sp, bp(dy), N, H, W, 40, (int)g, part.data_ptr<float>(),
                                     cur_stream(), bn ? bp(*bn_x) : nullptr, bn ? sc->data_ptr<float>() : nullptr,
                                     bn ? sh->data_ptr<float>() : nullptr, bn ? mean->data_ptr<float>() : nullptr,
                                     bn ? rstd->data_ptr<float>() : nullptr, bn ? fpo(gamma) : nullptr,
                                     bn ? mdz->data_ptr<float>() : nullptr, bn ? mdzx->data_ptr<float>() : nullptr),
                 "stem_bwd_weight");
    return sum0(part).view({40, 27});
}


std::vector<at::Tensor> attn_fwd(at::Tensor qkv, int64_t L, int64_t Kimg, double scale, double drop_p, int64_t seed,
                                 OptT seed_dev) {
    check_bf(qkv, "qkv");
    TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 128, "qkv must be [B, S, 3, H, 128]");
    const int B = (int)qkv.size(0), S = (int)qkv.size(1), H = (int)qkv.size(3);
    TORCH_CHECK(S >= 1 && S <= 256, "sequence length must be in [1, 256]");
    TORCH_CHECK(L > 0 && Kimg >= 0 && Kimg <= L, "bad token layout");
    auto out = at::empty({B, S, H, 128}, qkv.options());
    auto lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
    check_launch(rt1_attn_fwd(bp(qkv), bp(out), lse.data_ptr<float>(), B, S, H, (int)L, (int)Kimg, (float)scale,
                              (float)drop_p, (uint32_t)seed, seed_ptr(seed_dev), cur_stream()), "attn_fwd");
    return {out, lse};
}

// dqkv [B, S, 3, H, 128] for S <= 96 (one workgroup per (b, h), P and the dropout mask regenerated)
at::Tensor attn_bwd(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse, int64_t L, int64_t Kimg,
                    double scale, double drop_p, int64_t seed, OptT seed_dev) {
    check_bf(qkv, "qkv"); check_bf(out, "out"); check_bf(dout, "dout");
    TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 128, "qkv must be [B, S, 3, H, 128]");
    const int B = (int)qkv.size(0), S = (int)qkv.size(1), H = (int)qkv.size(3);
    TORCH_CHECK(S >= 1 && S <= 96, "attn_bwd supports S <= 96");
    TORCH_CHECK(out.sizes() == at::IntArrayRef({B, S, H, 128}) && dout.sizes() == out.sizes(), "out/dout [B,S,H,128]");
    check_f(lse, "lse", (int64_t)B * H * S);
    auto dqkv = at::empty_like(qkv);
    check_launch(rt1_attn_bwd(bp(qkv), bp(out), bp(dout), lse.data_ptr<float>(), bp(dqkv), B, S, H, (int)L, (int)Kimg,
                              (float)scale, (float)drop_p, (uint32_t)seed, seed_ptr(seed_dev), cur_stream()),
                 "attn_bwd");
    return dqkv;
}

at::Tensor attn_keepmask(int64_t BH, int64_t S, double drop_p, int64_t seed, at::Tensor like, OptT seed_dev) {
    TORCH_CHECK(like.is_cuda(), "like must be a GPU tensor");
    auto keep = at::empty({BH, S, S}, like.options().dtype(at::kByte));
    check_launch(rt1_attn_keepmask(keep.data_ptr<uint8_t>(), (int)BH, (int)S, (float)drop_p, (uint32_t)seed,
                                   seed_ptr(seed_dev), cur_stream()), "attn_keepmask");
    return keep;
}


at::Tensor se_bn_bwd_reduce(at::Tensor G, at::Tensor y, at::Tensor scale, at::Tensor shift, at::Tensor mean,
                            at::Tensor rstd) {
    check_bf(G, "G"); check_bf(y, "y");
    TORCH_CHECK(y.dim() == 3 && G.sizes() == y.sizes(), "G/y must be [N, HW, C]");
    const int N = (int)y.size(0), HW = (int)y.size(1), C = (int)y.size(2);
    TORCH_CHECK(C % 8 == 0, "C % 8");
    check_f(scale, "scale", C); check_f(shift, "shift", C); check_f(mean, "mean", C); check_f(rstd, "rstd", C);
    const int splits = rt1_frame_splits(N, HW, C);
    auto parts = at::empty({splits, 5, N, C}, f32(y));
    check_launch(rt1_se_bn_bwd_reduce(bp(G), bp(y), N, HW, C, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                      mean.data_ptr<float>(), rstd.data_ptr<float>(), splits, parts.data_ptr<float>(),
                                      cur_stream()), "se_bn_bwd_reduce");
    return splits > 1 ? sum0(parts) : parts[0];
}

// Project-conv backward of a skinny block from (dy3, y2) in one pass per frame (csrc/kernels/projbwd.hip):
// returns (red [5, N, Ce] -- the se_bn_bwd_reduce sums, computed through dA = dy3 @ Wp --, dWp [Cout, Ce] fp32)
std::vector<at::Tensor> proj_bwd(at::Tensor dy3, at::Tensor y2, at::Tensor Wp, at::Tensor gate, at::Tensor scale,
                                 at::Tensor shift, at::Tensor mean, at::Tensor rstd) {
    check_bf(dy3, "dy3"); check_bf(y2, "y2"); check_bf(Wp, "Wp");
    TORCH_CHECK(y2.dim() == 3, "proj_bwd: y2 must be [N, HW, Ce]");
    const int N = (int)y2.size(0), HW = (int)y2.size(1), Ce = (int)y2.size(2);
    TORCH_CHECK(dy3.dim() == 2 && dy3.size(0) == (int64_t)N * HW, "proj_bwd: dy3 must be [N*HW, Cout]");
    const int Cout = (int)dy3.size(1);
    TORCH_CHECK(rt1_proj_bwd_supported(Cout, Ce), "proj_bwd: no specialisation for Cout=", Cout, " Ce=", Ce);
    TORCH_CHECK(Wp.dim() == 2 && Wp.size(0) == Cout && Wp.size(1) == Ce, "proj_bwd: Wp must be [Cout, Ce]");
    TORCH_CHECK((int64_t)N * HW < ((int64_t)1 << 31), "proj_bwd: too many rows");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(dy3.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y2.data_ptr()) % 16 == 0,
                "proj_bwd: operands must be 16-byte aligned");
    check_f(gate, "gate", (int64_t)N * Ce);
    check_f(scale, "scale", Ce); check_f(shift, "shift", Ce); check_f(mean, "mean", Ce); check_f(rstd, "rstd", Ce);
    const int fs = rt1_proj_bwd_fsplit(N, HW, Ce);
    auto G = at::empty({fs, N, Cout, Ce}, f32(y2));
    auto R = at::empty({fs, 5, N, Ce}, f32(y2));
    check_launch(rt1_proj_bwd_frame(bp(dy3), bp(y2), N, HW, Cout, Ce, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                    mean.data_ptr<float>(), rstd.data_ptr<float>(), bp(Wp), fs, G.data_ptr<float>(),
                                    R.data_ptr<float>(), cur_stream()), "proj_bwd_frame");
    auto red = fs > 1 ? at::empty({5, N, Ce}, f32(y2)) : R[0];
    auto dW = at::empty({Cout, Ce}, f32(y2));
    check_launch(rt1_proj_bwd_finalize(G.data_ptr<float>(), R.data_ptr<float>(), gate.data_ptr<float>(), N, Cout, Ce, fs,
                                       red.data_ptr<float>(), dW.data_ptr<float>(), cur_stream()), "proj_bwd_finalize");
    return {red, dW};
}
bool proj_bwd_supported(int64_t Cout, int64_t Ce) { return rt1_proj_bwd_supported((int)Cout, (int)Ce) != 0; }

}  // namespace

// skinny kernel (with optional BN-stat epilogue) or the wide-N kernel (no epilogue)
bool pw_gemm_supported(int64_t K, int64_t N) {
    return rt1_pw_gemm_supported((int)K, (int)N) != 0 || rt1_pw_wide_supported((int)K, (int)N) != 0;
}
bool pw_stats_supported(int64_t K, int64_t N) { return rt1_pw_gemm_supported((int)K, (int)N) != 0; }

// C[M, N] = A[M, K] @ B[N, K]^T (bf16, fp32 accumulate) for the skinny 1x1-conv shapes; with stats=True
// also returns per-workgroup BN partial sums [G, N] of the stored C.  scale/shift [K] + gate [M / hw, K] (skinny
// shapes only): the operand is silu(A*scale + shift) * gate[row / hw], rebuilt in registers (project convs).
std::vector<at::Tensor> pw_gemm(at::Tensor A, at::Tensor B, int64_t max_blocks, bool stats, OptT scale, OptT shift,
                                OptT gate, int64_t hw, bool store_operand) {
    check_bf(A, "A"); check_bf(B, "B");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "pw_gemm: A [M,K], B [N,K]");
    const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
    TORCH_CHECK(M > 0 && M < (int64_t)1 << 31, "pw_gemm: bad M");
    const bool skinny = rt1_pw_gemm_supported((int)K, (int)N) != 0;
    TORCH_CHECK(skinny || (!stats && rt1_pw_wide_supported((int)K, (int)N)), "pw_gemm: no specialisation for K=", K,
                " N=", N, stats ? " with BN statistics" : "");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
                "pw_gemm: operands must be 16-byte aligned");
    const bool pro = scale.has_value() && scale->defined();
    if (pro) {
        TORCH_CHECK(skinny, "pw_gemm: the operand prologue needs a skinny specialisation (K=", K, " N=", N, ")");
        check_f(*scale, "scale", K);
        TORCH_CHECK(shift.has_value() && shift->defined() && gate.has_value() && gate->defined(),
                    "pw_gemm: prologue needs scale, shift and gate");
        check_f(*shift, "shift", K);
        TORCH_CHECK(hw > 0 && M % hw == 0, "pw_gemm: hw must divide M");
        check_f(*gate, "gate", (M / hw) * K);
    }
    TORCH_CHECK(!store_operand || pro, "pw_gemm: store_operand needs the prologue");
    auto C = at::empty({M, N}, A.options());
    at::Tensor aout;
    if (store_operand) aout = at::empty({M, K}, A.options());
    if (!skinny) {
        check_launch(rt1_pw_wide(bp(A), bp(B), (int)M, (int)K, (int)N, bp(C), (int)max_blocks, cur_stream()), "pw_wide");
        return {C};
    }
    at::Tensor ps, pq;
    if (stats) {
        const int g = rt1_pw_gemm_grid((int)M, (int)K, (int)N, (int)max_blocks);
        ps = at::empty({g, N}, f32(A));
        pq = at::empty({g, N}, f32(A));
    }
    check_launch(rt1_pw_gemm(bp(A), bp(B), (int)M, (int)K, (int)N, bp(C), stats ? ps.data_ptr<float>() : nullptr,
                             stats ? pq.data_ptr<float>() : nullptr, (int)max_blocks, fpo(scale), fpo(shift),
                             fpo(gate), (int)hw, store_operand ? bp(aout) : nullptr, cur_stream()), "pw_gemm");
    std::vector<at::Tensor> res{C};
    if (stats) { res.push_back(ps); res.push_back(pq); }
    if (store_operand) res.push_back(aout);
    return res;
}


// project data gradient with the BN3 backward in the operand prologue: dout, y3 [M, K] bf16, W [N, K] bf16 (= Wp^T),
// fmul [M / hw, K] fp32, keep [M / hw] fp32 or None, BN3 gamma / mean / rstd / mdz / mdzx [K] -> {dA [M, N], dy3 [M, K]}
bool pw_gemm_bnbwd_supported(int64_t K, int64_t N) { return rt1_pw_gemm_bnbwd_supported((int)K, (int)N) != 0; }
std::vector<at::Tensor> pw_gemm_bnbwd(at::Tensor dout, at::Tensor y, at::Tensor W, at::Tensor fmul, OptT keep,
                                      int64_t hw, OptT gamma, at::Tensor mean, at::Tensor rstd, at::Tensor mdz,
                                      at::Tensor mdzx, int64_t max_blocks) {
    check_bf(dout, "dout"); check_bf(y, "y"); check_bf(W, "W");
    TORCH_CHECK(dout.dim() == 2 && dout.sizes() == y.sizes() && W.dim() == 2 && W.size(1) == dout.size(1),
                "pw_gemm_bnbwd: dout, y [M, K], W [N, K]");
    const int64_t M = dout.size(0), K = dout.size(1), N = W.size(0);
    TORCH_CHECK(rt1_pw_gemm_bnbwd_supported((int)K, (int)N), "pw_gemm_bnbwd: no specialisation for K=", K, " N=", N);
    TORCH_CHECK(hw > 0 && M % hw == 0, "pw_gemm_bnbwd: hw must divide M");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(dout.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0, "pw_gemm_bnbwd: operands must be 16-byte aligned");
    check_f(fmul, "fmul", (M / hw) * K);
    check_opt_f(keep, "keep", M / hw); check_opt_f(gamma, "gamma", K);
    check_f(mean, "mean", K); check_f(rstd, "rstd", K); check_f(mdz, "mdz", K); check_f(mdzx, "mdzx", K);
    auto C = at::empty({M, N}, dout.options());
    auto dy = at::empty({M, K}, dout.options());
    check_launch(rt1_pw_gemm_bnbwd(bp(dout), bp(W), (int)M, (int)K, (int)N, bp(C), (int)max_blocks, bp(y),
                                   fmul.data_ptr<float>(), fpo(keep), (int)hw, fpo(gamma), mean.data_ptr<float>(),
                                   rstd.data_ptr<float>(), mdz.data_ptr<float>(), mdzx.data_ptr<float>(), bp(dy),
                                   cur_stream()), "pw_gemm_bnbwd");
    return {C, dy};
}

bool pw_bwd_supported(int64_t CE, int64_t CIN) { return rt1_pw_bwd_supported((int)CE, (int)CIN) != 0; }

// fused expand-stage backward: returns (dx [M, CIN] bf16, dWe [CE, CIN] fp32)
std::vector<at::Tensor> pw_bwd(at::Tensor dA, at::Tensor y, at::Tensor x, at::Tensor We, at::Tensor consts, OptT dout,
                               OptT fmul, int64_t HW, int64_t max_blocks) {
    check_bf(dA, "dA"); check_bf(y, "y"); check_bf(x, "x"); check_bf(We, "We");
    TORCH_CHECK(dA.dim() == 2 && y.sizes() == dA.sizes() && x.dim() == 2 && x.size(0) == dA.size(0),
                "pw_bwd: dA/y [M, CE], x [M, CIN]");
    const int64_t M = dA.size(0), CE = dA.size(1), CIN = x.size(1);
    TORCH_CHECK(M > 0 && M < (int64_t)1 << 31, "pw_bwd: bad M");
    TORCH_CHECK(rt1_pw_bwd_supported((int)CE, (int)CIN), "pw_bwd: no specialisation for CE=", CE, " CIN=", CIN);
    TORCH_CHECK(We.dim() == 2 && We.size(0) == CE && We.size(1) == CIN, "pw_bwd: We must be [CE, CIN]");
    check_f(consts, "consts", 5 * CE);
    const bool skip = dout.has_value() && dout->defined();
    if (skip) {
        check_opt_bf(dout, "dout", M * CIN);
        TORCH_CHECK(fmul.has_value() && fmul->defined() && HW > 0 && M % HW == 0, "pw_bwd: residual needs fmul, HW");
        check_f(*fmul, "fmul", (M / HW) * CIN);
    }
    const int g = rt1_pw_bwd_grid((int)M, (int)max_blocks);
    auto dx = at::empty({M, CIN}, x.options());
    auto dwp = at::empty({g, CE, CIN}, f32(x));
    check_launch(rt1_pw_bwd(bp(dA), bp(y), bp(x), bp(We), consts.data_ptr<float>(), (int)M, (int)CE, (int)CIN, bp(dx),
                            skip ? bp(*dout) : nullptr, skip ? fmul->data_ptr<float>() : nullptr, (int)HW,
                            dwp.data_ptr<float>(), g, cur_stream()), "pw_bwd");
    return {dx, sum0(dwp)};
}

// y-free fused expand backward (pwbwd.hip pw_bwd_z_kernel): dz [M, CE] = dA1 * silu'(bn1(y1)) as stored by the
// depthwise backward (dw_bwd_fused zout=True), x [M, CIN] the block input; consts [5, CE] from bn_bwd_finalize_pw.
// Returns (dx [M, CIN] bf16, dWe [CE, CIN] fp32); y1 is never read.
std::vector<at::Tensor> pw_bwd_z(at::Tensor dz, at::Tensor x, at::Tensor We, at::Tensor consts, OptT dout, OptT fmul,
                                 int64_t HW, int64_t max_blocks) {
    check_bf(dz, "dz"); check_bf(x, "x"); check_bf(We, "We");
    TORCH_CHECK(dz.dim() == 2 && x.dim() == 2 && x.size(0) == dz.size(0), "pw_bwd_z: dz [M, CE], x [M, CIN]");
    const int64_t M = dz.size(0), CE = dz.size(1), CIN = x.size(1);
    TORCH_CHECK(M > 0 && M < (int64_t)1 << 31, "pw_bwd_z: bad M");
    TORCH_CHECK(rt1_pw_bwd_supported((int)CE, (int)CIN), "pw_bwd_z: no specialisation for CE=", CE, " CIN=", CIN);
    TORCH_CHECK(We.dim() == 2 && We.size(0) == CE && We.size(1) == CIN, "pw_bwd_z: We must be [CE, CIN]");
    check_f(consts, "consts", 5 * CE);
    const bool skip = dout.has_value() && dout->defined();
    if (skip) {
        check_opt_bf(dout, "dout", M * CIN);
        TORCH_CHECK(fmul.has_value() && fmul->defined() && HW > 0 && M % HW == 0, "pw_bwd_z: residual needs fmul, HW");
        check_f(*fmul, "fmul", (M / HW) * CIN);
    }
    const int g = rt1_pw_bwd_grid((int)M, (int)max_blocks);
    auto dx = at::empty({M, CIN}, x.options());
    auto mk = at::empty({(int64_t)rt1_pw_bwd_z_mk_elems((int)CIN)}, x.options());
    auto r0 = at::empty({CIN}, f32(x));
    auto part = at::empty({g, (int64_t)rt1_pw_bwd_z_width((int)CE, (int)CIN)}, f32(x));
    check_launch(rt1_pw_bwd_z(bp(dz), bp(x), bp(We), consts.data_ptr<float>(), (int)M, (int)CE, (int)CIN, bp(mk),
                              r0.data_ptr<float>(), bp(dx), skip ? bp(*dout) : nullptr,
                              skip ? fmul->data_ptr<float>() : nullptr, (int)HW, part.data_ptr<float>(), g,
                              cur_stream()), "pw_bwd_z");
    auto S = sum0(part);
    auto dWe = at::empty({CE, CIN}, f32(x));
    check_launch(rt1_pw_bwd_z_finish(S.data_ptr<float>(), bp(We), consts.data_ptr<float>(), (int)CE, (int)CIN,
                                     dWe.data_ptr<float>(), cur_stream()), "pw_bwd_z_finish");
    return {dx, dWe};
}

// wide-layer y-free expand backward operands (pwbwd.hip, one launch): We [CE, CIN] bf16, consts [5, CE] ->
// (Wt = (diag(k1) We)^T [CIN, CE] bf16, Mk = We^T diag(k2) We [CIN, CIN] bf16, r0 = k0^T We [CIN] fp32)
std::vector<at::Tensor> pw_z_prep(at::Tensor We, at::Tensor consts) {
    check_bf(We, "We");
    TORCH_CHECK(We.dim() == 2, "pw_z_prep: We must be [CE, CIN]");
    const int64_t CE = We.size(0), CIN = We.size(1);
    check_f(consts, "consts", 5 * CE);
    auto wt = at::empty({CIN, CE}, We.options());
    auto mk = at::empty({CIN, CIN}, We.options());
    auto r0 = at::empty({CIN}, We.options().dtype(at::kFloat));
    check_launch(rt1_pw_z_prep(bp(We), consts.data_ptr<float>(), (int)CE, (int)CIN, bp(wt), bp(mk),
                               r0.data_ptr<float>(), cur_stream()), "pw_z_prep");
    return {wt, mk, r0};
}

// C = A @ W^T + A2 @ W2^T + bias (pwtall.hip pw_tall_tail): A [M, K], W [N, K], A2 [M, K2], W2 [N, K2] bf16,
// bias [N] fp32 -> C [M, N] bf16
at::Tensor pw_tall_tail(at::Tensor A, at::Tensor W, at::Tensor A2, at::Tensor W2, at::Tensor bias, OptT res,
                        OptT rmul, int64_t rhw) {
    check_bf(A, "A"); check_bf(W, "W"); check_bf(A2, "A2"); check_bf(W2, "W2");
    TORCH_CHECK(A.dim() == 2 && W.dim() == 2 && A.size(1) == W.size(1), "pw_tall_tail: A [M, K], W [N, K]");
    const int64_t M = A.size(0), K = A.size(1), N = W.size(0), K2 = A2.size(1);
    TORCH_CHECK(A2.dim() == 2 && A2.size(0) == M, "pw_tall_tail: A2 must be [M, K2]");
    TORCH_CHECK(W2.numel() == N * K2, "pw_tall_tail: W2 must be [N, K2]"); check_f(bias, "bias", N);
    TORCH_CHECK(rt1_pw_tall_preferred((int)K, (int)N) && K2 % 8 == 0, "pw_tall_tail: unsupported K=", K, " N=", N,
                " K2=", K2);
    const bool has_res = res.has_value() && res->defined();
    if (has_res) {
        check_opt_bf(res, "res", M * N);
        TORCH_CHECK(rmul.has_value() && rmul->defined() && rhw > 0 && M % rhw == 0, "pw_tall_tail: residual needs rmul");
        check_f(*rmul, "rmul", (M / rhw) * N);
    }
    auto C = at::empty({M, N}, A.options());
    check_launch(rt1_pw_tall_tail(bp(A), bp(W), (int)M, (int)K, (int)N, bp(A2), bp(W2), (int)K2,
                                  bias.data_ptr<float>(), has_res ? bp(*res) : nullptr,
                                  has_res ? rmul->data_ptr<float>() : nullptr, (int)rhw, bp(C), cur_stream()),
                 "pw_tall_tail");
    return C;
}

// dWe = diag(k1) S + diag(k2) We G + k0 (x) sx   (S [CE, CIN], G [CIN, CIN], sx [CIN] fp32)
// S: dz^T x [CE, CIN] or its row-split partials [splits, CE, CIN] (summed in the kernel)
at::Tensor pw_z_finish(at::Tensor S, at::Tensor G, at::Tensor sx, at::Tensor We, at::Tensor consts) {
    check_bf(We, "We");
    const int64_t CE = We.size(0), CIN = We.size(1);
    const int64_t splits = S.dim() == 3 ? S.size(0) : 1;
    check_f(S, "S", splits * CE * CIN); check_f(G, "G", CIN * CIN); check_f(sx, "sx", CIN);
    check_f(consts, "consts", 5 * CE);
    auto dWe = at::empty({CE, CIN}, f32(S));
    check_launch(rt1_pw_z_finish(S.data_ptr<float>(), (int)splits, G.data_ptr<float>(), sx.data_ptr<float>(), bp(We),
                                 consts.data_ptr<float>(), (int)CE, (int)CIN, dWe.data_ptr<float>(), cur_stream()),
                 "pw_z_finish");
    return dWe;
}

void check_rows512(const at::Tensor& t, const char* name, at::ScalarType dt) {
    check_dev(t, name, dt);
    TORCH_CHECK(t.dim() == 2 && t.size(1) == 512, name, " must be [T, 512]");
}

std::vector<at::Tensor> tf_ln_fwd(at::Tensor x, at::Tensor g, at::Tensor b, double eps) {
    check_rows512(x, "x", at::kFloat);
    check_f(g, "g", 512); check_f(b, "b", 512);
    const int T = (int)x.size(0);
    auto y = at::empty({T, 512}, x.options().dtype(at::kBFloat16));
    auto mu = at::empty({T}, x.options()), rs = at::empty({T}, x.options());
    check_launch(rt1_ln_fwd(x.data_ptr<float>(), g.data_ptr<float>(), b.data_ptr<float>(), T, (float)eps, bp(y),
                            mu.data_ptr<float>(), rs.data_ptr<float>(), cur_stream()), "ln_fwd");
    return {y, mu, rs};
}

// LayerNorm backward (+ dres); want_bf: also bf16(dx) and its column sums -> [dx, dg, db] (+ [dx_bf16, sum_rows dx])
std::vector<at::Tensor> tf_ln_bwd(at::Tensor dy, at::Tensor x, at::Tensor mu, at::Tensor rs, at::Tensor g, OptT dres,
                                  bool want_bf) {
    check_rows512(dy, "dy", at::kBFloat16); check_rows512(x, "x", at::kFloat);
    const int T = (int)x.size(0);
    TORCH_CHECK(dy.size(0) == T, "dy/x rows");
    check_f(mu, "mu", T); check_f(rs, "rs", T); check_f(g, "g", 512);
    if (dres.has_value() && dres->defined()) { check_rows512(*dres, "dres", at::kFloat); TORCH_CHECK(dres->size(0) == T, "dres rows"); }
    const int grid = rt1_tf_grid(T);
    auto dx = at::empty({T, 512}, x.options());
    auto part = at::empty({want_bf ? 3 : 2, grid, 512}, x.options());
    at::Tensor dxb;
    if (want_bf) dxb = at::empty({T, 512}, x.options().dtype(at::kBFloat16));
    check_launch(rt1_ln_bwd(bp(dy), x.data_ptr<float>(), mu.data_ptr<float>(), rs.data_ptr<float>(), g.data_ptr<float>(),
                            fpo(dres), T, dx.data_ptr<float>(), part[0].data_ptr<float>(), part[1].data_ptr<float>(),
                            want_bf ? bp(dxb) : nullptr, want_bf ? part[2].data_ptr<float>() : nullptr, grid,
                            cur_stream()), "ln_bwd");
    auto s = colsum3(part, want_bf ? 3 : 2, grid, 512);
    if (want_bf) return {dx, s[0], s[1], dxb, s[2]};
    return {dx, s[0], s[1]};
}

// out = x + dropout(a + bias); with (lg, lb): also the next LayerNorm of out -> [out] or [out, xn (bf16), mu, rstd]
std::vector<at::Tensor> tf_resid(at::Tensor x, at::Tensor a, at::Tensor bias, double p, int64_t seed, OptT seed_dev,
                                 OptT lg, OptT lb, double eps) {
    check_rows512(x, "x", at::kFloat); check_rows512(a, "a", at::kBFloat16);
    TORCH_CHECK(a.size(0) == x.size(0), "x/a rows");
    check_f(bias, "bias", 512);
    const int T = (int)x.size(0);
    const bool ln = lg.has_value() && lg->defined();
    if (ln) { check_f(*lg, "lg", 512); check_f(*lb, "lb", 512); }
    auto out = at::empty_like(x);
    at::Tensor xn, mu, rs;
    if (ln) {
        xn = at::empty({T, 512}, x.options().dtype(at::kBFloat16));
        mu = at::empty({T}, x.options());
        rs = at::empty({T}, x.options());
    }
    check_launch(rt1_resid(x.data_ptr<float>(), bp(a), bias.data_ptr<float>(), T, (float)p, (uint32_t)seed,
                           seed_ptr(seed_dev), out.data_ptr<float>(), fpo(lg), fpo(lb), (float)eps,
                           ln ? bp(xn) : nullptr, ln ? mu.data_ptr<float>() : nullptr,
                           ln ? rs.data_ptr<float>() : nullptr, cur_stream()), "resid");
    if (ln) return {out, xn, mu, rs};
    return {out};
}

std::vector<at::Tensor> tf_drop_bwd(at::Tensor dout, double p, int64_t seed, OptT seed_dev) {
    check_rows512(dout, "dout", at::kFloat);
    const int T = (int)dout.size(0);
    const int grid = rt1_tf_grid(T);
    auto dh = at::empty({T, 512}, dout.options().dtype(at::kBFloat16));
    auto part = at::empty({grid, 512}, dout.options());
    check_launch(rt1_drop_bwd(dout.data_ptr<float>(), T, (float)p, (uint32_t)seed, seed_ptr(seed_dev), bp(dh),
                              part.data_ptr<float>(), grid,
                              cur_stream()), "drop_bwd");
    return {dh, sum0(part)};
}


namespace rt1comm {
void register_comm(py::module_& m);
}
namespace rt1head {
void register_head(py::module_& m);
}

PYBIND11_MODULE(_rt1_hip, m) {
    m.doc() = "RT-1 HIP/CDNA4 kernels (gfx950)";
    m.def("flat_adam", &flat_adam, "fused Adam/AdamW over flat fp32 buffers");
    m.def("flat_adam_dev", &flat_adam_dev, "fused Adam/AdamW, step/lr read from a device tensor (graph-replayable)");
    m.def("bn_stats", &bn_stats);
    m.def("bn_finalize", &bn_finalize);
    m.def("xgram", &xgram);
    m.def("gemm_tail", &gemm_tail, py::arg("A"), py::arg("B"), py::arg("A2"), py::arg("B2"), py::arg("bias") = py::none(),
          py::arg("res") = py::none(), py::arg("rmul") = py::none(), py::arg("rhw") = 1, py::arg("cfg") = -1);
    m.def("gemm256", &gemm256, py::arg("A"), py::arg("B"), py::arg("nn") = false, py::arg("bias") = py::none(),
          py::arg("scale") = py::none(), py::arg("shift") = py::none(), py::arg("gate") = py::none(),
          py::arg("hw") = 0, py::arg("stats") = false, py::arg("store_a") = false, py::arg("bn") = 256);
    m.def("film_fwd", &film_fwd, py::arg("xe"), py::arg("K"), py::arg("w"), py::arg("bias"), py::arg("cmap"),
          py::arg("total"), py::arg("cfg") = -1);
    m.def("film_wgrad", &film_wgrad, py::arg("dflat"), py::arg("cmap"), py::arg("xe"), py::arg("K"),
          py::arg("splits") = 1, py::arg("tile") = 0);
    m.def("gemm", &gemm, py::arg("A"), py::arg("B"), py::arg("nn") = false, py::arg("bias") = py::none(),
          py::arg("scale") = py::none(), py::arg("shift") = py::none(), py::arg("gate") = py::none(),
          py::arg("hw") = 0, py::arg("out_f32") = false, py::arg("stats") = false, py::arg("cfg") = -1,
          py::arg("store_a") = false);
    m.def("x_bn_stats", &x_bn_stats);
    m.def("bn_from_gram", &bn_from_gram);
    m.def("dw_x_supported", &dw_x_supported);
    m.def("dw_tile_info", &dw_tile_info);
    m.def("dw_fwd_x", &dw_fwd_x);
    m.def("dw_bwd_fused_x", &dw_bwd_fused_x, py::arg("dA"), py::arg("y2"), py::arg("gate"), py::arg("rb"),
          py::arg("sc2"), py::arg("sh2"), py::arg("mu2"), py::arg("rs2"), py::arg("g2"), py::arg("mdz2"),
          py::arg("mdzx2"), py::arg("w"), py::arg("k"), py::arg("x"), py::arg("we"), py::arg("sc1"), py::arg("sh1"),
          py::arg("mu1"), py::arg("rs1"), py::arg("max_blocks"), py::arg("zout") = true);
    m.def("bn_apply", &bn_apply);
    m.def("bn_bwd_reduce", &bn_bwd_reduce);
    m.def("bn_bwd_finalize", &bn_bwd_finalize);
    m.def("bn_bwd_finalize_new", &bn_bwd_finalize_new);
    m.def("bn_bwd_finalize_pw", &bn_bwd_finalize_pw);
    m.def("bn_bwd_apply", &bn_bwd_apply, py::arg("G"), py::arg("rs"), py::arg("rb"), py::arg("HW"), py::arg("y"),
          py::arg("scale"), py::arg("shift"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("act"),
          py::arg("mdz"), py::arg("mdzx"), py::arg("keep") = py::none());
    m.def("dw_fwd", &dw_fwd);
    m.def("dw_bwd_data", &dw_bwd_data);
    m.def("dw_bwd_weight", &dw_bwd_weight);
    m.def("dw_bwd_fused", &dw_bwd_fused, py::arg("dA"), py::arg("y2"), py::arg("gate"), py::arg("rb"), py::arg("sc2"),
          py::arg("sh2"), py::arg("mu2"), py::arg("rs2"), py::arg("g2"), py::arg("mdz2"), py::arg("mdzx2"), py::arg("w"),
          py::arg("k"), py::arg("x1"), py::arg("sc1"), py::arg("sh1"), py::arg("act1"), py::arg("mu1"), py::arg("rs1"),
          py::arg("max_blocks"), py::arg("variant") = -1, py::arg("zout") = false, py::arg("res") = py::none(),
          py::arg("rmul") = py::none());
    m.def("gram", &gram, "{x^T x, sum_m x} fp32 of x [M, C] bf16 in one MFMA pass", py::arg("x"),
          py::arg("variant") = -1, py::arg("splits") = 0);
    m.def("wgrad", &wgrad, "1x1-conv weight gradient dy^T a on MFMA (optional BN/act/gate prologue on a)",
          py::arg("dy"), py::arg("a"), py::arg("scale") = py::none(), py::arg("shift") = py::none(),
          py::arg("gate") = py::none(), py::arg("act") = 0, py::arg("hw") = 0, py::arg("variant") = -1,
          py::arg("splits") = -1, py::arg("partials") = false, py::arg("sums") = false);
    m.def("crop_resize_u8", &crop_resize_u8, "Pillow-exact random-resized-crop of raw uint8 frames (GPU)");
    m.def("crop_resize_gather_u8", &crop_resize_gather_u8,
          "crop_resize_u8 over frames gathered by index from an HBM-resident [F, h, w, 3] table");
    m.def("multi_reduce_copy_", &multi_reduce_copy_, "dst[i] = fixed-order sum of splits[i] partials of src[i]",
          py::arg("dst"), py::arg("src"), py::arg("splits"), py::arg("sstride"));
    m.def("multi_copy_", &multi_copy_, "dst[i].copy_(src[i]) for many same-dtype tensors, 128 per launch");
    m.def("colsum", &colsum_py, "deterministic fixed-order sum over dim 0 (fp32/bf16 in, fp32 out)");
    m.def("frame_pool", &frame_pool);
    m.def("block_tail", &block_tail);
    m.def("tail_bwd_reduce", &tail_bwd_reduce);
    m.def("stem_fwd", &stem_fwd);
    m.def("stem_bwd_weight", &stem_bwd_weight, py::arg("img"), py::arg("shift"), py::arg("dy"), py::arg("max_blocks"),
          py::arg("bn_x") = py::none(), py::arg("scale") = py::none(), py::arg("shift_bn") = py::none(),
          py::arg("mean") = py::none(), py::arg("rstd") = py::none(), py::arg("gamma") = py::none(),
          py::arg("mdz") = py::none(), py::arg("mdzx") = py::none());
    m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("L"), py::arg("Kimg"), py::arg("scale"), py::arg("drop_p"),
          py::arg("seed"), py::arg("seed_dev") = py::none());
    m.def("se_bn_bwd_reduce", &se_bn_bwd_reduce);
    m.def("proj_bwd", &proj_bwd, "project-conv backward sums + dWp from (dy3, y2) per frame (skinny blocks)");
    m.def("proj_bwd_supported", &proj_bwd_supported);
    m.def("attn_keepmask", &attn_keepmask, py::arg("BH"), py::arg("S"), py::arg("drop_p"), py::arg("seed"),
          py::arg("like"), py::arg("seed_dev") = py::none());
    m.def("attn_bwd", &attn_bwd, py::arg("qkv"), py::arg("out"), py::arg("dout"), py::arg("lse"), py::arg("L"),
          py::arg("Kimg"), py::arg("scale"), py::arg("drop_p"), py::arg("seed"), py::arg("seed_dev") = py::none());
    m.def("tf_ln_fwd", &tf_ln_fwd);
    m.def("tf_ln_bwd", &tf_ln_bwd, py::arg("dy"), py::arg("x"), py::arg("mu"), py::arg("rs"), py::arg("g"),
          py::arg("dres") = py::none(), py::arg("want_bf") = false);
    m.def("tf_resid", &tf_resid, py::arg("x"), py::arg("a"), py::arg("bias"), py::arg("p"), py::arg("seed"),
          py::arg("seed_dev") = py::none(), py::arg("lg") = py::none(), py::arg("lb") = py::none(), py::arg("eps") = 1e-6);
    m.def("tf_drop_bwd", &tf_drop_bwd, py::arg("dout"), py::arg("p"), py::arg("seed"), py::arg("seed_dev") = py::none());
    m.def("pw_gemm_supported", &pw_gemm_supported);
    m.def("pw_stats_supported", &pw_stats_supported);
    m.def("add_scaled_", &add_scaled_);
    m.def("pw_bwd_supported", &pw_bwd_supported);
    m.def("pw_bwd", &pw_bwd);
    m.def("pw_bwd_z", &pw_bwd_z);
    m.def("pw_z_prep", &pw_z_prep);
    m.def("pw_gemm_bnbwd_supported", &pw_gemm_bnbwd_supported);
    m.def("pw_gemm_bnbwd", &pw_gemm_bnbwd);
    m.def("pw_tall_tail", &pw_tall_tail, py::arg("A"), py::arg("W"), py::arg("A2"), py::arg("W2"), py::arg("bias"),
          py::arg("res") = py::none(), py::arg("rmul") = py::none(), py::arg("rhw") = 1);
    m.def("pw_z_finish", &pw_z_finish);
    rt1comm::register_comm(m);
    rt1head::register_head(m);
    m.def("pw_gemm", &pw_gemm, py::arg("A"), py::arg("B"), py::arg("max_blocks"), py::arg("stats") = false,
          py::arg("scale") = py::none(), py::arg("shift") = py::none(), py::arg("gate") = py::none(),
          py::arg("hw") = 0, py::arg("store_operand") = false);
}
