// Python bindings for the fused action head (csrc/kernels/head.hip) and the streamed long-history
// attention backward (csrc/kernels/attention.hip, rt1_attn_bwd_long).  Same rules as bindings.cpp: every
// shape / dtype / device is validated on the host before a launch, launches go to torch's current stream.
#include <cstdlib>

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "rt1_kernels.h"

namespace rt1head {
namespace {

using OptT = c10::optional<at::Tensor>;

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

uint16_t* bp(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

const uint32_t* seed_ptr(const OptT& t) {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "seed_dev must be a GPU int32 tensor");
    return reinterpret_cast<const uint32_t*>(t->data_ptr());
}

bool head_ce_supported(int64_t V, int64_t E) { return rt1_head_ce_supported((int)V, (int)E) != 0; }

// hidden [B, S, 512] fp32, pos [P] int32 (values in [0, S), clamped in-kernel), W [V, 512] bf16, bias [V] fp32,
// target [B*P] int32  ->  ce [R] fp32, pred [R] int32, G [R, V] bf16, hb [R, 512] bf16   (R = B*P)
std::vector<at::Tensor> head_ce_fwd(at::Tensor hidden, at::Tensor pos, at::Tensor W, at::Tensor bias, at::Tensor target) {
    check_dev(hidden, "hidden", at::kFloat);
    check_dev(pos, "pos", at::kInt);
    check_dev(W, "W", at::kBFloat16);
    check_dev(bias, "bias", at::kFloat);
    check_dev(target, "target", at::kInt);
    TORCH_CHECK(hidden.dim() == 3, "hidden must be [B, S, E]");
    const int64_t B = hidden.size(0), S = hidden.size(1), E = hidden.size(2);
    TORCH_CHECK(W.dim() == 2 && W.size(1) == E, "W must be [V, E]");
    const int64_t V = W.size(0);
    TORCH_CHECK(rt1_head_ce_supported((int)V, (int)E), "head_ce: no specialisation for V=", V, " E=", E);
    TORCH_CHECK(bias.numel() == V, "bias must have V elements");
    TORCH_CHECK(pos.dim() == 1 && pos.numel() >= 1 && pos.numel() <= S, "pos must be [P], P <= S");
    const int64_t P = pos.numel(), R = B * P;
    TORCH_CHECK(target.numel() == R, "target must have B*P elements");
    TORCH_CHECK(R > 0 && R < (int64_t)1 << 30, "bad row count");
    auto ce = at::empty({R}, hidden.options());
    auto pred = at::empty({R}, pos.options());
    auto G = at::empty({R, V}, W.options());
    auto hb = at::empty({R, E}, W.options());
    check_launch(rt1_head_ce_fwd(hidden.data_ptr<float>(), pos.data_ptr<int>(), bp(W), bias.data_ptr<float>(),
                                 target.data_ptr<int>(), (int)R, (int)P, (int)S, (int)V, ce.data_ptr<float>(),
                                 pred.data_ptr<int>(), bp(G), bp(hb), cur_stream()), "head_ce_fwd");
    return {ce, pred, G, hb};
}

// action tokens of the concatenated components in one launch: comps[i] is Box fp32 [..., dims[i]] (dims[i] > 0) or
// Discrete int64 / int32 [...] (dims[i] == 0); low / high: one value per token.  -> (int64 [..., A], int32 [..., A])
std::vector<at::Tensor> action_tokenize(std::vector<at::Tensor> comps, std::vector<int64_t> dims, std::vector<double> low,
                                        std::vector<double> high, int64_t vocab) {
    TORCH_CHECK(!comps.empty() && comps.size() == dims.size() && comps.size() <= 8, "action_tokenize: 1..8 components");
    std::vector<const void*> ptrs;
    std::vector<int> kind, dim;
    int64_t rows = -1, A = 0;
    std::vector<int64_t> lead;
    for (size_t i = 0; i < comps.size(); ++i) {
        const at::Tensor& c = comps[i];
        TORCH_CHECK(c.is_cuda() && c.is_contiguous(), "action_tokenize: contiguous GPU components");
        int64_t r;
        if (dims[i] > 0) {
            TORCH_CHECK(c.scalar_type() == at::kFloat && c.size(-1) == dims[i], "action_tokenize: Box component ", i,
                        " must be fp32 [..., ", dims[i], "]");
            r = c.numel() / dims[i];
            kind.push_back(0);
            if (lead.empty()) lead = c.sizes().vec(), lead.pop_back();
        } else {
            TORCH_CHECK(c.scalar_type() == at::kLong || c.scalar_type() == at::kInt, "action_tokenize: Discrete ", i,
                        " must be int64 / int32");
            r = c.numel();
            kind.push_back(c.scalar_type() == at::kLong ? 1 : 2);
            if (lead.empty()) lead = c.sizes().vec();
        }
        TORCH_CHECK(rows < 0 || r == rows, "action_tokenize: components disagree on the number of rows");
        rows = r;
        dim.push_back(dims[i] > 0 ? (int)dims[i] : 1);
        A += dim.back();
        ptrs.push_back(c.data_ptr());
    }
    TORCH_CHECK(A <= 32 && (int64_t)low.size() == A && (int64_t)high.size() == A, "action_tokenize: low / high per token");
    TORCH_CHECK(rows > 0 && rows * A < ((int64_t)1 << 31), "action_tokenize: bad row count");
    std::vector<float> lo(low.begin(), low.end()), hi(high.begin(), high.end());
    lead.push_back(A);
    auto out64 = at::empty(lead, comps[0].options().dtype(at::kLong));
    auto out32 = at::empty(lead, comps[0].options().dtype(at::kInt));
    check_launch(rt1_action_tokenize(ptrs.data(), kind.data(), dim.data(), (int)comps.size(), lo.data(), hi.data(),
                                     (int)rows, (int)vocab, out64.data_ptr<int64_t>(), out32.data_ptr<int>(),
                                     cur_stream()), "action_tokenize");
    return {out64, out32};
}

// dz = G * dce[:, None] (bf16)
at::Tensor head_ce_scale(at::Tensor G, at::Tensor dce) {
    check_dev(G, "G", at::kBFloat16);
    check_dev(dce, "dce", at::kFloat);
    TORCH_CHECK(G.dim() == 2 && G.size(1) % 8 == 0, "G must be [R, V], V % 8 == 0");
    TORCH_CHECK(dce.numel() == G.size(0), "dce must have R elements");
    auto dz = at::empty_like(G);
    check_launch(rt1_head_ce_scale(bp(G), dce.data_ptr<float>(), (int)G.size(0), (int)G.size(1), bp(dz), cur_stream()),
                 "head_ce_scale");
    return dz;
}

// dqkv [B, S, 3, H, 128] for S <= 256 (two streamed kernels; the S <= 96 single-kernel path is attn_bwd)
at::Tensor attn_bwd_long(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse, int64_t L, int64_t Kimg,
                         double scale, double drop_p, int64_t seed, OptT seed_dev) {
    check_dev(qkv, "qkv", at::kBFloat16);
    check_dev(out, "out", at::kBFloat16);
    check_dev(dout, "dout", at::kBFloat16);
    check_dev(lse, "lse", at::kFloat);
    TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 128, "qkv must be [B, S, 3, H, 128]");
    const int B = (int)qkv.size(0), S = (int)qkv.size(1), H = (int)qkv.size(3);
    TORCH_CHECK(S >= 1 && S <= 256, "attn_bwd_long supports S <= 256");
    TORCH_CHECK(L > 0 && Kimg >= 0 && Kimg <= L, "bad token layout");
    TORCH_CHECK(out.sizes() == at::IntArrayRef({B, S, H, 128}) && dout.sizes() == out.sizes(), "out/dout [B,S,H,128]");
    TORCH_CHECK(lse.numel() == (int64_t)B * H * S, "lse must be [B, H, S]");
    auto dqkv = at::empty_like(qkv);
    check_launch(rt1_attn_bwd_long(bp(qkv), bp(out), bp(dout), lse.data_ptr<float>(), bp(dqkv), B, S, H, (int)L,
                                   (int)Kimg, (float)scale, (float)drop_p, (uint32_t)seed, seed_ptr(seed_dev),
                                   cur_stream()), "attn_bwd_long");
    return dqkv;
}

bool tl_supported(int64_t P, int64_t Cc, int64_t h1, int64_t t) {
    return rt1_tl_supported((int)P, (int)Cc, (int)h1, (int)t) != 0;
}

void check_f(const at::Tensor& t, const char* name, int64_t numel) {
    check_dev(t, name, at::kFloat);
    TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
}

// x [N, P, 512] bf16 -> out [N, 8, 512] bf16, mu / rstd [N, P], z1 [N, P, 64] bf16, s [N, 8, P] fp32
std::vector<at::Tensor> tl_fwd(at::Tensor x, at::Tensor gamma, at::Tensor beta, double eps, at::Tensor W1,
                               at::Tensor b1, at::Tensor W2, at::Tensor b2) {
    check_dev(x, "x", at::kBFloat16);
    TORCH_CHECK(x.dim() == 3 && x.size(2) == 512, "x must be [N, P, 512]");
    const int64_t N = x.size(0), P = x.size(1);
    TORCH_CHECK(rt1_tl_supported((int)P, 512, 64, 8), "tl_fwd: unsupported P=", P);
    check_f(gamma, "gamma", 512); check_f(beta, "beta", 512);
    check_dev(W1, "W1", at::kBFloat16);
    TORCH_CHECK(W1.numel() == 64 * 512, "W1 must be [64, 512]");
    check_f(b1, "b1", 64); check_f(W2, "W2", 8 * 64); check_f(b2, "b2", 8);
    auto f = x.options().dtype(at::kFloat);
    auto out = at::empty({N, 8, 512}, x.options());
    auto mu = at::empty({N, P}, f), rs = at::empty({N, P}, f);
    auto z1 = at::empty({N, P, 64}, x.options());
    auto s = at::empty({N, 8, P}, f);
    check_launch(rt1_tl_fwd(bp(x), gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)eps, bp(W1),
                            b1.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(), (int)N, (int)P, bp(out),
                            mu.data_ptr<float>(), rs.data_ptr<float>(), bp(z1), s.data_ptr<float>(), cur_stream()),
                 "tl_fwd");
    return {out, mu, rs, z1, s};
}

// -> dx [N, P, 512] bf16, dz1 [N*P, 64] bf16, xn [N*P, 512] bf16, pw2 [N, 8, 65] (dW2 | db2), pg [N, 2, 512]
std::vector<at::Tensor> tl_bwd(at::Tensor x, at::Tensor dO, at::Tensor s, at::Tensor z1, at::Tensor mu, at::Tensor rs,
                               at::Tensor gamma, at::Tensor beta, at::Tensor W1T, at::Tensor W2) {
    check_dev(x, "x", at::kBFloat16);
    TORCH_CHECK(x.dim() == 3 && x.size(2) == 512, "x must be [N, P, 512]");
    const int64_t N = x.size(0), P = x.size(1);
    TORCH_CHECK(rt1_tl_supported((int)P, 512, 64, 8), "tl_bwd: unsupported P=", P);
    check_dev(dO, "dO", at::kBFloat16);
    TORCH_CHECK(dO.numel() == N * 8 * 512, "dO must be [N, 8, 512]");
    check_f(s, "s", N * 8 * P);
    check_dev(z1, "z1", at::kBFloat16);
    TORCH_CHECK(z1.numel() == N * P * 64, "z1 must be [N, P, 64]");
    check_f(mu, "mu", N * P); check_f(rs, "rs", N * P); check_f(gamma, "gamma", 512); check_f(beta, "beta", 512);
    check_dev(W1T, "W1T", at::kBFloat16);
    TORCH_CHECK(W1T.numel() == 512 * 64, "W1T must be [512, 64]");
    check_f(W2, "W2", 8 * 64);
    auto f = x.options().dtype(at::kFloat);
    auto dx = at::empty_like(x);
    auto dz1 = at::empty({N * P, 64}, x.options());
    auto xn = at::empty({N * P, 512}, x.options());
    auto pw2 = at::empty({N, 8, 65}, f);
    auto pg = at::empty({N, 2, 512}, f);
    check_launch(rt1_tl_bwd(bp(x), bp(dO), s.data_ptr<float>(), bp(z1), mu.data_ptr<float>(), rs.data_ptr<float>(),
                            gamma.data_ptr<float>(), beta.data_ptr<float>(), bp(W1T), W2.data_ptr<float>(), (int)N,
                            (int)P, bp(dx), bp(dz1), bp(xn), pw2.data_ptr<float>(), pg.data_ptr<float>(), cur_stream()),
                 "tl_bwd");
    return {dx, dz1, xn, pw2, pg};
}


bool pw_tall_supported(int64_t K, int64_t N) { return rt1_pw_tall_supported((int)K, (int)N) != 0; }
bool pw_tall_preferred(int64_t K, int64_t N) { return rt1_pw_tall_preferred((int)K, (int)N) != 0; }

// A [M, K] bf16 @ W [N, K]^T bf16 -> C [M, N] bf16 (wide reduction, narrow output; csrc/kernels/pwtall.hip)
std::vector<at::Tensor> pw_tall(at::Tensor A, at::Tensor W, OptT scale, OptT shift, OptT gate, int64_t hw,
                                bool store_operand) {
    check_dev(A, "A", at::kBFloat16);
    check_dev(W, "W", at::kBFloat16);
    TORCH_CHECK(A.dim() == 2 && W.dim() == 2 && A.size(1) == W.size(1), "pw_tall: A [M, K], W [N, K] expected");
    const int64_t M = A.size(0), K = A.size(1), N = W.size(0);
    TORCH_CHECK(M > 0 && M < (int64_t)1 << 31, "pw_tall: M out of range");
    TORCH_CHECK(rt1_pw_tall_supported((int)K, (int)N), "pw_tall: unsupported shape K=", K, " N=", N);
    TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0,
                "pw_tall: operands must be 16-byte aligned");
    auto C = at::empty({M, N}, A.options());
    const bool pro = scale.has_value() && scale->defined();
    at::Tensor aout;
    if (pro) {
        check_dev(*scale, "scale", at::kFloat);
        TORCH_CHECK(shift.has_value() && shift->defined() && gate.has_value() && gate->defined(),
                    "pw_tall: the operand prologue needs scale, shift and gate");
        check_dev(*shift, "shift", at::kFloat);
        check_dev(*gate, "gate", at::kFloat);
        TORCH_CHECK(scale->numel() == K && shift->numel() == K && hw > 0 && M % hw == 0 && gate->numel() == (M / hw) * K,
                    "pw_tall: prologue shapes (scale/shift [K], gate [M / hw, K])");
        if (store_operand) aout = at::empty({M, K}, A.options());
    }
    check_launch(rt1_pw_tall(bp(A), bp(W), (int)M, (int)K, (int)N, bp(C), pro ? scale->data_ptr<float>() : nullptr,
                             pro ? shift->data_ptr<float>() : nullptr, pro ? gate->data_ptr<float>() : nullptr,
                             (int)hw, aout.defined() ? bp(aout) : nullptr, cur_stream()), "pw_tall");
    if (aout.defined()) return {C, aout};
    return {C};
}

// tokens [B, S, K] bf16, W [N, K] bf16, bias [N] fp32, pos [>= S, N] fp32 -> [B, S, N] fp32
at::Tensor embed_fwd(at::Tensor x, at::Tensor W, at::Tensor bias, at::Tensor pos) {
    check_dev(x, "x", at::kBFloat16);
    check_dev(W, "W", at::kBFloat16);
    TORCH_CHECK(x.dim() == 3 && W.dim() == 2 && x.size(2) == W.size(1), "embed_fwd: x [B, S, K], W [N, K]");
    const int64_t B = x.size(0), S = x.size(1), K = x.size(2), N = W.size(0);
    check_f(bias, "bias", N);
    check_dev(pos, "pos", at::kFloat);
    TORCH_CHECK(pos.dim() == 2 && pos.size(1) == N && pos.size(0) >= S, "embed_fwd: pos must be [>= S, N]");
    TORCH_CHECK(K % 8 == 0 && N % 16 == 0 && B * S > 0 && B * S < (int64_t)1 << 31, "embed_fwd: unsupported shape");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0,
                "embed_fwd: operands must be 16-byte aligned");
    auto out = at::empty({B, S, N}, x.options().dtype(at::kFloat));
    check_launch(rt1_embed_fwd(bp(x), bp(W), bias.data_ptr<float>(), pos.data_ptr<float>(), (int)(B * S), (int)K,
                               (int)N, (int)S, out.data_ptr<float>(), cur_stream()), "embed_fwd");
    return out;
}

// SE backward glue (csrc/kernels/se.hip).  dsum, gate [N, C] fp32 -> dz [N, C], db [C]
std::vector<at::Tensor> se_bwd_dz(at::Tensor dsum, at::Tensor gate) {
    check_dev(dsum, "dsum", at::kFloat);
    check_dev(gate, "gate", at::kFloat);
    TORCH_CHECK(dsum.dim() == 2 && gate.sizes() == dsum.sizes(), "se_bwd_dz: dsum / gate must be [N, C]");
    auto dz = at::empty_like(dsum);
    auto db = at::empty({dsum.size(1)}, dsum.options());
    check_launch(rt1_se_bwd_dz(dsum.data_ptr<float>(), gate.data_ptr<float>(), (int)dsum.size(0), (int)dsum.size(1),
                               dz.data_ptr<float>(), db.data_ptr<float>(), cur_stream()), "se_bwd_dz");
    return {dz, db};
}

// dzf2, h [N, S] fp32 -> dh [N, S], db [S]
std::vector<at::Tensor> se_bwd_dh(at::Tensor dzf2, at::Tensor h) {
    check_dev(dzf2, "dzf2", at::kFloat);
    check_dev(h, "h", at::kFloat);
    TORCH_CHECK(dzf2.dim() == 2 && h.sizes() == dzf2.sizes(), "se_bwd_dh: dzf2 / h must be [N, S]");
    auto dh = at::empty_like(dzf2);
    auto db = at::empty({dzf2.size(1)}, dzf2.options());
    check_launch(rt1_se_bwd_dh(dzf2.data_ptr<float>(), h.data_ptr<float>(), (int)dzf2.size(0), (int)dzf2.size(1),
                               dh.data_ptr<float>(), db.data_ptr<float>(), cur_stream()), "se_bwd_dh");
    return {dh, db};
}

// red [5, N, C], gate, rbraw [N, C] fp32 -> rb [N, C], sdz, sdzx, mdz, mdzx [C]
// Whole SE MLP forward (csrc/kernels/se.hip se_rowdot + se_rowmat): pool_sum [N, C] (frame_pool) -> {pool_sum (kept:
// the backward takes frame sums), h = fc1 pre-activation [N, S], gate = sigmoid(fc2(silu(h))) [N, C]};
// w1 [S, C], b1 [S], w2 [C, S], b2 [C] fp32.
std::vector<at::Tensor> se_fwd(at::Tensor pool_sum, double inv_hw, at::Tensor w1, at::Tensor b1, at::Tensor w2,
                               at::Tensor b2) {
    check_dev(pool_sum, "pool_sum", at::kFloat);
    TORCH_CHECK(pool_sum.dim() == 2, "se_fwd: pool_sum must be [N, C]");
    const int64_t N = pool_sum.size(0), C = pool_sum.size(1);
    check_dev(w1, "w1", at::kFloat); check_dev(b1, "b1", at::kFloat);
    check_dev(w2, "w2", at::kFloat); check_dev(b2, "b2", at::kFloat);
    const int64_t S = b1.numel();
    TORCH_CHECK(w1.numel() == S * C && w2.numel() == C * S && b2.numel() == C, "se_fwd: weight shapes");
    TORCH_CHECK(C % 4 == 0 && S <= 128, "se_fwd: C % 4 == 0 and S <= 128 required");
    auto gate = at::empty_like(pool_sum);
    auto h = at::empty({N, S}, pool_sum.options());
    auto part = at::empty({(int64_t)rt1_se_part_size((int)N, (int)C, (int)S)}, pool_sum.options());
    check_launch(rt1_se_fwd(pool_sum.data_ptr<float>(), (float)inv_hw, (int)N, (int)C, (int)S, w1.data_ptr<float>(),
                            b1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(), part.data_ptr<float>(),
                            h.data_ptr<float>(), gate.data_ptr<float>(), cur_stream()), "se_fwd");
    return {pool_sum, h, gate};
}

// Whole SE + BN2 backward glue (se_rowdot + se_rowmat + se_wsum_part + se_wsum_fin): red [5, N, C] from
// se_bn_bwd_reduce / proj_bwd, gate / pool SUMS [N, C], h [N, S] -> {dw2 [C, S], db2 [C], dw1 [S, C], db1 [S],
// rb [N, C], sdz, sdzx, mdz, mdzx [C]}
std::vector<at::Tensor> se_bwd(at::Tensor red, at::Tensor gate, at::Tensor h, at::Tensor pool, double inv_hw,
                               at::Tensor w1, at::Tensor w2, double count) {
    check_dev(red, "red", at::kFloat); check_dev(gate, "gate", at::kFloat);
    check_dev(h, "h", at::kFloat); check_dev(pool, "pool", at::kFloat);
    check_dev(w1, "w1", at::kFloat); check_dev(w2, "w2", at::kFloat);
    TORCH_CHECK(gate.dim() == 2 && pool.sizes() == gate.sizes(), "se_bwd: gate / pool must be [N, C]");
    const int64_t N = gate.size(0), C = gate.size(1), S = h.size(1);
    TORCH_CHECK(h.dim() == 2 && h.size(0) == N, "se_bwd: h must be [N, S]");
    TORCH_CHECK(red.dim() == 3 && red.size(0) == 5 && red.size(1) == N && red.size(2) == C, "red must be [5, N, C]");
    TORCH_CHECK(w1.numel() == S * C && w2.numel() == C * S, "se_bwd: weight shapes");
    TORCH_CHECK(C % 4 == 0 && S <= 128, "se_bwd: C % 4 == 0 and S <= 128 required");
    auto f = gate.options();
    auto rb = at::empty_like(gate);
    auto dh = at::empty({N, S}, f);
    auto part = at::empty({(int64_t)rt1_se_part_size((int)N, (int)C, (int)S)}, f);
    auto ws = at::empty({(int64_t)((rt1_se_wsum_ws_bytes((int)N, (int)C, (int)S) + 7) / 8)}, f.dtype(at::kDouble));
    auto dw2 = at::empty({C, S}, f), dw1 = at::empty({S, C}, f), db2 = at::empty({C}, f), db1 = at::empty({S}, f);
    auto sdz = at::empty({C}, f), sdzx = at::empty({C}, f), mdz = at::empty({C}, f), mdzx = at::empty({C}, f);
    check_launch(rt1_se_bwd_frame(red.data_ptr<float>(), gate.data_ptr<float>(), h.data_ptr<float>(), (float)inv_hw,
                                  (int)N, (int)C, (int)S, w1.data_ptr<float>(), w2.data_ptr<float>(),
                                  part.data_ptr<float>(), dh.data_ptr<float>(), rb.data_ptr<float>(), cur_stream()),
                 "se_bwd_frame");
    check_launch(rt1_se_bwd_wsum(red.data_ptr<float>(), gate.data_ptr<float>(), h.data_ptr<float>(),
                                 dh.data_ptr<float>(), pool.data_ptr<float>(), rb.data_ptr<float>(), (int)N, (int)C,
                                 (int)S, (float)inv_hw, count, ws.data_ptr<double>(), dw2.data_ptr<float>(),
                                 dw1.data_ptr<float>(), db2.data_ptr<float>(), db1.data_ptr<float>(),
                                 sdz.data_ptr<float>(), sdzx.data_ptr<float>(), mdz.data_ptr<float>(),
                                 mdzx.data_ptr<float>(), cur_stream()), "se_bwd_wsum");
    return {dw2, db2, dw1, db1, rb, sdz, sdzx, mdz, mdzx};
}

std::vector<at::Tensor> se_bwd_bnsum(at::Tensor red, at::Tensor gate, at::Tensor rbraw, double inv_hw, double count) {
    check_dev(red, "red", at::kFloat);
    check_dev(gate, "gate", at::kFloat);
    check_dev(rbraw, "rbraw", at::kFloat);
    TORCH_CHECK(gate.dim() == 2 && rbraw.sizes() == gate.sizes(), "se_bwd_bnsum: gate / rbraw must be [N, C]");
    const int64_t N = gate.size(0), C = gate.size(1);
    TORCH_CHECK(red.dim() == 3 && red.size(0) == 5 && red.size(1) == N && red.size(2) == C, "red must be [5, N, C]");
    auto rb = at::empty_like(gate);
    auto f = gate.options();
    auto sdz = at::empty({C}, f), sdzx = at::empty({C}, f), mdz = at::empty({C}, f), mdzx = at::empty({C}, f);
    check_launch(rt1_se_bwd_bnsum(red.data_ptr<float>(), gate.data_ptr<float>(), rbraw.data_ptr<float>(), (float)inv_hw,
                                  (int)N, (int)C, count, rb.data_ptr<float>(), sdz.data_ptr<float>(),
                                  sdzx.data_ptr<float>(), mdz.data_ptr<float>(), mdzx.data_ptr<float>(), cur_stream()),
                 "se_bwd_bnsum");
    return {rb, sdz, sdzx, mdz, mdzx};
}

}  // namespace

void register_head(py::module_& m) {
    m.def("action_tokenize", &action_tokenize);
    m.def("se_bwd_dz", &se_bwd_dz);
    m.def("se_bwd_dh", &se_bwd_dh);
    m.def("se_fwd", &se_fwd);
    m.def("se_bwd", &se_bwd);
    m.def("se_bwd_bnsum", &se_bwd_bnsum);
    m.def("embed_fwd", &embed_fwd);
    m.def("pw_tall_supported", &pw_tall_supported);
    m.def("pw_tall", &pw_tall, py::arg("A"), py::arg("W"), py::arg("scale") = py::none(), py::arg("shift") = py::none(),
          py::arg("gate") = py::none(), py::arg("hw") = 0, py::arg("store_operand") = false);
    m.def("pw_tall_preferred", &pw_tall_preferred);
    m.def("tl_supported", &tl_supported);
    m.def("tl_fwd", &tl_fwd);
    m.def("tl_bwd", &tl_bwd);
    m.def("head_ce_supported", &head_ce_supported);
    m.def("head_ce_fwd", &head_ce_fwd);
    m.def("head_ce_scale", &head_ce_scale);
    m.def("attn_bwd_long", &attn_bwd_long, py::arg("qkv"), py::arg("out"), py::arg("dout"), py::arg("lse"),
          py::arg("L"), py::arg("Kimg"), py::arg("scale"), py::arg("drop_p"), py::arg("seed"),
          py::arg("seed_dev") = py::none());
}

}  // namespace rt1head
