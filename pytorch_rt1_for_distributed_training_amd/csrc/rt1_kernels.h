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
// graph-replayable variant: state = {step, lr} on the device (the step is advanced by the caller's device op)
int rt1_flat_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* state, float beta1,
                      float beta2, float eps, float weight_decay, float grad_scale, hipStream_t stream);

}  // extern "C"

extern "C" {
typedef uint16_t rt1_bf16;

// bn.hip
int rt1_bn_stats(const rt1_bf16* x, int64_t M, int C, int P, float* psum, float* psq, hipStream_t st);
int rt1_bn_finalize(const float* psum, const float* psq, int P, int C, double count, const float* gamma,
                    const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                    float* scale, float* shift, float* save_mean, float* save_rstd, hipStream_t st);
int rt1_bn_apply(const rt1_bf16* y, int64_t M, int C, const float* scale, const float* shift, int act, const float* rs,
                 int64_t HW, rt1_bf16* out, hipStream_t st);
int rt1_bn_bwd_reduce(const rt1_bf16* G, const float* rs, const float* rb, int64_t HW, const rt1_bf16* y, int64_t M,
                      int C, const float* scale, const float* shift, const float* mean, const float* rstd, int act,
                      int P, float* pdz, float* pdzx, hipStream_t st);
int rt1_bn_bwd_finalize_consts(const float* pdz, const float* pdzx, int P, int C, double count, float* dgamma,
                               float* dbeta, float* mdz, float* mdzx, const float* scale, const float* shift,
                               const float* gamma, const float* mean, const float* rstd, float* consts,
                               hipStream_t st);
int rt1_bn_bwd_finalize(const float* pdz, const float* pdzx, int P, int C, double count, float* dgamma, float* dbeta,
                        float* mdz, float* mdzx, hipStream_t st, int accumulate);
int rt1_bn_bwd_apply(const rt1_bf16* G, const float* rs, const float* rb, int64_t HW, const rt1_bf16* y, int64_t M,
                     int C, const float* scale, const float* shift, const float* mean, const float* rstd,
                     const float* gamma, int act, const float* mdz, const float* mdzx, rt1_bf16* dy, hipStream_t st,
                     const float* keep = nullptr);   // keep [N]: rs[n] * keep[n] (the drop-path mask)

// dwconv.hip
int rt1_dw_grid(int N, int H, int W, int C, int k, int s, int max_blocks_x, int pro, int epi);
int rt1_dw_wgrad_grid(int N, int H, int W, int C, int k, int s, int max_blocks_x, int pro);
int rt1_dw_bwd_grid(int N, int H, int W, int C, int k, int s, int max_blocks_x, int epi);
int rt1_dw_fwd(const rt1_bf16* x, const float* w, const float* scale, const float* shift, int act, int N, int H, int W,
               int C, int k, int s, int grid_x, rt1_bf16* out, float* psum, float* psq, hipStream_t st);
int rt1_dw_bwd_data(const rt1_bf16* dy, const float* w, const float* wflip, int N, int H, int W, int C, int k, int s,
                    int grid_x,
                    rt1_bf16* dx, const rt1_bf16* y_in, const float* scale, const float* shift, const float* mean,
                    const float* rstd, float* pdz, float* pdzx, hipStream_t st);
int rt1_dw_bwd_weight(const rt1_bf16* dy, const rt1_bf16* x, const float* scale, const float* shift, int act, int N,
                      int H, int W, int C, int k, int s, int grid_x, float* dwp, hipStream_t st);
int rt1_dw_bwd_uses_uni(int variant, int pro, int epi);
int rt1_dw_bwd_fused_s2_grid(int N, int H, int W, int C, int k, int max_blocks_x, int epi, int cin);
int rt1_dw_bwd_fused_s2(const rt1_bf16* dA, const rt1_bf16* y2, const float* gate, const float* rb,
                        const float* scale2, const float* shift2, const float* mean2, const float* rstd2,
                        const float* gamma2, const float* mdz2, const float* mdzx2, const float* w,
                        const rt1_bf16* x1, const float* scale1, const float* shift1, const float* mean1,
                        const float* rstd1, int N, int H, int W, int C, int k, int grid_x, rt1_bf16* dx, float* pdz,
                        float* pdzx, float* dwp, hipStream_t st, int zout, const rt1_bf16* xin,
                        const rt1_bf16* we, int cin);
int rt1_dw_bwd_fused_grid(int N, int H, int W, int C, int k, int max_blocks_x, int pro, int epi, int variant,
                          int cin);
int rt1_dw_bwd_fused(const rt1_bf16* dA, const rt1_bf16* y2, const float* gate, const float* rb, const float* scale2,
                     const float* shift2, const float* mean2, const float* rstd2, const float* gamma2,
                     const float* mdz2, const float* mdzx2, const float* w, const float* wflip, const rt1_bf16* x1,
                     const float* scale1,
                     const float* shift1, int act1, const float* mean1, const float* rstd1, int N, int H, int W, int C,
                     int k, int grid_x, rt1_bf16* dx, float* pdz, float* pdzx, float* dwp, hipStream_t st,
                     int variant, int zout, const rt1_bf16* xin, const rt1_bf16* we, int cin,
                     const rt1_bf16* res = nullptr, const float* rmul = nullptr);
// x-mode (y1-free expand blocks): y1 = x @ we^T recomputed on MFMA inside the depthwise kernels
int rt1_dw_x_supported(int cin, int C, int k, int s);
int rt1_dw_grid_x(int N, int H, int W, int C, int k, int s, int cin, int max_blocks_x);
int rt1_dw_tile_info(int which, int H, int W, int C, int k, int s, int cin, int* out);
int rt1_dw_fwd_x(const rt1_bf16* x, int cin, const rt1_bf16* we, const float* w, const float* scale1,
                 const float* shift1, int N, int H, int W, int C, int k, int s, int grid_x, rt1_bf16* out, float* psum,
                 float* psq, hipStream_t st);
// gemm.hip: tiled MFMA GEMM, NT / NN operands, bias / BN-stat epilogues, BN+SiLU+gate A prologue
int rt1_gemm_tiles_m(int M, int N, int K, int cfg);
int rt1_gemm_cmap(const rt1_bf16* A, int lda, const rt1_bf16* B, float* C, int M, int N, int K, const float* bias,
                  const int* cmap, int cfg, hipStream_t st);
int rt1_gemm(const rt1_bf16* A, const rt1_bf16* B, void* C, int M, int N, int K, int nn, const float* bias,
             const float* scale, const float* shift, const float* gate, int hw, int out_f32, float* ps, float* pq,
             int cfg, rt1_bf16* aout, hipStream_t st);
int rt1_gemm_tail(const rt1_bf16* A, const rt1_bf16* B, int M, int N, int K, const rt1_bf16* A2, const rt1_bf16* B2,
                  int K2, const float* bias, const rt1_bf16* res, const float* rmul, int rhw, rt1_bf16* C, int cfg,
                  hipStream_t st);
// gemm256.hip: 256 x {256, 128} LDS-DMA MFMA GEMM, NT / NN operands, bias / BN-stat epilogues, PRO A prologue
int rt1_g256_tiles_m(int M);
int rt1_g256(const rt1_bf16* A, const rt1_bf16* B, rt1_bf16* C, int M, int N, int K, int nn, const float* bias,
             const float* scale, const float* shift, const float* gate, int hw, rt1_bf16* aout, float* ps, float* pq,
             int bn, hipStream_t st);
// xexpand.hip: BN1 batch statistics of y1 = x @ we^T from G = x^T x and sx = sum x (fp64), + running stats
int rt1_xgram_grid(int64_t M, int cin);
int rt1_xgram(const rt1_bf16* x, int64_t M, int cin, int grid, float* work, double* out, hipStream_t st);
int rt1_bn_from_gram(const double* G, const double* sx, const rt1_bf16* we, int cin, int C, double count,
                     const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                     float* running_var, float* scale, float* shift, float* save_mean, float* save_rstd,
                     hipStream_t st);
int rt1_bn_from_wg(const float* WG, const float* sx, const rt1_bf16* we, int cin, int C, double count,
                         const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                         float* running_var, float* scale, float* shift, float* save_mean, float* save_rstd,
                         hipStream_t st);

// block.hip
int rt1_frame_splits(int N, int HW, int C);
int rt1_frame_pool(const rt1_bf16* y, const rt1_bf16* G, int N, int HW, int C, const float* scale, const float* shift,
                   int act, int splits, float* pool, hipStream_t st);
int rt1_se_bn_bwd_reduce(const rt1_bf16* G, const rt1_bf16* y, int N, int HW, int C, const float* scale,
                         const float* shift, const float* mean, const float* rstd, int splits, float* out,
                         hipStream_t st);
int rt1_block_tail(const rt1_bf16* y3, int64_t M, int HW, int C, const float* scale, const float* shift,
                   const float* keep, const rt1_bf16* skip, const float* fmul, const float* fadd, rt1_bf16* out,
                   hipStream_t st);
int rt1_tail_bwd_reduce(const rt1_bf16* dout, const rt1_bf16* y3, int N, int HW, int C, const float* scale,
                        const float* shift, const float* mean, const float* rstd, const float* keep,
                        const rt1_bf16* skip, const float* fmul, int splits, float* dmul, float* dadd, float* pdz,
                        float* pdzx, hipStream_t st);

// stem.hip
int rt1_stem_grid(int N, int H, int W, int max_blocks);
int rt1_stem_fwd(const void* img, int img_is_u8, const int* shift, const float* w, int N, int H, int W, int Cout,
                 int grid, rt1_bf16* out, float* psum, float* psq, hipStream_t st);
// bn_x != nullptr: dy holds the gradient of silu(bn(bn_x)); the BN backward (constants as in rt1_bn_bwd_apply) is
// applied while staging (stem.hip StemBnBwd)
int rt1_stem_bwd_weight(const void* img, int img_is_u8, const int* shift, const rt1_bf16* dy, int N, int H, int W,
                        int Cout, int grid, float* dwp, hipStream_t st, const rt1_bf16* bn_x = nullptr,
                        const float* bn_scale = nullptr, const float* bn_shift = nullptr,
                        const float* bn_mean = nullptr, const float* bn_rstd = nullptr,
                        const float* bn_gamma = nullptr, const float* bn_mdz = nullptr,
                        const float* bn_mdzx = nullptr);

// attention.hip
int rt1_attn_fwd(const rt1_bf16* qkv, rt1_bf16* out, float* lse, int B, int S, int H, int L, int Kimg, float scale,
                 float drop_p, uint32_t seed, const uint32_t* seed_dev, hipStream_t st);
int rt1_attn_keepmask(uint8_t* keep, int BH, int S, float drop_p, uint32_t seed, const uint32_t* seed_dev,
                      hipStream_t st);
int rt1_attn_bwd(const rt1_bf16* qkv, const rt1_bf16* out, const rt1_bf16* dout, const float* lse, rt1_bf16* dqkv,
                 int B, int S, int H, int L, int Kimg, float scale, float drop_p, uint32_t seed,
                 const uint32_t* seed_dev, hipStream_t st);

int rt1_attn_bwd_long(const rt1_bf16* qkv, const rt1_bf16* out, const rt1_bf16* dout, const float* lse,
                      rt1_bf16* dqkv, int B, int S, int H, int L, int Kimg, float scale, float drop_p, uint32_t seed,
                      const uint32_t* seed_dev, hipStream_t st);

// head.hip (fused action head: gather + logits GEMM + CE + argmax)
int rt1_action_tokenize(const void* const* comps, const int* kind, const int* dim, int n, const float* low,
                        const float* high, int rows, int V, int64_t* out64, int* out32, hipStream_t st);
int rt1_head_ce_supported(int V, int E);
int rt1_head_ce_fwd(const float* hidden, const int* pos, const rt1_bf16* W, const float* bias, const int* target,
                    int R, int P, int S, int V, float* ce, int* pred, rt1_bf16* G, rt1_bf16* hb, hipStream_t st);
int rt1_head_ce_scale(const rt1_bf16* G, const float* dce, int R, int V, rt1_bf16* dz, hipStream_t st);

// tokenlearner.hip (one workgroup per frame; P <= 256, C = 512, bottleneck 64, 8 tokens)
int rt1_tl_supported(int P, int C, int h1, int t);
int rt1_tl_fwd(const rt1_bf16* x, const float* gamma, const float* beta, float eps, const rt1_bf16* W1, const float* b1,
               const float* W2, const float* b2, int N, int P, rt1_bf16* out, float* mu, float* rs, rt1_bf16* z1,
               float* s, hipStream_t st);
int rt1_tl_bwd(const rt1_bf16* x, const rt1_bf16* dO, const float* s, const rt1_bf16* z1, const float* mu,
               const float* rs, const float* gamma, const float* beta, const rt1_bf16* W1T, const float* W2, int N,
               int P, rt1_bf16* dx, rt1_bf16* dz1, rt1_bf16* xn, float* pw2, float* pg, hipStream_t st);


int rt1_add_scaled(rt1_bf16* x, const rt1_bf16* y, const float* sc, int64_t M, int HW, int C, hipStream_t st);

// pwgemm.hip
int rt1_pw_gemm_supported(int K, int N);
int rt1_pw_gemm_grid(int M, int K, int N, int max_blocks);
int rt1_pw_gemm(const rt1_bf16* A, const rt1_bf16* B, int M, int K, int N, rt1_bf16* C, float* ps, float* pq,
                int max_blocks, const float* scale, const float* shift, const float* gate, int hw, rt1_bf16* aout,
                hipStream_t st);
// dA = dy3 @ W^T with the BN3-backward operand dy3 = k1 * (dout * fmul[frame] * keep[frame]) + k2 * y3 + k0 built in the
// prologue (bn_bwd_apply's formula) and stored to dy_out (pwgemm.hip, project data gradients of blocks 0-7)
int rt1_pw_gemm_bnbwd_supported(int K, int N);
int rt1_pw_gemm_bnbwd(const rt1_bf16* dout, const rt1_bf16* B, int M, int K, int N, rt1_bf16* C, int max_blocks,
                      const rt1_bf16* y, const float* fmul, const float* keep, int hw, const float* gamma,
                      const float* mean, const float* rstd, const float* mdz, const float* mdzx, rt1_bf16* dy_out,
                      hipStream_t st);

// transformer.hip (E = 512)
int rt1_tf_grid(int T);
int rt1_ln_fwd(const float* x, const float* g, const float* b, int T, float eps, rt1_bf16* y, float* mu, float* rs,
               hipStream_t st);
int rt1_ln_bwd(const rt1_bf16* dy, const float* x, const float* mu, const float* rs, const float* g, const float* dres,
               int T, float* dx, float* dgp, float* dbp, rt1_bf16* dxb, float* dsp, int grid, hipStream_t st);
int rt1_resid(const float* x, const rt1_bf16* a, const float* bias, int T, float p, uint32_t seed,
              const uint32_t* seed_dev, float* out, const float* lg, const float* lb, float eps, rt1_bf16* xn, float* mu,
              float* rs, hipStream_t st);
int rt1_drop_bwd(const float* dout, int T, float p, uint32_t seed, const uint32_t* seed_dev, rt1_bf16* dh, float* dbp,
                 int grid, hipStream_t st);

// se.hip (SE + BN2 backward glue of an MBConv block)
int rt1_se_part_size(int N, int C, int S);
int rt1_se_fwd(const float* pool_sum, float inv_hw, int N, int C, int S, const float* w1, const float* b1,
               const float* w2, const float* b2, float* part, float* h, float* gate, hipStream_t st);
int rt1_se_bwd_frame(const float* dsum, const float* gate, const float* h, float inv_hw, int N, int C, int S,
                     const float* w1, const float* w2, float* part, float* dh, float* rb, hipStream_t st);
size_t rt1_se_wsum_ws_bytes(int N, int C, int S);
int rt1_se_bwd_wsum(const float* red, const float* gate, const float* h, const float* dh, const float* pool,
                    const float* rb, int N, int C, int S, float inv_hw, double count, void* ws, float* dw2,
                    float* dw1, float* db2, float* db1, float* sdz, float* sdzx, float* mdz, float* mdzx,
                    hipStream_t st);
int rt1_se_bwd_dz(const float* dsum, const float* gate, int N, int C, float* dz, float* db, hipStream_t st);
int rt1_se_bwd_dh(const float* dzf2, const float* h, int N, int S, float* dh, float* db, hipStream_t st);
int rt1_se_bwd_bnsum(const float* red, const float* gate, const float* rbraw, float inv_hw, int N, int C, double count,
                     float* rb, float* sdz, float* sdzx, float* mdz, float* mdzx, hipStream_t st);

// pwtall.hip (wide reduction, narrow output: K >= 256, N <= 384)
int rt1_pw_tall_supported(int K, int N);
int rt1_pw_tall_preferred(int K, int N);
int rt1_pw_tall(const rt1_bf16* A, const rt1_bf16* W, int M, int K, int N, rt1_bf16* C, const float* scale,
                const float* shift, const float* gate, int hw, rt1_bf16* aout, hipStream_t st);
int rt1_embed_fwd(const rt1_bf16* A, const rt1_bf16* W, const float* bias, const float* pos, int M, int K, int N, int S,
                  float* out, hipStream_t st);

int rt1_pw_wide_supported(int K, int N);
int rt1_pw_wide(const rt1_bf16* A, const rt1_bf16* B, int M, int K, int N, rt1_bf16* C, int max_blocks, hipStream_t st);

// reduce.hip (deterministic column sums; pass-1 chunks from rt1_colsum_chunks, tmp = B x [chunks, C] fp32)
int rt1_colsum_chunks(int64_t R, int C, int B);
// fp32 copies src[i] -> dst[i] (n[i] elements), count <= 32, one launch
int rt1_multi_copy(const float* const* src, float* const* dst, const int64_t* n, int count, hipStream_t st);
int rt1_multi_reduce_copy(const float* const* src, float* const* dst, const int64_t* n, const int64_t* sstride,
                          const int* splits, int count, hipStream_t st);
int rt1_colsum(const void* in, int in_is_bf16, int64_t R, int C, int B, float* out, float* tmp, int chunks,
               hipStream_t st);

// imgproc.hip (Pillow-exact random-resized-crop of raw HWC uint8 frames -> planar [N, 3, H, W] uint8)
int rt1_crop_resize_u8(const uint8_t* raw, const int* boxes, int N, int h, int w, int H, int W, uint8_t* out,
                       hipStream_t st);
int rt1_crop_resize_gather_u8(const uint8_t* raw, int64_t F, const int64_t* rows, const int* boxes, int N, int h,
                              int w, int H, int W, uint8_t* out, hipStream_t st);

// wgrad.hip (1x1-conv weight gradient on MFMA, split over pixels, optional BN/act/gate prologue on a)
int rt1_wgrad_splits(int64_t M, int Co, int Ci, int variant);   // variant < 0: the built-in tile pick
int rt1_wgrad_run(const rt1_bf16* dy, const rt1_bf16* a, int64_t M, int Co, int Ci, const float* scale,
                  const float* shift, const float* gate, int act, int hw, int splits, float* out, int variant,
                  int sums, hipStream_t st);   // sums: out [splits, Co * Ci + Co] with dy's column sums per split
int rt1_wgrad_dymap(const float* dyf, const int* map, const rt1_bf16* a, int64_t M, int Co, int Ci, int splits,
                    float* out, float* dbout, int tile, hipStream_t st);

// projbwd.hip (project-conv backward statistics + weight gradient of the skinny blocks, per frame)
int rt1_proj_bwd_supported(int Cout, int Ce);
int rt1_proj_bwd_fsplit(int N, int HW, int Ce);
int rt1_proj_bwd_frame(const rt1_bf16* dy, const rt1_bf16* y, int N, int HW, int Cout, int Ce, const float* scale,
                       const float* shift, const float* mean, const float* rstd, const rt1_bf16* Wp, int fsplit,
                       float* G, float* R, hipStream_t st);
int rt1_proj_bwd_finalize(const float* G, const float* R, const float* gate, int N, int Cout, int Ce, int fsplit,
                          float* red, float* dW, hipStream_t st);

// pwbwd.hip
int rt1_pw_bwd_supported(int CE, int CIN);
int rt1_pw_bwd_grid(int M, int max_blocks);
int rt1_pw_bwd(const rt1_bf16* dA, const rt1_bf16* y, const rt1_bf16* x, const rt1_bf16* We, const float* consts,
               int M, int CE, int CIN, rt1_bf16* dx, const rt1_bf16* dout, const float* fmul, int HW, float* dwp,
               int grid, hipStream_t st);
int rt1_pw_bwd_z_width(int CE, int CIN);
int rt1_pw_bwd_z_mk_elems(int CIN);
int rt1_pw_bwd_z(const rt1_bf16* dz, const rt1_bf16* x, const rt1_bf16* We, const float* consts, int M, int CE,
                 int CIN, rt1_bf16* mk, float* r0, rt1_bf16* dx, const rt1_bf16* dout, const float* fmul, int HW,
                 float* part, int grid, hipStream_t st);
int rt1_pw_tall_tail(const rt1_bf16* A, const rt1_bf16* W, int M, int K, int N, const rt1_bf16* A2, const rt1_bf16* W2,
                     int K2, const float* bias, const rt1_bf16* res, const float* rmul, int rhw, rt1_bf16* C,
                     hipStream_t st);
int rt1_pw_z_prep(const rt1_bf16* We, const float* consts, int CE, int CIN, rt1_bf16* wt, rt1_bf16* mk, float* r0,
                  hipStream_t st);
int rt1_pw_z_finish(const float* S, int splits, const float* G, const float* sx, const rt1_bf16* We,
                    const float* consts, int CE, int CIN, float* dWe, hipStream_t st);
int rt1_pw_bwd_z_finish(const float* S, const rt1_bf16* We, const float* consts, int CE, int CIN, float* dWe,
                        hipStream_t st);

}  // extern "C"
