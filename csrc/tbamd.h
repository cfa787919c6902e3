// Host-side launcher ABI shared by the HIP kernel files and the torch bindings.
// Kernel translation units include only <hip/hip_runtime.h> (fast builds);
// bindings.cpp includes torch and calls these with raw pointers + the current
// HIP stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>


namespace tbamd {

enum DTypeCode : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

// ---- fp32 conv weight gradient as split-bf16 passes of the MFMA wgrad kernel (conv_wgrad.hip)
int64_t conv_wgrad_split32_workspace(int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride,
                                     int pad);
void conv_wgrad_split32(const float* dy, const float* x, float* dw, uint16_t* dyh, uint16_t* dyl, uint16_t* xh,
                        uint16_t* xl, float* part, int N, int H, int W, int C, int K, int R, int S, int P, int Q,
                        int stride, int pad, int up, int reflect, hipStream_t st);

// f32 -> (hi, lo) bf16 pairs (n % 4 == 0), and the split-bf16 fp32 conv forward (conv.hip)
void split_bf16(const float* v, int64_t n, uint16_t* hi, uint16_t* lo, hipStream_t st);
void conv_fwd_split32(const void* xh, const void* xl, const void* wh, const void* wl, float* y, const float* bias,
                      bool relu, int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad,
                      hipStream_t st, float* part = nullptr);
// reduction splits conv_fwd_split32 uses for this shape (1: none); part holds splits * N*P*Q*K floats
int conv_fwd_splitk_bf16_ksplit(int N, int C, int K, int R, int S, int P, int Q);
void conv_fwd_splitk_bf16(const void* x, const void* w, void* y, const float* bias, bool relu, int N, int H, int W,
                          int C, int K, int R, int S, int P, int Q, int stride, int pad, float* part, int ns,
                          hipStream_t st);
int conv_fwd_split32_ksplit(int N, int C, int K, int R, int S, int P, int Q);

// ---- standalone activations (csrc/aux_ops.hip; act = kAct* of common.h, n % 8 == 0)
void act_forward(int dt, int act, const void* x, void* y, int64_t n, float slope, hipStream_t st);
void act_backward(int dt, int act, const void* x, const void* dy, void* dx, int64_t n, float slope, hipStream_t st);

// ---- completion-event hand-off (common.h tb_launch_ev, ops/streams.py): arm one event of a
// pool for the next tb_launch_ev launch of this thread; disarm returns whether a launch took it
int64_t stop_event_arm();
bool stop_event_disarm();
void stream_wait_stop_event(hipStream_t st, int64_t id);

// ---- BatchNorm (NHWC, [M, C]) ----
int bn_partial_blocks(int64_t M, int C);
void bn_forward_train(int dt, const void* x, int64_t M, int C, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                      float* psum, float* psq, int nblk, double* fin_ws, float* mean, float* invstd, float* scale,
                      float* shift, hipStream_t st);
// doubles of f64 workspace the BN finalize reductions need for nrows partial rows
int64_t colsum_workspace(int nrows, int C);
bool bn_backward_pool_ok(int H, int W, int C, int k, int s, int pad);
int bn_backward_pool_blocks(int N, int H, int W, int C);
void bn_backward_pool(int dt, const void* dyp, const uint8_t* idx, const void* x, int N, int H, int W, int C, int k,
                      int s, int pad, int act, float slope, const float* gamma, const float* mean,
                      const float* invstd, const float* scale, const float* shift, int training, float* pdb,
                      float* pdg, int nblk, double* fin_ws, float* coef, float* dgamma, float* dbeta, void* dx,
                      hipStream_t st);
void bn_backward_from_partials(int dt, const void* dy, const void* y, const void* x, int64_t M, int C, int act,
                               float slope, const float* gamma, const float* mean, const float* invstd,
                               const float* scale, const float* shift, int training, const float* part, int nrows,
                               double* fin_ws, float* coef, float* dgamma, float* dbeta, void* dx,
                               const uint8_t* maskin, hipStream_t st,
                               void* dres = nullptr,
                               const void* xds = nullptr, const float* mean_ds = nullptr, float* pds = nullptr);
// deferred apply (conv.hip GXF): finalize only -> coef [3][C], dgamma, dbeta; and the apply from coef
void bn_backward_coef(const float* part, int nrows, int64_t M, int C, const float* gamma, const float* mean,
                      const float* invstd, int training, double* fin_ws, float* coef, float* dgamma, float* dbeta,
                      hipStream_t st);
void bn_backward_apply_coef(int dt, const void* dy, const void* x, int64_t M, int C, int act, float slope,
                            const float* scale, const float* shift, const float* coef, void* dx,
                            const uint8_t* maskin, hipStream_t st);
// rows of bn_backward_from_partials's downsample-branch partials (pds [rows][2][C])
int bn_bwd_dsp_rows(int64_t M, int C);
void bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                    float eps, float* mean, float* invstd, float* scale, float* shift, hipStream_t st);
// mask (optional, residual + ReLU, C % 8 == 0): one bit per element (y > 0), [M][C/8] bytes
void bn_apply(int dt, const void* x, const void* res, const float* scale, const float* shift, int64_t M,
              int C, int act, float slope, void* y, uint8_t* mask, hipStream_t st, const float* rsc = nullptr,
              const float* rsh = nullptr);
// maskin (optional, residual + ReLU): take the ReLU mask from bn_apply's bits and do not write dres
void bn_backward(int dt, const void* dy, const void* y, const void* x, const void* res, int64_t M, int C,
                 int act, float slope, const float* gamma, const float* mean, const float* invstd,
                 const float* scale, const float* shift, int training, float* pdb, float* pdg, int nblk,
                 double* fin_ws, float* coef, float* dgamma, float* dbeta, void* dres, void* dx,
                 const uint8_t* maskin, hipStream_t st);

// ---- GroupNorm / InstanceNorm (NHWC, N samples x [HW, C]) ----
int norm_partial_blocks(int64_t M, int C, int S);
void norm_apply(int dt, const void* x, const void* res, const float* scale, const float* shift, int S,
                int64_t M, int C, int act, float slope, void* y, hipStream_t st);
void gn_forward_stats(int dt, const void* x, int N, int64_t HW, int C, int G, const float* gamma,
                      const float* beta, float eps, float* psum, float* psq, float* row0, int nblk, float* mean,
                      float* invstd, float* scale, float* shift, hipStream_t st);
void gn_backward(int dt, const void* dy, const void* y, const void* x, const void* res, int N, int64_t HW, int C,
                 int G, int act, float slope, const float* gamma, const float* mean, const float* invstd,
                 const float* scale, const float* shift, float* pdb, float* pdg, int nblk, float* coef,
                 float* dg_nc, float* db_nc, float* dgamma, float* dbeta, void* dres, void* dx, hipStream_t st);

// ---- LayerNorm (rows [M, C], C % 8 == 0) ----
int ln_bwd_blocks(int64_t M);
void ln_forward(int dt, const void* x, const void* res, const float* gamma, const float* beta, int64_t M, int C,
                float eps, void* y, void* xsum, float* mean, float* rstd, hipStream_t st);
void ln_backward(int dt, const void* dy, const void* x, const void* dadd, const float* gamma, const float* mean,
                 const float* rstd, int64_t M, int C, void* dx, float* pdg, float* pdb, int nblk, float* dgamma,
                 float* dbeta, hipStream_t st);

// ---- optimizers (multi-tensor, chunk table) ----
// hyper (optional, device f32): adamw [lr, bc1, bc2_sqrt] / sgd [lr] read by the kernel instead of
// the scalar arguments, so a captured hipGraph replays with the current schedule
void adamw_mt(int pdt, int gdt, bool master, bool ema, bool amsgrad, const void* chunks, int nchunks,
              const int64_t* table, float lr, float beta1, float beta2, float eps, float wd, float bc1,
              float bc2_sqrt, float ema_decay, const float* clip_coef, const float* inv_scale,
              const float* found_inf, hipStream_t st, const float* hyper = nullptr);
void sgd_mt(int pdt, int gdt, bool master, float momentum, float dampening, bool nesterov, float wd,
            float lr, int first_step, const void* chunks, int nchunks, const int64_t* table,
            const float* clip_coef, const float* inv_scale, const float* found_inf, hipStream_t st,
            const float* hyper = nullptr);
void grad_norm_mt(int gdt, const void* chunks, int nchunks, const int64_t* table, float max_norm,
                  const float* inv_scale, float* partial, float* out3, hipStream_t st);
// several (dtype) tables: Σg² of each into one partial array, one finalize -> [norm, coef, nonfinite]
void grad_norm_multi(int ngroups, const int* gdts, const void* const* chunks, const int* nchunks,
                     const int64_t* const* tables, float max_norm, const float* inv_scale, float* partial,
                     float* out3, hipStream_t st);
void scale_mt(int gdt, const void* chunks, int nchunks, const int64_t* table, const float* s,
              hipStream_t st);

// ---- cross entropy ----
void ce_forward(int dt, const void* logits, const int64_t* labels, int64_t N, int K, float smoothing,
                int64_t ignore_index, float* row_loss, float* row_lse, float* row_ok, float* out3,
                hipStream_t st);
void ce_backward(int dt, const void* logits, const int64_t* labels, const float* row_lse, const float* gout,
                 const float* stats3, int64_t N, int K, float smoothing, int64_t ignore_index,
                 void* dlogits, hipStream_t st);

// ---- implicit-GEMM conv (NHWC, bf16, MFMA) ----
int conv_fwd_supported(int C, int K);
// tuning override of the conv pipeline depth (0 = heuristic; 1..4 LDS stages)
void conv_set_stages(int s);
void conv_set_occupancy(int o);
int conv_fwd_pixel_tiles(int64_t NPQ, int K);
// rows of the BN-backward partials ([rows][2][K]) a dgrad conv_fwd call (bnb_mode != 0) writes
int conv_fwd_bnb_rows(int64_t NPQ, int C, int K, int R, int S, int stride, int pad);
// 1x1 stride-1 input gradient whose operand is a deferred BN backward apply (conv.hip GxfArgs):
// x = the BN output gradient g, gx_x the BN input, gx_coef [3][C]; gx_out (optional) receives dX
bool conv_dgrad_gxf_supported(int gxf, int add, int bnb_mode);
int conv_gxf_bnb_rows(int64_t NPQ, int K);
void conv_dgrad_gxf(const void* x, const void* w, void* y, const void* addend, const uint8_t* amask, int N, int H,
                    int W, int C, int K, hipStream_t st, int bnb_mode, const void* bnb_x, const float* bnb_scale,
                    const float* bnb_shift, const float* bnb_mean, const uint8_t* bnb_bits, float* bnb_part, int gxf,
                    const void* gx_x, const uint8_t* gx_bits, const float* gx_scale, const float* gx_shift,
                    const float* gx_coef, void* gx_out);
// big-tile (8-wave, 1 workgroup per CU) implicit-GEMM conv (csrc/conv_big.hip): the choice for a
// shape (0 = the 128x128 kernels), its encoding / pixel tile, the global mode (TBAMD_CONV_BIG)
int conv_big_choice(int64_t NPQ, int C, int K, int R, int S, int stride, int pad);
int conv_big_encode(int bm, int bn, int mf, int stages);
int conv_big_pixel_tile(int code);
void conv_set_big(int mode);
int conv_get_big();
void conv_big_set_call(int code);
int conv_big_mode_now();
void conv_big_fwd(const void* x, const void* w, void* y, const float* bias, float* stats, const void* addend,
                  const uint8_t* amask, bool relu, int N, int H, int W, int C, int K, int R, int S, int P, int Q,
                  int stride, int pad, hipStream_t st, int bnb_mode, const void* bnb_x, const float* bnb_scale,
                  const float* bnb_shift, const float* bnb_mean, const uint8_t* bnb_bits, float* bnb_part,
                  int code);
// rows of the forward's BatchNorm-statistics partials ([rows][2][K]) for this conv
void conv_set_persistent_1x1(bool on);
int conv_fwd_stats_rows(int64_t NPQ, int C, int K, int R, int S, int stride, int pad);
// ... of the 128x128 / persistent-1x1 kernels (the BN-in-operand forward)
int conv_fwd_stats_rows_tiled(int64_t NPQ, int C, int K, int R, int S, int stride, int pad);
// addend (optional, bf16 like y): y = conv(x) + addend (* addend_mask bits, [NPQ][K/8] bytes, if given);
// excludes bias/relu/stats
// bnb_mode (dgrad use): 0 off; 1/2/3 = also emit the backward partial sums of the BatchNorm whose
// output gradient y is (ReLU mask recomputed from bnb_x / from bnb_bits / no activation) into
// bnb_part [conv_fwd_pixel_tiles][2][K]
// ResNet stem (C = 3, 7x7, stride 2, pad 3) on the implicit-GEMM kernels: x [N][H][W][3] bf16 is
// re-laid as xp [N][Hp][Wp][4] (conv_stem_pad, conv_stem_workspace elements); weights packed
// [K][8][8][4] (window row, tap, channel; zero padded)
int64_t conv_stem_workspace(int N, int H, int W);
void stem_geometry(int H, int W, int* P, int* Q, int* Hp, int* Wp);
void conv_stem_pad(const void* x, void* xp, int N, int H, int W, hipStream_t st);
void conv_stem_fwd(const void* xp, const void* wp, void* y, float* stats, int N, int H, int W, int K,
                   hipStream_t st);
int64_t conv_stem_wgrad_workspace(int N, int Hp, int Wp, int K, int P, int Q);
void conv_stem_wgrad(const void* dy, const void* xp, void* dwp, float* workspace, int N, int Hp, int Wp, int K,
                     int P, int Q, hipStream_t st);
// stride-2 / stride-3 convolution input gradient as stride^2 output-phase classes on the
// implicit-GEMM kernel: dy [N][P][Q][Kf], wt = flip-transposed weights [Cf][R][S][Kf], dx [N][H][W][Cf]
// bnb_*: optional BN-backward partials of the BN whose output is the conv input (as conv_fwd's
// dgrad use), rows of the classes stacked: conv_dgrad_s2_tiles() rows
void conv_dgrad_s2(const void* dy, const void* wt, void* dx, int N, int P, int Q, int Kf, int Cf, int R, int S,
                   int pad, int H, int W, hipStream_t st, int bnb_mode = 0, const void* bnb_x = nullptr,
                   const float* bnb_scale = nullptr, const float* bnb_shift = nullptr,
                   const float* bnb_mean = nullptr, const uint8_t* bnb_bits = nullptr, float* bnb_part = nullptr,
                   int cs = 2);
int conv_dgrad_s2_tiles(int N, int H, int W, int Cf, int st = 2);
bool conv_dgrad_s2_supported(int R, int S, int st);
// forward conv of relu(x * scale + shift) (per input channel) with the transform applied in the
// kernel's operand staging: the BN output is never materialised (stats: conv_fwd_stats_rows rows)
// input channels the BN-in-operand forward keeps coefficients of in LDS (csrc/xf.h)
constexpr int kXfMaxC = 512;
// dW of a conv over relu(x * scale + shift) (csrc/xf.h transform in the X staging); workspace as conv_wgrad
// weight gradient of a 4x4 / 2 / pad-1 conv from a 3-channel input T and a 64-channel output
// gradient G (csrc/conv_tinyin_wgrad.hip); part: wgrad_tinyin_parts(N, P) * 64 * 48 floats
bool wgrad_tinyin_supported(int C, int K, int R, int S, int stride, int pad, int P, int Q, int H, int W);
int wgrad_tinyin_parts(int N, int P);
void wgrad_tinyin(const void* T, const void* G, void* dw, float* part, int N, int P, int H, int W, hipStream_t st);
void conv_wgrad_xf(const void* dy, const void* x, void* dw, float* workspace, const float* scale, const float* shift,
                   int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad,
                   hipStream_t st);
bool conv_fwd_xf_supported(int64_t NPQ, int C, int K, int R, int S, int stride, int pad);
void conv_fwd_xf(const void* x, const void* w, void* y, float* stats, const float* scale, const float* shift, int N,
                 int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad, hipStream_t st);
void conv_fwd(const void* x, const void* w, void* y, const float* bias, float* stats, const void* addend,
              const uint8_t* addend_mask, bool relu, int N, int H, int W, int C, int K, int R, int S, int P, int Q,
              int stride, int pad, hipStream_t st, int bnb_mode = 0, const void* bnb_x = nullptr,
              const float* bnb_scale = nullptr, const float* bnb_shift = nullptr, const float* bnb_mean = nullptr,
              const uint8_t* bnb_bits = nullptr, float* bnb_part = nullptr);
void bn_finalize_from_conv(const float* part, int nblk, int64_t M, int C, const float* gamma, const float* beta,
                           float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                           double* fin_ws, float* mean, float* invstd, float* scale, float* shift, hipStream_t st);
void conv_flip_transpose_weights_mt(const void* chunks, int nchunks, const int64_t* table, hipStream_t st);
void conv_flip_transpose_weight(const void* w, int K, int R, int S, int C, void* wt, hipStream_t st);
int conv_wgrad_supported(int C, int K, int64_t NPQ);
void conv_wgrad_set_occupancy(int o);
// floats of f32 workspace conv_wgrad needs (0: none)
int64_t conv_wgrad_workspace(int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad);
// convs over pad(upsample_nearest(x, up), pad, reflect|zero) on the 64-channel kernels (up = 1, 2, 4)
void conv_fwd_virtual(const void* x, const void* w, void* y, const float* bias, int N, int H, int W, int C, int K,
                      int R, int S, int P, int Q, int stride, int pad, int up, int reflect, hipStream_t st);
void conv_wgrad_virtual(const void* dy, const void* x, void* dw, float* workspace, int N, int H, int W, int C, int K,
                        int R, int S, int P, int Q, int stride, int pad, int up, int reflect, hipStream_t st);
void conv_wgrad(const void* dy, const void* x, void* dw, float* workspace, int N, int H, int W, int C, int K, int R,
                int S, int P, int Q, int stride, int pad, hipStream_t st);

// ---- fused attention (head dim 64, bf16) ----
// Strides are in elements over (batch, head, token); the head-dim stride is 1.
// Forward writes o and lse ([B][H][N] f32, natural log); backward reads q, k, v,
// o, dout, lse and writes dq, dk, dv and delta ([B][H][N] f32 scratch).
struct AttnArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  float* lse;
  int B, H, N;
  float scale;
  int64_t sq[3], sk[3], sv[3], so[3];
  const uint16_t* dout;
  int64_t sdo[3];
  uint16_t* dq;
  uint16_t* dk;
  uint16_t* dv;
  int64_t sdq[3], sdk[3], sdv[3];
  float* delta;
};
int attn_supported(int D);
// whole-head kernel mask (1 forward, 4 dK/dV); mask < 0 only reads it.  Returns the previous mask.
int attn_set_head_mask(int mask);
void attn_fwd(const AttnArgs& a, hipStream_t st);
void attn_bwd(const AttnArgs& a, hipStream_t st);

// ---- Gram matrix (NHWC bf16 features, C % 64 == 0) ----
void gram_sym(const float* dg, void* sym, int B, int C, float scale, hipStream_t st);
void im2col_nhwc(const void* x, void* col, int N, int H, int W, int C, int R, int S, int P, int Q, int stride,
                 int pad, int up, int reflect, int KP, hipStream_t st);
void col2im_nhwc(const void* col, void* dx, const void* bias, int N, int H, int W, int C, int R, int S, int P, int Q,
                 int stride, int pad, int KP, hipStream_t st);
int gram_tile(int C);
int64_t gram_workspace(int B, int C, int64_t HW);  // floats
// out[b] = F_b^T F_b * scale, F_b = [HW][C]; out is [B][C][C] f32
void gram(const void* f, int B, int64_t HW, int C, float scale, float* workspace, float* out, hipStream_t st);

// ---- column sums (Linear bias gradients), fused GELU backward ----
void gelu_forward(int dt, const void* z, void* y, int64_t n, hipStream_t st);  // y = GELU(z), n % 8 == 0
int colsum_splits(int64_t M, int C);
// out[c] = sum_r dy[r][c] (dtype dt); with z: dz = dy * GELU'(z) is written and summed instead.
// part: colsum_splits(M, C) * C floats.  C % 8 == 0, 16-B aligned rows.
void colsum(int dt, const void* dy, const void* z, void* dz, int64_t M, int C, float* part, void* out,
            hipStream_t st);

// ---- input pipeline ----
// ---- generic convolution (conv_any.hip): any channel counts / taps, fp32 or bf16, reflect
// padding and nearest upsampling (up) or input dilation (dil) folded into the addressing
struct ConvAnyShape {
  int N, H, W, C, K, R, S, P, Q, stride, pad, up, dil, reflect;
};
// narrow-output conv (K <= 16, C in {32, 64}, stride 1, halo tile in LDS; csrc/conv_narrow.hip)
int conv_narrow_supported(int C, int K, int R, int S, int stride, int up);
void conv_narrow_fwd(const void* x, const void* w16, const float* bias, void* y, int N, int H, int W, int C, int K,
                     int R, int S, int pad, int up, int reflect, hipStream_t st);
void conv_narrow_fwd_phase(const void* x, const void* w16, const float* bias, void* y, int N, int H, int W, int C,
                           int K, int R, int S, int pad_h, int pad_w, int P, int Q, int st, int a, int b, int YH,
                           int YW, hipStream_t st_);
int conv_tinyc_supported(int C, int K, int R, int S);
void conv_narrow_fwd32(const float* x, const void* w16h, const void* w16l, const float* bias, float* y, int N, int H,
                       int W, int C, int K, int R, int S, int pad, int up, int reflect, hipStream_t st);
int conv_tinyhalo_wgrad_blocks(int N, int H, int W, int R, int S, int pad);
int conv_tinyhalo_wgrad_cols(int R, int S);
void conv_tinyhalo_wgrad(bool f32, const void* x, const void* dy, float* part, void* dw, int N, int H, int W, int C,
                         int K, int R, int S, int pad, int reflect, hipStream_t st);
int conv_tinyhalo_supported(int C, int K, int R, int S, int stride, int up);
void conv_tinyhalo_fwd(bool f32, const void* x, const void* wph, const void* wpl, const float* bias, void* y, int N,
                       int H, int W, int C, int K, int R, int S, int pad, int reflect, bool relu, hipStream_t st);
void conv_tiny32_fwd(const float* x, const void* wph, const void* wpl, const int* tab, const float* bias, float* y,
                     int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int reflect, bool relu,
                     hipStream_t st);
void conv_tinyc_fwd(const void* x, const void* wp, const int* tab, const float* bias, void* y, int N, int H, int W,
                    int C, int K, int R, int S, int stride, int pad, int reflect, bool relu, hipStream_t st);
int conv_narrow_wgrad_splits(int N, int H, int W, int C, int R, int S, int pad, int up);
void conv_narrow_wgrad(const void* x, const void* dy, float* part, int splits, int N, int H, int W, int C, int K,
                       int R, int S, int pad, int up, int reflect, hipStream_t st);
void conv_any_fwd(int f32, const void* x, const void* w, const void* bias, void* y, const ConvAnyShape& s,
                  hipStream_t st);
int conv_any_wgrad_splits(const ConvAnyShape& s);
void conv_any_set_f32_split(bool on);
bool conv_any_f32_split();
void conv_any_wgrad(int f32, const void* x, const void* dy, float* part, int splits, void* dw,
                    const ConvAnyShape& s, hipStream_t st);
void conv_any_fold(int f32, const void* dxp, int Hg, int Wg, void* dx, const ConvAnyShape& s, hipStream_t st);
void bounds_probe(const float* x, int64_t n, int64_t i, float* out, hipStream_t st);
int augment_max_bytes();
void crop_flip_u8(int odt, const uint8_t* in, const int32_t* src, int B, int Hi, int Wi, int C, int Ho, int Wo,
                  const float* params, const float* mean, const float* inv_std, void* out, hipStream_t st);
void augment_u8(int odt, const uint8_t* in, const int32_t* src, int B, int Hi, int Wi, int C, int Ho, int Wo,
                const float* params, const float* mean, const float* inv_std, void* out, hipStream_t st);
void u8_crop_flip_normalize(int odt, const uint8_t* in, int N, int Hi, int Wi, int C, int Ho, int Wo,
                            const int32_t* offs, const uint8_t* flip, const float* mean, const float* inv_std,
                            void* out, hipStream_t st);

// ---- fused BN-apply + activation + max-pool (NHWC, C % 8 == 0) ----
void bn_act_maxpool_fwd(int dt, const void* x, const float* scale, const float* shift, int act, float slope, int N,
                        int H, int W, int C, int k, int s, int pad, void* y, uint8_t* idx, hipStream_t st);
void global_avgpool_fwd(int dt, const void* x, int N, int HW, int C, void* y, hipStream_t st);
void global_avgpool_bwd(int dt, const void* dy, int N, int HW, int C, void* dx, hipStream_t st);
void maxpool_bwd(int dt, const void* dy, const uint8_t* idx, int N, int H, int W, int C, int k, int s, int pad,
                 void* dx, hipStream_t st);

// ---- small fused losses / resampling (aux_ops.hip; K16, K17, K19-K22) ----
// scalar losses: `part` holds aux_partials() floats, out[0] = the reduced loss
int aux_partials();
void tv_forward(int dt, const void* x, int64_t total, int H, int W, int inner, float* part, float* out,
                hipStream_t st);
void tv_backward(int dt, const void* x, const float* gout, int64_t total, int H, int W, int inner, void* dx,
                 hipStream_t st);
void hinge_forward(int dt, const void* x, int64_t n, float margin, float sign, float* part, float* out,
                   hipStream_t st);
void hinge_backward(int dt, const void* x, const float* gout, int64_t n, float margin, float sign, void* dx,
                    hipStream_t st);
void bce_logits_forward(int dt, const void* x, const void* y, int64_t n, float* part, float* out, hipStream_t st);
void bce_logits_backward(int dt, const void* x, const void* y, const float* gout, int64_t n, void* dx,
                         hipStream_t st);
void kld_forward(int dt, const void* mu, const void* lv, int64_t n, int64_t rows, float* part, float* out,
                 hipStream_t st);
void kld_backward(int dt, const void* mu, const void* lv, const float* gout, int64_t n, int64_t rows, void* dmu,
                  void* dlv, hipStream_t st);
int64_t mean_std_workspace(int N, int C, int64_t S, bool channels_last);  // floats (0: none needed)
void mean_std_forward(int dt, const void* x, int N, int C, int64_t S, bool channels_last, float eps, float* mean,
                      float* std, hipStream_t st, float* ws = nullptr);
void mean_std_backward(int dt, const void* x, const float* mean, const float* std, const float* dmean,
                       const float* dstd, int N, int C, int64_t S, bool channels_last, void* dx, hipStream_t st,
                       float* coef = nullptr);  // coef: 2*N*C floats (NHWC fast path)
// NHWC tensors: x [N][H][W][C]
void reflect_pad_forward(int dt, const void* x, int N, int H, int W, int C, int pt, int pb, int pl, int pr,
                         void* y, hipStream_t st);
void reflect_pad_backward(int dt, const void* dy, int N, int H, int W, int C, int pt, int pb, int pl, int pr,
                          void* dx, hipStream_t st);
void upsample_nearest_forward(int dt, const void* x, int N, int H, int W, int C, int f, void* y, hipStream_t st);
void upsample_nearest_backward(int dt, const void* dy, int N, int H, int W, int C, int f, void* dx,
                               hipStream_t st);


// ---- dense GEMM engine (gemm.hip): Y[p][q] = epi(sum_k X[p][k] W(q,k)),
// W(q,k) = W[q][k] (tw = false) or W[k][q] (tw = true); epi 0 none, 1 +bias,
// 2 +bias then GELU (pre-activation -> Z), 3 +bias +res, 4 +res.  tile < 0: heuristic.
int gemm_num_tiles();
int gemm_pick_tile(int P, int Q, int K);
// 256x256 8-phase NT kernel (csrc/gemm8.hip): Y[p][q] = epi(sum_k X[p][k] W[q][k])
bool gemm8_supported(int P, int Q, int K, int64_t ldx);
// TN variant (csrc/gemm8.hip): Y[p][q] = sum_k X[k][p] W[k][q], split-K f32 partials in part
bool gemm8_tn_supported(int P, int Q, int K, int64_t ldx);
int gemm8_tn_splits(int KT, int splits);
// NN variant: Y[p][q] = sum_k X[p][k] W[k][q]; z != nullptr: Y = that * GELU'(z) and the column
// sums of Y per 256-row tile into bias_part ([ceil(P / 256)][Q] f32, summed by colsum_finalize)
bool gemm8_nn_supported(int P, int Q, int K, int64_t ldx);
void gemm8_nt_gelu_bwd_bf16(const void* X, int64_t ldx, const void* Wt, void* Y, int64_t ldy, const void* z,
                            float* bias_part, int P, int Q, int K, hipStream_t st);
void gemm8_nn_bf16(const void* X, int64_t ldx, const void* W, void* Y, int64_t ldy, const void* z, float* bias_part,
                   int P, int Q, int K, hipStream_t st);
// out[c] = sum over nsplit rows of part[s][c] (fixed order), stored as dt
void colsum_finalize(int dt, const float* part, int nsplit, int C, void* out, hipStream_t st);
void gemm8_tn_bf16(const void* X, int64_t ldx, const void* W, void* Y, int64_t ldy, int P, int Q, int K, int splits,
                   float* part, hipStream_t st);
void gemm8_set_stagger(int s);
void gemm8_bf16(const void* X, int64_t ldx, const void* W, void* Y, int64_t ldy, const void* bias, const void* res,
                void* Z, int P, int Q, int K, int epi, hipStream_t st);
void gemm_bf16(const void* X, int64_t ldx, bool tx, const void* W, bool tw, void* Y, int64_t ldy, const void* bias,
               const void* res, void* Z, int P, int Q, int K, int epi, int tile, int splits, float* part,
               hipStream_t st);
int gemm_pick_splits(int P, int Q, int K, int tile);

// ---- one-shot all-reduce over IPC-mapped peer buffers (csrc/oneshot.hip)
class OneShotComm {
 public:
  OneShotComm(int rank, int world, int64_t capacity_bytes, int64_t chunk_bytes, double timeout_s = 600.0);
  ~OneShotComm();
  OneShotComm(const OneShotComm&) = delete;
  OneShotComm& operator=(const OneShotComm&) = delete;
  std::string handles() const;                    // this rank's IPC handles (exchange them)
  void open(const std::vector<std::string>& all);  // every rank's handles, rank order
  // out = scale * sum over ranks of in (n elements of dtype dt, n % 8 == 0, n * size <= capacity)
  void allreduce(const void* in, void* out, int64_t n, int dt, float scale, hipStream_t st);
  bool error() const;  // a call timed out waiting for a peer (pinned host word: no sync)
  int64_t capacity() const { return cap_; }

 private:
  int rank_, world_, device_ = 0, nchunks_max_ = 0;
  int64_t cap_, chunk_bytes_;
  void* stage_ = nullptr;
  uint32_t* flags_ = nullptr;
  uint32_t* err_ = nullptr;       // device view of err_host_
  uint32_t* err_host_ = nullptr;  // hipHostMalloc'd, mapped
  uint64_t timeout_ticks_;
  void* peer_stage_[8];
  uint32_t* peer_flags_[8];
  uint32_t epoch_ = 0;
  bool opened_ = false;
};
}  // namespace tbamd
