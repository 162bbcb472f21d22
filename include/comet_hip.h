/*
 * comet_hip.h — C-ABI of libcomet_hip.so, the MI355X (gfx950) kernel library behind the
 * COMET Trajectory-Guided Temporal Modeling path.
 *
 * Conventions (SURVEY.md §8b "C-ABI the HIP library must export"):
 *   - every pointer is a device pointer owned by the caller (PyTorch caching allocator);
 *     the library allocates nothing and keeps no device state between calls;
 *   - every call only enqueues work on `stream` (a hipStream_t passed as void*), never syncs,
 *     and is safe to capture into a hipGraph;
 *   - return 0 on success, a negative COMET_E* code otherwise; comet_last_error() returns a
 *     thread-local message describing the last failure on the calling thread;
 *   - dtype codes: COMET_F32 = 0, COMET_BF16 = 1. Accumulation is always f32.
 *
 * Each entry point names the reference operator(s) it replaces (file:line under
 * wulibingbinglin/COMET-Pose-Estimation).
 */
#ifndef COMET_HIP_H_
#define COMET_HIP_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COMET_F32 0
#define COMET_BF16 1

#define COMET_OK 0
#define COMET_EINVAL -1     /* bad argument / unsupported shape */
#define COMET_ELAUNCH -2    /* kernel launch failed */

#define COMET_ACT_NONE 0
#define COMET_ACT_GELU 1    /* exact erf GELU, nn.GELU() (modules.py:127) */
#define COMET_ACT_RELU 2
#define COMET_ACT_SIGMOID 3

int comet_version(void);
const char* comet_last_error(void);

/* ---------------------------------------------------------------------------------------
 * GEMM with fused epilogue. Replaces every nn.Linear / packed MHA in_proj / out_proj
 * (modules.py:119-154, 248-344; torch.nn.MultiheadAttention), convolution GEMMs after
 * im2col (blocks.py:27-196, DINOv2 patch-embed) and the head's backward GEMMs.
 *
 *   v = alpha * sum_k A[m,k] * B[k,n]            (f32 accumulate, bf16 or f32 MFMA)
 *   v += bias  (per column n, or per row m)
 *   if aux: aux[m,n] = v                         (pre-activation, for backward)
 *   v = act(v)
 *   if resid: v += beta * resid[m,n]             (resid may alias c)
 *   c[m,n] = v
 *
 * layout_a 0: A[m*lda + k]; 1: A[k*lda + m].  layout_b 0: B[n*ldb + k] (Linear weight
 * [out,in]); 1: B[k*ldb + n]. Two batch dimensions: element base = b0*stride[0] + b1*stride[1].
 * Bias is always f32; c / resid / aux use dtype_c.
 *
 * Split-K: split_k 0 = library heuristic (splits K when the output tiles cannot fill the 256 CUs,
 * e.g. weight gradients reduced over every token), 1 = never, s > 1 = force s splits. A split
 * GEMM needs an f32 workspace of comet_gemm_workspace() bytes; with workspace == NULL (or too
 * small) the GEMM runs unsplit. Partials are summed in a fixed order: results are deterministic.
 * ------------------------------------------------------------------------------------- */
typedef struct comet_gemm_args {
  int32_t dtype_ab;
  int32_t dtype_c;
  int32_t layout_a;
  int32_t layout_b;
  int64_t m, n, k;
  int64_t batch[2];
  const void* a; int64_t lda; int64_t stride_a[2];
  const void* b; int64_t ldb; int64_t stride_b[2];
  void* c; int64_t ldc; int64_t stride_c[2];
  const float* bias; int32_t bias_mode; int64_t stride_bias[2];
  const void* resid; int64_t ldr; int64_t stride_r[2];
  void* aux; int64_t ldaux; int64_t stride_aux[2];
  float alpha; float beta;
  int32_t act;
  void* workspace; int64_t workspace_bytes;
  int32_t split_k;
  int32_t convert_a, convert_b;  /* 1: that operand is f32 in memory, rounded to bf16 on load
                                    (dtype_ab must be COMET_BF16; convert_b: layout_b 1 only) */
} comet_gemm_args;

int comet_gemm(const comet_gemm_args* args, void* stream);
/* Workspace bytes comet_gemm needs for these arguments (0 when it will not split K). */
int comet_gemm_workspace(const comet_gemm_args* args, int64_t* bytes);
/* Same, plus the kernel plan comet_gemm will launch: plan[0] = 0 skinny (N <= 64),
 * 1 256-row tile, 2 128 x 128 tile; plan[1] = the 256-row tile's BN; plan[2] = K splits.
 * Lets a profiler name the kernel instance a call lands on (bench.py roofline). */
int comet_gemm_plan(const comet_gemm_args* args, int64_t* bytes, int32_t* plan);

/* GEMM + row LayerNorm epilogue (AttnBlock / CrossAttnBlock of the tracker's update former,
 * blocks.py:205-348 over modules.py:248-344, all under no_grad): the f32 residual GEMM whose
 * output row v = x @ w^T + bias + beta*resid feeds LayerNorms (norm2 of the same block; norm1 /
 * norm_context of the next blocks) writes those LayerNorms itself:
 *   c   = v when raw_c != 0, else (v - mean(v)) / sqrt(var(v) + eps_y)        [f32]
 *   y16 = (v - mean(v)) / sqrt(var(v) + eps_y)                                  [bf16, optional]
 *   z16 = (v - mean(v)) / sqrt(var(v) + eps_z) * zw + zb                        [bf16, optional]
 * (biased variance, as nn.LayerNorm). Eligible (comet_gemm_rowln_ok): bf16 k-contiguous A / B,
 * K % 64 == 0, M >= 4096, N in {256, 384}, dtype_c f32 with resid, act NONE, no aux, no split. */
typedef struct comet_rowln_args {
  void* y16; int64_t ldy; float eps_y;
  void* z16; int64_t ldz; const float* zw; const float* zb; float eps_z;
  int32_t raw_c;
} comet_rowln_args;
int comet_gemm_rowln_ok(const comet_gemm_args* args);
/* Few rows (M <= 32 x CUs) and a long K: the row-LN GEMM runs as split-K partials + one LN reduce when
 * args->workspace holds comet_gemm_rowln_workspace() bytes (0: no split; without the workspace the
 * single-kernel path runs, same outputs within f32 summation order). */
int comet_gemm_rowln_workspace(const comet_gemm_args* args, int64_t* bytes);
int comet_gemm_rowln(const comet_gemm_args* args, const comet_rowln_args* ln, void* stream);

/* GEMM + activation backward (Mlp.fc2's input gradient fused with fc1's GELU backward and bias
 * gradient, modules.py:18-40 / timm Mlp under loss.backward(), train_eval_func_new_cp5.py:793):
 *   c[m, n]   = bf16( act'(pre[m, n]) * alpha * sum_k A[m, k] B[k, n] )     (act = GELU, erf form)
 *   dbias[n]  = sum_m c[m, n]   (the rounded values; zeroed first; may be NULL)
 * pre: bf16 [M, N] at row pitch ldpre (fc1's saved pre-activation). Replaces the dX GEMM + the
 * comet_act_bwd_colsum pass (the hidden gradient is written once instead of written, read and
 * written again). Eligible (comet_gemm_dact_ok): act GELU, bf16 A / B / C, A k-contiguous, no bias,
 * residual, aux or forward activation, one batch, N % 8 == 0, 16-B aligned C and pre, a 256-row
 * tile plan (comet_gemm_plan kind 1) without split-K. */
int comet_gemm_dact_ok(const comet_gemm_args* args, int32_t act, const void* pre, int64_t ldpre);
int comet_gemm_dact(const comet_gemm_args* args, int32_t act, const void* pre, int64_t ldpre, float* dbias,
                    void* stream);


/* ---------------------------------------------------------------------------------------
 * Implicit-GEMM convolution on channels-last activations (nn.Conv2d of BasicEncoder /
 * ShallowEncoder / ResidualBlock, blocks.py:27-202, modules.py:39-116): the im2col matrix is
 * never materialised; the GEMM's A tiles are gathered from x directly.
 *   y[(n*oh + oy)*ow + ox][co] = act(bias[co] + sum_{ky,kx,ci} x[n][oy*s-p+ky][ox*s-p+kx][ci]
 *                                    * weight[co][(ky*kw + kx)*c + ci]) + beta*resid[...]
 * x [n,h,w,c] bf16 contiguous with c % 8 == 0; weight [cout][ldw] bf16 (K = kh*kw*c <= ldw);
 * y / resid use dtype_y with row pitch ldy / ldr. (f32 or c % 8 != 0: im2col + comet_gemm.)
 * ------------------------------------------------------------------------------------- */
typedef struct comet_conv_args {
  int32_t dtype;      /* x and weight: COMET_BF16 */
  int32_t dtype_y;
  const void* x; int64_t n, h, w, c;
  const void* weight; int64_t cout, ldw;
  int32_t kh, kw, stride, pad;
  const float* bias;
  void* y; int64_t ldy;
  const void* resid; int64_t ldr; float beta;
  int32_t act;
} comet_conv_args;

int comet_conv2d_nhwc(const comet_conv_args* args, void* stream);

/* ---------------------------------------------------------------------------------------
 * Row LayerNorm over the last dim (nn.LayerNorm; also GroupNorm(1, C) on [rows, C] as used
 * by base_track_predictor.py:81,238). weight/bias f32 or NULL (elementwise_affine=False,
 * modules.py:261-317). mean/rstd (f32, [rows]) are written when non-NULL (for backward).
 * Output dtype may differ from input dtype (f32 residual stream -> bf16 GEMM operand).
 * ldx / ldy are row strides (elements); relu != 0 applies ReLU after the affine
 * (TrajectoryEncoder LN -> ReLU, camera_predictor10.py:79-81).
 * ------------------------------------------------------------------------------------- */
int comet_layernorm_fwd(int dtype_x, int dtype_y, const void* x, const float* weight,
                        const float* bias, void* y, void* y2, float* mean, float* rstd,
                        int64_t rows, int64_t cols, int64_t ldx, int64_t ldy, int64_t ldy2,
                        float eps, int relu, void* stream);
/* y2 (bf16, may be NULL; y may be NULL when y2 is given): a second copy of the output for the GEMM
 * that consumes it (AttnBlock: the normed x is both the in_proj input and the residual).
 * dx (dtype_dx) = LN backward of dy + dy2 (dy2 bf16, may be NULL); dweight/dbias (f32) are
 * ACCUMULATED (+=) when non-NULL. dx_accumulate != 0 adds into dx instead of overwriting. */
int comet_layernorm_bwd(int dtype_x, int dtype_dy, const void* x, const void* dy, const void* dy2,
                        const float* mean, const float* rstd, const float* weight,
                        int dtype_dx, void* dx, float* dweight, float* dbias, int64_t rows, int64_t cols,
                        int dx_accumulate, void* stream);
/* x + f(LN(x)) (modules.py:293-294, 342-343): dx (f32) = dres + LN backward of dy, one pass
 * (x f32, dy f32 / bf16, cols % 8 == 0, 32-B aligned rows). */
int comet_layernorm_bwd_res(int dtype_x, int dtype_dy, const void* x, const void* dy, const float* dres,
                            const float* mean, const float* rstd, const float* weight, float* dx,
                            float* dweight, float* dbias, int64_t rows, int64_t cols, void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused multi-head attention forward (flash style: LDS-staged K/V, online softmax, MFMA for
 * Q·Kᵀ and P·V). Replaces the explicit bmm-softmax-bmm path of nn.MultiheadAttention
 *  at every use site (head self/cross/T_P/trunk, tracker time/space,
 * DINOv2). Tensors are addressed [batch, head, token, d] with arbitrary element strides.
 * lse (f32, [batch, head, lq], may be NULL) receives log-sum-exp of the scaled scores.
 * ------------------------------------------------------------------------------------- */
typedef struct comet_attn_args {
  int32_t dtype;      /* q/k/v/o dtype */
  int32_t head_dim;   /* 32, 48, 64, 96 */
  int64_t batch, heads, lq, lk;
  const void* q; int64_t sq_b, sq_h, sq_l;
  const void* k; int64_t sk_b, sk_h, sk_l;
  const void* v; int64_t sv_b, sv_h, sv_l;
  void* o; int64_t so_b, so_h, so_l;
  float* lse;         /* contiguous [batch, heads, lq] */
  float scale;
  /* optional inner batch (0 / 1 = none): batch index b addresses (b / batch_inner) * s*_b +
   * (b % batch_inner) * s*_i -- attention over the tracks of a [B, N, T, C] tensor for every
   * (b, t) (EfficientUpdateFormer space blocks, blocks.py:322-340) without permuting it */
  int64_t batch_inner;
  int64_t sq_i, sk_i, sv_i, so_i;
} comet_attn_args;

int comet_attention_fwd(const comet_attn_args* args, void* stream);

/* Fused attention backward (bf16, flash style, nothing Lq x Lk in HBM): given q/k/v, the
 * forward output o, its lse and the incoming gradient dout, writes dq, dk, dv (bf16, any
 * 16-B-aligned strides). delta: f32 workspace [batch, heads, lq] (receives rowsum(dout*o)).
 * Replaces autograd through nn.MultiheadAttention's bmm-softmax-bmm. */
typedef struct comet_attn_bwd_args {
  int32_t dtype;      /* COMET_BF16 */
  int32_t head_dim;   /* 32, 48, 64, 96 */
  int64_t batch, heads, lq, lk;
  const void* q; int64_t sq_b, sq_h, sq_l;
  const void* k; int64_t sk_b, sk_h, sk_l;
  const void* v; int64_t sv_b, sv_h, sv_l;
  const void* o; int64_t so_b, so_h, so_l;
  const void* dout; int64_t sd_b, sd_h, sd_l;
  void* dq; int64_t sdq_b, sdq_h, sdq_l;
  void* dk; int64_t sdk_b, sdk_h, sdk_l;
  void* dv; int64_t sdv_b, sdv_h, sdv_l;
  const float* lse;   /* [batch, heads, lq], natural log, from comet_attention_fwd */
  float* delta;       /* workspace [batch, heads, lq] */
  float scale;
} comet_attn_bwd_args;

int comet_attention_bwd(const comet_attn_bwd_args* args, void* stream);

/* Attention backward helpers (materialised form, head_dim-agnostic):
 * probs[r, j] = exp(s[r, j]*scale - lse[r]); s is f32, probs has dtype_s (the compute dtype);
 * rows = batch*heads*lq, ld = row stride. */
int comet_attn_probs(int dtype_s, const void* s, const float* lse, void* p, int64_t rows,
                     int64_t cols, int64_t ld_s, int64_t ld_p, float scale, void* stream);
/* dS[r, j] = P[r, j] * (dP[r, j] - delta[r]) * scale, delta[r] = sum_d dO[r,d]*O[r,d]
 * (computed by comet_attn_delta). P and dS have dtype_p, dP is f32. */
int comet_attn_delta(int dtype, const void* dout, const void* out, float* delta, int64_t batch,
                     int64_t heads, int64_t lq, int64_t d, int64_t so_b, int64_t so_h,
                     int64_t so_l, int64_t sdo_b, int64_t sdo_h, int64_t sdo_l, void* stream);
int comet_attn_dsoftmax(int dtype_p, const void* p, const void* dp, const float* delta, void* ds,
                        int64_t rows, int64_t cols, int64_t ld, float scale, void* stream);

/* ---------------------------------------------------------------------------------------
 * Elementwise / reductions.
 * ------------------------------------------------------------------------------------- */
int comet_cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, void* stream);
/* dst[i][0:sizes[i]] = bf16(src[i][...]) for n_tensors f32 tensors in few launches (the bf16
 * copies of the trainable camera-head weights, refreshed after each AdamW step). */
int comet_cast_multi_f32_bf16(const float* const* src, void* const* dst, const int64_t* sizes,
                              int n_tensors, void* stream);
/* y = act(x) (f32 or bf16); gelu backward: dx = dy * gelu'(pre) */
int comet_act_bwd(int act, int dtype_pre, int dtype_dy, const void* pre, const void* dy,
                  void* dx, int dtype_dx, int64_t n, void* stream);
/* y = a*x + b*y (f32) */
int comet_axpby(const float* x, float* y, float a, float b, int64_t n, void* stream);
/* column sum: out[c] (+)= sum_r x[r*ld + c]  (bias gradients). */
int comet_colsum(int dtype, const void* x, float* out, int64_t rows, int64_t cols, int64_t ld,
                 int accumulate, void* stream);
/* Linear backward prologue in one pass (cols % 8 == 0, contiguous [rows, cols], 32-B aligned):
 * g = dy * act'(pre) (act NONE: g = dy, pre unused); if out: out = g (dtype_out);
 * if dbias: dbias[c] (+)= sum_r g[r, c] (of the rounded g when out is bf16). */
int comet_act_bwd_colsum(int act, int dtype_pre, const void* pre, int dtype_dy, const void* dy,
                         int dtype_out, void* out, float* dbias, int64_t rows, int64_t cols,
                         int accumulate, void* stream);
/* squared L2 norm of many tensors: out[0] += sum x_i^2  (clip_grad_norm_, train_eval_func_new_cp5.py:797),
 * in a fixed summation order (bit-identical across launches: the clip coefficient of every
 * data-parallel replica); partials: device scratch of COMET_SQ_NORM_PARTIALS floats, stream-ordered. */
#define COMET_SQ_NORM_PARTIALS 1024
int comet_sq_norm_multi(const float* const* ptrs, const int64_t* sizes, int n_tensors,
                        float* out, float* partials, void* stream);
/* fused AdamW over many f32 tensors (torch.optim.AdamW defaults, train_util.py:311-332);
 * grad scaled by clip = min(1, max_norm / (sqrt(*sqnorm) + 1e-6)) when sqnorm != NULL. */
int comet_adamw_multi(float* const* params, const float* const* grads, float* const* exp_avg,
                      float* const* exp_avg_sq, const int64_t* sizes, int n_tensors, float lr,
                      float beta1, float beta2, float eps, float weight_decay, int step,
                      const float* sqnorm, float max_norm, void* stream);

/* ---------------------------------------------------------------------------------------
 * Convolution / CNN operators (channels-last NHWC activations).
 * ------------------------------------------------------------------------------------- */
/* im2col for conv2d NHWC input [n, h, w, c] -> cols [n*oh*ow, ldc], column (ky*kw+kx)*c+ci,
 * columns [kh*kw*c, ldc) zero-filled (K padded to the GEMM vector width). */
int comet_im2col_nhwc(int dtype_in, int dtype_out, const void* x, void* cols, int64_t n,
                      int64_t h, int64_t w, int64_t c, int kh, int kw, int stride, int pad,
                      int64_t oh, int64_t ow, int64_t ldc, void* stream);
/* InstanceNorm2d (affine=False, eps 1e-5) on NHWC, optional residual add and ReLU:
 * o = IN(x); if res_norm_relu: o = relu(o); if res: o += res; if relu: o = relu(o).
 * (ResidualBlock tail relu(x + relu(IN(conv2(.)))), modules.py:108-116).
 * Large images are split over several workgroups per image; that path needs an f32 workspace
 * of comet_instnorm_workspace() bytes (with a NULL / short workspace one workgroup per image). */
int comet_instnorm_workspace(int64_t n, int64_t hw, int64_t c, int64_t* bytes);
int comet_instnorm_nhwc(int dtype, const void* x, const void* res, void* y, int64_t n,
                        int64_t hw, int64_t c, float eps, int relu, int res_norm_relu,
                        void* workspace, int64_t workspace_bytes, void* stream);
/* bilinear resize, align_corners=True, NCHW or NHWC (F.interpolate, blocks.py:179-202,
 * track_predictor.py:137, camera_predictor10.py:624). add != 0 accumulates into y. */
int comet_resize_bilinear(int dtype_in, int dtype_out, int nhwc, const void* x, void* y,
                          int64_t n, int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow,
                          int add, void* stream);
/* NHWC resize (align_corners=True) and the 2 x 2 / stride-2 average pool of its output in one pass
 * (refine_track.py fine features + blocks.py:371 F.avg_pool2d): y [n, oh, ow, c], pool
 * [n, oh / 2, ow / 2, c], both equal to comet_resize_bilinear followed by comet_avgpool2_nhwc.
 * c in {8, 16, 32, 64, 128, 256}, 16-B aligned, input image h * w * c elements of at most 32 KiB. */
int comet_resize_bilinear_pool_nhwc(int dtype_in, int dtype_out, const void* x, void* y, void* pool,
                                    int64_t n, int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow,
                                    void* stream);
/* The fine ShallowEncoder's tail (blocks.py:97-110 + the fine pyramid's pool, refine_track.py):
 * x2 = (x + up(up1)) + up(up2) (each sum rounded to bf16, as two resize-and-add calls; up1 / up2
 * optional, [n, h1, w1, c] / [n, h2, w2, c], align_corners=True), t = x2 + conv1x1(x2; weight
 * [c, c] bf16, bias f32) rounded as comet_gemm's narrow kernel does, y = resize(t) [n, oh, ow, c] and
 * pool = avgpool2(y), and optionally pool2 = avgpool2(pool) [n, oh / 4, ow / 4, c] (the pyramid's
 * next level), without writing x2 or t. bf16 tensors; c in {32, 64}, h * w % 16 == 0,
 * 2 * h * w * c * 2 (+ (oh / 2) * (ow / 2) * c * 2 with pool2) <= 64 KiB, 16-B aligned. */
int comet_conv1x1_resize_pool_nhwc(const void* x, const void* up1, int64_t h1, int64_t w1, const void* up2,
                                   int64_t h2, int64_t w2, const void* weight, const float* bias, void* y,
                                   void* pool, void* pool2, int64_t n, int64_t c, int64_t h, int64_t w,
                                   int64_t oh, int64_t ow, void* stream);
/* NHWC resize into a channel slice of a wider NHWC tensor (output pixel pitch ldy elements):
 * BasicEncoder's four up-sampled maps land directly in their torch.cat(dim=1) positions
 * (blocks.py:97-107), so the 416-channel concat is never copied. c, ldy % 8 == 0. */
int comet_resize_bilinear_nhwc_into(int dtype_in, int dtype_out, const void* x, void* y, int64_t n,
                                    int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow,
                                    int64_t ldy, int add, void* stream);

/* ---------------------------------------------------------------------------------------
 * Camera head (camera_predictor10.py:329-484) and encoders.
 * ------------------------------------------------------------------------------------- */
/* y = act(x) elementwise (ReLU / GELU / sigmoid of the T_P gating MLPs) */
int comet_act_fwd(int act, int dtype_x, int dtype_y, const void* x, void* y, int64_t n, void* stream);
/* op 0: y = a + b; 1: y = relu(a + b); 2: y = a * b (same dtype, same shape) */
int comet_binary(int op, int dtype, const void* a, const void* b, void* y, int64_t n, void* stream);
/* y[r, c] = x[r, c] + table[r % period, c] (positional / time embeddings, table f32) */
int comet_add_rows(int dtype_x, int dtype_y, const void* x, const float* table, void* y, int64_t rows,
                   int64_t cols, int64_t period, int64_t ldx, int64_t ldy, void* stream);
/* T_P confidence gating traj * w (camera_predictor10.py:332-333): y[r, :] = x[r, :] * w[r];
 * backward dx = dy * w, dw[r] = <dy[r], x[r]> (dx / dw may be NULL) */
int comet_rowscale_fwd(int dtype, const void* x, const float* w, void* y, int64_t rows, int64_t cols,
                       void* stream);
int comet_rowscale_bwd(int dtype, const void* x, const float* w, const float* dy, float* dx, float* dw,
                       int64_t rows, int64_t cols, void* stream);
/* 1-D sin/cos table (utils.py:807-832, double math, f32 out): out[m*ld + col0 + d] */
int comet_sincos_table(const float* pos, float* out, int64_t m, int dim, int64_t ld, int64_t col0,
                       void* stream);
/* HarmonicEmbedding (minipytorch3d/harmonic_embedding.py:127-158): x [rows, dim], optional
 * diag_cov [rows, dim], freqs [n] -> y [rows, dim*(2n + append)]; backward gives dx, dcov. */
int comet_harmonic_fwd(const float* x, const float* diag_cov, const float* freqs, float* y, int64_t rows,
                       int dim, int n_freqs, int append_input, void* stream);
int comet_harmonic_bwd(const float* x, const float* diag_cov, const float* freqs, const float* dy,
                       float* dx, float* dcov, int64_t rows, int dim, int n_freqs, int append_input,
                       void* stream);
/* camera_to_pose_encoding2 per sequence (utils.py:631-688): R [B*S,4], T_uvz [B*S,3],
 * focal [B*S,2] -> enc [B*S,8]; ratio as in the reference (float64): the host value, or, when
 * ratio_dev is non-NULL, the float64 read from that device address (no host sync for a ratio that
 * already lives in HBM). */
int comet_pose_encode(const float* R, const float* T_uvz, const float* focal, double ratio,
                      const double* ratio_dev, float* enc, int64_t B, int S, void* stream);
/* pose_encoding_to_camera2 per sequence (utils.py:312-403): enc [B*S,7] -> R [B*S,4] (f32),
 * T [B*S,3] (f64, as the reference's float64 promotion), intrinsics fx, fy, cx, cy. */
int comet_pose_decode(const float* enc, const float* R_gt, const float* T_uvz_gt, double ratio,
                      const double* ratio_dev, double fx,
                      double fy, double cx, double cy, float* R_out, double* T_out, int64_t B, int S,
                      void* stream);
/* Single-head ablations (camera_predictor_abl_uvz.py / _abl_all.py): camera_to_pose_encoding3
 * (utils.py:591-627) per sequence: enc [B*S,8] = (T_i - T_0 in xyz, q_i * q_0^-1 standardised,
 * 0 padding; frame 0 = (0,0,0,1,0,0,0,0)) -- the GAPR kernels take it like encoding 2; and
 * pose_encoding_to_camera3 (utils.py:270-310): enc [B*S,7] -> R = dq * q_0, T = T_0 + dxyz (f32). */
int comet_pose_encode3(const float* R, const float* T, float* enc, int64_t B, int S, void* stream);
int comet_pose_decode3(const float* enc, const float* R_gt, const float* T_gt, float* R_out, float* T_out,
                       int64_t B, int S, void* stream);
/* GAPR head + pose loss (camera_predictor10.py:385-460): F.normalize(rot, eps 1e-8), loss =
 * w_trans*100*MSE(uvd[1:]) + w_rot*100*MSE(q[1:]) (mean over sequences), frame-0 reset.
 * gt_enc may be NULL (no loss). qn [B*S,4] is kept for the backward. */
int comet_gapr_fwd(const float* rot, int64_t ld_rot, const float* uv, int64_t ld_uv, const float* d,
                   int64_t ld_d, const float* gt_enc, float* qn, float* enc, float* losses, int B, int S,
                   float w_trans, float w_rot, void* stream);
/* dlosses[3] = upstream grads of (loss, loss_trans, loss_rot) (device) -> drot [B*S,4],
 * duv [B*S,2], dd [B*S,1] */
int comet_gapr_bwd(const float* rot, int64_t ld_rot, const float* uv, int64_t ld_uv, const float* d,
                   int64_t ld_d, const float* gt_enc, const float* qn, const float* dlosses, float* drot,
                   float* duv, float* dd, int B, int S, float w_trans, float w_rot, void* stream);

/* ---------------------------------------------------------------------------------------
 * Point tracker (base_track_predictor.py, blocks.py:351-429, refine_track.py) and DINOv2 input.
 * Feature maps are NHWC [n, H, W, C]; track state is [B, N, S, .] (row t = (b*N + n)*S + s).
 * ------------------------------------------------------------------------------------- */
/* sample_features4d / bilinear_sampler (utils.py:874-974): align_corners=True pixel coords,
 * border (1) or zeros (0) padding; out f32 [B, R, C] (element strides given). */
int comet_sample_bilinear(int dtype, const void* fmap, int64_t bstride, int H, int W, int C,
                          const float* coords, int64_t cstride_b, int64_t cstride_r, float* out,
                          int64_t ostride_b, int64_t ostride_r, int64_t B, int64_t R, int border,
                          void* stream);
/* CorrBlock.corr + .sample fused (blocks.py:376-429): pyramid[l] NHWC [B*S, H_l, W_l, C],
 * feats f32 [B*N*S, C], coords f32 [B*N*S, 2] (level-0 units) -> out[t*ldo + col0 + l*(2r+1)^2 + k] */
int comet_corr_sample(int dtype_fmap, int dtype_feat, const void* const* pyramid, const int* heights,
                      const int* widths, int levels, int radius, int C, const void* feats,
                      const float* coords, float* out, int64_t ldo, int64_t col0, int64_t B, int64_t N,
                      int S, void* stream);
/* transformer input (base_track_predictor.py:170-221): [flow emb | flows | corr | feats | pad] + pos,
 * tdim columns at row pitch ldx >= tdim; columns tdim..ldx-1 are written as zeros (rows padded to
 * the consuming GEMM's 64-deep k-tile; ldx > tdim needs tdim, ldx % 4 == 0 and 16-B aligned pos). */
int comet_tracker_tokens(int dtype_out, const float* coords, const float* feats, int latent,
                         const float* corr, int64_t ldcorr, int corrdim, const float* pos, int tdim,
                         void* x, int64_t ldx, int64_t rows, int S, void* stream);
/* coords += delta[:, :2] (frame 0 pinned); preds [B, S, N, 2] = coords * scale (may be NULL) */
int comet_coords_update(int dtype_delta, float* coords, const void* delta, int64_t ldd, float* preds,
                        float scale, int64_t B, int64_t N, int S, void* stream);
/* F.avg_pool2d(2, 2) on NHWC (CorrBlock pyramid, blocks.py:369-374) */
int comet_avgpool2_nhwc(int dtype, const void* x, void* y, int64_t n, int H, int W, int C, void* stream);
/* refine_track.py:74-131: patches NHWC [B*N*S, P, P, cpad] in (b, n, s) order (RGB in channels
 * 0..2, channels 3..cpad-1 zero: cpad 8 lets the first conv run as an implicit GEMM), topleft
 * [B,S,N,2] (int, unclamped), query [B*N,2] = frac(coarse[:, 0]) + pradius */
int comet_patch_gather(int dtype_out, const float* images, const float* coarse, void* patches,
                       int* topleft, float* query, int64_t B, int S, int64_t N, int H, int W,
                       int pradius, int cpad, void* stream);
/* track_predictor.py:117-143: RGB NCHW f32 [n,3,H,W] -> [n, oh, ow, cpad] (channels 3.. zero),
 * align_corners bilinear resize when (oh, ow) != (H, W) (the x1/down_ratio interpolate). */
int comet_images_nhwc(int dtype_out, const float* images, void* out, int64_t n, int H, int W, int oh,
                      int ow, int cpad, void* stream);
/* refined[b,s,n] = fine[(b*N+n), s] + topleft[b,s,n]; frame 0 = coarse query (refine_track.py:143-153) */
int comet_refine_combine(const float* fine, const int* topleft, const float* coarse, float* refined,
                         int64_t B, int S, int64_t N, void* stream);
/* compute_score_fn + score inversion (refine_track.py:174-278, E2Epose2.py:232-236):
 * qfeat [B*N, C], pfeat NHWC [B*N, S, P, P, C], fine [B*N, S, 2] -> score, inv_score [B, S, N] */
int comet_track_score(int dtype_feat, const float* qfeat, const void* pfeat, const float* fine,
                      float* score, float* inv_score, int64_t B, int S, int64_t N, int P, int C,
                      int sradius, void* stream);
/* camera_predictor10.py:624-634 + DINOv2 patch_embed im2col: images [BS,3,H,W] -> resize to
 * R (align_corners) -> (x-mean)/std -> cols [BS*(R/p)^2, ldc], column ci*p*p + ky*p + kx */
int comet_dino_prep(int dtype_out, const float* images, void* cols, int64_t BS, int H, int W, int R,
                    int patch, int64_t ldc, const float* mean3, const float* std3, void* stream);

/* ---------------------------------------------------------------------------------------
 * Evaluation metrics (comet/models/metric.py; called by the eval block of
 * train_eval_func_new_cp5.py:633-671). f32, one thread per pair / frame.
 * comet_pose_pair_errors: camera_to_rel_deg3's all-pairs part (metric.py:214-245): world-to-view
 *   matrices [batch*frames, 4, 4] (PyTorch3D layout [[R, 0], [T, 1]], get_matrix()), pairs i < j of
 *   each sequence in torch.combinations order -> rotation_angle / translation_angle in degrees,
 *   [batch * frames*(frames-1)/2] each (metric.py:561-570, 611-701).
 * comet_pose_frame_errors: camera_to_rel_deg2 (the definition bound last, metric.py:391-451) per
 *   frame: translation_angle(gt[:, :3], pred[:, :3]) in degrees, geodesic angle of Rp·Rgᵀ in radians
 *   (metric.py:326-347) and the Euler angles of Rp·Rgᵀ [n, 3] (metric.py:302-323), from pose
 *   encodings pred [n, ld_pred >= 7] (u, v, d, qw, qx, qy, qz) and gt [n, ld_gt >= 7].
 * ------------------------------------------------------------------------------------- */
int comet_pose_pair_errors(const float* pred_w2v, const float* gt_w2v, int64_t batch, int64_t frames,
                           float* rot_deg, float* trans_deg, void* stream);
int comet_pose_frame_errors(const float* pred_enc, int64_t ld_pred, const float* gt_enc, int64_t ld_gt,
                            int64_t n, float* trans_deg, float* geo_rad, float* euler, void* stream);

/* ---------------------------------------------------------------------------------------
 * Data path (YTDataset.load_images_from_folder, kubric_movif_SFM_dataset_YT.py:236-266):
 * PIL Image.crop (black outside the frame) + Image.resize(crop_size, LANCZOS) + ImageNet
 * normalisation, byte-exact with Pillow's Resample.c.
 * comet_resample_coeffs (host): Pillow's precompute_coeffs + normalize_coeffs_8bpc for LANCZOS
 *   over the source span [in0, in1) of in_size pixels -> bounds [out_size*2] (first source pixel,
 *   tap count), coeffs [out_size*max_ksize] int32 (22 fraction bits); coeffs == NULL: only the
 *   table width *ksize.
 * comet_lanczos_crop_resize (device): frames [n][h][w][3] uint8 (frame_stride bytes apart), crop
 *   box origin (x0, y0) size (cw, ch), output (ow, oh): horizontal pass over crop rows
 *   ybase .. ybase + rows - 1 (bx / kx, width ksx; skipped when ow == cw) into tmp
 *   [n][rows][ow][3] uint8, vertical pass (by rebased to ybase / ky, width ksy; skipped when
 *   oh == ch) -> out [n][3][oh][ow] f32 = (u / 255 - mean[c]) / std[c]. */
int comet_resample_coeffs(int in_size, float in0, float in1, int out_size, int32_t* bounds, int32_t* coeffs,
                          int max_ksize, int* ksize);
int comet_lanczos_crop_resize(const uint8_t* frames, int64_t n, int h, int w, int64_t frame_stride, int x0, int y0,
                              int cw, int ch, int ow, int oh, const int32_t* bx, const int32_t* kx, int ksx,
                              const int32_t* by, const int32_t* ky, int ksy, int ybase, int rows, uint8_t* tmp,
                              const float* mean, const float* stdv, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Keypoint initialisation (train_eval_func_new_cp5.py:527-595: lightglue SuperPoint.extract on
 * frame 0, then filter_and_pad): the SuperPoint encoder / detector convolutions run on
 * comet_conv2d_nhwc; these are its other dense stages.
 * comet_sp_preprocess: x [B,3,H,W] f32 -> bilinear (align_corners=False) resize to OH x OW
 *   (up-sampling only) + grayscale (0.299, 0.587, 0.114) -> y [B,OH,OW,cpad] (channel 0; rest 0).
 * comet_maxpool2_nhwc: nn.MaxPool2d(2, 2) on NHWC.
 * comet_sp_scores: detector logits [B,h,w,65] f32 -> softmax, dustbin dropped, depth-to-space
 *   -> scores [B, 8h, 8w].
 * comet_maxfilt2d: (2r+1)^2 stride-1 max filter of [B,H,W] f32 (max_pool2d with padding r),
 *   tmp = B*H*W floats of workspace (simple_nms; filter_and_pad's 3x3 mask dilation). */
int comet_sp_preprocess(int dtype_y, const float* x, void* y, int B, int H, int W, int OH, int OW, int cpad,
                        void* stream);
int comet_maxpool2_nhwc(int dtype, const void* x, void* y, int64_t n, int H, int W, int C, void* stream);
int comet_sp_scores(const float* logits, float* scores, int B, int h, int w, void* stream);
int comet_maxfilt2d(const float* x, float* y, float* tmp, int B, int H, int W, int r, void* stream);

/* ---------------------------------------------------------------------------------------
 * Debug support (bounds asserts and a NaN / Inf check mode).
 * comet_count_nonfinite: adds the number of NaN / Inf elements of x (n elements, dtype) to
 *   *count (an int32 on the device; no host sync). Used by comet_amd.debug's finite-check hooks.
 * comet_debug_flags: the build's debug state. In a `make DEBUG=1` library (libcomet_hip_debug.so,
 *   compiled with COMET_DEBUG) every launch is followed by a device synchronise and a read of the
 *   device-side assertion word (index checks inside the kernels record a failed check there instead
 *   of trapping); the call returns that word and clears it (clear != 0). A release library returns
 *   -1. */
int comet_count_nonfinite(int dtype, const void* x, int64_t n, int32_t* count, void* stream);
int comet_debug_flags(int clear);
/* comet_lds_probe: LDS integrity probe for concurrency tests (tools/lds_race.py,
 *   tests/test_ops_gpu.py). `groups` workgroups each own the CU's whole LDS (160 KiB): per round
 *   they fill it with a pattern keyed by (workgroup, round), sleep about `spin` x 8k cycles and
 *   count the words that changed, adding the count to *bad (a uint32 on the device). A workgroup's
 *   LDS is its own, so any change is a write that landed after the CU handed the LDS over -- e.g.
 *   LDS-DMA of a kernel that ended with pieces in flight. */
int comet_lds_probe(int groups, int rounds, int spin, uint32_t* bad, void* stream);
/* comet_shfl_probe: cross-lane exchange probe for concurrency tests (tools/op_repeat.py). Each wave
 *   sums known integers over its 64 lanes `iters` times -- mode 0 by ds_bpermute (__shfl_xor), 1 by
 *   DPP + v_permlane swaps, 2 through its own LDS words -- and adds the number of wrong lane results
 *   to *bad (uint32 on the device). */
int comet_shfl_probe(int groups, int iters, int mode, uint32_t* bad, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* COMET_HIP_H_ */
