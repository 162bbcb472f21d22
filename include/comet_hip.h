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
} comet_gemm_args;

int comet_gemm(const comet_gemm_args* args, void* stream);

/* ---------------------------------------------------------------------------------------
 * Row LayerNorm over the last dim (nn.LayerNorm; also GroupNorm(1, C) on [rows, C] as used
 * by base_track_predictor.py:81,238). weight/bias f32 or NULL (elementwise_affine=False,
 * modules.py:261-317). mean/rstd (f32, [rows]) are written when non-NULL (for backward).
 * Output dtype may differ from input dtype (f32 residual stream -> bf16 GEMM operand).
 * ------------------------------------------------------------------------------------- */
int comet_layernorm_fwd(int dtype_x, int dtype_y, const void* x, const float* weight,
                        const float* bias, void* y, float* mean, float* rstd,
                        int64_t rows, int64_t cols, float eps, void* stream);
/* dx (f32) = LN backward; dweight/dbias (f32) are ACCUMULATED (+=) when non-NULL.
 * dx_accumulate != 0 adds into dx instead of overwriting. */
int comet_layernorm_bwd(int dtype_x, int dtype_dy, const void* x, const void* dy,
                        const float* mean, const float* rstd, const float* weight,
                        float* dx, float* dweight, float* dbias, int64_t rows, int64_t cols,
                        int dx_accumulate, void* stream);

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
} comet_attn_args;

int comet_attention_fwd(const comet_attn_args* args, void* stream);

/* Attention backward helpers (materialised form, head_dim-agnostic):
 * probs[r, j] = exp(s[r, j]*scale - lse[r]); rows = batch*heads*lq, ld = row stride. */
int comet_attn_probs(int dtype_s, const void* s, const float* lse, void* p, int64_t rows,
                     int64_t cols, int64_t ld_s, int64_t ld_p, float scale, void* stream);
/* dS[r, j] = P[r, j] * (dP[r, j] - delta[r]) * scale, delta[r] = sum_d dO[r,d]*O[r,d]
 * (computed by comet_attn_delta). */
int comet_attn_delta(int dtype, const void* dout, const void* out, float* delta, int64_t batch,
                     int64_t heads, int64_t lq, int64_t d, int64_t so_b, int64_t so_h,
                     int64_t so_l, int64_t sdo_b, int64_t sdo_h, int64_t sdo_l, void* stream);
int comet_attn_dsoftmax(int dtype_p, const void* p, const void* dp, const float* delta, void* ds,
                        int64_t rows, int64_t cols, int64_t ld, float scale, void* stream);

/* ---------------------------------------------------------------------------------------
 * Elementwise / reductions.
 * ------------------------------------------------------------------------------------- */
int comet_cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, void* stream);
/* y = act(x) (f32 or bf16); gelu backward: dx = dy * gelu'(pre) */
int comet_act_bwd(int act, int dtype_pre, int dtype_dy, const void* pre, const void* dy,
                  void* dx, int dtype_dx, int64_t n, void* stream);
/* y = a*x + b*y (f32) */
int comet_axpby(const float* x, float* y, float a, float b, int64_t n, void* stream);
/* column sum: out[c] (+)= sum_r x[r*ld + c]  (bias gradients). */
int comet_colsum(int dtype, const void* x, float* out, int64_t rows, int64_t cols, int64_t ld,
                 int accumulate, void* stream);
/* squared L2 norm of many tensors: out[0] += sum x_i^2  (clip_grad_norm_, train_eval_func_new_cp5.py:797) */
int comet_sq_norm_multi(const float* const* ptrs, const int64_t* sizes, int n_tensors,
                        float* out, void* stream);
/* fused AdamW over many f32 tensors (torch.optim.AdamW defaults, train_util.py:311-332);
 * grad scaled by clip = min(1, max_norm / (sqrt(*sqnorm) + 1e-6)) when sqnorm != NULL. */
int comet_adamw_multi(float* const* params, const float* const* grads, float* const* exp_avg,
                      float* const* exp_avg_sq, const int64_t* sizes, int n_tensors, float lr,
                      float beta1, float beta2, float eps, float weight_decay, int step,
                      const float* sqnorm, float max_norm, void* stream);

/* ---------------------------------------------------------------------------------------
 * Convolution / CNN operators (channels-last NHWC activations).
 * ------------------------------------------------------------------------------------- */
/* im2col for conv2d NHWC input [n, h, w, c] -> cols [n*oh*ow, kh*kw*c] (zero padding). */
int comet_im2col_nhwc(int dtype_in, int dtype_out, const void* x, void* cols, int64_t n,
                      int64_t h, int64_t w, int64_t c, int kh, int kw, int stride, int pad,
                      int64_t oh, int64_t ow, int64_t ldc, void* stream);
/* InstanceNorm2d (affine=False, eps 1e-5) on NHWC, optional residual add and ReLU:
 * y = relu?( IN(x) + (res ? res : 0) ). res may be NULL. */
int comet_instnorm_nhwc(int dtype, const void* x, const void* res, void* y, int64_t n,
                        int64_t hw, int64_t c, float eps, int relu, int res_norm_relu,
                        void* stream);
/* bilinear resize, align_corners=True, NCHW or NHWC (F.interpolate, blocks.py:179-202,
 * track_predictor.py:137, camera_predictor10.py:624). add != 0 accumulates into y. */
int comet_resize_bilinear(int dtype_in, int dtype_out, int nhwc, const void* x, void* y,
                          int64_t n, int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow,
                          int add, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* COMET_HIP_H_ */
