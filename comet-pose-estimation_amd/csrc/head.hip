// Camera-head kernels: elementwise helpers, sin/cos tables (T_F time encoder, 2-D patch
// embedding), HarmonicEmbedding, the fused GAPR head + pose loss, and the pose codec.
//
// Reference sites: camera_predictor10.py:329-484 (T_P gating, T_F, GAPR, loss, frame-0 reset),
// utils.py:312-403 (pose_encoding_to_camera2), utils.py:631-688 (camera_to_pose_encoding2),
// utils.py:724-832 (sin/cos tables), minipytorch3d/harmonic_embedding.py:14-158,
// minipytorch3d/rotation_conversions.py:382-449 (quaternion ops).
#include "common.hpp"

// The reference evaluates these formulas as separate f32 tensor ops: keep every product and sum
// rounded on its own (no FMA contraction) so the tiny head kernels match it to the ulp.
#pragma clang fp contract(off)

namespace comet {
namespace {

inline unsigned g1d(int64_t n) {
  int64_t g = cdiv(n, 256);
  return (unsigned)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}
#define GRID_STRIDE(i, n) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

template <typename TI, typename TO>
__global__ void act_fwd_kernel(int act, const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  GRID_STRIDE(i, n) y[i] = from_f32<TO>(apply_act(act, to_f32(x[i])));
}

// op 0: a + b, 1: relu(a + b), 2: a * b
template <typename T>
__global__ void binary_kernel(int op, const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, int64_t n) {
  GRID_STRIDE(i, n) {
    const float u = to_f32(a[i]), v = to_f32(b[i]);
    float o = op == 2 ? u * v : u + v;
    if (op == 1) o = o > 0.f ? o : 0.f;
    y[i] = from_f32<T>(o);
  }
}

template <typename TI, typename TO>
__global__ void add_rows_kernel(const TI* __restrict__ x, const float* __restrict__ table, TO* __restrict__ y,
                                int64_t rows, int64_t cols, int64_t period, int64_t ldx, int64_t ldy) {
  GRID_STRIDE(i, rows * cols) {
    const int64_t r = i / cols, c = i % cols;
    y[r * ldy + c] = from_f32<TO>(to_f32(x[r * ldx + c]) + table[(r % period) * cols + c]);
  }
}

// y = x + t elementwise (t f32, same shape), 4 elements per thread-step: the update formers' flow-head
// input (blocks.py:347, tokens + init) written straight in the GEMM's bf16 (one rounding of the f32 sum,
// as the reference's f32 add followed by autocast's cast)
template <typename TI, typename TO>
__global__ void add_cast4_kernel(const TI* __restrict__ x, const float* __restrict__ t, TO* __restrict__ y, int64_t n4) {
  GRID_STRIDE(i, n4) {
    float a[4], b[4];
    loadn<4>(x + 4 * i, a);
    loadn<4>(t + 4 * i, b);
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] += b[e];
    storen<4>(y + 4 * i, a);
  }
}

template <typename T>
__global__ void rowscale_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w, T* __restrict__ y,
                                    int64_t rows, int64_t cols) {
  GRID_STRIDE(i, rows * cols) y[i] = from_f32<T>(to_f32(x[i]) * w[i / cols]);
}

// one wave per row: dx = dy * w[r]; dw[r] = sum_c dy * x
template <typename T>
__global__ void rowscale_bwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                    const float* __restrict__ dy, float* __restrict__ dx,
                                    float* __restrict__ dw, int64_t rows, int64_t cols) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const float wr = w[r];
  float s = 0.f;
  for (int64_t c = lane; c < cols; c += 64) {
    const float g = dy[r * cols + c];
    s += g * to_f32(x[r * cols + c]);
    if (dx) dx[r * cols + c] = g * wr;
  }
  s = wave_sum(s);
  if (lane == 0 && dw) dw[r] = s;
}

// get_1d_sincos_pos_embed_from_grid (utils.py:807-832): double math, f32 out.
// out[m, d] = sin(pos[m] * omega_d) (d < D/2), cos(...) (d >= D/2); omega_d = 10000^(-d/(D/2))
__global__ void sincos_kernel(const float* __restrict__ pos, float* __restrict__ out, int64_t m, int dim,
                              int64_t ld, int64_t col0) {
  const int half = dim / 2;
  GRID_STRIDE(i, m * dim) {
    const int64_t r = i / dim;
    const int d = (int)(i % dim);
    const int k = d < half ? d : d - half;
    double om = (double)k / ((double)dim / 2.0);
    om = 1.0 / pow(10000.0, om);
    const double a = (double)pos[r] * om;
    out[r * ld + col0 + d] = (float)(d < half ? sin(a) : cos(a));
  }
}

// HarmonicEmbedding: out[r, p*dim*n + i*n + k] = sin(x[r,i]*f_k + p*pi/2) * att; (+ x appended)
__global__ void harmonic_fwd_kernel(const float* __restrict__ x, const float* __restrict__ cov,
                                    const float* __restrict__ freqs, float* __restrict__ y, int64_t rows,
                                    int dim, int n, int append) {
  const int64_t width = (int64_t)dim * (2 * n + append);
  const float half_pi = 1.5707963267948966f;
  GRID_STRIDE(t, rows * width) {
    const int64_t r = t / width;
    const int64_t c = t % width;
    float v;
    if (c >= 2ll * dim * n) {
      v = x[r * dim + (c - 2ll * dim * n)];
    } else {
      const int p = (int)(c / ((int64_t)dim * n));
      const int i = (int)((c / n) % dim), k = (int)(c % n);
      const float e = x[r * dim + i] * freqs[k] + (p ? half_pi : 0.f);  // f32, as the reference
      v = (float)sin((double)e);  // correctly rounded: large |x*f| would lose accuracy in sinf
      if (cov) v *= expf(-0.5f * (cov[r * dim + i] * (freqs[k] * freqs[k])));
    }
    y[t] = v;
  }
}

// one thread per (r, i): dx = sum_{p,k} dy * cos(e_p) * f_k * att + dy_append; dcov likewise.
__global__ void harmonic_bwd_kernel(const float* __restrict__ x, const float* __restrict__ cov,
                                    const float* __restrict__ freqs, const float* __restrict__ dy,
                                    float* __restrict__ dx, float* __restrict__ dcov, int64_t rows,
                                    int dim, int n, int append) {
  const int64_t width = (int64_t)dim * (2 * n + append);
  const float half_pi = 1.5707963267948966f;
  GRID_STRIDE(t, rows * dim) {
    const int64_t r = t / dim;
    const int i = (int)(t % dim);
    const float xv = x[r * dim + i];
    float gx = append ? dy[r * width + 2ll * dim * n + i] : 0.f, gc = 0.f;
    for (int p = 0; p < 2; ++p)
      for (int k = 0; k < n; ++k) {
        const float f = freqs[k];
        const float e = xv * f + (p ? half_pi : 0.f);
        const float att = cov ? expf(-0.5f * (cov[r * dim + i] * (f * f))) : 1.f;
        const float g = dy[r * width + (int64_t)p * dim * n + (int64_t)i * n + k];
        gx += g * (float)cos((double)e) * f * att;
        if (cov) gc += g * (float)sin((double)e) * att * (-0.5f * f * f);
      }
    dx[t] = gx;
    if (dcov) dcov[t] = gc;
  }
}

__device__ __forceinline__ void qmul_std(const float* a, const float* b, float* o) {
  // quaternion_multiply (rotation_conversions.py:398-432): raw product, then w >= 0
  const float aw = a[0], ax = a[1], ay = a[2], az = a[3];
  const float bw = b[0], bx = b[1], by = b[2], bz = b[3];
  float w = aw * bw - ax * bx - ay * by - az * bz;
  float x = aw * bx + ax * bw + ay * bz - az * by;
  float y = aw * by - ax * bz + ay * bw + az * bx;
  float z = aw * bz + ax * by - ay * bx + az * bw;
  if (w < 0.f) { w = -w; x = -x; y = -y; z = -z; }
  o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

// camera_to_pose_encoding2 per frame (per-sequence reference = frame 0 of each sequence)
__global__ void pose_encode_kernel(const float* __restrict__ R, const float* __restrict__ T,
                                   const float* __restrict__ focal, double ratio,
                                   const double* __restrict__ ratio_dev, float* __restrict__ enc,
                                   int64_t B, int S) {
  if (ratio_dev) ratio = *ratio_dev;
  GRID_STRIDE(t, B * S) {
    const int64_t b = t / S;
    const int s = (int)(t % S);
    const float* r0 = R + b * S * 4;
    const float* t0 = T + b * S * 3;
    float* e = enc + t * 8;
    float fl = focal[t * 2];
    fl = fminf(fmaxf(fl, 0.1f), 30.f);
    e[7] = fl;
    if (s == 0) {
      e[0] = e[1] = e[2] = 0.f; e[3] = 1.f; e[4] = e[5] = e[6] = 0.f;
      continue;
    }
    const float* ri = R + t * 4;
    const float* ti = T + t * 3;
    const float inv[4] = {r0[0], -r0[1], -r0[2], -r0[3]};
    float q[4];
    qmul_std(ri, inv, q);
    const float du32 = ti[0] - t0[0], dv32 = ti[1] - t0[1];
    const float dd32 = (ti[2] / t0[2]) - 1.f;
    e[0] = (float)((double)du32 * ratio / 128.0);
    e[1] = (float)((double)dv32 * ratio / 128.0);
    e[2] = (float)((double)dd32 * ratio);
    e[3] = q[0]; e[4] = q[1]; e[5] = q[2]; e[6] = q[3];
  }
}

// pose_encoding_to_camera2 per frame: enc [B*S, 7]; reference = frame 0 of each sequence's gt.
// T is produced in double (the reference promotes through the float64 `ratio`, B-15).
__global__ void pose_decode_kernel(const float* __restrict__ enc, const float* __restrict__ Rgt,
                                   const float* __restrict__ Tgt, double ratio,
                                   const double* __restrict__ ratio_dev, double fx, double fy,
                                   double cx, double cy, float* __restrict__ Rout, double* __restrict__ Tout,
                                   int64_t B, int S) {
  if (ratio_dev) ratio = *ratio_dev;
  GRID_STRIDE(t, B * S) {
    const int64_t b = t / S;
    const float* e = enc + t * 7;
    const float* q0 = Rgt + b * S * 4;
    const float* t0 = Tgt + b * S * 3;
    const double u = (double)t0[0] + (double)e[0] / ratio * 128.0;
    const double v = (double)t0[1] + (double)e[1] / ratio * 128.0;
    const double d = (double)t0[2] * ((double)e[2] / ratio + 1.0);
    Tout[t * 3 + 0] = (u - cx) * d / fx;
    Tout[t * 3 + 1] = (v - cy) * d / fy;
    Tout[t * 3 + 2] = d;
    qmul_std(e + 3, q0, Rout + t * 4);
  }
}

// camera_to_pose_encoding3 per frame (utils.py:591-627, the single-head ablations abl_uvz /
// abl_all): enc [rows, 8] = (T_i - T_0 (xyz), quaternion_multiply(q_i, q_0^-1), 0); frame 0 =
// (0, 0, 0, 1, 0, 0, 0, 0). Column 7 is padding so the GAPR kernels read it like encoding 2.
__global__ void pose_encode3_kernel(const float* __restrict__ R, const float* __restrict__ T,
                                    float* __restrict__ enc, int64_t B, int S) {
  GRID_STRIDE(t, B * S) {
    const int64_t b = t / S;
    const int s = (int)(t % S);
    const float* r0 = R + b * S * 4;
    const float* t0 = T + b * S * 3;
    float* e = enc + t * 8;
    e[7] = 0.f;
    if (s == 0) {
      e[0] = e[1] = e[2] = 0.f; e[3] = 1.f; e[4] = e[5] = e[6] = 0.f;
      continue;
    }
    const float inv[4] = {r0[0], -r0[1], -r0[2], -r0[3]};
    float q[4];
    qmul_std(R + t * 4, inv, q);
    const float* ti = T + t * 3;
    e[0] = ti[0] - t0[0]; e[1] = ti[1] - t0[1]; e[2] = ti[2] - t0[2];
    e[3] = q[0]; e[4] = q[1]; e[5] = q[2]; e[6] = q[3];
  }
}

// pose_encoding_to_camera3 per frame (utils.py:270-310): R = quaternion_multiply(dq, q_0),
// T = T_0 + dxyz (f32, the xyz translation of the sequence's frame 0).
__global__ void pose_decode3_kernel(const float* __restrict__ enc, const float* __restrict__ Rgt,
                                    const float* __restrict__ Tgt, float* __restrict__ Rout,
                                    float* __restrict__ Tout, int64_t B, int S) {
  GRID_STRIDE(t, B * S) {
    const int64_t b = t / S;
    const float* e = enc + t * 7;
    const float* t0 = Tgt + b * S * 3;
    Tout[t * 3 + 0] = t0[0] + e[0];
    Tout[t * 3 + 1] = t0[1] + e[1];
    Tout[t * 3 + 2] = t0[2] + e[2];
    qmul_std(e + 3, Rgt + b * S * 4, Rout + t * 4);
  }
}

// GAPR head (camera_predictor10.py:385-460). One block; rows t = b*S + s.
// rot raw [rows,4] (ld_rot), uv [rows,2] (ld_uv), dd [rows,1] (ld_d), gt [rows,8] or NULL.
// Outputs: qn [rows,4] normalized quats (pre-reset, kept for backward), enc [rows,7] with frame 0
// forced to (0,0,0,1,0,0,0), losses[3] = (loss, trans, rot) = mean over sequences.
__global__ void __launch_bounds__(256)
gapr_fwd_kernel(const float* __restrict__ rot, int64_t ld_rot, const float* __restrict__ uv, int64_t ld_uv,
                const float* __restrict__ dd, int64_t ld_d, const float* __restrict__ gt,
                float* __restrict__ qn_out, float* __restrict__ enc, float* __restrict__ losses,
                int B, int S, float w_trans, float w_rot) {
  __shared__ float red[2][256];
  float st = 0.f, sr = 0.f;  // sum over sequences of per-sequence MSE sums (scaled later)
  for (int t = threadIdx.x; t < B * S; t += 256) {
    const int s = t % S;
    const float* q = rot + (int64_t)t * ld_rot;
    const float nrm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const float den = fmaxf(nrm, 1e-8f);
    float qn[4];
    for (int j = 0; j < 4; ++j) { qn[j] = q[j] / den; qn_out[t * 4 + j] = qn[j]; }
    const float u = uv[(int64_t)t * ld_uv], v = uv[(int64_t)t * ld_uv + 1], d = dd[(int64_t)t * ld_d];
    if (gt && s > 0) {
      const float* g = gt + (int64_t)t * 8;
      const float e0 = u - g[0], e1 = v - g[1], e2 = d - g[2];
      st += e0 * e0 + e1 * e1 + e2 * e2;
      for (int j = 0; j < 4; ++j) { const float e = qn[j] - g[3 + j]; sr += e * e; }
    }
    float* o = enc + (int64_t)t * 7;
    if (s == 0) {
      o[0] = o[1] = o[2] = 0.f; o[3] = 1.f; o[4] = o[5] = o[6] = 0.f;
    } else {
      o[0] = u; o[1] = v; o[2] = d;
      for (int j = 0; j < 4; ++j) o[3 + j] = qn[j];
    }
  }
  red[0][threadIdx.x] = st;
  red[1][threadIdx.x] = sr;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      red[0][threadIdx.x] += red[0][threadIdx.x + off];
      red[1][threadIdx.x] += red[1][threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && gt && losses) {
    // every sequence has the same element count, so mean over sequences of per-sequence means
    // = global mean over all (S-1)*B rows
    const float tl = 100.f * red[0][0] / (float)(3 * (S - 1) * B);
    const float rl = 100.f * red[1][0] / (float)(4 * (S - 1) * B);
    losses[0] = w_trans * tl + w_rot * rl;
    losses[1] = tl;
    losses[2] = rl;
  }
}

__global__ void gapr_bwd_kernel(const float* __restrict__ rot, int64_t ld_rot, const float* __restrict__ uv,
                                int64_t ld_uv, const float* __restrict__ dd, int64_t ld_d,
                                const float* __restrict__ gt, const float* __restrict__ qn,
                                const float* __restrict__ dlosses, float* __restrict__ drot,
                                float* __restrict__ duv, float* __restrict__ ddd, int B, int S,
                                float w_trans, float w_rot) {
  const float gl = dlosses[0], gtl = dlosses[1], grl = dlosses[2];
  const float ct = (gl * w_trans + gtl) * 100.f * 2.f / (float)(3 * (S - 1) * B);
  const float cr = (gl * w_rot + grl) * 100.f * 2.f / (float)(4 * (S - 1) * B);
  GRID_STRIDE(t, (int64_t)B * S) {
    const int s = (int)(t % S);
    const float* g = gt + t * 8;
    float du = 0.f, dv = 0.f, dd_ = 0.f, dq[4] = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      du = ct * (uv[t * ld_uv] - g[0]);
      dv = ct * (uv[t * ld_uv + 1] - g[1]);
      dd_ = ct * (dd[t * ld_d] - g[2]);
      for (int j = 0; j < 4; ++j) dq[j] = cr * (qn[t * 4 + j] - g[3 + j]);
    }
    duv[t * 2] = du; duv[t * 2 + 1] = dv; ddd[t] = dd_;
    const float* q = rot + t * ld_rot;
    const float nrm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (nrm > 1e-8f) {
      float dot = 0.f;
      for (int j = 0; j < 4; ++j) dot += qn[t * 4 + j] * dq[j];
      for (int j = 0; j < 4; ++j) drot[t * 4 + j] = (dq[j] - qn[t * 4 + j] * dot) / nrm;
    } else {
      for (int j = 0; j < 4; ++j) drot[t * 4 + j] = dq[j] / 1e-8f;
    }
  }
}

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_act_fwd(int act, int dtype_x, int dtype_y, const void* x, void* y, int64_t n, void* stream) {
  COMET_CHECK_ARG(x && y, "comet_act_fwd: null pointer");
  if (n == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
#define AF(TI, TO) hipLaunchKernelGGL((act_fwd_kernel<TI, TO>), dim3(g1d(n)), dim3(256), 0, s, act, (const TI*)x, (TO*)y, n)
  if (dtype_x == COMET_F32 && dtype_y == COMET_F32) AF(float, float);
  else if (dtype_x == COMET_F32 && dtype_y == COMET_BF16) AF(float, __bf16);
  else if (dtype_x == COMET_BF16 && dtype_y == COMET_F32) AF(__bf16, float);
  else AF(__bf16, __bf16);
#undef AF
  COMET_CHECK_LAUNCH("comet_act_fwd");
  return COMET_OK;
}

extern "C" int comet_binary(int op, int dtype, const void* a, const void* b, void* y, int64_t n, void* stream) {
  COMET_CHECK_ARG(a && b && y && op >= 0 && op <= 2, "comet_binary: bad args");
  if (n == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((binary_kernel<float>), dim3(g1d(n)), dim3(256), 0, s, op, (const float*)a, (const float*)b, (float*)y, n);
  else
    hipLaunchKernelGGL((binary_kernel<__bf16>), dim3(g1d(n)), dim3(256), 0, s, op, (const __bf16*)a, (const __bf16*)b, (__bf16*)y, n);
  COMET_CHECK_LAUNCH("comet_binary");
  return COMET_OK;
}

extern "C" int comet_add_rows(int dtype_x, int dtype_y, const void* x, const float* table, void* y,
                              int64_t rows, int64_t cols, int64_t period, int64_t ldx, int64_t ldy, void* stream) {
  COMET_CHECK_ARG(x && table && y && period > 0, "comet_add_rows: bad args");
  if (rows == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  const int64_t n = rows * cols;
  if (period >= rows && ldx == cols && ldy == cols && n % 4 == 0 &&
      ((uintptr_t)x | (uintptr_t)table | (uintptr_t)y) % 16 == 0) {  // plain elementwise: vector path
#define AC(TI, TO) hipLaunchKernelGGL((add_cast4_kernel<TI, TO>), dim3(g1d(n / 4)), dim3(256), 0, s, (const TI*)x, table, (TO*)y, n / 4)
    if (dtype_x == COMET_F32 && dtype_y == COMET_F32) AC(float, float);
    else if (dtype_x == COMET_F32 && dtype_y == COMET_BF16) AC(float, __bf16);
    else if (dtype_x == COMET_BF16 && dtype_y == COMET_F32) AC(__bf16, float);
    else AC(__bf16, __bf16);
#undef AC
    COMET_CHECK_LAUNCH("comet_add_rows (elementwise)");
    return COMET_OK;
  }
  const unsigned g = g1d(rows * cols);
#define AR(TI, TO) hipLaunchKernelGGL((add_rows_kernel<TI, TO>), dim3(g), dim3(256), 0, s, (const TI*)x, table, (TO*)y, rows, cols, period, ldx, ldy)
  if (dtype_x == COMET_F32 && dtype_y == COMET_F32) AR(float, float);
  else if (dtype_x == COMET_F32 && dtype_y == COMET_BF16) AR(float, __bf16);
  else if (dtype_x == COMET_BF16 && dtype_y == COMET_F32) AR(__bf16, float);
  else AR(__bf16, __bf16);
#undef AR
  COMET_CHECK_LAUNCH("comet_add_rows");
  return COMET_OK;
}

extern "C" int comet_rowscale_fwd(int dtype, const void* x, const float* w, void* y, int64_t rows,
                                  int64_t cols, void* stream) {
  COMET_CHECK_ARG(x && w && y, "comet_rowscale_fwd: null pointer");
  if (rows == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((rowscale_fwd_kernel<float>), dim3(g1d(rows * cols)), dim3(256), 0, s, (const float*)x, w, (float*)y, rows, cols);
  else
    hipLaunchKernelGGL((rowscale_fwd_kernel<__bf16>), dim3(g1d(rows * cols)), dim3(256), 0, s, (const __bf16*)x, w, (__bf16*)y, rows, cols);
  COMET_CHECK_LAUNCH("comet_rowscale_fwd");
  return COMET_OK;
}

extern "C" int comet_rowscale_bwd(int dtype, const void* x, const float* w, const float* dy, float* dx,
                                  float* dw, int64_t rows, int64_t cols, void* stream) {
  COMET_CHECK_ARG(x && w && dy, "comet_rowscale_bwd: null pointer");
  if (rows == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  dim3 g((unsigned)cdiv(rows, 4));
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((rowscale_bwd_kernel<float>), g, dim3(256), 0, s, (const float*)x, w, dy, dx, dw, rows, cols);
  else
    hipLaunchKernelGGL((rowscale_bwd_kernel<__bf16>), g, dim3(256), 0, s, (const __bf16*)x, w, dy, dx, dw, rows, cols);
  COMET_CHECK_LAUNCH("comet_rowscale_bwd");
  return COMET_OK;
}

extern "C" int comet_sincos_table(const float* pos, float* out, int64_t m, int dim, int64_t ld, int64_t col0,
                                  void* stream) {
  COMET_CHECK_ARG(pos && out && dim % 2 == 0, "comet_sincos_table: bad args");
  if (m == 0) return COMET_OK;
  hipLaunchKernelGGL(sincos_kernel, dim3(g1d(m * dim)), dim3(256), 0, as_stream(stream), pos, out, m, dim, ld, col0);
  COMET_CHECK_LAUNCH("comet_sincos_table");
  return COMET_OK;
}

extern "C" int comet_harmonic_fwd(const float* x, const float* diag_cov, const float* freqs, float* y,
                                  int64_t rows, int dim, int n_freqs, int append_input, void* stream) {
  COMET_CHECK_ARG(x && freqs && y && dim > 0 && n_freqs > 0, "comet_harmonic_fwd: bad args");
  if (rows == 0) return COMET_OK;
  const int64_t width = (int64_t)dim * (2 * n_freqs + (append_input ? 1 : 0));
  hipLaunchKernelGGL(harmonic_fwd_kernel, dim3(g1d(rows * width)), dim3(256), 0, as_stream(stream), x, diag_cov,
                     freqs, y, rows, dim, n_freqs, append_input ? 1 : 0);
  COMET_CHECK_LAUNCH("comet_harmonic_fwd");
  return COMET_OK;
}

extern "C" int comet_harmonic_bwd(const float* x, const float* diag_cov, const float* freqs, const float* dy,
                                  float* dx, float* dcov, int64_t rows, int dim, int n_freqs, int append_input,
                                  void* stream) {
  COMET_CHECK_ARG(x && freqs && dy && dx, "comet_harmonic_bwd: bad args");
  if (rows == 0) return COMET_OK;
  hipLaunchKernelGGL(harmonic_bwd_kernel, dim3(g1d(rows * dim)), dim3(256), 0, as_stream(stream), x, diag_cov,
                     freqs, dy, dx, dcov, rows, dim, n_freqs, append_input ? 1 : 0);
  COMET_CHECK_LAUNCH("comet_harmonic_bwd");
  return COMET_OK;
}

extern "C" int comet_pose_encode(const float* R, const float* T_uvz, const float* focal, double ratio,
                                 const double* ratio_dev, float* enc, int64_t B, int S, void* stream) {
  COMET_CHECK_ARG(R && T_uvz && focal && enc && S >= 1, "comet_pose_encode: bad args");
  hipLaunchKernelGGL(pose_encode_kernel, dim3(g1d(B * S)), dim3(256), 0, as_stream(stream), R, T_uvz, focal,
                     ratio, ratio_dev, enc, B, S);
  COMET_CHECK_LAUNCH("comet_pose_encode");
  return COMET_OK;
}

extern "C" int comet_pose_decode(const float* enc, const float* R_gt, const float* T_uvz_gt, double ratio,
                                 const double* ratio_dev, double fx, double fy, double cx, double cy, float* R_out, double* T_out,
                                 int64_t B, int S, void* stream) {
  COMET_CHECK_ARG(enc && R_gt && T_uvz_gt && R_out && T_out, "comet_pose_decode: bad args");
  hipLaunchKernelGGL(pose_decode_kernel, dim3(g1d(B * S)), dim3(256), 0, as_stream(stream), enc, R_gt, T_uvz_gt,
                     ratio, ratio_dev, fx, fy, cx, cy, R_out, T_out, B, S);
  COMET_CHECK_LAUNCH("comet_pose_decode");
  return COMET_OK;
}

extern "C" int comet_pose_encode3(const float* R, const float* T, float* enc, int64_t B, int S, void* stream) {
  COMET_CHECK_ARG(R && T && enc && S >= 1, "comet_pose_encode3: bad args");
  if (B == 0) return COMET_OK;
  hipLaunchKernelGGL(pose_encode3_kernel, dim3(g1d(B * S)), dim3(256), 0, as_stream(stream), R, T, enc, B, S);
  COMET_CHECK_LAUNCH("comet_pose_encode3");
  return COMET_OK;
}

extern "C" int comet_pose_decode3(const float* enc, const float* R_gt, const float* T_gt, float* R_out, float* T_out,
                                  int64_t B, int S, void* stream) {
  COMET_CHECK_ARG(enc && R_gt && T_gt && R_out && T_out && S >= 1, "comet_pose_decode3: bad args");
  if (B == 0) return COMET_OK;
  hipLaunchKernelGGL(pose_decode3_kernel, dim3(g1d(B * S)), dim3(256), 0, as_stream(stream), enc, R_gt, T_gt, R_out,
                     T_out, B, S);
  COMET_CHECK_LAUNCH("comet_pose_decode3");
  return COMET_OK;
}

extern "C" int comet_gapr_fwd(const float* rot, int64_t ld_rot, const float* uv, int64_t ld_uv, const float* d,
                              int64_t ld_d, const float* gt_enc, float* qn, float* enc, float* losses, int B,
                              int S, float w_trans, float w_rot, void* stream) {
  COMET_CHECK_ARG(rot && uv && d && qn && enc && B > 0 && S > 0, "comet_gapr_fwd: bad args");
  COMET_CHECK_ARG(!gt_enc || S > 1, "comet_gapr_fwd: the pose loss needs S > 1");
  hipLaunchKernelGGL(gapr_fwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), rot, ld_rot, uv, ld_uv, d, ld_d,
                     gt_enc, qn, enc, losses, B, S, w_trans, w_rot);
  COMET_CHECK_LAUNCH("comet_gapr_fwd");
  return COMET_OK;
}

extern "C" int comet_gapr_bwd(const float* rot, int64_t ld_rot, const float* uv, int64_t ld_uv, const float* d,
                              int64_t ld_d, const float* gt_enc, const float* qn, const float* dlosses,
                              float* drot, float* duv, float* dd, int B, int S, float w_trans, float w_rot,
                              void* stream) {
  COMET_CHECK_ARG(rot && uv && d && gt_enc && qn && dlosses && drot && duv && dd, "comet_gapr_bwd: bad args");
  hipLaunchKernelGGL(gapr_bwd_kernel, dim3(g1d((int64_t)B * S)), dim3(256), 0, as_stream(stream), rot, ld_rot,
                     uv, ld_uv, d, ld_d, gt_enc, qn, dlosses, drot, duv, dd, B, S, w_trans, w_rot);
  COMET_CHECK_LAUNCH("comet_gapr_bwd");
  return COMET_OK;
}
