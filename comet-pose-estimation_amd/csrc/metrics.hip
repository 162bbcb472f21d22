// Evaluation metrics of the COMET eval path (reference comet/models/metric.py), as
// called by train_eval_func_new_cp5.py:633-671 after model(..., training=False):
//
//  comet_pose_pair_errors   camera_to_rel_deg3 (metric.py:183-247): for every frame pair i < j of a
//                           sequence (batched_all_pairs order, metric.py:561-570) the relative pose
//                           inverse(M_i) @ M_j of the world-to-view matrices (closed_form_inverse,
//                           metric.py:611-642, PyTorch3D row-vector layout [[R, 0], [T, 1]]) for
//                           prediction and ground truth, then rotation_angle (metric.py:645-659:
//                           quaternions by matrix_to_quaternion, minipytorch3d/rotation_conversions.py:
//                           104-172) and translation_angle (metric.py:675-701) in degrees.
//  comet_pose_frame_errors  camera_to_rel_deg2 as bound last in metric.py (391-451): per frame the
//                           translation direction angle of the uvd encodings, the geodesic angle of
//                           Rp·Rgᵀ (geodesic_distance_from_two_batches, 326-347) and its Euler angles
//                           (rotationMatrixToEulerAngles, 302-323).
//
// One thread per pair / frame; f32 arithmetic in the reference's operation order (the reference
// runs these in f32: its autocast(dtype=torch.double) is disabled for CUDA). Tiny, latency-bound
// launches (B * S * (S - 1) / 2 pairs).
#include "common.hpp"

namespace comet {
namespace {


// minipytorch3d matrix_to_quaternion: best-conditioned of the four candidates (first maximum of
// q_abs, as torch.argmax), standardised to w >= 0
__device__ void mat2quat(const float (&m)[3][3], float (&q)[4]) {
  const float m00 = m[0][0], m01 = m[0][1], m02 = m[0][2];
  const float m10 = m[1][0], m11 = m[1][1], m12 = m[1][2];
  const float m20 = m[2][0], m21 = m[2][1], m22 = m[2][2];
  float a[4] = {1.0f + m00 + m11 + m22, 1.0f + m00 - m11 - m22, 1.0f - m00 + m11 - m22,
                1.0f - m00 - m11 + m22};
  for (int i = 0; i < 4; ++i) a[i] = a[i] > 0.f ? sqrtf(a[i]) : 0.f;
  int best = 0;
  for (int i = 1; i < 4; ++i)
    if (a[i] > a[best]) best = i;
  float c[4];
  switch (best) {
    case 0: c[0] = a[0] * a[0]; c[1] = m21 - m12; c[2] = m02 - m20; c[3] = m10 - m01; break;
    case 1: c[0] = m21 - m12; c[1] = a[1] * a[1]; c[2] = m10 + m01; c[3] = m02 + m20; break;
    case 2: c[0] = m02 - m20; c[1] = m10 + m01; c[2] = a[2] * a[2]; c[3] = m12 + m21; break;
    default: c[0] = m10 - m01; c[1] = m20 + m02; c[2] = m21 + m12; c[3] = a[3] * a[3]; break;
  }
  const float den = 2.0f * fmaxf(a[best], 0.1f);
  for (int i = 0; i < 4; ++i) q[i] = c[i] / den;
  if (q[0] < 0.f)
    for (int i = 0; i < 4; ++i) q[i] = -q[i];
}

// metric.py compare_translation_by_angle + translation_angle (ambiguity=True), degrees
__device__ float trans_angle_deg(const float (&tg)[3], const float (&tp)[3]) {
  const float np_ = sqrtf(tp[0] * tp[0] + tp[1] * tp[1] + tp[2] * tp[2]);
  const float ng = sqrtf(tg[0] * tg[0] + tg[1] * tg[1] + tg[2] * tg[2]);
  float d = 0.f;
  for (int i = 0; i < 3; ++i) d += (tp[i] / (np_ + 1e-15f)) * (tg[i] / (ng + 1e-15f));
  const float loss = fmaxf(1.0f - d * d, 1e-15f);
  float err = acosf(sqrtf(1.0f - loss));
  if (isnan(err) || isinf(err)) err = 1e6f;
  const float deg = err * 180.0f / 3.14159265358979323846f;
  return fminf(deg, fabsf(180.0f - deg));
}

// closed_form_inverse(M_i) @ M_j for [[R, 0], [T, 1]] matrices (row-major 4x4)
__device__ void rel_pose(const float* Mi, const float* Mj, float (&rel)[4][4]) {
  float inv[4][4];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) inv[r][c] = Mi[c * 4 + r];  // Rᵀ
  for (int c = 0; c < 3; ++c) {                            // -T · Rᵀ
    float s = 0.f;
    for (int k = 0; k < 3; ++k) s += Mi[12 + k] * inv[k][c];
    inv[3][c] = -s;
  }
  for (int r = 0; r < 4; ++r) inv[r][3] = Mi[r * 4 + 3];   // right column kept as is
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      float s = 0.f;
      for (int k = 0; k < 4; ++k) s += inv[r][k] * Mj[k * 4 + c];
      rel[r][c] = s;
    }
}

__global__ void pose_pair_errors_kernel(const float* __restrict__ pred, const float* __restrict__ gt, int S,
                                        int64_t npairs_total, float* __restrict__ rot_deg,
                                        float* __restrict__ trans_deg) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npairs_total) return;
  const int P = S * (S - 1) / 2;
  const int64_t b = idx / P;
  int p = (int)(idx - b * P);
  // torch.combinations order: (0,1), (0,2), ..., (0,S-1), (1,2), ...
  int i = 0;
  while (p >= S - 1 - i) { p -= S - 1 - i; ++i; }
  const int j = i + 1 + p;
  float rg[4][4], rp[4][4];
  rel_pose(gt + (b * S + i) * 16, gt + (b * S + j) * 16, rg);
  rel_pose(pred + (b * S + i) * 16, pred + (b * S + j) * 16, rp);
  float mg[3][3], mp[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) { mg[r][c] = rg[r][c]; mp[r][c] = rp[r][c]; }
  float qg[4], qp[4];
  mat2quat(mg, qg);
  mat2quat(mp, qp);
  float d = 0.f;
  for (int k = 0; k < 4; ++k) d += qp[k] * qg[k];
  const float loss = fmaxf(1.0f - d * d, 1e-15f);
  rot_deg[idx] = acosf(1.0f - 2.0f * loss) * 180.0f / 3.14159265358979323846f;
  const float tg[3] = {rg[3][0], rg[3][1], rg[3][2]};
  const float tp[3] = {rp[3][0], rp[3][1], rp[3][2]};
  trans_deg[idx] = trans_angle_deg(tg, tp);
}

// minipytorch3d quaternion_to_matrix
__device__ void quat2mat(const float* q, float (&m)[3][3]) {
  const float r = q[0], i = q[1], j = q[2], k = q[3];
  const float two_s = 2.0f / (r * r + i * i + j * j + k * k);
  m[0][0] = 1 - two_s * (j * j + k * k); m[0][1] = two_s * (i * j - k * r); m[0][2] = two_s * (i * k + j * r);
  m[1][0] = two_s * (i * j + k * r); m[1][1] = 1 - two_s * (i * i + k * k); m[1][2] = two_s * (j * k - i * r);
  m[2][0] = two_s * (i * k - j * r); m[2][1] = two_s * (j * k + i * r); m[2][2] = 1 - two_s * (i * i + j * j);
}

__global__ void pose_frame_errors_kernel(const float* __restrict__ pred, int64_t ldp, const float* __restrict__ gt,
                                         int64_t ldg, int64_t n, float* __restrict__ trans_deg,
                                         float* __restrict__ geo_rad, float* __restrict__ euler) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const float* pe = pred + f * ldp;
  const float* ge = gt + f * ldg;
  const float tg[3] = {ge[0], ge[1], ge[2]};
  const float tp[3] = {pe[0], pe[1], pe[2]};
  trans_deg[f] = trans_angle_deg(tg, tp);
  float Rp[3][3], Rg[3][3], m[3][3];
  quat2mat(pe + 3, Rp);
  quat2mat(ge + 3, Rg);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      float s = 0.f;
      for (int k = 0; k < 3; ++k) s += Rp[r][k] * Rg[c][k];  // Rp · Rgᵀ
      m[r][c] = s;
    }
  float cs = (m[0][0] + m[1][1] + m[2][2] - 1.0f) / 2.0f;
  cs = fminf(cs, 1.0f);
  cs = fmaxf(cs, -1.0f);
  geo_rad[f] = acosf(cs);
  // rotationMatrixToEulerAngles (numpy on the f32 matrix, math.* in double)
  const double m00 = m[0][0], m10 = m[1][0], m11 = m[1][1], m12 = m[1][2], m20 = m[2][0], m21 = m[2][1],
               m22 = m[2][2];
  const double sy = sqrt(m00 * m00 + m10 * m10);
  double x, y, z;
  if (!(sy < 1e-6)) {
    z = atan2(m21, m22);
    y = atan2(-m20, sy);
    x = atan2(m10, m00);
  } else {
    z = atan2(-m12, m11);
    y = atan2(-m20, sy);
    x = 0.0;
  }
  euler[f * 3 + 0] = (float)x;
  euler[f * 3 + 1] = (float)y;
  euler[f * 3 + 2] = (float)z;
}

}  // namespace
}  // namespace comet

extern "C" int comet_pose_pair_errors(const float* pred_w2v, const float* gt_w2v, int64_t batch, int64_t frames,
                                      float* rot_deg, float* trans_deg, void* stream) {
  using namespace comet;
  COMET_CHECK_ARG(pred_w2v && gt_w2v && rot_deg && trans_deg, "comet_pose_pair_errors: null pointer");
  COMET_CHECK_ARG(batch >= 1 && frames >= 2 && frames < 46341, "comet_pose_pair_errors: batch >= 1, frames >= 2");
  const int64_t total = batch * (frames * (frames - 1) / 2);
  hipLaunchKernelGGL(pose_pair_errors_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, as_stream(stream),
                     pred_w2v, gt_w2v, (int)frames, total, rot_deg, trans_deg);
  COMET_CHECK_LAUNCH("comet_pose_pair_errors");
  return COMET_OK;
}

extern "C" int comet_pose_frame_errors(const float* pred_enc, int64_t ld_pred, const float* gt_enc, int64_t ld_gt,
                                       int64_t n, float* trans_deg, float* geo_rad, float* euler, void* stream) {
  using namespace comet;
  COMET_CHECK_ARG(pred_enc && gt_enc && trans_deg && geo_rad && euler, "comet_pose_frame_errors: null pointer");
  COMET_CHECK_ARG(n >= 0 && ld_pred >= 7 && ld_gt >= 7, "comet_pose_frame_errors: ld >= 7");
  if (n == 0) return COMET_OK;
  hipLaunchKernelGGL(pose_frame_errors_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream),
                     pred_enc, ld_pred, gt_enc, ld_gt, n, trans_deg, geo_rad, euler);
  COMET_CHECK_LAUNCH("comet_pose_frame_errors");
  return COMET_OK;
}
