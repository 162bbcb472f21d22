// Keypoint initialisation (train_eval_func_new_cp5.py:527-595): the dense parts of
// LightGlue's SuperPoint.extract on the GPU -- input resize + grayscale, 2x2 max pooling of the
// VGG encoder, the detector head's 65-way softmax + depth-to-space, and the max filter that its
// non-maximum suppression (simple_nms: three rounds of a (2r+1)^2 max pool) and filter_and_pad's
// mask dilation (a 3x3 max pool) are built from. The convolutions run on comet_conv2d_nhwc.
#include "common.hpp"

namespace comet {
namespace {

// kornia resize (F.interpolate bilinear, align_corners=False, up-sampling) of each RGB plane,
// then rgb_to_grayscale (0.299, 0.587, 0.114) -> NHWC with the gray value in channel 0 and zeros in
// channels 1..cpad-1 (the implicit-GEMM convolution takes c % 8 == 0).
template <typename TY>
__global__ void sp_preprocess_kernel(const float* __restrict__ x, TY* __restrict__ y, int B, int H, int W, int OH,
                                     int OW, int cpad) {
  const int64_t total = (int64_t)B * OH * OW;
  const float sh = (float)H / (float)OH, sw = (float)W / (float)OW;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(t % OW);
    const int64_t r = t / OW;
    const int oy = (int)(r % OH);
    const int b = (int)(r / OH);
    const float fy = fmaxf(sh * (oy + 0.5f) - 0.5f, 0.f), fx = fmaxf(sw * (ox + 0.5f) - 0.5f, 0.f);
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < H - 1), x1 = x0 + (x0 < W - 1);
    const float ly = fy - y0, lx = fx - x0;
    float g = 0.f;
    const float wgt[3] = {0.299f, 0.587f, 0.114f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* p = x + ((int64_t)b * 3 + c) * H * W;
      const float v = (1.f - ly) * ((1.f - lx) * p[y0 * W + x0] + lx * p[y0 * W + x1]) +
                      ly * ((1.f - lx) * p[y1 * W + x0] + lx * p[y1 * W + x1]);
      g += wgt[c] * v;
    }
    TY* o = y + t * cpad;
    o[0] = from_f32<TY>(g);
    for (int c = 1; c < cpad; ++c) o[c] = from_f32<TY>(0.f);
  }
}

// nn.MaxPool2d(2, 2) on NHWC
template <typename T>
__global__ void maxpool2_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int H, int W, int C) {
  const int OH = H / 2, OW = W / 2;
  const int64_t total = n * OH * OW * C;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    int64_t r = t / C;
    const int ox = (int)(r % OW);
    r /= OW;
    const int oy = (int)(r % OH);
    const int64_t b = r / OH;
    const T* p = x + ((b * H + 2 * oy) * W + 2 * ox) * C + c;
    const float m = fmaxf(fmaxf(to_f32(p[0]), to_f32(p[C])), fmaxf(to_f32(p[(int64_t)W * C]), to_f32(p[(int64_t)W * C + C])));
    y[t] = from_f32<T>(m);
  }
}

// Detector head decode: logits [B, h, w, 65] (f32 NHWC) -> softmax over the 65 channels, dustbin
// dropped, depth-to-space: scores[b][8i + a][8j + c] = p[b][i][j][8a + c].
__global__ void sp_scores_kernel(const float* __restrict__ logits, float* __restrict__ scores, int B, int h, int w) {
  const int64_t cells = (int64_t)B * h * w;
  const int lane = threadIdx.x & 63;
  const int64_t cell = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;  // one wave per cell
  if (cell >= cells) return;
  const float* p = logits + cell * 65;
  const float v = p[lane], v64 = p[64];
  const float m = fmaxf(wave_max(v), v64);
  const float e = __expf(v - m);
  const float s = wave_sum(e) + __expf(v64 - m);
  const int j = (int)(cell % w);
  const int64_t r = cell / w;
  const int i = (int)(r % h);
  const int b = (int)(r / h);
  const int a = lane >> 3, c = lane & 7;
  scores[((int64_t)b * 8 * h + 8 * i + a) * (8 * w) + 8 * j + c] = e / s;
}

// max over the (2r+1)-wide window along one axis (out-of-range taps ignored, as max_pool2d's -inf
// padding): axis 0 = along x (rows), 1 = along y (columns)
__global__ void maxfilt_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int H, int W, int r, int axis) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int xx = (int)(t % W);
    const int yy = (int)((t / W) % H);
    float m = -INFINITY;
    if (axis == 0) {
      const int lo = max(xx - r, 0), hi = min(xx + r, W - 1);
      const float* row = x + (t - xx);
      for (int k = lo; k <= hi; ++k) m = fmaxf(m, row[k]);
    } else {
      const int lo = max(yy - r, 0), hi = min(yy + r, H - 1);
      const float* col = x + (t - (int64_t)yy * W);
      for (int k = lo; k <= hi; ++k) m = fmaxf(m, col[(int64_t)k * W]);
    }
    y[t] = m;
  }
}

unsigned grid_for(int64_t n) {
  int64_t g = cdiv(n, 256);
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_sp_preprocess(int dtype_y, const float* x, void* y, int B, int H, int W, int OH, int OW, int cpad,
                                   void* stream) {
  COMET_CHECK_ARG(x && y && B > 0 && H > 0 && W > 0 && cpad >= 1, "comet_sp_preprocess: bad args");
  COMET_CHECK_ARG(OH >= H && OW >= W, "comet_sp_preprocess: up-sampling / identity only (no antialias path)");
  const unsigned g = grid_for((int64_t)B * OH * OW);
  if (dtype_y == COMET_BF16)
    hipLaunchKernelGGL((sp_preprocess_kernel<__bf16>), dim3(g), dim3(256), 0, as_stream(stream), x, (__bf16*)y, B, H, W,
                       OH, OW, cpad);
  else
    hipLaunchKernelGGL((sp_preprocess_kernel<float>), dim3(g), dim3(256), 0, as_stream(stream), x, (float*)y, B, H, W,
                       OH, OW, cpad);
  COMET_CHECK_LAUNCH("comet_sp_preprocess");
  return COMET_OK;
}

extern "C" int comet_maxpool2_nhwc(int dtype, const void* x, void* y, int64_t n, int H, int W, int C, void* stream) {
  COMET_CHECK_ARG(x && y && H >= 2 && W >= 2 && C > 0, "comet_maxpool2_nhwc: bad args");
  const unsigned g = grid_for(n * (H / 2) * (W / 2) * C);
  if (dtype == COMET_BF16)
    hipLaunchKernelGGL((maxpool2_kernel<__bf16>), dim3(g), dim3(256), 0, as_stream(stream), (const __bf16*)x, (__bf16*)y, n,
                       H, W, C);
  else
    hipLaunchKernelGGL((maxpool2_kernel<float>), dim3(g), dim3(256), 0, as_stream(stream), (const float*)x, (float*)y, n,
                       H, W, C);
  COMET_CHECK_LAUNCH("comet_maxpool2_nhwc");
  return COMET_OK;
}

extern "C" int comet_sp_scores(const float* logits, float* scores, int B, int h, int w, void* stream) {
  COMET_CHECK_ARG(logits && scores && B > 0 && h > 0 && w > 0, "comet_sp_scores: bad args");
  const int64_t threads = (int64_t)B * h * w * 64;
  hipLaunchKernelGGL(sp_scores_kernel, dim3((unsigned)cdiv(threads, 256)), dim3(256), 0, as_stream(stream), logits,
                     scores, B, h, w);
  COMET_CHECK_LAUNCH("comet_sp_scores");
  return COMET_OK;
}

// y = (2r+1) x (2r+1) max filter of x [B, H, W] f32 (stride 1, out-of-range taps ignored);
// tmp: caller workspace of B*H*W floats
extern "C" int comet_maxfilt2d(const float* x, float* y, float* tmp, int B, int H, int W, int r, void* stream) {
  COMET_CHECK_ARG(x && y && tmp && B > 0 && H > 0 && W > 0 && r >= 0, "comet_maxfilt2d: bad args");
  const unsigned g = grid_for((int64_t)B * H * W);
  hipLaunchKernelGGL(maxfilt_kernel, dim3(g), dim3(256), 0, as_stream(stream), x, tmp, B, H, W, r, 0);
  hipLaunchKernelGGL(maxfilt_kernel, dim3(g), dim3(256), 0, as_stream(stream), (const float*)tmp, y, B, H, W, r, 1);
  COMET_CHECK_LAUNCH("comet_maxfilt2d");
  return COMET_OK;
}
