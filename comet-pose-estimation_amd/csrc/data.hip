// Data path of YTDataset.load_images_from_folder (kubric_movif_SFM_dataset_YT.py:160-266, SURVEY
// §8(f2)): every selected frame is cropped to the sequence's square box (PIL Image.crop: pixels
// outside the frame are black), resized to crop_size with PIL's LANCZOS filter and normalised with
// the ImageNet mean / std into the model's [T, 3, H, W] float32 input.
//
// The resize reproduces Pillow's Resample.c bit for bit: separable passes (horizontal first, over
// only the source rows the vertical pass reads), int32 fixed-point coefficients with 22 fraction
// bits, rounding bias 1 << 21 and a clip to uint8 after each pass. The coefficient tables are built
// on the host by comet_resample_coeffs exactly as Pillow builds them (double math, same libm);
// the kernels only run the integer arithmetic, so the GPU frames equal PIL's byte for byte.
#include <cmath>
#include <vector>

#include "common.hpp"

namespace comet {
namespace {

constexpr int PB = 22;  // Resample.c PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8(int v) {
  if (v >= (1 << PB << 8)) return 255;
  if (v <= 0) return 0;
  return v >> PB;
}

// Horizontal pass: tmp[f][y][xx][c], y = crop rows ybase .. ybase + rows - 1. Source pixel (sx, sy)
// of the crop reads frame pixel (x0 + sx, y0 + sy), zero outside the frame (PIL crop fill).
__global__ void __launch_bounds__(256) lanczos_h_kernel(const uint8_t* __restrict__ frames, int64_t fstride,
                                                        int H, int W, int x0, int y0, int ybase, int rows,
                                                        int ow, const int* __restrict__ bx,
                                                        const int* __restrict__ kx, int ks,
                                                        uint8_t* __restrict__ tmp) {
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y, f = blockIdx.z;
  if (xx >= ow) return;
  const int sy = y0 + ybase + y;
  const int xmin = bx[2 * xx], xmax = bx[2 * xx + 1];
  const int* k = kx + (int64_t)xx * ks;
  int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
  if (sy >= 0 && sy < H) {
    const uint8_t* src = frames + f * fstride + (int64_t)sy * W * 3;
    for (int x = 0; x < xmax; ++x) {
      const int sx = x0 + xmin + x;
      if (sx < 0 || sx >= W) continue;
      const int w = k[x];
      s0 += (int)src[sx * 3 + 0] * w;
      s1 += (int)src[sx * 3 + 1] * w;
      s2 += (int)src[sx * 3 + 2] * w;
    }
  }
  uint8_t* o = tmp + (((int64_t)f * rows + y) * ow + xx) * 3;
  o[0] = (uint8_t)clip8(s0);
  o[1] = (uint8_t)clip8(s1);
  o[2] = (uint8_t)clip8(s2);
}

// No horizontal pass (crop width == output width): the crop rows themselves are the temp image.
__global__ void crop_rows_kernel(const uint8_t* __restrict__ frames, int64_t fstride, int H, int W, int x0, int y0,
                                 int rows, int cw, uint8_t* __restrict__ tmp) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y, f = blockIdx.z;
  if (x >= cw) return;
  const int sx = x0 + x, sy = y0 + y;
  const bool in = sx >= 0 && sx < W && sy >= 0 && sy < H;
  const uint8_t* src = frames + f * fstride + ((int64_t)sy * W + sx) * 3;
  uint8_t* o = tmp + (((int64_t)f * rows + y) * cw + x) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c] = in ? src[c] : (uint8_t)0;
}

// Vertical pass + normalisation: out[f][c][yy][xx] = (u / 255 - mean[c]) / std[c] (the reference's
// float32 ops in its order: video / 255.0, (video - mean) / std). need_v == 0: u = tmp row yy.
__global__ void __launch_bounds__(256) lanczos_v_kernel(const uint8_t* __restrict__ tmp, int rows, int ow, int oh,
                                                        int need_v, const int* __restrict__ by,
                                                        const int* __restrict__ ky, int ks,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ stdv, float* __restrict__ out) {
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  const int yy = blockIdx.y, f = blockIdx.z;
  if (xx >= ow) return;
  const uint8_t* t = tmp + (int64_t)f * rows * ow * 3;
  int u[3];
  if (need_v) {
    const int ymin = by[2 * yy], ymax = by[2 * yy + 1];
    const int* k = ky + (int64_t)yy * ks;
    int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
    for (int y = 0; y < ymax; ++y) {
      const uint8_t* p = t + ((int64_t)(ymin + y) * ow + xx) * 3;
      const int w = k[y];
      s0 += (int)p[0] * w;
      s1 += (int)p[1] * w;
      s2 += (int)p[2] * w;
    }
    u[0] = clip8(s0); u[1] = clip8(s1); u[2] = clip8(s2);
  } else {
    const uint8_t* p = t + ((int64_t)yy * ow + xx) * 3;
    u[0] = p[0]; u[1] = p[1]; u[2] = p[2];
  }
  const int64_t plane = (int64_t)oh * ow;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = __fdiv_rn((float)u[c], 255.0f);
    out[((int64_t)f * 3 + c) * plane + (int64_t)yy * ow + xx] = __fdiv_rn(v - mean[c], stdv[c]);
  }
}

// Resample.c lanczos_filter / sinc_filter (support 3)
double sinc_filter(double x) {
  if (x == 0.0) return 1.0;
  x = x * M_PI;
  return sin(x) / x;
}
double lanczos_filter(double x) {
  if (-3.0 <= x && x < 3.0) return sinc_filter(x) * sinc_filter(x / 3);
  return 0.0;
}

}  // namespace
}  // namespace comet

using namespace comet;

// Resample.c precompute_coeffs + normalize_coeffs_8bpc for the LANCZOS filter: output pixel xx
// reads source pixels bounds[2xx] .. bounds[2xx] + bounds[2xx+1] - 1 with int32 weights
// coeffs[xx * ksize + x]. coeffs == NULL: only *ksize is returned (table width to allocate).
extern "C" int comet_resample_coeffs(int in_size, float in0, float in1, int out_size, int32_t* bounds,
                                     int32_t* coeffs, int max_ksize, int* ksize) {
  COMET_CHECK_ARG(in_size > 0 && out_size > 0 && ksize != nullptr && in1 > in0, "comet_resample_coeffs: bad args");
  double scale = (double)(in1 - in0) / out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 3.0 * filterscale;
  const int ks = (int)ceil(support) * 2 + 1;
  *ksize = ks;
  if (coeffs == nullptr) return COMET_OK;
  COMET_CHECK_ARG(bounds != nullptr && max_ksize >= ks, "comet_resample_coeffs: table too narrow");
  std::vector<double> k(ks);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      const double w = lanczos_filter((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (int x = xmax; x < ks; ++x) k[x] = 0.0;
    for (int x = 0; x < ks; ++x)
      coeffs[(int64_t)xx * max_ksize + x] =
          k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << PB)) : (int32_t)(0.5 + k[x] * (1 << PB));
    for (int x = ks; x < max_ksize; ++x) coeffs[(int64_t)xx * max_ksize + x] = 0;
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return COMET_OK;
}

extern "C" int comet_lanczos_crop_resize(const uint8_t* frames, int64_t n, int h, int w, int64_t frame_stride,
                                         int x0, int y0, int cw, int ch, int ow, int oh, const int32_t* bx,
                                         const int32_t* kx, int ksx, const int32_t* by, const int32_t* ky,
                                         int ksy, int ybase, int rows, uint8_t* tmp, const float* mean,
                                         const float* stdv, float* out, void* stream) {
  COMET_CHECK_ARG(frames && tmp && mean && stdv && out && n >= 0 && h > 0 && w > 0 && cw > 0 && ch > 0 && ow > 0 &&
                      oh > 0 && rows > 0 && n <= 65535,
                  "comet_lanczos_crop_resize: bad args");
  if (n == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  const bool need_h = ow != cw, need_v = oh != ch;
  COMET_CHECK_ARG(!need_h || (bx && kx && ksx > 0), "comet_lanczos_crop_resize: horizontal tables missing");
  COMET_CHECK_ARG(!need_v || (by && ky && ksy > 0), "comet_lanczos_crop_resize: vertical tables missing");
  COMET_CHECK_ARG(need_v || rows == oh, "comet_lanczos_crop_resize: rows must equal oh without a vertical pass");
  const int tw = need_h ? ow : cw;
  if (need_h) {
    hipLaunchKernelGGL(lanczos_h_kernel, dim3((unsigned)cdiv(ow, 256), (unsigned)rows, (unsigned)n), dim3(256), 0, s,
                       frames, frame_stride, h, w, x0, y0, ybase, rows, ow, bx, kx, ksx, tmp);
  } else {
    hipLaunchKernelGGL(crop_rows_kernel, dim3((unsigned)cdiv(cw, 256), (unsigned)rows, (unsigned)n), dim3(256), 0, s,
                       frames, frame_stride, h, w, x0, y0 + ybase, rows, cw, tmp);
  }
  COMET_CHECK_LAUNCH("comet_lanczos_crop_resize (horizontal)");
  hipLaunchKernelGGL(lanczos_v_kernel, dim3((unsigned)cdiv(tw, 256), (unsigned)oh, (unsigned)n), dim3(256), 0, s,
                     tmp, rows, tw, oh, need_v ? 1 : 0, by, ky, ksy, mean, stdv, out);
  COMET_CHECK_LAUNCH("comet_lanczos_crop_resize (vertical)");
  return COMET_OK;
}
