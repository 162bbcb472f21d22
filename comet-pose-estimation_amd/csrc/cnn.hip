#include <cstdlib>
// CNN operators on channels-last activations: im2col for the tracker encoders / DINOv2
// patch-embed convolutions, and align_corners=True bilinear resize.
//
// Reference sites: blocks.py:27-111 (BasicEncoder: conv7x7 s2, 3x3, 1x1, bilinear
// up-sampling), blocks.py:114-202 (ShallowEncoder on 31x31 patches), modules.py:39-116
// (ResidualBlock), track_predictor.py:137-143 (x1/2 resize), camera_predictor10.py:624-630
// (512 -> 336 resize), DINOv2 patch_embed (conv 14x14 s14).
#include "common.hpp"

namespace comet {
namespace {

// cols[(n*oh + oy)*ow + ox][(ky*kw + kx)*c + ci] = x[n][oy*s - p + ky][ox*s - p + kx][ci]
template <typename TI, typename TO>
__global__ void im2col_nhwc_kernel(const TI* __restrict__ x, TO* __restrict__ cols, int64_t n,
                                   int64_t h, int64_t w, int64_t c, int kh, int kw, int stride,
                                   int pad, int64_t oh, int64_t ow, int64_t ldc) {
  const int64_t kk = (int64_t)kh * kw * c;
  const int64_t total = n * oh * ow * ldc;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int64_t col = i % ldc, pix = i / ldc;
    if (col >= kk) { cols[i] = from_f32<TO>(0.f); continue; }
    const int64_t ci = col % c, kx = (col / c) % kw, ky = col / (c * kw);
    const int64_t ox = pix % ow, oy = (pix / ow) % oh, ni = pix / (ow * oh);
    const int64_t iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
    float v = 0.f;
    if (iy >= 0 && iy < h && ix >= 0 && ix < w) v = to_f32(x[((ni * h + iy) * w + ix) * c + ci]);
    cols[pix * ldc + col] = from_f32<TO>(v);
  }
}

// align_corners=True bilinear: src = dst * (in-1)/(out-1). Contraction off here and in bilerp, so
// every kernel that inlines them rounds each product and sum the same way (the fused resize + pool
// kernel equals resize followed by avgpool2 bit for bit whatever hipcc fuses around it)
__device__ __forceinline__ void ac_coord(int64_t o, int64_t in, int64_t out, int64_t& i0,
                                         int64_t& i1, float& f) {
#pragma clang fp contract(off)
  const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float src = scale * (float)o;
  i0 = (int64_t)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + 1 < in ? i0 + 1 : in - 1;
  f = src - (float)i0;
}

// same association as ATen's upsample_bilinear2d: h0lambda*(w0l*v00 + w1l*v01) + h1lambda*(...)
__device__ __forceinline__ float bilerp(float v00, float v01, float v10, float v11, float fx, float fy) {
#pragma clang fp contract(off)
  return (1.f - fy) * ((1.f - fx) * v00 + fx * v01) + fy * ((1.f - fx) * v10 + fx * v11);
}

template <typename TI, typename TO>
__global__ void resize_kernel(const TI* __restrict__ x, TO* __restrict__ y, int nhwc, int64_t n,
                              int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow, int add) {
  const int64_t total = n * c * oh * ow;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gs) {
    int64_t ni, ci, oy, ox;
    if (nhwc) { ci = i % c; ox = (i / c) % ow; oy = (i / (c * ow)) % oh; ni = i / (c * ow * oh); }
    else { ox = i % ow; oy = (i / ow) % oh; ci = (i / (ow * oh)) % c; ni = i / (ow * oh * c); }
    int64_t y0, y1, x0, x1; float fy, fx;
    ac_coord(oy, h, oh, y0, y1, fy);
    ac_coord(ox, w, ow, x0, x1, fx);
    auto at = [&](int64_t yy, int64_t xx) -> float {
      return nhwc ? to_f32(x[((ni * h + yy) * w + xx) * c + ci])
                  : to_f32(x[((ni * c + ci) * h + yy) * w + xx]);
    };
    const float v00 = at(y0, x0), v01 = at(y0, x1), v10 = at(y1, x0), v11 = at(y1, x1);
    const float v = bilerp(v00, v01, v10, v11, fx, fy);
    float out = v;
    if (add) out += to_f32(y[i]);
    y[i] = from_f32<TO>(out);
  }
}

// NHWC with c % 8 == 0: one thread per (output pixel, 8 channels), 16-B (bf16) loads/stores.
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
resize_nhwc8_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n, int c, int h, int w,
                    int oh, int ow, int add) {
  const int cg8 = c / 8;
  const int64_t total = n * oh * ow * cg8;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int cg = (int)(i % cg8);
    const int64_t pix = i / cg8;
    const int ox = (int)(pix % ow);
    const int64_t t = pix / ow;
    const int oy = (int)(t % oh);
    const int64_t ni = t / oh;
    int64_t y0, y1, x0, x1;
    float fy, fx;
    ac_coord(oy, h, oh, y0, y1, fy);
    ac_coord(ox, w, ow, x0, x1, fx);
    const TI* b = x + ni * h * w * c + cg * 8;
    float v00[8], v01[8], v10[8], v11[8];
    load8(b + (y0 * w + x0) * c, v00);
    load8(b + (y0 * w + x1) * c, v01);
    load8(b + (y1 * w + x0) * c, v10);
    load8(b + (y1 * w + x1) * c, v11);
    float o[8];
    TO* yo = y + pix * c + cg * 8;
    if (add) load8(yo, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = bilerp(v00[e], v01[e], v10[e], v11[e], fx, fy);
      o[e] = add ? o[e] + v : v;
    }
    store8(yo, o);
  }
}

// Row-blocked variant (c % 8 == 0, 16-B aligned, n * oh < 2^31): output row (ni, oy) per
// RowBlock row, its y interpolation computed once, 8 channels per item.
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
resize_nhwc8_rows_kernel(const TI* __restrict__ x, TO* __restrict__ y, RowBlock rb, int c, int h, int w,
                         int oh, int ow, int add, int ldy) {
  const int rl = threadIdx.x / rb.R;
  const int row = blockIdx.x * rb.RB + rl;
  if (rl >= rb.RB || row >= rb.nrows) return;
  const int ni = row / oh, oy = row - ni * oh;
  int64_t y0, y1, x0, x1;
  float fy, fx;
  ac_coord(oy, h, oh, y0, y1, fy);
  const int cg8 = c / 8;
  const TI* b0 = x + ((int64_t)ni * h + y0) * w * c;
  const TI* b1 = x + ((int64_t)ni * h + y1) * w * c;
  TO* yrow = y + (int64_t)row * ow * ldy;
  const int step = rb.R > 256 ? 256 : rb.R;
  for (int it = threadIdx.x - rl * rb.R; it < rb.R; it += step) {
    const int ox = it / cg8, cg = it - ox * cg8;
    ac_coord(ox, w, ow, x0, x1, fx);
    float v00[8], v01[8], v10[8], v11[8];
    load8(b0 + x0 * c + cg * 8, v00);
    load8(b0 + x1 * c + cg * 8, v01);
    load8(b1 + x0 * c + cg * 8, v10);
    load8(b1 + x1 * c + cg * 8, v11);
    float o[8];
    TO* yo = yrow + (int64_t)ox * ldy + cg * 8;
    if (add) load8(yo, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = bilerp(v00[e], v01[e], v10[e], v11[e], fx, fy);
      o[e] = add ? o[e] + v : v;
    }
    store8(yo, o);
  }
}

// Small images (the fine ShallowEncoder's 16 x 16 -> 31 x 31 patch maps, 65536 of them): one
// workgroup per image stages the whole input image in LDS (<= 32 KiB) and writes the output
// image as one contiguous run of 16-B stores; the row kernel re-read each input pixel from L2 for
// every output it touches (4 x 16 B of L2 reads per 16 B written).
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
resize_nhwc8_img_kernel(const TI* __restrict__ x, TO* __restrict__ y, int c, int h, int w, int oh, int ow,
                        int add) {
  extern __shared__ uint4 img_lds[];
  const TI* img = reinterpret_cast<const TI*>(img_lds);
  const int64_t ni = blockIdx.x;
  const int nvec = (int)((int64_t)h * w * c * (int)sizeof(TI) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(x + ni * h * w * c);
  for (int i = threadIdx.x; i < nvec; i += 256) img_lds[i] = src[i];
  __syncthreads();
  const int cg8 = c / 8, items = oh * ow * cg8;
  TO* yo = y + ni * oh * ow * c;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int pix = it / cg8, cg = it - pix * cg8;
    const int oy = pix / ow, ox = pix - oy * ow;
    int64_t y0, y1, x0, x1;
    float fy, fx;
    ac_coord(oy, h, oh, y0, y1, fy);
    ac_coord(ox, w, ow, x0, x1, fx);
    float v00[8], v01[8], v10[8], v11[8];
    load8(img + ((int)y0 * w + (int)x0) * c + cg * 8, v00);
    load8(img + ((int)y0 * w + (int)x1) * c + cg * 8, v01);
    load8(img + ((int)y1 * w + (int)x0) * c + cg * 8, v10);
    load8(img + ((int)y1 * w + (int)x1) * c + cg * 8, v11);
    float o[8];
    if (add) load8(yo + (int64_t)it * 8, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = bilerp(v00[e], v01[e], v10[e], v11[e], fx, fy);
      o[e] = add ? o[e] + v : v;
    }
    store8(yo + (int64_t)it * 8, o);
  }
}

// resize_nhwc8_img_kernel with the 2 x 2 average pool of its output written by the same workgroup
// (the fine ShallowEncoder's 31 x 31 maps and the fine correlation pyramid's level 1, refine_track.py
// -> blocks.py:371 F.avg_pool2d(fmaps, 2, stride=2)). A lane owns one output column x (8 channels) of
// a row pair (2 py, 2 py + 1): its two pixels are stored by consecutive lanes as contiguous runs, and
// the pool value of columns (x, x + 1) is summed on the even lane from the stored (rounded) values,
// the odd lane's two by a shuffle, in avgpool2_rows_kernel's order ((a + b) + c) + d -- so y and the
// pool equal resize followed by avg_pool2d bit for bit without reading y back. A row pair's lanes
// are padded to an even column count so a column pair never straddles a wave (64 % (2 * c / 8) == 0:
// c in {8, 16, 32, 64, 128, 256}); the odd last row of y (floor pooling drops it) is written after.
// (workgroup body) y / pool of image ni from the staged input image `img` in LDS
// (and, when pl != nullptr, a copy of the image's pool in LDS, [oh / 2][ow / 2][c], for a second level)
template <typename TI, typename TO, bool NTS = false>
__device__ __forceinline__ void resize_pool_body(const TI* img, TO* __restrict__ y, TO* __restrict__ pool, int64_t ni,
                                                 int c, int h, int w, int oh, int ow, TO* pl = nullptr) {
  const int cg8 = c / 8, ph = oh / 2, pw = ow / 2;
  const int rpi = ((ow + 1) / 2) * 2 * cg8;  // lanes per row pair (even column count)
  const int lane = threadIdx.x & 63;
  TO* yo = y + ni * oh * ow * c;
  TO* po = pool + ni * ph * pw * c;
  auto put = [&](TO* p, const float (&o)[8]) {
    if constexpr (NTS) store8_nt(p, o);
    else store8(p, o);
  };
  auto pixel = [&](int oy, int ox, int cg, float (&o)[8]) {
    int64_t y0, y1, x0, x1;
    float fy, fx;
    ac_coord(oy, h, oh, y0, y1, fy);
    ac_coord(ox, w, ow, x0, x1, fx);
    float v00[8], v01[8], v10[8], v11[8];
    load8(img + ((int)y0 * w + (int)x0) * c + cg * 8, v00);
    load8(img + ((int)y0 * w + (int)x1) * c + cg * 8, v01);
    load8(img + ((int)y1 * w + (int)x0) * c + cg * 8, v10);
    load8(img + ((int)y1 * w + (int)x1) * c + cg * 8, v11);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bilerp(v00[e], v01[e], v10[e], v11[e], fx, fy);
  };
  const int items = ph * rpi;
  // whole waves per trip (the shuffles need every lane of the wave)
  for (int it0 = threadIdx.x - lane; it0 < items; it0 += 256) {
    const int it = it0 + lane;
    const int py = it / rpi, r = it - py * rpi, ox = r / cg8, cg = r - ox * cg8;
    const bool live = it < items && ox < ow;
    float a[8], cq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = cq[e] = 0.f;
    if (live) {
      pixel(2 * py, ox, cg, a);
      pixel(2 * py + 1, ox, cg, cq);
      put(yo + ((int64_t)(2 * py) * ow + ox) * c + cg * 8, a);
      put(yo + ((int64_t)(2 * py + 1) * ow + ox) * c + cg * 8, cq);
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // the values y holds
        a[e] = to_f32(from_f32<TO>(a[e]));
        cq[e] = to_f32(from_f32<TO>(cq[e]));
      }
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float b = __shfl_down(a[e], cg8, 64), d = __shfl_down(cq[e], cg8, 64);
      o[e] = (a[e] + b + cq[e] + d) * 0.25f;
    }
    if (live && (ox & 1) == 0 && ox / 2 < pw) {
      put(po + ((int64_t)py * pw + ox / 2) * c + cg * 8, o);
      if (pl != nullptr) store8(pl + (py * pw + ox / 2) * c + cg * 8, o);
    }
  }
  if (oh & 1) {  // the last row of y (no pool)
    for (int it = threadIdx.x; it < ow * cg8; it += 256) {
      const int ox = it / cg8, cg = it - ox * cg8;
      float o[8];
      pixel(oh - 1, ox, cg, o);
      put(yo + ((int64_t)(oh - 1) * ow + ox) * c + cg * 8, o);
    }
  }
}

template <typename TI, typename TO, bool NTS>
__global__ void __launch_bounds__(256)
resize_pool_nhwc8_img_kernel(const TI* __restrict__ x, TO* __restrict__ y, TO* __restrict__ pool, int c, int h,
                             int w, int oh, int ow) {
  extern __shared__ uint4 img_lds[];
  const int64_t ni = blockIdx.x;
  const int nvec = (int)((int64_t)h * w * c * (int)sizeof(TI) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(x + ni * h * w * c);
  for (int i = threadIdx.x; i < nvec; i += 256) img_lds[i] = src[i];
  __syncthreads();
  resize_pool_body<TI, TO, NTS>(reinterpret_cast<const TI*>(img_lds), y, pool, ni, c, h, w, oh, ow);
}

// The fine ShallowEncoder's tail in one pass per patch (blocks.py:97-110 with refine_track's pool):
//   x1 = x + up(u1) (rounded), x2 = x1 + up(u2) (rounded)  -- the two resize-and-add steps, optional
//   t = x2 + conv2(x2) (1x1, C x C, bias: the skinny GEMM's MFMA on the same operands; its epilogue at
//       alpha = beta = 1 is two exact-product fmas, i.e. the adds (acc + bias) + x2, rounded to bf16)
//   y = resize(t), pool = avgpool2(y)  (as resize_pool_nhwc8_img_kernel), pool2 = avgpool2(pool) (optional:
//       the fine correlation pyramid's level 2, base_track_predictor.py:83 / blocks.py:371)
// x2 and t stay in LDS (one image buffer, t written over x2): neither the [n, h, w, C] sums nor the
// conv2 output reach HBM (two resize-add passes and one 16.7M-row GEMM per step fewer). bf16,
// C = 16 x NT16 (one 32-deep k step per 32 input channels).
template <int NT16, bool NTS>
__global__ void __launch_bounds__(256)
conv1x1_resize_pool_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ u1, int h1, int w1,
                           const __bf16* __restrict__ u2, int h2, int w2, const __bf16* __restrict__ wt,
                           const float* __restrict__ bias, __bf16* __restrict__ y, __bf16* __restrict__ pool,
                           __bf16* __restrict__ pool2, int h, int w, int oh, int ow) {
  constexpr int C = NT16 * 16, KC = C / 32, CG8 = C / 8;
  // LDS: x (becomes x2, then t in place) | u1 | u2 | the pool's copy (pool2 only)
  extern __shared__ uint4 img_lds[];
  const int64_t ni = blockIdx.x;
  const int hw = h * w;
  const int nvec = hw * C * 2 / 16, n1 = u1 != nullptr ? h1 * w1 * C * 2 / 16 : 0,
            n2 = u2 != nullptr ? h2 * w2 * C * 2 / 16 : 0;
  {  // every global load of the workgroup's inputs issued before any wait
    const uint4* src = reinterpret_cast<const uint4*>(x + ni * hw * C);
    for (int i = threadIdx.x; i < nvec; i += 256) img_lds[i] = src[i];
    if (n1) {
      const uint4* s1 = reinterpret_cast<const uint4*>(u1 + ni * h1 * w1 * C);
      for (int i = threadIdx.x; i < n1; i += 256) img_lds[nvec + i] = s1[i];
    }
    if (n2) {
      const uint4* s2 = reinterpret_cast<const uint4*>(u2 + ni * h2 * w2 * C);
      for (int i = threadIdx.x; i < n2; i += 256) img_lds[nvec + n1 + i] = s2[i];
    }
  }
  __bf16* xs = reinterpret_cast<__bf16*>(img_lds);
  const __bf16* us1 = reinterpret_cast<const __bf16*>(img_lds + nvec);
  const __bf16* us2 = reinterpret_cast<const __bf16*>(img_lds + nvec + n1);
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  bf16x8 bf[NT16][KC];
#pragma unroll
  for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
    for (int k = 0; k < KC; ++k) bf[nt][k] = *reinterpret_cast<const bf16x8*>(wt + (nt * 16 + li) * C + 32 * k + 8 * g);
  float b4[NT16][4];
#pragma unroll
  for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) b4[nt][r] = bias != nullptr ? bias[nt * 16 + 4 * g + r] : 0.f;
  __syncthreads();
  // x2 = round(round(x + up(u1)) + up(u2)), in place (each item owns its 8 channels of one pixel)
  auto up = [&](const __bf16* ub, int hu, int wu, int oy, int ox, int cg, float (&o)[8]) {
    int64_t y0, y1, x0, x1;
    float fy, fx;
    ac_coord(oy, hu, h, y0, y1, fy);
    ac_coord(ox, wu, w, x0, x1, fx);
    float v00[8], v01[8], v10[8], v11[8];
    load8(ub + ((int)y0 * wu + (int)x0) * C + cg * 8, v00);
    load8(ub + ((int)y0 * wu + (int)x1) * C + cg * 8, v01);
    load8(ub + ((int)y1 * wu + (int)x0) * C + cg * 8, v10);
    load8(ub + ((int)y1 * wu + (int)x1) * C + cg * 8, v11);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bilerp(v00[e], v01[e], v10[e], v11[e], fx, fy);
  };
  if (n1 || n2) {
    for (int it = threadIdx.x; it < hw * CG8; it += 256) {
      const int pix = it / CG8, cg = it - pix * CG8;
      const int oy = pix / w, ox = pix - oy * w;
      float o[8], v[8];
      load8(xs + pix * C + cg * 8, o);
      if (n1) {
        up(us1, h1, w1, oy, ox, cg, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = to_f32(from_f32<__bf16>(o[e] + v[e]));  // the first add's stored value
      }
      if (n2) {
        up(us2, h2, w2, oy, ox, cg, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = o[e] + v[e];
      }
      store8(xs + pix * C + cg * 8, o);
    }
    __syncthreads();
  }
  // t = x2 + conv2(x2), written over x2: a wave reads its 16 rows (fragments, residual) before it
  // writes them (the writes depend on the MFMA that consumed the reads), and no other wave reads them
  for (int m0 = wv * 16; m0 < hw; m0 += 64) {  // 16 pixels per wave step (hw % 16 == 0, host-checked)
    const int m = m0 + li;
    f32x4 acc[NT16];
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(xs + m * C + 32 * k + 8 * g);
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[nt][k], a, acc[nt], 0, 0, 0);
    }
    float rr[NT16][4];
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) load4(xs + m * C + nt * 16 + 4 * g, rr[nt]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every read of these rows done before the writes
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[nt][r] + b4[nt][r];  // = fma(alpha = 1, acc, bias) exactly
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = rr[nt][r] + v[r];  // = fma(beta = 1, resid, v) exactly
      store4(xs + m * C + nt * 16 + 4 * g, v);
    }
  }
  __syncthreads();
  __bf16* pl = pool2 != nullptr ? reinterpret_cast<__bf16*>(img_lds + nvec + n1 + n2) : nullptr;
  resize_pool_body<__bf16, __bf16, NTS>(xs, y, pool, ni, C, h, w, oh, ow, pl);
  if (pool2 == nullptr) return;
  // the second pyramid level: avgpool2 of the pool, from its LDS copy (avgpool2_rows_kernel's order)
  __syncthreads();
  const int ph = oh / 2, pw = ow / 2, qh = ph / 2, qw = pw / 2;
  __bf16* qo = pool2 + ni * qh * qw * C;
  for (int it = threadIdx.x; it < qh * qw * CG8; it += 256) {
    const int q = it / CG8, cg = it - q * CG8, qy = q / qw, qx = q - qy * qw;
    const __bf16* r0 = pl + ((2 * qy) * pw + 2 * qx) * C + cg * 8;
    const __bf16* r1 = r0 + pw * C;
    float a[8], bq[8], cq[8], d[8], o[8];
    load8(r0, a);
    load8(r0 + C, bq);
    load8(r1, cq);
    load8(r1 + C, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (a[e] + bq[e] + cq[e] + d[e]) * 0.25f;
    if constexpr (NTS) store8_nt(qo + (int64_t)q * C + cg * 8, o);
    else store8(qo + (int64_t)q * C + cg * 8, o);
  }
}

inline unsigned g1d(int64_t n) {
  int64_t g = cdiv(n, 256);
  return (unsigned)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_im2col_nhwc(int dtype_in, int dtype_out, const void* x, void* cols, int64_t n,
                                 int64_t h, int64_t w, int64_t c, int kh, int kw, int stride,
                                 int pad, int64_t oh, int64_t ow, int64_t ldc, void* stream) {
  COMET_CHECK_ARG(x && cols && n > 0 && c > 0 && kh > 0 && kw > 0 && stride > 0, "comet_im2col_nhwc: bad args");
  hipStream_t s = as_stream(stream);
  COMET_CHECK_ARG(ldc >= (int64_t)kh * kw * c, "comet_im2col_nhwc: ldc < kh*kw*c");
  const unsigned g = g1d(n * oh * ow * ldc);
#define IC(TI, TO) hipLaunchKernelGGL((im2col_nhwc_kernel<TI, TO>), dim3(g), dim3(256), 0, s, (const TI*)x, (TO*)cols, n, h, w, c, kh, kw, stride, pad, oh, ow, ldc)
  if (dtype_in == COMET_F32 && dtype_out == COMET_F32) IC(float, float);
  else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) IC(float, __bf16);
  else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) IC(__bf16, __bf16);
  else IC(__bf16, float);
#undef IC
  COMET_CHECK_LAUNCH("comet_im2col_nhwc");
  return COMET_OK;
}

extern "C" int comet_resize_bilinear(int dtype_in, int dtype_out, int nhwc, const void* x, void* y,
                                     int64_t n, int64_t c, int64_t h, int64_t w, int64_t oh,
                                     int64_t ow, int add, void* stream) {
  COMET_CHECK_ARG(x && y && n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0, "comet_resize_bilinear: bad args");
  hipStream_t s = as_stream(stream);
  const int esz = dtype_in == COMET_F32 ? 4 : 2;
  if (nhwc && c % 8 == 0 && ((uintptr_t)x | (uintptr_t)y) % 16 == 0 && h * w * c * esz <= 32768 &&
      oh * ow * c < (1ll << 30) && n < (1ll << 31) && getenv("COMET_RESIZE_ROWS") == nullptr) {
    const size_t lds = (size_t)(h * w * c * esz);
#define RSI(TI, TO) hipLaunchKernelGGL((resize_nhwc8_img_kernel<TI, TO>), dim3((unsigned)n), dim3(256), lds, s, (const TI*)x, (TO*)y, (int)c, (int)h, (int)w, (int)oh, (int)ow, add)
    if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RSI(float, float);
    else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RSI(float, __bf16);
    else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RSI(__bf16, __bf16);
    else RSI(__bf16, float);
#undef RSI
    COMET_CHECK_LAUNCH("comet_resize_bilinear");
    return COMET_OK;
  }
  if (nhwc && c % 8 == 0 && ((uintptr_t)x | (uintptr_t)y) % 32 == 0 && n * oh < (1ll << 31) &&
      ow * (c / 8) < (1ll << 24) && h < (1 << 30) && w < (1 << 30) && getenv("COMET_RESIZE_FLAT") == nullptr) {
    const RowBlock rb = make_rowblock(n * oh, ow * (c / 8));
    const unsigned gr = (unsigned)cdiv(rb.nrows, rb.RB);
#define RSR(TI, TO) hipLaunchKernelGGL((resize_nhwc8_rows_kernel<TI, TO>), dim3(gr), dim3(256), 0, s, (const TI*)x, (TO*)y, rb, (int)c, (int)h, (int)w, (int)oh, (int)ow, add, (int)c)
    if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RSR(float, float);
    else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RSR(float, __bf16);
    else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RSR(__bf16, __bf16);
    else RSR(__bf16, float);
#undef RSR
    COMET_CHECK_LAUNCH("comet_resize_bilinear");
    return COMET_OK;
  }
  if (nhwc && c % 8 == 0 && ((uintptr_t)x | (uintptr_t)y) % 32 == 0 && h < (1 << 30) && w < (1 << 30)) {
    const unsigned g8 = g1d(n * oh * ow * (c / 8));
#define RS8(TI, TO) hipLaunchKernelGGL((resize_nhwc8_kernel<TI, TO>), dim3(g8), dim3(256), 0, s, (const TI*)x, (TO*)y, n, (int)c, (int)h, (int)w, (int)oh, (int)ow, add)
    if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RS8(float, float);
    else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RS8(float, __bf16);
    else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RS8(__bf16, __bf16);
    else RS8(__bf16, float);
#undef RS8
    COMET_CHECK_LAUNCH("comet_resize_bilinear");
    return COMET_OK;
  }
  const unsigned g = g1d(n * c * oh * ow);
#define RS(TI, TO) hipLaunchKernelGGL((resize_kernel<TI, TO>), dim3(g), dim3(256), 0, s, (const TI*)x, (TO*)y, nhwc, n, c, h, w, oh, ow, add)
  if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RS(float, float);
  else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RS(float, __bf16);
  else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RS(__bf16, __bf16);
  else RS(__bf16, float);
#undef RS
  COMET_CHECK_LAUNCH("comet_resize_bilinear");
  return COMET_OK;
}

// y / pool (/ pool2) of the resize + pool kernels written with streaming stores: write-once maps that no
// later kernel finds in L2 (1 % faster, profiles/r06_nt); COMET_RSP_NT=0 turns them off (read per call)
static bool rsp_streaming_stores() {
  const char* e = std::getenv("COMET_RSP_NT");
  return e == nullptr || e[0] != '0';
}

extern "C" int comet_resize_bilinear_pool_nhwc(int dtype_in, int dtype_out, const void* x, void* y, void* pool,
                                               int64_t n, int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow,
                                               void* stream) {
  COMET_CHECK_ARG(x && y && pool && n > 0 && c > 0 && h > 0 && w > 0 && oh >= 2 && ow >= 2,
                  "comet_resize_bilinear_pool_nhwc: bad args");
  const int esz = dtype_in == COMET_F32 ? 4 : 2;
  COMET_CHECK_ARG(c % 8 == 0 && c <= 256 && 64 % (2 * (c / 8)) == 0 &&
                      ((uintptr_t)x | (uintptr_t)y | (uintptr_t)pool) % 16 == 0 && h * w * c * esz <= 32768 &&
                      oh * ow * c < (1ll << 30) && n < (1ll << 31),
                  "comet_resize_bilinear_pool_nhwc: needs c in {8, 16, 32, 64, 128, 256}, 16-B aligned tensors and "
                  "an input image of at most 32 KiB");
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)(h * w * c * esz);
  const bool nts = rsp_streaming_stores();
#define RSP(TI, TO)                                                                                            \
  if (nts)                                                                                                     \
    hipLaunchKernelGGL((resize_pool_nhwc8_img_kernel<TI, TO, true>), dim3((unsigned)n), dim3(256), lds, s,     \
                       (const TI*)x, (TO*)y, (TO*)pool, (int)c, (int)h, (int)w, (int)oh, (int)ow);             \
  else                                                                                                         \
    hipLaunchKernelGGL((resize_pool_nhwc8_img_kernel<TI, TO, false>), dim3((unsigned)n), dim3(256), lds, s,    \
                       (const TI*)x, (TO*)y, (TO*)pool, (int)c, (int)h, (int)w, (int)oh, (int)ow)
  if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RSP(float, float);
  else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RSP(float, __bf16);
  else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RSP(__bf16, __bf16);
  else RSP(__bf16, float);
#undef RSP
  COMET_CHECK_LAUNCH("comet_resize_bilinear_pool_nhwc");
  return COMET_OK;
}

extern "C" int comet_conv1x1_resize_pool_nhwc(const void* x, const void* up1, int64_t h1, int64_t w1, const void* up2,
                                              int64_t h2, int64_t w2, const void* weight, const float* bias, void* y,
                                              void* pool, void* pool2, int64_t n, int64_t c, int64_t h, int64_t w,
                                              int64_t oh, int64_t ow, void* stream) {
  COMET_CHECK_ARG(x && weight && y && pool && n > 0 && h > 0 && w > 0 && oh >= 2 && ow >= 2,
                  "comet_conv1x1_resize_pool_nhwc: bad args");
  const int64_t lds_b = (h * w + (up1 ? h1 * w1 : 0) + (up2 ? h2 * w2 : 0)) * c * 2 +
                        (pool2 != nullptr ? (oh / 2) * (ow / 2) * c * 2 : 0);
  COMET_CHECK_ARG((c == 32 || c == 64) && (h * w) % 16 == 0 && lds_b <= 65536 && n < (1ll << 31) &&
                      oh * ow * c < (1ll << 30) && (pool2 == nullptr || (oh >= 4 && ow >= 4)) &&
                      ((uintptr_t)x | (uintptr_t)up1 | (uintptr_t)up2 | (uintptr_t)weight | (uintptr_t)y |
                       (uintptr_t)pool | (uintptr_t)pool2) % 16 == 0,
                  "comet_conv1x1_resize_pool_nhwc: needs c in {32, 64}, h * w % 16 == 0, the inputs (and the pool "
                  "copy) within 64 KiB of LDS and 16-B aligned tensors");
  COMET_CHECK_ARG((up1 == nullptr || (h1 > 0 && w1 > 0)) && (up2 == nullptr || (h2 > 0 && w2 > 0)),
                  "comet_conv1x1_resize_pool_nhwc: bad up-sampled input size");
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)lds_b;
  const bool nts = rsp_streaming_stores();
#define C1P(NT, NTS)                                                                                              \
  hipLaunchKernelGGL((conv1x1_resize_pool_kernel<NT, NTS>), dim3((unsigned)n), dim3(256), lds, s, (const __bf16*)x, \
                     (const __bf16*)up1, (int)h1, (int)w1, (const __bf16*)up2, (int)h2, (int)w2,                     \
                     (const __bf16*)weight, bias, (__bf16*)y, (__bf16*)pool, (__bf16*)pool2, (int)h, (int)w, (int)oh, \
                     (int)ow)
  if (c == 32 && nts) C1P(2, true);
  else if (c == 32) C1P(2, false);
  else if (nts) C1P(4, true);
  else C1P(4, false);
#undef C1P
  COMET_CHECK_LAUNCH("comet_conv1x1_resize_pool_nhwc");
  return COMET_OK;
}

extern "C" int comet_resize_bilinear_nhwc_into(int dtype_in, int dtype_out, const void* x, void* y, int64_t n,
                                               int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow,
                                               int64_t ldy, int add, void* stream) {
  COMET_CHECK_ARG(x && y && n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0, "comet_resize_bilinear_nhwc_into: bad args");
  COMET_CHECK_ARG(c % 8 == 0 && ldy % 8 == 0 && ldy >= c && ((uintptr_t)x | (uintptr_t)y) % 16 == 0,
                  "comet_resize_bilinear_nhwc_into: c, ldy multiples of 8, ldy >= c, 16-B aligned");
  COMET_CHECK_ARG(n * oh < (1ll << 31) && ow * (c / 8) < (1ll << 24) && ldy < (1ll << 24) && h < (1 << 30) && w < (1 << 30),
                  "comet_resize_bilinear_nhwc_into: sizes out of range");
  hipStream_t s = as_stream(stream);
  const RowBlock rb = make_rowblock(n * oh, ow * (c / 8));
  const unsigned gr = (unsigned)cdiv(rb.nrows, rb.RB);
#define RSR(TI, TO) hipLaunchKernelGGL((resize_nhwc8_rows_kernel<TI, TO>), dim3(gr), dim3(256), 0, s, (const TI*)x, (TO*)y, rb, (int)c, (int)h, (int)w, (int)oh, (int)ow, add, (int)ldy)
  if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RSR(float, float);
  else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RSR(float, __bf16);
  else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RSR(__bf16, __bf16);
  else RSR(__bf16, float);
#undef RSR
  COMET_CHECK_LAUNCH("comet_resize_bilinear_nhwc_into");
  return COMET_OK;
}
