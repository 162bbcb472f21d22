// Row LayerNorm forward/backward (nn.LayerNorm, GroupNorm(1, C) on token rows) and
// InstanceNorm2d on channels-last activations.
//
// Reference sites: modules.py:261-317 (non-affine eps 1e-6 / affine eps 1e-5),
// camera_predictor10.py:75-87 (TrajectoryEncoder LNs), base_track_predictor.py:81,238
// (GroupNorm(1, latent)), modules.py:86-90 + blocks.py:37-38,130-132 (InstanceNorm2d).
//
// One wave per row; the row (<= 1024 columns) is held in registers, mean and variance are
// two exact passes over the registers (wave shuffles), no LDS.
#include <cstdlib>

#include "common.hpp"

namespace comet {
namespace {

constexpr int LN_MAXV = 16;  // cols <= 64*16 = 1024

template <typename TX, typename TY>
__global__ void __launch_bounds__(256)
ln_fwd_kernel(const TX* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
              TY* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
              int64_t rows, int cols, int64_t ldx, int64_t ldy, float eps, int relu) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TX* xr = x + row * ldx;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    v[i] = c < cols ? to_f32(xr[c]) : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    const float d = c < cols ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float var = wave_sum(q) / cols;
  const float rstd = rsqrtf(var + eps);
  TY* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < cols) {
      float o = (v[i] - mean) * rstd;
      if (w) o = o * w[c];
      if (b) o = o + b[c];
      if (relu) o = o > 0.f ? o : 0.f;
      yr[c] = from_f32<TY>(o);
    }
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// Each block: 256 threads, ROWS_PER_BLOCK rows (4 waves x RPW rows). Weight/bias grads are
// kept per lane in registers, reduced across the 4 waves in LDS, one atomic per column/block.
constexpr int LN_RPW = 16;

template <typename TX, typename TD>
__global__ void __launch_bounds__(256)
ln_bwd_kernel(const TX* __restrict__ x, const TD* __restrict__ dy, const float* __restrict__ mean,
              const float* __restrict__ rstd, const float* __restrict__ w, float* __restrict__ dx,
              float* __restrict__ dw, float* __restrict__ db, int64_t rows, int cols, int accum) {
  __shared__ float red[2][4][1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gw[LN_MAXV], gb[LN_MAXV], wv[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    gw[i] = 0.f; gb[i] = 0.f;
    const int c = lane + i * 64;
    wv[i] = (w && c < cols) ? w[c] : 1.f;
  }
  const int64_t rbase = ((int64_t)blockIdx.x * 4 + wid) * LN_RPW;
  for (int rr = 0; rr < LN_RPW; ++rr) {
    const int64_t row = rbase + rr;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    float xh[LN_MAXV], g[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + i * 64;
      if (c < cols) {
        xh[i] = (to_f32(x[row * cols + c]) - mu) * rs;
        const float d = to_f32(dy[row * cols + c]);
        gw[i] += d * xh[i];
        gb[i] += d;
        g[i] = d * wv[i];
      } else {
        xh[i] = 0.f; g[i] = 0.f;
      }
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + i * 64;
      if (c < cols) {
        const float o = rs * (g[i] - s1 - xh[i] * s2);
        float* p = dx + row * cols + c;
        *p = accum ? *p + o : o;
      }
    }
  }
  if (!dw && !db) return;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < cols) { red[0][wid][c] = gw[i]; red[1][wid][c] = gb[i]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    if (dw) atomicAdd(dw + c, red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c]);
    if (db) atomicAdd(db + c, red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c]);
  }
}

// ---- vectorised LayerNorm (cols % 8 == 0, <= 1024, 32-B aligned rows) ------------------
// One wave per row, lane j owns columns 8j..8j+7 (and 512 + 8j.. when NV == 2): one 16-B (bf16)
// or 2 x 16-B (f32) access per lane per row. Forward may write a second copy of y (y2, bf16) for
// the GEMM that consumes it while y (f32) feeds a residual; backward sums two incoming
// gradients (dy f32/bf16 + dy2 bf16) and writes dx in f32 or bf16.
// Chunk CH = 4 (any f32 operand: 16-B f32 accesses) or 8 (all bf16: 16-B accesses); lane j owns
// chunks j, j + 64, ... (NK per lane): every wave-wide access is one contiguous run of the row.
template <typename TX, typename TY, int CH, int NK>
__global__ void __launch_bounds__(256)
ln_fwd_vec_kernel(const TX* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                  TY* __restrict__ y, __bf16* __restrict__ y2, float* __restrict__ mean_out,
                  float* __restrict__ rstd_out, int64_t rows, int cols, int64_t ldx, int64_t ldy,
                  int64_t ldy2, float eps, int relu) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[NK][CH];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = (lane + 64 * k) * CH;
    if (c0 < cols) {
      loadn<CH>(x + row * ldx + c0, v[k]);
    } else {
#pragma unroll
      for (int e = 0; e < CH; ++e) v[k][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < CH; ++e) s += v[k][e];
  }
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = (lane + 64 * k) * CH;
    if (c0 < cols)
#pragma unroll
      for (int e = 0; e < CH; ++e) { const float d = v[k][e] - mean; q += d * d; }
  }
  const float var = wave_sum(q) / cols;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = (lane + 64 * k) * CH;
    if (c0 >= cols) continue;
    float o[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      float t = (v[k][e] - mean) * rstd;
      if (w) t = t * w[c0 + e];
      if (b) t = t + b[c0 + e];
      if (relu) t = t > 0.f ? t : 0.f;
      o[e] = t;
    }
    if (y) storen<CH>(y + row * ldy + c0, o);
    if (y2) storen<CH>(y2 + row * ldy2 + c0, o);
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// Narrow rows (cols <= 8 x CH: the tracker's GroupNorm(1, 32) rows): RPW rows per wave, 64 / RPW
// lanes per row, one CH-chunk per lane. The sums are the segmented tail of wave_sum's
// butterfly (offsets 32 / RPW .. 1); in the one-row-per-wave kernel the larger offsets only add the
// idle lanes' zeros, so mean, variance and outputs are bit-identical to ln_fwd_vec_kernel.
template <typename TX, typename TY, int CH, int RPW>
__global__ void __launch_bounds__(256)
ln_fwd_narrow_kernel(const TX* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                     TY* __restrict__ y, __bf16* __restrict__ y2, float* __restrict__ mean_out,
                     float* __restrict__ rstd_out, int64_t rows, int cols, int64_t ldx, int64_t ldy,
                     int64_t ldy2, float eps, int relu) {
  constexpr int LPR = 64 / RPW;
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const int c0 = (lane % LPR) * CH;
  const bool live = row < rows && c0 < cols;
  float v[CH];
#pragma unroll
  for (int e = 0; e < CH; ++e) v[e] = 0.f;
  if (live) loadn<CH>(x + row * ldx + c0, v);
  auto seg_sum = [](float t) {
#pragma unroll
    for (int off = LPR / 2; off >= 1; off >>= 1) t += __shfl_xor(t, off, 64);
    return t;
  };
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < CH; ++e) s += v[e];
  const float mean = seg_sum(s) / cols;
  float q = 0.f;
  if (live) {
#pragma unroll
    for (int e = 0; e < CH; ++e) { const float d = v[e] - mean; q += d * d; }
  }
  const float var = seg_sum(q) / cols;
  const float rstd = rsqrtf(var + eps);
  if (!live) return;
  float o[CH];
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    float t = (v[e] - mean) * rstd;
    if (w) t = t * w[c0 + e];
    if (b) t = t + b[c0 + e];
    if (relu) t = t > 0.f ? t : 0.f;
    o[e] = t;
  }
  if (y) storen<CH>(y + row * ldy + c0, o);
  if (y2) storen<CH>(y2 + row * ldy2 + c0, o);
  if (c0 == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// Persistent-row form of ln_fwd_vec_kernel: each wave walks rows wave_id, wave_id + waves, ... and
// issues the next row's loads before reducing / storing the current one (a one-row-per-wave block
// lives mostly in load latency, so the short blocks held the forward near 3.8 TB/s).
template <typename TX, typename TY, int CH, int NK>
__global__ void __launch_bounds__(256)
ln_fwd_rows_kernel(const TX* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                   TY* __restrict__ y, __bf16* __restrict__ y2, float* __restrict__ mean_out,
                   float* __restrict__ rstd_out, int64_t rows, int cols, int64_t ldx, int64_t ldy,
                   int64_t ldy2, float eps, int relu) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float wv[NK][CH], bv[NK][CH];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int c = (lane + 64 * k) * CH + e;
      wv[k][e] = (w && c < cols) ? w[c] : 1.f;
      bv[k][e] = (b && c < cols) ? b[c] : 0.f;
    }
  float v[NK][CH], nx[NK][CH];
  auto load_row = [&](int64_t r, float (&dst)[NK][CH]) {
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (lane + 64 * k) * CH;
      if (c0 < cols) {
        loadn<CH>(x + r * ldx + c0, dst[k]);
      } else {
#pragma unroll
        for (int e = 0; e < CH; ++e) dst[k][e] = 0.f;
      }
    }
  };
  load_row(row, v);
  for (; row < rows; row += nw) {
    const int64_t nrow = row + nw;
    if (nrow < rows) load_row(nrow, nx);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int e = 0; e < CH; ++e) s += v[k][e];
    const float mean = wave_sum(s) / cols;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (lane + 64 * k) * CH;
      if (c0 < cols)
#pragma unroll
        for (int e = 0; e < CH; ++e) { const float d = v[k][e] - mean; q += d * d; }
    }
    const float var = wave_sum(q) / cols;
    const float rstd = rsqrtf(var + eps);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (lane + 64 * k) * CH;
      if (c0 >= cols) continue;
      float o[CH];
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        float t = (v[k][e] - mean) * rstd;
        if (w) t = t * wv[k][e];
        if (b) t = t + bv[k][e];
        if (relu) t = t > 0.f ? t : 0.f;
        o[e] = t;
      }
      if (y) storen<CH>(y + row * ldy + c0, o);
      if (y2) storen<CH>(y2 + row * ldy2 + c0, o);
    }
    if (lane == 0) {
      if (mean_out) mean_out[row] = mean;
      if (rstd_out) rstd_out[row] = rstd;
    }
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int e = 0; e < CH; ++e) v[k][e] = nx[k][e];
  }
}

template <typename TX, typename TD, typename TO, int CH, int NK>
__global__ void __launch_bounds__(256)
ln_bwd_vec_kernel(const TX* __restrict__ x, const TD* __restrict__ dy, const __bf16* __restrict__ dy2,
                  const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ w,
                  TO* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db, int64_t rows, int cols,
                  int accum, const float* __restrict__ dres = nullptr, int rpw = LN_RPW) {
  __shared__ float red[2][4][1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gw[NK][CH], gb[NK][CH], wv[NK][CH];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int c = (lane + 64 * k) * CH + e;
      gw[k][e] = 0.f; gb[k][e] = 0.f;
      wv[k][e] = (w && c < cols) ? w[c] : 1.f;
    }
  const int64_t rbase = ((int64_t)blockIdx.x * 4 + wid) * rpw;
  for (int rr = 0; rr < rpw; ++rr) {
    const int64_t row = rbase + rr;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    float xh[NK][CH], g[NK][CH];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (lane + 64 * k) * CH;
      if (c0 < cols) {
        float xv[CH], d[CH];
        loadn<CH>(x + row * cols + c0, xv);
        loadn<CH>(dy + row * cols + c0, d);
        if (dy2) {
          float d2[CH];
          loadn<CH>(dy2 + row * cols + c0, d2);
#pragma unroll
          for (int e = 0; e < CH; ++e) d[e] += d2[e];
        }
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          xh[k][e] = (xv[e] - mu) * rs;
          gw[k][e] += d[e] * xh[k][e];
          gb[k][e] += d[e];
          g[k][e] = d[e] * wv[k][e];
          s1 += g[k][e];
          s2 += g[k][e] * xh[k][e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < CH; ++e) { xh[k][e] = 0.f; g[k][e] = 0.f; }
      }
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (lane + 64 * k) * CH;
      if (c0 >= cols) continue;
      float o[CH];
#pragma unroll
      for (int e = 0; e < CH; ++e) o[e] = rs * (g[k][e] - s1 - xh[k][e] * s2);
      TO* p = dx + row * cols + c0;
      if (accum) {
        float prev[CH];
        loadn<CH>(p, prev);
#pragma unroll
        for (int e = 0; e < CH; ++e) o[e] += prev[e];
      }
      if (dres) {  // gradient of the residual branch that also reads x (x + f(LN(x)))
        float r[CH];
        loadn<CH>(dres + row * cols + c0, r);
#pragma unroll
        for (int e = 0; e < CH; ++e) o[e] += r[e];
      }
      storen<CH>(p, o);
    }
  }
  if (!dw && !db) return;
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int c = (lane + 64 * k) * CH + e;
      if (c < cols) { red[0][wid][c] = gw[k][e]; red[1][wid][c] = gb[k][e]; }
    }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    if (dw) atomicAdd(dw + c, red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c]);
    if (db) atomicAdd(db + c, red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c]);
  }
}

// InstanceNorm over H*W per (n, c) on NHWC input; one block per (n, 64-channel slab).
// Optional fused residual: res_norm_relu==0: y = relu?(IN(x) + res); the ResidualBlock
// tail relu(x + y) is expressed by the caller.
template <typename T>
__global__ void __launch_bounds__(256)
instnorm_nhwc_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
                     int64_t hw, int c, float eps, int relu, int relu_inner) {
  __shared__ float red_s[4][64], red_q[4][64];
  const int64_t n = blockIdx.x;
  const int c0 = blockIdx.y * 64;
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;  // 4 parts over hw
  const int ch = c0 + cl;
  const bool ok = ch < c;
  const T* xb = x + n * hw * c;
  // pass 1: mean
  float s = 0.f;
  if (ok)
    for (int64_t p = part; p < hw; p += 4) s += to_f32(xb[p * c + ch]);
  red_s[part][cl] = s;
  __syncthreads();
  const float mean = (red_s[0][cl] + red_s[1][cl] + red_s[2][cl] + red_s[3][cl]) / hw;
  // pass 2: variance (biased, as InstanceNorm2d)
  float q = 0.f;
  if (ok)
    for (int64_t p = part; p < hw; p += 4) {
      const float d = to_f32(xb[p * c + ch]) - mean;
      q += d * d;
    }
  red_q[part][cl] = q;
  __syncthreads();
  const float var = (red_q[0][cl] + red_q[1][cl] + red_q[2][cl] + red_q[3][cl]) / hw;
  const float rstd = rsqrtf(var + eps);
  if (!ok) return;
  T* yb = y + n * hw * c;
  const T* rb = res ? res + n * hw * c : nullptr;
  for (int64_t p = part; p < hw; p += 4) {
    float o = (to_f32(xb[p * c + ch]) - mean) * rstd;
    if (relu_inner) o = o > 0.f ? o : 0.f;
    if (rb) o += to_f32(rb[p * c + ch]);
    if (relu) o = o > 0.f ? o : 0.f;
    yb[p * c + ch] = from_f32<T>(o);
  }
}

// ---- InstanceNorm, vectorised (c % 8 == 0) ------------------------------------------------
// Each thread owns 8 channels of one pixel slot; a block covers `chunk` pixels of one image.
// Statistics are shifted sums (shift = the image's first pixel, per channel) so the variance is
// taken about a value near the mean: s1 = sum(x - K), s2 = sum((x - K)^2). Large images split
// over chunks: in_stats_kernel writes per-chunk partials, in_apply_kernel (or the fused kernel for
// a single chunk) combines them and normalises.
struct INGeo { int64_t hw, chunk; int c, chunks; float eps; int relu, relu_inner; };

template <typename T>
__device__ __forceinline__ void in_block_stats(const T* __restrict__ xb, const INGeo& g, int64_t p0,
                                               int64_t p1, float* __restrict__ red, float* out1,
                                               float* out2) {
  const int tpp = g.c / 8, ppp = 256 / tpp;
  const int t = threadIdx.x, cg = t % tpp, slot = t / tpp;
  float s1[8], s2[8], K[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  if (slot < ppp) {
    load8(xb + cg * 8, K);
    for (int64_t p = p0 + slot; p < p1; p += ppp) {
      float v[8];
      load8(xb + p * g.c + cg * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[e] - K[e];
        s1[e] += d;
        s2[e] += d * d;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[slot * g.c + cg * 8 + e] = s1[e];
      red[2048 + slot * g.c + cg * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  for (int ch = t; ch < g.c; ch += 256) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < ppp; ++q) {
      a += red[q * g.c + ch];
      b += red[2048 + q * g.c + ch];
    }
    out1[ch] = a;
    out2[ch] = b;
  }
}

template <typename T>
__device__ __forceinline__ void in_block_apply(const T* __restrict__ xb, const T* __restrict__ rb,
                                               T* __restrict__ yb, const INGeo& g, int64_t p0, int64_t p1,
                                               const float* mean, const float* rstd) {
  const int tpp = g.c / 8, ppp = 256 / tpp;
  const int t = threadIdx.x, cg = t % tpp, slot = t / tpp;
  if (slot >= ppp) return;
  float mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[cg * 8 + e];
    rs[e] = rstd[cg * 8 + e];
  }
  for (int64_t p = p0 + slot; p < p1; p += ppp) {
    float v[8];
    load8(xb + p * g.c + cg * 8, v);
    float r[8];
    if (rb) load8(rb + p * g.c + cg * 8, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float o = (v[e] - mu[e]) * rs[e];
      if (g.relu_inner) o = o > 0.f ? o : 0.f;
      if (rb) o += r[e];
      if (g.relu) o = o > 0.f ? o : 0.f;
      v[e] = o;
    }
    store8(yb + p * g.c + cg * 8, v);
  }
}

// mean / rstd of image n from its first-pixel shift K and the summed shifted moments
template <typename T>
__device__ __forceinline__ void in_finish(const T* __restrict__ xb, const INGeo& g, int ch, float S1,
                                          float S2, float* mean, float* rstd) {
  const float inv = 1.f / (float)g.hw;
  const float m1 = S1 * inv;
  float var = S2 * inv - m1 * m1;
  var = var > 0.f ? var : 0.f;
  mean[ch] = to_f32(xb[ch]) + m1;
  rstd[ch] = rsqrtf(var + g.eps);
}

template <typename T>
__global__ void __launch_bounds__(256)
in_fused_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y, INGeo g) {
  __shared__ float red[4096];
  __shared__ float st[4][256];
  const int64_t n = blockIdx.x;
  const T* xb = x + n * g.hw * g.c;
  in_block_stats(xb, g, 0, g.hw, red, st[0], st[1]);
  __syncthreads();
  for (int ch = threadIdx.x; ch < g.c; ch += 256) in_finish(xb, g, ch, st[0][ch], st[1][ch], st[2], st[3]);
  __syncthreads();
  in_block_apply(xb, res ? res + n * g.hw * g.c : nullptr, y + n * g.hw * g.c, g, 0, g.hw, st[2], st[3]);
}

template <typename T>
__global__ void __launch_bounds__(256)
in_stats_kernel(const T* __restrict__ x, float* __restrict__ part, INGeo g) {
  __shared__ float red[4096];
  const int64_t n = blockIdx.y, k = blockIdx.x;
  const int64_t p0 = k * g.chunk, p1 = p0 + g.chunk < g.hw ? p0 + g.chunk : g.hw;
  float* out = part + (n * g.chunks + k) * 2 * g.c;
  in_block_stats(x + n * g.hw * g.c, g, p0, p1, red, out, out + g.c);
}

template <typename T>
__global__ void __launch_bounds__(256)
in_apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
                const float* __restrict__ part, INGeo g) {
  __shared__ float st[2][256];
  const int64_t n = blockIdx.y, k = blockIdx.x;
  const T* xb = x + n * g.hw * g.c;
  for (int ch = threadIdx.x; ch < g.c; ch += 256) {
    float S1 = 0.f, S2 = 0.f;
    const float* pp = part + n * g.chunks * 2 * g.c;
    for (int q = 0; q < g.chunks; ++q) {
      S1 += pp[q * 2 * g.c + ch];
      S2 += pp[q * 2 * g.c + g.c + ch];
    }
    in_finish(xb, g, ch, S1, S2, st[0], st[1]);
  }
  __syncthreads();
  const int64_t p0 = k * g.chunk, p1 = p0 + g.chunk < g.hw ? p0 + g.chunk : g.hw;
  in_block_apply(xb, res ? res + n * g.hw * g.c : nullptr, y + n * g.hw * g.c, g, p0, p1, st[0], st[1]);
}

// Small bf16 images (the fine ShallowEncoder: 65536 images of 16x16 / 8x8 / 4x4 x 32): one wave
// per image holds the whole image in registers (NP 16-B vectors per lane), so the statistics need
// no LDS / barrier (xor shuffles over the lanes of one channel group) and the apply pass no second
// read; 4 images per workgroup. Same shifted-moment statistics as in_block_stats.
template <int NP>
__global__ void __launch_bounds__(256)
in_wave_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ res, __bf16* __restrict__ y, int64_t n,
               INGeo g) {
  const int lane = threadIdx.x & 63;
  const int64_t img = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (img >= n) return;
  const int tpp = g.c / 8, ppw = 64 / tpp;
  const int cg = lane % tpp, slot = lane / tpp;
  const int hw = (int)g.hw;
  const __bf16* xb = x + img * g.hw * g.c;
  uint4 raw[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int p = slot + k * ppw;
    raw[k] = p < hw ? *reinterpret_cast<const uint4*>(xb + (int64_t)p * g.c + cg * 8) : uint4{0, 0, 0, 0};
  }
  float K[8];
  load8(xb + cg * 8, K);
  auto unpack = [](const uint4& u, float (&v)[8]) {
    v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
    v[4] = bf16_lo(u.z); v[5] = bf16_hi(u.z); v[6] = bf16_lo(u.w); v[7] = bf16_hi(u.w);
  };
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    if (slot + k * ppw >= hw) break;
    float v[8];
    unpack(raw[k], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - K[e];
      s1[e] += d;
      s2[e] += d * d;
    }
  }
  const float inv = 1.f / (float)hw;
  float mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float a = s1[e], b = s2[e];
    for (int off = tpp; off < 64; off <<= 1) {
      a += __shfl_xor(a, off, 64);
      b += __shfl_xor(b, off, 64);
    }
    const float m1 = a * inv;
    float var = b * inv - m1 * m1;
    var = var > 0.f ? var : 0.f;
    mu[e] = K[e] + m1;
    rs[e] = rsqrtf(var + g.eps);
  }
  const __bf16* rb = res ? res + img * g.hw * g.c : nullptr;
  __bf16* yb = y + img * g.hw * g.c;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int p = slot + k * ppw;
    if (p >= hw) break;
    float v[8], r[8];
    unpack(raw[k], v);
    if (rb) load8(rb + (int64_t)p * g.c + cg * 8, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float o = (v[e] - mu[e]) * rs[e];
      if (g.relu_inner) o = o > 0.f ? o : 0.f;
      if (rb) o += r[e];
      if (g.relu) o = o > 0.f ? o : 0.f;
      v[e] = o;
    }
    store8(yb + (int64_t)p * g.c + cg * 8, v);
  }
}

// chunks per image: ~1024 blocks over the launch, >= 4 pixel passes per block
inline int in_chunks(int64_t n, int64_t hw, int64_t c) {
  const int64_t ppp = 256 / (c / 8);
  int64_t want = cdiv(1024, n);
  const int64_t most = hw / (ppp * 4);
  if (want > most) want = most;
  return (int)(want < 1 ? 1 : want);
}

}  // namespace
}  // namespace comet

using namespace comet;

static bool a32(const void* p) { return ((uintptr_t)p % 32) == 0; }

extern "C" int comet_layernorm_fwd(int dtype_x, int dtype_y, const void* x, const float* weight,
                                   const float* bias, void* y, void* y2, float* mean, float* rstd,
                                   int64_t rows, int64_t cols, int64_t ldx, int64_t ldy, int64_t ldy2,
                                   float eps, int relu, void* stream) {
  COMET_CHECK_ARG(cols > 0 && cols <= 64 * LN_MAXV, "comet_layernorm_fwd: cols must be in [1,1024]");
  COMET_CHECK_ARG(x && (y || y2), "comet_layernorm_fwd: null pointer");
  if (rows == 0) return COMET_OK;
  dim3 grid((unsigned)cdiv(rows, 4));
  hipStream_t s = as_stream(stream);
  const bool vec = cols % 8 == 0 && ldx % 8 == 0 && (y == nullptr || ldy % 8 == 0) && (y2 == nullptr || ldy2 % 8 == 0) &&
                   a32(x) && a32(y) && a32(y2);
  if (vec) {
    // persistent rows: <= 8 workgroups (32 waves) per CU, each wave prefetching its next row
    // (balanced: every wave gets the same number of rows +- 1); <= 2 rows per wave stays flat
    const bool flat = rows <= 2 * 2048 * 4 || getenv("COMET_LN_FLAT") != nullptr;
    const int64_t iters = cdiv(rows, 2048 * 4);
    const dim3 grid_rows((unsigned)cdiv(cdiv(rows, iters), 4));
    // narrow rows: 8 rows per wave for rows of <= 8 lanes x CH (65536 x 32 f32: 13.5 vs 16.2 us; at 32
    // lanes per row the persistent-row kernel's prefetch wins, 18.3 vs 23.8 us at 65536 x 128,
    // profiles/r06_tail/tail_ab_narrow.txt); COMET_LN_NO_NARROW=1: one row per wave
    const int ch_n = (dtype_x == COMET_F32 || (y && dtype_y == COMET_F32)) ? 4 : 8;
    const int lanes = (int)cdiv(cols, ch_n);
    const int rpw_n = lanes <= 8 ? 8 : 1;
    const bool narrow = rpw_n > 1 && getenv("COMET_LN_NO_NARROW") == nullptr;
#define LNN(TX, TY, CH)                                                                                        \
  do {                                                                                                         \
    const dim3 gn((unsigned)cdiv(rows, 4 * rpw_n));                                                            \
    hipLaunchKernelGGL((ln_fwd_narrow_kernel<TX, TY, CH, 8>), gn, dim3(256), 0, s, (const TX*)x, weight,        \
                       bias, (TY*)y, (__bf16*)y2, mean, rstd, rows, (int)cols, ldx, ldy, ldy2, eps, relu);     \
  } while (0)
#define LNV(TX, TY, CH, NK)                                                                                    \
  do {                                                                                                         \
    if (narrow && NK == 1) LNN(TX, TY, CH);                                                                    \
    else if (flat)                                                                                             \
      hipLaunchKernelGGL((ln_fwd_vec_kernel<TX, TY, CH, NK>), grid, dim3(256), 0, s, (const TX*)x, weight,      \
                         bias, (TY*)y, (__bf16*)y2, mean, rstd, rows, (int)cols, ldx, ldy, ldy2, eps, relu);   \
    else                                                                                                       \
      hipLaunchKernelGGL((ln_fwd_rows_kernel<TX, TY, CH, NK>), grid_rows, dim3(256), 0, s, (const TX*)x,       \
                         weight, bias, (TY*)y, (__bf16*)y2, mean, rstd, rows, (int)cols, ldx, ldy, ldy2, eps,  \
                         relu);                                                                                \
  } while (0)
#define LNV_CH(TX, TY, CH)                                                                                 \
  do {                                                                                                     \
    const int nk = (int)cdiv(cols, 64 * CH);                                                               \
    if (nk == 1) LNV(TX, TY, CH, 1); else if (nk == 2) LNV(TX, TY, CH, 2);                                 \
    else if (nk == 3) LNV(TX, TY, CH, 3); else LNV(TX, TY, CH, 4);                                         \
  } while (0)
#define LNV2(TX, TY)                                                                                       \
  do { if (sizeof(TX) == 4 || (y && sizeof(TY) == 4)) LNV_CH(TX, TY, 4); else LNV_CH(TX, TY, 8); } while (0)
    if (dtype_x == COMET_F32 && dtype_y == COMET_F32) LNV2(float, float);
    else if (dtype_x == COMET_F32 && dtype_y == COMET_BF16) LNV2(float, __bf16);
    else if (dtype_x == COMET_BF16 && dtype_y == COMET_F32) LNV2(__bf16, float);
    else if (dtype_x == COMET_BF16 && dtype_y == COMET_BF16) LNV2(__bf16, __bf16);
    else { set_error("comet_layernorm_fwd: bad dtype"); return COMET_EINVAL; }
#undef LNV2
#undef LNV_CH
#undef LNV
#undef LNN
    COMET_CHECK_LAUNCH("comet_layernorm_fwd");
    return COMET_OK;
  }
  COMET_CHECK_ARG(y2 == nullptr, "comet_layernorm_fwd: the second output needs cols % 8 == 0 and 32-B aligned rows");
#define LNF(TX, TY)                                                                        \
  hipLaunchKernelGGL((ln_fwd_kernel<TX, TY>), grid, dim3(256), 0, s, (const TX*)x, weight, \
                     bias, (TY*)y, mean, rstd, rows, (int)cols, ldx, ldy, eps, relu)
  if (dtype_x == COMET_F32 && dtype_y == COMET_F32) LNF(float, float);
  else if (dtype_x == COMET_F32 && dtype_y == COMET_BF16) LNF(float, __bf16);
  else if (dtype_x == COMET_BF16 && dtype_y == COMET_F32) LNF(__bf16, float);
  else if (dtype_x == COMET_BF16 && dtype_y == COMET_BF16) LNF(__bf16, __bf16);
  else { set_error("comet_layernorm_fwd: bad dtype"); return COMET_EINVAL; }
#undef LNF
  COMET_CHECK_LAUNCH("comet_layernorm_fwd");
  return COMET_OK;
}

// rows per wave of the LayerNorm backward: with affine gradients every workgroup ends in
// 2 x cols atomics, so waves take 16 rows; without them 2 rows per wave put more waves (and so
// more rows' loads) in flight: 184 -> 137 us (dual) and 219 -> 158 us (residual) at 69240 x 768,
// 4.0 -> 5.4 TB/s (tools/lnbwd_bench.py, profiles/r02_lnbwd). COMET_LNB_RPW overrides.
static int ln_bwd_rpw(const float* dweight, const float* dbias) {
  if (const char* e = getenv("COMET_LNB_RPW")) {
    const int v = atoi(e);
    if (v >= 1 && v <= 64) return v;
  }
  return (dweight || dbias) ? LN_RPW : 2;
}

extern "C" int comet_layernorm_bwd(int dtype_x, int dtype_dy, const void* x, const void* dy, const void* dy2,
                                   const float* mean, const float* rstd, const float* weight,
                                   int dtype_dx, void* dx, float* dweight, float* dbias, int64_t rows,
                                   int64_t cols, int dx_accumulate, void* stream) {
  COMET_CHECK_ARG(cols > 0 && cols <= 64 * LN_MAXV, "comet_layernorm_bwd: cols must be in [1,1024]");
  COMET_CHECK_ARG(x && dy && mean && rstd && dx, "comet_layernorm_bwd: null pointer");
  if (rows == 0) return COMET_OK;
  const int rpw = ln_bwd_rpw(dweight, dbias);
  dim3 grid((unsigned)cdiv(rows, 4 * rpw));
  hipStream_t s = as_stream(stream);
  const bool vec = cols % 8 == 0 && a32(x) && a32(dy) && a32(dy2) && a32(dx);
  if (vec) {
#define LBV(TX, TD, TO, CH, NK)                                                                           \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TX, TD, TO, CH, NK>), grid, dim3(256), 0, s, (const TX*)x, (const TD*)dy, \
                     (const __bf16*)dy2, mean, rstd, weight, (TO*)dx, dweight, dbias, rows, (int)cols, dx_accumulate, \
                     nullptr, rpw)
#define LBV_CH(TX, TD, TO, CH)                                                                             \
  do {                                                                                                     \
    const int nk = (int)cdiv(cols, 64 * CH);                                                               \
    if (nk == 1) LBV(TX, TD, TO, CH, 1); else if (nk == 2) LBV(TX, TD, TO, CH, 2);                         \
    else if (nk == 3) LBV(TX, TD, TO, CH, 3); else LBV(TX, TD, TO, CH, 4);                                 \
  } while (0)
#define LBV_NV(TX, TD, TO)                                                                                 \
  do { if (sizeof(TX) == 4 || sizeof(TD) == 4 || sizeof(TO) == 4) LBV_CH(TX, TD, TO, 4); else LBV_CH(TX, TD, TO, 8); } while (0)
#define LBV_O(TX, TD) do { if (dtype_dx == COMET_F32) LBV_NV(TX, TD, float); else LBV_NV(TX, TD, __bf16); } while (0)
#define LBV_D(TX) do { if (dtype_dy == COMET_F32) LBV_O(TX, float); else LBV_O(TX, __bf16); } while (0)
    if (dtype_x == COMET_F32) LBV_D(float); else LBV_D(__bf16);
#undef LBV_D
#undef LBV_O
#undef LBV_NV
#undef LBV_CH
#undef LBV
    COMET_CHECK_LAUNCH("comet_layernorm_bwd");
    return COMET_OK;
  }
  COMET_CHECK_ARG(dy2 == nullptr && dtype_dx == COMET_F32,
                  "comet_layernorm_bwd: dy2 / bf16 dx need cols % 8 == 0 and 32-B aligned rows");
#define LNB(TX, TD)                                                                           \
  hipLaunchKernelGGL((ln_bwd_kernel<TX, TD>), grid, dim3(256), 0, s, (const TX*)x, (const TD*)dy, \
                     mean, rstd, weight, (float*)dx, dweight, dbias, rows, (int)cols, dx_accumulate)
  if (dtype_x == COMET_F32 && dtype_dy == COMET_F32) LNB(float, float);
  else if (dtype_x == COMET_F32 && dtype_dy == COMET_BF16) LNB(float, __bf16);
  else if (dtype_x == COMET_BF16 && dtype_dy == COMET_F32) LNB(__bf16, float);
  else if (dtype_x == COMET_BF16 && dtype_dy == COMET_BF16) LNB(__bf16, __bf16);
  else { set_error("comet_layernorm_bwd: bad dtype"); return COMET_EINVAL; }
#undef LNB
  COMET_CHECK_LAUNCH("comet_layernorm_bwd");
  return COMET_OK;
}

extern "C" int comet_instnorm_workspace(int64_t n, int64_t hw, int64_t c, int64_t* bytes) {
  COMET_CHECK_ARG(bytes && n > 0 && hw > 0 && c > 0, "comet_instnorm_workspace: bad args");
  *bytes = 0;
  if (c % 8 == 0 && c <= 256) {
    const int chunks = in_chunks(n, hw, c);
    if (chunks > 1) *bytes = n * chunks * 2 * c * (int64_t)sizeof(float);
  }
  return COMET_OK;
}

extern "C" int comet_instnorm_nhwc(int dtype, const void* x, const void* res, void* y, int64_t n,
                                   int64_t hw, int64_t c, float eps, int relu, int res_norm_relu,
                                   void* workspace, int64_t workspace_bytes, void* stream) {
  COMET_CHECK_ARG(x && y && n > 0 && hw > 0 && c > 0, "comet_instnorm_nhwc: bad args");
  const bool aligned = ((uintptr_t)x | (uintptr_t)y | (uintptr_t)res) % 32 == 0;
  if (c % 8 == 0 && c <= 256 && aligned && n <= 65535ll * 65535ll) {
    hipStream_t s = as_stream(stream);
    int chunks = in_chunks(n, hw, c);
    if (chunks > 1 && (!workspace || workspace_bytes < n * chunks * 2 * c * (int64_t)sizeof(float))) chunks = 1;
    INGeo g{hw, cdiv(hw, chunks), (int)c, chunks, eps, relu, res_norm_relu};
    // small bf16 images: one wave per image (in_wave_kernel)
    const int tpp = (int)(c / 8), ppw = tpp > 0 && 64 % tpp == 0 ? 64 / tpp : 0;
    const int64_t np = ppw ? cdiv(hw, ppw) : 0;
    if (dtype == COMET_BF16 && chunks == 1 && ppw && np <= 16 && getenv("COMET_IN_NO_WAVE") == nullptr) {
      const unsigned gw = (unsigned)cdiv(n, 4);
      COMET_CHECK_ARG(cdiv(n, 4) < (1ll << 31), "comet_instnorm_nhwc: too many images");
#define INW(NP) hipLaunchKernelGGL((in_wave_kernel<NP>), dim3(gw), dim3(256), 0, s, (const __bf16*)x, (const __bf16*)res, (__bf16*)y, n, g)
      if (np <= 1) INW(1); else if (np <= 2) INW(2); else if (np <= 4) INW(4); else if (np <= 8) INW(8); else INW(16);
#undef INW
      COMET_CHECK_LAUNCH("comet_instnorm_nhwc (one wave per image)");
      return COMET_OK;
    }
#define INL(T)                                                                                           \
  if (chunks == 1) {                                                                                     \
    COMET_CHECK_ARG(n <= 2147483647ll, "comet_instnorm_nhwc: too many images");                         \
    hipLaunchKernelGGL((in_fused_kernel<T>), dim3((unsigned)n), dim3(256), 0, s, (const T*)x,            \
                       (const T*)res, (T*)y, g);                                                         \
  } else {                                                                                               \
    COMET_CHECK_ARG(n <= 65535, "comet_instnorm_nhwc: too many images for the chunked path");          \
    hipLaunchKernelGGL((in_stats_kernel<T>), dim3((unsigned)chunks, (unsigned)n), dim3(256), 0, s,       \
                       (const T*)x, (float*)workspace, g);                                               \
    hipLaunchKernelGGL((in_apply_kernel<T>), dim3((unsigned)chunks, (unsigned)n), dim3(256), 0, s,       \
                       (const T*)x, (const T*)res, (T*)y, (const float*)workspace, g);                   \
  }
    if (dtype == COMET_F32) { INL(float) }
    else if (dtype == COMET_BF16) { INL(__bf16) }
    else { set_error("comet_instnorm_nhwc: bad dtype"); return COMET_EINVAL; }
#undef INL
    COMET_CHECK_LAUNCH("comet_instnorm_nhwc");
    return COMET_OK;
  }
  COMET_CHECK_ARG(cdiv(c, 64) <= 65535, "comet_instnorm_nhwc: c too large");
  dim3 grid((unsigned)n, (unsigned)cdiv(c, 64));
  hipStream_t s = as_stream(stream);
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((instnorm_nhwc_kernel<float>), grid, dim3(256), 0, s, (const float*)x,
                       (const float*)res, (float*)y, hw, (int)c, eps, relu, res_norm_relu);
  else if (dtype == COMET_BF16)
    hipLaunchKernelGGL((instnorm_nhwc_kernel<__bf16>), grid, dim3(256), 0, s, (const __bf16*)x,
                       (const __bf16*)res, (__bf16*)y, hw, (int)c, eps, relu, res_norm_relu);
  else { set_error("comet_instnorm_nhwc: bad dtype"); return COMET_EINVAL; }
  COMET_CHECK_LAUNCH("comet_instnorm_nhwc");
  return COMET_OK;
}

// LayerNorm backward whose input also feeds a residual (x + Mlp(LN(x)), modules.py:293-294 /
// 342-343): dx = dres + LN backward of dy in one pass (no separate gradient add).
extern "C" int comet_layernorm_bwd_res(int dtype_x, int dtype_dy, const void* x, const void* dy, const float* dres,
                                       const float* mean, const float* rstd, const float* weight, float* dx,
                                       float* dweight, float* dbias, int64_t rows, int64_t cols, void* stream) {
  COMET_CHECK_ARG(cols > 0 && cols <= 64 * LN_MAXV, "comet_layernorm_bwd_res: cols must be in [1,1024]");
  COMET_CHECK_ARG(x && dy && dres && mean && rstd && dx, "comet_layernorm_bwd_res: null pointer");
  COMET_CHECK_ARG(cols % 8 == 0 && a32(x) && a32(dy) && a32(dres) && a32(dx),
                  "comet_layernorm_bwd_res: needs cols % 8 == 0 and 32-B aligned rows");
  if (rows == 0) return COMET_OK;
  const int rpw = ln_bwd_rpw(dweight, dbias);
  dim3 grid((unsigned)cdiv(rows, 4 * rpw));
  hipStream_t s = as_stream(stream);
#define LBR(TX, TD, NK)                                                                                          \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TX, TD, float, 4, NK>), grid, dim3(256), 0, s, (const TX*)x, (const TD*)dy, \
                     (const __bf16*)nullptr, mean, rstd, weight, dx, dweight, dbias, rows, (int)cols, 0, dres, rpw)
#define LBR_NK(TX, TD)                                                            \
  do {                                                                            \
    const int nk = (int)cdiv(cols, 64 * 4);                                       \
    if (nk == 1) LBR(TX, TD, 1); else if (nk == 2) LBR(TX, TD, 2);               \
    else if (nk == 3) LBR(TX, TD, 3); else LBR(TX, TD, 4);                        \
  } while (0)
  if (dtype_x == COMET_F32 && dtype_dy == COMET_F32) LBR_NK(float, float);
  else if (dtype_x == COMET_F32 && dtype_dy == COMET_BF16) LBR_NK(float, __bf16);
  else { set_error("comet_layernorm_bwd_res: x must be f32"); return COMET_EINVAL; }
#undef LBR_NK
#undef LBR
  COMET_CHECK_LAUNCH("comet_layernorm_bwd_res");
  return COMET_OK;
}
