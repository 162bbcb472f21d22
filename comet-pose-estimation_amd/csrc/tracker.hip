#include <cstdlib>
// Point-tracker kernels (coarse CoTracker-style predictor and fine refinement) + DINOv2 input
// preparation. All feature maps are channels-last (NHWC).
//
// Reference sites: base_track_predictor.py:95-284 (iteration: corr sample, flow embedding,
// transformer input, feature / coordinate update), blocks.py:351-429 (CorrBlock: avg-pool
// pyramid, corr = f·fmap/sqrt(C), 9x9 bilinear window, zeros padding), utils.py:835-974
// (get_2d_embedding, bilinear_sampler, sample_features4d), refine_track.py:26-278 (patch
// extraction, compute_score_fn), E2Epose2.py:232-236 (score inversion),
// camera_predictor10.py:622-634 (resize to 336, ImageNet normalisation) + DINOv2 patch_embed.
#include "common.hpp"

namespace comet {
namespace {

inline unsigned g1d(int64_t n) {
  int64_t g = cdiv(n, 256);
  return (unsigned)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}
#define GRID_STRIDE(i, n) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// torch grid_sample source index for align_corners=True after bilinear_sampler's
// normalisation: g = x * 2/max(size-1,1) - 1 ; ix = ((g + 1) / 2) * (size - 1)
__device__ __forceinline__ float src_index(float x, int size, bool border) {
  const float g = x * (2.f / (float)(size - 1 > 1 ? size - 1 : 1)) - 1.f;
  float ix = ((g + 1.f) / 2.f) * (float)(size - 1);
  if (border) ix = fminf(fmaxf(ix, 0.f), (float)(size - 1));
  return ix;
}

// sample_features4d: out[b, r, c] = bilinear(fmap[b], coords[b, r]) ; one wave per (b, r)
template <typename T>
__global__ void sample_kernel(const T* __restrict__ fmap, int64_t bstride, int H, int W, int C,
                              const float* __restrict__ coords, int64_t cstride_b, int64_t cstride_r,
                              float* __restrict__ out, int64_t ostride_b, int64_t ostride_r, int64_t B,
                              int64_t R, int border) {
  const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wv >= B * R) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = wv / R, r = wv % R;
  const float* cp = coords + b * cstride_b + r * cstride_r;
  const float ix = src_index(cp[0], W, border), iy = src_index(cp[1], H, border);
  const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  const int x1 = x0 + 1, y1 = y0 + 1;
  const float wnw = ((float)x1 - ix) * ((float)y1 - iy), wne = (ix - (float)x0) * ((float)y1 - iy);
  const float wsw = ((float)x1 - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
  const T* base = fmap + b * bstride;
  auto ok = [&](int x, int y) { return x >= 0 && x < W && y >= 0 && y < H; };
  for (int c = lane; c < C; c += 64) {
    float v = 0.f;
    if (ok(x0, y0)) v += to_f32(base[((int64_t)y0 * W + x0) * C + c]) * wnw;
    if (ok(x1, y0)) v += to_f32(base[((int64_t)y0 * W + x1) * C + c]) * wne;
    if (ok(x0, y1)) v += to_f32(base[((int64_t)y1 * W + x0) * C + c]) * wsw;
    if (ok(x1, y1)) v += to_f32(base[((int64_t)y1 * W + x1) * C + c]) * wse;
    out[b * ostride_b + r * ostride_r + c] = v;
  }
}

// CorrBlock.corr + CorrBlock.sample fused: for track (b, n, s) and level l, window (i, j)
// samples the correlation map f·fmap_l/sqrt(C) bilinearly (zeros padding) at
// (x/2^l + i - r, y/2^l + j - r) (the reference's meshgrid(dy, dx) puts the first window index on
// x). Correlation is linear, so the 4 corner dot products are formed on a (2r+4)^2 pixel grid
// around the window and shared by all (2r+1)^2 samples. One workgroup (256 threads) per track.
struct PyrTab {
  const void* p[8];
  int h[8];
  int w[8];
};

template <typename TF, typename TT, int C>
__global__ void __launch_bounds__(256)
corr_kernel(PyrTab tab, int levels, int radius, const TT* __restrict__ feats, const float* __restrict__ coords,
            float* __restrict__ out, int64_t ldo, int64_t col0, int64_t N, int S, float inv_sqrt_c) {
  constexpr int G = 16;  // max grid side (2r+4 <= 16 -> r <= 6)
  __shared__ float f[C];
  __shared__ float dots[G * G];
  const int64_t t = blockIdx.x;  // (b*N + n)*S + s
  const int s = (int)(t % S);
  const int64_t bn = t / S;
  const int64_t b = bn / N;
  for (int c = threadIdx.x; c < C; c += 256) f[c] = to_f32(feats[t * C + c]);
  const float cx = coords[t * 2], cy = coords[t * 2 + 1];
  const int win = 2 * radius + 1, gs = 2 * radius + 4;
  float* orow = out + t * ldo + col0;
  // dot products: LPP lanes per pixel, 16 channels each (2 x 16-B loads for bf16 maps), reduced
  // over the LPP lanes by xor shuffles; 256 / LPP pixels per pass
  constexpr int LPP = C / 16;
  const int sub = threadIdx.x % LPP, pslot = threadIdx.x / LPP;
  __syncthreads();
  float fr[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) fr[e] = f[sub * 16 + e];
  for (int l = 0; l < levels; ++l) {
    const int H = tab.h[l], W = tab.w[l];
    const TF* fm = reinterpret_cast<const TF*>(tab.p[l]) + (b * S + s) * (int64_t)H * W * C;
    const float scl = 1.f / (float)(1 << l);
    const float xl = cx * scl, yl = cy * scl;
    const int gx0 = (int)floorf(xl) - radius - 1, gy0 = (int)floorf(yl) - radius - 1;
    __syncthreads();  // previous level's dots consumed
    for (int p0 = 0; p0 < gs * gs; p0 += 256 / LPP) {
      const int p = p0 + pslot;
      const int px = gx0 + p % gs, py = gy0 + p / gs;
      float acc = 0.f;
      if (p < gs * gs && px >= 0 && px < W && py >= 0 && py < H) {
        const TF* pix = fm + ((int64_t)py * W + px) * C + sub * 16;
        float a[8], c8[8];
        load8(pix, a);
        load8(pix + 8, c8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += fr[e] * a[e] + fr[8 + e] * c8[e];
      }
#pragma unroll
      for (int o = LPP / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (sub == 0 && p < gs * gs) dots[(p / gs) * G + (p % gs)] = acc * inv_sqrt_c;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < win * win; k += 256) {
      const int i = k / win, j = k % win;
      const float ix = src_index(xl + (float)(i - radius), W, false);
      const float iy = src_index(yl + (float)(j - radius), H, false);
      const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
      const float wnw = ((float)(x0 + 1) - ix) * ((float)(y0 + 1) - iy), wne = (ix - (float)x0) * ((float)(y0 + 1) - iy);
      const float wsw = ((float)(x0 + 1) - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
      auto D = [&](int x, int y) -> float {
        const int gx = x - gx0, gy = y - gy0;
        return (gx >= 0 && gx < gs && gy >= 0 && gy < gs) ? dots[gy * G + gx] : 0.f;
      };
      orow[l * win * win + k] = D(x0, y0) * wnw + D(x0 + 1, y0) * wne + D(x0, y0 + 1) * wsw + D(x0 + 1, y0 + 1) * wse;
    }
  }
}

// corr_kernel with one wave per track row instead of one workgroup (the fine tracker: C = 32, r = 3,
// a 10 x 10 grid per level): no workgroup barriers, all 64 lanes busy on the grid's dot products
// (LPP = 2 lanes per pixel, 32 pixels per pass) and 49 of 64 on the window samples, four rows per
// workgroup. Per pixel and per sample the arithmetic -- the lane's 16-channel partial sums, the xor
// shuffle over the LPP lanes, the bilinear weights -- is corr_kernel's, so the outputs are bit-identical.
// 65536 fine rows: 184 vs 231 us (profiles/r06_tail/corr_wave_ab.txt; issuing all four passes' loads
// first measured 262 us: the extra registers cost more occupancy than the loads gained).
template <typename TF, typename TT, int C>
__global__ void __launch_bounds__(256)
corr_wave_kernel(PyrTab tab, int levels, int radius, const TT* __restrict__ feats, const float* __restrict__ coords,
                 float* __restrict__ out, int64_t ldo, int64_t col0, int64_t N, int S, float inv_sqrt_c, int64_t T) {
  constexpr int G = 16, LPP = C / 16, PPW = 64 / LPP;
  __shared__ float dots_w[4][G * G];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;  // (b*N + n)*S + s
  if (t >= T) return;  // whole waves; no workgroup barrier below
  const int s = (int)(t % S);
  const int64_t b = (t / S) / N;
  float* dots = dots_w[wv];
  const int sub = lane % LPP, pslot = lane / LPP;
  float fr[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) fr[e] = to_f32(feats[t * C + sub * 16 + e]);
  const float cx = coords[t * 2], cy = coords[t * 2 + 1];
  const int win = 2 * radius + 1, gs = 2 * radius + 4;
  float* orow = out + t * ldo + col0;
  for (int l = 0; l < levels; ++l) {
    const int H = tab.h[l], W = tab.w[l];
    const TF* fm = reinterpret_cast<const TF*>(tab.p[l]) + (b * S + s) * (int64_t)H * W * C;
    const float scl = 1.f / (float)(1 << l);
    const float xl = cx * scl, yl = cy * scl;
    const int gx0 = (int)floorf(xl) - radius - 1, gy0 = (int)floorf(yl) - radius - 1;
    __builtin_amdgcn_wave_barrier();  // the previous level's samples read dots before it is rewritten
    for (int p0 = 0; p0 < gs * gs; p0 += PPW) {
      const int p = p0 + pslot;
      const int px = gx0 + p % gs, py = gy0 + p / gs;
      float acc = 0.f;
      if (p < gs * gs && px >= 0 && px < W && py >= 0 && py < H) {
        const TF* pix = fm + ((int64_t)py * W + px) * C + sub * 16;
        float a[8], c8[8];
        load8(pix, a);
        load8(pix + 8, c8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += fr[e] * a[e] + fr[8 + e] * c8[e];
      }
#pragma unroll
      for (int o = LPP / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (sub == 0 && p < gs * gs) dots[(p / gs) * G + (p % gs)] = acc * inv_sqrt_c;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's dot products are in LDS
    __builtin_amdgcn_wave_barrier();
    for (int k = lane; k < win * win; k += 64) {
      const int i = k / win, j = k % win;
      const float ix = src_index(xl + (float)(i - radius), W, false);
      const float iy = src_index(yl + (float)(j - radius), H, false);
      const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
      const float wnw = ((float)(x0 + 1) - ix) * ((float)(y0 + 1) - iy), wne = (ix - (float)x0) * ((float)(y0 + 1) - iy);
      const float wsw = ((float)(x0 + 1) - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
      auto D = [&](int x, int y) -> float {
        const int gx = x - gx0, gy = y - gy0;
        return (gx >= 0 && gx < gs && gy >= 0 && gy < gs) ? dots[gy * G + gx] : 0.f;
      };
      orow[l * win * win + k] = D(x0, y0) * wnw + D(x0 + 1, y0) * wne + D(x0, y0 + 1) * wsw + D(x0 + 1, y0 + 1) * wse;
    }
  }
}

// The same CorrBlock step on the matrix cores, for bf16 maps with C = 128 (the coarse tracker:
// 512 tracks per frame on a 64 x 64 map). The tracks of one frame read overlapping windows, so
// the dot products are formed as dense MFMA tiles (16 map pixels x 16 tracks x 32 channels) over
// the bounding box of 16 tracks' (2r+4)^2 grids, walked in 8 x 2-pixel blocks, and each product
// inside a track's own grid is kept in an LDS table from which the (2r+1)^2 bilinear samples are
// taken as in corr_kernel. A workgroup (4 waves x 16 tracks) first ranks the frame's tracks by
// (8-pixel row band, column) of their level-0 position, so a wave's 16 tracks are neighbours and
// their box is small; the rank only groups tracks (each product is one MFMA output element, the
// same whatever the other rows of the tile), and every output row is written by its own track.
// The f32 track features enter as three bf16 terms (hi + mid + lo == f exactly), so the products
// are exact as in the f32 kernel and only the summation order differs.
typedef float f32x8 __attribute__((ext_vector_type(8)));

template <int C, int RING, int OCC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC)))
corr_mfma_kernel(PyrTab tab, int levels, int radius, const float* __restrict__ feats,
                 const float* __restrict__ coords, float* __restrict__ out, int64_t ldo, int64_t col0, int N, int S,
                 int frames, float inv_sqrt_c, int sort) {
  constexpr int KS = C / 32;  // 32-channel k-steps
  extern __shared__ __attribute__((aligned(16))) float csm[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, hg = lane >> 4;
  const int gs = 2 * radius + 4, g2 = gs * gs, win = 2 * radius + 1, nw = win * win;
  const int tiles = (N + 63) / 64;
  // XCD-aware order: workgroups are dealt to the 8 XCDs round-robin, so frame f's tiles all get
  // blockIdx = f (mod 8) and share one XCD's L2 (the frame's pyramid is read by all of them)
  const int xcd = (int)(blockIdx.x & 7), q = (int)(blockIdx.x >> 3);
  const int f = (q / tiles) * 8 + xcd, r0 = (q % tiles) * 64;
  if (f >= frames) return;
  const int b = f / S, s = f % S;
  float* dt = csm + wid * 16 * g2;  // this wave's [16 tracks][gs * gs] dots
  int* slot = reinterpret_cast<int*>(csm + 4 * 16 * g2);
  unsigned* keys = reinterpret_cast<unsigned*>(slot + 64);
  if (sort) {
    // key = band (10 bits) | column (11 bits) | track (11 bits, N <= 2048): distinct, so a track's
    // rank is the number of smaller keys
    const int np = (N + 3) & ~3;
    for (int n = tid; n < np; n += 256) {
      unsigned key = 0xffffffffu;
      if (n < N) {
        const float* c = coords + (((int64_t)b * N + n) * S + s) * 2;
        const float band = fminf(fmaxf(floorf(c[1] * 0.125f), -8.f), 1015.f) + 8.f;
        const float col = fminf(fmaxf(floorf(c[0]), -64.f), 1983.f) + 64.f;
        key = ((unsigned)band << 22) | ((unsigned)col << 11) | (unsigned)n;
      }
      keys[n] = key;
    }
    __syncthreads();
    for (int n0 = 0; n0 < N; n0 += 512) {
      const int na = n0 + tid, nb = n0 + 256 + tid;
      const unsigned ka = na < N ? keys[na] : 0u, kb = nb < N ? keys[nb] : 0u;
      int ra = 0, rb = 0;
      for (int m = 0; m < np; m += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(keys + m);
        ra += (v.x < ka) + (v.y < ka) + (v.z < ka) + (v.w < ka);
        rb += (v.x < kb) + (v.y < kb) + (v.z < kb) + (v.w < kb);
      }
      if (na < N && ra >= r0 && ra < r0 + 64) slot[ra - r0] = na;
      if (nb < N && rb >= r0 && rb < r0 + 64) slot[rb - r0] = nb;
    }
  } else if (tid < 64) {
    slot[tid] = r0 + tid;
  }
  __syncthreads();
  const bool act = r0 + wid * 16 + li < N;
  const int n = act ? slot[wid * 16 + li] : 0;
  const int64_t t = ((int64_t)b * N + n) * S + s;
  // track features as three bf16 terms, B operand layout: track li, channels 32 ks + 8 hg ..
  bf16x8 tf[3][KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    f32x8 v{};
    if (act) {
      const float4* p = reinterpret_cast<const float4*>(feats + t * C + 32 * ks + 8 * hg);
      const float4 x0 = p[0], x1 = p[1];
      v = f32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      tf[u][ks] = __builtin_convertvector(v, bf16x8);
      v -= __builtin_convertvector(tf[u][ks], f32x8);
    }
  }
  const float cx = act ? coords[t * 2] : 0.f, cy = act ? coords[t * 2 + 1] : 0.f;
  for (int l = 0; l < levels; ++l) {
    const int H = tab.h[l], W = tab.w[l];
    const __bf16* fm = reinterpret_cast<const __bf16*>(tab.p[l]) + (int64_t)f * H * W * C;
    const float scl = 1.f / (float)(1 << l);
    const float xl = cx * scl, yl = cy * scl;
    // grid origin, clamped so that NaN / huge coordinates give an empty intersection with the map
    const int gx0 = (int)fminf(fmaxf(floorf(xl), -65536.f), 65536.f) - radius - 1;
    const int gy0 = (int)fminf(fmaxf(floorf(yl), -65536.f), 65536.f) - radius - 1;
    int bx0 = act ? gx0 : 1 << 30, by0 = act ? gy0 : 1 << 30;
    int bx1 = act ? gx0 + gs - 1 : -(1 << 30), by1 = act ? gy0 + gs - 1 : -(1 << 30);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      bx0 = min(bx0, __shfl_xor(bx0, o, 64));
      by0 = min(by0, __shfl_xor(by0, o, 64));
      bx1 = max(bx1, __shfl_xor(bx1, o, 64));
      by1 = max(by1, __shfl_xor(by1, o, 64));
    }
    // the box is wave-uniform: say so, so that the block loop and its index math run on the SALU
    bx0 = __builtin_amdgcn_readfirstlane(max(bx0, 0));
    by0 = __builtin_amdgcn_readfirstlane(max(by0, 0));
    bx1 = __builtin_amdgcn_readfirstlane(min(bx1, W - 1));
    by1 = __builtin_amdgcn_readfirstlane(min(by1, H - 1));
    // 8 x 2-pixel blocks over the box: nbx across, nby down (none when the box misses the map)
    const int nbx = bx1 >= bx0 ? (bx1 - bx0 + 8) >> 3 : 0, nby = by1 >= by0 ? (by1 - by0 + 2) >> 1 : 0;
    const int nblk = nbx * nby;
    // zero the table (pixels outside the map keep a zero dot product)
    for (int i = lane; i < 4 * g2; i += 64) reinterpret_cast<float4*>(dt)[i] = float4{0.f, 0.f, 0.f, 0.f};
    // A operand: pixel li of the block = (bx0 + 8 cb + (li & 7), by0 + 2 rb + (li >> 3)); a pixel
    // past the box's edge loads the edge pixel instead (its output row is never stored), so the
    // loads are unconditional
    auto aload = [&](int blk, bf16x8 (&a)[KS]) {
      const int rb = blk / nbx, cb = blk - rb * nbx;
      const int px = min(bx0 + 8 * cb + (li & 7), bx1), py = min(by0 + 2 * rb + (li >> 3), by1);
      const __bf16* src = fm + ((int64_t)py * W + px) * C + 8 * hg;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) a[ks] = *reinterpret_cast<const bf16x8*>(src + 32 * ks);
    };
    // this lane's outputs: pixels 4 hg + e of the block = columns 4 (hg & 1) + e of row hg >> 1
    const int cxe = bx0 + 4 * (hg & 1), ry = by0 + (hg >> 1);
    auto blkstep = [&](int blk, const bf16x8 (&ac)[KS]) {
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int u = 0; u < 3; ++u) d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ac[ks], tf[u][ks], d, 0, 0, 0);
      const int rb = blk / nbx, cb = blk - rb * nbx;
      const int px = cxe + 8 * cb, py = ry + 2 * rb;
      const int gx = px - gx0, gy = py - gy0;
      if (act && py <= by1 && (unsigned)gy < (unsigned)gs) {
        float* trow = dt + li * g2 + gy * gs + gx;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (px + e <= bx1 && (unsigned)(gx + e) < (unsigned)gs) trow[e] = d[e] * inv_sqrt_c;
      }
    };
    // a ring of RING register buffers with static indices (a runtime index into a register array
    // becomes indexed-register moves): RING - 1 blocks of pixels load while a block's MFMAs run. The
    // prefetch is unconditional (past the last block it reloads the last one) so that the wait
    // before the MFMAs counts exactly the older block's loads
    bf16x8 ring[RING][KS];
    if (nblk > 0) {
#pragma unroll
      for (int u = 0; u < RING - 1; ++u) aload(min(u, nblk - 1), ring[u]);
    }
    for (int blk0 = 0; blk0 < nblk; blk0 += RING) {
#pragma unroll
      for (int u = 0; u < RING; ++u) {
        const int blk = blk0 + u;
        if (blk < nblk) {
          aload(min(blk + RING - 1, nblk - 1), ring[(u + RING - 1) % RING]);
          blkstep(blk, ring[u]);
        }
      }
    }
    asm volatile("" ::: "memory");
    // (2r+1)^2 bilinear samples per track from the table, the arithmetic of corr_kernel: one task per
    // (track, window column i) computes the x terms once and walks the window rows j
    for (int k0 = 0; k0 < 16 * win; k0 += 64) {  // uniform trip count: every lane joins the shuffles
      const int k = k0 + lane;
      const int ti = min(k / win, 15), i = k - ti * win;
      const float tx = __shfl(xl, ti, 64), ty = __shfl(yl, ti, 64);
      const int ox = __shfl(gx0, ti, 64), oy = __shfl(gy0, ti, 64), tn = __shfl(n, ti, 64);
      if (k >= 16 * win || r0 + wid * 16 + ti >= N) continue;
      float* orow = out + (((int64_t)b * N + tn) * S + s) * ldo + col0 + l * nw + i * win;
      const float ix = src_index(tx + (float)(i - radius), W, false);
      const int x0 = (int)floorf(ix);
      const int gxa = x0 - ox;
      const bool xa = (unsigned)gxa < (unsigned)gs, xb = (unsigned)(gxa + 1) < (unsigned)gs;
      const float* col = dt + ti * g2 + gxa;
      for (int j = 0; j < win; ++j) {
        const float iy = src_index(ty + (float)(j - radius), H, false);
        const int y0 = (int)floorf(iy);
        const float wnw = ((float)(x0 + 1) - ix) * ((float)(y0 + 1) - iy), wne = (ix - (float)x0) * ((float)(y0 + 1) - iy);
        const float wsw = ((float)(x0 + 1) - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
        const int gya = y0 - oy;
        const bool ya = (unsigned)gya < (unsigned)gs, yb = (unsigned)(gya + 1) < (unsigned)gs;
        const float* c0 = col + gya * gs;
        const float d00 = xa && ya ? c0[0] : 0.f, d10 = xb && ya ? c0[1] : 0.f;
        const float d01 = xa && yb ? c0[gs] : 0.f, d11 = xb && yb ? c0[gs + 1] : 0.f;
        orow[j] = d00 * wnw + d10 * wne + d01 * wsw + d11 * wse;
      }
    }
    asm volatile("" ::: "memory");
  }
}

template <typename TO>
__global__ void tokens_kernel(const float* __restrict__ coords, const float* __restrict__ feats, int latent,
                              const float* __restrict__ corr, int64_t ldcorr, int corrdim,
                              const float* __restrict__ pos, int tdim, TO* __restrict__ x, int64_t rows,
                              int S) {
  const int E = latent / 2;
  GRID_STRIDE(i, rows * tdim) {
    const int64_t t = i / tdim;
    const int c = (int)(i % tdim);
    const int64_t t0 = t - (t % S);
    float v;
    if (c < 2 * E + 2) {
      const float fx = coords[t * 2] - coords[t0 * 2], fy = coords[t * 2 + 1] - coords[t0 * 2 + 1];
      if (c >= 2 * E) {
        v = c == 2 * E ? fx : fy;
      } else {
        const float a = c < E ? fx : fy;
        const int cc = c < E ? c : c - E;
        const float div = (float)(cc & ~1) * (1000.0f / (float)E);
        v = (cc & 1) ? cosf(a * div) : sinf(a * div);
      }
    } else if (c < 2 * E + 2 + corrdim) {
      v = corr[t * ldcorr + (c - 2 * E - 2)];
    } else if (c < 2 * E + 2 + corrdim + latent) {
      v = feats[t * latent + (c - 2 * E - 2 - corrdim)];
    } else {
      v = 0.f;
    }
    x[i] = from_f32<TO>(v + pos[(t / S) * tdim + c]);
  }
}

// Row-blocked tokens_kernel: the row's flow, frame-0 row and position row are resolved once per
// thread (the flat form paid two 64-bit divisions per element).
template <typename TO>
__global__ void __launch_bounds__(256)
tokens_rows_kernel(const float* __restrict__ coords, const float* __restrict__ feats, int latent,
                   const float* __restrict__ corr, int64_t ldcorr, int corrdim,
                   const float* __restrict__ pos, int tdim, TO* __restrict__ x, RowBlock rb, int S) {
  const int rl = threadIdx.x / rb.R;
  const int t = blockIdx.x * rb.RB + rl;
  if (rl >= rb.RB || t >= rb.nrows) return;
  const int E = latent / 2;
  const int bn = t / S, t0 = bn * S;
  const float fx = coords[(int64_t)t * 2] - coords[(int64_t)t0 * 2];
  const float fy = coords[(int64_t)t * 2 + 1] - coords[(int64_t)t0 * 2 + 1];
  const float* prow = pos + (int64_t)bn * tdim;
  const float* crow = corr + (int64_t)t * ldcorr;
  const float* frow = feats + (int64_t)t * latent;
  TO* xrow = x + (int64_t)t * tdim;
  const int step = rb.R > 256 ? 256 : rb.R;
  for (int c = threadIdx.x - rl * rb.R; c < tdim; c += step) {
    float v;
    if (c < 2 * E + 2) {
      if (c >= 2 * E) {
        v = c == 2 * E ? fx : fy;
      } else {
        const float a = c < E ? fx : fy;
        const int cc = c < E ? c : c - E;
        const float div = (float)(cc & ~1) * (1000.0f / (float)E);
        v = (cc & 1) ? cosf(a * div) : sinf(a * div);
      }
    } else if (c < 2 * E + 2 + corrdim) {
      v = crow[c - 2 * E - 2];
    } else if (c < 2 * E + 2 + corrdim + latent) {
      v = frow[c - 2 * E - 2 - corrdim];
    } else {
      v = 0.f;
    }
    xrow[c] = from_f32<TO>(v + prow[c]);
  }
}

// One wave per token row, 4 consecutive columns per lane step (tdim % 4 == 0): the row's flow,
// frame-0 row and position row resolved once per wave, 8-B (bf16) / 16-B (f32) stores instead of the
// row-blocked kernel's 2-B ones (its 664-column rows also left 90 of 256 threads idle per block)
template <typename TO>
__global__ void __launch_bounds__(256)
tokens_wave4_kernel(const float* __restrict__ coords, const float* __restrict__ feats, int latent,
                    const float* __restrict__ corr, int64_t ldcorr, int corrdim,
                    const float* __restrict__ pos, int tdim, TO* __restrict__ x, int64_t ldx, int64_t rows, int S,
                    int pairs) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= rows) return;
  const int lane = threadIdx.x & 63;
  const int E = latent / 2, c_corr = 2 * E + 2, c_feat = c_corr + corrdim, c_pad = c_feat + latent;
  const int64_t bn = t / S, t0 = bn * S;
  const float fx = coords[t * 2] - coords[t0 * 2];
  const float fy = coords[t * 2 + 1] - coords[t0 * 2 + 1];
  const float* prow = pos + bn * tdim;
  const float* crow = corr + t * ldcorr;
  const float* frow = feats + t * latent;
  TO* xrow = x + t * ldx;
  const float dscale = 1000.0f / (float)E;
  for (int c0 = 4 * lane; c0 < ldx; c0 += 256) {
    float v[4];
    if (c0 >= tdim) {  // row padding (ldx > tdim: K of the consuming GEMM rounded up to its k-tile)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = 0.f;
      storen<4>(xrow + c0, v);
      continue;
    }
    loadn<4>(prow + c0, v);
    if (pairs && c0 < 2 * E && E % 2 == 0) {
      // flow embedding: columns (2k, 2k + 1) are sin and cos of one argument (E and c0 even: a pair
      // never straddles the x / y halves) -- one sincosf per pair, the values of sinf / cosf
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const int c = c0 + e;
        const float a = c < E ? fx : fy;
        const int cc = c < E ? c : c - E;
        float sn, cs;
        sincosf(a * ((float)cc * dscale), &sn, &cs);
        v[e] += sn;
        v[e + 1] += cs;
      }
      storen<4>(xrow + c0, v);
      continue;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      float u;
      if (c < 2 * E) {
        const float a = c < E ? fx : fy;
        const int cc = c < E ? c : c - E;
        const float arg = a * ((float)(cc & ~1) * dscale);
        u = (cc & 1) ? cosf(arg) : sinf(arg);
      } else if (c < c_corr) {
        u = c == 2 * E ? fx : fy;
      } else if (c < c_feat) {
        u = crow[c - c_corr];
      } else if (c < c_pad) {
        u = frow[c - c_feat];
      } else {
        u = 0.f;
      }
      v[e] += u;
    }
    storen<4>(xrow + c0, v);
  }
}

// coords[t] += delta[t, 0:2] for s > 0 (frame 0 pinned, base_track_predictor.py:247-254);
// preds[it][b, s, n] = coords * scale (layout [B, S, N, 2]).
template <typename TD>
__global__ void coords_update_kernel(float* __restrict__ coords, const TD* __restrict__ delta, int64_t ldd,
                                     float* __restrict__ preds, float scale, int64_t B, int64_t N, int S) {
  GRID_STRIDE(t, B * N * S) {
    const int s = (int)(t % S);
    const int64_t bn = t / S, b = bn / N, n = bn % N;
    float x = coords[t * 2], y = coords[t * 2 + 1];
    if (s > 0) {
      x += to_f32(delta[t * ldd]);
      y += to_f32(delta[t * ldd + 1]);
      coords[t * 2] = x;
      coords[t * 2 + 1] = y;
    }
    if (preds) {
      const int64_t o = ((b * S + s) * N + n) * 2;
      preds[o] = x * scale;
      preds[o + 1] = y * scale;
    }
  }
}

// avg_pool2d(2, stride 2) on NHWC
template <typename T>
__global__ void avgpool2_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int H, int W, int C) {
  const int OH = H / 2, OW = W / 2;
  GRID_STRIDE(i, n * OH * OW * C) {
    const int c = (int)(i % C);
    const int64_t p = i / C;
    const int ox = (int)(p % OW), oy = (int)((p / OW) % OH);
    const int64_t b = p / ((int64_t)OW * OH);
    const T* base = x + ((b * H + 2 * oy) * W + 2 * ox) * C + c;
    const float s = to_f32(base[0]) + to_f32(base[C]) + to_f32(base[(int64_t)W * C]) + to_f32(base[(int64_t)W * C + C]);
    y[i] = from_f32<T>(s * 0.25f);
  }
}

// Row-blocked, 8 channels (16 B of bf16 / 2 x 16 B of f32) per item (C % 8 == 0, aligned).
template <typename T>
__global__ void __launch_bounds__(256)
avgpool2_rows_kernel(const T* __restrict__ x, T* __restrict__ y, RowBlock rb, int H, int W, int C) {
  const int rl = threadIdx.x / rb.R;
  const int row = blockIdx.x * rb.RB + rl;
  if (rl >= rb.RB || row >= rb.nrows) return;
  const int OH = H / 2, OW = W / 2, cg8 = C / 8;
  const int b = row / OH, oy = row - b * OH;
  const T* r0 = x + ((int64_t)b * H + 2 * oy) * W * C;
  const T* r1 = r0 + (int64_t)W * C;
  T* yrow = y + (int64_t)row * OW * C;
  const int step = rb.R > 256 ? 256 : rb.R;
  for (int it = threadIdx.x - rl * rb.R; it < rb.R; it += step) {
    const int ox = it / cg8, cg = it - ox * cg8;
    const int64_t o = (int64_t)(2 * ox) * C + cg * 8;
    float a[8], bq[8], cq[8], d[8], out[8];
    load8(r0 + o, a);
    load8(r0 + o + C, bq);
    load8(r1 + o, cq);
    load8(r1 + o + C, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = (a[e] + bq[e] + cq[e] + d[e]) * 0.25f;
    store8(yrow + (int64_t)ox * C + cg * 8, out);
  }
}

// refine_track.py:74-131: integer patch origins, 31x31 RGB patches (NHWC) and the fine query points.
// images [B, S, 3, H, W] f32; coarse [B, S, N, 2]; patches [B*N*S, P, P, 3] in (b, n, s) order
// (the rearrange '(b s n) -> (b n) s' of refine_track.py:123 folded into the gather);
// topleft [B, S, N, 2] (int, unclamped), query [B*N, 2] = frac(coarse[:, 0]) + pradius.
template <typename TO>
__global__ void patch_gather_kernel(const float* __restrict__ images, const float* __restrict__ coarse,
                                    TO* __restrict__ patches, int* __restrict__ topleft, float* __restrict__ query,
                                    int64_t B, int S, int64_t N, int H, int W, int pradius, int cpad) {
  const int P = 2 * pradius + 1;
  GRID_STRIDE(q, B * S * N * P * P) {  // one thread per patch pixel, cpad channels (3.. zero)
    const int px = (int)(q % P), py = (int)((q / P) % P);
    const int64_t tp = q / ((int64_t)P * P);  // patch order (b*N + n)*S + s (fine-tracker layout)
    const int sp = (int)(tp % S);
    const int64_t np_ = (tp / S) % N, bp = tp / ((int64_t)S * N);
    const int64_t t = (bp * S + sp) * N + np_;  // coarse / topleft order (b*S + s)*N + n
    const float cx = coarse[t * 2], cy = coarse[t * 2 + 1];
    const int ix = (int)floorf(cx), iy = (int)floorf(cy);
    const int tlx = ix - pradius, tly = iy - pradius;
    const int lim = H - P;  // the reference clamps both axes with H (assumes H == W)
    const int x0 = tlx < 0 ? 0 : (tlx > lim ? lim : tlx);
    const int y0 = tly < 0 ? 0 : (tly > lim ? lim : tly);
    const int64_t bs = t / N;
    // the patch must lie inside the frame: the reference's H-for-both-axes clamp needs W >= H, and
    // a NaN track coordinate has no defined floor
    COMET_DASSERT(x0 >= 0 && x0 + P <= W && y0 >= 0 && y0 + P <= H && cx == cx && cy == cy);
    const int64_t pix = (int64_t)(y0 + py) * W + (x0 + px), plane = (int64_t)H * W;
    const float* src = images + bs * 3 * plane + pix;
    TO* dst = patches + q * cpad;
    if (cpad == 8) {
      float v[8] = {src[0], src[plane], src[2 * plane], 0.f, 0.f, 0.f, 0.f, 0.f};
      store8(dst, v);
    } else {
      for (int c = 0; c < cpad; ++c) dst[c] = from_f32<TO>(c < 3 ? src[c * plane] : 0.f);
    }
    if (px == 0 && py == 0) {
      topleft[t * 2] = tlx;
      topleft[t * 2 + 1] = tly;
      const int s = (int)(bs % S);
      if (s == 0) {
        const int64_t b = bs / S, n = t % N;
        query[(b * N + n) * 2] = (cx - (float)ix) + (float)pradius;
        query[(b * N + n) * 2 + 1] = (cy - (float)iy) + (float)pradius;
      }
    }
  }
}

// NCHW RGB f32 -> channels-last [n, oh, ow, cpad] (channels 3.. zero) in the compute dtype, with the
// align_corners bilinear resize of track_predictor.py:137 when (oh, ow) != (H, W).
template <typename TO>
__global__ void images_nhwc_kernel(const float* __restrict__ x, TO* __restrict__ y, int64_t n, int H, int W,
                                   int oh, int ow, int cpad) {
  GRID_STRIDE(q, n * oh * ow) {
    const int ox = (int)(q % ow);
    const int64_t t = q / ow;
    const int oy = (int)(t % oh);
    const int64_t ni = t / oh;
    const float* xb = x + ni * 3 * (int64_t)H * W;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (oh == H && ow == W) {
      for (int c = 0; c < 3; ++c) v[c] = xb[((int64_t)c * H + oy) * W + ox];
    } else {
      const float sy = oh > 1 ? (float)(H - 1) / (float)(oh - 1) : 0.f;
      const float sx = ow > 1 ? (float)(W - 1) / (float)(ow - 1) : 0.f;
      const float fy = sy * (float)oy, fx = sx * (float)ox;
      int y0 = (int)fy, x0 = (int)fx;
      y0 = y0 > H - 1 ? H - 1 : y0;
      x0 = x0 > W - 1 ? W - 1 : x0;
      const int y1 = y0 + 1 < H ? y0 + 1 : H - 1, x1 = x0 + 1 < W ? x0 + 1 : W - 1;
      const float ly = fy - (float)y0, lx = fx - (float)x0;
      for (int c = 0; c < 3; ++c) {
        const float* pl = xb + (int64_t)c * H * W;
        const float v00 = pl[(int64_t)y0 * W + x0], v01 = pl[(int64_t)y0 * W + x1];
        const float v10 = pl[(int64_t)y1 * W + x0], v11 = pl[(int64_t)y1 * W + x1];
        v[c] = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
      }
    }
    TO* dst = y + q * cpad;
    if (cpad == 8) {
      store8(dst, v);
    } else {
      for (int c = 0; c < cpad; ++c) dst[c] = from_f32<TO>(v[c]);
    }
  }
}

// refined[b, s, n] = fine_last[(b*N+n), s] + topleft[b, s, n]; frame 0 = coarse query point.
__global__ void refine_combine_kernel(const float* __restrict__ fine, const int* __restrict__ topleft,
                                      const float* __restrict__ coarse, float* __restrict__ refined,
                                      int64_t B, int S, int64_t N) {
  GRID_STRIDE(t, B * S * N) {
    const int64_t n = t % N, bs = t / N, s = bs % S, b = bs / S;
    if (s == 0) {
      refined[t * 2] = coarse[(b * S * N + n) * 2];
      refined[t * 2 + 1] = coarse[(b * S * N + n) * 2 + 1];
    } else {
      const int64_t f = ((b * N + n) * S + s) * 2;
      refined[t * 2] = fine[f] + (float)topleft[t * 2];
      refined[t * 2 + 1] = fine[f + 1] + (float)topleft[t * 2 + 1];
    }
  }
}

// compute_score_fn (refine_track.py:174-278) + score inversion (E2Epose2.py:232-236), one thread
// per (b, n). Reproduces the reference's indexing: the feature map of every window is patch
// (s = 0, n = 0) of the sequence (batch_indices = arange(B) indexes the flat (b s n) axis), and
// the window origin for output (b, s, n) is read from the fine track at flat position
// m = (b*S + s)*N + n of its (b n, s) layout. Window row = clamp(floor(y)-r), col = clamp(floor(x)-r).
template <typename TF>
__global__ void score_kernel(const float* __restrict__ qfeat, const TF* __restrict__ pfeat,
                             const float* __restrict__ fine, float* __restrict__ score,
                             float* __restrict__ inv_score, int64_t B, int S, int64_t N, int P, int C,
                             int sradius) {
  const int ss = 2 * sradius + 1;
  const float lin_step = 2.f / (float)(ss - 1);
  GRID_STRIDE(t, B * N) {
    const int64_t b = t / N, n = t % N;
    const float* q = qfeat + t * C;
    // feature map f = patch (b, s=0, n=0): row (b*N + 0) of [B*N, S, P, P, C], frame 0
    const TF* fm = pfeat + (b * N * S) * (int64_t)P * P * C;
    float inv_max = 0.f;
    for (int s = 0; s < S; ++s) {
      float sc = 1.f;
      if (s > 0) {
        const int64_t m = (b * S + s) * N + n;  // flat (b s n) position
        const int64_t bn2 = m / S;              // read in (b n, s) order
        const int s2 = (int)(m % S);
        const float fx = fine[(bn2 * S + s2) * 2], fy = fine[(bn2 * S + s2) * 2 + 1];
        int tx = (int)floorf(fx) - sradius, ty = (int)floorf(fy) - sradius;
        const int lim = P - ss;
        tx = tx < 0 ? 0 : (tx > lim ? lim : tx);
        ty = ty < 0 ? 0 : (ty > lim ? lim : ty);
        float sim[25];
        float mx = -INFINITY;
        for (int a = 0; a < ss; ++a)
          for (int c2 = 0; c2 < ss; ++c2) {
            const TF* pix = fm + ((int64_t)(ty + a) * P + (tx + c2)) * C;
            float d = 0.f;
            for (int c = 0; c < C; ++c) d += q[c] * to_f32(pix[c]);
            d *= 1.f / sqrtf((float)C);
            sim[a * ss + c2] = d;
            mx = fmaxf(mx, d);
          }
        float den = 0.f;
        for (int k = 0; k < ss * ss; ++k) { sim[k] = expf(sim[k] - mx); den += sim[k]; }
        float ex = 0.f, ey = 0.f, ex2 = 0.f, ey2 = 0.f;
        for (int a = 0; a < ss; ++a)
          for (int c2 = 0; c2 < ss; ++c2) {
            const float p = sim[a * ss + c2] / den;
            const float gx = -1.f + lin_step * (float)c2, gy = -1.f + lin_step * (float)a;
            ex += p * gx; ey += p * gy; ex2 += p * gx * gx; ey2 += p * gy * gy;
          }
        sc = sqrtf(fmaxf(ex2 - ex * ex, 1e-10f)) + sqrtf(fmaxf(ey2 - ey * ey, 1e-10f));
      }
      score[(b * S + s) * N + n] = sc;
      const float iv = 1.f / (sc + 1e-6f);
      inv_score[(b * S + s) * N + n] = iv;
      inv_max = fmaxf(inv_max, iv);
    }
    for (int s = 0; s < S; ++s) inv_score[(b * S + s) * N + n] /= inv_max;
  }
}

// Parallel form of score_kernel (the per-track loop ran 4096 threads for the whole chip): one
// thread per (b, s, n) window, channels 8 at a time (C % 8 == 0), then a per-track pass that
// divides by the max inverse score over s. Same arithmetic and reads as score_kernel.
template <typename TF>
__global__ void __launch_bounds__(256)
score_items_kernel(const float* __restrict__ qfeat, const TF* __restrict__ pfeat, const float* __restrict__ fine,
                   float* __restrict__ score, float* __restrict__ inv_score, int B, int S, int N, int P, int C,
                   int sradius) {
  const int item = blockIdx.x * 256 + threadIdx.x;  // (b*S + s)*N + n
  if (item >= B * S * N) return;
  const int n = item % N, t = item / N, s = t % S, b = t / S;
  float sc = 1.f;
  if (s > 0) {
    const int ss = 2 * sradius + 1;
    const float lin_step = 2.f / (float)(ss - 1);
    const float* q = qfeat + ((int64_t)b * N + n) * C;
    const TF* fm = pfeat + ((int64_t)b * N * S) * P * P * C;
    const int m = item;  // flat (b s n) position, read in (b n, s) order
    const int bn2 = m / S, s2 = m - bn2 * S;
    const float fx = fine[((int64_t)bn2 * S + s2) * 2], fy = fine[((int64_t)bn2 * S + s2) * 2 + 1];
    int tx = (int)floorf(fx) - sradius, ty = (int)floorf(fy) - sradius;
    const int lim = P - ss;
    tx = tx < 0 ? 0 : (tx > lim ? lim : tx);
    ty = ty < 0 ? 0 : (ty > lim ? lim : ty);
    float sim[25];
    float mx = -INFINITY;
    const float rs = 1.f / sqrtf((float)C);
    for (int a = 0; a < ss; ++a)
      for (int c2 = 0; c2 < ss; ++c2) {
        const TF* pix = fm + ((int64_t)(ty + a) * P + (tx + c2)) * C;
        float d = 0.f;
        for (int c = 0; c < C; c += 8) {
          float pv[8], qv[8];
          load8(pix + c, pv);
          load8(q + c, qv);
#pragma unroll
          for (int e = 0; e < 8; ++e) d += qv[e] * pv[e];
        }
        d *= rs;
        sim[a * ss + c2] = d;
        mx = fmaxf(mx, d);
      }
    float den = 0.f;
    for (int k = 0; k < ss * ss; ++k) { sim[k] = expf(sim[k] - mx); den += sim[k]; }
    float ex = 0.f, ey = 0.f, ex2 = 0.f, ey2 = 0.f;
    for (int a = 0; a < ss; ++a)
      for (int c2 = 0; c2 < ss; ++c2) {
        const float p = sim[a * ss + c2] / den;
        const float gx = -1.f + lin_step * (float)c2, gy = -1.f + lin_step * (float)a;
        ex += p * gx; ey += p * gy; ex2 += p * gx * gx; ey2 += p * gy * gy;
      }
    sc = sqrtf(fmaxf(ex2 - ex * ex, 1e-10f)) + sqrtf(fmaxf(ey2 - ey * ey, 1e-10f));
  }
  score[item] = sc;
  inv_score[item] = 1.f / (sc + 1e-6f);
}

__global__ void __launch_bounds__(256)
score_norm_kernel(float* __restrict__ inv_score, int B, int S, int N) {
  const int t = blockIdx.x * 256 + threadIdx.x;  // b*N + n
  if (t >= B * N) return;
  const int b = t / N, n = t - b * N;
  float mx = 0.f;
  for (int s = 0; s < S; ++s) mx = fmaxf(mx, inv_score[((int64_t)b * S + s) * N + n]);
  for (int s = 0; s < S; ++s) inv_score[((int64_t)b * S + s) * N + n] /= mx;
}

// DINOv2 input: x [BS, 3, H, W] f32 -> bilinear(align_corners) to R x R -> (x - mean)/std ->
// patch rows cols[(f*g + py)*g + px][ci*p*p + ky*p + kx] (conv weight flatten order), K padded.
template <typename TO>
__global__ void dino_prep_kernel(const float* __restrict__ x, TO* __restrict__ cols, int64_t BS, int H, int W,
                                 int R, int patch, int64_t ldc, float m0, float m1, float m2, float s0, float s1,
                                 float s2) {
  const int g = R / patch;
  const int kk = 3 * patch * patch;
  const float scy = R > 1 ? (float)(H - 1) / (float)(R - 1) : 0.f;
  const float scx = R > 1 ? (float)(W - 1) / (float)(R - 1) : 0.f;
  GRID_STRIDE(i, BS * g * g * ldc) {
    const int64_t col = i % ldc, row = i / ldc;
    if (col >= kk) { cols[i] = from_f32<TO>(0.f); continue; }
    const int ci = (int)(col / (patch * patch)), ky = (int)((col / patch) % patch), kx = (int)(col % patch);
    const int px = (int)(row % g), py = (int)((row / g) % g);
    const int64_t f = row / ((int64_t)g * g);
    const int oy = py * patch + ky, ox = px * patch + kx;
    const float sy = scy * (float)oy, sx = scx * (float)ox;
    int y0 = (int)sy; if (y0 > H - 1) y0 = H - 1;
    int x0 = (int)sx; if (x0 > W - 1) x0 = W - 1;
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
    const float ly = sy - (float)y0, lx = sx - (float)x0;
    const float* pl = x + (f * 3 + ci) * (int64_t)H * W;
    const float v = (1.f - ly) * ((1.f - lx) * pl[(int64_t)y0 * W + x0] + lx * pl[(int64_t)y0 * W + x1]) +
                    ly * ((1.f - lx) * pl[(int64_t)y1 * W + x0] + lx * pl[(int64_t)y1 * W + x1]);
    const float mean = ci == 0 ? m0 : (ci == 1 ? m1 : m2);
    const float sd = ci == 0 ? s0 : (ci == 1 ? s1 : s2);
    cols[i] = from_f32<TO>((v - mean) / sd);
  }
}

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_sample_bilinear(int dtype, const void* fmap, int64_t bstride, int H, int W, int C,
                                     const float* coords, int64_t cstride_b, int64_t cstride_r, float* out,
                                     int64_t ostride_b, int64_t ostride_r, int64_t B, int64_t R, int border,
                                     void* stream) {
  COMET_CHECK_ARG(fmap && coords && out && H > 0 && W > 0 && C > 0, "comet_sample_bilinear: bad args");
  if (B * R == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  dim3 g((unsigned)cdiv(B * R, 4));
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((sample_kernel<float>), g, dim3(256), 0, s, (const float*)fmap, bstride, H, W, C, coords,
                       cstride_b, cstride_r, out, ostride_b, ostride_r, B, R, border);
  else
    hipLaunchKernelGGL((sample_kernel<__bf16>), g, dim3(256), 0, s, (const __bf16*)fmap, bstride, H, W, C, coords,
                       cstride_b, cstride_r, out, ostride_b, ostride_r, B, R, border);
  COMET_CHECK_LAUNCH("comet_sample_bilinear");
  return COMET_OK;
}

extern "C" int comet_corr_sample(int dtype_fmap, int dtype_feat, const void* const* pyramid, const int* heights,
                                 const int* widths, int levels, int radius, int C, const void* feats,
                                 const float* coords, float* out, int64_t ldo, int64_t col0, int64_t B,
                                 int64_t N, int S, void* stream) {
  COMET_CHECK_ARG(levels >= 1 && levels <= 8 && radius >= 1 && radius <= 6, "comet_corr_sample: levels in [1,8], radius in [1,6]");
  COMET_CHECK_ARG(C == 128 || C == 32, "comet_corr_sample: C must be 128 (coarse) or 32 (fine)");
  COMET_CHECK_ARG(pyramid && heights && widths && feats && coords && out, "comet_corr_sample: null pointer");
  COMET_CHECK_ARG(dtype_feat == COMET_F32, "comet_corr_sample: track features must be f32");
  const int64_t T = B * N * S;
  if (T == 0) return COMET_OK;
  COMET_CHECK_ARG(T < (1ll << 31), "comet_corr_sample: too many tracks");
  PyrTab tab{};
  for (int l = 0; l < levels; ++l) {
    COMET_CHECK_ARG(pyramid[l] != nullptr, "comet_corr_sample: null level");
    tab.p[l] = pyramid[l]; tab.h[l] = heights[l]; tab.w[l] = widths[l];
  }
  hipStream_t s = as_stream(stream);
  const float isc = 1.f / sqrtf((float)C);
  const bool valu = std::getenv("COMET_CORR_VALU") != nullptr;  // the VALU kernel for every shape (A/B, tests)
  if (dtype_fmap == COMET_BF16 && C == 128 && N >= 16 && !valu) {
    // matrix-core path (corr_mfma_kernel): 4 waves x 16 tracks per workgroup
    const int gs = 2 * radius + 4, sort = N <= 2048;
    const size_t lds = (size_t)4 * 16 * gs * gs * 4 + 64 * 4 + (sort ? (size_t)((N + 3) & ~3) * 4 : 0);
    const int64_t frames = B * S, grid = (frames + 7) / 8 * 8 * ((N + 63) / 64);
    COMET_CHECK_ARG(grid < (1ll << 31) && N < (1ll << 30), "comet_corr_sample: too many tracks");
    const char* rs = std::getenv("COMET_CORR_RING");
    const int ring = rs ? std::atoi(rs) : 2;
    // default: the 2-deep ring at 4 waves per SIMD (128 VGPRs; 242 vs 274 us at 3 waves, profiles/r04_corr)
    const bool occ3 = std::getenv("COMET_CORR_OCC3") != nullptr || rs != nullptr;
#define CM(R, O) hipLaunchKernelGGL((corr_mfma_kernel<128, R, O>), dim3((unsigned)grid), dim3(256), lds, s, tab, levels, \
                                    radius, (const float*)feats, coords, out, ldo, col0, (int)N, S, (int)frames, isc, sort)
    if (!occ3) CM(2, 4); else if (ring >= 4) CM(4, 1); else if (ring == 3) CM(3, 1); else CM(2, 1);
#undef CM
    COMET_CHECK_LAUNCH("comet_corr_sample");
    return COMET_OK;
  }
  if (C == 32 && std::getenv("COMET_CORR_BLOCK") == nullptr) {
    // the fine tracker: one wave per track row (corr_wave_kernel; COMET_CORR_BLOCK=1: a workgroup per row)
#define CW(TF) hipLaunchKernelGGL((corr_wave_kernel<TF, float, 32>), dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, tab, \
                                  levels, radius, (const float*)feats, coords, out, ldo, col0, N, S, isc, T)
    if (dtype_fmap == COMET_F32) CW(float); else CW(__bf16);
#undef CW
    COMET_CHECK_LAUNCH("comet_corr_sample");
    return COMET_OK;
  }
#define CK(TF, CC) hipLaunchKernelGGL((corr_kernel<TF, float, CC>), dim3((unsigned)T), dim3(256), 0, s, tab, levels, radius, (const float*)feats, coords, out, ldo, col0, N, S, isc)
  if (dtype_fmap == COMET_F32) { if (C == 128) CK(float, 128); else CK(float, 32); }
  else { if (C == 128) CK(__bf16, 128); else CK(__bf16, 32); }
#undef CK
  COMET_CHECK_LAUNCH("comet_corr_sample");
  return COMET_OK;
}

extern "C" int comet_tracker_tokens(int dtype_out, const float* coords, const float* feats, int latent,
                                    const float* corr, int64_t ldcorr, int corrdim, const float* pos, int tdim,
                                    void* x, int64_t ldx, int64_t rows, int S, void* stream) {
  COMET_CHECK_ARG(coords && feats && corr && pos && x && tdim >= latent * 2 + 2 + corrdim && ldx >= tdim,
                  "comet_tracker_tokens: bad args");
  if (rows == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  const bool al = ((uintptr_t)x % (dtype_out == COMET_F32 ? 16 : 8)) == 0 && (uintptr_t)pos % 16 == 0;
  const bool wave4 = tdim % 4 == 0 && ldx % 4 == 0 && al && S > 0;
  COMET_CHECK_ARG(ldx == tdim || wave4, "comet_tracker_tokens: padded rows (ldx > tdim) need tdim, ldx % 4 == 0 and "
                                        "aligned x / pos");
  if (wave4 && (ldx != tdim || (getenv("COMET_TOKENS_ROWS") == nullptr && getenv("COMET_TOKENS_FLAT") == nullptr))) {
    const unsigned gr = (unsigned)cdiv(rows, 4);
    const int pairs = getenv("COMET_TOKENS_NO_SINCOS") == nullptr;  // measurement: sinf / cosf per column
    if (dtype_out == COMET_F32)
      hipLaunchKernelGGL((tokens_wave4_kernel<float>), dim3(gr), dim3(256), 0, s, coords, feats, latent, corr, ldcorr, corrdim, pos, tdim, (float*)x, ldx, rows, S, pairs);
    else
      hipLaunchKernelGGL((tokens_wave4_kernel<__bf16>), dim3(gr), dim3(256), 0, s, coords, feats, latent, corr, ldcorr, corrdim, pos, tdim, (__bf16*)x, ldx, rows, S, pairs);
  } else if (rows < (1ll << 31) && S > 0 && getenv("COMET_TOKENS_FLAT") == nullptr) {
    const RowBlock rb = make_rowblock(rows, tdim);
    const unsigned gr = (unsigned)cdiv(rb.nrows, rb.RB);
    if (dtype_out == COMET_F32)
      hipLaunchKernelGGL((tokens_rows_kernel<float>), dim3(gr), dim3(256), 0, s, coords, feats, latent, corr, ldcorr, corrdim, pos, tdim, (float*)x, rb, S);
    else
      hipLaunchKernelGGL((tokens_rows_kernel<__bf16>), dim3(gr), dim3(256), 0, s, coords, feats, latent, corr, ldcorr, corrdim, pos, tdim, (__bf16*)x, rb, S);
  } else if (dtype_out == COMET_F32)
    hipLaunchKernelGGL((tokens_kernel<float>), dim3(g1d(rows * tdim)), dim3(256), 0, s, coords, feats, latent, corr, ldcorr, corrdim, pos, tdim, (float*)x, rows, S);
  else
    hipLaunchKernelGGL((tokens_kernel<__bf16>), dim3(g1d(rows * tdim)), dim3(256), 0, s, coords, feats, latent, corr, ldcorr, corrdim, pos, tdim, (__bf16*)x, rows, S);
  COMET_CHECK_LAUNCH("comet_tracker_tokens");
  return COMET_OK;
}

extern "C" int comet_coords_update(int dtype_delta, float* coords, const void* delta, int64_t ldd, float* preds,
                                   float scale, int64_t B, int64_t N, int S, void* stream) {
  COMET_CHECK_ARG(coords && delta, "comet_coords_update: null pointer");
  if (B * N * S == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (dtype_delta == COMET_F32)
    hipLaunchKernelGGL((coords_update_kernel<float>), dim3(g1d(B * N * S)), dim3(256), 0, s, coords, (const float*)delta, ldd, preds, scale, B, N, S);
  else
    hipLaunchKernelGGL((coords_update_kernel<__bf16>), dim3(g1d(B * N * S)), dim3(256), 0, s, coords, (const __bf16*)delta, ldd, preds, scale, B, N, S);
  COMET_CHECK_LAUNCH("comet_coords_update");
  return COMET_OK;
}

extern "C" int comet_avgpool2_nhwc(int dtype, const void* x, void* y, int64_t n, int H, int W, int C, void* stream) {
  COMET_CHECK_ARG(x && y && H >= 2 && W >= 2, "comet_avgpool2_nhwc: bad args");
  hipStream_t s = as_stream(stream);
  const int64_t tot = n * (H / 2) * (W / 2) * C;
  if (C % 8 == 0 && ((uintptr_t)x | (uintptr_t)y) % 32 == 0 && n * (H / 2) < (1ll << 31) && getenv("COMET_POOL_FLAT") == nullptr) {
    const RowBlock rb = make_rowblock(n * (H / 2), (int64_t)(W / 2) * (C / 8));
    const unsigned gr = (unsigned)cdiv(rb.nrows, rb.RB);
    if (dtype == COMET_F32)
      hipLaunchKernelGGL((avgpool2_rows_kernel<float>), dim3(gr), dim3(256), 0, s, (const float*)x, (float*)y, rb, H, W, C);
    else
      hipLaunchKernelGGL((avgpool2_rows_kernel<__bf16>), dim3(gr), dim3(256), 0, s, (const __bf16*)x, (__bf16*)y, rb, H, W, C);
    COMET_CHECK_LAUNCH("comet_avgpool2_nhwc");
    return COMET_OK;
  }
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((avgpool2_kernel<float>), dim3(g1d(tot)), dim3(256), 0, s, (const float*)x, (float*)y, n, H, W, C);
  else
    hipLaunchKernelGGL((avgpool2_kernel<__bf16>), dim3(g1d(tot)), dim3(256), 0, s, (const __bf16*)x, (__bf16*)y, n, H, W, C);
  COMET_CHECK_LAUNCH("comet_avgpool2_nhwc");
  return COMET_OK;
}

extern "C" int comet_patch_gather(int dtype_out, const float* images, const float* coarse, void* patches,
                                  int* topleft, float* query, int64_t B, int S, int64_t N, int H, int W,
                                  int pradius, int cpad, void* stream) {
  COMET_CHECK_ARG(images && coarse && patches && topleft && query, "comet_patch_gather: null pointer");
  COMET_CHECK_ARG(H >= 2 * pradius + 1 && W >= 2 * pradius + 1, "comet_patch_gather: image smaller than a patch");
  COMET_CHECK_ARG(cpad >= 3 && cpad <= 8, "comet_patch_gather: cpad must be in [3, 8]");
  COMET_CHECK_ARG(cpad != 8 || (uintptr_t)patches % 32 == 0, "comet_patch_gather: cpad 8 needs a 32-B aligned output");
  const int P = 2 * pradius + 1;
  const int64_t tot = B * S * N * P * P;
  if (tot == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (dtype_out == COMET_F32)
    hipLaunchKernelGGL((patch_gather_kernel<float>), dim3(g1d(tot)), dim3(256), 0, s, images, coarse, (float*)patches, topleft, query, B, S, N, H, W, pradius, cpad);
  else
    hipLaunchKernelGGL((patch_gather_kernel<__bf16>), dim3(g1d(tot)), dim3(256), 0, s, images, coarse, (__bf16*)patches, topleft, query, B, S, N, H, W, pradius, cpad);
  COMET_CHECK_LAUNCH("comet_patch_gather");
  return COMET_OK;
}

extern "C" int comet_images_nhwc(int dtype_out, const float* images, void* out, int64_t n, int H, int W, int oh,
                                 int ow, int cpad, void* stream) {
  COMET_CHECK_ARG(images && out && n > 0 && H > 0 && W > 0 && oh > 0 && ow > 0, "comet_images_nhwc: bad args");
  COMET_CHECK_ARG(cpad >= 3 && cpad <= 8, "comet_images_nhwc: cpad must be in [3, 8]");
  COMET_CHECK_ARG(cpad != 8 || (uintptr_t)out % 32 == 0, "comet_images_nhwc: cpad 8 needs a 32-B aligned output");
  hipStream_t s = as_stream(stream);
  const int64_t tot = n * oh * ow;
  if (dtype_out == COMET_F32)
    hipLaunchKernelGGL((images_nhwc_kernel<float>), dim3(g1d(tot)), dim3(256), 0, s, images, (float*)out, n, H, W, oh, ow, cpad);
  else
    hipLaunchKernelGGL((images_nhwc_kernel<__bf16>), dim3(g1d(tot)), dim3(256), 0, s, images, (__bf16*)out, n, H, W, oh, ow, cpad);
  COMET_CHECK_LAUNCH("comet_images_nhwc");
  return COMET_OK;
}

extern "C" int comet_refine_combine(const float* fine, const int* topleft, const float* coarse, float* refined,
                                    int64_t B, int S, int64_t N, void* stream) {
  COMET_CHECK_ARG(fine && topleft && coarse && refined, "comet_refine_combine: null pointer");
  if (B * S * N == 0) return COMET_OK;
  hipLaunchKernelGGL(refine_combine_kernel, dim3(g1d(B * S * N)), dim3(256), 0, as_stream(stream), fine, topleft,
                     coarse, refined, B, S, N);
  COMET_CHECK_LAUNCH("comet_refine_combine");
  return COMET_OK;
}

extern "C" int comet_track_score(int dtype_feat, const float* qfeat, const void* pfeat, const float* fine,
                                 float* score, float* inv_score, int64_t B, int S, int64_t N, int P, int C,
                                 int sradius, void* stream) {
  COMET_CHECK_ARG(qfeat && pfeat && fine && score && inv_score, "comet_track_score: null pointer");
  COMET_CHECK_ARG(sradius >= 1 && sradius <= 2 && P > 2 * sradius, "comet_track_score: sradius must be 1 or 2");
  if (B * N == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (C % 8 == 0 && (uintptr_t)pfeat % 16 == 0 && (uintptr_t)qfeat % 16 == 0 && B * S * N < (1ll << 31) &&
      getenv("COMET_SCORE_SERIAL") == nullptr) {
    const unsigned g = (unsigned)cdiv(B * S * N, 256), g2 = (unsigned)cdiv(B * N, 256);
    if (dtype_feat == COMET_F32)
      hipLaunchKernelGGL((score_items_kernel<float>), dim3(g), dim3(256), 0, s, qfeat, (const float*)pfeat, fine, score,
                         inv_score, (int)B, S, (int)N, P, C, sradius);
    else
      hipLaunchKernelGGL((score_items_kernel<__bf16>), dim3(g), dim3(256), 0, s, qfeat, (const __bf16*)pfeat, fine, score,
                         inv_score, (int)B, S, (int)N, P, C, sradius);
    hipLaunchKernelGGL(score_norm_kernel, dim3(g2), dim3(256), 0, s, inv_score, (int)B, S, (int)N);
    COMET_CHECK_LAUNCH("comet_track_score");
    return COMET_OK;
  }
  if (dtype_feat == COMET_F32)
    hipLaunchKernelGGL((score_kernel<float>), dim3(g1d(B * N)), dim3(256), 0, s, qfeat, (const float*)pfeat, fine, score, inv_score, B, S, N, P, C, sradius);
  else
    hipLaunchKernelGGL((score_kernel<__bf16>), dim3(g1d(B * N)), dim3(256), 0, s, qfeat, (const __bf16*)pfeat, fine, score, inv_score, B, S, N, P, C, sradius);
  COMET_CHECK_LAUNCH("comet_track_score");
  return COMET_OK;
}

extern "C" int comet_dino_prep(int dtype_out, const float* images, void* cols, int64_t BS, int H, int W, int R,
                               int patch, int64_t ldc, const float* mean3, const float* std3, void* stream) {
  COMET_CHECK_ARG(images && cols && mean3 && std3 && R % patch == 0 && ldc >= 3 * patch * patch, "comet_dino_prep: bad args");
  const int g = R / patch;
  const int64_t tot = BS * g * g * ldc;
  if (tot == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (dtype_out == COMET_F32)
    hipLaunchKernelGGL((dino_prep_kernel<float>), dim3(g1d(tot)), dim3(256), 0, s, images, (float*)cols, BS, H, W, R, patch, ldc,
                       mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  else
    hipLaunchKernelGGL((dino_prep_kernel<__bf16>), dim3(g1d(tot)), dim3(256), 0, s, images, (__bf16*)cols, BS, H, W, R, patch, ldc,
                       mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  COMET_CHECK_LAUNCH("comet_dino_prep");
  return COMET_OK;
}
