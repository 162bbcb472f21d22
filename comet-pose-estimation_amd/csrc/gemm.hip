// Batched MFMA GEMM with fused bias / activation / residual epilogue (comet_gemm).
//
// Replaces nn.Linear / MHA in_proj+out_proj / conv-after-im2col of the reference
// (modules.py:119-154, 248-344; blocks.py:27-348; camera_predictor10.py:75-87,126-280) and the
// head's backward GEMMs (dX = dY.W, dW = dY^T.X).
//
// Tile 128x128, 256 threads = 4 waves (2x2), each wave owns 64x64 = 4x4 MFMA 16x16 tiles.
//
// bf16 kernel: v_mfma_f32_16x16x32_bf16, BK = 64 (two 32-deep MFMA steps per k-tile).
//   Each operand keeps the LDS image its global layout gives for free:
//   * k-contiguous (layout 0): [128 rows][64 k + 8 pad]   (144-B pitch: ds_read_b128, conflict-free)
//   * row-contiguous (layout 1): [64 k][128 rows + 16 pad] (288-B pitch), fragments read with
//     ds_read_b64_tr_b16 (lane gets 4 k of one row per read, two reads = the 8 k of a fragment).
//     k rows are stored with bits 2 and 3 of k swapped so the 8 rows one half-wave reads fall on
//     8 distinct 32-B bank groups.
//   Global -> register staging, write of tile t+1 after the barrier of tile t-1, loads of tile t+2
//   issued right after (one barrier per k-tile).
// f32 kernel (parity precision): v_mfma_f32_16x16x4_f32, BK = 16, both operands k-contiguous in LDS.
//
// Split-K: when the output has fewer tiles than the chip has CUs and K is long (the weight-gradient
// GEMMs: K = all tokens of the batch), blockIdx.z splits K; every split writes an f32 partial tile
// into the caller's workspace and a second kernel sums the splits in a fixed order (deterministic)
// and applies the epilogue.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace comet {


namespace {

constexpr int BM = 128, BN = 128, NT = 256;

struct Epi {
  const float* bias; int bias_mode; int64_t sb0, sb1;
  const void* resid; int64_t ldr, sr0, sr1; float beta;
  void* aux; int64_t ldaux, sx0, sx1;
  float alpha; int act;
  int vec;  // output / resid / aux rows allow 8-wide vector access (host-checked)
  int wide = 0;  // persistent kernel: 16-B bf16 stores (C 16-B aligned, ldc % 8 == 0; host-checked)
  int prio = 0;  // persistent kernel: s_setprio 1 for waves 4-7 (COMET_GEMM_PRIO=1, measurement)
  int bpark = 0;  // persistent kernel: bf16-park epilogue (COMET_GEMM_NO_BPARK=1: the direct / f32-park paths)
  int raster = 0;  // persistent kernel: per-XCD contiguous tile ranges (COMET_GEMM_RASTER=1, measurement)
  // 256-row kernel, DACT instances (comet_gemm_dact): C = act'(pre) * acc with pre [M, N] bf16 at
  // row pitch ldg, and dcol[n] += sum over rows of the stored (rounded) values
  const __bf16* gpre = nullptr; int64_t ldg = 0; float* dcol = nullptr;
};

// Split-K partials: ws[((z * nb) + bz) * M * N + row * N + col], f32.
struct Split {
  float* ws; int64_t kchunk;  // k range of split z: [z*kchunk, min(K, (z+1)*kchunk))
};

template <typename TC>
__device__ __forceinline__ void epi_store(const Epi& epi, TC* __restrict__ C, int64_t ldc,
                                          const TC* R, TC* X, const float* bias,
                                          int64_t row, int64_t col, float acc) {
  float v = epi.alpha * acc;
  if (bias) v += epi.bias_mode == 1 ? bias[col] : bias[row];
  if (X) X[row * epi.ldaux + col] = from_f32<TC>(v);
  v = apply_act(epi.act, v);
  if (R) v += epi.beta * to_f32(R[row * epi.ldr + col]);
  C[row * ldc + col] = from_f32<TC>(v);
}

// Write the 128x128 accumulator tile: either the fused epilogue or the raw split-K partial.
template <typename TC, bool SPLIT>
__device__ __forceinline__ void write_tile(const f32x4 (&acc)[4][4], const Epi& epi, TC* __restrict__ C,
                                           int64_t ldc, int64_t b0, int64_t b1, int64_t bz,
                                           int64_t m0, int64_t n0, int64_t M, int64_t N,
                                           const Split& sp, int wm, int wn, int lane) {
  const int cl = lane & 15, rq = (lane >> 4) * 4;
  if (SPLIT) {
    float* W = sp.ws + ((int64_t)blockIdx.z * gridDim.y + bz) * M * N;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t col = n0 + wn * 64 + j * 16 + cl;
      if (col >= N) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = m0 + wm * 64 + i * 16 + rq + r;
          if (row < M) W[row * N + col] = acc[i][j][r];
        }
    }
    return;
  }
  const TC* R = epi.resid ? reinterpret_cast<const TC*>(epi.resid) + b0 * epi.sr0 + b1 * epi.sr1 : nullptr;
  TC* X = epi.aux ? reinterpret_cast<TC*>(epi.aux) + b0 * epi.sx0 + b1 * epi.sx1 : nullptr;
  const float* bias = epi.bias ? epi.bias + b0 * epi.sb0 + b1 * epi.sb1 : nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = n0 + wn * 64 + j * 16 + cl;
    if (col >= N) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + rq + r;
        if (row < M) epi_store<TC>(epi, C, ldc, R, X, bias, row, col, acc[i][j][r]);
      }
  }
}

// Epilogue through LDS (bf16 kernel): the 128x128 f32 accumulator tile is parked in LDS, then each
// thread owns 8 consecutive columns of 8 rows, so bias / residual / aux / output move as 16-B
// (bf16) or 32-B (f32) vectors instead of 2-4-B column-strided scalars.
constexpr int CP = 132;  // f32 pitch of the parked tile: conflict-free fragment writes

template <typename TC, bool SPLIT, int MI = 4>
__device__ __forceinline__ void write_tile_lds(const f32x4 (&acc)[MI][4], float* __restrict__ cs,
                                               const Epi& epi, TC* __restrict__ C, int64_t ldc,
                                               int64_t b0, int64_t b1, int64_t bz, int64_t m0, int64_t n0,
                                               int64_t M, int64_t N, const Split& sp, int wm, int wn, int lane) {
  const int cl = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[(wm * 16 * MI + i * 16 + rq + r) * CP + wn * 64 + j * 16 + cl] = acc[i][j][r];
  __syncthreads();
  const int t = threadIdx.x, cg = t & 15, rb = t >> 4;
  const int64_t col0 = n0 + cg * 8;
  if (col0 >= N) return;
  const bool full = epi.vec && col0 + 8 <= N;
  if (SPLIT) {
    float* W = sp.ws + ((int64_t)blockIdx.z * gridDim.y + bz) * M * N;
#pragma unroll 2
    for (int q = 0; q < 8; ++q) {
      const int64_t row = m0 + rb + 16 * q;
      if (row >= M) break;
      float v[8];
      load8(cs + (rb + 16 * q) * CP + cg * 8, v);
      if (full) {
        store8(W + row * N + col0, v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col0 + e < N) W[row * N + col0 + e] = v[e];
      }
    }
    return;
  }
  const TC* R = epi.resid ? reinterpret_cast<const TC*>(epi.resid) + b0 * epi.sr0 + b1 * epi.sr1 : nullptr;
  TC* X = epi.aux ? reinterpret_cast<TC*>(epi.aux) + b0 * epi.sx0 + b1 * epi.sx1 : nullptr;
  const float* bias = epi.bias ? epi.bias + b0 * epi.sb0 + b1 * epi.sb1 : nullptr;
  float bc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bc[e] = (bias && epi.bias_mode == 1 && col0 + e < N) ? bias[col0 + e] : 0.f;
#pragma unroll 2
  for (int q = 0; q < 8; ++q) {
    const int64_t row = m0 + rb + 16 * q;
    if (row >= M) break;
    float v[8];
    load8(cs + (rb + 16 * q) * CP + cg * 8, v);
    const float br = (bias && epi.bias_mode == 2) ? bias[row] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = epi.alpha * v[e] + bc[e] + br;
    if (full) {
      if (X) store8(X + row * epi.ldaux + col0, v);
      apply_act_n<8>(epi.act, v);
      if (R) {
        float r[8];
        load8(R + row * epi.ldr + col0, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += epi.beta * r[e];
      }
      store8(C + row * ldc + col0, v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int64_t col = col0 + e;
        if (col >= N) break;
        float o = v[e];
        if (X) X[row * epi.ldaux + col] = from_f32<TC>(o);
        o = apply_act(epi.act, o);
        if (R) o += epi.beta * to_f32(R[row * epi.ldr + col]);
        C[row * ldc + col] = from_f32<TC>(o);
      }
    }
  }
}

// ============================== bf16 kernel ===============================================
namespace bf {
constexpr int BK = 64;
constexpr int P0 = BK + 8;       // layout-0 image pitch (elements)
constexpr int P1 = 128 + 16;     // layout-1 image pitch (elements)
constexpr int IMG = 128 * P0;    // == 64 * P1 == 9216 elements per operand per stage
static_assert(128 * P0 == 64 * P1, "image sizes");
static_assert(2 * 2 * IMG * 2 >= 128 * CP * 4, "parked C tile must fit in the staging LDS");

__device__ __forceinline__ int krow_phys(int k) { return (k & ~12) | ((k >> 1) & 4) | ((k << 1) & 8); }

__device__ __forceinline__ uint4 pack8(const unsigned short (&s)[8]) {
  uint4 u;
  u.x = (unsigned)s[0] | ((unsigned)s[1] << 16);
  u.y = (unsigned)s[2] | ((unsigned)s[3] << 16);
  u.z = (unsigned)s[4] | ((unsigned)s[5] << 16);
  u.w = (unsigned)s[6] | ((unsigned)s[7] << 16);
  return u;
}

// One operand's 128 x 64 tile, 4 x 16-B (8 x bf16) vectors per thread.
// KIND 0: bf16, element loads (misaligned / ragged operands); 1: bf16, 16-B vector loads;
// 2: f32 in memory, 2 x 16-B loads converted to bf16 (round to nearest even) in the staging
//    registers -- the GEMM reads f32 activations / gradients without a separate cast pass.
enum { K_BF16_SCALAR = 0, K_BF16_VEC = 1, K_F32_CVT = 2 };

__device__ __forceinline__ uint4 cvt8(const float* p) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  return uint4{pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w), pack_bf16x2(b.x, b.y), pack_bf16x2(b.z, b.w)};
}

template <int LAYOUT, int KIND>
struct Loader {
  uint4 reg[4];

  __device__ __forceinline__ void load(const void* __restrict__ base, int64_t ld, int64_t r0,
                                       int64_t rmax, int64_t k0, int64_t kmax) {
    const unsigned short* b16 = reinterpret_cast<const unsigned short*>(base);
    const float* f32 = reinterpret_cast<const float*>(base);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = threadIdx.x + i * NT;
      int64_t gr, gk, off;
      bool ok;
      if (LAYOUT == 0) {
        const int row = v >> 3, kv = (v & 7) * 8;
        gr = r0 + row; gk = k0 + kv;
        off = gr * ld + gk;
      } else {
        const int krow = v >> 4, rv = (v & 15) * 8;
        gk = k0 + krow; gr = r0 + rv;
        off = gk * ld + gr;
      }
      ok = gr < rmax && gk < kmax;
      if (KIND == K_BF16_VEC) {
        reg[i] = ok ? *reinterpret_cast<const uint4*>(b16 + off) : uint4{0, 0, 0, 0};
      } else if (KIND == K_F32_CVT) {
        reg[i] = ok ? cvt8(f32 + off) : uint4{0, 0, 0, 0};
      } else {
        unsigned short s[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool oke = LAYOUT == 0 ? (gr < rmax && gk + e < kmax) : (gk < kmax && gr + e < rmax);
          s[e] = oke ? b16[off + e] : (unsigned short)0;
        }
        reg[i] = pack8(s);
      }
    }
  }

  __device__ __forceinline__ void store(__bf16* __restrict__ img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = threadIdx.x + i * NT;
      if (LAYOUT == 0) {
        const int row = v >> 3, kv = (v & 7) * 8;
        *reinterpret_cast<uint4*>(img + row * P0 + kv) = reg[i];
      } else {
        const int krow = v >> 4, rv = (v & 15) * 8;
        *reinterpret_cast<uint4*>(img + krow_phys(krow) * P1 + rv) = reg[i];
      }
    }
  }
};

// Implicit-GEMM convolution A operand (NHWC input, k order (ky, kx, ci), c % 8 == 0): the
// 128 x 64 tile of the virtual im2col matrix is gathered straight from the activation, 16 B
// (8 channels of one tap) per load; padding taps and rows >= M load zeros.
struct ConvGeo {
  const __bf16* x; int h, w, c, kw, stride, pad, oh, ow;
};

struct ConvLoader {
  uint4 reg[4];
  int64_t base[4];
  int iy0[4], ix0[4];
  ConvGeo g;

  __device__ __forceinline__ void init(const ConvGeo& geo, int64_t m0, int64_t M) {
    g = geo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = m0 + (threadIdx.x >> 3) + 32 * i;
      if (row < M) {
        const int ox = (int)(row % g.ow);
        const int64_t t = row / g.ow;
        const int oy = (int)(t % g.oh);
        const int64_t ni = t / g.oh;
        iy0[i] = oy * g.stride - g.pad;
        ix0[i] = ox * g.stride - g.pad;
        base[i] = ni * g.h * g.w * g.c;
      } else {
        iy0[i] = -(1 << 29);
        ix0[i] = 0;
        base[i] = 0;
      }
    }
  }

  __device__ __forceinline__ void load(const void*, int64_t, int64_t, int64_t, int64_t k0, int64_t kmax) {
    const int k = (int)k0 + (threadIdx.x & 7) * 8;
    const int tap = k / g.c, ci = k - tap * g.c;
    const int ky = tap / g.kw, kx = tap - ky * g.kw;
    const unsigned short* x16 = reinterpret_cast<const unsigned short*>(g.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      const bool ok = k < kmax && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      reg[i] = ok ? *reinterpret_cast<const uint4*>(x16 + base[i] + ((int64_t)iy * g.w + ix) * g.c + ci)
                  : uint4{0, 0, 0, 0};
    }
  }

  __device__ __forceinline__ void store(__bf16* __restrict__ img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = threadIdx.x + i * NT;
      *reinterpret_cast<uint4*>(img + (v >> 3) * P0 + (v & 7) * 8) = reg[i];
    }
  }
};

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// MFMA operand fragment: lane l gets rows rbase + (l & 15), k = s*32 + 8*(l >> 4) + 0..7.
template <int LAYOUT>
__device__ __forceinline__ bf16x8 frag(const __bf16* __restrict__ img, int rbase, int s, int lane) {
  if (LAYOUT == 0) {
    return *reinterpret_cast<const bf16x8*>(img + (rbase + (lane & 15)) * P0 + s * 32 + (lane >> 4) * 8);
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int k = s * 32 + 8 * g + q;
    const __bf16* a0 = img + krow_phys(k) * P1 + rbase + 4 * p;
    const __bf16* a1 = img + krow_phys(k + 4) * P1 + rbase + 4 * p;
    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

// N64: outputs with N <= 64 (the 64-channel convolutions): the 4 waves split the 128 rows
// (32 x 64 wave tiles) instead of a 2 x 2 grid whose right half would multiply zero columns.
template <typename TC, int LA, int LB, int KA, int KB, bool SPLIT, bool CONV = false, bool N64 = false>
__global__ void __launch_bounds__(NT, 2)
gemm_bf16_kernel(const void* __restrict__ A, int64_t lda, int64_t sa0, int64_t sa1,
                 const void* __restrict__ B, int64_t ldb, int64_t sb0, int64_t sb1,
                 TC* __restrict__ C, int64_t ldc, int64_t sc0, int64_t sc1,
                 int64_t M, int64_t N, int64_t K, int64_t nb1, int tiles_n, Epi epi, Split sp,
                 ConvGeo geo = ConvGeo{}) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][2][IMG];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int64_t bz = blockIdx.y, b0 = bz / nb1, b1 = bz % nb1;
  A = reinterpret_cast<const char*>(A) + (b0 * sa0 + b1 * sa1) * (KA == K_F32_CVT ? 4 : 2);
  B = reinterpret_cast<const char*>(B) + (b0 * sb0 + b1 * sb1) * (KB == K_F32_CVT ? 4 : 2);
  C += b0 * sc0 + b1 * sc1;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  int64_t kbeg = 0, kend = K;
  if (SPLIT) {
    kbeg = (int64_t)blockIdx.z * sp.kchunk;
    kend = kbeg + sp.kchunk < K ? kbeg + sp.kchunk : K;
  }

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = N64 ? wid : wid >> 1, wn = N64 ? 0 : wid & 1;
  constexpr int MI = N64 ? 2 : 4;  // 16-row fragments per wave (N64: 32-row wave tiles)
  constexpr int WR = 16 * MI;

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typename std::conditional<CONV, ConvLoader, Loader<LA, KA>>::type la;
  Loader<LB, KB> lb;
  if constexpr (CONV) la.init(geo, m0, M);
  const int nk = (int)((kend - kbeg + BK - 1) / BK);

  if (nk > 0) {
    la.load(A, lda, m0, M, kbeg, kend);
    lb.load(B, ldb, n0, N, kbeg, kend);
    la.store(smem[0][0]);
    lb.store(smem[0][1]);
    if (nk > 1) {
      la.load(A, lda, m0, M, kbeg + BK, kend);
      lb.load(B, ldb, n0, N, kbeg + BK, kend);
    }
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {  // buffer cur^1 was last read in iteration kt-1 (barrier passed)
      la.store(smem[cur ^ 1][0]);
      lb.store(smem[cur ^ 1][1]);
      if (kt + 2 < nk) {
        la.load(A, lda, m0, M, kbeg + (int64_t)(kt + 2) * BK, kend);
        lb.load(B, ldb, n0, N, kbeg + (int64_t)(kt + 2) * BK, kend);
      }
    }
    const __bf16* As = smem[cur][0];
    const __bf16* Bs = smem[cur][1];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[MI], b[4];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = frag<LA>(As, wm * WR + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag<LB>(Bs, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  write_tile_lds<TC, SPLIT, MI>(acc, reinterpret_cast<float*>(&smem[0][0][0]), epi, C, ldc, b0, b1, bz, m0, n0, M, N,
                                sp, wm, wn, lane);
}
}  // namespace bf

// ============================== f32 kernel ================================================
namespace f32 {
constexpr int BK = 16, PAD = 4, LDW = BK + PAD;

template <int LAYOUT, bool VEC>
struct Loader {
  static constexpr int NV = 128 * BK / 4 / NT;  // float4 per thread (=2)
  float4 reg[NV];

  __device__ __forceinline__ void load(const float* __restrict__ base, int64_t ld, int64_t r0,
                                       int64_t rmax, int64_t k0, int64_t kmax) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * NT;
      float t[4];
      if (LAYOUT == 0) {
        const int row = v / (BK / 4), kv = (v % (BK / 4)) * 4;
        const int64_t gr = r0 + row, gk = k0 + kv;
        if (VEC) {
          reg[i] = (gr < rmax && gk < kmax) ? *reinterpret_cast<const float4*>(base + gr * ld + gk) : float4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = (gr < rmax && gk + e < kmax) ? base[gr * ld + gk + e] : 0.f;
      } else {
        const int krow = v / 32, rv = (v % 32) * 4;
        const int64_t gk = k0 + krow, gr = r0 + rv;
        if (VEC) {
          reg[i] = (gk < kmax && gr < rmax) ? *reinterpret_cast<const float4*>(base + gk * ld + gr) : float4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = (gk < kmax && gr + e < rmax) ? base[gk * ld + gr + e] : 0.f;
      }
      reg[i] = float4{t[0], t[1], t[2], t[3]};
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * NT;
      if (LAYOUT == 0) {
        const int row = v / (BK / 4), kv = (v % (BK / 4)) * 4;
        *reinterpret_cast<float4*>(lds + row * LDW + kv) = reg[i];
      } else {
        const int krow = v / 32, rv = (v % 32) * 4;
        lds[(rv + 0) * LDW + krow] = reg[i].x;
        lds[(rv + 1) * LDW + krow] = reg[i].y;
        lds[(rv + 2) * LDW + krow] = reg[i].z;
        lds[(rv + 3) * LDW + krow] = reg[i].w;
      }
    }
  }
};

template <typename TC, int LA, int LB, bool VA, bool VB, bool SPLIT>
__global__ void __launch_bounds__(NT)
gemm_f32_kernel(const float* __restrict__ A, int64_t lda, int64_t sa0, int64_t sa1,
                const float* __restrict__ B, int64_t ldb, int64_t sb0, int64_t sb1,
                TC* __restrict__ C, int64_t ldc, int64_t sc0, int64_t sc1,
                int64_t M, int64_t N, int64_t K, int64_t nb1, int tiles_n, Epi epi, Split sp) {
  __shared__ __attribute__((aligned(16))) float smem[2][2][128 * LDW];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int64_t bz = blockIdx.y, b0 = bz / nb1, b1 = bz % nb1;
  A += b0 * sa0 + b1 * sa1;
  B += b0 * sb0 + b1 * sb1;
  C += b0 * sc0 + b1 * sc1;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  int64_t kbeg = 0, kend = K;
  if (SPLIT) {
    kbeg = (int64_t)blockIdx.z * sp.kchunk;
    kend = kbeg + sp.kchunk < K ? kbeg + sp.kchunk : K;
  }

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Loader<LA, VA> la;
  Loader<LB, VB> lb;
  const int nk = (int)((kend - kbeg + BK - 1) / BK);

  if (nk > 0) {
    la.load(A, lda, m0, M, kbeg, kend);
    lb.load(B, ldb, n0, N, kbeg, kend);
    la.store(smem[0][0]);
    lb.store(smem[0][1]);
  }
  __syncthreads();

  const int r = lane & 15, kq = (lane >> 4) * 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(A, lda, m0, M, kbeg + (int64_t)(kt + 1) * BK, kend);
      lb.load(B, ldb, n0, N, kbeg + (int64_t)(kt + 1) * BK, kend);
    }
    f32x4 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const f32x4*>(smem[cur][0] + (wm * 64 + i * 16 + r) * LDW + kq);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const f32x4*>(smem[cur][1] + (wn * 64 + j * 16 + r) * LDW + kq);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
    if (more) {
      la.store(smem[cur ^ 1][0]);
      lb.store(smem[cur ^ 1][1]);
    }
    __syncthreads();
  }
  write_tile<TC, SPLIT>(acc, epi, C, ldc, b0, b1, bz, m0, n0, M, N, sp, wm, wn, lane);
}
}  // namespace f32

// Sum the split-K partials in split order and apply the epilogue. One thread per 4 columns.
template <typename TC>
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(const float* __restrict__ ws, int splits, int64_t nb, int64_t nb1,
                     TC* __restrict__ C, int64_t ldc, int64_t sc0, int64_t sc1,
                     int64_t M, int64_t N, Epi epi) {
  const int64_t n4 = (N + 3) / 4;
  const int64_t total = nb * M * n4;
  const int64_t plane = nb * M * N;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c4 = t % n4, rowg = t / n4;
    const int64_t row = rowg % M, bz = rowg / M;
    const int64_t b0 = bz / nb1, b1 = bz % nb1;
    const int64_t col0 = c4 * 4;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const float* p = ws + bz * M * N + row * N + col0;
    if (N % 4 == 0) {
      for (int z = 0; z < splits; ++z) {
        const float4 v = *reinterpret_cast<const float4*>(p + z * plane);
        s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
      }
    } else {
      for (int z = 0; z < splits; ++z)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col0 + e < N) s[e] += p[z * plane + e];
    }
    TC* Cb = C + b0 * sc0 + b1 * sc1;
    const TC* R = epi.resid ? reinterpret_cast<const TC*>(epi.resid) + b0 * epi.sr0 + b1 * epi.sr1 : nullptr;
    TC* X = epi.aux ? reinterpret_cast<TC*>(epi.aux) + b0 * epi.sx0 + b1 * epi.sx1 : nullptr;
    const float* bias = epi.bias ? epi.bias + b0 * epi.sb0 + b1 * epi.sb1 : nullptr;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (col0 + e < N) epi_store<TC>(epi, Cb, ldc, R, X, bias, row, col0 + e, s[e]);
  }
}

// ============================== skinny GEMM (N <= 64) =========================================
// C[M, N] = epilogue(A[M, K] · B[N, K]ᵀ) for a narrow output (1x1 convs of the fine ShallowEncoder:
// M = 16.7M pixels, N = K = 32): a 128-wide tile would waste 3/4 of every MFMA and epilogue pass.
// Each wave keeps all of B (N x K) in registers as MFMA A fragments and streams 16 rows of A per
// step as the B operand of Cᵀ = B·Aᵀ, so each lane ends with 4 consecutive output columns of one
// row (8-B bf16 / 16-B f32 stores). Purely HBM-bound: A, resid and C move once.
template <typename TC, int NT16, int KC>
__global__ void __launch_bounds__(256)
gemm_skinny_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
                   TC* __restrict__ C, int64_t ldc, int64_t M, int N, int K, Epi epi) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  bf16x8 bf[NT16][KC];
#pragma unroll
  for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int n = nt * 16 + li, k0 = 32 * c + 8 * g;
      bf[nt][c] = (n < N && k0 < K) ? *reinterpret_cast<const bf16x8*>(B + (int64_t)n * ldb + k0) : bf16x8{};
    }
  float bias4[NT16][4];
#pragma unroll
  for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nt * 16 + 4 * g + r;
      bias4[nt][r] = (epi.bias && n < N) ? epi.bias[n] : 0.f;
    }
  const TC* R = reinterpret_cast<const TC*>(epi.resid);
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * 256) >> 6;
  for (int64_t m0 = wave * 16; m0 < M; m0 += nwaves * 16) {
    const int64_t m = m0 + li;
    const bool mok = m < M;
    f32x4 acc[NT16];
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int k0 = 32 * c + 8 * g;
      const bf16x8 a = (mok && k0 < K) ? *reinterpret_cast<const bf16x8*>(A + m * lda + k0) : bf16x8{};
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[nt][c], a, acc[nt], 0, 0, 0);
    }
    if (!mok) continue;
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) {
      const int n0 = nt * 16 + 4 * g;
      if (n0 >= N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = epi.alpha * acc[nt][r] + bias4[nt][r];
      apply_act_n<4>(epi.act, v);
      if (R) {
        float rr[4];
        load4(R + m * epi.ldr + n0, rr);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += epi.beta * rr[r];
      }
      store4(C + m * ldc + n0, v);
    }
  }
}

// Eligible: bf16 A/B k-contiguous, 16-B aligned rows, N % 16 == 0, N <= 64, K % 8 == 0, K <= 256,
// one batch, no aux, row-major C/resid with 8-B (bf16) / 16-B (f32) aligned 4-column groups.
bool skinny_ok(const comet_gemm_args& a) {
  if (a.dtype_ab != COMET_BF16 || a.layout_a != 0 || a.layout_b != 0 || a.convert_a || a.convert_b) return false;
  if (a.batch[0] * a.batch[1] != 1 || a.aux != nullptr || (a.bias && a.bias_mode != 1)) return false;
  if (a.n % 16 != 0 || a.n > 64 || a.k % 8 != 0 || a.k > 256 || a.m < 16384) return false;
  const int es = a.dtype_c == COMET_F32 ? 4 : 2;
  auto al = [](const void* p, int bytes) { return p == nullptr || (uintptr_t)p % bytes == 0; };
  if (!al(a.a, 16) || a.lda % 8 != 0 || !al(a.b, 16) || a.ldb % 8 != 0) return false;
  if ((uintptr_t)a.c % (4 * es) != 0 || a.ldc % 4 != 0) return false;
  if (a.resid && ((uintptr_t)a.resid % (4 * es) != 0 || a.ldr % 4 != 0)) return false;
  return true;
}

template <typename TC>
int launch_skinny(const comet_gemm_args& a, hipStream_t s) {
  Epi e{a.bias, a.bias_mode, 0, 0, a.resid, a.ldr, 0, 0, a.beta, nullptr, 0, 0, 0, a.alpha, a.act, 0};
  const int64_t tiles = cdiv(a.m, 16);
  int64_t blocks = cdiv(tiles, 4 * 8);  // ~8 row tiles per wave
  if (blocks > 4096) blocks = 4096;
  const int nt = (int)(a.n / 16), kc = (int)cdiv(a.k, 32);
#define SK(NT, KC)                                                                                          \
  hipLaunchKernelGGL((gemm_skinny_kernel<TC, NT, KC>), dim3((unsigned)blocks), dim3(256), 0, s,            \
                     (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (TC*)a.c, a.ldc, a.m, (int)a.n, (int)a.k, e)
#define SK_K(NT) do { if (kc == 1) SK(NT, 1); else if (kc == 2) SK(NT, 2); else if (kc <= 4) SK(NT, 4); else SK(NT, 8); } while (0)
  if (nt == 1) SK_K(1); else if (nt == 2) SK_K(2); else if (nt == 3) SK_K(3); else SK_K(4);
#undef SK_K
#undef SK
  COMET_CHECK_LAUNCH("comet_gemm (skinny)");
  return COMET_OK;
}

// ============================== 256 x BN bf16 kernel (k-contiguous A and B) ===================
// The forward Linear / 1x1 GEMMs of the step (M = all tokens, N = 384..3072, K = 256..3072).
// 8 waves; BN = 256: 2 x 4 waves of 128 x 64, BN = 128: 4 x 2 waves of 64 x 64 (MFMA 16x16x32,
// 8 or 4 x 4 accumulator tiles). BK = 64, two LDS stages of A[256][64] and B[BN][64] in one
// __shared__ array, filled by global_load_lds (16 B per lane, no register staging); tile t+1 is
// in flight while tile t is multiplied, one raw s_barrier per k-tile. LDS rows are 128 B; the 16-B
// chunk c of row r lives at chunk c ^ ((r >> 1) & 7) -- applied on the global source address (glds
// writes lane-linearly) and on the ds_read address -- so the 16 rows a ds_read_b128 lane group
// touches fall on 16 distinct bank slots. The k-step-1 fragments are read while the k-step-0
// MFMAs run (sched_group_barrier). Requires K % 64 == 0, 16-B aligned rows, one batch; M / N tails
// clamp the source row (those rows are never stored).
namespace big {
constexpr int BM = 256, BK = 64, NT = 512;
constexpr int ASTAGE = BM * BK;  // bf16 elements of one A stage (32 KiB)
constexpr int CPW = 64;          // parked f32 pitch per wave (64 x 64, swizzled)

typedef __attribute__((address_space(3))) void lds_void;

// rows x 64 bf16 tile, chunks of 1 KiB (8 rows) spread over the 8 waves
template <int ROWS>
__device__ __forceinline__ void glds_tile(const __bf16* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                          int64_t k0, __bf16* __restrict__ img, int wid, int lane) {
  constexpr int PER_WAVE = ROWS / 8 / 8;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int c = wid * PER_WAVE + i;
    const int row = c * 8 + (lane >> 3), pch = lane & 7;
    const int lch = pch ^ ((row >> 1) & 7);
    int64_t gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    const __bf16* gp = src + gr * ld + k0 + lch * 8;
    __builtin_amdgcn_global_load_lds((const void*)gp, (lds_void*)(img + c * 512), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag(const __bf16* __restrict__ img, int row, int lchunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((lchunk ^ ((row >> 1) & 7)) << 3));
}

// Row-contiguous operands (layout 1: element (r, k) at src[k * ld + r]; the weight of dX = dY.W
// and both operands of dW = dYᵀ.X): image [64 k][ROWS r]; 32-B unit u of k-row k lives at
// u ^ f(k), f(k) = (k & 3) | ((k >> 3) & 1) << 2, so the 8 k-rows a half-wave reads with
// ds_read_b64_tr_b16 hit 8 distinct 32-B bank groups. Requires rmax % 8 == 0.
__device__ __forceinline__ int tswz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

template <int ROWS>
__device__ __forceinline__ void glds_tile_t(const __bf16* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                            int64_t k0, __bf16* __restrict__ img, int wid, int lane) {
  constexpr int CPR = ROWS / 8;           // 16-B chunks per k-row
  constexpr int KPC = 64 / CPR;           // k-rows per 1-KiB wave chunk
  constexpr int PER_WAVE = ROWS / 8 / 8;  // wave chunks per wave (64 x ROWS x 2 B / 1 KiB / 8)
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int c = wid * PER_WAVE + i;
    const int krow = c * KPC + lane / CPR, pch = lane % CPR;
    const int lch = pch ^ (tswz(krow) << 1);
    int64_t gr = r0 + lch * 8;
    gr = gr < rmax ? gr : rmax - 8;
    const __bf16* gp = src + (k0 + krow) * ld + gr;
    __builtin_amdgcn_global_load_lds((const void*)gp, (lds_void*)(img + c * 512), 16, 0, 0);
  }
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4g;

// MFMA operand of rows rbase + (lane & 15), k = 32 s + 8 g + 0..7 from a transposed image
template <int ROWS>
__device__ __forceinline__ bf16x8 frag_t(const __bf16* __restrict__ img, int rbase, int s, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int u = rbase >> 4;
  const int k0 = s * 32 + 8 * g + q, k1 = k0 + 4;
  const __bf16* a0 = img + k0 * ROWS + ((u ^ tswz(k0)) << 4) + 4 * p;
  const __bf16* a1 = img + k1 * ROWS + ((u ^ tswz(k1)) << 4) + 4 * p;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4g*)(a0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4g*)(a1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <typename TC, int BN, int LA, int LB, bool SPLIT, int VAR = 0, bool DACT = false>
__global__ void __launch_bounds__(NT, 1)
gemm_big_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
                TC* __restrict__ C, int64_t ldc, int64_t M, int64_t N, int64_t K, int tiles_n, Epi epi,
                Split sp) {
  constexpr int WN = BN / 64, WM = 8 / WN;   // wave grid
  constexpr int MI = BM / WM / 16;           // 16-row tiles per wave (8 or 4)
  constexpr int BSTAGE = BN * BK;
  constexpr int STAGING = 2 * ASTAGE + 2 * BSTAGE, PARKING = 8 * 64 * CPW * 2;  // bf16 elements
  __shared__ __attribute__((aligned(1024))) __bf16 smem[STAGING > PARKING ? STAGING : PARKING];
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int li = lane & 15, g = lane >> 4;
  __bf16* const Asm = smem;
  __bf16* const Bsm = smem + 2 * ASTAGE;

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int64_t kbeg = 0, kend = K;
  if (SPLIT) {
    kbeg = (int64_t)blockIdx.y * sp.kchunk;
    kend = kbeg + sp.kchunk < K ? kbeg + sp.kchunk : K;
  }
  const int nk = (int)((kend - kbeg) / BK);
  auto load_tiles = [&](int64_t k0, int stage) {
    if constexpr (LA == 0) glds_tile<BM>(A, lda, m0, M, k0, Asm + stage * ASTAGE, wid, lane);
    else glds_tile_t<BM>(A, lda, m0, M, k0, Asm + stage * ASTAGE, wid, lane);
    if constexpr (LB == 0) glds_tile<BN>(B, ldb, n0, N, k0, Bsm + stage * BSTAGE, wid, lane);
    else glds_tile_t<BN>(B, ldb, n0, N, k0, Bsm + stage * BSTAGE, wid, lane);
  };
  auto afrag = [&](const __bf16* img, int rbase, int s) {
    if constexpr (LA == 0) return frag(img, rbase + li, 4 * s + g);
    else return frag_t<BM>(img, rbase, s, lane);
  };
  auto bfrag = [&](const __bf16* img, int rbase, int s) {
    if constexpr (LB == 0) return frag(img, rbase + li, 4 * s + g);
    else return frag_t<BN>(img, rbase, s, lane);
  };
  if (nk > 0) load_tiles(kbeg, 0);

  // one barrier per k-tile: it publishes tile kt (every wave drained its own glds first) and
  // frees the other stage (every wave finished tile kt-1), which then receives tile kt+1 while
  // tile kt is multiplied. The body is branch-free (the last tile is peeled) so the scheduler can
  // interleave the next tile's glds, this tile's fragment reads and the MFMAs.
  auto body = [&](int kt, auto load_next) {
    constexpr bool LOAD = decltype(load_next)::value;
    const int cur = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    const __bf16* a_img = Asm + cur * ASTAGE;
    const __bf16* b_img = Bsm + cur * BSTAGE;
    bf16x8 a0[MI], b0[4], a1[MI], b1[4];
    if constexpr (LOAD && VAR != 3) load_tiles(kbeg + (int64_t)(kt + 1) * BK, cur ^ 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) b0[j] = bfrag(b_img, wc * 64 + j * 16, 0);
#pragma unroll
    for (int i = 0; i < MI; ++i) a0[i] = afrag(a_img, wr * (MI * 16) + i * 16, 0);
    if constexpr (LOAD && VAR == 3) load_tiles(kbeg + (int64_t)(kt + 1) * BK, cur ^ 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) b1[j] = bfrag(b_img, wc * 64 + j * 16, 1);
#pragma unroll
    for (int i = 0; i < MI; ++i) a1[i] = afrag(a_img, wr * (MI * 16) + i * 16, 1);
    if constexpr (VAR == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
    if constexpr (VAR == 1) __builtin_amdgcn_s_setprio(0);
    constexpr int RD = MI * (LA ? 2 : 1) + 4 * (LB ? 2 : 1);  // ds_read instructions per k-step
    if constexpr (VAR == 3) {
      constexpr int NG = LOAD ? BM / 64 + BN / 64 : 0;       // glds per thread per tile
      __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
#pragma unroll
      for (int q = 0; q < RD; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8 * MI - 2 * NG - RD, 0);
    } else if constexpr (VAR != 2) {
      // the k-step-0 reads, then {1 read, 2 MFMA} for the k-step-1 reads, then the rest
      constexpr int PAIRS = RD < 4 * MI ? RD : 4 * MI;
      __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
#pragma unroll
      for (int q = 0; q < PAIRS; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, RD - PAIRS, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8 * MI - 2 * PAIRS, 0);
    }
  };
  for (int kt = 0; kt + 1 < nk; ++kt) body(kt, std::true_type{});
  if (nk > 0) body(nk - 1, std::false_type{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");  // all fragment reads done before the LDS is reused

  // ---- epilogue: each wave parks 64 x 64 f32 in its own 16 KiB of LDS (MI / 4 rounds), then
  // writes 8-column runs with the fused bias / act / aux / residual ----
  float* park = reinterpret_cast<float*>(smem) + wid * 64 * CPW;
  const TC* R = reinterpret_cast<const TC*>(epi.resid);
  TC* X = reinterpret_cast<TC*>(epi.aux);
  const int rq = g * 4;
  const int cg = lane & 7, rb = lane >> 3;
  const int64_t col0 = n0 + wc * 64 + cg * 8;
  float bc[8], cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bc[e] = (epi.bias && epi.bias_mode == 1 && col0 + e < N) ? epi.bias[col0 + e] : 0.f;
    cs[e] = 0.f;
  }
#pragma unroll
  for (int h = 0; h < MI / 4; ++h) {
    if (h) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + rq + r, col = j * 16 + li;
          park[row * CPW + (col ^ ((row & 3) << 4))] = acc[h * 4 + i][j][r];
        }
#pragma unroll 2
    for (int q = 0; q < 8; ++q) {
      const int rl = rb + 8 * q;
      const int64_t row = m0 + wr * (MI * 16) + h * 64 + rl;
      float v[8];
      load8(park + rl * CPW + ((cg * 8) ^ ((rl & 3) << 4)), v);
      if (row >= M || col0 >= N) continue;
      if constexpr (SPLIT) {  // raw f32 partial of split blockIdx.y; epilogue in the reduce
        float* W = sp.ws + (int64_t)blockIdx.y * M * N + row * N + col0;
        if (N % 8 == 0) {
          store8(W, v);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (col0 + e < N) W[e] = v[e];
        }
        continue;
      }
      if constexpr (DACT) {  // backward of an activation: act'(pre) * dH, rounded, column sums
        float pr[8];
        load8(epi.gpre + row * epi.ldg + col0, pr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gq = to_f32(from_f32<TC>(epi.alpha * v[e] * gelu_grad_fast(pr[e])));
          v[e] = gq;
          cs[e] += gq;
        }
        store8(C + row * ldc + col0, v);
        continue;
      }
      const float br = (epi.bias && epi.bias_mode == 2) ? epi.bias[row] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = epi.alpha * v[e] + bc[e] + br;
      if (epi.vec && col0 + 8 <= N) {
        if (X) store8(X + row * epi.ldaux + col0, v);
        apply_act_n<8>(epi.act, v);
        if (R) {
          float rr[8];
          load8(R + row * epi.ldr + col0, rr);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += epi.beta * rr[e];
        }
        store8(C + row * ldc + col0, v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int64_t col = col0 + e;
          if (col >= N) break;
          float o = v[e];
          if (X) X[row * epi.ldaux + col] = from_f32<TC>(o);
          o = apply_act(epi.act, o);
          if (R) o += epi.beta * to_f32(R[row * epi.ldr + col]);
          C[row * ldc + col] = from_f32<TC>(o);
        }
      }
    }
  }
  if constexpr (DACT) {
    // the 8 row lanes of each column group (lanes cg + 8 rb) meet by shuffles; one atomic per column
    // per wave (the act_bwd_colsum kernel sums its row blocks the same way)
    if (epi.dcol != nullptr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = cs[e];
        x += __shfl_xor(x, 8, 64);
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        cs[e] = x;
      }
      if (rb == 0 && col0 < N) {
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(epi.dcol + col0 + e, cs[e]);
      }
    }
  }
}
}  // namespace big

// ============================== persistent 256 x 256 kernel ======================================
// The forward Linear shapes (k-contiguous bf16 A and B, K % 64 == 0). What the 256-row kernel above
// loses per tile (measured on M 74368, N 3072, K 768: MFMA busy 28 % of the SIMD cycles) is the
// lock-step [barrier -> glds burst + ds_read burst -> wait -> MFMA] body of its waves, the
// park-in-LDS epilogue and the tile prologue's load latency. Here:
//  * each 32-deep k-step of a wave is one MFMA stream with the next k-step's fragment reads (and,
//    in the second k-step, this wave's LDS-DMA pieces of k-tile q+2) issued one by one between the
//    MFMAs (sched_group_barrier), fragments double-buffered in registers;
//  * one barrier per 64-deep k-tile, between its two k-steps: it retires every wave's reads of
//    buffer q&1 (which the second k-step then refills with k-tile q+2) and every wave's LDS-DMA of
//    k-tile q+1 (whose first-k-step fragments the second k-step reads);
//  * persistent: one workgroup per CU walks its tiles (XCD-banded order) and the k-tile stream runs
//    on across tile boundaries, so the next tile's first two k-tiles load during this epilogue;
//  * Cᵀ = W·Xᵀ per MFMA (operands swapped): a lane holds 4 consecutive output columns of one row
//    and the epilogue stores straight from the accumulators (no LDS park).
// NW = 8: 2 x 4 waves of 128 x 64 (two waves per SIMD); NW = 4: 2 x 2 waves of 128 x 128.
namespace w4 {
constexpr int BK = 64;
constexpr int WGM = 8;  // logical tiles run down groups of WGM tile rows, column by column

// logical tile -> (tile row, tile column): an XCD's 32 consecutive tiles form an 8 x 4 patch
// (A blocks shared by 4 workgroups, B blocks by 8) instead of a 32-wide strip of one tile row
__device__ __forceinline__ void tile_rc(int L, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int gsz = WGM * tiles_n, grp = L / gsz, rem = L - grp * gsz;
  const int rows = min(WGM, tiles_m - grp * WGM);
  tm = grp * WGM + rem % rows;
  tn = rem / rows;
}

typedef __attribute__((address_space(3))) void lds_void;

constexpr int SG_MFMA = 0x008, SG_DSR = 0x100, SG_VMR = 0x020;

#ifdef COMET_GEMM_STAMPS
// Diagnostic build only (make STAMPS=1 -> libcomet_hip_stamp.so): wave 0 of each workgroup records
// the shader clock at the start of each tile's k-loop (0), before (1) and after (2) its epilogue,
// past the second k-tile's barrier (3), and around the row-LN statistics barrier (4, 5); written by
// lane 0 with a vector store into g_stamps[workgroup][tile][phase] (tools/gemm_stamps.py).
constexpr int ST_WG = 256, ST_TILES = 64;
__device__ unsigned long long g_stamps[ST_WG * ST_TILES * 8];
__device__ __forceinline__ void stamp(int bid, int wid, int tile, int ph) {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if (wid == 0 && bid < ST_WG && tile < ST_TILES && (threadIdx.x & 63) == 0)
    g_stamps[((bid * ST_TILES + tile) << 3) + ph + (threadIdx.x & 63)] = t;
}
// intra-k-tile stamps of waves 0 and 4 (the two waves of one SIMD) on k-tile 3 of tiles 0..31:
// wave 4 records into tile slot + 32 (phases 3: k-tile start, 4: k-step 0 issued, 5: past the
// waits, 6: past the barrier, 7: k-step 1 issued; tools/gemm_stamps.py ksteps)
__device__ __forceinline__ void kstamp(int bid, int wid, int tile, int ph) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if ((wid == 0 || wid == 4) && bid < ST_WG && tile < 32 && (threadIdx.x & 63) == 0)
    g_stamps[((bid * ST_TILES + tile + (wid == 4 ? 32 : 0)) << 3) + ph] = t;
  __builtin_amdgcn_sched_barrier(0);
}
#define COMET_STAMP(tile, ph) stamp(bid, wid, (tile), (ph))
#define COMET_KSTAMP(tile, ph) kstamp(bid, wid, (tile), (ph))
#else
#define COMET_STAMP(tile, ph) ((void)0)
#define COMET_KSTAMP(tile, ph) ((void)0)
#endif

// Row LayerNorm fused into the f32 epilogue when one tile spans the whole output row (N == TBN:
// the tracker's hidden sizes 384 / 256). With v = the epilogue value of a row (bias, residual):
//   C   = v (raw_c) or (v - mean) * rstd(eps_y)                [f32: residual stream / dual copy]
//   y16 = (v - mean) * rstd(eps_y)                             [bf16, optional: next GEMM operand]
//   z16 = (v - mean) * rstd(eps_z) * zw + zb                   [bf16, optional: affine context LN]
// Mean and variance are two-pass over the values kept in registers; the four waves of a tile row
// exchange their partial sums through a small LDS table (two workgroup barriers per tile).
struct RowLN {
  __bf16* y16; int64_t ldy; float eps_y;
  __bf16* z16; int64_t ldz; const float* zw; const float* zb; float eps_z;
  int raw_c;
};

template <typename TC, int ACT, bool HASR, int NW, int TBM, int TBN, bool LN = false, bool PING = false>
__global__ void __launch_bounds__(NW * 64, 1)
gemm_w4_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
               TC* __restrict__ C, int64_t ldc, int64_t M, int64_t N, int64_t K, int tiles_n, int ntiles,
               Epi epi, RowLN ln) {
  constexpr int WN = NW / 2;        // wave grid 2 x WN
  constexpr int WROWS = TBM / 2;    // wave tile rows (128 or 64)
  constexpr int WCOLS = TBN / WN;   // wave tile columns (64 or 96)
  constexpr int MI = WROWS / 16;    // row fragments per wave
  constexpr int NI = WCOLS / 16;    // column fragments per wave
  constexpr int ASTAGE = TBM * BK;  // bf16 elements of the A image of one k-tile
  constexpr int BUF = (TBM + TBN) * BK;  // A + B images of one k-tile (64 KiB)
  // LDS-DMA pieces (8 rows x 64 k = 1 KiB) per wave and k-tile; a 32-row A image has 4 pieces for
  // 8 waves: waves 4-7 load the same pieces as waves 0-3 (identical bytes to the same LDS words), so
  // every wave issues the same count and the counted waits stay uniform
  constexpr int APC = TBM / 8;
  constexpr int PA = APC >= NW ? APC / NW : 1, PB = TBN / 8 / NW;
  constexpr int NMF = MI * NI;      // MFMAs per k-step
  constexpr int NRD = MI + NI;      // fragment reads per k-step
  // f32 outputs park each 8-row half block in LDS and store whole 128-B lines (the direct
  // 4-column f32 stores ran at half speed); so do bf16 outputs without an activation when the wave
  // tile is 64 wide (tools/gpu/kscan.sh: the direct 4-column stores of 16 rows per instruction
  // cost ~3-4 us per 256 x 256 tile, 10-18 % of a K = 384-768 GEMM). With GELU the parked path
  // serialises the activation behind the LDS round trips (+27 %): those keep the direct stores.
  constexpr bool BPARK = std::is_same<TC, __bf16>::value && !HASR && !LN && WCOLS == 64 && ACT == COMET_ACT_NONE;  // see below
  constexpr bool PARK = std::is_same<TC, float>::value || (WCOLS % 64 == 0 && ACT == COMET_ACT_NONE && !BPARK);
  // direct bf16 stores of interior tiles without a residual: fragments j, j+1 exchange halves by
  // v_permlane16_swap so every lane stores 16 B (8 columns) instead of 8 B -- half the store
  // instructions for the same bytes (the epilogue tail is store-issue bound: cdna_hip_programming.md
  // T21). COMET_GEMM_NO_WIDE=1 at launch selects the 8-B stores (measurement A/B).
  constexpr bool WIDE = !PARK && !BPARK && !HASR && std::is_same<TC, __bf16>::value && (NI % 2 == 0);
  // parked f32 row pitch: 64-wide slabs XOR-swizzle their 16-B chunks (c ^ pswz(r): the 8 rows
  // one ds_write_b128 lane group writes hit 8 distinct chunks and the 4 (row, 4-chunk) quads of
  // each ds_read_b128 lane group of the re-read are disjoint); 96-wide slabs pad rows to 100
  // bf16 outputs without a residual or activation on 64-wide wave tiles (interior tiles, epi.bpark):
  // the epilogue value (alpha * acc + bias) is parked as bf16, one 16-row block at a time, in a
  // per-wave slab (two alternate), re-read as 8 rows x 128 B per ds_read_b128 and stored as whole
  // 128-B lines: half the LDS bytes and write instructions of the f32 park (epilogue 8.9k -> 5.4k
  // cycles per 256 x 256 tile, tools/gemm_stamps.py). GELU outputs keep the direct 16-B stores: their
  // epilogue is VALU-bound on the activation and the park round trip measured 4 % slower.
  constexpr int BSLAB = 16 * WCOLS;                   // bf16 elements of one slab
  constexpr int BPARK_B = BPARK ? NW * 2 * BSLAB : 0;  // bf16 elements of the bf16 park region
  constexpr bool PSWZ = (WCOLS & (WCOLS - 1)) == 0;
  constexpr int PPITCH = PSWZ ? WCOLS : WCOLS + 4;
  constexpr int PARK_F = PARK ? NW * 8 * PPITCH : 0;  // f32 elements of the park region
  auto pswz = [](int r) { return PSWZ ? ((r & 7) | ((r & 2) << 2)) : 0; };
  static_assert(!LN || (PARK && std::is_same<TC, float>::value), "row LN epilogue: parked f32 outputs only");
  static_assert(!LN || !BPARK, "row LN epilogue: no bf16 park");
  constexpr int STATS_F = LN ? 2 * TBM * WN : 0;  // f32 row-partial table (sum, sum of squares)
  constexpr int PARK_ELEMS = 2 * PARK_F > BPARK_B ? 2 * PARK_F : BPARK_B;
  // A-operand lookahead (AR): the A images (activation rows, streamed from HBM once when tiles_n is
  // small) run in a 3-slot ring one k-tile ahead of the 2-slot B ring (weights, L2-resident). Within
  // an issue batch the B pieces go first, so the barrier wait can leave the batch's A pieces in
  // flight (vmcnt counts in issue order): each A load gets two k-tiles of MFMA work to land in
  // instead of one. Taken by every instance whose LDS still fits (the row tiles up to 128 x 384 /
  // 128 x 256 without an f32 park of 128 x 384); COMET_GEMM_NO_AR at build time disables it (A/B).
#ifdef COMET_GEMM_NO_AR
  constexpr bool AR = false;
#else
  constexpr bool AR = 2 * (3 * ASTAGE + 2 * TBN * BK + PARK_ELEMS + 2 * STATS_F) <= 160 * 1024 && TBM <= 128;
#endif
  constexpr int NA = AR ? 3 : 2;                  // A ring slots
  constexpr int BSTAGE = TBN * BK;                // bf16 elements of the B image of one k-tile
  constexpr int BRING = NA * ASTAGE;              // B ring base (A ring first)
  constexpr int RING = NA * ASTAGE + 2 * BSTAGE;  // both rings (= 2 * BUF without AR)
  constexpr int XA = AR ? PA : 0;                 // A pieces a barrier wait may leave in flight
  static_assert(AR || RING == 2 * BUF, "ring layout");
  __shared__ __attribute__((aligned(1024))) __bf16 smem[RING + PARK_ELEMS + 2 * STATS_F];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int li = lane & 15, g = lane >> 4;
  const int nk = (int)(K / BK);
  const int G = gridDim.x, bid = blockIdx.x;
  const int tiles_m = ntiles / tiles_n;
  const bool single = ntiles <= G;
  // tile it of this workgroup is logical tile off + it * strd, below lim. Default: wave it of the
  // grid takes logical tiles [it * G, (it + 1) * G), XCD x (= bid & 7) the x-th 32 of them. With
  // epi.raster (COMET_GEMM_RASTER=1, measurement) each XCD walks its own contiguous eighth of the
  // logical tiles instead, so an A row block is fetched into at most two XCDs' L2.
  int off = single ? xcd_remap(bid, G) : (bid & 7) * (G >> 3) + (bid >> 3), strd = G, lim = ntiles;
  if (!single && epi.raster && (G & 7) == 0) {
    const int x = bid & 7, per = ntiles >> 3, rem = ntiles & 7, base = x * per + min(x, rem);
    lim = base + per + (x < rem ? 1 : 0);
    off = base + (bid >> 3);
    strd = G >> 3;
  }
  const int my_tiles = single ? 1 : (off < lim ? (lim - off + strd - 1) / strd : 0);
  const int T = my_tiles * nk;
  if (T == 0) return;

  // ---- load stream: a wave issues LDS-DMA pieces wid*PA + p (A) and wid*PB + p (B) of the images (8 rows x 64 k
  // = 1 KiB each; 16-B chunk c of row r stored at c ^ ((r >> 1) & 7)); source rows clamped (tails
  // re-read the last row, never stored)
  // first A piece of this wave: the wrap is compile-time absent unless the A image has fewer pieces
  // than waves (32-row tiles), so the other instances keep the plain wid * PA addressing
#ifdef COMET_APIECE_WRAP_ALL  // round-4 form (wrap in every instance; A/B build only, profiles/r05_rowln)
  const int pieca = (wid * PA) % APC;
#else
  const int pieca = APC < NW ? (wid * PA) % APC : wid * PA;
#endif
  const int prowa = pieca * 8 + (lane >> 3), prowb = wid * PB * 8 + (lane >> 3);  // + p * 8
  // load-stream state: the k-tile the next issue_cur() loads (tile ld_it of this workgroup, k-tile
  // ld_kt of it); per tile, uniform row-block bases and per-lane 32-bit element offsets
  // (two streams, A and B: with AR the A stream runs one k-tile ahead, otherwise in lockstep)
  int la_it = 0, la_kt = 0, lb_it = 0, lb_kt = 0;
  const __bf16* ldA = A;
  const __bf16* ldB = B;
  int offA[PA], offB[PB];
  // chunk swizzle of image row r: c ^ ((r >> 1) & 7) (r = this lane's row in the image)
  auto lch = [&](int r) { return ((lane & 7) ^ ((r >> 1) & 7)) * 8; };
  auto set_tile_a = [&](int it) {
    int tm, tn;
    tile_rc(off + it * strd, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * TBM;
    ldA = A + (int64_t)m0 * lda;
#pragma unroll
    for (int p = 0; p < PA; ++p)
      offA[p] = (min(m0 + prowa + p * 8, (int)M - 1) - m0) * (int)lda + lch(prowa + p * 8);
  };
  auto set_tile_b = [&](int it) {
    int tm, tn;
    tile_rc(off + it * strd, tiles_m, tiles_n, tm, tn);
    const int n0 = tn * TBN;
    ldB = B + (int64_t)n0 * ldb;
#pragma unroll
    for (int p = 0; p < PB; ++p)
      offB[p] = (min(n0 + prowb + p * 8, (int)N - 1) - n0) * (int)ldb + lch(prowb + p * 8);
  };
  auto issue_a = [&](int slot) {
    const __bf16* pa = ldA + la_kt * BK;
#pragma unroll
    for (int p = 0; p < PA; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(pa + offA[p]), (lds_void*)(smem + slot * ASTAGE + (pieca + p) * 512), 16, 0, 0);
  };
  auto issue_b = [&](int slot) {
    const __bf16* pb = ldB + lb_kt * BK;
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(pb + offB[p]),
                                       (lds_void*)(smem + BRING + slot * BSTAGE + (wid * PB + p) * 512), 16, 0, 0);
  };
  // one batch: A and B pieces interleaved (lockstep), or all B pieces before the A pieces (AR)
  auto issue_cur = [&](int aslot, int bslot) {
    if constexpr (AR) {
      issue_b(bslot);
      issue_a(aslot);
    } else {
      const __bf16* pa = ldA + la_kt * BK;
      const __bf16* pb = ldB + lb_kt * BK;
#pragma unroll
      for (int p = 0; p < (PA > PB ? PA : PB); ++p) {
        if (p < PA)
          __builtin_amdgcn_global_load_lds((const void*)(pa + offA[p]), (lds_void*)(smem + aslot * ASTAGE + (pieca + p) * 512), 16, 0, 0);
        if (p < PB)
          __builtin_amdgcn_global_load_lds((const void*)(pb + offB[p]),
                                           (lds_void*)(smem + BRING + bslot * BSTAGE + (wid * PB + p) * 512), 16, 0, 0);
      }
    }
  };
  // past the last k-tile a stream keeps re-loading it (into a slot nothing reads again)
  auto advance_a = [&]() {
    if (++la_kt == nk) {
      if (la_it + 1 < my_tiles) { la_kt = 0; set_tile_a(++la_it); }
      else la_kt = nk - 1;
    }
  };
  auto advance_b = [&]() {
    if (++lb_kt == nk) {
      if (lb_it + 1 < my_tiles) { lb_kt = 0; set_tile_b(++lb_it); }
      else lb_kt = nk - 1;
    }
  };
  auto advance = [&]() {
    advance_a();
    advance_b();
  };

  bf16x8 a0[MI], b0[NI], a1[MI], b1[NI];
  auto read_frags = [&](int aslot, int bslot, int s, bf16x8 (&af)[MI], bf16x8 (&bf)[NI]) {
    const __bf16* aimg = smem + aslot * ASTAGE;
    const __bf16* bimg = smem + BRING + bslot * BSTAGE;
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = big::frag(aimg, wr * WROWS + i * 16 + li, 4 * s + g);
#pragma unroll
    for (int j = 0; j < NI; ++j) bf[j] = big::frag(bimg, wc * WCOLS + j * 16 + li, 4 * s + g);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](const bf16x8 (&af)[MI], const bf16x8 (&bf)[NI]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
  };

  // static priority for the younger half of the workgroup (cdna_hip_programming.md T5, static
  // form): the second-dispatched waves lose VALU / issue arbitration on every segment otherwise
  if (!PING && epi.prio && wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  int pend = 0;  // 1: the last epilogue's stores are the newest VMEM ops (count known)
  // epilogue of tile tix (q_: its last k-tile, qa1_: the A slot of k-tile q_ + 1, for the re-read of
  // the next tile's first fragments the lock-step loop needs after it)
  auto tile_epilogue = [&](const int tix, const int q_, const int qa1_) {
      COMET_STAMP(tix, 1);
      // ---- epilogue of the tile, straight from the accumulators: lane (li, g) of fragment
      // (i, j) holds C[row0 + i*16 + li][col0 + j*16 + 4g + r], r = 0..3
      int tm, tn;
      tile_rc(off + tix * strd, tiles_m, tiles_n, tm, tn);
      const int64_t row0 = (int64_t)tm * TBM + wr * WROWS + li;
      const int64_t col0 = (int64_t)tn * TBN + wc * WCOLS + 4 * g;
      const TC* R = reinterpret_cast<const TC*>(epi.resid);
      TC* X = reinterpret_cast<TC*>(epi.aux);
      const bool interior = (int64_t)tm * TBM + TBM <= M && (int64_t)tn * TBN + TBN <= N;
      // loads first (bias, the first residual row), then a store stream with no wait in it: the
      // residual rows are prefetched one ahead, so their waits only cover the previous row's stores.
      // Interior tiles take a branch-free copy (no per-store exec branches, whose joins make the
      // compiler drain every outstanding store before each block).
      auto epilogue = [&](auto edge_t) {
        constexpr bool EDGE = decltype(edge_t)::value;
        const bool bias_c = epi.bias != nullptr;  // per-column bias only (pp_ok)
        float bc[NI][4];
  #pragma unroll
        for (int j = 0; j < NI; ++j)
  #pragma unroll
          for (int r = 0; r < 4; ++r) bc[j][r] = 0.f;
        if (bias_c) {  // one uniform branch around straight-line loads (clamped: tail columns never stored)
  #pragma unroll
          for (int j = 0; j < NI; ++j)
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int64_t col = col0 + j * 16 + r;
              bc[j][r] = epi.bias[EDGE ? (col < N ? col : N - 1) : col];
            }
        }
        float rc[NI][4], rn[NI][4];
        auto load_resid = [&](int i, float (&rv)[NI][4]) {
          const int64_t row = row0 + i * 16;
  #pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int64_t col = col0 + j * 16;
            if (!EDGE || (row < M && col < N)) load4(R + row * epi.ldr + col, rv[j]);
          }
        };
        if constexpr (HASR) load_resid(0, rc);
  #pragma unroll
        for (int i = 0; i < MI; ++i) {
          if constexpr (HASR) {
            if (i + 1 < MI) load_resid(i + 1, rn);
          }
          const int64_t row = row0 + i * 16;
  #pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int64_t col = col0 + j * 16;
            if (!EDGE || (row < M && col < N)) {
              float v[4];
  #pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = epi.alpha * acc[i][j][r] + bc[j][r];
              if (X) store4(X + row * epi.ldaux + col, v);
              apply_act_n<4>(ACT, v);
              if constexpr (HASR) {
  #pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += epi.beta * rc[j][r];
              }
              store4(C + row * ldc + col, v);
            }
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
          if constexpr (HASR) {
  #pragma unroll
            for (int j = 0; j < NI; ++j)
  #pragma unroll
              for (int r = 0; r < 4; ++r) rc[j][r] = rn[j][r];
          }
        }
      };
      if constexpr (LN) {
        // row-LN epilogue (tiles_n == 1, N == TBN). Pass 1 is the parked pass of the plain f32
        // epilogue; each lane's final values (8 lanes x NV columns of one row per wave) go back into
        // the accumulator registers they were parked from, and the lane's row sum and sum of squares
        // are reduced over the 8 lanes of the row, then over the WN waves of the tile row through
        // the LDS table st (one barrier; var = E[v^2] - mean^2, clamped at 0). Pass 2 writes the
        // outputs with the statistics read back per row (no per-row arrays in registers).
        constexpr int CPL = 4, NTC = WCOLS / (8 * CPL), NV = NTC * CPL;
        float* park = reinterpret_cast<float*>(smem + RING) + wid * 8 * PPITCH;
        float* st = reinterpret_cast<float*>(smem + RING + 2 * PARK_F);
        const int rr = lane >> 3, cc = lane & 7;
        const int64_t prow0 = (int64_t)tm * TBM + wr * WROWS + rr;  // + i*16 + h*8
        // (tn is always 0 here; keeping it in the column makes the bias / affine loads tile-dependent
        // so they are not hoisted out of the k-loop, where they would hold ~36 registers)
        const int pc0 = tn * TBN + wc * WCOLS + cc * CPL;  // + t*8*CPL + e
        const float invn = 1.f / (float)N;
        auto VK = [&](int i, int h, int u) -> float { return acc[i][h * NTC + (u >> 2)][u & 3]; };
        auto lrow = [&](int i, int h) { return (wr * WROWS + i * 16 + h * 8 + rr) * WN; };
        auto red8 = [](float x) {
          x += __shfl_xor(x, 1, 64);
          x += __shfl_xor(x, 2, 64);
          x += __shfl_xor(x, 4, 64);
          return x;
        };
        // (mean, biased variance) of row (i, h) from the WN (sum, sum of squares) partials
        auto rowstats = [&](int i, int h, float& mu, float& var) {
          float x = 0.f, q = 0.f;
  #pragma unroll
          for (int w = 0; w < WN; ++w) {
            const float2 p = *reinterpret_cast<const float2*>(st + 2 * (lrow(i, h) + w));
            x += p.x;
            q += p.y;
          }
          mu = x * invn;
          var = fmaxf(q * invn - mu * mu, 0.f);
        };
        auto lnepilogue = [&](auto edge_t) {
          constexpr bool EDGE = decltype(edge_t)::value;
          float bcp[NV];
  #pragma unroll
          for (int u = 0; u < NV; ++u) bcp[u] = 0.f;
          if (epi.bias != nullptr) {
  #pragma unroll
            for (int t = 0; t < NTC; ++t) load4(epi.bias + pc0 + t * 8 * CPL, *reinterpret_cast<float(*)[4]>(bcp + t * CPL));
          }
          // residual rows are loaded one (i, h) step ahead (a 2-slot register ring), so each step's HBM
          // latency overlaps the previous step's park / reduce / store work instead of being exposed
          // MI x 2 times (a 3-slot ring measured 4 % slower on the 64 x 384 tiles; round 4: every residual
          // row of a 64 x 384 tile issued at once, and a 4-slot ring on the 128-row tiles, 1-6 % slower,
          // profiles/r04_rowln)
          constexpr int RDL = 2;
          auto rload = [&](int ih, float (&dst)[NTC][CPL]) {
            const int64_t row = prow0 + (ih >> 1) * 16 + (ih & 1) * 8;
  #pragma unroll
            for (int t = 0; t < NTC; ++t)
  #pragma unroll
              for (int e = 0; e < CPL; ++e) dst[t][e] = 0.f;
            if constexpr (HASR) {
  #pragma unroll
              for (int t = 0; t < NTC; ++t)
                if (!EDGE || row < M) loadn<CPL>(R + row * epi.ldr + pc0 + t * 8 * CPL, dst[t]);
            }
          };
          float rring[RDL][NTC][CPL];
  #pragma unroll
          for (int d = 0; d < RDL - 1; ++d) rload(d, rring[d]);
  #pragma unroll
          for (int i = 0; i < MI; ++i) {
            float vh[2][NV];
  #pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int64_t row = prow0 + i * 16 + h * 8;
              const bool live = !EDGE || row < M;
              const int ih = 2 * i + h;
              float (&rc)[NTC][CPL] = rring[ih % RDL];
              if (ih + RDL - 1 < 2 * MI) rload(ih + RDL - 1, rring[(ih + RDL - 1) % RDL]);
              if ((li >> 3) == h) {
  #pragma unroll
                for (int j = 0; j < NI; ++j)
                  *reinterpret_cast<f32x4*>(park + (li & 7) * PPITCH + (((j * 4 + g) ^ pswz(li & 7)) << 2)) = acc[i][j];
              }
              asm volatile("" ::: "memory");
              float s = 0.f, sq = 0.f;
  #pragma unroll
              for (int t = 0; t < NTC; ++t) {
                float v[CPL];
                const int lc = (t * 8 * CPL + cc * CPL) >> 2;
                const f32x4 p4 = *reinterpret_cast<const f32x4*>(park + rr * PPITCH + ((lc ^ pswz(rr)) << 2));
                v[0] = p4[0]; v[1] = p4[1]; v[2] = p4[2]; v[3] = p4[3];
  #pragma unroll
                for (int e = 0; e < CPL; ++e) {
                  float o = apply_act(ACT, epi.alpha * v[e] + bcp[t * CPL + e]);
                  if constexpr (HASR) o += epi.beta * rc[t][e];
                  v[e] = o;
                  vh[h][t * CPL + e] = o;
                  s += o;
                  sq = fmaf(o, o, sq);
                }
                if (ln.raw_c && live) storen<CPL>(C + row * ldc + pc0 + t * 8 * CPL, v);
              }
              s = red8(s);
              sq = red8(sq);
              if (cc == 0) *reinterpret_cast<float2*>(st + 2 * (lrow(i, h) + wc)) = float2{s, sq};
              asm volatile("" ::: "memory");
            }
  #pragma unroll
            for (int h = 0; h < 2; ++h)
  #pragma unroll
              for (int t = 0; t < NTC; ++t)
                acc[i][h * NTC + t] = f32x4{vh[h][4 * t], vh[h][4 * t + 1], vh[h][4 * t + 2], vh[h][4 * t + 3]};
          }
          float zw[NV], zb[NV];
          if (ln.z16 != nullptr) {
  #pragma unroll
            for (int t = 0; t < NTC; ++t) {
              load4(ln.zw + pc0 + t * 8 * CPL, *reinterpret_cast<float(*)[4]>(zw + t * CPL));
              load4(ln.zb + pc0 + t * 8 * CPL, *reinterpret_cast<float(*)[4]>(zb + t * CPL));
            }
          }
          COMET_STAMP(tix, 4);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          COMET_STAMP(tix, 5);
          // pass 2: outputs, row by row (mean / rstd once per row, affine weights loaded before the
          // barrier: a load issued after this epilogue's stores would wait for them)
  #pragma unroll
          for (int i = 0; i < MI; ++i)
  #pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int64_t row = prow0 + i * 16 + h * 8;
              if (EDGE && row >= M) continue;
              float mu, var;
              rowstats(i, h, mu, var);
              const float ry = rsqrtf(var + ln.eps_y), rz = rsqrtf(var + ln.eps_z);
  #pragma unroll
              for (int t = 0; t < NTC; ++t) {
                const int col = pc0 + t * 8 * CPL;
                float y[CPL];
  #pragma unroll
                for (int e = 0; e < CPL; ++e) y[e] = (VK(i, h, t * CPL + e) - mu) * ry;
                if (!ln.raw_c) storen<CPL>(C + row * ldc + col, y);
                if (ln.y16 != nullptr) store4(ln.y16 + row * ln.ldy + col, y);
                if (ln.z16 != nullptr) {
                  float z[CPL];
  #pragma unroll
                  for (int e = 0; e < CPL; ++e)
                    z[e] = (VK(i, h, t * CPL + e) - mu) * rz * zw[t * CPL + e] + zb[t * CPL + e];
                  store4(ln.z16 + row * ln.ldz + col, z);
                }
              }
            }
  #pragma unroll
          for (int i = 0; i < MI; ++i)
  #pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        };
        if (interior) lnepilogue(std::false_type{});
        else lnepilogue(std::true_type{});
        // the next tile's k-step-0 fragments again (buffer (q+1)&1 still holds k-tile q+1): the
        // copies read during k-step 1 are dead here, so their registers serve the epilogue
        if constexpr (!PING) read_frags(qa1_, (q_ + 1) & 1, 0, a0, b0);
      } else if (BPARK && interior && epi.bpark) {
        if constexpr (BPARK) {
          __bf16* slab0 = smem + RING + wid * 2 * BSLAB;
          const int rr = lane >> 3, cc = lane & 7;
          float bc[NI][4];
  #pragma unroll
          for (int j = 0; j < NI; ++j)
  #pragma unroll
            for (int e = 0; e < 4; ++e) bc[j][e] = 0.f;
          if (epi.bias != nullptr) {  // one uniform branch around straight-line loads
  #pragma unroll
            for (int j = 0; j < NI; ++j)
  #pragma unroll
              for (int e = 0; e < 4; ++e) bc[j][e] = epi.bias[col0 + j * 16 + e];
          }
          // per-lane output bases: rows srow0 + i*16 + h*8 (the block offsets are uniform)
          const int64_t srow0 = (int64_t)tm * TBM + wr * WROWS + rr;
          const int64_t scol = (int64_t)tn * TBN + wc * WCOLS + cc * 8;
          TC* cbase = C + srow0 * ldc + scol;
          // slab layout: row r (0..15) of the block, 16-B chunk k stored at chunk k ^ (r & 7), and the
          // two 8-B halves of a chunk swapped for rows 8..15 (the fragment writes -- rows li and li + 8
          // in one lane group -- then hit distinct banks; the row reads are conflict-free)
          const int wofs = li * WCOLS + ((g & 1) ^ (li >> 3)) * 4;
          const int rofs = rr * WCOLS + ((cc ^ rr) << 3);
          // PRE: the activation is applied before parking (no pre-activation copy); otherwise the parked
          // pre-activation is stored to X and the activation applied to the re-read values. Two
          // straight-line bodies: a per-element branch on X splits the GELU chains into basic blocks.
          auto body = [&](auto pre_t) {
            constexpr bool PRE = decltype(pre_t)::value;
            TC* xbase = PRE ? nullptr : X + srow0 * epi.ldaux + scol;
  #pragma unroll
            for (int i = 0; i < MI; ++i) {
              __bf16* slab = slab0 + (i & 1) * BSLAB;
  #pragma unroll
              for (int j = 0; j < NI; ++j) {
                float v[4];
  #pragma unroll
                for (int e = 0; e < 4; ++e) {
                  v[e] = epi.alpha * acc[i][j][e] + bc[j][e];
                  if constexpr (PRE) v[e] = apply_act(ACT, v[e]);
                }
                *reinterpret_cast<uint2*>(slab + wofs + (((2 * j + (g >> 1)) ^ (li & 7)) << 3)) =
                    uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
                acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
              }
              asm volatile("" ::: "memory");
  #pragma unroll
              for (int h = 0; h < 2; ++h) {
                uint4 d = *reinterpret_cast<const uint4*>(slab + h * 8 * WCOLS + rofs);
                if (h == 1) d = uint4{d.z, d.w, d.x, d.y};
                const int64_t roff = (int64_t)(i * 16 + h * 8);
                if constexpr (!PRE) {
                  *reinterpret_cast<uint4*>(xbase + roff * epi.ldaux) = d;
                  const unsigned u[4] = {d.x, d.y, d.z, d.w};
                  unsigned o[4];
  #pragma unroll
                  for (int e = 0; e < 4; ++e)
                    o[e] = pack_bf16x2(apply_act(ACT, bf16_lo(u[e])), apply_act(ACT, bf16_hi(u[e])));
                  d = uint4{o[0], o[1], o[2], o[3]};
                }
                *reinterpret_cast<uint4*>(cbase + roff * ldc) = d;
              }
              asm volatile("" ::: "memory");
            }
          };
          if (X == nullptr) body(std::true_type{});
          else body(std::false_type{});
          if constexpr (!PING) read_frags(qa1_, (q_ + 1) & 1, 0, a0, b0);
        }
      } else if constexpr (BPARK) {
        epilogue(std::true_type{});  // edge tiles (or unaligned outputs): masked direct stores
      } else if constexpr (PARK) {
        // parked epilogue: per 8-row half of each 16-row block the wave parks its 8 x WCOLS raw
        // accumulators in its own LDS slab (no barrier: only this wave touches it) and re-reads them
        // row-contiguously, so every store / residual load instruction covers 8 rows x 128 B
        constexpr int CPL = 16 / (int)sizeof(TC);       // output columns per lane per access (16 B)
        constexpr int NTC = WCOLS / (8 * CPL);          // column passes per row
        float* park = reinterpret_cast<float*>(smem + RING) + wid * 8 * PPITCH;
        const int rr = lane >> 3, cc = lane & 7;
        const int64_t prow0 = (int64_t)tm * TBM + wr * WROWS + rr;        // + i*16 + h*8
        const int64_t pcol0 = (int64_t)tn * TBN + wc * WCOLS + cc * CPL;  // + t*8*CPL
        auto pepilogue = [&](auto edge_t) {
          constexpr bool EDGE = decltype(edge_t)::value;
          const bool bias_c = epi.bias != nullptr;  // per-column bias only (pp_ok)
          float bcp[NTC][CPL];
  #pragma unroll
          for (int t = 0; t < NTC; ++t)
  #pragma unroll
            for (int e = 0; e < CPL; ++e) bcp[t][e] = 0.f;
          if (bias_c) {
  #pragma unroll
            for (int t = 0; t < NTC; ++t)
  #pragma unroll
              for (int e = 0; e < CPL; ++e) {
                const int64_t col = pcol0 + t * 8 * CPL + e;
                bcp[t][e] = epi.bias[EDGE ? (col < N ? col : N - 1) : col];
              }
          }
          // residual rows prefetched RD (i, h) steps ahead into a register ring (the next tile's
          // k-step-0 fragments are re-read after the epilogue, so their registers hold the ring):
          // each step's residual load then has RD - 1 steps of park / store work to land in (3 steps:
          // epilogue 39.5k -> 32.1k cycles per 256 x 256 f32 tile, K 3072 GEMM 835 -> 900 TF/s)
          constexpr int NSTEP = 2 * MI, RD = HASR ? 4 : 1;
          float rq[RD][NTC][CPL];
          auto rld = [&](int st, float (&dst)[NTC][CPL]) {
            const int64_t row = prow0 + (st >> 1) * 16 + (st & 1) * 8;
  #pragma unroll
            for (int t = 0; t < NTC; ++t) {
              const int64_t col = pcol0 + t * 8 * CPL;
              if (!EDGE || (row < M && col < N)) loadn<CPL>(R + row * epi.ldr + col, dst[t]);
            }
          };
          if constexpr (HASR) {
  #pragma unroll
            for (int d = 0; d < RD; ++d)
              if (d < NSTEP) rld(d, rq[d]);
          }
  #pragma unroll
          for (int i = 0; i < MI; ++i)
  #pragma unroll
            for (int h = 0; h < 2; ++h) {
              float (&rc)[NTC][CPL] = rq[(2 * i + h) % RD];
              const int64_t row = prow0 + i * 16 + h * 8;
              if ((li >> 3) == h) {
  #pragma unroll
                for (int j = 0; j < NI; ++j)
                  *reinterpret_cast<f32x4*>(park + (li & 7) * PPITCH + (((j * 4 + g) ^ pswz(li & 7)) << 2)) = acc[i][j];
              }
              asm volatile("" ::: "memory");
  #pragma unroll
              for (int t = 0; t < NTC; ++t) {
                const int64_t col = pcol0 + t * 8 * CPL;
                float v[CPL];
  #pragma unroll
                for (int e = 0; e < CPL; e += 4) {
                  const int lc = (t * 8 * CPL + cc * CPL + e) >> 2;
                  const f32x4 p4 = *reinterpret_cast<const f32x4*>(park + rr * PPITCH + ((lc ^ pswz(rr)) << 2));
                  v[e] = p4[0]; v[e + 1] = p4[1]; v[e + 2] = p4[2]; v[e + 3] = p4[3];
                }
                if (!EDGE || (row < M && col < N)) {
  #pragma unroll
                  for (int e = 0; e < CPL; ++e) v[e] = epi.alpha * v[e] + bcp[t][e];
                  if (X) storen<CPL>(X + row * epi.ldaux + col, v);
                  apply_act_n<CPL>(ACT, v);
                  if constexpr (HASR) {
  #pragma unroll
                    for (int e = 0; e < CPL; ++e) v[e] += epi.beta * rc[t][e];
                  }
                  storen<CPL>(C + row * ldc + col, v);
                }
              }
              if constexpr (HASR) {
                if (2 * i + h + RD < NSTEP) rld(2 * i + h + RD, rc);
              }
              asm volatile("" ::: "memory");
              if (h == 1) {
  #pragma unroll
                for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
              }
            }
        };
        if (interior) pepilogue(std::false_type{});
        else pepilogue(std::true_type{});
        if constexpr (HASR) if constexpr (!PING) read_frags(qa1_, (q_ + 1) & 1, 0, a0, b0);
      } else {
      if constexpr (WIDE) {
        if (interior && X == nullptr && epi.wide) {
          // lane (li, g) of fragment (i, j) holds row li, columns 16j + 4g .. +3 (bf16-packed as uint2);
          // permlane16_swap(frag j, frag j+1) exchanges 16-lane groups 1 <-> 0 and 3 <-> 2, after which
          // group g holds 8 contiguous columns: 16(j + (g & 1)) + 8(g >> 1) .. +7
          const bool bias_c = epi.bias != nullptr;
          float bc[NI][4];
  #pragma unroll
          for (int j = 0; j < NI; ++j)
  #pragma unroll
            for (int e = 0; e < 4; ++e) bc[j][e] = bias_c ? epi.bias[col0 + j * 16 + e] : 0.f;
          const int64_t wcol = (int64_t)tn * TBN + wc * WCOLS + 16 * (g & 1) + 8 * (g >> 1);
  #pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int64_t row = row0 + i * 16;
  #pragma unroll
            for (int j = 0; j < NI; j += 2) {
              unsigned pk[2][2];
  #pragma unroll
              for (int u = 0; u < 2; ++u) {
                float v[4];
  #pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = epi.alpha * acc[i][j + u][e] + bc[j + u][e];
                apply_act_n<4>(ACT, v);
                pk[u][0] = pack_bf16x2(v[0], v[1]);
                pk[u][1] = pack_bf16x2(v[2], v[3]);
                acc[i][j + u] = f32x4{0.f, 0.f, 0.f, 0.f};
              }
              const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
              const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
              *reinterpret_cast<uint4*>(C + row * ldc + wcol + 16 * j) = uint4{s0[0], s1[0], s0[1], s1[1]};
            }
          }
        } else if (interior) {
          epilogue(std::false_type{});
        } else {
          epilogue(std::true_type{});
        }
      } else {
      if (interior) epilogue(std::false_type{});
      else epilogue(std::true_type{});
      }
      }
      // interior: every VMEM op this epilogue issued came after the LDS-DMA of k-tile q+2 and their
      // count is fixed, so the next barrier wait leaves them in flight
      if (BPARK && interior && epi.bpark) pend = X != nullptr ? 3 : 2;
      else if constexpr (WIDE) pend = (interior && X == nullptr && epi.wide) ? 1 : 0;
      else pend = interior ? 1 : 0;
      COMET_STAMP(tix, 2);
  };
  if constexpr (PING) {
    // ---- ping-pong k-loop (256 x 256 tiles; PING instances): 32-deep k-steps through a 4-slot ring
    // of [A 256 x 32 | B 256 x 32] images (the 128 KiB of the lock-step ring). Waves 4-7 run one
    // barrier behind waves 0-3, and each k-step of a wave is a memory segment (its 12 fragments of
    // this k-step, its LDS-DMA pieces of k-step p + 3, the waits) and an MFMA segment (32 MFMAs at
    // raised priority), each closed by a barrier: one group's MFMAs always run beside the other
    // group's reads, DMA issue and barrier waits, where the lock-step loop had both SIMD partners
    // waiting at once (profiles/r05_l: ~1.2k of ~4k cycles per k-tile with the MFMA pipe idle).
    // Fragments are single-buffered (read in the segment that precedes their MFMAs).
    // Hazards (p = global k-step, slot p % 4): the DMA of k-step p + 3 refills the slot of k-step
    // p - 1, whose last reads (group 1's, retired by lgkmcnt(0) before its first barrier of k-step
    // p - 1, which is group 0's second) precede every wave's memory segment of k-step p; the
    // pieces of k-step p + 1 are retired (vmcnt: the two younger k-steps' 8 pieces stay in flight)
    // before the first barrier of k-step p, two barriers before any read of them.
    constexpr int KSA = TBM * 32, KSL = (TBM + TBN) * 32;  // bf16 elements: A image, one slot
    static_assert(TBM == 256 && TBN == 256 && NW == 8 && !LN, "ping-pong k-loop: 256 x 256 tiles, 8 waves");
    static_assert(4 * KSL <= RING, "ping-pong ring");
    const int nks = (int)(K / 32);
    const int P = my_tiles * nks;
    const int grp = wid >> 2;
    // one LDS-DMA piece = 16 rows x 32 k: lane -> row lane >> 2 of the piece, LDS chunk lane & 3
    // holding source chunk (lane & 3) ^ ((row >> 1) & 3); per wave and k-step pieces 2 wid, 2 wid + 1
    // of the A image and of the B image (rows clamped: tail rows re-read the last row, never stored)
    int s_it = 0, s_ks = 0;
    const __bf16* sA = A;
    const __bf16* sB = B;
    int oA[2], oB[2];
    auto pset = [&](int it) {
      int tm, tn;
      tile_rc(off + it * strd, tiles_m, tiles_n, tm, tn);
      const int m0 = tm * TBM, n0 = tn * TBN;
      sA = A + (int64_t)m0 * lda;
      sB = B + (int64_t)n0 * ldb;
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int r = (wid * 2 + pp) * 16 + (lane >> 2);
        const int sw = ((lane & 3) ^ ((r >> 1) & 3)) * 8;
        oA[pp] = (min(m0 + r, (int)M - 1) - m0) * (int)lda + sw;
        oB[pp] = (min(n0 + r, (int)N - 1) - n0) * (int)ldb + sw;
      }
    };
    // the pieces of the stream's next k-step into `slot`; past the end a re-load of the last one.
    // Issued from inline asm: hipcc cannot tell the slot a ds_read reads from the slots the DMA
    // fills and, seeing the builtin, waits vmcnt(0) before every k-step's first read -- that would
    // cut the 2-k-step landing time of each piece to one. The counted waits below order them.
    auto glds_asm = [](const __bf16* src, const __bf16* dst) {
      const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const lds_void*)dst);
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" :: "s"(la), "v"(src) : "m0");
    };
    auto pissue = [&](int slot) {
      const __bf16* a = sA + s_ks * 32;
      const __bf16* b = sB + s_ks * 32;
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) glds_asm(a + oA[pp], smem + slot * KSL + (wid * 2 + pp) * 512);
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) glds_asm(b + oB[pp], smem + slot * KSL + KSA + (wid * 2 + pp) * 512);
      if (++s_ks == nks) {
        if (s_it + 1 < my_tiles) { s_ks = 0; pset(++s_it); }
        else s_ks = nks - 1;
      }
    };
    bf16x8 fa[MI], fb[NI];
    auto pread = [&](int slot) {
      const __bf16* ai = smem + slot * KSL;
      const __bf16* bi = ai + KSA;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = wr * WROWS + i * 16 + li;
        fa[i] = *reinterpret_cast<const bf16x8*>(ai + r * 32 + ((g ^ ((r >> 1) & 3)) << 3));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int r = wc * WCOLS + j * 16 + li;
        fb[j] = *reinterpret_cast<const bf16x8*>(bi + r * 32 + ((g ^ ((r >> 1) & 3)) << 3));
      }
    };
    pset(0);
    pissue(0);
    pissue(1);
    pissue(2);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's pieces of k-step 0
    asm volatile("s_barrier" ::: "memory");
    if (grp) asm volatile("s_barrier" ::: "memory");  // waves 4-7: one barrier behind from here on
    // tiles outer, k-steps inner: the inner loop holds no load hipcc tracks, so the waits it owes to
    // the epilogue's loads land once before it (a single loop over all k-steps put them, as
    // vmcnt(0), at the top of every k-step: the DMA of the next two k-steps drained each time)
    int p = 0;
    for (int it = 0; it < my_tiles; ++it) {
      for (int kk = 0; kk < nks; ++kk, ++p) {
        pread(p & 3);
        pissue((p + 3) & 3);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // k-step p + 1 landed (this wave's pieces)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (!(grp && p + 1 == P)) asm volatile("s_barrier" ::: "memory");  // waves 4-7 skip their last
        __builtin_amdgcn_sched_barrier(0);
      }
      pend = 0;
      tile_epilogue(it, 0, 0);
      pend = 0;
      // drain the epilogue's stores with a builtin (not asm) wait: hipcc's wait insertion sees it.
      // Left in flight, the stores' data registers stay pending in hipcc's model and it waits
      // vmcnt(0) before the first fragment read of every k-step (those registers are reused),
      // draining the DMA of the next two k-steps each time; here it drains once per tile.
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt unchanged
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stream's trailing re-loads land before exit
  } else {
  // ---- prologue: k-tiles 0 and 1 in flight, k-tile 0 landed, its first-k-step fragments read
  set_tile_a(0);
  set_tile_b(0);
  if constexpr (AR) {
    // B0 A0 A1 | B1 A2: the wait leaves A1 and the second batch in flight (past the end of a short
    // stream the extra pieces re-load the last k-tile into slots nothing reads)
    issue_b(0);
    advance_b();
    issue_a(0);
    advance_a();
    issue_a(1);
    advance_a();
    issue_cur(2, 1);
    advance();
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PA + PB) : "memory");
  } else {
    issue_cur(0, 0);
    advance();
    if (T > 1) {
      issue_cur(1, 1);
      advance();
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PA + PB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  asm volatile("s_barrier" ::: "memory");
  read_frags(0, 0, 0, a0, b0);
  int qa = 0;  // q % NA: the A slot of k-tile q (its B slot is q & 1)

  for (int q = 0; q < T; ++q) {
    const int qa1 = qa + 1 == NA ? 0 : qa + 1;
    if (q % nk == 0) COMET_STAMP(q / nk, 0);
#ifdef COMET_GEMM_STAMPS
    const bool kst = nk > 4 && q % nk == 3;
    if (kst) COMET_KSTAMP(q / nk, 3);
#endif
    // ---- k-step 0 of k-tile q: MFMAs on (a0, b0), reads of the k-step-1 fragments (a1, b1)
    read_frags(qa, q & 1, 1, a1, b1);
    mfmas(a0, b0);
#pragma unroll
    for (int t = 0; t < NRD; ++t) {
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DSR, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF / NRD - 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF % NRD, 0);
    // every wave's reads of buffer q&1 and LDS-DMA of k-tile q+1 are done past this barrier; after
    // an interior tile's epilogue its stores (all issued after that LDS-DMA) stay in flight
#ifdef COMET_GEMM_STAMPS
    if (kst) COMET_KSTAMP(q / nk, 4);
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (pend == 2) {  // bf16-park epilogue: 2 x MI stores
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + 2 * MI > 63 ? 63 : XA + 2 * MI) : "memory");
      pend = 0;
    } else if (pend == 3) {  // bf16-park epilogue with the pre-activation copy: 4 x MI stores
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + 4 * MI > 63 ? 63 : XA + 4 * MI) : "memory");
      pend = 0;
    } else if (pend) {
      // VMEM ops per output kind of one epilogue: direct MI x NI, parked 2 x MI x (WCOLS / (8 * CPL))
      constexpr int PER = PARK ? 2 * MI * (WCOLS / (8 * (16 / (int)sizeof(TC)))) : (WIDE ? MI * NI / 2 : MI * NI);
      constexpr int E = PER * (1 + (HASR ? 1 : 0)) + PER;  // C stores (+ resid loads) (+ aux stores)
      if constexpr (LN) {
        // C stores (+ resid loads) + one store per (row half, column pass) of each bf16 output
        // (a lower bound of the VMEM ops issued after the LDS-DMA: bias / affine loads only add)
        constexpr int E1 = E - PER, E2 = E1 + PER, E3 = E1 + 2 * PER;
        const int nb = (ln.y16 != nullptr) + (ln.z16 != nullptr);
        if (nb == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + E1 > 63 ? 63 : XA + E1) : "memory");
        else if (nb == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + E2 > 63 ? 63 : XA + E2) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + E3 > 63 ? 63 : XA + E3) : "memory");
      } else if (epi.aux) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + E > 63 ? 63 : XA + E) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA + E - PER > 63 ? 63 : XA + E - PER) : "memory");
      pend = 0;
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA) : "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
#ifdef COMET_GEMM_STAMPS
    if (kst) COMET_KSTAMP(q / nk, 5);
#endif
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#ifdef COMET_GEMM_STAMPS
    if (kst) COMET_KSTAMP(q / nk, 6);
#endif
    // ---- k-step 1: MFMAs on (a1, b1); LDS-DMA of k-tile q+2 into buffer q&1 (past the end of the
    // stream: a re-load of the last k-tile that nothing reads); reads of k-tile q+1's k-step-0
    // fragments (a0, b0) from buffer (q+1)&1 (garbage past the end, never used). Branch-free.
    const bool tile_end = (q + 1) % nk == 0;
    {
      issue_cur(qa, q & 1);
      read_frags(qa1, (q + 1) & 1, 0, a0, b0);
      mfmas(a1, b1);
      // per group of NMF / NRD MFMAs: one fragment read; LDS-DMA pieces (PA + PB) spread evenly
#pragma unroll
      for (int t = 0; t < NRD; ++t) {
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
        if (t < PA + PB) __builtin_amdgcn_sched_group_barrier(SG_VMR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DSR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF / NRD - 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF % NRD, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#ifdef COMET_GEMM_STAMPS
    if (kst) COMET_KSTAMP(q / nk, 7);
#endif
    advance();
    qa = qa1;
    if (!tile_end) continue;
    tile_epilogue(q / nk, q, qa1);
  }
  // The k-tile stream runs two k-tiles past the last one (re-loads nothing reads), so up to two
  // batches of LDS-DMA pieces can still be in flight here when the last epilogue issued no load of
  // its own (bf16 outputs of a Linear without bias: the tracker's q / kv projections). Drained so
  // no workgroup ends with LDS writes pending (round 6: comet_lds_probe workgroups placed on a CU as
  // these leave saw no late write with or without this wait, tools/lds_race.py; one wait per
  // workgroup and kernel, kept as the guarantee)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}
}  // namespace w4


int g_num_cus = 0;
int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}

// Eligible: bf16 k-contiguous A / B (16-B aligned rows), K % 64 == 0, one batch, no split, output /
// residual / aux rows allow 4-column vector access, N a multiple of 4 and a 256-column tile
// wasting <= 15 % of the columns, enough rows to fill the chip.
bool pp_ok(const comet_gemm_args& a) {
  if (getenv("COMET_GEMM_NO_PP") != nullptr) return false;
  if (a.dtype_ab != COMET_BF16 || a.convert_a || a.convert_b || a.layout_a != 0 || a.layout_b != 0) return false;
  if (a.batch[0] * a.batch[1] != 1 || a.k % 64 != 0 || a.k == 0 || a.split_k > 1) return false;
  if (a.bias && a.bias_mode != 1) return false;
  if ((uintptr_t)a.a % 16 != 0 || (uintptr_t)a.b % 16 != 0 || a.lda % 8 != 0 || a.ldb % 8 != 0) return false;
  if (a.m < 4096 || a.n < 256 || a.n % 4 != 0 || a.m >= (1ll << 31) || a.n >= (1ll << 31)) return false;
  if (a.n == 384 && getenv("COMET_GEMM_NO_PP384") != nullptr) return false;
  if (a.lda * 384 + 64 >= (1ll << 31) || a.ldb * 384 + 64 >= (1ll << 31)) return false;  // 32-bit offsets
  // in-step per-shape profile (tools/gemm_shapes.py): with a second (aux) output its direct
  // 8-byte-per-lane bf16 stores lose to the parked 16-B row stores of the 256-row kernel
  if (a.aux != nullptr && getenv("COMET_GEMM_PP_ALL_K") == nullptr) return false;
  const int64_t w256 = cdiv(a.n, 256) * 256 - a.n;
  if (a.n != 384 && w256 * 100 > 15 * a.n && getenv("COMET_GEMM_PP_ANY_N") == nullptr) return false;
  const int es = a.dtype_c == COMET_F32 ? 4 : 2;
  auto v4 = [&](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % (4 * es) == 0 && ld % 4 == 0); };
  return v4(a.c, a.ldc) && v4(a.resid, a.ldr) && v4(a.aux, a.ldaux);
}

// Tile of the persistent kernel: 128 x 384 for N = 384 (the tracker's hidden size: each A row
// block read once), else 256 x 256; half-height (64 x 384, 128 x 256) when the full-height tiles
// leave CUs idle (M = 8192: the tracker's virtual tracks x frames x batch).
void pp_tile_base(const comet_gemm_args& a, int& tbm, int& tbn) {
  int cus = num_cus();
  cus -= cus % 8;
  tbn = a.n == 384 ? 384 : 256;
  tbm = a.n == 384 ? 128 : 256;
  if (cdiv(a.m, tbm) * cdiv(a.n, tbn) < cus) tbm /= 2;
}

// plain GEMMs: the base tile, or COMET_PP_TILE=256x256 | 128x256 | 128x384 | 64x384 (measurement
// override, tools/tile_bench.py)
void pp_tile(const comet_gemm_args& a, int& tbm, int& tbn) {
  pp_tile_base(a, tbm, tbn);
  // small M (the tracker's virtual tracks, M = 8192): when 128 x 384 tiles fill 75-100 % of the
  // CUs in one round they beat the 1.5-round 128 x 256 grid (N = 1536: 23.7 vs 30.1 us; N = 1152:
  // 19.6 vs 22.8 us; profiles/r02_tile)
  int cus = num_cus();
  cus -= cus % 8;
  const int64_t t384 = cdiv(a.m, 128) * (a.n / 384);
  if (a.n != 384 && a.n % 384 == 0 && 4 * t384 >= 3 * (int64_t)cus && t384 <= cus && getenv("COMET_PP_NO_384") == nullptr) {
    tbm = 128;
    tbn = 384;
  }
  if (const char* t = getenv("COMET_PP_TILE")) {
    int m = 0, n = 0;
    if (sscanf(t, "%dx%d", &m, &n) == 2 && ((n == 256 && (m == 256 || m == 128)) || (n == 384 && (m == 128 || m == 64)))) {
      tbm = m;
      tbn = n;
    }
  }
}

// Few-row row-LN GEMMs (M <= 32 x CUs: the tracker's 8192 virtual-track tokens) with a long K: the
// persistent row-LN kernel gives each CU one 32 x 384 tile whose 24 k-tiles of weights (48 KiB each)
// run behind one load in flight (33.6 us at M 8192 K 1536). Instead: split-K partials of the plain
// 256-row kernel (raw f32, K / S each, tiles x S ~ one round of CUs), then one reduce that sums the
// partials in split order, adds bias and residual and writes the LayerNorm outputs, one wave per
// row (rowln_reduce_kernel). 0 = not taken (COMET_ROWLN_NOSPLIT=1 disables it).
int rowln_splits(const comet_gemm_args& a) {
  if ((a.n != 384 && a.n != 256) || getenv("COMET_ROWLN_NOSPLIT") != nullptr) return 0;
  const int grid = num_cus();
  if (cdiv(a.m, 32) > grid) return 0;
  const int64_t tiles = cdiv(a.m, big::BM) * cdiv(a.n, 128), ktiles = a.k / 64;
  int64_t sp = grid / tiles;
  if (sp > ktiles / 6) sp = ktiles / 6;  // >= 6 k-tiles per split
  return sp >= 2 ? (int)sp : 0;
}

int64_t rowln_ws_bytes(const comet_gemm_args& a, int splits) {
  return (int64_t)splits * a.m * a.n * (int64_t)sizeof(float);
}

// One wave per row, N <= 512 and N % 4 == 0: lane l owns columns 4l + 256j. v = alpha * sum of the
// partials (split order) + bias + beta * resid, then the RowLN outputs (two-pass-free: sum and sum of
// squares by wave shuffles, var = E[v^2] - mean^2 clamped at 0, as the persistent kernel).
__global__ void __launch_bounds__(256)
rowln_reduce_kernel(const float* __restrict__ ws, int splits, int64_t M, int N, const float* __restrict__ bias,
                    const float* __restrict__ resid, int64_t ldr, float alpha, float beta, float* __restrict__ C,
                    int64_t ldc, w4::RowLN ln) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[2][4];
  float s = 0.f, sq = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = 4 * lane + 256 * j;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[j][e] = 0.f;
    if (col >= N) continue;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < splits; ++z) {
      const f32x4 p = *reinterpret_cast<const f32x4*>(ws + ((int64_t)z * M + row) * N + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += p[e];
    }
    const f32x4 r = *reinterpret_cast<const f32x4*>(resid + row * ldr + col);
    f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bias != nullptr) b = *reinterpret_cast<const f32x4*>(bias + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float o = alpha * acc[e] + b[e] + beta * r[e];
      v[j][e] = o;
      s += o;
      sq = fmaf(o, o, sq);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    s += __shfl_xor(s, m, 64);
    sq += __shfl_xor(sq, m, 64);
  }
  const float invn = 1.f / (float)N;
  const float mu = s * invn, var = fmaxf(sq * invn - mu * mu, 0.f);
  const float ry = rsqrtf(var + ln.eps_y), rz = rsqrtf(var + ln.eps_z);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = 4 * lane + 256 * j;
    if (col >= N) continue;
    float y[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = (v[j][e] - mu) * ry;
    *reinterpret_cast<f32x4*>(C + row * ldc + col) =
        ln.raw_c ? f32x4{v[j][0], v[j][1], v[j][2], v[j][3]} : f32x4{y[0], y[1], y[2], y[3]};
    if (ln.y16 != nullptr) store4(ln.y16 + row * ln.ldy + col, y);
    if (ln.z16 != nullptr) {
      const f32x4 zw = *reinterpret_cast<const f32x4*>(ln.zw + col), zb = *reinterpret_cast<const f32x4*>(ln.zb + col);
      float z[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) z[e] = (v[j][e] - mu) * rz * zw[e] + zb[e];
      store4(ln.z16 + row * ln.ldz + col, z);
    }
  }
}

int launch_rowln_split(const comet_gemm_args& a, const w4::RowLN& ln, int splits, hipStream_t s) {
  Epi e{nullptr, 0, 0, 0, nullptr, 0, 0, 0, 0.f, nullptr, 0, 0, 0, 1.f, COMET_ACT_NONE, 1};
  const int64_t tiles_m = cdiv(a.m, big::BM), tiles_n = cdiv(a.n, 128);
  const int64_t kchunk = cdiv(a.k / 64, splits) * 64;
  splits = (int)cdiv(a.k, kchunk);
  Split sp{reinterpret_cast<float*>(a.workspace), kchunk};
  hipLaunchKernelGGL((big::gemm_big_kernel<float, 128, 0, 0, true>), dim3((unsigned)(tiles_m * tiles_n), (unsigned)splits),
                     dim3(big::NT), 0, s, (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (float*)nullptr, a.ldc,
                     a.m, a.n, a.k, (int)tiles_n, e, sp);
  COMET_CHECK_LAUNCH("comet_gemm_rowln (split-K partials)");
  hipLaunchKernelGGL(rowln_reduce_kernel, dim3((unsigned)cdiv(a.m, 4)), dim3(256), 0, s, sp.ws, splits, a.m, (int)a.n,
                     a.bias_mode == 1 ? a.bias : nullptr, reinterpret_cast<const float*>(a.resid), a.ldr, a.alpha,
                     a.beta, reinterpret_cast<float*>(a.c), a.ldc, ln);
  COMET_CHECK_LAUNCH("comet_gemm_rowln (LN reduce)");
  return COMET_OK;
}

// Row-LN launch (comet_gemm_rowln): f32 output with a residual, no activation / aux, one tile
// spanning the row. Instances: 128 x 384 / 64 x 384 / 32 x 384 (N = 384), 128 x 256 (N = 256).
int launch_pp_rowln(const comet_gemm_args& a, const w4::RowLN& ln, hipStream_t s) {
  if (const int sp = rowln_splits(a)) {
    if (a.workspace != nullptr && a.workspace_bytes >= rowln_ws_bytes(a, sp)) return launch_rowln_split(a, ln, sp, s);
  }
  Epi e{a.bias, a.bias_mode, 0, 0, a.resid, a.ldr, 0, 0, a.beta, nullptr, 0, 0, 0, a.alpha, COMET_ACT_NONE, 1};
  e.prio = getenv("COMET_GEMM_PRIO") != nullptr;
  e.raster = getenv("COMET_GEMM_RASTER") != nullptr && getenv("COMET_GEMM_RASTER")[0] == '1';
  int grid = num_cus();
  grid -= grid % 8;
  int tbm, tbn;
  pp_tile_base(a, tbm, tbn);
  // tile rows: full-height 128 x 384 only for long K (K >= 1024: fc2), else the half-height tiles
  // (the full-height LN instances run at 256 VGPRs with spills; tools/rowln_bench.py)
  const bool full = tbn == 384 && a.k >= 1024 && getenv("COMET_ROWLN_HALF") == nullptr;
  if (!full && tbm == (tbn == 384 ? 128 : 256)) tbm /= 2;
  // quarter-height 32 x 384 tiles when the 64-row grid fills at most half the CUs (M = 8192: the
  // tracker's virtual tracks): every CU gets a tile. Default since round 5 (2-5 % faster on every
  // M = 8192 shape, same box, profiles/r05_rowln); COMET_ROWLN_NO32=1 keeps the 64-row tiles
  if (tbn == 384 && tbm == 64 && 2 * cdiv(a.m, 64) <= grid && getenv("COMET_ROWLN_NO32") == nullptr) tbm = 32;
  // measurement: 32-row tiles for every N = 384 shape (COMET_ROWLN_32ALL=1)
  if (tbn == 384 && tbm == 64 && getenv("COMET_ROWLN_32ALL") != nullptr) tbm = 32;
  const int64_t tiles_m = cdiv(a.m, tbm);
  COMET_CHECK_ARG(tbn == a.n && tiles_m < (1ll << 30), "comet_gemm_rowln: the row must fit one tile");
  const int ntiles = (int)tiles_m;
  if (ntiles <= grid) grid = ntiles;
#define PPLN(BMT, BNT)                                                                                         \
  hipLaunchKernelGGL((w4::gemm_w4_kernel<float, COMET_ACT_NONE, true, 8, BMT, BNT, true>), dim3((unsigned)grid), \
                     dim3(512), 0, s, (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (float*)a.c, a.ldc,  \
                     a.m, a.n, a.k, 1, ntiles, e, ln)
  if (tbn == 384) { if (tbm == 32) PPLN(32, 384); else if (tbm == 64) PPLN(64, 384); else PPLN(128, 384); }
  else PPLN(128, 256);
#undef PPLN
  COMET_CHECK_LAUNCH("comet_gemm_rowln (persistent, row LN epilogue)");
  return COMET_OK;
}

template <typename TC>
int launch_pp(const comet_gemm_args& a, hipStream_t s) {
  Epi e{a.bias, a.bias_mode, 0, 0, a.resid, a.ldr, 0, 0, a.beta, a.aux, a.ldaux, 0, 0, a.alpha, a.act, 1};
  e.wide = (uintptr_t)a.c % 16 == 0 && a.ldc % 8 == 0 && getenv("COMET_GEMM_NO_WIDE") == nullptr;
  e.prio = getenv("COMET_GEMM_PRIO") != nullptr;
  // per-XCD contiguous tile ranges: measurement only (COMET_GEMM_RASTER=1). Alone, 4-5 % faster on the
  // K = 768 shapes and 1-6 % slower at K 384 / 3072, with 22 % more L2 fill traffic; as the default
  // for K 512..1024 the step measured 0.1 ms slower (tools/raster_ab.py, profiles/r06_raster)
  e.raster = getenv("COMET_GEMM_RASTER") != nullptr && getenv("COMET_GEMM_RASTER")[0] == '1';
  e.bpark = (uintptr_t)a.c % 16 == 0 && a.ldc % 8 == 0 && (a.aux == nullptr || ((uintptr_t)a.aux % 16 == 0 && a.ldaux % 8 == 0)) &&
            getenv("COMET_GEMM_NO_BPARK") == nullptr;
  const w4::RowLN noln{};
  // N = 384 (the tracker's hidden size): 128 x 384 tiles (each A row block read once);
  // otherwise 256 x 256
  int grid = num_cus();
  grid -= grid % 8;
  int tbm, tbn;
  pp_tile(a, tbm, tbn);
  const bool n384 = tbn == 384, half = tbm == (n384 ? 64 : 128);
  const int64_t tiles_m = cdiv(a.m, tbm), tiles_n = cdiv(a.n, tbn);
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 30), "comet_gemm: too many tiles");
  const int ntiles = (int)(tiles_m * tiles_n);
  if (ntiles <= grid) grid = ntiles;
  // 256 x 256 tiles: the ping-pong k-loop (PING instances) for bf16 outputs without activation,
  // residual or pre-activation copy at K >= 768, and for any output / residual at K >= 2048
  // (profiles/r05_n: 8192^3 +8..14 %, M 74368 N 2304 K 768 +4 %, the f32 + residual K 3072 shape
  // +1..2 %; with GELU at K 768 even, K <= 384 5-9 % slower -- the tile's two wave groups then run
  // their epilogues one after the other and drain the stores once per tile). COMET_GEMM_PING=1 / =0
  // forces it on / off (measurement; read per call, so one test process can run both loops).
  const char* ping_env = getenv("COMET_GEMM_PING");
  const bool ping = ping_env != nullptr ? ping_env[0] == '1'
                                        : (a.aux == nullptr && a.act == COMET_ACT_NONE &&
                                           ((a.k >= 768 && a.dtype_c == COMET_BF16 && a.resid == nullptr) ||
                                            a.k >= 2048));
#define PPKT(ACT, HR, BMT, BNT, PG)                                                                           \
  hipLaunchKernelGGL((w4::gemm_w4_kernel<TC, ACT, HR, 8, BMT, BNT, false, PG>), dim3((unsigned)grid), dim3(512), 0, s, \
                     (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (TC*)a.c, a.ldc, a.m, a.n, a.k,     \
                     (int)tiles_n, ntiles, e, noln)
#define PPK(ACT, HR)                                                                                          \
  do {                                                                                                        \
    if (n384) { if (half) PPKT(ACT, HR, 64, 384, false); else PPKT(ACT, HR, 128, 384, false); }             \
    else if (half) PPKT(ACT, HR, 128, 256, false);                                                            \
    else if (ping) PPKT(ACT, HR, 256, 256, true);                                                             \
    else PPKT(ACT, HR, 256, 256, false);                                                                      \
  } while (0)
#define PPR(ACT) do { if (a.resid) PPK(ACT, true); else PPK(ACT, false); } while (0)
  switch (a.act) {
    case COMET_ACT_GELU: PPR(COMET_ACT_GELU); break;
    case COMET_ACT_RELU: PPR(COMET_ACT_RELU); break;
    case COMET_ACT_SIGMOID: PPR(COMET_ACT_SIGMOID); break;
    default: PPR(COMET_ACT_NONE);
  }
#undef PPR
#undef PPK
#undef PPKT
  COMET_CHECK_LAUNCH("comet_gemm (persistent 256 x 256, 4 waves)");
  return COMET_OK;
}

// 0: not eligible, else the column tile (256 or 128) wasting the fewest columns
int big_bn(const comet_gemm_args& a) {
  if (getenv("COMET_GEMM_NO_BIG") != nullptr) return 0;
  if (a.dtype_ab != COMET_BF16 || a.convert_a || a.convert_b) return 0;
  const bool wide = a.layout_a == 1 || a.layout_b == 1;  // transposed: dX / dW shapes
  // K % 64 != 0: dW shapes over a ragged token count (e.g. 8 x 15 x 577) run the 64-multiple part
  // here as split-K partials and the < 64 remainder as one more partial (comet_gemm)
  const bool ragged_ok = wide && a.k >= 1024 && getenv("COMET_GEMM_NO_RAGGED") == nullptr;
  if (a.batch[0] * a.batch[1] != 1 || (a.k % 64 != 0 && !ragged_ok) || a.k == 0) return 0;
  if ((uintptr_t)a.a % 16 != 0 || (uintptr_t)a.b % 16 != 0 || a.lda % 8 != 0 || a.ldb % 8 != 0) return 0;
  if ((a.layout_a == 1 && a.m % 8 != 0) || (a.layout_b == 1 && a.n % 8 != 0)) return 0;
  if (!wide && a.m < 4096) return 0;
  if (a.m < 256 || a.n < 128) return 0;
  // short-K weight gradients over few 256-row tiles (M = N = 768, K = 128 tokens: 9 workgroups)
  // run faster as 36 128 x 128 tiles
  if (wide && a.k < 16 * 64 && cdiv(a.m, 256) * cdiv(a.n, 256) * 4 <= 256 && getenv("COMET_GEMM_NO_SMALLSPLIT") == nullptr)
    return 0;
  const int64_t w256 = cdiv(a.n, 256) * 256 - a.n, w128 = cdiv(a.n, 128) * 128 - a.n;
  if (a.n >= 512 && w256 * 100 <= 15 * a.n) return 256;
  if (a.n % 256 == 0 || (a.n >= 512 && w128 * 100 <= 15 * a.n)) return 128;  // N = 384: 128 x 128 measured faster
  return 0;
}

struct Plan {
  int kind;      // 0 skinny, 1 256-row tile, 2 128 x 128 tile, 3 persistent tile kernel,
                 // 4 two-workgroups-per-CU 256 x 128 kernel (removed)
  int bn;        // kind 1, 3: column tile
  int splits;    // requested K splits (before the workspace check)
  int bm = 0;    // kind 3: row tile
  int tail = 0;  // kind 1: K % 64 (one extra split-K partial computed by the 128 x 128 kernel)
};

Plan make_plan(const comet_gemm_args& a);
int64_t plan_workspace(const comet_gemm_args& a, const Plan& p) {
  if (p.tail) return (int64_t)(p.splits + 1) * a.m * a.n * (int64_t)sizeof(float);
  if (p.splits <= 1) return 0;
  return (int64_t)p.splits * a.batch[0] * a.batch[1] * a.m * a.n * (int64_t)sizeof(float);
}

// extra > 0: split mode even for one split, and the reduce also sums `extra` partial slots that
// precede a.workspace (the ragged-K remainder)
template <typename TC, int BN, int LA, int LB>
int launch_big(const comet_gemm_args& a, int splits, hipStream_t s, int extra = 0) {
  auto v8 = [](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 32 == 0 && ld % 8 == 0); };
  const int vec = a.n % 8 == 0 && v8(a.c, a.ldc) && v8(a.resid, a.ldr) && v8(a.aux, a.ldaux);
  Epi e{a.bias, a.bias_mode, 0, 0, a.resid, a.ldr, 0, 0, a.beta, a.aux, a.ldaux, 0, 0, a.alpha, a.act, vec};
  const int64_t tiles_m = cdiv(a.m, big::BM), tiles_n = cdiv(a.n, BN);
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "comet_gemm: too many tiles");
  int64_t kchunk = a.k;
  if (splits > 1) {
    kchunk = cdiv(a.k / 64, splits) * 64;
    splits = (int)cdiv(a.k, kchunk);
  }
  Split sp{reinterpret_cast<float*>(a.workspace), kchunk};
  dim3 grid((unsigned)(tiles_m * tiles_n), (unsigned)splits);
  if (splits > 1 || extra > 0) {
    hipLaunchKernelGGL((big::gemm_big_kernel<float, BN, LA, LB, true>), grid, dim3(big::NT), 0, s,
                       (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (float*)nullptr, a.ldc, a.m, a.n, a.k,
                       (int)tiles_n, e, sp);
    COMET_CHECK_LAUNCH("comet_gemm (256-row tile, split)");
    const int64_t work = a.m * cdiv(a.n, 4);
    int64_t blocks = cdiv(work, 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL((splitk_reduce_kernel<TC>), dim3((unsigned)blocks), dim3(256), 0, s,
                       sp.ws - (int64_t)extra * a.m * a.n, splits + extra, (int64_t)1,
                       (int64_t)1, (TC*)a.c, a.ldc, (int64_t)0, (int64_t)0, a.m, a.n, e);
    COMET_CHECK_LAUNCH("comet_gemm split-K reduce");
    return COMET_OK;
  }
  hipLaunchKernelGGL((big::gemm_big_kernel<TC, BN, LA, LB, false>), grid, dim3(big::NT), 0, s,
                     (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (TC*)a.c, a.ldc, a.m, a.n, a.k,
                     (int)tiles_n, e, sp);
  COMET_CHECK_LAUNCH("comet_gemm (256-row tile)");
  return COMET_OK;
}

template <typename TC, int BN>
int launch_big_layout(const comet_gemm_args& a, int splits, hipStream_t s, int extra = 0) {
  if (a.layout_a == 0 && a.layout_b == 0) return launch_big<TC, BN, 0, 0>(a, splits, s, extra);
  if (a.layout_a == 0 && a.layout_b == 1) return launch_big<TC, BN, 0, 1>(a, splits, s, extra);
  if (a.layout_a == 1 && a.layout_b == 0) return launch_big<TC, BN, 1, 0>(a, splits, s, extra);
  return launch_big<TC, BN, 1, 1>(a, splits, s, extra);
}

// ---- host side --------------------------------------------------------------------------
constexpr int kCUs = 256;

// Number of K splits: only when the output tiles cannot fill the chip and each split still
// runs >= 8 k-tiles (splits * tiles ~ 2 waves of workgroups over the CUs).
int choose_splits(const comet_gemm_args& a) {
  if (a.split_k >= 1) return a.split_k;
  const int64_t tiles = cdiv(a.m, BM) * cdiv(a.n, BN) * a.batch[0] * a.batch[1];
  const int bk = a.dtype_ab == COMET_BF16 ? bf::BK : f32::BK;
  const int64_t ktiles = cdiv(a.k, bk);
  if (tiles >= kCUs || ktiles < 16) {
    // few tiles over a short K (the camera trunk's M = 128 token GEMMs: 6 tiles ran 12 serial
    // k-tiles each on 6 CUs): split while every split keeps >= 2 k-tiles (bf16 operands only)
    if (a.dtype_ab == COMET_BF16 && tiles * 4 <= kCUs && ktiles >= 4 && getenv("COMET_GEMM_NO_SMALLSPLIT") == nullptr) {
      int64_t s = cdiv(2 * kCUs, tiles);
      if (s > ktiles / 2) s = ktiles / 2;
      if (s > 64) s = 64;
      return s < 1 ? 1 : (int)s;
    }
    return 1;
  }
  int64_t s = cdiv(2 * kCUs, tiles);
  const int64_t smax = ktiles / 8;
  if (s > smax) s = smax;
  if (s > 64) s = 64;
  return s < 1 ? 1 : (int)s;
}

Plan make_plan(const comet_gemm_args& a) {
  if (skinny_ok(a)) return Plan{0, 0, 1};
  if (pp_ok(a)) {
    int tbm, tbn;
    pp_tile(a, tbm, tbn);
    return Plan{3, tbn, 1, tbm};
  }
  if (const int bn = big_bn(a)) {
    int sp = 1;
    if (a.split_k >= 1) {
      sp = a.split_k;
    } else {
      const int64_t tiles = cdiv(a.m, big::BM) * cdiv(a.n, bn), ktiles = a.k / 64;
      if (tiles < kCUs && ktiles >= 16) {
        // one full round of workgroups (one 256-row workgroup per CU): 36 dW tiles x 7 splits run
        // K/7 per CU, where ~2 rounds (x 15) ran 3 rounds of K/15 and doubled the partials
        int64_t s2 = kCUs / tiles;
        if (s2 > ktiles / 8) s2 = ktiles / 8;
        if (s2 > 64) s2 = 64;
        sp = s2 < 1 ? 1 : (int)s2;
      }
    }
    return Plan{1, bn, sp, 0, (int)(a.k % 64)};
  }
  return Plan{2, 0, choose_splits(a)};
}

int64_t workspace_bytes(const comet_gemm_args& a, int splits) {
  if (splits <= 1) return 0;
  return (int64_t)splits * a.batch[0] * a.batch[1] * a.m * a.n * (int64_t)sizeof(float);
}

struct LaunchCfg {
  Epi e; Split sp; dim3 grid; int tiles_n; int splits;
};

// Epilogue flags, split count and grid shared by the bf16 and f32 launchers.
int prepare(const comet_gemm_args& a, int bk, LaunchCfg& L) {
  const int64_t tiles_m = cdiv(a.m, BM), tiles_n = cdiv(a.n, BN);
  const int64_t nb = a.batch[0] * a.batch[1];
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "comet_gemm: too many tiles");
  COMET_CHECK_ARG(nb <= 65535, "comet_gemm: batch too large (max 65535)");
  auto v8 = [](const void* p, int64_t ld, const int64_t* st) {
    return p == nullptr || ((uintptr_t)p % 32 == 0 && ld % 8 == 0 && st[0] % 8 == 0 && st[1] % 8 == 0);
  };
  const int vec = a.n % 8 == 0 && v8(a.c, a.ldc, a.stride_c) && v8(a.resid, a.ldr, a.stride_r) &&
                  v8(a.aux, a.ldaux, a.stride_aux);
  L.e = Epi{a.bias, a.bias_mode, a.stride_bias[0], a.stride_bias[1],
            a.resid, a.ldr, a.stride_r[0], a.stride_r[1], a.beta,
            a.aux, a.ldaux, a.stride_aux[0], a.stride_aux[1], a.alpha, a.act, vec};
  int splits = choose_splits(a);
  if (splits > 1 && (a.workspace == nullptr || a.workspace_bytes < workspace_bytes(a, splits))) splits = 1;
  int64_t kchunk = a.k;
  if (splits > 1) {
    kchunk = cdiv(cdiv(a.k, bk), splits) * bk;
    splits = (int)cdiv(a.k, kchunk);
  }
  L.sp = Split{reinterpret_cast<float*>(a.workspace), kchunk};
  L.grid = dim3((unsigned)(tiles_m * tiles_n), (unsigned)nb, (unsigned)splits);
  L.tiles_n = (int)tiles_n;
  L.splits = splits;
  return COMET_OK;
}

template <typename TC>
int reduce_splits(const comet_gemm_args& a, const LaunchCfg& L, hipStream_t s) {
  const int64_t nb = a.batch[0] * a.batch[1];
  const int64_t work = nb * a.m * cdiv(a.n, 4);
  int64_t blocks = cdiv(work, 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL((splitk_reduce_kernel<TC>), dim3((unsigned)blocks), dim3(256), 0, s,
                     L.sp.ws, L.splits, nb, a.batch[1], reinterpret_cast<TC*>(a.c), a.ldc, a.stride_c[0],
                     a.stride_c[1], a.m, a.n, L.e);
  COMET_CHECK_LAUNCH("comet_gemm split-K reduce");
  return COMET_OK;
}

template <typename TC, int LA, int LB, int KA, int KB>
int launch_bf16(const comet_gemm_args& a, hipStream_t s) {
  LaunchCfg L;
  int rc = prepare(a, bf::BK, L);
  if (rc != COMET_OK) return rc;
  // split partials are f32 whatever the output type (tiny dW GEMMs like Linear(1, 32) over all
  // tokens have ragged operands and need the split most)
  constexpr bool can_split = true;
  if (!can_split && L.splits > 1) {
    L.splits = 1;
    L.sp.kchunk = a.k;
    L.grid.z = 1;
  }
  if constexpr (can_split) {
    if (L.splits > 1) {
      hipLaunchKernelGGL((bf::gemm_bf16_kernel<float, LA, LB, KA, KB, true>), L.grid, dim3(NT), 0, s,
                         a.a, a.lda, a.stride_a[0], a.stride_a[1], a.b, a.ldb, a.stride_b[0], a.stride_b[1],
                         (float*)nullptr, a.ldc, a.stride_c[0], a.stride_c[1], a.m, a.n, a.k, a.batch[1],
                         L.tiles_n, L.e, L.sp);
      COMET_CHECK_LAUNCH("comet_gemm");
      return reduce_splits<TC>(a, L, s);
    }
  }
  hipLaunchKernelGGL((bf::gemm_bf16_kernel<TC, LA, LB, KA, KB, false>), L.grid, dim3(NT), 0, s,
                     a.a, a.lda, a.stride_a[0], a.stride_a[1], a.b, a.ldb, a.stride_b[0], a.stride_b[1],
                     reinterpret_cast<TC*>(a.c), a.ldc, a.stride_c[0], a.stride_c[1], a.m, a.n, a.k, a.batch[1],
                     L.tiles_n, L.e, L.sp);
  COMET_CHECK_LAUNCH("comet_gemm");
  return COMET_OK;
}

template <typename TC, int LA, int LB, bool VA, bool VB>
int launch_f32(const comet_gemm_args& a, hipStream_t s) {
  LaunchCfg L;
  int rc = prepare(a, f32::BK, L);
  if (rc != COMET_OK) return rc;
  const float* A = reinterpret_cast<const float*>(a.a);
  const float* B = reinterpret_cast<const float*>(a.b);
  if (L.splits > 1) {
    hipLaunchKernelGGL((f32::gemm_f32_kernel<TC, LA, LB, VA, VB, true>), L.grid, dim3(NT), 0, s,
                       A, a.lda, a.stride_a[0], a.stride_a[1], B, a.ldb, a.stride_b[0], a.stride_b[1],
                       reinterpret_cast<TC*>(a.c), a.ldc, a.stride_c[0], a.stride_c[1], a.m, a.n, a.k, a.batch[1],
                       L.tiles_n, L.e, L.sp);
    COMET_CHECK_LAUNCH("comet_gemm");
    return reduce_splits<TC>(a, L, s);
  }
  hipLaunchKernelGGL((f32::gemm_f32_kernel<TC, LA, LB, VA, VB, false>), L.grid, dim3(NT), 0, s,
                     A, a.lda, a.stride_a[0], a.stride_a[1], B, a.ldb, a.stride_b[0], a.stride_b[1],
                     reinterpret_cast<TC*>(a.c), a.ldc, a.stride_c[0], a.stride_c[1], a.m, a.n, a.k, a.batch[1],
                     L.tiles_n, L.e, L.sp);
  COMET_CHECK_LAUNCH("comet_gemm");
  return COMET_OK;
}

// 16-B vector access: base, ld and batch strides multiples of 8 elements (bf16 or converted f32,
// whose 8-element runs are read as 2 x 16 B) or 4 (f32 kernel), contiguous extent likewise.
inline bool vec_ok(const void* p, int64_t ld, const int64_t* st, int64_t contig_extent, int V) {
  return ((uintptr_t)p % 16 == 0) && ld % V == 0 && st[0] % V == 0 && st[1] % V == 0 && contig_extent % V == 0;
}

template <typename TC, int LA, int LB, int KA>
int dispatch_kb(const comet_gemm_args& a, hipStream_t s) {
  const bool vb = vec_ok(a.b, a.ldb, a.stride_b, LB == 0 ? a.k : a.n, 8);
  if (a.convert_b) {
    if constexpr (LB == 1) {
      COMET_CHECK_ARG(vb, "comet_gemm: convert_b needs 16-B aligned f32 B with ld, strides and n multiples of 8");
      return launch_bf16<TC, LA, LB, KA, bf::K_F32_CVT>(a, s);
    }
    set_error("comet_gemm: convert_b is supported for layout_b == 1 only");
    return COMET_EINVAL;
  }
  if (vb) return launch_bf16<TC, LA, LB, KA, bf::K_BF16_VEC>(a, s);
  return launch_bf16<TC, LA, LB, KA, bf::K_BF16_SCALAR>(a, s);
}

template <typename TC, int LA, int LB>
int dispatch_bf16(const comet_gemm_args& a, hipStream_t s) {
  const bool va = vec_ok(a.a, a.lda, a.stride_a, LA == 0 ? a.k : a.m, 8);
  if (a.convert_a) {
    COMET_CHECK_ARG(va, "comet_gemm: convert_a needs 16-B aligned f32 A with ld, strides and contiguous extent multiples of 8");
    return dispatch_kb<TC, LA, LB, bf::K_F32_CVT>(a, s);
  }
  if (va) return dispatch_kb<TC, LA, LB, bf::K_BF16_VEC>(a, s);
  return dispatch_kb<TC, LA, LB, bf::K_BF16_SCALAR>(a, s);
}

template <typename TC, int LA, int LB>
int dispatch_f32(const comet_gemm_args& a, hipStream_t s) {
  const bool va = vec_ok(a.a, a.lda, a.stride_a, LA == 0 ? a.k : a.m, 4);
  const bool vb = vec_ok(a.b, a.ldb, a.stride_b, LB == 0 ? a.k : a.n, 4);
  if (va && vb) return launch_f32<TC, LA, LB, true, true>(a, s);
  if (va) return launch_f32<TC, LA, LB, true, false>(a, s);
  if (vb) return launch_f32<TC, LA, LB, false, true>(a, s);
  return launch_f32<TC, LA, LB, false, false>(a, s);
}

template <typename T, typename TC>
int dispatch_layout(const comet_gemm_args& a, hipStream_t s) {
  if constexpr (std::is_same<T, __bf16>::value) {
    if (a.layout_a == 0 && a.layout_b == 0) return dispatch_bf16<TC, 0, 0>(a, s);
    if (a.layout_a == 0 && a.layout_b == 1) return dispatch_bf16<TC, 0, 1>(a, s);
    if (a.layout_a == 1 && a.layout_b == 0) return dispatch_bf16<TC, 1, 0>(a, s);
    return dispatch_bf16<TC, 1, 1>(a, s);
  } else {
    if (a.layout_a == 0 && a.layout_b == 0) return dispatch_f32<TC, 0, 0>(a, s);
    if (a.layout_a == 0 && a.layout_b == 1) return dispatch_f32<TC, 0, 1>(a, s);
    if (a.layout_a == 1 && a.layout_b == 0) return dispatch_f32<TC, 1, 0>(a, s);
    return dispatch_f32<TC, 1, 1>(a, s);
  }
}

int validate(const comet_gemm_args* args) {
  COMET_CHECK_ARG(args != nullptr, "comet_gemm: null args");
  const comet_gemm_args& a = *args;
  COMET_CHECK_ARG(a.m >= 0 && a.n >= 0 && a.k >= 0, "comet_gemm: negative dims");
  COMET_CHECK_ARG(a.layout_a == 0 || a.layout_a == 1, "comet_gemm: bad layout_a");
  COMET_CHECK_ARG(a.layout_b == 0 || a.layout_b == 1, "comet_gemm: bad layout_b");
  COMET_CHECK_ARG(a.batch[0] >= 1 && a.batch[1] >= 1, "comet_gemm: batch dims must be >= 1");
  COMET_CHECK_ARG(a.bias_mode >= 0 && a.bias_mode <= 2, "comet_gemm: bad bias_mode");
  COMET_CHECK_ARG(a.split_k >= 0 && a.split_k <= 256, "comet_gemm: split_k must be in [0, 256]");
  COMET_CHECK_ARG(a.workspace_bytes >= 0, "comet_gemm: negative workspace_bytes");
  COMET_CHECK_ARG(a.convert_a == 0 || a.convert_a == 1, "comet_gemm: convert_a must be 0 or 1");
  COMET_CHECK_ARG(a.convert_b == 0 || a.convert_b == 1, "comet_gemm: convert_b must be 0 or 1");
  COMET_CHECK_ARG(a.dtype_ab == COMET_BF16 || (a.convert_a == 0 && a.convert_b == 0),
                  "comet_gemm: convert_a / convert_b need dtype_ab == COMET_BF16");
  return COMET_OK;
}

// Narrow-output implicit convolution (cout <= 64: the fine ShallowEncoder's 32-channel convs over
// 65536 patches): the skinny-GEMM structure (weights in registers as MFMA A fragments, 16 output
// pixels per wave step as the B operand, Cᵀ = W·Xᵀ) with the B fragment of pixel m gathered from
// the NHWC input tap by tap (each 8-element k chunk = 8 channels of one tap, c % 8 == 0).
template <typename TC, int NT16, int KC>
__global__ void __launch_bounds__(256)
conv_skinny_kernel(const __bf16* __restrict__ X, int H, int W, int Cin, int KW, int stride, int pad, int OH, int OW,
                   const __bf16* __restrict__ Wt, int64_t ldw, TC* __restrict__ Y, int64_t ldy, int64_t M, int N,
                   int K, Epi epi) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  bf16x8 wf[NT16][KC];
#pragma unroll
  for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int n = nt * 16 + li, k0 = 32 * c + 8 * g;
      wf[nt][c] = (n < N && k0 < K) ? *reinterpret_cast<const bf16x8*>(Wt + (int64_t)n * ldw + k0) : bf16x8{};
    }
  float bias4[NT16][4];
#pragma unroll
  for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nt * 16 + 4 * g + r;
      bias4[nt][r] = (epi.bias && n < N) ? epi.bias[n] : 0.f;
    }
  // per-lane tap decomposition of its k chunks (fixed for the whole kernel)
  int tky[KC], tkx[KC], tci[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int k0 = 32 * c + 8 * g;
    const int tap = k0 / Cin;
    tci[c] = k0 - tap * Cin;
    tky[c] = tap / KW;
    tkx[c] = tap - tky[c] * KW;
  }
  const TC* R = reinterpret_cast<const TC*>(epi.resid);
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * 256) >> 6;
  const unsigned short* x16 = reinterpret_cast<const unsigned short*>(X);
  // input fragments of the next 16-pixel step are gathered right after this step's MFMAs (software
  // pipelined: the gather latency overlaps the epilogue); pixel -> (image, oy, ox) in 32-bit
  // arithmetic (M < 2^31, host-checked: three 64-bit divisions per step cost more than its MFMAs)
  auto gather = [&](int64_t m0, bf16x8 (&xf)[KC]) {
    const int m = (int)m0 + li;
    const bool mok = m < M;
    int iy0 = 0, ix0 = 0;
    int64_t base = 0;
    if (mok) {
      const unsigned t = (unsigned)m / (unsigned)OW;
      const int ox = m - (int)t * OW;
      const unsigned ni = t / (unsigned)OH;
      const int oy = (int)t - (int)ni * OH;
      iy0 = oy * stride - pad;
      ix0 = ox * stride - pad;
      base = (int64_t)ni * H * W * Cin;
    }
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int k0 = 32 * c + 8 * g;
      const int iy = iy0 + tky[c], ix = ix0 + tkx[c];
      const bool ok = mok && k0 < K && iy >= 0 && iy < H && ix >= 0 && ix < W;
      xf[c] = ok ? *reinterpret_cast<const bf16x8*>(x16 + base + ((int64_t)iy * W + ix) * Cin + tci[c]) : bf16x8{};
    }
  };
  // 16-B bf16 stores (epi.wide, host-checked: cout % 32 == 0, Y 16-B aligned, ldy % 8 == 0): channel
  // blocks nt, nt + 1 exchange lane-group halves by v_permlane16_swap so a lane stores 8 channels
  constexpr bool WIDE = std::is_same<TC, __bf16>::value && NT16 % 2 == 0;
  auto mfmas = [&](const bf16x8 (&xc)[KC], f32x4 (&acc)[NT16]) {
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt][c], xc[c], acc[nt], 0, 0, 0);
  };
  auto epilogue = [&](int64_t m0, const f32x4 (&acc)[NT16]) {
    const int64_t m = m0 + li;
    if (m >= M) return;
    float v[NT16][4];
#pragma unroll
    for (int nt = 0; nt < NT16; ++nt) {
      const int n0 = nt * 16 + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[nt][r] = acc[nt][r] + bias4[nt][r];
      apply_act_n<4>(epi.act, v[nt]);
      if (R && n0 < N) {
        float rr[4];
        load4(R + m * epi.ldr + n0, rr);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[nt][r] += epi.beta * rr[r];
      }
    }
    if (WIDE && epi.wide) {
      if constexpr (WIDE) {
        const int wcol = 16 * (g & 1) + 8 * (g >> 1);
#pragma unroll
        for (int nt = 0; nt < NT16; nt += 2) {
          const unsigned p00 = pack_bf16x2(v[nt][0], v[nt][1]), p01 = pack_bf16x2(v[nt][2], v[nt][3]);
          const unsigned p10 = pack_bf16x2(v[nt + 1][0], v[nt + 1][1]), p11 = pack_bf16x2(v[nt + 1][2], v[nt + 1][3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(p00, p10, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(p01, p11, false, false);
          *reinterpret_cast<uint4*>(Y + m * ldy + 16 * nt + wcol) = uint4{s0[0], s1[0], s0[1], s1[1]};
        }
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt) {
        const int n0 = nt * 16 + 4 * g;
        if (n0 < N) store4(Y + m * ldy + n0, v[nt]);
      }
    }
  };
  const int64_t mstep = nwaves * 16;
  bf16x8 xa[KC], xb[KC];
  gather(wave * 16, xa);
  if constexpr (KC >= 6) {
    // long K (many taps): the next step's gather is issued before this step's MFMAs and two steps
    // per trip swap the buffers, so its latency overlaps the MFMAs and the epilogue (3x3 s2 16^2:
    // 418 -> 389 us; the short-K steps lose occupancy to the second buffer: gathered after the MFMAs)
    for (int64_t m0 = wave * 16; m0 < M; m0 += 2 * mstep) {
      f32x4 acc[NT16];
      if (m0 + mstep < M) gather(m0 + mstep, xb);
      mfmas(xa, acc);
      epilogue(m0, acc);
      if (m0 + mstep >= M) break;
      if (m0 + 2 * mstep < M) gather(m0 + 2 * mstep, xa);
      mfmas(xb, acc);
      epilogue(m0 + mstep, acc);
    }
  } else {
    for (int64_t m0 = wave * 16; m0 < M; m0 += mstep) {
      f32x4 acc[NT16];
      mfmas(xa, acc);
      if (m0 + mstep < M) gather(m0 + mstep, xb);
#pragma unroll
      for (int c = 0; c < KC; ++c) xa[c] = xb[c];
      epilogue(m0, acc);
    }
  }
}

template <typename TC>
int launch_conv_skinny(const comet_conv_args& a, int64_t M, int OH, int OW, int K, hipStream_t s) {
  Epi e{a.bias, a.bias ? 1 : 0, 0, 0, a.resid, a.ldr, 0, 0, a.beta, nullptr, 0, 0, 0, 1.f, a.act, 0};
  e.wide = a.cout % 32 == 0 && (uintptr_t)a.y % 16 == 0 && a.ldy % 8 == 0 && getenv("COMET_CONV_NO_WIDE") == nullptr;
  COMET_CHECK_ARG(M + 64 < (1ll << 31), "comet_conv2d_nhwc (narrow): too many output pixels");
  int64_t blocks = cdiv(cdiv(M, 16), 4 * 8);
  if (blocks > 4096) blocks = 4096;
  const int nt = (int)(a.cout / 16), kc = (int)cdiv(K, 32);
#define CSK(NT, KC)                                                                                        \
  hipLaunchKernelGGL((conv_skinny_kernel<TC, NT, KC>), dim3((unsigned)blocks), dim3(256), 0, s,           \
                     (const __bf16*)a.x, (int)a.h, (int)a.w, (int)a.c, a.kw, a.stride, a.pad, OH, OW,      \
                     (const __bf16*)a.weight, a.ldw, (TC*)a.y, a.ldy, M, (int)a.cout, K, e)
#define CSK_K(NT)                                                                                          \
  do {                                                                                                     \
    if (kc <= 1) CSK(NT, 1); else if (kc <= 2) CSK(NT, 2); else if (kc <= 3) CSK(NT, 3);                   \
    else if (kc <= 4) CSK(NT, 4); else if (kc <= 6) CSK(NT, 6); else if (kc <= 8) CSK(NT, 8);              \
    else if (NT <= 2 && kc <= 9) CSK(NT, 9); else if (NT <= 2 && kc <= 16) CSK(NT, 16);                     \
  } while (0)
  if (nt == 1) CSK_K(1); else if (nt == 2) CSK_K(2);
  else if (nt == 3) { if (kc <= 8) CSK_K(3); }
  else { if (kc <= 8) CSK_K(4); else if (kc <= 13) CSK(4, 13); }
#undef CSK_K
#undef CSK
  COMET_CHECK_LAUNCH("comet_conv2d_nhwc (narrow)");
  return COMET_OK;
}

// ============================== 3x3 stride-1 convolution, rows resident in LDS ==================
// BasicEncoder's 64 -> 64 3x3 convolutions at 128 x 128 (ResidualBlock, modules.py:39-116): one
// workgroup per CU holds the whole weight (64 x 576 bf16) and a ring of four input rows (row + 2
// zero pad columns, 16 B of pad per pixel so the b128 reads of 32 consecutive pixels are
// conflict-free) in LDS, and walks a contiguous range of output rows: each output row needs one new
// input row (prefetched into registers before the row's MFMAs, written to the ring after them),
// so the input is read from HBM once instead of being gathered 9 times per tap from L2. Per row,
// Cᵀ[cout][px] = W·Xᵀ on 32x32x16 MFMAs: 8 waves (2 per SIMD, so one hides the other's LDS latency)
// each own 32 pixels x 32 outputs, 36 k-steps (9 taps x 64 channels).
namespace cr {
constexpr int CI = 64, CO = 64, KK = 9 * CI;  // channels, outputs, k
constexpr int WP = KK + 8;                     // weight row pitch (elements)
constexpr int PXP = CI + 8;                    // pixel pitch in a ring row (elements)
constexpr int MAXW = 128;
constexpr int RP = (MAXW + 2) * PXP;           // ring row (elements)
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <typename TC>
__global__ void __launch_bounds__(512, 1)
conv3_rows_kernel(const __bf16* __restrict__ x, int h, int w, const __bf16* __restrict__ wt, int64_t ldw,
                  TC* __restrict__ y, int64_t ldy, int64_t rows_total, int rows_per, Epi epi) {
  extern __shared__ __attribute__((aligned(16))) __bf16 lds[];
  __bf16* Ws = lds;                 // [CO][WP]
  __bf16* Xr = lds + CO * WP;       // [4][RP]
  constexpr int NT = 512;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int pb = wid & 3, cb = wid >> 2;  // wave: pixels 32 pb.., outputs 32 cb..
  const int64_t R0 = (int64_t)blockIdx.x * rows_per;
  const int64_t R1 = R0 + rows_per < rows_total ? R0 + rows_per : rows_total;
  if (R0 >= R1) return;

  // weights (once) and the ring's pad columns (pixel 0 and w + 1 of every slot: zero forever)
  for (int i = tid; i < CO * (KK / 8); i += NT) {
    const int co = i / (KK / 8), c = i % (KK / 8);
    *reinterpret_cast<uint4*>(Ws + co * WP + 8 * c) = *reinterpret_cast<const uint4*>(wt + (int64_t)co * ldw + 8 * c);
  }
  for (int i = tid; i < 4 * 2 * (CI / 8); i += NT) {
    const int slot = i / (2 * (CI / 8)), rem = i % (2 * (CI / 8));
    const int px = (rem / (CI / 8)) ? w + 1 : 0;
    *reinterpret_cast<uint4*>(Xr + slot * RP + px * PXP + 8 * (rem % (CI / 8))) = uint4{0, 0, 0, 0};
  }
  const int nch = w * (CI / 8);  // 16-B chunks of one input row
  constexpr int MAXCH = MAXW * (CI / 8) / NT;  // per thread
  uint4 st[MAXCH];
  // input row `row` (may be -1 or h: zeros) of image ni -> registers
  auto rload = [&](int64_t ni, int row) {
    const bool in = row >= 0 && row < h;
    const __bf16* src = x + ((ni * h + (in ? row : 0)) * (int64_t)w) * CI;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int idx = tid + i * NT;
      st[i] = (in && idx < nch) ? *reinterpret_cast<const uint4*>(src + (int64_t)idx * 8) : uint4{0, 0, 0, 0};
    }
  };
  auto rstore = [&](int row) {
    COMET_DASSERT(row >= -1 && row <= h);  // the ring holds rows -1 .. h (zero pad rows included)
    __bf16* dst = Xr + ((row + 1) & 3) * RP;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int idx = tid + i * NT;
      if (idx < nch) *reinterpret_cast<uint4*>(dst + ((idx >> 3) + 1) * PXP + 8 * (idx & 7)) = st[i];
    }
  };
  const int px = pb * 32 + r;  // this lane's output pixel (B operand column / output row)
  const bool pxok = px < w;
  const __bf16* wbase = Ws + (cb * 32 + r) * WP + 8 * hh;

  int64_t ni = R0 / h;
  int oy = (int)(R0 % h);
  for (int dr = -1; dr <= 1; ++dr) {  // window of the first output row
    rload(ni, oy + dr);
    rstore(oy + dr);
  }
  __syncthreads();
  for (int64_t R = R0; R < R1; ++R) {
    const bool next_same = R + 1 < R1 && oy + 1 < h;
    if (next_same) rload(ni, oy + 2);
    f32x16 acc = f32x16{};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const __bf16* xb = Xr + ((oy + ky) & 3) * RP + px * PXP + 8 * hh;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int c = 0; c < CI; c += 16) {
          const bf16x8 bx = *reinterpret_cast<const bf16x8*>(xb + kx * PXP + c);
          const bf16x8 aw = *reinterpret_cast<const bf16x8*>(wbase + (ky * 3 + kx) * CI + c);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aw, bx, acc, 0, 0, 0);
        }
    }
    // epilogue: lane holds couts 32 cb + 8u + 4hh + (0..3) of pixel px; f32 values of the (u, u + 1)
    // pair are exchanged with the partner half so each lane owns 8 consecutive couts
    TC* yrow = y + (R * w + px) * ldy;
    const TC* rrow = reinterpret_cast<const TC*>(epi.resid) + (R * w + px) * epi.ldr;
#pragma unroll
    for (int u = 0; u < 4; u += 2) {
      float v[2][4];
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int co = 32 * cb + 8 * (u + e) + 4 * hh + q;
          v[e][q] = apply_act(epi.act, acc[4 * (u + e) + q] + (epi.bias ? epi.bias[co] : 0.f));
        }
      float o[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0][q]), __float_as_uint(v[1][q]), false, false);
        o[q] = __uint_as_float(sw[0]);
        o[4 + q] = __uint_as_float(sw[1]);
      }
      const int co0 = 32 * cb + 8 * u + 8 * hh;
      if (pxok) {
        if (epi.resid) {
          float rv[8];
          load8(rrow + co0, rv);
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] += epi.beta * rv[q];
        }
        store8(yrow + co0, o);
      }
    }
    if (next_same) rstore(oy + 2);
    __syncthreads();  // ring slot of row oy - 1 (refilled above) and this row's reads are done
    ++oy;
    if (oy == h && R + 1 < R1) {  // next image: a fresh window
      ++ni;
      oy = 0;
      for (int dr = -1; dr <= 1; ++dr) {
        rload(ni, dr);
        rstore(dr);
      }
      __syncthreads();
    }
  }
}
}  // namespace cr

// eligible: 3x3 / stride 1 / pad 1, c = cout = 64, w <= 128 with w % 32 == 0, 16-B aligned rows
template <typename TC>
bool conv_rows_ok(const comet_conv_args& a) {
  if (getenv("COMET_CONV_NO_ROWS") != nullptr) return false;
  if (a.kh != 3 || a.kw != 3 || a.stride != 1 || a.pad != 1 || a.c != cr::CI || a.cout != cr::CO) return false;
  // w >= 96: all four waves own pixels (at w = 64 the implicit GEMM is faster, tools/conv_bench.py)
  if (a.w > cr::MAXW || a.w < 96 || a.w % 32 != 0 || a.ldw < cr::KK || a.ldw % 8 != 0 || a.n * a.h < 256) return false;
  const uintptr_t al = 8 * sizeof(TC) >= 16 ? 16 : 8 * sizeof(TC);
  if ((uintptr_t)a.y % al != 0 || a.ldy % 8 != 0) return false;
  if (a.resid && ((uintptr_t)a.resid % al != 0 || a.ldr % 8 != 0)) return false;
  return true;
}

template <typename TC>
int launch_conv_rows(const comet_conv_args& a, hipStream_t s) {
  Epi e{a.bias, a.bias ? 1 : 0, 0, 0, a.resid, a.ldr, 0, 0, a.beta, nullptr, 0, 0, 0, 1.f, a.act, 1};
  const int64_t rows = a.n * a.h;
  int grid = num_cus();
  const int rows_per = (int)cdiv(rows, grid);
  grid = (int)cdiv(rows, rows_per);
  const size_t lds = (size_t)(cr::CO * cr::WP + 4 * cr::RP) * sizeof(__bf16);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)cr::conv3_rows_kernel<TC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((cr::conv3_rows_kernel<TC>), dim3((unsigned)grid), dim3(512), lds, s, (const __bf16*)a.x,
                     (int)a.h, (int)a.w, (const __bf16*)a.weight, a.ldw, (TC*)a.y, a.ldy, rows, rows_per, e);
  COMET_CHECK_LAUNCH("comet_conv2d_nhwc (3x3 rows in LDS)");
  return COMET_OK;
}

template <typename TC>
int launch_conv(const comet_conv_args& a, hipStream_t s) {
  const int64_t oh = (a.h + 2 * a.pad - a.kh) / a.stride + 1, ow = (a.w + 2 * a.pad - a.kw) / a.stride + 1;
  const int64_t M = a.n * oh * ow, N = a.cout, K = (int64_t)a.kh * a.kw * a.c;
  const int64_t tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "comet_conv2d_nhwc: too many tiles");
  const int vec = a.cout % 8 == 0 && (uintptr_t)a.y % 32 == 0 && a.ldy % 8 == 0 &&
                  (a.resid == nullptr || ((uintptr_t)a.resid % 32 == 0 && a.ldr % 8 == 0));
  Epi e{a.bias, a.bias ? 1 : 0, 0, 0, a.resid, a.ldr, 0, 0, a.beta, nullptr, 0, 0, 0, 1.f, a.act, vec};
  bf::ConvGeo g{reinterpret_cast<const __bf16*>(a.x), (int)a.h, (int)a.w, (int)a.c, a.kw, a.stride, a.pad,
                (int)oh, (int)ow};
  if (conv_rows_ok<TC>(a)) return launch_conv_rows<TC>(a, s);
  // narrow outputs: weights fit the registers (cout/16 x ceil(K/32) fragments <= 32)
  const int64_t kcs = cdiv(K, 32);
  // (and the BasicEncoder's 7x7 stem, cout 64 x K 392: 52 fragments, 208 registers at one wave per SIMD)
  const bool stem = a.cout == 64 && kcs > 8 && kcs <= 13 && getenv("COMET_CONV_NO_STEM") == nullptr;
  if (a.cout % 16 == 0 && a.cout <= 64 && ((a.cout / 16) * kcs <= 32 || stem) && kcs <= 16 && M >= 16384 &&
      (uintptr_t)a.y % (4 * sizeof(TC)) == 0 && a.ldy % 4 == 0 && getenv("COMET_CONV_NO_SKINNY") == nullptr &&
      (a.resid == nullptr || ((uintptr_t)a.resid % (4 * sizeof(TC)) == 0 && a.ldr % 4 == 0)))
    return launch_conv_skinny<TC>(a, M, (int)oh, (int)ow, (int)K, s);
  Split sp{nullptr, K};
  if (N <= 64 && getenv("COMET_CONV_NO_N64") == nullptr)  // 4 x 1 waves over 128 x 64: no zero columns
    hipLaunchKernelGGL((bf::gemm_bf16_kernel<TC, 0, 0, bf::K_BF16_VEC, bf::K_BF16_VEC, false, true, true>),
                       dim3((unsigned)(tiles_m * tiles_n), 1, 1), dim3(NT), 0, s,
                       nullptr, 0, 0, 0, reinterpret_cast<const __bf16*>(a.weight), a.ldw, 0, 0,
                       reinterpret_cast<TC*>(a.y), a.ldy, 0, 0, M, N, K, 1, (int)tiles_n, e, sp, g);
  else
    hipLaunchKernelGGL((bf::gemm_bf16_kernel<TC, 0, 0, bf::K_BF16_VEC, bf::K_BF16_VEC, false, true>),
                       dim3((unsigned)(tiles_m * tiles_n), 1, 1), dim3(NT), 0, s,
                       nullptr, 0, 0, 0, reinterpret_cast<const __bf16*>(a.weight), a.ldw, 0, 0,
                       reinterpret_cast<TC*>(a.y), a.ldy, 0, 0, M, N, K, 1, (int)tiles_n, e, sp, g);
  COMET_CHECK_LAUNCH("comet_conv2d_nhwc");
  return COMET_OK;
}

}  // namespace

}  // namespace comet

extern "C" int comet_conv2d_nhwc(const comet_conv_args* args, void* stream) {
  using namespace comet;
  COMET_CHECK_ARG(args != nullptr, "comet_conv2d_nhwc: null args");
  const comet_conv_args& a = *args;
  COMET_CHECK_ARG(a.dtype == COMET_BF16, "comet_conv2d_nhwc: x/weight must be bf16 (use im2col + comet_gemm for f32)");
  COMET_CHECK_ARG(a.c > 0 && a.c % 8 == 0, "comet_conv2d_nhwc: channels must be a positive multiple of 8");
  COMET_CHECK_ARG(a.n > 0 && a.h > 0 && a.w > 0 && a.cout > 0 && a.kh > 0 && a.kw > 0 && a.stride > 0 && a.pad >= 0,
                  "comet_conv2d_nhwc: bad geometry");
  COMET_CHECK_ARG(a.h + 2 * a.pad >= a.kh && a.w + 2 * a.pad >= a.kw, "comet_conv2d_nhwc: kernel larger than padded input");
  COMET_CHECK_ARG(a.ldw >= (int64_t)a.kh * a.kw * a.c && a.ldw % 8 == 0, "comet_conv2d_nhwc: ldw < kh*kw*c or not a multiple of 8");
  COMET_CHECK_ARG(a.x && a.weight && a.y, "comet_conv2d_nhwc: null pointer");
  COMET_CHECK_ARG((uintptr_t)a.x % 16 == 0 && (uintptr_t)a.weight % 16 == 0, "comet_conv2d_nhwc: x/weight must be 16-byte aligned");
  COMET_CHECK_ARG(a.n * a.h * a.w * a.c < (1ll << 40), "comet_conv2d_nhwc: input too large");
  hipStream_t s = as_stream(stream);
  if (a.dtype_y == COMET_BF16) return launch_conv<__bf16>(a, s);
  if (a.dtype_y == COMET_F32) return launch_conv<float>(a, s);
  set_error("comet_conv2d_nhwc: bad dtype_y");
  return COMET_EINVAL;
}

extern "C" int comet_gemm_workspace(const comet_gemm_args* args, int64_t* bytes) {
  using namespace comet;
  const int rc = validate(args);
  if (rc != COMET_OK) return rc;
  COMET_CHECK_ARG(bytes != nullptr, "comet_gemm_workspace: null bytes");
  *bytes = plan_workspace(*args, make_plan(*args));
  return COMET_OK;
}

extern "C" int comet_gemm_plan(const comet_gemm_args* args, int64_t* bytes, int32_t* plan) {
  using namespace comet;
  const int rc = validate(args);
  if (rc != COMET_OK) return rc;
  COMET_CHECK_ARG(bytes != nullptr && plan != nullptr, "comet_gemm_plan: null output");
  const Plan p = make_plan(*args);
  *bytes = plan_workspace(*args, p);
  plan[0] = p.kind;
  plan[1] = p.bn;
  plan[2] = (p.kind == 3 || p.kind == 4) ? p.bm : p.splits;
  return COMET_OK;
}

// Row-LN GEMM (see w4::RowLN): eligibility shared by comet_gemm_rowln_ok and comet_gemm_rowln.
static bool rowln_ok(const comet_gemm_args& a, const comet_rowln_args* ln) {
  using namespace comet;
  if (!pp_ok(a) || a.dtype_c != COMET_F32 || a.resid == nullptr || a.aux != nullptr || a.act != COMET_ACT_NONE) return false;
  if (a.n != 384 && a.n != 256) return false;
  int tbm, tbn;
  pp_tile_base(a, tbm, tbn);
  if (tbn != a.n) return false;
  // the epilogues (persistent and split reduce) read bias / zw / zb as f32x4 per 4 columns
  auto a16 = [](const void* p) { return p == nullptr || (uintptr_t)p % 16 == 0; };
  if (!a16(a.bias)) return false;
  if (ln == nullptr) return true;
  auto b4 = [](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 8 == 0 && ld % 4 == 0); };
  if (!b4(ln->y16, ln->ldy) || !b4(ln->z16, ln->ldz)) return false;
  if (ln->z16 != nullptr && (ln->zw == nullptr || ln->zb == nullptr)) return false;
  if (!a16(ln->zw) || !a16(ln->zb)) return false;
  return true;
}

extern "C" int comet_gemm_rowln_workspace(const comet_gemm_args* args, int64_t* bytes) {
  using namespace comet;
  COMET_CHECK_ARG(bytes != nullptr, "comet_gemm_rowln_workspace: null bytes");
  *bytes = 0;
  const int rc = validate(args);
  if (rc != COMET_OK) return rc;
  if (rowln_ok(*args, nullptr)) {
    if (const int sp = rowln_splits(*args)) *bytes = rowln_ws_bytes(*args, sp);
  }
  return COMET_OK;
}

extern "C" int comet_gemm_rowln_ok(const comet_gemm_args* args) {
  using namespace comet;
  if (args == nullptr || validate(args) != COMET_OK) return 0;
  return rowln_ok(*args, nullptr) ? 1 : 0;
}

extern "C" int comet_gemm_rowln(const comet_gemm_args* args, const comet_rowln_args* ln, void* stream) {
  using namespace comet;
  const int rc = validate(args);
  if (rc != COMET_OK) return rc;
  COMET_CHECK_ARG(ln != nullptr && args->a && args->b && args->c, "comet_gemm_rowln: null operand");
  COMET_CHECK_ARG(rowln_ok(*args, ln), "comet_gemm_rowln: not eligible (bf16 k-contiguous operands, K % 64 == 0, "
                                       "M >= 4096, N in {256, 384}, f32 output with a residual, no activation / aux)");
  if (args->m == 0) return COMET_OK;
  w4::RowLN r{reinterpret_cast<__bf16*>(ln->y16), ln->ldy, ln->eps_y, reinterpret_cast<__bf16*>(ln->z16), ln->ldz,
              ln->zw, ln->zb, ln->eps_z, ln->raw_c};
  return launch_pp_rowln(*args, r, as_stream(stream));
}

// ---- GEMM + activation backward (comet_gemm_dact) --------------------------------------------
// dPre = act'(pre) * (A.B) in bf16 with the bias gradient dcol = column sums of dPre: the
// hidden-layer gradient of an MLP (fc2's dX GEMM fused with fc1's GELU backward and bias gradient),
// on the 256-row kernel without split-K.
namespace comet {
namespace {
bool dact_ok(const comet_gemm_args& a, int act, const void* pre, int64_t ldpre) {
  if (act != COMET_ACT_GELU || a.dtype_ab != COMET_BF16 || a.dtype_c != COMET_BF16 || a.layout_a != 0) return false;
  if (a.bias || a.resid || a.aux || a.act != COMET_ACT_NONE || a.batch[0] * a.batch[1] != 1) return false;
  if (a.n % 8 != 0 || (uintptr_t)a.c % 16 != 0 || a.ldc % 8 != 0) return false;
  if (pre == nullptr || (uintptr_t)pre % 16 != 0 || ldpre % 8 != 0 || ldpre < a.n) return false;
  // one predicate with the planner: the fused epilogue exists on the 256-row kernel without split-K
  const Plan p = make_plan(a);
  return p.kind == 1 && p.splits == 1 && p.tail == 0 && p.bn == big_bn(a);
}

template <int BN, int LB>
int launch_big_dact(const comet_gemm_args& a, const __bf16* pre, int64_t ldpre, float* dcol, hipStream_t s) {
  Epi e{nullptr, 0, 0, 0, nullptr, 0, 0, 0, 0.f, nullptr, 0, 0, 0, a.alpha, COMET_ACT_NONE, 1};
  e.gpre = pre; e.ldg = ldpre; e.dcol = dcol;
  const int64_t tiles_m = cdiv(a.m, big::BM), tiles_n = cdiv(a.n, BN);
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "comet_gemm_dact: too many tiles");
  if (dcol != nullptr && hipMemsetAsync(dcol, 0, a.n * sizeof(float), s) != hipSuccess) {
    set_error("comet_gemm_dact: memset failed");
    return COMET_ELAUNCH;
  }
  Split sp{nullptr, a.k};
  hipLaunchKernelGGL((big::gemm_big_kernel<__bf16, BN, 0, LB, false, 0, true>), dim3((unsigned)(tiles_m * tiles_n)),
                     dim3(big::NT), 0, s, (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (__bf16*)a.c, a.ldc,
                     a.m, a.n, a.k, (int)tiles_n, e, sp);
  COMET_CHECK_LAUNCH("comet_gemm_dact");
  return COMET_OK;
}
}  // namespace
}  // namespace comet

extern "C" int comet_gemm_dact_ok(const comet_gemm_args* args, int32_t act, const void* pre, int64_t ldpre) {
  using namespace comet;
  if (args == nullptr || validate(args) != COMET_OK) return 0;
  return dact_ok(*args, act, pre, ldpre) ? 1 : 0;
}

extern "C" int comet_gemm_dact(const comet_gemm_args* args, int32_t act, const void* pre, int64_t ldpre, float* dbias,
                               void* stream) {
  using namespace comet;
  const int rc = validate(args);
  if (rc != COMET_OK) return rc;
  COMET_CHECK_ARG(args->a && args->b && args->c, "comet_gemm_dact: null operand");
  COMET_CHECK_ARG(dact_ok(*args, act, pre, ldpre), "comet_gemm_dact: not eligible (GELU, bf16 operands and output, "
                                                   "A k-contiguous, no bias / residual / aux / activation, one batch, "
                                                   "N % 8 == 0, 16-B aligned C and pre, a 256-row tile plan without split-K)");
  if (args->m == 0) return COMET_OK;
  const comet_gemm_args& a = *args;
  const __bf16* pre16 = reinterpret_cast<const __bf16*>(pre);
  hipStream_t s = as_stream(stream);
  const int bn = big_bn(a);
  if (bn == 256) return a.layout_b ? launch_big_dact<256, 1>(a, pre16, ldpre, dbias, s) : launch_big_dact<256, 0>(a, pre16, ldpre, dbias, s);
  return a.layout_b ? launch_big_dact<128, 1>(a, pre16, ldpre, dbias, s) : launch_big_dact<128, 0>(a, pre16, ldpre, dbias, s);
}

#ifdef COMET_GEMM_STAMPS
// diagnostic build: copy out / clear the per-tile clock stamps of the persistent GEMM
extern "C" int comet_gemm_stamps(unsigned long long* host, int64_t n, int clear) {
  using namespace comet;
  const int64_t cap = (int64_t)w4::ST_WG * w4::ST_TILES * 8;
  if (n > cap) n = cap;
  if (host != nullptr && hipMemcpyFromSymbol(host, HIP_SYMBOL(w4::g_stamps), n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess) return COMET_ELAUNCH;
  if (clear) {
    static unsigned long long* zero = nullptr;
    if (zero == nullptr) zero = (unsigned long long*)calloc(cap, 8);
    if (hipMemcpyToSymbol(HIP_SYMBOL(w4::g_stamps), zero, cap * 8, 0, hipMemcpyHostToDevice) != hipSuccess) return COMET_ELAUNCH;
  }
  return (int)n;
}
#endif

extern "C" int comet_gemm(const comet_gemm_args* args, void* stream) {
  using namespace comet;
  const int rc = validate(args);
  if (rc != COMET_OK) return rc;
  const comet_gemm_args& a = *args;
  COMET_CHECK_ARG(a.a && a.b && a.c, "comet_gemm: null operand");
  if (a.m == 0 || a.n == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  const Plan plan = make_plan(a);
  if (plan.kind == 0) return a.dtype_c == COMET_BF16 ? launch_skinny<__bf16>(a, s) : launch_skinny<float>(a, s);
  if (plan.kind == 3) return a.dtype_c == COMET_BF16 ? launch_pp<__bf16>(a, s) : launch_pp<float>(a, s);
  if (plan.kind == 1 && plan.tail && a.workspace != nullptr && a.workspace_bytes >= plan_workspace(a, plan)) {
    // slot 0: the K % 64 remainder (128 x 128 kernel, plain f32 output); slots 1..: the 256-row
    // kernel's split partials over the 64-multiple part; one reduce applies the epilogue
    const int64_t kt = plan.tail, km = a.k - kt;
    float* ws = reinterpret_cast<float*>(a.workspace);
    comet_gemm_args t{};
    t.dtype_ab = a.dtype_ab;
    t.dtype_c = COMET_F32;
    t.layout_a = a.layout_a;
    t.layout_b = a.layout_b;
    t.m = a.m; t.n = a.n; t.k = kt;
    t.a = reinterpret_cast<const __bf16*>(a.a) + (a.layout_a == 0 ? km : km * a.lda);
    t.b = reinterpret_cast<const __bf16*>(a.b) + (a.layout_b == 0 ? km : km * a.ldb);
    t.lda = a.lda; t.ldb = a.ldb;
    t.c = ws; t.ldc = a.n;
    t.batch[0] = t.batch[1] = 1;
    t.alpha = 1.f;
    t.split_k = 1;
    int rc = dispatch_layout<__bf16, float>(t, s);
    if (rc != COMET_OK) return rc;
    comet_gemm_args m = a;
    m.k = km;
    m.workspace = ws + a.m * a.n;
    m.workspace_bytes = a.workspace_bytes - a.m * a.n * (int64_t)sizeof(float);
    if (plan.bn == 256)
      return a.dtype_c == COMET_BF16 ? launch_big_layout<__bf16, 256>(m, plan.splits, s, 1) : launch_big_layout<float, 256>(m, plan.splits, s, 1);
    return a.dtype_c == COMET_BF16 ? launch_big_layout<__bf16, 128>(m, plan.splits, s, 1) : launch_big_layout<float, 128>(m, plan.splits, s, 1);
  }
  if (plan.kind == 1 && !plan.tail) {
    int sp = plan.splits;
    if (sp > 1 && (a.workspace == nullptr || a.workspace_bytes < plan_workspace(a, plan))) sp = 1;
    if (plan.bn == 256)
      return a.dtype_c == COMET_BF16 ? launch_big_layout<__bf16, 256>(a, sp, s) : launch_big_layout<float, 256>(a, sp, s);
    return a.dtype_c == COMET_BF16 ? launch_big_layout<__bf16, 128>(a, sp, s) : launch_big_layout<float, 128>(a, sp, s);
  }
  if (a.dtype_ab == COMET_BF16 && a.dtype_c == COMET_BF16) return dispatch_layout<__bf16, __bf16>(a, s);
  if (a.dtype_ab == COMET_BF16 && a.dtype_c == COMET_F32) return dispatch_layout<__bf16, float>(a, s);
  if (a.dtype_ab == COMET_F32 && a.dtype_c == COMET_F32) return dispatch_layout<float, float>(a, s);
  if (a.dtype_ab == COMET_F32 && a.dtype_c == COMET_BF16) return dispatch_layout<float, __bf16>(a, s);
  set_error("comet_gemm: unsupported dtype combination");
  return COMET_EINVAL;
}
