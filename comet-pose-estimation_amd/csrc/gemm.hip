// Batched MFMA GEMM with fused bias / activation / residual epilogue (comet_gemm).
//
// Replaces nn.Linear / MHA in_proj+out_proj / conv-after-im2col of the reference
// (modules.py:119-154, 248-344; blocks.py:27-348; camera_predictor10.py:75-87,126-280).
//
// Tile 128x128, 256 threads = 4 waves (2x2), each wave owns 64x64 = 4x4 MFMA 16x16 tiles.
//  bf16: v_mfma_f32_16x16x32_bf16, BK = 32   (lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15])
//  f32 : v_mfma_f32_16x16x4_f32,  BK = 16   (lane reads 4 consecutive k; instruction e uses
//        k = 4(l>>4)+e for A and B alike, so one ds_read_b128 feeds 4 MFMAs)
// LDS holds both operands k-contiguous ([row][BK+pad]); row pitch 80 B keeps the 16-lane
// ds_read_b128 groups conflict-free. Global->register loads of tile t+1 are issued before the
// MFMAs of tile t and written to the other LDS buffer afterwards (one barrier per k-tile).
#include "common.hpp"

namespace comet {

namespace {

constexpr int BM = 128, BN = 128, NT = 256;

template <typename T> struct Cfg;
template <> struct Cfg<__bf16> { static constexpr int BK = 32, VEC = 8, PAD = 8; };
template <> struct Cfg<float>  { static constexpr int BK = 16, VEC = 4, PAD = 4; };

template <typename T> struct VecT;
template <> struct VecT<__bf16> { typedef uint4 type; };   // 8 x bf16
template <> struct VecT<float>  { typedef float4 type; };  // 4 x f32

struct Epi {
  const float* bias; int bias_mode; int64_t sb0, sb1;
  const void* resid; int64_t ldr, sr0, sr1; float beta;
  void* aux; int64_t ldaux, sx0, sx1;
  float alpha; int act;
};

// Load one operand tile (ROWS x BK of the k-contiguous LDS image) from global into registers.
// layout 0: element (r, k) at base[r*ld + k]; layout 1: at base[k*ld + r].
template <typename T, int LAYOUT, bool VEC>
struct TileLoader {
  static constexpr int BK = Cfg<T>::BK, V = Cfg<T>::VEC;
  static constexpr int NV = 128 * BK / V / NT;  // vectors per thread (=2)
  typedef typename VecT<T>::type vec_t;
  vec_t reg[NV];

  __device__ __forceinline__ void load(const T* __restrict__ base, int64_t ld, int64_t r0,
                                       int64_t rmax, int64_t k0, int64_t kmax) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * NT;
      T tmp[V];
      if (LAYOUT == 0) {
        const int row = v / (BK / V), kv = (v % (BK / V)) * V;
        const int64_t gr = r0 + row, gk = k0 + kv;
        if (VEC) {
          if (gr < rmax && gk < kmax) {
            reg[i] = *reinterpret_cast<const vec_t*>(base + gr * ld + gk);
          } else {
            reg[i] = vec_t{};
          }
          continue;
        }
#pragma unroll
        for (int e = 0; e < V; ++e)
          tmp[e] = (gr < rmax && gk + e < kmax) ? base[gr * ld + gk + e] : T(0.f);
      } else {
        const int krow = v / (128 / V), rv = (v % (128 / V)) * V;
        const int64_t gk = k0 + krow, gr = r0 + rv;
        if (VEC) {
          if (gk < kmax && gr < rmax) {
            reg[i] = *reinterpret_cast<const vec_t*>(base + gk * ld + gr);
          } else {
            reg[i] = vec_t{};
          }
          continue;
        }
#pragma unroll
        for (int e = 0; e < V; ++e)
          tmp[e] = (gk < kmax && gr + e < rmax) ? base[gk * ld + gr + e] : T(0.f);
      }
      reg[i] = *reinterpret_cast<vec_t*>(tmp);
    }
  }

  __device__ __forceinline__ void store(T* __restrict__ lds) const {
    constexpr int LDW = BK + Cfg<T>::PAD;
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * NT;
      if (LAYOUT == 0) {
        const int row = v / (BK / V), kv = (v % (BK / V)) * V;
        *reinterpret_cast<vec_t*>(lds + row * LDW + kv) = reg[i];
      } else {
        const int krow = v / (128 / V), rv = (v % (128 / V)) * V;
        const T* t = reinterpret_cast<const T*>(&reg[i]);
#pragma unroll
        for (int e = 0; e < V; ++e) lds[(rv + e) * LDW + krow] = t[e];
      }
    }
  }
};

template <typename T>
__device__ __forceinline__ void mma_tile(const T* __restrict__ As, const T* __restrict__ Bs,
                                         f32x4 (&acc)[4][4], int wm, int wn, int lane);

template <>
__device__ __forceinline__ void mma_tile<__bf16>(const __bf16* __restrict__ As,
                                                 const __bf16* __restrict__ Bs,
                                                 f32x4 (&acc)[4][4], int wm, int wn, int lane) {
  constexpr int LDW = 32 + 8;
  bf16x8 a[4], b[4];
  const int r = lane & 15, kq = (lane >> 4) * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + r) * LDW + kq);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 16 + r) * LDW + kq);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

template <>
__device__ __forceinline__ void mma_tile<float>(const float* __restrict__ As,
                                                const float* __restrict__ Bs,
                                                f32x4 (&acc)[4][4], int wm, int wn, int lane) {
  constexpr int LDW = 16 + 4;
  f32x4 a[4], b[4];
  const int r = lane & 15, kq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a[i] = *reinterpret_cast<const f32x4*>(As + (wm * 64 + i * 16 + r) * LDW + kq);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    b[j] = *reinterpret_cast<const f32x4*>(Bs + (wn * 64 + j * 16 + r) * LDW + kq);
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
}

template <typename T, typename TC, int LA, int LB, bool VA, bool VB>
__global__ void __launch_bounds__(NT)
gemm_kernel(const T* __restrict__ A, int64_t lda, int64_t sa0, int64_t sa1,
            const T* __restrict__ B, int64_t ldb, int64_t sb0, int64_t sb1,
            TC* __restrict__ C, int64_t ldc, int64_t sc0, int64_t sc1,
            int64_t M, int64_t N, int64_t K, int64_t nb1, int tiles_n, Epi epi) {
  constexpr int BK = Cfg<T>::BK, LDW = BK + Cfg<T>::PAD;
  __shared__ __attribute__((aligned(16))) T smem[2][2][128 * LDW];

  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int64_t bz = blockIdx.y, b0 = bz / nb1, b1 = bz % nb1;
  A += b0 * sa0 + b1 * sa1;
  B += b0 * sb0 + b1 * sb1;
  C += b0 * sc0 + b1 * sc1;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  TileLoader<T, LA, VA> la;
  TileLoader<T, LB, VB> lb;
  const int nk = (int)((K + BK - 1) / BK);

  la.load(A, lda, m0, M, 0, K);
  lb.load(B, ldb, n0, N, 0, K);
  la.store(smem[0][0]);
  lb.store(smem[0][1]);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(A, lda, m0, M, (int64_t)(kt + 1) * BK, K);
      lb.load(B, ldb, n0, N, (int64_t)(kt + 1) * BK, K);
    }
    mma_tile<T>(smem[cur][0], smem[cur][1], acc, wm, wn, lane);
    if (more) {
      la.store(smem[cur ^ 1][0]);
      lb.store(smem[cur ^ 1][1]);
    }
    __syncthreads();
  }

  // ---- epilogue: C layout col = lane&15, row = 4*(lane>>4)+r ----
  const TC* R = epi.resid ? reinterpret_cast<const TC*>(epi.resid) + b0 * epi.sr0 + b1 * epi.sr1 : nullptr;
  TC* X = epi.aux ? reinterpret_cast<TC*>(epi.aux) + b0 * epi.sx0 + b1 * epi.sx1 : nullptr;
  const float* bias = epi.bias ? epi.bias + b0 * epi.sb0 + b1 * epi.sb1 : nullptr;
  const int cl = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = n0 + wn * 64 + j * 16 + cl;
    if (col >= N) continue;
    const float bcol = (bias && epi.bias_mode == 1) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + rq + r;
        if (row >= M) continue;
        float v = epi.alpha * acc[i][j][r] + bcol;
        if (bias && epi.bias_mode == 2) v += bias[row];
        if (X) X[row * epi.ldaux + col] = from_f32<TC>(v);
        v = apply_act(epi.act, v);
        if (R) v += epi.beta * to_f32(R[row * epi.ldr + col]);
        C[row * ldc + col] = from_f32<TC>(v);
      }
    }
  }
}

template <typename T, typename TC, int LA, int LB, bool VA, bool VB>
int launch(const comet_gemm_args& a, hipStream_t s) {
  const int64_t tiles_m = cdiv(a.m, BM), tiles_n = cdiv(a.n, BN);
  const int64_t nb = a.batch[0] * a.batch[1];
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "comet_gemm: too many tiles");
  COMET_CHECK_ARG(nb <= 65535, "comet_gemm: batch too large (max 65535)");
  Epi e{a.bias, a.bias_mode, a.stride_bias[0], a.stride_bias[1],
        a.resid, a.ldr, a.stride_r[0], a.stride_r[1], a.beta,
        a.aux, a.ldaux, a.stride_aux[0], a.stride_aux[1], a.alpha, a.act};
  dim3 grid((unsigned)(tiles_m * tiles_n), (unsigned)nb);
  hipLaunchKernelGGL((gemm_kernel<T, TC, LA, LB, VA, VB>), grid, dim3(NT), 0, s,
                     reinterpret_cast<const T*>(a.a), a.lda, a.stride_a[0], a.stride_a[1],
                     reinterpret_cast<const T*>(a.b), a.ldb, a.stride_b[0], a.stride_b[1],
                     reinterpret_cast<TC*>(a.c), a.ldc, a.stride_c[0], a.stride_c[1],
                     a.m, a.n, a.k, a.batch[1], (int)tiles_n, e);
  COMET_CHECK_LAUNCH("comet_gemm");
  return COMET_OK;
}

template <typename T, typename TC, int LA, int LB>
int dispatch_vec(const comet_gemm_args& a, hipStream_t s) {
  constexpr int V = Cfg<T>::VEC;
  // A vector needs 16-byte alignment of every vector start: base, ld and strides multiples of V.
  auto aligned = [&](const void* p, int64_t ld, const int64_t* st, int64_t contig_extent) {
    return ((uintptr_t)p % 16 == 0) && ld % V == 0 && st[0] % V == 0 && st[1] % V == 0 &&
           contig_extent % V == 0;
  };
  const bool va = aligned(a.a, a.lda, a.stride_a, LA == 0 ? a.k : a.m);
  const bool vb = aligned(a.b, a.ldb, a.stride_b, LB == 0 ? a.k : a.n);
  if (va && vb) return launch<T, TC, LA, LB, true, true>(a, s);
  if (va) return launch<T, TC, LA, LB, true, false>(a, s);
  if (vb) return launch<T, TC, LA, LB, false, true>(a, s);
  return launch<T, TC, LA, LB, false, false>(a, s);
}

template <typename T, typename TC>
int dispatch_layout(const comet_gemm_args& a, hipStream_t s) {
  if (a.layout_a == 0 && a.layout_b == 0) return dispatch_vec<T, TC, 0, 0>(a, s);
  if (a.layout_a == 0 && a.layout_b == 1) return dispatch_vec<T, TC, 0, 1>(a, s);
  if (a.layout_a == 1 && a.layout_b == 0) return dispatch_vec<T, TC, 1, 0>(a, s);
  return dispatch_vec<T, TC, 1, 1>(a, s);
}

}  // namespace

}  // namespace comet

extern "C" int comet_gemm(const comet_gemm_args* args, void* stream) {
  using namespace comet;
  COMET_CHECK_ARG(args != nullptr, "comet_gemm: null args");
  const comet_gemm_args& a = *args;
  COMET_CHECK_ARG(a.m >= 0 && a.n >= 0 && a.k >= 0, "comet_gemm: negative dims");
  COMET_CHECK_ARG(a.layout_a == 0 || a.layout_a == 1, "comet_gemm: bad layout_a");
  COMET_CHECK_ARG(a.layout_b == 0 || a.layout_b == 1, "comet_gemm: bad layout_b");
  COMET_CHECK_ARG(a.batch[0] >= 1 && a.batch[1] >= 1, "comet_gemm: batch dims must be >= 1");
  COMET_CHECK_ARG(a.bias_mode >= 0 && a.bias_mode <= 2, "comet_gemm: bad bias_mode");
  COMET_CHECK_ARG(a.a && a.b && a.c, "comet_gemm: null operand");
  if (a.m == 0 || a.n == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (a.dtype_ab == COMET_BF16 && a.dtype_c == COMET_BF16) return dispatch_layout<__bf16, __bf16>(a, s);
  if (a.dtype_ab == COMET_BF16 && a.dtype_c == COMET_F32) return dispatch_layout<__bf16, float>(a, s);
  if (a.dtype_ab == COMET_F32 && a.dtype_c == COMET_F32) return dispatch_layout<float, float>(a, s);
  if (a.dtype_ab == COMET_F32 && a.dtype_c == COMET_BF16) return dispatch_layout<float, __bf16>(a, s);
  set_error("comet_gemm: unsupported dtype combination");
  return COMET_EINVAL;
}
