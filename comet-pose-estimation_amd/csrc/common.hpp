// Shared helpers for the gfx950 kernels of libcomet_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/comet_hip.h"

namespace comet {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

void set_error(const std::string& msg);

#define COMET_CHECK_ARG(cond, msg)          \
  do {                                      \
    if (!(cond)) {                          \
      ::comet::set_error(msg);              \
      return COMET_EINVAL;                  \
    }                                       \
  } while (0)

#ifdef COMET_DEBUG
// debug build: synchronise after every launch (a fault is attributed to the op that caused it) and
// read this translation unit's device assertion word, which the kernels' COMET_DASSERT checks set
static __device__ int g_dbg_word = 0;  // (inside namespace comet)
void debug_record(const char* name, int word);
#define COMET_CHECK_LAUNCH(name)                                                              \
  do {                                                                                        \
    hipError_t e_ = hipGetLastError();                                                        \
    if (e_ == hipSuccess) e_ = hipDeviceSynchronize();                                        \
    if (e_ != hipSuccess) {                                                                   \
      ::comet::set_error(std::string(name) + ": " + hipGetErrorString(e_));                   \
      return COMET_ELAUNCH;                                                                   \
    }                                                                                         \
    int w_ = 0;                                                                               \
    (void)hipMemcpyFromSymbol(&w_, HIP_SYMBOL(::comet::g_dbg_word), sizeof(int));             \
    if (w_ != 0) {                                                                            \
      const int z_ = 0;                                                                       \
      (void)hipMemcpyToSymbol(HIP_SYMBOL(::comet::g_dbg_word), &z_, sizeof(int));             \
      ::comet::debug_record(name, w_);                                                        \
      return COMET_ELAUNCH;                                                                   \
    }                                                                                         \
  } while (0)
// a failed check records its source line (mod 31) in the word -- no trap: a faulting wave can take
// the whole device down; the access the check guards still happens
#define COMET_DASSERT(cond)                                                      \
  do {                                                                           \
    if (!(cond)) atomicOr(&::comet::g_dbg_word, 1 << (__LINE__ % 31));           \
  } while (0)
#else
#define COMET_CHECK_LAUNCH(name)                                                 \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      ::comet::set_error(std::string(name) + ": " + hipGetErrorString(e_));      \
      return COMET_ELAUNCH;                                                      \
    }                                                                            \
  } while (0)
#define COMET_DASSERT(cond) do { } while (0)
#endif

// ---- scalar conversions -------------------------------------------------------------------
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__bf16 x) { return static_cast<float>(x); }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ __bf16 from_f32<__bf16>(float x) { return static_cast<__bf16>(x); }

// ---- 8-element vector loads / stores (16 B of bf16, 32 B of f32) as f32 -------------------
__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ void load8(const __bf16* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
  v[4] = bf16_lo(u.z); v[5] = bf16_hi(u.z); v[6] = bf16_lo(u.w); v[7] = bf16_hi(u.w);
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return (unsigned)__builtin_bit_cast(unsigned short, static_cast<__bf16>(a)) |
         ((unsigned)__builtin_bit_cast(unsigned short, static_cast<__bf16>(b)) << 16);
}
__device__ __forceinline__ void store8(__bf16* p, const float (&v)[8]) {
  uint4 u;
  u.x = pack_bf16x2(v[0], v[1]); u.y = pack_bf16x2(v[2], v[3]);
  u.z = pack_bf16x2(v[4], v[5]); u.w = pack_bf16x2(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  reinterpret_cast<float4*>(p)[0] = float4{v[0], v[1], v[2], v[3]};
  reinterpret_cast<float4*>(p)[1] = float4{v[4], v[5], v[6], v[7]};
}
// streaming (non-temporal) variants, for write-once outputs no later kernel of the step finds in L2
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
__device__ __forceinline__ void store8_nt(__bf16* p, const float (&v)[8]) {
  u32x4 u;
  u.x = pack_bf16x2(v[0], v[1]); u.y = pack_bf16x2(v[2], v[3]);
  u.z = pack_bf16x2(v[4], v[5]); u.w = pack_bf16x2(v[6], v[7]);
  __builtin_nontemporal_store(u, reinterpret_cast<u32x4*>(p));
}
__device__ __forceinline__ void store8_nt(float* p, const float (&v)[8]) {
  __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(p));
  __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(p) + 1);
}

// 4-element variants (16 B of f32, 8 B of bf16)
__device__ __forceinline__ void load4(const float* p, float (&v)[4]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
__device__ __forceinline__ void load4(const __bf16* p, float (&v)[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
}
__device__ __forceinline__ void store4(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void store4(__bf16* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
}
// N in {4, 8}
template <int N, typename T> __device__ __forceinline__ void loadn(const T* p, float (&v)[N]) {
  if constexpr (N == 4) load4(p, v); else load8(p, v);
}
template <int N, typename T> __device__ __forceinline__ void storen(T* p, const float (&v)[N]) {
  if constexpr (N == 4) store4(p, v); else store8(p, v);
}

// ---- wave (64-lane) reductions ------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// block-wide sum for blockDim.x == 64*NW; scratch must hold NW floats
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// nn.GELU() (exact erf form), written as x Phi(x) = relu(x) - |x| Phi(-|x|) with Phi(-a) = 2^q(a):
// q is a degree-6 fit of log2 Phi(-a) on a = min(|x|, 6) (Phi(-6) = 9.9e-10), weighted by a Phi(-a)
// so the GELU error is even: |err| <= 2.8e-7 over the f32 line (fit and check: tools/gelu_fit.py;
// the Abramowitz-Stegun 7.1.26 erf form used before: 4.6e-7). One v_exp_f32 and 9 VALU operations
// against two transcendentals and ~15: the GELU GEMM epilogues are VALU-bound. Non-finite inputs give
// NaN, as torch's f32 GELU does (fmaxf / fminf drop a NaN operand, so the relu term is fma(x, 0, relu):
// x * 0 is 0 for finite x and NaN for NaN / +-inf; one more fma per value, one packed fma per pair).
// The last step multiplies by the clamped a rather than |x|: for |x| > 6 the term is below 6e-9 either
// way (and nearer the true GELU with a); the pair form below then needs no second |x| register.
__device__ __forceinline__ float gelu_erf(float x) {
  const float a = fminf(fabsf(x), 6.0f);
  float q = fmaf(3.309693057e-05f, a, -7.692557992e-04f);
  q = fmaf(q, a, 8.080835454e-03f);
  q = fmaf(q, a, -5.341228843e-02f);
  q = fmaf(q, a, -4.587708414e-01f);
  q = fmaf(q, a, -1.151201725e+00f);
  q = fmaf(q, a, -9.999930859e-01f);
  return fmaf(-a, __builtin_amdgcn_exp2f(q), fmaf(x, 0.f, fmaxf(x, 0.f)));
}
// The same GELU on two values with packed f32 math (v_pk_fma_f32: the six polynomial steps and the
// final fma issue once per pair): 13 VALU instructions per pair instead of 21, bit-identical to
// gelu_erf (one fma rounding per step either way). The GELU GEMM epilogues run it on adjacent columns.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_erf2(float& x0, float& x1) {
  const f32x2_t a = {fminf(fabsf(x0), 6.0f), fminf(fabsf(x1), 6.0f)};
  f32x2_t q = __builtin_elementwise_fma((f32x2_t)(3.309693057e-05f), a, (f32x2_t)(-7.692557992e-04f));
  q = __builtin_elementwise_fma(q, a, (f32x2_t)(8.080835454e-03f));
  q = __builtin_elementwise_fma(q, a, (f32x2_t)(-5.341228843e-02f));
  q = __builtin_elementwise_fma(q, a, (f32x2_t)(-4.587708414e-01f));
  q = __builtin_elementwise_fma(q, a, (f32x2_t)(-1.151201725e+00f));
  q = __builtin_elementwise_fma(q, a, (f32x2_t)(-9.999930859e-01f));
  const f32x2_t e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2_t xv = {x0, x1};
  const f32x2_t r = __builtin_elementwise_fma(xv, (f32x2_t)(0.f), (f32x2_t){fmaxf(x0, 0.f), fmaxf(x1, 0.f)});
  const f32x2_t o = __builtin_elementwise_fma(-a, e, r);
  x0 = o.x;
  x1 = o.y;
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// d/dx of gelu_erf with the same branch-free erf (A&S 7.1.26, |err| <= 1.5e-7) and one exp shared
// by the cdf and pdf terms (libm erff branches on |x| < 1 and made the GELU backward VALU-bound);
// shared by comet_act_bwd_colsum and the GEMM epilogue that applies a GELU backward (gemm.hip)
__device__ __forceinline__ float gelu_grad_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __expf(-z * z);  // = exp(-x^2 / 2)
  const float erf_v = copysignf(1.0f - p * t * e, x);
  return 0.5f * (1.0f + erf_v) + x * (0.39894228040143267794f * e);
}

__device__ __forceinline__ float apply_act(int act, float v) {
  switch (act) {
    case COMET_ACT_GELU: return gelu_erf(v);
    case COMET_ACT_RELU: return v > 0.f ? v : 0.f;
    case COMET_ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    default: return v;
  }
}
// apply_act over NV (even) consecutive values: GELU in pairs (gelu_erf2), the others one by one
template <int NV>
__device__ __forceinline__ void apply_act_n(int act, float* v) {
  if (act == COMET_ACT_GELU) {
#pragma unroll
    for (int e = 0; e < NV; e += 2) gelu_erf2(v[e], v[e + 1]);
  } else {
#pragma unroll
    for (int e = 0; e < NV; ++e) v[e] = apply_act(act, v[e]);
  }
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 T1):
// blocks b, b+8, b+16 ... land on one XCD; give each XCD a contiguous chunk of tiles.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int xcd = bid & 7, local = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

// (x, y) block coordinates of a 2-D grid remapped so that consecutive x of one y run on one XCD:
// the hardware deals linear ids (x fastest) round-robin over the 8 XCDs, so without this the
// query / key tiles of one attention head (x) are spread over every XCD and each XCD's L2 fetches
// that head's shared operand again.
__device__ __forceinline__ void xcd_remap2(int& x, int& y) {
  const int gx = gridDim.x;
  const int r = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gridDim.y);
  y = r / gx;
  x = r - y * gx;
}

// Row-blocked NHWC launches (resize / pooling): R = items per output row (ow x channel groups),
// a 256-thread block covers RB = max(1, 256 / R) output rows (n, oy) and loops over a row's items
// when R > 256. Index math is 32-bit and done once per thread, not per element (the flat 64-bit
// div / mod decomposition of a grid-stride loop made these kernels VALU-bound).
struct RowBlock {
  int R, RB, nrows;
};
inline RowBlock make_rowblock(int64_t nrows, int64_t items) {
  RowBlock rb;
  rb.R = (int)items;
  rb.RB = items >= 256 ? 1 : (int)(256 / items);
  rb.nrows = (int)nrows;
  return rb;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace comet
