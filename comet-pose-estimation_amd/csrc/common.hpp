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

#define COMET_CHECK_LAUNCH(name)                                                 \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      ::comet::set_error(std::string(name) + ": " + hipGetErrorString(e_));      \
      return COMET_ELAUNCH;                                                      \
    }                                                                            \
  } while (0)

// ---- scalar conversions -------------------------------------------------------------------
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__bf16 x) { return static_cast<float>(x); }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ __bf16 from_f32<__bf16>(float x) { return static_cast<__bf16>(x); }

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

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float apply_act(int act, float v) {
  switch (act) {
    case COMET_ACT_GELU: return gelu_erf(v);
    case COMET_ACT_RELU: return v > 0.f ? v : 0.f;
    case COMET_ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    default: return v;
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

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace comet
