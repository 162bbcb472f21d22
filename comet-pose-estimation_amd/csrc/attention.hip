// Fused multi-head attention forward + materialised-backward helpers.
//
// Replaces nn.MultiheadAttention's explicit q·kᵀ·scale → softmax → ·v path (SURVEY Appendix
// B-17; modules.py:290,339) at every use site of the hot path: head self/cross attention
// (camera_predictor10.py:663-683), T_P cross attention (329-348), trunk (382), tracker time /
// space blocks (blocks.py:312-340) and the DINOv2 backbone.
//
// Forward structure (one workgroup = 4 waves = 64 queries of one (batch, head)):
//  * each wave owns 16 queries, Q fragments live in registers for the whole kernel;
//  * K/V tiles of 64 keys are staged global -> registers -> LDS (next tile's global loads are
//    issued before the current tile's MFMAs);
//  * Sᵀ = K·Qᵀ is computed ("swapped" product): the accumulator has the query on the lane and
//    the keys in registers, so the running max / sum of a query are lane-local plus two
//    shuffles over the four 16-lane groups;
//  * Oᵀ = Vᵀ·Pᵀ takes P straight from the Sᵀ registers as the B operand (k order permuted
//    consistently for both operands); the Vᵀ fragments come from a row-major V tile via
//    ds_read_b64_tr_b16 (bf16) or plain ds_read_b32 (f32).
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace comet {
namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

template <typename T, int D> struct ACfg;
template <int D> struct ACfg<__bf16, D> {
  static constexpr int DA = ((D + 31) / 32) * 32;  // k-dim of the Q·Kᵀ MFMA (x32)
  static constexpr int KP = DA + 8;                 // LDS row pitch (elements)
  static constexpr int VEC = 8;
};
template <int D> struct ACfg<float, D> {
  static constexpr int DA = ((D + 15) / 16) * 16;
  static constexpr int KP = DA + 4;
  static constexpr int VEC = 4;
};

// optional inner batch: batch index b = (b / n) * s*_b + (b % n) * s*  (the tracker's space
// attention runs over tracks of a [B, N, T, C] tensor for every (b, t) without permuting it)
struct Inner { int64_t n, sq, sk, sv, so; };

template <typename T> struct AVec;
template <> struct AVec<__bf16> { typedef uint4 type; };
template <> struct AVec<float> { typedef float4 type; };

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// max of two scores without fmaxf's NaN canonicalisation of both operands (two extra v_max_f32 per
// call on permlane results); the scores are finite or -inf
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
typedef __attribute__((address_space(3))) void lds_void;

template <typename T, int D>
__global__ void __launch_bounds__(256)
attn_fwd_kernel(const T* __restrict__ Q, int64_t sq_b, int64_t sq_h, int64_t sq_l,
                const T* __restrict__ K, int64_t sk_b, int64_t sk_h, int64_t sk_l,
                const T* __restrict__ V, int64_t sv_b, int64_t sv_h, int64_t sv_l,
                T* __restrict__ O, int64_t so_b, int64_t so_h, int64_t so_l,
                float* __restrict__ LSE, int heads, int lq, int lk, float scale_log2, Inner in) {
  typedef ACfg<T, D> C;
  constexpr int DA = C::DA, KP = C::KP, VEC = C::VEC;
  constexpr int DT = (D + 15) / 16;
  constexpr bool BF = sizeof(T) == 2;
  constexpr int NVROW = D / VEC;                    // vectors per key row
  constexpr int NVT = (64 * NVROW + 255) / 256;     // vectors per thread per tile
  typedef typename AVec<T>::type vec_t;

  __shared__ __attribute__((aligned(16))) T Ks[64 * KP];
  __shared__ __attribute__((aligned(16))) T Vs[64 * KP];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, hg = lane >> 4;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by;
  const int64_t b = bh / heads, h = bh % heads;
  const int64_t bo = b / in.n, bi = b % in.n;
  Q += bo * sq_b + bi * in.sq + h * sq_h;
  K += bo * sk_b + bi * in.sk + h * sk_h;
  V += bo * sv_b + bi * in.sv + h * sv_h;
  O += bo * so_b + bi * in.so + h * so_h;

  // zero LDS once: pad columns [D, DA) stay zero for the whole kernel
  for (int i = tid; i < 64 * KP; i += 256) { Ks[i] = T(0.f); Vs[i] = T(0.f); }

  // ---- Q fragments (registers) ----
  const int q = bx * 64 + wid * 16 + li;
  const bool qok = q < lq;
  constexpr int NQC = BF ? DA / 32 : DA / 16;
  typedef typename std::conditional<BF, bf16x8, f32x4>::type qfrag_t;
  qfrag_t qf[NQC];
#pragma unroll
  for (int c = 0; c < NQC; ++c) {
    const int d0 = BF ? 32 * c + 8 * hg : 16 * c + 4 * hg;
    if (qok && d0 < D) {
      qf[c] = *reinterpret_cast<const qfrag_t*>(Q + (int64_t)q * sq_l + d0);
    } else {
      qf[c] = qfrag_t{};
    }
  }

  f32x4 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int ntiles = (lk + 63) / 64;
  vec_t kreg[NVT], vreg[NVT];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NVROW, cv = (idx % NVROW) * VEC;
      const int key = t * 64 + row;
      if (idx < 64 * NVROW && key < lk) {
        kreg[i] = *reinterpret_cast<const vec_t*>(K + (int64_t)key * sk_l + cv);
        vreg[i] = *reinterpret_cast<const vec_t*>(V + (int64_t)key * sv_l + cv);
      } else {
        kreg[i] = vec_t{};
        vreg[i] = vec_t{};
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NVROW) {
        const int row = idx / NVROW, cv = (idx % NVROW) * VEC;
        *reinterpret_cast<vec_t*>(Ks + row * KP + cv) = kreg[i];
        *reinterpret_cast<vec_t*>(Vs + row * KP + cv) = vreg[i];
      }
    }
  };

  gload(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();  // previous tile fully consumed (and LDS zeroing done)
    lstore();
    __syncthreads();
    if (t + 1 < ntiles) gload(t + 1);

    // ---- Sᵀ = K·Qᵀ : 4 subtiles of 16 keys ----
    f32x4 s[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = f32x4{0.f, 0.f, 0.f, 0.f};
      const T* krow = Ks + (st * 16 + li) * KP;
      if constexpr (BF) {
#pragma unroll
        for (int c = 0; c < NQC; ++c) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(krow + 32 * c + 8 * hg);
          s[st] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[c], s[st], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int c = 0; c < NQC; ++c) {
          const f32x4 kf = *reinterpret_cast<const f32x4*>(krow + 16 * c + 4 * hg);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            s[st] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[e], qf[c][e], s[st], 0, 0, 0);
        }
      }
    }
    // ---- online softmax (log2 domain); key of s[st][r] = t*64 + st*16 + 4*hg + r ----
    float mt = -INFINITY;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = t * 64 + st * 16 + 4 * hg + r;
        const float v = key < lk ? s[st][r] * scale_log2 : -INFINITY;
        s[st][r] = v;
        mt = fmaxf(mt, v);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = exp2f(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[st][r] - m_new);
        s[st][r] = p;
        ls += p;
      }
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < DT; ++i) o[i] *= alpha;

    // ---- Oᵀ += Vᵀ·Pᵀ ----
    if constexpr (BF) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bf16x4 p0 = __builtin_convertvector(s[2 * u], bf16x4);
        const bf16x4 p1 = __builtin_convertvector(s[2 * u + 1], bf16x4);
        const bf16x8 pf = __builtin_shufflevector(p0, p1, 0, 1, 2, 3, 4, 5, 6, 7);
        const int qq = li >> 2, pp = li & 3;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const T* a0 = Vs + (16 * (2 * u) + 4 * hg + qq) * KP + 16 * dt + 4 * pp;
          const T* a1 = Vs + (16 * (2 * u + 1) + 4 * hg + qq) * KP + 16 * dt + 4 * pp;
          const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
          const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
          const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const T* vrow = Vs + (16 * st + 4 * hg + r) * KP + li;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vrow[16 * dt], s[st][r], o[dt], 0, 0, 0);
        }
    }
  }

  // ---- epilogue ----
  float l_tot = l_run;
  l_tot += __shfl_xor(l_tot, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (!qok) return;
  const float inv = 1.f / l_tot;
  T* orow = O + (int64_t)q * so_l;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int d0 = 16 * dt + 4 * hg;
    if (d0 < D) {
      if constexpr (BF) {
        bf16x4 w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = static_cast<__bf16>(o[dt][r] * inv);
        *reinterpret_cast<bf16x4*>(orow + d0) = w;
      } else {
        f32x4 w = o[dt] * inv;
        *reinterpret_cast<f32x4*>(orow + d0) = w;
      }
    }
  }
  if (LSE && hg == 0) LSE[bh * lq + q] = (m_run + log2f(l_tot)) * LN2;
}

// bf16 forward, QG query groups of 16 per wave (one workgroup = 4 waves = 64*QG queries).
// Same Sᵀ = K·Qᵀ / Oᵀ = Vᵀ·Pᵀ formulation as attn_fwd_kernel, trimmed for the VALU budget that
// bounds attention at these head dims (a 16x16x32 MFMA leaves 8 issue cycles for the vector
// unit; the softmax costs ~20 cycles of VALU per score-per-lane):
//  * every K / Vᵀ fragment read from LDS feeds QG MFMAs (one per query group);
//  * the softmax scale is folded into one FMA per score, exp2 is the bare v_exp_f32;
//  * the key mask runs only on the last tile;
//  * O is rescaled only when some lane's running max moved (exact: alpha == 1 otherwise).
template <int D, int QG, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
attn_fwd_bf16_kernel(const __bf16* __restrict__ Q, int64_t sq_b, int64_t sq_h, int64_t sq_l,
                     const __bf16* __restrict__ K, int64_t sk_b, int64_t sk_h, int64_t sk_l,
                     const __bf16* __restrict__ V, int64_t sv_b, int64_t sv_h, int64_t sv_l,
                     __bf16* __restrict__ O, int64_t so_b, int64_t so_h, int64_t so_l,
                     float* __restrict__ LSE, int heads, int lq, int lk, float scale_log2, Inner in) {
  constexpr int DA = ((D + 31) / 32) * 32;
  // LDS row pitch: K is read by ds_read_b128 (lane (li, hg) takes row li, 16-B chunk 4c + hg; the
  // four 16-lane groups {0-3,12-15,20-27}, ... each need 16 distinct 16-B slots of the 256-B bank row:
  // slot = (KP / 8) li + hg + 4c mod 16), V by ds_read_b64_tr_b16 (rows 4 hg + qq of 8 dwords each per
  // 32-lane half: distinct 8-dword windows mod 64). KP / 8 = 10 (DA <= 64) or 14 (DA = 96) satisfies
  // both; the round-4 pitch DA + 8 (9 or 13 slots) put ~2 conflict cycles on every K read
  // (SQ_LDS_BANK_CONFLICT 11.3 M for 5.7 M LDS instructions, profiles/r04_attn/pmc_fwd_d64.txt)
  constexpr int KP = DA <= 64 ? 80 : 112;
  static_assert(DA <= 96, "attn_fwd_bf16_kernel: D <= 96");
  constexpr int DT = (D + 15) / 16, NQC = DA / 32;
  constexpr int NVROW = D / 8, NVT = (64 * NVROW + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 Ks[64 * KP];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[64 * KP];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, hg = lane >> 4;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by;
  const int64_t b = bh / heads, h = bh % heads;
  const int64_t bo = b / in.n, bi = b % in.n;
  Q += bo * sq_b + bi * in.sq + h * sq_h;
  K += bo * sk_b + bi * in.sk + h * sk_h;
  V += bo * sv_b + bi * in.sv + h * sv_h;
  O += bo * so_b + bi * in.so + h * so_h;

  if constexpr (DA != D) {  // pad columns [D, DA) of K stay zero for the whole kernel
    for (int i = tid; i < 64 * KP; i += 256) Ks[i] = __bf16(0.f);
  }

  bf16x8 qf[QG][NQC];
  int qrow[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    qrow[g] = bx * (64 * QG) + (wid * QG + g) * 16 + li;
#pragma unroll
    for (int c = 0; c < NQC; ++c) {
      const int d0 = 32 * c + 8 * hg;
      qf[g][c] = (qrow[g] < lq && d0 < D) ? *reinterpret_cast<const bf16x8*>(Q + (int64_t)qrow[g] * sq_l + d0) : bf16x8{};
    }
  }
  // lacc: the row sums of P on the matrix core -- Oᵀ's extra 16-row tile with an all-ones A operand,
  // so every register of a lane holds its query's sum over the keys so far (the sum of the bf16 P
  // that the PV MFMAs consume, rescaled with O): 4 MFMAs per tile instead of 16 v_add_f32 per query
  // group (the kernel is bound by vector issue)
  f32x4 o[QG][DT], lacc[QG];
  float m_run[QG];
  const bf16x8 ones = __builtin_bit_cast(bf16x8, uint4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    m_run[g] = -INFINITY;
    lacc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < DT; ++i) o[g][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int ntiles = (lk + 63) / 64;
  uint4 kreg[NVT], vreg[NVT];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NVROW, cv = (idx % NVROW) * 8;
      const int key = t * 64 + row;
      const bool ok = idx < 64 * NVROW && key < lk;
      kreg[i] = ok ? *reinterpret_cast<const uint4*>(K + (int64_t)key * sk_l + cv) : uint4{0, 0, 0, 0};
      vreg[i] = ok ? *reinterpret_cast<const uint4*>(V + (int64_t)key * sv_l + cv) : uint4{0, 0, 0, 0};
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NVROW) {
        const int row = idx / NVROW, cv = (idx % NVROW) * 8;
        *reinterpret_cast<uint4*>(Ks + row * KP + cv) = kreg[i];
        *reinterpret_cast<uint4*>(Vs + row * KP + cv) = vreg[i];
      }
    }
  };

  // one 64-key tile; MASK only for a ragged last tile
  auto tile = [&](int t, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    f32x4 s[QG][4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
#pragma unroll
      for (int g = 0; g < QG; ++g) s[g][st] = f32x4{0.f, 0.f, 0.f, 0.f};
      const __bf16* krow = Ks + (st * 16 + li) * KP + 8 * hg;
#pragma unroll
      for (int c = 0; c < NQC; ++c) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(krow + 32 * c);
#pragma unroll
        for (int g = 0; g < QG; ++g) s[g][st] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[g][c], s[g][st], 0, 0, 0);
      }
    }
    bf16x8 pf[QG][2];
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      if constexpr (MASK) {
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t * 64 + st * 16 + 4 * hg + r >= lk) s[g][st][r] = -INFINITY;
      }
      // the 16 scores of the lane: a v_max3 tree (8 instructions); the 4 lane groups of a query meet by
      // v_permlane16_swap / v_permlane32_swap (no LDS round trip as with ds_bpermute)
      const float* sv = reinterpret_cast<const float*>(&s[g][0]);
      float mt = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), sv[2]), fmaxf(fmaxf(sv[3], sv[4]), sv[5]));
      mt = fmaxf(fmaxf(mt, fmaxf(fmaxf(sv[6], sv[7]), sv[8])), fmaxf(fmaxf(sv[9], sv[10]), sv[11]));
      mt = fmaxf(fmaxf(mt, fmaxf(fmaxf(sv[12], sv[13]), sv[14])), sv[15]);
      {
        const auto w16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(mt), __float_as_uint(mt), false, false);
        mt = vmax_raw(__uint_as_float(w16[0]), __uint_as_float(w16[1]));
        const auto w32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(mt), __float_as_uint(mt), false, false);
        mt = vmax_raw(__uint_as_float(w32[0]), __uint_as_float(w32[1]));
      }
      const float m_new = fmaxf(m_run[g], mt * scale_log2);
      if (__ballot(m_new > m_run[g]) != 0) {
        const float alpha = __builtin_amdgcn_exp2f(m_run[g] - m_new);
        lacc[g] *= alpha;
#pragma unroll
        for (int i = 0; i < DT; ++i) o[g][i] *= alpha;
        m_run[g] = m_new;
      }
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[g][st][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[g][st][r], scale_log2, -m_new));
#pragma unroll
      for (int u = 0; u < 2; ++u)
        pf[g][u] = __builtin_shufflevector(__builtin_convertvector(s[g][2 * u], bf16x4),
                                           __builtin_convertvector(s[g][2 * u + 1], bf16x4), 0, 1, 2, 3, 4, 5, 6, 7);
    }
    const int qq = li >> 2, pp = li & 3;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const __bf16* a0 = Vs + (16 * (2 * u) + 4 * hg + qq) * KP + 16 * dt + 4 * pp;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 16 * KP));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int g = 0; g < QG; ++g) o[g][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[g][u], o[g][dt], 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < QG; ++g) lacc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[g][u], lacc[g], 0, 0, 0);
    }
  };

  // full tiles unmasked; the last tile (peeled: one masked instantiation outside the loop keeps
  // the loop's register allocation that of the unmasked body) masks keys >= lk
  gload(0);
  for (int t = 0; t < ntiles - 1; ++t) {
    __syncthreads();  // previous tile consumed (and LDS zeroing done)
    lstore();
    __syncthreads();
    gload(t + 1);
    tile(t, std::false_type{});
  }
  __syncthreads();
  lstore();
  __syncthreads();
  tile(ntiles - 1, std::true_type{});

#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const float l_tot = lacc[g][0];
    if (qrow[g] >= lq) continue;
    const float inv = 1.f / l_tot;
    __bf16* orow = O + (int64_t)qrow[g] * so_l;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d0 = 16 * dt + 4 * hg;
      if (d0 < D) *reinterpret_cast<bf16x4*>(orow + d0) = __builtin_convertvector(o[g][dt] * inv, bf16x4);
    }
    if (LSE && hg == 0) LSE[bh * lq + qrow[g]] = (m_run[g] + log2f(l_tot)) * LN2;
  }
}

// bf16 forward on 32x32x16 MFMAs (D = 32, 48, 64, 96), one workgroup = 4 waves = 128 queries of one
// (batch, head), 2 workgroups per CU. Per wave: 32 queries; per 64-key tile
//  * Sᵀ = K·Qᵀ as two 32x32 blocks (keys x queries; D / 16 k-steps each, Q fragments in registers):
//    a lane holds one query and 16 keys of each block, so the row max / sum are 32 lane-local values
//    plus one v_permlane32_swap with the partner half;
//  * P stays in the accumulator registers: registers 8s..8s+7 of a block, packed to bf16, are the
//    B fragment of k-step s of Oᵀ = Vᵀ·Pᵀ, whose k order (16s + 8(j>>2) + 4h + (j&3)) the Vᵀ
//    fragments follow: two ds_read_b64_tr_b16 of 4 consecutive keys each;
//  * K / V tiles: global loads into registers issued before the tile's MFMAs, written to the other
//    LDS buffer after them, one barrier per tile (rows padded by 16 B: conflict-free b128 and
//    tr16 reads).
// A 32x32x16 MFMA carries twice the work of a 16x16x32 one for the same 8 cycles of vector issue,
// which the softmax (about 20 cycles of VALU per score per lane) needs.
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int D>
__global__ void __launch_bounds__(256, 2)
attn_fwd32_kernel(const __bf16* __restrict__ Q, int64_t sq_b, int64_t sq_h, int64_t sq_l,
                  const __bf16* __restrict__ K, int64_t sk_b, int64_t sk_h, int64_t sk_l,
                  const __bf16* __restrict__ V, int64_t sv_b, int64_t sv_h, int64_t sv_l,
                  __bf16* __restrict__ O, int64_t so_b, int64_t so_h, int64_t so_l,
                  float* __restrict__ LSE, int heads, int lq, int lk, float scale_log2, Inner in) {
  static_assert(D % 16 == 0 && D <= 128, "D: multiple of 16");
  constexpr int NKS = D / 16;            // k-steps of Sᵀ = K·Qᵀ
  constexpr int DB = (D + 31) / 32;      // 32-row blocks of Oᵀ
  constexpr int KP = D + 8;              // K row pitch (elements): ds_read_b128 slots 7r, 9r, 13r mod 16 distinct
  // V row pitch; columns [D, 32 DB) stay zero. The Vᵀ tr16 reads of a 32-lane half cover 4 rows x 16
  // dwords: a pitch of 16 or 48 dwords mod 64 puts them on 4 disjoint quarters of the bank row (the
  // round-4 pitch 32 DB + 8 overlapped neighbouring rows: 2-way conflicts)
  constexpr int VP = DB == 1 ? 32 : DB <= 3 ? 96 : 160;
  static_assert(VP >= DB * 32 && ((VP / 2) % 64 == 16 || (VP / 2) % 64 == 48), "V pitch");
  constexpr int NCH = D / 8;             // 16-B chunks per key row
  constexpr int NST = (64 * NCH + 255) / 256;  // chunks per thread per tile (K and V each)
  __shared__ __attribute__((aligned(16))) __bf16 Ks[2][64 * KP];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[2][64 * VP];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by;
  const int64_t b = bh / heads, hd = bh % heads;
  const int64_t bo = b / in.n, bi = b % in.n;
  Q += bo * sq_b + bi * in.sq + hd * sq_h;
  K += bo * sk_b + bi * in.sk + hd * sk_h;
  V += bo * sv_b + bi * in.sv + hd * sv_h;
  O += bo * so_b + bi * in.so + hd * so_h;

  if constexpr (DB * 32 != D) {  // zero V's pad columns once (both buffers)
    for (int i = tid; i < 2 * 64 * (DB * 32 - D); i += 256) {
      const int buf = i / (64 * (DB * 32 - D)), rem = i % (64 * (DB * 32 - D));
      Vs[buf][(rem / (DB * 32 - D)) * VP + D + rem % (DB * 32 - D)] = __bf16(0.f);
    }
  }

  const int qrow = bx * 128 + wid * 32 + r;
  bf16x8 qf[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s)
    qf[s] = qrow < lq ? *reinterpret_cast<const bf16x8*>(Q + (int64_t)qrow * sq_l + 16 * s + 8 * h) : bf16x8{};

  // lacc: the row sums of P on the matrix core (an all-ones A operand beside the PV MFMAs: every
  // register of a lane holds its query's sum of the bf16 P consumed so far, rescaled with O), in
  // place of 32 v_add_f32 per tile
  f32x16 oacc[DB], lacc = f32x16{};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, uint4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
#pragma unroll
  for (int i = 0; i < DB; ++i) oacc[i] = f32x16{};
  float m_run = -INFINITY;

  uint4 kst[NST], vst[NST];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NCH, c = idx % NCH;
      const int key = t * 64 + row;
      const bool ok = idx < 64 * NCH && key < lk;
      kst[i] = ok ? *reinterpret_cast<const uint4*>(K + (int64_t)key * sk_l + 8 * c) : uint4{0, 0, 0, 0};
      vst[i] = ok ? *reinterpret_cast<const uint4*>(V + (int64_t)key * sv_l + 8 * c) : uint4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NCH) {
        const int row = idx / NCH, c = idx % NCH;
        *reinterpret_cast<uint4*>(&Ks[buf][row * KP + 8 * c]) = kst[i];
        *reinterpret_cast<uint4*>(&Vs[buf][row * VP + 8 * c]) = vst[i];
      }
    }
  };
  // per-lane part of the Vᵀ tr16 read address: 16-lane group g, lane 4q + p of it reads key row q,
  // columns 4p..4p+3 of the group's 16-column slice
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int voff = (4 * (tg >> 1) + tq) * VP + 16 * (tg & 1) + 4 * tp;

  auto tile = [&](int t, int buf, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const __bf16* ks = Ks[buf];
    const __bf16* vs = Vs[buf];
    f32x16 sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      sacc[kb] = f32x16{};
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + (kb * 32 + r) * KP + 16 * s + 8 * h);
        sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kb], 0, 0, 0);
      }
    }
    if constexpr (MASK) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (t * 64 + kb * 32 + (j & 3) + 8 * (j >> 2) + 4 * h >= lk) sacc[kb][j] = -INFINITY;
    }
    // the lane's 32 scores: a v_max3 tree (16 instructions), then the partner half by permlane32
    float mt = fmaxf(fmaxf(sacc[0][0], sacc[0][1]), sacc[0][2]);
#pragma unroll
    for (int j = 3; j < 15; j += 2) mt = fmaxf(fmaxf(mt, sacc[0][j]), sacc[0][j + 1]);
    mt = fmaxf(fmaxf(mt, sacc[0][15]), sacc[1][0]);
#pragma unroll
    for (int j = 1; j < 15; j += 2) mt = fmaxf(fmaxf(mt, sacc[1][j]), sacc[1][j + 1]);
    mt = fmaxf(mt, sacc[1][15]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mt), __float_as_uint(mt), false, false);
      mt = vmax_raw(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const float m_new = fmaxf(m_run, mt * scale_log2);
    if (__ballot(m_new > m_run) != 0) {  // exact: alpha == 1 for every lane otherwise
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      lacc *= alpha;
#pragma unroll
      for (int i = 0; i < DB; ++i) oacc[i] *= alpha;
      m_run = m_new;
    }
    bf16x8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int j = 0; j < 16; ++j) sacc[kb][j] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kb][j], scale_log2, -m_new));
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f32x4 lo = {sacc[kb][8 * s], sacc[kb][8 * s + 1], sacc[kb][8 * s + 2], sacc[kb][8 * s + 3]};
        const f32x4 hi = {sacc[kb][8 * s + 4], sacc[kb][8 * s + 5], sacc[kb][8 * s + 6], sacc[kb][8 * s + 7]};
        pf[kb][s] = __builtin_shufflevector(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4),
                                            0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[kb][s], lacc, 0, 0, 0);
        const __bf16* va = vs + (kb * 32 + 16 * s) * VP + voff;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(va + 32 * db));
          const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(va + 8 * VP + 32 * db));
          const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][s], oacc[db], 0, 0, 0);
        }
      }
  };

  const int ntiles = (lk + 63) / 64;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int t = 0; t < ntiles - 1; ++t) {
    gload(t + 1);  // lands during this tile's MFMAs
    tile(t, t & 1, std::false_type{});
    lstore((t + 1) & 1);  // that buffer's last reader (tile t - 1) finished before the last barrier
    __syncthreads();
  }
  tile(ntiles - 1, (ntiles - 1) & 1, std::true_type{});

  const float l_tot = lacc[0];
  // O rows: lane (r, h) holds d = 32 db + 8u + 4h + (0..3); a v_permlane32_swap per dword of the
  // (u, u + 1) pair gives each lane 8 contiguous d (16-B stores, cdna_hip_programming.md T21)
  const float inv = 1.f / l_tot;
  __bf16* orow = O + (int64_t)qrow * so_l;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int u = 0; u < 4; u += 2) {
      if (32 * db + 8 * u >= D) continue;  // D % 16 == 0: a pair is all in or all out
      uint2 pk[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x4 w = f32x4{oacc[db][4 * (u + e)], oacc[db][4 * (u + e) + 1], oacc[db][4 * (u + e) + 2],
                              oacc[db][4 * (u + e) + 3]} * inv;
        pk[e] = __builtin_bit_cast(uint2, __builtin_convertvector(w, bf16x4));
      }
      const auto sx = __builtin_amdgcn_permlane32_swap(pk[0].x, pk[1].x, false, false);
      const auto sy = __builtin_amdgcn_permlane32_swap(pk[0].y, pk[1].y, false, false);
      if (qrow < lq) *reinterpret_cast<uint4*>(orow + 32 * db + 8 * u + 8 * h) = uint4{sx[0], sy[0], sx[1], sy[1]};
    }
  if (LSE && h == 0 && qrow < lq) LSE[bh * lq + qrow] = (m_run + log2f(l_tot)) * LN2;
}

// Short sequences (Lq, Lk <= 16: the tracker's per-track time attention over S = 16 frames,
// blocks.py:312-321): one wave per (batch, head) instead of a 64 x 64 tile that would be 1/16
// occupied. Sᵀ = K·Qᵀ in one 16x16 MFMA tile per 32 of d (K and Q fragments straight from
// global), column softmax over the 4 lane groups, Oᵀ = Vᵀ·Pᵀ with v_mfma_f32_16x16x16_bf16 whose
// k = 4g + j matches the Sᵀ accumulator layout, Vᵀ fragments via ds_read_b64_tr_b16.
template <int D>
__global__ void __launch_bounds__(256)
attn_small_kernel(const __bf16* __restrict__ Q, int64_t sq_b, int64_t sq_h, int64_t sq_l,
                  const __bf16* __restrict__ K, int64_t sk_b, int64_t sk_h, int64_t sk_l,
                  const __bf16* __restrict__ V, int64_t sv_b, int64_t sv_h, int64_t sv_l,
                  __bf16* __restrict__ O, int64_t so_b, int64_t so_h, int64_t so_l,
                  float* __restrict__ LSE, int heads, int lq, int lk, float scale_log2, int64_t nbh, Inner in) {
  constexpr int DA = ((D + 31) / 32) * 32, NQC = DA / 32, DT = D / 16, KP = D + 8, NV = D / 8;
  __shared__ __attribute__((aligned(16))) __bf16 Vs[4][16 * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int64_t bh = (int64_t)blockIdx.x * 4 + w;
  const bool valid = bh < nbh;
  const int64_t b = valid ? bh / heads : 0, h = valid ? bh % heads : 0;
  const int64_t bo = b / in.n, bi = b % in.n;
  Q += bo * sq_b + bi * in.sq + h * sq_h;
  K += bo * sk_b + bi * in.sk + h * sk_h;
  V += bo * sv_b + bi * in.sv + h * sv_h;
  __bf16* vs = Vs[w];
  for (int idx = lane; idx < 16 * NV; idx += 64) {
    const int row = idx / NV, cv = (idx % NV) * 8;
    const uint4 v = (valid && row < lk) ? *reinterpret_cast<const uint4*>(V + (int64_t)row * sv_l + cv) : uint4{0, 0, 0, 0};
    *reinterpret_cast<uint4*>(vs + row * KP + cv) = v;
  }
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NQC; ++c) {
    const int d0 = 32 * c + 8 * g;
    const bf16x8 qf = (valid && li < lq && d0 < D) ? *reinterpret_cast<const bf16x8*>(Q + (int64_t)li * sq_l + d0) : bf16x8{};
    const bf16x8 kf = (valid && li < lk && d0 < D) ? *reinterpret_cast<const bf16x8*>(K + (int64_t)li * sk_l + d0) : bf16x8{};
    s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, s, 0, 0, 0);
  }
  float m = -INFINITY;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float v = (4 * g + r) < lk ? s[r] * scale_log2 : -INFINITY;
    s[r] = v;
    m = fmaxf(m, v);
  }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    s[r] = exp2f(s[r] - m);
    l += s[r];
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const s16x4 pb = __builtin_bit_cast(s16x4, __builtin_convertvector(s, bf16x4));
  __syncthreads();  // V tiles staged
  const int qq = li >> 2, pp = li & 3;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vs + (4 * g + qq) * KP + 16 * dt + 4 * pp));
    o[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  if (!valid || li >= lq) return;
  const float inv = 1.f / l;
  __bf16* orow = O + bo * so_b + bi * in.so + h * so_h + (int64_t)li * so_l;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
    *reinterpret_cast<bf16x4*>(orow + 16 * dt + 4 * g) = __builtin_convertvector(o[dt] * inv, bf16x4);
  if (LSE && g == 0) LSE[bh * lq + li] = (m + log2f(l)) * LN2;
}

inline Inner inner_of(const comet_attn_args& a) {
  if (a.batch_inner <= 1) return Inner{1, 0, 0, 0, 0};
  return Inner{a.batch_inner, a.sq_i, a.sk_i, a.sv_i, a.so_i};
}

template <int D>
int launch_small(const comet_attn_args& a, hipStream_t s) {
  const int64_t nbh = a.batch * a.heads;
  hipLaunchKernelGGL((attn_small_kernel<D>), dim3((unsigned)cdiv(nbh, 4)), dim3(256), 0, s,
                     (const __bf16*)a.q, a.sq_b, a.sq_h, a.sq_l, (const __bf16*)a.k, a.sk_b, a.sk_h, a.sk_l,
                     (const __bf16*)a.v, a.sv_b, a.sv_h, a.sv_l, (__bf16*)a.o, a.so_b, a.so_h, a.so_l,
                     a.lse, (int)a.heads, (int)a.lq, (int)a.lk, a.scale * LOG2E, nbh, inner_of(a));
  COMET_CHECK_LAUNCH("comet_attention_fwd (short)");
  return COMET_OK;
}

template <typename T, int D>
int launch_fwd(const comet_attn_args& a, hipStream_t s) {
  dim3 grid((unsigned)cdiv(a.lq, 64), (unsigned)(a.batch * a.heads));
  hipLaunchKernelGGL((attn_fwd_kernel<T, D>), grid, dim3(256), 0, s,
                     (const T*)a.q, a.sq_b, a.sq_h, a.sq_l, (const T*)a.k, a.sk_b, a.sk_h, a.sk_l,
                     (const T*)a.v, a.sv_b, a.sv_h, a.sv_l, (T*)a.o, a.so_b, a.so_h, a.so_l,
                     a.lse, (int)a.heads, (int)a.lq, (int)a.lk, a.scale * LOG2E, inner_of(a));
  COMET_CHECK_LAUNCH("comet_attention_fwd");
  return COMET_OK;
}

template <int D>
int launch_fwd_bf16(const comet_attn_args& a, hipStream_t s) {
  // two query groups per wave when both sequences span several tiles (measured on the COMET
  // shapes, tools/attn_bench.py: DINO 581x581 D64 497 -> 317 us, head 577x577 D96 419 -> 273 us);
  // with a single key tile the halved grid costs more than the K/V fragment reuse saves
  const bool two = a.lq > 64 && a.lk > 64;
  dim3 grid((unsigned)cdiv(a.lq, two ? 128 : 64), (unsigned)(a.batch * a.heads));
  auto kern = two ? attn_fwd_bf16_kernel<D, 2, (D > 64 ? 3 : 2)> : attn_fwd_bf16_kernel<D, 1, 4>;
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s,
                     (const __bf16*)a.q, a.sq_b, a.sq_h, a.sq_l, (const __bf16*)a.k, a.sk_b, a.sk_h, a.sk_l,
                     (const __bf16*)a.v, a.sv_b, a.sv_h, a.sv_l, (__bf16*)a.o, a.so_b, a.so_h, a.so_l,
                     a.lse, (int)a.heads, (int)a.lq, (int)a.lk, a.scale * LOG2E, inner_of(a));
  COMET_CHECK_LAUNCH("comet_attention_fwd");
  return COMET_OK;
}

template <int D>
int launch_fwd32(const comet_attn_args& a, hipStream_t s) {
  dim3 grid((unsigned)cdiv(a.lq, 128), (unsigned)(a.batch * a.heads));
  hipLaunchKernelGGL((attn_fwd32_kernel<D>), grid, dim3(256), 0, s,
                     (const __bf16*)a.q, a.sq_b, a.sq_h, a.sq_l, (const __bf16*)a.k, a.sk_b, a.sk_h, a.sk_l,
                     (const __bf16*)a.v, a.sv_b, a.sv_h, a.sv_l, (__bf16*)a.o, a.so_b, a.so_h, a.so_l,
                     a.lse, (int)a.heads, (int)a.lq, (int)a.lk, a.scale * LOG2E, inner_of(a));
  COMET_CHECK_LAUNCH("comet_attention_fwd (32x32)");
  return COMET_OK;
}

template <typename T>
int dispatch_d(const comet_attn_args& a, hipStream_t s) {
  if (std::is_same<T, __bf16>::value && a.lq <= 16 && a.lk <= 16 && a.batch * a.heads < (1ll << 31) * 4) {
    switch (a.head_dim) {
      case 32: return launch_small<32>(a, s);
      case 48: return launch_small<48>(a, s);
      case 64: return launch_small<64>(a, s);
      case 96: return launch_small<96>(a, s);
      default: break;
    }
  }
  // 32x32x16 kernel for every bf16 shape past the one-wave kernel's; COMET_ATTN_FWD16=1 selects the
  // 16x16x32 kernel (A/B measurement)
  // 32x32x16 kernel where it measured faster (profiles/r03_attn_v*.txt): head dims <= 48 with
  // lq > 64 (the tracker's point -> virtual cross attention, +30 %); the 16x16x32 kernel for
  // D = 64 / 96 (DINOv2 and the camera head: equal or up to 10 % faster) and for lq <= 64 (its
  // 64-query workgroups waste nothing there). COMET_ATTN_FWD32=1 / COMET_ATTN_FWD16=1 force one.
  if (std::is_same<T, __bf16>::value && a.lq > 64 && getenv("COMET_ATTN_FWD16") == nullptr &&
      (a.head_dim <= 48 || getenv("COMET_ATTN_FWD32") != nullptr)) {
    switch (a.head_dim) {
      case 32: return launch_fwd32<32>(a, s);
      case 48: return launch_fwd32<48>(a, s);
      case 64: return launch_fwd32<64>(a, s);
      case 96: return launch_fwd32<96>(a, s);
      default: break;
    }
  }
  if (std::is_same<T, __bf16>::value) {
    switch (a.head_dim) {
      case 32: return launch_fwd_bf16<32>(a, s);
      case 48: return launch_fwd_bf16<48>(a, s);
      case 64: return launch_fwd_bf16<64>(a, s);
      case 96: return launch_fwd_bf16<96>(a, s);
      default: break;
    }
  }
  switch (a.head_dim) {
    case 32: return launch_fwd<T, 32>(a, s);
    case 48: return launch_fwd<T, 48>(a, s);
    case 64: return launch_fwd<T, 64>(a, s);
    case 96: return launch_fwd<T, 96>(a, s);
    default: set_error("comet_attention_fwd: head_dim must be 32, 48, 64 or 96"); return COMET_EINVAL;
  }
}

// ---- materialised backward helpers ----
template <typename T>
__global__ void probs_kernel(const float* __restrict__ S, const float* __restrict__ lse,
                             T* __restrict__ P, int64_t rows, int64_t cols, int64_t lds,
                             int64_t ldp, float scale) {
  const int64_t r = blockIdx.y * (int64_t)gridDim.z + blockIdx.z;
  if (r >= rows) return;
  const float l = lse[r];
  for (int64_t c = blockIdx.x * 256 + threadIdx.x; c < cols; c += (int64_t)gridDim.x * 256)
    P[r * ldp + c] = from_f32<T>(__expf(S[r * lds + c] * scale - l));
}

template <typename T>
__global__ void delta_kernel(const T* __restrict__ dO, const T* __restrict__ Out,
                             float* __restrict__ delta, int64_t heads, int64_t lq, int64_t d,
                             int64_t so_b, int64_t so_h, int64_t so_l, int64_t sd_b,
                             int64_t sd_h, int64_t sd_l, int64_t rows) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t bh = r / lq, qi = r % lq, b = bh / heads, h = bh % heads;
  const T* o = Out + b * so_b + h * so_h + qi * so_l;
  const T* g = dO + b * sd_b + h * sd_h + qi * sd_l;
  float acc = 0.f;
  for (int64_t i = lane; i < d; i += 64) acc += to_f32(o[i]) * to_f32(g[i]);
  acc = wave_sum(acc);
  if (lane == 0) delta[r] = acc;
}

template <typename T>
__global__ void dsoftmax_kernel(const T* __restrict__ P, const float* __restrict__ dP,
                                const float* __restrict__ delta, T* __restrict__ dS,
                                int64_t rows, int64_t cols, int64_t ld, float scale) {
  const int64_t r = blockIdx.y * (int64_t)gridDim.z + blockIdx.z;
  if (r >= rows) return;
  const float dl = delta[r];
  for (int64_t c = blockIdx.x * 256 + threadIdx.x; c < cols; c += (int64_t)gridDim.x * 256) {
    const int64_t i = r * ld + c;
    dS[i] = from_f32<T>(to_f32(P[i]) * (dP[i] - dl) * scale);
  }
}

inline dim3 row_grid(int64_t rows, int64_t cols) {
  const unsigned gx = (unsigned)(cdiv(cols, 256) < 4 ? cdiv(cols, 256) : 4);
  // rows split over y*z to stay under the 65535 limit
  int64_t gz = rows < 65535 ? rows : 65535;
  int64_t gy = cdiv(rows, gz);
  return dim3(gx, (unsigned)gy, (unsigned)gz);
}

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_attention_fwd(const comet_attn_args* args, void* stream) {
  COMET_CHECK_ARG(args != nullptr, "comet_attention_fwd: null args");
  const comet_attn_args& a = *args;
  COMET_CHECK_ARG(a.q && a.k && a.v && a.o, "comet_attention_fwd: null tensor");
  COMET_CHECK_ARG(a.batch > 0 && a.heads > 0 && a.lq >= 0 && a.lk > 0, "comet_attention_fwd: bad sizes");
  COMET_CHECK_ARG(a.batch * a.heads <= 65535 || (a.lq <= 16 && a.lk <= 16 && a.dtype == COMET_BF16),
                  "comet_attention_fwd: batch*heads > 65535");
  const int vec = a.dtype == COMET_BF16 ? 8 : 4;
  COMET_CHECK_ARG(a.batch_inner >= 0 && (a.batch_inner <= 1 || a.batch % a.batch_inner == 0),
                  "comet_attention_fwd: batch must be a multiple of batch_inner");
  const int64_t strides[] = {a.sq_b, a.sq_h, a.sq_l, a.sk_b, a.sk_h, a.sk_l,
                             a.sv_b, a.sv_h, a.sv_l, a.so_b, a.so_h, a.so_l, a.sq_i, a.sk_i, a.sv_i, a.so_i};
  for (int64_t st : strides) COMET_CHECK_ARG(st % vec == 0, "comet_attention_fwd: strides must be multiples of 16 bytes");
  COMET_CHECK_ARG(((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v | (uintptr_t)a.o) % 16 == 0,
                  "comet_attention_fwd: tensors must be 16-byte aligned");
  if (a.lq == 0) return COMET_OK;
  hipStream_t s = as_stream(stream);
  if (a.dtype == COMET_BF16) return dispatch_d<__bf16>(a, s);
  if (a.dtype == COMET_F32) return dispatch_d<float>(a, s);
  set_error("comet_attention_fwd: bad dtype");
  return COMET_EINVAL;
}

extern "C" int comet_attn_probs(int dtype_s, const void* s, const float* lse, void* p, int64_t rows,
                                int64_t cols, int64_t ld_s, int64_t ld_p, float scale, void* stream) {
  COMET_CHECK_ARG(s && lse && p, "comet_attn_probs: null pointer");
  if (rows == 0 || cols == 0) return COMET_OK;
  hipStream_t st = as_stream(stream);
  dim3 g = row_grid(rows, cols);
  if (dtype_s == COMET_F32)
    hipLaunchKernelGGL((probs_kernel<float>), g, dim3(256), 0, st, (const float*)s, lse, (float*)p, rows, cols, ld_s, ld_p, scale);
  else
    hipLaunchKernelGGL((probs_kernel<__bf16>), g, dim3(256), 0, st, (const float*)s, lse, (__bf16*)p, rows, cols, ld_s, ld_p, scale);
  COMET_CHECK_LAUNCH("comet_attn_probs");
  return COMET_OK;
}

extern "C" int comet_attn_delta(int dtype, const void* dout, const void* out, float* delta,
                                int64_t batch, int64_t heads, int64_t lq, int64_t d, int64_t so_b,
                                int64_t so_h, int64_t so_l, int64_t sdo_b, int64_t sdo_h,
                                int64_t sdo_l, void* stream) {
  COMET_CHECK_ARG(dout && out && delta, "comet_attn_delta: null pointer");
  const int64_t rows = batch * heads * lq;
  if (rows == 0) return COMET_OK;
  hipStream_t st = as_stream(stream);
  dim3 g((unsigned)cdiv(rows, 4));
  if (dtype == COMET_F32)
    hipLaunchKernelGGL((delta_kernel<float>), g, dim3(256), 0, st, (const float*)dout, (const float*)out, delta, heads, lq, d, so_b, so_h, so_l, sdo_b, sdo_h, sdo_l, rows);
  else
    hipLaunchKernelGGL((delta_kernel<__bf16>), g, dim3(256), 0, st, (const __bf16*)dout, (const __bf16*)out, delta, heads, lq, d, so_b, so_h, so_l, sdo_b, sdo_h, sdo_l, rows);
  COMET_CHECK_LAUNCH("comet_attn_delta");
  return COMET_OK;
}

extern "C" int comet_attn_dsoftmax(int dtype_p, const void* p, const void* dp, const float* delta,
                                   void* ds, int64_t rows, int64_t cols, int64_t ld, float scale,
                                   void* stream) {
  COMET_CHECK_ARG(p && dp && delta && ds, "comet_attn_dsoftmax: null pointer");
  if (rows == 0 || cols == 0) return COMET_OK;
  hipStream_t st = as_stream(stream);
  dim3 g = row_grid(rows, cols);
  if (dtype_p == COMET_F32)
    hipLaunchKernelGGL((dsoftmax_kernel<float>), g, dim3(256), 0, st, (const float*)p, (const float*)dp, delta, (float*)ds, rows, cols, ld, scale);
  else
    hipLaunchKernelGGL((dsoftmax_kernel<__bf16>), g, dim3(256), 0, st, (const __bf16*)p, (const float*)dp, delta, (__bf16*)ds, rows, cols, ld, scale);
  COMET_CHECK_LAUNCH("comet_attn_dsoftmax");
  return COMET_OK;
}
