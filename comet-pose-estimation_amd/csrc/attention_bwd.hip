// Fused multi-head attention backward (flash style, bf16) -- comet_attention_bwd.
//
// Replaces the autograd backward of nn.MultiheadAttention's softmax(q kᵀ·scale)·v
//  for the camera head's self / cross-frame / T_P / trunk attention
// (camera_predictor10.py:329-348, 365-382, 663-683): nothing of size Lq x Lk reaches HBM.
//
//   P = exp(S - lse),  S = scale·Q Kᵀ        (lse from the forward)
//   dV = Pᵀ dO,  dP = dO Vᵀ,  dS = P ∘ (dP - Δ),  Δ_q = Σ_d dO·O
//   dQ = scale·dS K,  dK = scale·dSᵀ Q
//
// Two kernels, no atomics:
//  * dkdv: one workgroup per 64 keys (4 waves x 16 keys, K/V fragments in registers), walks all
//    query tiles; S and dP are computed with the query on the MFMA row so P / dS land in exactly
//    the register layout of an A operand for dV += Pᵀ·dO and dK += dSᵀ·Q, whose B operands
//    (dO, Q columns) come from the LDS tile by ds_read_b64_tr_b16.
//  * dq: one workgroup per 64 queries, structured like the forward (Sᵀ = K·Qᵀ with the query on
//    the lane), adds dPᵀ = V·dOᵀ and accumulates dQᵀ += Kᵀ·dSᵀ with Kᵀ fragments read by
//    ds_read_b64_tr_b16.
// The k index of the P/dS operands is permuted (32u + 4g + j, 32u + 16 + 4g + j) identically
// on both MFMA operands, as in the forward's P·V.
#include <cstdlib>

#include "common.hpp"

namespace comet {
namespace {

constexpr float LOG2E_B = 1.4426950408889634f;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4b;

template <int D> struct BCfg {
  static constexpr int DA = ((D + 31) / 32) * 32;  // k-dim of Q·Kᵀ (x32, zero padded)
  static constexpr int KP = DA + 8;                 // LDS row pitch (bf16 elements)
  static constexpr int NQC = DA / 32;               // 32-deep MFMA steps over d
  static constexpr int DT = D / 16;                 // 16-wide output tiles over d
  static constexpr int NVROW = D / 8;               // 16-B vectors per row
  static constexpr int NVT = (64 * NVROW + 255) / 256;
};

__device__ __forceinline__ bf16x8 frag_rows(const __bf16* base, int row, int col) {
  return *reinterpret_cast<const bf16x8*>(base + row + col);
}

// 4 consecutive d of rows r0+{0..3} (lane's column) for both k halves: the B / A operand with the
// permuted k order (rows 32u + 4g + qq and 32u + 16 + 4g + qq of a [64][KP] tile)
template <int KP>
__device__ __forceinline__ bf16x8 frag_tr(const __bf16* tile, int u, int g, int qq, int pp, int col0) {
  const __bf16* a0 = tile + (32 * u + 4 * g + qq) * KP + col0 + 4 * pp;
  const __bf16* a1 = tile + (32 * u + 16 + 4 * g + qq) * KP + col0 + 4 * pp;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4b*)(a0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4b*)(a1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ bf16x8 pack_operand(const f32x4& lo, const f32x4& hi) {
  const bf16x4 p0 = __builtin_convertvector(lo, bf16x4);
  const bf16x4 p1 = __builtin_convertvector(hi, bf16x4);
  return __builtin_shufflevector(p0, p1, 0, 1, 2, 3, 4, 5, 6, 7);
}

struct BwdPtrs {
  const __bf16* q; int64_t sq_b, sq_h, sq_l;
  const __bf16* k; int64_t sk_b, sk_h, sk_l;
  const __bf16* v; int64_t sv_b, sv_h, sv_l;
  const __bf16* dout; int64_t sd_b, sd_h, sd_l;
  __bf16* dq; int64_t sdq_b, sdq_h, sdq_l;
  __bf16* dk; int64_t sdk_b, sdk_h, sdk_l;
  __bf16* dv; int64_t sdv_b, sdv_h, sdv_l;
  const float* lse; const float* delta;
  int heads, lq, lk; float scale;
};

// Load one 16-row x D register fragment set (row = lane & 15, d = 32c + 8g + j) from global.
template <int D>
__device__ __forceinline__ void load_frags(const __bf16* base, int64_t sl, int row, bool ok, int g,
                                           bf16x8 (&f)[BCfg<D>::NQC]) {
#pragma unroll
  for (int c = 0; c < BCfg<D>::NQC; ++c) {
    const int d0 = 32 * c + 8 * g;
    f[c] = (ok && d0 < D) ? *reinterpret_cast<const bf16x8*>(base + (int64_t)row * sl + d0) : bf16x8{};
  }
}

// ---------------------------------------------------------------- dK, dV  /  dQ
// G row groups per wave (every LDS fragment feeds G MFMAs; G = 1 is dispatched: at G = 2 the
// D = 96 instances fall to 1-2 waves per SIMD), the 64-row tile processed in two 32-row halves
// to bound the live S / dP registers, lse / Δ read as float4, and
// P = exp2(fma(s, scale·log2e, -lse·log2e)) on the bare v_exp_f32.
template <int D, int G>
__global__ void __launch_bounds__(256)
attn_bwd_dkdv2_kernel(BwdPtrs p) {
  typedef BCfg<D> C;
  constexpr int KP = C::KP, NQC = C::NQC, DT = C::DT, NVROW = C::NVROW, NVT = C::NVT;
  __shared__ __attribute__((aligned(16))) __bf16 Qs[64 * KP];
  __shared__ __attribute__((aligned(16))) __bf16 Gs[64 * KP];  // dO tile
  __shared__ __attribute__((aligned(16))) float lse_s[64];
  __shared__ __attribute__((aligned(16))) float dl_s[64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4, qq = li >> 2, pp = li & 3;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by, b = bh / p.heads, h = bh % p.heads;
  const __bf16* Q = p.q + b * p.sq_b + h * p.sq_h;
  const __bf16* K = p.k + b * p.sk_b + h * p.sk_h;
  const __bf16* V = p.v + b * p.sv_b + h * p.sv_h;
  const __bf16* Gd = p.dout + b * p.sd_b + h * p.sd_h;
  const float* LSE = p.lse + bh * p.lq;
  const float* DL = p.delta + bh * p.lq;
  const float sl2 = p.scale * LOG2E_B;

  if constexpr (C::DA != D) {  // pad columns of the Q / dO tiles read by the S / dP MFMAs
    for (int i = tid; i < 64 * KP; i += 256) { Qs[i] = __bf16(0.f); Gs[i] = __bf16(0.f); }
  }

  int key0[G];
  bf16x8 kf[G][NQC], vf[G][NQC];
  f32x4 dv[G][DT], dk[G][DT];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    key0[k] = bx * (64 * G) + (wid * G + k) * 16;
    load_frags<D>(K, p.sk_l, key0[k] + li, key0[k] + li < p.lk, g, kf[k]);
    load_frags<D>(V, p.sv_l, key0[k] + li, key0[k] + li < p.lk, g, vf[k]);
#pragma unroll
    for (int i = 0; i < DT; ++i) { dv[k][i] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[k][i] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  }

  uint4 qreg[NVT], greg[NVT];
  float lreg = 0.f, dreg = 0.f;
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NVROW, cv = (idx % NVROW) * 8;
      const int q = t * 64 + row;
      const bool ok = idx < 64 * NVROW && q < p.lq;
      qreg[i] = ok ? *reinterpret_cast<const uint4*>(Q + (int64_t)q * p.sq_l + cv) : uint4{0, 0, 0, 0};
      greg[i] = ok ? *reinterpret_cast<const uint4*>(Gd + (int64_t)q * p.sd_l + cv) : uint4{0, 0, 0, 0};
    }
    if (tid < 64) {
      const int q = t * 64 + tid;
      lreg = q < p.lq ? LSE[q] * LOG2E_B : INFINITY;  // invalid queries: P = 0
      dreg = q < p.lq ? DL[q] : 0.f;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NVROW) {
        const int row = idx / NVROW, cv = (idx % NVROW) * 8;
        *reinterpret_cast<uint4*>(Qs + row * KP + cv) = qreg[i];
        *reinterpret_cast<uint4*>(Gs + row * KP + cv) = greg[i];
      }
    }
    if (tid < 64) { lse_s[tid] = lreg; dl_s[tid] = dreg; }
  };

  const int ntiles = (p.lq + 63) / 64;
  gload(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (t + 1 < ntiles) gload(t + 1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      // S, dP of queries 32u + 16j + 4g + r (row) x the wave's keys (lane)
      f32x4 s[G][2], dp[G][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int st = 2 * u + j;
#pragma unroll
        for (int k = 0; k < G; ++k) { s[k][j] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[k][j] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
        for (int c = 0; c < NQC; ++c) {
          const bf16x8 qa = frag_rows(Qs, (st * 16 + li) * KP, 32 * c + 8 * g);
          const bf16x8 ga = frag_rows(Gs, (st * 16 + li) * KP, 32 * c + 8 * g);
#pragma unroll
          for (int k = 0; k < G; ++k) {
            s[k][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[k][c], s[k][j], 0, 0, 0);
            dp[k][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, vf[k][c], dp[k][j], 0, 0, 0);
          }
        }
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(lse_s + st * 16 + 4 * g);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(dl_s + st * 16 + 4 * g);
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pr = __builtin_amdgcn_exp2f(__builtin_fmaf(s[k][j][r], sl2, -l4[r]));
            s[k][j][r] = pr;                         // P
            dp[k][j][r] = pr * (dp[k][j][r] - d4[r]);  // dS (unscaled)
          }
      }
      bf16x8 pa[G], da[G];
#pragma unroll
      for (int k = 0; k < G; ++k) { pa[k] = pack_operand(s[k][0], s[k][1]); da[k] = pack_operand(dp[k][0], dp[k][1]); }
      // dV += Pᵀ dO, dK += dSᵀ Q over these 32 queries (permuted k order)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const bf16x8 gb = frag_tr<KP>(Gs, u, g, qq, pp, 16 * dt);
        const bf16x8 qb = frag_tr<KP>(Qs, u, g, qq, pp, 16 * dt);
#pragma unroll
        for (int k = 0; k < G; ++k) {
          dv[k][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[k], gb, dv[k][dt], 0, 0, 0);
          dk[k][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[k], qb, dk[k][dt], 0, 0, 0);
        }
      }
    }
  }

  __bf16* dK = p.dk + b * p.sdk_b + h * p.sdk_h;
  __bf16* dV = p.dv + b * p.sdv_b + h * p.sdv_h;
#pragma unroll
  for (int k = 0; k < G; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kr = key0[k] + 4 * g + r;
      if (kr >= p.lk) continue;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dV[(int64_t)kr * p.sdv_l + 16 * dt + li] = static_cast<__bf16>(dv[k][dt][r]);
        dK[(int64_t)kr * p.sdk_l + 16 * dt + li] = static_cast<__bf16>(dk[k][dt][r] * p.scale);
      }
    }
}

template <int D, int G>
__global__ void __launch_bounds__(256)
attn_bwd_dq2_kernel(BwdPtrs p) {
  typedef BCfg<D> C;
  constexpr int KP = C::KP, NQC = C::NQC, DT = C::DT, NVROW = C::NVROW, NVT = C::NVT;
  __shared__ __attribute__((aligned(16))) __bf16 Ks[64 * KP];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[64 * KP];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4, qq = li >> 2, pp = li & 3;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by, b = bh / p.heads, h = bh % p.heads;
  const __bf16* Q = p.q + b * p.sq_b + h * p.sq_h;
  const __bf16* K = p.k + b * p.sk_b + h * p.sk_h;
  const __bf16* V = p.v + b * p.sv_b + h * p.sv_h;
  const __bf16* Gd = p.dout + b * p.sd_b + h * p.sd_h;
  const float sl2 = p.scale * LOG2E_B;

  if constexpr (C::DA != D) {
    for (int i = tid; i < 64 * KP; i += 256) { Ks[i] = __bf16(0.f); Vs[i] = __bf16(0.f); }
  }

  int qrow[G];
  bf16x8 qf[G][NQC], gf[G][NQC];
  float lse2[G], dl[G];
  f32x4 acc[G][DT];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    qrow[k] = bx * (64 * G) + (wid * G + k) * 16 + li;
    const bool ok = qrow[k] < p.lq;
    load_frags<D>(Q, p.sq_l, qrow[k], ok, g, qf[k]);
    load_frags<D>(Gd, p.sd_l, qrow[k], ok, g, gf[k]);
    lse2[k] = ok ? p.lse[bh * p.lq + qrow[k]] * LOG2E_B : INFINITY;
    dl[k] = ok ? p.delta[bh * p.lq + qrow[k]] : 0.f;
#pragma unroll
    for (int i = 0; i < DT; ++i) acc[k][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  uint4 kreg[NVT], vreg[NVT];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NVT; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NVROW, cv = (idx % NVROW) * 8;
      const int kk = t * 64 + row;
      const bool ok = idx < 64 * NVROW && kk < p.lk;
      kreg[i] = ok ? *reinterpret_cast<const uint4*>(K + (int64_t)kk * p.sk_l + cv) : uint4{0, 0, 0, 0};
      vreg[i] = ok ? *reinterpret_cast<const uint4*>(V + (int64_t)kk * p.sv_l + cv) : uint4{0, 0, 0, 0};
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

  const int ntiles = (p.lk + 63) / 64;
  gload(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (t + 1 < ntiles) gload(t + 1);
    const bool ragged = t * 64 + 64 > p.lk;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x4 dp[G][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int st = 2 * u + j;
        f32x4 s[G];
#pragma unroll
        for (int k = 0; k < G; ++k) { s[k] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[k][j] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
        for (int c = 0; c < NQC; ++c) {
          const bf16x8 ka = frag_rows(Ks, (st * 16 + li) * KP, 32 * c + 8 * g);
          const bf16x8 va = frag_rows(Vs, (st * 16 + li) * KP, 32 * c + 8 * g);
#pragma unroll
          for (int k = 0; k < G; ++k) {
            s[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[k][c], s[k], 0, 0, 0);
            dp[k][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, gf[k][c], dp[k][j], 0, 0, 0);
          }
        }
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float pr = __builtin_amdgcn_exp2f(__builtin_fmaf(s[k][r], sl2, -lse2[k]));
            if (ragged && t * 64 + st * 16 + 4 * g + r >= p.lk) pr = 0.f;
            dp[k][j][r] = pr * (dp[k][j][r] - dl[k]);  // dS (unscaled)
          }
      }
      // dQᵀ += Kᵀ dSᵀ over these 32 keys (permuted k order)
      bf16x8 db[G];
#pragma unroll
      for (int k = 0; k < G; ++k) db[k] = pack_operand(dp[k][0], dp[k][1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const bf16x8 ka = frag_tr<KP>(Ks, u, g, qq, pp, 16 * dt);
#pragma unroll
        for (int k = 0; k < G; ++k) acc[k][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, db[k], acc[k][dt], 0, 0, 0);
      }
    }
  }

#pragma unroll
  for (int k = 0; k < G; ++k) {
    if (qrow[k] >= p.lq) continue;
    __bf16* dQ = p.dq + b * p.sdq_b + h * p.sdq_h + (int64_t)qrow[k] * p.sdq_l;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      *reinterpret_cast<bf16x4*>(dQ + 16 * dt + 4 * g) = __builtin_convertvector(acc[k][dt] * p.scale, bf16x4);
  }
}

// ---------------------------------------------------------------- 32x32x16 MFMA kernels
// Same two-kernel split, on v_mfma_f32_32x32x16_bf16 (half the vector-issue cost per FLOP of the
// 16x16x32 form, twice the operand reuse per LDS fragment), one barrier per tile (the next tile's
// global loads are issued before this tile's MFMAs and written to the other LDS buffer after them):
//  * dkdv32: one wave = 32 keys (K / V fragments in registers), workgroup = 128 keys; per 32-query
//    block S = Q·Kᵀ and dP = dO·Vᵀ with the key on the lane (queries in the registers), then
//    dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS with P / dS straight from the accumulators as B operands and
//    the dOᵀ / Qᵀ A fragments read transposed (ds_read_b64_tr_b16) in the accumulator's permuted
//    query order;
//  * dq32: one wave = 32 queries (Q / dO fragments in registers, lse / Δ lane-local), per 32-key
//    block Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ, dQᵀ += Kᵀ·dSᵀ.
// Outputs leave as 16-B rows: lane pairs (l, l + 32) swap halves with v_permlane32_swap.
typedef __attribute__((ext_vector_type(16))) float f32x16b;

template <int D> struct B32 {
  static constexpr int NKS = D / 16;              // k-steps over d of S / dP
  static constexpr int DB = (D + 31) / 32;        // 32-row output blocks over d
  static constexpr int TP = D + 8;                // LDS row pitch of the Q / dO (K / V) tiles
  static constexpr int TPV = DB * 32 + 8;         // pitch of tiles read transposed (pad cols zero)
  static constexpr int NCH = D / 8;               // 16-B chunks per row
  static constexpr int NST = (64 * NCH + 255) / 256;
};

// 16 consecutive-d values of a [d-block][lane] accumulator row set -> one 16-B row store per lane
// pair: lane (r, h) holds d = 32 db + 8u + 4h + (0..3) of its row r
template <int D>
__device__ __forceinline__ void store_rows32(__bf16* row_ptr, bool ok, const f32x16b (&acc)[B32<D>::DB], float mul, int h) {
#pragma unroll
  for (int db = 0; db < B32<D>::DB; ++db)
#pragma unroll
    for (int u = 0; u < 4; u += 2) {
      if (32 * db + 8 * u >= D) continue;
      uint2 pk[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x4 w = f32x4{acc[db][4 * (u + e)], acc[db][4 * (u + e) + 1], acc[db][4 * (u + e) + 2],
                              acc[db][4 * (u + e) + 3]} * mul;
        pk[e] = __builtin_bit_cast(uint2, __builtin_convertvector(w, bf16x4));
      }
      const auto sx = __builtin_amdgcn_permlane32_swap(pk[0].x, pk[1].x, false, false);
      const auto sy = __builtin_amdgcn_permlane32_swap(pk[0].y, pk[1].y, false, false);
      if (ok) *reinterpret_cast<uint4*>(row_ptr + 32 * db + 8 * u + 8 * h) = uint4{sx[0], sy[0], sx[1], sy[1]};
    }
}

__device__ __forceinline__ bf16x8 pack16(const f32x16b& x, int s) {
  const f32x4 lo = {x[8 * s], x[8 * s + 1], x[8 * s + 2], x[8 * s + 3]};
  const f32x4 hi = {x[8 * s + 4], x[8 * s + 5], x[8 * s + 6], x[8 * s + 7]};
  return __builtin_shufflevector(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4), 0, 1, 2, 3,
                                 4, 5, 6, 7);
}

// A fragment of k-step s (16 rows: r0 + 16s + 8(j>>2) + 4h + (j&3)) x 32 columns (c0 + lane's 16-lane
// group slice) of a row-major LDS tile, transposed (Xᵀ rows = columns of the tile)
__device__ __forceinline__ bf16x8 frag_tr32(const __bf16* tile, int pitch, int r0, int c0, int lane) {
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const __bf16* a = tile + (r0 + 4 * (tg >> 1) + tq) * pitch + c0 + 16 * (tg & 1) + 4 * tp;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4b*)(a));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4b*)(a + 8 * pitch));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int D>
__global__ void __launch_bounds__(256, 2)
attn_bwd_dkdv32_kernel(BwdPtrs p) {
  typedef B32<D> C;
  constexpr int NKS = C::NKS, DB = C::DB, TP = C::TPV, NCH = C::NCH, NST = C::NST;
  __shared__ __attribute__((aligned(16))) __bf16 Qs[2][64 * TP];
  __shared__ __attribute__((aligned(16))) __bf16 Gs[2][64 * TP];
  __shared__ __attribute__((aligned(16))) float lse_s[2][64];
  __shared__ __attribute__((aligned(16))) float dl_s[2][64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by, b = bh / p.heads, hd = bh % p.heads;
  const __bf16* Q = p.q + b * p.sq_b + hd * p.sq_h;
  const __bf16* K = p.k + b * p.sk_b + hd * p.sk_h;
  const __bf16* V = p.v + b * p.sv_b + hd * p.sv_h;
  const __bf16* Gd = p.dout + b * p.sd_b + hd * p.sd_h;
  const float* LSE = p.lse + bh * p.lq;
  const float* DL = p.delta + bh * p.lq;
  const float sl2 = p.scale * LOG2E_B;

  if constexpr (DB * 32 != D) {  // pad columns of the tiles read transposed stay zero
    constexpr int PADC = DB * 32 - D;
    for (int i = tid; i < 2 * 64 * PADC; i += 256) {
      const int buf = i / (64 * PADC), rem = i % (64 * PADC);
      Qs[buf][(rem / PADC) * TP + D + rem % PADC] = __bf16(0.f);
      Gs[buf][(rem / PADC) * TP + D + rem % PADC] = __bf16(0.f);
    }
  }

  const int key = bx * 128 + wid * 32 + r;
  const bool kok = key < p.lk;
  bf16x8 kf[NKS], vf[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    kf[s] = kok ? *reinterpret_cast<const bf16x8*>(K + (int64_t)key * p.sk_l + 16 * s + 8 * h) : bf16x8{};
    vf[s] = kok ? *reinterpret_cast<const bf16x8*>(V + (int64_t)key * p.sv_l + 16 * s + 8 * h) : bf16x8{};
  }
  f32x16b dv[DB], dk[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) { dv[i] = f32x16b{}; dk[i] = f32x16b{}; }

  uint4 qst[NST], gst[NST];
  float lreg = 0.f, dreg = 0.f;
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NCH, c = idx % NCH;
      const int q = t * 64 + row;
      const bool ok = idx < 64 * NCH && q < p.lq;
      qst[i] = ok ? *reinterpret_cast<const uint4*>(Q + (int64_t)q * p.sq_l + 8 * c) : uint4{0, 0, 0, 0};
      gst[i] = ok ? *reinterpret_cast<const uint4*>(Gd + (int64_t)q * p.sd_l + 8 * c) : uint4{0, 0, 0, 0};
    }
    if (tid < 64) {
      const int q = t * 64 + tid;
      lreg = q < p.lq ? LSE[q] * LOG2E_B : INFINITY;  // queries past lq: P = 0
      dreg = q < p.lq ? -DL[q] : 0.f;                 // -Δ: the dPᵀ accumulators start from it
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NCH) {
        const int row = idx / NCH, c = idx % NCH;
        *reinterpret_cast<uint4*>(&Qs[buf][row * TP + 8 * c]) = qst[i];
        *reinterpret_cast<uint4*>(&Gs[buf][row * TP + 8 * c]) = gst[i];
      }
    }
    if (tid < 64) { lse_s[buf][tid] = lreg; dl_s[buf][tid] = dreg; }
  };

  auto tile = [&](int buf) {
    const __bf16* qs = Qs[buf];
    const __bf16* gs = Gs[buf];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      // register j: query qb*32 + 8(j>>2) + 4h + (j&3); dPᵀ - Δ accumulates onto the -Δ of its query
      // (one v_mul per score below instead of v_sub + v_mul)
      f32x16b sacc = f32x16b{}, pacc;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&dl_s[buf][qb * 32 + 8 * u + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e) pacc[4 * u + e] = d4[e];
      }
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(qs + (qb * 32 + r) * TP + 16 * s + 8 * h);
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(gs + (qb * 32 + r) * TP + 16 * s + 8 * h);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, vf[s], pacc, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(&lse_s[buf][qb * 32 + 8 * u + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pr = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[4 * u + e], sl2, -l4[e]));
          sacc[4 * u + e] = pr;                     // P
          pacc[4 * u + e] = pr * pacc[4 * u + e];   // dS (unscaled)
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pb = pack16(sacc, s2), sb = pack16(pacc, s2);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const bf16x8 ga = frag_tr32(gs, TP, qb * 32 + 16 * s2, 32 * db, lane);
          const bf16x8 qa = frag_tr32(qs, TP, qb * 32 + 16 * s2, 32 * db, lane);
          dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, pb, dv[db], 0, 0, 0);
          dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, sb, dk[db], 0, 0, 0);
        }
      }
    }
  };

  const int ntiles = (p.lq + 63) / 64;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) gload(t + 1);
    tile(t & 1);
    if (t + 1 < ntiles) lstore((t + 1) & 1);
    __syncthreads();
  }
  __bf16* dK = p.dk + b * p.sdk_b + hd * p.sdk_h + (int64_t)key * p.sdk_l;
  __bf16* dV = p.dv + b * p.sdv_b + hd * p.sdv_h + (int64_t)key * p.sdv_l;
  store_rows32<D>(dV, kok, dv, 1.f, h);
  store_rows32<D>(dK, kok, dk, p.scale, h);
}

template <int D>
__global__ void __launch_bounds__(256, 2)
attn_bwd_dq32_kernel(BwdPtrs p) {
  typedef B32<D> C;
  constexpr int NKS = C::NKS, DB = C::DB, TP = C::TPV, NCH = C::NCH, NST = C::NST;
  __shared__ __attribute__((aligned(16))) __bf16 Ks[2][64 * TP];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[2][64 * TP];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  int bx, by;
  xcd_remap2(bx, by);
  const int64_t bh = by, b = bh / p.heads, hd = bh % p.heads;
  const __bf16* Q = p.q + b * p.sq_b + hd * p.sq_h;
  const __bf16* K = p.k + b * p.sk_b + hd * p.sk_h;
  const __bf16* V = p.v + b * p.sv_b + hd * p.sv_h;
  const __bf16* Gd = p.dout + b * p.sd_b + hd * p.sd_h;
  const float sl2 = p.scale * LOG2E_B;

  if constexpr (DB * 32 != D) {
    constexpr int PADC = DB * 32 - D;
    for (int i = tid; i < 2 * 64 * PADC; i += 256) {
      const int buf = i / (64 * PADC), rem = i % (64 * PADC);
      Ks[buf][(rem / PADC) * TP + D + rem % PADC] = __bf16(0.f);
    }
  }

  const int qrow = bx * 128 + wid * 32 + r;
  const bool qok = qrow < p.lq;
  bf16x8 qf[NKS], gf[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    qf[s] = qok ? *reinterpret_cast<const bf16x8*>(Q + (int64_t)qrow * p.sq_l + 16 * s + 8 * h) : bf16x8{};
    gf[s] = qok ? *reinterpret_cast<const bf16x8*>(Gd + (int64_t)qrow * p.sd_l + 16 * s + 8 * h) : bf16x8{};
  }
  const float lse2 = qok ? p.lse[bh * p.lq + qrow] * LOG2E_B : INFINITY;
  const float dl = qok ? p.delta[bh * p.lq + qrow] : 0.f;
  f32x16b acc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) acc[i] = f32x16b{};

  uint4 kst[NST], vst[NST];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NCH, c = idx % NCH;
      const int kk = t * 64 + row;
      const bool ok = idx < 64 * NCH && kk < p.lk;
      kst[i] = ok ? *reinterpret_cast<const uint4*>(K + (int64_t)kk * p.sk_l + 8 * c) : uint4{0, 0, 0, 0};
      vst[i] = ok ? *reinterpret_cast<const uint4*>(V + (int64_t)kk * p.sv_l + 8 * c) : uint4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NCH) {
        const int row = idx / NCH, c = idx % NCH;
        *reinterpret_cast<uint4*>(&Ks[buf][row * TP + 8 * c]) = kst[i];
        *reinterpret_cast<uint4*>(&Vs[buf][row * TP + 8 * c]) = vst[i];
      }
    }
  };

  // MASK only for the ragged last key tile (peeled: the per-score key test and select cost ~95 vector
  // instructions per tile when evaluated on every tile)
  auto tile = [&](int t, int buf, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const __bf16* ks = Ks[buf];
    const __bf16* vs = Vs[buf];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // dPᵀ - Δ accumulates onto -Δ of the lane's query: one v_mul per score below
      f32x16b sacc = f32x16b{}, pacc;
#pragma unroll
      for (int j = 0; j < 16; ++j) pacc[j] = -dl;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(ks + (kb * 32 + r) * TP + 16 * s + 8 * h);
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(vs + (kb * 32 + r) * TP + 16 * s + 8 * h);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, gf[s], pacc, 0, 0, 0);
      }
      // register j: key t*64 + kb*32 + 8(j>>2) + 4h + (j&3)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        float pr = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[j], sl2, -lse2));
        if (MASK && t * 64 + kb * 32 + 8 * (j >> 2) + 4 * h + (j & 3) >= p.lk) pr = 0.f;
        pacc[j] = pr * pacc[j];  // dS (unscaled)
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 sb = pack16(pacc, s2);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const bf16x8 ka = frag_tr32(ks, TP, kb * 32 + 16 * s2, 32 * db, lane);
          acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, sb, acc[db], 0, 0, 0);
        }
      }
    }
  };

  const int ntiles = (p.lk + 63) / 64;
  gload(0);
  lstore(0);
  __syncthreads();
  // every tile but the last is full; the last runs the masked instantiation, peeled out of the loop
  // (one instantiation inside the loop keeps its register allocation that of the unmasked body)
  for (int t = 0; t < ntiles - 1; ++t) {
    gload(t + 1);
    tile(t, t & 1, std::false_type{});
    lstore((t + 1) & 1);
    __syncthreads();
  }
  tile(ntiles - 1, (ntiles - 1) & 1, std::true_type{});
  __bf16* dQ = p.dq + b * p.sdq_b + hd * p.sdq_h + (int64_t)qrow * p.sdq_l;
  store_rows32<D>(dQ, qok, acc, p.scale, h);
}

// Δ = rowsum(dO ∘ O), one wave per 4 query rows... one lane group of 8 per row (D <= 128)
__global__ void __launch_bounds__(256)
attn_delta_bf16_kernel(const __bf16* __restrict__ dO, const __bf16* __restrict__ O, float* __restrict__ delta,
                       int heads, int lq, int D, int64_t so_b, int64_t so_h, int64_t so_l, int64_t sd_b,
                       int64_t sd_h, int64_t sd_l, int64_t rows) {
  const int64_t r = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  const int sub = threadIdx.x & 7;
  float acc = 0.f;
  if (r < rows) {
    const int64_t bh = r / lq, qi = r % lq, b = bh / heads, h = bh % heads;
    const __bf16* o = O + b * so_b + h * so_h + qi * so_l;
    const __bf16* g = dO + b * sd_b + h * sd_h + qi * sd_l;
    for (int d = sub * 8; d < D; d += 64) {
      float x[8], y[8];
      load8(o + d, x);
      load8(g + d, y);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += x[e] * y[e];
    }
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (r < rows && sub == 0) delta[r] = acc;
}

template <int D>
int launch_bwd32(const BwdPtrs& p, int64_t bh, hipStream_t s) {
  hipLaunchKernelGGL((attn_bwd_dkdv32_kernel<D>), dim3((unsigned)cdiv(p.lk, 128), (unsigned)bh), dim3(256), 0, s, p);
  COMET_CHECK_LAUNCH("comet_attention_bwd (dk, dv; 32x32)");
  hipLaunchKernelGGL((attn_bwd_dq32_kernel<D>), dim3((unsigned)cdiv(p.lq, 128), (unsigned)bh), dim3(256), 0, s, p);
  COMET_CHECK_LAUNCH("comet_attention_bwd (dq; 32x32)");
  return COMET_OK;
}

template <int D>
int launch_bwd(const BwdPtrs& p, int64_t bh, hipStream_t s) {
  // one row group per wave: at G = 2 the D = 96 kernels drop to 1-2 waves per SIMD and lose
  // more than the halved LDS traffic gains (tools/attn_bench.py)
  hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<D, 1>), dim3((unsigned)cdiv(p.lk, 64), (unsigned)bh), dim3(256), 0, s, p);
  COMET_CHECK_LAUNCH("comet_attention_bwd (dk, dv)");
  hipLaunchKernelGGL((attn_bwd_dq2_kernel<D, 1>), dim3((unsigned)cdiv(p.lq, 64), (unsigned)bh), dim3(256), 0, s, p);
  COMET_CHECK_LAUNCH("comet_attention_bwd (dq)");
  return COMET_OK;
}

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_attention_bwd(const comet_attn_bwd_args* args, void* stream) {
  COMET_CHECK_ARG(args != nullptr, "comet_attention_bwd: null args");
  const comet_attn_bwd_args& a = *args;
  COMET_CHECK_ARG(a.dtype == COMET_BF16, "comet_attention_bwd: bf16 only (f32 uses the materialised backward)");
  COMET_CHECK_ARG(a.q && a.k && a.v && a.o && a.dout && a.dq && a.dk && a.dv && a.lse && a.delta,
                  "comet_attention_bwd: null tensor");
  COMET_CHECK_ARG(a.batch > 0 && a.heads > 0 && a.lq > 0 && a.lk > 0 && a.lq < (1ll << 30) && a.lk < (1ll << 30),
                  "comet_attention_bwd: bad sizes");
  COMET_CHECK_ARG(a.batch * a.heads <= 65535, "comet_attention_bwd: batch*heads > 65535");
  const int64_t strides[] = {a.sq_b, a.sq_h, a.sq_l, a.sk_b, a.sk_h, a.sk_l, a.sv_b, a.sv_h, a.sv_l,
                             a.so_b, a.so_h, a.so_l, a.sd_b, a.sd_h, a.sd_l, a.sdq_b, a.sdq_h, a.sdq_l,
                             a.sdk_b, a.sdk_h, a.sdk_l, a.sdv_b, a.sdv_h, a.sdv_l};
  for (int64_t st : strides) COMET_CHECK_ARG(st % 8 == 0, "comet_attention_bwd: strides must be multiples of 8 elements");
  COMET_CHECK_ARG(((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v | (uintptr_t)a.o | (uintptr_t)a.dout |
                   (uintptr_t)a.dq) % 16 == 0, "comet_attention_bwd: tensors must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int64_t bh = a.batch * a.heads, rows = bh * a.lq;
  hipLaunchKernelGGL(attn_delta_bf16_kernel, dim3((unsigned)cdiv(rows, 32)), dim3(256), 0, s,
                     (const __bf16*)a.dout, (const __bf16*)a.o, a.delta, (int)a.heads, (int)a.lq, (int)a.head_dim,
                     a.so_b, a.so_h, a.so_l, a.sd_b, a.sd_h, a.sd_l, rows);
  COMET_CHECK_LAUNCH("comet_attention_bwd (delta)");
  BwdPtrs p{(const __bf16*)a.q, a.sq_b, a.sq_h, a.sq_l, (const __bf16*)a.k, a.sk_b, a.sk_h, a.sk_l,
            (const __bf16*)a.v, a.sv_b, a.sv_h, a.sv_l, (const __bf16*)a.dout, a.sd_b, a.sd_h, a.sd_l,
            (__bf16*)a.dq, a.sdq_b, a.sdq_h, a.sdq_l, (__bf16*)a.dk, a.sdk_b, a.sdk_h, a.sdk_l,
            (__bf16*)a.dv, a.sdv_b, a.sdv_h, a.sdv_l, a.lse, a.delta, (int)a.heads, (int)a.lq, (int)a.lk, a.scale};
  // 32x32x16 kernels (16-B dK / dV / dQ row stores: 16-B aligned outputs); COMET_ATTN_BWD16=1
  // selects the 16x16x32 kernels (A/B measurement)
  // (128-row workgroups: short query / key sequences -- T_P's Lq = 1, the trunk's 16 -- stay on
  // the 64-row kernels)
  const bool wide = ((uintptr_t)a.dk | (uintptr_t)a.dv) % 16 == 0 && a.lq >= 64 && a.lk >= 64 &&
                    getenv("COMET_ATTN_BWD16") == nullptr;
  if (wide) {
    switch (a.head_dim) {
      case 32: return launch_bwd32<32>(p, bh, s);
      case 48: return launch_bwd32<48>(p, bh, s);
      case 64: return launch_bwd32<64>(p, bh, s);
      case 96: return launch_bwd32<96>(p, bh, s);
      default: break;
    }
  }
  switch (a.head_dim) {
    case 32: return launch_bwd<32>(p, bh, s);
    case 48: return launch_bwd<48>(p, bh, s);
    case 64: return launch_bwd<64>(p, bh, s);
    case 96: return launch_bwd<96>(p, bh, s);
    default: set_error("comet_attention_bwd: head_dim must be 32, 48, 64 or 96"); return COMET_EINVAL;
  }
}
