// Two-workgroups-per-CU bf16 GEMM for the forward Linear shapes of the step (comet_gemm):
//   C[M, N] = epilogue(A[M, K] · B[N, K]ᵀ),  A = activations, B = nn.Linear weight (k-contiguous).
//
// Why a second structure beside the persistent one-workgroup-per-CU kernel (gemm.hip, w4): on the
// step's shapes (M ~ 65-74 k tokens, N 384..3072, K 384..1536) a tile runs only 6-24 64-deep
// k-tiles, and w4's epilogue -- bias / GELU / residual / stores of a 256 x 256 tile -- leaves the
// CU's matrix pipe idle: measured ~10-14 us of fixed cost per tile against 1.5 us per k-tile
// (tools/gpu/kscan.sh: t(K) = rounds x (a + K/64 x 1.51 us), a = 10-14 us), 30-50 % of the GEMM.
// Here two independent 4-wave workgroups share each CU (one wave of each per SIMD, <= 256 VGPRs,
// 80 KiB of LDS each), so one workgroup's epilogue (VALU + stores + residual latency) runs while
// the other's MFMAs keep the pipe busy, and the hardware dispatcher desynchronises the CUs' store
// bursts. Per workgroup:
//  * tile TBM x TBN = 256 x 128, waves 2 x 2 of 128 x 64 (8 x 4 MFMA 16x16x32 accumulators);
//  * K in 32-deep stages (one MFMA k-step), a 3-stage LDS ring filled by global_load_lds
//    (16 B per lane, no register staging), stage q+2 issued after stage q's barrier: two stages of
//    load latency hidden, one raw s_barrier per stage, counted vmcnt (never 0 in the loop);
//  * image rows are 64 B (32 k); 16-B chunk c of row r lives at c ^ swz(r), swz(r) =
//    (-(r >> 2)) & 3: the 16 lanes of each ds_read_b128 lane group hit 64 distinct banks
//    (checked exhaustively for the fragment pattern); the swizzle is applied on the DMA's global
//    source address (the LDS side of global_load_lds is lane-linear) and on the ds_read address;
//  * Cᵀ = W·Xᵀ per MFMA, so a lane holds 4 consecutive output columns of one row; the epilogue
//    parks each 8-row half block of a wave in LDS and stores whole 128-B lines (16 B per lane).
// Requires: bf16 A / B with 16-B aligned k-contiguous rows, K % 32 == 0, N % 128 == 0, one batch.
#include <type_traits>

#include "common.hpp"

namespace comet {

namespace w2 {

constexpr int BK = 32, NS = 3, NT = 256, WGM = 8;

typedef __attribute__((address_space(3))) void lds_void;

struct Epi2 {
  const float* bias;    // [N] or nullptr
  const void* resid;    // [M, ldr] TC or nullptr (C = act(alpha * acc + bias) + beta * resid)
  int64_t ldr;
  float beta;
  void* aux;            // [M, ldaux] TC pre-activation copy or nullptr
  int64_t ldaux;
  float alpha;
};

__device__ __forceinline__ int swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

// logical tile -> (tile row, tile column): consecutive ids run down groups of WGM tile rows,
// column by column (an XCD's resident workgroups share A row blocks and B column blocks in L2)
__device__ __forceinline__ void tile_rc(int L, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int gsz = WGM * tiles_n, grp = L / gsz, rem = L - grp * gsz;
  const int rows = min(WGM, tiles_m - grp * WGM);
  tm = grp * WGM + rem % rows;
  tn = rem / rows;
}

template <typename TC, int ACT, bool HASR, int TBM, int TBN>
__global__ void __launch_bounds__(NT, 2)
gemm_w2_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
               TC* __restrict__ C, int64_t ldc, int M, int K, int tiles_m, int tiles_n, Epi2 epi) {
  constexpr int WR = TBM / 2, WC = TBN / 2;      // wave tile
  constexpr int MI = WR / 16, NI = WC / 16;      // accumulator fragments
  constexpr int SA = TBM * BK, STG = (TBM + TBN) * BK;  // bf16 elements: A image, whole stage
  constexpr int PA = TBM / 64, PB = TBN / 64;    // 1-KiB LDS-DMA pieces per wave and stage
  constexpr int PIECES = PA + PB;
  constexpr int CPL = 16 / (int)sizeof(TC);      // epilogue: output columns per lane per access
  constexpr int NTC = WC / (8 * CPL);            // column passes per parked row
  constexpr int PPITCH = WC;                     // parked f32 row pitch (16-B chunks XOR-swizzled)
  static_assert((WC & (WC - 1)) == 0 && NTC >= 1, "wave tile width");
  __shared__ __attribute__((aligned(1024))) __bf16 smem[NS * STG + 2 * 4 * 8 * PPITCH];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int li = lane & 15, g = lane >> 4;
  int tm, tn;
  tile_rc(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * TBM, n0 = tn * TBN;
  const int nk = K / BK;

  // ---- load stream: piece p of a stage = image rows 16p .. 16p+15 (lane -> row 16p + lane/4,
  // slot lane%4 holding source chunk slot ^ swz(row)); A pieces first, then B; rows past M clamp
  const __bf16* ldA = A + (int64_t)m0 * lda;
  const __bf16* ldB = B + (int64_t)n0 * ldb;
  int offA[PA], offB[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int r = (wid * PA + p) * 16 + (lane >> 2);
    offA[p] = (min(m0 + r, M - 1) - m0) * (int)lda + (((lane & 3) ^ swz(r)) << 3);
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int r = (wid * PB + p) * 16 + (lane >> 2);
    offB[p] = r * (int)ldb + (((lane & 3) ^ swz(r)) << 3);
  }
  auto issue = [&](int q, int st) {
    const __bf16* pa = ldA + q * BK;
    const __bf16* pb = ldB + q * BK;
    __bf16* img = smem + st * STG;
#pragma unroll
    for (int p = 0; p < PA; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(pa + offA[p]), (lds_void*)(img + (wid * PA + p) * 512), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(pb + offB[p]), (lds_void*)(img + SA + (wid * PB + p) * 512), 16, 0, 0);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fsw = (g ^ swz(li)) << 3;  // fragment chunk offset (rows are 16-aligned + li)
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  int st = 0;
  for (int q = 0; q < nk; ++q) {
    // stage q landed for this wave (stage q+1 may stay in flight), and every wave's reads of the
    // stage refilled below (read at step q-1) are done past the barrier
    if (q + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (q + 2 < nk) issue(q + 2, st == 0 ? 2 : st - 1);
    const __bf16* img = smem + st * STG;
    bf16x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(img + (wr * WR + i * 16 + li) * BK + fsw);
#pragma unroll
    for (int j = 0; j < NI; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(img + SA + (wc * WC + j * 16 + li) * BK + fsw);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    st = st == NS - 1 ? 0 : st + 1;
  }

  // ---- epilogue: per 8-row half of each 16-row block the wave parks its 8 x WC accumulators in
  // its own LDS slab (only this wave touches it: no barrier) and re-reads them row-contiguously,
  // so every store / residual load instruction covers 8 rows x 128 B
  float* park = reinterpret_cast<float*>(smem + NS * STG) + wid * 8 * PPITCH;
  auto pswz = [](int r) { return (r & 7) | ((r & 2) << 2); };
  const int rr = lane >> 3, cc = lane & 7;
  const int64_t prow0 = (int64_t)m0 + wr * WR + rr;     // + i*16 + h*8
  const int pcol0 = n0 + wc * WC + cc * CPL;            // + t*8*CPL
  const TC* R = reinterpret_cast<const TC*>(epi.resid);
  TC* X = reinterpret_cast<TC*>(epi.aux);
  float bcp[NTC][CPL];
#pragma unroll
  for (int t = 0; t < NTC; ++t)
#pragma unroll
    for (int e = 0; e < CPL; ++e) bcp[t][e] = epi.bias ? epi.bias[pcol0 + t * 8 * CPL + e] : 0.f;
  const bool interior = m0 + TBM <= M;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t row = prow0 + i * 16 + h * 8;
      const bool ok = interior || row < M;
      float rc[NTC][CPL];
      if constexpr (HASR) {
#pragma unroll
        for (int t = 0; t < NTC; ++t)
          if (ok) loadn<CPL>(R + row * epi.ldr + pcol0 + t * 8 * CPL, rc[t]);
      }
      if ((li >> 3) == h) {
#pragma unroll
        for (int j = 0; j < NI; ++j)
          *reinterpret_cast<f32x4*>(park + (li & 7) * PPITCH + (((j * 4 + g) ^ pswz(li & 7)) << 2)) = acc[i][j];
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < NTC; ++t) {
        float v[CPL];
#pragma unroll
        for (int e = 0; e < CPL; e += 4) {
          const int lc = (t * 8 * CPL + cc * CPL + e) >> 2;
          const f32x4 p4 = *reinterpret_cast<const f32x4*>(park + rr * PPITCH + ((lc ^ pswz(rr)) << 2));
          v[e] = p4[0]; v[e + 1] = p4[1]; v[e + 2] = p4[2]; v[e + 3] = p4[3];
        }
        if (ok) {
          const int64_t col = pcol0 + t * 8 * CPL;
#pragma unroll
          for (int e = 0; e < CPL; ++e) v[e] = epi.alpha * v[e] + bcp[t][e];
          if (X) storen<CPL>(X + row * epi.ldaux + col, v);
#pragma unroll
          for (int e = 0; e < CPL; ++e) v[e] = apply_act(ACT, v[e]);
          if constexpr (HASR) {
#pragma unroll
            for (int e = 0; e < CPL; ++e) v[e] += epi.beta * rc[t][e];
          }
          storen<CPL>(C + row * ldc + col, v);
        }
      }
      asm volatile("" ::: "memory");
    }
}

}  // namespace w2

// Eligible: bf16 k-contiguous A / B with 16-B aligned rows, K % 32 == 0, N % 128 == 0, one batch,
// no split, per-column bias, output / residual / aux rows 16-B vectorisable, activation none /
// GELU / ReLU, enough tiles to fill the chip twice over.
bool w2_ok(const comet_gemm_args& a) {
  // measured slower than the persistent kernel on the step's shapes (its two workgroups per CU
  // stay in phase: their epilogues coincide), kept opt-in for comparison
  if (getenv("COMET_GEMM_W2") == nullptr) return false;
  if (a.dtype_ab != COMET_BF16 || a.convert_a || a.convert_b || a.layout_a != 0 || a.layout_b != 0) return false;
  if (a.batch[0] * a.batch[1] != 1 || a.k % 32 != 0 || a.k == 0 || a.split_k > 1) return false;
  if (a.bias && a.bias_mode != 1) return false;
  if (a.act != COMET_ACT_NONE && a.act != COMET_ACT_GELU && a.act != COMET_ACT_RELU) return false;
  if ((uintptr_t)a.a % 16 != 0 || (uintptr_t)a.b % 16 != 0 || a.lda % 8 != 0 || a.ldb % 8 != 0) return false;
  if (a.n % 128 != 0 || a.m < 2048 || a.m >= (1ll << 31) || a.n >= (1ll << 31)) return false;
  if (a.lda * 256 + 64 >= (1ll << 31) || a.ldb * 128 + 64 >= (1ll << 31)) return false;  // 32-bit offsets
  if (cdiv(a.m, 256) * (a.n / 128) < 1024) return false;  // < 2 rounds of 512 resident workgroups
  const int es = a.dtype_c == COMET_F32 ? 4 : 2;
  auto v16 = [&](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 16 == 0 && (ld * es) % 16 == 0); };
  return v16(a.c, a.ldc) && v16(a.resid, a.ldr) && v16(a.aux, a.ldaux);
}

template <typename TC>
int launch_w2(const comet_gemm_args& a, hipStream_t s) {
  constexpr int TBM = 256, TBN = 128;
  const int64_t tiles_m = cdiv(a.m, TBM), tiles_n = a.n / TBN;
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "comet_gemm: too many tiles");
  w2::Epi2 e{a.bias, a.resid, a.ldr, a.beta, a.aux, a.ldaux, a.alpha};
  const dim3 grid((unsigned)(tiles_m * tiles_n));
#define W2K(ACT, HR)                                                                                         \
  hipLaunchKernelGGL((w2::gemm_w2_kernel<TC, ACT, HR, TBM, TBN>), grid, dim3(w2::NT), 0, s,                  \
                     (const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, (TC*)a.c, a.ldc, (int)a.m, (int)a.k, \
                     (int)tiles_m, (int)tiles_n, e)
#define W2R(ACT) do { if (a.resid) W2K(ACT, true); else W2K(ACT, false); } while (0)
  switch (a.act) {
    case COMET_ACT_GELU: W2R(COMET_ACT_GELU); break;
    case COMET_ACT_RELU: W2R(COMET_ACT_RELU); break;
    default: W2R(COMET_ACT_NONE);
  }
#undef W2R
#undef W2K
  COMET_CHECK_LAUNCH("comet_gemm (2 workgroups per CU, 256 x 128)");
  return COMET_OK;
}

int launch_w2_any(const comet_gemm_args& a, hipStream_t s) {
  return a.dtype_c == COMET_BF16 ? launch_w2<__bf16>(a, s) : launch_w2<float>(a, s);
}

}  // namespace comet
