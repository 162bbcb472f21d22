// Fused tracker MLP block: x = resid + fc2(GELU(fc1(xn))) with the consumers' LayerNorms in the
// epilogue -- the second half of every AttnBlock / CrossAttnBlock of the update former
// (modules.py:119-154, 285-294, 334-343; blocks.py:205-348), always under no_grad.
//
// Per workgroup a block of 128 rows (8 waves, 2 x 4 wave grid). The hidden activation never leaves
// the CU: for each chunk of 128 hidden units
//   GEMM1  Hc[128 x 128] = xn[128 x C] . W1[chunk]^T     (K = C, 64-deep k-tiles)
//          + b1, GELU (erf), bf16 -> LDS
//   GEMM2  Out[128 x C] += Hc . W2[:, chunk]^T            (K = 128, two 64-deep k-tiles)
// and Out (f32 accumulators, 96 per lane for C = 384) + b2 + resid goes through the row-LN
// epilogue of comet_gemm_rowln (raw or normalised f32 residual stream, bf16 LayerNorm copies).
// At M = 65536 this removes the [M, 4C] bf16 hidden tensor (2 x 201 MB of HBM traffic per block).
//
// Operand tiles are staged global -> registers -> LDS (double-buffered, one barrier per 64-deep
// step) as 128-B rows with XOR-swizzled 16-B chunks; every step of the chunk loop (C / 64 GEMM1
// steps, 2 GEMM2 steps) prefetches the next step's tile while its MFMAs run.
// MFMA: v_mfma_f32_16x16x32_bf16 with the operands swapped (Cᵀ = W . Xᵀ): a lane holds 4
// consecutive output columns of one row, so the GELU result packs straight into a 64-bit LDS write.
//
// Measured (tools/mlp_bench.py, profiles/r02_mlp): correct, but 711 us vs 300 us for the unfused
// pair at M = 65536, C = 384 -- a 64-deep step is ~0.2 us of MFMA per SIMD while its weight tile
// arrives from L2 in ~1-2 us, so one step of register-staged prefetch leaves the kernel latency
// bound, and every 128-row block re-streams all 2.4 MB of W1 / W2 through L2 -> LDS. Opt-in only
// (COMET_FUSED_MLP=1); a competitive version needs a multi-step LDS-DMA ring.
#include "common.hpp"

namespace comet {
namespace {

namespace mlp {
constexpr int TBM = 128, HC = 128, NT = 512, BK = 64;

struct LN {
  __bf16* y16; int64_t ldy; float eps_y;
  __bf16* z16; int64_t ldz; const float* zw; const float* zb; float eps_z;
  int raw_c;
};

// element offset of (row, 16-B chunk ck) in a [rows][64] image, chunks XOR-swizzled by row
__device__ __forceinline__ int img_off(int row, int ck) { return row * BK + ((ck ^ (row & 7)) << 3); }
// [128][128] hidden tile: 16 chunks per row, low 3 chunk bits swizzled
__device__ __forceinline__ int h_off(int row, int ck) { return row * HC + ((ck ^ (row & 7)) << 3); }

template <int C>
__global__ void __launch_bounds__(NT, 1)
mlp_rowln_kernel(const __bf16* __restrict__ X, int64_t ldx, const __bf16* __restrict__ W1,
                 const float* __restrict__ b1, const __bf16* __restrict__ W2, const float* __restrict__ b2,
                 const float* __restrict__ R, int64_t ldr, float* __restrict__ Cout, int64_t ldc, int64_t M,
                 int hidden, LN ln) {
  constexpr int KT1 = C / BK;               // GEMM1 steps per chunk
  constexpr int SPC = KT1 + 2;              // steps per chunk
  constexpr int NI2 = C / 64;               // GEMM2 column fragments per wave (wave tile 64 x C/4)
  constexpr int IMG1 = 2 * TBM * BK;        // GEMM1 stage: xn tile + W1 tile
  constexpr int IMG2 = C * BK;              // GEMM2 stage: W2 tile
  constexpr int STAGE = IMG1 > IMG2 ? IMG1 : IMG2;
  constexpr int LD1 = IMG1 / 8 / NT;        // 16-B loads per thread, GEMM1 step (4)
  constexpr int LD2 = IMG2 / 8 / NT;        // GEMM2 step (6 for C = 384)
  constexpr int LDM = LD1 > LD2 ? LD1 : LD2;
  static_assert(C % 64 == 0 && IMG2 % (8 * NT) == 0, "C must be a multiple of 64 (and of 128 for the W2 loads)");
  __shared__ __attribute__((aligned(1024))) __bf16 smem[2 * STAGE + TBM * HC];
  __bf16* hbuf = smem + 2 * STAGE;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int li = lane & 15, g = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * TBM;
  const int nchunks = hidden / HC;
  static_assert(SPC % 2 == 0, "an even number of steps per chunk keeps the buffer parity per chunk");

  // ---- register-staged loads: step (c, k) of chunk c, k < KT1: GEMM1 k-tile k; k >= KT1: the
  // GEMM2 W2 tile k - KT1. Steps run chunk by chunk; step (c, k) + 1 / + 2 computed statically
  // inside the unrolled step loops, so acc1 is dead (not carried) through the GEMM2 steps.
  uint4 stg[LDM];
  // per-thread 32-bit element offsets (row tid/8 + 64j, 16-B chunk tid%8) against wave-uniform
  // bases, so the loads take scalar base + vector offset addressing
  const int trow = tid >> 3, tck = (tid & 7) * 8;
  int xo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int64_t gr = m0 + trow + 64 * j;
    gr = gr < M ? gr : M - 1;
    xo[j] = (int)(gr - m0) * (int)ldx + tck;
  }
  const int w1o = trow * C + tck, w2o = trow * hidden + tck;
  const __bf16* Xb = X + m0 * ldx;
  auto load_step = [&](int c, int k) {
    if (k < KT1) {
      const __bf16* wb = W1 + (int64_t)c * HC * C + k * BK;
#pragma unroll
      for (int j = 0; j < 2; ++j) stg[j] = *reinterpret_cast<const uint4*>(Xb + k * BK + xo[j]);
#pragma unroll
      for (int j = 0; j < LD1 - 2; ++j) stg[2 + j] = *reinterpret_cast<const uint4*>(wb + j * 64 * C + w1o);
    } else {
      const __bf16* wb = W2 + c * HC + (k - KT1) * BK;  // hidden columns c*128 + (k-KT1)*64 ..
#pragma unroll
      for (int j = 0; j < LD2; ++j) stg[j] = *reinterpret_cast<const uint4*>(wb + (int64_t)j * 64 * hidden + w2o);
    }
  };
  auto store_step = [&](int c, int k, __bf16* buf) {
    if (k < KT1) {
#pragma unroll
      for (int j = 0; j < LD1; ++j) {
        const int q = tid + j * NT;
        const int which = q >= TBM * 8;
        const int qq = q - which * TBM * 8;
        *reinterpret_cast<uint4*>(buf + which * TBM * BK + img_off(qq >> 3, qq & 7)) = stg[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < LD2; ++j) {
        const int q = tid + j * NT;
        *reinterpret_cast<uint4*>(buf + img_off(q >> 3, q & 7)) = stg[j];
      }
    }
  };
  // (c, k) + d steps
  auto nxt = [&](int c, int k, int d, int& c2, int& k2) {
    k2 = k + d;
    c2 = c;
    if (k2 >= SPC) { k2 -= SPC; ++c2; }
  };
  // end of step (c, k) whose stage buffer is `cur`: stage step +1 into the other buffer, start the
  // loads of step +2, one barrier
  auto advance = [&](int c, int k, int cur) {
    int c1, k1, c2, k2;
    nxt(c, k, 1, c1, k1);
    nxt(c, k, 2, c2, k2);
    // past the last chunk the stream re-loads its last tiles into a buffer nothing reads again
    // (branch-free: the staging registers stay in VGPRs)
    c1 = c1 < nchunks ? c1 : nchunks - 1;
    c2 = c2 < nchunks ? c2 : nchunks - 1;
    store_step(c1, k1, smem + (cur ^ 1) * STAGE);
    load_step(c2, k2);
    __syncthreads();
  };

  f32x4 acc2[4][NI2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_step(0, 0);
  store_step(0, 0, smem);
  load_step(0, 1);
  __syncthreads();

  // stage buffer of step (c, k) is k & 1 (SPC is even: every chunk starts on buffer 0)
  for (int c = 0; c < nchunks; ++c) {
    f32x4 acc1[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KT1; ++k) {
      const int cur = k & 1;
      const __bf16* buf = smem + cur * STAGE;
      // GEMM1: wave tile rows wr*64 + 16i, hidden columns wc*32 + 16j
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[4], b[2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(buf + img_off(wr * 64 + i * 16 + li, 4 * ks + g));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(buf + TBM * BK + img_off(wc * 32 + j * 16 + li, 4 * ks + g));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc1[i][j], 0, 0, 0);
      }
      if (k == KT1 - 1) {
        // + b1, GELU, bf16 -> hidden tile (read by this chunk's GEMM2 steps after the barrier;
        // the previous chunk's GEMM2 reads of it ended before this chunk's first barrier)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = wc * 32 + j * 16 + 4 * g;  // within the chunk
          float bb[4];
          load4(b1 + c * HC + col, bb);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = wr * 64 + i * 16 + li;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = gelu_erf(acc1[i][j][r] + bb[r]);
            store4(hbuf + h_off(row, col >> 3) + (col & 7), v);
          }
        }
      }
      advance(c, k, cur);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cur = (KT1 + kk) & 1;
      const __bf16* buf = smem + cur * STAGE;
      // GEMM2: hidden k = kk*64 .. +63 of this chunk; output rows wr*64 + 16i, cols wc*(C/4) + 16j
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[4], b[NI2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(hbuf + h_off(wr * 64 + i * 16 + li, kk * 8 + 4 * ks + g));
#pragma unroll
        for (int j = 0; j < NI2; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(buf + img_off(wc * (C / 4) + j * 16 + li, 4 * ks + g));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NI2; ++j) acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc2[i][j], 0, 0, 0);
      }
      advance(c, KT1 + kk, cur);
    }
  }

  // ---- epilogue: v = acc2 + b2 + resid, row statistics, outputs (fragment layout: lane holds
  // row wr*64 + 16i + li, columns wc*(C/4) + 16j + 4g + r) ----
  float* st = reinterpret_cast<float*>(hbuf);  // [TBM][4] (sum, sum of squares) pairs
  const float invn = 1.f / (float)C;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int lrow = wr * 64 + i * 16 + li;
    const int64_t row = m0 + lrow;
    const bool live = row < M;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NI2; ++j) {
      const int col = wc * (C / 4) + j * 16 + 4 * g;
      float bb[4], rr[4] = {0.f, 0.f, 0.f, 0.f};
      load4(b2 + col, bb);
      if (live) load4(R + row * ldr + col, rr);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc2[i][j][r] + bb[r] + rr[r];
        acc2[i][j][r] = v[r];
        s1 += v[r];
        s2 = fmaf(v[r], v[r], s2);
      }
      if (ln.raw_c && live) store4(Cout + row * ldc + col, v);
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (g == 0) *reinterpret_cast<float2*>(st + 2 * (lrow * 4 + wc)) = float2{s1, s2};
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int lrow = wr * 64 + i * 16 + li;
    const int64_t row = m0 + lrow;
    if (row >= M) continue;
    float x = 0.f, q = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float2 p = *reinterpret_cast<const float2*>(st + 2 * (lrow * 4 + w));
      x += p.x;
      q += p.y;
    }
    const float mu = x * invn, var = fmaxf(q * invn - mu * mu, 0.f);
    const float ry = rsqrtf(var + ln.eps_y), rz = rsqrtf(var + ln.eps_z);
#pragma unroll
    for (int j = 0; j < NI2; ++j) {
      const int col = wc * (C / 4) + j * 16 + 4 * g;
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = (acc2[i][j][r] - mu) * ry;
      if (!ln.raw_c) store4(Cout + row * ldc + col, y);
      if (ln.y16 != nullptr) store4(ln.y16 + row * ln.ldy + col, y);
      if (ln.z16 != nullptr) {
        float zw[4], zb[4], z[4];
        load4(ln.zw + col, zw);
        load4(ln.zb + col, zb);
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = (acc2[i][j][r] - mu) * rz * zw[r] + zb[r];
        store4(ln.z16 + row * ln.ldz + col, z);
      }
    }
  }
}
}  // namespace mlp

}  // namespace
}  // namespace comet

using namespace comet;

extern "C" int comet_mlp_rowln_ok(int64_t m, int c_dim, int hidden) {
  return (c_dim == 384 || c_dim == 256) && hidden % mlp::HC == 0 && hidden > 0 && m > 0 && m < (1ll << 31) ? 1 : 0;
}

extern "C" int comet_mlp_rowln(const comet_mlp_args* a, const comet_rowln_args* ln, void* stream) {
  COMET_CHECK_ARG(a != nullptr && ln != nullptr, "comet_mlp_rowln: null args");
  COMET_CHECK_ARG(a->x && a->w1 && a->b1 && a->w2 && a->b2 && a->resid && a->c, "comet_mlp_rowln: null operand");
  COMET_CHECK_ARG(comet_mlp_rowln_ok(a->m, a->c_dim, a->hidden), "comet_mlp_rowln: C must be 256 or 384, hidden a multiple of 128");
  auto a16 = [](const void* p, int64_t ld) { return (uintptr_t)p % 16 == 0 && ld % 8 == 0; };
  auto a8 = [](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 8 == 0 && ld % 4 == 0); };
  COMET_CHECK_ARG(a16(a->x, a->ldx) && a16(a->w1, 8) && a16(a->w2, 8) && a16(a->resid, a->ldr) && a16(a->c, a->ldc) &&
                      a8(ln->y16, ln->ldy) && a8(ln->z16, ln->ldz) && (ln->z16 == nullptr || (ln->zw && ln->zb)),
                  "comet_mlp_rowln: operands must be 16-B aligned with row strides % 8 == 0");
  if (a->m == 0) return COMET_OK;
  mlp::LN l{reinterpret_cast<__bf16*>(ln->y16), ln->ldy, ln->eps_y, reinterpret_cast<__bf16*>(ln->z16), ln->ldz,
            ln->zw, ln->zb, ln->eps_z, ln->raw_c};
  const dim3 grid((unsigned)cdiv(a->m, mlp::TBM));
  hipStream_t s = as_stream(stream);
#define MLPK(CC)                                                                                                   \
  hipLaunchKernelGGL((mlp::mlp_rowln_kernel<CC>), grid, dim3(mlp::NT), 0, s, (const __bf16*)a->x, a->ldx,         \
                     (const __bf16*)a->w1, a->b1, (const __bf16*)a->w2, a->b2, a->resid, a->ldr, a->c, a->ldc, a->m, \
                     a->hidden, l)
  if (a->c_dim == 384) MLPK(384);
  else MLPK(256);
#undef MLPK
  COMET_CHECK_LAUNCH("comet_mlp_rowln");
  return COMET_OK;
}
