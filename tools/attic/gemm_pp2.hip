// Persistent bf16 GEMM whose epilogue overlaps the next tile's MFMAs (comet_gemm, plan kind 5).
//
// The forward Linear shapes of the path (k-contiguous bf16 X [M, K] and W [N, K], K % 64 == 0,
// K >= 256, per-column bias, optional GELU / ReLU, bf16 output, or f32 output + f32 residual):
// modules.py:119-154 (Mlp fc1 / fc2), 248-344 (MHA in_proj / out_proj), blocks.py:205-348 (the
// tracker's update former), camera_predictor10.py:601-687 (DINOv2 blocks, the head's blocks).
//
// What the round-3 persistent kernel (gemm.hip, w4::gemm_w4_kernel) loses: each 256 x 256 tile runs
// its k-loop, then the same 8 waves run the epilogue while the matrix pipes idle (5.3k cycles per
// tile for bf16 outputs, ~16-21k with GELU, 31k for f32 outputs with a residual, against ~18-37k
// of k-loop at K = 384-768; DESIGN.md section 7 stamps). Here every wave owns TWO accumulator sets
// of a 64 x 64 wave tile (2 x 64 registers) and alternates them tile by tile: while tile t
// accumulates into one set, the other set -- tile t-1's finished 64 x 64 block -- is written out in
// eight slices, one per 32-deep k-step of tile t's first four k-tiles (slice = one 16-row fragment
// row x 32 columns: 8 values per lane). The slices' VALU (bias, GELU, bf16 packing) and stores issue
// beside the MFMAs of both waves of the SIMD instead of after them.
//
// Structure (per workgroup = one CU, 8 waves, 2 per SIMD):
//  * tile 256 (rows of X) x 128 (rows of W = output columns); wave grid 4 x 2, 64 x 64 per wave,
//    4 x 4 fragments of v_mfma_f32_16x16x32_bf16 computing C^T = W X^T (a lane holds 4 consecutive
//    output columns of one row);
//  * k-tiles of 64 through LDS by LDS-DMA (global_load_lds, 16-B chunks XOR-swizzled by row), A in a
//    3-slot ring one k-tile ahead of the 2-slot B ring, one barrier per k-tile, the load stream
//    running on across tile boundaries (as the w4 kernel; 128 KiB of LDS, no epilogue staging);
//  * tiles walked in XCD-banded, 8-tile-row-grouped order, one persistent workgroup per CU;
//  * slices store straight from the registers: bf16 outputs 16 B per lane (two fragments' halves
//    exchanged by v_permlane16_swap), f32 outputs 16 B per fragment row, the residual of slice s+1
//    loaded during slice s; edge tiles clamp their loads and send out-of-range stores to a sink
//    buffer, so every tile issues the same memory operations (the k-loop's counted vmcnt waits
//    stay exact) and no store sits behind a per-lane branch.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace comet {
namespace pp2 {

constexpr int BK = 64, TBM = 256, TBN = 128, NW = 8, WN = 2;
constexpr int MI = 4, NI = 4;                 // fragments per wave (64 x 64)
constexpr int ASTAGE = TBM * BK;              // bf16 elements of one A image
constexpr int BSTAGE = TBN * BK;              // bf16 elements of one B image
constexpr int PA = TBM / 8 / NW, PB = TBN / 8 / NW;  // LDS-DMA pieces (1 KiB) per wave and k-tile
constexpr int NA = 3;                         // A ring slots
constexpr int BRING = NA * ASTAGE;
constexpr int RING = NA * ASTAGE + 2 * BSTAGE;
constexpr int NMF = MI * NI, NRD = MI + NI;   // MFMAs / fragment reads per k-step
constexpr int WGM = 8;

typedef __attribute__((address_space(3))) void lds_void;
constexpr int SG_VALU = 0x002, SG_MFMA = 0x008, SG_DSR = 0x100, SG_VMR = 0x020;

__device__ __forceinline__ void tile_rc(int L, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int gsz = WGM * tiles_n, grp = L / gsz, rem = L - grp * gsz;
  const int rows = min(WGM, tiles_m - grp * WGM);
  tm = grp * WGM + rem % rows;
  tn = rem / rows;
}

__device__ __forceinline__ bf16x8 frag(const __bf16* __restrict__ img, int row, int lchunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((lchunk ^ ((row >> 1) & 7)) << 3));
}

struct Args {
  const __bf16* A; int64_t lda;
  const __bf16* B; int64_t ldb;
  void* C; int64_t ldc;
  const float* bias;
  const float* R; int64_t ldr;
  float alpha, beta;
  int M, N, K, tiles_n, ntiles;
  int c_bytes, r_bytes, b_bytes;  // buffer-descriptor ranges (M rows of C / R, N bias values; 0 = absent)
};

template <int V>
using ic = std::integral_constant<int, V>;

template <typename TC, int ACT, bool HASR>
__global__ void __launch_bounds__(NW * 64, 1) gemm_pp2_kernel(Args p) {
  __shared__ __attribute__((aligned(1024))) __bf16 smem[RING];
  constexpr bool F32 = std::is_same<TC, float>::value;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int li = lane & 15, g = lane >> 4;
  const int nk = p.K / BK;
  const int G = gridDim.x, bid = blockIdx.x;
  const int tiles_m = p.ntiles / p.tiles_n;
  const bool single = p.ntiles <= G;
  const int off = single ? xcd_remap(bid, G) : (bid & 7) * (G >> 3) + (bid >> 3);
  const int my_tiles = single ? 1 : (off < p.ntiles ? (p.ntiles - off + G - 1) / G : 0);
  if (my_tiles == 0) return;
  const int M = p.M, N = p.N;

  // ---- load stream (as w4): wave pieces wid*PA + q (A) and wid*PB + q (B) of each image
  const int prowa = wid * PA * 8 + (lane >> 3), prowb = wid * PB * 8 + (lane >> 3);
  int la_it = 0, la_kt = 0, lb_it = 0, lb_kt = 0;
  const __bf16* ldA = p.A;
  const __bf16* ldB = p.B;
  int offA[PA], offB[PB];
  auto lch = [&](int r) { return ((lane & 7) ^ ((r >> 1) & 7)) * 8; };
  auto set_tile_a = [&](int it) {
    int tm, tn;
    tile_rc(off + it * G, tiles_m, p.tiles_n, tm, tn);
    const int m0 = tm * TBM;
    ldA = p.A + (int64_t)m0 * p.lda;
#pragma unroll
    for (int q = 0; q < PA; ++q) offA[q] = (min(m0 + prowa + q * 8, M - 1) - m0) * (int)p.lda + lch(prowa + q * 8);
  };
  auto set_tile_b = [&](int it) {
    int tm, tn;
    tile_rc(off + it * G, tiles_m, p.tiles_n, tm, tn);
    const int n0 = tn * TBN;
    ldB = p.B + (int64_t)n0 * p.ldb;
#pragma unroll
    for (int q = 0; q < PB; ++q) offB[q] = (min(n0 + prowb + q * 8, N - 1) - n0) * (int)p.ldb + lch(prowb + q * 8);
  };
  auto issue_a = [&](int slot) {
    const __bf16* pa = ldA + la_kt * BK;
#pragma unroll
    for (int q = 0; q < PA; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(pa + offA[q]), (lds_void*)(smem + slot * ASTAGE + (wid * PA + q) * 512), 16, 0, 0);
  };
  auto issue_b = [&](int slot) {
    const __bf16* pb = ldB + lb_kt * BK;
#pragma unroll
    for (int q = 0; q < PB; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(pb + offB[q]), (lds_void*)(smem + BRING + slot * BSTAGE + (wid * PB + q) * 512), 16, 0, 0);
  };
  // past the last k-tile a stream keeps re-loading it into a slot nothing reads again
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

  bf16x8 a0[MI], b0[NI], a1[MI], b1[NI];
  auto read_frags = [&](int aslot, int bslot, int s, bf16x8 (&af)[MI], bf16x8 (&bf)[NI]) {
    const __bf16* aimg = smem + aslot * ASTAGE;
    const __bf16* bimg = smem + BRING + bslot * BSTAGE;
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = frag(aimg, wr * 64 + i * 16 + li, 4 * s + g);
#pragma unroll
    for (int j = 0; j < NI; ++j) bf[j] = frag(bimg, wc * 64 + j * 16 + li, 4 * s + g);
  };

  f32x4 acc0[MI][NI], acc1[MI][NI];
  f32x4 binit[NI];                            // the next tile's bias (this lane's 4 columns per fragment)
  f32x4 rinit[HASR ? MI : 1][HASR ? NI : 1];  // ... and residual (f32 outputs with a residual)
  // MFMAs of one k-step into `acc`; FIRST: the tile's first k-step accumulates onto the bias (+ beta
  // * residual), so the epilogue has no bias / residual work left
  auto mfmas = [&](f32x4 (&acc)[MI][NI], const bf16x8 (&af)[MI], const bf16x8 (&bf)[NI], auto first_t) {
    constexpr bool FIRST = decltype(first_t)::value;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        f32x4 c;
        if constexpr (!FIRST) c = acc[i][j];
        else if constexpr (HASR) c = p.beta * rinit[i][j] + binit[j];
        else c = binit[j];
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], c, 0, 0, 0);
      }
  };

  // ---- tile state and the epilogue. Every epilogue access goes through a buffer descriptor
  // (uniform 128-bit base + a 32-bit per-lane offset, hardware range check): loads beyond the
  // buffer return 0 (edge rows of the residual; a missing bias: zero records) and stores beyond it
  // are dropped -- edge rows by the range itself, edge columns by an out-of-range offset -- so edge
  // tiles run the same branch-free instruction stream as interior ones.
  constexpr int ES = F32 ? 4 : 2;
  const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, p.c_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc((void*)p.R, (short)0, p.r_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.bias, (short)0, p.b_bytes, 0x00020000);
  const int ccol = F32 ? 4 * g : 16 * (g & 1) + 8 * (g >> 1);  // lane's first column in a fragment (pair)
  const int voff_c = (li * (int)p.ldc + ccol) * ES;            // lane's byte offset in the output tile
  constexpr int DROP = 0x7fffffff;                              // beyond every buffer: dropped store
  int e_cbase = 0;                                              // tile being written out: element offset
  int e_vc[4];                                                  // per store of a slice: voff_c or DROP
  // initial accumulators of tile it: its bias (+ residual) into binit (+ rinit), NL buffer loads,
  // consumed by the tile's first MFMAs
  auto load_init = [&](int it) {
    int tm, tn;
    tile_rc(off + it * G, tiles_m, p.tiles_n, tm, tn);
    const int row0 = tm * TBM + wr * 64, col0 = tn * TBN + wc * 64;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      binit[j] = __builtin_amdgcn_raw_buffer_load_b128(rB, 16 * g, __builtin_amdgcn_readfirstlane((col0 + 16 * j) * 4), 0);
    if constexpr (HASR) {
      const int vr = (li * (int)p.ldr + 4 * g) * 4;
      const int rb = __builtin_amdgcn_readfirstlane(row0 * (int)p.ldr + col0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          rinit[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rR, vr, (rb + i * 16 * (int)p.ldr + 16 * j) * 4, 0);
    }
  };
  constexpr int NL = HASR ? NI + MI * NI : NI;  // VMEM operations of load_init
  // the tile whose accumulators move to the write-out set
  auto begin_tile = [&](int it) {
    int tm, tn;
    tile_rc(off + it * G, tiles_m, p.tiles_n, tm, tn);
    const int row0 = tm * TBM + wr * 64, col0 = tn * TBN + wc * 64;
    e_cbase = __builtin_amdgcn_readfirstlane(row0 * (int)p.ldc + col0);
    // edge columns: a lane's bf16 store covers 8 columns, an f32 store 4 (rows beyond M fall past
    // the end of the buffer by themselves)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = F32 ? col0 + 16 * q + ccol : col0 + 32 * q + ccol;
      e_vc[q] = c + (F32 ? 4 : 8) <= N ? voff_c : DROP;
    }
  };
  // slice s of the write-out set: fragment row i = s & 3, column pair cp = s >> 2 (fragments
  // (i, 2cp), (i, 2cp + 1)); the activation, then the stores
  auto slice = [&](f32x4 (&acc)[MI][NI], auto s_t) {
    constexpr int s = decltype(s_t)::value;
    constexpr int i = s & 3, cp = s >> 2;
    float v[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[u][e] = acc[i][2 * cp + u][e];
      apply_act_n<4>(ACT, v[u]);
    }
    const int so = e_cbase + i * 16 * (int)p.ldc + 32 * cp;
    if constexpr (F32) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(f32x4{v[u][0], v[u][1], v[u][2], v[u][3]}, rC, e_vc[2 * cp + u],
                                               (so + 16 * u) * ES, 0);
    } else {
      // fragments 2cp, 2cp+1 exchange 16-lane groups 1 <-> 0 and 3 <-> 2: group g then holds the 8
      // contiguous columns 16 (g & 1) + 8 (g >> 1) of the pair
      const unsigned p00 = pack_bf16x2(v[0][0], v[0][1]), p01 = pack_bf16x2(v[0][2], v[0][3]);
      const unsigned p10 = pack_bf16x2(v[1][0], v[1][1]), p11 = pack_bf16x2(v[1][2], v[1][3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(p00, p10, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(p01, p11, false, false);
      typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{s0[0], s1[0], s0[1], s1[1]}, rC, e_vc[cp], so * ES, 0);
    }
  };
  constexpr int VS = F32 ? 2 : 1;  // VMEM operations of one slice

  // ---- prologue: the first tile's initial accumulators, then B0 A0 A1 | B1 A2 in flight, k-tile
  // 0 landed, its first-k-step fragments read
  load_init(0);
  set_tile_a(0);
  set_tile_b(0);
  issue_b(0);
  advance_b();
  issue_a(0);
  advance_a();
  issue_a(1);
  advance_a();
  issue_b(1);
  issue_a(2);
  advance_b();
  advance_a();
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PA + PB) : "memory");
  asm volatile("s_barrier" ::: "memory");
  read_frags(0, 0, 0, a0, b0);
  int qa = 0, qb = 0;  // A slot (mod 3) and B slot (mod 2) of the current k-tile

  // The barrier of k-tile q waits for the B pieces of k-tile q+1, issued one k-tile ago in a
  // batch (B q+1, A q+2): younger than them are that batch's PA A pieces (left in flight) and
  // whatever was issued since -- slice stores (VS each), the next tile's initial-accumulator loads
  // (NL) -- counted exactly per call site so they stay in flight across the barrier.
  auto kstep0 = [&](f32x4 (&acc)[MI][NI], auto first_t) {
    constexpr bool FIRST = decltype(first_t)::value;
    read_frags(qa, qb, 1, a1, b1);
    mfmas(acc, a0, b0, first_t);
    if constexpr (FIRST && HASR) {
      // each MFMA's initial accumulator (beta * residual + bias: 4 VALU) right before it, so the 16
      // are not all materialised up front
#pragma unroll
      for (int t = 0; t < NRD; ++t) {
        __builtin_amdgcn_sched_group_barrier(SG_VALU, 4, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DSR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_VALU, 4, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF / NRD - 1, 0);
      }
    } else {
#pragma unroll
      for (int t = 0; t < NRD; ++t) {
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DSR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF / NRD - 1, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  auto kbarrier = [&](auto n_t) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(decltype(n_t)::value > 63 ? 63 : decltype(n_t)::value) : "memory");
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto kstep1 = [&](f32x4 (&acc)[MI][NI]) {
    const int qa1 = qa + 1 == NA ? 0 : qa + 1;
    issue_b(qb);
    issue_a(qa);
    read_frags(qa1, qb ^ 1, 0, a0, b0);
    mfmas(acc, a1, b1, std::false_type{});
#pragma unroll
    for (int t = 0; t < NRD; ++t) {
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      if (t < PA + PB) __builtin_amdgcn_sched_group_barrier(SG_VMR, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DSR, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, NMF / NRD - 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    qa = qa1;
    qb ^= 1;
    advance_b();
    advance_a();
  };

  // One tile into `acc` (K >= 320: five or more k-tiles). PREV: the previous tile (`prv`,
  // begin_tile state) is written out in slices 2kt, 2kt+1 during k-tiles kt = 0..3. next: the last
  // k-tile loads tile `nit`'s initial accumulators before its barrier, so those loads are older than
  // the batch the next tile's first MFMAs wait behind (their registers are free by then: the
  // write-out set finished at k-tile 3).
  auto tile = [&](f32x4 (&acc)[MI][NI], f32x4 (&prv)[MI][NI], auto prev_t, bool next, int nit) {
    constexpr bool PREV = decltype(prev_t)::value;
    auto kt_pre = [&](auto kt_t) {
      constexpr int kt = decltype(kt_t)::value;
      kstep0(acc, std::integral_constant<bool, kt == 0>{});
      if constexpr (PREV) {
        slice(prv, ic<2 * kt>{});
        asm volatile("" ::: "memory");
        kbarrier(ic<PA + (kt > 0 ? 2 * VS : VS)>{});
      } else {
        kbarrier(ic<PA>{});
      }
      kstep1(acc);
      if constexpr (PREV) slice(prv, ic<2 * kt + 1>{});
      asm volatile("" ::: "memory");
    };
    kt_pre(ic<0>{});
    kt_pre(ic<1>{});
    kt_pre(ic<2>{});
    kt_pre(ic<3>{});
    // k-tiles 4 .. nk-2 (k-tile 4 still has slice 7's stores younger than the batch it waits for)
    if (nk > 5) {
      kstep0(acc, std::false_type{});
      if constexpr (PREV) kbarrier(ic<PA + VS>{});
      else kbarrier(ic<PA>{});
      kstep1(acc);
      for (int kt = 5; kt < nk - 1; ++kt) {
        kstep0(acc, std::false_type{});
        kbarrier(ic<PA>{});
        kstep1(acc);
      }
    }
    // the last k-tile, nk - 1 >= 4
    kstep0(acc, std::false_type{});
    const bool s7 = PREV && nk == 5;
    if (next) {
      load_init(nit);
      asm volatile("" ::: "memory");
      if (s7) kbarrier(ic<PA + VS + NL>{});
      else kbarrier(ic<PA + NL>{});
    } else {
      if (s7) kbarrier(ic<PA + VS>{});
      else kbarrier(ic<PA>{});
    }
    kstep1(acc);
  };

  // tile 0 (nothing to write out yet), then tiles 1..: each accumulates into acc0 while acc1 (the
  // previous tile, moved there at its end) is written out; after the loop the last tile is written
  // out serially
  tile(acc0, acc1, std::false_type{}, my_tiles > 1, 1);
  begin_tile(0);
  for (int it = 1; it < my_tiles; ++it) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc1[i][j] = acc0[i][j];
    tile(acc0, acc1, std::true_type{}, it + 1 < my_tiles, it + 1);
    begin_tile(it);
  }
  auto one = [&](auto s_t) {
    slice(acc0, s_t);
    __builtin_amdgcn_sched_barrier(0);
  };
  one(ic<0>{}); one(ic<1>{}); one(ic<2>{}); one(ic<3>{});
  one(ic<4>{}); one(ic<5>{}); one(ic<6>{}); one(ic<7>{});
}

}  // namespace pp2

// ------------------------------------------------------------------------------------------------
int g_pp2_cus = 0;
static int pp2_cus() {
  if (g_pp2_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_pp2_cus = n;
    else
      g_pp2_cus = 256;
  }
  return g_pp2_cus;
}

// Eligible: bf16 k-contiguous A / B with 16-B aligned rows, K % 64 == 0 and K >= 320 (four k-tiles
// carry the previous tile's eight slices and a fifth the next tile's initial-accumulator loads), one
// batch, no split, per-column bias or none, alpha 1, no aux output; bf16 output (N % 8, 16-B
// aligned rows) without residual, or f32 output (N % 4, 16-B aligned rows) with an f32 residual and
// no activation or without a residual; act none / GELU / ReLU; M large enough to fill the chip.
// COMET_GEMM_NO_PP2=1: the w4 kernel instead (measurement A/B).
bool pp2_ok(const comet_gemm_args& a) {
  if (getenv("COMET_GEMM_NO_PP2") != nullptr) return false;
  if (a.dtype_ab != COMET_BF16 || a.convert_a || a.convert_b || a.layout_a != 0 || a.layout_b != 0) return false;
  if (a.batch[0] * a.batch[1] != 1 || a.k % 64 != 0 || a.k < 320 || a.split_k > 1 || a.aux != nullptr) return false;
  // the bias (and beta * residual) are the accumulators' initial values: alpha must be 1, and an
  // activation comes before the residual in comet_gemm, so a residual goes with act none only
  if (a.alpha != 1.0f || (a.resid != nullptr && a.act != COMET_ACT_NONE)) return false;
  // f32 outputs with a residual: the 64 residual registers of the initial accumulators spill at
  // 256 VGPRs (hipcc 7.2); they stay on the w4 kernel unless COMET_PP2_RESID=1 (measurement)
  if (a.resid != nullptr && getenv("COMET_PP2_RESID") == nullptr) return false;
  if (a.bias && a.bias_mode != 1) return false;
  if (a.act != COMET_ACT_NONE && a.act != COMET_ACT_GELU && a.act != COMET_ACT_RELU) return false;
  if ((uintptr_t)a.a % 16 != 0 || (uintptr_t)a.b % 16 != 0 || a.lda % 8 != 0 || a.ldb % 8 != 0) return false;
  const int64_t minm = getenv("COMET_PP2_MINM") ? atoll(getenv("COMET_PP2_MINM")) : 16384;
  if (a.m < minm || a.n < 128 || a.m >= (1ll << 31) || a.n >= (1ll << 31)) return false;
  if (a.lda * 256 + 64 >= (1ll << 31) || a.ldb * 128 + 64 >= (1ll << 31)) return false;  // 32-bit offsets
  // epilogue buffer descriptors: 32-bit byte offsets over the output / residual, with the rows of a
  // partial last tile still below 2^31 (their offsets fall past the range and are dropped)
  const int64_t es = a.dtype_c == COMET_F32 ? 4 : 2;
  if ((a.m + 256) * a.ldc * es >= (1ll << 31) || (a.resid && (a.m + 256) * a.ldr * 4 >= (1ll << 31))) return false;
  if (a.bias && (uintptr_t)a.bias % 16 != 0) return false;
  if ((uintptr_t)a.c % 16 != 0) return false;
  if (a.dtype_c == COMET_BF16) {
    if (a.resid != nullptr || a.n % 8 != 0 || a.ldc % 8 != 0) return false;
  } else if (a.dtype_c == COMET_F32) {
    if (a.n % 4 != 0 || a.ldc % 4 != 0) return false;
    if (a.resid != nullptr && ((uintptr_t)a.resid % 16 != 0 || a.ldr % 4 != 0)) return false;
  } else {
    return false;
  }
  return true;
}

int launch_pp2(const comet_gemm_args& a, hipStream_t s) {
  using namespace pp2;
  int grid = pp2_cus();
  grid -= grid % 8;
  const int64_t tiles_m = cdiv(a.m, TBM), tiles_n = cdiv(a.n, TBN);
  COMET_CHECK_ARG(tiles_m * tiles_n < (1ll << 30), "comet_gemm: too many tiles");
  const int ntiles = (int)(tiles_m * tiles_n);
  if (ntiles <= grid) grid = ntiles;
  const int es = a.dtype_c == COMET_F32 ? 4 : 2;
  Args p{(const __bf16*)a.a, a.lda, (const __bf16*)a.b, a.ldb, a.c, a.ldc, a.bias,
         (const float*)a.resid, a.ldr, a.alpha, a.beta, (int)a.m, (int)a.n, (int)a.k, (int)tiles_n, ntiles,
         (int)(a.m * a.ldc * es), a.resid ? (int)(a.m * a.ldr * 4) : 0, a.bias ? (int)(a.n * 4) : 0};
#define PP2K(TC, ACT, HR) hipLaunchKernelGGL((gemm_pp2_kernel<TC, ACT, HR>), dim3((unsigned)grid), dim3(NW * 64), 0, s, p)
  if (a.dtype_c == COMET_BF16) {
    if (a.act == COMET_ACT_GELU) PP2K(__bf16, COMET_ACT_GELU, false);
    else if (a.act == COMET_ACT_RELU) PP2K(__bf16, COMET_ACT_RELU, false);
    else PP2K(__bf16, COMET_ACT_NONE, false);
  } else if (a.resid != nullptr) {
    PP2K(float, COMET_ACT_NONE, true);
  } else {
    if (a.act == COMET_ACT_GELU) PP2K(float, COMET_ACT_GELU, false);
    else if (a.act == COMET_ACT_RELU) PP2K(float, COMET_ACT_RELU, false);
    else PP2K(float, COMET_ACT_NONE, false);
  }
#undef PP2K
  COMET_CHECK_LAUNCH("comet_gemm (persistent 256 x 128, overlapped epilogue)");
  return COMET_OK;
}

}  // namespace comet
