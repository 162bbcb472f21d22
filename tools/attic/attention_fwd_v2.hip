// Moved out of csrc/attention.hip (round 3): opt-in LDS-DMA 3-stage attention forward,
// measured equal (D = 96) or 7 % slower (D = 64) than attn_fwd_bf16_kernel (profiles/r02_attn).
// Not compiled; kept for reference.
// bf16 forward v2 for the long-sequence head dims (D = 64: DINOv2 L 581; D = 96: head self L 577,
// cross Lq 8655 / Lk 577). Same Sᵀ = K·Qᵀ / Oᵀ = Vᵀ·Pᵀ formulation as attn_fwd_bf16_kernel; what
// the PMC pass of that kernel showed (profiles/r02_attn: 8.9 / 6.8 VALU instructions per MFMA at
// D = 64 / 96, 36-41 % of LDS cycles lost to bank conflicts, 24-31 % of wave time in barriers) is
// removed here:
//  * K / V tiles (64 keys) arrive by LDS-DMA (global_load_lds, 16 B per lane, per-lane source
//    address) into a 3-stage ring: tile t+2 is issued right after tile t's barrier, so the load
//    path costs no VALU / ds_write and one barrier per tile (was register staging + 2 barriers);
//  * LDS images are unpadded [64][D] rows with the 16-B chunks XOR-swizzled per row (chunk c of
//    row r at c ^ (r & 7) for D = 64; within groups of 4 chunks, c ^ ((r ^ r >> 1) & 2), for
//    D = 96): both the K ds_read_b128 fragments and the V ds_read_b64_tr_b16 reads are
//    bank-conflict free (checked exhaustively over every lane group);
//  * the row max runs on v_max3_f32 (8 per 16 scores; plain fmaxf on MFMA results also emitted a
//    canonicalising v_max per operand).
template <int D, int QG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
attn_fwd_v2_kernel(const __bf16* __restrict__ Q, int64_t sq_b, int64_t sq_h, int64_t sq_l,
                   const __bf16* __restrict__ K, int64_t sk_b, int64_t sk_h, int64_t sk_l,
                   const __bf16* __restrict__ V, int64_t sv_b, int64_t sv_h, int64_t sv_l,
                   __bf16* __restrict__ O, int64_t so_b, int64_t so_h, int64_t so_l,
                   float* __restrict__ LSE, int heads, int lq, int lk, float scale_log2, Inner in) {
  static_assert(D == 64 || D == 96, "v2 forward: D = 64 or 96");
  constexpr int NQC = D / 32, DT = D / 16;
  constexpr int ROWB = 2 * D;                      // bytes per key row
  constexpr int TE = 64 * D;                       // bf16 elements of one K (or V) tile
  constexpr int NS = D == 64 ? 4 : 3;              // LDS ring stages (<= 80 KiB: 2 workgroups / CU)
  constexpr int PW = D / 32;                       // 1-KiB DMA pieces per wave per matrix and tile
  __shared__ __attribute__((aligned(1024))) __bf16 smem[NS * 2 * TE];
  auto swz = [](int r, int c) {
    if constexpr (D == 64) return c ^ (r & 7);
    else return (c & ~3) | ((c ^ ((r ^ (r >> 1)) & 2)) & 3);
  };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  // ---- DMA: piece p of a tile image = bytes [1024 p, 1024 p + 1024): lane -> row r, slot s,
  // source chunk swz(r, s) (the swizzle is an involution)
  int prow[PW], pcol[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int byte = (wid * PW + i) * 1024 + lane * 16;
    prow[i] = byte / ROWB;
    pcol[i] = swz(prow[i], (byte % ROWB) / 16) * 8;
  }
  const int ntiles = (lk + 63) / 64;
  auto issue = [&](int t, int st) {
    __bf16* kimg = smem + st * 2 * TE;
    __bf16* vimg = kimg + TE;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int key = min(t * 64 + prow[i], lk - 1);  // rows past lk re-read a real row (masked)
      __builtin_amdgcn_global_load_lds((const void*)(K + (int64_t)key * sk_l + pcol[i]),
                                       (lds_void*)(kimg + (wid * PW + i) * 512), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(V + (int64_t)key * sv_l + pcol[i]),
                                       (lds_void*)(vimg + (wid * PW + i) * 512), 16, 0, 0);
    }
  };
  bf16x8 qf[QG][NQC];
  int qrow[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    qrow[g] = bx * (64 * QG) + (wid * QG + g) * 16 + li;
#pragma unroll
    for (int c = 0; c < NQC; ++c)
      qf[g][c] = qrow[g] < lq ? *reinterpret_cast<const bf16x8*>(Q + (int64_t)qrow[g] * sq_l + 32 * c + 8 * hg) : bf16x8{};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // Q landed before the DMA stream starts
  issue(0, 0);
  if (ntiles > 1) issue(1, 1);
  if (NS == 4 && ntiles > 2) issue(2, 2);
  f32x4 o[QG][DT];
  float m_run[QG], l_run[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    m_run[g] = -INFINITY;
    l_run[g] = 0.f;
#pragma unroll
    for (int i = 0; i < DT; ++i) o[g][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto max3 = [](float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  };
  const int qq = li >> 2, pp = li & 3;

  typedef f32x4 sblk[QG][4];
  // Sᵀ = K·Qᵀ of the tile in stage st
  auto qk = [&](int st, sblk& sv) {
    const __bf16* kimg = smem + st * 2 * TE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = j * 16 + li;
#pragma unroll
      for (int c = 0; c < NQC; ++c) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kimg + r * D + swz(r, 4 * c + hg) * 8);
#pragma unroll
        for (int g = 0; g < QG; ++g)
          sv[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[g][c], c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : sv[g][j], 0, 0, 0);
      }
    }
  };
  // online softmax of one tile: running max / rescale (branch-free: alpha == 1 when the max did
  // not move), P = exp2(S * scale - m) as bf16 PV operands, row sums
  auto softmax = [&](sblk& sv, bf16x8 (&pf)[QG][2]) {
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      float mt = max3(sv[g][0][0], sv[g][0][1], sv[g][0][2]);
      mt = max3(mt, sv[g][0][3], sv[g][1][0]);
      mt = max3(mt, sv[g][1][1], sv[g][1][2]);
      mt = max3(mt, sv[g][1][3], sv[g][2][0]);
      mt = max3(mt, sv[g][2][1], sv[g][2][2]);
      mt = max3(mt, sv[g][2][3], sv[g][3][0]);
      mt = max3(mt, sv[g][3][1], sv[g][3][2]);
      mt = fmaxf(mt, sv[g][3][3]);
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float m_new = fmaxf(m_run[g], mt * scale_log2);
      const float alpha = __builtin_amdgcn_exp2f(m_run[g] - m_new);
      m_run[g] = m_new;
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv[g][j][e], scale_log2, -m_new));
          sv[g][j][e] = p;
          ls += p;
        }
      l_run[g] = l_run[g] * alpha + ls;
#pragma unroll
      for (int i = 0; i < DT; ++i) o[g][i] *= alpha;
#pragma unroll
      for (int u = 0; u < 2; ++u)
        pf[g][u] = __builtin_shufflevector(__builtin_convertvector(sv[g][2 * u], bf16x4),
                                           __builtin_convertvector(sv[g][2 * u + 1], bf16x4), 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };
  // Oᵀ += Vᵀ·Pᵀ with the V tile in stage st
  auto pv = [&](int st, const bf16x8 (&pf)[QG][2]) {
    const __bf16* vimg = smem + st * 2 * TE + TE;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r0 = 32 * u + 4 * hg + qq, r1 = r0 + 16;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int ch = 2 * dt + (pp >> 1), sub = (pp & 1) * 4;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vimg + r0 * D + swz(r0, ch) * 8 + sub));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vimg + r1 * D + swz(r1, ch) * 8 + sub));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int g = 0; g < QG; ++g) o[g][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[g][u], o[g][dt], 0, 0, 0);
      }
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // Software pipeline: iteration t runs softmax(t) on the VALU beside the MFMAs of Sᵀ(t+1) (no
  // dependency between them, one basic block), then Oᵀ += Vᵀ(t)·Pᵀ(t). Tile j is issued at the
  // top of iteration j - (NS - 1) into stage j % NS (free: its previous tile's K was read in
  // iteration j - NS - 1, its V in iteration j - NS, both before the barrier that precedes the
  // issue); the top of iteration t waits for tile t+1 (K for Sᵀ(t+1)).
  if (NS == 4) {
    if (ntiles > 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 * PW) : "memory");
    else if (ntiles > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (ntiles > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  sync();
  // one non-last iteration: cur = Sᵀ(t) -> Oᵀ; nxt = Sᵀ(t+1). The loop is unrolled by two with the
  // roles of the two score blocks swapped (no register copies) and the ragged last tile peeled
  // (no per-element mask in the loop body)
  auto iter = [&](int t, int st, sblk& cur, sblk& nxt) {
    if (NS == 4 && t + 2 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sync();
    if (t + NS - 1 < ntiles) issue(t + NS - 1, st == 0 ? NS - 1 : st - 1);
    qk(st == NS - 1 ? 0 : st + 1, nxt);
    bf16x8 pf[QG][2];
    softmax(cur, pf);
    pv(st, pf);
  };
  auto last = [&](int t, int st, sblk& cur) {
#pragma unroll
    for (int g = 0; g < QG; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (t * 64 + j * 16 + 4 * hg + e >= lk) cur[g][j][e] = -INFINITY;
    bf16x8 pf[QG][2];
    softmax(cur, pf);
    pv(st, pf);
  };
  auto nxt_st = [](int st) { return st == NS - 1 ? 0 : st + 1; };
  sblk sa, sb;
  qk(0, sa);
  int t = 0, st = 0;
  for (; t + 2 < ntiles; t += 2) {
    iter(t, st, sa, sb);
    st = nxt_st(st);
    iter(t + 1, st, sb, sa);
    st = nxt_st(st);
  }
  if (t + 1 < ntiles) {
    iter(t, st, sa, sb);
    last(t + 1, nxt_st(st), sb);
  } else {
    last(t, st, sa);
  }

#pragma unroll
  for (int g = 0; g < QG; ++g) {
    float l_tot = l_run[g];
    l_tot += __shfl_xor(l_tot, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (qrow[g] >= lq) continue;
    const float inv = 1.f / l_tot;
    __bf16* orow = O + (int64_t)qrow[g] * so_l;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      *reinterpret_cast<bf16x4*>(orow + 16 * dt + 4 * hg) = __builtin_convertvector(o[g][dt] * inv, bf16x4);
    if (LSE && hg == 0) LSE[bh * lq + qrow[g]] = (m_run[g] + log2f(l_tot)) * LN2;
  }
}


template <int D>
int launch_fwd_v2(const comet_attn_args& a, hipStream_t s) {
  constexpr int QG = 2;
  dim3 grid((unsigned)cdiv(a.lq, 64 * QG), (unsigned)(a.batch * a.heads));
  hipLaunchKernelGGL((attn_fwd_v2_kernel<D, QG>), grid, dim3(256), 0, s,
                     (const __bf16*)a.q, a.sq_b, a.sq_h, a.sq_l, (const __bf16*)a.k, a.sk_b, a.sk_h, a.sk_l,
                     (const __bf16*)a.v, a.sv_b, a.sv_h, a.sv_l, (__bf16*)a.o, a.so_b, a.so_h, a.so_l,
                     a.lse, (int)a.heads, (int)a.lq, (int)a.lk, a.scale * LOG2E, inner_of(a));
  COMET_CHECK_LAUNCH("comet_attention_fwd (v2)");
  return COMET_OK;
}


  // v2 (LDS-DMA ring, swizzled conflict-free images, software-pipelined softmax) for the long
  // D = 64 / 96 sequences: opt-in (COMET_ATTN_V2=1). Measured equal (D = 96) or 7 % slower
  // (D = 64) than attn_fwd_bf16_kernel on the step's shapes although its LDS conflicts are gone
  // and its VALU per MFMA dropped 8.9 -> 8.1 / 6.8 -> 6.3 (profiles/r02_attn): both kernels are
  // bound by the per-wave dependency chain softmax -> PV at two waves per SIMD, not by LDS.
  const bool v2_ok = a.lq > 64 && a.lk > 64 && a.sk_l % 8 == 0 && a.sv_l % 8 == 0 && (uintptr_t)a.k % 16 == 0 &&
                     (uintptr_t)a.v % 16 == 0 && a.sk_h % 8 == 0 && a.sv_h % 8 == 0 && a.sk_b % 8 == 0 &&
                     a.sv_b % 8 == 0 && (a.batch_inner <= 1 || (a.sk_i % 8 == 0 && a.sv_i % 8 == 0)) &&
                     getenv("COMET_ATTN_V2") != nullptr;
  if (std::is_same<T, __bf16>::value && v2_ok) {
    if (a.head_dim == 64) return launch_fwd_v2<64>(a, s);
    if (a.head_dim == 96) return launch_fwd_v2<96>(a, s);
  }
