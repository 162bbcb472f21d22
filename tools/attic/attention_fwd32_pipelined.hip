// Moved out of csrc/attention.hip (round 3): software-pipelined 32x32 forward (next tile's S
// MFMAs interleaved with this tile's softmax by sched_group_barrier). Measured 20-25 % slower than
// the plain 32x32 kernel on the DINO / head shapes (profiles/r03_attn_v3_*.txt). Not compiled.
// Software-pipelined variant of attn_fwd32_kernel: the next key tile's Sᵀ MFMAs are issued
// between the VALU of this tile's softmax (sched_group_barrier), so the matrix pipe runs while
// the vector unit exponentiates (cdna_hip_programming.md T15). K and V have separate double
// buffers: iteration t reads K(t+1) and V(t), and refills K(t+2) / V(t+1) after its MFMAs.
template <int D>
__global__ void __launch_bounds__(256, 2)
attn_fwd32p_kernel(const __bf16* __restrict__ Q, int64_t sq_b, int64_t sq_h, int64_t sq_l,
                   const __bf16* __restrict__ K, int64_t sk_b, int64_t sk_h, int64_t sk_l,
                   const __bf16* __restrict__ V, int64_t sv_b, int64_t sv_h, int64_t sv_l,
                   __bf16* __restrict__ O, int64_t so_b, int64_t so_h, int64_t so_l,
                   float* __restrict__ LSE, int heads, int lq, int lk, float scale_log2, Inner in) {
  static_assert(D % 16 == 0 && D <= 128, "D: multiple of 16");
  constexpr int NKS = D / 16, DB = (D + 31) / 32;
  constexpr int KP = D + 8, VP = DB * 32 + 8, NCH = D / 8;
  constexpr int NST = (64 * NCH + 255) / 256;
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

  if constexpr (DB * 32 != D) {
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
  f32x16 oacc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) oacc[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;

  uint4 kst[NST], vst[NST];
  auto gload = [&](uint4 (&dst)[NST], const __bf16* src, int64_t sl, int t) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / NCH, c = idx % NCH;
      const int key = t * 64 + row;
      dst[i] = (idx < 64 * NCH && key < lk) ? *reinterpret_cast<const uint4*>(src + (int64_t)key * sl + 8 * c)
                                            : uint4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](const uint4 (&src)[NST], __bf16* img, int pitch) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int idx = tid + i * 256;
      if (idx < 64 * NCH) *reinterpret_cast<uint4*>(img + (idx / NCH) * pitch + 8 * (idx % NCH)) = src[i];
    }
  };
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int voff = (4 * (tg >> 1) + tq) * VP + 16 * (tg & 1) + 4 * tp;

  auto smm = [&](f32x16 (&sc)[2], const __bf16* ks) {  // Sᵀ of one key tile
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      sc[kb] = f32x16{};
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + (kb * 32 + r) * KP + 16 * s + 8 * h);
        sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sc[kb], 0, 0, 0);
      }
    }
  };
  // softmax of tile t (in sc) -> P fragments; then O += Vᵀ·Pᵀ
  auto softmax_pv = [&](int t, f32x16 (&sc)[2], const __bf16* vs, bool mask) {
    if (mask) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (t * 64 + kb * 32 + (j & 3) + 8 * (j >> 2) + 4 * h >= lk) sc[kb][j] = -INFINITY;
    }
    float mt = fmaxf(sc[0][0], sc[1][0]);
#pragma unroll
    for (int j = 1; j < 16; ++j) mt = fmaxf(mt, fmaxf(sc[0][j], sc[1][j]));
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mt), __float_as_uint(mt), false, false);
      mt = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const float m_new = fmaxf(m_run, mt * scale_log2);
    if (__ballot(m_new > m_run) != 0) {
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < DB; ++i) oacc[i] *= alpha;
      m_run = m_new;
    }
    float ls = 0.f;
    bf16x8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][j], scale_log2, -m_new));
        sc[kb][j] = pv;
        ls += pv;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const f32x4 lo = {sc[kb][8 * s2], sc[kb][8 * s2 + 1], sc[kb][8 * s2 + 2], sc[kb][8 * s2 + 3]};
        const f32x4 hi = {sc[kb][8 * s2 + 4], sc[kb][8 * s2 + 5], sc[kb][8 * s2 + 6], sc[kb][8 * s2 + 7]};
        pf[kb][s2] = __builtin_shufflevector(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4),
                                             0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    l_run += ls;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const __bf16* va = vs + (kb * 32 + 16 * s2) * VP + voff;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(va + 32 * db));
          const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(va + 8 * VP + 32 * db));
          const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][s2], oacc[db], 0, 0, 0);
        }
      }
  };

  const int n = (lk + 63) / 64;
  // prologue: K(0), V(0) -> buffers 0, K(1) -> Ks[1]; S(0)
  gload(kst, K, sk_l, 0);
  gload(vst, V, sv_l, 0);
  lstore(kst, Ks[0], KP);
  lstore(vst, Vs[0], VP);
  if (n > 1) {
    gload(kst, K, sk_l, 1);
    lstore(kst, Ks[1], KP);
  }
  __syncthreads();
  f32x16 sA[2], sB[2];
  smm(sA, Ks[0]);
  __syncthreads();  // every wave's S(0) reads of Ks[0] precede iteration 0's refill of it

  // iteration t: S(t+1) (into the other register set) interleaved with softmax(t), O += V(t)·P(t),
  // refill Ks[t&1] <- K(t+2), Vs[(t+1)&1] <- V(t+1)
  auto step = [&](int t, f32x16 (&cur)[2], f32x16 (&nxt)[2]) {
    const bool more = t + 1 < n;
    if (t + 2 < n) gload(kst, K, sk_l, t + 2);
    if (more) gload(vst, V, sv_l, t + 1);
    if (more) smm(nxt, Ks[(t + 1) & 1]);
    softmax_pv(t, cur, Vs[t & 1], t == n - 1);
    if (more) {
      // MFMAs of S(t+1) spread over the softmax VALU
#pragma unroll
      for (int i = 0; i < 2 * NKS; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
      }
    }
    if (t + 2 < n) lstore(kst, Ks[t & 1], KP);
    if (more) lstore(vst, Vs[(t + 1) & 1], VP);
    __syncthreads();
  };
  int t = 0;
  for (; t + 1 < n; t += 2) {
    step(t, sA, sB);
    step(t + 1, sB, sA);
  }
  if (t < n) step(t, sA, sB);

  float l_tot = l_run;
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_tot), __float_as_uint(l_tot), false, false);
    l_tot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = 1.f / l_tot;
  __bf16* orow = O + (int64_t)qrow * so_l;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int u = 0; u < 4; u += 2) {
      if (32 * db + 8 * u >= D) continue;
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

