// Moved out of csrc/tracker.hip (round 3): opt-in correlation sampling with hoisted grid loads
// (COMET_CORR_PF), equal in isolation, 10-15 % slower inside the step. Not compiled.
// corr_kernel with the grid loads hoisted: every lane issues all NP of its grid-pixel
// loads for a level at once (out-of-map cells clamp to a valid address and are zeroed after the
// dot product), and the next level's loads are issued before this level's window sampling, so a
// track costs about one memory round trip per level instead of one per 256/LPP-pixel pass.
template <typename TF>
__device__ __forceinline__ void unpack16(const uint4 (&r)[16 * sizeof(TF) / 16], float (&a)[16]) {
  if constexpr (sizeof(TF) == 2) {
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const unsigned u[4] = {r[v].x, r[v].y, r[v].z, r[v].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[8 * v + 2 * i] = bf16_lo(u[i]); a[8 * v + 2 * i + 1] = bf16_hi(u[i]); }
    }
  } else {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      a[4 * v] = __uint_as_float(r[v].x); a[4 * v + 1] = __uint_as_float(r[v].y);
      a[4 * v + 2] = __uint_as_float(r[v].z); a[4 * v + 3] = __uint_as_float(r[v].w);
    }
  }
}

template <typename TF, typename TT, int C, int NP>
__global__ void __launch_bounds__(256)
corr_pf_kernel(PyrTab tab, int levels, int radius, const TT* __restrict__ feats, const float* __restrict__ coords,
               float* __restrict__ out, int64_t ldo, int64_t col0, int64_t N, int S, float inv_sqrt_c) {
  constexpr int G = 16;
  constexpr int LPP = C / 16, PPP = 256 / LPP;     // lanes per pixel, pixels per pass
  constexpr int NV = 16 * (int)sizeof(TF) / 16;    // 16-B vectors per lane per pixel
  __shared__ float f[C];
  __shared__ float dots[G * G];
  const int64_t t = blockIdx.x;  // (b*N + n)*S + s
  const int s = (int)(t % S);
  const int64_t b = (t / S) / N;
  for (int c = threadIdx.x; c < C; c += 256) f[c] = to_f32(feats[t * C + c]);
  const float cx = coords[t * 2], cy = coords[t * 2 + 1];
  const int win = 2 * radius + 1;
  float* orow = out + t * ldo + col0;
  const int sub = threadIdx.x % LPP, pslot = threadIdx.x / LPP;
  // Level geometry: the pixel grid is exactly the corners the window taps touch -- floor of the
  // first / last tap's source index (src_index is monotone) -- normally (2r+2)^2 pixels.
  struct Geo { int gx0, gy0, gw, gh; float xl, yl; };
  auto geo = [&](int l) {
    Geo g;
    const float scl = 1.f / (float)(1 << l);
    g.xl = cx * scl;
    g.yl = cy * scl;
    const int W = tab.w[l], H = tab.h[l];
    g.gx0 = (int)floorf(src_index(g.xl - (float)radius, W, false));
    g.gy0 = (int)floorf(src_index(g.yl - (float)radius, H, false));
    g.gw = (int)floorf(src_index(g.xl + (float)radius, W, false)) + 2 - g.gx0;
    g.gh = (int)floorf(src_index(g.yl + (float)radius, H, false)) + 2 - g.gy0;
    return g;
  };
  int cgx[NP], cgy[NP];
  uint4 raw[NP][NV];
  bool okm[NP];
  auto issue = [&](int l, const Geo& g) {
    const int H = tab.h[l], W = tab.w[l];
    const TF* fm = reinterpret_cast<const TF*>(tab.p[l]) + (b * S + s) * (int64_t)H * W * C + sub * 16;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int p = q * PPP + pslot;
      cgy[q] = p / g.gw;
      cgx[q] = p - cgy[q] * g.gw;
      const int px = g.gx0 + cgx[q], py = g.gy0 + cgy[q];
      const bool ok = cgy[q] < g.gh && px >= 0 && px < W && py >= 0 && py < H;
      okm[q] = ok;
      const uint4* src = reinterpret_cast<const uint4*>(fm + (ok ? ((int64_t)py * W + px) * C : 0));
#pragma unroll
      for (int v = 0; v < NV; ++v) raw[q][v] = src[v];
    }
  };
  Geo cur = geo(0);
  issue(0, cur);
  __syncthreads();
  float fr[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) fr[e] = f[sub * 16 + e];
  for (int l = 0; l < levels; ++l) {
    const int H = tab.h[l], W = tab.w[l];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      float a[16];
      unpack16<TF>(raw[q], a);
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += fr[e] * a[e] + fr[8 + e] * a[8 + e];
      acc = okm[q] ? acc : 0.f;
#pragma unroll
      for (int o = LPP / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (sub == 0 && cgy[q] < cur.gh) dots[cgy[q] * G + cgx[q]] = acc * inv_sqrt_c;
    }
    const Geo g = cur;
    if (l + 1 < levels) {
      cur = geo(l + 1);
      issue(l + 1, cur);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < win * win; k += 256) {
      const int i = k / win, j = k % win;
      const float ix = src_index(g.xl + (float)(i - radius), W, false);
      const float iy = src_index(g.yl + (float)(j - radius), H, false);
      const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
      const float wnw = ((float)(x0 + 1) - ix) * ((float)(y0 + 1) - iy), wne = (ix - (float)x0) * ((float)(y0 + 1) - iy);
      const float wsw = ((float)(x0 + 1) - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
      auto D = [&](int x, int y) -> float {
        const int gx = x - g.gx0, gy = y - g.gy0;
        return (gx >= 0 && gx < g.gw && gy >= 0 && gy < g.gh) ? dots[gy * G + gx] : 0.f;
      };
      orow[l * win * win + k] = D(x0, y0) * wnw + D(x0 + 1, y0) * wne + D(x0, y0 + 1) * wsw + D(x0 + 1, y0 + 1) * wse;
    }
    __syncthreads();  // dots consumed before the next level overwrites them
  }
}

// Transformer input of one iteration, [B*N*S, tdim] rows t = (b*N + n)*S + s (compute dtype):
// [ flows_emb(2*E) | flows(2) | corr (already written, f32 scratch) | track feats | 0 pad ] + pos
// where flows = coords[t] - coords[(b,n,0)], emb = get_2d_embedding(flows, E) (sin/cos
// interleaved per axis, freqs 2k*1000/E), pos = sampled 2-D sincos row of (b, n).

  // hoisted-load variant: opt-in (equal in isolation, 10-15 % slower inside the step, r01 profiles)
  if (getenv("COMET_CORR_PF") != nullptr) {
    const int npix = (2 * radius + 3) * (2 * radius + 3);  // largest exact grid
    const int np = (int)cdiv(npix, 256 / (C / 16));  // C = 128: 1..6 passes, C = 32: 1..2
#define CKP(TF, CC, NPV) hipLaunchKernelGGL((corr_pf_kernel<TF, float, CC, NPV>), dim3((unsigned)T), dim3(256), 0, s, tab, levels, radius, (const float*)feats, coords, out, ldo, col0, N, S, isc)
#define CKP_C(TF)                                                                                   \
  do {                                                                                              \
    if (C == 32) { if (np == 1) CKP(TF, 32, 1); else CKP(TF, 32, 2); }                              \
    else switch (np) {                                                                              \
      case 1: CKP(TF, 128, 1); break; case 2: CKP(TF, 128, 2); break; case 3: CKP(TF, 128, 3); break; \
      case 4: CKP(TF, 128, 4); break; case 5: CKP(TF, 128, 5); break; case 6: CKP(TF, 128, 6); break; \
      case 7: CKP(TF, 128, 7); break; default: CKP(TF, 128, 8); break;                               \
    }                                                                                               \
  } while (0)
    if (dtype_fmap == COMET_F32) CKP_C(float); else CKP_C(__bf16);
#undef CKP_C
#undef CKP
    COMET_CHECK_LAUNCH("comet_corr_sample");
    return COMET_OK;
  }
