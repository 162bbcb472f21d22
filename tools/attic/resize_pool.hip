// Moved out of csrc/cnn.hip (round 3): opt-in fused up-sample + 2x2 pool (COMET_RESIZE_POOL),
// bit-identical, 0.6 % slower in the step. Not compiled.
// ShallowEncoder's final up-sample fused with the fine pyramid's first 2x2 average pool
// (blocks.py:199-202 -> base_track_predictor.py CorrBlock pyramid): one workgroup per image stages
// the input image in LDS, writes the resized image y, and writes p = the 2x2 average of y's values
// recomputed from the LDS input and rounded to TO exactly as stored -- the avg_pool2d pass no longer
// re-reads y from HBM (2 GB at B*N*S = 65536 31x31x32 bf16 maps).
template <typename TI, typename TO>
__device__ __forceinline__ void bilerp8(const TI* img, int c, int h, int w, int oh, int ow, int oy, int ox, int cg,
                                        float (&o)[8]) {
  int64_t y0, y1, x0, x1;
  float fy, fx;
  ac_coord(oy, h, oh, y0, y1, fy);
  ac_coord(ox, w, ow, x0, x1, fx);
  float v00[8], v01[8], v10[8], v11[8];
  load8(img + ((int)y0 * w + (int)x0) * c + cg * 8, v00);
  load8(img + ((int)y0 * w + (int)x1) * c + cg * 8, v01);
  load8(img + ((int)y1 * w + (int)x0) * c + cg * 8, v10);
  load8(img + ((int)y1 * w + (int)x1) * c + cg * 8, v11);
#pragma unroll
  for (int e = 0; e < 8; ++e)
    o[e] = (1.f - fy) * ((1.f - fx) * v00[e] + fx * v01[e]) + fy * ((1.f - fx) * v10[e] + fx * v11[e]);
}

template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
resize_pool_img_kernel(const TI* __restrict__ x, TO* __restrict__ y, TO* __restrict__ p, int c, int h, int w, int oh,
                       int ow) {
  extern __shared__ uint4 lds[];
  const TI* img = reinterpret_cast<const TI*>(lds);
  const int64_t ni = blockIdx.x;
  const int nvec = (int)((int64_t)h * w * c * (int)sizeof(TI) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(x + ni * h * w * c);
  for (int i = threadIdx.x; i < nvec; i += 256) lds[i] = src[i];
  __syncthreads();
  const int cg8 = c / 8, items = oh * ow * cg8;
  TO* yo = y + ni * oh * ow * c;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int pix = it / cg8, cg = it - pix * cg8;
    const int oy = pix / ow, ox = pix - oy * ow;
    float o[8];
    bilerp8<TI, TO>(img, c, h, w, oh, ow, oy, ox, cg, o);
    store8(yo + (int64_t)it * 8, o);
  }
  const int ph = oh / 2, pw = ow / 2, pitems = ph * pw * cg8;
  TO* po = p + ni * ph * pw * c;
  for (int it = threadIdx.x; it < pitems; it += 256) {
    const int pix = it / cg8, cg = it - pix * cg8;
    const int py = pix / pw, px = pix - py * pw;
    float q[4][8], o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bilerp8<TI, TO>(img, c, h, w, oh, ow, 2 * py + (k >> 1), 2 * px + (k & 1), cg, q[k]);
#pragma unroll
      for (int e = 0; e < 8; ++e) q[k][e] = to_f32(from_f32<TO>(q[k][e]));  // y's stored value
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (q[0][e] + q[1][e] + q[2][e] + q[3][e]) * 0.25f;  // avgpool2_rows_kernel's sum
    store8(po + (int64_t)it * 8, o);
  }
}


extern "C" int comet_resize_pool_nhwc(int dtype_in, int dtype_out, const void* x, void* y, void* p, int64_t n,
                                      int64_t c, int64_t h, int64_t w, int64_t oh, int64_t ow, void* stream) {
  COMET_CHECK_ARG(x && y && p && n > 0 && c % 8 == 0 && h > 0 && w > 0 && oh >= 2 && ow >= 2 && n < (1ll << 31),
                  "comet_resize_pool_nhwc: bad args");
  const int esi = dtype_in == COMET_F32 ? 4 : 2, eso = dtype_out == COMET_F32 ? 4 : 2;
  (void)eso;
  const int64_t in_b = h * w * c * esi;
  COMET_CHECK_ARG(in_b <= 32768 && ((uintptr_t)x | (uintptr_t)y | (uintptr_t)p) % 16 == 0,
                  "comet_resize_pool_nhwc: the input image must fit 32 KiB of LDS, 16-B aligned");
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)in_b;
#define RP(TI, TO) hipLaunchKernelGGL((resize_pool_img_kernel<TI, TO>), dim3((unsigned)n), dim3(256), lds, s, (const TI*)x, (TO*)y, (TO*)p, (int)c, (int)h, (int)w, (int)oh, (int)ow)
  if (dtype_in == COMET_F32 && dtype_out == COMET_F32) RP(float, float);
  else if (dtype_in == COMET_F32 && dtype_out == COMET_BF16) RP(float, __bf16);
  else if (dtype_in == COMET_BF16 && dtype_out == COMET_BF16) RP(__bf16, __bf16);
  else RP(__bf16, float);
#undef RP
  COMET_CHECK_LAUNCH("comet_resize_pool_nhwc");
  return COMET_OK;
}

