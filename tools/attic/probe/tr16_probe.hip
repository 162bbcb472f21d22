// Probe: lane mapping of ds_read_b64_tr_b16 on gfx950 (debug tool, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short sm[16 * 32];
  for (int i = threadIdx.x; i < 16 * 32; i += 64) sm[i] = (short)((i / 32) * 100 + (i % 32));  // row*100+col, 32 cols
  __syncthreads();
  int l = threadIdx.x, i = l & 15, g = l >> 4;
  int q = i >> 2, p = i & 3;
  // group g reads rows 4g+q, cols 4p..4p+3
  const short* a = sm + (4 * g + q) * 32 + 4 * p;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  k<<<1, 64>>>(d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
  return 0;
}
