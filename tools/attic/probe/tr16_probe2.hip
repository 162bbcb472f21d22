// Probe 2: ds_read_b64_tr_b16 with a 40-element row pitch, a non-zero LDS base and
// immediate offsets (the attention kernel's addressing). Debug tool, not product code.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
template <int VAR>
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short A[64 * 40];
  __shared__ __attribute__((aligned(16))) short Bv[64 * 40];
  for (int i = threadIdx.x; i < 64 * 40; i += 64) { A[i] = -1; Bv[i] = (short)((i / 40) * 100 + (i % 40)); }
  __syncthreads();
  int l = threadIdx.x, i = l & 15, g = l >> 4;
  int q = i >> 2, p = i & 3;
  const short* base = (VAR == 0) ? Bv : Bv + 16 * 40;  // VAR 1: rows 16.. via immediate-able offset
  const short* a = base + (4 * g + q) * 40 + 4 * p;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
  A[l] = v[0];
}
int main() {
  short* d; (void)hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  k<0><<<1, 64>>>(d); (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("VAR0 lane0: %d %d %d %d lane5: %d %d %d %d lane17: %d %d %d %d\n", h[0], h[1], h[2], h[3], h[20], h[21], h[22], h[23], h[68], h[69], h[70], h[71]);
  k<1><<<1, 64>>>(d); (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("VAR1 lane0: %d %d %d %d lane5: %d %d %d %d lane17: %d %d %d %d\n", h[0], h[1], h[2], h[3], h[20], h[21], h[22], h[23], h[68], h[69], h[70], h[71]);
  return 0;
}
