// Probe of ds_read_b64_tr_b16 lane semantics on gfx950: LDS holds u16 value
// (row * 256 + col) for a [8][64] u16 image (128-B rows); lane 4q+p of each
// 16-lane group addresses row q, columns 16*(g&1) + 4p (g = lane / 16); prints
// what every lane receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void probe(unsigned short* out) {
  __shared__ __attribute__((aligned(16))) unsigned short img[8 * 64];
  for (int i = threadIdx.x; i < 8 * 64; i += 64) img[i] = (unsigned short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const unsigned short* a = img + (q + 4 * (g >> 1)) * 64 + 16 * (g & 1) + 4 * p;
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = (unsigned short)r[e];
}
int main() {
  unsigned short* d;
  hipMalloc(&d, 256 * 2);
  probe<<<1, 64>>>(d);
  unsigned short h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) printf(" (r%d,c%2d)", h[l * 4 + e] >> 8, h[l * 4 + e] & 255);
    printf("\n");
  }
  return 0;
}
