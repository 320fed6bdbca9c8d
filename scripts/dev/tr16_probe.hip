// Probe the lane mapping of ds_read_b64_tr_b16 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__global__ void k(int* out) {
  __shared__ short t[64 * 16];  // 64 rows x 16 cols, value = row*100+col
  for (int i = threadIdx.x; i < 64 * 16; i += 64) t[i] = (short)((i / 16) * 100 + (i % 16));
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 4 * g + q, col = 4 * p;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + row * 16 + col));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  int* d; hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  int h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) { printf("lane %2d:", l); for (int e = 0; e < 4; ++e) printf(" %4d", h[l*4+e]); printf("\n"); }
  return 0;
}
