// MFMA throughput ceiling on this box: every SIMD of every CU issues back-to-back independent
// v_mfma_f32_16x16x4_f32 (16 accumulators per wave) — the fp32 conv kernels' instruction — and
// v_mfma_f32_16x16x32_bf16 for the bf16 path; TFLOP/s from hipEvent timing of a 256 x k grid.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <bool BF16>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float seed) {
  f32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const float a = seed * (threadIdx.x + 1), b = seed * 0.5f;
  bf16x8 av, bv;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    av[i] = (__bf16)a;
    bv[i] = (__bf16)b;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (BF16)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i], 0, 0, 0);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int bf = 0; bf < 2; ++bf)
    for (int wgs = 256; wgs <= 1024; wgs *= 2) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (bf)
          hipLaunchKernelGGL(mfma_loop<true>, dim3(wgs), dim3(256), 0, 0, out, iters, 1e-3f);
        else
          hipLaunchKernelGGL(mfma_loop<false>, dim3(wgs), dim3(256), 0, 0, out, iters, 1e-3f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flop_per = bf ? 2.0 * 16 * 16 * 32 : 2.0 * 16 * 16 * 4;
        const double flops = flop_per * 16.0 * iters * 4.0 * wgs;
        if (rep) printf("{\"mfma\": \"%s\", \"workgroups\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n",
                        bf ? "16x16x32_bf16" : "16x16x4_f32", wgs, ms, flops / ms / 1e9);
      }
    }
  return 0;
}
