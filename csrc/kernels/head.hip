// Classifier head: global average pool -> Linear(512 -> classes) -> softmax cross-entropy,
// forward and backward fused in one launch (one workgroup per sample).
//
// Replaces nn.AdaptiveAvgPool2d((1,1)), nn.Linear and nn.CrossEntropyLoss of the reference
// (reference: src/parameter_server/server.py:56-57,73-75; src/workers/worker.py:133,342) and
// the accuracy count of evaluate_model (worker.py:324-326).
#include "common.hpp"

namespace psx {

// act: NHWC [B][HW][C] bf16; fcw: [K][C] fp32; fcb: [K] fp32; labels int32 [B]
// outputs: pooled [B][C] fp32, dlogits [B][K] fp32 (already divided by B), dact (bf16, same
// shape as act; nullable for eval), loss [B] fp32, correct (atomic int counter, nullable).
template <bool BWD>
__global__ __launch_bounds__(256) void head_kernel(const uint16_t* __restrict__ act, int HW, int C,
                                                   const float* __restrict__ fcw, const float* __restrict__ fcb, int K,
                                                   const int* __restrict__ labels, float* __restrict__ pooled,
                                                   float* __restrict__ dlogits, uint16_t* __restrict__ dact,
                                                   float* __restrict__ loss, int* __restrict__ correct, float invB) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* sp = sh;          // [C]   pooled
  float* sl = sh + C;      // [K]   logits -> dlogits
  float* red = sl + 1024;  // scratch
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint16_t* a = act + (size_t)b * HW * C;
  const float inv_hw = 1.f / (float)HW;
  for (int c = tid; c < C; c += 256) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += bf2f(a[(size_t)p * C + c]);
    s *= inv_hw;
    sp[c] = s;
    if (pooled) pooled[(size_t)b * C + c] = s;
  }
  __syncthreads();
  // logits: each wave computes K/4 rows, lanes stride the C dot product
  const int lane = tid & 63, wid = tid >> 6;
  for (int k = wid; k < K; k += 4) {
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += fcw[(size_t)k * C + c] * sp[c];
    s = wave_sum(s);
    if (lane == 0) sl[k] = s + fcb[k];
  }
  __syncthreads();
  // softmax / loss / argmax (wave 0)
  if (wid == 0) {
    float mx = -INFINITY;
    int arg = 0;
    for (int k = lane; k < K; k += 64) {
      const float v = sl[k];
      if (v > mx) {
        mx = v;
        arg = k;
      }
    }
    // wave argmax (first index on ties)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(arg, o, 64);
      if (om > mx || (om == mx && oa < arg)) {
        mx = om;
        arg = oa;
      }
    }
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += __expf(sl[k] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    const int y = labels[b];
    if (lane == 0) {
      if (loss) loss[b] = lse - sl[y];
      if (correct && arg == y) atomicAdd(correct, 1);
    }
    if (BWD) {
      for (int k = lane; k < K; k += 64) {
        const float pr = __expf(sl[k] - lse);
        const float d = (pr - (k == y ? 1.f : 0.f)) * invB;
        sl[k] = d;
        dlogits[(size_t)b * K + k] = d;
      }
    }
  }
  if (!BWD) return;
  __syncthreads();
  // dpooled[c] = sum_k dlogits[k] * W[k][c]; dact = dpooled / HW broadcast over pixels
  for (int c = tid; c < C; c += 256) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += sl[k] * fcw[(size_t)k * C + c];
    const uint16_t v = f2bf(s * inv_hw);
    for (int p = 0; p < HW; ++p) dact[((size_t)b * HW + p) * C + c] = v;
  }
  (void)red;
}

// dW[k][c] = sum_b dlogits[b][k] * pooled[b][c]; db[k] = sum_b dlogits[b][k]
template <typename GT>
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ dlogits,
                                                         const float* __restrict__ pooled, int B, int K, int C,
                                                         GT* __restrict__ dw, GT* __restrict__ db, float gscale) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = K * C + K;
  if (idx >= total) return;
  float s = 0.f;
  if (idx < K * C) {
    const int k = idx / C, c = idx - k * C;
    for (int b = 0; b < B; ++b) s += dlogits[(size_t)b * K + k] * pooled[(size_t)b * C + c];
  } else {
    const int k = idx - K * C;
    for (int b = 0; b < B; ++b) s += dlogits[(size_t)b * K + k];
  }
  s *= gscale;
  GT* dst = idx < K * C ? dw + idx : db + (idx - K * C);
  if constexpr (sizeof(GT) == 2)
    *dst = __builtin_bit_cast(uint16_t, (_Float16)s);
  else
    *dst = s;
}

}  // namespace psx

using namespace psx;

extern "C" {

int psx_head_fwd_bwd(const void* act, int B, int HW, int C, const float* fcw, const float* fcb, int K,
                     const int* labels, float* pooled, float* dlogits, void* dact, float* loss, int* correct,
                     hipStream_t st) {
  if (K > 1024) return -2;
  const size_t lds = (size_t)(C + 1024 + 64) * sizeof(float);
  if (dact)
    hipLaunchKernelGGL(head_kernel<true>, dim3(B), dim3(256), lds, st, (const uint16_t*)act, HW, C, fcw, fcb, K,
                       labels, pooled, dlogits, (uint16_t*)dact, loss, correct, 1.f / (float)B);
  else
    hipLaunchKernelGGL(head_kernel<false>, dim3(B), dim3(256), lds, st, (const uint16_t*)act, HW, C, fcw, fcb, K,
                       labels, pooled, dlogits, (uint16_t*)nullptr, loss, correct, 1.f / (float)B);
  return (int)hipGetLastError();
}

int psx_head_wgrad(const float* dlogits, const float* pooled, int B, int K, int C, void* dw, void* db, float gscale,
                   int grad_fp16, hipStream_t st) {
  const int total = K * C + K;
  const dim3 grid((total + 255) / 256);
  if (grad_fp16)
    hipLaunchKernelGGL(head_wgrad_kernel<uint16_t>, grid, dim3(256), 0, st, dlogits, pooled, B, K, C, (uint16_t*)dw,
                       (uint16_t*)db, gscale);
  else
    hipLaunchKernelGGL(head_wgrad_kernel<float>, grid, dim3(256), 0, st, dlogits, pooled, B, K, C, (float*)dw,
                       (float*)db, gscale);
  return (int)hipGetLastError();
}

}  // extern "C"
