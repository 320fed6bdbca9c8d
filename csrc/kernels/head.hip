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
// One workgroup per sample; C must be a multiple of 512 or <= 512 and even, K <= 256.
template <bool BWD>
__global__ __launch_bounds__(256) void head_kernel(const uint16_t* __restrict__ act, int HW, int C,
                                                   const float* __restrict__ fcw, const float* __restrict__ fcb, int K,
                                                   const int* __restrict__ labels, float* __restrict__ pooled,
                                                   float* __restrict__ dlogits, uint16_t* __restrict__ dact,
                                                   float* __restrict__ loss, int* __restrict__ correct, float invB) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* sp = sh;      // [C]  pooled
  float* sl = sh + C;  // [K]  logits -> dlogits
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint16_t* a = act + (size_t)b * HW * C;
  const float inv_hw = 1.f / (float)HW;
  // global average pool, 2 channels per thread per pass (4-byte loads, coalesced)
  for (int c = 2 * tid; c < C; c += 512) {
    float s0 = 0.f, s1 = 0.f;
    for (int p = 0; p < HW; ++p) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(a + (size_t)p * C + c);
      s0 += lo_bf(v);
      s1 += hi_bf(v);
    }
    s0 *= inv_hw;
    s1 *= inv_hw;
    sp[c] = s0;
    sp[c + 1] = s1;
    if (pooled) {
      pooled[(size_t)b * C + c] = s0;
      pooled[(size_t)b * C + c + 1] = s1;
    }
  }
  __syncthreads();
  // logits: 4 lanes per class row, each lane a quarter of the C-long dot product
  for (int r = tid >> 2; r < K; r += 64) {
    const int part = tid & 3, len = C >> 2;
    const float4* w4 = reinterpret_cast<const float4*>(fcw + (size_t)r * C + part * len);
    const float* x = sp + part * len;
    float s = 0.f;
    for (int j = 0; j < (len >> 2); ++j) {
      const float4 w = w4[j];
      s += w.x * x[4 * j] + w.y * x[4 * j + 1] + w.z * x[4 * j + 2] + w.w * x[4 * j + 3];
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (part == 0) sl[r] = s + fcb[r];
  }
  __syncthreads();
  const int lane = tid & 63, wid = tid >> 6;
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
        const float d = (__expf(sl[k] - lse) - (k == y ? 1.f : 0.f)) * invB;
        sl[k] = d;
        dlogits[(size_t)b * K + k] = d;
      }
    }
  }
  if (!BWD) return;
  __syncthreads();
  // dpooled[c] = sum_k dlogits[k] * W[k][c]; dact = dpooled / HW broadcast over the pixels
  for (int c = 2 * tid; c < C; c += 512) {
    float s0 = 0.f, s1 = 0.f;
    for (int k = 0; k < K; ++k) {
      const float2 w = *reinterpret_cast<const float2*>(fcw + (size_t)k * C + c);
      s0 += sl[k] * w.x;
      s1 += sl[k] * w.y;
    }
    const uint32_t v = pack_bf2(s0 * inv_hw, s1 * inv_hw);
    for (int p = 0; p < HW; ++p) *reinterpret_cast<uint32_t*>(dact + ((size_t)b * HW + p) * C + c) = v;
  }
}

// dW[k][c] = sum_b dlogits[b][k] * pooled[b][c]; db[k] = sum_b dlogits[b][k].
// Block: 8 classes x 256 channels; dlogits for those classes staged in LDS.
template <typename GT>
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ dlogits,
                                                         const float* __restrict__ pooled, int B, int K, int C,
                                                         GT* __restrict__ dw, GT* __restrict__ db, float gscale) {
  extern __shared__ __attribute__((aligned(16))) float sdl[];  // [B][8]
  const int k0 = blockIdx.y * 8, c = blockIdx.x * 256 + threadIdx.x;
  for (int i = threadIdx.x; i < B * 8; i += 256) {
    const int bb = i >> 3, kk = i & 7;
    sdl[i] = (k0 + kk < K) ? dlogits[(size_t)bb * K + k0 + kk] : 0.f;
  }
  __syncthreads();
  float acc[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) acc[kk] = 0.f;
  if (c < C) {
    for (int bb = 0; bb < B; ++bb) {
      const float pv = pooled[(size_t)bb * C + c];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) acc[kk] += sdl[bb * 8 + kk] * pv;
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (k0 + kk >= K) break;
      const float v = acc[kk] * gscale;
      if constexpr (sizeof(GT) == 2)
        dw[(size_t)(k0 + kk) * C + c] = __builtin_bit_cast(uint16_t, (_Float16)v);
      else
        dw[(size_t)(k0 + kk) * C + c] = v;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 8 && k0 + threadIdx.x < K) {
    float s = 0.f;
    for (int bb = 0; bb < B; ++bb) s += sdl[bb * 8 + threadIdx.x];
    s *= gscale;
    if constexpr (sizeof(GT) == 2)
      db[k0 + threadIdx.x] = __builtin_bit_cast(uint16_t, (_Float16)s);
    else
      db[k0 + threadIdx.x] = s;
  }
}

}  // namespace psx

using namespace psx;

extern "C" {

int psx_head_fwd_bwd(const void* act, int B, int HW, int C, const float* fcw, const float* fcb, int K,
                     const int* labels, float* pooled, float* dlogits, void* dact, float* loss, int* correct,
                     hipStream_t st) {
  if (K > 1024 || C % 16 || (C > 512 && C % 512)) return -2;
  const size_t lds = (size_t)(C + K + 64) * sizeof(float);
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
  const dim3 grid((C + 255) / 256, (K + 7) / 8);
  const size_t lds = (size_t)B * 8 * sizeof(float);
  if (grad_fp16)
    hipLaunchKernelGGL(head_wgrad_kernel<uint16_t>, grid, dim3(256), lds, st, dlogits, pooled, B, K, C, (uint16_t*)dw,
                       (uint16_t*)db, gscale);
  else
    hipLaunchKernelGGL(head_wgrad_kernel<float>, grid, dim3(256), lds, st, dlogits, pooled, B, K, C, (float*)dw,
                       (float*)db, gscale);
  return (int)hipGetLastError();
}

}  // extern "C"
