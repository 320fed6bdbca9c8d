// Classifier head: global average pool -> Linear(512 -> classes) -> softmax cross-entropy,
// forward and backward fused in one launch (one workgroup per sample).
//
// Replaces nn.AdaptiveAvgPool2d((1,1)), nn.Linear and nn.CrossEntropyLoss of the reference
// (reference: src/parameter_server/server.py:56-57,73-75; src/workers/worker.py:133,342) and
// the accuracy count of evaluate_model (worker.py:324-326).
#include "bnfin.hpp"
#include <algorithm>

#include "common.hpp"

namespace psx {

// Optional BN-backward reduction of the layer whose output the head consumes (same layout as
// conv_v2.hip BwdStatsDesc): slot rows part[T][2][C] += (sum dz, sum dz * xhat) over this
// sample's pixels, dz = dact * [o > 0] with o = act, xhat = (y1 - mean) * invstd, saved1 =
// [2][C] (mean, invstd) — what bn_bwd_reduce would compute in its own pass over dact, act, y1.
struct HeadBnStats {
  float* part;
  const void* o;
  const void* y1;
  const void* y2;
  const float* saved1;
  const float* saved2;
};

// act: NHWC [B][HW][C] of storage type T (bf16 bits or fp32); fcw: [K][C] fp32; fcb: [K] fp32;
// labels int32 [B]. outputs: pooled [B][C] fp32, dlogits [B][K] fp32 (already divided by B),
// dact (T, same shape as act; nullable for eval), loss [B] fp32, correct (atomic int counter,
// nullable). One workgroup per sample; C must be a multiple of 512 or <= 512 and even, K <= 256.
template <typename T, bool BWD>
__global__ __launch_bounds__(256) void head_kernel(const T* __restrict__ act, int HW, int C,
                                                   const float* __restrict__ fcw, const float* __restrict__ fcb, int K,
                                                   const int* __restrict__ labels, float* __restrict__ pooled,
                                                   float* __restrict__ dlogits, T* __restrict__ dact,
                                                   float* __restrict__ loss, int* __restrict__ correct, float invB,
                                                   HeadBnStats bs, DetRed det) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* sp = sh;      // [C]  pooled
  float* sl = sh + C;  // [K]  logits -> dlogits
  const int b = blockIdx.x, tid = threadIdx.x;
  const T* a = act + (size_t)b * HW * C;
  const float inv_hw = 1.f / (float)HW;
  // global average pool, 2 channels per thread per pass (coalesced pair loads)
  for (int c = 2 * tid; c < C; c += 512) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll 16
    for (int p = 0; p < HW; ++p) {
      float v0, v1;
      ld2(a + (size_t)p * C + c, v0, v1);
      s0 += v0;
      s1 += v1;
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
    // unrolled: the row's L2 loads are issued back to back instead of one latency per step
#pragma unroll 8
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
#pragma unroll 10
    for (int k = 0; k < K; ++k) {
      const float2 w = *reinterpret_cast<const float2*>(fcw + (size_t)k * C + c);
      s0 += sl[k] * w.x;
      s1 += sl[k] * w.y;
    }
    float g0 = s0 * inv_hw, g1 = s1 * inv_hw;
    for (int p = 0; p < HW; ++p) {
      float q0 = g0, q1 = g1;
      st2(dact + ((size_t)b * HW + p) * C + c, q0, q1);
      if (p == HW - 1) {  // the gradient as stored
        g0 = q0;
        g1 = q1;
      }
    }
    if (bs.part) {  // BN-backward sums of the consumed layer (see HeadBnStats)
      const float m0 = bs.saved1[c], i0 = bs.saved1[C + c], m1 = bs.saved1[c + 1], i1 = bs.saved1[C + c + 1];
      const T* y = reinterpret_cast<const T*>(bs.y1) + (size_t)b * HW * C + c;
      float z0 = 0.f, z1 = 0.f, x0 = 0.f, x1 = 0.f;
#pragma unroll 8
      for (int p = 0; p < HW; ++p) {
        float o0, o1, y0, y1v;
        ld2(a + (size_t)p * C + c, o0, o1);
        ld2(y + (size_t)p * C, y0, y1v);
        const float d0 = o0 > 0.f ? g0 : 0.f, d1 = o1 > 0.f ? g1 : 0.f;
        z0 += d0;
        z1 += d1;
        x0 += d0 * (y0 - m0) * i0;
        x1 += d1 * (y1v - m1) * i1;
      }
      float* dst = bs.part + (size_t)(b & (PSX_STAT_SLOTS - 1)) * 2 * C;
      stat_add(det, dst, c, z0);
      stat_add(det, dst, c + 1, z1);
      stat_add(det, dst, C + c, x0);
      stat_add(det, dst, C + c + 1, x1);
    }
  }
}

// dW[k][c] = sum_b dlogits[b][k] * pooled[b][c]; db[k] = sum_b dlogits[b][k].
// Block: 8 classes x 256 channels; dlogits for those classes staged in LDS. (The small-head
// variant below trades the 8-class register block for 4x more workgroups.)
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

// ---- large heads (ResNet-50: 2048 -> 1000): the fused kernel above streams the whole FC matrix
// through every per-sample workgroup twice (2 x 8 MB x B); split into pool -> logits GEMM ->
// softmax/xent -> dpooled GEMM (+ broadcast to dact), each matrix read once per 32-sample tile.

// pooled[b][c] = mean over the HW pixels; grid (B, ceil(C / 512)), 2 channels per thread
// also zeroes zbuf[0, nz) (the split-K logits accumulator)
template <typename T>
__global__ __launch_bounds__(256) void head_pool_kernel(const T* __restrict__ act, int HW, int C,
                                                        float* __restrict__ pooled, float* __restrict__ zbuf,
                                                        long nz) {
  const long gt = ((long)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
  for (long i = gt; i < nz; i += (long)gridDim.x * gridDim.y * 256) zbuf[i] = 0.f;
  const int b = blockIdx.x, c = blockIdx.y * 512 + 2 * threadIdx.x;
  if (c >= C) return;
  const T* a = act + (size_t)b * HW * C + c;
  float s0 = 0.f, s1 = 0.f;
  for (int p = 0; p < HW; ++p) {
    float v0, v1;
    ld2(a + (size_t)p * C, v0, v1);
    s0 += v0;
    s1 += v1;
  }
  const float inv = 1.f / (float)HW;
  *reinterpret_cast<float2*>(pooled + (size_t)b * C + c) = make_float2(s0 * inv, s1 * inv);
}

// out[m][n] = sum_k A[m][k] * B(k, n), fp32, 32 x 64 tile per workgroup (2 x 4 per thread), k in
// chunks of 32 through LDS. BT: B(k, n) = Bm[n][k] (FC rows: logits); else Bm[k][n] (dpooled).
// EPI 0: out += partial (+ bias[n] from split 0), fp32 atomics, split-K over blockIdx.z (out
// zeroed beforehand); EPI 1: dact (T) = out / HW written to all HW pixels of sample m (no split).
template <bool BT, int EPI, typename T = uint16_t>
__global__ __launch_bounds__(256) void head_gemm_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                        int M, int N, int Kd, const float* __restrict__ bias,
                                                        float* __restrict__ out, T* __restrict__ dact,
                                                        int HW) {
  __shared__ float As[32][33];
  __shared__ float Bs[32][68];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 64;
  const int kper = ((Kd + gridDim.z * 32 - 1) / (gridDim.z * 32)) * 32;  // 32-aligned split ranges
  const int kbeg = blockIdx.z * kper, kend = min(Kd, kbeg + kper);
  float acc[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int k0 = kbeg; k0 < kend; k0 += 32) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A tile 32 x 32, coalesced along k
      const int idx = i * 256 + tid, mm = idx >> 5, kk = idx & 31;
      As[mm][kk] = (m0 + mm < M && k0 + kk < kend) ? A[(size_t)(m0 + mm) * Kd + k0 + kk] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // B tile 32 (k) x 64 (n)
      const int idx = i * 256 + tid;
      if (BT) {  // coalesced along k of row n
        const int nn = idx >> 5, kk = idx & 31;
        Bs[kk][nn] = (n0 + nn < N && k0 + kk < kend) ? Bm[(size_t)(n0 + nn) * Kd + k0 + kk] : 0.f;
      } else {   // coalesced along n of row k
        const int kk = idx >> 6, nn = idx & 63;
        Bs[kk][nn] = (n0 + nn < N && k0 + kk < kend) ? Bm[(size_t)(k0 + kk) * N + n0 + nn] : 0.f;
      }
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      const float a0 = As[2 * ty][kk], a1 = As[2 * ty + 1][kk];
      const float4 bv = *reinterpret_cast<const float4*>(&Bs[kk][4 * tx]);
      acc[0][0] += a0 * bv.x; acc[0][1] += a0 * bv.y; acc[0][2] += a0 * bv.z; acc[0][3] += a0 * bv.w;
      acc[1][0] += a1 * bv.x; acc[1][1] += a1 * bv.y; acc[1][2] += a1 * bv.z; acc[1][3] += a1 * bv.w;
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + 2 * ty + i;
    if (m >= M) continue;
    const int n = n0 + 4 * tx;
    if (EPI == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < N) atomicAdd(out + (size_t)m * N + n + j, acc[i][j] + (blockIdx.z == 0 ? bias[n + j] : 0.f));
    } else if (n + 3 < N) {  // N (channels) is a multiple of 64 on this path
      const float inv = 1.f / (float)HW;
      for (int p = 0; p < HW; ++p) {
        float v0 = acc[i][0] * inv, v1 = acc[i][1] * inv, v2 = acc[i][2] * inv, v3 = acc[i][3] * inv;
        T* d = dact + ((size_t)m * HW + p) * N + n;
        st2(d, v0, v1);
        st2(d + 2, v2, v3);
      }
    }
  }
}

// one wave per sample: logits row (in dl) -> loss, accuracy, dlogits = (softmax - onehot) / B in place
__global__ __launch_bounds__(64) void head_softmax_kernel(float* __restrict__ dl, int K, const int* __restrict__ labels,
                                                          float* __restrict__ loss, int* __restrict__ correct,
                                                          float invB, int bwd) {
  const int b = blockIdx.x, lane = threadIdx.x;
  float* row = dl + (size_t)b * K;
  float mx = -INFINITY;
  int arg = 0;
  for (int k = lane; k < K; k += 64) {
    const float v = row[k];
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
  for (int k = lane; k < K; k += 64) se += __expf(row[k] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const int y = labels[b];
  const float ly = row[y];
  if (lane == 0) {
    if (loss) loss[b] = lse - ly;
    if (correct && arg == y) atomicAdd(correct, 1);
  }
  if (bwd)
    for (int k = lane; k < K; k += 64) row[k] = (__expf(row[k] - lse) - (k == y ? 1.f : 0.f)) * invB;
}

// Small heads (ResNet-18: 100 x 512, B = 128): one output per thread, workgroup = 4 classes x 64
// channels (200 workgroups instead of 26); dlogits of the 4 classes staged in LDS, pooled read
// coalesced along the channels; db by the first channel block.
template <typename GT>
__global__ __launch_bounds__(256) void head_wgrad_small_kernel(const float* __restrict__ dlogits,
                                                               const float* __restrict__ pooled, int B, int K,
                                                               int C, GT* __restrict__ dw, GT* __restrict__ db,
                                                               float gscale) {
  extern __shared__ __attribute__((aligned(16))) float sdl4[];  // [B][4]
  const int k0 = blockIdx.y * 4, kk = threadIdx.x >> 6, c = blockIdx.x * 64 + (threadIdx.x & 63);
  for (int i = threadIdx.x; i < B * 4; i += 256) {
    const int bb = i >> 2, j = i & 3;
    sdl4[i] = (k0 + j < K) ? dlogits[(size_t)bb * K + k0 + j] : 0.f;
  }
  __syncthreads();
  const int k = k0 + kk;
  if (k >= K) return;
  float acc = 0.f, accb = 0.f;
  if (c < C) {
#pragma unroll 16
    for (int bb = 0; bb < B; ++bb) acc += sdl4[bb * 4 + kk] * pooled[(size_t)bb * C + c];
    const float v = acc * gscale;
    if constexpr (sizeof(GT) == 2)
      dw[(size_t)k * C + c] = __builtin_bit_cast(uint16_t, (_Float16)v);
    else
      dw[(size_t)k * C + c] = v;
  }
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) {
    for (int bb = 0; bb < B; ++bb) accb += sdl4[bb * 4 + kk];
    accb *= gscale;
    if constexpr (sizeof(GT) == 2)
      db[k] = __builtin_bit_cast(uint16_t, (_Float16)accb);
    else
      db[k] = accb;
  }
}

}  // namespace psx

using namespace psx;

namespace {

template <typename T>
int head_fwd_bwd_t(const void* act, int B, int HW, int C, const float* fcw, const float* fcb, int K,
                   const int* labels, float* pooled, float* dlogits, void* dact, float* loss, int* correct,
                   const HeadBnStats* bst, hipStream_t st) {
  if ((long)K * C > (1L << 18) && C % 64 == 0 && pooled && dlogits) {  // large head: split path
    hipLaunchKernelGGL(head_pool_kernel<T>, dim3(B, (C + 511) / 512), dim3(256), 0, st, (const T*)act, HW, C,
                       pooled, dlogits, (long)B * K);
    // logits: split-K over the C-long dot products (a 2048 x 1000 head at B = 128 is only 64
    // output tiles; 16 splits of 128 channels fill the chip)
    const int ks = det_enabled() ? 1 : (C >= 1024 ? 16 : 4);  // deterministic mode: one add per logit
    hipLaunchKernelGGL((head_gemm_kernel<true, 0>), dim3((K + 63) / 64, (B + 31) / 32, ks), dim3(256), 0, st,
                       pooled, fcw, B, K, C, fcb, dlogits, (uint16_t*)nullptr, HW);
    hipLaunchKernelGGL(head_softmax_kernel, dim3(B), dim3(64), 0, st, dlogits, K, labels, loss, correct,
                       1.f / (float)B, dact ? 1 : 0);
    if (dact)
      hipLaunchKernelGGL((head_gemm_kernel<false, 1, T>), dim3(C / 64, (B + 31) / 32), dim3(256), 0, st, dlogits,
                         fcw, B, C, K, (const float*)nullptr, (float*)nullptr, (T*)dact, HW);
    const int e = (int)hipGetLastError();
    return e ? -e : 0;
  }
  if (K > 1024 || C % 16 || (C > 512 && C % 512)) return -2;
  // >= 16 + 1024 bytes: the deterministic-mode reduction's flag + scratch (bnfin.hpp det_finish)
  const size_t lds = std::max<size_t>((size_t)(C + K + 64) * sizeof(float), 1040);
  const HeadBnStats bs = (bst && dact) ? *bst : HeadBnStats{};
  const DetRed det = bs.part ? det_for(bs.part) : DetRed{};
  if (dact)
    hipLaunchKernelGGL((head_kernel<T, true>), dim3(B), dim3(256), lds, st, (const T*)act, HW, C, fcw, fcb, K,
                       labels, pooled, dlogits, (T*)dact, loss, correct, 1.f / (float)B, bs, det);
  else
    hipLaunchKernelGGL((head_kernel<T, false>), dim3(B), dim3(256), lds, st, (const T*)act, HW, C, fcw, fcb, K,
                       labels, pooled, dlogits, (T*)nullptr, loss, correct, 1.f / (float)B, bs, DetRed{});
  const int e = (int)hipGetLastError();
  return e ? -e : (bs.part ? 1 : 0);
}

}  // namespace

extern "C" {

// bst (nullable, fused path only, needs dact): the BN-backward sums of the consumed layer.
// Returns 1 when they were produced (the caller then skips its bn_bwd_reduce), 0 otherwise.
// f32: act / dact (and bst's operands) are fp32 instead of bf16.
int psx_head_fwd_bwd(const void* act, int B, int HW, int C, const float* fcw, const float* fcb, int K,
                     const int* labels, float* pooled, float* dlogits, void* dact, float* loss, int* correct,
                     const HeadBnStats* bst, int f32, hipStream_t st) {
  return f32 ? head_fwd_bwd_t<float>(act, B, HW, C, fcw, fcb, K, labels, pooled, dlogits, dact, loss, correct, bst, st)
             : head_fwd_bwd_t<uint16_t>(act, B, HW, C, fcw, fcb, K, labels, pooled, dlogits, dact, loss, correct, bst,
                                        st);
}

int psx_head_wgrad(const float* dlogits, const float* pooled, int B, int K, int C, void* dw, void* db, float gscale,
                   int grad_fp16, hipStream_t st) {
  if ((long)K * C <= (1L << 18)) {  // small head: more, smaller workgroups
    const dim3 grid((C + 63) / 64, (K + 3) / 4);
    const size_t lds = (size_t)B * 4 * sizeof(float);
    if (grad_fp16)
      hipLaunchKernelGGL(head_wgrad_small_kernel<uint16_t>, grid, dim3(256), lds, st, dlogits, pooled, B, K, C,
                         (uint16_t*)dw, (uint16_t*)db, gscale);
    else
      hipLaunchKernelGGL(head_wgrad_small_kernel<float>, grid, dim3(256), lds, st, dlogits, pooled, B, K, C,
                         (float*)dw, (float*)db, gscale);
    return (int)hipGetLastError();
  }
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
