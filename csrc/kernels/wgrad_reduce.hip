// Weight-gradient split-K reduction: the split slabs of the implicit-GEMM weight-gradient
// kernels (wgrad_v2.hip) are summed in a fixed order, permuted from the GEMM layout
// (oc, r, s, c) to the reference OIHW layout (oc, c, r, s) with the channel padding dropped,
// scaled, and written straight into the gradient wire (fp16 codec or fp32). The reference's
// gradients come out of autograd (src/workers/worker.py:345) and are cast to fp16 for the push
// (worker.py:264-268); here that cast is this kernel's store.
//   wgrad_reduce_kernel        any R*S / channel count (one thread per partial column)
//   wgrad_reduce2_kernel       R*S <= 49, IC % 16 == 0: workgroup = (oc, channel chunk) x all taps,
//                              16-byte loads split over slot groups, LDS transpose to contiguous
//                              OIHW runs
//   wgrad_reduce2_batch_kernel the layers of one residual block in ONE launch (engine.py
//                              _flush_reduces)
#include <stdlib.h>

#include "common.hpp"

namespace psx {
// Sum the split-K partials, permute (oc, r, s, c) -> reference OIHW (oc, c, r, s), drop the
// channel padding and emit the gradient straight into the wire buffer (fp16 codec or fp32).
// Block = 4 waves; each lane owns 4 consecutive partial columns (16-byte loads), the waves split
// the split-K slabs 4 ways (fixed order => deterministic) and combine through LDS.
// Pre-pass of a small layer with many splits (the stem: 64 x 64 columns = 16 workgroups of the
// final reduce over 256 slabs, latency-bound at ~70 us): workgroup (column block, slab group)
// sums the kPre slabs of its group in fixed order and stores the sum over the group's FIRST slab,
// which no other workgroup reads; the final reduce then walks every kPre-th slab.
constexpr int kPre = 16;

__global__ __launch_bounds__(256) void wgrad_presum_kernel(float* __restrict__ part, int splits, size_t slab) {
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t base = (size_t)blockIdx.x * 256 + lane * 4;
  const int s0 = blockIdx.y * kPre;
  f32x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int sp = s0 + g + 4 * u;
    acc[u] = sp < splits ? *reinterpret_cast<const f32x4*>(part + (size_t)sp * slab + base)
                         : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  red[g][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (g != 0) return;
  *reinterpret_cast<f32x4*>(part + (size_t)s0 * slab + base) =
      (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int OC,
                                                           int Kg, int Cin, int IC, int R, int S, float scale,
                                                           OutT* __restrict__ out, int sstride) {
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t slab = (size_t)OC * Kg * sstride;  // every sstride-th slab (after the pre-pass)
  const size_t base = (size_t)blockIdx.x * 256 + lane * 4;
  // the 4 waves split the slabs 4 ways; 8 independent 16-byte loads in flight per lane (the
  // reduce is bandwidth work, and with as few as 144 workgroups for a 64x576 layer it is
  // latency-bound unless each lane keeps several slab loads outstanding)
  f32x4 acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int sp = g;
  for (; sp + 28 < splits; sp += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += *reinterpret_cast<const f32x4*>(part + (size_t)(sp + 4 * u) * slab + base);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (sp + 4 * u < splits) acc[u] += *reinterpret_cast<const f32x4*>(part + (size_t)(sp + 4 * u) * slab + base);
  red[g][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (g != 0) return;
  const f32x4 v = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  const int RS = R * S;
  const int oc = (int)(base / Kg);
  int k = (int)(base - (size_t)oc * Kg);  // the 4 columns never straddle a row (Kg % 64 == 0)
  int tap = k / IC, c = k - tap * IC;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (tap < RS && c < Cin) {
      const float val = v[e] * scale;
      const size_t o = ((size_t)oc * Cin + c) * RS + tap;
      if constexpr (sizeof(OutT) == 2) {
        out[o] = __builtin_bit_cast(uint16_t, (_Float16)val);
      } else {
        out[o] = val;
      }
    }
    if (++c == IC) {
      c = 0;
      ++tap;
    }
  }
}

// v2 mapping: workgroup = (output channel oc, chunk of CW input channels) x all R*S taps, so
// its OIHW output [oc][c0..c0+CW)[taps] is one contiguous run (written from an LDS transpose).
// Threads = (item, split group): an item is 4 channels of one tap (one 16-byte load per split),
// G groups take splits g, g+G, ... so a layer with few items still keeps 256 lanes x several
// 16-byte loads in flight (the partials are 2-16 MB per layer; the v1 mapping was latency-bound
// at ~1 TB/s with 4-byte loads and 64 workgroups on layer1).
template <typename OutT>
PSX_DEV void wgrad_reduce2_tile(const float* __restrict__ part, int splits, int Kg, int Cin, int IC, int RS, int CW,
                                float scale, OutT* __restrict__ out, int oc, int c0, int OC, float4* acc,
                                float* tile) {
  const int q = CW >> 2;           // channel quads per tap
  const int items = RS * q;
  const int G = items >= 256 ? 1 : min(splits, 256 / items);
  const size_t slab = (size_t)OC * Kg;
  const float* row = part + (size_t)oc * Kg + c0;
  for (int base = 0; base < items; base += 256 / G) {
    const int t = threadIdx.x;
    const int per = 256 / G;            // items handled per pass
    const int it = base + t % per, g = t / per;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool live = g < G && t % per + base < items && it < items;
    if (live) {
      const int tap = it / q, cq = it % q;
      const float4* src = reinterpret_cast<const float4*>(row + (size_t)tap * IC + cq * 4);
      const size_t st4 = slab / 4;
      // 8 independent 16-byte loads in flight per thread: a 3x3 layer's workgroup (144 items, G = 1)
      // walks all splits itself, and 4 per round trip left the batched reduction latency-bound
      // (ResNet-50: 64-split 3x3 layers, 16 round trips per workgroup)
      int sp = g;
      f32x4 acc8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc8[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
      const f32x4* src4 = reinterpret_cast<const f32x4*>(src);
      for (; sp + 7 * G < splits; sp += 8 * G) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src4[(size_t)(sp + u * G) * st4];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc8[u] += v[u];
      }
      for (; sp < splits; sp += G) acc8[0] += src4[(size_t)sp * st4];
      const f32x4 t4 = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
      s = make_float4(t4[0], t4[1], t4[2], t4[3]);
    }
    acc[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < per && base + threadIdx.x < items) {
      float4 r = acc[threadIdx.x];
      for (int gg = 1; gg < G; ++gg) {
        const float4 v = acc[gg * per + threadIdx.x];
        r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
      }
      const int it2 = base + threadIdx.x, tap = it2 / q, c = (it2 % q) * 4;
      tile[(c + 0) * RS + tap] = r.x;
      tile[(c + 1) * RS + tap] = r.y;
      tile[(c + 2) * RS + tap] = r.z;
      tile[(c + 3) * RS + tap] = r.w;
    }
    __syncthreads();
  }
  const int cv = min(CW, Cin - c0);  // valid (unpadded) input channels of this chunk
  if (cv <= 0) return;
  OutT* dst = out + ((size_t)oc * Cin + c0) * RS;
  for (int j = threadIdx.x; j < cv * RS; j += 256) {
    const float val = tile[j] * scale;
    if constexpr (sizeof(OutT) == 2) {
      dst[j] = __builtin_bit_cast(uint16_t, (_Float16)val);
    } else {
      dst[j] = val;
    }
  }
}

template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce2_kernel(const float* __restrict__ part, int splits, int Kg,
                                                            int Cin, int IC, int RS, int CW, float scale,
                                                            OutT* __restrict__ out) {
  __shared__ float4 acc[256];
  __shared__ float tile[64 * 49];  // [c][tap], CW*RS <= 64*49
  wgrad_reduce2_tile<OutT>(part, splits, Kg, Cin, IC, RS, CW, scale, out, blockIdx.x, blockIdx.y * CW, gridDim.x, acc,
                           tile);
}

// Several layers' reductions in one launch (the weight gradients of one residual block are
// reduced together at the end of its backward): flat grid, desc j owns blocks [blk0, blk0 + OC*IC/CW).
constexpr int kWrMax = 4;
struct WrDesc {
  const float* part;
  void* out;
  int splits, Kg, Cin, IC, RS, CW, OC, blk0;
};
struct WrBatch {
  WrDesc d[kWrMax];
  int n;
  float scale;
};

template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce2_batch_kernel(WrBatch b) {
  __shared__ float4 acc[256];
  __shared__ float tile[64 * 49];
  int j = 0;
  while (j + 1 < b.n && b.d[j + 1].blk0 <= (int)blockIdx.x) ++j;
  const WrDesc& d = b.d[j];
  const int local = blockIdx.x - d.blk0;
  const int oc = local % d.OC, c0 = (local / d.OC) * d.CW;
  wgrad_reduce2_tile<OutT>(d.part, d.splits, d.Kg, d.Cin, d.IC, d.RS, d.CW, b.scale, (OutT*)d.out, oc, c0, d.OC, acc,
                           tile);
}

}  // namespace psx

// ------------------------------------------------------------------------------------
// C ABI launchers
// ------------------------------------------------------------------------------------

using namespace psx;

extern "C" {

static int reduce2_cw(int OC, int IC) {
  // chunk width: widest of 64/32/16 channels that still gives >= 1024 workgroups
  int CW = IC < 64 ? IC : 64;
  while (CW > 16 && (long)OC * (IC / CW) < 1024) CW >>= 1;
  return CW;
}

// n <= 4 layers: part/out/splits/OC/Kg/Cin/IC/RS arrays of n entries (host memory); every layer
// needs the v2 reduce (R*S <= 49, IC % 16 == 0). One launch for all of them.
int psx_wgrad_reduce_batch(int n, const float* const* part, void* const* out, const int* splits, const int* OC,
                           const int* Kg, const int* Cin, const int* IC, const int* RS, float scale, int out_fp16,
                           hipStream_t st) {
  if (n < 1 || n > kWrMax) return -2;
  WrBatch b{};
  b.n = n;
  b.scale = scale;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    if (RS[i] > 49 || IC[i] % 16) return -3;
    const int CW = reduce2_cw(OC[i], IC[i]);
    b.d[i] = WrDesc{part[i], out[i], splits[i], Kg[i], Cin[i], IC[i], RS[i], CW, OC[i], blk};
    blk += OC[i] * (IC[i] / CW);
  }
  if (out_fp16)
    hipLaunchKernelGGL(wgrad_reduce2_batch_kernel<uint16_t>, dim3(blk), dim3(256), 0, st, b);
  else
    hipLaunchKernelGGL(wgrad_reduce2_batch_kernel<float>, dim3(blk), dim3(256), 0, st, b);
  return (int)hipGetLastError();
}

int psx_wgrad_reduce(const float* part, int splits, int OC, int Kg, int Cin, int IC, int R, int S, float scale,
                     void* out, int out_fp16, hipStream_t st) {
  if (R * S <= 49 && IC % 16 == 0) {
    const int CW = reduce2_cw(OC, IC);
    const dim3 grid(OC, IC / CW);
    if (out_fp16)
      hipLaunchKernelGGL(wgrad_reduce2_kernel<uint16_t>, grid, dim3(256), 0, st, part, splits, Kg, Cin, IC, R * S,
                         CW, scale, (uint16_t*)out);
    else
      hipLaunchKernelGGL(wgrad_reduce2_kernel<float>, grid, dim3(256), 0, st, part, splits, Kg, Cin, IC, R * S, CW,
                         scale, (float*)out);
    return (int)hipGetLastError();
  }
  if (((long)OC * Kg) % 256) return -2;
  const int grid = (int)(((long)OC * Kg) / 256);
  int sstride = 1;
  if (grid < 128 && splits > 2 * kPre) {
    // few columns, many slabs: spread the slab sum over grid x splits/kPre workgroups first
    const int groups = (splits + kPre - 1) / kPre;
    hipLaunchKernelGGL(wgrad_presum_kernel, dim3(grid, groups), dim3(256), 0, st, const_cast<float*>(part), splits,
                       (size_t)OC * Kg);
    splits = groups;
    sstride = kPre;
  }
  if (out_fp16)
    hipLaunchKernelGGL(wgrad_reduce_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, part, splits, OC, Kg, Cin, IC,
                       R, S, scale, (uint16_t*)out, sstride);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<float>, dim3(grid), dim3(256), 0, st, part, splits, OC, Kg, Cin, IC, R,
                       S, scale, (float*)out, sstride);
  return (int)hipGetLastError();
}

}  // extern "C"
