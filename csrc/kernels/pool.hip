// 3x3 / stride-2 / pad-1 max-pool of the ResNet-50 ImageNet stem (torchvision
// nn.MaxPool2d(3, 2, 1)), NHWC bf16 or fp32 (template T), forward + backward.
//
// Forward keeps, per output element, the window position (0..8) of its maximum in a uint8
// side buffer; backward is a *gather* over the (at most 2x2) windows covering each input
// pixel, so every input gradient is written exactly once (no atomics, deterministic, and the
// same first-max tie rule as PyTorch's CPU/GPU max-pool).
// Forward: one thread = 8 channels of one output pixel.
#include "common.hpp"

namespace psx {

template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                             uint8_t* __restrict__ arg, int B, int H, int W, int C,
                                                             int OH, int OW) {
  const int cv = C >> 3;
  const int total = B * OH * OW * cv;  // < 2^31 (host check): 32-bit index math
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    const int c8 = t % cv, p = t / cv;
    const int ow = p % OW, q = p / OW;
    const int oh = q % OH, b = q / OH;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ih = oh * 2 - 1 + r;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int iw = ow * 2 - 1 + s;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[8];
        ld8(x + (((size_t)b * H + ih) * W + iw) * C + c8 * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = v[e];
          if (f > best[e]) {  // strict: first maximum in window order wins
            best[e] = f;
            bi[e] = (uint8_t)(r * 3 + s);
          }
        }
      }
    }
    u32x2 ai;
    ai[0] = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    ai[1] = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    const size_t off = (size_t)p * C + c8 * 8;
    st8(y + off, best);
    *reinterpret_cast<u32x2*>(arg + off) = ai;
  }
}

// Backward: one thread = 8 channels of one 2x2 block of input pixels (2m + dh, 2n + dw). The
// windows covering the block are those of the outputs (m + doh, n + dow), doh, dow in {0, 1}, and
// input row 2m + dh is tap r = dh + 1 - 2 doh of output row m + doh — known at compile time per
// (dh, doh), so the gather has no data-dependent branches: 4 (dy, arg) chunk loads, 4 dx stores.
// (A thread per input pixel with 64-bit index math and parity branches took 474 us on the
// ResNet-50 stem at batch 128, ~4.5x its 540 MB traffic floor.)
template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const T* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg,
                                                             T* __restrict__ dx, int B, int H, int W, int C,
                                                             int OH, int OW) {
  const int cv = C >> 3, BH = (H + 1) >> 1, BW = (W + 1) >> 1;
  const int total = B * BH * BW * cv;  // < 2^31 (host check)
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    const int c8 = t % cv, p = t / cv;
    const int n = p % BW, q = p / BW;
    const int m = q % BH, b = q / BH;
    float acc[2][2][8];
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[dh][dw][e] = 0.f;
#pragma unroll
    for (int doh = 0; doh < 2; ++doh) {
      const int oh = m + doh;
      if (oh >= OH) continue;
#pragma unroll
      for (int dow = 0; dow < 2; ++dow) {
        const int ow = n + dow;
        if (ow >= OW) continue;
        const size_t off = (((size_t)b * OH + oh) * OW + ow) * C + c8 * 8;
        const u32x2 ai = *reinterpret_cast<const u32x2*>(arg + off);
        float g[8];
        ld8(dy + off, g);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const int r = dh + 1 - 2 * doh;
          if (r < 0) continue;  // compile-time
#pragma unroll
          for (int dw = 0; dw < 2; ++dw) {
            const int sx = dw + 1 - 2 * dow;
            if (sx < 0) continue;  // compile-time
            const uint32_t want = (uint32_t)(r * 3 + sx);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t a = (ai[e >> 2] >> (8 * (e & 3))) & 0xffu;
              if (a == want) acc[dh][dw][e] += g[e];
            }
          }
        }
      }
    }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int ih = 2 * m + dh;
      if (ih >= H) continue;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int iw = 2 * n + dw;
        if (iw >= W) continue;
        st8(dx + (((size_t)b * H + ih) * W + iw) * C + c8 * 8, acc[dh][dw]);
      }
    }
  }
}

}  // namespace psx

using namespace psx;

static int pool_grid(long work) {
  long g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

extern "C" {

int psx_maxpool3s2_fwd(const void* x, void* y, void* arg, int B, int H, int W, int C, int f32, hipStream_t st) {
  if (C % 8) return -2;
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  // the grid-stride index t < total + grid * 256 must stay below 2^31 (32-bit index math)
  if ((long)B * OH * OW * (C / 8) + 8192L * 256 >= (1L << 31)) return -2;
  const dim3 grid(pool_grid((long)B * OH * OW * (C / 8)));
  if (f32)
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<float>, grid, dim3(256), 0, st, (const float*)x, (float*)y,
                       (uint8_t*)arg, B, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<uint16_t>, grid, dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)y,
                       (uint8_t*)arg, B, H, W, C, OH, OW);
  return (int)hipGetLastError();
}

int psx_maxpool3s2_bwd(const void* dy, const void* arg, void* dx, int B, int H, int W, int C, int f32,
                       hipStream_t st) {
  if (C % 8) return -2;
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const long blocks = (long)B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  if (blocks + 8192L * 256 >= (1L << 31)) return -2;  // grid-stride t stays < 2^31
  const dim3 grid(pool_grid(blocks));
  if (f32)
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<float>, grid, dim3(256), 0, st, (const float*)dy, (const uint8_t*)arg,
                       (float*)dx, B, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<uint16_t>, grid, dim3(256), 0, st, (const uint16_t*)dy,
                       (const uint8_t*)arg, (uint16_t*)dx, B, H, W, C, OH, OW);
  return (int)hipGetLastError();
}

}  // extern "C"
