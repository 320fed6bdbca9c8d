// 3x3 / stride-2 / pad-1 max-pool of the ResNet-50 ImageNet stem (torchvision
// nn.MaxPool2d(3, 2, 1)), NHWC bf16 or fp32 (template T), forward + backward.
//
// Forward keeps, per output element, the window position (0..8) of its maximum in a uint8
// side buffer; backward is a *gather* over the (at most 2x2) windows covering each input
// pixel, so every input gradient is written exactly once (no atomics, deterministic, and the
// same first-max tie rule as PyTorch's CPU/GPU max-pool).
// One thread = 8 channels of one pixel.
#include "common.hpp"

namespace psx {

template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                             uint8_t* __restrict__ arg, int B, int H, int W, int C,
                                                             int OH, int OW) {
  const int cv = C >> 3;
  const long total = (long)B * OH * OW * cv;
  for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int c8 = (int)(t % cv);
    const long p = t / cv;
    const int ow = (int)(p % OW);
    const long q = p / OW;
    const int oh = (int)(q % OH);
    const int b = (int)(q / OH);
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

template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const T* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg,
                                                             T* __restrict__ dx, int B, int H, int W, int C,
                                                             int OH, int OW) {
  const int cv = C >> 3;
  const long total = (long)B * H * W * cv;
  for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int c8 = (int)(t % cv);
    const long p = t / cv;
    const int iw = (int)(p % W);
    const long q = p / W;
    const int ih = (int)(q % H);
    const int b = (int)(q / H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // output (oh, ow) covers ih iff ih = 2*oh - 1 + r, r in [0, 3)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int th = ih + 1 - r;
      if (th & 1) continue;
      const int oh = th >> 1;
      if ((unsigned)oh >= (unsigned)OH) continue;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int tw = iw + 1 - s;
        if (tw & 1) continue;
        const int ow = tw >> 1;
        if ((unsigned)ow >= (unsigned)OW) continue;
        const size_t off = (((size_t)b * OH + oh) * OW + ow) * C + c8 * 8;
        const u32x2 ai = *reinterpret_cast<const u32x2*>(arg + off);
        float g[8];
        ld8(dy + off, g);
        const uint32_t want = (uint32_t)(r * 3 + s);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t a = (ai[e >> 2] >> (8 * (e & 3))) & 0xffu;
          if (a == want) acc[e] += g[e];
        }
      }
    }
    st8(dx + (size_t)p * C + c8 * 8, acc);
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
  const dim3 grid(pool_grid((long)B * H * W * (C / 8)));
  if (f32)
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<float>, grid, dim3(256), 0, st, (const float*)dy, (const uint8_t*)arg,
                       (float*)dx, B, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<uint16_t>, grid, dim3(256), 0, st, (const uint16_t*)dy,
                       (const uint8_t*)arg, (uint16_t*)dx, B, H, W, C, OH, OW);
  return (int)hipGetLastError();
}

}  // extern "C"
