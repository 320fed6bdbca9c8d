// Device-side data pipeline: CIFAR-shaped uint8 dataset resident in HBM, per-step batch
// gather + RandomCrop(32, padding=4) + RandomHorizontalFlip + Normalize(mean, std) fused into
// one kernel that writes the network input directly as NHWC bf16 with channels padded 3 -> 8,
// or as NHWC fp32 padded 3 -> 4 (the fp32 path: one 16-byte chunk per pixel either way).
//
// Replaces the torchvision transform pipeline + DataLoader worker processes of the reference
// (reference: src/workers/worker.py:145-155,182-197; baseline/baseline_training.py:13-23).
// The synthetic generator produces a learnable, class-conditioned CIFAR-100-shaped dataset
// (there is no network access for the real dataset; utils/data.py can load real CIFAR binaries).
#include "common.hpp"

namespace psx {

PSX_DEV uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
PSX_DEV uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return hash32(a ^ hash32(b ^ hash32(c + 0x9e3779b9u))); }

// images: [N][H][W][3] uint8, labels: [N] int32. Class prototypes are low-frequency colour
// patterns fixed by `seed`; each sample = prototype + per-pixel noise, so the task is learnable.
// `offset` selects a disjoint sample range (train set offset 0, test set a large offset) over
// the same class prototypes.
__global__ void synth_gen_kernel(uint8_t* __restrict__ img, int* __restrict__ labels, int N, int H, int W,
                                 int classes, uint32_t seed, uint32_t offset) {
  const long total = (long)N * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i / (H * W));
    const int hw = (int)(i - (long)n * H * W);
    const int h = hw / W, w = hw - (hw / W) * W;
    const int y = (int)(hash3(seed, (uint32_t)n + offset, 77u) % (uint32_t)classes);
    if (hw == 0) labels[n] = y;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      // prototype: sum of two class-specific sinusoid-like integer patterns
      const uint32_t hp = hash3(seed ^ 0xabcdu, (uint32_t)y, (uint32_t)c);
      const int fx = 1 + (hp & 3), fy = 1 + ((hp >> 2) & 3), ph = (hp >> 4) & 31;
      const int tri_x = ((h * fx + ph) & 31), tri_y = ((w * fy + (ph >> 1)) & 31);
      const int proto = ((tri_x < 16 ? tri_x : 31 - tri_x) + (tri_y < 16 ? tri_y : 31 - tri_y)) * 8;  // 0..240
      const int noise = (int)(hash3(seed + offset, (uint32_t)i, (uint32_t)c) & 63) - 32;
      int v = proto + noise;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      img[i * 3 + c] = (uint8_t)v;
    }
  }
}

struct AugArgs {
  const uint8_t* img;  // [N][H][W][3]
  const int* labels;   // [N]
  const int* index;    // [B] sample indices of this batch
  void* out;           // [B][H][W][8] bf16 or [B][H][W][4] fp32 (f32)
  int* out_labels;     // [B]
  int B, H, W, pad;
  uint32_t seed;
  const unsigned* step;  // device scalar, so a captured graph sees the live step counter
  int train;           // 1: random crop + flip, 0: centre (eval transform)
  int f32;
  float mean[3], inv_std[3];
  uint32_t* zero0;  // optional 32-bit words zeroed by the same launch (the step's BN statistic
  long nzero0;      // slots and accuracy counter: two fewer launches per step)
  uint32_t* zero1;
  long nzero1;
  const uint32_t* copy_src;  // optional word copy of the same launch: the BN statistic shifts
  uint32_t* copy_dst;        // (bnfin.hpp BnFin::sshift) the previous step's finalizes wrote
  long ncopy;
};

__global__ __launch_bounds__(256) void augment_kernel(AugArgs a) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.nzero0; i += stride) a.zero0[i] = 0u;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.nzero1; i += stride) a.zero1[i] = 0u;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.ncopy; i += stride) a.copy_dst[i] = a.copy_src[i];
  const long total = (long)a.B * a.H * a.W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / (a.H * a.W));
    const int hw = (int)(i - (long)b * a.H * a.W);
    const int h = hw / a.W, w = hw - h * a.W;
    const int n = a.index[b];
    int dy = 0, dx = 0;
    bool flip = false;
    if (a.train) {
      const uint32_t r = hash3(a.seed, *a.step, (uint32_t)b);
      dy = (int)(r % (uint32_t)(2 * a.pad + 1)) - a.pad;
      dx = (int)((r >> 8) % (uint32_t)(2 * a.pad + 1)) - a.pad;
      flip = (r >> 20) & 1;
    }
    if (hw == 0) a.out_labels[b] = a.labels[n];
    const int sw = flip ? (a.W - 1 - w) : w;  // flip applied after the crop, as torchvision
    const int ih = h + dy, iw = sw + dx;
    float v[3] = {0.f, 0.f, 0.f};
    const bool in = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float px = in ? (float)a.img[(((long)n * a.H + ih) * a.W + iw) * 3 + c] * (1.f / 255.f) : 0.f;
      v[c] = (px - a.mean[c]) * a.inv_std[c];
    }
    if (a.f32) {
      reinterpret_cast<f32x4*>(a.out)[i] = (f32x4){v[0], v[1], v[2], 0.f};
    } else {
      u32x4 o;
      o[0] = pack_bf2(v[0], v[1]);
      o[1] = pack_bf2(v[2], 0.f);
      o[2] = 0u;
      o[3] = 0u;
      reinterpret_cast<u32x4*>(a.out)[i] = o;
    }
  }
}

// NCHW fp32 (e.g. a torch batch) -> NHWC (bf16 or fp32) with channel padding to Cp
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int H, int W,
                                    int Cp) {
  const long total = (long)N * H * W * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    long t = i / Cp;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const float v = c < C ? x[(((long)n * C + c) * H + h) * W + w] : 0.f;
    st1(y + i, v);
  }
}

}  // namespace psx

using namespace psx;

extern "C" {

int psx_synth_gen(void* img, int* labels, int N, int H, int W, int classes, unsigned seed, unsigned offset,
                  hipStream_t st) {
  long total = (long)N * H * W;
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(synth_gen_kernel, dim3((unsigned)g), dim3(256), 0, st, (uint8_t*)img, labels, N, H, W, classes,
                     (uint32_t)seed, (uint32_t)offset);
  return (int)hipGetLastError();
}

int psx_augment(const void* img, const int* labels, const int* index, void* out, int* out_labels, int B, int H, int W,
                int pad, unsigned seed, const unsigned* step, int train, const float* mean3, const float* std3,
                void* zero0, long nzero0, void* zero1, long nzero1, const void* copy_src, void* copy_dst, long ncopy,
                int f32, hipStream_t st) {
  AugArgs a{};
  a.copy_src = (const uint32_t*)copy_src;
  a.copy_dst = (uint32_t*)copy_dst;
  a.ncopy = copy_src && copy_dst ? ncopy : 0;
  a.zero0 = (uint32_t*)zero0;
  a.nzero0 = zero0 ? nzero0 : 0;
  a.zero1 = (uint32_t*)zero1;
  a.nzero1 = zero1 ? nzero1 : 0;
  a.img = (const uint8_t*)img;
  a.labels = labels;
  a.index = index;
  a.out = out;
  a.f32 = f32;
  a.out_labels = out_labels;
  a.B = B; a.H = H; a.W = W; a.pad = pad;
  a.seed = seed; a.step = step; a.train = train;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = mean3[c];
    a.inv_std[c] = 1.f / std3[c];
  }
  long total = (long)B * H * W;
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(augment_kernel, dim3((unsigned)g), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

int psx_nchw_to_nhwc(const float* x, void* y, int N, int C, int H, int W, int Cp, int f32, hipStream_t st) {
  long total = (long)N * H * W * Cp;
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  if (f32)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3((unsigned)g), dim3(256), 0, st, x, (float*)y, N, C, H, W, Cp);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<uint16_t>, dim3((unsigned)g), dim3(256), 0, st, x, (uint16_t*)y, N, C, H,
                       W, Cp);
  return (int)hipGetLastError();
}

}  // extern "C"
