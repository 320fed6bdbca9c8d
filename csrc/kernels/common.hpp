// Shared device helpers for the psx CDNA4 (gfx950) kernel library.
//
// Conventions used by every kernel in csrc/kernels:
//   * activations are NHWC bf16 (channels padded to a multiple of 8 so a 16-byte
//     chunk is always 8 channels of one pixel),
//   * conv weights used for compute are bf16 "KRSC" rows (GEMM-K contiguous),
//   * master parameters / optimizer state are fp32 in the reference state_dict
//     layout (OIHW), see models/layout.py,
//   * wave = 64 lanes; every block size is a multiple of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PSX_DEV __device__ __forceinline__

// Cross-workgroup per-channel reductions (BN statistics, BN backward sums) are accumulated with
// fp32 atomics into this many slot rows; consumers sum the slots in a fixed order. 8 rows keep
// the atomic contention of a 1024-workgroup conv epilogue low while letting every workgroup of
// the consuming BN pass re-derive the affine from the slots itself (the folded finalize,
// bnfin.hpp bn_fin_lds): 1.999 vs 2.019 ms/step against 32 rows + separate finalize kernels.
#ifndef PSX_STAT_SLOTS
#define PSX_STAT_SLOTS 8
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace psx {

PSX_DEV float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN preserved as quiet NaN).
PSX_DEV uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

PSX_DEV uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

PSX_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
PSX_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

PSX_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
PSX_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of NT threads (NT multiple of 64); `red` must hold NT/64 floats.
template <int NT>
PSX_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 'XCD swizzle must be
// bijective'): consecutive logical tiles land on the same XCD so neighbouring tiles that
// share operand panels hit the same L2. Speed only; correctness never depends on it.
PSX_DEV int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

}  // namespace psx
