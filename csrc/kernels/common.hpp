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
#include <stdlib.h>
#include <string.h>

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

// Developer tuning overrides — the planners' tile sweeps and A/B switches — in ONE environment
// variable, PSX_TUNE="key=value[,key=value...]" (e.g. PSX_TUNE=cv_bm=128,wg_splits=12; a bare
// key means "1"; the Python side reads the same variable, psx/utils/tune.py). Read at every
// planning call (tests and sweeps change it inside one process). Returns the value (a per-thread
// buffer) or nullptr when the key is absent. Production runs set nothing.
static inline const char* tune(const char* key) {
  const char* e = getenv("PSX_TUNE");
  if (!e) return nullptr;
  thread_local char buf[64];
  const size_t kl = strlen(key);
  for (const char* p = e; *p;) {
    const char* comma = strchr(p, ',');
    const size_t len = comma ? (size_t)(comma - p) : strlen(p);
    if (len >= kl && !strncmp(p, key, kl) && (len == kl || p[kl] == '=')) {
      size_t vl = len == kl ? 1 : len - kl - 1;
      if (vl >= sizeof buf) vl = sizeof buf - 1;
      if (len == kl)
        buf[0] = '1';
      else
        memcpy(buf, p + kl + 1, vl);
      buf[vl] = 0;
      return buf;
    }
    if (!comma) break;
    p = comma + 1;
  }
  return nullptr;
}

PSX_DEV float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN preserved as quiet NaN).
// fp32 -> bf16, round to nearest even: gfx950's v_cvt_pk_bf16_f32 (one instruction per pair; the
// integer-arithmetic rounding it replaces was ~7 VALU per value, a third of the bf16 conv epilogue)
// (A/B builds: -D PSX_SW_BF16 keeps the integer version)
typedef __bf16 psx_bf16x2 __attribute__((ext_vector_type(2)));
typedef float psx_f32x2 __attribute__((ext_vector_type(2)));
#ifdef PSX_SW_BF16
PSX_DEV uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
PSX_DEV uint32_t pack_bf2(float lo, float hi) { return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16); }
#else
PSX_DEV uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

PSX_DEV uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((psx_f32x2){lo, hi}, psx_bf16x2));
}
#endif

PSX_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
PSX_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// ---- activation storage types ----------------------------------------------------------
// Every activation-touching kernel is templated on its storage type T: uint16_t (bf16 bits, the
// fast path) or float (fp32, the reference's training precision: src/workers/worker.py:333-348
// runs torch CPU fp32). A 16-byte chunk holds kEPC<T> channels of one pixel and a 128-byte
// implicit-GEMM k-step row kKS<T> of them, so the LDS tile images, the DMA staging and the
// swizzles are byte-identical for both types; only the MFMA and the epilogue conversions differ.
template <typename T>
constexpr int kEPC = 16 / (int)sizeof(T);
template <typename T>
constexpr int kKS = 128 / (int)sizeof(T);

// 8 consecutive channels <-> 8 floats (one u32x4 for bf16, two f32x4 for fp32)
PSX_DEV void ld8(const uint16_t* p, float (&v)[8]) {
  const u32x4 w = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = lo_bf(w[j]);
    v[2 * j + 1] = hi_bf(w[j]);
  }
}
PSX_DEV void ld8(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = a[j];
    v[4 + j] = b[j];
  }
}
// store, then leave in v the value as stored (the BN statistics are taken of the stored tensor)
PSX_DEV void st8(uint16_t* p, float (&v)[8]) {
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = pack_bf2(v[2 * j], v[2 * j + 1]);
  *reinterpret_cast<u32x4*>(p) = o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = lo_bf(o[j]);
    v[2 * j + 1] = hi_bf(o[j]);
  }
}
PSX_DEV void st8(float* p, float (&v)[8]) {
  *reinterpret_cast<f32x4*>(p) = (f32x4){v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = (f32x4){v[4], v[5], v[6], v[7]};
}
// 2 consecutive channels (4-byte bf16 pair / 8-byte fp32 pair)
PSX_DEV void ld2(const uint16_t* p, float& a, float& b) {
  const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
  a = lo_bf(w);
  b = hi_bf(w);
}
PSX_DEV void ld2(const float* p, float& a, float& b) {
  const float2 w = *reinterpret_cast<const float2*>(p);
  a = w.x;
  b = w.y;
}
PSX_DEV void st2(uint16_t* p, float& a, float& b) {
  const uint32_t w = pack_bf2(a, b);
  *reinterpret_cast<uint32_t*>(p) = w;
  a = lo_bf(w);
  b = hi_bf(w);
}
PSX_DEV void st2(float* p, float& a, float& b) { *reinterpret_cast<float2*>(p) = make_float2(a, b); }
PSX_DEV float ld1(const uint16_t* p) { return bf2f(*p); }
PSX_DEV float ld1(const float* p) { return *p; }
PSX_DEV void st1(uint16_t* p, float v) { *p = f2bf(v); }
PSX_DEV void st1(float* p, float v) { *p = v; }

// One 16x16 output tile += A-fragment x B-fragment of one 16-byte chunk per lane (lane l: row
// l & 15, k-group l >> 4). bf16: one v_mfma_f32_16x16x32_bf16. fp32: four v_mfma_f32_16x16x4_f32
// (exact f32, cdna_hip_programming.md §3) — element j of the chunk feeds the j-th, so MFMA j sums
// k = 4*(l>>4) + j over the four lane groups; A and B share the permutation, the sum is the
// same set of products. The fp32 form is issued j-outermost over a wave's tiles (mma_tiles) so
// consecutive MFMAs never chain on one accumulator (40-cycle dependent latency, 32-cycle issue).
PSX_DEV void mma_chunk(f32x4& acc, const u32x4& a, const u32x4& b, uint16_t) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                0, 0, 0);
}
template <int MT, int NT, typename T>
PSX_DEV void mma_tiles(f32x4 (&acc)[MT][NT], const u32x4 (&fa)[MT], const u32x4 (&fb)[NT]) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) mma_chunk(acc[m][n], fa[m], fb[n], uint16_t{});
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(fa[m][j]), __uint_as_float(fb[n][j]),
                                                           acc[m][n], 0, 0, 0);
  }
}

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
