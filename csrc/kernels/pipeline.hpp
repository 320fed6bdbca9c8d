// Shared building blocks of the LDS-DMA pipelined kernels (conv_v2.hip, wgrad_v2.hip).
#pragma once
#include <type_traits>

#include "common.hpp"

namespace psx {

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// One wave-instruction moves 64 x 16 B from per-lane global addresses into 1 KiB of LDS at a
// wave-uniform base (lane l lands at base + 16 l) — global_load_lds_dwordx4.
PSX_DEV void glds16(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds, 16, 0, 0);
}

// Counted wait on this wave's outstanding vector-memory ops (LDS-DMA included).
template <int N>
PSX_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS reads outside hipcc's waitcnt tracking. hipcc puts an s_waitcnt lgkmcnt(0) in front of
// every MFMA group that consumes LDS fragments, so a prefetch of the next group's fragments is
// waited for too and its latency is exposed each time; reads issued through these wrappers are
// invisible to that pass, and the kernel waits for exactly the ones a group consumes with a
// counted lgkm_wait<N> (LDS operations retire in order; no scalar loads may be in flight, they
// share the counter). The counter is 4 bits: more than 15 reads in flight stall the issue, and
// waits are capped at 15, which stays correct (in-order retirement).
// PSX_CONV_ASMRD = 0 builds the mainloops with plain LDS loads (A/B variant).
#ifndef PSX_CONV_ASMRD
#define PSX_CONV_ASMRD 0
#endif

typedef __attribute__((address_space(3))) unsigned char lds_u8;

PSX_DEV unsigned lds_off(const void* p) { return (unsigned)(size_t)(const lds_u8*)p; }

PSX_DEV float ds_read32(unsigned off) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(off));
  return v;
}

PSX_DEV u32x4 ds_read128u(unsigned off) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(off));
  return v;
}

template <int N>
PSX_DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N > 15 ? 15 : N) : "memory");
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
PSX_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Division by a runtime-invariant divisor via multiply-high (Granlund-Montgomery), valid for
// 0 <= n < 2^31 and 1 <= d < 2^31. Host computes (m, l) once per launch.
struct FastDiv {
  unsigned m;
  int l;
  int d;
};

static inline FastDiv make_fastdiv(int d) {
  FastDiv f;
  f.d = d;
  int l = 0;
  while ((1u << l) < (unsigned)d) ++l;
  f.l = l;
  f.m = (unsigned)((((unsigned long long)1 << 32) * (((unsigned long long)1 << l) - (unsigned)d)) / (unsigned)d + 1);
  return f;
}

PSX_DEV int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.l);
}

}  // namespace psx
