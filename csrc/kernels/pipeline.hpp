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

// (Round 4 measured LDS fragment reads issued through inline asm with exact counted lgkmcnt
// waits: the fp32 step 3.37 -> 3.41 ms, wgrad2f +8-10 %; removed in round 5.)

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
