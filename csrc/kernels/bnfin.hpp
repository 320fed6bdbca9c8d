// In-launch BatchNorm finalize: the last workgroup of the kernel that produced a BN layer's
// per-slot partial sums turns them into the layer's affine (forward) or backward coefficients,
// replacing a separate one-block finalize launch per BN layer (40 launches per ResNet-18 step).
//
// Hand-off (cdna_hip_programming.md §6 Guideline 16, counter form; payload = agent-scope
// atomic adds): every wave drains its stat atomics (s_waitcnt vmcnt(0)), workgroup barrier,
// lane 0 draws a relaxed agent-scope ticket; the workgroup drawing nblocks-1 does an
// agent-scope acquire fence + drain, barrier, then loads the slot rows. No release fence: the
// payload is float atomics, which execute at the memory side (MI355X_MICROARCH.md §Global
// float atomics) and leave no dirty L2 line to write back — a per-workgroup buffer_wbl2 here
// measured +0.9 ms per ResNet-18 step. Correct for any placement of the producers over XCDs.
// Counters live in the slot buffer the engine zeroes once per step.
// The flag and the reduction scratch reuse the caller's dynamic-LDS array (no second
// __shared__ object beside an LDS-DMA staging array).
#pragma once
#include "common.hpp"

namespace psx {

struct BnFin {  // forward: batch statistics -> affine (+ running statistics)
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  float* scale;
  float* shift;
  float* save_mean;
  float* save_invstd;
  unsigned* counter;
  float count, eps, momentum;
  int C;
  // Shifted sums (nullable = 0): the producer summed (x - k_c) and (x - k_c)^2 with k = sshift,
  // the previous step's batch mean, so the variance E[(x-k)^2] - E[x-k]^2 never cancels two
  // large numbers (|mean| >> std); the finalize writes this batch's mean to sshift_next, which
  // becomes the next step's sshift (engine.py: copied by the next step's first launch).
  const float* sshift;
  float* sshift_next;
  int det;  // the slot rows hold exact fixed-point pairs (deterministic mode; set by the launcher)
};

// batch moments from the (shifted) sums: mean = k + s/n, var = ss/n - (s/n)^2 (biased)
PSX_DEV void bn_moments(double s, double ss, float count, float k, double& mean, double& var) {
  const double m1 = s / count;
  mean = (double)k + m1;
  var = ss / count - m1 * m1;
  if (var < 0.0) var = 0.0;
}

struct BnBwdFin {  // backward: sum(dz), sum(dz*xhat) -> coefficients + dgamma/dbeta
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* coef;
  void* dgamma;
  void* dbeta;
  unsigned* counter;
  float count, gscale;
  int C, grad_fp16;
  int det;  // the slot rows hold exact fixed-point pairs (deterministic mode; set by the launcher)
};

// All threads of the block call this after issuing their stat atomics. Returns true in the
// last-arriving block only (after its acquire).
PSX_DEV bool last_block_arrive(unsigned* counter, unsigned nblocks, unsigned char* lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  volatile int* flag = reinterpret_cast<volatile int*>(lds);
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == nblocks - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __syncthreads();  // the flag word is scratch below
  return last;
}

// ---------------------------------------------------------------------------------------
// Deterministic mode (psx_set_deterministic, bn.hip): every producer of per-channel sums adds its
// workgroup partials as exact fixed-point numbers instead of floats. A partial v (fp32) becomes
// the 104-bit value round(v * 2^64) split into hi = floor(v * 2^24) and lo = frac(v * 2^24) *
// 2^40, each added with a 64-bit integer atomic: integer addition is associative, so the sums —
// and with them every BN statistic and the whole step — are the same bits whatever order the
// workgroups arrive in. The exact range is |sum| < 2^39 with an absolute resolution of 2^-64 (a
// partial below 2^-41 in magnitude truncates its lowest bits, deterministically); a non-finite or
// out-of-range partial poisons its entry (kFixPoison below: the statistic reads NaN).
// The pairs live IN the slot buffer: entry i of the float layout [PSX_STAT_SLOTS][NS][C] becomes
// the 16-byte pair at byte 16 i (the engine sizes its slot buffers 4x in this mode; they are
// zeroed every step with the float ones), so producers spread over the same 8 slot rows and no
// launch needs an arrival counter or a conversion pass: the consumers (the finalize paths below,
// the Winograd kernels' folded finalizes) sum the slots' pairs as integers and convert once.
// (A first version kept rotating per-launch accumulators and converted in the launch's last
// workgroup: the arrival + conversion tail cost 0.27 ms of the 0.65 ms its mode added to the
// ResNet-18 fp32 step, profiles/r5_deterministic_ab.jsonl.)
struct DetRed {
  unsigned long long* fix;  // nullptr: deterministic mode off; else the slot buffer's base (pairs)
};

// Poison: a partial that is not finite or is too large for the exact range (|v| >= 2^38: a
// double -> int64 conversion past 2^63 is undefined, and a channel sum past 2^39 would wrap) sets
// bit 63 of the pair's low word instead of being added. Legitimate low words stay below 2^56 (each
// add < 2^40, fewer than 2^16 adds per entry), so the bit is sticky under the other adds and every
// reader (slot_sum, slot_sum_rt, ops/kernels.py det_slot_values) turns a poisoned entry into NaN —
// as the float-atomic mode would let an Inf / NaN through to the statistics.
constexpr unsigned long long kFixPoison = 1ull << 63;

PSX_DEV void fix_add(unsigned long long* p, float v) {
  if (!(fabsf(v) < 274877906944.0f)) {  // 2^38; false for NaN too
    atomicOr(p + 1, kFixPoison);
    return;
  }
  const double x = (double)v * 16777216.0;  // 2^24: exact
  const double h = floor(x);
  const long long hi = (long long)h;
  const unsigned long long lo = (unsigned long long)((x - h) * 1099511627776.0);  // 2^40: exact above 2^-41
  atomicAdd(p, (unsigned long long)hi);
  atomicAdd(p + 1, lo);
}

// sum of fixed-point pairs -> double (the one rounding of the whole reduction); NaN when poisoned
PSX_DEV double fix_value(long long H, unsigned long long L, bool poison = false) {
  if (poison) return __builtin_nan("");
  return (double)H * (1.0 / 16777216.0) + (double)L * 5.421010862427522e-20;  // 2^-24, 2^-64
}

// One per-channel partial into slot row `dst` (a row of the launch's slot buffer) at index `off`:
// a float atomic, or in deterministic mode the fixed-point pair of the same float-layout index.
PSX_DEV void stat_add(const DetRed& d, float* dst, int off, float v) {
  if (d.fix) {
    const size_t i = (size_t)(dst - reinterpret_cast<float*>(d.fix)) + off;
    fix_add(d.fix + 2 * i, v);
  } else {
    atomicAdd(dst + off, v);
  }
}

// Sum over T slots of float-layout entry i0 + t * stride: doubles of the float slots, or the
// exact integer sum of the fixed-point pairs (det). All loads issued back to back.
template <int T>
PSX_DEV double slot_sum(const float* part, size_t i0, size_t stride, bool det) {
  if (det) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(part);
    long long H = 0;
    unsigned long long L = 0, P = 0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const size_t i = i0 + (size_t)t * stride;
      const unsigned long long lw = q[2 * i + 1];
      H += (long long)q[2 * i];
      L += lw & ~kFixPoison;
      P |= lw;
    }
    return fix_value(H, L, (P & kFixPoison) != 0);
  }
  double s = 0.0;
#pragma unroll
  for (int t = 0; t < T; ++t) s += part[i0 + (size_t)t * stride];
  return s;
}

// runtime slot count (the standalone finalize kernels)
PSX_DEV double slot_sum_rt(const float* part, size_t i0, size_t stride, int T, bool det) {
  if (det) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(part);
    long long H = 0;
    unsigned long long L = 0, P = 0;
    for (int t = 0; t < T; ++t) {
      const size_t i = i0 + (size_t)t * stride;
      const unsigned long long lw = q[2 * i + 1];
      H += (long long)q[2 * i];
      L += lw & ~kFixPoison;
      P |= lw;
    }
    return fix_value(H, L, (P & kFixPoison) != 0);
  }
  double s = 0.0;
  for (int t = 0; t < T; ++t) s += part[i0 + (size_t)t * stride];
  return s;
}

// host: the DetRed of a launch whose sums go to slot buffer `part` (disabled outside
// deterministic mode)
DetRed det_for(const float* part);
bool det_enabled();

// part: [T][2][C] slot rows (sum, sum of squares). Same math as bn_finalize_kernel (bn.hip).
// One thread per channel, all T slot loads issued back to back: the slot sums sit at the
// memory side (float atomics bypass L2), so a per-channel-group LDS reduction would pay one
// memory round trip per 32 channels; this pays about one in total. blockDim = 256.
template <int T>
PSX_DEV void bn_finalize_block(const float* part, const BnFin& f) {
  for (int c = threadIdx.x; c < f.C; c += 256) {
    const double s = slot_sum<T>(part, c, 2 * (size_t)f.C, f.det), ss = slot_sum<T>(part, f.C + c, 2 * (size_t)f.C, f.det);
    double mean, var;
    bn_moments(s, ss, f.count, f.sshift ? f.sshift[c] : 0.f, mean, var);
    const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    const float sc = f.gamma[c] * invstd;
    f.scale[c] = sc;
    f.shift[c] = f.beta[c] - (float)mean * sc;
    f.save_mean[c] = (float)mean;
    f.save_invstd[c] = invstd;
    if (f.sshift_next) f.sshift_next[c] = (float)mean;
    if (f.run_mean) {
      const double unb = f.count > 1.f ? var * f.count / (f.count - 1.0) : var;
      f.run_mean[c] = (1.f - f.momentum) * f.run_mean[c] + f.momentum * (float)mean;
      f.run_var[c] = (1.f - f.momentum) * f.run_var[c] + f.momentum * (float)unb;
    }
  }
}

// part: [T][NS][C] (row 0 = sum dz, row `which` = sum dz*xhat). Same math as
// bn_bwd_finalize_kernel (bn.hip); layout of the work as bn_finalize_block.
template <int T>
PSX_DEV void bn_bwd_finalize_block(const float* part, int NS, int which, const BnBwdFin& f) {
  for (int c = threadIdx.x; c < f.C; c += 256) {
    const size_t st = (size_t)NS * f.C;
    const double sdz = slot_sum<T>(part, c, st, f.det), sxh = slot_sum<T>(part, (size_t)which * f.C + c, st, f.det);
    const float mdz = (float)(sdz / f.count), mxh = (float)(sxh / f.count);
    const float is = f.invstd[c], gm = f.gamma[c];
    f.coef[c] = gm * is;
    f.coef[f.C + c] = -gm * is * is * mxh;
    f.coef[2 * f.C + c] = -gm * is * mdz + gm * is * is * f.mean[c] * mxh;
    const float dg = (float)sxh * f.gscale, db = (float)sdz * f.gscale;
    if (f.grad_fp16) {
      reinterpret_cast<uint16_t*>(f.dgamma)[c] = __builtin_bit_cast(uint16_t, (_Float16)dg);
      reinterpret_cast<uint16_t*>(f.dbeta)[c] = __builtin_bit_cast(uint16_t, (_Float16)db);
    } else {
      reinterpret_cast<float*>(f.dgamma)[c] = dg;
      reinterpret_cast<float*>(f.dbeta)[c] = db;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Consumer-side finalize: every workgroup of the BN-apply launch that consumes a layer's slot
// sums recomputes the per-channel affine (forward) or coefficients (backward) into LDS, and
// workgroup 0 also writes the global side outputs (affine, saved statistics, running
// statistics / coefficients, dgamma and dbeta on the gradient wire). This replaces one
// finalize launch per BN layer (~4-5 us of dispatch and drain each, 40 per ResNet-18 step)
// with 2*T*C redundant slot loads per workgroup: L2 hits after the first reader on each XCD.
// The producer is a previous launch, so no fence is needed. tpc threads share a channel
// (adjacent lanes, combined with shuffles) so 256 threads cover small C in one pass.
// Slot reduction of two stat rows (ra, rb of NS per slot) for all C channels into LDS red[2][C]
// (double sums, as bn_finalize_kernel). Thread = (float4 column of 4 channels, slot
// group g of G); all of a thread's 16-byte loads are independent, so the whole reduction costs
// about one memory round trip. LDS scratch: 8 * 256 floats (caller's sbn tail).
template <int T>
PSX_DEV void slot_reduce2(const float* part, int NS, int ra, int rb, int C, double* red, float* scratch,
                          bool det = false) {
  if (det) {  // fixed-point pairs: one thread per (row, channel), exact integer sums
    for (int j = threadIdx.x; j < 2 * C; j += blockDim.x) {
      const int row = j < C ? ra : rb, c = j < C ? j : j - C;
      red[j] = slot_sum<T>(part, (size_t)row * C + c, (size_t)NS * C, true);
    }
    __syncthreads();
    return;
  }
  const int C4 = C >> 2;
  for (int cb = 0; cb < C4; cb += 256) {
    const int ncol = min(256, C4 - cb);
    const int G = max(1, min(T, 256 / ncol));
    const int col = threadIdx.x % ncol, g = threadIdx.x / ncol;
    double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    if (g < G) {
      const float4* pa = reinterpret_cast<const float4*>(part + (size_t)ra * C) + cb + col;
      const float4* pb = reinterpret_cast<const float4*>(part + (size_t)rb * C) + cb + col;
      const size_t st4 = (size_t)NS * C / 4;
#pragma unroll 8
      for (int t = g; t < T; t += G) {
        const float4 va = pa[t * st4], vb = pb[t * st4];
        a[0] += va.x; a[1] += va.y; a[2] += va.z; a[3] += va.w;
        b[0] += vb.x; b[1] += vb.y; b[2] += vb.z; b[3] += vb.w;
      }
    }
    // combine the G slot groups of each column through LDS (G = 1: direct)
    if (G == 1) {
      if (g == 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          red[(cb + col) * 4 + k] = a[k];
          red[C + (cb + col) * 4 + k] = b[k];
        }
    } else {
      double* sd = reinterpret_cast<double*>(scratch);  // [256][2] doubles per component pass
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        __syncthreads();
        sd[threadIdx.x * 2 + 0] = a[k];
        sd[threadIdx.x * 2 + 1] = b[k];
        __syncthreads();
        if (threadIdx.x < ncol) {
          double sa = 0.0, sb = 0.0;
          for (int q = 0; q < G; ++q) {
            sa += sd[(q * ncol + threadIdx.x) * 2 + 0];
            sb += sd[(q * ncol + threadIdx.x) * 2 + 1];
          }
          red[(cb + threadIdx.x) * 4 + k] = sa;
          red[C + (cb + threadIdx.x) * 4 + k] = sb;
        }
      }
    }
  }
  __syncthreads();
}

// sc/sh: LDS [C]; red: LDS [2][C] doubles; scratch: LDS 512 doubles.
template <int T>
PSX_DEV void bn_fin_lds(const float* part, const BnFin& f, float* sc, float* sh, double* red, float* scratch) {
  slot_reduce2<T>(part, 2, 0, 1, f.C, red, scratch, f.det);
  for (int c = threadIdx.x; c < f.C; c += 256) {
    double mean, var;
    bn_moments(red[c], red[f.C + c], f.count, f.sshift ? f.sshift[c] : 0.f, mean, var);
    const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    const float scv = f.gamma[c] * invstd, shv = f.beta[c] - (float)mean * scv;
    sc[c] = scv;
    sh[c] = shv;
    if (blockIdx.x == 0) {
      f.scale[c] = scv;
      f.shift[c] = shv;
      f.save_mean[c] = (float)mean;
      f.save_invstd[c] = invstd;
      if (f.sshift_next) f.sshift_next[c] = (float)mean;
      if (f.run_mean) {
        const double unb = f.count > 1.f ? var * f.count / (f.count - 1.0) : var;
        f.run_mean[c] = (1.f - f.momentum) * f.run_mean[c] + f.momentum * (float)mean;
        f.run_var[c] = (1.f - f.momentum) * f.run_var[c] + f.momentum * (float)unb;
      }
    }
  }
}

// part: [T][NS][C] (row 0 = sum dz, row `which` = sum dz*xhat); coef (LDS): [3][C].
template <int T>
PSX_DEV void bn_bwd_fin_lds(const float* part, int NS, int which, const BnBwdFin& f, float* coef, double* red,
                            float* scratch) {
  slot_reduce2<T>(part, NS, 0, which, f.C, red, scratch, f.det);
  const int C = f.C;
  for (int c = threadIdx.x; c < C; c += 256) {
    const double sdz = red[c], sxh = red[C + c];
    const float mdz = (float)(sdz / f.count), mxh = (float)(sxh / f.count);
    const float is = f.invstd[c], gm = f.gamma[c];
    const float k1 = gm * is, k2 = -gm * is * is * mxh, k3 = -gm * is * mdz + gm * is * is * f.mean[c] * mxh;
    coef[c] = k1;
    coef[C + c] = k2;
    coef[2 * C + c] = k3;
    if (blockIdx.x == 0) {
      f.coef[c] = k1;
      f.coef[C + c] = k2;
      f.coef[2 * C + c] = k3;
      const float dg = (float)sxh * f.gscale, db = (float)sdz * f.gscale;
      if (f.grad_fp16) {
        reinterpret_cast<uint16_t*>(f.dgamma)[c] = __builtin_bit_cast(uint16_t, (_Float16)dg);
        reinterpret_cast<uint16_t*>(f.dbeta)[c] = __builtin_bit_cast(uint16_t, (_Float16)db);
      } else {
        reinterpret_cast<float*>(f.dgamma)[c] = dg;
        reinterpret_cast<float*>(f.dbeta)[c] = db;
      }
    }
  }
}

}  // namespace psx
