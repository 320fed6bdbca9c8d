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
// Deterministic mode (psx_set_deterministic, bn.hip): a launch that produces per-channel sums
// adds each workgroup's partial row into a row of its own of a scratch slab [rows][NS][C] —
// exactly one add per location into zeros, so the value is exact whatever the order. The rows
// are then summed in a fixed order by a two-level tree:
//   level 1: rows are grouped `group` at a time; the workgroup arriving last among a group's
//            writers (`nper` per row: e.g. the channel tiles of a conv) sums the group's rows in
//            row order into row g of a second slab [ngroups][NS][C] (again one add per location)
//            and re-zeroes the group's rows and counter;
//   level 2: the last group reducer sums the ngroups rows in order into slot row 0 of the usual
//            [PSX_STAT_SLOTS][NS][C] buffer (the other slot rows stay zero), re-zeroes the second
//            slab and the launch counter.
// Groups of ~sqrt(rows) rows keep both levels short (the one-level form, one workgroup reading
// every row, read up to 1 MB from one CU per launch; both levels are latency-bound chains of
// dependent loads, det_rows). The consumers are
// unchanged and sum the slot rows in a fixed order, so every BN statistic — and with it the
// whole step — is bit-reproducible. All payload adds are memory-side float atomics (no release
// needed, as for the slots); the slab lines a reducer reads were never cached by this launch,
// and kernel boundaries write back and invalidate the non-coherent L2 lines of the previous
// launch's re-zeroing.
struct DetRed {
  float* slab;        // nullptr: deterministic mode off
  float* slab2;       // level-2 rows [ngroups][NS][C]
  unsigned* counter;  // [0]: level 2, [1 + g]: group g; zero at launch, re-zeroed by the reducers
  int rows, group, ngroups, nper;
};

// Fixed-order sum of rows [r0, r1) of a [rows][n] slab into dst[j] (j < n), by the whole block:
// value j is summed by `lanes` = max(1, 256 / n) threads over interleaved row subsets (8 loads in
// flight each: the reduction is latency-bound), combined through LDS in lane order. Every value's
// sum has the same association for a given (r0, r1, n), whatever the launch's timing.
// add = true: dst receives one atomic add (onto zero: exact); else a plain store. Re-zeroes the rows.
PSX_DEV void det_rows(float* slab, int r0, int r1, int n, float* dst, bool add, float* scratch) {
  const int lanes = n >= 256 ? 1 : 256 / n;
  for (int jb = 0; jb < n; jb += 256) {
    // the first 256 threads do the work (blocks of 384, wino.hip's split transforms, call it too)
    const int t = threadIdx.x, k = lanes > 1 ? t / n : 0, j = jb + (lanes > 1 ? t % n : t);
    const bool act = t < 256;
    float acc = 0.f;
    if (act && k < lanes && j < n) {
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int r = r0 + k;
      for (; r + 7 * lanes < r1; r += 8 * lanes) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += slab[(size_t)(r + u * lanes) * n + j];
      }
      for (int u = 0; r < r1; r += lanes, ++u) a[u & 7] += slab[(size_t)r * n + j];
      acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      for (r = r0 + k; r < r1; r += lanes) slab[(size_t)r * n + j] = 0.f;
    }
    if (lanes > 1) {
      __syncthreads();
      if (act && k < lanes && j < n) scratch[k * n + (j - jb)] = acc;
      __syncthreads();
      if (t < n) {
        float v = 0.f;
        for (int q = 0; q < lanes; ++q) v += scratch[q * n + t];
        if (add) atomicAdd(dst + t, v);
        else dst[t] = v;
      }
    } else if (act && j < n) {
      if (add) atomicAdd(dst + j, acc);
      else dst[j] = acc;
    }
  }
}

// every workgroup of the launch calls this (block-uniformly) after its slab adds into row `row`;
// returns true in the last-arriving workgroup (after the fixed-order reduction, so an in-launch
// finalize of the same sums can follow). lds: >= 16 + 1024 bytes of the caller's LDS.
PSX_DEV bool det_finish(const DetRed& d, int NS, int C, float* part, int row, unsigned char* lds) {
  const int g = row / d.group;
  const int r0 = g * d.group, r1 = min(d.rows, r0 + d.group);
  if (!last_block_arrive(d.counter + 1 + g, (unsigned)(d.nper * (r1 - r0)), lds)) return false;
  float* scratch = reinterpret_cast<float*>(lds + 16);
  const int n = NS * C;
  det_rows(d.slab, r0, r1, n, d.slab2 + (size_t)g * n, true, scratch);
  if (threadIdx.x == 0) __hip_atomic_store(d.counter + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!last_block_arrive(d.counter, (unsigned)d.ngroups, lds)) return false;
  det_rows(d.slab2, 0, d.ngroups, n, part, false, scratch);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(d.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// host: the DetRed of the next producing launch (slab rows for `rows` x NS x C sums, `nper`
// writer workgroups per row). Deterministic mode off: a disabled one. The slab too small for
// the launch is a hard error (bn.hip det_next aborts): a silent fall back to the atomic slots
// would break bit-reproducibility unnoticed.
DetRed det_next(int rows, int NS, int C, int nper = 1);
bool det_enabled();

// part: [T][2][C] slot rows (sum, sum of squares). Same math as bn_finalize_kernel (bn.hip).
// One thread per channel, all T slot loads issued back to back: the slot sums sit at the
// memory side (float atomics bypass L2), so a per-channel-group LDS reduction would pay one
// memory round trip per 32 channels; this pays about one in total. blockDim = 256.
template <int T>
PSX_DEV void bn_finalize_block(const float* part, const BnFin& f) {
  for (int c = threadIdx.x; c < f.C; c += 256) {
    float v1[T], v2[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      v1[t] = part[((size_t)t * 2 + 0) * f.C + c];
      v2[t] = part[((size_t)t * 2 + 1) * f.C + c];
    }
    double s = 0.0, ss = 0.0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      s += v1[t];
      ss += v2[t];
    }
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
    float va[T], vb[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      va[t] = part[((size_t)t * NS + 0) * f.C + c];
      vb[t] = part[((size_t)t * NS + which) * f.C + c];
    }
    double sdz = 0.0, sxh = 0.0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      sdz += va[t];
      sxh += vb[t];
    }
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
PSX_DEV void slot_reduce2(const float* part, int NS, int ra, int rb, int C, double* red, float* scratch) {
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
  slot_reduce2<T>(part, 2, 0, 1, f.C, red, scratch);
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
  slot_reduce2<T>(part, NS, 0, which, f.C, red, scratch);
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
