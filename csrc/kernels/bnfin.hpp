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
};

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
    const double mean = s / f.count;
    double var = ss / f.count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    const float sc = f.gamma[c] * invstd;
    f.scale[c] = sc;
    f.shift[c] = f.beta[c] - (float)mean * sc;
    f.save_mean[c] = (float)mean;
    f.save_invstd[c] = invstd;
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

}  // namespace psx
