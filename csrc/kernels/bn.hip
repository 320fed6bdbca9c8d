// Training-mode BatchNorm2d (+ReLU, +residual) on NHWC activations (bf16 bits or fp32: every
// elementwise kernel is templated on the storage type T, common.hpp ld8/st8).
//
// Replaces nn.BatchNorm2d / torch.relu / `out += shortcut` of the reference BasicBlock
// (reference: src/parameter_server/server.py:21-41, identical copies in worker.py:20-76).
// Semantics follow torch: batch statistics over (N,H,W), biased variance for normalisation,
// running_var updated with the unbiased variance, momentum 0.1, eps 1e-5.
//
// Forward statistics come from the conv epilogue as per-tile partial (sum, sumsq) slabs
// ([T][2][C]); bn_finalize reduces them (fp64, fixed order => deterministic), produces the
// per-channel affine (scale, shift) and updates the running stats. Every elementwise pass is
// vectorised at 8 channels per lane (16 B bf16 / 32 B fp32).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "bnfin.hpp"
#include "common.hpp"

namespace psx {

__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ part, int T, int C, float count,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, float momentum,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          float* __restrict__ scale, float* __restrict__ shift,
                                                          float* __restrict__ save_mean,
                                                          float* __restrict__ save_invstd,
                                                          const float* __restrict__ sshift,
                                                          float* __restrict__ sshift_next, int det) {
  // 8 slot groups x 32 channels per block (T slot rows read with 8-way parallelism)
  __shared__ double red[2][8][32];
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float fs = 0.f, fss = 0.f;
  if (c < C && !det) {
    for (int t = grp; t < T; t += 8) {
      fs += part[((size_t)t * 2 + 0) * C + c];
      fss += part[((size_t)t * 2 + 1) * C + c];
    }
  }
  red[0][grp][cl] = fs;
  red[1][grp][cl] = fss;
  __syncthreads();
  if (grp == 0 && c < C) {
    double s = 0.0, ss = 0.0;
    if (det) {  // fixed-point slot pairs: exact integer sums (bnfin.hpp DetRed)
      s = slot_sum_rt(part, c, 2 * (size_t)C, T, true);
      ss = slot_sum_rt(part, (size_t)C + c, 2 * (size_t)C, T, true);
    } else {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        s += red[0][g][cl];
        ss += red[1][g][cl];
      }
    }
    double mean, var;  // shifted sums (bnfin.hpp BnFin::sshift)
    bn_moments(s, ss, count, sshift ? sshift[c] : 0.f, mean, var);
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * invstd;
    scale[c] = sc;
    shift[c] = beta[c] - (float)mean * sc;
    save_mean[c] = (float)mean;
    save_invstd[c] = invstd;
    if (sshift_next) sshift_next[c] = (float)mean;
    if (run_mean) {
      const double unb = count > 1.f ? var * count / (count - 1.0) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
    }
  }
}

// Eval-mode affine from running statistics.
__global__ void bn_eval_affine_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                      float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    const float sc = gamma[c] * rsqrtf(rv[c] + eps);
    scale[c] = sc;
    shift[c] = beta[c] - rm[c] * sc;
  }
}

// out = act( y*scale + shift  [+ res]  [+ res2*scale2 + shift2] )
// MODE 0: no residual, 1: identity residual, 2: BN'd residual.
template <typename T, int MODE, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ res,
                                                       const float* __restrict__ scale2,
                                                       const float* __restrict__ shift2, T* __restrict__ out,
                                                       size_t nvec, int C) {
  const int cvec = C >> 3;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cvec) << 3;
    float v[8], rv[8];
    ld8(y + i * 8, v);
    if (MODE != 0) ld8(res + i * 8, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float t = v[j] * scale[c] + shift[c];
      if (MODE == 1) t += rv[j];
      else if (MODE == 2) t += rv[j] * scale2[c] + shift2[c];
      v[j] = RELU ? fmaxf(t, 0.f) : t;
    }
    st8(out + i * 8, v);
  }
}

// Backward pass 1: per-channel partials of sum(dz), sum(dz*xhat1) [, sum(dz*xhat2)], with
// dz = g * (o > 0) (ReLU mask from the stored activation) or dz = g.
// part layout: [PSX_STAT_SLOTS][NS][C] (pre-zeroed, fp32 atomics), NS = 2 or 3.
template <typename T, bool MASK, bool TWO>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ g, const T* __restrict__ o,
                                                            const T* __restrict__ y1,
                                                            const float* __restrict__ mean1,
                                                            const float* __restrict__ invstd1,
                                                            const T* __restrict__ y2,
                                                            const float* __restrict__ mean2,
                                                            const float* __restrict__ invstd2, float* __restrict__ part,
                                                            int npix, int C, int pix_per_block, int fuse_fin,
                                                            BnBwdFin fin1, BnBwdFin fin2, DetRed det) {
  constexpr int NS = TWO ? 3 : 2;
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [256][NS*8]
  const int cvec = C >> 3;
  const int tpp = 256 / cvec;  // threads per pixel row set (pixels processed per iteration)
  const int cg = threadIdx.x % cvec, pr = threadIdx.x / cvec;
  const int c0 = cg * 8;
  float m1[8], i1[8], m2[8], i2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m1[j] = mean1[c0 + j];
    i1[j] = invstd1[c0 + j];
    if (TWO) {
      m2[j] = mean2[c0 + j];
      i2[j] = invstd2[c0 + j];
    }
  }
  float sdz[8], sx1[8], sx2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sdz[j] = sx1[j] = sx2[j] = 0.f;
  const int pbeg = blockIdx.x * pix_per_block;
  const int pend = min(npix, pbeg + pix_per_block);
  for (int p = pbeg + pr; p < pend; p += tpp) {
    const size_t e0 = ((size_t)p * cvec + cg) * 8;
    float gv[8], ov[8], yv[8], y2v[8];
    ld8(g + e0, gv);
    if (MASK) ld8(o + e0, ov);
    ld8(y1 + e0, yv);
    if (TWO) ld8(y2 + e0, y2v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d = gv[j];
      if (MASK && !(ov[j] > 0.f)) d = 0.f;
      sdz[j] += d;
      sx1[j] += d * (yv[j] - m1[j]) * i1[j];
      if (TWO) sx2[j] += d * (y2v[j] - m2[j]) * i2[j];
    }
  }
  float* mine = sred + threadIdx.x * (NS * 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mine[j] = sdz[j];
    mine[8 + j] = sx1[j];
    if (TWO) mine[16 + j] = sx2[j];
  }
  __syncthreads();
  // reduce over pr (threads with the same cg): thread t < cvec*NS*8 sums one (cg, stat, j)
  for (int t = threadIdx.x; t < cvec * NS * 8; t += 256) {
    const int cgi = t / (NS * 8), sj = t - cgi * (NS * 8);
    float acc = 0.f;
    for (int q = 0; q < tpp; ++q) acc += sred[(q * cvec + cgi) * (NS * 8) + sj];
    const int stat = sj >> 3, j = sj & 7;
    stat_add(det, part + (size_t)(blockIdx.x & (PSX_STAT_SLOTS - 1)) * NS * C, stat * C + cgi * 8 + j, acc);
  }
  // in-launch finalize (bnfin.hpp): the last block computes the coefficients + dgamma/dbeta
  if (fuse_fin && last_block_arrive(fin1.counter, gridDim.x, reinterpret_cast<unsigned char*>(sred))) {
    bn_bwd_finalize_block<PSX_STAT_SLOTS>(part, NS, 1, fin1);
    if (TWO) bn_bwd_finalize_block<PSX_STAT_SLOTS>(part, NS, 2, fin2);
  }
}

// Backward finalize: dgamma = sum(dz*xhat), dbeta = sum(dz); dx = k1*dz + k2*y + k3.
// Writes dgamma/dbeta (scaled) into the gradient sink (fp16 wire codec or fp32).
template <typename GT>
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int T, int NS, int which, int C, float count,
                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ coef,
                                       GT* __restrict__ dgamma, GT* __restrict__ dbeta, float gscale, int det) {
  // 8 slot groups x 32 channels per block: the T slot rows are read with 8-way parallelism
  __shared__ float red[2][8][32];
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float a = 0.f, b = 0.f;
  if (c < C && !det) {
    for (int t = grp; t < T; t += 8) {
      a += part[((size_t)t * NS + 0) * C + c];
      b += part[((size_t)t * NS + which) * C + c];
    }
  }
  red[0][grp][cl] = a;
  red[1][grp][cl] = b;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  double sdz = 0.0, sxh = 0.0;
  if (det) {  // fixed-point slot pairs: exact integer sums (bnfin.hpp DetRed)
    sdz = slot_sum_rt(part, c, (size_t)NS * C, T, true);
    sxh = slot_sum_rt(part, (size_t)which * C + c, (size_t)NS * C, T, true);
  } else {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      sdz += red[0][g][cl];
      sxh += red[1][g][cl];
    }
  }
  const float mdz = (float)(sdz / count), mxh = (float)(sxh / count);
  const float is = invstd[c], gm = gamma[c];
  const float k1 = gm * is;
  const float k2 = -gm * is * is * mxh;
  const float k3 = -gm * is * mdz + gm * is * is * mean[c] * mxh;
  coef[c] = k1;
  coef[C + c] = k2;
  coef[2 * C + c] = k3;
  const float dg = (float)sxh * gscale, db = (float)sdz * gscale;
  if constexpr (sizeof(GT) == 2) {
    dgamma[c] = __builtin_bit_cast(uint16_t, (_Float16)dg);
    dbeta[c] = __builtin_bit_cast(uint16_t, (_Float16)db);
  } else {
    dgamma[c] = dg;
    dbeta[c] = db;
  }
}

// dx1 = k1*dz + k2*y1 + k3 [, dx2 = k1'*dz + k2'*y2 + k3'] [, dzout = dz]
template <typename T, bool MASK, bool TWO, bool DZOUT>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ g, const T* __restrict__ o,
                                                           const T* __restrict__ y1, const float* __restrict__ coef1,
                                                           T* __restrict__ dx1, const T* __restrict__ y2,
                                                           const float* __restrict__ coef2, T* __restrict__ dx2,
                                                           T* __restrict__ dzout, size_t nvec, int C) {
  const int cvec = C >> 3;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cvec) << 3;
    float d[8], ov[8], yv[8], y2v[8], r1[8], r2[8];
    ld8(g + i * 8, d);
    if (MASK) ld8(o + i * 8, ov);
    ld8(y1 + i * 8, yv);
    if (TWO) ld8(y2 + i * 8, y2v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      if (MASK && !(ov[j] > 0.f)) d[j] = 0.f;
      r1[j] = coef1[c] * d[j] + coef1[C + c] * yv[j] + coef1[2 * C + c];
      if (TWO) r2[j] = coef2[c] * d[j] + coef2[C + c] * y2v[j] + coef2[2 * C + c];
    }
    st8(dx1 + i * 8, r1);
    if (TWO) st8(dx2 + i * 8, r2);
    if (DZOUT) st8(dzout + i * 8, d);
  }
}

// Opt-in (PSX_TUNE bnfin_apply=1) variant of bn_apply_kernel with the training-mode finalize folded in:
// every workgroup computes the affine(s) from the stat slots (bnfin.hpp bn_fin_lds). Separate
// kernels so the default path keeps its exact code (an A/B showed +38 us/step otherwise).
template <typename T, int MODE, bool RELU, bool FIN = true>
__global__ __launch_bounds__(256) void bn_apply_fin_kernel(const T* __restrict__ y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ res,
                                                       const float* __restrict__ scale2,
                                                       const float* __restrict__ shift2, T* __restrict__ out,
                                                       size_t nvec, int C, const float* __restrict__ part1,
                                                       const float* __restrict__ part2, BnFin f1, BnFin f2) {
  extern __shared__ __attribute__((aligned(16))) float sbn[];  // FIN: [scale1|shift1|scale2|shift2] x C, red, scratch
  if constexpr (FIN) {
    double* red = reinterpret_cast<double*>(sbn + 4 * C);
    float* scratch = sbn + 8 * C;
    bn_fin_lds<PSX_STAT_SLOTS>(part1, f1, sbn, sbn + C, red, scratch);
    if constexpr (MODE == 2) {
      __syncthreads();
      bn_fin_lds<PSX_STAT_SLOTS>(part2, f2, sbn + 2 * C, sbn + 3 * C, red, scratch);
    }
    __syncthreads();
  }
  auto SC = [&](int c) -> float { if constexpr (FIN) return sbn[c]; else return scale[c]; };
  auto SH = [&](int c) -> float { if constexpr (FIN) return sbn[C + c]; else return shift[c]; };
  auto SC2 = [&](int c) -> float { if constexpr (FIN) return sbn[2 * C + c]; else return scale2[c]; };
  auto SH2 = [&](int c) -> float { if constexpr (FIN) return sbn[3 * C + c]; else return shift2[c]; };
  const int cvec = C >> 3;
  // a thread's channel group is fixed when the grid stride is a multiple of C/8: keep its 8
  // channels' parameters in registers (scalar per-element reads of LDS at an 8-float lane
  // stride are 8-way bank conflicts)
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  // (global-memory parameters: re-read per iteration, L1 hits the compiler schedules with the
  // data loads; hoisting them behind a first-iteration branch measured slower)
  const bool fixed = FIN && stride % cvec == 0;
  float k[4][8];
  int cur = -1;
  auto load = [&](int c0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k[0][j] = SC(c0 + j);
      k[1][j] = SH(c0 + j);
      if (MODE == 2) {
        k[2][j] = SC2(c0 + j);
        k[3][j] = SH2(c0 + j);
      }
    }
    cur = c0;
  };
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int c0 = (int)(i % cvec) << 3;
    if (!fixed || cur < 0) load(c0);
    float v[8], rv[8];
    ld8(y + i * 8, v);
    if (MODE != 0) ld8(res + i * 8, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j] * k[0][j] + k[1][j];
      if (MODE == 1) t += rv[j];
      else if (MODE == 2) t += rv[j] * k[2][j] + k[3][j];
      v[j] = RELU ? fmaxf(t, 0.f) : t;
    }
    st8(out + i * 8, v);
  }
}

// Opt-in variant of bn_bwd_apply_kernel: coefficients from the slot sums part [T][NS][C] per
// workgroup (bnfin.hpp bn_bwd_fin_lds).
template <typename T, bool MASK, bool TWO, bool DZOUT, bool FIN = true>
__global__ __launch_bounds__(256) void bn_bwd_apply_fin_kernel(const T* __restrict__ g, const T* __restrict__ o,
                                                           const T* __restrict__ y1,
                                                           const float* __restrict__ coef1, T* __restrict__ dx1,
                                                           const T* __restrict__ y2,
                                                           const float* __restrict__ coef2, T* __restrict__ dx2,
                                                           T* __restrict__ dzout,
                                                           size_t nvec, int C, const float* __restrict__ part,
                                                           BnBwdFin f1, BnBwdFin f2) {
  extern __shared__ __attribute__((aligned(16))) float sbn[];  // FIN: coef1 [3][C] | coef2 [3][C] | red | scratch
  if constexpr (FIN) {
    constexpr int NS = TWO ? 3 : 2;
    double* red = reinterpret_cast<double*>(sbn + 6 * C);
    float* scratch = sbn + 10 * C;
    bn_bwd_fin_lds<PSX_STAT_SLOTS>(part, NS, 1, f1, sbn, red, scratch);
    if constexpr (TWO) {
      __syncthreads();
      bn_bwd_fin_lds<PSX_STAT_SLOTS>(part, NS, 2, f2, sbn + 3 * C, red, scratch);
    }
    __syncthreads();
  }
  auto K1 = [&](int c) -> float { if constexpr (FIN) return sbn[c]; else return coef1[c]; };
  auto K2 = [&](int c) -> float { if constexpr (FIN) return sbn[3 * C + c]; else return coef2[c]; };
  const int cvec = C >> 3;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const bool fixed = FIN && stride % cvec == 0;  // see bn_apply_kernel
  float k1[3][8], k2[3][8];
  int cur = -1;
  auto load = [&](int c0) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        k1[r][j] = K1(r * C + c0 + j);
        if (TWO) k2[r][j] = K2(r * C + c0 + j);
      }
    cur = c0;
  };
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int c0 = (int)(i % cvec) << 3;
    if (!fixed || cur < 0) load(c0);
    float d[8], ov[8], yv[8], y2v[8], r1[8], r2[8];
    ld8(g + i * 8, d);
    if (MASK) ld8(o + i * 8, ov);
    ld8(y1 + i * 8, yv);
    if (TWO) ld8(y2 + i * 8, y2v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MASK && !(ov[j] > 0.f)) d[j] = 0.f;
      r1[j] = k1[0][j] * d[j] + k1[1][j] * yv[j] + k1[2][j];
      if (TWO) r2[j] = k2[0][j] * d[j] + k2[1][j] * y2v[j] + k2[2][j];
    }
    st8(dx1 + i * 8, r1);
    if (TWO) st8(dx2 + i * 8, r2);
    if (DZOUT) st8(dzout + i * 8, d);
  }
}

// ---- deterministic mode host state (bnfin.hpp DetRed): on / off
namespace {
bool g_det = false;
}  // namespace

bool det_enabled() { return g_det; }

DetRed det_for(const float* part) {
  DetRed d{};
  if (g_det) d.fix = reinterpret_cast<unsigned long long*>(const_cast<float*>(part));
  return d;
}

}  // namespace psx

using namespace psx;

// workgroup cap of the folded-finalize apply launches (each workgroup recomputes the affine)
// (1024 vs 2048: 1.852 vs 1.867-1.875 ms/step, round 4; round 6, same box: 512 vs 1024 fp32
// 3.262 -> 3.254, bf16 1.605 -> 1.581; 256 worse in bf16: profiles/r6_bn_fin_grid_ab.jsonl)
static int fin_grid_cap() { return 512; }

static int ew_grid(size_t nvec) {
  size_t g = (nvec + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

// Deterministic mode on (on != 0) or off. Every later producer of BN sums (conv epilogues, split-K
// epilogue, bn_bwd_reduce, the Winograd output transforms, the head, the stems) adds exact
// fixed-point pairs into its slot buffer — which the caller sizes psx_det_slot_scale() times the
// float layout — and every consumer reads them as such (bnfin.hpp DetRed). Host state only: set
// it before a HIP graph is captured.
int psx_det_slot_scale() { return 4; }

int psx_set_deterministic(int on) {
  g_det = on != 0;
  return 0;
}

int psx_bn_finalize(const float* part, int T, int C, float count, const float* gamma, const float* beta, float eps,
                    float momentum, float* run_mean, float* run_var, float* scale, float* shift, float* save_mean,
                    float* save_invstd, const float* sshift, float* sshift_next, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 31) / 32), dim3(256), 0, st, part, T, C, count, gamma, beta, eps,
                     momentum, run_mean, run_var, scale, shift, save_mean, save_invstd, sshift, sshift_next,
                     (int)det_enabled());
  return (int)hipGetLastError();
}

int psx_bn_eval_affine(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                       float* scale, float* shift, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, rm, rv, eps,
                     scale, shift);
  return (int)hipGetLastError();
}

// mode: 0 plain, 1 +identity residual, 2 +BN'd residual
int psx_bn_apply(const void* y, const float* scale, const float* shift, const void* res, const float* scale2,
                 const float* shift2, void* out, long nelem, int C, int mode, int relu, int f32, hipStream_t st) {
  if (C % 8 || nelem % 8) return -2;
  const size_t nvec = (size_t)nelem / 8;
  const int grid = ew_grid(nvec);
#define PSX_BNA(M, R)                                                                                           \
  do {                                                                                                          \
    if (f32)                                                                                                    \
      hipLaunchKernelGGL((bn_apply_kernel<float, M, R>), dim3(grid), dim3(256), 0, st, (const float*)y, scale,  \
                         shift, (const float*)res, scale2, shift2, (float*)out, nvec, C);                       \
    else                                                                                                        \
      hipLaunchKernelGGL((bn_apply_kernel<uint16_t, M, R>), dim3(grid), dim3(256), 0, st, (const uint16_t*)y,   \
                         scale, shift, (const uint16_t*)res, scale2, shift2, (uint16_t*)out, nvec, C);          \
  } while (0)
  if (mode == 0 && relu) PSX_BNA(0, true);
  else if (mode == 0) PSX_BNA(0, false);
  else if (mode == 1 && relu) PSX_BNA(1, true);
  else if (mode == 1) PSX_BNA(1, false);
  else if (mode == 2 && relu) PSX_BNA(2, true);
  else if (mode == 2) PSX_BNA(2, false);
  else return -3;
#undef PSX_BNA
  return (int)hipGetLastError();
}

// Returns the number of partial rows T (query with part == nullptr).
int psx_bn_bwd_reduce(const void* g, const void* o, const void* y1, const float* mean1, const float* invstd1,
                      const void* y2, const float* mean2, const float* invstd2, float* part, int npix, int C,
                      const BnBwdFin* fin1, const BnBwdFin* fin2, int f32, hipStream_t st) {
  if (C % 8 || 256 % (C / 8)) return -2;
  const int fuse = fin1 != nullptr;
  BnBwdFin f1{}, f2{};
  if (fin1) f1 = *fin1;
  if (fin2) f2 = *fin2;
  f1.det = f2.det = (int)det_enabled();
  if (fuse && (f1.C != C || (y2 && (!fin2 || f2.C != C)))) return -10;
  // ~512 blocks, at least 64 pixels each
  int ppb = (npix + 511) / 512;
  if (ppb < 64) ppb = 64;
  const int T = (npix + ppb - 1) / ppb;
  if (!part) return PSX_STAT_SLOTS;
  const bool mask = o != nullptr, two = y2 != nullptr;
  const size_t lds = 256 * (two ? 3 : 2) * 8 * sizeof(float);
  const DetRed det = det_for(part);
#define PSX_BBR(M, TW)                                                                                         \
  do {                                                                                                         \
    if (f32)                                                                                                   \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<float, M, TW>), dim3(T), dim3(256), lds, st, (const float*)g,   \
                         (const float*)o, (const float*)y1, mean1, invstd1, (const float*)y2, mean2, invstd2,  \
                         part, npix, C, ppb, fuse, f1, f2, det);                                               \
    else                                                                                                       \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<uint16_t, M, TW>), dim3(T), dim3(256), lds, st,                 \
                         (const uint16_t*)g, (const uint16_t*)o, (const uint16_t*)y1, mean1, invstd1,          \
                         (const uint16_t*)y2, mean2, invstd2, part, npix, C, ppb, fuse, f1, f2, det);          \
  } while (0)
  if (mask && two) PSX_BBR(true, true);
  else if (mask) PSX_BBR(true, false);
  else if (two) PSX_BBR(false, true);
  else PSX_BBR(false, false);
#undef PSX_BBR
  const int e = (int)hipGetLastError();
  return e ? -e : PSX_STAT_SLOTS;
}

int psx_bn_bwd_finalize(const float* part, int T, int NS, int which, int C, float count, const float* gamma,
                        const float* mean, const float* invstd, float* coef, void* dgamma, void* dbeta, float gscale,
                        int grad_fp16, hipStream_t st) {
  const dim3 grid((C + 31) / 32);
  if (grad_fp16)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<uint16_t>, grid, dim3(256), 0, st, part, T, NS, which, C, count, gamma,
                       mean, invstd, coef, (uint16_t*)dgamma, (uint16_t*)dbeta, gscale, (int)det_enabled());
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<float>, grid, dim3(256), 0, st, part, T, NS, which, C, count, gamma,
                       mean, invstd, coef, (float*)dgamma, (float*)dbeta, gscale, (int)det_enabled());
  return (int)hipGetLastError();
}

int psx_bn_bwd_apply(const void* g, const void* o, const void* y1, const float* coef1, void* dx1, const void* y2,
                     const float* coef2, void* dx2, void* dzout, long nelem, int C, int f32, hipStream_t st) {
  if (C % 8 || nelem % 8) return -2;
  const size_t nvec = (size_t)nelem / 8;
  const int grid = ew_grid(nvec);
  const bool mask = o != nullptr, two = y2 != nullptr, dz = dzout != nullptr;
#define PSX_BBA(M, TW, DZ)                                                                                      \
  do {                                                                                                          \
    if (f32)                                                                                                    \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<float, M, TW, DZ>), dim3(grid), dim3(256), 0, st, (const float*)g, \
                         (const float*)o, (const float*)y1, coef1, (float*)dx1, (const float*)y2, coef2,         \
                         (float*)dx2, (float*)dzout, nvec, C);                                                  \
    else                                                                                                        \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<uint16_t, M, TW, DZ>), dim3(grid), dim3(256), 0, st,              \
                         (const uint16_t*)g, (const uint16_t*)o, (const uint16_t*)y1, coef1, (uint16_t*)dx1,    \
                         (const uint16_t*)y2, coef2, (uint16_t*)dx2, (uint16_t*)dzout, nvec, C);                \
  } while (0)
  if (mask && two && dz) PSX_BBA(true, true, true);
  else if (mask && two) PSX_BBA(true, true, false);
  else if (mask && dz) PSX_BBA(true, false, true);
  else if (mask) PSX_BBA(true, false, false);
  else if (two && dz) PSX_BBA(false, true, true);
  else if (two) PSX_BBA(false, true, false);
  else if (dz) PSX_BBA(false, false, true);
  else PSX_BBA(false, false, false);
#undef PSX_BBA
  return (int)hipGetLastError();
}

// Training-mode apply with the finalize folded in: part1/part2 = [PSX_STAT_SLOTS][2][C] slot
// sums of the layer (and of the shortcut BN for mode 2); fin1/fin2 name the side outputs.
int psx_bn_apply_fin(const void* y, const float* part1, const BnFin* fin1, const void* res, const float* part2,
                     const BnFin* fin2, void* out, long nelem, int C, int mode, int relu, int f32, hipStream_t st) {
  if (!fin1) return -10;
  if (C % 8 || nelem % 8) return -2;
  if (fin1->C != C || (mode == 2 && (!fin2 || fin2->C != C))) return -10;
  const size_t nvec = (size_t)nelem / 8;
  int grid = ew_grid(nvec);
  if (grid > fin_grid_cap()) grid = fin_grid_cap();
  const size_t lds = (size_t)(8 * C + 1024) * sizeof(float);  // affines, red [2][C] f64, scratch
  BnFin f1 = *fin1;
  BnFin f2 = fin2 ? *fin2 : BnFin{};
  f1.det = f2.det = (int)det_enabled();
#define PSX_BNAF(M, R)                                                                                        \
  do {                                                                                                        \
    if (f32)                                                                                                  \
      hipLaunchKernelGGL((bn_apply_fin_kernel<float, M, R>), dim3(grid), dim3(256), lds, st, (const float*)y,  \
                         nullptr, nullptr, (const float*)res, nullptr, nullptr, (float*)out, nvec, C, part1,   \
                         part2, f1, f2);                                                                      \
    else                                                                                                      \
      hipLaunchKernelGGL((bn_apply_fin_kernel<uint16_t, M, R>), dim3(grid), dim3(256), lds, st,               \
                         (const uint16_t*)y, nullptr, nullptr, (const uint16_t*)res, nullptr, nullptr,        \
                         (uint16_t*)out, nvec, C, part1, part2, f1, f2);                                      \
  } while (0)
  if (mode == 0 && relu) PSX_BNAF(0, true);
  else if (mode == 0) PSX_BNAF(0, false);
  else if (mode == 1 && relu) PSX_BNAF(1, true);
  else if (mode == 1) PSX_BNAF(1, false);
  else if (mode == 2 && relu) PSX_BNAF(2, true);
  else if (mode == 2) PSX_BNAF(2, false);
  else return -3;
#undef PSX_BNAF
  return (int)hipGetLastError();
}

// Backward apply with the finalize folded in: part = [PSX_STAT_SLOTS][NS][C] slot sums
// (NS = 3 with y2); fin1/fin2 name the coefficient and dgamma/dbeta outputs.
int psx_bn_bwd_apply_fin(const void* g, const void* o, const void* y1, const float* part, const BnBwdFin* fin1,
                         void* dx1, const void* y2, const BnBwdFin* fin2, void* dx2, void* dzout, long nelem, int C,
                         int f32, hipStream_t st) {
  if (!fin1) return -10;
  if (C % 8 || nelem % 8) return -2;
  const bool mask = o != nullptr, two = y2 != nullptr, dz = dzout != nullptr;
  if (fin1->C != C || (two && (!fin2 || fin2->C != C))) return -10;
  const size_t nvec = (size_t)nelem / 8;
  int grid = ew_grid(nvec);
  if (grid > fin_grid_cap()) grid = fin_grid_cap();
  const size_t lds = (size_t)(10 * C + 1024) * sizeof(float);  // coefs, red [2][C] f64, scratch
  BnBwdFin f1 = *fin1;
  BnBwdFin f2 = fin2 ? *fin2 : BnBwdFin{};
  f1.det = f2.det = (int)det_enabled();
#define PSX_BBAF(M, TW, DZ)                                                                                     \
  do {                                                                                                         \
    if (f32)                                                                                                   \
      hipLaunchKernelGGL((bn_bwd_apply_fin_kernel<float, M, TW, DZ>), dim3(grid), dim3(256), lds, st,          \
                         (const float*)g, (const float*)o, (const float*)y1, nullptr, (float*)dx1,             \
                         (const float*)y2, nullptr, (float*)dx2, (float*)dzout, nvec, C, part, f1, f2);        \
    else                                                                                                       \
      hipLaunchKernelGGL((bn_bwd_apply_fin_kernel<uint16_t, M, TW, DZ>), dim3(grid), dim3(256), lds, st,       \
                         (const uint16_t*)g, (const uint16_t*)o, (const uint16_t*)y1, nullptr, (uint16_t*)dx1, \
                         (const uint16_t*)y2, nullptr, (uint16_t*)dx2, (uint16_t*)dzout, nvec, C, part, f1,   \
                         f2);                                                                                  \
  } while (0)
  if (mask && two && dz) PSX_BBAF(true, true, true);
  else if (mask && two) PSX_BBAF(true, true, false);
  else if (mask && dz) PSX_BBAF(true, false, true);
  else if (mask) PSX_BBAF(true, false, false);
  else if (two && dz) PSX_BBAF(false, true, true);
  else if (two) PSX_BBAF(false, true, false);
  else if (dz) PSX_BBAF(false, false, true);
  else PSX_BBAF(false, false, false);
#undef PSX_BBAF
  return (int)hipGetLastError();
}

}  // extern "C"
