// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16.
//
// Replaces the nn.Conv2d forward/backward of the reference ResNet-18
// (reference: src/parameter_server/server.py:24,26,32,48 and the autograd of
// src/workers/worker.py:345) with three hand-written kernels:
//
//   conv_fwd   : Y[pix][oc]   = sum_k im2col(X)[pix][k] * Wf[oc][k]        k = (r,s,c)
//   conv_dgrad : dX[pix][c]   = sum_k im2col'(dY)[pix][k] * Wd[c][k]       k = (r,s,oc)
//   conv_wgrad : dW[oc][k]    = sum_pix dY[pix][oc] * im2col(X)[pix][k]    (split-K over pix)
//
// fwd and dgrad share one kernel body (both GEMM operands K-contiguous, LDS tiles read with
// ds_read_b128); wgrad reduces over the pixel dimension, which is the strided dimension of
// both operands, so its LDS tiles are pixel-major and its MFMA fragments are fetched with the
// gfx950 transposing LDS read ds_read_b64_tr_b16.
//
// MFMA orientation: A = weights (rows = output channels), B = im2col pixels, so the
// accumulator of one lane holds 4 consecutive output channels of one pixel -> each lane
// stores 8 contiguous bytes of the NHWC output.
#include <stdlib.h>

#include "common.hpp"

namespace psx {

struct ConvArgs {
  const uint16_t* in;   // gathered activation, NHWC [Nb][IH][IW][IC]
  const uint16_t* w;    // weights [OC][Kg]  (bf16, K-contiguous, zero padded to Kg)
  uint16_t* out;        // NHWC [Nb][OH][OW][OC]
  const uint16_t* res;  // optional residual added in the epilogue (same shape as out)
  float* stats;         // optional BN partial sums [PSX_STAT_SLOTS][2][OC], pre-zeroed
  int Nb, IH, IW, IC;   // IC: power of two, multiple of 8
  int OH, OW, OC;
  int R, S, pad, stride;
  int Kg;               // padded GEMM-K (multiple of 64)
  int log2_icc;         // log2(IC / 8)
  int npix;             // Nb*OH*OW
  int n_oc_tiles, n_pix_tiles;
};

// LDS byte offset of 16-byte chunk c (0..7) of row r in a K-major tile with 128-byte rows.
// Conflict-free for the ds_read_b128 fragment reads below (lane groups of MI355X_MICROARCH §LDS).
PSX_DEV int kmaj_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int MODE>  // 0 = forward conv gather, 1 = data-grad gather (stride 1), 2 = dgrad stride 2
PSX_DEV u32x4 gather_chunk(const ConvArgs& a, int nbase, int hb, int wb, bool pvalid, int gk) {
  u32x4 v = {0u, 0u, 0u, 0u};
  const int tap = gk >> a.log2_icc;
  const int c0 = (gk & ((1 << a.log2_icc) - 1)) << 3;
  if (!pvalid || tap >= a.R * a.S) return v;
  const int r = tap / a.S;
  const int s = tap - r * a.S;
  int ih, iw;
  if (MODE == 0) {
    ih = hb + r;
    iw = wb + s;
  } else {
    const int th = hb - r, tw = wb - s;
    if (MODE == 2) {
      if ((th | tw) & 1) return v;
      ih = th >> 1;
      iw = tw >> 1;
    } else {
      ih = th;
      iw = tw;
    }
  }
  if ((unsigned)ih >= (unsigned)a.IH || (unsigned)iw >= (unsigned)a.IW) return v;
  const uint16_t* p = a.in + ((size_t)(nbase + ih * a.IW + iw) * a.IC + c0);
  return *reinterpret_cast<const u32x4*>(p);
}

// BM: output-channel tile (MFMA rows); BN: pixel tile (MFMA cols). 4 waves in 2x2.
template <int BM, int BN, int MODE, bool HAS_RES>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  constexpr int BK = 64;
  constexpr int MT = BM / 32, NT = BN / 32;      // 16x16 MFMA tiles per wave
  constexpr int LA = BM / 32, LB = BN / 32;      // 16-byte chunks per thread per k-step
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* sA = smem;                       // [2][BM][128B]
  unsigned char* sB = smem + 2 * BM * 128;        // [2][BN][128B]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nwg = a.n_oc_tiles * a.n_pix_tiles;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int oc_t = tile % a.n_oc_tiles, pix_t = tile / a.n_oc_tiles;
  const int oc0 = oc_t * BM, pix0 = pix_t * BN;

  const int kc = tid & 7;  // this thread's chunk column in every row it loads
  // Per-row gather state for the B (pixel) operand.
  int nbase[LB], hb[LB], wb[LB];
  bool pv[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int pix = pix0 + (tid >> 3) + 32 * i;
    pv[i] = pix < a.npix;
    const int pp = pv[i] ? pix : 0;
    const int ohw = a.OH * a.OW;
    const int n = pp / ohw, rem = pp - n * ohw;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    nbase[i] = n * a.IH * a.IW;
    if (MODE == 0) {
      hb[i] = oh * a.stride - a.pad;
      wb[i] = ow * a.stride - a.pad;
    } else {
      hb[i] = oh + a.pad;
      wb[i] = ow + a.pad;
    }
  }

  const uint16_t* wrow = a.w + (size_t)(oc0 + (tid >> 3)) * a.Kg + kc * 8;
  const int nk = a.Kg / BK;

  u32x4 ra[LA], rb[LB];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < LA; ++i)
      ra[i] = *reinterpret_cast<const u32x4*>(wrow + (size_t)32 * i * a.Kg + ks * BK);
#pragma unroll
    for (int i = 0; i < LB; ++i) rb[i] = gather_chunk<MODE>(a, nbase[i], hb[i], wb[i], pv[i], ks * 8 + kc);
  };
  auto lstore = [&](int stage) {
    unsigned char* A = sA + stage * BM * 128;
    unsigned char* B = sB + stage * BN * 128;
#pragma unroll
    for (int i = 0; i < LA; ++i) *reinterpret_cast<u32x4*>(A + kmaj_off((tid >> 3) + 32 * i, kc)) = ra[i];
#pragma unroll
    for (int i = 0; i < LB; ++i) *reinterpret_cast<u32x4*>(B + kmaj_off((tid >> 3) + 32 * i, kc)) = rb[i];
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();

  const int frow = lane & 15, fchunk = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) gload(ks + 1);
    const unsigned char* A = sA + cur * BM * 128;
    const unsigned char* B = sB + cur * BN * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[MT], fb[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        fa[m] = *reinterpret_cast<const bf16x8*>(A + kmaj_off(wm * (BM / 2) + m * 16 + frow, kk * 4 + fchunk));
#pragma unroll
      for (int n = 0; n < NT; ++n)
        fb[n] = *reinterpret_cast<const bf16x8*>(B + kmaj_off(wn * (BN / 2) + n * 16 + frow, kk * 4 + fchunk));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
    if (ks + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bf16 NHWC store (+residual), optional BN partial statistics ----
  float s1[MT][4], s2[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) s1[m][i] = s2[m][i] = 0.f;

#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int pix = pix0 + wn * (BN / 2) + n * 16 + (lane & 15);
    const bool ok = pix < a.npix;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int oc = oc0 + wm * (BM / 2) + m * 16 + 4 * (lane >> 4);
      float v0 = acc[m][n][0], v1 = acc[m][n][1], v2 = acc[m][n][2], v3 = acc[m][n][3];
      if (ok) {
        const size_t off = (size_t)pix * a.OC + oc;
        if (HAS_RES) {
          const u32x2 rr = *reinterpret_cast<const u32x2*>(a.res + off);
          v0 += lo_bf(rr[0]); v1 += hi_bf(rr[0]); v2 += lo_bf(rr[1]); v3 += hi_bf(rr[1]);
        }
        u32x2 o;
        o[0] = pack_bf2(v0, v1);
        o[1] = pack_bf2(v2, v3);
        *reinterpret_cast<u32x2*>(a.out + off) = o;
        if (a.stats) {  // statistics of the stored (bf16-rounded) values
          const float q0 = lo_bf(o[0]), q1 = hi_bf(o[0]), q2 = lo_bf(o[1]), q3 = hi_bf(o[1]);
          s1[m][0] += q0; s2[m][0] += q0 * q0;
          s1[m][1] += q1; s2[m][1] += q1 * q1;
          s1[m][2] += q2; s2[m][2] += q2 * q2;
          s1[m][3] += q3; s2[m][3] += q3 * q3;
        }
      }
    }
  }
  if (a.stats) {
    // reduce over the 16 pixel lanes that share (lane>>4)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[m][i] += __shfl_xor(s1[m][i], o, 64);
          s2[m][i] += __shfl_xor(s2[m][i], o, 64);
        }
      }
    __syncthreads();  // LDS reuse
    float* red = reinterpret_cast<float*>(smem);  // [2 wn][2][BM]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * (BM / 2) + m * 16 + 4 * (lane >> 4) + i;
          red[(wn * 2 + 0) * BM + row] = s1[m][i];
          red[(wn * 2 + 1) * BM + row] = s2[m][i];
        }
    }
    __syncthreads();
    // fire-and-forget fp32 atomics into one of PSX_STAT_SLOTS slot rows (zeroed once per step);
    // spreading blocks over slots keeps per-address contention low.
    float* dst = a.stats + (size_t)(pix_t & (PSX_STAT_SLOTS - 1)) * 2 * a.OC;
    for (int j = tid; j < 2 * BM; j += 256) {
      const int which = j / BM, row = j - which * BM;
      const float v = red[(0 * 2 + which) * BM + row] + red[(1 * 2 + which) * BM + row];
      atomicAdd(dst + which * a.OC + oc0 + row, v);
    }
  }
}

// ------------------------------------------------------------------------------------
// Weight gradient: dW[oc][k] = sum_pix dY[pix][oc] * im2col(X)[pix][k]
// MFMA rows = k (im2col column), cols = oc. Both LDS tiles are pixel-major [64 pix][64 col]
// and the K=pixel fragments are read with ds_read_b64_tr_b16.
// ------------------------------------------------------------------------------------
struct WgradArgs {
  const uint16_t* x;   // NHWC [Nb][IH][IW][IC]
  const uint16_t* dy;  // NHWC [Nb][OH][OW][OC]
  float* part;         // [splits][OC][Kg] fp32 partial sums
  int Nb, IH, IW, IC, OH, OW, OC, R, S, pad, stride;
  int Kg, log2_icc, npix;
  int n_k_tiles, n_oc_tiles, splits, pix_per_split;  // pix_per_split multiple of 64
};

// Pixel-major tile, 128-byte rows: swizzle chosen so that the 8 rows one 32-lane half of a
// ds_read_b64_tr_b16 touches (rows 8a..8a+7) and their 32-byte column pairs are bank-disjoint.
PSX_DEV int pmaj_off(int r, int c) { return r * 128 + ((c ^ (((r >> 1) & 3) << 1)) << 4); }

PSX_DEV s16x4 tr_read(const unsigned char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + byte_off));
}

__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int BR = 64, BC = 64, BKP = 64;  // k rows, oc cols, pixels per step
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* sX = smem;               // [2][64 pix][128B]
  unsigned char* sD = smem + 2 * 64 * 128;  // [2][64 pix][128B]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = a.n_k_tiles * a.n_oc_tiles;
  const int nwg = ntile * a.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int split = bid / ntile, t = bid - split * ntile;
  const int oc_t = t % a.n_oc_tiles, k_t = t / a.n_oc_tiles;
  const int k0 = k_t * BR, oc0 = oc_t * BC;
  const int pbeg = split * a.pix_per_split;
  const int pend = min(a.npix, pbeg + a.pix_per_split);

  const int kc = tid & 7;
  const int prow = tid >> 3;  // rows prow and prow+32
  const int gk = (k0 >> 3) + kc;
  const int tap = gk >> a.log2_icc;
  const int c0 = (gk & ((1 << a.log2_icc) - 1)) << 3;
  const bool tap_ok = tap < a.R * a.S;
  const int r = tap_ok ? tap / a.S : 0, s = tap_ok ? tap - r * a.S : 0;
  const int ohw = a.OH * a.OW;

  u32x4 rx[2], rd[2];
  auto gload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pix = p0 + prow + 32 * i;
      u32x4 vx = {0u, 0u, 0u, 0u}, vd = {0u, 0u, 0u, 0u};
      if (pix < pend) {
        vd = *reinterpret_cast<const u32x4*>(a.dy + (size_t)pix * a.OC + oc0 + kc * 8);
        if (tap_ok) {
          const int n = pix / ohw, rem = pix - n * ohw;
          const int oh = rem / a.OW, ow = rem - oh * a.OW;
          const int ih = oh * a.stride - a.pad + r, iw = ow * a.stride - a.pad + s;
          if ((unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW)
            vx = *reinterpret_cast<const u32x4*>(a.x + ((size_t)(n * a.IH + ih) * a.IW + iw) * a.IC + c0);
        }
      }
      rx[i] = vx;
      rd[i] = vd;
    }
  };
  auto lstore = [&](int stage) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<u32x4*>(sX + stage * 8192 + pmaj_off(prow + 32 * i, kc)) = rx[i];
      *reinterpret_cast<u32x4*>(sD + stage * 8192 + pmaj_off(prow + 32 * i, kc)) = rd[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nsteps = (pend - pbeg + BKP - 1) / BKP;
  if (nsteps > 0) {
    gload(pbeg);
    lstore(0);
  }
  __syncthreads();

  // tr-read addressing: lane l, group g = l>>4, i = l&15, q = i>>2, p = i&3.
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    if (st + 1 < nsteps) gload(pbeg + (st + 1) * BKP);
    const unsigned char* X = sX + cur * 8192;
    const unsigned char* D = sD + cur * 8192;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      // element j = 4h+e of lane (g, i) <-> pixel row kk*32 + 16h + 4g + e (same for A and B)
      const int row0 = kk * 32 + 4 * g + q, row1 = row0 + 16;
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int col = wm * 32 + m * 16 + 4 * p;  // bf16 column within the 64-col tile
        const s16x4 lo = tr_read(X, pmaj_off(row0, col >> 3) + ((col & 7) << 1));
        const s16x4 hi = tr_read(X, pmaj_off(row1, col >> 3) + ((col & 7) << 1));
        fa[m] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = wn * 32 + n * 16 + 4 * p;
        const s16x4 lo = tr_read(D, pmaj_off(row0, col >> 3) + ((col & 7) << 1));
        const s16x4 hi = tr_read(D, pmaj_off(row1, col >> 3) + ((col & 7) << 1));
        fb[n] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
    if (st + 1 < nsteps) lstore(cur ^ 1);
    __syncthreads();
  }

  // D[row = k][col = oc]: lane holds k = 4(l>>4)+i for oc = l&15 -> 16-byte fp32 store
  float* part = a.part + (size_t)split * a.OC * a.Kg;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int k = k0 + wm * 32 + m * 16 + 4 * (lane >> 4);
      const int oc = oc0 + wn * 32 + n * 16 + (lane & 15);
      *reinterpret_cast<f32x4*>(part + (size_t)oc * a.Kg + k) = acc[m][n];
    }
}

// Sum the split-K partials, permute (oc, r, s, c) -> reference OIHW (oc, c, r, s), drop the
// channel padding and emit the gradient straight into the wire buffer (fp16 codec or fp32).
// Block = 4 waves; each lane owns 4 consecutive partial columns (16-byte loads), the waves split
// the split-K slabs 4 ways (fixed order => deterministic) and combine through LDS.
template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int OC,
                                                           int Kg, int Cin, int IC, int R, int S, float scale,
                                                           OutT* __restrict__ out) {
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t slab = (size_t)OC * Kg;
  const size_t base = (size_t)blockIdx.x * 256 + lane * 4;
  // the 4 waves split the slabs 4 ways; 8 independent 16-byte loads in flight per lane (the
  // reduce is bandwidth work, and with as few as 144 workgroups for a 64x576 layer it is
  // latency-bound unless each lane keeps several slab loads outstanding)
  f32x4 acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int sp = g;
  for (; sp + 28 < splits; sp += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += *reinterpret_cast<const f32x4*>(part + (size_t)(sp + 4 * u) * slab + base);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (sp + 4 * u < splits) acc[u] += *reinterpret_cast<const f32x4*>(part + (size_t)(sp + 4 * u) * slab + base);
  red[g][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (g != 0) return;
  const f32x4 v = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  const int RS = R * S;
  const int oc = (int)(base / Kg);
  int k = (int)(base - (size_t)oc * Kg);  // the 4 columns never straddle a row (Kg % 64 == 0)
  int tap = k / IC, c = k - tap * IC;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (tap < RS && c < Cin) {
      const float val = v[e] * scale;
      const size_t o = ((size_t)oc * Cin + c) * RS + tap;
      if constexpr (sizeof(OutT) == 2) {
        out[o] = __builtin_bit_cast(uint16_t, (_Float16)val);
      } else {
        out[o] = val;
      }
    }
    if (++c == IC) {
      c = 0;
      ++tap;
    }
  }
}

// v2 mapping: workgroup = (output channel oc, chunk of CW input channels) x all R*S taps, so
// its OIHW output [oc][c0..c0+CW)[taps] is one contiguous run (written from an LDS transpose).
// Threads = (item, split group): an item is 4 channels of one tap (one 16-byte load per split),
// G groups take splits g, g+G, ... so a layer with few items still keeps 256 lanes x several
// 16-byte loads in flight (the partials are 2-16 MB per layer; the v1 mapping was latency-bound
// at ~1 TB/s with 4-byte loads and 64 workgroups on layer1).
template <typename OutT>
PSX_DEV void wgrad_reduce2_tile(const float* __restrict__ part, int splits, int Kg, int Cin, int IC, int RS, int CW,
                                float scale, OutT* __restrict__ out, int oc, int c0, int OC, float4* acc,
                                float* tile) {
  const int q = CW >> 2;           // channel quads per tap
  const int items = RS * q;
  const int G = items >= 256 ? 1 : min(splits, 256 / items);
  const size_t slab = (size_t)OC * Kg;
  const float* row = part + (size_t)oc * Kg + c0;
  for (int base = 0; base < items; base += 256 / G) {
    const int t = threadIdx.x;
    const int per = 256 / G;            // items handled per pass
    const int it = base + t % per, g = t / per;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool live = g < G && t % per + base < items && it < items;
    if (live) {
      const int tap = it / q, cq = it % q;
      const float4* src = reinterpret_cast<const float4*>(row + (size_t)tap * IC + cq * 4);
      const size_t st4 = slab / 4;
      int sp = g;
      float4 a1 = s, a2 = s, a3 = s;
      for (; sp + 3 * G < splits; sp += 4 * G) {
        const float4 v0 = src[(size_t)sp * st4], v1 = src[(size_t)(sp + G) * st4];
        const float4 v2 = src[(size_t)(sp + 2 * G) * st4], v3 = src[(size_t)(sp + 3 * G) * st4];
        s.x += v0.x; s.y += v0.y; s.z += v0.z; s.w += v0.w;
        a1.x += v1.x; a1.y += v1.y; a1.z += v1.z; a1.w += v1.w;
        a2.x += v2.x; a2.y += v2.y; a2.z += v2.z; a2.w += v2.w;
        a3.x += v3.x; a3.y += v3.y; a3.z += v3.z; a3.w += v3.w;
      }
      for (; sp < splits; sp += G) {
        const float4 v = src[(size_t)sp * st4];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      s.x += a1.x + a2.x + a3.x; s.y += a1.y + a2.y + a3.y;
      s.z += a1.z + a2.z + a3.z; s.w += a1.w + a2.w + a3.w;
    }
    acc[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < per && base + threadIdx.x < items) {
      float4 r = acc[threadIdx.x];
      for (int gg = 1; gg < G; ++gg) {
        const float4 v = acc[gg * per + threadIdx.x];
        r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
      }
      const int it2 = base + threadIdx.x, tap = it2 / q, c = (it2 % q) * 4;
      tile[(c + 0) * RS + tap] = r.x;
      tile[(c + 1) * RS + tap] = r.y;
      tile[(c + 2) * RS + tap] = r.z;
      tile[(c + 3) * RS + tap] = r.w;
    }
    __syncthreads();
  }
  const int cv = min(CW, Cin - c0);  // valid (unpadded) input channels of this chunk
  if (cv <= 0) return;
  OutT* dst = out + ((size_t)oc * Cin + c0) * RS;
  for (int j = threadIdx.x; j < cv * RS; j += 256) {
    const float val = tile[j] * scale;
    if constexpr (sizeof(OutT) == 2) {
      dst[j] = __builtin_bit_cast(uint16_t, (_Float16)val);
    } else {
      dst[j] = val;
    }
  }
}

template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce2_kernel(const float* __restrict__ part, int splits, int Kg,
                                                            int Cin, int IC, int RS, int CW, float scale,
                                                            OutT* __restrict__ out) {
  __shared__ float4 acc[256];
  __shared__ float tile[64 * 49];  // [c][tap], CW*RS <= 64*49
  wgrad_reduce2_tile<OutT>(part, splits, Kg, Cin, IC, RS, CW, scale, out, blockIdx.x, blockIdx.y * CW, gridDim.x, acc,
                           tile);
}

// Several layers' reductions in one launch (the weight gradients of one residual block are
// reduced together at the end of its backward): flat grid, desc j owns blocks [blk0, blk0 + OC*IC/CW).
constexpr int kWrMax = 4;
struct WrDesc {
  const float* part;
  void* out;
  int splits, Kg, Cin, IC, RS, CW, OC, blk0;
};
struct WrBatch {
  WrDesc d[kWrMax];
  int n;
  float scale;
};

template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce2_batch_kernel(WrBatch b) {
  __shared__ float4 acc[256];
  __shared__ float tile[64 * 49];
  int j = 0;
  while (j + 1 < b.n && b.d[j + 1].blk0 <= (int)blockIdx.x) ++j;
  const WrDesc& d = b.d[j];
  const int local = blockIdx.x - d.blk0;
  const int oc = local % d.OC, c0 = (local / d.OC) * d.CW;
  wgrad_reduce2_tile<OutT>(d.part, d.splits, d.Kg, d.Cin, d.IC, d.RS, d.CW, b.scale, (OutT*)d.out, oc, c0, d.OC, acc,
                           tile);
}

}  // namespace psx

// ------------------------------------------------------------------------------------
// C ABI launchers
// ------------------------------------------------------------------------------------
using namespace psx;

template <int BM, int BN, int MODE, bool RES>
static int launch_conv(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.n_oc_tiles = a.OC / BM;
  b.n_pix_tiles = (a.npix + BN - 1) / BN;
  const size_t lds = (size_t)2 * (BM + BN) * 128;
  const int grid = b.n_oc_tiles * b.n_pix_tiles;
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE, RES>), dim3(grid), dim3(256), lds, st, b);
  return (int)hipGetLastError();
}

template <int MODE, bool RES>
static int dispatch_tile(int tile_cfg, const ConvArgs& a, hipStream_t st) {
  switch (tile_cfg) {
    case 0: return launch_conv<64, 128, MODE, RES>(a, st);
    case 1: return launch_conv<128, 128, MODE, RES>(a, st);
    case 2: return launch_conv<64, 64, MODE, RES>(a, st);
    case 3: return launch_conv<128, 64, MODE, RES>(a, st);
    default: return -1;
  }
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

// Tile selection: output-channel tile (BM) must divide OC; prefer >= 512 workgroups.
static int pick_tile(int OC, int npix) {
  if (OC % 128 == 0 && (long)(OC / 128) * ((npix + 127) / 128) >= 512) return 1;
  if ((long)(OC / 64) * ((npix + 127) / 128) >= 256) return 0;
  if (OC % 128 == 0 && (long)(OC / 128) * ((npix + 63) / 64) >= 256) return 3;
  return 2;
}

extern "C" {

// Forward conv. x: NHWC [Nb][H][W][IC]; wf: [OC][Kg]; y: NHWC [Nb][P][Q][OC].
// stats (nullable, pre-zeroed): BN partial sums [PSX_STAT_SLOTS][2][OC]; *ntiles = PSX_STAT_SLOTS.
int psx_conv_fwd(const void* x, const void* wf, void* y, float* stats, int Nb, int H, int W, int IC, int OC, int R,
                 int S, int stride, int pad, int Kg, int tile_cfg, int* ntiles, hipStream_t st) {
  ConvArgs a{};
  a.in = (const uint16_t*)x;
  a.w = (const uint16_t*)wf;
  a.out = (uint16_t*)y;
  a.res = nullptr;
  a.stats = stats;
  a.Nb = Nb; a.IH = H; a.IW = W; a.IC = IC;
  a.OH = (H + 2 * pad - R) / stride + 1;
  a.OW = (W + 2 * pad - S) / stride + 1;
  a.OC = OC; a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2(IC / 8);
  a.npix = Nb * a.OH * a.OW;
  if (OC % 64 || Kg % 64 || IC % 8 || (IC & (IC - 1))) return -2;
  if (tile_cfg < 0) tile_cfg = pick_tile(OC, a.npix);
  if ((tile_cfg == 1 || tile_cfg == 3) && OC % 128) tile_cfg = (tile_cfg == 1) ? 0 : 2;
  const int BN = (tile_cfg == 0 || tile_cfg == 1) ? 128 : 64;
  if (ntiles) *ntiles = PSX_STAT_SLOTS;
  (void)BN;
  return dispatch_tile<0, false>(tile_cfg, a, st);
}

// Data gradient. dy: NHWC [Nb][P][Q][OC_fwd]; wd: [IC_fwd][Kg'] with Kg' >= R*S*OC_fwd;
// dx: NHWC [Nb][H][W][IC_fwd]; res (nullable) is added to dx.
int psx_conv_dgrad(const void* dy, const void* wd, void* dx, const void* res, int Nb, int H, int W, int IC_fwd,
                   int OC_fwd, int R, int S, int stride, int pad, int Kg, int tile_cfg, hipStream_t st) {
  ConvArgs a{};
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  a.in = (const uint16_t*)dy;
  a.w = (const uint16_t*)wd;
  a.out = (uint16_t*)dx;
  a.res = (const uint16_t*)res;
  a.stats = nullptr;
  a.Nb = Nb; a.IH = P; a.IW = Q; a.IC = OC_fwd;
  a.OH = H; a.OW = W; a.OC = IC_fwd;
  a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2(OC_fwd / 8);
  a.npix = Nb * H * W;
  if (IC_fwd % 64 || Kg % 64 || (OC_fwd & (OC_fwd - 1))) return -2;
  if (tile_cfg < 0) tile_cfg = pick_tile(IC_fwd, a.npix);
  if ((tile_cfg == 1 || tile_cfg == 3) && IC_fwd % 128) tile_cfg = (tile_cfg == 1) ? 0 : 2;
  if (stride == 1) return res ? dispatch_tile<1, true>(tile_cfg, a, st) : dispatch_tile<1, false>(tile_cfg, a, st);
  if (stride == 2) return res ? dispatch_tile<2, true>(tile_cfg, a, st) : dispatch_tile<2, false>(tile_cfg, a, st);
  return -4;
}

// Weight-gradient partials; returns the number of splits used (partials buffer must hold
// splits*OC*Kg floats; query with part == nullptr).
int psx_conv_wgrad(const void* x, const void* dy, float* part, int Nb, int H, int W, int IC, int OC, int R, int S,
                   int stride, int pad, int Kg, int splits, hipStream_t st) {
  WgradArgs a{};
  a.x = (const uint16_t*)x;
  a.dy = (const uint16_t*)dy;
  a.part = part;
  a.Nb = Nb; a.IH = H; a.IW = W; a.IC = IC;
  a.OH = (H + 2 * pad - R) / stride + 1;
  a.OW = (W + 2 * pad - S) / stride + 1;
  a.OC = OC; a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2(IC / 8);
  a.npix = Nb * a.OH * a.OW;
  a.n_k_tiles = Kg / 64;
  a.n_oc_tiles = OC / 64;
  if (OC % 64 || Kg % 64) return -2;
  const int tiles = a.n_k_tiles * a.n_oc_tiles;
  if (splits <= 0) {
    // aim for ~512 workgroups (2 per CU), at least 16 pixel-steps (1024 pixels) per split
    const int max_splits = (a.npix + 1023) / 1024;
    splits = (512 + tiles - 1) / tiles;
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
  }
  int pps = (a.npix + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  splits = (a.npix + pps - 1) / pps;
  a.splits = splits;
  a.pix_per_split = pps;
  if (!part) return splits;
  const size_t lds = 2 * 2 * 64 * 128;
  hipLaunchKernelGGL(conv_wgrad_kernel, dim3(tiles * splits), dim3(256), lds, st, a);
  const int e = (int)hipGetLastError();
  return e ? -e : splits;
}

static int reduce2_cw(int OC, int IC) {
  // chunk width: widest of 64/32/16 channels that still gives >= 1024 workgroups
  int CW = IC < 64 ? IC : 64;
  while (CW > 16 && (long)OC * (IC / CW) < 1024) CW >>= 1;
  return CW;
}

// n <= 4 layers: part/out/splits/OC/Kg/Cin/IC/RS arrays of n entries (host memory); every layer
// needs the v2 reduce (R*S <= 49, IC % 16 == 0). One launch for all of them.
int psx_wgrad_reduce_batch(int n, const float* const* part, void* const* out, const int* splits, const int* OC,
                           const int* Kg, const int* Cin, const int* IC, const int* RS, float scale, int out_fp16,
                           hipStream_t st) {
  if (n < 1 || n > kWrMax) return -2;
  WrBatch b{};
  b.n = n;
  b.scale = scale;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    if (RS[i] > 49 || IC[i] % 16) return -3;
    const int CW = reduce2_cw(OC[i], IC[i]);
    b.d[i] = WrDesc{part[i], out[i], splits[i], Kg[i], Cin[i], IC[i], RS[i], CW, OC[i], blk};
    blk += OC[i] * (IC[i] / CW);
  }
  if (out_fp16)
    hipLaunchKernelGGL(wgrad_reduce2_batch_kernel<uint16_t>, dim3(blk), dim3(256), 0, st, b);
  else
    hipLaunchKernelGGL(wgrad_reduce2_batch_kernel<float>, dim3(blk), dim3(256), 0, st, b);
  return (int)hipGetLastError();
}

int psx_wgrad_reduce(const float* part, int splits, int OC, int Kg, int Cin, int IC, int R, int S, float scale,
                     void* out, int out_fp16, hipStream_t st) {
  if (R * S <= 49 && IC % 16 == 0 && !getenv("PSX_WGRAD_REDUCE_V1")) {
    const int CW = reduce2_cw(OC, IC);
    const dim3 grid(OC, IC / CW);
    if (out_fp16)
      hipLaunchKernelGGL(wgrad_reduce2_kernel<uint16_t>, grid, dim3(256), 0, st, part, splits, Kg, Cin, IC, R * S,
                         CW, scale, (uint16_t*)out);
    else
      hipLaunchKernelGGL(wgrad_reduce2_kernel<float>, grid, dim3(256), 0, st, part, splits, Kg, Cin, IC, R * S, CW,
                         scale, (float*)out);
    return (int)hipGetLastError();
  }
  if (((long)OC * Kg) % 256) return -2;
  const int grid = (int)(((long)OC * Kg) / 256);
  if (out_fp16)
    hipLaunchKernelGGL(wgrad_reduce_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, part, splits, OC, Kg, Cin, IC,
                       R, S, scale, (uint16_t*)out);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<float>, dim3(grid), dim3(256), 0, st, part, splits, OC, Kg, Cin, IC, R,
                       S, scale, (float*)out);
  return (int)hipGetLastError();
}

}  // extern "C"
