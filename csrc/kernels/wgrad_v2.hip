// Weight-gradient implicit GEMM v2: dW[oc][k] = sum_pix dY[pix][oc] * im2col(X)[pix][k]
// (reduction over N*P*Q pixels, split-K over pixel ranges), LDS-DMA staged, 3-stage ring.
//
// Both operands are pixel-major in HBM, so the LDS tiles are pixel-major and the MFMA
// (v_mfma_f32_16x16x32_bf16) fragments along the pixel (reduction) axis are fetched with the
// gfx950 transposing LDS read ds_read_b64_tr_b16. Compared with v1 (conv_gemm.hip):
//   * tiles up to 128 (k) x 128 (oc) — half the LDS fragment traffic per MFMA,
//   * global->LDS by global_load_lds with a per-lane im2col source address (padding = zero
//     page) and the transposed-read swizzle folded into the source address,
//   * pixel -> (n, oh, ow) and tap -> (r, s) by multiply-high division (no integer divide in
//     the main loop), 3 LDS stages with counted vmcnt waits and one barrier per 64 pixels.
// Partial sums go to fp32 slabs [split][OC][Kg] reduced by wgrad_reduce (conv_gemm.hip),
// which also permutes to OIHW and emits the fp16 wire codec.
#include <stdlib.h>

#include "pipeline.hpp"

namespace psx {

struct Wgrad2Args {
  const uint16_t* x;     // NHWC [Nb][IH][IW][IC]
  const uint16_t* dy;    // NHWC [Nb][OH][OW][OC]
  float* part;           // [splits][OC][Kg]
  const uint16_t* zero;  // 16-byte zero page
  int IH, IW, IC, OC, R, S, pad, stride, Kg, log2_icc, npix;
  FastDiv div_ohw, div_ow, div_s;
  int n_k_tiles, n_oc_tiles, splits, steps_per_split;  // steps of 64 pixels
};

// pixel-major tile swizzle for the transposed reads (see conv_gemm.hip pmaj_off for the 128 B
// case; 256 B rows put each row on its own bank row, so 8 rows x 2 chunks need (r&7)<<1).
template <int ROWB>
PSX_DEV int pm2(int r, int c) {
  if constexpr (ROWB == 128) return r * 128 + ((c ^ (((r >> 1) & 3) << 1)) << 4);
  return r * 256 + ((c ^ ((r & 7) << 1)) << 4);
}

PSX_DEV s16x4 tr_read2(const unsigned char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off));
}

template <int BR, int BC, int NS>
__global__ __launch_bounds__(256) void wgrad2_kernel(Wgrad2Args a) {
  constexpr int XROWB = BR * 2, DROWB = BC * 2;           // bytes per pixel row
  constexpr int XCPR = XROWB / 16, DCPR = DROWB / 16;     // 16-byte chunks per row
  constexpr int XRPI = 64 / XCPR, DRPI = 64 / DCPR;       // rows per DMA instruction
  constexpr int LX = 64 / XRPI / 4, LD = 64 / DRPI / 4;   // DMA instructions per wave per stage
  constexpr int XT = 64 * XROWB, DT = 64 * DROWB, STAGE = XT + DT;
  constexpr int MT = BR / 32, NT = BC / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = a.n_k_tiles * a.n_oc_tiles;
  const int bid = xcd_remap(blockIdx.x, ntile * a.splits);
  const int split = bid / ntile, t = bid - split * ntile;
  const int oc_t = t % a.n_oc_tiles, k_t = t / a.n_oc_tiles;
  const int k0 = k_t * BR, oc0 = oc_t * BC;
  const int pbeg = split * a.steps_per_split * 64;
  const int nsteps = min(a.steps_per_split, (a.npix - pbeg + 63) / 64);

  // ---- per-lane DMA state ----
  // X: this lane's row within each instruction and its (logical) k-chunk -> tap / channel
  int xrow[LX], xtap_r[LX], xtap_s[LX], xc0[LX];
  bool xtap_ok[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int row = (i * 4 + wid) * XRPI + lane / XCPR;
    const int pos = lane % XCPR;
    const int c = (XROWB == 128) ? (pos ^ (((row >> 1) & 3) << 1)) : (pos ^ ((row & 7) << 1));
    xrow[i] = row;
    const int gk = (k0 >> 3) + c;
    const int tap = gk >> a.log2_icc;
    xc0[i] = (gk & ((1 << a.log2_icc) - 1)) << 3;
    xtap_ok[i] = tap < a.R * a.S;
    const int r = fdiv(tap, a.div_s);
    xtap_r[i] = r;
    xtap_s[i] = tap - r * a.S;
  }
  int drow[LD], dchunk[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int row = (i * 4 + wid) * DRPI + lane / DCPR;
    const int pos = lane % DCPR;
    drow[i] = row;
    dchunk[i] = (DROWB == 128) ? (pos ^ (((row >> 1) & 3) << 1)) : (pos ^ ((row & 7) << 1));
  }
  const int OW = a.div_ow.d;

  auto issue = [&](int st, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int p0 = pbeg + st * 64;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int pix = p0 + xrow[i];
      const uint16_t* src = a.zero;
      if (pix < a.npix && xtap_ok[i]) {
        const int n = fdiv(pix, a.div_ohw);
        const int rem = pix - n * a.div_ohw.d;
        const int oh = fdiv(rem, a.div_ow);
        const int ow = rem - oh * OW;
        const int ih = oh * a.stride - a.pad + xtap_r[i], iw = ow * a.stride - a.pad + xtap_s[i];
        if ((unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW)
          src = a.x + ((size_t)(n * a.IH + ih) * a.IW + iw) * a.IC + xc0[i];
      }
      glds16(src, base + (i * 4 + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int pix = p0 + drow[i];
      const uint16_t* src = pix < a.npix ? a.dy + (size_t)pix * a.OC + oc0 + dchunk[i] * 8 : a.zero;
      glds16(src, base + XT + (i * 4 + wid) * 1024);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // NS-stage ring: steps st+1 .. st+NS-2 may still be in flight while step st is consumed
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nsteps) issue(i, i);
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  int stage = 0;
  for (int st = 0; st < nsteps; ++st) {
    const int ahead = min(NS - 2, nsteps - 1 - st);  // groups issued after step st's
    if (ahead >= NS - 2)
      wait_vmcnt<(NS - 2) * (LX + LD)>();
    else if (NS > 3 && ahead == 1)
      wait_vmcnt<LX + LD>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + NS - 1 < nsteps) issue(st + NS - 1, stage == 0 ? NS - 1 : stage - 1);
    const unsigned char* X = smem + stage * STAGE;
    const unsigned char* D = X + XT;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int row0 = kk * 32 + 4 * g + q, row1 = row0 + 16;
      bf16x8 fa[MT], fb[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int col = wm * (BR / 2) + m * 16 + 4 * p;
        const s16x4 lo = tr_read2(X, pm2<XROWB>(row0, col >> 3) + ((col & 7) << 1));
        const s16x4 hi = tr_read2(X, pm2<XROWB>(row1, col >> 3) + ((col & 7) << 1));
        fa[m] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int col = wn * (BC / 2) + n * 16 + 4 * p;
        const s16x4 lo = tr_read2(D, pm2<DROWB>(row0, col >> 3) + ((col & 7) << 1));
        const s16x4 hi = tr_read2(D, pm2<DROWB>(row1, col >> 3) + ((col & 7) << 1));
        fb[n] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
    stage = stage == NS - 1 ? 0 : stage + 1;
  }

  float* part = a.part + (size_t)split * a.OC * a.Kg;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int k = k0 + wm * (BR / 2) + m * 16 + 4 * (lane >> 4);
      const int oc = oc0 + wn * (BC / 2) + n * 16 + (lane & 15);
      *reinterpret_cast<f32x4*>(part + (size_t)oc * a.Kg + k) = acc[m][n];
    }
}

}  // namespace psx

using namespace psx;

namespace {

struct WPlan {
  int BR, BC, NS, splits, sps;
};

// LDS bytes per workgroup of an NS-stage BR x BC tile (64 pixels per stage).
constexpr int wlds(int BR, int BC, int NS) { return NS * 64 * (BR + BC) * 2; }

// Occupancy-aware plan: tiles x splits workgroups should fill whole rounds of the
// 256 CUs x (workgroups per CU that the LDS allows), with >= 8 pixel-steps per split; among
// the tile shapes the one with the lowest modelled time wins (per-step costs measured on
// MI355X with rocprofv3: 128x128 ~1.2 us at 1 WG/CU, 64x64 ~0.7 us at 3 WG/CU; +3 us
// prologue/epilogue per workgroup; split-K partials cost a write + a read at ~5 TB/s).
WPlan wplan(int OC, int Kg, int npix) {
  WPlan best{64, 64, 3, 1, 0};
  double best_t = 1e30;
  const int steps = (npix + 63) / 64;
  const int brs[2] = {128, 64}, bcs[2] = {128, 64};
  for (int ib = 0; ib < 2; ++ib)
    for (int ic = 0; ic < 2; ++ic) {
      const int BR = brs[ib], BC = bcs[ic];
      if (Kg % BR || OC % BC || (BR == 128 && Kg < 256)) continue;
      const int NS = (BR == 128 && BC == 128) ? 4 : 3;
      int occ = 163840 / wlds(BR, BC, NS);
      if (occ > 3) occ = 3;
      if (occ < 1) continue;
      const int slots = 256 * occ;
      const long tiles = (long)(Kg / BR) * (OC / BC);
      const double step_us = 0.55 + 0.15 * (double)(BR * BC) / 4096.0;
      int smax = steps / 8 > 0 ? steps / 8 : 1;
      for (int sp = 1; sp <= smax && sp <= 64; ++sp) {
        const int sps = (steps + sp - 1) / sp;
        const int spl = (steps + sps - 1) / sps;
        const long wgs = tiles * spl;
        const long rounds = (wgs + slots - 1) / slots;
        const double t = rounds * (sps * step_us + 3.0) + (spl > 1 ? spl * (double)OC * Kg * 8.0 / 5e6 : 0.0);
        if (t < best_t) {
          best_t = t;
          best = WPlan{BR, BC, NS, spl, sps};
        }
      }
    }
  return best;
}

template <int BR, int BC, int NS>
int launch_w2(const Wgrad2Args& a, hipStream_t st) {
  const size_t lds = (size_t)wlds(BR, BC, NS);
  hipLaunchKernelGGL((wgrad2_kernel<BR, BC, NS>), dim3(a.n_k_tiles * a.n_oc_tiles * a.splits), dim3(256), lds, st,
                     a);
  return (int)hipGetLastError();
}

int ilog2w(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

}  // namespace

extern "C" {

// Returns the split count (query with part == nullptr); partials need splits*OC*Kg floats.
int psx_conv_wgrad2(const void* x, const void* dy, float* part, const void* zero, int Nb, int H, int W, int IC, int OC,
                    int R, int S, int stride, int pad, int Kg, hipStream_t st) {
  Wgrad2Args a{};
  const int OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  a.x = (const uint16_t*)x;
  a.dy = (const uint16_t*)dy;
  a.part = part;
  a.zero = (const uint16_t*)zero;
  a.IH = H; a.IW = W; a.IC = IC; a.OC = OC; a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2w(IC / 8);
  a.npix = Nb * OH * OW;
  a.div_ohw = make_fastdiv(OH * OW);
  a.div_ow = make_fastdiv(OW);
  a.div_s = make_fastdiv(S);
  if (OC % 64 || Kg % 64) return -2;
  WPlan p = wplan(OC, Kg, a.npix);
  // experiment overrides (tile sweep): PSX_WG_BR / PSX_WG_BC / PSX_WG_SPLITS
  if (const char* e = getenv("PSX_WG_BR")) p.BR = atoi(e);
  if (const char* e = getenv("PSX_WG_BC")) p.BC = atoi(e);
  if (const char* e = getenv("PSX_WG_SPLITS")) {
    const int steps = (a.npix + 63) / 64;
    p.sps = (steps + atoi(e) - 1) / atoi(e);
    p.splits = (steps + p.sps - 1) / p.sps;
  }
  if (Kg % p.BR || OC % p.BC) return -2;
  a.n_k_tiles = Kg / p.BR;
  a.n_oc_tiles = OC / p.BC;
  a.splits = p.splits;
  a.steps_per_split = p.sps;
  if (!part) return p.splits;
  int e;
  if (p.BR == 128 && p.BC == 128) e = launch_w2<128, 128, 4>(a, st);
  else if (p.BR == 128) e = launch_w2<128, 64, 3>(a, st);
  else if (p.BC == 128) e = launch_w2<64, 128, 3>(a, st);
  else e = launch_w2<64, 64, 3>(a, st);
  return e ? -e : p.splits;
}

}  // extern "C"
