// Implicit-GEMM convolution v2: LDS-DMA (global_load_lds) operand staging, 3-stage LDS ring
// with counted vmcnt waits, optional split-K. Forward conv and data-gradient conv.
//
// Same math as conv_gemm.hip (v1) — see there for the GEMM formulation and the MFMA
// orientation — but the mainloop is built for CDNA4 latency hiding:
//   * operands go HBM/L2 -> LDS with `global_load_lds_dwordx4` (no VGPR staging). The im2col
//     gather is expressed through the per-lane *source* address (any pixel / tap / channel
//     chunk, zero padding = a pointer to a 16-byte zero page), while the LDS destination stays
//     lane-linear (cdna_hip_programming.md §5 'Async global->LDS copy', rule 21): the XOR swizzle
//     of the K-major tile is applied on the source side and undone on the fragment read.
//   * 3 LDS stages: k-step t+2 is in flight while t is consumed; one raw s_barrier per k-step,
//     preceded by a counted `s_waitcnt vmcnt(N)` that retires only the stage about to be read.
//   * split-K over the GEMM-K dimension (blockIdx.y) for the small-M layers (ResNet stages 3-4),
//     writing fp32 slabs that conv_splitk_epilogue reduces (+ bf16 store, residual, BN stats).
// Kernel selection lives in psx_conv_fwd2 / psx_conv_dgrad2 (shape-driven).
#include <stdlib.h>

#include "bnfin.hpp"
#include "pipeline.hpp"

namespace psx {

struct Conv2Args {
  const uint16_t* in;    // NHWC [Nb][IH][IW][IC] gathered operand
  const uint16_t* w;     // [OC][Kg] bf16 (K-contiguous, zero padded)
  uint16_t* out;         // NHWC [Nb][OH][OW][OC]
  const uint16_t* res;   // optional residual (same shape as out)
  float* stats;          // optional BN partial sums [PSX_STAT_SLOTS][2][OC]
  float* part;           // split-K fp32 slabs [splits][npix][OC]
  const uint16_t* zero;  // 16-byte zero page (DMA source for padding)
  int Nb, IH, IW, IC, OH, OW, OC, R, S, pad, stride;
  int Kg, log2_icc, npix;
  int n_oc_tiles, n_pix_tiles, splits, kps;  // kps: k-steps per split
  int fuse_fin;                              // last workgroup finalizes the BN layer (bnfin.hpp)
  BnFin fin;
  // optional fused BatchNorm-backward reduction over this launch's bf16 output g (dgrad): slot
  // rows [PSX_STAT_SLOTS][bns][OC] of sum(dz), sum(dz*xhat1) [, sum(dz*xhat2)], dz = g*[o > 0],
  // xhat = (y - mean) * invstd — what bn_bwd_reduce (bn.hip) would compute in a separate pass.
  float* bpart;
  const uint16_t* bo;
  const uint16_t* by1;
  const uint16_t* by2;
  const float* bsaved1;  // [2][OC] mean, invstd
  const float* bsaved2;
  int bns;
};

PSX_DEV int kmaj2(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int MODE>
PSX_DEV const uint16_t* gather_src(const Conv2Args& a, int nbase, int hb, int wb, bool pv, int gk) {
  const int tap = gk >> a.log2_icc;
  const int c0 = (gk & ((1 << a.log2_icc) - 1)) << 3;
  if (!pv || tap >= a.R * a.S) return a.zero;
  const int r = tap / a.S, s = tap - r * a.S;
  int ih, iw;
  if (MODE == 0) {
    ih = hb + r;
    iw = wb + s;
  } else {
    const int th = hb - r, tw = wb - s;
    if (MODE == 2) {
      if ((th | tw) & 1) return a.zero;
      ih = th >> 1;
      iw = tw >> 1;
    } else {
      ih = th;
      iw = tw;
    }
  }
  if ((unsigned)ih >= (unsigned)a.IH || (unsigned)iw >= (unsigned)a.IW) return a.zero;
  return a.in + ((size_t)(nbase + ih * a.IW + iw) * a.IC + c0);
}

// WGM = waves along the output-channel (M) axis, 4 / WGM along pixels: 2 (2x2 waves, wave tile
// BM/2 x BN/2) or 1 (1x4 waves: every wave holds all BM channels of a BN/4 pixel slice, e.g. a
// 64x64 wave tile for BM = 64, BN = 256 — 2/3 of the LDS fragment bytes per MFMA of 32x64).
//
// TAPR (3x3 / stride 1 / pad 1, MODE 0 or 1, tiles of whole image rows): tap-reuse mainloop.
// A macro step = (kernel row r, 64-channel chunk): the three weight tiles of taps (r, 0..2) and
// ONE window X of the tile's BN pixels at (row r, centre column) are staged; pixel j of tap s
// reads window slot j + d(s) (d = s - 1 forward, 1 - s dgrad: ih = oh + pad - r there) or a zero
// row when its column leaves the image row. The im2col operand is staged once per kernel row
// instead of once per tap (1/3 of the L2->LDS bytes of the gathered operand); 2 LDS stages.
// TAPR = 1: tiles of whole image rows (power-of-two widths); TAPR = 2 ("halo", any width, e.g.
// ResNet-50's 56/28/14/7): the window also holds the pixel before and after the tile (slot k =
// pixel pix0 - 1 + k), so a shift never leaves the staged rows; the zero row sits at slot BN + 2.
template <int BM, int BN, int MODE, bool HAS_RES, bool SPLIT, int WGM = 2, int TAPR = 0>
__global__ __launch_bounds__(256) void conv2_kernel(Conv2Args a) {
  constexpr int NSTAGE = 3;
  constexpr int WGN = 4 / WGM;
  constexpr int MT = BM / (16 * WGM), NT = BN / (16 * WGN);  // 16x16 MFMA tiles per wave
  constexpr int LA = BM / 32, LB = BN / 32;   // DMA instructions per wave per stage
  constexpr int STAGE = (BM + BN) * 128;      // bytes per stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int nwg = a.n_oc_tiles * a.n_pix_tiles;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int oc_t = tile % a.n_oc_tiles, pix_t = tile / a.n_oc_tiles;
  const int oc0 = oc_t * BM, pix0 = pix_t * BN;
  const int split = SPLIT ? blockIdx.y : 0;
  const int ks0 = split * a.kps;
  int nk = SPLIT ? min(a.kps, a.Kg / 64 - ks0) : a.Kg / 64;
  // MODE 3 = stride-2 dgrad, one parity class (py, px) of dx per blockIdx.y: dx(2i+py, 2j+px)
  // only receives taps r = r0, r0+2, .. and s = s0, s0+2, .. (r0 = (py+pad)&1), i.e. a dense
  // GEMM over 1, 2, 2 or 4 of the 9 taps instead of 9 with 3/4 of the products zero.
  const int cls = MODE == 3 ? blockIdx.y : 0;
  const int py = cls >> 1, px = cls & 1;
  const int CH = (a.OH - py + 1) >> 1, CW = (a.OW - px + 1) >> 1;
  const int r0 = (py + a.pad) & 1, s0 = (px + a.pad) & 1;
  const int nr = r0 < a.R ? (a.R - r0 + 1) >> 1 : 0, nsx = s0 < a.S ? (a.S - s0 + 1) >> 1 : 0;
  const int npix_c = MODE == 3 ? a.Nb * CH * CW : a.npix;
  if (MODE == 3) {
    nk = (nr * nsx) << (a.log2_icc - 3);
    if (pix0 >= npix_c) return;  // whole workgroup: this class has fewer tiles
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if constexpr (TAPR) {
    static_assert(MODE == 0 || MODE == 1, "tap reuse: forward or stride-1 dgrad");
    constexpr bool HALO = TAPR == 2;
    constexpr int XROWS = HALO ? BN + 8 : BN + 1, ZS = HALO ? BN + 2 : BN;  // window rows, zero slot
    constexpr int XOFF = 3 * BM * 128, TST = XOFF + XROWS * 128;            // A0 A1 A2 | X
    const int nch = a.IC >> 6, nmac = 3 * nch;
    const int W = a.OW, log2w = __builtin_ctz(W);
    const int lrow = lane >> 3, lpos = lane & 7;
    if (!HALO && tid < 16)  // (the halo DMA writes zeros into slots BN+2.. of every stage itself)
      *reinterpret_cast<uint4*>(smem + (tid >> 3) * TST + XOFF + BN * 128 + (tid & 7) * 16) = uint4{0u, 0u, 0u, 0u};
    const uint16_t* wsrc[LA];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = (i * 4 + wid) * 8 + lrow;
      wsrc[i] = a.w + (size_t)(oc0 + row) * a.Kg + (lpos ^ ((row >> 1) & 7)) * 8;
    }
    // window rows: the tile's own pixels (input pixel index == output pixel index at s1/p1);
    // halo mode: slot k = pixel pix0 - 1 + k, and wave 0 also stages slots BN .. BN+7 (the two
    // halo pixels, then zeros from the zero page)
    constexpr int LX = LB + (HALO ? 1 : 0);
    const uint16_t* xsrc[LX];
    int xoh[LX];
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int row = i < LB ? (i * 4 + wid) * 8 + lrow : BN + lrow;
      const int pix = pix0 + row - (HALO ? 1 : 0);
      const bool ok = HALO ? (pix >= 0 && pix < a.npix && (i < LB || lrow < 2)) : true;
      xoh[i] = !ok ? -(1 << 20) : HALO ? (pix / W) % a.OH : (pix >> log2w) & (a.OH - 1);
      xsrc[i] = ok ? a.in + (size_t)pix * a.IC + (lpos ^ ((row >> 1) & 7)) * 8 : a.zero;
    }
    auto issue_t = [&](int t, int stage) {
      unsigned char* base = smem + stage * TST;
      const int r = __builtin_amdgcn_readfirstlane(t / nch);
      const int cc = t - r * nch;
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const int kofs = (r * 3 + sx) * a.IC + cc * 64;
#pragma unroll
        for (int i = 0; i < LA; ++i) glds16(wsrc[i] + kofs, base + sx * BM * 128 + (i * 4 + wid) * 1024);
      }
      const int dr = MODE == 0 ? r - 1 : 1 - r;
      const long uoff = (long)dr * W * a.IC + cc * 64;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const uint16_t* src = (unsigned)(xoh[i] + dr) < (unsigned)a.OH ? xsrc[i] + uoff : a.zero;
        glds16(src, base + XOFF + (i * 4 + wid) * 1024);
      }
      if (HALO && wid == 0) {
        const uint16_t* src = (unsigned)(xoh[LX - 1] + dr) < (unsigned)a.OH ? xsrc[LX - 1] + uoff : a.zero;
        glds16(src, base + XOFF + BN * 128);
      }
    };
    // per-lane B-fragment byte offsets of the three taps (tile starts on an image row)
    const int frow = lane & 15, fch = lane >> 4;
    int boff[NT][3];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int prow = wn * (BN / WGN) + n * 16 + frow;
      const int ow = HALO ? (pix0 + prow) % W : prow & (W - 1);
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const int d = MODE == 0 ? sx - 1 : 1 - sx;
        const int slot = (unsigned)(ow + d) < (unsigned)W ? prow + d + (HALO ? 1 : 0) : ZS;
        boff[n][sx] = slot * 128 + ((fch ^ ((slot >> 1) & 7)) << 4);
      }
    }
    __syncthreads();  // zero rows written
    if (nmac > 0) issue_t(0, 0);
    for (int t = 0; t < nmac; ++t) {
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + 1 < nmac) issue_t(t + 1, (t + 1) & 1);
      const unsigned char* base = smem + (t & 1) * TST;
      const unsigned char* X = base + XOFF;
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const unsigned char* A = base + sx * BM * 128;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 fa[MT], fb[NT];
#pragma unroll
          for (int m = 0; m < MT; ++m)
            fa[m] = *reinterpret_cast<const bf16x8*>(A + kmaj2(wm * (BM / WGM) + m * 16 + frow, kk * 4 + fch));
#pragma unroll
          for (int n = 0; n < NT; ++n) fb[n] = *reinterpret_cast<const bf16x8*>(X + (boff[n][sx] ^ (kk << 6)));
#pragma unroll
          for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
        }
      }
    }
  } else {
  // ---- per-lane DMA source state (fixed across k-steps) ----
  const int lrow = lane >> 3, lpos = lane & 7;
  const uint16_t* wsrc[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = (i * 4 + wid) * 8 + lrow;
    const int c = lpos ^ ((row >> 1) & 7);
    wsrc[i] = a.w + (size_t)(oc0 + row) * a.Kg + c * 8;
  }
  int nbase[LB], hb[LB], wb[LB], bc[LB];
  bool pv[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int row = (i * 4 + wid) * 8 + lrow;
    bc[i] = lpos ^ ((row >> 1) & 7);
    const int pix = pix0 + row;
    pv[i] = pix < npix_c;
    const int pp = pv[i] ? pix : 0;
    const int pw = MODE == 3 ? CW : a.OW;
    const int ohw = (MODE == 3 ? CH : a.OH) * pw;
    const int n = pp / ohw, rem = pp - n * ohw;
    const int oh = rem / pw, ow = rem - oh * pw;
    nbase[i] = n * a.IH * a.IW;
    if (MODE == 3) {  // class-local (i, j)
      hb[i] = oh;
      wb[i] = ow;
    } else if (MODE == 0) {
      hb[i] = oh * a.stride - a.pad;
      wb[i] = ow * a.stride - a.pad;
    } else {
      hb[i] = oh + a.pad;
      wb[i] = ow + a.pad;
    }
  }

  // Uniform-tap fast path: with >= 64 (padded) channels a 64-wide k-step lies inside one tap,
  // so tap -> (r, s) and the channel offset are per-step scalars and a lane only adds a
  // uniform offset to its precomputed pixel pointer (+ two bounds compares). The generic
  // gather_src (integer division per lane per DMA) left the kernel VALU-bound: 14 VALU per
  // MFMA measured with rocprofv3 (SQ_INSTS_VALU / SQ_INSTS_MFMA); -7% time per conv.
  // (A persistent variant that streams the ring across tiles was measured 1.3-2x slower: the
  // epilogue's stores/atomics share vmcnt with the prefetches and force a drain per tile.)
  const bool utap = a.log2_icc >= 3;
  const uint16_t* pbase[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    // MODE 0: pixel (hb, wb) = top-left tap; MODE 1: (hb, wb) = (oh, ow) + pad, taps subtract
    const long off = MODE == 2 ? 0 : ((long)nbase[i] + (long)hb[i] * a.IW + wb[i]) * a.IC + bc[i] * 8;
    // MODE 3: pbase = dy(n, i, j); a class tap adds the uniform offset (dr, ds) = ((py+pad-r)/2, ..)
    pbase[i] = a.in + off;
  }
  const int ksh = a.log2_icc - 3;  // k-steps per tap = 1 << ksh (utap only)

  auto issue = [&](int ks, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int kglob = ks0 + ks;
    if (MODE == 3) {
      const int t = __builtin_amdgcn_readfirstlane(ks >> ksh);
      const int cofs = __builtin_amdgcn_readfirstlane((ks & ((1 << ksh) - 1)) << 6);
      const int tr = __builtin_amdgcn_readfirstlane(t / nsx);
      const int r = r0 + 2 * tr, sx = s0 + 2 * (t - tr * nsx);
      const int kg = ((r * a.S + sx) << ksh) + (ks & ((1 << ksh) - 1));  // k-step in the full weights
#pragma unroll
      for (int i = 0; i < LA; ++i) glds16(wsrc[i] + kg * 64, base + (i * 4 + wid) * 1024);
      const int dr = (py + a.pad - r) >> 1, ds = (px + a.pad - sx) >> 1;
      const long uoff = ((long)dr * a.IW + ds) * a.IC + cofs;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const uint16_t* src = a.zero;
        if (pv[i] && (unsigned)(hb[i] + dr) < (unsigned)a.IH && (unsigned)(wb[i] + ds) < (unsigned)a.IW)
          src = pbase[i] + uoff;
        glds16(src, base + BM * 128 + (i * 4 + wid) * 1024);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) glds16(wsrc[i] + kglob * 64, base + (i * 4 + wid) * 1024);
    if (utap) {
      const int tap = __builtin_amdgcn_readfirstlane(kglob >> ksh);
      const int cofs = __builtin_amdgcn_readfirstlane((kglob & ((1 << ksh) - 1)) << 6);
      const int r = __builtin_amdgcn_readfirstlane(tap / a.S);
      const int sx = tap - r * a.S;
      const bool tap_ok = tap < a.R * a.S;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const uint16_t* src = a.zero;
        if (MODE == 0) {
          const long uoff = ((long)r * a.IW + sx) * a.IC + cofs;
          if (tap_ok && pv[i] && (unsigned)(hb[i] + r) < (unsigned)a.IH && (unsigned)(wb[i] + sx) < (unsigned)a.IW)
            src = pbase[i] + uoff;
        } else if (MODE == 1) {
          const long uoff = cofs - ((long)r * a.IW + sx) * a.IC;
          if (tap_ok && pv[i] && (unsigned)(hb[i] - r) < (unsigned)a.IH && (unsigned)(wb[i] - sx) < (unsigned)a.IW)
            src = pbase[i] + uoff;
        } else {
          const int th = hb[i] - r, tw = wb[i] - sx;
          if (tap_ok && pv[i] && !((th | tw) & 1) && (unsigned)(th >> 1) < (unsigned)a.IH &&
              (unsigned)(tw >> 1) < (unsigned)a.IW)
            src = a.in + ((size_t)(nbase[i] + (th >> 1) * a.IW + (tw >> 1)) * a.IC + cofs + bc[i] * 8);
        }
        glds16(src, base + BM * 128 + (i * 4 + wid) * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < LB; ++i)
        glds16(gather_src<MODE>(a, nbase[i], hb[i], wb[i], pv[i], kglob * 8 + bc[i]),
               base + BM * 128 + (i * 4 + wid) * 1024);
    }
  };

  if (nk > 0) issue(0, 0);
  if (nk > 1) issue(1, 1);
  const int frow = lane & 15, fch = lane >> 4;
  int stage = 0;
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk)
      wait_vmcnt<LA + LB>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ks + 2 < nk) issue(ks + 2, stage == 0 ? 2 : stage - 1);
    const unsigned char* A = smem + stage * STAGE;
    const unsigned char* B = A + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[MT], fb[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        fa[m] = *reinterpret_cast<const bf16x8*>(A + kmaj2(wm * (BM / WGM) + m * 16 + frow, kk * 4 + fch));
#pragma unroll
      for (int n = 0; n < NT; ++n)
        fb[n] = *reinterpret_cast<const bf16x8*>(B + kmaj2(wn * (BN / WGN) + n * 16 + frow, kk * 4 + fch));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
    stage = stage == 2 ? 0 : stage + 1;
  }
  }  // generic mainloop

  if constexpr (SPLIT) {
    float* dst = a.part + (size_t)split * a.npix * a.OC;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int pix = pix0 + wn * (BN / WGN) + n * 16 + (lane & 15);
      if (pix >= a.npix) continue;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int oc = oc0 + wm * (BM / WGM) + m * 16 + 4 * (lane >> 4);
        *reinterpret_cast<f32x4*>(dst + (size_t)pix * a.OC + oc) = acc[m][n];
      }
    }
    return;
  }

  // ---- LDS-staged epilogue (PSX_CV_EPI=0 builds keep the fragment epilogue) ----
  // The fp32 tile goes through LDS once; then every thread owns 8 channels of a pixel row, so the
  // bf16 output, the residual and the BN-backward operands o / y move as whole 16-byte chunks of
  // 128-byte rows (the fragment layout touched 32-byte pieces of 16 rows per instruction), and
  // the per-channel sums need one shuffle tree + one LDS pass per workgroup.
#ifndef PSX_CV_EPI
#define PSX_CV_EPI 1
#endif
  if constexpr (PSX_CV_EPI) {
    constexpr int TS = BM + 4;      // fp32 row stride of the staged tile (spreads the banks)
    constexpr int CPR = BM / 8;     // 16-byte bf16 chunks per pixel row
    constexpr int RPP = 256 / CPR;  // pixel rows per pass
    constexpr int LDSB = TAPR ? 2 * (3 * BM * 128 + (TAPR == 2 ? BN + 8 : BN + 1) * 128)
                              : 3 * (BM + BN) * 128;  // launched
    static_assert(256 % CPR == 0 && BN * TS * 4 <= LDSB, "staged tile fits the mainloop LDS");
    float* T = reinterpret_cast<float*>(smem);
    __syncthreads();  // every wave is done with the mainloop's LDS
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int pr = wn * (BN / WGN) + n * 16 + (lane & 15);
#pragma unroll
      for (int m = 0; m < MT; ++m)
        *reinterpret_cast<f32x4*>(T + pr * TS + wm * (BM / WGM) + m * 16 + 4 * (lane >> 4)) = acc[m][n];
    }
    __syncthreads();
    const bool bwd = a.bpart != nullptr, two = a.by2 != nullptr, st = a.stats != nullptr;
    const int cc = tid % CPR, ch0 = oc0 + cc * 8;
    float s1[8], s2[8], s3[8], bm1[8], bi1[8], bm2[8], bi2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s1[i] = s2[i] = s3[i] = 0.f;
      bm1[i] = bi1[i] = bm2[i] = bi2[i] = 0.f;
      if (bwd) {
        bm1[i] = a.bsaved1[ch0 + i];
        bi1[i] = a.bsaved1[a.OC + ch0 + i];
        if (two) {
          bm2[i] = a.bsaved2[ch0 + i];
          bi2[i] = a.bsaved2[a.OC + ch0 + i];
        }
      }
    }
    for (int pr = tid / CPR; pr < BN; pr += RPP) {
      const int pix = pix0 + pr;
      if (pix >= npix_c) break;
      const float* src = T + pr * TS + cc * 8;
      const f32x4 va = *reinterpret_cast<const f32x4*>(src), vb = *reinterpret_cast<const f32x4*>(src + 4);
      float v[8] = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
      size_t opix = (size_t)pix;
      if (MODE == 3) {  // class-local (n, i, j) -> dx (n, 2i+py, 2j+px)
        const int nn = pix / (CH * CW), rem = pix - nn * CH * CW, ii = rem / CW, jj = rem - ii * CW;
        opix = ((size_t)nn * a.OH + 2 * ii + py) * a.OW + 2 * jj + px;
      }
      const size_t off = opix * a.OC + ch0;
      if (HAS_RES) {
        const u32x4 rr = *reinterpret_cast<const u32x4*>(a.res + off);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += lo_bf(rr[k]);
          v[2 * k + 1] += hi_bf(rr[k]);
        }
      }
      u32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
      *reinterpret_cast<u32x4*>(a.out + off) = o;
      if (st) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float q0 = lo_bf(o[k]), q1 = hi_bf(o[k]);
          s1[2 * k] += q0; s2[2 * k] += q0 * q0;
          s1[2 * k + 1] += q1; s2[2 * k + 1] += q1 * q1;
        }
      }
      if (bwd) {
        const u32x4 om = *reinterpret_cast<const u32x4*>(a.bo + off);
        const u32x4 yv = *reinterpret_cast<const u32x4*>(a.by1 + off);
        u32x4 y2v = {0u, 0u, 0u, 0u};
        if (two) y2v = *reinterpret_cast<const u32x4*>(a.by2 + off);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = i >> 1;
          const bool hi = i & 1;
          const float g = hi ? hi_bf(o[k]) : lo_bf(o[k]);
          const float dz = (hi ? hi_bf(om[k]) : lo_bf(om[k])) > 0.f ? g : 0.f;
          s1[i] += dz;
          s2[i] += dz * ((hi ? hi_bf(yv[k]) : lo_bf(yv[k])) - bm1[i]) * bi1[i];
          if (two) s3[i] += dz * ((hi ? hi_bf(y2v[k]) : lo_bf(y2v[k])) - bm2[i]) * bi2[i];
        }
      }
    }
    if (!st && !bwd) return;
    // lanes of one wave that own the same channels differ in the lane bits >= log2(CPR)
#pragma unroll
    for (int sh = CPR; sh < 64; sh <<= 1)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s1[i] += __shfl_xor(s1[i], sh, 64);
        s2[i] += __shfl_xor(s2[i], sh, 64);
        if (two) s3[i] += __shfl_xor(s3[i], sh, 64);
      }
    __syncthreads();  // the staged tile is no longer read
    float* red = T;   // [4 waves][3][BM]
    if (lane < CPR) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        red[(wid * 3 + 0) * BM + cc * 8 + i] = s1[i];
        red[(wid * 3 + 1) * BM + cc * 8 + i] = s2[i];
        red[(wid * 3 + 2) * BM + cc * 8 + i] = s3[i];
      }
    }
    __syncthreads();
    const int nst = bwd ? a.bns : 2;
    float* dst = (bwd ? a.bpart : a.stats) + (size_t)(pix_t & (PSX_STAT_SLOTS - 1)) * nst * a.OC;
    for (int j = tid; j < nst * BM; j += 256) {
      const int which = j / BM, row = j - which * BM;
      const float v = red[which * BM + row] + red[(3 + which) * BM + row] + red[(6 + which) * BM + row] +
                      red[(9 + which) * BM + row];
      atomicAdd(dst + which * a.OC + oc0 + row, v);
    }
    if (st && a.fuse_fin && last_block_arrive(a.fin.counter, gridDim.x, smem))
      bn_finalize_block<PSX_STAT_SLOTS>(a.stats, a.fin);
    return;
  }

  // ---- epilogue: bf16 NHWC store (+residual), BN partial statistics ----
  float s1[MT][4], s2[MT][4], s3[MT][4];
  float bm1[MT][4], bi1[MT][4], bm2[MT][4], bi2[MT][4];
  const bool bwd = a.bpart != nullptr, two = a.by2 != nullptr;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s1[m][i] = s2[m][i] = s3[m][i] = 0.f;
      const int ch = oc0 + wm * (BM / WGM) + m * 16 + 4 * (lane >> 4) + i;
      if (bwd) {
        bm1[m][i] = a.bsaved1[ch];
        bi1[m][i] = a.bsaved1[a.OC + ch];
        if (two) {
          bm2[m][i] = a.bsaved2[ch];
          bi2[m][i] = a.bsaved2[a.OC + ch];
        }
      }
    }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int pix = pix0 + wn * (BN / WGN) + n * 16 + (lane & 15);
    const bool ok = pix < npix_c;
    size_t opix = (size_t)pix;
    if (MODE == 3 && ok) {  // class-local (n, i, j) -> dx (n, 2i+py, 2j+px)
      const int nn = pix / (CH * CW), rem = pix - nn * CH * CW, ii = rem / CW, jj = rem - ii * CW;
      opix = ((size_t)nn * a.OH + 2 * ii + py) * a.OW + 2 * jj + px;
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int oc = oc0 + wm * (BM / WGM) + m * 16 + 4 * (lane >> 4);
      float v0 = acc[m][n][0], v1 = acc[m][n][1], v2 = acc[m][n][2], v3 = acc[m][n][3];
      if (ok) {
        const size_t off = opix * a.OC + oc;
        if (HAS_RES) {
          const u32x2 rr = *reinterpret_cast<const u32x2*>(a.res + off);
          v0 += lo_bf(rr[0]); v1 += hi_bf(rr[0]); v2 += lo_bf(rr[1]); v3 += hi_bf(rr[1]);
        }
        u32x2 o;
        o[0] = pack_bf2(v0, v1);
        o[1] = pack_bf2(v2, v3);
        *reinterpret_cast<u32x2*>(a.out + off) = o;
        if (a.stats) {
          const float q0 = lo_bf(o[0]), q1 = hi_bf(o[0]), q2 = lo_bf(o[1]), q3 = hi_bf(o[1]);
          s1[m][0] += q0; s2[m][0] += q0 * q0;
          s1[m][1] += q1; s2[m][1] += q1 * q1;
          s1[m][2] += q2; s2[m][2] += q2 * q2;
          s1[m][3] += q3; s2[m][3] += q3 * q3;
        }
        if (bwd) {
          const u32x2 om = *reinterpret_cast<const u32x2*>(a.bo + off);
          const u32x2 yv = *reinterpret_cast<const u32x2*>(a.by1 + off);
          u32x2 y2v = {0u, 0u};
          if (two) y2v = *reinterpret_cast<const u32x2*>(a.by2 + off);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t w = i < 2 ? o[0] : o[1], mw = i < 2 ? om[0] : om[1];
            const uint32_t yw = i < 2 ? yv[0] : yv[1], y2w = i < 2 ? y2v[0] : y2v[1];
            const bool hi = i & 1;
            const float g = hi ? hi_bf(w) : lo_bf(w);
            const float dz = (hi ? hi_bf(mw) : lo_bf(mw)) > 0.f ? g : 0.f;
            s1[m][i] += dz;
            s2[m][i] += dz * ((hi ? hi_bf(yw) : lo_bf(yw)) - bm1[m][i]) * bi1[m][i];
            if (two) s3[m][i] += dz * ((hi ? hi_bf(y2w) : lo_bf(y2w)) - bm2[m][i]) * bi2[m][i];
          }
        }
      }
    }
  }
  if (bwd) {  // [2 wn][NS][BM] in LDS, then one atomic per (stat, channel) into the slot row
    const int NSr = a.bns;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[m][i] += __shfl_xor(s1[m][i], o, 64);
          s2[m][i] += __shfl_xor(s2[m][i], o, 64);
          if (two) s3[m][i] += __shfl_xor(s3[m][i], o, 64);
        }
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * (BM / WGM) + m * 16 + 4 * (lane >> 4) + i;
          red[(wn * 3 + 0) * BM + row] = s1[m][i];
          red[(wn * 3 + 1) * BM + row] = s2[m][i];
          red[(wn * 3 + 2) * BM + row] = s3[m][i];
        }
    }
    __syncthreads();
    float* dst = a.bpart + (size_t)(pix_t & (PSX_STAT_SLOTS - 1)) * NSr * a.OC;
    for (int j = tid; j < NSr * BM; j += 256) {
      const int which = j / BM, row = j - which * BM;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WGN; ++w) v += red[(w * 3 + which) * BM + row];
      atomicAdd(dst + which * a.OC + oc0 + row, v);
    }
  }
  if (a.stats) {
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
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [2 wn][2][BM]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * (BM / WGM) + m * 16 + 4 * (lane >> 4) + i;
          red[(wn * 2 + 0) * BM + row] = s1[m][i];
          red[(wn * 2 + 1) * BM + row] = s2[m][i];
        }
    }
    __syncthreads();
    float* dst = a.stats + (size_t)(pix_t & (PSX_STAT_SLOTS - 1)) * 2 * a.OC;
    for (int j = tid; j < 2 * BM; j += 256) {
      const int which = j / BM, row = j - which * BM;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WGN; ++w) v += red[(w * 2 + which) * BM + row];
      atomicAdd(dst + which * a.OC + oc0 + row, v);
    }
    if (a.fuse_fin && last_block_arrive(a.fin.counter, gridDim.x, smem))
      bn_finalize_block<PSX_STAT_SLOTS>(a.stats, a.fin);
  }
}

// Split-K epilogue: out = bf16(sum_s part[s] (+res)); BN partial statistics into slot rows.
// Block = 256 threads; thread owns 8 channels of a pixel; blocks stride over pixel ranges.
template <bool HAS_RES>
__global__ __launch_bounds__(256) void conv_splitk_epilogue(const float* __restrict__ part, int splits, int npix,
                                                            int OC, uint16_t* __restrict__ out,
                                                            const uint16_t* __restrict__ res,
                                                            float* __restrict__ stats, int pix_per_block,
                                                            int fuse_fin, BnFin fin, float* __restrict__ bpart,
                                                            const uint16_t* __restrict__ bo,
                                                            const uint16_t* __restrict__ by1,
                                                            const uint16_t* __restrict__ by2,
                                                            const float* __restrict__ bsaved1,
                                                            const float* __restrict__ bsaved2, int bns) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [256][24]
  const int cvec = OC >> 3, tpp = 256 / cvec;
  const int cg = threadIdx.x % cvec, pr = threadIdx.x / cvec;
  const size_t slab = (size_t)npix * OC;
  // per-thread partial sums: fwd stats (sum, sumsq) or fused BN-backward (dz, dz*xh1, dz*xh2)
  const bool bwd = bpart != nullptr, two = by2 != nullptr;
  const int nst = bwd ? bns : 2;
  float st[3][8], m1[8], i1[8], m2[8], i2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    st[0][j] = st[1][j] = st[2][j] = 0.f;
    if (bwd) {
      m1[j] = bsaved1[cg * 8 + j];
      i1[j] = bsaved1[OC + cg * 8 + j];
      if (two) {
        m2[j] = bsaved2[cg * 8 + j];
        i2[j] = bsaved2[OC + cg * 8 + j];
      }
    }
  }
  const int pbeg = blockIdx.x * pix_per_block, pend = min(npix, pbeg + pix_per_block);
  for (int p = pbeg + pr; p < pend; p += tpp) {
    const size_t off = (size_t)p * OC + cg * 8;
    f32x4 x0 = *reinterpret_cast<const f32x4*>(part + off);
    f32x4 x1 = *reinterpret_cast<const f32x4*>(part + off + 4);
    for (int s = 1; s < splits; ++s) {
      x0 += *reinterpret_cast<const f32x4*>(part + s * slab + off);
      x1 += *reinterpret_cast<const f32x4*>(part + s * slab + off + 4);
    }
    float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    if (HAS_RES) {
      const u32x4 r = *reinterpret_cast<const u32x4*>(res + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] += lo_bf(r[j]);
        v[2 * j + 1] += hi_bf(r[j]);
      }
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf2(v[2 * j], v[2 * j + 1]);
    *reinterpret_cast<u32x4*>(out + off) = o;
    if (stats) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float q0 = lo_bf(o[j]), q1 = hi_bf(o[j]);
        st[0][2 * j] += q0; st[1][2 * j] += q0 * q0;
        st[0][2 * j + 1] += q1; st[1][2 * j + 1] += q1 * q1;
      }
    } else if (bwd) {
      const u32x4 om = *reinterpret_cast<const u32x4*>(bo + off);
      const u32x4 yv = *reinterpret_cast<const u32x4*>(by1 + off);
      u32x4 y2v = {0u, 0u, 0u, 0u};
      if (two) y2v = *reinterpret_cast<const u32x4*>(by2 + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool hi = e & 1;
        const uint32_t w = o[e >> 1], mw = om[e >> 1], yw = yv[e >> 1], y2w = y2v[e >> 1];
        const float g = hi ? hi_bf(w) : lo_bf(w);
        const float dz = (hi ? hi_bf(mw) : lo_bf(mw)) > 0.f ? g : 0.f;
        st[0][e] += dz;
        st[1][e] += dz * ((hi ? hi_bf(yw) : lo_bf(yw)) - m1[e]) * i1[e];
        if (two) st[2][e] += dz * ((hi ? hi_bf(y2w) : lo_bf(y2w)) - m2[e]) * i2[e];
      }
    }
  }
  if (!stats && !bwd) return;
  float* mine = sred + threadIdx.x * 24;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mine[j] = st[0][j];
    mine[8 + j] = st[1][j];
    mine[16 + j] = st[2][j];
  }
  __syncthreads();
  float* dst = (bwd ? bpart : stats) + (size_t)(blockIdx.x & (PSX_STAT_SLOTS - 1)) * nst * OC;
  for (int t = threadIdx.x; t < cvec * nst * 8; t += 256) {
    const int cgi = t / (nst * 8), sj = t - cgi * (nst * 8);
    float acc = 0.f;
    for (int q = 0; q < tpp; ++q) acc += sred[(q * cvec + cgi) * 24 + sj];
    const int which = sj >> 3, j = sj & 7;
    atomicAdd(dst + which * OC + cgi * 8 + j, acc);
  }
  if (!stats) return;
  if (fuse_fin && last_block_arrive(fin.counter, gridDim.x, reinterpret_cast<unsigned char*>(sred)))
    bn_finalize_block<PSX_STAT_SLOTS>(stats, fin);
}

}  // namespace psx

using namespace psx;

namespace {

int ilog2i(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

struct Plan {
  int BM, BN, splits, WGM = 2;
};

// Tile / split-K plan: prefer >= 2 workgroups per CU; split-K only while each split keeps
// >= 8 k-steps.
Plan plan_for(int OC, int npix, int ksteps) {
  Plan p{64, 128, 1};
  if (OC % 128 == 0 && (long)(OC / 128) * ((npix + 127) / 128) >= 512) {
    p.BM = 128;
    p.BN = 128;
  } else if ((long)(OC / 64) * ((npix + 127) / 128) >= 512) {
    p.BM = 64;
    p.BN = 128;
  } else {
    p.BM = 64;
    p.BN = 64;
  }
  const long tiles = (long)(OC / p.BM) * ((npix + p.BN - 1) / p.BN);
  while (p.splits < 8 && tiles * p.splits < 512 && ksteps / (p.splits * 2) >= 8) p.splits *= 2;
  // experiment overrides (tile sweep, bench/conv_sweep.py): PSX_CV_BM / PSX_CV_BN / PSX_CV_SPLITS
  if (const char* e = getenv("PSX_CV_BM")) p.BM = atoi(e);
  if (const char* e = getenv("PSX_CV_BN")) p.BN = atoi(e);
  if (const char* e = getenv("PSX_CV_SPLITS")) p.splits = atoi(e);
  if (const char* e = getenv("PSX_CV_WGM")) p.WGM = atoi(e);
  if (OC % p.BM) p.BM = 64;
  if (p.splits > ksteps) p.splits = ksteps;
  return p;
}

template <int BM, int BN, int MODE, bool RES, bool SPLIT, int WGM = 2>
int launch2(const Conv2Args& a, hipStream_t st) {
  const size_t lds = (size_t)3 * (BM + BN) * 128;
  dim3 grid(a.n_oc_tiles * a.n_pix_tiles, SPLIT ? a.splits : (MODE == 3 ? 4 : 1));
  hipLaunchKernelGGL((conv2_kernel<BM, BN, MODE, RES, SPLIT, WGM>), grid, dim3(256), lds, st, a);
  return (int)hipGetLastError();
}

template <int MODE, bool RES>
int dispatch2(const Plan& p, const Conv2Args& a, hipStream_t st) {
  const bool sp = p.splits > 1;
#define PSX_L2(BM_, BN_, W_)                                                                   \
  if (p.BM == BM_ && p.BN == BN_ && p.WGM == W_)                                               \
    return sp ? launch2<BM_, BN_, MODE, false, true, W_>(a, st) : launch2<BM_, BN_, MODE, RES, false, W_>(a, st);
  PSX_L2(128, 128, 2)
  PSX_L2(64, 128, 2)
  PSX_L2(64, 64, 2)
  PSX_L2(64, 256, 1)
  PSX_L2(64, 128, 1)
  PSX_L2(128, 256, 2)
#undef PSX_L2
  return -7;
}

template <int BM, int BN, int MODE, bool RES, int WGM, int TP = 1>
int launch_tapr(const Conv2Args& a, hipStream_t st) {
  const size_t lds = (size_t)2 * (3 * BM * 128 + (TP == 2 ? BN + 8 : BN + 1) * 128);
  hipLaunchKernelGGL((conv2_kernel<BM, BN, MODE, RES, false, WGM, TP>), dim3(a.n_oc_tiles * a.n_pix_tiles),
                     dim3(256), lds, st, a);
  return (int)hipGetLastError();
}

// Pixel-tile width of the tap-reuse path for this layer, 0 = not applicable: 3x3 / stride 1 /
// pad 1, square power-of-two images whose rows tile BN exactly, 64-channel chunks; no split-K.
// PSX_CV_TAPR=0 disables it, PSX_CV_TAPR_BN=64|128|256 forces the width (sweeps). Other widths
// (and PSX_CV_TAPR_HALO=1, a test override) take the halo mode with 64-pixel tiles: returns -64.
int tapr_bn(int R, int S, int stride, int pad, int H, int W, int IC, int OC, int npix) {
  if (const char* e = getenv("PSX_CV_TAPR"))
    if (e[0] == '0') return 0;
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || IC % 64 || OC % 64) return 0;
  const char* he = getenv("PSX_CV_TAPR_HALO");
  const bool halo_off = he && he[0] == '0', halo_force = he && he[0] == '1';
  if (halo_force || H != W || (W & (W - 1)) || 64 % W) return halo_off ? 0 : -64;
  int force = 0;
  if (const char* e = getenv("PSX_CV_TAPR_BN")) force = atoi(e);
  // measured (bench/tapr_probe.py, ResNet-18 B=128, us fwd/dgrad): 64-pixel tiles (2 workgroups
  // per CU) win or tie on every layer — 32x32x64: 27.3/20.9 vs generic 26.3/23.0; 16x16x128:
  // 18.7/15.8 vs 20.6/19.3; 8x8x256: 14.8/13.7 vs 25.5/23.4; 4x4x512: 20.5/19.2 vs 29.3/28.0
  // (generic = split-K + epilogue launch there); 128/256-pixel tiles (1 workgroup per CU) lose.
  const int BN = force ? force : 64;
  if ((BN != 64 && BN != 128 && BN != 256) || BN % W || npix % BN) return 0;
  return BN;
}

template <int MODE, bool RES>
int dispatch_tapr(int bn, Conv2Args& a, hipStream_t st) {
  a.n_oc_tiles = a.OC / 64;
  a.splits = 1;
  a.kps = a.Kg / 64;
  if (bn < 0) {  // halo mode
    a.n_pix_tiles = (a.npix + 63) / 64;
    return launch_tapr<64, 64, MODE, RES, 2, 2>(a, st);
  }
  a.n_pix_tiles = a.npix / bn;
  if (bn == 256) return launch_tapr<64, 256, MODE, RES, 1>(a, st);
  if (bn == 128) return launch_tapr<64, 128, MODE, RES, 2>(a, st);
  return launch_tapr<64, 64, MODE, RES, 2>(a, st);
}

int finish_split(const Conv2Args& a, hipStream_t st) {
  const int cvec = a.OC / 8;
  if (256 % cvec) return -8;
  int ppb = (a.npix + 511) / 512;
  if (ppb < 8) ppb = 8;
  const int grid = (a.npix + ppb - 1) / ppb;
  const size_t lds = 256 * 24 * sizeof(float);
  if (a.res)
    hipLaunchKernelGGL(conv_splitk_epilogue<true>, dim3(grid), dim3(256), lds, st, a.part, a.splits, a.npix, a.OC,
                       a.out, a.res, a.stats, ppb, a.fuse_fin, a.fin, a.bpart, a.bo, a.by1, a.by2, a.bsaved1,
                       a.bsaved2, a.bns);
  else
    hipLaunchKernelGGL(conv_splitk_epilogue<false>, dim3(grid), dim3(256), lds, st, a.part, a.splits, a.npix, a.OC,
                       a.out, (const uint16_t*)nullptr, a.stats, ppb, a.fuse_fin, a.fin, a.bpart, a.bo, a.by1,
                       a.by2, a.bsaved1, a.bsaved2, a.bns);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// Bytes of fp32 split-K workspace the v2 conv needs for this problem (0 = no split).
long psx_conv2_workspace(int Nb, int OH, int OW, int OC, int Kg) {
  const int npix = Nb * OH * OW;
  const Plan p = plan_for(OC, npix, Kg / 64);
  return p.splits > 1 ? (long)p.splits * npix * OC * 4 : 0;
}

// Forward conv (v2). Same operands as psx_conv_fwd plus a 16-byte zero page and a split-K
// workspace (>= psx_conv2_workspace bytes, may be null when that is 0).
// fin (nullable, needs stats): the BN layer fed by this conv is finalized by the kernel's last
// workgroup (bnfin.hpp) instead of a separate psx_bn_finalize launch.
int psx_conv_fwd2(const void* x, const void* wf, void* y, float* stats, const void* zero, float* ws, int Nb, int H,
                  int W, int IC, int OC, int R, int S, int stride, int pad, int Kg, const BnFin* fin, hipStream_t st) {
  Conv2Args a{};
  if (fin && stats) {
    if (fin->C != OC) return -10;
    a.fuse_fin = 1;
    a.fin = *fin;
  }
  a.in = (const uint16_t*)x;
  a.w = (const uint16_t*)wf;
  a.out = (uint16_t*)y;
  a.res = nullptr;
  a.stats = stats;
  a.part = ws;
  a.zero = (const uint16_t*)zero;
  a.Nb = Nb; a.IH = H; a.IW = W; a.IC = IC;
  a.OH = (H + 2 * pad - R) / stride + 1;
  a.OW = (W + 2 * pad - S) / stride + 1;
  a.OC = OC; a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2i(IC / 8);
  a.npix = Nb * a.OH * a.OW;
  if (OC % 64 || Kg % 64 || IC % 8 || (IC & (IC - 1))) return -2;
  if (const int tbn = tapr_bn(R, S, stride, pad, H, W, IC, OC, a.npix)) return dispatch_tapr<0, false>(tbn, a, st);
  const Plan p = plan_for(OC, a.npix, Kg / 64);
  a.n_oc_tiles = OC / p.BM;
  a.n_pix_tiles = (a.npix + p.BN - 1) / p.BN;
  a.splits = p.splits;
  a.kps = (Kg / 64 + p.splits - 1) / p.splits;
  if (p.splits > 1 && !ws) return -9;
  int e = dispatch2<0, false>(p, a, st);
  if (e || p.splits == 1) return e;
  return finish_split(a, st);
}

struct BwdStatsDesc {  // fused BN-backward reduction over the dgrad output (see Conv2Args)
  float* part;
  const void* o;
  const void* y1;
  const void* y2;
  const float* saved1;
  const float* saved2;
};

int psx_conv_dgrad2(const void* dy, const void* wd, void* dx, const void* res, const void* zero, float* ws, int Nb,
                    int H, int W, int IC_fwd, int OC_fwd, int R, int S, int stride, int pad, int Kg,
                    const BwdStatsDesc* bst, hipStream_t st) {
  Conv2Args a{};
  if (bst) {
    a.bpart = bst->part;
    a.bo = (const uint16_t*)bst->o;
    a.by1 = (const uint16_t*)bst->y1;
    a.by2 = (const uint16_t*)bst->y2;
    a.bsaved1 = bst->saved1;
    a.bsaved2 = bst->saved2;
    a.bns = bst->y2 ? 3 : 2;
  }
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  a.in = (const uint16_t*)dy;
  a.w = (const uint16_t*)wd;
  a.out = (uint16_t*)dx;
  a.res = (const uint16_t*)res;
  a.stats = nullptr;
  a.part = ws;
  a.zero = (const uint16_t*)zero;
  a.Nb = Nb; a.IH = P; a.IW = Q; a.IC = OC_fwd;
  a.OH = H; a.OW = W; a.OC = IC_fwd;
  a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2i(OC_fwd / 8);
  a.npix = Nb * H * W;
  if (IC_fwd % 64 || Kg % 64 || (OC_fwd & (OC_fwd - 1))) return -2;
  if (const int tbn = tapr_bn(R, S, stride, pad, H, W, OC_fwd, IC_fwd, a.npix))
    return res ? dispatch_tapr<1, true>(tbn, a, st) : dispatch_tapr<1, false>(tbn, a, st);
  const Plan p = plan_for(IC_fwd, a.npix, Kg / 64);
  a.n_oc_tiles = IC_fwd / p.BM;
  a.n_pix_tiles = (a.npix + p.BN - 1) / p.BN;
  a.splits = p.splits;
  a.kps = (Kg / 64 + p.splits - 1) / p.splits;
  if (p.splits > 1 && !ws) return -9;
  int e;
  if (stride == 1)
    e = res ? dispatch2<1, true>(p, a, st) : dispatch2<1, false>(p, a, st);
  else if (stride == 2 && a.log2_icc >= 3 && !getenv("PSX_DGRAD_S2_GATHER")) {
    // parity classes: each class GEMM covers dx pixels (2i+py, 2j+px), ~1/4 of them
    Plan q = plan_for(IC_fwd, (a.npix + 3) / 4, Kg / 64);
    q.splits = 1;
    a.n_oc_tiles = IC_fwd / q.BM;
    a.n_pix_tiles = (Nb * ((H + 1) / 2) * ((W + 1) / 2) + q.BN - 1) / q.BN;
    a.splits = 1;
    a.kps = Kg / 64;
    return res ? dispatch2<3, true>(q, a, st) : dispatch2<3, false>(q, a, st);
  } else if (stride == 2)
    e = res ? dispatch2<2, true>(p, a, st) : dispatch2<2, false>(p, a, st);
  else
    return -4;
  if (e || p.splits == 1) return e;
  return finish_split(a, st);
}

}  // extern "C"
