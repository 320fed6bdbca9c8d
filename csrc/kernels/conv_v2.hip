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

// fp32 register double buffer of the MFMA fragments (A/B builds: csrc/build.py --variant):
// bit 0 the tap-reuse mainloop, bit 1 the generic one. Same-box A/B (fp32 layers, B=128, us
// fwd/dgrad): tap reuse 32x32 102.2/96.7 -> 98.9/94.6, 8x8 89.7/87.9 -> 87.1/83.7, 4x4
// 103.0/96.3 -> 92.9/89.5 (bench 5.15 -> 5.03 ms/step); the generic loop (stride 2, 1x1)
// measured neutral to 4 % slower, so only bit 0 is on.
#ifndef PSX_CONV_PF
#define PSX_CONV_PF 1
#endif
// bf16: the same double buffer in the tap-reuse loop. Same-box A/B (bf16 layers, us fwd/dgrad):
// 32x32 30.9/23.0 -> 25.5/22.0, 16x16 22.9/19.4 -> 18.9/17.3, 4x4 23.5/22.0 -> 21.1/19.7 (the
// bf16 tile widths: tapr_bn)
#ifndef PSX_CONV_PF_BF16
#define PSX_CONV_PF_BF16 1
#endif
// epilogue rows whose global loads are issued together (A/B builds: -D PSX_EPI_U=1)
#ifndef PSX_EPI_U
#define PSX_EPI_U 4
#endif
#ifndef PSX_TAPR_F32_128
#define PSX_TAPR_F32_128 1
#endif

namespace psx {

struct Conv2Args {
  // activation / weight operands are of the launch's storage type T (bf16 bits or fp32)
  const void* in;        // NHWC [Nb][IH][IW][IC] gathered operand
  const void* w;         // [OC][Kg] (K-contiguous, zero padded)
  void* out;             // NHWC [Nb][OH][OW][OC]
  const void* res;       // optional residual (same shape as out)
  float* stats;          // optional BN partial sums [PSX_STAT_SLOTS][2][OC]
  float* part;           // split-K fp32 slabs [splits][npix][OC]
  const void* zero;      // 16-byte zero page (DMA source for padding)
  int Nb, IH, IW, IC, OH, OW, OC, R, S, pad, stride;
  int Kg, log2_icc, npix;
  int n_oc_tiles, n_pix_tiles, splits, kps;  // kps: k-steps per split
  int fuse_fin;                              // last workgroup finalizes the BN layer (bnfin.hpp)
  BnFin fin;
  // optional fused BatchNorm-backward reduction over this launch's bf16 output g (dgrad): slot
  // rows [PSX_STAT_SLOTS][bns][OC] of sum(dz), sum(dz*xhat1) [, sum(dz*xhat2)], dz = g*[o > 0],
  // xhat = (y - mean) * invstd — what bn_bwd_reduce (bn.hip) would compute in a separate pass.
  float* bpart;
  const void* bo;
  const void* by1;
  const void* by2;
  const float* bsaved1;  // [2][OC] mean, invstd
  const float* bsaved2;
  int bns;
  // bmask: store dz = g*[o > 0] instead of g, so the BN-backward apply that consumes this output
  // needs no ReLU-mask operand (one full activation read less per BN layer)
  int bmask;
  DetRed det;  // deterministic mode: the launch's row slab (bnfin.hpp)
  // forward statistics: per-channel shift k subtracted before summing (nullable = 0; bnfin.hpp
  // BnFin::sshift): the slots hold sum(y - k), sum((y - k)^2)
  const float* sshift;
  // MODE 3 with the block's 1x1 / stride-2 shortcut folded in (nullable in2): the shortcut's data
  // gradient only reaches the (0, 0) parity class, one tap deep, so that class runs its 3x3 tap
  // and then the shortcut's as extra k-steps: operand dy_sc (in2, same shape as in) against the
  // shortcut's data-gradient weights (w2, rows of Kg2) — no separate launch and no residual pass
  const void* in2;
  const void* w2;
  int Kg2;
  // LDS ring depth of the generic mainloop: 3 (default, 0) or 2 — a 2-deep ring halves nothing
  // per k-step but fits 5 instead of 3 fp32 64x64 workgroups per CU (32 vs 48 KB), the batched
  // Winograd GEMMs' 1152-workgroup grids then run in one round (launch2 / psx_bgemm_f32_split)
  int nstg;
};

// Winograd F(4x4,3x3) output transform A^T (wino.hip has the matrices): y = A^T P A
__constant__ float kWinoAT[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                    {0.f, 1.f, -1.f, 2.f, -2.f, 0.f},
                                    {0.f, 1.f, 1.f, 4.f, 4.f, 0.f},
                                    {0.f, 1.f, -1.f, 8.f, -8.f, 1.f}};

PSX_DEV int kmaj2(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int MODE, typename T>
PSX_DEV const T* gather_src(const Conv2Args& a, int nbase, int hb, int wb, bool pv, int gk) {
  const T* zero = (const T*)a.zero;
  const int tap = gk >> a.log2_icc;
  const int c0 = (gk & ((1 << a.log2_icc) - 1)) * kEPC<T>;
  if (!pv || tap >= a.R * a.S) return zero;
  const int r = tap / a.S, s = tap - r * a.S;
  int ih, iw;
  if (MODE == 0) {
    ih = hb + r;
    iw = wb + s;
  } else {
    const int th = hb - r, tw = wb - s;
    if (MODE == 2) {
      if ((th | tw) & 1) return zero;
      ih = th >> 1;
      iw = tw >> 1;
    } else {
      ih = th;
      iw = tw;
    }
  }
  if ((unsigned)ih >= (unsigned)a.IH || (unsigned)iw >= (unsigned)a.IW) return zero;
  return (const T*)a.in + ((size_t)(nbase + ih * a.IW + iw) * a.IC + c0);
}

// WGM = waves along the output-channel (M) axis, 4 / WGM along pixels: 2 (2x2 waves, wave tile
// BM/2 x BN/2) or 1 (1x4 waves: every wave holds all BM channels of a BN/4 pixel slice, e.g. a
// 64x64 wave tile for BM = 64, BN = 256 — 2/3 of the LDS fragment bytes per MFMA of 32x64).
//
// TAPR (3x3 / stride 1 / pad 1, MODE 0 or 1, tiles of whole image rows): tap-reuse mainloop.
// A macro step = (kernel row r, 64-channel chunk): the three weight tiles of taps (r, 0..2) and
// ONE window X of the tile's BN pixels at (row r, centre column) are staged; pixel j of tap s
// reads window slot j + d(s) (d = s - 1 forward, 1 - s dgrad: ih = oh + pad - r there); when its
// column leaves the image row the fragment is zeroed in registers (a per-lane mask fixed for the
// whole kernel: no zero row in LDS, so a 128-pixel stage fits two workgroups per CU). The im2col
// operand is staged once per kernel row
// instead of once per tap (1/3 of the L2->LDS bytes of the gathered operand); 2 LDS stages.
// TAPR = 1: tiles of whole image rows (power-of-two widths); TAPR = 2 ("halo", any width, e.g.
// ResNet-50's 56/28/14/7): the window also holds the pixel before and after the tile (slot k =
// pixel pix0 - 1 + k), so a shift never leaves the staged rows; a zero row sits at slot BN + 2.
//
// T: activation / weight storage type (common.hpp kEPC/kKS): one k-step is a 128-byte row of
// every operand = 64 bf16 or 32 fp32 channels; the staging below is written in 16-byte chunks
// and bytes, so only the element strides (EPC per chunk, KS per k-step) depend on T.
template <typename T, int BM, int BN, int MODE, bool HAS_RES, bool SPLIT, int WGM = 2, int TAPR = 0>
__global__ __launch_bounds__(256) void conv2_kernel(Conv2Args a) {
  constexpr int EPC = kEPC<T>, KS = kKS<T>;
  const T* const in = (const T*)a.in;
  const T* const wts = (const T*)a.w;
  const T* const zero = (const T*)a.zero;
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
  int nk = SPLIT ? min(a.kps, a.Kg / KS - ks0) : a.Kg / KS;
  // MODE 3 = stride-2 dgrad, one parity class (py, px) of dx per blockIdx.y: dx(2i+py, 2j+px)
  // only receives taps r = r0, r0+2, .. and s = s0, s0+2, .. (r0 = (py+pad)&1), i.e. a dense
  // GEMM over 1, 2, 2 or 4 of the 9 taps instead of 9 with 3/4 of the products zero.
  // classes in decreasing work order (the (1,1) class has 4 of the 9 taps, (0,0) one): the
  // dispatcher walks blockIdx.y last, so the longest workgroups start first
  const int cls = MODE == 3 ? 3 - (int)blockIdx.y : 0;
  const int py = cls >> 1, px = cls & 1;
  const int CH = (a.OH - py + 1) >> 1, CW = (a.OW - px + 1) >> 1;
  const int r0 = (py + a.pad) & 1, s0 = (px + a.pad) & 1;
  const int nr = r0 < a.R ? (a.R - r0 + 1) >> 1 : 0, nsx = s0 < a.S ? (a.S - s0 + 1) >> 1 : 0;
  const int npix_c = MODE == 3 ? a.Nb * CH * CW : a.npix;
  const bool sc = MODE == 3 && a.in2 != nullptr && cls == 0;  // class (0, 0) + the folded shortcut
  if (MODE == 3) {
    nk = (nr * nsx + (sc ? 1 : 0)) << (a.log2_icc - 3);
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
    constexpr int XROWS = HALO ? BN + 8 : BN, ZS = BN + 2;  // window rows; the halo mode's zero slot
    constexpr int XOFF = 3 * BM * 128, TST = XOFF + XROWS * 128;  // A0 A1 A2 | X
    const int nch = a.IC / KS, nmac = 3 * nch;
    const int W = a.OW, log2w = __builtin_ctz(W);
    const int lrow = lane >> 3, lpos = lane & 7;
    const T* wsrc[LA];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = (i * 4 + wid) * 8 + lrow;
      wsrc[i] = wts + (size_t)(oc0 + row) * a.Kg + (lpos ^ ((row >> 1) & 7)) * EPC;
    }
    // window rows: the tile's own pixels (input pixel index == output pixel index at s1/p1);
    // halo mode: slot k = pixel pix0 - 1 + k, and wave 0 also stages slots BN .. BN+7 (the two
    // halo pixels, then zeros from the zero page)
    constexpr int LX = LB + (HALO ? 1 : 0);
    const T* xsrc[LX];
    int xoh[LX];
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int row = i < LB ? (i * 4 + wid) * 8 + lrow : BN + lrow;
      const int pix = pix0 + row - (HALO ? 1 : 0);
      const bool ok = HALO ? (pix >= 0 && pix < a.npix && (i < LB || lrow < 2)) : true;
      xoh[i] = !ok ? -(1 << 20) : HALO ? (pix / W) % a.OH : (pix >> log2w) & (a.OH - 1);
      xsrc[i] = ok ? in + (size_t)pix * a.IC + (lpos ^ ((row >> 1) & 7)) * EPC : zero;
    }
    auto issue_t = [&](int t, int stage) {
      unsigned char* base = smem + stage * TST;
      const int r = __builtin_amdgcn_readfirstlane(t / nch);
      const int cc = t - r * nch;
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const int kofs = (r * 3 + sx) * a.IC + cc * KS;
#pragma unroll
        for (int i = 0; i < LA; ++i) glds16(wsrc[i] + kofs, base + sx * BM * 128 + (i * 4 + wid) * 1024);
      }
      const int dr = MODE == 0 ? r - 1 : 1 - r;
      const long uoff = (long)dr * W * a.IC + cc * KS;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const T* src = (unsigned)(xoh[i] + dr) < (unsigned)a.OH ? xsrc[i] + uoff : zero;
        glds16(src, base + XOFF + (i * 4 + wid) * 1024);
      }
      if (HALO && wid == 0) {
        const T* src = (unsigned)(xoh[LX - 1] + dr) < (unsigned)a.OH ? xsrc[LX - 1] + uoff : zero;
        glds16(src, base + XOFF + BN * 128);
      }
    };
    // per-lane B-fragment byte offsets of the three taps (tile starts on an image row)
    const int frow = lane & 15, fch = lane >> 4;
    int boff[NT][3];
    bool keep[NT][3];  // (whole-row tiles) the tap's column is inside the image row
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int prow = wn * (BN / WGN) + n * 16 + frow;
      const int ow = HALO ? (pix0 + prow) % W : prow & (W - 1);
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const int d = MODE == 0 ? sx - 1 : 1 - sx;
        const bool in = (unsigned)(ow + d) < (unsigned)W;
        const int slot = in ? prow + d + (HALO ? 1 : 0) : (HALO ? ZS : prow);
        keep[n][sx] = HALO || in;
        boff[n][sx] = slot * 128 + ((fch ^ ((slot >> 1) & 7)) << 4);
      }
    }
    if constexpr ((sizeof(T) == 4 || PSX_CONV_PF_BF16) && (PSX_CONV_PF & 1)) {
      // Fragments are double-buffered in registers: a macro step is 6 sub-steps q = (tap sx = q/2,
      // half kk = q%2), and the LDS reads of sub-step q+1 are issued before the MFMAs of q, so the
      // read latency (one s_waitcnt lgkmcnt(0) in front of every sub-step's MFMAs before) hides
      // behind them. At the last sub-step the stage boundary comes first — this wave's DMA of the
      // next stage retired, its own reads of this stage retired (lgkmcnt), barrier, DMA of step t+2
      // into the stage just drained, reads of the next stage's first sub-step — then its MFMAs.
      auto load_frags = [&](const unsigned char* base, int q, u32x4(&fa)[MT], u32x4(&fb)[NT]) {
        const int sx = q >> 1, kk = q & 1;
        const unsigned char* A = base + sx * BM * 128;
        const unsigned char* X = base + XOFF;
#pragma unroll
        for (int m = 0; m < MT; ++m)
          fa[m] = *reinterpret_cast<const u32x4*>(A + kmaj2(wm * (BM / WGM) + m * 16 + frow, kk * 4 + fch));
#pragma unroll
        for (int n = 0; n < NT; ++n) fb[n] = *reinterpret_cast<const u32x4*>(X + (boff[n][sx] ^ (kk << 6)));
      };
      u32x4 fa0[MT], fb0[NT], fa1[MT], fb1[NT];
      if (HALO) __syncthreads();
      if (nmac > 0) {
        issue_t(0, 0);
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (nmac > 1) issue_t(1, 1);
        load_frags(smem, 0, fa0, fb0);
      }
      for (int t = 0; t < nmac; ++t) {
        const unsigned char* base = smem + (t & 1) * TST;
        auto sub = [&](auto qc, u32x4(&fa)[MT], u32x4(&fb)[NT], u32x4(&na)[MT], u32x4(&nb)[NT]) {
          constexpr int q = decltype(qc)::value, sx = q >> 1;
          if constexpr (q < 5) {
            load_frags(base, q + 1, na, nb);
          } else if (t + 1 < nmac) {
            wait_vmcnt<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (t + 2 < nmac) issue_t(t + 2, t & 1);
            load_frags(smem + ((t + 1) & 1) * TST, 0, na, nb);
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (!HALO && sx != 1) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
              if (!keep[n][sx]) fb[n] = u32x4{0u, 0u, 0u, 0u};
          }
          mma_tiles<MT, NT, T>(acc, fa, fb);
        };
        sub(std::integral_constant<int, 0>{}, fa0, fb0, fa1, fb1);
        sub(std::integral_constant<int, 1>{}, fa1, fb1, fa0, fb0);
        sub(std::integral_constant<int, 2>{}, fa0, fb0, fa1, fb1);
        sub(std::integral_constant<int, 3>{}, fa1, fb1, fa0, fb0);
        sub(std::integral_constant<int, 4>{}, fa0, fb0, fa1, fb1);
        sub(std::integral_constant<int, 5>{}, fa1, fb1, fa0, fb0);
      }
    } else {
      // single fragment set (PSX_CONV_PF_BF16=0 builds)
      if (HALO) __syncthreads();
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
            u32x4 fa[MT], fb[NT];
#pragma unroll
            for (int m = 0; m < MT; ++m)
              fa[m] = *reinterpret_cast<const u32x4*>(A + kmaj2(wm * (BM / WGM) + m * 16 + frow, kk * 4 + fch));
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              fb[n] = *reinterpret_cast<const u32x4*>(X + (boff[n][sx] ^ (kk << 6)));
              if (!HALO && sx != 1 && !keep[n][sx]) fb[n] = u32x4{0u, 0u, 0u, 0u};
            }
            mma_tiles<MT, NT, T>(acc, fa, fb);
          }
        }
      }
    }
  } else {
  // ---- per-lane DMA source state (fixed across k-steps) ----
  const int lrow = lane >> 3, lpos = lane & 7;
  const T* wsrc[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = (i * 4 + wid) * 8 + lrow;
    const int c = lpos ^ ((row >> 1) & 7);
    wsrc[i] = wts + (size_t)(oc0 + row) * a.Kg + c * EPC;
  }
  const T* wsrc2[MODE == 3 ? LA : 1];
  if constexpr (MODE == 3) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = (i * 4 + wid) * 8 + lrow;
      wsrc2[i] = sc ? (const T*)a.w2 + (size_t)(oc0 + row) * a.Kg2 + (lpos ^ ((row >> 1) & 7)) * EPC : wts;
    }
  }
  int nbase[LB], hb[LB], wb[LB], bc[LB];
  bool pv[LB];
  // a pure GEMM needs no (n, oh, ow) decomposition: two integer divisions (~70 VALU) per staged
  // row, which a one- or two-k-step 1x1 layer otherwise pays as much as its whole epilogue
#ifdef PSX_NO_GEMM1X1  // A/B builds
  const bool gemm1x1 = false;
#else
  const bool gemm1x1 = (MODE == 0 || MODE == 1) && a.R == 1 && a.S == 1 && a.stride == 1 && a.pad == 0;
#endif
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int row = (i * 4 + wid) * 8 + lrow;
    bc[i] = lpos ^ ((row >> 1) & 7);
    const int pix = pix0 + row;
    pv[i] = pix < npix_c;
    const int pp = pv[i] ? pix : 0;
    if (gemm1x1) {  // 1x1 / stride 1 / no padding: the gathered operand is the plain [npix][IC] matrix
      nbase[i] = pp;
      hb[i] = wb[i] = 0;  // (the bounds checks of tap (0, 0) always pass)
      continue;
    }
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
  const T* pbase[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    // MODE 0: pixel (hb, wb) = top-left tap; MODE 1: (hb, wb) = (oh, ow) + pad, taps subtract
    const long off = MODE == 2 ? 0 : ((long)nbase[i] + (long)hb[i] * a.IW + wb[i]) * a.IC + bc[i] * EPC;
    // MODE 3: pbase = dy(n, i, j); a class tap adds the uniform offset (dr, ds) = ((py+pad-r)/2, ..)
    pbase[i] = in + off;
  }
  const int ksh = a.log2_icc - 3;  // k-steps per tap = 1 << ksh (utap only)

  auto issue = [&](int ks, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int kglob = ks0 + ks;
    if (MODE == 3) {
      const int t = __builtin_amdgcn_readfirstlane(ks >> ksh);
      const int cofs = __builtin_amdgcn_readfirstlane((ks & ((1 << ksh) - 1)) * KS);
      if (sc && t == nr * nsx) {  // the folded 1x1 / stride-2 shortcut: tap (0, 0) of dy_sc
#pragma unroll
        for (int i = 0; i < LA; ++i) glds16(wsrc2[i] + cofs, base + (i * 4 + wid) * 1024);
#pragma unroll
        for (int i = 0; i < LB; ++i) {
          const T* src = pv[i] ? (const T*)a.in2 + (pbase[i] - in) + cofs : zero;
          glds16(src, base + BM * 128 + (i * 4 + wid) * 1024);
        }
        return;
      }
      const int tr = __builtin_amdgcn_readfirstlane(t / nsx);
      const int r = r0 + 2 * tr, sx = s0 + 2 * (t - tr * nsx);
      const int kg = ((r * a.S + sx) << ksh) + (ks & ((1 << ksh) - 1));  // k-step in the full weights
#pragma unroll
      for (int i = 0; i < LA; ++i) glds16(wsrc[i] + kg * KS, base + (i * 4 + wid) * 1024);
      const int dr = (py + a.pad - r) >> 1, ds = (px + a.pad - sx) >> 1;
      const long uoff = ((long)dr * a.IW + ds) * a.IC + cofs;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const T* src = zero;
        if (pv[i] && (unsigned)(hb[i] + dr) < (unsigned)a.IH && (unsigned)(wb[i] + ds) < (unsigned)a.IW)
          src = pbase[i] + uoff;
        glds16(src, base + BM * 128 + (i * 4 + wid) * 1024);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) glds16(wsrc[i] + kglob * KS, base + (i * 4 + wid) * 1024);
    if (utap) {
      const int tap = __builtin_amdgcn_readfirstlane(kglob >> ksh);
      const int cofs = __builtin_amdgcn_readfirstlane((kglob & ((1 << ksh) - 1)) * KS);
      const int r = __builtin_amdgcn_readfirstlane(tap / a.S);
      const int sx = tap - r * a.S;
      const bool tap_ok = tap < a.R * a.S;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const T* src = zero;
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
            src = in + ((size_t)(nbase[i] + (th >> 1) * a.IW + (tw >> 1)) * a.IC + cofs + bc[i] * EPC);
        }
        glds16(src, base + BM * 128 + (i * 4 + wid) * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < LB; ++i)
        glds16(gather_src<MODE, T>(a, nbase[i], hb[i], wb[i], pv[i], kglob * 8 + bc[i]),
               base + BM * 128 + (i * 4 + wid) * 1024);
    }
  };

  const int frow = lane & 15, fch = lane >> 4;
  auto load_frags = [&](int stg, int kk, u32x4(&fa)[MT], u32x4(&fb)[NT]) {
    const unsigned char* A = smem + stg * STAGE;
    const unsigned char* B = A + BM * 128;
#pragma unroll
    for (int m = 0; m < MT; ++m)
      fa[m] = *reinterpret_cast<const u32x4*>(A + kmaj2(wm * (BM / WGM) + m * 16 + frow, kk * 4 + fch));
#pragma unroll
    for (int n = 0; n < NT; ++n)
      fb[n] = *reinterpret_cast<const u32x4*>(B + kmaj2(wn * (BN / WGN) + n * 16 + frow, kk * 4 + fch));
  };
  if (a.nstg != 2) {
    if (nk > 0) issue(0, 0);
    if (nk > 1) issue(1, 1);
  }
  if constexpr (sizeof(T) == 4 && (PSX_CONV_PF & 2)) {
    // fp32: the fragments of the next half k-step are read before the MFMAs of the current one
    // (register double buffer, as in the tap-reuse loop); the stage boundary — DMA of k-step
    // ks+1 retired, this wave's reads of stage ks retired, barrier, DMA of ks+3 into stage ks —
    // sits between the two halves of k-step ks.
    u32x4 fa0[MT], fb0[NT], fa1[MT], fb1[NT];
    if (nk > 0) {
      if (nk > 1)
        wait_vmcnt<LA + LB>();
      else
        wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (nk > 2) issue(2, 2);
      load_frags(0, 0, fa0, fb0);
    }
    int stage = 0;
    for (int ks = 0; ks < nk; ++ks) {
      const int nxt = stage == 2 ? 0 : stage + 1;
      load_frags(stage, 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      mma_tiles<MT, NT, T>(acc, fa0, fb0);
      if (ks + 1 < nk) {
        if (ks + 2 < nk)
          wait_vmcnt<LA + LB>();
        else
          wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks + 3 < nk) issue(ks + 3, stage);
        load_frags(nxt, 0, fa0, fb0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma_tiles<MT, NT, T>(acc, fa1, fb1);
      stage = nxt;
    }
  } else if (a.nstg == 2) {
    // 2-deep ring: k-step ks + 1 is issued into the other stage once every wave has passed the
    // barrier, i.e. finished reading it (k-step ks - 1); its DMA overlaps k-step ks's MFMAs
    for (int ks = 0; ks < nk; ++ks) {
      const int stage = ks & 1;
      if (ks == 0) issue(0, 0);  // (the shared prologue above issued nothing: nstg == 2 skips it)
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (ks + 1 < nk) issue(ks + 1, stage ^ 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4 fa[MT], fb[NT];
        load_frags(stage, kk, fa, fb);
        mma_tiles<MT, NT, T>(acc, fa, fb);
      }
    }
  } else {
    int stage = 0;
    for (int ks = 0; ks < nk; ++ks) {
      if (ks + 1 < nk)
        wait_vmcnt<LA + LB>();
      else
        wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (ks + 2 < nk) issue(ks + 2, stage == 0 ? 2 : stage - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4 fa[MT], fb[NT];
        load_frags(stage, kk, fa, fb);
        mma_tiles<MT, NT, T>(acc, fa, fb);
      }
      stage = stage == 2 ? 0 : stage + 1;
    }
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

  // ---- LDS-staged epilogue ----
  // The fp32 tile goes through LDS once; then every thread owns 8 channels of a pixel row, so the
  // output, the residual and the BN-backward operands o / y move as whole 16- (bf16) or 32-byte
  // (fp32) pieces of their rows (the fragment layout touched 32-byte pieces of 16 rows per
  // instruction), and the per-channel sums need one shuffle tree + one LDS pass per workgroup.
  {
    constexpr int TS = BM + 4;      // fp32 row stride of the staged tile (spreads the banks)
    constexpr int CPR = BM / 8;     // 8-channel groups per pixel row
    constexpr int RPP = 256 / CPR;  // pixel rows per pass
    constexpr int LDSB = TAPR ? 2 * (3 * BM * 128 + (TAPR == 2 ? BN + 8 : BN) * 128)
                              : 3 * (BM + BN) * 128;  // launched
    static_assert(256 % CPR == 0 && BN * TS * 4 <= LDSB, "staged tile fits the mainloop LDS");
    float* Ts = reinterpret_cast<float*>(smem);
    __syncthreads();  // every wave is done with the mainloop's LDS
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int pr = wn * (BN / WGN) + n * 16 + (lane & 15);
#pragma unroll
      for (int m = 0; m < MT; ++m)
        *reinterpret_cast<f32x4*>(Ts + pr * TS + wm * (BM / WGM) + m * 16 + 4 * (lane >> 4)) = acc[m][n];
    }
    __syncthreads();
    const bool bwd = a.bpart != nullptr, two = a.by2 != nullptr, st = a.stats != nullptr;
    const int cc = tid % CPR, ch0 = oc0 + cc * 8;
    float s1[8], s2[8], s3[8], bm1[8], bi1[8], bm2[8], bi2[8], ksh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s1[i] = s2[i] = s3[i] = 0.f;
      bm1[i] = bi1[i] = bm2[i] = bi2[i] = 0.f;
      ksh[i] = (st && a.sshift) ? a.sshift[ch0 + i] : 0.f;
      if (bwd) {
        bm1[i] = a.bsaved1[ch0 + i];
        bi1[i] = a.bsaved1[a.OC + ch0 + i];
        if (two) {
          bm2[i] = a.bsaved2[ch0 + i];
          bi2[i] = a.bsaved2[a.OC + ch0 + i];
        }
      }
    }
    // The pixel rows of a thread in chunks of U: every global load of a chunk (residual, the
    // BN-backward operands o / y) is issued before the first is used, so a workgroup pays one
    // memory round trip per chunk instead of one per row (a 1x1 layer with one or two k-steps is
    // all epilogue: ResNet-50's 64 -> 256 forward / 256 -> 64 data gradient at 56x56 ran 3-5x
    // slower than their HBM bytes with the row loop serialised on its loads).
    constexpr int NIT = BN / RPP;
    constexpr int UMAX = MODE == 3 ? (PSX_EPI_U < 2 ? PSX_EPI_U : 2) : PSX_EPI_U;  // MODE 3: 4 spills
    constexpr int U = NIT < UMAX ? NIT : UMAX;
    static_assert(NIT % U == 0, "whole chunks");
    const int pr0 = tid / CPR;
#pragma unroll
    for (int it0 = 0; it0 < NIT; it0 += U) {
      size_t offs[U];
      bool ok[U];
      float rr[U][8], om[U][8], yv[U][8], y2v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pix = pix0 + pr0 + (it0 + u) * RPP;
        ok[u] = pix < npix_c;
        const int pp = ok[u] ? pix : pix0;  // an in-range stand-in row: loaded, never stored
        size_t opix = (size_t)pp;
        if (MODE == 3) {  // class-local (n, i, j) -> dx (n, 2i+py, 2j+px)
          const int nn = pp / (CH * CW), rem = pp - nn * CH * CW, ii = rem / CW, jj = rem - ii * CW;
          opix = ((size_t)nn * a.OH + 2 * ii + py) * a.OW + 2 * jj + px;
        }
        offs[u] = opix * a.OC + ch0;
        if (HAS_RES) ld8((const T*)a.res + offs[u], rr[u]);
        if (bwd) {
          ld8((const T*)a.bo + offs[u], om[u]);
          ld8((const T*)a.by1 + offs[u], yv[u]);
          if (two) ld8((const T*)a.by2 + offs[u], y2v[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const float* src = Ts + (pr0 + (it0 + u) * RPP) * TS + cc * 8;
        const f32x4 va = *reinterpret_cast<const f32x4*>(src), vb = *reinterpret_cast<const f32x4*>(src + 4);
        float v[8] = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
        const size_t off = offs[u];
        if (HAS_RES) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += rr[u][k];
        }
        if (!bwd) st8((T*)a.out + off, v);  // v = the stored values from here on
        if (st) {  // packed f32 pairs (v_pk_add_f32 / v_pk_fma_f32): half the VALU of the sums
#pragma unroll
          for (int k = 0; k < 8; k += 2) {
            const psx_f32x2 d = (psx_f32x2){v[k], v[k + 1]} - (psx_f32x2){ksh[k], ksh[k + 1]};
            psx_f32x2 a1 = (psx_f32x2){s1[k], s1[k + 1]} + d;
            psx_f32x2 a2 = __builtin_elementwise_fma(d, d, (psx_f32x2){s2[k], s2[k + 1]});
            s1[k] = a1[0];
            s1[k + 1] = a1[1];
            s2[k] = a2[0];
            s2[k + 1] = a2[1];
          }
        }
        if (bwd) {
          if constexpr (sizeof(T) == 2) {  // bf16: the stored (rounded) g feeds the sums
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = bf2f(f2bf(v[i]));
          }
          float dzv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float dz = om[u][i] > 0.f ? v[i] : 0.f;
            dzv[i] = dz;
            s1[i] += dz;
            s2[i] += dz * (yv[u][i] - bm1[i]) * bi1[i];
            if (two) s3[i] += dz * (y2v[u][i] - bm2[i]) * bi2[i];
          }
          if (a.bmask)
            st8((T*)a.out + off, dzv);
          else
            st8((T*)a.out + off, v);
        }
      }
    }
    if (!st && !bwd) return;
    // per-channel sums over the RPP row groups through LDS: every thread writes its 8 channels'
    // partials (16-byte stores), then one thread per (statistic, channel) adds the RPP of them in
    // row-group order (cross-lane shuffles here cost 3 x 8 x 2-3 ds_bpermute per thread)
    __syncthreads();  // the staged tile is no longer read
    float* red = Ts;  // [RPP][3][BM] (launch2 sizes the LDS for it)
    {
      float* rw = red + (size_t)pr0 * 3 * BM + cc * 8;
      *reinterpret_cast<f32x4*>(rw) = (f32x4){s1[0], s1[1], s1[2], s1[3]};
      *reinterpret_cast<f32x4*>(rw + 4) = (f32x4){s1[4], s1[5], s1[6], s1[7]};
      *reinterpret_cast<f32x4*>(rw + BM) = (f32x4){s2[0], s2[1], s2[2], s2[3]};
      *reinterpret_cast<f32x4*>(rw + BM + 4) = (f32x4){s2[4], s2[5], s2[6], s2[7]};
      if (two) {
        *reinterpret_cast<f32x4*>(rw + 2 * BM) = (f32x4){s3[0], s3[1], s3[2], s3[3]};
        *reinterpret_cast<f32x4*>(rw + 2 * BM + 4) = (f32x4){s3[4], s3[5], s3[6], s3[7]};
      }
    }
    __syncthreads();
    const int nst = bwd ? a.bns : 2;
    float* dst = (bwd ? a.bpart : a.stats) + (size_t)(pix_t & (PSX_STAT_SLOTS - 1)) * nst * a.OC;
    for (int j = tid; j < nst * BM; j += 256) {
      const int which = j / BM, row = j - which * BM;
      float v = 0.f;
#pragma unroll 8
      for (int g = 0; g < RPP; ++g) v += red[((size_t)g * 3 + which) * BM + row];
      stat_add(a.det, dst, which * a.OC + oc0 + row, v);
    }
    if (st && a.fuse_fin && last_block_arrive(a.fin.counter, gridDim.x, smem))
      bn_finalize_block<PSX_STAT_SLOTS>(a.stats, a.fin);
    return;
  }

}

// Split-K epilogue: out = T(sum_s part[s] (+res)); BN partial statistics into slot rows.
// Block = 256 threads; thread owns 8 channels of a pixel; blocks stride over pixel ranges.
template <typename T, bool HAS_RES>
__global__ __launch_bounds__(256) void conv_splitk_epilogue(const float* __restrict__ part, int splits, int npix,
                                                            int OC, T* __restrict__ out,
                                                            const T* __restrict__ res,
                                                            float* __restrict__ stats, int pix_per_block,
                                                            int fuse_fin, BnFin fin, float* __restrict__ bpart,
                                                            const T* __restrict__ bo,
                                                            const T* __restrict__ by1,
                                                            const T* __restrict__ by2,
                                                            const float* __restrict__ bsaved1,
                                                            const float* __restrict__ bsaved2, int bns,
                                                            int bmask, DetRed det, const float* __restrict__ sshift) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [256][24]
  const int cvec = OC >> 3, tpp = 256 / cvec;
  const int cg = threadIdx.x % cvec, pr = threadIdx.x / cvec;
  const size_t slab = (size_t)npix * OC;
  // per-thread partial sums: fwd stats (sum, sumsq) or fused BN-backward (dz, dz*xh1, dz*xh2)
  const bool bwd = bpart != nullptr, two = by2 != nullptr;
  const int nst = bwd ? bns : 2;
  float st[3][8], m1[8], i1[8], m2[8], i2[8], ksh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    st[0][j] = st[1][j] = st[2][j] = 0.f;
    ksh[j] = (stats && sshift) ? sshift[cg * 8 + j] : 0.f;
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
  // PP pixel rows per thread at a time: their split slabs are loaded together (one round trip
  // per split instead of one per row and split)
  constexpr int PP = 4;
  for (int pg = pbeg + pr; pg < pend; pg += PP * tpp) {
    f32x4 xs0[PP], xs1[PP];
    size_t offs[PP];
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int pu = pg + u * tpp;
      offs[u] = (size_t)(pu < pend ? pu : pg) * OC + cg * 8;
      xs0[u] = *reinterpret_cast<const f32x4*>(part + offs[u]);
      xs1[u] = *reinterpret_cast<const f32x4*>(part + offs[u] + 4);
    }
    for (int s = 1; s < splits; ++s)
#pragma unroll
      for (int u = 0; u < PP; ++u) {
        xs0[u] += *reinterpret_cast<const f32x4*>(part + s * slab + offs[u]);
        xs1[u] += *reinterpret_cast<const f32x4*>(part + s * slab + offs[u] + 4);
      }
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    if (pg + u * tpp >= pend) break;
    const size_t off = offs[u];
    const f32x4 x0 = xs0[u], x1 = xs1[u];
    float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    if (HAS_RES) {
      float r[8];
      ld8(res + off, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    if (!bwd) st8(out + off, v);  // v = the stored values from here on
    if (stats) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - ksh[j];
        st[0][j] += d;
        st[1][j] += d * d;
      }
    } else if (bwd) {
      float om[8], yv[8], y2v[8];
      if constexpr (sizeof(T) == 2) {  // bf16: the stored (rounded) g feeds the sums
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e]));
      }
      ld8(bo + off, om);
      ld8(by1 + off, yv);
      if (two) ld8(by2 + off, y2v);
      float dzv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = om[e] > 0.f ? v[e] : 0.f;
        dzv[e] = dz;
        st[0][e] += dz;
        st[1][e] += dz * (yv[e] - m1[e]) * i1[e];
        if (two) st[2][e] += dz * (y2v[e] - m2[e]) * i2[e];
      }
      if (bmask)
        st8(out + off, dzv);
      else
        st8(out + off, v);
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
    stat_add(det, dst, which * OC + cgi * 8 + j, acc);
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
// >= 8 k-steps. fp32 (f32 = true): MFMA-bound (1/16 of the bf16 rate), so 128-row tiles (one
// 96 KiB workgroup per CU) are not used and the split-K target is the same workgroup count at
// twice the k-steps of a bf16 layer.
// Round 5 sweep (bench/r50_tiles.py, profiles/r5_r50_conv_tiles.jsonl, ResNet-50's 1x1 / strided
// layers, B = 128): bf16 128x128 tiles lose to 64x128 on every layer (by up to 1.4x: one 96 KB
// workgroup per CU), fp32 64x64 beats 64x128 on most (the data gradients by 3-9 %). Steps, same box
// (r5_call15): ResNet-50 bf16 19.33 -> 17.35 ms, fp32 36.89 -> 36.06; the fp32 64x64 choice costs
// ResNet-18 +0.2 % (its power-of-two 32x32 / 16x16 layers, tuned on 64x128 in round 2,
// bench/conv_sweep.py), so fp32 layers with a power-of-two pixel count keep 64x128.
Plan plan_for(int OC, int npix, int ksteps, bool f32 = false) {
  Plan p{64, 128, 1};
  if ((!f32 || !(npix & (npix - 1))) && (long)(OC / 64) * ((npix + 127) / 128) >= 512) {
    p.BM = 64;
    p.BN = 128;
  } else {
    p.BM = 64;
    p.BN = 64;
  }
  const long tiles = (long)(OC / p.BM) * ((npix + p.BN - 1) / p.BN);
  while (p.splits < 8 && tiles * p.splits < 512 && ksteps / (p.splits * 2) >= 8) p.splits *= 2;
  // experiment overrides (tile sweep, bench/conv_sweep.py): PSX_TUNE cv_bm / PSX_TUNE cv_bn / PSX_TUNE cv_splits
  if (const char* e = tune("cv_bm")) p.BM = atoi(e);
  if (const char* e = tune("cv_bn")) p.BN = atoi(e);
  if (const char* e = tune("cv_splits")) p.splits = atoi(e);
  if (const char* e = tune("cv_wgm")) p.WGM = atoi(e);
  if (OC % p.BM || (f32 && p.BM == 128 && !tune("cv_bm"))) p.BM = 64;
  if (p.splits > ksteps) p.splits = ksteps;
  return p;
}

// deterministic mode: this launch's slab rows (one per pixel tile, per parity class for MODE 3)
void with_det(Conv2Args& b, int rows) {
  (void)rows;
  if (b.stats || b.bpart) b.det = det_for(b.bpart ? b.bpart : b.stats);
}

template <typename T, int BM, int BN, int MODE, bool RES, bool SPLIT, int WGM = 2>
int launch2(const Conv2Args& a, hipStream_t st) {
  // LDS: the ring's stages in use (a 1x1 layer with one or two k-steps needs one or two of the
  // three) or the staged epilogue tile, whichever is larger — the short-reduction layers (the
  // 64-channel 1x1s of ResNet-50) then fit more workgroups per CU, so one's epilogue stores
  // overlap another's loads (a 128x128 bf16 tile: 96 -> 67.6 KB, 1 -> 2 per CU; measured neutral on
  // the ResNet-50 step, r5_call13, kept as the tighter bound)
  const int nk_max = SPLIT ? a.kps : (MODE == 3 ? 3 : a.Kg / kKS<T>);
  const int stages = nk_max < 3 ? (nk_max < 1 ? 1 : nk_max) : (a.nstg == 2 ? 2 : 3);
  const size_t ring = (size_t)stages * (BM + BN) * 128, epi = (size_t)BN * (BM + 4) * 4;
  const size_t red = (size_t)(256 / (BM / 8)) * 3 * BM * 4;  // the epilogue's statistic reduction
  const size_t epr = epi > red ? epi : red;
  const size_t lds = SPLIT ? ring : (ring > epr ? ring : epr);
  dim3 grid(a.n_oc_tiles * a.n_pix_tiles, SPLIT ? a.splits : (MODE == 3 ? 4 : 1));
  Conv2Args b = a;
  if (!SPLIT) with_det(b, a.n_pix_tiles * (MODE == 3 ? 4 : 1));
  hipLaunchKernelGGL((conv2_kernel<T, BM, BN, MODE, RES, SPLIT, WGM>), grid, dim3(256), lds, st, b);
  return (int)hipGetLastError();
}

template <typename T, int MODE, bool RES>
int dispatch2(const Plan& p, const Conv2Args& a, hipStream_t st) {
  const bool sp = p.splits > 1;
#define PSX_L2(BM_, BN_, W_)                                                                             \
  if (p.BM == BM_ && p.BN == BN_ && p.WGM == W_)                                                         \
    return sp ? launch2<T, BM_, BN_, MODE, false, true, W_>(a, st) : launch2<T, BM_, BN_, MODE, RES, false, W_>(a, st);
  PSX_L2(128, 128, 2)
  if constexpr (sizeof(T) == 2) PSX_L2(128, 256, 2)
  PSX_L2(64, 128, 2)
  PSX_L2(64, 64, 2)
  PSX_L2(64, 256, 1)
  PSX_L2(64, 128, 1)
#undef PSX_L2
  return -7;
}

template <typename T, int BM, int BN, int MODE, bool RES, int WGM, int TP = 1>
int launch_tapr(const Conv2Args& a, hipStream_t st) {
  const size_t lds = (size_t)2 * (3 * BM * 128 + (TP == 2 ? BN + 8 : BN) * 128);
  Conv2Args b = a;
  with_det(b, a.n_pix_tiles);
  hipLaunchKernelGGL((conv2_kernel<T, BM, BN, MODE, RES, false, WGM, TP>), dim3(a.n_oc_tiles * a.n_pix_tiles),
                     dim3(256), lds, st, b);
  return (int)hipGetLastError();
}

// Pixel-tile width of the tap-reuse path for this layer, 0 = not applicable: 3x3 / stride 1 /
// pad 1, square power-of-two images whose rows tile BN exactly, 64-channel chunks; no split-K.
// PSX_TUNE cv_tapr=0 disables it, PSX_TUNE cv_tapr_bn=64|128|256 forces the width (sweeps). Other widths
// (and PSX_TUNE cv_tapr_halo=1, a test override) take the halo mode with 64-pixel tiles: returns -64.
int tapr_bn(int R, int S, int stride, int pad, int H, int W, int IC, int OC, int npix, bool f32 = false) {
  if (const char* e = tune("cv_tapr"))
    if (e[0] == '0') return 0;
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || IC % 64 || OC % 64) return 0;
  const char* he = tune("cv_tapr_halo");
  const bool halo_off = he && he[0] == '0', halo_force = he && he[0] == '1';
  if (halo_force || H != W || (W & (W - 1)) || 64 % W) return halo_off ? 0 : -64;
  int force = 0;
  if (const char* e = tune("cv_tapr_bn")) force = atoi(e);
  // measured (bench/tapr_probe.py, ResNet-18 B=128, us fwd/dgrad): 64-pixel tiles (2 workgroups
  // per CU) win or tie on every layer — 32x32x64: 27.3/20.9 vs generic 26.3/23.0; 16x16x128:
  // 18.7/15.8 vs 20.6/19.3; 8x8x256: 14.8/13.7 vs 25.5/23.4; 4x4x512: 20.5/19.2 vs 29.3/28.0
  // (generic = split-K + epilogue launch there); 128/256-pixel tiles (1 workgroup per CU) lose.
  // fp32 (scripts/dev/f32_tapr_sweep.sh, us fwd/dgrad): 256-pixel tiles with 64x64 wave tiles (WGM 1)
  // win while the grid still has >= 256 workgroups — 32x32x64: 95/94 vs 103/97, 16x16x128: 85/84
  // vs 94/92 — and lose below (8x8x256: 148 vs 89); the f32 MFMA work per stage then hides the
  // DMA wait at one workgroup per CU
  int BN = force ? force : 64;
  if (!force && f32 && npix % 256 == 0 && 256 % W == 0 && (long)(npix / 256) * (OC / 64) >= 256) BN = 256;
  // bf16: 128-pixel tiles (two workgroups per CU: one's epilogue — the BN statistics or the BN-backward
  // sums — runs under the other's mainloop) where they fill two rounds of the chip, 64 below. Round 6,
  // same box (bench/conv_layers.py, profiles/r6_tapr_split_sweep.txt, us fwd / dgrad + BN-backward sums):
  // 32x32x64 24.3 / 31.8 (256-pixel tiles, the round-5 choice) -> 21.5 / 26.9, 16x16x128 18.3 / 20.1 ->
  // 17.2 / 20.6; the bf16 step 1.660 -> 1.605 ms (3 interleaved pairs, profiles/r6_numbers.jsonl)
  if (!force && !f32 && npix % 128 == 0 && 128 % W == 0 && (long)(npix / 128) * (OC / 64) >= 512) BN = 128;
#if PSX_TAPR_F32_128
  // fp32 with the register double buffer: 128-pixel tiles (two workgroups per CU, one's epilogue
  // under the other's mainloop) where they fill two full rounds of the chip. Same-box A/B: 32x32x64
  // 102.9/96.8 -> 99.2/94.0 us fwd/dgrad, 16x16 equal; bench 4.977 -> 4.936/4.946 ms/step
  if (!force && f32 && npix % 128 == 0 && 128 % W == 0 && (long)(npix / 128) * (OC / 64) >= 512) BN = 128;
#endif
  if ((BN != 64 && BN != 128 && BN != 256) || BN % W || npix % BN) return 0;
  return BN;
}

// (Round 6 measured split-K over the tap-reuse macro steps, partials through conv_splitk_epilogue,
// at every tile width x 2-8 splits on ResNet-18's four 3x3 layers, bench/conv_layers.py: slower on
// every one — the 4x4x512 layer's best 23.6 vs 21.2 us unsplit — profiles/r6_tapr_split_sweep.txt.)
template <typename T, int MODE, bool RES>
int dispatch_tapr(int bn, Conv2Args& a, hipStream_t st) {
  a.n_oc_tiles = a.OC / 64;
  a.splits = 1;
  a.kps = a.Kg / kKS<T>;
  if (bn < 0) {  // halo mode
    a.n_pix_tiles = (a.npix + 63) / 64;
    return launch_tapr<T, 64, 64, MODE, RES, 2, 2>(a, st);
  }
  a.n_pix_tiles = a.npix / bn;
  if (bn == 256) return launch_tapr<T, 64, 256, MODE, RES, 1>(a, st);
  if (bn == 128) return launch_tapr<T, 64, 128, MODE, RES, 2>(a, st);
  return launch_tapr<T, 64, 64, MODE, RES, 2>(a, st);
}

template <typename T>
int finish_split(const Conv2Args& a, hipStream_t st) {
  const int cvec = a.OC / 8;
  if (256 % cvec) return -8;
  // 32 pixels per workgroup (was >= 8, ~512 workgroups): every workgroup adds one set of
  // per-channel BN partials with same-address atomics, and fewer, longer workgroups halve that
  // traffic; their slab loads are batched 4 rows at a time. ResNet-18's one split-K layer
  // (4x4x512, 2048 pixels -> 64 workgroups): step fp32 3.268 -> 3.258 ms, bf16 1.580 -> 1.569
  // (profiles/r6_splitk_epilogue_ab.jsonl)
  const int ppb = 32;
  const int grid = (a.npix + ppb - 1) / ppb;
  const size_t lds = 256 * 24 * sizeof(float);
  DetRed det{};
  if (a.stats || a.bpart) det = det_for(a.bpart ? a.bpart : a.stats);
  if (a.res)
    hipLaunchKernelGGL((conv_splitk_epilogue<T, true>), dim3(grid), dim3(256), lds, st, a.part, a.splits, a.npix,
                       a.OC, (T*)a.out, (const T*)a.res, a.stats, ppb, a.fuse_fin, a.fin, a.bpart, (const T*)a.bo,
                       (const T*)a.by1, (const T*)a.by2, a.bsaved1, a.bsaved2, a.bns, a.bmask, det, a.sshift);
  else
    hipLaunchKernelGGL((conv_splitk_epilogue<T, false>), dim3(grid), dim3(256), lds, st, a.part, a.splits, a.npix,
                       a.OC, (T*)a.out, (const T*)nullptr, a.stats, ppb, a.fuse_fin, a.fin, a.bpart, (const T*)a.bo,
                       (const T*)a.by1, (const T*)a.by2, a.bsaved1, a.bsaved2, a.bns, a.bmask, det, a.sshift);
  return (int)hipGetLastError();
}

}  // namespace

struct BwdStatsDesc {  // fused BN-backward reduction over the dgrad output (see Conv2Args)
  float* part;
  const void* o;
  const void* y1;
  const void* y2;
  const float* saved1;
  const float* saved2;
  int mask_store;  // store dz = g*[o > 0] instead of g (Conv2Args::bmask)
};

namespace {

template <typename T>
int conv_fwd2_t(Conv2Args& a, float* ws, hipStream_t st) {
  constexpr int KS = kKS<T>;
  const int IC = a.IC, OC = a.OC, Kg = a.Kg;
  a.log2_icc = ilog2i(IC / kEPC<T>);
  if (OC % 64 || Kg % KS || IC % kEPC<T> || (IC & (IC - 1))) return -2;
  if (const int tbn = tapr_bn(a.R, a.S, a.stride, a.pad, a.IH, a.IW, IC, OC, a.npix, sizeof(T) == 4))
    return dispatch_tapr<T, 0, false>(tbn, a, st);
  const Plan p = plan_for(OC, a.npix, Kg / KS, sizeof(T) == 4);
  a.n_oc_tiles = OC / p.BM;
  a.n_pix_tiles = (a.npix + p.BN - 1) / p.BN;
  a.splits = p.splits;
  a.kps = (Kg / KS + p.splits - 1) / p.splits;
  if (p.splits > 1 && !ws) return -9;
  int e = dispatch2<T, 0, false>(p, a, st);
  if (e || p.splits == 1) return e;
  return finish_split<T>(a, st);
}

template <typename T>
int conv_dgrad2_t(Conv2Args& a, float* ws, hipStream_t st) {
  constexpr int KS = kKS<T>;
  const int OC_fwd = a.IC, IC_fwd = a.OC, Kg = a.Kg, Nb = a.Nb, H = a.OH, W = a.OW;
  a.log2_icc = ilog2i(OC_fwd / kEPC<T>);
  if (IC_fwd % 64 || Kg % KS || (OC_fwd & (OC_fwd - 1)) || OC_fwd % kEPC<T>) return -2;
  const bool res = a.res != nullptr;
  if (const int tbn = tapr_bn(a.R, a.S, a.stride, a.pad, H, W, OC_fwd, IC_fwd, a.npix, sizeof(T) == 4))
    return res ? dispatch_tapr<T, 1, true>(tbn, a, st) : dispatch_tapr<T, 1, false>(tbn, a, st);
  const Plan p = plan_for(IC_fwd, a.npix, Kg / KS, sizeof(T) == 4);
  a.n_oc_tiles = IC_fwd / p.BM;
  a.n_pix_tiles = (a.npix + p.BN - 1) / p.BN;
  a.splits = p.splits;
  a.kps = (Kg / KS + p.splits - 1) / p.splits;
  const bool parity = a.stride == 2 && a.log2_icc >= 3;
  if (p.splits > 1 && !ws && !parity) return -9;  // the parity-class path never splits K
  int e;
  if (a.stride == 1)
    e = res ? dispatch2<T, 1, true>(p, a, st) : dispatch2<T, 1, false>(p, a, st);
  else if (a.in2 && !(a.stride == 2 && a.log2_icc >= 3))
    return -11;  // the shortcut folds only into the parity-class path
  else if (parity) {
    // parity classes: each class GEMM covers dx pixels (2i+py, 2j+px), ~1/4 of them
    Plan q = plan_for(IC_fwd, (a.npix + 3) / 4, Kg / KS, sizeof(T) == 4);
    q.splits = 1;
    if (IC_fwd % q.BM) q.BM = 64;
    a.n_oc_tiles = IC_fwd / q.BM;
    a.n_pix_tiles = (Nb * ((H + 1) / 2) * ((W + 1) / 2) + q.BN - 1) / q.BN;
    a.splits = 1;
    a.kps = Kg / KS;
    return res ? dispatch2<T, 3, true>(q, a, st) : dispatch2<T, 3, false>(q, a, st);
  } else if (a.stride == 2)
    e = res ? dispatch2<T, 2, true>(p, a, st) : dispatch2<T, 2, false>(p, a, st);
  else
    return -4;
  if (e || p.splits == 1) return e;
  return finish_split<T>(a, st);
}

}  // namespace

extern "C" {

// Bytes of fp32 split-K workspace the v2 conv needs for this problem (0 = no split).
// f32: the operands are fp32 (32-channel k-steps) instead of bf16.
long psx_conv2_workspace(int Nb, int OH, int OW, int OC, int Kg, int f32) {
  const int npix = Nb * OH * OW;
  const Plan p = plan_for(OC, npix, Kg / (f32 ? 32 : 64), f32 != 0);
  return p.splits > 1 ? (long)p.splits * npix * OC * 4 : 0;
}

// Forward conv (v2). Same operands as psx_conv_fwd plus a 16-byte zero page and a split-K
// workspace (>= psx_conv2_workspace bytes, may be null when that is 0).
// fin (nullable, needs stats): the BN layer fed by this conv is finalized by the kernel's last
// workgroup (bnfin.hpp) instead of a separate psx_bn_finalize launch.
// f32: x, wf, y are fp32 (the reference's precision) instead of bf16.
// sshift (nullable): per-channel shift of the BN statistics (Conv2Args::sshift)
int psx_conv_fwd2(const void* x, const void* wf, void* y, float* stats, const void* zero, float* ws, int Nb, int H,
                  int W, int IC, int OC, int R, int S, int stride, int pad, int Kg, const BnFin* fin, int f32,
                  const float* sshift, hipStream_t st) {
  Conv2Args a{};
  a.sshift = sshift;
  if (fin && stats) {
    if (fin->C != OC) return -10;
    a.fuse_fin = 1;
    a.fin = *fin;
    a.fin.det = (int)det_enabled();
  }
  a.in = x;
  a.w = wf;
  a.out = y;
  a.res = nullptr;
  a.stats = stats;
  a.part = ws;
  a.zero = zero;
  a.Nb = Nb; a.IH = H; a.IW = W; a.IC = IC;
  a.OH = (H + 2 * pad - R) / stride + 1;
  a.OW = (W + 2 * pad - S) / stride + 1;
  a.OC = OC; a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.npix = Nb * a.OH * a.OW;
  return f32 ? conv_fwd2_t<float>(a, ws, st) : conv_fwd2_t<uint16_t>(a, ws, st);
}

int psx_conv_dgrad2_sc(const void* dy, const void* wd, void* dx, const void* res, const void* zero, float* ws,
                       int Nb, int H, int W, int IC_fwd, int OC_fwd, int R, int S, int stride, int pad, int Kg,
                       const BwdStatsDesc* bst, int f32, const void* dy_sc, const void* wd_sc, int Kg_sc,
                       hipStream_t st);

int psx_conv_dgrad2(const void* dy, const void* wd, void* dx, const void* res, const void* zero, float* ws, int Nb,
                    int H, int W, int IC_fwd, int OC_fwd, int R, int S, int stride, int pad, int Kg,
                    const BwdStatsDesc* bst, int f32, hipStream_t st) {
  return psx_conv_dgrad2_sc(dy, wd, dx, res, zero, ws, Nb, H, W, IC_fwd, OC_fwd, R, S, stride, pad, Kg, bst, f32,
                            nullptr, nullptr, 0, st);
}

// psx_conv_dgrad2 of a 3x3 / stride-2 / pad-1 conv with its block's 1x1 / stride-2 / pad-0
// shortcut folded in: dx = dgrad(dy, wd) + dgrad_sc(dy_sc, wd_sc) in one launch (Conv2Args in2;
// the parity-class path only). dy_sc: the shortcut's output gradient (the shape of dy), wd_sc:
// its data-gradient weights, rows of Kg_sc (= OC_fwd). -11: this layer cannot fold (caller runs
// the two launches).
int psx_conv_dgrad2_sc(const void* dy, const void* wd, void* dx, const void* res, const void* zero, float* ws,
                       int Nb, int H, int W, int IC_fwd, int OC_fwd, int R, int S, int stride, int pad, int Kg,
                       const BwdStatsDesc* bst, int f32, const void* dy_sc, const void* wd_sc, int Kg_sc,
                       hipStream_t st) {
  Conv2Args a{};
  if (dy_sc) {
    if (R != 3 || S != 3 || stride != 2 || pad != 1 || res || Kg_sc != OC_fwd || !wd_sc) return -11;
    a.in2 = dy_sc;
    a.w2 = wd_sc;
    a.Kg2 = Kg_sc;
  }
  if (bst) {
    a.bpart = bst->part;
    a.bo = bst->o;
    a.by1 = bst->y1;
    a.by2 = bst->y2;
    a.bsaved1 = bst->saved1;
    a.bsaved2 = bst->saved2;
    a.bns = bst->y2 ? 3 : 2;
    a.bmask = bst->mask_store;
  }
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  a.in = dy;
  a.w = wd;
  a.out = dx;
  a.res = res;
  a.stats = nullptr;
  a.part = ws;
  a.zero = zero;
  a.Nb = Nb; a.IH = P; a.IW = Q; a.IC = OC_fwd;
  a.OH = H; a.OW = W; a.OC = IC_fwd;
  a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.npix = Nb * H * W;
  return f32 ? conv_dgrad2_t<float>(a, ws, st) : conv_dgrad2_t<uint16_t>(a, ws, st);
}

// nb independent fp32 GEMMs P[b][M][N] = A[b] . B[:, b, :]^T with A [nb][M][Kd] (batch-major
// rows) and B [N][nb][Kd], Kd a power of two >= 32, on the conv mainloop: an implicit GEMM over M
// "pixels" whose nb "taps" are the batches — the operand is an image of nb rows x M columns
// (R = nb, S = 1: tap b reads row b, i.e. A[b]) — split-K into nb slabs of Kd, so split s is
// exactly batch s (the Winograd GEMMs, wino.hip). cfg: tile (0: 64x64, 1: 64x128, 2: 64x256 /
// 1x4 waves, 3: 64x128 / 1x4 waves; N rows x M pixels).
// s2 > 1: each batch's Kd-long reduction as s2 ranges (whole k-steps) writing s2 partial slabs
// P[b s2 + j][M][N] (the Winograd output transform sums them, wino.hip psx_wino_conv)
// LDS ring depth of the batched GEMMs (Conv2Args::nstg): 2 (5 fp32 64x64 workgroups per CU
// instead of 3). Same box, wino_conv forward us 3-deep / 2-deep (bench/wino_gemm_ab.py,
// profiles/r6_wino_gemm_stages_ab.jsonl): 8x8x256 51.0 / 49.9, 4x4x512 45.9 / 44.8, 14x14x256
// 144.8 / 139.8, 7x7x512 120.9 / 120.1
static int bgemm_stages() { return 2; }

int psx_bgemm_f32_split(const float* A, const float* B, float* P, const void* zero, int M, int N, int Kd, int nb,
                        int s2, int cfg, hipStream_t st) {
  if (N % 64 || Kd < kKS<float> || (Kd & (Kd - 1)) || M < 1 || nb < 1 || s2 < 1 || (Kd / kKS<float>) % s2) return -2;
  Plan p{64, 64, nb * s2, 2};
  if (cfg == 1) p.BN = 128;
  if (cfg == 2) { p.BN = 256; p.WGM = 1; }
  if (cfg == 3) { p.BN = 128; p.WGM = 1; }
  Conv2Args a{};
  a.in = A;
  a.w = B;
  a.out = nullptr;
  a.part = P;
  a.zero = zero;
  a.Nb = 1; a.IH = nb; a.IW = M; a.OH = 1; a.OW = M;
  a.IC = Kd;
  a.OC = N;
  a.R = nb; a.S = 1; a.pad = 0; a.stride = 1;
  a.Kg = nb * Kd;
  a.log2_icc = ilog2i(Kd / kEPC<float>);
  a.npix = M;
  a.n_oc_tiles = N / 64;
  a.n_pix_tiles = (M + p.BN - 1) / p.BN;
  a.splits = nb * s2;
  a.kps = Kd / kKS<float> / s2;
  a.nstg = bgemm_stages();
  return nb * s2 > 1 ? dispatch2<float, 0, false>(p, a, st) : -2;
}

int psx_bgemm_f32(const float* A, const float* B, float* P, const void* zero, int M, int N, int Kd, int nb, int cfg,
                  hipStream_t st) {
  return psx_bgemm_f32_split(A, B, P, zero, M, N, Kd, nb, 1, cfg, st);
}

}  // extern "C"
