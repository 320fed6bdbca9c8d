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
  const void* x;         // NHWC [Nb][IH][IW][IC] (bf16 bits, or fp32 for wgrad2f_kernel)
  const void* dy;        // NHWC [Nb][OH][OW][OC]
  float* part;           // [splits][OC][Kg]
  const void* zero;      // 16-byte zero page
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

  const uint16_t* const xg = (const uint16_t*)a.x;
  const uint16_t* const dyg = (const uint16_t*)a.dy;
  const uint16_t* const zero = (const uint16_t*)a.zero;
  // 1x1 / stride 1 / pad 0 (most of ResNet-50's weight gradients): output pixel == input pixel,
  // no (n, oh, ow) decomposition per staged row
  const bool ident = a.R == 1 && a.S == 1 && a.stride == 1 && a.pad == 0;
  auto issue = [&](int st, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int p0 = pbeg + st * 64;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int pix = p0 + xrow[i];
      const uint16_t* src = zero;
      if (ident) {
        if (pix < a.npix && xtap_ok[i]) src = xg + (size_t)pix * a.IC + xc0[i];
      } else if (pix < a.npix && xtap_ok[i]) {
        const int n = fdiv(pix, a.div_ohw);
        const int rem = pix - n * a.div_ohw.d;
        const int oh = fdiv(rem, a.div_ow);
        const int ow = rem - oh * OW;
        const int ih = oh * a.stride - a.pad + xtap_r[i], iw = ow * a.stride - a.pad + xtap_s[i];
        if ((unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW)
          src = xg + ((size_t)(n * a.IH + ih) * a.IW + iw) * a.IC + xc0[i];
      }
      glds16(src, base + (i * 4 + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int pix = p0 + drow[i];
      const uint16_t* src = pix < a.npix ? dyg + (size_t)pix * a.OC + oc0 + dchunk[i] * 8 : zero;
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
  // unrolled by NS: compile-time stage offsets (see wgrad3_kernel)
  auto step = [&](const int st, auto sc) {
    constexpr int stage = decltype(sc)::value;
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
  };
  for (int st0 = 0; st0 < nsteps; st0 += NS)
    static_for<0, NS>([&](auto sc) {
      const int st = st0 + decltype(sc)::value;
      if (st < nsteps) step(st, sc);
    });

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

// ---------------------------------------------------------------------------------------
// wgrad2f: the fp32 weight gradient (the reference's training precision). Same GEMM, grid and
// LDS-DMA ring as wgrad2_kernel, fp32 operands: a stage holds 32 pixels x (BR + BC) fp32 columns
// and the reduction runs on v_mfma_f32_16x16x4_f32 (exact f32). Its A/B fragments hold ONE
// element per lane (lane l: column l & 15 of pixel 4s + (l >> 4)), so the pixel-major tiles need
// no transposed read: one ds_read_b32 per operand per MFMA. Rows are 256/512 B (a multiple of
// the 32 banks), so the 16-byte chunk index is XOR-ed with bit 2 on odd rows (applied to the DMA
// source address, the LDS destination stays lane-linear): the two rows a 32-lane read group
// touches then sit 16 banks apart, conflict-free.
template <int BR, int BC, int NS>
__global__ __launch_bounds__(256) void wgrad2f_kernel(Wgrad2Args a) {
  constexpr int PS = 32;                                  // pixels per stage
  constexpr int XROWB = BR * 4, DROWB = BC * 4;           // bytes per pixel row
  constexpr int XCPR = XROWB / 16, DCPR = DROWB / 16;     // 16-byte chunks per row
  constexpr int XRPI = 64 / XCPR, DRPI = 64 / DCPR;       // rows per DMA instruction
  constexpr int LX = PS / XRPI / 4, LD = PS / DRPI / 4;   // DMA instructions per wave per stage
  constexpr int XT = PS * XROWB, DT = PS * DROWB, STAGE = XT + DT;
  constexpr int MT = BR / 32, NT = BC / 32;
  static_assert(LX >= 1 && LD >= 1, "tile too narrow for the 32-pixel stage");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = a.n_k_tiles * a.n_oc_tiles;
  const int bid = xcd_remap(blockIdx.x, ntile * a.splits);
  const int split = bid / ntile, t = bid - split * ntile;
  const int oc_t = t % a.n_oc_tiles, k_t = t / a.n_oc_tiles;
  const int k0 = k_t * BR, oc0 = oc_t * BC;
  const int pbeg = split * a.steps_per_split * PS;
  const int nsteps = min(a.steps_per_split, (a.npix - pbeg + PS - 1) / PS);
  const float* const xg = (const float*)a.x;
  const float* const dyg = (const float*)a.dy;
  const float* const zero = (const float*)a.zero;

  int xrow[LX], xtap_r[LX], xtap_s[LX], xc0[LX];
  bool xtap_ok[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int row = (i * 4 + wid) * XRPI + lane / XCPR;
    const int c = (lane % XCPR) ^ ((row & 1) << 2);  // logical chunk of this lane's slot
    xrow[i] = row;
    const int gk = (k0 >> 2) + c;
    const int tap = gk >> a.log2_icc;
    xc0[i] = (gk & ((1 << a.log2_icc) - 1)) << 2;
    xtap_ok[i] = tap < a.R * a.S;
    const int r = fdiv(tap, a.div_s);
    xtap_r[i] = r;
    xtap_s[i] = tap - r * a.S;
  }
  int drow[LD], dchunk[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int row = (i * 4 + wid) * DRPI + lane / DCPR;
    drow[i] = row;
    dchunk[i] = (lane % DCPR) ^ ((row & 1) << 2);
  }
  const int OW = a.div_ow.d;
  const bool ident = a.R == 1 && a.S == 1 && a.stride == 1 && a.pad == 0;  // (see wgrad2_kernel)

  auto issue = [&](int st, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int p0 = pbeg + st * PS;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int pix = p0 + xrow[i];
      const float* src = zero;
      if (ident) {
        if (pix < a.npix && xtap_ok[i]) src = xg + (size_t)pix * a.IC + xc0[i];
      } else if (pix < a.npix && xtap_ok[i]) {
        const int n = fdiv(pix, a.div_ohw);
        const int rem = pix - n * a.div_ohw.d;
        const int oh = fdiv(rem, a.div_ow);
        const int ow = rem - oh * OW;
        const int ih = oh * a.stride - a.pad + xtap_r[i], iw = ow * a.stride - a.pad + xtap_s[i];
        if ((unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW)
          src = xg + ((size_t)(n * a.IH + ih) * a.IW + iw) * a.IC + xc0[i];
      }
      glds16(src, base + (i * 4 + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int pix = p0 + drow[i];
      const float* src = pix < a.npix ? dyg + (size_t)pix * a.OC + oc0 + dchunk[i] * 4 : zero;
      glds16(src, base + XT + (i * 4 + wid) * 1024);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // per-lane fragment byte offsets within a row (odd rows: chunk bit 2 flipped)
  const int kq = lane >> 4, col = lane & 15;
  int aoff[MT], boff[NT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int c = wm * (BR / 2) + m * 16 + col;
    aoff[m] = (((c >> 2) ^ ((kq & 1) << 2)) << 4) + ((c & 3) << 2);
  }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int c = wn * (BC / 2) + n * 16 + col;
    boff[n] = (((c >> 2) ^ ((kq & 1) << 2)) << 4) + ((c & 3) << 2);
  }

#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nsteps) issue(i, i);
  // unrolled by NS: compile-time stage offsets (see wgrad3_kernel)
  auto step = [&](const int st, auto sc) {
    constexpr int stage = decltype(sc)::value;
    const int ahead = min(NS - 2, nsteps - 1 - st);
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
    for (int s4 = 0; s4 < PS / 4; ++s4) {
      const int row = 4 * s4 + kq;
      float fa[MT], fb[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m) fa[m] = *reinterpret_cast<const float*>(X + row * XROWB + aoff[m]);
#pragma unroll
      for (int n = 0; n < NT; ++n) fb[n] = *reinterpret_cast<const float*>(D + row * DROWB + boff[n]);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
  };
  for (int st0 = 0; st0 < nsteps; st0 += NS)
    static_for<0, NS>([&](auto sc) {
      const int st = st0 + decltype(sc)::value;
      if (st < nsteps) step(st, sc);
    });

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

// ---------------------------------------------------------------------------------------
// wgrad3: 3x3 / stride 1 / pad 1 with tap reuse. For one kernel row r, the three taps s=0,1,2
// read the same input row shifted by -1/0/+1 pixels, so one LDS window of 64 input pixels
// x(n, oh+r-1, ow) (plus one zero row for the row edges) feeds a 192-row output tile
// (3 taps x 64 channels) instead of three 64-row tiles each gathering its own copy. Each lane's
// transposed-read address picks slot (pixel + s - 1), or the zero row when ow + s - 1 leaves
// the image row; 64-pixel steps hold whole rows because W is a power of two <= 64. Staged
// bytes per step stay ~16 KB while the MFMA work per step triples (wgrad2 is LDS-DMA bound).
// G (general widths, e.g. ResNet-50's 56 / 28 / 14 / 7): a step takes PIX = 56 pixels — whole
// rows of any W dividing 56 — in the 64-row tiles; rows 56..63 are zero on both operands (1/8 of
// the MFMA work idle), pixel -> (oh, ow) by multiply-high division.
struct Wgrad3Args {
  const uint16_t* x;
  const uint16_t* dy;
  float* part;
  const uint16_t* zero;  // (bf16 only)
  int H, W, log2w, IC, OC, Kg, npix;
  int n_c_tiles, n_oc_tiles, splits, steps_per_split;
  int pix;               // pixels per step (G: 56)
  FastDiv div_w, div_h;  // (G)
};

// wait until at most `ahead` later stage groups (PER DMA ops each) are still in flight
template <int PER, int MAXA>
PSX_DEV void wait_ahead(int ahead) {
  if constexpr (MAXA <= 0) {
    wait_vmcnt<0>();
  } else {
    if (ahead >= MAXA)
      wait_vmcnt<MAXA * PER>();
    else
      wait_ahead<PER, MAXA - 1>(ahead);
  }
}

template <int BC, int NS, bool G>
__global__ __launch_bounds__(256) void wgrad3_kernel(Wgrad3Args a) {
  constexpr int DROWB = BC * 2, DCPR = DROWB / 16, DRPI = 64 / DCPR, LD = 64 / DRPI / 4;
  constexpr int XT = 65 * 128, DT = 64 * DROWB, STAGE = XT + DT;
  constexpr int NT = BC / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = 3 * a.n_c_tiles * a.n_oc_tiles;
  const int bid = xcd_remap(blockIdx.x, ntile * a.splits);
  const int split = bid / ntile, t = bid - split * ntile;
  const int oc_t = t % a.n_oc_tiles, rest = t / a.n_oc_tiles;
  const int c_t = rest % a.n_c_tiles, r = rest / a.n_c_tiles;
  const int c0 = c_t * 64, oc0 = oc_t * BC;
  const int PIX = G ? a.pix : 64;
  const int pbeg = split * a.steps_per_split * PIX;
  const int nsteps = min(a.steps_per_split, (a.npix - pbeg + PIX - 1) / PIX);
  const int W = a.W;

  // zero row (slot 64) of every stage; the DMA never writes it
  if (tid < NS * 8) *reinterpret_cast<uint4*>(smem + (tid >> 3) * STAGE + 64 * 128 + (tid & 7) * 16) = uint4{0, 0, 0, 0};

  // ---- per-lane DMA state ----
  int xrow[2], xcol[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (i * 4 + wid) * 8 + (lane >> 3);
    xrow[i] = row;
    xcol[i] = c0 + (((lane & 7) ^ (((row >> 1) & 3) << 1)) << 3);
  }
  int drow[LD], dchunk[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int row = (i * 4 + wid) * DRPI + lane / DCPR;
    const int pos = lane % DCPR;
    drow[i] = row;
    dchunk[i] = (DROWB == 128) ? (pos ^ (((row >> 1) & 3) << 1)) : (pos ^ ((row & 7) << 1));
  }
  const long xshift = (long)(r - 1) * W;

  auto issue = [&](int st, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int p0 = pbeg + st * PIX;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pix = p0 + xrow[i];
      int ih;
      if constexpr (G) {
        const int q = fdiv(pix, a.div_w);
        ih = q - fdiv(q, a.div_h) * a.H + r - 1;
      } else {
        ih = ((pix >> a.log2w) & (a.H - 1)) + r - 1;
      }
      const uint16_t* src = a.zero;
      if ((!G || xrow[i] < PIX) && pix < a.npix && (unsigned)ih < (unsigned)a.H)
        src = a.x + ((long)pix + xshift) * a.IC + xcol[i];
      glds16(src, base + (i * 4 + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int pix = p0 + drow[i];
      const bool ok = (!G || drow[i] < PIX) && pix < a.npix;
      const uint16_t* src = ok ? a.dy + (size_t)pix * a.OC + oc0 + dchunk[i] * 8 : a.zero;
      glds16(src, base + XT + (i * 4 + wid) * 1024);
    }
  };

  // per-lane window slots: logical K row (pixel) -> physical LDS row for tap s
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  int soff[2][2][3], sxr[2][2][3];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = kk * 32 + h * 16 + 4 * g + q;
      const int ow = G ? row - fdiv(row, a.div_w) * W : row & (W - 1);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int iw = ow + s - 1;
        const int slot = ((!G || row < PIX) && (unsigned)iw < (unsigned)W) ? row + s - 1 : 64;
        soff[kk][h][s] = slot * 128 + ((4 * p & 7) << 1);
        sxr[kk][h][s] = ((slot >> 1) & 3) << 1;
      }
    }

  f32x4 acc[6][NT];
#pragma unroll
  for (int m = 0; m < 6; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  __syncthreads();
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nsteps) issue(i, i);
  // The step loop is unrolled by NS so that every step's stage is a compile-time constant: the
  // fragment reads then address LDS as per-lane offsets hoisted out of the loop + an immediate
  // (a runtime stage base cost one v_add per read, ~2 of wgrad3's 5.3 VALU per MFMA).
  auto step = [&](const int st, auto sc) {
    constexpr int stage = decltype(sc)::value;
    wait_ahead<2 + LD, NS - 2>(min(NS - 2, nsteps - 1 - st));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + NS - 1 < nsteps) issue(st + NS - 1, stage == 0 ? NS - 1 : stage - 1);
    const unsigned char* X = smem + stage * STAGE;
    const unsigned char* D = X + XT;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int row0 = kk * 32 + 4 * g + q, row1 = row0 + 16;
      bf16x8 fa[6], fb[NT];
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        const int s = m >> 1;
        const int cc = ((wm * 32 + (m & 1) * 16) >> 3) + (p >> 1);  // 16-byte chunk of the channel
        const s16x4 lo = tr_read2(X, soff[kk][0][s] + ((cc ^ sxr[kk][0][s]) << 4));
        const s16x4 hi = tr_read2(X, soff[kk][1][s] + ((cc ^ sxr[kk][1][s]) << 4));
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
      for (int m = 0; m < 6; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
  };
  for (int st0 = 0; st0 < nsteps; st0 += NS)
    static_for<0, NS>([&](auto sc) {
      const int st = st0 + decltype(sc)::value;
      if (st < nsteps) step(st, sc);
    });

  float* part = a.part + (size_t)split * a.OC * a.Kg;
#pragma unroll
  for (int m = 0; m < 6; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int k = (r * 3 + (m >> 1)) * a.IC + c0 + wm * 32 + (m & 1) * 16 + 4 * (lane >> 4);
      const int oc = oc0 + wn * (BC / 2) + n * 16 + (lane & 15);
      *reinterpret_cast<f32x4*>(part + (size_t)oc * a.Kg + k) = acc[m][n];
    }
}

// ---------------------------------------------------------------------------------------
// wgrad3f: the fp32 tap-reuse weight gradient (3x3 / stride 1 / pad 1, power-of-two W <= 32).
// Same decomposition as wgrad3 — one workgroup = kernel row r x 64 input channels x BC output
// channels x a pixel range, its 192-row tile covering the taps s = 0, 1, 2 — on the exact-f32
// v_mfma_f32_16x16x4_f32. A stage holds 32 pixels (whole image rows: W divides 32) of x shifted
// by r - 1 rows and of dy; the A fragment of tap s is the x window read one slot left / in place /
// one slot right (lane l: channel l & 15 of pixel 4k + (l >> 4) + s - 1). Slots that leave the
// image row (ow + s - 1 outside [0, W)) are zeroed in registers from a per-lane bit mask over the
// 8 k-steps, computed once. Compared with wgrad2f (64x64 tiles, one tap per row) the MFMA work
// per staged byte triples: x is staged once per kernel row instead of once per tap. Rows are
// 256 B (x) / 256-512 B (dy); the 16-byte chunk index is XOR-ed with bit 2 on odd slots (in the
// DMA source address), so the two slots a 32-lane read group touches sit 16 banks apart. A
// 256-byte guard row in front of every stage's x tile absorbs the masked slot -1 read.
template <int BC, int NS>
__global__ __launch_bounds__(256) void wgrad3f_kernel(Wgrad3Args a) {
  constexpr int PS = 32;
  constexpr int DROWB = BC * 4, DCPR = DROWB / 16, DRPI = 64 / DCPR;
  constexpr int LX = PS / 4 / 4, LD = PS / DRPI / 4;  // DMA instructions per wave per stage
  constexpr int GUARD = 256, XT = PS * 256, DT = PS * DROWB, STAGE = GUARD + XT + DT;
  constexpr int NT = BC / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = 3 * a.n_c_tiles * a.n_oc_tiles;
  const int bid = xcd_remap(blockIdx.x, ntile * a.splits);
  const int split = bid / ntile, t = bid - split * ntile;
  const int oc_t = t % a.n_oc_tiles, rest = t / a.n_oc_tiles;
  const int c_t = rest % a.n_c_tiles, r = rest / a.n_c_tiles;
  const int c0 = c_t * 64, oc0 = oc_t * BC;
  const int pbeg = split * a.steps_per_split * PS;
  const int nsteps = min(a.steps_per_split, (a.npix - pbeg) / PS);
  const int W = a.W;
  const float* const xg = (const float*)a.x;
  const float* const dyg = (const float*)a.dy;
  const float* const zero = (const float*)a.zero;

  // ---- per-lane DMA state ----
  int xrow[LX], xcol[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int row = (i * 4 + wid) * 4 + (lane >> 4);
    xrow[i] = row;
    xcol[i] = c0 + (((lane & 15) ^ ((row & 1) << 2)) << 2);
  }
  int drow[LD], dcol[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int row = (i * 4 + wid) * DRPI + lane / DCPR;
    drow[i] = row;
    dcol[i] = oc0 + (((lane % DCPR) ^ ((row & 1) << 2)) << 2);
  }
  const long xshift = (long)(r - 1) * W;

  auto issue = [&](int st, int stage) {
    unsigned char* base = smem + stage * STAGE + GUARD;
    const int p0 = pbeg + st * PS;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int pix = p0 + xrow[i];
      const int ih = ((pix >> a.log2w) & (a.H - 1)) + r - 1;
      const float* src = (unsigned)ih < (unsigned)a.H ? xg + ((long)pix + xshift) * a.IC + xcol[i] : zero;
      glds16(src, base + (i * 4 + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < LD; ++i) glds16(dyg + (size_t)(p0 + drow[i]) * a.OC + dcol[i], base + XT + (i * 4 + wid) * 1024);
  };

  // per-lane fragment offsets (relative to the k-step's first slot row) and tap masks
  const int kq = lane >> 4, col = lane & 15;
  int aoff[3][2], boff[NT];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int c = wm * 32 + m * 16 + col;
      aoff[s][m] = (kq + s - 1) * 256 + ((((c >> 2) ^ (((kq + s + 1) & 1) << 2)) << 4) + ((c & 3) << 2));
    }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int c = wn * (BC / 2) + n * 16 + col;
    boff[n] = kq * DROWB + ((((c >> 2) ^ ((kq & 1) << 2)) << 4) + ((c & 3) << 2));
  }
  unsigned lmask = 0, rmask = 0;  // bit k: slot of tap 0 / tap 2 inside the image row at k-step k
#pragma unroll
  for (int k = 0; k < PS / 4; ++k) {
    const int ow = (4 * k + kq) & (W - 1);
    lmask |= (ow != 0 ? 1u : 0u) << k;
    rmask |= (ow != W - 1 ? 1u : 0u) << k;
  }

  f32x4 acc[3][2][NT];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[s][m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nsteps) issue(i, i);
  int stage = 0;
  for (int st = 0; st < nsteps; ++st) {
    wait_ahead<LX + LD, NS - 2>(min(NS - 2, nsteps - 1 - st));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + NS - 1 < nsteps) issue(st + NS - 1, stage == 0 ? NS - 1 : stage - 1);
    const unsigned char* X = smem + stage * STAGE + GUARD;
    const unsigned char* D = X + XT;
#pragma unroll
    for (int k = 0; k < PS / 4; ++k) {
      float fa[3][2], fb[NT];
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const float v = *reinterpret_cast<const float*>(X + k * 1024 + aoff[s][m]);
          fa[s][m] = s == 1 ? v : (((s == 0 ? lmask : rmask) >> k) & 1u) ? v : 0.f;
        }
#pragma unroll
      for (int n = 0; n < NT; ++n) fb[n] = *reinterpret_cast<const float*>(D + k * 4 * DROWB + boff[n]);
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < NT; ++n)
            acc[s][m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s][m], fb[n], acc[s][m][n], 0, 0, 0);
    }
    stage = stage == NS - 1 ? 0 : stage + 1;
  }

  float* part = a.part + (size_t)split * a.OC * a.Kg;
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int k = (r * 3 + s) * a.IC + c0 + wm * 32 + m * 16 + 4 * (lane >> 4);
        const int oc = oc0 + wn * (BC / 2) + n * 16 + (lane & 15);
        *reinterpret_cast<f32x4*>(part + (size_t)oc * a.Kg + k) = acc[s][m][n];
      }
}

}  // namespace psx

using namespace psx;

namespace {

struct WPlan {
  int BR, BC, NS, splits, sps;
};

// Workgroup slots of the chip the weight gradient plans for (256 CUs x occupancy).
int wg_slots(int occ) { return 256 * occ; }

// LDS bytes per workgroup of an NS-stage BR x BC tile (64 pixels per stage).
constexpr int wlds(int BR, int BC, int NS) { return NS * 64 * (BR + BC) * 2; }

// Occupancy-aware plan: tiles x splits workgroups should fill whole rounds of the
// 256 CUs x (workgroups per CU that the LDS allows), with >= 8 pixel-steps per split; among
// the tile shapes the one with the lowest modelled time wins (per-step costs measured on
// MI355X with rocprofv3: 128x128 ~1.2 us at 1 WG/CU, 64x64 ~0.7 us at 3 WG/CU; +3 us
// prologue/epilogue per workgroup; split-K partials cost a write + a read at ~5 TB/s).
// fbr / fbc (> 0): only that tile (its split count still from the model).
WPlan wplan(int OC, int Kg, int npix, int fbr = 0, int fbc = 0) {
  WPlan best{64, 64, 3, 1, 0};
  double best_t = 1e30;
  const int steps = (npix + 63) / 64;
  const int brs[2] = {128, 64}, bcs[2] = {128, 64};
  for (int ib = 0; ib < 2; ++ib)
    for (int ic = 0; ic < 2; ++ic) {
      const int BR = brs[ib], BC = bcs[ic];
      if ((fbr && BR != fbr) || (fbc && BC != fbc)) continue;
      if (Kg % BR || OC % BC || (BR == 128 && Kg < 256)) continue;
      const int NS = (BR == 128 && BC == 128) ? 4 : 3;
      int occ = 163840 / wlds(BR, BC, NS);
      if (occ > 3) occ = 3;
      if (occ < 1) continue;
      const int slots = wg_slots(occ);
      const long tiles = (long)(Kg / BR) * (OC / BC);
      const double step_us = 0.55 + 0.15 * (double)(BR * BC) / 4096.0;
      int smax = steps / 8 > 0 ? steps / 8 : 1;
      // (cap 64 until round 6: ResNet-50's 56x56 1x1 layers sat at it with ~98 steps per
      // workgroup; 256 measured -2 % on its bf16 step, profiles/r6_wgrad_split_cap_ab.jsonl)
      for (int sp = 1; sp <= smax && sp <= 256; ++sp) {
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

constexpr int wlds3(int BC, int NS) { return NS * (65 * 128 + 64 * BC * 2); }

// wgrad3 plan, same model as wplan with wgrad3's per-step costs.
WPlan wplan3(int OC, int IC, int Kg, int npix, int pix = 64) {
  WPlan best{0, 64, 3, 1, 0};
  double best_t = 1e30;
  const int steps = npix / pix;
  for (int cfg = 0; cfg < 4; ++cfg) {
    const int BC = cfg & 1 ? 128 : 64, NS = cfg & 2 ? 6 : 3;
    if (OC % BC) continue;
    int occ = 163840 / wlds3(BC, NS);
    if (occ > 3) occ = 3;
    if (occ < 1) continue;
    const int slots = wg_slots(occ);
    const long tiles = 3L * (IC / 64) * (OC / BC);
    const double step_us = (BC == 64 ? 0.9 : 1.3) * (NS == 6 ? 0.8 : 1.0);
    const int smax = steps / 4 > 0 ? steps / 4 : 1;
    // split cap 128 (256 until round 6): fewer partial slabs to write and reduce; ResNet-18 bf16
    // -9.5 us twice, ResNet-50 bf16 -24 us, 64 +30 us (profiles/r6_wgrad3_split_cap_ab.jsonl)
    for (int sp = 1; sp <= smax && sp <= 128; ++sp) {
      const int sps = (steps + sp - 1) / sp;
      const int spl = (steps + sps - 1) / sps;
      const long wgs = tiles * spl;
      const long rounds = (wgs + slots - 1) / slots;
      const double t = rounds * (sps * step_us + 3.0) + (spl > 1 ? spl * (double)OC * Kg * 8.0 / 5e6 : 0.0);
      if (t < best_t) {
        best_t = t;
        best = WPlan{0, BC, NS, spl, sps};
      }
    }
  }
  return best;
}

template <int BC, int NS, bool G = false>
int launch_w3(const Wgrad3Args& a, hipStream_t st) {
  hipLaunchKernelGGL((wgrad3_kernel<BC, NS, G>), dim3(3 * a.n_c_tiles * a.n_oc_tiles * a.splits), dim3(256),
                     (size_t)wlds3(BC, NS), st, a);
  return (int)hipGetLastError();
}

// fp32 plan (wgrad2f_kernel): workgroups run in rounds of 256 CUs x k co-resident workgroups
// (k <= the LDS occupancy); a round's length is its workgroups' stages x the f32 MFMA time of a
// stage (BR*BC/4 cycles per wave) x k / eff(k) — a lone wave per SIMD leaves every stage's DMA wait
// and barrier exposed — plus ~1.5 us of prologue / partial-tile store, and the split-K partial
// traffic (written here, read by the reduction) comes on top. Round quantisation dominates: the
// 64-channel 32x32 layer takes 100 us at 84 splits (756 workgroups: one round at k = 3) and 131 us
// at 86 (774: a second round for 6 workgroups). eff measured with scripts/dev/wgf_splits.py:
// 64x64 0.55 / 0.65 / 0.72 at k = 1 / 2 / 3.
WPlan wplanf(int OC, int Kg, int npix) {
  WPlan best{64, 64, 3, 1, 0};
  double best_t = 1e30;
  const int steps = (npix + 31) / 32;
  const int brs[2] = {128, 64}, bcs[2] = {128, 64};
  for (int ib = 0; ib < 2; ++ib)
    for (int ic = 0; ic < 2; ++ic) {
      const int BR = brs[ib], BC = bcs[ic];
      if (Kg % BR || OC % BC) continue;
      const int NS = 3;
      int occ = 163840 / (NS * 32 * (BR + BC) * 4);
      if (occ > 3) occ = 3;
      if (occ < 1) continue;
      const bool sq = BR == 64 && BC == 64;
      const long tiles = (long)(Kg / BR) * (OC / BC);
      const double step_us = (double)(BR * BC) / 4.0 / 2100.0;  // one stage at full f32 MFMA rate
      auto eff = [&](int k) { return sq ? (k <= 1 ? 0.55 : k == 2 ? 0.65 : 0.72) : (k <= 1 ? 0.60 : 0.68); };
      for (int sp = 1; sp <= 256 && sp <= steps; ++sp) {
        const int sps = (steps + sp - 1) / sp;
        const int spl = (steps + sps - 1) / sps;
        if (sp > 1 && spl != sp) continue;
        const long wgs = tiles * spl, full = wgs / (256L * occ), rest = wgs - full * 256L * occ;
        const int krest = (int)((rest + 255) / 256);
        double t = full * (sps * step_us * occ / eff(occ) + 1.5);
        if (rest) t += sps * step_us * krest / eff(krest) + 1.5;
        if (spl > 1) t += spl * (double)OC * Kg * 6.0 / 6e6;  // reduction read + extra store
        if (t < best_t) {
          best_t = t;
          best = WPlan{BR, BC, NS, spl, sps};
        }
      }
    }
  return best;
}

constexpr int wlds3f(int BC, int NS) { return NS * (256 + 32 * 256 + 32 * BC * 4); }

// wgrad3f plan: the wplanf round model with the tap-reuse tile (192 x BC per workgroup, 3 x 64 x
// BC x 32 MACs per stage). eff(k) as measured for the tap-reuse conv mainloops (64-66 % at 2-3
// co-resident workgroups).
WPlan wplan3f(int OC, int IC, int Kg, int npix) {
  WPlan best{0, 64, 3, 1, 0};
  double best_t = 1e30;
  const int steps = npix / 32;
  for (int BC = 64; BC <= 128; BC *= 2) {
    if (OC % BC) continue;
    const int NS = 3;
    int occ = 163840 / wlds3f(BC, NS);
    if (occ > 3) occ = 3;
    const long tiles = 3L * (IC / 64) * (OC / BC);
    const double step_us = 3.0 * 64 * BC / 4.0 / 2100.0;
    auto eff = [&](int k) { return k <= 1 ? 0.55 : k == 2 ? 0.66 : 0.70; };
    for (int sp = 1; sp <= 512 && sp <= steps; ++sp) {
      const int sps = (steps + sp - 1) / sp;
      const int spl = (steps + sps - 1) / sps;
      if (sp > 1 && spl != sp) continue;
      const long wgs = tiles * spl, full = wgs / (256L * occ), rest = wgs - full * 256L * occ;
      const int krest = (int)((rest + 255) / 256);
      double t = full * (sps * step_us * occ / eff(occ) + 1.5);
      if (rest) t += sps * step_us * krest / eff(krest) + 1.5;
      if (spl > 1) t += spl * (double)OC * Kg * 6.0 / 6e6;
      if (t < best_t) {
        best_t = t;
        best = WPlan{0, BC, NS, spl, sps};
      }
    }
  }
  return best;
}

template <int BC>
int launch_w3f(const Wgrad3Args& a, hipStream_t st) {
  hipLaunchKernelGGL((wgrad3f_kernel<BC, 3>), dim3(3 * a.n_c_tiles * a.n_oc_tiles * a.splits), dim3(256),
                     (size_t)wlds3f(BC, 3), st, a);
  return (int)hipGetLastError();
}

template <int BR, int BC>
int launch_w2f(const Wgrad2Args& a, hipStream_t st) {
  const size_t lds = (size_t)3 * 32 * (BR + BC) * 4;
  hipLaunchKernelGGL((wgrad2f_kernel<BR, BC, 3>), dim3(a.n_k_tiles * a.n_oc_tiles * a.splits), dim3(256), lds, st,
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

// Batched TN GEMMs part[b * q + j][K][C] = sum over tiles t in range j of D[b][t][:]^T . X[b][t][:]
// with X [nb][T][C], D [nb][T][K] (the Winograd weight gradient, wino.hip): wgrad2f_kernel as a
// 1x1 weight gradient over nb * T pixels whose split s = b * q + j covers T / q pixels of batch b.
// T % (32 q) == 0; BR | C, BC | K (64 or 128); C a power of two.
int psx_bgemm_tn_f32(const float* X, const float* D, float* part, const void* zero, int T, int C, int K, int nb, int q,
                     int BR, int BC, hipStream_t st) {
  if (q < 1 || T % (32 * q) || C % BR || K % BC || (C & (C - 1)) || (BR != 64 && BR != 128) || (BC != 64 && BC != 128))
    return -2;
  Wgrad2Args a{};
  a.x = X;
  a.dy = D;
  a.part = part;
  a.zero = zero;
  a.IH = a.IW = 1; a.IC = C; a.OC = K; a.R = a.S = 1; a.pad = 0; a.stride = 1;
  a.Kg = C;
  a.log2_icc = ilog2w(C / 4);
  a.npix = nb * T;
  a.div_ohw = make_fastdiv(1);
  a.div_ow = make_fastdiv(1);
  a.div_s = make_fastdiv(1);
  a.n_k_tiles = C / BR;
  a.n_oc_tiles = K / BC;
  a.splits = nb * q;
  a.steps_per_split = T / q / 32;
  if (BR == 128 && BC == 128) return launch_w2f<128, 128>(a, st);
  if (BR == 128) return launch_w2f<128, 64>(a, st);
  if (BC == 128) return launch_w2f<64, 128>(a, st);
  return launch_w2f<64, 64>(a, st);
}

// Returns the split count (query with part == nullptr); partials need splits*OC*Kg floats.
// f32: x / dy are fp32 (wgrad2f_kernel) instead of bf16.
extern "C" int psx_stem7_wgrad(const float* x, const float* dy, float* part, int Nb, int IH, int IW, int cin, int cp,
                               int OC, int Kg, hipStream_t st);

int psx_conv_wgrad2(const void* x, const void* dy, float* part, const void* zero, int Nb, int H, int W, int IC, int OC,
                    int R, int S, int stride, int pad, int Kg, int f32, hipStream_t st) {
  Wgrad2Args a{};
  const int OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  a.x = x;
  a.dy = dy;
  a.part = part;
  a.zero = zero;
  a.IH = H; a.IW = W; a.IC = IC; a.OC = OC; a.R = R; a.S = S; a.pad = pad; a.stride = stride;
  a.Kg = Kg;
  a.log2_icc = ilog2w(IC / 8);
  a.npix = Nb * OH * OW;
  a.div_ohw = make_fastdiv(OH * OW);
  a.div_ow = make_fastdiv(OW);
  a.div_s = make_fastdiv(S);
  if (OC % 64 || Kg % 64) return -2;
  if (f32 && IC == 4 && R == 7 && S == 7 && stride == 2 && pad == 3 && OC == 64 && H == 224 && W == 224) {
    // the ImageNet stem: its own MFMA kernel with the input patch in LDS (stem.hip)
    const int e = psx_stem7_wgrad((const float*)x, (const float*)dy, part, Nb, H, W, 3, 4, OC, Kg, st);
    if (e != -11) return e;
  }
  const bool w3ok = R == 3 && S == 3 && stride == 1 && pad == 1 && IC % 64 == 0;
  if (f32 && w3ok && (W & (W - 1)) == 0 && (H & (H - 1)) == 0 && W <= 32 && W >= 2 && a.npix % 32 == 0 &&
      Kg == 9 * IC) {
    // 3x3 stride-1 layers: fp32 tap-reuse kernel
    WPlan p = wplan3f(OC, IC, Kg, a.npix);
    if (OC % p.BC) return -2;
    if (!part) return p.splits;
    Wgrad3Args b{};
    b.x = (const uint16_t*)x; b.dy = (const uint16_t*)dy; b.part = part; b.zero = (const uint16_t*)zero;
    b.H = H; b.W = W; b.log2w = ilog2w(W); b.IC = IC; b.OC = OC; b.Kg = Kg; b.npix = a.npix;
    b.n_c_tiles = IC / 64; b.n_oc_tiles = OC / p.BC; b.splits = p.splits; b.steps_per_split = p.sps;
    b.pix = 32;
    const int e = p.BC == 128 ? launch_w3f<128>(b, st) : launch_w3f<64>(b, st);
    return e ? -e : p.splits;
  }
  if (f32) {
    a.log2_icc = ilog2w(IC / 4);
    if (IC % 4 || (IC & (IC - 1))) return -2;
    WPlan p = wplanf(OC, Kg, a.npix);
    if (Kg % p.BR || OC % p.BC) return -2;
    a.n_k_tiles = Kg / p.BR;
    a.n_oc_tiles = OC / p.BC;
    a.splits = p.splits;
    a.steps_per_split = p.sps;
    if (!part) return p.splits;
    int e;
    if (p.BR == 128 && p.BC == 128) e = launch_w2f<128, 128>(a, st);
    else if (p.BR == 128) e = launch_w2f<128, 64>(a, st);
    else if (p.BC == 128) e = launch_w2f<64, 128>(a, st);
    else e = launch_w2f<64, 64>(a, st);
    return e ? -e : p.splits;
  }
  // 3x3 stride-1 layers, tap-reuse kernel: power-of-two rows (64-pixel
  // steps), or widths dividing 56 (ResNet-50: 56-pixel steps of whole rows, G)
  const bool pow2 = (W & (W - 1)) == 0 && (H & (H - 1)) == 0 && W <= 64 && W >= 2 && a.npix % 64 == 0;
  const bool gen = !pow2 && W >= 2 && 56 % W == 0 && a.npix % 56 == 0;
  if (w3ok && (pow2 || gen)) {
    const int pix = pow2 ? 64 : 56;
    WPlan p = wplan3(OC, IC, Kg, a.npix, pix);
    if (OC % p.BC) return -2;
    if (!part) return p.splits;
    Wgrad3Args b{};
    b.x = (const uint16_t*)a.x; b.dy = (const uint16_t*)a.dy; b.part = part; b.zero = (const uint16_t*)a.zero;
    b.H = H; b.W = W; b.log2w = ilog2w(W); b.IC = IC; b.OC = OC; b.Kg = Kg; b.npix = a.npix;
    b.n_c_tiles = IC / 64; b.n_oc_tiles = OC / p.BC; b.splits = p.splits; b.steps_per_split = p.sps;
    b.pix = pix;
    b.div_w = make_fastdiv(W);
    b.div_h = make_fastdiv(H);
    int e;
    if (pow2)
      e = p.BC == 128 ? (p.NS == 6 ? launch_w3<128, 6>(b, st) : launch_w3<128, 3>(b, st))
                      : (p.NS == 6 ? launch_w3<64, 6>(b, st) : launch_w3<64, 3>(b, st));
    else
      e = p.BC == 128 ? (p.NS == 6 ? launch_w3<128, 6, true>(b, st) : launch_w3<128, 3, true>(b, st))
                      : (p.NS == 6 ? launch_w3<64, 6, true>(b, st) : launch_w3<64, 3, true>(b, st));
    return e ? -e : p.splits;
  }
  // Tile: the round-5 sweep (bench/r50_wgrad_tiles.py, profiles/r5_r50_wgrad_tiles.jsonl, ResNet-50's
  // 1x1 layers): 64 (k) x 128 (oc) wins by 10-20 % on every layer up to 28x28 with OC % 128 == 0
  // (128x512x28 42.0 -> 34.7 us, 1024x2048x14/s2 64.3 -> 55.4), 64x64 on the 56x56 ones (the
  // model's choice there).
  const bool t128 = OC % 128 == 0 && Kg % 64 == 0 && a.npix <= 128 * 28 * 28;
  WPlan p = t128 ? wplan(OC, Kg, a.npix, 64, 128) : wplan(OC, Kg, a.npix);
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
