// Fused fp32 Winograd F(3x3,4x4) weight gradient: input transform, dy transform and the 36
// tile-reduction GEMMs in ONE launch (+ the small output-transform launch psx_wino_wout).
//
// The three-launch path (wino.hip psx_wino_wgrad) writes D = A dy A^T (36 x T x K floats, 2.25x
// dy: 75 MB per ResNet-18 32x32x64 conv at B = 128) and re-reads it together with the forward's
// stored V = B^T x B (another 75 MB, written by the forward only for this consumer). Here every
// lane transforms its own tile in registers straight from x and dy, so neither D nor V exists:
// the launch reads x (or the pre-BN y with the BN + ReLU of the forward folded into the load)
// and dy (or dz with the BN-backward apply folded in) once, and writes only the q partial slabs
// the output transform reduces.
//
// Mapping onto v_mfma_f32_16x16x4f32 (exact f32). For one Winograd point b = (r, s) the GEMM is
//   M[b][k][c] = sum_t D[b][t][k] * V[b][t][c]       (t over the tiles of the batch)
// A 16 (k) x 4 (t) operand and a 4 (t) x 16 (c) operand per MFMA: lane l supplies A[k = l & 15][t =
// l >> 4] and B[t = l >> 4][c = l & 15], i.e. lane l owns TILE l >> 4 of a group of four and
// CHANNEL l & 15 — and computes that tile's complete 6x6 transforms for its channel, D for channel
// k0 + (l & 15) of dy and V for channel c0 + (l & 15) of x. No LDS, no exchange: 36 MFMAs (one per
// point, 36 independent accumulators, never a dependent chain) per group of four tiles.
//   workgroup = 4 waves on one 16 (k) x 16 (c) output block; the waves take alternate tile
//               groups of the workgroup's tile range; at the end the four waves' 36 x 16 x 16
//               partial sums are added through LDS (9 points at a time) in fixed order and the
//               workgroup writes one partial slab part[b * q + range][k][c]
//   grid      = (K/16)(C/16) blocks x q tile ranges, XCD-remapped so that one XCD runs every
//               block of a few tile ranges (they share the same x / dy lines in its L2)
// Per group and wave: 52 loads + ~400 VALU (both transforms, the folds, the padding masks) beside
// 36 MFMAs x 32 cycles; two waves per SIMD overlap one's transforms with the other's MFMAs.
// Numerics: fp32 transforms and fp32 MFMA accumulation, fixed summation order (deterministic).
#include <stdlib.h>

#include "bnfin.hpp"
#include "common.hpp"
#include "wino.hpp"

extern "C" int psx_wino_wout(const float* part, void* out, int out_fp16, float scale, int K, int C, int q,
                             hipStream_t st);

namespace psx {

struct WinoWgradArgs {
  const float* x;      // [N][H][W][C]: the conv input, or (xaff) the pre-BN output y of the previous BN
  const float* xaff;   // nullable [2][C]: x operand = relu(scale * y + shift), zero padding after it
  const float* dy;     // [N][H][W][K]: the output gradient, or (bpart) dz of the BN behind the conv
  const float* ybn;    // bpart: that BN's input (its backward apply dy = k1 dz + k2 ybn + k3)
  const float* bpart;  // nullable: slot sums [PSX_STAT_SLOTS][2][K] of that BN's backward (wino.hpp)
  BnBwdFin bfin;
  float* part;         // [36 * q][K][C]
  int H, W, C, K, T, q, tpr;  // tpr = tiles per range = T / q
  int xbytes, ybytes;         // N H W C * 4, N H W K * 4 (< 2^30)
};

// PSX_WGF_PF = 1: the next tile group's 52 (BWD: 68) loads are issued before the current group's
// transforms and MFMAs (one wave per SIMD: the accumulators move to AGPRs); 0 (default): load,
// then compute, two waves per SIMD hiding each other's load latency. Same box, B = 128, us incl.
// the output transform (bench/wino_wgrad_ab.py): 32x32x64 82.8 vs 58.4, 16x16x128 72.1 vs 55.3,
// 8x8x256 73.2 vs 53.7, 4x4x512 85.8 vs 61.7 — one wave per SIMD cannot overlap its own
// transforms with its MFMAs.
#ifndef PSX_WGF_PF
#define PSX_WGF_PF 0
#endif

// one axis of B^T d with explicit FMAs (the file is built without FP contraction, so every
// template instance rounds identically: the folded and unfolded paths give the same bits)
PSX_DEV void bt6f(const float (&d)[6], float (&r)[6]) {
  r[0] = fmaf(4.f, d[0], fmaf(-5.f, d[2], d[4]));
  r[1] = fmaf(-4.f, d[1] + d[2], d[3] + d[4]);
  r[2] = fmaf(4.f, d[1] - d[2], d[4] - d[3]);
  r[3] = fmaf(2.f, d[3] - d[1], d[4] - d[2]);
  r[4] = fmaf(2.f, d[1] - d[3], d[4] - d[2]);
  r[5] = fmaf(4.f, d[1], fmaf(-5.f, d[3], d[5]));
}

PSX_DEV void a4f(const float (&y)[4], float (&r)[6]) {
  const float e = y[0] + y[2], o = y[1] + y[3], e4 = fmaf(4.f, y[2], y[0]), o2 = fmaf(8.f, y[3], 2.f * y[1]);
  r[0] = y[0];
  r[1] = e + o;
  r[2] = e - o;
  r[3] = e4 + o2;
  r[4] = e4 - o2;
  r[5] = y[3];
}

template <bool BWD>
struct WgfRaw {  // one tile group's loads, per lane (its tile, its channel)
  float x[6][6];
  float y[4][4];
  float yb[BWD ? 4 : 1][BWD ? 4 : 1];
  bool r0, r5, c0, c5;  // the patch's first / last row / column inside the image
};

template <bool AFF, bool BWD>
__global__ __launch_bounds__(256, PSX_WGF_PF ? 1 : 2) void wino_wgrad_fused_kernel(WinoWgradArgs a) {
  __shared__ float red[4][9][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nkb = a.K >> 4, nblk = nkb * (a.C >> 4);
  // logical id = range-major: an XCD gets consecutive ranges' blocks (same x / dy lines)
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int range = lid / nblk, blk = lid - range * nblk;
  const int kb = blk % nkb, cb = blk / nkb;
  const int ch = lane & 15, tl = lane >> 4;
  const int k = kb * 16 + ch, c = cb * 16 + ch;
  const int H = a.H, W = a.W, C = a.C, K = a.K;
  const int tw = W >> 2, tpi = (H >> 2) * tw;

  float sc = 1.f, sh = 0.f;
  if constexpr (AFF) {
    sc = a.xaff[c];
    sh = a.xaff[C + c];
  }
  float k1 = 1.f, k2 = 0.f, k3 = 0.f;
  if constexpr (BWD) {
    double sdz, sxh;
    wino_bwd_coef(a.bpart, a.bfin, k, k1, k2, k3, sdz, sxh);
  }

  f32x4 acc[36];
#pragma unroll
  for (int b = 0; b < 36; ++b) acc[b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // buffer descriptors: x loads use per-element offsets whose padding rows / columns carry kBad
  // (past the buffer: the load returns 0, no mask, no 64-bit address math); the dy tile never
  // pads, so its 16 loads are one per-lane base + 16 wave-uniform offsets
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, a.xbytes, 0x00020000);
  const auto dr_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dy), 0, a.ybytes, 0x00020000);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.ybn), 0, BWD ? a.ybytes : 0, 0x00020000);
  constexpr unsigned kBad = 0x40000000u;  // > any tensor's bytes; kBad + kBad + offset still > them
  const unsigned rowb = (unsigned)W * C * 4, colb = (unsigned)C * 4;
  const int t0 = range * a.tpr;

  auto load = [&](int g, WgfRaw<BWD>& R) {
    const int t = t0 + g + tl;
    const int n = t / tpi, rem = t - n * tpi, ti = rem / tw, tj = rem - ti * tw;
    // x patch (6x6 at (4 ti - 1, 4 tj - 1), zero padded) of channel c: only rows / columns 0 and
    // 5 can fall outside the image
    const int h0 = 4 * ti - 1, w0 = 4 * tj - 1;
    R.r0 = h0 >= 0;
    R.r5 = h0 + 5 < H;
    R.c0 = w0 >= 0;
    R.c5 = w0 + 5 < W;
    unsigned ro[6], co[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const bool oh = i == 0 ? R.r0 : (i == 5 ? R.r5 : true), ow = i == 0 ? R.c0 : (i == 5 ? R.c5 : true);
      ro[i] = oh ? (unsigned)(n * H + h0 + i) * rowb + (unsigned)c * 4 : kBad;
      co[i] = ow ? (unsigned)(w0 + i) * colb : kBad;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j)
        R.x[i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, ro[i] + co[j], 0, 0));
    // dy tile (4x4 at (4 ti, 4 tj)) of channel k
    const unsigned yo = (unsigned)(((n * H + 4 * ti) * W + 4 * tj) * K + k) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int so = (i * W + j) * K * 4;  // wave-uniform
        R.y[i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(dr_, yo, so, 0));
        if constexpr (BWD) R.yb[i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yr, yo, so, 0));
      }
  };

  auto compute = [&](const WgfRaw<BWD>& R) {
    // column transforms: tb[r][j] = (B^T d)[r][j], u[r][j] = (A y)[r][j]
    float tb[6][6], u[6][4];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float col[6], o[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        float v = R.x[i][j];
        if constexpr (AFF) {  // zero padding stays zero after BN + ReLU (border elements only);
          // fmaf = the BN apply's contracted y * scale + shift: the operand is bit-identical to
          // the activation the unfolded path writes
          const float e = fmaxf(fmaf(v, sc, sh), 0.f);
          const bool oh = i == 0 ? R.r0 : (i == 5 ? R.r5 : true), ow = j == 0 ? R.c0 : (j == 5 ? R.c5 : true);
          v = (oh && ow) ? e : 0.f;
        }
        col[i] = v;
      }
      bt6f(col, o);
#pragma unroll
      for (int r = 0; r < 6; ++r) tb[r][j] = o[r];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float col[4], o[6];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (BWD)
          col[i] = wino_bwd_apply(R.y[i][j], R.yb[i][j], k1, k2, k3);
        else
          col[i] = R.y[i][j];
      }
      a4f(col, o);
#pragma unroll
      for (int r = 0; r < 6; ++r) u[r][j] = o[r];
    }
    // row r: V[r][s] = (tb B)[r][s], D[r][s] = (u A^T)[r][s]; one MFMA per point (r, s)
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      float vr[6], dr[6];
      bt6f(tb[r], vr);
      a4f(u[r], dr);
#pragma unroll
      for (int s = 0; s < 6; ++s)
        acc[r * 6 + s] = __builtin_amdgcn_mfma_f32_16x16x4f32(dr[s], vr[s], acc[r * 6 + s], 0, 0, 0);
    }
  };

#if PSX_WGF_PF
  WgfRaw<BWD> cur;
  int g = wv * 4;
  if (g < a.tpr) load(g, cur);
  for (; g < a.tpr; g += 16) {
    WgfRaw<BWD> nxt;
    const bool more = g + 16 < a.tpr;
    if (more) load(g + 16, nxt);
    compute(cur);
    if (more) cur = nxt;  // register moves (a two-set ping-pong unrolled into spills)
  }
#else#else
  for (int g = wv * 4; g < a.tpr; g += 16) {
    WgfRaw<BWD> cur;
    load(g, cur);
    compute(cur);
  }
#endif

  // the four waves' partial sums, 9 points at a time, added in wave order; lane l holds
  // M[b][k = 4 (l >> 4) + j][c = l & 15] in acc[b][j]
  float* out = a.part + ((size_t)range * K + kb * 16) * C + cb * 16;
  const size_t bstride = (size_t)a.q * K * C;
  const int ok_ = threadIdx.x >> 4, oc_ = threadIdx.x & 15;
#pragma unroll
  for (int c9 = 0; c9 < 4; ++c9) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wv][i][(4 * tl + j) * 16 + ch] = acc[c9 * 9 + i][j];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const float v = ((red[0][i][threadIdx.x] + red[1][i][threadIdx.x]) + red[2][i][threadIdx.x]) + red[3][i][threadIdx.x];
      out[(size_t)(c9 * 9 + i) * bstride + (size_t)ok_ * C + oc_] = v;
    }
    __syncthreads();
  }
}

}  // namespace psx

using namespace psx;

extern "C" {

// Tile ranges q of the fused weight gradient (0: not applicable): ~512 workgroups, ranges of
// whole groups of 16 tiles (four per wave) and >= 64 tiles.
int psx_wino_wgrad_fused_q(int N, int H, int W, int C, int K) {
  if (H % 4 || W % 4 || C % 16 || K % 16 || C < 16 || K < 16) return 0;
  const int T = N * (H / 4) * (W / 4);
  if (T % 16) return 0;
  const long nblk = (long)(K / 16) * (C / 16);
  int q = 1;
  while (nblk * q * 2 <= 512 && T % (16 * q * 2) == 0 && T / (q * 2) >= 64) q *= 2;
  return (T % (16 * q) == 0 && nblk * q < (1L << 30)) ? q : 0;
}

// Weight gradient of a 3x3 / stride-1 / pad-1 fp32 conv (Winograd F(3x3,4x4), fused: see the
// header). x [N][H][W][C] (xaff nullable [2][C]: x = relu(scale y + shift) of the stored pre-BN y),
// dy [N][H][W][K] (ybn / bpart / bbfin nullable: dy = k1 dz + k2 ybn + k3 of the stored dz, as
// wino.hip psx_wino_wgrad). part: 36 * q * K * C floats (q = psx_wino_wgrad_fused_q). out: OIHW
// gradient, fp16 (out_fp16: the wire) or fp32, times scale.
int psx_wino_wgrad_fused(const float* x, const float* xaff, const float* dy, const float* ybn, const float* bpart,
                         const BnBwdFin* bbfin, float* part, void* out, int out_fp16, float scale, int N, int H, int W,
                         int C, int K, hipStream_t st) {
  const int q = psx_wino_wgrad_fused_q(N, H, W, C, K);
  if (q < 1) return -2;
  if (bpart && (!ybn || !bbfin || bbfin->C != K)) return -3;
  WinoWgradArgs a{};
  a.x = x;
  a.xaff = xaff;
  a.dy = dy;
  a.ybn = ybn;
  a.bpart = bpart;
  if (bpart) a.bfin = *bbfin;
  a.bfin.det = (int)det_enabled();
  a.part = part;
  a.H = H;
  a.W = W;
  a.C = C;
  a.K = K;
  a.T = N * (H / 4) * (W / 4);
  a.q = q;
  a.tpr = a.T / q;
  const long xb = (long)N * H * W * C * 4, yb = (long)N * H * W * K * 4;
  if (xb >= (1L << 30) || yb >= (1L << 30)) return -4;  // 32-bit buffer offsets (kernel kBad)
  a.xbytes = (int)xb;
  a.ybytes = (int)yb;
  const unsigned nwg = (unsigned)((K / 16) * (C / 16) * q);
  using Kern = void (*)(WinoWgradArgs);
  static const Kern kk[2][2] = {{wino_wgrad_fused_kernel<false, false>, wino_wgrad_fused_kernel<false, true>},
                                {wino_wgrad_fused_kernel<true, false>, wino_wgrad_fused_kernel<true, true>}};
  hipLaunchKernelGGL(kk[xaff != nullptr][bpart != nullptr], dim3(nwg), dim3(256), 0, st, a);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return (int)e;
  return psx_wino_wout(part, out, out_fp16, scale, K, C, q, st);
}

}  // extern "C"
