// fp32 Winograd F(4x4, 3x3) convolution for the small-image 3x3 / stride-1 / pad-1 layers
// (ResNet-18 CIFAR stages 2-4: 16x16x128, 8x8x256 and 4x4x512, forward and data gradient).
// Same-box per layer (B=128, us fwd / dgrad, direct -> Winograd incl. transforms): 16x16 85/82 ->
// 54/54, 8x8 86/84 -> 44/44, 4x4 91/89 -> 46/45; 32x32x64 ties (98 vs 98: its transformed
// operands, 75 MB each, make the transforms the cost), so it stays direct.
//
// Why: on those layers the direct implicit GEMM is MFMA-bound at fp32 (v_mfma_f32_16x16x4_f32,
// 1/16 of the bf16 rate) while the activations are small (8.4 / 4.2 MB at B=128), so trading
// multiplies for transform traffic pays: F(4x4,3x3) does 36 products per 16 outputs instead of
// 144 (4x fewer MFMA flops) for ~2.25x the activation bytes in the transformed domain. The
// arithmetic stays fp32 end to end (transforms, MFMA operands, fp32 accumulation): relative
// error vs an fp64 reference ~3e-6 (direct fp32: ~2e-7) — the algorithm MIOpen / cuDNN pick for
// fp32 3x3 convolutions. PSX_TUNE wino=0 (engine) keeps the direct kernels.
//
// Layouts (T = N * (H/4) * (W/4) output tiles, tile t = (n, ti, tj)):
//   V [36][T][C]   input tiles d (6x6 window at (4ti-1, 4tj-1), zero padded) -> B^T d B
//   U [K][36][C]   weights g (3x3) -> G g G^T           (dgrad: U'[C][36][K] of rot180(g)^T)
//   P [36][T][K]   36 independent GEMMs P[b] = V[b] . U[:, b, :]^T, run as ONE launch of the
//                  conv_v2 LDS-DMA mainloop (an implicit GEMM over T pixels whose 36 "taps" are
//                  the batches, split-K into 36 slabs of C = exactly the 36 batches; psx_bgemm_f32)
//   y [N][H][W][K] A^T P A per tile (+ residual) and the BN partial sums of y (slot rows, as the
//                  conv epilogue writes them)
// Weight gradient (F(3x3,4x4) by transposition: dg = G^T [sum_t (A dy_t A^T) . V_t] G):
//   D [36][T][K]   dy tiles -> A dy A^T
//   M [36][K][C]   M[b] = D[b]^T . V[b]: 36 TN GEMMs reduced over the T tiles, ONE launch of the
//                  fp32 weight-gradient mainloop (wgrad2f_kernel as a 1x1 wgrad over 36*T pixels
//                  whose split s covers exactly batch s (x q tile ranges); psx_bgemm_tn_f32)
//   dW [K][C][3][3] G^T M G straight into the gradient wire (fp16 codec or fp32)
// Matrices (points 0, +-1, +-2, inf; checked against torch float64 in tests/test_wino_gpu.py):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
#include <stdlib.h>

#include "bnfin.hpp"
#include "common.hpp"
#include "wino.hpp"

extern "C" int psx_bgemm_f32_split(const float* A, const float* B, float* P, const void* zero, int M, int N, int Kd,
                                   int nb, int s2, int cfg, hipStream_t st);
extern "C" int psx_wino_wout(const float* part, void* out, int out_fp16, float scale, int K, int C, int q,
                             hipStream_t st);
extern "C" int psx_bgemm_tn_f32(const float* X, const float* D, float* part, const void* zero, int T, int C, int K,
                                int nb, int q, int BR, int BC, hipStream_t st);

namespace psx {

__constant__ float kWinoG[6][3] = {{0.25f, 0.f, 0.f},
                                   {-1.f / 6.f, -1.f / 6.f, -1.f / 6.f},
                                   {-1.f / 6.f, 1.f / 6.f, -1.f / 6.f},
                                   {1.f / 24.f, 1.f / 12.f, 1.f / 6.f},
                                   {1.f / 24.f, -1.f / 12.f, 1.f / 6.f},
                                   {0.f, 0.f, 1.f}};

// the 36 transformed weights (G g G^T) of one 3x3 kernel, rounding pinned by explicit FMAs so
// every transform kernel produces the same bits
PSX_DEV void wino_g36(const float (&gg)[3][3], float (&v)[36]) {
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float gr[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) gr[q] = fmaf(kWinoG[r][0], gg[0][q], fmaf(kWinoG[r][1], gg[1][q], kWinoG[r][2] * gg[2][q]));
#pragma unroll
    for (int s = 0; s < 6; ++s) v[r * 6 + s] = fmaf(kWinoG[s][0], gr[0], fmaf(kWinoG[s][1], gr[1], kWinoG[s][2] * gr[2]));
  }
}

// U[row][b][col] = (G g G^T)[b], g = w[k][c] (fwd: row k, col c) or rot180(w[k][c]) (dgrad: row
// c, col k). One thread per (row, col) pair — every weight read once — col fastest (each of its
// 36 stores is a coalesced 256-byte wave row), 64-thread workgroups so a 128-channel layer still
// spreads over 256 CUs. Measured alternatives (B=128 per-layer bench, fwd + flipped pair, 512
// channels): a thread per (pair, output row) 45.6 us (6 scattered re-reads of every weight in the
// flipped case), a thread per output element 225 us; this one 22.8 us.
__global__ __launch_bounds__(64) void wino_w_kernel(const float* __restrict__ w, float* __restrict__ U, int K, int C,
                                                    int flip) {
  const int rows = flip ? C : K, cols = flip ? K : C;
  const long i = (long)blockIdx.x * 64 + threadIdx.x;
  if (i >= (long)rows * cols) return;
  const int row = (int)(i / cols), col = (int)(i - (long)row * cols);
  const int k = flip ? col : row, c = flip ? row : col;
  const float* g = w + ((size_t)k * C + c) * 9;
  float gg[3][3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int q = 0; q < 3; ++q) gg[p][q] = flip ? g[(2 - p) * 3 + (2 - q)] : g[p * 3 + q];
  float* dst = U + (size_t)row * 36 * cols + col;
  float v[36];
  wino_g36(gg, v);
#pragma unroll
  for (int b = 0; b < 36; ++b) dst[(size_t)b * cols] = v[b];
}

// All layers' weight transforms of a step in one launch: descriptor j covers pairs
// [p0_j, p0_{j+1}) of layer j's (row, col) grid (the per-layer launches were ~6 us each, mostly
// launch and tail latency: 26 per ResNet-18 step).
struct WinoWDesc {
  const float* w;
  float* U;
  int K, C, flip, layout;
  long p0;
};
constexpr int kWinoWMax = 40;
struct WinoWBatch {
  WinoWDesc d[kWinoWMax];
  int n;
  long total;
};

__global__ __launch_bounds__(64) void wino_w_multi_kernel(WinoWBatch bt) {
  const long i = (long)blockIdx.x * 64 + threadIdx.x;
  if (i >= bt.total) return;
  int j = 0;
  while (j + 1 < bt.n && i >= bt.d[j + 1].p0) ++j;
  const WinoWDesc& d = bt.d[j];
  const int flip = d.flip, K = d.K, C = d.C;
  const int cols = flip ? K : C;
  const long li = i - d.p0;
  // layout 0: U[row][36][col] (the batched GEMM's operand), thread = (row, col), col fastest;
  // 1: the fused kernel's MFMA B-operand order (wino_fused.hip): [row/16][col/4][slot 10][lane =
  // (col%4)*16 + row%16][4], slot 5h + i (i < 4) = points 18h + 4i .. +3, slot 5h + 4 = points
  // 18h + 16, 18h + 17 and two zeros; thread = destination lane, so each slot is one coalesced
  // 16-byte store per thread (the (row, col) order scattered every store: 90 us per step)
  int row, col;
  if (d.layout) {
    const int ln = (int)(li & 63);
    const long blk = li >> 6;
    const int cq = cols >> 2;
    const int rg = (int)(blk / cq), cs = (int)(blk - (long)rg * cq);
    row = rg * 16 + (ln & 15);
    col = cs * 4 + (ln >> 4);
  } else {
    row = (int)(li / cols);
    col = (int)(li - (long)row * cols);
  }
  const int k = flip ? col : row, c = flip ? row : col;
  const float* g = d.w + ((size_t)k * C + c) * 9;
  float gg[3][3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int q = 0; q < 3; ++q) gg[p][q] = flip ? g[(2 - p) * 3 + (2 - q)] : g[p * 3 + q];
  float v[36];
  wino_g36(gg, v);
  if (d.layout) {
    f32x4* dst = reinterpret_cast<f32x4*>(d.U) + (li >> 6) * 640 + (li & 63);
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int b = 18 * hb + 4 * q;
        dst[(5 * hb + q) * 64] = (f32x4){v[b], v[b + 1], v[b + 2], v[b + 3]};
      }
      dst[(5 * hb + 4) * 64] = (f32x4){v[18 * hb + 16], v[18 * hb + 17], 0.f, 0.f};
    }
  } else {
    float* dst = d.U + (size_t)row * 36 * cols + col;
#pragma unroll
    for (int b = 0; b < 36; ++b) dst[(size_t)b * cols] = v[b];
  }
}

// ---- Transforms: one tile per 6-wave workgroup iteration, one transform row per wave ----
// (A thread per whole tile — 36 loads + 36 stores of one (tile, channel) — left the 4x4 / 8x8
// layers at 1-4 waves per CU, each one long dependent chain, at 2-4x their byte time; that form
// was removed in round 5.) Here a workgroup = 64 channels x 6 waves takes a tile per
// iteration: wave r loads row r of the tile (6 loads), applies the row transform, hands the 6
// results over LDS (double-buffered: one barrier per tile), and wave s then applies the column
// transform to column s and stores it (6 stores). 6x the waves, 1/6 of the chain per wave, the
// next tile's row prefetched behind the current tile's transform.
constexpr int kXfWaves = 6;

// grid.y of the split kernels: ~4 workgroups per CU over the channel blocks, at most a tile each
// (8 per CU until round 6: each workgroup also adds one set of BN partial sums, and 1024 vs 2048
// workgroups measured ResNet-18 fp32 3.277 -> 3.257 ms, ResNet-50 35.50 -> 35.47; 512 the same
// as 1024, 256 +2 %, 4096 neutral: profiles/r6_wino_xf_grid_ab.jsonl)
int wino_xf_grid(int T, int cblocks) {
  int gy = 1024 / cblocks;
  if (gy < 1) gy = 1;
  return gy > T ? T : gy;
}

// V[b][t][c] = B^T d B of the 6x6 input window of tile t (zero padded).
// bnpart (nullable): x is the PRE-BatchNorm conv output z of the previous layer, and the operand
// is relu(BN(z)) — the training-mode BN finalize (batch statistics from the slot rows
// bnpart[slot][2][C], as bnfin.hpp bn_fin_lds computes them) and the BN + ReLU apply are folded
// into this load, so the activation relu(BN(z)) is never written. The workgroups of tile row 0
// publish the affine, saved statistics and running statistics of their channels.
__global__ __launch_bounds__(384) void wino_in_xf_kernel(const float* __restrict__ x, float* __restrict__ V, int T,
                                                         int H, int W, int C, const float* __restrict__ bnpart,
                                                         WinoBnFin fin) {
  __shared__ float xf[2][6][6][64];
  __shared__ float aff[2][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int tw = (W + 3) >> 2, tpi = ((H + 3) >> 2) * tw;  // partial edge tiles
  const size_t bs = (size_t)T * C;
  auto load = [&](int t, float (&d)[6], unsigned& okc, bool& okr) {
    const int n = t / tpi, rem = t - n * tpi, ti = rem / tw, tj = rem - ti * tw;
    const int h = 4 * ti - 1 + wv, w0 = 4 * tj - 1;
    okr = (unsigned)h < (unsigned)H;
    okc = 0;
    const float* xr = x + ((size_t)n * H + (okr ? h : 0)) * W * C + c;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const bool ok = (unsigned)(w0 + s) < (unsigned)W;
      okc |= (unsigned)ok << s;
      d[s] = xr[(size_t)(ok ? w0 + s : 0) * C];  // unconditional (zeroed below when padding)
    }
  };
  int t = blockIdx.y;
  float d[6];
  unsigned okc = 0;
  bool okr = false;
  if (t < T) load(t, d, okc, okr);
  float sc = 1.f, sh = 0.f;
  if (bnpart) {
    if (wv == 0) {  // BN finalize of the workgroup's 64 channels
      const double s = slot_sum<PSX_STAT_SLOTS>(bnpart, c, 2 * (size_t)C, fin.det);
      const double ss = slot_sum<PSX_STAT_SLOTS>(bnpart, (size_t)C + c, 2 * (size_t)C, fin.det);
      double mean, var;
      bn_moments(s, ss, fin.count, fin.sshift ? fin.sshift[c] : 0.f, mean, var);
      const float invstd = (float)(1.0 / sqrt(var + (double)fin.eps));
      const float a = fin.gamma[c] * invstd, b = fin.beta[c] - (float)mean * a;
      aff[0][lane] = a;
      aff[1][lane] = b;
      if (blockIdx.y == 0) {
        fin.scale[c] = a;
        fin.shift[c] = b;
        fin.save_mean[c] = (float)mean;
        fin.save_invstd[c] = invstd;
        if (fin.sshift_next) fin.sshift_next[c] = (float)mean;
        if (fin.run_mean) {
          const double unb = fin.count > 1.f ? var * fin.count / (fin.count - 1.0) : var;
          fin.run_mean[c] = (1.f - fin.momentum) * fin.run_mean[c] + fin.momentum * (float)mean;
          fin.run_var[c] = (1.f - fin.momentum) * fin.run_var[c] + fin.momentum * (float)unb;
        }
      }
    }
    __syncthreads();
    sc = aff[0][lane];
    sh = aff[1][lane];
  }
  for (int p = 0; t < T; t += gridDim.y, p ^= 1) {
    float cur[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const float v = bnpart ? fmaxf(d[s] * sc + sh, 0.f) : d[s];
      cur[s] = (okr && ((okc >> s) & 1u)) ? v : 0.f;  // zero padding stays zero after BN + ReLU
    }
    const int tn = t + gridDim.y;
    if (tn < T) load(tn, d, okc, okr);
    float e[6];  // row wv of d B
    wino_bt6(cur, e);
#pragma unroll
    for (int s = 0; s < 6; ++s) xf[p][wv][s][lane] = e[s];
    __syncthreads();
    float col[6], o[6];  // column wv of (d B): B^T applied
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = xf[p][r][wv][lane];
    wino_bt6(col, o);
    float* vt = V + (size_t)t * C + c;
#pragma unroll
    for (int r = 0; r < 6; ++r) vt[(r * 6 + wv) * bs] = o[r];
  }
}

// Weight gradient, dy side: D[b][t][k] = (A dy_t A^T)[b] for the 4x4 output tile dy_t
// (A = (A^T)^T, 6x4): waves 0-3 load the 4 rows of the dy tile
// ybn / bpart (nullable): dy is the BN backward k1 dz + k2 ybn + k3 of dz (the dy argument) —
// the BN-backward apply folded in (wino.hpp wino_bwd_coef: the same coefficients and rounding as
// the fused data gradient that consumes the same dy)
__global__ __launch_bounds__(384) void wino_dy_xf_kernel(const float* __restrict__ dy, float* __restrict__ D, int T,
                                                         int H, int W, int K, const float* __restrict__ ybn,
                                                         const float* __restrict__ bpart, BnBwdFin bfin) {
  __shared__ float xf[2][4][6][64];
  __shared__ float kc[3][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int tw = (W + 3) >> 2, tpi = ((H + 3) >> 2) * tw;  // partial edge tiles
  const size_t bs = (size_t)T * K;
  float k1 = 1.f, k2 = 0.f, k3 = 0.f;
  if (bpart) {
    if (wv == 0) {
      double sdz, sxh;
      wino_bwd_coef(bpart, bfin, k, k1, k2, k3, sdz, sxh);
      kc[0][lane] = k1;
      kc[1][lane] = k2;
      kc[2][lane] = k3;
    }
    __syncthreads();
    k1 = kc[0][lane];
    k2 = kc[1][lane];
    k3 = kc[2][lane];
  }
  auto load = [&](int t, float (&y)[4]) {
    const int n = t / tpi, rem = t - n * tpi, ti = rem / tw, tj = rem - ti * tw;
    // partial edge tiles: row 4 ti + wv / columns 4 tj + j outside the image are zero dy (after
    // the BN-backward fold too: its k3 would make them non-zero); their loads read in bounds
    const bool rok = 4 * ti + wv < H;
    const int vj = min(4, W - 4 * tj);
    const size_t off = (((size_t)n * H + (rok ? 4 * ti + wv : 4 * ti)) * W + 4 * tj) * K + k;
    const float* src = dy + off;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = src[(size_t)(j < vj ? j : 0) * K];
    if (bpart) {
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = wino_bwd_apply(y[j], ybn[off + (size_t)(j < vj ? j : 0) * K], k1, k2, k3);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = (rok && j < vj) ? y[j] : 0.f;
  };
  int t = blockIdx.y;
  float y[4];
  if (t < T && wv < 4) load(t, y);
  for (int p = 0; t < T; t += gridDim.y, p ^= 1) {
    if (wv < 4) {
      float cur[4] = {y[0], y[1], y[2], y[3]}, e[6];
      const int tn = t + gridDim.y;
      if (tn < T) load(tn, y);
      wino_a4(cur, e);  // row wv of dy A^T
#pragma unroll
      for (int s = 0; s < 6; ++s) xf[p][wv][s][lane] = e[s];
    }
    __syncthreads();
    float col[4] = {xf[p][0][wv][lane], xf[p][1][wv][lane], xf[p][2][wv][lane], xf[p][3][wv][lane]}, o[6];
    wino_a4(col, o);
    float* dt = D + (size_t)t * K + k;
#pragma unroll
    for (int r = 0; r < 6; ++r) dt[(r * 6 + wv) * bs] = o[r];
  }
}

// y = A^T P A (+ res); forward: BN partial sums (sum y - k, (y - k)^2) of the stored values into
// slot rows stats[slot][2][K]; data gradient (bs.part): the BN-backward sums of the consumer BN
// instead (what the direct dgrad epilogue fuses). Wave r loads row r of the 6x6 tile and applies
// A^T to it; waves 0-3 then each finish output column j (pixels (i, j), i = 0..3) with its
// epilogue. Deterministic mode (det.fix): the sums go to exact fixed-point accumulators and the
// launch's last workgroup writes them into slot row 0 (bnfin.hpp DetRed).
template <bool RES, bool BWD, bool MAFF, bool TWO>
__global__ __launch_bounds__(384) void wino_out_xf_kernel(const float* __restrict__ P, float* __restrict__ y,
                                                          const float* __restrict__ res, float* __restrict__ stats,
                                                          int T, int H, int W, int K, WinoBwdStats bs, DetRed det,
                                                          const float* __restrict__ sshift, int nsplit) {
  __shared__ float xf[2][6][4][64];
  __shared__ float red[3][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int tw = (W + 3) >> 2, tpi = ((H + 3) >> 2) * tw;  // partial edge tiles
  const size_t bstride = (size_t)T * K;
  constexpr bool bwd = BWD, two = BWD && TWO;
  float m1 = 0.f, i1 = 0.f, m2 = 0.f, i2 = 0.f, msc = 0.f, msh = 0.f;
  if constexpr (bwd) {
    m1 = bs.saved1[k];
    i1 = bs.saved1[K + k];
    if constexpr (MAFF) {
      msc = bs.mask_aff[k];
      msh = bs.mask_aff[K + k];
    }
    if constexpr (two) {
      m2 = bs.saved2[k];
      i2 = bs.saved2[K + k];
    }
  }
  const float kshift = (!bwd && sshift) ? sshift[k] : 0.f;  // forward statistics: shifted sums
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
  // P holds nsplit partial slabs per point (the GEMM's reduction split, psx_wino_conv): summed here
  auto load = [&](int t, float (&m)[6]) {
    const float* pt = P + (size_t)t * K + k + (size_t)(wv * 6) * nsplit * bstride;
    if (nsplit == 1) {
#pragma unroll
      for (int s = 0; s < 6; ++s) m[s] = pt[s * bstride];
      return;
    }
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      float v = pt[(size_t)s * nsplit * bstride];
      for (int j = 1; j < nsplit; ++j) v += pt[((size_t)s * nsplit + j) * bstride];
      m[s] = v;
    }
  };
  int t = blockIdx.y;
  float m[6];
  if (t < T) load(t, m);
  for (int p = 0; t < T; t += gridDim.y, p ^= 1) {
    {
      float cur[6] = {m[0], m[1], m[2], m[3], m[4], m[5]}, q[4];
      const int tn = t + gridDim.y;
      if (tn < T) load(tn, m);
      wino_at6(cur, q);  // row wv of P A
#pragma unroll
      for (int j = 0; j < 4; ++j) xf[p][wv][j][lane] = q[j];
    }
    const int n = t / tpi, rem = t - n * tpi, ti = rem / tw, tj = rem - ti * tw;
    // partial edge tiles: this wave's output column 4 tj + wv and rows 4 ti + i must be inside the
    // image (a missing pixel's loads read the tile's first pixel, in bounds, and are discarded)
    const int vi = min(4, H - 4 * ti);
    const bool cok = 4 * tj + wv < W;
    const size_t base0 = (((size_t)n * H + 4 * ti) * W + 4 * tj) * K + k;
    const size_t base = cok ? base0 + (size_t)wv * K : base0;  // pixel (0, wv)
    float rv[4], y1v[4], ov[4], y2v[4];
    if (wv < 4) {  // the epilogue's operands, issued before the barrier
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t off = base + (size_t)(i < vi ? i : 0) * W * K;
        if constexpr (RES) rv[i] = res[off];
        if constexpr (bwd) {
          y1v[i] = bs.y1[off];
          if constexpr (!MAFF) ov[i] = bs.o[off];
          if constexpr (two) y2v[i] = bs.y2[off];
        }
      }
    }
    __syncthreads();
    if (wv < 4) {
      float col[6], o[4];
#pragma unroll
      for (int r = 0; r < 6; ++r) col[r] = xf[p][r][wv][lane];
      wino_at6(col, o);  // output column wv: A^T applied
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!cok || i >= vi) continue;
        const size_t off = base + (size_t)i * W * K;
        float v = o[i];
        if constexpr (RES) v += rv[i];
        if constexpr (bwd) {
          const float y1 = y1v[i];
          bool pos;
          if constexpr (MAFF)
            pos = y1 * msc + msh > 0.f;
          else
            pos = ov[i] > 0.f;
          const float dz = pos ? v : 0.f;
          s1 += dz;
          s2 += dz * (y1 - m1) * i1;
          if constexpr (two) s3 += dz * (y2v[i] - m2) * i2;
          y[off] = bs.mask_store ? dz : v;
        } else {
          y[off] = v;
          const float dd = v - kshift;
          s1 += dd;
          s2 += dd * dd;
        }
      }
    }
  }
  float* dst = bwd ? bs.part : stats;
  if (!dst) return;
  const int nst = bwd ? (two ? 3 : 2) : 2;
  if (wv < 4) {
    red[0][wv][lane] = s1;
    red[1][wv][lane] = s2;
    red[2][wv][lane] = s3;
  }
  __syncthreads();
  float* row = dst + (size_t)(blockIdx.y & (PSX_STAT_SLOTS - 1)) * nst * K;
  if (threadIdx.x < 64 * nst) {
    const int which = threadIdx.x >> 6;
    const float v = red[which][0][lane] + red[which][1][lane] + red[which][2][lane] + red[which][3][lane];
    stat_add(det, row, which * K + k, v);
  }
}

// dW[k][c][3][3] = scale * G^T M G, M[b] = sum of the q partial slabs part[b * q + j][k][c] (the
// batched TN GEMM's split of each batch over tile ranges); OutT = uint16_t: the fp16 wire
// (reference codec), float: fp32 gradients; OIHW like wgrad_reduce's output. A workgroup = 64 (k, c) pairs x 6 waves; wave r
// sums the q partial slabs of row r of M (6 q loads in flight, unrolled for Q > 0) and applies G
// along the row, waves 0-2 then take column j of the result through LDS, and the workgroup's
// 64 x 9 outputs leave as one contiguous run. The one-thread-per-pair kernel issued 36 q
// loads per thread from (K C / 256) workgroups: 16 for a 64 x 64 layer, a latency chain
// (q = 8 with its runtime loop: +50 us).
template <typename OutT, int Q>
__global__ __launch_bounds__(384) void wino_wout_xf_kernel(const float* __restrict__ part, OutT* __restrict__ out,
                                                           int K, int C, int q, float scale) {
  __shared__ float mg[6][3][64];
  __shared__ float stage[64 * 9];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long i0 = (long)blockIdx.x * 64, n = (long)K * C;
  const long i = i0 + lane;
  const int qq = Q > 0 ? Q : q;
  const size_t slab = (size_t)K * C;
  if (i < n) {
    float m6[6], o[3];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const float* p = part + (size_t)(wv * 6 + s) * qq * slab + i;
      float v = p[0];
      if constexpr (Q > 0) {
#pragma unroll
        for (int j = 1; j < Q; ++j) v += p[j * slab];
      } else {
        for (int j = 1; j < qq; ++j) v += p[j * slab];
      }
      m6[s] = v;
    }
    wino_gt6(m6, o);  // row wv of M G
#pragma unroll
    for (int j = 0; j < 3; ++j) mg[wv][j][lane] = o[j];
  }
  __syncthreads();
  if (wv < 3 && i < n) {
    float col[6], o[3];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = mg[r][wv][lane];
    wino_gt6(col, o);  // column wv of G^T (M G)
#pragma unroll
    for (int p = 0; p < 3; ++p) stage[lane * 9 + p * 3 + wv] = o[p] * scale;
  }
  __syncthreads();
  const long lim = (n - i0 < 64 ? n - i0 : 64) * 9;
  OutT* dst = out + i0 * 9;
  for (int j = threadIdx.x; j < lim; j += 384) {
    const float v = stage[j];
    if constexpr (sizeof(OutT) == 2)
      dst[j] = __builtin_bit_cast(uint16_t, (_Float16)v);
    else
      dst[j] = v;
  }
}

}  // namespace psx

using namespace psx;

extern "C" {

// Floats of one Winograd conv's transformed operands: V = T*36*C (input tiles, kept per layer for
// the weight gradient) and P = 36*T*K (GEMM output / dy tiles).
// T = N * ceil(H / 4) * ceil(W / 4) output tiles (partial edge tiles: ResNet-50's 14x14 / 7x7)
static long wino_tiles(int N, int H, int W) { return (long)N * ((H + 3) / 4) * ((W + 3) / 4); }

long psx_wino_v_floats(int N, int H, int W, int C) { return wino_tiles(N, H, W) * 36 * C; }

// Reduction split s2 of the 36 GEMMs (a pure function of the shape: psx_wino_p_floats sizes the
// caller's P buffer with it, so no run-time override may change it later): each point's C-long reduction
// runs as s2 workgroup ranges writing s2 partial slabs of P, summed by the output transform. 2 when
// the 64x64 tiles give fewer than 768 workgroups (3 per CU: the last round part-empty): ResNet-18's
// 4x4x512 points (576), fwd / dgrad 47.6 / 46.8 -> 45.6 / 43.8 us; 8x8x256 (1152 workgroups) and
// ResNet-50's 14x14 / 7x7 points are slower split (profiles/r5_wino_split_ab.jsonl).
static int wino_gemm_split(int T, int C, int K) {
  int s2 = 36L * ((T + 63) / 64) * (K / 64) < 768 ? 2 : 1;
  while (s2 > 1 && (C / 32) % s2) s2 >>= 1;  // whole k-steps (32 fp32 channels) per range
  return s2;
}

// floats of the GEMM output P of psx_wino_conv (36 x T x K x the reduction split)
long psx_wino_p_floats(int N, int H, int W, int C, int K) {
  const long T = wino_tiles(N, H, W);
  return 36 * T * K * wino_gemm_split((int)T, C, K);
}

long psx_wino_workspace(int N, int H, int W, int C, int K) {
  return psx_wino_v_floats(N, H, W, C) + psx_wino_v_floats(N, H, W, K);
}

// 1 when psx_wino_conv handles this layer: 3x3 / stride 1 / pad 1, H, W >= 4 (not a multiple of
// 4: the edge tiles are partial — zero padded in, clipped out: 14x14 -> 16 tiles of 16 pixels),
// channels powers of two >= 64 (transform blocks, the GEMM's per-batch channel decode).
int psx_wino_ok(int H, int W, int C, int K) {
  return H >= 4 && W >= 4 && C >= 64 && K >= 64 && !(C & (C - 1)) && !(K & (K - 1));
}

// fwd (flip = 0): U[K][36][C] from w [K][C][3][3]; dgrad (flip = 1): U[C][36][K] of rot180(w)^T.
int psx_wino_weights(const float* w, float* U, int K, int C, int flip, hipStream_t st) {
  const long n = (long)K * C;
  hipLaunchKernelGGL(wino_w_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, w, U, K, C, flip);
  return (int)hipGetLastError();
}

// n (<= 40) weight transforms in one launch: w[j] OIHW [K[j]][C[j]][3][3] -> U[j] (flip[j] as in
// psx_wino_weights).
// layout (nullable): per item 1 = the fused kernel's operand order (rows and columns multiples of
// 16 and 4).
int psx_wino_weights_multi(const float* const* w, float* const* U, const int* K, const int* C, const int* flip, int n,
                           const int* layout, hipStream_t st) {
  if (n < 1 || n > kWinoWMax) return -2;
  WinoWBatch b{};
  long p = 0;
  for (int j = 0; j < n; ++j) {
    const int lay = layout ? layout[j] : 0;
    if (lay && ((flip[j] ? C[j] : K[j]) % 16 || (flip[j] ? K[j] : C[j]) % 4)) return -3;
    b.d[j] = WinoWDesc{w[j], U[j], K[j], C[j], flip[j], lay, p};
    p += (long)K[j] * C[j];
  }
  b.n = n;
  b.total = p;
  hipLaunchKernelGGL(wino_w_multi_kernel, dim3((unsigned)((p + 63) / 64)), dim3(64), 0, st, b);
  return (int)hipGetLastError();
}

// y[N][H][W][K] = conv3x3(x[N][H][W][C]) (+ res) with the pre-transformed weights U [K][36][C];
// stats (nullable): BN partial sums into slot rows [PSX_STAT_SLOTS][2][K] (pre-zeroed); bst
// (nullable, data gradient): the consumer BN's backward sums instead (conv_v2 BwdStatsDesc).
// bnpart + bnfin (nullable, forward): x is the previous layer's pre-BN output; its BN finalize +
// BN + ReLU run inside the input transform (wino_in_kernel).
// V: psx_wino_v_floats(C) (the transformed input, left there for psx_wino_wgrad), P: 36*T*K
// floats. cfg: GEMM tile (psx_bgemm_f32).
int psx_wino_conv(const float* x, const float* U, float* y, const float* res, float* stats, float* V, float* P,
                  const void* zero, int N, int H, int W, int C, int K, int cfg, const WinoBwdStats* bst,
                  const float* bnpart, const WinoBnFin* bnfin, const float* sshift, hipStream_t st) {
  if (bnpart && (!bnfin || bnfin->C != C)) return -3;
  if (!psx_wino_ok(H, W, C, K)) return -2;
  const int T = (int)wino_tiles(N, H, W);
  WinoBnFin bf{};
  if (bnpart) bf = *bnfin;
  bf.det = (int)det_enabled();
  hipLaunchKernelGGL(wino_in_xf_kernel, dim3(C / 64, wino_xf_grid(T, C / 64)), dim3(64 * kXfWaves), 0, st, x, V, T, H,
                     W, C, bnpart, bf);
  // the 36 GEMMs: the conv_v2 mainloop. (Measured slower and removed in round 5: a stream-K GEMM,
  // 8x8x256 40.6 vs 33.7 us, profiles/r4_sk_gemm_probes.jsonl; the GEMM with the output transform
  // in its epilogue, 64 output registers per accumulator forcing 16x16 wave tiles: neutral where
  // it had >= 256 workgroups, 1.8x slower elsewhere, profiles/r4_numbers.jsonl r4_call16.)
  const int s2 = wino_gemm_split(T, C, K);
  int e = psx_bgemm_f32_split(V, U, P, zero, T, K, C, 36, s2, cfg, st);
  if (e) return e;
  WinoBwdStats bs{};
  if (bst) bs = *bst;
  const int gyo = wino_xf_grid(T, K / 64);
  DetRed det{};
  if (bst || stats) det = det_for(bst ? bst->part : stats);
  using OutK = void (*)(const float*, float*, const float*, float*, int, int, int, int, WinoBwdStats, DetRed,
                       const float*, int);
  // [res][variant]: forward, backward (ReLU mask from o / from the affine) x (one / two BN sums)
  static const OutK kOutXf[2][5] = {
      {wino_out_xf_kernel<false, false, false, false>, wino_out_xf_kernel<false, true, false, false>,
       wino_out_xf_kernel<false, true, false, true>, wino_out_xf_kernel<false, true, true, false>,
       wino_out_xf_kernel<false, true, true, true>},
      {wino_out_xf_kernel<true, false, false, false>, wino_out_xf_kernel<true, true, false, false>,
       wino_out_xf_kernel<true, true, false, true>, wino_out_xf_kernel<true, true, true, false>,
       wino_out_xf_kernel<true, true, true, true>}};
  const int var = bst ? 1 + 2 * (bs.mask_aff != nullptr) + (bs.y2 != nullptr) : 0;
  hipLaunchKernelGGL(kOutXf[res != nullptr][var], dim3(K / 64, gyo), dim3(64 * kXfWaves), 0, st, P, y, res,
                     bst ? nullptr : stats, T, H, W, K, bs, det, sshift, s2);
  return (int)hipGetLastError();
}

// Weight-gradient GEMM tile (BR = BC): 64 (3 workgroups per CU).
static int wino_wtile(int, int) { return 64; }

// Tile-range splits q of the weight-gradient GEMM: 36 * q * (C/BR) * (K/BC) workgroups, each
// over T / q tiles (a multiple of 32): the smallest q reaching 1024 workgroups while a split keeps
// >= 256 tiles, at most 8. Same-box sweep with the split output transform (B=128,
// us incl. dy transform, q = 1 / 2 / 4 / 8 / 16): 32x32x64 244 / 134 / 79 / 69 / 83, 16x16x128
// 72 / 62 / 51 / 48 / 69, 8x8x256 51 / 46 / 47 / 55 / 81, 4x4x512 47 / 54 / 75 (bench/wino_fused_ab.py).
// 0 = not applicable.
int psx_wino_wgrad_q(int N, int H, int W, int C, int K) {
  const int T = (int)wino_tiles(N, H, W);
  if (!psx_wino_ok(H, W, C, K) || T % 32) return 0;
  const int bt = wino_wtile(C, K);
  int q = 1;
  while (36L * q * (C / bt) * (K / bt) < 1024 && q < 8 && T % (32 * 2 * q) == 0 && T / (2 * q) >= 256) q *= 2;
  return T % (32 * q) ? 0 : q;
}

// Weight gradient of psx_wino_conv: V = that call's transformed input, dy [N][H][W][K]; D: 36*T*K
// floats of scratch, part: 36*q*K*C floats (q = psx_wino_wgrad_q). out: OIHW gradient, fp16
// (out_fp16, the wire) or fp32, times scale.
// ybn / bpart / bbfin (nullable): dy is dz of a BN whose backward apply is folded into the dy
// transform (wino_dy_xf_kernel); the fused data gradient of the same layer publishes that BN's
// coefficients and dgamma / dbeta.
int psx_wino_wgrad(const float* V, const float* dy, float* D, float* part, void* out, int out_fp16, float scale,
                   const void* zero, int N, int H, int W, int C, int K, const float* ybn, const float* bpart,
                   const BnBwdFin* bbfin, hipStream_t st) {
  const int q = psx_wino_wgrad_q(N, H, W, C, K);
  if (q < 1) return -2;
  if (bpart && (!ybn || !bbfin || bbfin->C != K)) return -3;
  const int T = (int)wino_tiles(N, H, W);
  BnBwdFin bb{};
  if (bpart) bb = *bbfin;
  bb.det = (int)det_enabled();
  hipLaunchKernelGGL(wino_dy_xf_kernel, dim3(K / 64, wino_xf_grid(T, K / 64)), dim3(64 * kXfWaves), 0, st, dy, D, T, H,
                     W, K, ybn, bpart, bb);
  const int bt = wino_wtile(C, K);
  int e = psx_bgemm_tn_f32(V, D, part, zero, T, C, K, 36, q, bt, bt, st);
  if (e) return e;
  return psx_wino_wout(part, out, out_fp16, scale, K, C, q, st);
}

// dW[k][c][3][3] = scale * G^T M G with M[b] = sum_j part[b * q + j][k][c]: the output transform
// of a Winograd weight gradient (its 36 x q partial slabs [36 * q][K][C] from psx_bgemm_tn_f32 or
// from the fused weight-gradient kernel, wino_wgrad.hip). out: OIHW, fp16 (out_fp16) or fp32.
int psx_wino_wout(const float* part, void* out, int out_fp16, float scale, int K, int C, int q, hipStream_t st) {
  const long n = (long)K * C;
  const dim3 gx((unsigned)((n + 63) / 64));
#define PSX_WOUT(OT, QV) \
  hipLaunchKernelGGL((wino_wout_xf_kernel<OT, QV>), gx, dim3(64 * kXfWaves), 0, st, part, (OT*)out, K, C, q, scale)
#define PSX_WOUT_Q(OT)                \
  if (q == 1) PSX_WOUT(OT, 1);        \
  else if (q == 2) PSX_WOUT(OT, 2);   \
  else if (q == 4) PSX_WOUT(OT, 4);   \
  else if (q == 8) PSX_WOUT(OT, 8);   \
  else if (q == 16) PSX_WOUT(OT, 16); \
  else if (q == 32) PSX_WOUT(OT, 32); \
  else PSX_WOUT(OT, 0)
  if (out_fp16) {
    PSX_WOUT_Q(uint16_t);
  } else {
    PSX_WOUT_Q(float);
  }
#undef PSX_WOUT_Q
#undef PSX_WOUT
  return (int)hipGetLastError();
}

}  // extern "C"
