// fp32 Winograd F(4x4,3x3) conv with both transforms fused into the GEMM: ONE launch per conv, the
// transformed input V and the 36 GEMM outputs P never reach HBM (wino.hip runs input transform ->
// 36 batched GEMMs -> output transform as three launches, V and P 2.25x the activation each way:
// on the 32x32x64 layer ~300 MB of the ~370 MB a conv moves).
//
// Workgroup = 16 Winograd tiles x 64 output channels, 8 waves (two per SIMD, <= 256 registers,
// 84 KB LDS: one workgroup per CU). Wave w = (kq = w & 3, h = w >> 2) owns output channels
// [16 kq, 16 kq + 16) of the block and Winograd points 18h .. 18h + 17 (rows 3h .. 3h + 2 of the
// 6x6): acc[m] is one v_mfma_f32_16x16x4_f32 tile per point (72 accumulator registers), so lane l
// ends holding M_b[tile 4(l>>4)+i][channel l&15] for its 18 points and i = 0..3. 144 per wave (all
// 36 points, one wave per SIMD) ran the same speed: the transform and the MFMAs serialise; here
// waves 0-3 transform while waves 4-7 multiply.
//
// The reduction runs over C in groups of 16 channels = 4 MFMA k-steps. Per group waves 0-3
// transform the block's 16 tiles x 16 channels (lane = (tile 4 kq + (l>>4), channel l&15): each of
// the 36 patch loads is 4 runs of 64 contiguous bytes — one (tile, channel) per lane with 16 tiles
// per instruction measured 87 vs 63 us on 32x32x64; clamped rows / columns through buffer loads,
// the optional folded BN + ReLU of the previous layer, zero padding, B^T d B in registers) and
// write the 36 values into the LDS group buffer in the MFMA A-operand order (slots of four points,
// ds_write_b128). After one barrier per group every wave runs its 4 x 18 MFMAs, A from LDS
// (4 ds_read_b128 + 1 ds_read_b64 per k-step), B (the transformed weights, laid out in the
// B-operand order by the weight transform, layout 1) straight from L2 by buffer loads prefetched
// one k-step ahead. Waves 0-3 transform group g + 1 first (patch loaded during group g - 1) while
// waves 4-7 already multiply group g; the group buffer is double-buffered. The group loop is fully
// unrolled (4 or 8 groups: 64 / 128 input channels), which also keeps hipcc from copying the
// loop-carried accumulators between register files every group.
//
// Epilogue: per tile the row pass Z = (M rows) A of the wave's 3 rows, its share of y = A^T M A,
// the partner wave's share of two of the four tiles through LDS, then (same contract as wino.hip
// wino_out_kernel) forward (+ residual) with BN slot sums of y (shifted), or data gradient with the
// consumer BN's backward sums (ReLU mask from o or from the affine, one or two BNs) and the masked
// store; deterministic mode through the slab (DetRed). V (nullable): the forward also stores the
// transformed input [36][T][C] for the Winograd weight gradient (wino.hip psx_wino_wgrad).
#include "bnfin.hpp"
#include "common.hpp"
#include "wino.hpp"

// diagnostics (A/B builds only, wrong results): bit 1 no B loads, 2 no patch loads, 4 no transform
// VALU, 8 no V stores, 16 no A reads from LDS, 32 no transform at all (VALU + LDS writes)
#ifndef PSX_WF_PROBE
#define PSX_WF_PROBE 0
#endif
// bit 1: B operands loaded two k-steps ahead (else one); bit 2: the next k-step's A operands read
// before this k-step's MFMAs (inside a group)
#ifndef PSX_WF_PF
#define PSX_WF_PF 0
#endif
#ifndef PSX_WF_SWZ
#define PSX_WF_SWZ 1
#endif

namespace psx {

PSX_DEV void mfma_f32_16x16x4(f32x4& acc, float a, float b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}

constexpr int kWfT = 16;  // tiles per workgroup (the MFMA's 16 rows)
constexpr int kWfK = 64;  // output channels per workgroup (4 waves x 16)

struct WinoFusedArgs {
  const float* x;  // [N][H][W][C]
  const float* U;  // transformed weights, layout 1 (wino.hip wino_w_multi_kernel)
  float* y;        // [N][H][W][K]
  const float* res;
  float* stats;
  float* V;  // nullable: [36][T][C]
  const float* bnpart;
  const float* sshift;
  const float* ybn;    // BN-backward fold (data gradient): the BN's forward input y (nullable)
  const float* bpart;  // its backward slot sums [PSX_STAT_SLOTS][2][C]
  int H, W, C, K, T, nkb;
  int xbytes, ubytes, vbytes, ybytes;
};

template <int GG, bool RES, bool BWD, bool MAFF, bool TWO>
__global__ __launch_bounds__(512, 1) void wino_fused_kernel(WinoFusedArgs a, WinoBnFin fin, WinoBwdStats bs,
                                                            DetRed det, BnBwdFin bfin) {
  // [buffer][k-step][slot][lane]: slot 5h + i (i < 4) = points 18h + 4i .. +3, slot 5h + 4 = points
  // 18h + 16, 18h + 17 (+ 2 unused floats)
  __shared__ f32x4 vb[2][4][10][64];
  __shared__ float aff[3][256];
  __shared__ float red[3][4][16];
  const int l = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kq = w & 3, h = w >> 2;  // channel quarter, Winograd point half
  const int id = xcd_remap(blockIdx.x, gridDim.x);  // a tile block's channel blocks on one XCD
  const int tb = id / a.nkb, kb = id - tb * a.nkb;
  const int H = a.H, W = a.W, C = a.C, K = a.K;
  const int tw = W >> 2, tpi = (H >> 2) * tw;
  const bool bnin = a.bnpart != nullptr;
  // BN-backward fold (data gradient whose input dy = BNbwd(dz, y) was never written): x is dz,
  // the operand is k1 dz + k2 y + k3 with the coefficients finalized here from the slot sums
  const bool bwdin = a.bpart != nullptr;
  // the transform applies max(x * aff0 + aff1, lo) unconditionally (one branch-free group body):
  // identity (1, 0, -inf) without a folded BN
  const float lo = bnin ? 0.f : -__builtin_inff();
  if (bwdin) {
    for (int c = threadIdx.x; c < C; c += 512) {
      float k1, k2, k3;
      double sdz, sxh;
      wino_bwd_coef(a.bpart, bfin, c, k1, k2, k3, sdz, sxh);
      aff[0][c] = k1;
      aff[1][c] = k3;
      aff[2][c] = k2;
      if (id == 0) {  // one workgroup publishes the coefficients and dgamma / dbeta (the wire)
        bfin.coef[c] = k1;
        bfin.coef[C + c] = k2;
        bfin.coef[2 * C + c] = k3;
        const float dg = (float)sxh * bfin.gscale, db = (float)sdz * bfin.gscale;
        if (bfin.grad_fp16) {
          reinterpret_cast<uint16_t*>(bfin.dgamma)[c] = __builtin_bit_cast(uint16_t, (_Float16)dg);
          reinterpret_cast<uint16_t*>(bfin.dbeta)[c] = __builtin_bit_cast(uint16_t, (_Float16)db);
        } else {
          reinterpret_cast<float*>(bfin.dgamma)[c] = dg;
          reinterpret_cast<float*>(bfin.dbeta)[c] = db;
        }
      }
    }
  } else if (!bnin) {
    for (int c = threadIdx.x; c < C; c += 512) {
      aff[0][c] = 1.f;
      aff[1][c] = 0.f;
    }
  } else {  // BN finalize of the input channels (wino.hip wino_in_kernel), all C of them
    for (int c = threadIdx.x; c < C; c += 512) {
      const double s = slot_sum<PSX_STAT_SLOTS>(a.bnpart, c, 2 * (size_t)C, fin.det);
      const double ss = slot_sum<PSX_STAT_SLOTS>(a.bnpart, (size_t)C + c, 2 * (size_t)C, fin.det);
      double mean, var;
      bn_moments(s, ss, fin.count, fin.sshift ? fin.sshift[c] : 0.f, mean, var);
      const float invstd = (float)(1.0 / sqrt(var + (double)fin.eps));
      const float sc = fin.gamma[c] * invstd, sh = fin.beta[c] - (float)mean * sc;
      aff[0][c] = sc;
      aff[1][c] = sh;
      if (id == 0) {
        fin.scale[c] = sc;
        fin.shift[c] = sh;
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
  }
  __syncthreads();

  // ---- transform role (waves 0-3, wave kq = k-step kq of a group): lane = (tile l&15, channel l>>4)
  // (tiles 4 kq .. 4 kq + 3 x the group's 16 channels: a patch load is 4 runs of 64 contiguous
  // bytes; the value for (tile tl, channel cl) goes to A-operand lane (cl & 3) * 16 + tl of k-step
  // cl >> 2)
  const int tl = 4 * kq + (l >> 4), cl = l & 15;
  const int t = tb * kWfT + tl;
  const int la = (cl & 3) * 16 + tl, qa = cl >> 2;
  int rowoff[6], coloff[6];
  unsigned okr = 0, okc = 0;
  {
    const int n = t / tpi, rem = t - n * tpi, ti = rem / tw, tj = rem - ti * tw;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int hh = 4 * ti - 1 + r, wc = 4 * tj - 1 + r;
      const bool oh = (unsigned)hh < (unsigned)H, ow = (unsigned)wc < (unsigned)W;
      okr |= (unsigned)oh << r;
      okc |= (unsigned)ow << r;
      // clamped in-image row / column: a padding position loads a real pixel, zeroed below
      rowoff[r] = (((n * H + (oh ? hh : (hh < 0 ? 0 : H - 1))) * W) * C + cl) * 4;
      coloff[r] = (ow ? wc : (wc < 0 ? 0 : W - 1)) * C * 4;
    }
  }
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, a.xbytes, 0x00020000);
  const auto ybr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.ybn), 0, bwdin ? a.xbytes : 0, 0x00020000);
  const auto ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
  const int S4 = C >> 2;  // MFMA k-steps
  // B operand of wave (kq, h): k-step s at ubase + s * 10 KB, its slots 5h .. 5h + 4
  const int ubase = ((kb * 4 + kq) * S4 * 10 + h * 5) * 1024;
  constexpr int G = GG;  // 16-channel groups (C / 16): the group loop is fully unrolled
  // V side output through a buffer descriptor: stores of the pipeline's one dummy transform (past
  // the last group) go to a zero-record descriptor and are dropped
  const auto vr = __builtin_amdgcn_make_buffer_rsrc(a.V, 0, a.V ? a.vbytes : 0, 0x00020000);
  const auto vnull = __builtin_amdgcn_make_buffer_rsrc(a.V, 0, 0, 0x00020000);
  const int voff = (t * C + cl) * 4;

  // LDS image unit of (k-step q, A-operand lane u): XOR-swizzled within the k-step's 1 KB slot
  // block so the transform's ds_write_b128 (16 lanes of one tile = 16 channels scatter over the 4
  // k-steps and 4 lane groups) hit 16 different bank groups instead of one; the MFMA reads stay a
  // permutation of one contiguous 1 KB block (conflict-free)
  auto swz = [](int q, int u) { return PSX_WF_SWZ ? (u ^ ((((u >> 4) << 2) + q) & 15)) : u; };
  float d[36], yb[36];
  auto load_patch = [&](int g) {
    const int so = g * 16 * 4;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int s = 0; s < 6; ++s)
        d[r * 6 + s] = (PSX_WF_PROBE & 2) ? (float)(rowoff[r] + coloff[s] + so)
                                          : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, rowoff[r] + coloff[s], so, 0));
    if (bwdin) {
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int s = 0; s < 6; ++s)
          yb[r * 6 + s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ybr, rowoff[r] + coloff[s], so, 0));
    }
  };
  auto xform = [&](int g, int p, bool real) {
    if constexpr ((PSX_WF_PROBE & 32) != 0) return;
    const int ch0 = g * 16;  // wave-uniform
    const float sc = aff[0][ch0 + cl], sh = aff[1][ch0 + cl];
    float e[36];
    if (bwdin) {  // dy = k1 dz + k2 y + k3 (k2 in aff[2]), padding stays zero
      const float k2 = aff[2][ch0 + cl];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int s = 0; s < 6; ++s) d[r * 6 + s] = wino_bwd_apply(d[r * 6 + s], yb[r * 6 + s], sc, k2, sh);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const float v = bwdin ? d[r * 6 + s] : fmaxf(d[r * 6 + s] * sc + sh, lo);
        e[r * 6 + s] = ((okr >> r) & (okc >> s) & 1u) ? v : 0.f;  // zero padding stays zero after BN + ReLU
      }
#pragma unroll
    for (int s = 0; s < 6; ++s) {  // columns: B^T d
      float col[6] = {e[s], e[6 + s], e[12 + s], e[18 + s], e[24 + s], e[30 + s]}, o[6];
      wino_bt6(col, o);
#pragma unroll
      for (int r = 0; r < 6; ++r) e[r * 6 + s] = o[r];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {  // rows: (B^T d) B
      float row[6] = {e[r * 6], e[r * 6 + 1], e[r * 6 + 2], e[r * 6 + 3], e[r * 6 + 4], e[r * 6 + 5]}, o[6];
      wino_bt6(row, o);
#pragma unroll
      for (int s = 0; s < 6; ++s) e[r * 6 + s] = o[s];
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 18 * hh + 4 * i;
        vb[p][qa][5 * hh + i][swz(qa, la)] = (f32x4){e[b], e[b + 1], e[b + 2], e[b + 3]};
      }
      vb[p][qa][5 * hh + 4][swz(qa, la)] = (f32x4){e[18 * hh + 16], e[18 * hh + 17], 0.f, 0.f};
    }
    // one channel block writes V (the others' transforms are the same values): the 16x16x128 forward
    // (two blocks) stored every value twice
    const auto rs = (real && kb == 0) ? vr : vnull;
    if ((PSX_WF_PROBE & 8) == 0 && a.V)  // the stores cost ~4 us on 32x32x64 even when dropped
#pragma unroll
    for (int b = 0; b < 36; ++b)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(e[b]), rs, voff, (b * a.T * C + ch0) * 4, 0);
  };

  // acc[m]: local point m = 0..17 of this wave's half (point 18h + m)
  f32x4 acc[18];
#pragma unroll
  for (int m = 0; m < 18; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
  constexpr int UD = (PSX_WF_PF & 1) ? 2 : 1;  // B prefetch distance (k-steps)
  f32x4 ub[UD][4];
  float2 uh[UD];
  auto load_u = [&](int s, int slot) {
    const int so = ubase + s * 10 * 1024;
    if constexpr ((PSX_WF_PROBE & 1) != 0) {  // diagnostic: B from registers
#pragma unroll
      for (int i = 0; i < 4; ++i) ub[slot][i] = (f32x4){(float)so, 1.f, 2.f, (float)i};
      uh[slot] = make_float2((float)so, 1.f);
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      ub[slot][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ur, l * 16 + i * 1024, so, 0));
    uh[slot] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(ur, l * 16 + 4 * 1024, so, 0));
  };
#pragma unroll
  for (int i = 0; i < UD; ++i) load_u(i < S4 ? i : S4 - 1, i);
  if (h == 0) {
    load_patch(0);
    xform(0, 0, true);
    load_patch(G > 1 ? 1 : 0);
  }
  __syncthreads();
  // Per group g: waves 0-3 first transform group g + 1 (patch loaded during the previous group)
  // into the other buffer and issue the patch loads of g + 2, while waves 4-7 — the other wave on
  // each SIMD — already run their MFMAs of g; then waves 0-3 run theirs. The MFMA pipe sees 72 + 72
  // MFMAs per SIMD and group with the transform in between hidden. The group past the last is a
  // dummy (clamped loads, dropped V stores, its LDS image never read).
  f32x4 an[4];
  float2 ah;
  auto load_a = [&](int p, int q) {
    if constexpr ((PSX_WF_PROBE & 16) != 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) an[i] = (f32x4){(float)p, (float)q, (float)i, 1.f};
      ah = make_float2((float)q, 2.f);
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) an[i] = vb[p][q][5 * h + i][swz(q, l)];
    ah = *reinterpret_cast<const float2*>(&vb[p][q][5 * h + 4][swz(q, l)]);
  };
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int p = g & 1;
    if (h == 0) {
      xform(g + 1, p ^ 1, g + 1 < G);
      load_patch(g + 2 < G ? g + 2 : G - 1);
    }
    if constexpr ((PSX_WF_PF & 2) != 0) load_a(p, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s = g * 4 + q;
      if constexpr ((PSX_WF_PF & 2) == 0) load_a(p, q);
      const f32x4 a0 = an[0], a1 = an[1], a2 = an[2], a3 = an[3];
      const float2 a4 = ah;
      if constexpr ((PSX_WF_PF & 2) != 0)
        if (q < 3) load_a(p, q + 1);
      const int us = s % UD;
      const f32x4 u0 = ub[us][0], u1 = ub[us][1], u2 = ub[us][2], u3 = ub[us][3];
      const float2 u4 = uh[us];
      load_u(s + UD < S4 ? s + UD : S4 - 1, us);  // UD k-steps ahead (past the end: re-loads the last)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mfma_f32_16x16x4(acc[j], a0[j], u0[j]);
        mfma_f32_16x16x4(acc[4 + j], a1[j], u1[j]);
        mfma_f32_16x16x4(acc[8 + j], a2[j], u2[j]);
        mfma_f32_16x16x4(acc[12 + j], a3[j], u3[j]);
      }
      mfma_f32_16x16x4(acc[16], a4.x, u4.x);
      mfma_f32_16x16x4(acc[17], a4.y, u4.y);
    }
    __syncthreads();
  }

  // ---- epilogue. Lane l holds M_b[tile 4(l>>4)+i][channel l&15] for this half's points b = 18h +
  // m (rows 3h .. 3h + 2 of the 6x6), i = 0..3. Per tile: Z = (M rows) A (row pass, 3 x 4), then
  // this half's share of y = A^T M A: Y_h[r][j] = sum_rr A^T[r][3h + rr] Z[rr][j]. Wave h keeps
  // tiles 2h, 2h + 1, hands the other two's partials to its partner (kq, 1 - h) through LDS
  // (the group buffers are free) and finishes its two tiles with the partner's partials.
  // A^T columns 3h .. 3h + 2 (rows r = 0..3): h = 0: [1 1 1; 0 1 -1; 0 1 1; 0 1 -1],
  // h = 1: [1 1 0; 2 -2 0; 4 4 0; 8 -8 1]
  float at[4][3];
  {
    const float c0[4][3] = {{1.f, 1.f, 1.f}, {0.f, 1.f, -1.f}, {0.f, 1.f, 1.f}, {0.f, 1.f, -1.f}};
    const float c1[4][3] = {{1.f, 1.f, 0.f}, {2.f, -2.f, 0.f}, {4.f, 4.f, 0.f}, {8.f, -8.f, 1.f}};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) at[r][rr] = h ? c1[r][rr] : c0[r][rr];
  }
  float yp[4][16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float z[3][4];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      float row[6] = {acc[6 * rr][i], acc[6 * rr + 1][i], acc[6 * rr + 2][i],
                      acc[6 * rr + 3][i], acc[6 * rr + 4][i], acc[6 * rr + 5][i]};
      wino_at6(row, z[rr]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) yp[i][r * 4 + j] = at[r][0] * z[0][j] + at[r][1] * z[1][j] + at[r][2] * z[2][j];
  }
  // hand-off: xb[kq][h][lane][36] (32 used: the partner's two tiles x 16 pixels; the 144-byte lane
  // stride keeps the b128 accesses conflict-free), h uniform: no per-value selects
  float* xb = reinterpret_cast<float*>(&vb[0][0][0][0]);
  float* mine = xb + ((size_t)(kq * 2 + h) * 64 + l) * 36;
  const float* theirs = xb + ((size_t)(kq * 2 + (1 - h)) * 64 + l) * 36;
  float yv[2][16];
  if (h) {
#pragma unroll
    for (int e = 0; e < 32; e += 4)
      *reinterpret_cast<f32x4*>(mine + e) =
          (f32x4){yp[e >> 4][e & 15], yp[e >> 4][(e & 15) + 1], yp[e >> 4][(e & 15) + 2], yp[e >> 4][(e & 15) + 3]};
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int e = 0; e < 16; ++e) yv[ii][e] = yp[2 + ii][e];
  } else {
#pragma unroll
    for (int e = 0; e < 32; e += 4)
      *reinterpret_cast<f32x4*>(mine + e) = (f32x4){yp[2 + (e >> 4)][e & 15], yp[2 + (e >> 4)][(e & 15) + 1],
                                                    yp[2 + (e >> 4)][(e & 15) + 2], yp[2 + (e >> 4)][(e & 15) + 3]};
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int e = 0; e < 16; ++e) yv[ii][e] = yp[ii][e];
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 32; e += 4) {
    const f32x4 t4 = *reinterpret_cast<const f32x4*>(theirs + e);
#pragma unroll
    for (int j = 0; j < 4; ++j) yv[e >> 4][(e & 15) + j] += t4[j];
  }

  const int k = kb * kWfK + kq * 16 + (l & 15);
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
  const float kshift = (!bwd && a.sshift) ? a.sshift[k] : 0.f;  // forward statistics: shifted sums
  // the output-sized tensors through buffer descriptors: 32-bit lane offsets, the pixel step in
  // the (uniform) soffset
  const int ybytes = a.ybytes;
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, ybytes, 0x00020000);
#ifdef PSX_WF_RES_BUF
  const auto rr_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.res), 0, RES ? ybytes : 0, 0x00020000);
#endif
  const auto y1r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bs.y1), 0, bwd ? ybytes : 0, 0x00020000);
  const auto orr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bs.o), 0, (bwd && !MAFF) ? ybytes : 0,
                                                     0x00020000);
  const auto y2r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bs.y2), 0, two ? ybytes : 0, 0x00020000);
  const bool mstore = bwd && bs.mask_store;
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
  for (int ii = 0; ii < 2; ++ii) {
    const int tt = tb * kWfT + 4 * (l >> 4) + 2 * h + ii;
    const int n = tt / tpi, rem = tt - n * tpi, ti = rem / tw, tj = rem - ti * tw;
    const int base = ((((n * H + 4 * ti) * W + 4 * tj) * K) + k) * 4;
    float rv[16], y1v[16], ov[16], y2v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int so = ((e >> 2) * W + (e & 3)) * K * 4;
      // the residual through a flat load: its buffer descriptor's 4 SGPRs pushed the residual +
      // data-gradient variants into SGPR spills held in VGPR lanes and then 25-144 VGPR spills to
      // scratch (113 vs 66 us per 32x32x64 call, profiles/README.md round-5 leads)
#ifdef PSX_WF_RES_BUF  // A/B builds: the buffer load
      if constexpr (RES) rv[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr_, base, so, 0));
#else
      if constexpr (RES) rv[e] = a.res[(base + so) >> 2];
#endif
      if constexpr (bwd) {
        y1v[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(y1r, base, so, 0));
        if constexpr (!MAFF) ov[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(orr, base, so, 0));
        if constexpr (two) y2v[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(y2r, base, so, 0));
      }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int so = ((e >> 2) * W + (e & 3)) * K * 4;
      float v = yv[ii][e];
      if constexpr (RES) v += rv[e];
      if constexpr (bwd) {
        const float y1 = y1v[e];
        bool pos;
        if constexpr (MAFF)
          pos = y1 * msc + msh > 0.f;
        else
          pos = ov[e] > 0.f;
        const float dz = pos ? v : 0.f;
        s1 += dz;
        s2 += dz * (y1 - m1) * i1;
        if constexpr (two) s3 += dz * (y2v[e] - m2) * i2;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mstore ? dz : v), yr, base, so, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), yr, base, so, 0);
        const float dd = v - kshift;
        s1 += dd;
        s2 += dd * dd;
      }
    }
  }
  float* dst = bwd ? bs.part : a.stats;
  if (!dst) return;
  const int nst = bwd ? (two ? 3 : 2) : 2;
  // lanes l, l^16, l^32, l^48 hold the same channel; then the wave pair (kq, 0 / 1) through LDS
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  if constexpr (two) {
    s3 += __shfl_xor(s3, 16, 64);
    s3 += __shfl_xor(s3, 32, 64);
  }
  if (h == 1 && l < 16) {
    red[0][kq][l] = s1;
    red[1][kq][l] = s2;
    red[2][kq][l] = s3;
  }
  __syncthreads();
  // deterministic mode: exact fixed-point accumulators (bnfin.hpp DetRed)
  float* row = dst + (size_t)(tb & (PSX_STAT_SLOTS - 1)) * nst * K;
  if (h == 0 && l < 16) {
    stat_add(det, row, k, s1 + red[0][kq][l]);
    stat_add(det, row, K + k, s2 + red[1][kq][l]);
    if constexpr (two) stat_add(det, row, 2 * K + k, s3 + red[2][kq][l]);
  }
}

}  // namespace psx

using namespace psx;

extern "C" {

// 1 when psx_wino_fused handles the layer: the Winograd conditions (wino.hip psx_wino_ok), whole
// 16-tile blocks, 64-channel output blocks, 64 or 128 input channels (the fully unrolled group
// loop is instantiated for 4 and 8 groups) and 32-bit byte offsets.
int psx_wino_fused_ok(int N, int H, int W, int C, int K) {
  if (H % 4 || W % 4 || (C != 64 && C != 128) || K % kWfK) return 0;  // instantiated: 4 / 8 groups
  const long T = (long)N * (H / 4) * (W / 4);
  return T % kWfT == 0 && (long)N * H * W * (long)(C > K ? C : K) * 4 < (1L << 31) && 40L * C * K * 4 < (1L << 31) &&
         36L * T * C < (1L << 31);
}

// y[N][H][W][K] = conv3x3(x[N][H][W][C]) (+ res) from the layout-1 transformed weights Uf; the rest
// as psx_wino_conv (wino.hip). V (nullable): the transformed input [36][T][C] for psx_wino_wgrad.
// ybn / bpart / bbfin (nullable, data gradient): x is dz and the operand is the BN backward
// k1 dz + k2 ybn + k3 of the BN whose backward sums are bpart (the BN-backward apply folded in;
// the launch publishes the coefficients and dgamma / dbeta, bnfin.hpp BnBwdFin).
int psx_wino_fused(const float* x, const float* Uf, float* y, const float* res, float* stats, float* V, int N, int H,
                   int W, int C, int K, const WinoBwdStats* bst, const float* bnpart, const WinoBnFin* bnfin,
                   const float* sshift, const float* ybn, const float* bpart, const BnBwdFin* bbfin,
                   hipStream_t st) {
  if (!psx_wino_fused_ok(N, H, W, C, K)) return -2;
  if (bnpart && (!bnfin || bnfin->C != C)) return -3;
  if (bpart && (!bbfin || bbfin->C != C || !ybn || bnpart)) return -3;
  const int T = N * (H / 4) * (W / 4);
  WinoFusedArgs a{x, Uf, y, res, bst ? nullptr : stats, V, bnpart, sshift, bpart ? ybn : nullptr, bpart, H, W, C, K, T,
                  K / kWfK,
                  (int)((long)N * H * W * C * 4), (int)(40L * C * K * 4), (int)(36L * T * C * 4),
                  (int)((long)N * H * W * K * 4)};
  WinoBnFin bf{};
  if (bnpart) bf = *bnfin;
  bf.det = (int)det_enabled();
  WinoBwdStats bs{};
  if (bst) bs = *bst;
  const int rows = T / kWfT;
  DetRed det{};
  if (bst || stats) det = det_for(bst ? bst->part : stats);
  using FK = void (*)(WinoFusedArgs, WinoBnFin, WinoBwdStats, DetRed, BnBwdFin);
  BnBwdFin bb{};
  if (bpart) bb = *bbfin;
  bb.det = (int)det_enabled();
#define PSX_WF_ROW(G, R)                                                                                     \
  {wino_fused_kernel<G, R, false, false, false>, wino_fused_kernel<G, R, true, false, false>,                 \
   wino_fused_kernel<G, R, true, false, true>, wino_fused_kernel<G, R, true, true, false>,                    \
   wino_fused_kernel<G, R, true, true, true>}
  // [C / 16 == 8][res][variant]: forward, backward (ReLU mask from o / from the affine) x (one / two BN sums)
  static const FK kF[2][2][5] = {{PSX_WF_ROW(4, false), PSX_WF_ROW(4, true)}, {PSX_WF_ROW(8, false), PSX_WF_ROW(8, true)}};
#undef PSX_WF_ROW
  const int var = bst ? 1 + 2 * (bs.mask_aff != nullptr) + (bs.y2 != nullptr) : 0;
  hipLaunchKernelGGL(kF[C == 128][res != nullptr][var], dim3((unsigned)(rows * (K / kWfK))), dim3(512), 0, st, a, bf, bs, det, bb);
  return (int)hipGetLastError();
}

}  // extern "C"
