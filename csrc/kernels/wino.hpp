// Shared pieces of the fp32 Winograd F(4x4,3x3) kernels (wino.hip: separate transforms + batched
// GEMMs; wino_fused.hip: transforms fused into the GEMM). Matrices in wino.hip's header comment.
#pragma once
#include "bnfin.hpp"
#include "common.hpp"

namespace psx {

PSX_DEV void wino_bt6(const float (&d)[6], float (&r)[6]) {
  r[0] = 4.f * d[0] - 5.f * d[2] + d[4];
  r[1] = -4.f * (d[1] + d[2]) + d[3] + d[4];
  r[2] = 4.f * (d[1] - d[2]) - d[3] + d[4];
  r[3] = 2.f * (d[3] - d[1]) - d[2] + d[4];
  r[4] = 2.f * (d[1] - d[3]) - d[2] + d[4];
  r[5] = 4.f * d[1] - 5.f * d[3] + d[5];
}

PSX_DEV void wino_at6(const float (&m)[6], float (&o)[4]) {
  const float a = m[1] + m[2], b = m[1] - m[2], c = m[3] + m[4], d = m[3] - m[4];
  o[0] = m[0] + a + c;
  o[1] = b + 2.f * d;
  o[2] = a + 4.f * c;
  o[3] = b + 8.f * d + m[5];
}

// one axis of A dy A^T (the dy transform of the weight gradient): 4 dy values -> 6
PSX_DEV void wino_a4(const float (&y)[4], float (&r)[6]) {
  const float e = y[0] + y[2], o = y[1] + y[3], e4 = y[0] + 4.f * y[2], o2 = 2.f * y[1] + 8.f * y[3];
  r[0] = y[0];
  r[1] = e + o;
  r[2] = e - o;
  r[3] = e4 + o2;
  r[4] = e4 - o2;
  r[5] = y[3];
}

PSX_DEV void wino_gt6(const float (&m)[6], float (&o)[3]) {
  const float a = m[1] + m[2], b = m[1] - m[2], c = m[3] + m[4], d = m[3] - m[4];
  o[0] = 0.25f * m[0] - a * (1.f / 6.f) + c * (1.f / 24.f);
  o[1] = -b * (1.f / 6.f) + d * (1.f / 12.f);
  o[2] = -a * (1.f / 6.f) + c * (1.f / 6.f) + m[5];
}

// Forward BN finalize descriptor (the layout of bnfin.hpp BnFin)
struct WinoBnFin {
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
  const float* sshift;  // shifted sums (bnfin.hpp BnFin::sshift)
  float* sshift_next;
  int det;  // fixed-point slot pairs (bnfin.hpp BnFin::det)
};

// Fused BN-backward sums over a data-gradient output (the layout of conv_v2.hip BwdStatsDesc):
// dz = g * [o > 0], slot rows [PSX_STAT_SLOTS][bns][K] of sum dz, sum dz * xhat1 (, * xhat2);
// mask_store: store dz instead of g.
struct WinoBwdStats {
  float* part;
  const float* o;
  const float* y1;
  const float* y2;
  const float* saved1;  // [2][K] mean, invstd
  const float* saved2;
  int mask_store;
  const float* mask_aff;  // nullable: ReLU mask = [y1 * scale + shift > 0] (affine [2][K]) instead of o
};


// BN-backward fold into a consumer's operand loads (wino_fused.hip data gradient, wino.hip dy
// transform): the coefficients of channel c from the consumer-producing dgrad's slot rows
// part[PSX_STAT_SLOTS][2][C] (row 0 sum dz, row 1 sum dz*xhat; fixed slot order, double), as
// bnfin.hpp bn_bwd_fin_lds: dx = k1 dz + k2 y + k3. Both consumers call this, so they read the
// same bits.
PSX_DEV void wino_bwd_coef(const float* part, const BnBwdFin& f, int c, float& k1, float& k2, float& k3, double& sdz,
                           double& sxh) {
  const int C = f.C;
  sdz = slot_sum<PSX_STAT_SLOTS>(part, c, 2 * (size_t)C, f.det);
  sxh = slot_sum<PSX_STAT_SLOTS>(part, (size_t)C + c, 2 * (size_t)C, f.det);
  const float mdz = (float)(sdz / f.count), mxh = (float)(sxh / f.count);
  const float is = f.invstd[c], gm = f.gamma[c];
  k1 = gm * is;
  k2 = -gm * is * is * mxh;
  k3 = -gm * is * mdz + gm * is * is * f.mean[c] * mxh;
}

// the folded operand: dx = k1 dz + k2 y + k3 (one rounding order for every consumer)
PSX_DEV float wino_bwd_apply(float dz, float y, float k1, float k2, float k3) { return fmaf(k1, dz, fmaf(k2, y, k3)); }

}  // namespace psx
