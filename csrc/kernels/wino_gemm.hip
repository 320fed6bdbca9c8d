// Stream-K fp32 batched NT GEMM for the Winograd layers whose 36 per-point GEMMs are too small to
// fill the chip in tiles (ResNet-18's 8x8x256 / 4x4x512: P[b] = V[b] . U[:, b, :]^T, 36 GEMMs of
// 512 x 256 x 256 / 128 x 512 x 512).
//
// Why: on those shapes every tiled launch is either a fraction of a round of 256 CUs or a pile of
// short-K workgroups whose pipeline fill (first loads ~2 us) rivals their MFMA time: the conv_v2
// mainloop (psx_bgemm_f32) and torch.bmm (hipBLASLt) both measure 64-72 TF on them, ~45 % of
// the 157 TF fp32 MFMA peak (bench/bgemm_f32.py). Here exactly G <= 256 workgroups (one per CU,
// four waves) split the flat list of (tile, 32-wide k-chunk) units evenly: a workgroup streams
// its units through one 3-stage LDS-DMA ring without draining it at tile boundaries, so the chip
// runs one balanced round at the mainloop's steady-state rate.
//
// Tile 128 x BN (BN = 128 or 64), 4 waves = 2 x 2 of 64 x BN/2, v_mfma_f32_32x32x2_f32 (exact
// fp32) on 32 x 32 blocks. One k-chunk = 32 floats = one 128-byte LDS row per operand row, the
// 16-byte chunks XOR-swizzled by row (the DMA source address carries the swizzle, the LDS side
// stays lane-linear). The reduction order inside a chunk is permuted so that each lane's operand
// run is contiguous: lane l (i = l & 31, h = l >> 5) feeds k = 16 h + j to the j-th MFMA, i.e.
// A[i][16h .. 16h + 15] — four ds_read_b128 per 32-row block per chunk, the same permutation on
// both operands. Within a unit the four quarters' fragments are double-buffered in registers (the
// next quarter's ds_reads go out before this quarter's 16 MFMAs).
//
// Tile ends: a unit range covers >= kc units (G <= units / kc), so a tile is split between at most
// two neighbouring workgroups — the head part ends workgroup w's range, the tail part starts
// w + 1's. Both store their partial (register order) into the workspace slot of w, fence, and
// count; the second to arrive adds the other's partial to its own (fp32 addition is commutative:
// head + tail bit-identical whoever arrives last, so results are run-to-run deterministic), stores
// the tile and re-zeroes the counter. Nobody waits on anybody: no spin, no co-residency
// assumption. Unsplit tiles are stored directly.
#include <stdlib.h>

#include <type_traits>

#include "pipeline.hpp"

namespace psx {

struct SkArgs {
  const float* A;  // A[b][m][k] at A + b * sa_b + m * sa_row + k
  const float* B;  // B[b][n][k] at B + b * sb_b + n * sb_row + k
  float* C;        // C[b][m][n] at C + b * sc_b + m * sc_row + n
  const float* zero;
  float* ws;      // [G][2][128 * BN]
  unsigned* cnt;  // [G], zero between launches
  long sa_row, sa_b, sb_row, sb_b, sc_row, sc_b;
  int M, N, Kd, nb;
  int tm, tn, kc, units, G;
};

// diagnostics builds only (wrong results; profiles/r4_sk_gemm_probes.jsonl): 1 no DMA, 2 no MFMA,
// 4 no flush, 8 no split hand-off, 16 no C stores
#ifndef PSX_SK_PROBE
#define PSX_SK_PROBE 0
#endif

constexpr int kSkBM = 128;
constexpr int kSkNS = 3;

// The XCD that runs remapped workgroup w of an nwg-workgroup launch (common.hpp xcd_remap: XCD x
// owns the contiguous range of w starting at its base).
PSX_DEV int xcd_of(int w, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  return w < r * (q + 1) ? w / (q + 1) : r + (w - r * (q + 1)) / q;
}

// ds_read_b128 outside hipcc's waitcnt tracking (pipeline.hpp ds_read128u, as fp32)
PSX_DEV f32x4 ds_read128(unsigned off) { return __builtin_bit_cast(f32x4, ds_read128u(off)); }

PSX_DEV f32x16 mfma32(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

template <int BN>
__global__ __launch_bounds__(256, 1) void sk_gemm_kernel(SkArgs a) {
  constexpr int BM = kSkBM, NS = kSkNS;
  constexpr int ROWS = BM + BN, STAGE = ROWS * 128;
  constexpr int LPW = ROWS / 32;  // DMA instructions per wave per stage (8 rows each, 4 waves)
  constexpr int WN = BN / 2, NBK = WN / 32, MBK = 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int w = xcd_remap(blockIdx.x, a.G);
  const int u0 = (int)((long)w * a.units / a.G), u1 = (int)((long)(w + 1) * a.units / a.G);
  const int n = u1 - u0;

  // DMA lane state: instruction i covers rows (4 i + wid) * 8 + (lane >> 3), 16-byte slot lane & 7
  long off[LPW];
  int rowi[LPW];
#pragma unroll
  for (int i = 0; i < LPW; ++i) {
    const int r = (i * 4 + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);  // the logical chunk this slot holds
    rowi[i] = r;
    off[i] = r < BM ? (long)r * a.sa_row + c * 4 : (long)(r - BM) * a.sb_row + c * 4;
  }
  auto issue = [&](int u, int slot) {
    if (PSX_SK_PROBE & 1) return;
    const int t = __builtin_amdgcn_readfirstlane(u / a.kc);
    const int ch = u - t * a.kc;
    const int bt = __builtin_amdgcn_readfirstlane(t / (a.tm * a.tn));
    const int rem = t - bt * a.tm * a.tn;
    const int mt = rem / a.tn, nt = rem - (rem / a.tn) * a.tn;
    const float* pa = a.A + bt * a.sa_b + (long)mt * BM * a.sa_row + ch * 32;
    const float* pb = a.B + bt * a.sb_b + (long)nt * BN * a.sb_row + ch * 32;
    unsigned char* base = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < LPW; ++i) {
      const float* src;
      if (rowi[i] < BM)  // wave-uniform per instruction (8-row groups never straddle BM)
        src = mt * BM + rowi[i] < a.M ? pa + off[i] : a.zero;
      else
        src = pb + off[i];
      glds16(src, base + (i * 4 + wid) * 1024);
    }
  };

  // fragment reads: block rows of this wave, lane row i, logical chunks 4 h .. 4 h + 3
  const int fi = lane & 31, fh = lane >> 5;
  int aro[MBK], bro[NBK];
#pragma unroll
  for (int m = 0; m < MBK; ++m) aro[m] = (wm * 64 + m * 32 + fi) * 128;
#pragma unroll
  for (int q = 0; q < NBK; ++q) bro[q] = (BM + wn * WN + q * 32 + fi) * 128;
  const int sw = fi & 7;  // row & 7 (block rows start at multiples of 32)
  // quarter q of a unit's fragments: logical chunk 4 h + q of every block row (k = 16 h + 4 q + e)
  auto readq = [&](int slot, int q, f32x4(&fa)[MBK], f32x4(&fb)[NBK]) {
    const unsigned char* base = smem + slot * STAGE;
    const int so = (((fh * 4 + q) ^ sw) << 4);
#pragma unroll
    for (int m = 0; m < MBK; ++m) fa[m] = *reinterpret_cast<const f32x4*>(base + aro[m] + so);
#pragma unroll
    for (int b = 0; b < NBK; ++b) fb[b] = *reinterpret_cast<const f32x4*>(base + bro[b] + so);
  };

  f32x16 acc[MBK][NBK];
  auto zero_acc = [&]() {
#pragma unroll
    for (int m = 0; m < MBK; ++m)
#pragma unroll
      for (int b = 0; b < NBK; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][b][r] = 0.f;
  };
  zero_acc();

  auto mmaq = [&](const f32x4(&fa)[MBK], const f32x4(&fb)[NBK]) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int m = 0; m < MBK; ++m)
#pragma unroll
        for (int b = 0; b < NBK; ++b) acc[m][b] = mfma32(fb[b][e], fa[m][e], acc[m][b]);  // C^T: lane = row of C
  };

  // tile store / split-tile fixup of the segment ending at unit u (inclusive)
  __shared__ int sk_flag;
  auto flush = [&](int u, int seg0) {
    const int t = u / a.kc;
    const bool head = seg0 % a.kc == 0, tail = (u + 1) % a.kc == 0;
    const int bt = t / (a.tm * a.tn), rem = t - bt * a.tm * a.tn;
    const int mt = rem / a.tn, nt = rem - (rem / a.tn) * a.tn;
    if (!(head && tail) && !(PSX_SK_PROBE & 8)) {
      // The partials cross workgroups, possibly XCDs (each XCD has its own L2): they are written
      // through to memory (sc0 sc1 stores) and read past the L2 (sc0 sc1 loads), so no
      // whole-cache writeback / invalidate fence is needed (an agent-scope release / acquire
      // compiles to buffer_wbl2 / buffer_inv of the entire L2: ~60 us for a 256-workgroup launch).
      const int slot = head ? w : w - 1;  // head part ends w's range; the tail part starts w+1's
      const auto mr = __builtin_amdgcn_make_buffer_rsrc(a.ws + ((long)slot * 2 + (head ? 0 : 1)) * BM * BN, 0,
                                                         BM * BN * 4, 0x00020000);
      const auto orr = __builtin_amdgcn_make_buffer_rsrc(a.ws + ((long)slot * 2 + (head ? 1 : 0)) * BM * BN, 0,
                                                          BM * BN * 4, 0x00020000);
      // partners on one XCD share its L2: stores land there (the CU's L1 is write-through) and
      // sc0 loads skip the reader's L1, so the hand-off never leaves the L2. Partners on two XCDs
      // (7 of the 255 neighbour pairs: xcd_remap gives each XCD a contiguous range of w) go
      // through memory: sc0 | sc1 = write-through / miss-always.
      const bool cross = xcd_of(slot, a.G) != xcd_of(slot + 1, a.G);
#pragma unroll
      for (int m = 0; m < MBK; ++m)
#pragma unroll
        for (int b = 0; b < NBK; ++b)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const int idx = (((wid * MBK + m) * NBK + b) * 4 + r4) * 64 + lane;
            const f32x4 v = {acc[m][b][4 * r4], acc[m][b][4 * r4 + 1], acc[m][b][4 * r4 + 2], acc[m][b][4 * r4 + 3]};
            if (cross)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), mr, idx * 16, 0, 1 | 16);
            else
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), mr, idx * 16, 0, 0);
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.cnt + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sk_flag = (int)old;
      }
      __syncthreads();
      const int second = sk_flag;
      __syncthreads();
      if (!second) return;  // the partner adds ours
      asm volatile("" ::: "memory");
#pragma unroll
      for (int m = 0; m < MBK; ++m)
#pragma unroll
        for (int b = 0; b < NBK; ++b)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const int idx = (((wid * MBK + m) * NBK + b) * 4 + r4) * 64 + lane;
            const f32x4 o = __builtin_bit_cast(
                f32x4, cross ? __builtin_amdgcn_raw_buffer_load_b128(orr, idx * 16, 0, 1 | 16)
                             : __builtin_amdgcn_raw_buffer_load_b128(orr, idx * 16, 0, 1));
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[m][b][4 * r4 + e] += o[e];
          }
      if (threadIdx.x == 0) __hip_atomic_store(a.cnt + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (PSX_SK_PROBE & 16) return;
    // the accumulators hold C^T blocks (the B operand's rows on the MFMA's row axis): a lane owns
    // one row of C (its tile) and each register quad four consecutive columns, so the tile goes
    // out as 16-byte stores
    float* cb = a.C + bt * a.sc_b;
#pragma unroll
    for (int m = 0; m < MBK; ++m) {
      const int row = mt * BM + wm * 64 + m * 32 + fi;
      if (row >= a.M) continue;
#pragma unroll
      for (int b = 0; b < NBK; ++b)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int col = nt * BN + wn * WN + b * 32 + 8 * r4 + 4 * fh;
          *reinterpret_cast<f32x4*>(cb + (long)row * a.sc_row + col) =
              (f32x4){acc[m][b][4 * r4], acc[m][b][4 * r4 + 1], acc[m][b][4 * r4 + 2], acc[m][b][4 * r4 + 3]};
        }
    }
  };

  // prologue: units 0 and 1 in flight
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < n) issue(u0 + s, s);
  // one unit: its DMA landed (its successor's may still fly), barrier (every wave is done with
  // the slot of unit k - 1), refill that slot with unit k + 2, then the unit's four quarters with
  // the next quarter's fragments read before this quarter's MFMAs
  auto step = [&](int k) {
    if (k + 1 < n)
      wait_vmcnt<LPW>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + 2 < n) issue(u0 + k + 2, (k + 2) % NS);
    const int slot = k % NS;
    // the unit's fragment reads go out ahead (inline asm: hipcc does not count them; <= 12 in
    // flight), quarter q waits only for its own (LDS retires in order):
    // hipcc's own waitcnt placement put an lgkmcnt(0) in front of every MFMA group, exposing the
    // read latency of the next group's prefetch each time
    const unsigned lbase = lds_off(smem) + slot * STAGE;
    f32x4 fa[4][MBK], fb[4][NBK];
    auto rq = [&](int q) {
      const unsigned so = (((fh * 4 + q) ^ sw) << 4);
#pragma unroll
      for (int m = 0; m < MBK; ++m) fa[q][m] = ds_read128(lbase + aro[m] + so);
#pragma unroll
      for (int b = 0; b < NBK; ++b) fb[q][b] = ds_read128(lbase + bro[b] + so);
    };
    constexpr int RQ = MBK + NBK;  // reads per quarter; at most 3 quarters (<= 12) in flight
    rq(0);
    rq(1);
    rq(2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < 2) lgkm_wait<2 * RQ>();
      if (q == 2) lgkm_wait<RQ>();
      if (q == 3) lgkm_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
      if (!(PSX_SK_PROBE & 2)) mmaq(fa[q], fb[q]);
      __builtin_amdgcn_sched_barrier(0);
      if (q == 0) rq(3);
    }
  };
  // segments = the parts of tiles in this range; the accumulators stay in the MFMA registers
  // across a segment's units (no flush inside the inner loop)
  int k = 0;
  while (k < n) {
    const int seg0 = u0 + k;
    const int kend = min(n, k + (a.kc - seg0 % a.kc));
    for (; k < kend; ++k) step(k);
    if (!(PSX_SK_PROBE & 4)) flush(u0 + k - 1, seg0);
    zero_acc();
  }
}

float* g_ws = nullptr;
unsigned* g_cnt = nullptr;
long g_ws_floats = 0;
int g_ncnt = 0;

template <int BN>
int sk_plan(int M, int N, int Kd, int nb, SkArgs& a) {
  if (N % BN || Kd % 32) return -1;
  a.tm = (M + kSkBM - 1) / kSkBM;
  a.tn = N / BN;
  a.kc = Kd / 32;
  const long tiles = (long)nb * a.tm * a.tn;
  a.units = (int)(tiles * a.kc);
  // one workgroup per CU; PSX_SK_G: more (two per CU fit the 64-wide tile's 72 KB of LDS)
  static const int gmax = [] {
    const char* e = getenv("PSX_SK_G");
    return e && atoi(e) > 0 ? atoi(e) : 256;
  }();
  a.G = (int)(tiles < gmax ? tiles : gmax);
  return a.G;
}

}  // namespace psx

using namespace psx;

extern "C" {

// The fixup workspace (>= 256 * 2 * 128 * 128 floats) and counters (>= 256, zeroed): set once by
// the engine (models/engine.py) before any capture; unset, psx_sk_gemm_nt returns -5 and callers
// keep their tiled path.
int psx_sk_set_workspace(float* ws, long ws_floats, unsigned* cnt, int ncnt) {
  g_ws = ws;
  g_ws_floats = ws_floats;
  g_cnt = cnt;
  g_ncnt = ncnt;
  return 0;
}

long psx_sk_workspace_floats() { return 256L * 2 * kSkBM * 128; }

// nb batched C[b] = A[b] . B[b]^T (see SkArgs for the strides); Kd a multiple of 32, N of 64.
// bn: 0 = the plan's choice (the tile width giving the most workgroups, 128 on ties), else 64 / 128.
int psx_sk_gemm_nt(const float* A, const float* B, float* C, long sa_row, long sa_b, long sb_row, long sb_b,
                   long sc_row, long sc_b, int M, int N, int Kd, int nb, const void* zero, int bn, hipStream_t st) {
  if (!g_ws || g_ws_floats < psx_sk_workspace_floats() || g_ncnt < 256) return -5;
  if (M < 1 || nb < 1 || Kd < 32) return -2;
  // 16-byte DMA sources and 16-byte C stores
  if ((sa_row | sa_b | sb_row | sb_b | sc_row | sc_b) & 3) return -2;
  if (((size_t)A | (size_t)B | (size_t)C) & 15) return -2;
  SkArgs a{};
  a.A = A; a.B = B; a.C = C; a.zero = (const float*)zero; a.ws = g_ws; a.cnt = g_cnt;
  a.sa_row = sa_row; a.sa_b = sa_b; a.sb_row = sb_row; a.sb_b = sb_b; a.sc_row = sc_row; a.sc_b = sc_b;
  a.M = M; a.N = N; a.Kd = Kd; a.nb = nb;
  SkArgs a128 = a, a64 = a;
  const int g128 = sk_plan<128>(M, N, Kd, nb, a128), g64 = sk_plan<64>(M, N, Kd, nb, a64);
  int use = bn;
  if (!use) use = g128 >= g64 && g128 > 0 ? 128 : 64;
  if (const char* e = getenv("PSX_SK_BN"); e && atoi(e) > 0) use = atoi(e);
  const SkArgs& p = use == 128 ? a128 : a64;
  if ((use == 128 ? g128 : g64) < 1) return -2;
  if (p.units / p.G < p.kc) return -3;  // a tile would span three workgroups
  if (use == 128)
    hipLaunchKernelGGL(sk_gemm_kernel<128>, dim3(p.G), dim3(256), (size_t)kSkNS * (kSkBM + 128) * 128, st, p);
  else
    hipLaunchKernelGGL(sk_gemm_kernel<64>, dim3(p.G), dim3(256), (size_t)kSkNS * (kSkBM + 64) * 128, st, p);
  return (int)hipGetLastError();
}

}  // extern "C"
