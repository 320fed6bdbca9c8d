// Top-k gradient sparsification with error feedback (the BASELINE.json "top-k grad compression"
// codec; the reference only casts to fp16, src/workers/worker.py:264-268).
//
// Worker side, one push:
//   acc   = resid + g                        (error feedback: what was not sent last time)
//   T     = k-th largest |acc|               (exact, radix select on the 31 magnitude bits)
//   send    { (i, fp16(acc[i])) : |acc[i]| > T } + enough |acc[i]| == T ties to make exactly k
//   resid = acc - sent                       (incl. the fp16 rounding error of sent values)
//
// Two passes over the gradient, five launches, no host round trip (stream-ordered,
// graph-capturable):
//   A  (1024 chunks, four per 1024-thread workgroup — one workgroup per CU, one 256-thread group
//      per chunk) acc = resid + g in place and a 4096-bin LDS histogram per chunk of the top 12
//      magnitude bits (exponent + 4 mantissa bits), kept as the chunk's suffix sums and flushed
//      to 16 global copies (chunk-group & 15: 256 same-address atomics per bin serialise at the
//      memory side) with sparse atomics;
//   S  (one workgroup) the bin b0 holding the k-th largest;
//   B  (1024 workgroups of 256 threads, the same chunks) sums its chunk's bases from the rows
//      (counts above b0 — "sure" — and inside it — "candidates" — of the preceding chunks), writes
//      the sure entries to the payload in index order (ranks from wave ballots plus one
//      cross-wave prefix per tile; resid -= fp16 value), compacts the candidates (index, acc) in
//      index order and histograms their remaining 19 bits: 1024 coarse bins (bits 18..9, LDS,
//      flushed to 8 copies) and the full 2^19 fine bins (global atomics);
//   Rc (256 workgroups over the candidates) every workgroup finds the exact threshold T from the
//      two histograms (coarse bin, then its 512 fine bins) and counts its range's candidates
//      above T and equal to T;
//   Rw (same) appends its selected candidates in index order (base = prefix of the preceding
//      ranges' counts; ties at T taken lowest index first), updates resid, clears the histograms
//      and writes the header.
// With error feedback the unsent mass piles up just below the threshold (10x the candidates of a
// Gaussian), so the candidate stage is grid-parallel. Deterministic: positions come from ordered
// scans, never from same-address atomics. The previous encoder made three full histogram passes
// + count / scan / write (5 passes, 11 launches). Round 6 (ResNet-18 step, 11.2 M values: 91 ->
// ~75 us): pipelined loads without exec-masked fallbacks (full vmcnt waits before), histogram
// copies, bases summed in B instead of S; profiles/r6_topk_*.
//
// Payload (int32 words): [count, kcap, n, 0 | idx[kcap] | fp16 val[kcap] (packed)]
// Server side: dst[idx] += scale * val (decode into a dense fp32 buffer, or straight into the
// fp32 master parameters with scale = -lr * weight when there is no optimizer state).
#include <type_traits>

#include "common.hpp"

namespace psx {

enum { TK_KREM = 0, TK_B0 = 1, TK_CNTGT = 2, TK_NC = 3, TK_T = 4, TK_NEED = 5, TK_STATE_WORDS = 16 };
constexpr int TK_RB = 256;                 // workgroups of the candidate stage
constexpr int TK_FINE = 1 << 19;           // fine bins: magnitude bits 18..0
constexpr int TK_NB0 = 4096, TK_SH0 = 19;  // first-level bins: magnitude bits 30..19
constexpr int TK_MAXBLK = 1024;            // chunks of passes A / B
constexpr int TK_ROW = TK_NB0 + 1;         // per-chunk suffix row (entry 4096 = 0)
// The global histograms are spread over copies (chunk & (copies - 1)): every chunk finishes at
// about the same time, and 256 same-address atomics per bin serialise at the memory side (pass A
// 37 -> 22.5 us without them at ResNet-18 size); the consumers sum the copies.
constexpr int TK_HCOPY = 16;               // copies of the 4096-bin histogram (pass A -> S)
constexpr int TK_CCOPY = 8;                // copies of the candidates' 1024-bin histogram (B -> Rc)

PSX_DEV uint32_t mag_key(float a) { return __float_as_uint(a) & 0x7fffffffu; }

// exclusive scan of v over the workgroup in thread order (NT threads); *total = the sum
template <int NT>
PSX_DEV uint32_t tk_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const uint32_t x = wsum[i];
    if (i < w) base += x;
    tot += x;
  }
  __syncthreads();  // wsum reusable
  *total = tot;
  return base + incl - v;
}

PSX_DEV uint16_t tk_half(float a) {
  return __builtin_bit_cast(uint16_t, (_Float16)fminf(fmaxf(a, -65504.f), 65504.f));
}

template <typename GT>
PSX_DEV float tk_load_g(const GT* g, long i) {
  if constexpr (sizeof(GT) == 2) return (float)reinterpret_cast<const _Float16*>(g)[i];
  else return (float)g[i];
}

// S: one workgroup of 1024 threads. The bin b0 holding the k-th largest, summing the histogram
// copies; clears them for the next encode. (Each pass-B workgroup sums its chunk's bases from the
// rows itself: done here, the 1024 dependent row reads and scans made this launch 10 us. Run by
// pass A's last-arriving workgroup instead, A measured 47 us vs 30 + 7 here.)
__global__ __launch_bounds__(1024) void tk_select0(uint32_t* __restrict__ ghist, uint32_t* __restrict__ state, int k) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t sb[2];
  const int t = threadIdx.x;
  // thread t owns bins 4095 - 4 t - j (j < 4): the 16-byte word at bin 4092 - 4 t of every copy
  u32x4 cv = {0u, 0u, 0u, 0u};
  u32x4* const hv = reinterpret_cast<u32x4*>(ghist) + (TK_NB0 / 4 - 1 - t);
#pragma unroll
  for (int h = 0; h < TK_HCOPY; ++h) cv += hv[h * (TK_NB0 / 4)];
  uint32_t c[4] = {cv[3], cv[2], cv[1], cv[0]}, local = c[0] + c[1] + c[2] + c[3];
  if (t == 0) sb[0] = sb[1] = 0;
  uint32_t tot;
  uint32_t above = tk_excl_scan<1024>(local, wsum, &tot);
  const uint32_t kk = (uint32_t)k;
  if (above < kk && above + local >= kk) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (above + c[j] >= kk) {
        sb[0] = (uint32_t)(TK_NB0 - 1 - (4 * t + j));
        sb[1] = above;
        break;
      }
      above += c[j];
    }
  }
  __syncthreads();
  const uint32_t b0 = sb[0], cnt_gt = sb[1];
#pragma unroll
  for (int h = 0; h < TK_HCOPY; ++h) hv[h * (TK_NB0 / 4)] = u32x4{0u, 0u, 0u, 0u};
  if (t == 0) {
    state[TK_KREM] = kk - cnt_gt;
    state[TK_B0] = b0;
    state[TK_CNTGT] = cnt_gt;
  }
}

// Pass A: acc = resid + g (g may be null), 4096-bin histogram -> global + per-chunk suffix rows.
// One workgroup of 1024 threads per CU runs four chunks, one per 256-thread group (LDS histogram
// copy = group): pass B runs the same chunks as 256-thread workgroups (its per-tile rank barrier
// is cheaper over 4 waves than over 16), while 256-thread workgroups here measured 2.5x slower
// (65 vs 26 us at ResNet-18 size: four times the workgroup epilogues and LDS clears per CU).
template <typename GT, bool HASG>
__global__ __launch_bounds__(1024) void tk_pass_a(const GT* __restrict__ g, float* __restrict__ resid, long n,
                                                  long chunk, uint32_t* __restrict__ ghist,
                                                  uint32_t* __restrict__ rows) {
  constexpr int NT = 256, TILE = 4 * NT;  // per group; a tile = 4 consecutive elements per thread
  __shared__ uint32_t lh4[4 * TK_NB0];
  __shared__ uint32_t wsum[16];
  for (int i = threadIdx.x; i < 4 * TK_NB0; i += 1024) lh4[i] = 0;
  __syncthreads();
  const int gq = threadIdx.x >> 8, t = threadIdx.x & (NT - 1);
  const int vb = 4 * blockIdx.x + gq;  // this group's chunk
  uint32_t* const lh = lh4 + gq * TK_NB0;
  const long lo = (long)vb * chunk;
  const long hi = lo + chunk < n ? lo + chunk : n;
  // Full tiles (no bounds checks, so no exec-masked fallback loads that force a full vmcnt wait),
  // PF of them in flight: the loop is unrolled by PF and tile u's registers are refilled (tile
  // u + PF) right after they are consumed, so the loads stay queued behind the atomics; the
  // chunk's partial last tile (the last chunk only) after the loop.
  constexpr int PF = 3;
  constexpr bool hasg = HASG;  // compile-time: a runtime flag leaves register merges (copies of
                               // tiles still in flight) in the loop
  const long nfull = hi > lo ? (hi - lo) / TILE : 0;
  using GV = std::conditional_t<sizeof(GT) == 2, u32x2, f32x4>;  // raw g in the ring (fp16: converted
                                                                 // when consumed, not when loaded)
  auto load = [&](long i, f32x4& r, GV& gv) {
    r = *reinterpret_cast<const f32x4*>(resid + i);
    if constexpr (hasg) gv = *reinterpret_cast<const GV*>(g + i);
  };
  auto consume = [&](const f32x4& rv, const GV& gv, long i) {
    f32x4 r = rv;
    if constexpr (hasg) {
      if constexpr (sizeof(GT) == 2) {
        const _Float16* hp = reinterpret_cast<const _Float16*>(&gv);
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] += (float)hp[e];
      } else {
        r += gv;
      }
      *reinterpret_cast<f32x4*>(resid + i) = r;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(&lh[mag_key(r[e]) >> TK_SH0], 1u);
  };
  // groups of PF tiles with straight-line bodies (the last group's refills re-load its own tiles,
  // unused): a skipped refill would leave the wait counter's bookkeeping with a full wait
  const long ng = nfull / PF;
  f32x4 br[PF];
  GV bg[PF];
  if (ng > 0) {
#pragma unroll
    for (int u = 0; u < PF; ++u) load(lo + (long)u * TILE + 4 * t, br[u], bg[u]);
  }
  for (long gi = 0; gi < ng; ++gi) {
    const long nxt = gi + 1 < ng ? PF * TILE : 0;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const long i = lo + (gi * PF + u) * TILE + 4 * t;
      const f32x4 r = br[u];
      const GV gv = bg[u];
      load(i + nxt, br[u], bg[u]);
      consume(r, gv, i);
      // keep the refill here: hoisted to the top of the body, the scheduler would have to wait
      // for every tile in flight before overwriting their registers
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (long tt = ng * PF; tt < nfull; ++tt) {  // leftover full tiles
    f32x4 r;
    GV gv;
    const long i = lo + tt * TILE + 4 * t;
    load(i, r, gv);
    consume(r, gv, i);
  }
  for (long i = lo + nfull * TILE + t; i < hi; i += NT) {  // partial tile
    float a = resid[i];
    if (hasg) {
      a += tk_load_g(g, i);
      resid[i] = a;
    }
    atomicAdd(&lh[mag_key(a) >> TK_SH0], 1u);
  }
  __syncthreads();
  // the group's suffix row, descending bins: thread t owns bins 4095 - 16 t - j (j < 16); the
  // exclusive scan runs over the group's 4 waves
  constexpr int BT = TK_NB0 / NT;
  uint32_t c[BT], local = 0;
#pragma unroll
  for (int j = 0; j < BT; ++j) {
    c[j] = lh[TK_NB0 - 1 - (BT * t + j)];
    local += c[j];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o, 64);
    if (lane >= o) incl += x;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t above = incl - local;
  for (int i = gq * 4; i < w; ++i) above += wsum[i];
  uint32_t* row = rows + (size_t)vb * TK_ROW;
#pragma unroll
  for (int j = 0; j < BT; ++j) {
    above += c[j];
    row[TK_NB0 - 1 - (BT * t + j)] = above;  // # elements of this chunk in bins >= bin
  }
  if (t == 0) row[TK_NB0] = 0;
  // the global histogram: the four groups' counts summed, one atomic per non-empty bin
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = 4 * (int)threadIdx.x + j;
    const uint32_t v = lh4[b] + lh4[TK_NB0 + b] + lh4[2 * TK_NB0 + b] + lh4[3 * TK_NB0 + b];
    if (v) atomicAdd(&ghist[(blockIdx.x & (TK_HCOPY - 1)) * TK_NB0 + b], v);
  }
}


// B: sure entries -> payload (index order), candidates -> (cidx, cval) (index order) + their
// coarse / fine histograms. Tiles of 4096 elements, 4 consecutive ones per thread (one 16-byte
// load, three tiles in flight ahead); an element's rank = the preceding waves' counts (one
// cross-wave prefix per tile, double-buffered so one barrier suffices) + the wave's ballots below
// it + its own earlier flags.
__global__ __launch_bounds__(256) void tk_pass_b(float* __restrict__ resid, long n, long chunk,
                                                   uint32_t* __restrict__ state,
                                                   const uint32_t* __restrict__ rows, int* __restrict__ payload,
                                                   int kcap, int* __restrict__ cidx, float* __restrict__ cval,
                                                   uint32_t* __restrict__ coarse, uint32_t* __restrict__ fine) {
  constexpr int TK_NT = 256, NW = TK_NT / 64, TK_TILE = 4 * TK_NT;
  __shared__ uint32_t wsum[2][NW];
  __shared__ uint32_t lh[1024];
  for (int i = threadIdx.x; i < 1024; i += TK_NT) lh[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t b0 = state[TK_B0];
  int* idx = payload + 4;
  uint16_t* val = reinterpret_cast<uint16_t*>(payload + 4 + kcap);
  const long lo = (long)blockIdx.x * chunk;
  const long hi = lo + chunk < n ? lo + chunk : n;
  // this chunk's payload / candidate bases: the preceding chunks' counts above b0 and in b0 (their
  // suffix rows at b0 + 1 and b0); the last chunk also publishes the candidate total
  uint32_t rs = 0, rc = 0;
  {
    const int vb = blockIdx.x;
    const bool last = vb == (int)gridDim.x - 1;
    uint32_t s1 = 0, s0 = 0;
    for (int c = threadIdx.x; c < vb || (last && c == vb); c += TK_NT) {
      const uint32_t* row = rows + (size_t)c * TK_ROW;
      s1 += row[b0 + 1];
      s0 += row[b0];
    }
    // (each count < 2^31: the chunk sums of s1 and of s0 - s1 fit; reduce both packed as 64-bit)
    unsigned long long v = ((unsigned long long)(s0 - s1) << 32) | s1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __shared__ unsigned long long bred[NW];
    if (lane == 0) bred[w] = v;
    __syncthreads();
    v = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) v += bred[j];
    if (last) {  // v includes this chunk: the candidate total
      if (threadIdx.x == 0) state[TK_NC] = (uint32_t)(v >> 32);
      const uint32_t* row = rows + (size_t)vb * TK_ROW;
      v -= ((unsigned long long)(row[b0] - row[b0 + 1]) << 32) | row[b0 + 1];
    }
    rs = (uint32_t)v;
    rc = (uint32_t)(v >> 32);
  }
  int it = 0;
  // one tile: a = this thread's 4 elements at i0 (in = the first nin of them exist)
  auto tile = [&](const f32x4& a, long i0, int nin) {
    uint32_t fs = 0, fc = 0;  // per-element flags (bit e): sure / candidate
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool in = e < nin;
      const uint32_t bin = mag_key(a[e]) >> TK_SH0;
      fs |= (uint32_t)(in && bin > b0) << e;
      fc |= (uint32_t)(in && bin == b0) << e;
    }
    uint32_t ws = 0, wc = 0, ts = 0, tc = 0;  // this lane's rank in the wave, the wave's totals
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned long long bs = __ballot((fs >> e) & 1u), bc = __ballot((fc >> e) & 1u);
      ws += __popcll(bs & below);
      wc += __popcll(bc & below);
      ts += __popcll(bs);
      tc += __popcll(bc);
    }
    if (lane == 0) wsum[it][w] = ts | (tc << 16);
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const uint32_t x = wsum[it][j];
      pre += j < w ? x : 0u;
      tot += x;
    }
    it ^= 1;
    uint32_t ps = rs + (pre & 0xffffu) + ws, pc = rc + (pre >> 16) + wc;
    rs += tot & 0xffffu;
    rc += tot >> 16;
    if (fs | fc) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long i = i0 + e;
        if ((fs >> e) & 1u) {
          if (ps < (uint32_t)kcap) {
            const uint16_t h = tk_half(a[e]);
            idx[ps] = (int)i;
            val[ps] = h;
            resid[i] = a[e] - (float)__builtin_bit_cast(_Float16, h);
          }
          ++ps;
        } else if ((fc >> e) & 1u) {
          const uint32_t key = mag_key(a[e]);
          cidx[pc] = (int)i;
          cval[pc] = a[e];
          ++pc;
          atomicAdd(&lh[(key >> 9) & 1023u], 1u);
          atomicAdd(&fine[key & (TK_FINE - 1)], 1u);
        }
      }
    }
  };
  // full tiles, PF in flight (unrolled ring without bounds checks, as in pass A), then the partial one
  constexpr int PF = 3;
  const long nfull = hi > lo ? (hi - lo) / TK_TILE : 0;
  const long ng = nfull / PF;
  f32x4 nx[PF];
  if (ng > 0) {
#pragma unroll
    for (int u = 0; u < PF; ++u) nx[u] = *reinterpret_cast<const f32x4*>(resid + lo + (long)u * TK_TILE + 4 * threadIdx.x);
  }
  for (long gi = 0; gi < ng; ++gi) {
    const long nxt = gi + 1 < ng ? PF * TK_TILE : 0;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const long i0 = lo + (gi * PF + u) * TK_TILE + 4 * threadIdx.x;
      const f32x4 a = nx[u];
      nx[u] = *reinterpret_cast<const f32x4*>(resid + i0 + nxt);
      tile(a, i0, 4);
      __builtin_amdgcn_sched_barrier(0);  // (see pass A)
    }
  }
  for (long tt = ng * PF; tt < nfull; ++tt) {  // leftover full tiles
    const long i0 = lo + tt * TK_TILE + 4 * threadIdx.x;
    tile(*reinterpret_cast<const f32x4*>(resid + i0), i0, 4);
  }
  if (lo + nfull * TK_TILE < hi) {
    const long i0 = lo + nfull * TK_TILE + 4 * threadIdx.x;
    f32x4 a;
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = i0 + e < hi ? resid[i0 + e] : 0.f;
    const long left = hi - i0;
    tile(a, i0, left <= 0 ? 0 : left >= 4 ? 4 : (int)left);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += TK_NT)
    if (lh[i]) atomicAdd(&coarse[(blockIdx.x & (TK_CCOPY - 1)) * 1024 + i], lh[i]);
}

PSX_DEV void tk_crange(uint32_t nc, uint32_t& lo, uint32_t& hi) {
  const uint32_t per = (nc + TK_RB - 1) / TK_RB;
  lo = blockIdx.x * per;
  hi = lo + per < nc ? lo + per : nc;
  if (lo > hi) lo = hi;
}

// Rc: exact threshold (every workgroup, from the histograms) + this range's > T / == T counts.
__global__ __launch_bounds__(256) void tk_refine_count(const float* __restrict__ cval, uint32_t* __restrict__ state,
                                                       const uint32_t* __restrict__ coarse,
                                                       const uint32_t* __restrict__ fine,
                                                       uint32_t* __restrict__ counts) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t sb[4];
  const int t = threadIdx.x;
  const uint32_t nc = state[TK_NC], b0 = state[TK_B0];
  const uint32_t krem = state[TK_KREM];
  if (t == 0) sb[0] = sb[1] = sb[2] = sb[3] = 0;
  // coarse bins, descending: thread t owns 1023 - 4t - j
  uint32_t c[4], local = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = 0;
#pragma unroll
    for (int h = 0; h < TK_CCOPY; ++h) c[j] += coarse[h * 1024 + 1023 - (4 * t + j)];
    local += c[j];
  }
  uint32_t tot;
  uint32_t above = tk_excl_scan<256>(local, wsum, &tot);
  if (above < krem && above + local >= krem) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (above + c[j] >= krem) {
        sb[0] = 1023u - (4 * t + j);
        sb[1] = above;
        break;
      }
      above += c[j];
    }
  }
  __syncthreads();
  const uint32_t b1 = sb[0], k1 = krem - sb[1];
  // fine bins of coarse bin b1, descending: thread t owns 511 - 2t - j
  uint32_t f[2];
  local = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    f[j] = fine[(b1 << 9) | (511u - (2 * t + j))];
    local += f[j];
  }
  above = tk_excl_scan<256>(local, wsum, &tot);
  if (above < k1 && above + local >= k1) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (above + f[j] >= k1) {
        sb[2] = 511u - (2 * t + j);
        sb[3] = above;
        break;
      }
      above += f[j];
    }
  }
  __syncthreads();
  const uint32_t T = (b0 << TK_SH0) | (b1 << 9) | sb[2];
  if (blockIdx.x == 0 && t == 0) {
    state[TK_T] = T;
    state[TK_NEED] = k1 - sb[3];  // ties at T to take (>= 1)
  }
  uint32_t lo, hi;
  tk_crange(nc, lo, hi);
  uint32_t ng = 0, ne = 0;
  for (uint32_t i = lo + t; i < hi; i += 256) {
    const uint32_t key = mag_key(cval[i]);
    ng += key > T;
    ne += key == T;
  }
  uint32_t tg, te;
  tk_excl_scan<256>(ng, wsum, &tg);
  tk_excl_scan<256>(ne, wsum, &te);
  if (t == 0) {
    counts[2 * blockIdx.x] = tg;
    counts[2 * blockIdx.x + 1] = te;
  }
}

// Rw: ordered append of the selected candidates of this range; clears the histograms.
__global__ __launch_bounds__(256) void tk_refine_write(float* __restrict__ resid, const int* __restrict__ cidx,
                                                       const float* __restrict__ cval,
                                                       const uint32_t* __restrict__ state,
                                                       const uint32_t* __restrict__ counts, int* __restrict__ payload,
                                                       int kcap, long n, int k, uint32_t* __restrict__ coarse,
                                                       uint32_t* __restrict__ fine) {
  __shared__ uint32_t wsum[4];
  const int t = threadIdx.x;
  const uint32_t nc = state[TK_NC], T = state[TK_T], need = state[TK_NEED], cnt_gt = state[TK_CNTGT];
  // bases: # > T and # == T in the preceding ranges (one value per thread, TK_RB == 256)
  const bool prev = (uint32_t)t < blockIdx.x;
  uint32_t sg, se;
  tk_excl_scan<256>(prev ? counts[2 * t] : 0u, wsum, &sg);
  tk_excl_scan<256>(prev ? counts[2 * t + 1] : 0u, wsum, &se);
  uint32_t lo, hi;
  tk_crange(nc, lo, hi);
  // selected before this range = # > T + min(# == T, need) over the preceding ranges
  uint32_t run_sel = sg + (se < need ? se : need), run_tie = se;
  int* idx = payload + 4;
  uint16_t* val = reinterpret_cast<uint16_t*>(payload + 4 + kcap);
  for (uint32_t base = lo; base < hi; base += 256) {
    const uint32_t i = base + t;
    const bool in = i < hi;
    const float a = in ? cval[i] : 0.f;
    const uint32_t key = mag_key(a);
    const bool gt = in && key > T, eq = in && key == T;
    uint32_t teq, tsel;
    const uint32_t tie = run_tie + tk_excl_scan<256>(eq ? 1u : 0u, wsum, &teq);
    const bool sel = gt || (eq && tie < need);
    const uint32_t pos = cnt_gt + run_sel + tk_excl_scan<256>(sel ? 1u : 0u, wsum, &tsel);
    if (in) fine[key & (TK_FINE - 1)] = 0;  // this candidate's fine bin (read by Rc, done)
    if (sel && pos < (uint32_t)kcap) {
      const uint16_t hv = tk_half(a);
      const int gi = cidx[i];
      idx[pos] = gi;
      val[pos] = hv;
      resid[gi] = a - (float)__builtin_bit_cast(_Float16, hv);
    }
    run_sel += tsel;
    run_tie += teq;
  }
  if (blockIdx.x == 0) {
    for (int i = t; i < TK_CCOPY * 1024; i += 256) coarse[i] = 0;
    if (t == 0) {
      payload[0] = k < kcap ? k : kcap;
      payload[1] = kcap;
      payload[2] = (int)n;
      payload[3] = 0;
    }
  }
}

__global__ __launch_bounds__(256) void topk_decode_add_kernel(const int* __restrict__ payload, float* __restrict__ dst,
                                                              float scale) {
  const int count = payload[0], kcap = payload[1];
  const int* idx = payload + 4;
  const _Float16* val = reinterpret_cast<const _Float16*>(payload + 4 + kcap);
  const int lim = count < kcap ? count : kcap;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < lim; i += gridDim.x * 256)
    dst[idx[i]] += scale * (float)val[i];  // indices of one payload are unique
}

}  // namespace psx

using namespace psx;

static long tk_chunk(long n, int nblk, int tile) { return ((n + nblk - 1) / nblk + tile - 1) / tile * tile; }

extern "C" {

// int32 words of workspace for gradients of n elements (state, histogram copies, per-chunk
// suffix rows, candidate buffers of n entries — never overflow, whatever the distribution —,
// the candidates' coarse / fine histograms and the candidate stage's range counts).
long psx_topk_workspace_words(long n) {
  return (long)TK_STATE_WORDS + (long)TK_HCOPY * TK_NB0 + (long)TK_MAXBLK * TK_ROW +
         2L * (((n > 0 ? n : 1) + 3) / 4 * 4) + (long)TK_CCOPY * 1024 + TK_FINE + 2L * TK_RB;
}

int psx_topk_payload_words(int kcap) { return 4 + kcap + (kcap + 1) / 2; }

// g: fp16 (g_fp16=1) or fp32 gradient, or NULL (select from resid as is); resid: fp32 error
// feedback buffer (updated in place); ws: psx_topk_workspace_words(n) uint32, zeroed once at
// allocation (every encode leaves its histogram zeroed).
int psx_topk_encode(const void* g, int g_fp16, float* resid, long n, int k, int kcap, int* payload, uint32_t* ws,
                    hipStream_t st) {
  if (k > kcap) k = kcap;
  if ((long)k > n) k = (int)n;
  if (k < 1 || n < 1) return (int)hipErrorInvalidValue;
  if (((uintptr_t)resid & 15) || (g && ((uintptr_t)g & (g_fp16 ? 7 : 15)))) return (int)hipErrorInvalidValue;
  uint32_t* state = ws;  // (bench/topk_bench.py reads the candidate count, word TK_NC)
  uint32_t* hist = state + TK_STATE_WORDS;
  uint32_t* rows = hist + TK_HCOPY * TK_NB0;
  int* cidx = (int*)(rows + (size_t)TK_MAXBLK * TK_ROW);
  float* cval = (float*)(cidx + (n + 3) / 4 * 4);
  uint32_t* coarse = (uint32_t*)(cval + (n + 3) / 4 * 4);
  uint32_t* fine = coarse + TK_CCOPY * 1024;
  uint32_t* rcounts = fine + TK_FINE;
  const long chunk = tk_chunk(n, TK_MAXBLK, 1024);  // pass A: 4 chunks per workgroup
  if (!g)
    hipLaunchKernelGGL((tk_pass_a<float, false>), dim3(TK_MAXBLK / 4), dim3(1024), 0, st, (const float*)nullptr, resid,
                       n, chunk, hist, rows);
  else if (g_fp16)
    hipLaunchKernelGGL((tk_pass_a<uint16_t, true>), dim3(TK_MAXBLK / 4), dim3(1024), 0, st, (const uint16_t*)g, resid,
                       n, chunk, hist, rows);
  else
    hipLaunchKernelGGL((tk_pass_a<float, true>), dim3(TK_MAXBLK / 4), dim3(1024), 0, st, (const float*)g, resid, n,
                       chunk, hist, rows);
  hipLaunchKernelGGL(tk_select0, dim3(1), dim3(1024), 0, st, hist, state, k);
  hipLaunchKernelGGL(tk_pass_b, dim3(TK_MAXBLK), dim3(256), 0, st, resid, n, chunk, state, rows, payload, kcap, cidx,
                     cval, coarse, fine);
  hipLaunchKernelGGL(tk_refine_count, dim3(TK_RB), dim3(256), 0, st, cval, state, coarse, fine, rcounts);
  hipLaunchKernelGGL(tk_refine_write, dim3(TK_RB), dim3(256), 0, st, resid, cidx, cval, state, rcounts, payload, kcap,
                     n, k, coarse, fine);
  return (int)hipGetLastError();
}

int psx_topk_decode_add(const int* payload, float* dst, float scale, int kcap, hipStream_t st) {
  int grid = (kcap + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(topk_decode_add_kernel, dim3(grid), dim3(256), 0, st, payload, dst, scale);
  return (int)hipGetLastError();
}

}  // extern "C"
