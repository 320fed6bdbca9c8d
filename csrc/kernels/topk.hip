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
//   A  (1024 workgroups, one contiguous chunk each) acc = resid + g in place and a 4096-bin LDS
//      histogram of the top 12 magnitude bits (exponent + 4 mantissa bits); flushed to a global
//      histogram with sparse atomics, and kept per workgroup as suffix sums;
//   S  (one workgroup) the bin b0 holding the k-th largest; every chunk's count of elements above
//      b0 ("sure") and inside it ("candidates") is two lookups in its suffix row: exclusive scans
//      give each chunk its write bases;
//   B  (1024 workgroups, same chunks) writes the sure entries to the payload in index order
//      (workgroup-scan ranks; resid -= fp16 value), compacts the candidates (index, acc) in index
//      order and histograms their remaining 19 bits: 1024 coarse bins (bits 18..9, LDS) and the
//      full 2^19 fine bins (global atomics);
//   Rc (256 workgroups over the candidates) every workgroup finds the exact threshold T from the
//      two histograms (coarse bin, then its 512 fine bins) and counts its range's candidates
//      above T and equal to T;
//   Rw (same) appends its selected candidates in index order (base = prefix of the preceding
//      ranges' counts; ties at T taken lowest index first), updates resid, clears the histograms
//      and writes the header.
// With error feedback the unsent mass piles up just below the threshold (10x the candidates of a
// Gaussian), so the candidate stage is grid-parallel. Deterministic: positions come from ordered
// scans, never from same-address atomics. The previous encoder made three full histogram passes
// + count / scan / write (5 passes, 11 launches).
//
// Payload (int32 words): [count, kcap, n, 0 | idx[kcap] | fp16 val[kcap] (packed)]
// Server side: dst[idx] += scale * val (decode into a dense fp32 buffer, or straight into the
// fp32 master parameters with scale = -lr * weight when there is no optimizer state).
#include "common.hpp"

namespace psx {

enum { TK_KREM = 0, TK_B0 = 1, TK_CNTGT = 2, TK_NC = 3, TK_T = 4, TK_NEED = 5, TK_STATE_WORDS = 16 };
constexpr int TK_RB = 256;                 // workgroups of the candidate stage
constexpr int TK_FINE = 1 << 19;           // fine bins: magnitude bits 18..0
constexpr int TK_NB0 = 4096, TK_SH0 = 19;  // first-level bins: magnitude bits 30..19
constexpr int TK_BLOCKS = 1024;            // chunks of passes A / B
constexpr int TK_ROW = TK_NB0 + 1;         // per-chunk suffix row (entry 4096 = 0)

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

// Pass A: acc = resid + g (g may be null), 4096-bin histogram -> global + per-chunk suffix row.
template <typename GT>
__global__ __launch_bounds__(256) void tk_pass_a(const GT* __restrict__ g, float* __restrict__ resid, long n,
                                                 long chunk, uint32_t* __restrict__ ghist,
                                                 uint32_t* __restrict__ rows) {
  __shared__ uint32_t lh2[2 * TK_NB0];  // two copies (waves 0-1 / 2-3): half the same-bin contention
  __shared__ uint32_t wsum[4];
  const int t = threadIdx.x;
  for (int i = t; i < 2 * TK_NB0; i += 256) lh2[i] = 0;
  __syncthreads();
  uint32_t* const lh = lh2 + (t >> 7) * TK_NB0;
  const long lo = (long)blockIdx.x * chunk;
  const long hi = lo + chunk < n ? lo + chunk : n;
  // 4 tiles of 1024 per iteration: their loads are all in flight before the first add / atomic
  constexpr int U = 4;
  long i = lo + 4 * t;
  for (; i + (U - 1) * 1024 + 3 < hi; i += U * 1024) {
    f32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = *reinterpret_cast<const f32x4*>(resid + i + u * 1024);
    if (g != nullptr) {
      if constexpr (sizeof(GT) == 2) {
        u32x2 hv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) hv[u] = *reinterpret_cast<const u32x2*>(g + i + u * 1024);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const _Float16* hp = reinterpret_cast<const _Float16*>(&hv[u]);
#pragma unroll
          for (int e = 0; e < 4; ++e) r[u][e] += (float)hp[e];
        }
      } else {
        f32x4 gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) gv[u] = *reinterpret_cast<const f32x4*>(g + i + u * 1024);
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] += gv[u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) *reinterpret_cast<f32x4*>(resid + i + u * 1024) = r[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) atomicAdd(&lh[mag_key(r[u][e]) >> TK_SH0], 1u);
  }
  for (; i < hi; i += 1024) {
    if (i + 3 < hi) {
      f32x4 r = *reinterpret_cast<const f32x4*>(resid + i);
      if (g != nullptr) {
        if constexpr (sizeof(GT) == 2) {
          const u32x2 h = *reinterpret_cast<const u32x2*>(g + i);
          const _Float16* hp = reinterpret_cast<const _Float16*>(&h);
#pragma unroll
          for (int e = 0; e < 4; ++e) r[e] += (float)hp[e];
        } else {
          r += *reinterpret_cast<const f32x4*>(g + i);
        }
        *reinterpret_cast<f32x4*>(resid + i) = r;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) atomicAdd(&lh[mag_key(r[e]) >> TK_SH0], 1u);
    } else {
      for (long j = i; j < hi; ++j) {
        float a = resid[j];
        if (g != nullptr) {
          a += tk_load_g(g, j);
          resid[j] = a;
        }
        atomicAdd(&lh[mag_key(a) >> TK_SH0], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = t; i < TK_NB0; i += 256) lh2[i] += lh2[TK_NB0 + i];
  __syncthreads();
  // suffix sums in descending bin order: thread t owns bins 4095 - 16 t - j (j < 16)
  uint32_t c[16], local = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    c[j] = lh2[TK_NB0 - 1 - (16 * t + j)];
    local += c[j];
  }
  uint32_t tot;
  uint32_t above = tk_excl_scan<256>(local, wsum, &tot);
  uint32_t* row = rows + (size_t)blockIdx.x * TK_ROW;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    above += c[j];
    row[TK_NB0 - 1 - (16 * t + j)] = above;  // # elements of this chunk in bins >= bin
  }
  if (t == 0) row[TK_NB0] = 0;
  for (int i = t; i < TK_NB0; i += 256)
    if (lh2[i]) atomicAdd(&ghist[i], lh2[i]);
}

// S: one workgroup of 1024 threads. The bin b0 holding the k-th largest; per-chunk bases of the
// sure entries and of the candidates; clears the global histogram for the next encode.
__global__ __launch_bounds__(1024) void tk_select0(uint32_t* __restrict__ ghist, const uint32_t* __restrict__ rows,
                                                   uint32_t* __restrict__ state, uint32_t* __restrict__ bases, int k) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t sb[2];
  const int t = threadIdx.x;
  uint32_t c[4], local = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = ghist[TK_NB0 - 1 - (4 * t + j)];
    local += c[j];
  }
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
  for (int j = 0; j < 4; ++j) ghist[4 * t + j] = 0;
  // chunk t: sure = bins > b0, candidates = bin b0
  const uint32_t* row = rows + (size_t)t * TK_ROW;
  const uint32_t sure = row[b0 + 1], cand = row[b0] - sure;
  uint32_t ts, tc;
  const uint32_t bs = tk_excl_scan<1024>(sure, wsum, &ts);
  const uint32_t bc = tk_excl_scan<1024>(cand, wsum, &tc);
  bases[2 * t] = bs;
  bases[2 * t + 1] = bc;
  if (t == 0) {
    state[TK_KREM] = kk - cnt_gt;
    state[TK_B0] = b0;
    state[TK_CNTGT] = cnt_gt;
    state[TK_NC] = tc;
  }
}

// B: sure entries -> payload (index order), candidates -> (cidx, cval) (index order) + their
// coarse / fine histograms. Tiles of 1024 elements, 4 consecutive ones per thread (one 16-byte
// load), ranks by a workgroup scan.
__global__ __launch_bounds__(256) void tk_pass_b(float* __restrict__ resid, long n, long chunk,
                                                 const uint32_t* __restrict__ state,
                                                 const uint32_t* __restrict__ bases, int* __restrict__ payload,
                                                 int kcap, int* __restrict__ cidx, float* __restrict__ cval,
                                                 uint32_t* __restrict__ coarse, uint32_t* __restrict__ fine) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t lh[1024];
  for (int i = threadIdx.x; i < 1024; i += 256) lh[i] = 0;
  const uint32_t b0 = state[TK_B0];
  int* idx = payload + 4;
  uint16_t* val = reinterpret_cast<uint16_t*>(payload + 4 + kcap);
  const long lo = (long)blockIdx.x * chunk;
  const long hi = lo + chunk < n ? lo + chunk : n;
  uint32_t rs = bases[2 * blockIdx.x], rc = bases[2 * blockIdx.x + 1];
  auto load4 = [&](long i0, float (&a)[4]) {
    if (i0 + 3 < hi) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(resid + i0);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = i0 + e < hi ? resid[i0 + e] : 0.f;
    }
  };
  float nx1[4], nx2[4];  // tiles t + 1 and t + 2 are in flight while tile t is ranked and written
  load4(lo + 4 * threadIdx.x, nx1);
  load4(lo + 1024 + 4 * threadIdx.x, nx2);
  for (long base = lo; base < hi; base += 1024) {
    const long i0 = base + 4 * threadIdx.x;
    float a[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = nx1[e];
      nx1[e] = nx2[e];
    }
    if (base + 2048 < hi) load4(i0 + 2048, nx2);
    uint32_t ns = 0, ncnd = 0, fs = 0, fc = 0;  // counts and per-element flags (bit e)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool in = i0 + e < hi;
      const uint32_t bin = mag_key(a[e]) >> TK_SH0;
      if (in && bin > b0) {
        fs |= 1u << e;
        ++ns;
      } else if (in && bin == b0) {
        fc |= 1u << e;
        ++ncnd;
      }
    }
    uint32_t tp;  // one scan of both counts packed (each <= 1024 per tile)
    const uint32_t ex = tk_excl_scan<256>(ns | (ncnd << 16), wsum, &tp);
    const uint32_t ts = tp & 0xffffu, tc = tp >> 16;
    uint32_t ps = rs + (ex & 0xffffu), pc = rc + (ex >> 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long i = i0 + e;
      if (fs >> e & 1u) {
        if (ps < (uint32_t)kcap) {
          const uint16_t h = tk_half(a[e]);
          idx[ps] = (int)i;
          val[ps] = h;
          resid[i] = a[e] - (float)__builtin_bit_cast(_Float16, h);
        }
        ++ps;
      } else if (fc >> e & 1u) {
        const uint32_t key = mag_key(a[e]);
        cidx[pc] = (int)i;
        cval[pc] = a[e];
        ++pc;
        atomicAdd(&lh[(key >> 9) & 1023u], 1u);
        atomicAdd(&fine[key & (TK_FINE - 1)], 1u);
      }
    }
    rs += ts;
    rc += tc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 256)
    if (lh[i]) atomicAdd(&coarse[i], lh[i]);
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
    c[j] = coarse[1023 - (4 * t + j)];
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
    for (int i = t; i < 1024; i += 256) coarse[i] = 0;
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

static long tk_chunk(long n) { return ((n + TK_BLOCKS - 1) / TK_BLOCKS + 1023) / 1024 * 1024; }

extern "C" {

// int32 words of workspace for gradients of n elements (histogram, state, chunk bases, per-chunk
// suffix rows, candidate buffers of n entries — never overflow, whatever the distribution —,
// the candidates' coarse / fine histograms and the candidate stage's range counts).
long psx_topk_workspace_words(long n) {
  return (long)TK_NB0 + TK_STATE_WORDS + 2L * TK_BLOCKS + (long)TK_BLOCKS * TK_ROW + 2L * (((n > 0 ? n : 1) + 3) / 4 * 4) +
         1024 + TK_FINE + 2L * TK_RB;
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
  uint32_t* hist = ws;
  uint32_t* state = hist + TK_NB0;
  uint32_t* bases = state + TK_STATE_WORDS;
  uint32_t* rows = bases + 2 * TK_BLOCKS;
  int* cidx = (int*)(rows + (size_t)TK_BLOCKS * TK_ROW);
  float* cval = (float*)(cidx + (n + 3) / 4 * 4);
  uint32_t* coarse = (uint32_t*)(cval + (n + 3) / 4 * 4);
  uint32_t* fine = coarse + 1024;
  uint32_t* rcounts = fine + TK_FINE;
  const long chunk = tk_chunk(n);
  if (g_fp16)
    hipLaunchKernelGGL((tk_pass_a<uint16_t>), dim3(TK_BLOCKS), dim3(256), 0, st, (const uint16_t*)g, resid, n, chunk,
                       hist, rows);
  else
    hipLaunchKernelGGL((tk_pass_a<float>), dim3(TK_BLOCKS), dim3(256), 0, st, (const float*)g, resid, n, chunk, hist,
                       rows);
  hipLaunchKernelGGL(tk_select0, dim3(1), dim3(1024), 0, st, hist, rows, state, bases, k);
  hipLaunchKernelGGL(tk_pass_b, dim3(TK_BLOCKS), dim3(256), 0, st, resid, n, chunk, state, bases, payload, kcap,
                     cidx, cval, coarse, fine);
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
