// Top-k gradient sparsification with error feedback (the BASELINE.json "top-k grad compression"
// codec; the reference only casts to fp16, src/workers/worker.py:264-268).
//
// Worker side, one push:
//   acc   = resid + g                        (error feedback: what was not sent last time)
//   T     = k-th largest |acc|               (exact, radix select on the 31 magnitude bits)
//   send    { (i, fp16(acc[i])) : |acc[i]| > T } + enough |acc[i]| == T ties to make exactly k
//   resid = acc - sent                       (incl. the fp16 rounding error of sent values)
//
// The select never leaves the device: three histogram passes over the magnitude bits
// (11 + 11 + 9 bits, LDS histograms flushed with sparse global atomics), each followed by a
// one-block "select" kernel that finds the bin holding the k-th element and refines the
// (prefix, mask, k_remaining) state in HBM; a count / scan / write compaction then emits the
// payload in index order (deterministic, no same-address atomics). No host round trip, so the
// whole encode is stream-ordered and graph-capturable.
//
// Payload (int32 words): [count, kcap, n, 0 | idx[kcap] | fp16 val[kcap] (packed)]
// Server side: dst[idx] += scale * val (decode into a dense fp32 buffer, or straight into the
// fp32 master parameters with scale = -lr * weight when there is no optimizer state).
#include "common.hpp"

namespace psx {

enum { TK_KREM = 0, TK_PREFIX = 1, TK_MASK = 2, TK_CNTGT = 3, TK_TIES = 4, TK_STATE_WORDS = 16 };
constexpr int TK_HIST = 2048;

template <int PASS>
struct TkPass {
  static constexpr int SHIFT = PASS == 0 ? 20 : (PASS == 1 ? 9 : 0);
  static constexpr int NB = PASS == 2 ? 512 : 2048;
};

PSX_DEV uint32_t mag_key(float a) { return __float_as_uint(a) & 0x7fffffffu; }

__global__ __launch_bounds__(256) void topk_init_kernel(uint32_t* state, uint32_t* hist, int* payload, int k,
                                                        int kcap, long n) {
  for (int i = threadIdx.x; i < TK_HIST; i += 256) hist[i] = 0;
  if (threadIdx.x < TK_STATE_WORDS) state[threadIdx.x] = threadIdx.x == TK_KREM ? (uint32_t)k : 0u;
  if (threadIdx.x == 0) {
    payload[0] = 0;
    payload[1] = kcap;
    payload[2] = (int)n;
    payload[3] = 0;
  }
}

// PASS 0 also forms acc = resid + g in place.
template <int PASS, typename GT>
__global__ __launch_bounds__(256) void topk_hist_kernel(const GT* __restrict__ g, float* __restrict__ resid, long n,
                                                        const uint32_t* __restrict__ state, uint32_t* __restrict__ hist) {
  using P = TkPass<PASS>;
  __shared__ uint32_t lh[P::NB];
  for (int i = threadIdx.x; i < P::NB; i += 256) lh[i] = 0;
  __syncthreads();
  const uint32_t prefix = state[TK_PREFIX], pmask = state[TK_MASK];
  auto bump = [&](float a) {
    const uint32_t key = mag_key(a);
    if ((key & pmask) == prefix) atomicAdd(&lh[(key >> P::SHIFT) & (P::NB - 1)], 1u);
  };
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    f32x4 r = reinterpret_cast<const f32x4*>(resid)[i];
    if (PASS == 0 && g != nullptr) {
      if constexpr (sizeof(GT) == 2) {
        const u32x2 h = reinterpret_cast<const u32x2*>(g)[i];
        const _Float16* hp = reinterpret_cast<const _Float16*>(&h);
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] += (float)hp[e];
      } else {
        const f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
        r += gv;
      }
      reinterpret_cast<f32x4*>(resid)[i] = r;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) bump(r[e]);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {  // scalar tail
    const long i = (n4 << 2) + threadIdx.x;
    float a = resid[i];
    if (PASS == 0 && g != nullptr) {
      if constexpr (sizeof(GT) == 2) a += (float)reinterpret_cast<const _Float16*>(g)[i];
      else a += (float)g[i];
      resid[i] = a;
    }
    bump(a);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P::NB; i += 256)
    if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

// One block: locate the bin (scanning from the largest magnitudes down) that holds the k-th
// element, fold it into the prefix, and clear the histogram for the next pass.
template <int PASS>
__global__ __launch_bounds__(256) void topk_select_kernel(uint32_t* __restrict__ hist, uint32_t* __restrict__ state) {
  using P = TkPass<PASS>;
  constexpr int PER = P::NB / 256;
  __shared__ uint32_t wtot[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t c[PER];
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    c[j] = hist[P::NB - 1 - (t * PER + j)];  // thread 0 owns the highest bins
    local += c[j];
  }
  const uint32_t krem = state[TK_KREM];
  // block exclusive scan of `local` in thread order
  uint32_t incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  uint32_t above = incl - local;
  for (int i = 0; i < w; ++i) above += wtot[i];
  if (above < krem && above + local >= krem) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (above + c[j] >= krem) {
        const uint32_t b = (uint32_t)(P::NB - 1 - (t * PER + j));
        state[TK_CNTGT] += above;
        state[TK_KREM] = krem - above;
        state[TK_PREFIX] |= b << P::SHIFT;
        state[TK_MASK] |= (uint32_t)(P::NB - 1) << P::SHIFT;
        break;
      }
      above += c[j];
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) hist[P::NB - 1 - (t * PER + j)] = 0;
}

// Deterministic two-phase compaction (no same-address atomics): block b owns the contiguous
// chunk [b*chunk, (b+1)*chunk). Phase 1 counts its "greater" and "tie" elements, a one-block
// scan turns the counts into bases, phase 2 writes the selected entries in index order:
//   pos(i) = #gt(< i) + min(#eq(< i), ties_needed)
constexpr int TK_BLOCKS = 1024;

PSX_DEV void tk_flags(const float* resid, long i, long end, uint32_t T, bool& gt, bool& eq, float& a) {
  const bool in = i < end;
  a = in ? resid[i] : 0.f;
  const uint32_t key = mag_key(a);
  gt = in && key > T;
  eq = in && key == T;
}

__global__ __launch_bounds__(256) void topk_count_kernel(const float* __restrict__ resid, long n, long chunk,
                                                         const uint32_t* __restrict__ state,
                                                         uint32_t* __restrict__ counts) {
  __shared__ uint32_t red[2][4];
  const uint32_t T = state[TK_PREFIX];
  const long lo = (long)blockIdx.x * chunk;
  const long hi = lo + chunk < n ? lo + chunk : n;
  uint32_t cg = 0, ce = 0;
  for (long base = lo; base < hi; base += 256) {
    bool gt, eq;
    float a;
    tk_flags(resid, base + threadIdx.x, hi, T, gt, eq, a);
    cg += (uint32_t)__popcll(__ballot(gt));
    ce += (uint32_t)__popcll(__ballot(eq));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = cg;
    red[1][w] = ce;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    counts[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    counts[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// One block of 256 threads, TK_BLOCKS/256 blocks' counts per thread: exclusive scans.
__global__ __launch_bounds__(256) void topk_scan_kernel(const uint32_t* __restrict__ counts,
                                                        uint32_t* __restrict__ bases) {
  constexpr int PER = TK_BLOCKS / 256;
  __shared__ uint32_t wt[2][4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t g[PER], e[PER], sg = 0, se = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    g[j] = counts[2 * (t * PER + j)];
    e[j] = counts[2 * (t * PER + j) + 1];
    sg += g[j];
    se += e[j];
  }
  uint32_t ig = sg, ie = se;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t vg = __shfl_up(ig, o, 64), ve = __shfl_up(ie, o, 64);
    if (lane >= o) {
      ig += vg;
      ie += ve;
    }
  }
  if (lane == 63) {
    wt[0][w] = ig;
    wt[1][w] = ie;
  }
  __syncthreads();
  uint32_t bg = ig - sg, be = ie - se;
  for (int i = 0; i < w; ++i) {
    bg += wt[0][i];
    be += wt[1][i];
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    bases[2 * (t * PER + j)] = bg;
    bases[2 * (t * PER + j) + 1] = be;
    bg += g[j];
    be += e[j];
  }
}

__global__ __launch_bounds__(256) void topk_write_kernel(float* __restrict__ resid, long n, long chunk,
                                                         const uint32_t* __restrict__ state,
                                                         const uint32_t* __restrict__ bases,
                                                         int* __restrict__ payload, int kcap) {
  __shared__ uint32_t wt[2][4];
  const uint32_t T = state[TK_PREFIX];
  const uint32_t need = state[TK_KREM];  // ties to take
  int* idx = payload + 4;
  uint16_t* val = reinterpret_cast<uint16_t*>(payload + 4 + kcap);
  const long lo = (long)blockIdx.x * chunk;
  const long hi = lo + chunk < n ? lo + chunk : n;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t rg = bases[2 * blockIdx.x], re = bases[2 * blockIdx.x + 1];  // running #gt / #eq before tile
  for (long base = lo; base < hi; base += 256) {
    bool gt, eq;
    float a;
    const long i = base + threadIdx.x;
    tk_flags(resid, i, hi, T, gt, eq, a);
    const uint64_t mg = __ballot(gt), me = __ballot(eq);
    __syncthreads();  // previous tile's wt reads are done
    if (lane == 0) {
      wt[0][w] = (uint32_t)__popcll(mg);
      wt[1][w] = (uint32_t)__popcll(me);
    }
    __syncthreads();
    uint32_t pg = rg, pe = re, tg = 0, te = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < w) {
        pg += wt[0][j];
        pe += wt[1][j];
      }
      tg += wt[0][j];
      te += wt[1][j];
    }
    pg += (uint32_t)__popcll(mg & lt);
    pe += (uint32_t)__popcll(me & lt);
    const bool sel = gt || (eq && pe < need);
    if (sel) {
      const uint32_t pos = pg + (pe < need ? pe : need);
      if (pos < (uint32_t)kcap) {
        const _Float16 h = (_Float16)fminf(fmaxf(a, -65504.f), 65504.f);
        idx[pos] = (int)i;
        val[pos] = __builtin_bit_cast(uint16_t, h);
        resid[i] = a - (float)h;
      }
    }
    rg += tg;
    re += te;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const uint32_t total = rg + (re < need ? re : need);
    payload[0] = (int)(total < (uint32_t)kcap ? total : (uint32_t)kcap);
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

static int tk_grid(long n) {
  long b = (n / 4 + 255) / 256;
  if (b > 1024) b = 1024;
  return (int)(b < 1 ? 1 : b);
}

extern "C" {

int psx_topk_workspace_words() { return TK_HIST + TK_STATE_WORDS + 4 * TK_BLOCKS; }

int psx_topk_payload_words(int kcap) { return 4 + kcap + (kcap + 1) / 2; }

// g: fp16 (g_fp16=1) or fp32 gradient, or NULL (select from resid as is); resid: fp32 error
// feedback buffer (updated in place); ws: psx_topk_workspace_words() uint32.
int psx_topk_encode(const void* g, int g_fp16, float* resid, long n, int k, int kcap, int* payload, uint32_t* ws,
                    hipStream_t st) {
  if (k > kcap) k = kcap;
  if ((long)k > n) k = (int)n;
  if (((uintptr_t)resid & 15) || (g && ((uintptr_t)g & (g_fp16 ? 7 : 15)))) return (int)hipErrorInvalidValue;
  uint32_t* hist = ws;
  uint32_t* state = ws + TK_HIST;
  const int grid = tk_grid(n);
  hipLaunchKernelGGL(topk_init_kernel, dim3(1), dim3(256), 0, st, state, hist, payload, k, kcap, n);
  if (g_fp16)
    hipLaunchKernelGGL((topk_hist_kernel<0, uint16_t>), dim3(grid), dim3(256), 0, st, (const uint16_t*)g, resid, n,
                       state, hist);
  else
    hipLaunchKernelGGL((topk_hist_kernel<0, float>), dim3(grid), dim3(256), 0, st, (const float*)g, resid, n, state,
                       hist);
  hipLaunchKernelGGL(topk_select_kernel<0>, dim3(1), dim3(256), 0, st, hist, state);
  hipLaunchKernelGGL((topk_hist_kernel<1, float>), dim3(grid), dim3(256), 0, st, nullptr, resid, n, state, hist);
  hipLaunchKernelGGL(topk_select_kernel<1>, dim3(1), dim3(256), 0, st, hist, state);
  hipLaunchKernelGGL((topk_hist_kernel<2, float>), dim3(grid), dim3(256), 0, st, nullptr, resid, n, state, hist);
  hipLaunchKernelGGL(topk_select_kernel<2>, dim3(1), dim3(256), 0, st, hist, state);
  uint32_t* counts = state + TK_STATE_WORDS;
  uint32_t* bases = counts + 2 * TK_BLOCKS;
  const long chunk = ((n + TK_BLOCKS - 1) / TK_BLOCKS + 255) / 256 * 256;
  hipLaunchKernelGGL(topk_count_kernel, dim3(TK_BLOCKS), dim3(256), 0, st, resid, n, chunk, state, counts);
  hipLaunchKernelGGL(topk_scan_kernel, dim3(1), dim3(256), 0, st, counts, bases);
  hipLaunchKernelGGL(topk_write_kernel, dim3(TK_BLOCKS), dim3(256), 0, st, resid, n, chunk, state, bases, payload,
                     kcap);
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
