// Direct CIFAR stem conv (3 -> 64 channels, 3x3 / stride 1 / pad 1) on the vector ALUs, with the
// BN statistics of its output.
//
// The stem's implicit GEMM has K = 27 (padded to one or two 128-byte k-steps), so the conv_v2
// MFMA kernel spends its time in the pipeline prologue and the LDS-staged epilogue: measured
// 27 us at batch 128 in fp32 (bench/stem_probe.py), the same with a pre-built im2col operand,
// against a 7 us store floor for the 33.5 MB output. Here a thread computes 4 consecutive
// pixels x 16 output channels with FMAs against weights read from LDS, each 16-byte weight read
// feeding 16 FMAs (one pixel x 64 channels per thread was bound by the LDS return path of the
// broadcast reads, 23 us; weights as scalar-register operands through the scalar cache, 40 us).
// The workgroup's 256 x 64 tile is staged in LDS once for the per-channel statistics
// (conflict-free column sums) and leaves as contiguous 16-byte stores — the tile is one
// contiguous NHWC block.
// Reference: the CIFAR ResNet-18's first conv, nn.Conv2d(3, 64, 3, 1, 1, bias=False)
// (src/workers/worker.py:48, src/parameter_server/server.py:48).
#include "bnfin.hpp"
#include "common.hpp"

namespace psx {

template <typename T, int CIN>
__global__ __launch_bounds__(256) void stem_conv_kernel(const T* __restrict__ x, const T* __restrict__ wf,
                                                        T* __restrict__ y, float* __restrict__ stats,
                                                        const float* __restrict__ sshift, int Nb, int H, int W,
                                                        int Kg, DetRed det) {
  constexpr int CP = kEPC<T>;  // input channels per pixel as stored (one 16-byte chunk)
  constexpr int OC = 64, NK = 9 * CIN, TS = OC + 4;
  static_assert(CIN <= 4 && CIN <= CP, "the stem's channels fit one chunk");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const ws = sm;              // [NK][OC] weights, k = tap * CIN + c; later statistic partials
  float* const tile = sm + NK * OC;  // [256][TS] output tile
  const int tid = threadIdx.x;
  for (int i = tid; i < NK * OC; i += 256) {
    const int k = i / OC, oc = i - k * OC;
    const int tap = k / CIN, c = k - tap * CIN;
    ws[i] = ld1(wf + (size_t)oc * Kg + tap * CP + c);
  }
  const int npix = Nb * H * W, pix0 = blockIdx.x * 256;
  // thread = 4 consecutive pixels of one image row (W % 4 == 0) x 16 output channels: one LDS
  // weight read (4 channels) feeds 16 FMAs
  const int og = tid & 3, p0 = pix0 + (tid >> 2) * 4;
  float xw[3][6][CIN];  // rows h-1..h+1, columns w-1..w+4 of the 4-pixel group
  {
    const int pp = p0 < npix ? p0 : 0;
    const int n = pp / (H * W), rem = pp - n * (H * W), h = rem / W, w = rem - h * W;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) {
        const int ih = h + r - 1, iw = w + cc - 1;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
          const T* src = x + ((size_t)(n * H + ih) * W + iw) * CP;
          if constexpr (sizeof(T) == 4) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(src);
            v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
          } else {
            const u32x2 q = *reinterpret_cast<const u32x2*>(src);
            v[0] = lo_bf(q[0]); v[1] = hi_bf(q[0]); v[2] = lo_bf(q[1]); v[3] = hi_bf(q[1]);
          }
        }
#pragma unroll
        for (int c = 0; c < CIN; ++c) xw[r][cc][c] = v[c];
      }
  }
  __syncthreads();
  f32x4 acc[4][4];  // [pixel][4-channel group]
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int o = 0; o < 4; ++o) acc[p][o] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int sx = 0; sx < 3; ++sx)
#pragma unroll
      for (int c = 0; c < CIN; ++c) {
        const float* wk = ws + ((r * 3 + sx) * CIN + c) * OC + og * 16;
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const f32x4 wv = *reinterpret_cast<const f32x4*>(wk + o * 4);
#pragma unroll
          for (int p = 0; p < 4; ++p) acc[p][o] += xw[r][p + sx][c] * wv;
        }
      }
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      *reinterpret_cast<f32x4*>(tile + ((tid >> 2) * 4 + p) * TS + og * 16 + o * 4) = acc[p][o];
    }
  __syncthreads();
  const int nvalid = min(256, npix - pix0);
  if (stats) {
    // wave q sums pixels [64 q, 64 q + 64) of channel lane; then the four partial sums meet in LDS
    const int oc = tid & 63, q = tid >> 6;
    const float k = sshift ? sshift[oc] : 0.f;
    float s1 = 0.f, s2 = 0.f;
    for (int p = q * 64; p < min(q * 64 + 64, nvalid); ++p) {
      float v = tile[p * TS + oc];
      if constexpr (sizeof(T) == 2) v = bf2f(f2bf(v));  // the statistics of the stored tensor
      const float d = v - k;
      s1 += d;
      s2 += d * d;
    }
    ws[q * 128 + oc] = s1;
    ws[q * 128 + 64 + oc] = s2;
    __syncthreads();
    if (tid < 128) {
      const float v = ws[tid] + ws[128 + tid] + ws[256 + tid] + ws[384 + tid];
      stat_add(det, stats + (size_t)(blockIdx.x & (PSX_STAT_SLOTS - 1)) * 2 * OC, tid, v);
    }
  }
  // the tile is one contiguous [nvalid][64] block of y: 16-byte stores in address order
  constexpr int EPS = 16 / (int)sizeof(T);  // elements per 16-byte store
  T* const dst = y + (size_t)pix0 * OC;
  for (int i = tid; i < nvalid * (OC / EPS); i += 256) {
    const int p = i / (OC / EPS), c = (i - p * (OC / EPS)) * EPS;
    const float* src = tile + p * TS + c;
    if constexpr (sizeof(T) == 4) {
      *reinterpret_cast<f32x4*>(dst + (size_t)p * OC + c) = *reinterpret_cast<const f32x4*>(src);
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>(src), b = *reinterpret_cast<const f32x4*>(src + 4);
      u32x4 o = {pack_bf2(a[0], a[1]), pack_bf2(a[2], a[3]), pack_bf2(b[0], b[1]), pack_bf2(b[2], b[3])};
      *reinterpret_cast<u32x4*>(dst + (size_t)p * OC + c) = o;
    }
  }
}


// ---------------------------------------------------------------------------------------
// ImageNet stem (ResNet-50: 3 -> 64 channels, 7x7 / stride 2 / pad 3, 224 -> 112) on the exact-f32
// MFMA, with the BN statistics of its output. conv_v2 runs it as an implicit GEMM whose k-steps
// are 8 taps of the 4-channel (padded) input: the per-lane gather is a division chain per DMA
// (no uniform-tap fast path below 32 channels) and the step ran at 47 TF (631 us at batch 128,
// profiles/r5_r50_layers_f32_isolated.jsonl). Here a workgroup owns 2 output rows x all 112
// columns x 64 channels of one image: the 9-row input patch it needs is staged in LDS (columns
// de-interleaved by parity, so a wave's 16 stride-2 pixels read 16 consecutive 16-byte slots: no
// bank conflicts). Wave w computes output row w / 4 for channel tile w % 4 (16 channels) as 7
// pixel tiles of v_mfma_f32_16x16x4_f32, one tap (4 channels = one k-group) per MFMA: A = its 49
// weight fragments, held in registers for the whole kernel, B = the patch. 33 KB of LDS and ~100
// VGPRs: two workgroups share a CU. Measured (B = 128, isolated): 571 us, the same as a first
// version with all 64 channels per wave and the weights in LDS (98 KB, one workgroup per CU:
// 574 us) — so the overlap of one workgroup's loads with another's MFMAs is not what bounds it
// (profiles/r5_numbers.jsonl; the PMC pass is in profiles/r5_pmc_r50_layers.txt). The output
// leaves as 16-byte (4-channel) stores per pixel.
constexpr int kS7Rows = 2, kS7W = 112, kS7PW = 115, kS7PR = 2 * kS7Rows + 5;  // 9 patch rows
constexpr int kS7PFloats = kS7PR * 2 * kS7PW * 4;

__global__ __launch_bounds__(512) void stem7_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wf,
                                                        float* __restrict__ y, float* __restrict__ stats,
                                                        const float* __restrict__ sshift, int Kg, int IH, int IW,
                                                        DetRed det) {
  __shared__ __attribute__((aligned(16))) float pt[kS7PFloats];  // [9 rows][parity][115][4]
  __shared__ float red[2][2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ri = w >> 2, m = w & 3;
  const int n = blockIdx.x / (kS7W / kS7Rows), oh0 = (blockIdx.x % (kS7W / kS7Rows)) * kS7Rows;
  const int j = lane & 15, c = lane >> 4;
  // this lane's A fragments: output channel 16 m + j, input channel c, every tap
  float wa[49];
  const float* wrow = wf + (size_t)(16 * m + j) * Kg + c;
#pragma unroll
  for (int t = 0; t < 49; ++t) wa[t] = wrow[4 * t];
  const int ih0 = 2 * oh0 - 3;
  for (int i = tid; i < kS7PR * 2 * kS7PW; i += 512) {  // patch pixel (row rr, padded column pc)
    const int rr = i / (2 * kS7PW), pc = i - rr * (2 * kS7PW);
    const int ih = ih0 + rr, iw = pc - 3;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW)
      v = *reinterpret_cast<const f32x4*>(x + (((size_t)n * IH + ih) * IW + iw) * 4);
    *reinterpret_cast<f32x4*>(pt + ((rr * 2 + (pc & 1)) * kS7PW + (pc >> 1)) * 4) = v;
  }
  __syncthreads();
  f32x4 acc[7];
#pragma unroll
  for (int t = 0; t < 7; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const float* prow = pt + ((2 * ri + r) * 2) * kS7PW * 4 + j * 4 + c;
#pragma unroll
    for (int sx = 0; sx < 7; ++sx) {
      const float* pb = prow + ((sx & 1) * kS7PW + (sx >> 1)) * 4;
      float b[7];
#pragma unroll
      for (int t = 0; t < 7; ++t) b[t] = pb[t * 64];
#pragma unroll
      for (int t = 0; t < 7; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[r * 7 + sx], b[t], acc[t], 0, 0, 0);
    }
  }
  // lane: pixels ow = 16 t + j, channels oc = 16 m + 4 c + e
  float* const yrow = y + (((size_t)n * kS7W + oh0 + ri) * kS7W) * 64 + 16 * m + 4 * c;
  f32x4 k4 = {0.f, 0.f, 0.f, 0.f};
  if (sshift) k4 = *reinterpret_cast<const f32x4*>(sshift + 16 * m + 4 * c);
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    *reinterpret_cast<f32x4*>(yrow + (size_t)(16 * t + j) * 64) = acc[t];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = acc[t][e] - k4[e];
      s1[e] += d;
      s2[e] += d * d;
    }
  }
  if (!stats) return;
#pragma unroll
  for (int sh = 1; sh < 16; sh <<= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] += __shfl_xor(s1[e], sh, 64);
      s2[e] += __shfl_xor(s2[e], sh, 64);
    }
  if (j == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[ri][0][16 * m + 4 * c + e] = s1[e];
      red[ri][1][16 * m + 4 * c + e] = s2[e];
    }
  }
  __syncthreads();
  float* dst = stats + (size_t)(blockIdx.x & (PSX_STAT_SLOTS - 1)) * 2 * 64;
  if (tid < 128) {
    const int which = tid >> 6, oc = tid & 63;
    stat_add(det, dst, tid, red[0][which][oc] + red[1][which][oc]);  // [sum | sum of squares][oc]
  }
}

// bf16 ImageNet stem (ResNet-50 --dtype bf16): the same workgroup / wave layout and LDS patch as
// stem7_fwd_kernel (a bf16 pixel of the 8-channel padded input is also 16 bytes), on
// v_mfma_f32_16x16x32_bf16: one MFMA covers 4 taps x 8 channels, so a pixel tile is 13 MFMAs
// (taps 49..51 read zero weights), lane l supplying the 8 channels of its pixel l & 15 at tap
// 4 j + (l >> 4) — a per-lane patch offset fixed for the kernel. conv_v2 ran it as an implicit
// GEMM with the per-lane im2col gather (one tap per 16-byte chunk): 291 us at batch 128
// (profiles/r5_r50_bf16_kernels.txt); the output is the cost here (205 MB of bf16).
__global__ __launch_bounds__(512) void stem7_fwd_bf16_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ wf, uint16_t* __restrict__ y,
                                                             float* __restrict__ stats, const float* __restrict__ sshift,
                                                             int Kg, int IH, int IW, DetRed det) {
  __shared__ __attribute__((aligned(16))) u32x4 pt[kS7PR * 2 * kS7PW];  // [9 rows][parity][115] x 8 bf16
  __shared__ float red[2][2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ri = w >> 2, m = w & 3;
  const int n = blockIdx.x / (kS7W / kS7Rows), oh0 = (blockIdx.x % (kS7W / kS7Rows)) * kS7Rows;
  const int j = lane & 15, g = lane >> 4;
  // A fragments: output channel 16 m + j, taps 4 q + g (8 channels each); taps >= 49 are zero
  u32x4 wa[13];
  const uint16_t* wrow = wf + (size_t)(16 * m + j) * Kg;
#pragma unroll
  for (int q = 0; q < 13; ++q) {
    const int tap = 4 * q + g;
    wa[q] = tap < 49 ? *reinterpret_cast<const u32x4*>(wrow + tap * 8) : u32x4{0u, 0u, 0u, 0u};
  }
  // B fragment offsets (u32x4 units) of this lane's taps, pixel tile 0: row 2 ri + r, parity s & 1,
  // column j + (s >> 1); the pixel tile t adds 16 t. Taps past 48 read a real pixel (zero weights)
  int boff[13];
#pragma unroll
  for (int q = 0; q < 13; ++q) {
    const int tap = min(4 * q + g, 48), r = tap / 7, sx = tap - r * 7;
    boff[q] = ((2 * ri + r) * 2 + (sx & 1)) * kS7PW + (sx >> 1) + j;
  }
  const int ih0 = 2 * oh0 - 3;
  for (int i = tid; i < kS7PR * 2 * kS7PW; i += 512) {
    const int rr = i / (2 * kS7PW), pc = i - rr * (2 * kS7PW);
    const int ih = ih0 + rr, iw = pc - 3;
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW)
      v = *reinterpret_cast<const u32x4*>(x + (((size_t)n * IH + ih) * IW + iw) * 8);
    pt[(rr * 2 + (pc & 1)) * kS7PW + (pc >> 1)] = v;
  }
  __syncthreads();
  f32x4 acc[7];
#pragma unroll
  for (int t = 0; t < 7; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 13; ++q) {
    u32x4 b[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) b[t] = pt[boff[q] + 16 * t];
#pragma unroll
    for (int t = 0; t < 7; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[q]), __builtin_bit_cast(bf16x8, b[t]),
                                                       acc[t], 0, 0, 0);
  }
  // lane: pixels ow = 16 t + j, channels oc = 16 m + 4 g + e; the sums are of the stored bf16 values
  uint16_t* const yrow = y + (((size_t)n * kS7W + oh0 + ri) * kS7W) * 64 + 16 * m + 4 * g;
  f32x4 k4 = {0.f, 0.f, 0.f, 0.f};
  if (sshift) k4 = *reinterpret_cast<const f32x4*>(sshift + 16 * m + 4 * g);
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    const uint32_t lo = pack_bf2(acc[t][0], acc[t][1]), hi = pack_bf2(acc[t][2], acc[t][3]);
    *reinterpret_cast<u32x2*>(yrow + (size_t)(16 * t + j) * 64) = u32x2{lo, hi};
    const float v[4] = {lo_bf(lo), hi_bf(lo), lo_bf(hi), hi_bf(hi)};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[e] - k4[e];
      s1[e] += d;
      s2[e] += d * d;
    }
  }
  if (!stats) return;
#pragma unroll
  for (int sh = 1; sh < 16; sh <<= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] += __shfl_xor(s1[e], sh, 64);
      s2[e] += __shfl_xor(s2[e], sh, 64);
    }
  if (j == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[ri][0][16 * m + 4 * g + e] = s1[e];
      red[ri][1][16 * m + 4 * g + e] = s2[e];
    }
  }
  __syncthreads();
  float* dst = stats + (size_t)(blockIdx.x & (PSX_STAT_SLOTS - 1)) * 2 * 64;
  if (tid < 128) {
    const int which = tid >> 6, oc = tid & 63;
    stat_add(det, dst, tid, red[0][which][oc] + red[1][which][oc]);
  }
}

// Weight gradient of the ImageNet stem (fp32): dW[oc][tap][c] = sum over output pixels of
// dy[px][oc] * x[2 oh + r - 3][2 ow + s - 3][c], as the v_mfma_f32_16x16x4_f32 GEMM M = 64 output
// channels x N = 196 (tap, channel) columns x K = pixels, 4 pixels per MFMA. A persistent grid of
// kS7WGrid workgroups walks the 4-row x 112-column output tiles of the forward kernel: each tile's
// input patch is staged in LDS (the forward's de-interleaved layout), the A operand (dy) comes
// straight from global memory — a lane's one 16-byte load per pixel quad holds its 4 channel tiles
// (channel oc = 4 i + m of row i of tile m) — and B from the patch with a per-lane (tap, channel)
// offset fixed for the whole kernel. 13 column tiles x 4 channel tiles of accumulators live across
// all of a workgroup's tiles; at the end the 4 waves meet in LDS and the workgroup writes one
// [64][Kg] fp32 slab of the split-K partials that wgrad_reduce sums (split = workgroup).
constexpr int kS7WGrid = 256;
constexpr int kS7WRows = 4, kS7WPR = 2 * kS7WRows + 5;  // the weight gradient's tiles: 4 rows, 13 patch rows

__global__ __launch_bounds__(256) void stem7_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          float* __restrict__ part, int ntiles, int Kg, int IH,
                                                          int IW) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const pt = sm;  // [13 rows][parity][115][4]; after the loop: the wave reduction [4][64][196]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, j = lane & 15;
  // this lane's column of each of the 13 column tiles: k = 16 nt + j = tap * 4 + c
  int toff[13];
  unsigned kvalid = 0;
#pragma unroll
  for (int nt = 0; nt < 13; ++nt) {
    const int k = 16 * nt + j, tap = k >> 2, c = k & 3, r = tap / 7, sx = tap - r * 7;
    toff[nt] = tap < 49 ? ((r * 2 + (sx & 1)) * kS7PW + (sx >> 1)) * 4 + c : 0;
    kvalid |= (unsigned)(tap < 49) << nt;
  }
  f32x4 acc[4][13];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nt = 0; nt < 13; ++nt) acc[m][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / (kS7W / kS7WRows), oh0 = (tile % (kS7W / kS7WRows)) * kS7WRows;
    const int ih0 = 2 * oh0 - 3;
    __syncthreads();  // the previous tile's patch reads are done
    for (int i = tid; i < kS7WPR * 2 * kS7PW; i += 256) {
      const int rr = i / (2 * kS7PW), pc = i - rr * (2 * kS7PW);
      const int ih = ih0 + rr, iw = pc - 3;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW)
        v = *reinterpret_cast<const f32x4*>(x + (((size_t)n * IH + ih) * IW + iw) * 4);
      *reinterpret_cast<f32x4*>(pt + ((rr * 2 + (pc & 1)) * kS7PW + (pc >> 1)) * 4) = v;
    }
    __syncthreads();
    // wave w: output row oh0 + w; pixel quad g = output columns 4 g .. 4 g + 3, lane's column 4 g + q
    const float* dyrow = dy + (((size_t)n * kS7W + oh0 + w) * kS7W) * 64 + 4 * j;
    const float* prow = pt + (2 * w) * 2 * kS7PW * 4 + q * 4;
    // dy loads run kAhead pixel quads ahead of the MFMAs (one quad of MFMAs is ~0.7 us: a single
    // quad of lookahead left the HBM latency exposed)
    constexpr int kAhead = 4;
    f32x4 ar[kAhead];
#pragma unroll
    for (int u = 0; u < kAhead; ++u) ar[u] = *reinterpret_cast<const f32x4*>(dyrow + (size_t)(4 * u + q) * 64);
#pragma unroll kAhead
    for (int g = 0; g < kS7W / 4; ++g) {
      const f32x4 a = ar[g % kAhead];
      if (g + kAhead < kS7W / 4) ar[g % kAhead] = *reinterpret_cast<const f32x4*>(dyrow + (size_t)(4 * (g + kAhead) + q) * 64);
      const float* pb = prow + g * 16;
      float b[13];
#pragma unroll
      for (int nt = 0; nt < 13; ++nt) b[nt] = ((kvalid >> nt) & 1u) ? pb[toff[nt]] : 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nt = 0; nt < 13; ++nt) acc[m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], b[nt], acc[m][nt], 0, 0, 0);
    }
  }
  // D[i][col] of tile (m, nt): lane holds rows i = 4 q + e (output channel 4 i + m), column 16 nt + j
  __syncthreads();
  float* red = sm;  // [4 waves][64 oc][196]: 200,704 B would not fit; reduce in two halves of 2 waves
  for (int half = 0; half < 2; ++half) {
    if ((w >> 1) == half) {
      float* rw = red + (size_t)(w & 1) * 64 * 196;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nt = 0; nt < 13; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int col = 16 * nt + j;
            if (col < 196) {
              const int oc = 4 * (4 * q + e) + m;
              if (half == 0)
                rw[oc * 196 + col] = acc[m][nt][e];
              else
                rw[oc * 196 + col] += acc[m][nt][e];
            }
          }
    }
    __syncthreads();
  }
  float* dst = part + (size_t)blockIdx.x * 64 * Kg;
  for (int i = tid; i < 64 * 196; i += 256) {
    const int oc = i / 196, col = i - oc * 196;
    dst[(size_t)oc * Kg + col] = red[i] + red[64 * 196 + i];
  }
}

}  // namespace psx

using namespace psx;

extern "C" {

// y = conv3x3(x, wf) (stride 1, pad 1) of the 3-channel stem into 64 channels, + the BN
// statistics [PSX_STAT_SLOTS][2][64] (nullable) of (y - sshift) (sshift nullable). x: NHWC with
// cp = one 16-byte chunk of channels (4 fp32 / 8 bf16, zero padded); wf: the conv_v2 forward
// weights [64][Kg], k = tap * cp + c. -11: not this shape (the caller runs psx_conv_fwd2 instead).
int psx_stem_conv(const void* x, const void* wf, void* y, float* stats, const float* sshift, int Nb, int H, int W,
                  int cin, int cp, int OC, int Kg, int f32, hipStream_t st) {
  if (cin != 3 || OC != 64 || cp != (f32 ? 4 : 8) || Kg < 9 * cp || W % 4) return -11;
  const long npix = (long)Nb * H * W;
  if (npix <= 0 || npix > (1L << 30)) return -2;
  const dim3 grid((unsigned)((npix + 255) / 256));
  const DetRed det = stats ? det_for(stats) : DetRed{};
  const size_t lds = (size_t)(27 * 64 + 256 * 68) * sizeof(float);
  if (f32)
    hipLaunchKernelGGL((stem_conv_kernel<float, 3>), grid, dim3(256), lds, st, (const float*)x, (const float*)wf,
                       (float*)y, stats, sshift, Nb, H, W, Kg, det);
  else
    hipLaunchKernelGGL((stem_conv_kernel<uint16_t, 3>), grid, dim3(256), lds, st, (const uint16_t*)x,
                       (const uint16_t*)wf, (uint16_t*)y, stats, sshift, Nb, H, W, Kg, det);
  return (int)hipGetLastError();
}


// y = conv7x7/s2/p3(x, wf) of the ImageNet stem (3 -> 64 channels), fp32 (f32) or bf16, + the BN
// statistics [PSX_STAT_SLOTS][2][64] (nullable) of (y - sshift). x: NHWC [Nb][IH][IW][cp] (cp = 4
// fp32 / 8 bf16 channels, the padding zero); wf: the conv_v2 forward weights [64][Kg],
// k = tap * cp + c (tap = r * 7 + s), Kg >= 49 cp.
// The output is 112 x 112 (IH = IW = 224). -11: not this shape (the caller runs psx_conv_fwd2).
int psx_stem7_conv(const void* x, const void* wf, void* y, float* stats, const float* sshift, int Nb, int IH,
                   int IW, int cin, int cp, int OC, int Kg, int f32, hipStream_t st) {
  if (cin != 3 || cp != (f32 ? 4 : 8) || OC != 64 || Kg < 49 * cp || IH != 224 || IW != 224 || Nb < 1) return -11;
  const unsigned grid = (unsigned)Nb * (kS7W / kS7Rows);
  const DetRed det = stats ? det_for(stats) : DetRed{};
  if (f32)
    hipLaunchKernelGGL(stem7_fwd_kernel, dim3(grid), dim3(512), 0, st, (const float*)x, (const float*)wf, (float*)y,
                       stats, sshift, Kg, IH, IW, det);
  else
    hipLaunchKernelGGL(stem7_fwd_bf16_kernel, dim3(grid), dim3(512), 0, st, (const uint16_t*)x, (const uint16_t*)wf,
                       (uint16_t*)y, stats, sshift, Kg, IH, IW, det);
  return (int)hipGetLastError();
}


// Weight gradient of psx_stem7_conv (fp32): split-K partials part[kS7WGrid][64][Kg] (columns
// k = tap * 4 + c < 196 written) for wgrad_reduce, from the stem input x (NHWC, cp = 4) and the
// output gradient dy [Nb][112][112][64]. part == nullptr: returns the split count (the
// psx_conv_wgrad2 query). -11: not this shape.
int psx_stem7_wgrad(const float* x, const float* dy, float* part, int Nb, int IH, int IW, int cin, int cp, int OC,
                    int Kg, hipStream_t st) {
  if (cin != 3 || cp != 4 || OC != 64 || Kg < 196 || IH != 224 || IW != 224 || Nb < 1) return -11;
  if (!part) return kS7WGrid;
  const int ntiles = Nb * (kS7W / kS7WRows);
  const size_t lds = (size_t)2 * 64 * 196 * sizeof(float);  // >= the patch (47,840 B)
  hipLaunchKernelGGL(stem7_wgrad_kernel, dim3(kS7WGrid), dim3(256), lds, st, x, dy, part, ntiles, Kg, IH, IW);
  const int e = (int)hipGetLastError();
  return e ? -e : kS7WGrid;
}

}  // extern "C"
