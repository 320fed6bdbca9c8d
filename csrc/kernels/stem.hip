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
                                                        int Kg) {
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
      atomicAdd(stats + (size_t)(blockIdx.x & (PSX_STAT_SLOTS - 1)) * 2 * OC + tid, v);
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

}  // namespace psx

using namespace psx;

extern "C" {

// y = conv3x3(x, wf) (stride 1, pad 1) of the 3-channel stem into 64 channels, + the BN
// statistics [PSX_STAT_SLOTS][2][64] (nullable) of (y - sshift) (sshift nullable). x: NHWC with
// cp = one 16-byte chunk of channels (4 fp32 / 8 bf16, zero padded); wf: the conv_v2 forward
// weights [64][Kg], k = tap * cp + c. -11: not this shape, or deterministic mode (the caller
// runs psx_conv_fwd2 instead).
int psx_stem_conv(const void* x, const void* wf, void* y, float* stats, const float* sshift, int Nb, int H, int W,
                  int cin, int cp, int OC, int Kg, int f32, hipStream_t st) {
  if (const char* e = tune("stem_direct"))
    if (e[0] == '0') return -11;
  if (cin != 3 || OC != 64 || cp != (f32 ? 4 : 8) || Kg < 9 * cp || W % 4 || det_enabled()) return -11;
  const long npix = (long)Nb * H * W;
  if (npix <= 0 || npix > (1L << 30)) return -2;
  const dim3 grid((unsigned)((npix + 255) / 256));
  const size_t lds = (size_t)(27 * 64 + 256 * 68) * sizeof(float);
  if (f32)
    hipLaunchKernelGGL((stem_conv_kernel<float, 3>), grid, dim3(256), lds, st, (const float*)x, (const float*)wf,
                       (float*)y, stats, sshift, Nb, H, W, Kg);
  else
    hipLaunchKernelGGL((stem_conv_kernel<uint16_t, 3>), grid, dim3(256), lds, st, (const uint16_t*)x,
                       (const uint16_t*)wf, (uint16_t*)y, stats, sshift, Nb, H, W, Kg);
  return (int)hipGetLastError();
}

}  // extern "C"
