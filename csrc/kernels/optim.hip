// Parameter-server numerics on HBM-resident flat arenas:
//   * sgd_apply     : the server update p <- p - lr * w * g  (reference server.py:126-143,
//                     apply_gradients; w = 1/W for sync averaging server.py:166-167 or the
//                     async staleness weight server.py:178), optionally with momentum and
//                     weight decay (baseline optimizer, baseline_training.py:223),
//                     reading fp16 wire gradients directly (codec unpack fused).
//   * grad_aggregate: N-input gradient sum (reference aggregate_gradients_sync, server.py:145-169)
//   * fp16 codec    : pack/unpack (reference compress_gradients worker.py:264-268 /
//                     decompress_gradients server.py:232-237)
//   * param_unpack  : fp32 OIHW master weights -> bf16 implicit-GEMM operands (KRSC for the
//                     forward conv, transposed CRSK for the data-gradient conv); one launch for
//                     every conv of the model, table-driven.
#include "common.hpp"

namespace psx {

PSX_DEV float ld_grad(const uint16_t* g, size_t i) { return (float)__builtin_bit_cast(_Float16, g[i]); }
PSX_DEV float ld_grad(const float* g, size_t i) { return g[i]; }

// img (optional): bf16 image of the updated parameters, written in the same pass — the fetch
// wire / the workers' conv-operand source (parallel/codec.py), so no separate pack kernel.
template <typename GT, bool MOM>
__global__ __launch_bounds__(256) void sgd_apply_kernel(float* __restrict__ p, const GT* __restrict__ g,
                                                        float* __restrict__ buf, size_t n, float lr, float gscale,
                                                        float momentum, float wd, int first,
                                                        uint16_t* __restrict__ img) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float d = ld_grad(g, i) * gscale;
    const float pv = p[i];
    if (wd != 0.f) d += wd * pv;
    if (MOM) {
      const float v = first ? d : momentum * buf[i] + d;
      buf[i] = v;
      d = v;
    }
    const float nv = pv - lr * d;
    p[i] = nv;
    if (img) img[i] = f2bf(nv);
  }
}

// vectorised fp16-gradient fast path (no momentum): 8 elements per lane
template <bool IMG>
__global__ __launch_bounds__(256) void sgd_apply_h8_kernel(float* __restrict__ p, const uint16_t* __restrict__ g,
                                                           size_t n, float step, float wd_step,
                                                           uint16_t* __restrict__ img) {
  const size_t n8 = n >> 3;
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {  // tail (n % 8 elements)
    const size_t i = (n8 << 3) + threadIdx.x;
    const float nv = p[i] - (step * (float)__builtin_bit_cast(_Float16, g[i]) + wd_step * p[i]);
    p[i] = nv;
    if (IMG) img[i] = f2bf(nv);
  }
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 gv = reinterpret_cast<const u32x4*>(g)[i];
    f32x4 p0 = reinterpret_cast<f32x4*>(p)[2 * i];
    f32x4 p1 = reinterpret_cast<f32x4*>(p)[2 * i + 1];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t w0 = gv[j], w1 = gv[2 + j];
      const float a = (float)__builtin_bit_cast(_Float16, (uint16_t)(w0 & 0xffff));
      const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(w0 >> 16));
      const float c = (float)__builtin_bit_cast(_Float16, (uint16_t)(w1 & 0xffff));
      const float d = (float)__builtin_bit_cast(_Float16, (uint16_t)(w1 >> 16));
      p0[2 * j] -= step * a + wd_step * p0[2 * j];
      p0[2 * j + 1] -= step * b + wd_step * p0[2 * j + 1];
      p1[2 * j] -= step * c + wd_step * p1[2 * j];
      p1[2 * j + 1] -= step * d + wd_step * p1[2 * j + 1];
    }
    reinterpret_cast<f32x4*>(p)[2 * i] = p0;
    reinterpret_cast<f32x4*>(p)[2 * i + 1] = p1;
    if (IMG) {
      const u32x4 o = {pack_bf2(p0[0], p0[1]), pack_bf2(p0[2], p0[3]), pack_bf2(p1[0], p1[1]),
                       pack_bf2(p1[2], p1[3])};
      reinterpret_cast<u32x4*>(img)[i] = o;
    }
  }
}

// Sync-round update straight from the W gathered gradient wires (reference server.py:232-237
// decompress_gradients + :145-169 aggregate_gradients_sync + :126-143 apply_gradients):
//   p <- p - lr * (gscale * sum_k decode(g_k) [+ wd p]) [momentum], gscale = 1/W,
// every wire decoded to fp32 and summed in fp32 in the fixed source order k = 0..W-1 (what the
// reference's numpy loop does; an RCCL fp16 reduce would round the running sum to fp16 at every
// hop). One pass over the W wires + the parameters; img (optional) receives the bf16 image.
constexpr int kMaxSrc = 32;  // reference server.py:424-426 caps the job at 32 workers
struct SrcList {
  const void* p[kMaxSrc];
  int n;
};

template <typename GT, bool MOM>
__global__ __launch_bounds__(256) void sgd_apply_multi_kernel(float* __restrict__ p, SrcList srcs,
                                                              float* __restrict__ buf, size_t n, float lr,
                                                              float gscale, float momentum, float wd, int first,
                                                              uint16_t* __restrict__ img) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < srcs.n; ++k) s += ld_grad(reinterpret_cast<const GT*>(srcs.p[k]), i);
    float d = s * gscale;
    const float pv = p[i];
    if (wd != 0.f) d += wd * pv;
    if (MOM) {
      const float v = first ? d : momentum * buf[i] + d;
      buf[i] = v;
      d = v;
    }
    const float nv = pv - lr * d;
    p[i] = nv;
    if (img) img[i] = f2bf(nv);
  }
}

// vectorised fp16-wire form (no momentum / weight decay): 8 elements per lane, every source's
// 16-byte chunk loaded before the fixed-order sum
// (same arithmetic as sgd_apply_multi_kernel: d = sum * gscale, p -= lr * d)
template <bool IMG>
__global__ __launch_bounds__(256) void sgd_apply_multi_h8_kernel(float* __restrict__ p, SrcList srcs, size_t n,
                                                                 float lr, float gscale, uint16_t* __restrict__ img) {
  const size_t n8 = n >> 3;
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {  // tail (n % 8 elements)
    const size_t i = (n8 << 3) + threadIdx.x;
    float s = 0.f;
    for (int k = 0; k < srcs.n; ++k) s += ld_grad(reinterpret_cast<const uint16_t*>(srcs.p[k]), i);
    const float nv = p[i] - lr * (s * gscale);
    p[i] = nv;
    if (IMG) img[i] = f2bf(nv);
  }
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < srcs.n; ++k) {
      const u32x4 gv = reinterpret_cast<const u32x4*>(srcs.p[k])[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[2 * j] += (float)__builtin_bit_cast(_Float16, (uint16_t)(gv[j] & 0xffff));
        s[2 * j + 1] += (float)__builtin_bit_cast(_Float16, (uint16_t)(gv[j] >> 16));
      }
    }
    f32x4 p0 = reinterpret_cast<f32x4*>(p)[2 * i];
    f32x4 p1 = reinterpret_cast<f32x4*>(p)[2 * i + 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p0[j] -= lr * (s[j] * gscale);
      p1[j] -= lr * (s[4 + j] * gscale);
    }
    reinterpret_cast<f32x4*>(p)[2 * i] = p0;
    reinterpret_cast<f32x4*>(p)[2 * i + 1] = p1;
    if (IMG) {
      const u32x4 o = {pack_bf2(p0[0], p0[1]), pack_bf2(p0[2], p0[3]), pack_bf2(p1[0], p1[1]),
                       pack_bf2(p1[2], p1[3])};
      reinterpret_cast<u32x4*>(img)[i] = o;
    }
  }
}

// dst = sum_i src_i * scale  (fp16 or fp32 sources; fp32 or fp16 destination)
template <typename ST, typename DT>
__global__ __launch_bounds__(256) void aggregate_kernel(const ST* const* __restrict__ srcs, int nsrc,
                                                        DT* __restrict__ dst, size_t n, float scale, int accumulate) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nsrc; ++k) s += ld_grad(srcs[k], i);
    s *= scale;
    if constexpr (sizeof(DT) == 2) {
      if (accumulate) s += ld_grad(dst, i);
      dst[i] = __builtin_bit_cast(uint16_t, (_Float16)s);
    } else {
      if (accumulate) s += dst[i];
      dst[i] = s;
    }
  }
}

__global__ __launch_bounds__(256) void fp16_pack_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                        size_t n, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = __builtin_bit_cast(uint16_t, (_Float16)(src[i] * scale));
}
__global__ __launch_bounds__(256) void fp16_unpack_kernel(const uint16_t* __restrict__ src, float* __restrict__ dst,
                                                          size_t n, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = (float)__builtin_bit_cast(_Float16, src[i]) * scale;
}

__global__ __launch_bounds__(256) void gather_f32_kernel(const float* __restrict__ src, const long* __restrict__ idx,
                                                         size_t n, float* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

struct UnpackDesc {
  long src_off;  // element offset of the OIHW fp32 weight in the arena
  long wf_off;   // element offset of the bf16 [OC][Kg] forward operand
  long wd_off;   // element offset of the bf16 [Cp][Kgd] dgrad operand, -1 if none
  int OC, Cin, R, S, Cp, Kg, Kgd;
  int tile0;     // first flat tile index of this conv (param_unpack_tiles_kernel grid)
};

PSX_DEV uint16_t to_bf(const float* s, size_t i) { return f2bf(s[i]); }
PSX_DEV uint16_t to_bf(const uint16_t* s, size_t i) { return s[i]; }
// operand element of type DT from the source (bf16 bits from fp32 / bf16, or fp32 from fp32)
template <typename DT, typename ST>
PSX_DEV DT to_op(const ST* s, size_t i) {
  if constexpr (sizeof(DT) == 2) return to_bf(s, i);
  else return s[i];
}

// Flat-grid unpack: one workgroup per (conv, 64 oc x 64 c tile, chunk of <= 3 taps), staged
// through LDS. Every global store is a 4-byte pair and every (oc, tap) row of
// wf / (c, tap) row of wd a full 128-byte line (the 32x32-tile version wrote 64-byte halves from
// two workgroups and ran at 0.8 TB/s). The source is the fp32 arena or the server's bf16 weight
// image (the bits sgd_apply wrote next to the fp32 update, parallel/codec.py), so a worker
// never needs fp32 conv weights.
constexpr int kUnpackTile = 64;

PSX_DEV void store_pair(uint16_t* p, uint16_t a, uint16_t b) {
  *reinterpret_cast<uint32_t*>(p) = (uint32_t)a | ((uint32_t)b << 16);
}
PSX_DEV void store_pair(float* p, float a, float b) { *reinterpret_cast<float2*>(p) = make_float2(a, b); }

// DT: operand type (bf16 bits, or fp32 for the fp32 path). The (oc, tap) rows of wf and (c, tap)
// rows of wd are written as element pairs (4-byte bf16 / 8-byte fp32 stores).
template <int NT, typename ST, typename DT>
PSX_DEV void unpack_chunk(const UnpackDesc& d, const ST* __restrict__ src, int oc0, int c0, int tap0, int RS,
                          DT* __restrict__ wbuf, DT* tile) {
  // odd dword pitch -> oc-strided reads hit distinct banks
  constexpr int PITCH = 64 * NT + (sizeof(DT) == 2 ? 2 : 1);
  const int nc_src = min(64, d.Cin - c0);  // real input channels in this tile (<= 0: all padding)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // stage tile[oc][c*NT + tp] = W[oc0+oc][c0+c][tap0+tp]: all 16*NT loads of a lane in flight
  // before the first LDS write (a load -> wait -> write loop per row was latency-bound)
  DT v[16][NT];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int oc = wv + 4 * i;
    const bool ok = oc0 + oc < d.OC && lane < nc_src;
    const ST* p = src + ((size_t)(oc0 + oc) * d.Cin + c0 + lane) * RS + tap0;
#pragma unroll
    for (int tp = 0; tp < NT; ++tp) v[i][tp] = ok ? to_op<DT>(p, tp) : (DT)0;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int tp = 0; tp < NT; ++tp) tile[(wv + 4 * i) * PITCH + lane * NT + tp] = v[i][tp];
  __syncthreads();
  const int half = lane >> 5, l2 = (lane & 31) * 2;  // a wave writes two 128-byte rows
  // wf[oc][tap*Cp + c]
  for (int q = wv * 2 + half; q < 64 * NT; q += 8) {
    const int oc = q / NT, tp = q - oc * NT;
    if (oc0 + oc < d.OC && c0 + l2 < d.Cp)
      store_pair(wbuf + d.wf_off + (size_t)(oc0 + oc) * d.Kg + (tap0 + tp) * d.Cp + c0 + l2,
                 tile[oc * PITCH + l2 * NT + tp], tile[oc * PITCH + (l2 + 1) * NT + tp]);
  }
  if (d.wd_off >= 0) {  // wd[c][tap*OC + oc]
    for (int q = wv * 2 + half; q < 64 * NT; q += 8) {
      const int c = q / NT, tp = q - c * NT;
      if (oc0 + l2 < d.OC && c0 + c < d.Cp)
        store_pair(wbuf + d.wd_off + (size_t)(c0 + c) * d.Kgd + (tap0 + tp) * d.OC + oc0 + l2,
                   tile[l2 * PITCH + c * NT + tp], tile[(l2 + 1) * PITCH + c * NT + tp]);
    }
  }
}

// The fp32 remainder of a fetch (BN affine, FC, BN buffers) scattered into the worker's arena by
// workgroups appended to the unpack grid (one launch instead of unpack + index_copy):
// dst[idx[j]] = src[j] (the wire's small region) or src[idx[j]] (gather = 1: straight from the
// server's fp32 arena when the worker shares the server's device and round).
struct SmallScatter {
  const float* src;
  const long* idx;
  long n;
  float* dst;
  int gather;
  const long* sidx;  // optional source positions: dst[idx[j]] = src[sidx[j]] (sharded wire)
};
constexpr int kScatterPerBlock = 2048;

template <typename ST, typename DT>
__global__ __launch_bounds__(256) void param_unpack_tiles_kernel(const ST* __restrict__ src_all,
                                                                 const UnpackDesc* __restrict__ descs, int ndesc,
                                                                 DT* __restrict__ wbuf, int ntiles,
                                                                 SmallScatter sc) {
  if ((int)blockIdx.x >= ntiles) {  // scatter workgroups (block-uniform exit)
    const long base = (long)(blockIdx.x - ntiles) * kScatterPerBlock;
#pragma unroll
    for (int r = 0; r < kScatterPerBlock / 256; ++r) {
      const long j = base + r * 256 + threadIdx.x;
      if (j < sc.n) {
        const long k = sc.idx[j];
        sc.dst[k] = sc.src[sc.sidx ? sc.sidx[j] : (sc.gather ? k : j)];
      }
    }
    return;
  }
  __shared__ DT tile[64 * (64 * 3 + 2)];
  __shared__ int first_tile[256];
  // which conv owns this workgroup: all descs' tile0 fetched in parallel
  for (int k = threadIdx.x; k < 256; k += 256) first_tile[k] = k < ndesc ? descs[k].tile0 : 0x7fffffff;
  __syncthreads();
  int j = 0;
  while (j + 1 < ndesc && first_tile[j + 1] <= (int)blockIdx.x) ++j;
  const UnpackDesc d = descs[j];
  // unit = (64x64 tile, chunk of <= 3 taps): one workgroup each
  const int RS = d.R * d.S;
  const int nchunk = (RS + 2) / 3;
  const int u = blockIdx.x - d.tile0;
  const int t = u / nchunk, tap0 = (u - t * nchunk) * 3;
  const int n_c = (d.Cp + kUnpackTile - 1) / kUnpackTile;
  const int oc0 = (t / n_c) * kUnpackTile, c0 = (t % n_c) * kUnpackTile;
  const ST* src = src_all + d.src_off;
  const int nt = min(3, RS - tap0);
  if (nt == 3) unpack_chunk<3, ST, DT>(d, src, oc0, c0, tap0, RS, wbuf, tile);
  else if (nt == 2) unpack_chunk<2, ST, DT>(d, src, oc0, c0, tap0, RS, wbuf, tile);
  else unpack_chunk<1, ST, DT>(d, src, oc0, c0, tap0, RS, wbuf, tile);
}

// One workgroup per (32 oc x 32 c) tile of one conv (blockIdx.y = conv). For every tap the
// tile goes through LDS so both destination layouts are written with contiguous runs:
// wf[oc][tap*Cp + c] (c fastest) and wd[c][tap*OC + oc] (oc fastest). Channels c >= Cin of the
// forward operand are written as zeros; the Kg tail beyond R*S*Cp is zeroed once at allocation.
__global__ __launch_bounds__(256) void param_unpack_kernel(const float* __restrict__ arena,
                                                           const UnpackDesc* __restrict__ descs,
                                                           uint16_t* __restrict__ wbuf) {
  __shared__ float tile[32][33];
  const UnpackDesc d = descs[blockIdx.y];
  const float* src = arena + d.src_off;
  const int RS = d.R * d.S;
  const int n_oc = (d.OC + 31) / 32, n_c = (d.Cp + 31) / 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int t = blockIdx.x; t < n_oc * n_c; t += gridDim.x) {
    const int oc0 = (t / n_c) * 32, c0 = (t % n_c) * 32;
    for (int tap = 0; tap < RS; ++tap) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // tile[oc][c] = W[oc0+oc][c0+c][tap]
        const int oc = ty + 8 * j, c = tx;
        float v = 0.f;
        if (oc0 + oc < d.OC && c0 + c < d.Cin) v = src[((size_t)(oc0 + oc) * d.Cin + (c0 + c)) * RS + tap];
        tile[oc][c] = v;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int oc = ty + 8 * j, c = tx;  // wf: c contiguous
        if (oc0 + oc < d.OC && c0 + c < d.Cp)
          wbuf[d.wf_off + (size_t)(oc0 + oc) * d.Kg + tap * d.Cp + c0 + c] = f2bf(tile[oc][c]);
      }
      if (d.wd_off >= 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = ty + 8 * j, oc = tx;  // wd: oc contiguous
          if (oc0 + oc < d.OC && c0 + c < d.Cp)
            wbuf[d.wd_off + (size_t)(c0 + c) * d.Kgd + tap * d.OC + oc0 + oc] = f2bf(tile[oc][c]);
        }
      }
    }
  }
}

}  // namespace psx

using namespace psx;

static int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

// p -= lr * (gscale*g + wd*p) [with momentum buffer]; grads fp16 (wire) or fp32.
// img (optional, nullptr = none): bf16 image of the updated parameters (n elements).
int psx_sgd_apply(float* p, const void* g, float* buf, long n, float lr, float gscale, float momentum, float wd,
                  int first, int grad_fp16, void* img, hipStream_t st) {
  const bool mom = buf != nullptr && momentum != 0.f;
  uint16_t* im = (uint16_t*)img;
  if (!mom && grad_fp16 && n >= 8 && ((uintptr_t)p % 32 == 0) && ((uintptr_t)g % 16 == 0) &&
      ((uintptr_t)img % 16 == 0)) {
    if (im)
      hipLaunchKernelGGL(sgd_apply_h8_kernel<true>, dim3(grid_for(n / 8)), dim3(256), 0, st, p, (const uint16_t*)g,
                         (size_t)n, lr * gscale, lr * wd, im);
    else
      hipLaunchKernelGGL(sgd_apply_h8_kernel<false>, dim3(grid_for(n / 8)), dim3(256), 0, st, p, (const uint16_t*)g,
                         (size_t)n, lr * gscale, lr * wd, im);
    return (int)hipGetLastError();
  }
  const int grid = grid_for(n);
  if (grad_fp16) {
    if (mom)
      hipLaunchKernelGGL((sgd_apply_kernel<uint16_t, true>), dim3(grid), dim3(256), 0, st, p, (const uint16_t*)g, buf,
                         (size_t)n, lr, gscale, momentum, wd, first, im);
    else
      hipLaunchKernelGGL((sgd_apply_kernel<uint16_t, false>), dim3(grid), dim3(256), 0, st, p, (const uint16_t*)g,
                         buf, (size_t)n, lr, gscale, momentum, wd, first, im);
  } else {
    if (mom)
      hipLaunchKernelGGL((sgd_apply_kernel<float, true>), dim3(grid), dim3(256), 0, st, p, (const float*)g, buf,
                         (size_t)n, lr, gscale, momentum, wd, first, im);
    else
      hipLaunchKernelGGL((sgd_apply_kernel<float, false>), dim3(grid), dim3(256), 0, st, p, (const float*)g, buf,
                         (size_t)n, lr, gscale, momentum, wd, first, im);
  }
  return (int)hipGetLastError();
}

// p -= lr * (gscale * sum_k g_k + wd * p) [momentum] over nsrc gradient wires (host array of
// nsrc <= 32 device pointers, all fp16 or all fp32), summed in fp32 in source order.
// img (optional): bf16 image of the updated parameters.
int psx_sgd_apply_multi(float* p, const void* const* srcs, int nsrc, float* buf, long n, float lr, float gscale,
                        float momentum, float wd, int first, int grad_fp16, void* img, hipStream_t st) {
  if (nsrc < 1 || nsrc > kMaxSrc) return (int)hipErrorInvalidValue;
  SrcList sl{};
  sl.n = nsrc;
  bool aligned = ((uintptr_t)p % 32 == 0) && ((uintptr_t)img % 16 == 0);
  for (int k = 0; k < nsrc; ++k) {
    sl.p[k] = srcs[k];
    aligned = aligned && ((uintptr_t)srcs[k] % 16 == 0);
  }
  const bool mom = buf != nullptr && momentum != 0.f;
  uint16_t* im = (uint16_t*)img;
  if (!mom && wd == 0.f && grad_fp16 && n >= 8 && aligned) {
    if (im)
      hipLaunchKernelGGL(sgd_apply_multi_h8_kernel<true>, dim3(grid_for(n / 8)), dim3(256), 0, st, p, sl, (size_t)n,
                         lr, gscale, im);
    else
      hipLaunchKernelGGL(sgd_apply_multi_h8_kernel<false>, dim3(grid_for(n / 8)), dim3(256), 0, st, p, sl, (size_t)n,
                         lr, gscale, im);
    return (int)hipGetLastError();
  }
  const int grid = grid_for(n);
#define PSX_SAM(G, M)                                                                                              \
  hipLaunchKernelGGL((sgd_apply_multi_kernel<G, M>), dim3(grid), dim3(256), 0, st, p, sl, buf, (size_t)n, lr, gscale, \
                     momentum, wd, first, im)
  if (grad_fp16 && mom) PSX_SAM(uint16_t, true);
  else if (grad_fp16) PSX_SAM(uint16_t, false);
  else if (mom) PSX_SAM(float, true);
  else PSX_SAM(float, false);
#undef PSX_SAM
  return (int)hipGetLastError();
}

// srcs: device array of nsrc device pointers.
int psx_grad_aggregate(const void* const* srcs, int nsrc, int src_fp16, void* dst, int dst_fp16, long n, float scale,
                       int accumulate, hipStream_t st) {
  const int grid = grid_for(n);
#define PSX_AGG(S, D)                                                                                      \
  hipLaunchKernelGGL((aggregate_kernel<S, D>), dim3(grid), dim3(256), 0, st, (const S* const*)srcs, nsrc, \
                     (D*)dst, (size_t)n, scale, accumulate)
  if (src_fp16 && dst_fp16) PSX_AGG(uint16_t, uint16_t);
  else if (src_fp16) PSX_AGG(uint16_t, float);
  else if (dst_fp16) PSX_AGG(float, uint16_t);
  else PSX_AGG(float, float);
#undef PSX_AGG
  return (int)hipGetLastError();
}

int psx_fp16_pack(const float* src, void* dst, long n, float scale, hipStream_t st) {
  hipLaunchKernelGGL(fp16_pack_kernel, dim3(grid_for(n)), dim3(256), 0, st, src, (uint16_t*)dst, (size_t)n, scale);
  return (int)hipGetLastError();
}

int psx_fp16_unpack(const void* src, float* dst, long n, float scale, hipStream_t st) {
  hipLaunchKernelGGL(fp16_unpack_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const uint16_t*)src, dst, (size_t)n,
                     scale);
  return (int)hipGetLastError();
}

// descs: device array of ndesc UnpackDesc (see struct layout above: 3 int64 + 8 int32)
int psx_param_unpack(const float* arena, const void* descs, int ndesc, void* wbuf, hipStream_t st) {
  hipLaunchKernelGGL(param_unpack_kernel, dim3(64, ndesc), dim3(256), 0, st, arena, (const UnpackDesc*)descs,
                     (uint16_t*)wbuf);
  return (int)hipGetLastError();
}

// Flat-grid unpack (one workgroup per 32x32 tile of every conv; ntiles = sum of the tiles, each
// desc's tile0 = its first tile). src_bf16: the source is a bf16 image instead of the fp32 arena.
// sc_src/sc_idx/sc_n/sc_dst/sc_gather/sc_sidx: optional SmallScatter (sc_n = 0: none), see above.
// f32: fp32 operands (the fp32 compute path; source must be the fp32 arena).
int psx_param_unpack_tiles(const void* src, int src_bf16, const void* descs, int ndesc, int ntiles, void* wbuf,
                           const float* sc_src, const long* sc_idx, long sc_n, float* sc_dst, int sc_gather,
                           const long* sc_sidx, int f32, hipStream_t st) {
  if (ntiles <= 0 || ndesc <= 0) return 0;
  if (ndesc > 256) return (int)hipErrorInvalidValue;  // the kernel's LDS desc table
  const SmallScatter sc{sc_src, sc_idx, sc_n > 0 ? sc_n : 0, sc_dst, sc_gather, sc_sidx};
  const long nsb = (sc.n + kScatterPerBlock - 1) / kScatterPerBlock;
  const dim3 grid((unsigned)(ntiles + nsb));
  if (f32 && src_bf16) return (int)hipErrorInvalidValue;  // fp32 operands come from fp32 weights
  if (f32)
    hipLaunchKernelGGL((param_unpack_tiles_kernel<float, float>), grid, dim3(256), 0, st, (const float*)src,
                       (const UnpackDesc*)descs, ndesc, (float*)wbuf, ntiles, sc);
  else if (src_bf16)
    hipLaunchKernelGGL((param_unpack_tiles_kernel<uint16_t, uint16_t>), grid, dim3(256), 0, st, (const uint16_t*)src,
                       (const UnpackDesc*)descs, ndesc, (uint16_t*)wbuf, ntiles, sc);
  else
    hipLaunchKernelGGL((param_unpack_tiles_kernel<float, uint16_t>), grid, dim3(256), 0, st, (const float*)src,
                       (const UnpackDesc*)descs, ndesc, (uint16_t*)wbuf, ntiles, sc);
  return (int)hipGetLastError();
}

int psx_unpack_desc_size() { return (int)sizeof(UnpackDesc); }

// dst[i] = src[idx[i]] (fp32, int64 indices): the fp32 remainder of the fetch payload
// (parallel/codec.py WeightWire.small) for the native server loop (csrc/server/event_loop.cpp).
int psx_gather_f32(const float* src, const long* idx, long n, float* dst, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gather_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, src, idx, (size_t)n, dst);
  return (int)hipGetLastError();
}

}  // extern "C"
