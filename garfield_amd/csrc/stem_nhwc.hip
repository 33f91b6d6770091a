// The ResNet stem as an implicit-GEMM MFMA convolution (gfx950): 7x7, stride 2,
// padding 3, over 3 input channels, NHWC bf16, for the grouped step's k workers.
//
// The generic path of the grouped executor runs this layer as im2col (a [pixels, 152]
// patch matrix: 156 MB for 2000 CIFAR images, written by 8 scalar 2-byte gathers per
// 16-byte store) + a hipBLASLt GEMM that reads it back, and keeps the matrix alive
// for the weight gradient (~170 us forward + ~57 us weight-gradient GEMM per step,
// profiles/r3). Here nothing but the input (12 MB) and the output (65 MB) touch HBM:
//
// * forward: a workgroup owns 128 consecutive output pixels of one image. It stages
//   the input rows they read (zero-padded borders) and the [64][160] weight matrix
//   (K = 7*7*3 = 147 padded to 5 k-steps of 32) in LDS; v_mfma_f32_16x16x32_bf16
//   with the WEIGHT as the A operand (D's lane = 4 consecutive output channels of
//   one pixel) and the patch values gathered from LDS as B (per-lane tap offsets);
//   the tile leaves through LDS as 16-byte row segments.
// * weight gradient (per worker, no patch matrix): a workgroup owns a slice of one
//   worker's images and accumulates dW[64][160] over their pixels with the
//   pixel index as the MFMA reduction dimension: A = dyᵀ (a [64][32] LDS tile
//   written transposed), B = the patch values of those 32 pixels, gathered from the
//   staged input rows. The fp32 slabs of the slices are summed by the deferred
//   split-K reduction of the exchange rows (GradSink.queue_split).
#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kC = 3, kKH = 7, kKW = 7, kS = 2, kP = 3, kCout = 64;
constexpr int kK = kKH * kKW * kC;        // 147
constexpr int kKP = 160;                   // padded to 5 k-steps of 32
constexpr int kTile = 128;                 // output pixels per forward workgroup
constexpr int kThreads = 256;
constexpr int kMaxPatch = 24576;           // elements (48 KB) of staged input per workgroup

struct StemGeo {
  int N, H, W, Ho, Wo;
  int pw;          // staged row width in pixels = W + 2P
};

// patch offset (elements) of reduction index k = (ky * 7 + kx) * 3 + ci inside the
// staged rows (row width pw pixels); k >= 147 maps to `zero` (a 0 element)
__device__ __forceinline__ int tap_offset(int k, int pw, int zero) {
  if (k >= kK) return zero;
  const int ky = k / (kKW * kC), r = k - ky * (kKW * kC);
  const int kx = r / kC, ci = r - kx * kC;
  return (ky * pw + kx) * kC + ci;
}

// Stage input rows [iy0, iy0 + rows) of image n into LDS as [rows][pw][3] (zero outside the image).
// A staged row is the image row's 3W contiguous elements between 3P zero elements on each side;
// the (row, column) position advances without divisions, and each thread issues kStageBatch
// independent loads before its LDS stores (one memory latency per batch, not per element).
constexpr int kStageBatch = 8;
__device__ __forceinline__ void stage_rows(const uint16_t* __restrict__ x, const StemGeo& g, int n, int iy0, int rows,
                                           uint16_t* patch) {
  const int per_row = g.pw * kC, row_len = g.W * kC;
  const int total = rows * per_row;
  const uint16_t* src = x + static_cast<int64_t>(n) * g.H * row_len - kP * kC;   // (iy, c) at src + iy*row_len + c
  const int dr = kThreads / per_row, dc = kThreads - dr * per_row;
  int e = threadIdx.x, r = e / per_row, c = e - r * per_row;
  while (e < total) {
    uint16_t v[kStageBatch];
    int pos[kStageBatch];
#pragma unroll
    for (int b = 0; b < kStageBatch; ++b) {
      const int iy = iy0 + r;
      v[b] = 0;
      if (e < total && iy >= 0 && iy < g.H && c >= kP * kC && c < kP * kC + row_len)
        v[b] = src[static_cast<int64_t>(iy) * row_len + c];
      pos[b] = e;
      e += kThreads;
      c += dc;
      r += dr;
      if (c >= per_row) {
        c -= per_row;
        ++r;
      }
    }
#pragma unroll
    for (int b = 0; b < kStageBatch; ++b)
      if (pos[b] < total) patch[pos[b]] = v[b];
  }
}

__global__ __launch_bounds__(kThreads) void k_stem_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                       StemGeo g, uint16_t* __restrict__ y) {
  // LDS (dynamic, sized by the host for this geometry): weights [64][160] | staged input rows
  // (+1 zero); the [128][64] output tile reuses the whole area
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* wl = lds;
  uint16_t* patch = lds + kCout * kKP;
  const int tiles = (g.Ho * g.Wo + kTile - 1) / kTile;
  const int n = blockIdx.x / tiles;
  const int p0 = (blockIdx.x - n * tiles) * kTile;
  const int npix = g.Ho * g.Wo - p0 < kTile ? g.Ho * g.Wo - p0 : kTile;
  const int oy0 = p0 / g.Wo, oy1 = (p0 + npix - 1) / g.Wo;
  const int iy0 = oy0 * kS - kP;
  const int rows = (oy1 - oy0) * kS + kKH;
  // weights: the zero-padded [64][160] bf16 matrix (columns in the channels_last weight's
  // (ky, kx, ci) order), 16-byte loads
  for (int e = threadIdx.x; e < kCout * kKP / 8; e += kThreads)
    reinterpret_cast<uint4*>(wl)[e] = reinterpret_cast<const uint4*>(w)[e];
  stage_rows(x, g, n, iy0, rows, patch);
  const int zero = rows * g.pw * kC;
  if (threadIdx.x == 0) patch[zero] = 0;
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  // this wave's pixels: [wave * 32, wave * 32 + 32) of the tile, two 16-pixel fragments
  int pbase[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    int p = p0 + wave * 32 + f * 16 + fr;
    if (p > p0 + npix - 1) p = p0 + npix - 1;   // clamp: computed, never stored
    const int oy = p / g.Wo, ox = p - oy * g.Wo;
    pbase[f] = ((oy * kS - kP - iy0) * g.pw + ox * kS) * kC;
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[f][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kKP / 32; ++s) {
    const int kb = s * 32 + fq * 8;
    int off[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) off[j] = tap_offset(kb + j, g.pw, zero);
    bf16x8 bx[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint16_t v = off[j] == zero ? uint16_t(0) : patch[pbase[f] + off[j]];
        bx[f][j] = __builtin_bit_cast(__bf16, v);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 aw = *reinterpret_cast<const bf16x8*>(wl + (c * 16 + fr) * kKP + kb);
#pragma unroll
      for (int f = 0; f < 2; ++f) acc[f][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, bx[f], acc[f][c], 0, 0, 0);
    }
  }
  // epilogue: D lane = pixel fr of fragment f, channels 16c + 4fq .. +3 -> LDS tile [128][64] -> 16-byte rows
  __syncthreads();   // every wave's weight and patch reads are done: reuse the area
  uint16_t* tile = lds;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int pl = wave * 32 + f * 16 + fr;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint2 o;
      o.x = static_cast<uint32_t>(f_to_bf16(acc[f][c][0])) | (static_cast<uint32_t>(f_to_bf16(acc[f][c][1])) << 16);
      o.y = static_cast<uint32_t>(f_to_bf16(acc[f][c][2])) | (static_cast<uint32_t>(f_to_bf16(acc[f][c][3])) << 16);
      *reinterpret_cast<uint2*>(tile + pl * kCout + c * 16 + fq * 4) = o;
    }
  }
  __syncthreads();
  uint16_t* out = y + (static_cast<int64_t>(n) * g.Ho * g.Wo + p0) * kCout;
  for (int e = threadIdx.x; e < npix * (kCout / 8); e += kThreads)
    *reinterpret_cast<uint4*>(out + e * 8) = *reinterpret_cast<const uint4*>(tile + e * 8);
}

// Weight gradient: workgroup (slice s, worker g) sums over images [i0, i1) of worker g.
// Pixels are processed 32 at a time (one MFMA reduction step): the dy tile [32][64] is
// written transposed into LDS ([64][32 + pad]); each of the 4 waves owns 16 output
// channels and all 10 k-blocks of 16 (160 padded taps): acc[10] f32x4.
constexpr int kDyPitch = 40;   // bf16 per transposed dy row (32 + 8: 16-byte aligned, conflict-spread)

__global__ __launch_bounds__(kThreads) void k_stem_wgrad(const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ dy, StemGeo g, int imgs_per_worker,
                                                         int slices, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];   // dynamic: sized by the host
  uint16_t* dyt = lds;                       // [64][kDyPitch]
  uint16_t* patch = lds + kCout * kDyPitch;  // one image's input rows
  const int s = blockIdx.x, grp = blockIdx.y;
  const int per = (imgs_per_worker + slices - 1) / slices;
  const int i0 = grp * imgs_per_worker + s * per;
  int i1 = i0 + per;
  if (i1 > (grp + 1) * imgs_per_worker) i1 = (grp + 1) * imgs_per_worker;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int rows = (g.Ho - 1) * kS + kKH;    // every input row an image's outputs read
  const int zero = rows * g.pw * kC;
  // this lane's 10 taps (k = 16 kb + fr), as staged-row offsets
  int toff[kKP / 16];
#pragma unroll
  for (int kb = 0; kb < kKP / 16; ++kb) toff[kb] = tap_offset(kb * 16 + fr, g.pw, zero);
  f32x4 acc[kKP / 16];
#pragma unroll
  for (int kb = 0; kb < kKP / 16; ++kb) acc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int npix = g.Ho * g.Wo;
  for (int n = i0; n < i1; ++n) {
    __syncthreads();   // the previous image's patch reads are done
    stage_rows(x, g, n, -kP, rows, patch);
    if (threadIdx.x == 0) patch[zero] = 0;
    const uint16_t* dyi = dy + static_cast<int64_t>(n) * npix * kCout;
    // this thread's 16 bytes of a dy tile: pixel q0 + pq, channels 8 cv .. +7; the next
    // tile's load is issued before the current tile's MFMAs (one latency per image, not per tile)
    const int pq = threadIdx.x >> 3, cv = threadIdx.x & 7;
    auto load_dy = [&](int q0) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (q0 + pq < npix) v = *reinterpret_cast<const uint4*>(dyi + static_cast<int64_t>(q0 + pq) * kCout + cv * 8);
      return v;
    };
    uint4 vnext = load_dy(0);
    for (int q0 = 0; q0 < npix; q0 += 32) {
      __syncthreads();   // previous dy tile consumed (and, first time, the patch staged)
      {
        const uint32_t wv[4] = {vnext.x, vnext.y, vnext.z, vnext.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dyt[(cv * 8 + 2 * i) * kDyPitch + pq] = static_cast<uint16_t>(wv[i] & 0xffffu);
          dyt[(cv * 8 + 2 * i + 1) * kDyPitch + pq] = static_cast<uint16_t>(wv[i] >> 16);
        }
      }
      if (q0 + 32 < npix) vnext = load_dy(q0 + 32);
      __syncthreads();
      // A = dyᵀ: lane holds channel (16 wave + fr), pixels q0 + 8 fq .. +7
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(dyt + (wave * 16 + fr) * kDyPitch + fq * 8);
      // B: pixels q0 + 8 fq + j (rows of the reduction), tap k = 16 kb + fr (column)
      // (the 8 pixels are consecutive: one division, then column steps with a row wrap)
      int pb[8];
      {
        const int p = q0 + fq * 8;
        int oy = p / g.Wo, ox = p - oy * g.Wo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[j] = p + j < npix ? (oy * kS * g.pw + ox * kS) * kC : -1;   // rows staged from input row -P
          if (++ox == g.Wo) {
            ox = 0;
            ++oy;
          }
        }
      }
#pragma unroll
      for (int kb = 0; kb < kKP / 16; ++kb) {
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint16_t v = (pb[j] < 0 || toff[kb] == zero) ? uint16_t(0) : patch[pb[j] + toff[kb]];
          b[j] = __builtin_bit_cast(__bf16, v);
        }
        acc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[kb], 0, 0, 0);
      }
    }
  }
  // D[co][k]: col = k = 16 kb + fr, rows co = 16 wave + 4 fq + r; slab [slices][G][64][147]
  float* o = part + (static_cast<int64_t>(s) * gridDim.y + grp) * kCout * kK;
#pragma unroll
  for (int kb = 0; kb < kKP / 16; ++kb) {
    const int k = kb * 16 + fr;
    if (k >= kK) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[(wave * 16 + fq * 4 + r) * kK + k] = acc[kb][r];
  }
}

StemGeo geo(int N, int H, int W) {
  StemGeo g{};
  g.N = N;
  g.H = H;
  g.W = W;
  g.Ho = (H + 2 * kP - kKH) / kS + 1;
  g.Wo = (W + 2 * kP - kKW) / kS + 1;
  g.pw = W + 2 * kP;
  return g;
}

int fwd_rows(const StemGeo& g) { return ((kTile + g.Wo - 1) / g.Wo) * kS + kKH; }   // max staged rows per tile
int wg_rows(const StemGeo& g) { return (g.Ho - 1) * kS + kKH; }                     // every row an image reads

}  // namespace

bool stem_supported(int H, int W) {
  if (H <= 0 || W <= 0) return false;
  const StemGeo g = geo(1, H, W);
  return fwd_rows(g) * g.pw * kC < kMaxPatch && wg_rows(g) * g.pw * kC < kMaxPatch;
}

void stem_fwd(const uint16_t* x, const uint16_t* w, int N, int H, int W, uint16_t* y, hipStream_t stream) {
  const StemGeo g = geo(N, H, W);
  const int tiles = (g.Ho * g.Wo + kTile - 1) / kTile;
  const size_t lds = (static_cast<size_t>(kCout) * kKP + static_cast<size_t>(fwd_rows(g)) * g.pw * kC + 8) * 2;
  hipLaunchKernelGGL(k_stem_fwd, dim3(N * tiles), dim3(kThreads), lds, stream, x, w, g, y);
}

void stem_wgrad(const uint16_t* x, const uint16_t* dy, int N, int H, int W, int groups, int slices, float* part,
                hipStream_t stream) {
  const StemGeo g = geo(N, H, W);
  const size_t lds = (static_cast<size_t>(kCout) * kDyPitch + static_cast<size_t>(wg_rows(g)) * g.pw * kC + 8) * 2;
  hipLaunchKernelGGL(k_stem_wgrad, dim3(slices, groups), dim3(kThreads), lds, stream, x, dy, g, N / groups, slices,
                     part);
}

}  // namespace gpu
}  // namespace garfield
