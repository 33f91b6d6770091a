// The ResNet stem as an implicit-GEMM MFMA convolution (gfx950): 7x7, stride 2,
// padding 3, over 3 input channels, NHWC, for the grouped step's k workers.
//
// The generic path of the grouped executor runs this layer as im2col (a [pixels, 152]
// patch matrix: 156 MB for 2000 CIFAR images, written by 8 scalar 2-byte gathers per
// 16-byte store) + a hipBLASLt GEMM that reads it back, and keeps the matrix alive
// for the weight gradient (~170 us forward + ~57 us weight-gradient GEMM per step,
// profiles/r3). Here nothing but the input and the output touch HBM:
//
// * forward: a workgroup owns 256 (bf16; split: 128) consecutive output pixels of one image. It stages
//   the input rows they read (zero-padded borders) and the [64][160] weight matrix
//   (K = 7*7*3 = 147 padded to 5 k-steps of 32) in LDS; v_mfma_f32_16x16x32_bf16
//   with the WEIGHT as the A operand (D's lane = 4 consecutive output channels of
//   one pixel) and the patch values gathered from LDS as B (per-lane tap offsets);
//   the tile leaves through LDS as 16-byte row segments.
// * weight gradient (per worker, no patch matrix): a workgroup owns a slice of one
//   worker's images and accumulates dW[64][160] over their pixels with the
//   pixel index as the MFMA reduction dimension: A = dyᵀ (a [64][32] LDS tile
//   written transposed), B = the patch values of those 32 pixels, gathered from the
//   staged input rows. An image is processed in BANDS of output rows whose input rows
//   fit the LDS budget (one band for CIFAR sizes, 8 bands at 224 x 224). The fp32 slabs
//   of the slices are summed by the deferred split-K reduction of the exchange rows
//   (GradSink.queue_split).
//
// SPLIT (the reference-precision fp32 step): fp32 input / dy / output; every staged value
// is split into three bf16 pieces (LDS holds all three), the weight comes as its three pieces, and
// each product is the six piece products of order <= 2 on the bf16 MFMA with fp32 accumulation
// (see conv_f32.hip).
#include <type_traits>

#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kC = 3, kCout = 64;
// Geometry of the stem: the ResNet-50 / ImageNet 7x7 / stride 2 / pad 3, or the CIFAR ResNet-18
// 3x3 / stride 1 / pad 1 (its 27-deep reduction is one 32-wide k-step). K: taps x channels, KP: K
// padded to whole 32-wide k-steps.
template <int KH_, int S_, int P_>
struct StemShape {
  static constexpr int KH = KH_, KW = KH_, S = S_, P = P_;
  static constexpr int K = KH * KW * kC;
  static constexpr int KP = (K + 31) / 32 * 32;
};
using Stem7 = StemShape<7, 2, 3>;   // K 147, KP 160
using Stem3 = StemShape<3, 1, 1>;   // K 27, KP 32
// output pixels per forward workgroup: 64 * F (F 16-pixel fragments per wave); bf16 takes F = 4
// (a 256-pixel tile stages its input rows and the weights once per ~2.3 ImageNet output rows:
// 3.38 -> 2.52 ms per ImageNet step), the split form F = 2 (three pieces of every operand in registers)
constexpr int kFwdFragBf16 = 4, kFwdFragSplit = 2;
constexpr int kThreads = 256;
constexpr int kMaxPatch = 24576;           // elements of staged input per workgroup (bf16)
constexpr int kMaxPatchSplit = 16384;      // ... per piece array of the split (fp32) form
constexpr int kNP = 3;                     // bf16 pieces per fp32 value (split form)

struct StemGeo {
  int N, H, W, Ho, Wo;
  int pw;          // staged row width in pixels = W + 2P
  int band;        // output rows per weight-gradient band
};

// patch offset (elements) of reduction index k = (ky * 7 + kx) * 3 + ci inside the
// staged rows (row width pw pixels); k >= 147 maps to `zero` (a 0 element)
template <class SH>
__device__ __forceinline__ int tap_offset(int k, int pw, int zero) {
  if (k >= SH::K) return zero;
  const int ky = k / (SH::KW * kC), r = k - ky * (SH::KW * kC);
  const int kx = r / kC, ci = r - kx * kC;
  return (ky * pw + kx) * kC + ci;
}

// Stage input rows [iy0, iy0 + rows) of image n into LDS as [rows][pw][3] (zero outside the image).
// A staged row is the image row's 3W contiguous elements between 3P zero elements on each side;
// the (row, column) position advances without divisions, and each thread issues kStageBatch
// independent loads before its LDS stores (one memory latency per batch, not per element).
// SPLIT: x is fp32 and each value lands as three pieces in patch, patch + pstride, patch + 2 pstride.
constexpr int kStageBatch = 8;
template <class SH, bool SPLIT>
__device__ __forceinline__ void stage_rows(const void* __restrict__ xv, const StemGeo& g, int n, int iy0, int rows,
                                           uint16_t* patch, int pstride) {
  const int per_row = g.pw * kC, row_len = g.W * kC;
  const int total = rows * per_row;
  const int64_t img = static_cast<int64_t>(n) * g.H * row_len - SH::P * kC;   // (iy, c) at img + iy*row_len + c
  const int dr = kThreads / per_row, dc = kThreads - dr * per_row;
  int e = threadIdx.x, r = e / per_row, c = e - r * per_row;
  while (e < total) {
    float v[kStageBatch];
    int pos[kStageBatch];
#pragma unroll
    for (int b = 0; b < kStageBatch; ++b) {
      const int iy = iy0 + r;
      v[b] = 0.f;
      if (e < total && iy >= 0 && iy < g.H && c >= SH::P * kC && c < SH::P * kC + row_len) {
        const int64_t o = img + static_cast<int64_t>(iy) * row_len + c;
        if constexpr (SPLIT) v[b] = static_cast<const float*>(xv)[o];
        else v[b] = bf16_to_f(static_cast<const uint16_t*>(xv)[o]);
      }
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
      if (pos[b] < total) {
        if constexpr (SPLIT) {
          float r = v[b];
#pragma unroll
          for (int i = 0; i < kNP; ++i) {
            const uint16_t h = f_to_bf16(r);
            patch[i * pstride + pos[b]] = h;
            r -= bf16_to_f(h);
          }
        } else {
          patch[pos[b]] = f_to_bf16(v[b]);
        }
      }
  }
}

__device__ __forceinline__ bf16x8 u8_to_bf16x8(const uint16_t (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = __builtin_bit_cast(__bf16, v[j]);
  return r;
}

// the six piece products of order <= 2 (split form), the small terms first
__device__ __forceinline__ f32x4 mma6(const bf16x8 (&a)[kNP], const bf16x8 (&b)[kNP], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
}

template <class SH, bool SPLIT, int F>
__global__ __launch_bounds__(kThreads) void k_stem_fwd(const void* __restrict__ x, const uint16_t* __restrict__ w,
                                                       StemGeo g, void* __restrict__ y, int wpitch) {
  // LDS (dynamic, sized by the host for this geometry): weights [64][160] (x3 split) | staged
  // input rows (+1 zero) (x3 split); the output tile reuses the whole area
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int NP = SPLIT ? kNP : 1;
  uint16_t* wl = lds;
  constexpr int kTile = 64 * F;
  const int tiles = (g.Ho * g.Wo + kTile - 1) / kTile;
  const int n = blockIdx.x / tiles;
  const int p0 = (blockIdx.x - n * tiles) * kTile;
  const int npix = g.Ho * g.Wo - p0 < kTile ? g.Ho * g.Wo - p0 : kTile;
  const int oy0 = p0 / g.Wo, oy1 = (p0 + npix - 1) / g.Wo;
  const int iy0 = oy0 * SH::S - SH::P;
  const int rows = (oy1 - oy0) * SH::S + SH::KH;
  const int zero = rows * g.pw * kC;
  uint16_t* patch = lds + NP * kCout * SH::KP;
  const int pstride = zero + 8;   // elements between the piece arrays of the staged rows
  // weights: the zero-padded [64][160] bf16 matrix (columns in the channels_last weight's
  // (ky, kx, ci) order; split: its three pieces one after the other), 16-byte loads; or
  // (wpitch = 147) the channels_last bf16 weight itself, padded while it is staged (no per-step
  // padding copy)
  if (wpitch == SH::KP) {
    for (int e = threadIdx.x; e < NP * kCout * SH::KP / 8; e += kThreads)
      reinterpret_cast<uint4*>(wl)[e] = reinterpret_cast<const uint4*>(w)[e];
  } else {   // 64 x 147 contiguous bf16 (18816 bytes, 16-byte aligned): 16-byte loads, scattered into rows
    for (int e = threadIdx.x; e < kCout * SH::K / 8; e += kThreads) {
      const uint4 v = reinterpret_cast<const uint4*>(w)[e];
      const uint32_t h[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int q = e * 8 + i, r = q / SH::K, c = q - (q / SH::K) * SH::K;
        wl[r * SH::KP + c] = static_cast<uint16_t>((i & 1) ? (h[i >> 1] >> 16) : (h[i >> 1] & 0xffffu));
      }
    }
    for (int e = threadIdx.x; e < kCout * (SH::KP - SH::K); e += kThreads) {
      const int r = e / (SH::KP - SH::K);
      wl[r * SH::KP + SH::K + (e - r * (SH::KP - SH::K))] = 0;
    }
  }
  stage_rows<SH, SPLIT>(x, g, n, iy0, rows, patch, pstride);
  if (threadIdx.x < NP) patch[threadIdx.x * pstride + zero] = 0;
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  // this wave's pixels: [wave * 16F, wave * 16F + 16F) of the tile, F 16-pixel fragments
  int pbase[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    int p = p0 + wave * 16 * F + f * 16 + fr;
    if (p > p0 + npix - 1) p = p0 + npix - 1;   // clamp: computed, never stored
    const int oy = p / g.Wo, ox = p - oy * g.Wo;
    pbase[f] = ((oy * SH::S - SH::P - iy0) * g.pw + ox * SH::S) * kC;
  }
  f32x4 acc[F][4];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[f][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < SH::KP / 32; ++s) {
    const int kb = s * 32 + fq * 8;
    int off[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) off[j] = tap_offset<SH>(kb + j, g.pw, zero);
    bf16x8 bx[F][NP];
#pragma unroll
    for (int f = 0; f < F; ++f) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        uint16_t vh[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) vh[j] = patch[i * pstride + (off[j] == zero ? zero : pbase[f] + off[j])];
        bx[f][i] = u8_to_bf16x8(vh);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bf16x8 aw[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i)
        aw[i] = *reinterpret_cast<const bf16x8*>(wl + i * kCout * SH::KP + (c * 16 + fr) * SH::KP + kb);
#pragma unroll
      for (int f = 0; f < F; ++f) {
        if constexpr (SPLIT) acc[f][c] = mma6(aw, bx[f], acc[f][c]);
        else acc[f][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[0], bx[f][0], acc[f][c], 0, 0, 0);
      }
    }
  }
  // epilogue: D lane = pixel fr of fragment f, channels 16c + 4fq .. +3 -> LDS tile [128][64] -> 16-byte rows
  __syncthreads();   // every wave's weight and patch reads are done: reuse the area
  if constexpr (SPLIT) {
    float* tile = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const int pl = wave * 16 * F + f * 16 + fr;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        *reinterpret_cast<float4*>(tile + pl * kCout + c * 16 + fq * 4) =
            make_float4(acc[f][c][0], acc[f][c][1], acc[f][c][2], acc[f][c][3]);
    }
    __syncthreads();
    float* out = static_cast<float*>(y) + (static_cast<int64_t>(n) * g.Ho * g.Wo + p0) * kCout;
    for (int e = threadIdx.x; e < npix * (kCout / 4); e += kThreads)
      *reinterpret_cast<float4*>(out + e * 4) = *reinterpret_cast<const float4*>(tile + e * 4);
  } else {
    uint16_t* tile = lds;
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const int pl = wave * 16 * F + f * 16 + fr;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint2 o;
        o.x = pack_bf16x2(acc[f][c][0], acc[f][c][1]);
        o.y = pack_bf16x2(acc[f][c][2], acc[f][c][3]);
        *reinterpret_cast<uint2*>(tile + pl * kCout + c * 16 + fq * 4) = o;
      }
    }
    __syncthreads();
    uint16_t* out = static_cast<uint16_t*>(y) + (static_cast<int64_t>(n) * g.Ho * g.Wo + p0) * kCout;
    for (int e = threadIdx.x; e < npix * (kCout / 8); e += kThreads)
      *reinterpret_cast<uint4*>(out + e * 8) = *reinterpret_cast<const uint4*>(tile + e * 8);
  }
}

// bf16 7x7 stem forward on a channel-padded staging: input rows as [rows][pw][4] (channel 3 = 0) and the
// weight as [64][7 ky][8 kx][4 ci] (kx 7 and ci 3 zero; written once per call by k_stem_wprep), so k-step
// s is kernel row ky and a lane's 8 consecutive reduction elements (taps kx = 2 fq, 2 fq + 1, 4 channels
// each) of one pixel are ONE aligned ds_read_b128 (even staged row width) instead of k_stem_fwd's 8
// scalar LDS gathers: 7 k-steps of 32 instead of 5 (40% more MFMA work on zeros). The output tile leaves
// through LDS rows of 72 elements (a 64-element pitch put the 16 pixels of a fragment in one bank).
constexpr int kKP4 = 7 * 32;
constexpr int kTileP = kCout + 8;

__global__ __launch_bounds__(kThreads) void k_stem_wprep(const uint16_t* __restrict__ w, int wpitch,
                                                         uint16_t* __restrict__ wp4) {
  const int e = blockIdx.x * kThreads + threadIdx.x;
  if (e >= kCout * kKP4) return;
  const int co = e / kKP4, k4 = e - co * kKP4;
  const int ky = k4 >> 5, kx = (k4 >> 2) & 7, ci = k4 & 3;
  wp4[e] = (kx < 7 && ci < 3) ? w[co * wpitch + (ky * 7 + kx) * 3 + ci] : static_cast<uint16_t>(0);
}

__device__ __forceinline__ void stage_rows4(const uint16_t* __restrict__ x, const StemGeo& g, int n, int iy0, int rows,
                                            uint16_t* patch) {
  const int total = rows * g.pw;   // staged pixels
  const int64_t img = static_cast<int64_t>(n) * g.H * g.W;
  for (int e0 = threadIdx.x; e0 < total; e0 += kThreads * kStageBatch) {
    uint32_t lo[kStageBatch], hi[kStageBatch];
#pragma unroll
    for (int b = 0; b < kStageBatch; ++b) {
      const int e = e0 + b * kThreads;
      const int r = e / g.pw, c = e - r * g.pw - Stem7::P;   // staged pixel -> image column
      const int iy = iy0 + r;
      lo[b] = 0u;
      hi[b] = 0u;
      if (e < total && iy >= 0 && iy < g.H && c >= 0 && c < g.W) {
        const uint16_t* px = x + (img + static_cast<int64_t>(iy) * g.W + c) * kC;
        lo[b] = static_cast<uint32_t>(px[0]) | (static_cast<uint32_t>(px[1]) << 16);
        hi[b] = px[2];
      }
    }
#pragma unroll
    for (int b = 0; b < kStageBatch; ++b) {
      const int e = e0 + b * kThreads;
      if (e < total) *reinterpret_cast<uint2*>(patch + static_cast<int64_t>(e) * 4) = make_uint2(lo[b], hi[b]);
    }
  }
}

// stats (optional): the consuming BatchNorm's statistics of this tile's stored bf16 values, in
// gemm_nt.hip's tile layout ([tile][entry 1][slot 2][n, Σy, Σ(y - ȳ)²][64], slot 0 only: a tile lies in
// one image, so in one worker), merged by bn_finalize_tiles: the BatchNorm forward then has no partial pass
template <int F>
__global__ __launch_bounds__(kThreads) void k_stem_fwd4(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wp4,
                                                        StemGeo g, uint16_t* __restrict__ y, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* wl = lds;                         // [64][224]
  uint16_t* patch = lds + kCout * kKP4;       // [rows][pw][4]
  constexpr int kTile = 64 * F;
  const int tiles = (g.Ho * g.Wo + kTile - 1) / kTile;
  const int n = blockIdx.x / tiles;
  const int p0 = (blockIdx.x - n * tiles) * kTile;
  const int npix = g.Ho * g.Wo - p0 < kTile ? g.Ho * g.Wo - p0 : kTile;
  const int oy0 = p0 / g.Wo, oy1 = (p0 + npix - 1) / g.Wo;
  const int iy0 = oy0 * Stem7::S - Stem7::P;
  const int rows = (oy1 - oy0) * Stem7::S + Stem7::KH;
  for (int e = threadIdx.x; e < kCout * kKP4 / 8; e += kThreads)
    reinterpret_cast<uint4*>(wl)[e] = reinterpret_cast<const uint4*>(wp4)[e];
  stage_rows4(x, g, n, iy0, rows, patch);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  int pbase[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    int p = p0 + wave * 16 * F + f * 16 + fr;
    if (p > p0 + npix - 1) p = p0 + npix - 1;   // clamp: computed, never stored
    const int oy = p / g.Wo, ox = p - oy * g.Wo;
    pbase[f] = ((oy * Stem7::S - Stem7::P - iy0) * g.pw + ox * Stem7::S + 2 * fq) * 4;
  }
  f32x4 acc[F][4];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[f][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    bf16x8 bx[F];
#pragma unroll
    for (int f = 0; f < F; ++f) bx[f] = *reinterpret_cast<const bf16x8*>(patch + pbase[f] + s * g.pw * 4);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 aw = *reinterpret_cast<const bf16x8*>(wl + (c * 16 + fr) * kKP4 + s * 32 + fq * 8);
#pragma unroll
      for (int f = 0; f < F; ++f) acc[f][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, bx[f], acc[f][c], 0, 0, 0);
    }
  }
  __syncthreads();   // every wave's weight and patch reads are done: reuse the area
  uint16_t* tile = lds;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int pl = wave * 16 * F + f * 16 + fr;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint2 o;
      o.x = pack_bf16x2(acc[f][c][0], acc[f][c][1]);
      o.y = pack_bf16x2(acc[f][c][2], acc[f][c][3]);
      *reinterpret_cast<uint2*>(tile + pl * kTileP + c * 16 + fq * 4) = o;
    }
  }
  __syncthreads();
  uint16_t* out = y + (static_cast<int64_t>(n) * g.Ho * g.Wo + p0) * kCout;
  for (int e = threadIdx.x; e < npix * (kCout / 8); e += kThreads)
    *reinterpret_cast<uint4*>(out + e * 8) = *reinterpret_cast<const uint4*>(tile + (e >> 3) * kTileP + (e & 7) * 8);
  if (stats == nullptr) return;
  // channel c = thread % 64 over every 4th pixel from part = thread / 64, shifted by the tile's first
  // stored value (no cancellation whatever |mean| / std), the 4 parts summed in order through LDS
  const int c = threadIdx.x & 63, part = threadIdx.x >> 6;
  const float sh = bf16_to_f(tile[c]);
  float sd = 0.f, sq = 0.f;
  for (int p = part; p < npix; p += 4) {
    const float d = bf16_to_f(tile[p * kTileP + c]) - sh;
    sd += d;
    sq = fmaf(d, d, sq);
  }
  __syncthreads();   // the tile reads are done: reuse its first bytes for the parts
  float* red = reinterpret_cast<float*>(lds);
  red[part * 64 + c] = sd;
  red[256 + part * 64 + c] = sq;
  __syncthreads();
  if (part == 0) {
    const float D = red[c] + red[64 + c] + red[128 + c] + red[192 + c];
    const float Q = red[256 + c] + red[320 + c] + red[384 + c] + red[448 + c];
    const float nn = static_cast<float>(npix);
    float* ps = stats + static_cast<int64_t>(blockIdx.x) * 2 * 3 * kCout;   // tile = blockIdx.x, slot 0
    ps[c] = nn;
    ps[kCout + c] = D + nn * sh;
    ps[2 * kCout + c] = fmaxf(Q - D * D / nn, 0.f);
  }
}

// Weight gradient: workgroup (slice s, worker g) sums over images [i0, i1) of worker g, each in
// bands of g.band output rows. Pixels are processed 32 at a time (one MFMA reduction step): the
// dy tile [32][64] is written transposed into LDS ([64][32 + pad]). The 7x7 stem (10 k-blocks of 16
// taps): each of the 4 waves owns every output channel (4 dyT fragments) and the k-blocks
// wave, wave + 4, wave + 8, so each patch column is gathered from LDS once per tile, not once per
// wave (the gathers were 80 scalar LDS reads per lane per tile, 4x redundant); the 3x3 stem (2
// k-blocks): each wave owns 16 output channels and both k-blocks.
// bf16 per transposed dy row: 34 (17 dwords), so the 8 rows a wave's transposing 2-byte stores hit at once
// (channels 8 cv + i, cv = 0..7) fall in 8 different bank groups; the A fragments are then read as four
// dwords (rows are 4-byte, not 16-byte, aligned). A 40-element pitch put them 4 / 8 to a bank.
constexpr int kDyPitch = 34;

template <class SH, bool SPLIT>
__global__ __launch_bounds__(kThreads) void k_stem_wgrad(const void* __restrict__ x, const void* __restrict__ dy,
                                                         StemGeo g, int imgs_per_worker, int slices,
                                                         float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];   // dynamic: sized by the host
  constexpr int NP = SPLIT ? kNP : 1;
  uint16_t* dyt = lds;                            // [64][kDyPitch] (x3 split: the pieces one after the other)
  const int brows = (g.band - 1) * SH::S + SH::KH;   // input rows a band's outputs read
  const int zero = brows * g.pw * kC;
  uint16_t* patch = lds + NP * kCout * kDyPitch;  // one band's input rows (x3 split)
  const int pstride = zero + 8;
  const int s = blockIdx.x, grp = blockIdx.y;
  const int per = (imgs_per_worker + slices - 1) / slices;
  const int i0 = grp * imgs_per_worker + s * per;
  int i1 = i0 + per;
  if (i1 > (grp + 1) * imgs_per_worker) i1 = (grp + 1) * imgs_per_worker;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  constexpr int NKB = SH::KP / 16;
  constexpr bool KSPLIT = NKB >= 8;                  // k-blocks dealt to the waves (the 7x7 stem)
  constexpr int KBW = KSPLIT ? (NKB + 3) / 4 : NKB;  // k-blocks per wave
  constexpr int CF = KSPLIT ? 4 : 1;                 // 16-channel dyT fragments per wave
  // this lane's taps (k = 16 kb + fr of its k-blocks), as staged-row offsets
  int toff[KBW];
#pragma unroll
  for (int i = 0; i < KBW; ++i) {
    const int kb = KSPLIT ? wave + 4 * i : i;
    // padded taps (k >= K) read any staged value: their D columns are never stored
    toff[i] = kb < NKB && kb * 16 + fr < SH::K ? tap_offset<SH>(kb * 16 + fr, g.pw, zero) : 0;
  }
  f32x4 acc[CF][KBW];
#pragma unroll
  for (int c = 0; c < CF; ++c)
#pragma unroll
    for (int i = 0; i < KBW; ++i) acc[c][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int npix = g.Ho * g.Wo;
  const int pq = threadIdx.x >> 3, cv = threadIdx.x & 7;   // this thread's 8 channels of one dy pixel
  for (int n = i0; n < i1; ++n) {
    for (int ob0 = 0; ob0 < g.Ho; ob0 += g.band) {
      const int ob1 = ob0 + g.band < g.Ho ? ob0 + g.band : g.Ho;
      const int q_lo = ob0 * g.Wo, q_hi = ob1 * g.Wo;      // the band's pixels [q_lo, q_hi)
      __syncthreads();   // the previous band's patch reads are done
      stage_rows<SH, SPLIT>(x, g, n, ob0 * SH::S - SH::P, (ob1 - ob0 - 1) * SH::S + SH::KH, patch, pstride);
      if (threadIdx.x < NP) patch[threadIdx.x * pstride + zero] = 0;
      const int64_t dyi = static_cast<int64_t>(n) * npix * kCout;
      // the next tile's load is issued before the current tile's MFMAs (one latency per band, not per tile)
      // (bf16: the raw 16-byte vector, written to LDS as loaded)
      auto load_dy = [&](int q0, float (&v)[8], uint4& raw) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.f;
        raw = make_uint4(0u, 0u, 0u, 0u);
        if (q0 + pq < q_hi) {
          if constexpr (SPLIT) load_vec<kF32, 8>(dy, dyi + static_cast<int64_t>(q0 + pq) * kCout + cv * 8, v);
          else raw = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(dy) + dyi +
                                                    static_cast<int64_t>(q0 + pq) * kCout + cv * 8);
        }
      };
      float vnext[8];
      uint4 rnext;
      load_dy(q_lo, vnext, rnext);
      for (int q0 = q_lo; q0 < q_hi; q0 += 32) {
        __syncthreads();   // previous dy tile consumed (and, first time, the band staged)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (SPLIT) {
            float r = vnext[i];
#pragma unroll
            for (int pc = 0; pc < NP; ++pc) {
              const uint16_t h = f_to_bf16(r);
              dyt[pc * kCout * kDyPitch + (cv * 8 + i) * kDyPitch + pq] = h;
              r -= bf16_to_f(h);
            }
          } else {
            const uint32_t wd = i < 2 ? rnext.x : (i < 4 ? rnext.y : (i < 6 ? rnext.z : rnext.w));
            dyt[(cv * 8 + i) * kDyPitch + pq] = static_cast<uint16_t>((i & 1) ? (wd >> 16) : (wd & 0xffffu));
          }
        }
        if (q0 + 32 < q_hi) load_dy(q0 + 32, vnext, rnext);
        __syncthreads();
        // A = dyᵀ: lane holds channel (16 c + fr; c = wave without KSPLIT), pixels q0 + 8 fq .. +7
        bf16x8 a[CF][NP];
#pragma unroll
        for (int c = 0; c < CF; ++c)
#pragma unroll
          for (int pc = 0; pc < NP; ++pc)
          {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(dyt + pc * kCout * kDyPitch +
                                                                    ((KSPLIT ? c : wave) * 16 + fr) * kDyPitch + fq * 8);
            a[c][pc] = __builtin_bit_cast(bf16x8, make_uint4(src[0], src[1], src[2], src[3]));
          }
        // B: pixels q0 + 8 fq + j (rows of the reduction), tap k = 16 kb + fr (column)
        // (the 8 pixels are consecutive: one division, then column steps with a row wrap)
        int pb[8];
        {
          const int p = q0 + fq * 8;
          int oy = p / g.Wo, ox = p - oy * g.Wo;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            // band staged from row ob0*S - P; pixels past the band (dy zero-filled) read the first staged value
            pb[j] = p + j < q_hi ? ((oy - ob0) * SH::S * g.pw + ox * SH::S) * kC : 0;
            if (++ox == g.Wo) {
              ox = 0;
              ++oy;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < KBW; ++i) {
          if (KSPLIT && wave + 4 * i >= NKB) continue;   // wave-uniform: waves 2, 3 own two k-blocks
          bf16x8 b[NP];
#pragma unroll
          for (int pc = 0; pc < NP; ++pc) {
            uint16_t vh[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
              vh[j] = patch[pc * pstride + pb[j] + toff[i]];
            b[pc] = u8_to_bf16x8(vh);
          }
#pragma unroll
          for (int c = 0; c < CF; ++c) {
            if constexpr (SPLIT) acc[c][i] = mma6(a[c], b, acc[c][i]);
            else acc[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c][0], b[0], acc[c][i], 0, 0, 0);
          }
        }
      }
    }
  }
  // D[co][k]: col = k = 16 kb + fr, rows co = 16 c + 4 fq + r (c = wave without KSPLIT); slab [slices][G][64][K]
  float* o = part + (static_cast<int64_t>(s) * gridDim.y + grp) * kCout * SH::K;
#pragma unroll
  for (int i = 0; i < KBW; ++i) {
    const int kb = KSPLIT ? wave + 4 * i : i;
    const int k = kb * 16 + fr;
    if (kb >= NKB || k >= SH::K) continue;
#pragma unroll
    for (int c = 0; c < CF; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(((KSPLIT ? c : wave) * 16) + fq * 4 + r) * SH::K + k] = acc[c][i][r];
  }
}

template <class SH>
StemGeo geo(int N, int H, int W, bool split = false) {
  StemGeo g{};
  g.N = N;
  g.H = H;
  g.W = W;
  g.Ho = (H + 2 * SH::P - SH::KH) / SH::S + 1;
  g.Wo = (W + 2 * SH::P - SH::KW) / SH::S + 1;
  g.pw = W + 2 * SH::P;
  // weight-gradient bands: as many output rows as the staged input rows allow
  const int max_rows = (split ? kMaxPatchSplit : kMaxPatch) / (g.pw * kC) - 1;
  int band = max_rows >= SH::KH ? (max_rows - SH::KH) / SH::S + 1 : 0;
  g.band = band > g.Ho ? g.Ho : band;
  return g;
}

template <class SH>
int fwd_rows(const StemGeo& g, int tile) { return ((tile + g.Wo - 1) / g.Wo) * SH::S + SH::KH; }   // max staged rows per tile

template <class K>
void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(bytes));
}

template <class SH>
bool supported_t(int H, int W) {
  if (H <= 0 || W <= 0) return false;
  const StemGeo g = geo<SH>(1, H, W), gs = geo<SH>(1, H, W, true);
  return fwd_rows<SH>(g, 64 * kFwdFragBf16) * g.pw * kC < kMaxPatch &&
         fwd_rows<SH>(g, 64 * kFwdFragSplit) * g.pw * kC < kMaxPatchSplit && g.band >= 1 && gs.band >= 1;
}

template <class SH>
void fwd_t(const void* x, const uint16_t* w, bool split, int N, int H, int W, void* y, hipStream_t stream, int wpitch,
           uint16_t* scratch, float* stats) {
  const StemGeo g = geo<SH>(N, H, W, split);
  const int T = 64 * (split ? kFwdFragSplit : kFwdFragBf16);
  const int tiles = (g.Ho * g.Wo + T - 1) / T;
  const int np = split ? kNP : 1;
  size_t lds = (static_cast<size_t>(np) * kCout * SH::KP +
                np * (static_cast<size_t>(fwd_rows<SH>(g, T)) * g.pw * kC + 8)) * 2;
  const size_t tile = static_cast<size_t>(T) * kCout * (split ? 4 : 2);
  if (lds < tile) lds = tile;
  if (split) {
    allow_lds(k_stem_fwd<SH, true, kFwdFragSplit>, lds);
    hipLaunchKernelGGL((k_stem_fwd<SH, true, kFwdFragSplit>), dim3(N * tiles), dim3(kThreads), lds, stream, x, w, g, y,
                       SH::KP);
  } else if (std::is_same<SH, Stem7>::value && g.pw % 2 == 0 && scratch != nullptr) {   // channel-padded form
    const int wp = wpitch == SH::K ? SH::K : SH::KP;
    hipLaunchKernelGGL(k_stem_wprep, dim3((kCout * kKP4 + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, w, wp,
                       scratch);
    size_t lds4 = (static_cast<size_t>(kCout) * kKP4 + static_cast<size_t>(fwd_rows<SH>(g, T)) * g.pw * 4) * 2;
    const size_t tile4 = static_cast<size_t>(T) * kTileP * 2;
    if (lds4 < tile4) lds4 = tile4;
    allow_lds(k_stem_fwd4<kFwdFragBf16>, lds4);
    hipLaunchKernelGGL((k_stem_fwd4<kFwdFragBf16>), dim3(N * tiles), dim3(kThreads), lds4, stream,
                       static_cast<const uint16_t*>(x), scratch, g, static_cast<uint16_t*>(y), stats);
  } else {
    allow_lds(k_stem_fwd<SH, false, kFwdFragBf16>, lds);
    hipLaunchKernelGGL((k_stem_fwd<SH, false, kFwdFragBf16>), dim3(N * tiles), dim3(kThreads), lds, stream, x, w, g, y,
                       wpitch == SH::K ? SH::K : SH::KP);
  }
}

template <class SH>
void wgrad_t(const void* x, const void* dy, int N, int H, int W, int groups, int slices, float* part, bool split,
             hipStream_t stream) {
  const StemGeo g = geo<SH>(N, H, W, split);
  const int np = split ? kNP : 1;
  const size_t brows = static_cast<size_t>((g.band - 1) * SH::S + SH::KH);
  const size_t lds = (static_cast<size_t>(np) * kCout * kDyPitch + np * (brows * g.pw * kC + 8)) * 2;
  if (split) {
    allow_lds(k_stem_wgrad<SH, true>, lds);
    hipLaunchKernelGGL((k_stem_wgrad<SH, true>), dim3(slices, groups), dim3(kThreads), lds, stream, x, dy, g,
                       N / groups, slices, part);
  } else {
    allow_lds(k_stem_wgrad<SH, false>, lds);
    hipLaunchKernelGGL((k_stem_wgrad<SH, false>), dim3(slices, groups), dim3(kThreads), lds, stream, x, dy, g,
                       N / groups, slices, part);
  }
}

}  // namespace

int stem_k(int kind) { return kind == kStem3x3 ? Stem3::K : Stem7::K; }
int stem_kp(int kind) { return kind == kStem3x3 ? Stem3::KP : Stem7::KP; }

bool stem_supported(int H, int W, int kind) {
  return kind == kStem3x3 ? supported_t<Stem3>(H, W) : supported_t<Stem7>(H, W);
}

int stem_fwd_scratch(int kind) { return kind == kStem3x3 ? 0 : kCout * kKP4; }

int64_t stem_fwd_stat_tiles(int N, int H, int W, int kind) {
  if (kind == kStem3x3) return 0;
  const StemGeo g = geo<Stem7>(N, H, W);
  const int T = 64 * kFwdFragBf16;
  if (g.pw % 2 != 0 || (g.Ho * g.Wo) % T != 0) return 0;   // the channel-padded form, tiles of whole images
  return static_cast<int64_t>(N) * (g.Ho * g.Wo / T);
}

void stem_fwd(const void* x, const uint16_t* w, bool split, int N, int H, int W, void* y, hipStream_t stream,
              int wpitch, int kind, uint16_t* scratch, float* stats) {
  if (kind == kStem3x3) fwd_t<Stem3>(x, w, split, N, H, W, y, stream, wpitch, nullptr, nullptr);
  else fwd_t<Stem7>(x, w, split, N, H, W, y, stream, wpitch, scratch, split ? nullptr : stats);
}

void stem_wgrad(const void* x, const void* dy, int N, int H, int W, int groups, int slices, float* part, bool split,
                hipStream_t stream, int kind) {
  if (kind == kStem3x3) wgrad_t<Stem3>(x, dy, N, H, W, groups, slices, part, split, stream);
  else wgrad_t<Stem7>(x, dy, N, H, W, groups, slices, part, split, stream);
}

}  // namespace gpu
}  // namespace garfield
