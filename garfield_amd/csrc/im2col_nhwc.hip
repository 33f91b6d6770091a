// NHWC im2col / col2im (bf16) for the worker-grouped convolutions
// (garfield_amd/ops/grouped.py). With the k logical workers batched, every
// k x k convolution of the grouped step is three GEMMs on hipBLASLt around these
// two gathers, no MIOpen call (MIOpen's NHWC solvers are not HIP-graph replay
// safe on ROCm 7 / gfx950: weight gradients go non-finite from a replay on):
//
//   forward : col = im2col(x);  y = col · Wᵀ              (W: [Cout, KH*KW*Cin], the
//                                                         channels_last weight's memory order)
//   dgrad   : dcol = dy · W;    dx = col2im(dcol)
//   wgrad   : dW_g = dy_gᵀ · col_g for every worker g     (ONE strided-batched GEMM; col's
//                                                         (kh, kw, ci) column order IS the
//                                                         weight's memory order, so each dW_g
//                                                         lands in the exchange row as it is)
//
// col2im is written as a gather (each input pixel sums the taps that read it),
// so it needs no atomics and is deterministic.
#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kThreads = 256;

// Vector path (C % 8 == 0): one thread per 16-byte channel vector of one
// (output pixel, kernel tap); a workgroup covers whole col rows, so every index
// is 32-bit except the final element offsets.
__global__ __launch_bounds__(kThreads) void k_im2col_vec(const uint16_t* __restrict__ x, Im2col g,
                                                        uint16_t* __restrict__ col, int rows_per_wg) {
  const int cv = g.C / 8;
  const int K = g.KH * g.KW * cv;  // vectors per col row
  const int rows = g.N * g.Ho * g.Wo;
  for (int t = threadIdx.x; t < rows_per_wg * K; t += kThreads) {
    const int m = blockIdx.x * rows_per_wg + t / K;
    if (m >= rows) break;
    const int r = t % K;
    const int kp = r / cv, v = r % cv;
    const int i = kp / g.KW, j = kp % g.KW;
    const int wo = m % g.Wo;
    const int ho = (m / g.Wo) % g.Ho;
    const int n = m / (g.Wo * g.Ho);
    const int hi = ho * g.sh - g.ph + i * g.dh;
    const int wi = wo * g.sw - g.pw + j * g.dw;
    uint4 val = make_uint4(0u, 0u, 0u, 0u);
    if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
      val = *reinterpret_cast<const uint4*>(x + ((static_cast<int64_t>(n) * g.H + hi) * g.W + wi) * g.C + v * 8);
    *reinterpret_cast<uint4*>(col + static_cast<int64_t>(m) * g.ldc + static_cast<int64_t>(r) * 8) = val;
  }
}

// Scalar path (any C, e.g. the 3-channel stem); also zero-fills the pad columns.
__global__ __launch_bounds__(kThreads) void k_im2col_scalar(const uint16_t* __restrict__ x, Im2col g,
                                                           uint16_t* __restrict__ col, int rows_per_wg) {
  const int K = g.KH * g.KW * g.C;
  const int L = g.ldc;
  const int rows = g.N * g.Ho * g.Wo;
  for (int t = threadIdx.x; t < rows_per_wg * L; t += kThreads) {
    const int m = blockIdx.x * rows_per_wg + t / L;
    if (m >= rows) break;
    const int r = t % L;
    uint16_t val = 0;
    if (r < K) {
      const int kp = r / g.C, c = r % g.C;
      const int i = kp / g.KW, j = kp % g.KW;
      const int wo = m % g.Wo;
      const int ho = (m / g.Wo) % g.Ho;
      const int n = m / (g.Wo * g.Ho);
      const int hi = ho * g.sh - g.ph + i * g.dh;
      const int wi = wo * g.sw - g.pw + j * g.dw;
      if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
        val = x[((static_cast<int64_t>(n) * g.H + hi) * g.W + wi) * g.C + c];
    }
    col[static_cast<int64_t>(m) * L + r] = val;
  }
}

// Chunked path (any C, ldc % 8 == 0, e.g. the 3-channel stem padded to 152
// columns): one thread gathers 8 consecutive columns of one col row and writes
// them with one 16-byte store. C_/KW_/L8_ != 0 fix the channel count, kernel
// width and 16-byte chunks per row at compile time (the ResNet stem: 3, 7, 19),
// turning the per-element divisions into multiplies; out-of-range taps load a
// clamped in-bounds element and are zeroed by a select (no branch per load).
template <int C_, int KW_, int L8_>
__global__ __launch_bounds__(kThreads) void k_im2col_chunk8(const uint16_t* __restrict__ x, Im2col g,
                                                           uint16_t* __restrict__ col, int rows_per_wg) {
  const int C = C_ ? C_ : g.C;
  const int KW = KW_ ? KW_ : g.KW;
  const int L8 = L8_ ? L8_ : g.ldc / 8;
  const int K = g.KH * KW * C;
  const int rows = g.N * g.Ho * g.Wo;
  for (int t = threadIdx.x; t < rows_per_wg * L8; t += kThreads) {
    const int m = blockIdx.x * rows_per_wg + t / L8;
    if (m >= rows) break;
    const int r0 = (t % L8) * 8;
    const int wo = m % g.Wo;
    const int ho = (m / g.Wo) % g.Ho;
    const int n = m / (g.Wo * g.Ho);
    const int h0 = ho * g.sh - g.ph, w0 = wo * g.sw - g.pw;
    const int64_t nbase = static_cast<int64_t>(n) * g.H;
    uint32_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = r0 + e;
      const int kp = r / C, c = r - (r / C) * C;
      const int hi = h0 + (kp / KW) * g.dh;
      const int wi = w0 + (kp - (kp / KW) * KW) * g.dw;
      const bool ok = r < K && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
      const uint16_t val = x[((nbase + (ok ? hi : 0)) * g.W + (ok ? wi : 0)) * C + (ok ? c : 0)];
      v[e] = ok ? val : 0u;
    }
    uint4 w;
    w.x = v[0] | (v[1] << 16); w.y = v[2] | (v[3] << 16);
    w.z = v[4] | (v[5] << 16); w.w = v[6] | (v[7] << 16);
    *reinterpret_cast<uint4*>(col + static_cast<int64_t>(m) * g.ldc + r0) = w;
  }
}

// (hi, wi) -> output pixel of tap (i, j), or -1.
__device__ __forceinline__ int tap_row(const Im2col& g, int n, int hi, int wi, int i, int j) {
  const int a = hi + g.ph - i * g.dh;
  const int b = wi + g.pw - j * g.dw;
  if (a < 0 || b < 0 || a % g.sh || b % g.sw) return -1;
  const int ho = a / g.sh, wo = b / g.sw;
  if (ho >= g.Ho || wo >= g.Wo) return -1;
  return (n * g.Ho + ho) * g.Wo + wo;
}

// col2im vector path: one thread per 8-channel vector of one input pixel. ACC adds
// into dx (the other branch's gradient of the same input, e.g. a residual block's
// conv1 and downsample), instead of a separate elementwise add.
template <bool ACC>
__global__ __launch_bounds__(kThreads) void k_col2im_vec(const uint16_t* __restrict__ dcol, Im2col g,
                                                        uint16_t* __restrict__ dx) {
  const int cv = g.C / 8;
  const int64_t total = static_cast<int64_t>(g.N) * g.H * g.W * cv;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int v = static_cast<int>(t % cv);
    const int pix = static_cast<int>(t / cv);
    const int wi = pix % g.W;
    const int hi = (pix / g.W) % g.H;
    const int n = pix / (g.W * g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ACC) load_vec<kBF16, 8>(dx, static_cast<int64_t>(pix) * g.C + v * 8, acc);
    for (int i = 0; i < g.KH; ++i) {
      for (int j = 0; j < g.KW; ++j) {
        const int m = tap_row(g, n, hi, wi, i, j);
        if (m < 0) continue;
        float a[8];
        load_vec<kBF16, 8>(dcol, static_cast<int64_t>(m) * g.ldc + (i * g.KW + j) * g.C + v * 8, a);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += a[e];
      }
    }
    store_vec<8>(dx, kBF16, static_cast<int64_t>(pix) * g.C + v * 8, acc);
  }
}

template <bool ACC>
__global__ __launch_bounds__(kThreads) void k_col2im_scalar(const uint16_t* __restrict__ dcol, Im2col g,
                                                           uint16_t* __restrict__ dx) {
  const int64_t total = static_cast<int64_t>(g.N) * g.H * g.W * g.C;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int c = static_cast<int>(t % g.C);
    const int pix = static_cast<int>(t / g.C);
    const int wi = pix % g.W;
    const int hi = (pix / g.W) % g.H;
    const int n = pix / (g.W * g.H);
    float acc = ACC ? bf16_to_f(dx[t]) : 0.f;
    for (int i = 0; i < g.KH; ++i)
      for (int j = 0; j < g.KW; ++j) {
        const int m = tap_row(g, n, hi, wi, i, j);
        if (m >= 0) acc += bf16_to_f(dcol[static_cast<int64_t>(m) * g.ldc + (i * g.KW + j) * g.C + c]);
      }
    dx[t] = f_to_bf16(acc);
  }
}

// Max pooling (NHWC, bf16, C % 8 == 0), forward keeping the window position of
// every output element's maximum as one byte, backward as a gather over the
// windows that cover an input pixel (no scatter, no atomics, no zero fill).
// Ties and NaN follow ATen: the first maximum in (i, j) scan order wins, a NaN
// always wins.
template <int DT>
__global__ __launch_bounds__(kThreads) void k_maxpool_fwd(const void* __restrict__ x, Im2col g,
                                                         void* __restrict__ y, uint8_t* __restrict__ idx) {
  const int cv = g.C / 8;
  const int64_t total = static_cast<int64_t>(g.N) * g.Ho * g.Wo * cv;
  const bool narrow = total <= 0x7fffffff;   // 32-bit index math (the 64-bit divisions dominated)
  const bool pool3s2 = g.KH == 3 && g.KW == 3 && g.sh == 2 && g.sw == 2 && g.ph == 1 && g.pw == 1 && g.dh == 1 &&
                       g.dw == 1;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int v = narrow ? static_cast<int>(t) % cv : static_cast<int>(t % cv);
    const int m = narrow ? static_cast<int>(t) / cv : static_cast<int>(t / cv);
    const int wo = m % g.Wo;
    const int ho = (m / g.Wo) % g.Ho;
    const int n = m / (g.Wo * g.Ho);
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -__builtin_inff(); arg[e] = 0; }
    if (pool3s2) {
      // the ResNet stem pool (3x3, stride 2, pad 1): all nine window loads issued before the first
      // comparison (rows / columns outside the image read a clamped neighbour and are skipped)
      float a[9][8];
      bool ok[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int hi = 2 * ho - 1 + i, wi = 2 * wo - 1 + j;
          ok[i * 3 + j] = hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
          const int hc = hi < 0 ? 0 : (hi >= g.H ? g.H - 1 : hi), wc = wi < 0 ? 0 : (wi >= g.W ? g.W - 1 : wi);
          load_vec<DT, 8>(x, ((static_cast<int64_t>(n) * g.H + hc) * g.W + wc) * g.C + v * 8, a[i * 3 + j]);
        }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (!ok[tap]) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (a[tap][e] > best[e] || (a[tap][e] != a[tap][e] && best[e] == best[e])) { best[e] = a[tap][e]; arg[e] = tap; }
      }
    } else
    for (int i = 0; i < g.KH; ++i) {
      const int hi = ho * g.sh - g.ph + i * g.dh;
      if (hi < 0 || hi >= g.H) continue;
      for (int j = 0; j < g.KW; ++j) {
        const int wi = wo * g.sw - g.pw + j * g.dw;
        if (wi < 0 || wi >= g.W) continue;
        float a[8];
        load_vec<DT, 8>(x, ((static_cast<int64_t>(n) * g.H + hi) * g.W + wi) * g.C + v * 8, a);
        const int tap = i * g.KW + j;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (a[e] > best[e] || (a[e] != a[e] && best[e] == best[e])) { best[e] = a[e]; arg[e] = tap; }
      }
    }
    const int64_t o = static_cast<int64_t>(m) * g.C + v * 8;
    store_vec<8>(y, DT, o, best);
    uint2 packed;
    packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (static_cast<uint32_t>(arg[3]) << 24);
    packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (static_cast<uint32_t>(arg[7]) << 24);
    *reinterpret_cast<uint2*>(idx + o) = packed;
  }
}

template <int DT>
__global__ __launch_bounds__(kThreads) void k_maxpool_bwd(const void* __restrict__ dy,
                                                         const uint8_t* __restrict__ idx, Im2col g,
                                                         void* __restrict__ dx) {
  const int cv = g.C / 8;
  const int64_t total = static_cast<int64_t>(g.N) * g.H * g.W * cv;
  const bool narrow = total <= 0x7fffffff;
  // undilated windows: only the output rows / columns whose window covers (hi, wi) are visited
  // (1-4 of the 9 taps of a 3x3 / 2 pool), in the generic loop's (i, j) order
  const bool unit = g.dh == 1 && g.dw == 1;
  const bool pool3s2 = unit && g.KH == 3 && g.KW == 3 && g.sh == 2 && g.sw == 2 && g.ph == 1 && g.pw == 1;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int v = narrow ? static_cast<int>(t) % cv : static_cast<int>(t % cv);
    const int pix = narrow ? static_cast<int>(t) / cv : static_cast<int>(t / cv);
    const int wi = pix % g.W;
    const int hi = (pix / g.W) % g.H;
    const int n = pix / (g.W * g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto take = [&](int m, int tap) {
      const int64_t o = static_cast<int64_t>(m) * g.C + v * 8;
      const uint2 p = *reinterpret_cast<const uint2*>(idx + o);
      float d[8];
      load_vec<DT, 8>(dy, o, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t word = e < 4 ? p.x : p.y;
        if (static_cast<int>((word >> (8 * (e & 3))) & 0xffu) == tap) acc[e] += d[e];
      }
    };
    if (pool3s2) {
      // 3x3 / 2 / pad 1: at most two covering rows and columns; their four (idx, dy) loads issued before
      // the sums, which run in the general loop's order (ho, then wo, descending)
      const int ah = hi + 1, aw = wi + 1;
      const int ho1 = ah / 2 < g.Ho - 1 ? ah / 2 : g.Ho - 1, wo1 = aw / 2 < g.Wo - 1 ? aw / 2 : g.Wo - 1;
      const int ho0 = ah - 2 <= 0 ? 0 : (ah - 1) / 2, wo0 = aw - 2 <= 0 ? 0 : (aw - 1) / 2;
      uint2 pk[4];
      float d[4][8];
      int tp[4];
      bool ok[4];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int ho = ho1 - a, wo = wo1 - b;
          const int q = a * 2 + b;
          ok[q] = ho >= ho0 && wo >= wo0;
          const int hc = ok[q] ? ho : ho1, wcl = ok[q] ? wo : wo1;
          const int64_t o = (static_cast<int64_t>((n * g.Ho + hc) * g.Wo + wcl)) * g.C + v * 8;
          pk[q] = *reinterpret_cast<const uint2*>(idx + o);
          load_vec<DT, 8>(dy, o, d[q]);
          tp[q] = (ah - ho * 2) * 3 + (aw - wo * 2);
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!ok[q]) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t word = e < 4 ? pk[q].x : pk[q].y;
          if (static_cast<int>((word >> (8 * (e & 3))) & 0xffu) == tp[q]) acc[e] += d[q][e];
        }
      }
    } else if (unit) {
      // window (ho, wo) covers hi iff i = hi + ph - ho*sh lies in [0, KH)
      const int ah = hi + g.ph, aw = wi + g.pw;
      int ho1 = ah / g.sh, wo1 = aw / g.sw;
      if (ho1 > g.Ho - 1) ho1 = g.Ho - 1;
      if (wo1 > g.Wo - 1) wo1 = g.Wo - 1;
      const int lh = ah - g.KH + 1, lw = aw - g.KW + 1;
      const int ho0 = lh <= 0 ? 0 : (lh + g.sh - 1) / g.sh, wo0 = lw <= 0 ? 0 : (lw + g.sw - 1) / g.sw;
      for (int ho = ho1; ho >= ho0; --ho)          // i ascending
        for (int wo = wo1; wo >= wo0; --wo)        // j ascending
          take((n * g.Ho + ho) * g.Wo + wo, (ah - ho * g.sh) * g.KW + (aw - wo * g.sw));
    } else {
      for (int i = 0; i < g.KH; ++i)
        for (int j = 0; j < g.KW; ++j) {
          const int m = tap_row(g, n, hi, wi, i, j);
          if (m >= 0) take(m, i * g.KW + j);
        }
    }
    store_vec<8>(dx, DT, static_cast<int64_t>(pix) * g.C + v * 8, acc);
  }
}

}  // namespace

void im2col_nhwc(const uint16_t* x, const Im2col& g, uint16_t* col, hipStream_t stream) {
  const int rows = g.N * g.Ho * g.Wo;
  if (rows <= 0) return;
  const bool vec = g.C % 8 == 0 && g.ldc == g.KH * g.KW * g.C;
  const bool chunk8 = !vec && g.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(col) & 15) == 0;
  const int K = vec ? g.KH * g.KW * (g.C / 8) : (chunk8 ? g.ldc / 8 : g.ldc);
  int rpw = kThreads * 4 / K;  // ~4 items per thread
  if (rpw < 1) rpw = 1;
  const dim3 grid((rows + rpw - 1) / rpw);
  if (vec) hipLaunchKernelGGL(k_im2col_vec, grid, dim3(kThreads), 0, stream, x, g, col, rpw);
  else if (chunk8 && g.C == 3 && g.KW == 7 && g.ldc == 152)
    hipLaunchKernelGGL((k_im2col_chunk8<3, 7, 19>), grid, dim3(kThreads), 0, stream, x, g, col, rpw);
  else if (chunk8) hipLaunchKernelGGL((k_im2col_chunk8<0, 0, 0>), grid, dim3(kThreads), 0, stream, x, g, col, rpw);
  else hipLaunchKernelGGL(k_im2col_scalar, grid, dim3(kThreads), 0, stream, x, g, col, rpw);
}

void col2im_nhwc(const uint16_t* dcol, const Im2col& g, uint16_t* dx, bool accumulate, hipStream_t stream) {
  const bool vec = g.C % 8 == 0 && g.ldc % 8 == 0;
  const int64_t items = static_cast<int64_t>(g.N) * g.H * g.W * (vec ? g.C / 8 : g.C);
  if (items <= 0) return;
  int64_t blocks = (items + kThreads - 1) / kThreads;
  if (blocks > 65536) blocks = 65536;  // grid-stride beyond
  const dim3 grid(static_cast<unsigned>(blocks));
  if (vec && accumulate) hipLaunchKernelGGL(k_col2im_vec<true>, grid, dim3(kThreads), 0, stream, dcol, g, dx);
  else if (vec) hipLaunchKernelGGL(k_col2im_vec<false>, grid, dim3(kThreads), 0, stream, dcol, g, dx);
  else if (accumulate) hipLaunchKernelGGL(k_col2im_scalar<true>, grid, dim3(kThreads), 0, stream, dcol, g, dx);
  else hipLaunchKernelGGL(k_col2im_scalar<false>, grid, dim3(kThreads), 0, stream, dcol, g, dx);
}

namespace {
unsigned grid_for(int64_t items) {
  int64_t blocks = (items + kThreads - 1) / kThreads;
  if (blocks > 65536) blocks = 65536;  // grid-stride beyond
  return static_cast<unsigned>(blocks < 1 ? 1 : blocks);
}
}  // namespace

void maxpool_fwd_nhwc(const void* x, const Im2col& g, void* y, uint8_t* idx, hipStream_t stream, int dt) {
  const int64_t items = static_cast<int64_t>(g.N) * g.Ho * g.Wo * (g.C / 8);
  if (items <= 0) return;
  if (dt == kF32) hipLaunchKernelGGL(k_maxpool_fwd<kF32>, dim3(grid_for(items)), dim3(kThreads), 0, stream, x, g, y, idx);
  else hipLaunchKernelGGL(k_maxpool_fwd<kBF16>, dim3(grid_for(items)), dim3(kThreads), 0, stream, x, g, y, idx);
}

void maxpool_bwd_nhwc(const void* dy, const uint8_t* idx, const Im2col& g, void* dx, hipStream_t stream, int dt) {
  const int64_t items = static_cast<int64_t>(g.N) * g.H * g.W * (g.C / 8);
  if (items <= 0) return;
  if (dt == kF32) hipLaunchKernelGGL(k_maxpool_bwd<kF32>, dim3(grid_for(items)), dim3(kThreads), 0, stream, dy, idx, g, dx);
  else hipLaunchKernelGGL(k_maxpool_bwd<kBF16>, dim3(grid_for(items)), dim3(kThreads), 0, stream, dy, idx, g, dx);
}

}  // namespace gpu
}  // namespace garfield
