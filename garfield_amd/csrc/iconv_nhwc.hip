// Implicit-GEMM NHWC convolution on MFMA (bf16 in, fp32 accumulate), gfx950.
//
// The grouped ResNet step (garfield_amd/ops/grouped.py) used to run every k x k
// convolution as im2col -> hipBLASLt GEMM (-> col2im for the data gradient). For
// CIFAR-shape activations those GEMMs are tiny in FLOPs (layer1's 3x3: 9.4 GFLOP
// for 8 workers x 250 images) and the 9x-inflated col matrix (147 MB written,
// then read) is what the step pays for. Here the patch gather happens inside the
// MFMA loop: no col is ever written.
//
//   y[m, co] = Σ_{i, j, ci} x[n, ho*sh - ph + i*dh, wo*sw - pw + j*dw, ci] · W[co, i, j, ci]  (+ add[m, co])
//
// GEMM view D[co, m] = W[co, k] · X[k, m] with k = (i, j, ci): the weight is the A
// operand and the gathered input the B operand of v_mfma_f32_16x16x32_bf16, so
// both fragments are 16 contiguous bytes in memory:
//   A lane l: W[co = l&15][k = 8(l>>4) .. +7]      (channels_last weight = [Cout, KH, KW, C])
//   B lane l: X[k = 8(l>>4) .. +7][pixel = l&15]   (8 consecutive input channels of one tap)
//   D lane l: rows co = 4(l>>4) .. +3, column pixel l&15 -> one 8-byte store of 4 channels.
// The data gradient of a stride-1 convolution is the same kernel on dy with the
// flipped, transposed weight (W'[ci, i', j', co] = W[co, KH-1-i', KW-1-j', ci],
// padding KH-1-ph); ``add`` folds in the gradient of the residual branch.
//
// Workgroup: 4 waves, wave tile = 16*PM pixels x 64 output channels (PM pixel
// fragments x 4 channel fragments), so a workgroup covers 64*PM pixels x 64
// channels; grid (ceil(M / (64*PM)), Cout / 64). Requires C % 32 == 0 and
// Cout % 64 == 0 (checked by the host wrapper). Out-of-range taps read a clamped
// in-bounds address and are zeroed in registers (no branch around the load).
#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kWaves = 4;

template <int PM>
struct Frags {
  bf16x8 a[4];
  bf16x8 b[PM];
};

template <int PM, bool ADD>
__global__ __launch_bounds__(256) void k_iconv(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                               Im2col g, int Cout, uint16_t* y, const uint16_t* add) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int pl = lane & 15;   // pixel (B column) / channel (A row) inside a fragment
  const int kq = lane >> 4;   // 8-element k slice
  const int M = g.N * g.Ho * g.Wo;
  const int K = g.KH * g.KW * g.C;
  const int m0 = blockIdx.x * (kWaves * 16 * PM) + wave * 16 * PM;
  const int co0 = blockIdx.y * 64;

  int hb[PM], wb[PM], nb[PM];
  bool pv[PM];
#pragma unroll
  for (int r = 0; r < PM; ++r) {
    const int m = m0 + r * 16 + pl;
    pv[r] = m < M;
    const int mm = pv[r] ? m : 0;
    const int wo = mm % g.Wo;
    const int t = mm / g.Wo;
    hb[r] = (t % g.Ho) * g.sh - g.ph;
    wb[r] = wo * g.sw - g.pw;
    nb[r] = t / g.Ho;
  }
  const uint16_t* wp[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wp[c] = w + static_cast<int64_t>(co0 + c * 16 + pl) * K + kq * 8;

  const int csteps = g.C / 32;
  const int steps = g.KH * g.KW * csteps;

  auto load = [&](int s, Frags<PM>& f) {
    const int tap = s / csteps;
    const int c0 = (s - tap * csteps) * 32;
    const int i = tap / g.KW, j = tap - (tap / g.KW) * g.KW;
    const int koff = tap * g.C + c0;
#pragma unroll
    for (int c = 0; c < 4; ++c) f.a[c] = *reinterpret_cast<const bf16x8*>(wp[c] + koff);
#pragma unroll
    for (int r = 0; r < PM; ++r) {
      const int hi = hb[r] + i * g.dh, wi = wb[r] + j * g.dw;
      const bool ok = pv[r] && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
      const int64_t pix = (static_cast<int64_t>(nb[r]) * g.H + (ok ? hi : 0)) * g.W + (ok ? wi : 0);
      const uint4 v = *reinterpret_cast<const uint4*>(x + pix * g.C + c0 + kq * 8);
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
      f.b[r] = __builtin_bit_cast(bf16x8, ok ? v : z);
    }
  };

  f32x4 acc[PM][4];
#pragma unroll
  for (int r = 0; r < PM; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](const Frags<PM>& f) {
#pragma unroll
    for (int r = 0; r < PM; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[c], f.b[r], acc[r][c], 0, 0, 0);
  };

  // one step of loads in flight while the previous step multiplies; the
  // latency is hidden across waves (4 per SIMD at PM = 2), not inside one
  Frags<PM> cur, nxt;
  load(0, cur);
  for (int s = 0; s < steps; ++s) {
    if (s + 1 < steps) load(s + 1, nxt);
    mma(cur);
    cur = nxt;
  }

  // D[co = 4*kq + e][pixel = pl] of every (r, c) fragment: 4 consecutive channels of one pixel
#pragma unroll
  for (int r = 0; r < PM; ++r) {
    if (!pv[r]) continue;
    const int64_t rowoff = static_cast<int64_t>(m0 + r * 16 + pl) * Cout;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t off = rowoff + co0 + c * 16 + kq * 4;
      float v[4] = {acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]};
      if constexpr (ADD) {
        const uint2 a = *reinterpret_cast<const uint2*>(add + off);
        v[0] += bf16_to_f(static_cast<uint16_t>(a.x & 0xffffu));
        v[1] += bf16_to_f(static_cast<uint16_t>(a.x >> 16));
        v[2] += bf16_to_f(static_cast<uint16_t>(a.y & 0xffffu));
        v[3] += bf16_to_f(static_cast<uint16_t>(a.y >> 16));
      }
      uint2 o;
      o.x = static_cast<uint32_t>(f_to_bf16(v[0])) | (static_cast<uint32_t>(f_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f_to_bf16(v[2])) | (static_cast<uint32_t>(f_to_bf16(v[3])) << 16);
      *reinterpret_cast<uint2*>(y + off) = o;
    }
  }
}

template <int PM>
void launch(const uint16_t* x, const uint16_t* w, const Im2col& g, int Cout, uint16_t* y, const uint16_t* add,
            hipStream_t stream) {
  const int M = g.N * g.Ho * g.Wo;
  const dim3 grid((M + kWaves * 16 * PM - 1) / (kWaves * 16 * PM), Cout / 64);
  if (add) hipLaunchKernelGGL((k_iconv<PM, true>), grid, dim3(256), 0, stream, x, w, g, Cout, y, add);
  else hipLaunchKernelGGL((k_iconv<PM, false>), grid, dim3(256), 0, stream, x, w, g, Cout, y, add);
}

}  // namespace

void iconv_nhwc(const uint16_t* x, const uint16_t* w, const Im2col& g, int Cout, uint16_t* y, const uint16_t* add,
                int pm, hipStream_t stream) {
  const int M = g.N * g.Ho * g.Wo;
  if (M <= 0) return;
  if (pm <= 0) {  // measured (scripts/bench_iconv.py): the largest pixel tile that keeps ~256 workgroups
    const int64_t ncb = Cout / 64;
    pm = 4;
    while (pm > 1 && ((M + 64 * pm - 1) / (64 * pm)) * ncb < 250) pm /= 2;
  }
  if (pm >= 4) launch<4>(x, w, g, Cout, y, add, stream);
  else if (pm == 2) launch<2>(x, w, g, Cout, y, add, stream);
  else launch<1>(x, w, g, Cout, y, add, stream);
}

}  // namespace gpu
}  // namespace garfield
