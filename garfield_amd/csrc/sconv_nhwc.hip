// 3x3 / stride-1 / pad-1 convolutions on tiny images (H, W <= 2: ResNet-50 CIFAR layer3 at 2x2 and
// layer4 at 1x1) as dense GEMMs, gfx950.
//
// On a 2x2 image every output pixel sees only four of the nine taps (on 1x1 only the centre one), so
// the implicit-GEMM kernel (iconv_nhwc.hip) streams 2.25x (9x) the useful work, and a 1x1 image falls
// back to im2col + GEMM over a 9x zero-padded patch matrix. With P = H * W pixels per image, the NHWC
// image is already the row x[n, (p, ci)] of a [N, P * Cin] matrix and
//
//   y[n, (p', co)] = Σ_{(p, ci)} x[n, (p, ci)] · Wbig[(p', co), (p, ci)],
//   Wbig[(p', co), (p, ci)] = W[co, h - h' + 1, w - w' + 1, ci]   (0 when the tap falls outside 3x3)
//
// is one dense GEMM (gemm_nt.hip) with exactly the convolution's FLOPs; the data gradient multiplies
// by Wbigᵀ, and the per-worker weight gradient is the 1x1 weight gradient of [N, P*Cout] x [N, P*Cin]
// (iconv_nhwc.hip, rows = images), folded back onto the nine taps here: dW[co, i, j, ci] = Σ over the
// (p', p) pairs of tap (i, j) of dWbig[(p', co), (p, ci)].
//
// This file: the per-step expansion W -> Wbig, Wbigᵀ of every such layer in ONE launch, and the fold.
#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

// one thread per 8 consecutive elements of a Wbig row (8 ci: one 16-byte load and store) or of a
// Wbigᵀ row (8 co: 8 strided 2-byte loads of the L2-resident weight, one 16-byte store); the first
// start[count] units are Wbig's, the next as many Wbigᵀ's
__global__ __launch_bounds__(256) void k_sc_expand(ScExpandJobs jobs) {
  const int64_t u0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t half = jobs.start[jobs.count];
  if (u0 >= 2 * half) return;
  const bool tr = u0 >= half;
  const int64_t u = tr ? u0 - half : u0;
  int jb = 0;
  while (jb + 1 < jobs.count && u >= jobs.start[jb + 1]) ++jb;
  const ScExpandJob& J = jobs.job[jb];
  const int P = J.H * J.W;
  const int64_t v = u - jobs.start[jb];
  if (!tr) {
    const int rowu = P * J.cin / 8;   // 8-element units per Wbig row
    const int r = static_cast<int>(v / rowu), c8 = static_cast<int>(v - static_cast<int64_t>(r) * rowu);
    const int pq = r / J.cout, co = r - pq * J.cout;
    const int col = c8 * 8;
    const int p = col / J.cin, ci = col - p * J.cin;
    const int i = p / J.W - pq / J.W + 1, j = p % J.W - pq % J.W + 1;
    uint4 val = make_uint4(0u, 0u, 0u, 0u);
    if (i >= 0 && i < 3 && j >= 0 && j < 3)
      val = *reinterpret_cast<const uint4*>(J.w + (static_cast<int64_t>(co) * 9 + i * 3 + j) * J.cin + ci);
    *reinterpret_cast<uint4*>(J.big + static_cast<int64_t>(r) * P * J.cin + col) = val;
  } else {
    const int rowu = P * J.cout / 8;   // 8-element units per Wbigᵀ row (p, ci): columns (p', co)
    const int r = static_cast<int>(v / rowu), c8 = static_cast<int>(v - static_cast<int64_t>(r) * rowu);
    const int p = r / J.cin, ci = r - p * J.cin;
    const int col = c8 * 8;
    const int pq = col / J.cout, co = col - pq * J.cout;
    const int i = p / J.W - pq / J.W + 1, j = p % J.W - pq % J.W + 1;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (i >= 0 && i < 3 && j >= 0 && j < 3) {
      const uint16_t* src = J.w + (static_cast<int64_t>(co) * 9 + i * 3 + j) * J.cin + ci;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        w[e >> 1] |= static_cast<uint32_t>(src[static_cast<int64_t>(e) * 9 * J.cin]) << (16 * (e & 1));
    }
    *reinterpret_cast<uint4*>(J.bigT + static_cast<int64_t>(r) * P * J.cout + col) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// out[g][co][(i*3 + j)*Cin + ci] = Σ_s Σ_{pairs of tap (i, j)} slab[s][g][(p', co)][(p, ci)], 8 ci per thread
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void k_sc_fold(const float* __restrict__ slab, int S, int G, int H, int W, int cout,
                                                 int cin, void* out, int64_t gstride) {
  const int64_t u = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int c8n = cin / 8;
  const int64_t total = static_cast<int64_t>(G) * cout * 9 * c8n;
  if (u >= total) return;
  const int c8 = static_cast<int>(u % c8n);
  int64_t t = u / c8n;
  const int tap = static_cast<int>(t % 9);
  t /= 9;
  const int co = static_cast<int>(t % cout);
  const int g = static_cast<int>(t / cout);
  const int i = tap / 3, j = tap - (tap / 3) * 3;
  const int P = H * W;
  const int64_t ldk = static_cast<int64_t>(P) * cin;               // slab row length
  const int64_t gsz = static_cast<int64_t>(P) * cout * ldk;        // one worker's slab
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int hq = 0; hq < H; ++hq)
    for (int wq = 0; wq < W; ++wq) {
      const int h = hq + i - 1, w = wq + j - 1;
      if (h < 0 || h >= H || w < 0 || w >= W) continue;
      const int64_t off = static_cast<int64_t>(g) * gsz + static_cast<int64_t>((hq * W + wq) * cout + co) * ldk +
                          (h * W + w) * cin + c8 * 8;
      for (int s = 0; s < S; ++s) {
        const float4 a = *reinterpret_cast<const float4*>(slab + s * G * gsz + off);
        const float4 b = *reinterpret_cast<const float4*>(slab + s * G * gsz + off + 4);
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      }
    }
  const int64_t o = static_cast<int64_t>(g) * gstride + (static_cast<int64_t>(co) * 9 + tap) * cin + c8 * 8;
  if constexpr (OUT_BF16) {
    uint4 r;
    r.x = static_cast<uint32_t>(f_to_bf16(acc[0])) | (static_cast<uint32_t>(f_to_bf16(acc[1])) << 16);
    r.y = static_cast<uint32_t>(f_to_bf16(acc[2])) | (static_cast<uint32_t>(f_to_bf16(acc[3])) << 16);
    r.z = static_cast<uint32_t>(f_to_bf16(acc[4])) | (static_cast<uint32_t>(f_to_bf16(acc[5])) << 16);
    r.w = static_cast<uint32_t>(f_to_bf16(acc[6])) | (static_cast<uint32_t>(f_to_bf16(acc[7])) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(out) + o) = r;
  } else {
    float* d = static_cast<float*>(out) + o;
    *reinterpret_cast<float4*>(d) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(d + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

}  // namespace

void sc_expand(const ScExpandJobs& jobs, hipStream_t stream) {
  const int64_t total = 2 * jobs.start[jobs.count];   // Wbig units, then as many Wbigᵀ units
  if (total <= 0) return;
  hipLaunchKernelGGL(k_sc_expand, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, stream, jobs);
}

void sc_fold(const float* slab, int S, int G, int H, int W, int cout, int cin, void* out, bool out_bf16,
             int64_t gstride, hipStream_t stream) {
  const int64_t total = static_cast<int64_t>(G) * cout * 9 * (cin / 8);
  if (total <= 0) return;
  const dim3 grid(static_cast<unsigned>((total + 255) / 256));
  if (out_bf16)
    hipLaunchKernelGGL((k_sc_fold<true>), grid, dim3(256), 0, stream, slab, S, G, H, W, cout, cin, out, gstride);
  else
    hipLaunchKernelGGL((k_sc_fold<false>), grid, dim3(256), 0, stream, slab, S, G, H, W, cout, cin, out, gstride);
}

}  // namespace gpu
}  // namespace garfield
