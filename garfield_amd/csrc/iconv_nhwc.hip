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
#include <cstdlib>

#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kWaves = 4;

// BatchNorm prologue of a weight gradient's input fragment (the 1x1 consumers of a BatchNorm + ReLU whose
// output was never written): 8 pixels of one channel of one worker, bf16(max(x * sc + sh, 0)). A 1x1
// stride-1 unpadded convolution has no padding pixels; rows past the worker's end are zeros whose dy
// rows are zeros too.
__device__ __forceinline__ bf16x8 pro_frag(bf16x8 b, float sc, float sh) {
  const uint4 u = __builtin_bit_cast(uint4, b);
  const float x[8] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                      __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u),
                      __uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u),
                      __uint_as_float(u.w << 16), __uint_as_float(u.w & 0xffff0000u)};
  float y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) y[i] = fmaxf(fmaf(x[i], sc, sh), 0.f);
  return __builtin_bit_cast(bf16x8, make_uint4(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]),
                                               pack_bf16x2(y[4], y[5]), pack_bf16x2(y[6], y[7])));
}

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

// ---------------------------------------------------------------------------
// LDS-staged variant (C % 64 == 0): every 64-deep k-step (one tap, 64 input
// channels) of the workgroup's W tile [64 co x 64 k] and X tile [64*PM pixels x
// 64 k] is copied global -> LDS by global_load_lds (16 B per lane, no VGPR
// round trip), NS stages deep, so a wave keeps NS-1 stages of loads in flight
// instead of one (the register variant above is one load latency per k-step).
// LDS images are [row][8 x 16-byte chunks] with the chunk index XOR-swizzled by
// (row & 7) on the GLOBAL side (glds writes lane-linear): the fragment reads
// (16 rows x one chunk) then hit 8 different bank groups.

__device__ __attribute__((aligned(16))) uint4 g_iconv_zero[8];  // 128 zero bytes: source of padded taps

using lds_ptr = __attribute__((address_space(3))) void*;
typedef short s16x4 __attribute__((ext_vector_type(4)));

// Bank swizzle of the transposed-read tiles of the weight gradients: a half-wave's ds_read_b64_tr_b16
// touches pixel rows {0..3, 8..11} (+ 16) at one chunk pair; with plain 128-byte rows rows 0, 2, 8, 10
// share banks (4-way conflicts). Row r's 16-byte chunks are stored XOR 2 tr_g(r) (the global side of
// the LDS-DMA picks the chunk), which spreads those rows over distinct banks.
__device__ __forceinline__ int tr_g(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 1); }

// TW: w is the FORWARD weight of a stride-1 convolution and this launch computes its data
// gradient (x = dy, C = the forward's output channels, Cout = its input channels, padding
// KH-1-ph): A[o][(i', j', c)] = Wf[c][KH-1-i'][KW-1-j'][o]. The W tile is staged as plain
// [c][o] rows and its fragments are read transposed (ds_read_b64_tr_b16), so no flipped /
// transposed weight copy is made.
// S2 (with TW): the data gradient of a STRIDE-2 convolution, without a dcol matrix or col2im. The
// output pixels split by parity into four classes (blockIdx.z = 2p + q: dx rows 2u + p, columns
// 2v + q); class (p, q) is a stride-1 correlation of dy with the sub-kernel of the forward taps
// i = i0 + 2a (i0 = (p + ph) & 1), which read dy row u + (p + ph - i) / 2 (and likewise for the
// columns): 1 / 2 / 2 / 4 taps for a 3x3 pad-1 kernel, 1 / 0 / 0 / 0 for a 1x1 pad-0 one (a class
// with no tap writes zeros, or add). Here g is the forward geometry seen from dy: H, W = dy's
// spatial size, C = dy's channels, Ho, Wo = dx's (even), sh = sw = 2.
// magic divisors of the output-pixel decomposition (the class grid's for S2): m -> (n, row, column)
struct PixDiv {
  FastDiv fw, fh;
};

template <int PM, int NS, bool ADD, bool TW, bool S2>
__global__ __launch_bounds__(256) void k_iconv_lds(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                   Im2col g, int Cout, uint16_t* y, const uint16_t* add, PixDiv pd) {
  static_assert(!S2 || TW, "the stride-2 data gradient reads the forward weight transposed");
  constexpr int BM = 64 * PM;          // pixels per workgroup
  constexpr int XB = BM * 128;         // X tile bytes per stage
  constexpr int WB = 64 * 128;         // W tile bytes per stage
  constexpr int SB = XB + WB;
  constexpr int XI = XB / 1024 / 4;    // X glds instructions per wave per stage
  constexpr int WI = WB / 1024 / 4;    // W glds instructions per wave per stage (2)
  __shared__ __attribute__((aligned(16))) char lds[NS * SB];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // S2: this class's output grid (HoC x WoC) and its taps along each axis (count, first forward
  // tap, dy offset of the first tap; tap a: forward index i0 + 2a, dy offset d0 - a)
  const int cp = S2 ? static_cast<int>(blockIdx.z >> 1) : 0, cq = S2 ? static_cast<int>(blockIdx.z & 1) : 0;
  const int HoC = S2 ? g.Ho >> 1 : g.Ho, WoC = S2 ? g.Wo >> 1 : g.Wo;
  const int i0h = (cp + g.ph) & 1, i0w = (cq + g.pw) & 1;
  const int nth = S2 ? (g.KH - i0h + 1) >> 1 : g.KH, ntw = S2 ? (g.KW - i0w + 1) >> 1 : g.KW;
  const int d0h = (cp + g.ph - i0h) >> 1, d0w = (cq + g.pw - i0w) >> 1;
  const int M = g.N * HoC * WoC;
  const int K = g.KH * g.KW * g.C;
  const int m0 = blockIdx.x * BM;
  const int co0 = blockIdx.y * 64;
  const int lrow = lane >> 3, lchunk = lane & 7;

  // this lane's sources: X rows (wave*XI + u)*8 + lrow, W rows (wave*WI + u)*8 + lrow
  int xh[XI], xw[XI], xn[XI], xq[XI];
  bool xv[XI];
#pragma unroll
  for (int u = 0; u < XI; ++u) {
    const int px = (wave * XI + u) * 8 + lrow;
    const int m = m0 + px;
    xv[u] = m < M;
    const int mm = xv[u] ? m : 0;
    const int t = static_cast<int>(fdiv(static_cast<uint32_t>(mm), pd.fw));
    const int wo = mm - t * WoC;
    const int tn = static_cast<int>(fdiv(static_cast<uint32_t>(t), pd.fh));
    const int ho = t - tn * HoC;
    if constexpr (S2) {   // class pixel (u, v): dy rows u + offset
      xh[u] = ho;
      xw[u] = wo;
    } else {
      xh[u] = ho * g.sh - g.ph;
      xw[u] = wo * g.sw - g.pw;
    }
    xn[u] = tn;
    xq[u] = lchunk ^ (px & 7);
  }
  const uint16_t* wsrc[WI];
  const int KF = g.KH * g.KW * Cout;   // TW: row stride of the forward weight
#pragma unroll
  for (int u = 0; u < WI; ++u) {
    const int row = (wave * WI + u) * 8 + lrow;
    // TW: the transposed fragment reads' bank swizzle (tr_g): row r's 16-byte chunks XOR 2 tr_g(r)
    if constexpr (TW) wsrc[u] = w + static_cast<int64_t>(row) * KF + co0 + (lchunk ^ (2 * tr_g(row))) * 8;
    else wsrc[u] = w + static_cast<int64_t>(co0 + row) * K + (lchunk ^ (row & 7)) * 8;
  }
  const uint16_t* zsrc = reinterpret_cast<const uint16_t*>(g_iconv_zero) + lchunk * 8;

  const int csteps = g.C / 64;
  const int steps = nth * ntw * csteps;

  auto issue = [&](int s, int slot) {
    const int tap = s / csteps;
    const int c0 = (s - tap * csteps) * 64;
    const int a = tap / ntw, b = tap - (tap / ntw) * ntw;
    char* base = lds + slot * SB;
    int64_t woff;
    int oh, ow;   // dy offsets of this tap
    if constexpr (S2) {
      woff = static_cast<int64_t>(c0) * KF + ((i0h + 2 * a) * g.KW + (i0w + 2 * b)) * Cout;
      oh = d0h - a;
      ow = d0w - b;
    } else {
      if constexpr (TW) woff = static_cast<int64_t>(c0) * KF + ((g.KH - 1 - a) * g.KW + (g.KW - 1 - b)) * Cout;
      else woff = tap * g.C + c0;
      oh = a * g.dh;
      ow = b * g.dw;
    }
#pragma unroll
    for (int u = 0; u < WI; ++u)
      __builtin_amdgcn_global_load_lds(wsrc[u] + woff, (lds_ptr)(base + XB + (wave * WI + u) * 1024), 16, 0, 0);
#pragma unroll
    for (int u = 0; u < XI; ++u) {
      const int hi = xh[u] + oh, wi = xw[u] + ow;
      const bool ok = xv[u] && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
      // both addresses computed, then one select (a conditional address expression
      // becomes a branch around each load)
      const int hc = ok ? hi : 0, wc = ok ? wi : 0;
      const uint64_t ax = reinterpret_cast<uint64_t>(
          x + ((static_cast<int64_t>(xn[u]) * g.H + hc) * g.W + wc) * g.C + c0 + xq[u] * 8);
      const uint64_t az = reinterpret_cast<uint64_t>(zsrc);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? ax : az),
                                       (lds_ptr)(base + (wave * XI + u) * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[PM][4];
#pragma unroll
  for (int r = 0; r < PM; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets inside a stage (row-major 128-B rows, swizzled chunks)
  const int fr = lane & 15, fq = lane >> 4;   // row in fragment, 8-element k slice
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);

  for (int s = 0; s < steps; ++s) {
    // stage s has landed when at most (stages issued after it) x (glds per stage) are outstanding
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (WI + XI)) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WI + XI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    const char* base = lds + (s % NS) * SB;
    s16x4 tr[TW ? 16 : 1];
    if constexpr (TW) {
      // A fragments of both 32-deep halves: lane (group grp, 4q+p) reads W-tile row
      // 32*ks + 8*grp + 4h + q, columns 16c + 4p .. +3 (inline asm: see k_iwgrad); column block c
      // of that row is stored at block c ^ tr_g(8*grp + q) (the staging's swizzle: no 4-way conflicts
      // between rows 0, 2, 8, 10 of a half-wave)
      const int tq = 8 * (lane >> 4) + ((lane & 15) >> 2), tg = tr_g(tq);
      const uint32_t ab = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)base)) + XB + tq * 128 +
                          8 * (lane & 3);
      const uint32_t a0 = ab + 32 * (0 ^ tg), a1 = ab + 32 * (1 ^ tg), a2 = ab + 32 * (2 ^ tg),
                     a3 = ab + 32 * (3 ^ tg);
      asm volatile(
            "ds_read_b64_tr_b16 %0, %16 offset:0\n\t"
            "ds_read_b64_tr_b16 %1, %16 offset:512\n\t"
            "ds_read_b64_tr_b16 %2, %17 offset:0\n\t"
            "ds_read_b64_tr_b16 %3, %17 offset:512\n\t"
            "ds_read_b64_tr_b16 %4, %18 offset:0\n\t"
            "ds_read_b64_tr_b16 %5, %18 offset:512\n\t"
            "ds_read_b64_tr_b16 %6, %19 offset:0\n\t"
            "ds_read_b64_tr_b16 %7, %19 offset:512\n\t"
            "ds_read_b64_tr_b16 %8, %16 offset:4096\n\t"
            "ds_read_b64_tr_b16 %9, %16 offset:4608\n\t"
            "ds_read_b64_tr_b16 %10, %17 offset:4096\n\t"
            "ds_read_b64_tr_b16 %11, %17 offset:4608\n\t"
            "ds_read_b64_tr_b16 %12, %18 offset:4096\n\t"
            "ds_read_b64_tr_b16 %13, %18 offset:4608\n\t"
            "ds_read_b64_tr_b16 %14, %19 offset:4096\n\t"
            "ds_read_b64_tr_b16 %15, %19 offset:4608\n\t"
            "s_waitcnt lgkmcnt(0)"
          : "=&v"(tr[0]), "=&v"(tr[1]), "=&v"(tr[2]), "=&v"(tr[3]), "=&v"(tr[4]), "=&v"(tr[5]), "=&v"(tr[6]),
            "=&v"(tr[7]), "=&v"(tr[8]), "=&v"(tr[9]), "=&v"(tr[10]), "=&v"(tr[11]), "=&v"(tr[12]), "=&v"(tr[13]),
            "=&v"(tr[14]), "=&v"(tr[15])
          : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
          : "memory");
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4], b[PM];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if constexpr (TW) {
          const s16x4 lo = tr[ks * 8 + 2 * c], hi = tr[ks * 8 + 2 * c + 1];
          const short v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          a[c] = __builtin_bit_cast(bf16x8, v);
        } else {
          const int row = c * 16 + fr;
          const int chunk = (ks * 4 + fq) ^ (row & 7);
          a[c] = *reinterpret_cast<const bf16x8*>(base + XB + row * 128 + chunk * 16);
        }
      }
#pragma unroll
      for (int r = 0; r < PM; ++r) {
        const int row = (wave * PM + r) * 16 + fr;
        const int chunk = (ks * 4 + fq) ^ (row & 7);
        b[r] = *reinterpret_cast<const bf16x8*>(base + row * 128 + chunk * 16);
      }
#pragma unroll
      for (int r = 0; r < PM; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[r], acc[r][c], 0, 0, 0);
    }
    // every wave's fragment reads of this slot retire before the barrier that lets it be refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

#pragma unroll
  for (int r = 0; r < PM; ++r) {
    const int m = m0 + (wave * PM + r) * 16 + fr;
    if (m >= M) continue;
    int64_t orow = m;
    if constexpr (S2) {   // class pixel -> dx pixel (n, 2u + p, 2v + q)
      const int t = static_cast<int>(fdiv(static_cast<uint32_t>(m), pd.fw)), v = m - t * WoC;
      const int tn = static_cast<int>(fdiv(static_cast<uint32_t>(t), pd.fh));
      orow = (static_cast<int64_t>(tn) * g.Ho + 2 * (t - tn * HoC) + cp) * g.Wo + 2 * v + cq;
    }
    const int64_t rowoff = orow * Cout;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t off = rowoff + co0 + c * 16 + fq * 4;
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

template <int PM, int NS>
void launch_lds(const uint16_t* x, const uint16_t* w, const Im2col& g, int Cout, uint16_t* y, const uint16_t* add,
                bool tw, hipStream_t stream) {
  const int M = g.N * g.Ho * g.Wo;
  const dim3 grid((M + 64 * PM - 1) / (64 * PM), Cout / 64);
  const PixDiv pd{make_fastdiv(static_cast<uint32_t>(g.Wo)), make_fastdiv(static_cast<uint32_t>(g.Ho))};
  if (tw) {
    if (add) hipLaunchKernelGGL((k_iconv_lds<PM, NS, true, true, false>), grid, dim3(256), 0, stream, x, w, g, Cout, y, add, pd);
    else hipLaunchKernelGGL((k_iconv_lds<PM, NS, false, true, false>), grid, dim3(256), 0, stream, x, w, g, Cout, y, add, pd);
  } else {
    if (add) hipLaunchKernelGGL((k_iconv_lds<PM, NS, true, false, false>), grid, dim3(256), 0, stream, x, w, g, Cout, y, add, pd);
    else hipLaunchKernelGGL((k_iconv_lds<PM, NS, false, false, false>), grid, dim3(256), 0, stream, x, w, g, Cout, y, add, pd);
  }
}

template <int PM, int NS>
void launch_s2(const uint16_t* dy, const uint16_t* w, const Im2col& g, int Cout, uint16_t* dx, const uint16_t* add,
               hipStream_t stream) {
  const int M = g.N * (g.Ho >> 1) * (g.Wo >> 1);
  const dim3 grid((M + 64 * PM - 1) / (64 * PM), Cout / 64, 4);
  const PixDiv pd{make_fastdiv(static_cast<uint32_t>(g.Wo >> 1)), make_fastdiv(static_cast<uint32_t>(g.Ho >> 1))};
  if (add) hipLaunchKernelGGL((k_iconv_lds<PM, NS, true, true, true>), grid, dim3(256), 0, stream, dy, w, g, Cout, dx, add, pd);
  else hipLaunchKernelGGL((k_iconv_lds<PM, NS, false, true, true>), grid, dim3(256), 0, stream, dy, w, g, Cout, dx, add, pd);
}

// ---------------------------------------------------------------------------
// Implicit weight gradient, per worker, on MFMA:
//
//   dW_g[co, (i, j, ci)] = Σ_{m in worker g} dy[m, co] · x[pixel(m, i, j), ci]
//
// (the reduction runs over output pixels m, so both operands need a transpose
// from their natural [pixel][channel] rows: the tiles are staged with
// global_load_lds as plain 128-byte rows and read with ds_read_b64_tr_b16, whose
// 16-lane groups gather 4 rows x 16 columns and hand lane i column i). No im2col
// matrix is written or read. Workgroup tile: 64 output channels x 64 k-columns
// (one tap, 64 input channels) of one worker, 32 pixels per k-step, NS-deep glds
// ring; the worker's pixels are split ``splits`` ways (fp32 partial slabs summed
// afterwards) when the tile grid alone cannot fill the chip.


template <int NS, bool OUT_BF16, bool PRO>
__global__ __launch_bounds__(256) void k_iwgrad(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                Im2col g, int Cout, int64_t rg, int64_t per_split, void* out,
                                                int64_t split_stride, int64_t group_stride,
                                                const float* __restrict__ psc, const float* __restrict__ psh) {
  constexpr int TB = 32 * 128;  // one 32-pixel x 64-channel tile
  constexpr int SB = 2 * TB;    // dy tile + x tile per stage
  __shared__ __attribute__((aligned(16))) char lds[NS * SB];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int K = g.KH * g.KW * g.C;
  const int nkb = K / 64;
  const int kb = blockIdx.x % nkb, cb = blockIdx.x / nkb;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int k0 = kb * 64, co0 = cb * 64;
  const int tap = k0 / g.C, c0 = k0 - tap * g.C;
  const int ti = tap / g.KW, tj = tap - ti * g.KW;
  const int64_t mbeg = static_cast<int64_t>(gi) * rg + static_cast<int64_t>(sp) * per_split;
  int64_t mend = mbeg + per_split;
  if (mend > static_cast<int64_t>(gi + 1) * rg) mend = static_cast<int64_t>(gi + 1) * rg;
  const int steps = mend > mbeg ? static_cast<int>((mend - mbeg + 31) / 32) : 0;

  const int lrow = wave * 8 + (lane >> 3), lchunk = lane & 7;   // this lane's glds row / 16-byte chunk
  const int lsw = lchunk ^ (2 * tr_g(lrow));                      // the global chunk it stages (swizzle)
  const uint16_t* zsrc = reinterpret_cast<const uint16_t*>(g_iconv_zero) + lchunk * 8;
  const uint64_t az = reinterpret_cast<uint64_t>(zsrc);

  const FastDiv fWo = make_fastdiv(g.Wo), fHo = make_fastdiv(g.Ho);
  auto issue = [&](int s, int slot) {
    const int m = static_cast<int>(mbeg) + s * 32 + lrow;   // < 2^31: checked by the host wrapper
    const bool mv = m < static_cast<int>(mend);
    const int mm = mv ? m : 0;
    char* base = lds + slot * SB;
    const uint64_t ady = reinterpret_cast<uint64_t>(dy + static_cast<int64_t>(mm) * Cout + co0 + lsw * 8);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(mv ? ady : az), (lds_ptr)(base + wave * 1024), 16,
                                     0, 0);
    uint32_t t_, wo_, n_, ho_;
    fdivmod(static_cast<uint32_t>(mm), fWo, t_, wo_);
    fdivmod(t_, fHo, n_, ho_);
    const int wo = static_cast<int>(wo_), ho = static_cast<int>(ho_), n = static_cast<int>(n_);
    const int hi = ho * g.sh - g.ph + ti * g.dh, wi = wo * g.sw - g.pw + tj * g.dw;
    const bool ok = mv && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
    const uint64_t ax = reinterpret_cast<uint64_t>(
        x + ((static_cast<int64_t>(n) * g.H + (ok ? hi : 0)) * g.W + (ok ? wi : 0)) * g.C + c0 + lsw * 8);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? ax : az),
                                     (lds_ptr)(base + TB + wave * 1024), 16, 0, 0);
  };

  // wave tile: output-channel fragments {cf0, cf0+1} x k-column fragments {kf0, kf0+1}
  const int cf0 = 2 * (wave >> 1), kf0 = 2 * (wave & 1);
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Transposed fragments: lane i of 16-lane group grp gets tile column 16f + i at rows
  // 8*grp .. 8*grp+7 (two ds_read_b64_tr_b16: lane 4q+p addresses row 8*grp + 4h + q, columns
  // 16f + 4p .. +3). The reads are inline asm with their own lgkmcnt wait: as a builtin, hipcc
  // puts a vmcnt(0) in front of them (it cannot tell them from the in-flight LDS-DMA ring
  // stages), which serialises the ring.
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)lds));
  // staged rows carry their 16-byte chunks XOR-swizzled by 2 tr_g(row) (see the staging): fragment f of
  // row r sits at chunk pair f ^ tr_g(r); the second fragment of a pair is dtr = +-32 bytes away
  const int tg = tr_g(8 * grp + q);
  const uint32_t offA = (8 * grp + q) * 128 + 32 * (cf0 ^ tg) + 8 * p;
  const uint32_t offB = TB + (8 * grp + q) * 128 + 32 * (kf0 ^ tg) + 8 * p;
  const uint32_t dtr = (tg & 1) ? static_cast<uint32_t>(-32) : 32u;
  float psv[2] = {0.f, 0.f}, phv[2] = {0.f, 0.f};   // PRO: this lane's two input channels (1x1: k = channel)
  if constexpr (PRO) {
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int64_t o = static_cast<int64_t>(gi) * g.C + c0 + (kf0 + v) * 16 + li;
      psv[v] = psc[o];
      phv[v] = psh[o];
    }
  }

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);
  for (int s = 0; s < steps; ++s) {
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t sb = lds0 + (s % NS) * SB;
    s16x4 r[8];
    asm volatile(
        "ds_read_b64_tr_b16 %0, %8\n\t"
        "ds_read_b64_tr_b16 %1, %8 offset:512\n\t"
        "ds_read_b64_tr_b16 %2, %10\n\t"
        "ds_read_b64_tr_b16 %3, %10 offset:512\n\t"
        "ds_read_b64_tr_b16 %4, %9\n\t"
        "ds_read_b64_tr_b16 %5, %9 offset:512\n\t"
        "ds_read_b64_tr_b16 %6, %11\n\t"
        "ds_read_b64_tr_b16 %7, %11 offset:512\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
        : "v"(sb + offA), "v"(sb + offB), "v"(sb + offA + dtr), "v"(sb + offB + dtr)
        : "memory");
    // every wave's reads of this slot are done (waited above) before the next barrier lets it be refilled
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    bf16x8 a[2], b[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const short va[8] = {r[2 * u][0], r[2 * u][1], r[2 * u][2], r[2 * u][3],
                           r[2 * u + 1][0], r[2 * u + 1][1], r[2 * u + 1][2], r[2 * u + 1][3]};
      const short vb[8] = {r[4 + 2 * u][0], r[4 + 2 * u][1], r[4 + 2 * u][2], r[4 + 2 * u][3],
                           r[5 + 2 * u][0], r[5 + 2 * u][1], r[5 + 2 * u][2], r[5 + 2 * u][3]};
      a[u] = __builtin_bit_cast(bf16x8, va);   // dy tile: A[co][m]
      b[u] = __builtin_bit_cast(bf16x8, vb);   // x tile:  B[m][k]
      if constexpr (PRO) b[u] = pro_frag(b[u], psv[u], phv[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[v], acc[u][v], 0, 0, 0);
  }

  // D[co = 4*grp + e][k = li] of each (u, v) fragment
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + (cf0 + u) * 16 + 4 * grp + e;
        const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                          static_cast<int64_t>(co) * K + k0 + (kf0 + v) * 16 + li;
        if constexpr (OUT_BF16) static_cast<uint16_t*>(out)[o] = f_to_bf16(acc[u][v][e]);
        else static_cast<float*>(out)[o] = acc[u][v][e];
      }
}


// Weight gradient of all THREE taps of NR kernel rows per workgroup (KW == 3, NR = 1 or
// KH): the k-step's 32-pixel dy tile is staged once and feeds 3*NR taps' MFMAs (the per-tap
// kernel above re-reads it for every tap: 9x dy traffic on a 3x3 layer; 3x at NR = 1, 1x at
// NR = 3). Stage = dy tile + 3*NR shifted x tiles; wave tile = 2 output-channel fragments x 2
// k-fragments per tap.
template <int NS, bool OUT_BF16, int NR>
__global__ __launch_bounds__(256) void k_iwgrad_rows(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                     Im2col g, int Cout, int64_t rg, int64_t per_split, void* out,
                                                     int64_t split_stride, int64_t group_stride) {
  constexpr int TB = 32 * 128;   // one 32-pixel x 64-channel tile
  constexpr int NT = 3;          // taps per kernel row
  constexpr int NX = NR * NT;    // x tiles per stage
  constexpr int SB = (1 + NX) * TB;
  __shared__ __attribute__((aligned(16))) char lds[NS * SB];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int K = g.KH * g.KW * g.C;
  const int ncb = g.C / 64;
  const int nq = (g.KH / NR) * ncb;
  const int qb = blockIdx.x % nq, cb = blockIdx.x / nq;
  const int ti0 = (qb / ncb) * NR, c0 = (qb - (qb / ncb) * ncb) * 64;
  const int co0 = cb * 64;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int64_t mbeg = static_cast<int64_t>(gi) * rg + static_cast<int64_t>(sp) * per_split;
  int64_t mend = mbeg + per_split;
  if (mend > static_cast<int64_t>(gi + 1) * rg) mend = static_cast<int64_t>(gi + 1) * rg;
  const int steps = mend > mbeg ? static_cast<int>((mend - mbeg + 31) / 32) : 0;

  const int lrow = wave * 8 + (lane >> 3), lchunk = lane & 7;
  const int lsw = lchunk ^ (2 * tr_g(lrow));   // the global chunk this lane stages (bank swizzle)
  const uint16_t* zsrc = reinterpret_cast<const uint16_t*>(g_iconv_zero) + lchunk * 8;
  const uint64_t az = reinterpret_cast<uint64_t>(zsrc);

  const FastDiv fWo = make_fastdiv(g.Wo), fHo = make_fastdiv(g.Ho);
  auto issue = [&](int s, int slot) {
    const int m = static_cast<int>(mbeg) + s * 32 + lrow;
    const bool mv = m < static_cast<int>(mend);
    const int mm = mv ? m : 0;
    char* base = lds + slot * SB;
    const uint64_t ady = reinterpret_cast<uint64_t>(dy + static_cast<int64_t>(mm) * Cout + co0 + lsw * 8);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(mv ? ady : az), (lds_ptr)(base + wave * 1024), 16,
                                     0, 0);
    uint32_t t_, wo_, n_, ho_;
    fdivmod(static_cast<uint32_t>(mm), fWo, t_, wo_);
    fdivmod(t_, fHo, n_, ho_);
    const int wo = static_cast<int>(wo_), ho = static_cast<int>(ho_), n = static_cast<int>(n_);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int hi = ho * g.sh - g.ph + (ti0 + r) * g.dh;
      const bool rok = mv && hi >= 0 && hi < g.H;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int wi = wo * g.sw - g.pw + j * g.dw;
        const bool ok = rok && wi >= 0 && wi < g.W;
        const uint64_t ax = reinterpret_cast<uint64_t>(
            x + ((static_cast<int64_t>(n) * g.H + (ok ? hi : 0)) * g.W + (ok ? wi : 0)) * g.C + c0 + lsw * 8);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? ax : az),
                                         (lds_ptr)(base + TB * (1 + r * NT + j) + wave * 1024), 16, 0, 0);
      }
    }
  };

  const int cf0 = 2 * (wave >> 1), kf0 = 2 * (wave & 1);
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[NX][2][2];
#pragma unroll
  for (int j = 0; j < NX; ++j)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[j][a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)lds));
  // staged rows carry their 16-byte chunks XOR-swizzled by 2 tr_g(row) (see the staging): fragment f of
  // row r sits at chunk pair f ^ tr_g(r); the second fragment of a pair is dtr = +-32 bytes away
  const int tg = tr_g(8 * grp + q);
  const uint32_t offA = (8 * grp + q) * 128 + 32 * (cf0 ^ tg) + 8 * p;
  const uint32_t offB = TB + (8 * grp + q) * 128 + 32 * (kf0 ^ tg) + 8 * p;
  const uint32_t dtr = (tg & 1) ? static_cast<uint32_t>(-32) : 32u;

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);
  for (int s = 0; s < steps; ++s) {
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (1 + NX)) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + NX) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t sb = lds0 + (s % NS) * SB;
    s16x4 ra[4], rb[NR][12];
    // A (dy) fragments + the first row's three B (x) fragments, then the other rows' B fragments
    asm volatile(
        "ds_read_b64_tr_b16 %0, %16\n\t"
        "ds_read_b64_tr_b16 %1, %16 offset:512\n\t"
        "ds_read_b64_tr_b16 %2, %20\n\t"
        "ds_read_b64_tr_b16 %3, %20 offset:512\n\t"
        "ds_read_b64_tr_b16 %4, %17\n\t"
        "ds_read_b64_tr_b16 %5, %17 offset:512\n\t"
        "ds_read_b64_tr_b16 %6, %21\n\t"
        "ds_read_b64_tr_b16 %7, %21 offset:512\n\t"
        "ds_read_b64_tr_b16 %8, %18\n\t"
        "ds_read_b64_tr_b16 %9, %18 offset:512\n\t"
        "ds_read_b64_tr_b16 %10, %22\n\t"
        "ds_read_b64_tr_b16 %11, %22 offset:512\n\t"
        "ds_read_b64_tr_b16 %12, %19\n\t"
        "ds_read_b64_tr_b16 %13, %19 offset:512\n\t"
        "ds_read_b64_tr_b16 %14, %23\n\t"
        "ds_read_b64_tr_b16 %15, %23 offset:512\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(ra[0]), "=&v"(ra[1]), "=&v"(ra[2]), "=&v"(ra[3]), "=&v"(rb[0][0]), "=&v"(rb[0][1]), "=&v"(rb[0][2]),
          "=&v"(rb[0][3]), "=&v"(rb[0][4]), "=&v"(rb[0][5]), "=&v"(rb[0][6]), "=&v"(rb[0][7]), "=&v"(rb[0][8]),
          "=&v"(rb[0][9]), "=&v"(rb[0][10]), "=&v"(rb[0][11])
        : "v"(sb + offA), "v"(sb + offB), "v"(sb + offB + TB), "v"(sb + offB + 2 * TB), "v"(sb + offA + dtr), "v"(sb + offB + dtr), "v"(sb + offB + TB + dtr), "v"(sb + offB + 2 * TB + dtr)
        : "memory");
#pragma unroll
    for (int r = 1; r < NR; ++r) {
      const uint32_t ob = sb + offB + static_cast<uint32_t>(r * NT) * TB;
      asm volatile(
          "ds_read_b64_tr_b16 %0, %12\n\t"
          "ds_read_b64_tr_b16 %1, %12 offset:512\n\t"
          "ds_read_b64_tr_b16 %2, %15\n\t"
          "ds_read_b64_tr_b16 %3, %15 offset:512\n\t"
          "ds_read_b64_tr_b16 %4, %13\n\t"
          "ds_read_b64_tr_b16 %5, %13 offset:512\n\t"
          "ds_read_b64_tr_b16 %6, %16\n\t"
          "ds_read_b64_tr_b16 %7, %16 offset:512\n\t"
          "ds_read_b64_tr_b16 %8, %14\n\t"
          "ds_read_b64_tr_b16 %9, %14 offset:512\n\t"
          "ds_read_b64_tr_b16 %10, %17\n\t"
          "ds_read_b64_tr_b16 %11, %17 offset:512\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(rb[r][0]), "=&v"(rb[r][1]), "=&v"(rb[r][2]), "=&v"(rb[r][3]), "=&v"(rb[r][4]), "=&v"(rb[r][5]),
            "=&v"(rb[r][6]), "=&v"(rb[r][7]), "=&v"(rb[r][8]), "=&v"(rb[r][9]), "=&v"(rb[r][10]), "=&v"(rb[r][11])
          : "v"(ob), "v"(ob + TB), "v"(ob + 2 * TB), "v"(ob + dtr), "v"(ob + TB + dtr), "v"(ob + 2 * TB + dtr)
        : "memory");
    }
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    bf16x8 a[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const short va[8] = {ra[2 * u][0], ra[2 * u][1], ra[2 * u][2], ra[2 * u][3],
                           ra[2 * u + 1][0], ra[2 * u + 1][1], ra[2 * u + 1][2], ra[2 * u + 1][3]};
      a[u] = __builtin_bit_cast(bf16x8, va);   // dy tile: A[co][m]
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const int o = 4 * j + 2 * v;
          const short vb[8] = {rb[r][o][0], rb[r][o][1], rb[r][o][2], rb[r][o][3],
                               rb[r][o + 1][0], rb[r][o + 1][1], rb[r][o + 1][2], rb[r][o + 1][3]};
          const bf16x8 bx = __builtin_bit_cast(bf16x8, vb);   // x tile of tap (r, j): B[m][k]
#pragma unroll
          for (int u = 0; u < 2; ++u)
            acc[r * NT + j][u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], bx, acc[r * NT + j][u][v], 0, 0, 0);
        }
  }

#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int k0 = ((ti0 + r) * g.KW + j) * g.C + c0;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int co = co0 + (cf0 + u) * 16 + 4 * grp + e;
            const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                              static_cast<int64_t>(co) * K + k0 + (kf0 + v) * 16 + li;
            if constexpr (OUT_BF16) static_cast<uint16_t*>(out)[o] = f_to_bf16(acc[r * NT + j][u][v][e]);
            else static_cast<float*>(out)[o] = acc[r * NT + j][u][v][e];
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
                int pm, bool transpose_w, hipStream_t stream) {
  const int M = g.N * g.Ho * g.Wo;
  if (M <= 0) return;
  if (pm <= 0) {  // measured (scripts/bench_iconv.py): the largest pixel tile that keeps ~500 workgroups
    constexpr int64_t min_wg = 500;
    const int64_t ncb = Cout / 64;
    pm = 4;
    while (pm > 1 && ((M + 64 * pm - 1) / (64 * pm)) * ncb < min_wg) pm /= 2;
    if (g.C % 64 == 0) pm += 10;   // the LDS-staged kernel whenever its k-step fits
  }
  // pm 11 / 12 / 14: the LDS-staged kernel with 1 / 2 / 4 pixel fragments per wave (C % 64 == 0)
  if (pm > 10 && g.C % 64 == 0) {
    if (pm == 11) launch_lds<1, 4>(x, w, g, Cout, y, add, transpose_w, stream);
    else if (pm == 12) launch_lds<2, 3>(x, w, g, Cout, y, add, transpose_w, stream);
    else launch_lds<4, 2>(x, w, g, Cout, y, add, transpose_w, stream);
    return;
  }
  if (pm > 10) pm -= 10;
  if (transpose_w) {  // only the LDS-staged kernel reads the weight transposed (the wrapper checks C % 64)
    if (pm >= 4) launch_lds<4, 2>(x, w, g, Cout, y, add, true, stream);
    else if (pm == 2) launch_lds<2, 3>(x, w, g, Cout, y, add, true, stream);
    else launch_lds<1, 4>(x, w, g, Cout, y, add, true, stream);
    return;
  }
  if (pm >= 4) launch<4>(x, w, g, Cout, y, add, stream);
  else if (pm == 2) launch<2>(x, w, g, Cout, y, add, stream);
  else launch<1>(x, w, g, Cout, y, add, stream);
}

bool dgrad_s2_ok(const Im2col& g, int Cout) {
  return g.sh == 2 && g.sw == 2 && g.dh == 1 && g.dw == 1 && g.C % 64 == 0 && Cout % 64 == 0 && g.KH <= 3 &&
         g.KW <= 3 && g.ph <= 1 && g.pw <= 1 && g.Ho % 2 == 0 && g.Wo % 2 == 0 &&
         g.H == (g.Ho + 2 * g.ph - g.KH) / 2 + 1 && g.W == (g.Wo + 2 * g.pw - g.KW) / 2 + 1;
}

void dgrad_s2_nhwc(const uint16_t* dy, const uint16_t* w, const Im2col& g, int Cout, uint16_t* dx, const uint16_t* add,
                   int pm, hipStream_t stream) {
  const int64_t M = static_cast<int64_t>(g.N) * (g.Ho >> 1) * (g.Wo >> 1);
  if (M <= 0) return;
  if (pm <= 0) {   // the iconv rule over all four classes: the largest pixel tile keeping ~500 workgroups
    pm = 4;
    while (pm > 1 && ((M + 64 * pm - 1) / (64 * pm)) * (Cout / 64) * 4 < 500) pm /= 2;
  }
  if (pm >= 4) launch_s2<4, 2>(dy, w, g, Cout, dx, add, stream);
  else if (pm == 2) launch_s2<2, 3>(dy, w, g, Cout, dx, add, stream);
  else launch_s2<1, 4>(dy, w, g, Cout, dx, add, stream);
}

// Weight gradient of a 1x1 convolution with NT 64-channel input blocks per workgroup: the
// k-step's 32-pixel dy tile is staged once for NT x tiles (the per-tap kernel re-reads it for
// every input-channel block). NT = 2 or 4.
template <int NS, bool OUT_BF16, int NT, bool PRO>
__global__ __launch_bounds__(256) void k_iwgrad_1x1(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                    Im2col g, int Cout, int64_t rg, int64_t per_split, void* out,
                                                    int64_t split_stride, int64_t group_stride,
                                                    const float* __restrict__ psc, const float* __restrict__ psh) {
  constexpr int TB = 32 * 128;
  constexpr int SB = (1 + NT) * TB;
  __shared__ __attribute__((aligned(16))) char lds[NS * SB];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int K = g.C;
  const int nq = g.C / (64 * NT);
  const int qb = blockIdx.x % nq, cb = blockIdx.x / nq;
  const int c0 = qb * 64 * NT, co0 = cb * 64;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int64_t mbeg = static_cast<int64_t>(gi) * rg + static_cast<int64_t>(sp) * per_split;
  int64_t mend = mbeg + per_split;
  if (mend > static_cast<int64_t>(gi + 1) * rg) mend = static_cast<int64_t>(gi + 1) * rg;
  const int steps = mend > mbeg ? static_cast<int>((mend - mbeg + 31) / 32) : 0;

  const int lrow = wave * 8 + (lane >> 3), lchunk = lane & 7;
  const int lsw = lchunk ^ (2 * tr_g(lrow));   // the global chunk this lane stages (bank swizzle)
  const uint16_t* zsrc = reinterpret_cast<const uint16_t*>(g_iconv_zero) + lchunk * 8;
  const uint64_t az = reinterpret_cast<uint64_t>(zsrc);

  const FastDiv fWo = make_fastdiv(g.Wo), fHo = make_fastdiv(g.Ho);
  const bool ident = g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0 && g.H == g.Ho && g.W == g.Wo;
  auto issue = [&](int s, int slot) {
    const int m = static_cast<int>(mbeg) + s * 32 + lrow;
    const bool mv = m < static_cast<int>(mend);
    const int mm = mv ? m : 0;
    char* base = lds + slot * SB;
    const uint64_t ady = reinterpret_cast<uint64_t>(dy + static_cast<int64_t>(mm) * Cout + co0 + lsw * 8);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(mv ? ady : az), (lds_ptr)(base + wave * 1024), 16,
                                     0, 0);
    bool ok = mv;
    int64_t xo = mm;   // a stride-1 unpadded 1x1 convolution reads the output pixel's own input row
    if (!ident) {
      uint32_t t_, wo_, n_, ho_;
      fdivmod(static_cast<uint32_t>(mm), fWo, t_, wo_);
      fdivmod(t_, fHo, n_, ho_);
      const int hi = static_cast<int>(ho_) * g.sh - g.ph, wi = static_cast<int>(wo_) * g.sw - g.pw;
      ok = mv && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
      xo = (static_cast<int64_t>(n_) * g.H + (ok ? hi : 0)) * g.W + (ok ? wi : 0);
    }
    const uint16_t* xr = x + xo * g.C + c0 + lsw * 8;
#pragma unroll
    for (int j = 0; j < NT; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? reinterpret_cast<uint64_t>(xr + j * 64) : az),
                                       (lds_ptr)(base + TB * (1 + j) + wave * 1024), 16, 0, 0);
  };

  const int cf0 = 2 * (wave >> 1), kf0 = 2 * (wave & 1);
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[NT][2][2];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[j][a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)lds));
  // staged rows carry their 16-byte chunks XOR-swizzled by 2 tr_g(row) (see the staging): fragment f of
  // row r sits at chunk pair f ^ tr_g(r); the second fragment of a pair is dtr = +-32 bytes away
  const int tg = tr_g(8 * grp + q);
  const uint32_t offA = (8 * grp + q) * 128 + 32 * (cf0 ^ tg) + 8 * p;
  const uint32_t offB = TB + (8 * grp + q) * 128 + 32 * (kf0 ^ tg) + 8 * p;
  const uint32_t dtr = (tg & 1) ? static_cast<uint32_t>(-32) : 32u;
  float psv[NT][2] = {}, phv[NT][2] = {};   // PRO: this lane's input channels
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int64_t o = static_cast<int64_t>(gi) * g.C + c0 + j * 64 + (kf0 + v) * 16 + li;
        psv[j][v] = psc[o];
        phv[j][v] = psh[o];
      }
  }

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);
  for (int s = 0; s < steps; ++s) {
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (1 + NT)) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + NT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // inline-asm transposed reads (a ds_read_tr16 builtin makes the compiler drain every
    // outstanding LDS-DMA load first: no prefetch would survive)
    const uint32_t sb = lds0 + (s % NS) * SB;
    s16x4 ra[4], rb[NT][4];
    asm volatile(
        "ds_read_b64_tr_b16 %0, %12\n\t"
        "ds_read_b64_tr_b16 %1, %12 offset:512\n\t"
        "ds_read_b64_tr_b16 %2, %15\n\t"
        "ds_read_b64_tr_b16 %3, %15 offset:512\n\t"
        "ds_read_b64_tr_b16 %4, %13\n\t"
        "ds_read_b64_tr_b16 %5, %13 offset:512\n\t"
        "ds_read_b64_tr_b16 %6, %16\n\t"
        "ds_read_b64_tr_b16 %7, %16 offset:512\n\t"
        "ds_read_b64_tr_b16 %8, %14\n\t"
        "ds_read_b64_tr_b16 %9, %14 offset:512\n\t"
        "ds_read_b64_tr_b16 %10, %17\n\t"
        "ds_read_b64_tr_b16 %11, %17 offset:512\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(ra[0]), "=&v"(ra[1]), "=&v"(ra[2]), "=&v"(ra[3]), "=&v"(rb[0][0]), "=&v"(rb[0][1]), "=&v"(rb[0][2]),
          "=&v"(rb[0][3]), "=&v"(rb[1][0]), "=&v"(rb[1][1]), "=&v"(rb[1][2]), "=&v"(rb[1][3])
        : "v"(sb + offA), "v"(sb + offB), "v"(sb + offB + TB), "v"(sb + offA + dtr), "v"(sb + offB + dtr), "v"(sb + offB + TB + dtr)
        : "memory");
    if constexpr (NT == 4) {
      asm volatile(
          "ds_read_b64_tr_b16 %0, %8\n\t"
          "ds_read_b64_tr_b16 %1, %8 offset:512\n\t"
          "ds_read_b64_tr_b16 %2, %10\n\t"
          "ds_read_b64_tr_b16 %3, %10 offset:512\n\t"
          "ds_read_b64_tr_b16 %4, %9\n\t"
          "ds_read_b64_tr_b16 %5, %9 offset:512\n\t"
          "ds_read_b64_tr_b16 %6, %11\n\t"
          "ds_read_b64_tr_b16 %7, %11 offset:512\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(rb[2][0]), "=&v"(rb[2][1]), "=&v"(rb[2][2]), "=&v"(rb[2][3]), "=&v"(rb[3][0]), "=&v"(rb[3][1]),
            "=&v"(rb[3][2]), "=&v"(rb[3][3])
          : "v"(sb + offB + 2 * TB), "v"(sb + offB + 3 * TB), "v"(sb + offB + 2 * TB + dtr), "v"(sb + offB + 3 * TB + dtr)
        : "memory");
    }
    // the refilled slot was read in the previous k-step, before every wave passed this barrier
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    bf16x8 a[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) a[u] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ra[2 * u], ra[2 * u + 1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        bf16x8 bx =
            __builtin_bit_cast(bf16x8, __builtin_shufflevector(rb[j][2 * v], rb[j][2 * v + 1], 0, 1, 2, 3, 4, 5, 6, 7));
        if constexpr (PRO) bx = pro_frag(bx, psv[j][v], phv[j][v]);
#pragma unroll
        for (int u = 0; u < 2; ++u)
          acc[j][u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], bx, acc[j][u][v], 0, 0, 0);
      }
  }

#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int k0 = c0 + j * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + (cf0 + u) * 16 + 4 * grp + e;
          const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                            static_cast<int64_t>(co) * K + k0 + (kf0 + v) * 16 + li;
          if constexpr (OUT_BF16) static_cast<uint16_t*>(out)[o] = f_to_bf16(acc[j][u][v][e]);
          else static_cast<float*>(out)[o] = acc[j][u][v][e];
        }
  }
}

// 1x1 weight gradient with 128 output channels x 128 input channels per workgroup (Cout, C % 128 == 0):
// each wave computes 4 x 4 fragments (64 x 64) -- four times the MFMAs per staged byte and per barrier of
// the 2 x 2-fragment kernel above, which is latency-bound (one 32-pixel step = 8 MFMAs per wave between
// barriers). A stage is 64 pixels (two 32-deep MFMA steps): dy [64 px][128 co] and x [64 px][128 ci] as
// four [64][64] bf16 sub-tiles of 128-byte rows, staged by LDS-DMA with the bank swizzle (tr_g), read
// transposed; 3-deep ring (96 KB: one workgroup per CU).
constexpr int kW1Stage = 4 * 64 * 128;   // bytes per stage: dy0 | dy1 | x0 | x1

// NS: ring depth (3: 96 KB, one workgroup per CU; 2: 64 KB, two, for splits of at most four 64-pixel
// stages, where a workgroup's whole K loop is shorter than the load latency the third stage hides:
// ResNet-50 CIFAR layer4, 10.9-21.8 vs 13.6-26.3 us per call, profiles/r6/iwgrad_wide/). (A 16-byte
// LDS-staged epilogue measured no faster than the 2-byte stores, which merge in L2.)
template <bool OUT_BF16, bool PRO, int NS = 3>
__global__ __launch_bounds__(256) void k_iwgrad_1x1_wide(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                         Im2col g, int Cout, int64_t rg, int64_t per_split, void* out,
                                                         int64_t split_stride, int64_t group_stride,
                                                         const float* __restrict__ psc, const float* __restrict__ psh) {
  constexpr int SUB = 64 * 128;          // one [64 px][64 ch] sub-tile
  extern __shared__ __attribute__((aligned(16))) char wlds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = g.C;
  const int nq = g.C / 128;
  const int qb = blockIdx.x % nq, cb = blockIdx.x / nq;
  const int c0 = qb * 128, co0 = cb * 128;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int64_t mbeg = static_cast<int64_t>(gi) * rg + static_cast<int64_t>(sp) * per_split;
  int64_t mend = mbeg + per_split;
  if (mend > static_cast<int64_t>(gi + 1) * rg) mend = static_cast<int64_t>(gi + 1) * rg;
  const int steps = mend > mbeg ? static_cast<int>((mend - mbeg + 63) / 64) : 0;
  const FastDiv fWo = make_fastdiv(g.Wo), fHo = make_fastdiv(g.Ho);
  const bool ident = g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0 && g.H == g.Ho && g.W == g.Wo;

  // staging: instruction u (0..7) of this wave covers sub-tile u / 2, rows 8 ((u & 1) * 4 + wave) + lane / 8
  const int lchunk = lane & 7;
  const uint16_t* zsrc = reinterpret_cast<const uint16_t*>(g_iconv_zero) + lchunk * 8;
  const uint64_t az = reinterpret_cast<uint64_t>(zsrc);
  auto issue = [&](int s, int slot) {
    char* base = wlds + slot * kW1Stage;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const int row = 8 * (hb * 4 + wave) + (lane >> 3);
      const int lsw = lchunk ^ (2 * tr_g(row));
      const int m = static_cast<int>(mbeg) + s * 64 + row;   // < 2^31: checked by the host wrapper
      const bool mv = m < static_cast<int>(mend);
      const int mm = mv ? m : 0;
      bool ok = mv;
      int64_t xo = mm;   // a stride-1 unpadded 1x1 convolution reads the output pixel's own input row
      if (!ident) {
        uint32_t t, wo, n, ho;
        fdivmod(static_cast<uint32_t>(mm), fWo, t, wo);
        fdivmod(t, fHo, n, ho);
        const int hi = static_cast<int>(ho) * g.sh - g.ph, wi = static_cast<int>(wo) * g.sw - g.pw;
        ok = mv && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
        xo = (static_cast<int64_t>(n) * g.H + (ok ? hi : 0)) * g.W + (ok ? wi : 0);
      }
      const uint16_t* dr = dy + static_cast<int64_t>(mm) * Cout + co0 + lsw * 8;
      const uint16_t* xr = x + xo * g.C + c0 + lsw * 8;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(mv ? reinterpret_cast<uint64_t>(dr + 64 * b) : az),
                                         (lds_ptr)(base + b * SUB + (hb * 4 + wave) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? reinterpret_cast<uint64_t>(xr + 64 * b) : az),
                                         (lds_ptr)(base + (2 + b) * SUB + (hb * 4 + wave) * 1024), 16, 0, 0);
      }
    }
  };

  // wave (sa, sb): co sub-tile sa = wave >> 1 (fragments 4 sa ..), ci sub-tile sb = wave & 1
  const int sa = wave >> 1, sbk = wave & 1;
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int trow = 8 * grp + q, tg = tr_g(trow);
  uint32_t offA[4], offB[4];   // fragment k: chunk pair k ^ tg of row trow (+ 4 rows at offset 512)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    offA[k] = sa * SUB + trow * 128 + 32 * (k ^ tg) + 8 * p;
    offB[k] = (2 + sbk) * SUB + trow * 128 + 32 * (k ^ tg) + 8 * p;
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)wlds));
  float psv[4] = {}, phv[4] = {};   // PRO: this lane's four input channels
  if constexpr (PRO) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t o = static_cast<int64_t>(gi) * g.C + c0 + (4 * sbk + v) * 16 + li;
      psv[v] = psc[o];
      phv[v] = psh[o];
    }
  }

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);
  for (int s = 0; s < steps; ++s) {
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // the next stage's 8 glds may stay in flight
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    const uint32_t sbase = lds0 + (s % NS) * kW1Stage;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {   // pixel rows 32 ks .. 32 ks + 31
      const uint32_t b0 = sbase + ks * 4096;
      s16x4 ra[8], rb[8];
      asm volatile(
          "ds_read_b64_tr_b16 %0, %16\n\t"
          "ds_read_b64_tr_b16 %1, %16 offset:512\n\t"
          "ds_read_b64_tr_b16 %2, %17\n\t"
          "ds_read_b64_tr_b16 %3, %17 offset:512\n\t"
          "ds_read_b64_tr_b16 %4, %18\n\t"
          "ds_read_b64_tr_b16 %5, %18 offset:512\n\t"
          "ds_read_b64_tr_b16 %6, %19\n\t"
          "ds_read_b64_tr_b16 %7, %19 offset:512\n\t"
          "ds_read_b64_tr_b16 %8, %20\n\t"
          "ds_read_b64_tr_b16 %9, %20 offset:512\n\t"
          "ds_read_b64_tr_b16 %10, %21\n\t"
          "ds_read_b64_tr_b16 %11, %21 offset:512\n\t"
          "ds_read_b64_tr_b16 %12, %22\n\t"
          "ds_read_b64_tr_b16 %13, %22 offset:512\n\t"
          "ds_read_b64_tr_b16 %14, %23\n\t"
          "ds_read_b64_tr_b16 %15, %23 offset:512\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(ra[0]), "=&v"(ra[1]), "=&v"(ra[2]), "=&v"(ra[3]), "=&v"(ra[4]), "=&v"(ra[5]), "=&v"(ra[6]),
            "=&v"(ra[7]), "=&v"(rb[0]), "=&v"(rb[1]), "=&v"(rb[2]), "=&v"(rb[3]), "=&v"(rb[4]), "=&v"(rb[5]),
            "=&v"(rb[6]), "=&v"(rb[7])
          : "v"(b0 + offA[0]), "v"(b0 + offA[1]), "v"(b0 + offA[2]), "v"(b0 + offA[3]), "v"(b0 + offB[0]),
            "v"(b0 + offB[1]), "v"(b0 + offB[2]), "v"(b0 + offB[3])
          : "memory");
      bf16x8 a[4], b[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ra[2 * k], ra[2 * k + 1], 0, 1, 2, 3, 4, 5, 6, 7));
        b[k] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(rb[2 * k], rb[2 * k + 1], 0, 1, 2, 3, 4, 5, 6, 7));
        if constexpr (PRO) b[k] = pro_frag(b[k], psv[k], phv[k]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[v], acc[u][v], 0, 0, 0);
    }
  }

#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + (4 * sa + u) * 16 + 4 * grp + e;
        const int k = c0 + (4 * sbk + v) * 16 + li;
        const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                          static_cast<int64_t>(co) * K + k;
        if constexpr (OUT_BF16) static_cast<uint16_t*>(out)[o] = f_to_bf16(acc[u][v][e]);
        else static_cast<float*>(out)[o] = acc[u][v][e];
      }
}

// Taps per weight-gradient workgroup: a 3x3 kernel's row of three taps shares each staged dy tile
// (profiles/r2/ab_iwgrad_9tap.log: all nine taps leave one wave per SIMD and lose); a 1x1
// convolution's two 64-channel input blocks share it (profiles/r2/iwgrad_wg_nt_sweep.log).
int iwgrad_taps_per_block(int kw, int kh, int C, int Cout) {
  if (kw == 1 && kh == 1) return C % 128 == 0 ? (Cout % 128 == 0 ? 4 : 2) : 1;   // 4: the 128 x 128 tile
  return kw == 3 ? 3 : 1;
}

template <bool PRO>
void iwgrad_launch(const uint16_t* x, const uint16_t* dy, const Im2col& g, int Cout, int groups, int64_t rg,
                   int splits, void* out, bool out_bf16, int64_t split_stride, int64_t group_stride, hipStream_t stream,
                   const float* psc, const float* psh) {
  const int K = g.KH * g.KW * g.C;
  if (splits < 1) splits = 1;
  const int64_t per_split = (rg + splits - 1) / splits;
  const int tpb = iwgrad_taps_per_block(g.KW, g.KH, g.C, Cout);
  if (tpb == 4 && g.KW == 1) {   // 1x1, C and Cout % 128: the 128 x 128-tile kernel
    static bool once = (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_iwgrad_1x1_wide<true, PRO>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 3 * kW1Stage),
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_iwgrad_1x1_wide<false, PRO>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 3 * kW1Stage),
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_iwgrad_1x1_wide<true, PRO, 2>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kW1Stage),
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_iwgrad_1x1_wide<false, PRO, 2>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kW1Stage),
                        true);
    (void)once;
    const dim3 grid((g.C / 128) * (Cout / 128), groups, splits);
    const bool ns2 = (per_split + 63) / 64 <= 4;
    if (out_bf16 && ns2)
      hipLaunchKernelGGL((k_iwgrad_1x1_wide<true, PRO, 2>), grid, dim3(256), 2 * kW1Stage, stream, x, dy, g, Cout, rg,
                         per_split, out, split_stride, group_stride, psc, psh);
    else if (out_bf16)
      hipLaunchKernelGGL((k_iwgrad_1x1_wide<true, PRO>), grid, dim3(256), 3 * kW1Stage, stream, x, dy, g, Cout, rg,
                         per_split, out, split_stride, group_stride, psc, psh);
    else if (ns2)
      hipLaunchKernelGGL((k_iwgrad_1x1_wide<false, PRO, 2>), grid, dim3(256), 2 * kW1Stage, stream, x, dy, g, Cout, rg,
                         per_split, out, split_stride, group_stride, psc, psh);
    else
      hipLaunchKernelGGL((k_iwgrad_1x1_wide<false, PRO>), grid, dim3(256), 3 * kW1Stage, stream, x, dy, g, Cout, rg,
                         per_split, out, split_stride, group_stride, psc, psh);
    return;
  }
  if (tpb == 2 && g.KW == 1) {   // 1x1: two 64-channel input blocks per workgroup, 3 pipeline stages
    const dim3 grid((g.C / 128) * (Cout / 64), groups, splits);
    if (out_bf16)
      hipLaunchKernelGGL((k_iwgrad_1x1<3, true, 2, PRO>), grid, dim3(256), 0, stream, x, dy, g, Cout, rg, per_split,
                         out, split_stride, group_stride, psc, psh);
    else
      hipLaunchKernelGGL((k_iwgrad_1x1<3, false, 2, PRO>), grid, dim3(256), 0, stream, x, dy, g, Cout, rg, per_split,
                         out, split_stride, group_stride, psc, psh);
    return;
  }
  if constexpr (!PRO) {
    if (tpb == 3) {                // the three taps of a kernel row per workgroup
      const dim3 grid(g.KH * (g.C / 64) * (Cout / 64), groups, splits);
      if (out_bf16)
        hipLaunchKernelGGL((k_iwgrad_rows<3, true, 1>), grid, dim3(256), 0, stream, x, dy, g, Cout, rg, per_split, out,
                           split_stride, group_stride);
      else
        hipLaunchKernelGGL((k_iwgrad_rows<3, false, 1>), grid, dim3(256), 0, stream, x, dy, g, Cout, rg, per_split, out,
                           split_stride, group_stride);
      return;
    }
  }
  const dim3 grid((K / 64) * (Cout / 64), groups, splits);
  if (out_bf16)
    hipLaunchKernelGGL((k_iwgrad<3, true, PRO>), grid, dim3(256), 0, stream, x, dy, g, Cout, rg, per_split, out,
                       split_stride, group_stride, psc, psh);
  else
    hipLaunchKernelGGL((k_iwgrad<3, false, PRO>), grid, dim3(256), 0, stream, x, dy, g, Cout, rg, per_split, out,
                       split_stride, group_stride, psc, psh);
}

void iwgrad_nhwc(const uint16_t* x, const uint16_t* dy, const Im2col& g, int Cout, int groups, int64_t rg,
                 int splits, void* out, bool out_bf16, int64_t split_stride, int64_t group_stride, hipStream_t stream,
                 const float* pro_scale, const float* pro_shift) {
  if (pro_scale)   // 1x1 / stride 1 / no padding only (host-checked): the kernels' input has no padding pixel
    iwgrad_launch<true>(x, dy, g, Cout, groups, rg, splits, out, out_bf16, split_stride, group_stride, stream,
                        pro_scale, pro_shift);
  else
    iwgrad_launch<false>(x, dy, g, Cout, groups, rg, splits, out, out_bf16, split_stride, group_stride, stream, nullptr,
                         nullptr);
}

}  // namespace gpu
}  // namespace garfield
