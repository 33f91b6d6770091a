// fp32 NHWC convolutions for the reference-precision grouped step, on bf16 MFMA (gfx950).
//
// The reference trains in fp32 (pytorch_impl/applications/Garfield_CC/trainer.py:296-303, no
// autocast). gfx950 has no xf32 MFMA and its f32-input MFMA runs at the f32 vector rate (1/16 of
// bf16: 157 TF/s), so an fp32 product is formed from bf16 pieces: every fp32 operand is split as
//   v = v0 + v1 + v2 + r,  v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1),  |r| <~ 2^-27 |v|
// and a·b ≈ Σ_{i + j <= 2} a_i·b_j (a0b0 + a0b1 + a1b0 + a0b2 + a2b0 + a1b1; the dropped terms are
// ~2^-26 of the product, under fp32's own rounding): six v_mfma_f32_16x16x32_bf16 with fp32
// accumulation, 96 cycles per 16x16x32 block against 256 for the f32 MFMA. Two pieces (three
// products) leave ~2^-17 per product, which a BatchNorm network's backward (cancellation in
// dz - mean(dz) - x̂·mean(dz·x̂)) amplifies to ~1e-2 of the gradient: not the reference's precision.
// Activations stay fp32 in HBM; the weights are split once per step (k_wsplit: W -> the three
// pieces [3][Cout][K] and the channel-transposed pieces [3][Cin][KH][KW][Cout] of the data gradient).
//
// * k_cf32_conv: implicit-GEMM convolution y[m, co] = Σ_{tap, c} src[pixel(m, tap), c] · A[co, tap, c]
//   (+ add). Forward: src = x, A = W [Cout][KH][KW][Cin]. Data gradient (DG): src = dy, A = Wt
//   [Cin][KH][KW][Cout], and input pixel (h, w) gathers dy[(h + ph - i·dh) / sh, (w + pw - j·dw) / sw]
//   where the division is exact (the transposed convolution; any stride). The weight is the
//   MFMA A operand (a lane holds 8 consecutive k of one output channel: 16 bytes of each piece),
//   the activation the B operand (8 consecutive channels of one pixel: two float4 loads, split in
//   registers); the loads of k-step s + 1 are in flight while step s multiplies. Workgroup: 4 waves
//   x 16·PM pixels x 64 output channels.
// * k_cf32_wgrad: per-worker weight gradient dW_g[co, (tap, ci)] = Σ_{m in worker g} dy[m, co] ·
//   x[pixel(m, tap), ci]: the reduction runs over pixels, so both operands are staged (fp32 ->
//   split in registers -> [32 pixel][64 channel] bf16 piece tiles in LDS, double-buffered) and read
//   with ds_read_b64_tr_b16 (16 lanes gather 4 rows x 16 columns). Tile: 64 co x 64 k, 32 pixels
//   per k-step, the worker's pixels optionally split into `splits` fp32 slabs.
// * k_f32_linear_*: the classifier (per-worker dW, db straight into the exchange rows), and the
//   global average pool: VALU kernels (tens of MFLOP), so the fp32 step runs no library GEMM.
#include "bn_gpu.hpp"
#include "conv_f32.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

using lds_ptr = __attribute__((address_space(3))) void*;
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int kNP = 3;   // bf16 pieces per fp32 value

// (a, b) -> three packed bf16 pairs p[0..2] with a ≈ Σ p_i.lo, b ≈ Σ p_i.hi
__device__ __forceinline__ void split2(float a, float b, uint32_t (&p)[kNP]) {
#pragma unroll
  for (int i = 0; i < kNP; ++i) {
    p[i] = pack_bf16x2(a, b);
    a -= __uint_as_float(p[i] << 16);
    b -= __uint_as_float(p[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void split8(const float4& a, const float4& b, bf16x8 (&v)[kNP]) {
  uint32_t q[4][kNP];
  split2(a.x, a.y, q[0]);
  split2(a.z, a.w, q[1]);
  split2(b.x, b.y, q[2]);
  split2(b.z, b.w, q[3]);
#pragma unroll
  for (int i = 0; i < kNP; ++i) v[i] = __builtin_bit_cast(bf16x8, make_uint4(q[0][i], q[1][i], q[2][i], q[3][i]));
}

// acc += Σ_{i + j <= 2} a_i · b_j, the small terms first
__device__ __forceinline__ f32x4 mma6(const bf16x8 (&a)[kNP], const bf16x8 (&b)[kNP], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// implicit-GEMM convolution

template <int PM>
struct Step {
  bf16x8 a[4][kNP];
  float4 b0[PM], b1[PM];
};

// GATHER (a forward over Cs % 32 != 0 channels, e.g. the 3-channel CIFAR stem): the reduction
// runs over the flattened (tap, channel) index k < K padded to Kp = 32·steps, each lane gathering its
// 8 consecutive k one element at a time; the weight rows are [Co][Kp] (zero padding).
template <int PM, bool DG, bool ADD, bool GATHER>
__global__ __launch_bounds__(256) void k_cf32_conv(const float* __restrict__ src, const uint16_t* __restrict__ w3,
                                                   ConvF32Geo g, float* __restrict__ out, const float* __restrict__ add) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pl = lane & 15, kq = lane >> 4;
  const int M = g.N * g.Ho * g.Wo;
  const int Kr = g.KH * g.KW * g.Cs;                        // real reduction length
  const int K = GATHER ? (Kr + 31) / 32 * 32 : Kr;          // weight row stride
  const int m0 = blockIdx.x * (64 * PM) + wave * 16 * PM;
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
    const int ho = t % g.Ho;
    nb[r] = t / g.Ho;
    if constexpr (DG) {
      hb[r] = ho + g.ph;
      wb[r] = wo + g.pw;
    } else {
      hb[r] = ho * g.sh - g.ph;
      wb[r] = wo * g.sw - g.pw;
    }
  }
  // w3: the weight's three pieces [3][Co][K]
  const int64_t piece = static_cast<int64_t>(g.Co) * K;
  const uint16_t* wp[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wp[c] = w3 + static_cast<int64_t>(co0 + c * 16 + pl) * K + kq * 8;
  const int csteps = GATHER ? 1 : g.Cs / 32;
  const int steps = GATHER ? K / 32 : g.KH * g.KW * csteps;

  auto load = [&](int s, Step<PM>& f) {
    const int tap = s / csteps;
    const int c0 = (s - tap * csteps) * 32;
    const int i = tap / g.KW, j = tap - (tap / g.KW) * g.KW;
    const int koff = GATHER ? s * 32 : tap * g.Cs + c0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < kNP; ++i) f.a[c][i] = *reinterpret_cast<const bf16x8*>(wp[c] + i * piece + koff);
    if constexpr (GATHER) {
#pragma unroll
      for (int r = 0; r < PM; ++r) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = s * 32 + kq * 8 + e;
          const int tp = k / g.Cs, ch = k - tp * g.Cs;
          const int ti = tp / g.KW, tj = tp - ti * g.KW;
          const int hs = hb[r] + ti * g.dh, ws = wb[r] + tj * g.dw;
          const bool ok = pv[r] && k < Kr && hs >= 0 && hs < g.Hs && ws >= 0 && ws < g.Ws;
          const int64_t pix = (static_cast<int64_t>(nb[r]) * g.Hs + (ok ? hs : 0)) * g.Ws + (ok ? ws : 0);
          const float a = src[pix * g.Cs + (ok ? ch : 0)];
          v[e] = ok ? a : 0.f;
        }
        f.b0[r] = make_float4(v[0], v[1], v[2], v[3]);
        f.b1[r] = make_float4(v[4], v[5], v[6], v[7]);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < PM; ++r) {
      int hs, ws;
      bool ok;
      if constexpr (DG) {
        const int th = hb[r] - i * g.dh, tw = wb[r] - j * g.dw;
        hs = th / g.sh;
        ws = tw / g.sw;
        ok = pv[r] && th >= 0 && tw >= 0 && hs * g.sh == th && ws * g.sw == tw && hs < g.Hs && ws < g.Ws;
      } else {
        hs = hb[r] + i * g.dh;
        ws = wb[r] + j * g.dw;
        ok = pv[r] && hs >= 0 && hs < g.Hs && ws >= 0 && ws < g.Ws;
      }
      const int64_t pix = (static_cast<int64_t>(nb[r]) * g.Hs + (ok ? hs : 0)) * g.Ws + (ok ? ws : 0);
      const float* p = src + pix * g.Cs + c0 + kq * 8;
      const float4 a = *reinterpret_cast<const float4*>(p);
      const float4 b = *reinterpret_cast<const float4*>(p + 4);
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      f.b0[r] = ok ? a : z;
      f.b1[r] = ok ? b : z;
    }
  };

  f32x4 acc[PM][4];
#pragma unroll
  for (int r = 0; r < PM; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  Step<PM> cur, nxt;
  load(0, cur);
  for (int s = 0; s < steps; ++s) {
    if (s + 1 < steps) load(s + 1, nxt);
#pragma unroll
    for (int r = 0; r < PM; ++r) {
      bf16x8 b[kNP];
      split8(cur.b0[r], cur.b1[r], b);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = mma6(cur.a[c], b, acc[r][c]);
    }
    cur = nxt;
  }

  // D[co = 4*kq + e][pixel = pl]: four consecutive output channels of one pixel per lane
#pragma unroll
  for (int r = 0; r < PM; ++r) {
    if (!pv[r]) continue;
    const int64_t rowoff = static_cast<int64_t>(m0 + r * 16 + pl) * g.Co;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t off = rowoff + co0 + c * 16 + kq * 4;
      float4 v = make_float4(acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]);
      if constexpr (ADD) {
        const float4 a = *reinterpret_cast<const float4*>(add + off);
        v.x += a.x;
        v.y += a.y;
        v.z += a.z;
        v.w += a.w;
      }
      *reinterpret_cast<float4*>(out + off) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-staged implicit-GEMM convolution (Cs % 32 == 0): every k-step (one tap, 32 source channels)
// stages the three weight pieces [3][64 co][32 k] bf16 and the activation tile [64·PM pixels][32
// channels] fp32 by global_load_lds (no VGPR round trip; chunks XOR-swizzled on the global side so
// the fragment reads below spread over the banks) through an NS-deep ring: NS-1 k-steps of loads in
// flight. A wave reads its B fragments as fp32 (two ds_read_b128) and splits them in registers.
// Data gradient of a strided convolution: the output pixels are processed in parity classes
// (blockIdx.z = (h mod sh, w mod sw)); a class gathers dy only through the taps that hit it
// (i ≡ h + ph mod sh), so no MFMA is spent on the zero taps of the transposed convolution
// (9 taps over the 4 classes of a 3x3 / stride-2 layer, not 36).

__device__ __attribute__((aligned(16))) float g_cf32_zero[8];   // 32 zero bytes: source of padded taps

// Split-K (ksplit > 1: layers with few output tiles and a long reduction, e.g. 256 channels of 3x3
// at 2x2 pixels): blockIdx.z = class * ksplit + kz, split kz runs k-steps [kz·chunk, (kz+1)·chunk) and
// writes its fp32 partial tile into slab kz of `out` (k_cf32_ksum then adds the slabs, + add).
template <int PM, int NS, bool DG, bool ADD>
__global__ __launch_bounds__(256) void k_cf32_conv_lds(const float* __restrict__ src, const uint16_t* __restrict__ w3,
                                                       ConvF32Geo g, float* __restrict__ out,
                                                       const float* __restrict__ add, int ksplit) {
  constexpr int BM = 64 * PM;
  constexpr int WB = kNP * 64 * 64;     // weight pieces per stage (bytes): 3 x 64 rows x 64 B
  constexpr int XB = BM * 128;          // activation tile per stage (bytes): BM rows x 128 B
  constexpr int SB = WB + XB;
  constexpr int WI = WB / 1024 / 4;     // glds per wave per stage: weights (3)
  constexpr int XI = XB / 1024 / 4;     // ... activations (2 PM)
  constexpr int PER = WI + XI;
  __shared__ __attribute__((aligned(16))) char lds[NS * SB];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = g.KH * g.KW * g.Cs;
  // parity class of this workgroup's output pixels (data gradient of a strided convolution)
  const int csh = DG ? g.sh : 1, csw = DG ? g.sw : 1;
  const int cls = static_cast<int>(blockIdx.z) / ksplit, kz = static_cast<int>(blockIdx.z) - cls * ksplit;
  const int ca = DG ? cls / g.sw : 0, cb = DG ? cls % g.sw : 0;
  const int Hc = (g.Ho - ca + csh - 1) / csh, Wc = (g.Wo - cb + csw - 1) / csw;
  const int Mc = g.N * Hc * Wc;
  const int m0 = blockIdx.x * BM;
  if (m0 >= Mc) return;   // whole workgroup (a class with fewer pixels than the grid covers)
  const int co0 = blockIdx.y * 64;
  // taps of this class: i = ti0 + t * tstep_i (forward: every tap)
  int ti0 = 0, tj0 = 0, tsi = 1, tsj = 1;
  if constexpr (DG) {
    ti0 = (ca + g.ph) % g.sh;
    tj0 = (cb + g.pw) % g.sw;
    tsi = g.sh;
    tsj = g.sw;
  }
  const int ni = ti0 < g.KH ? (g.KH - ti0 + tsi - 1) / tsi : 0;
  const int nj = tj0 < g.KW ? (g.KW - tj0 + tsj - 1) / tsj : 0;
  const int csteps = g.Cs / 32;
  const int all_steps = ni * nj * csteps;
  const int chunk = (all_steps + ksplit - 1) / ksplit;
  const int sbeg = kz * chunk < all_steps ? kz * chunk : all_steps;
  const int steps = (sbeg + chunk < all_steps ? sbeg + chunk : all_steps) - sbeg;
  if (ksplit > 1) out += static_cast<int64_t>(kz) * g.N * g.Ho * g.Wo * g.Co;   // this split's slab

  // taps of the class in k-step order t = ti * nj + tj: source offset (di, dj) of tap t relative to
  // the row's base pixel -- forward (i·dh, j·dw); data gradient (dI0 - ti, dJ0 - tj) with
  // dI0 = (ca + ph - ti0) / sh (exact in this class)
  const int dI0 = DG ? (ca + g.ph - ti0) / g.sh : 0, dJ0 = DG ? (cb + g.pw - tj0) / g.sw : 0;
  auto tap_di = [&](int ti) { return DG ? dI0 - ti : (ti0 + ti * tsi) * g.dh; };
  auto tap_dj = [&](int tj) { return DG ? dJ0 - tj : (tj0 + tj * tsj) * g.dw; };

  // this lane's activation rows: rows (wave * XI + u) * 8 + lane / 8 of the tile, chunk lane % 8. Per
  // row: its base element offset (with the lane's swizzled chunk) and the bit mask of the taps whose
  // source pixel is inside the image (KH * KW <= 32), so a k-step costs a shift, an add and a select.
  const int xr = lane >> 3, xc = lane & 7;
  int xoff[XI];
  uint32_t xmask[XI];
#pragma unroll
  for (int u = 0; u < XI; ++u) {
    const int row = (wave * XI + u) * 8 + xr;
    const int m = m0 + row;
    const int mm = m < Mc ? m : 0;
    const int wc = mm % Wc;
    const int t = mm / Wc;
    const int hc = t % Hc, n = t / Hc;
    const int hb = DG ? hc : hc * g.sh - g.ph, wb = DG ? wc : wc * g.sw - g.pw;
    uint32_t mask = 0;
    if (m < Mc)
      for (int ti = 0; ti < ni; ++ti) {
        const int hs = hb + tap_di(ti);
        if (hs < 0 || hs >= g.Hs) continue;
        for (int tj = 0; tj < nj; ++tj) {
          const int ws = wb + tap_dj(tj);
          if (ws >= 0 && ws < g.Ws) mask |= 1u << (ti * nj + tj);
        }
      }
    xmask[u] = mask;
    const int swz = (row >> 1) & 7;   // chunk swizzle: 16 consecutive rows of one fragment read hit 16 bank groups
    xoff[u] = ((n * g.Hs + hb) * g.Ws + wb) * g.Cs + (xc ^ swz) * 4;
  }
  // weight rows: glds block q covers rows 16 q .. 16 q + 15 of one piece, lane -> row lane / 4, chunk lane % 4
  const int wr = lane >> 2, wcn = lane & 3;
  const int64_t piece = static_cast<int64_t>(g.Co) * K;
  const uint16_t* wsrc[WI];
#pragma unroll
  for (int u = 0; u < WI; ++u) {
    const int q = wave * WI + u;                 // 0 .. 11: piece q / 4, rows 16 (q % 4) + wr
    const int row = 16 * (q & 3) + wr;
    wsrc[u] = w3 + (q >> 2) * piece + static_cast<int64_t>(co0 + row) * K + ((wcn ^ ((row >> 2) & 3)) * 8);
  }
  const uint64_t az = reinterpret_cast<uint64_t>(g_cf32_zero);

  // k-step walk (issue order): tap (ti, tj), channel block c0 -- no divisions in the loop
  int it_ti, it_tj, it_c0;
  {
    const int tap = sbeg / csteps;
    it_c0 = (sbeg - tap * csteps) * 32;
    it_ti = nj ? tap / nj : 0;
    it_tj = tap - it_ti * nj;
  }
  auto issue = [&](int slot) {
    const int i = ti0 + it_ti * tsi, j = tj0 + it_tj * tsj;
    const int tbit = it_ti * nj + it_tj;
    char* base = lds + slot * SB;
    const int koff = (i * g.KW + j) * g.Cs + it_c0;
#pragma unroll
    for (int u = 0; u < WI; ++u)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(wsrc[u] + koff),
                                       (lds_ptr)(base + (wave * WI + u) * 1024), 16, 0, 0);
    const int toff = (tap_di(it_ti) * g.Ws + tap_dj(it_tj)) * g.Cs + it_c0;
#pragma unroll
    for (int u = 0; u < XI; ++u) {
      const bool ok = (xmask[u] >> tbit) & 1u;
      const uint64_t ax = reinterpret_cast<uint64_t>(src + (xoff[u] + toff));
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? ax : az),
                                       (lds_ptr)(base + WB + (wave * XI + u) * 1024), 16, 0, 0);
    }
    it_c0 += 32;
    if (it_c0 == g.Cs) {
      it_c0 = 0;
      if (++it_tj == nj) {
        it_tj = 0;
        ++it_ti;
      }
    }
  };

  f32x4 acc[PM][4];
#pragma unroll
  for (int r = 0; r < PM; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0);
  for (int s = 0; s < steps; ++s) {
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < steps) issue((s + NS - 1) % NS);
    const char* base = lds + (s % NS) * SB;
    bf16x8 a[4][kNP];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int row = c * 16 + fr;
#pragma unroll
      for (int i = 0; i < kNP; ++i)
        a[c][i] = *reinterpret_cast<const bf16x8*>(base + i * 4096 + row * 64 + ((fq ^ ((row >> 2) & 3)) * 16));
    }
#pragma unroll
    for (int r = 0; r < PM; ++r) {
      const int row = (wave * PM + r) * 16 + fr;
      const int swz = (row >> 1) & 7;
      const float4 v0 = *reinterpret_cast<const float4*>(base + WB + row * 128 + ((2 * fq) ^ swz) * 16);
      const float4 v1 = *reinterpret_cast<const float4*>(base + WB + row * 128 + ((2 * fq + 1) ^ swz) * 16);
      bf16x8 b[kNP];
      split8(v0, v1, b);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = mma6(a[c], b, acc[r][c]);
    }
    // every wave's fragment reads of this slot retire before the barrier that lets it be refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // D[co = 4*fq + e][pixel = fr]: four consecutive output channels of one pixel per lane
#pragma unroll
  for (int r = 0; r < PM; ++r) {
    const int m = m0 + (wave * PM + r) * 16 + fr;
    if (m >= Mc) continue;
    const int wc = m % Wc;
    const int t = m / Wc;
    const int hc = t % Hc, n = t / Hc;
    const int64_t pix = (static_cast<int64_t>(n) * g.Ho + hc * csh + ca) * g.Wo + wc * csw + cb;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t off = pix * g.Co + co0 + c * 16 + fq * 4;
      float4 v = make_float4(acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]);
      if constexpr (ADD) {
        const float4 a4 = *reinterpret_cast<const float4*>(add + off);
        v.x += a4.x;
        v.y += a4.y;
        v.z += a4.z;
        v.w += a4.w;
      }
      *reinterpret_cast<float4*>(out + off) = v;
    }
  }
}

template <int PM, int NS, bool DG>
void launch_conv_lds(const float* src, const uint16_t* w3, const ConvF32Geo& g, float* out, const float* add,
                     int ksplit, hipStream_t stream) {
  const int csh = DG ? g.sh : 1, csw = DG ? g.sw : 1;
  const int Mc = g.N * ((g.Ho + csh - 1) / csh) * ((g.Wo + csw - 1) / csw);   // the largest class (0, 0)
  const dim3 grid((Mc + 64 * PM - 1) / (64 * PM), g.Co / 64, csh * csw * ksplit);
  if (add && ksplit == 1)
    hipLaunchKernelGGL((k_cf32_conv_lds<PM, NS, DG, true>), grid, dim3(256), 0, stream, src, w3, g, out, add, 1);
  else
    hipLaunchKernelGGL((k_cf32_conv_lds<PM, NS, DG, false>), grid, dim3(256), 0, stream, src, w3, g, out, nullptr,
                       ksplit);
}

// out[i] = Σ_s part[s][i] (+ add[i]), float4 lanes (the slab is a multiple of 64 floats)
__global__ __launch_bounds__(256) void k_cf32_ksum(const float* __restrict__ part, int S, int64_t slab,
                                                   float* __restrict__ out, const float* __restrict__ add) {
  const int64_t n4 = slab / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    float4 acc = add ? reinterpret_cast<const float4*>(add)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) {
      const float4 v = reinterpret_cast<const float4*>(part + s * slab)[i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
}

template <int PM, bool DG>
void launch_conv(const float* src, const uint16_t* w3, const ConvF32Geo& g, float* out, const float* add,
                 hipStream_t stream) {
  const int M = g.N * g.Ho * g.Wo;
  const dim3 grid((M + 64 * PM - 1) / (64 * PM), g.Co / 64);
  if (!DG && g.Cs % 32 != 0) {
    if (add) hipLaunchKernelGGL((k_cf32_conv<PM, false, true, true>), grid, dim3(256), 0, stream, src, w3, g, out, add);
    else hipLaunchKernelGGL((k_cf32_conv<PM, false, false, true>), grid, dim3(256), 0, stream, src, w3, g, out, add);
    return;
  }
  if (add) hipLaunchKernelGGL((k_cf32_conv<PM, DG, true, false>), grid, dim3(256), 0, stream, src, w3, g, out, add);
  else hipLaunchKernelGGL((k_cf32_conv<PM, DG, false, false>), grid, dim3(256), 0, stream, src, w3, g, out, add);
}

// ---------------------------------------------------------------------------------------------
// per-worker weight gradient

// transposed fragment read through the compiler builtin (the compiler tracks the returned registers,
// so a step's reads are all in flight before the first wait)
__device__ __forceinline__ s16x4 tr16(uint32_t lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      reinterpret_cast<__attribute__((address_space(3))) s16x4*>(static_cast<uintptr_t>(lds_addr)));
}

// LDS swizzle of the transposed-read tiles: 8-byte unit u of pixel row r is stored at u ^ 4 tr_swz(r),
// so the 32 (row, unit) pairs one half-wave's ds_read_b64_tr_b16 touches (rows {0..3, 8..11} + 16 j,
// four units) fall on distinct bank pairs (unswizzled: 4-way conflicts, 60 % of the LDS cycles)
__device__ __forceinline__ int tr_swz(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 1); }
constexpr int kTB = 32 * 128;          // one [32 pixel][64 channel] bf16 tile
constexpr int kSB = 2 * kNP * kTB;     // dy pieces 0..2 | x pieces 0..2

// GATHER (Cs % 64 != 0, e.g. the 3-channel CIFAR stem): k-blocks of 64 consecutive flattened
// (tap, channel) indices (K padded to a multiple of 64, the padding never stored), the x tile gathered
// one element at a time.
template <bool GATHER>
__global__ __launch_bounds__(256) void k_cf32_wgrad(const float* __restrict__ x, const float* __restrict__ dy,
                                                    ConvF32Geo g, int64_t rg, int64_t per_split, float* __restrict__ out,
                                                    int64_t split_stride, int64_t group_stride) {
  // g: the forward geometry (Hs/Ws/Cs = x's, Ho/Wo/Co = dy's)
  __shared__ __attribute__((aligned(16))) char lds[2 * kSB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = g.KH * g.KW * g.Cs;
  const int nkb = (K + 63) / 64;
  const int kb = blockIdx.x % nkb, cb = blockIdx.x / nkb;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int k0 = kb * 64, co0 = cb * 64;
  const int tap = k0 / g.Cs, c0 = k0 - tap * g.Cs;
  const int ti = tap / g.KW, tj = tap - ti * g.KW;
  const int64_t mbeg = static_cast<int64_t>(gi) * rg + static_cast<int64_t>(sp) * per_split;
  int64_t mend = mbeg + per_split;
  if (mend > static_cast<int64_t>(gi + 1) * rg) mend = static_cast<int64_t>(gi + 1) * rg;
  const int steps = mend > mbeg ? static_cast<int>((mend - mbeg + 31) / 32) : 0;
  const FastDiv fWo = make_fastdiv(g.Wo), fHo = make_fastdiv(g.Ho);

  // staging: thread t owns rows (t >> 4) and (t >> 4) + 16 of the step's 32 pixels, channels 4 (t & 15) .. +3
  const int srow = threadIdx.x >> 4, sch = threadIdx.x & 15;
  float4 rd[2], rx[2];
  auto load = [&](int s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t m = mbeg + static_cast<int64_t>(s) * 32 + srow + 16 * h;
      const bool mv = m < mend;
      const int64_t mm = mv ? m : 0;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 d = *reinterpret_cast<const float4*>(dy + mm * g.Co + co0 + sch * 4);
      rd[h] = mv ? d : z;
      uint32_t t, uwo, un, uho;   // m < 2^31 (checked by the host)
      fdivmod(static_cast<uint32_t>(mm), fWo, t, uwo);
      fdivmod(t, fHo, un, uho);
      const int wo = static_cast<int>(uwo), ho = static_cast<int>(uho);
      const int64_t n = un;
      if constexpr (GATHER) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = k0 + sch * 4 + e;
          const int tp = k / g.Cs, ch = k - tp * g.Cs;
          const int ki = tp / g.KW, kj = tp - ki * g.KW;
          const int hi = ho * g.sh - g.ph + ki * g.dh, wi = wo * g.sw - g.pw + kj * g.dw;
          const bool ok = mv && k < K && hi >= 0 && hi < g.Hs && wi >= 0 && wi < g.Ws;
          const float a = x[((n * g.Hs + (ok ? hi : 0)) * g.Ws + (ok ? wi : 0)) * g.Cs + (ok ? ch : 0)];
          v[e] = ok ? a : 0.f;
        }
        rx[h] = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const int hi = ho * g.sh - g.ph + ti * g.dh, wi = wo * g.sw - g.pw + tj * g.dw;
        const bool ok = mv && hi >= 0 && hi < g.Hs && wi >= 0 && wi < g.Ws;
        const float4 v = *reinterpret_cast<const float4*>(
            x + ((n * g.Hs + (ok ? hi : 0)) * g.Ws + (ok ? wi : 0)) * g.Cs + c0 + sch * 4);
        rx[h] = ok ? v : z;
      }
    }
  };
  auto stage = [&](int slot) {
    char* base = lds + slot * kSB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = srow + 16 * h;
      const int off = row * 128 + ((sch ^ (4 * tr_swz(row))) * 8);   // bank swizzle (see tr_swz)
      uint32_t p0[kNP], p1[kNP];
      split2(rd[h].x, rd[h].y, p0);
      split2(rd[h].z, rd[h].w, p1);
#pragma unroll
      for (int i = 0; i < kNP; ++i) *reinterpret_cast<uint2*>(base + i * kTB + off) = make_uint2(p0[i], p1[i]);
      split2(rx[h].x, rx[h].y, p0);
      split2(rx[h].z, rx[h].w, p1);
#pragma unroll
      for (int i = 0; i < kNP; ++i)
        *reinterpret_cast<uint2*>(base + (kNP + i) * kTB + off) = make_uint2(p0[i], p1[i]);
    }
  };

  const int cf0 = 2 * (wave >> 1), kf0 = 2 * (wave & 1);
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)lds));
  // fragment k of a tile: 8-byte unit 4 k + p of row 8 grp + q, stored at unit (4 k + p) ^ 4 tr_swz(row)
  const int trow = 8 * grp + q, tsw = tr_swz(trow);
  const uint32_t offA0 = trow * 128 + (4 * (cf0 ^ tsw) + p) * 8, offA1 = trow * 128 + (4 * ((cf0 + 1) ^ tsw) + p) * 8;
  const uint32_t offB0 = kNP * kTB + trow * 128 + (4 * (kf0 ^ tsw) + p) * 8;
  const uint32_t offB1 = kNP * kTB + trow * 128 + (4 * ((kf0 + 1) ^ tsw) + p) * 8;

  if (steps > 0) load(0);
  for (int s = 0; s < steps; ++s) {
    // slot s & 1 was last read in step s - 2, before every wave passed step s - 1's barrier
    stage(s & 1);
    if (s + 1 < steps) load(s + 1);
    __syncthreads();
    const uint32_t sb = lds0 + (s & 1) * kSB;
    // transposed fragments (see k_iwgrad in iconv_nhwc.hip) of one piece tile: two fragments u
    auto tr_read = [&](uint32_t a0, uint32_t a1, bf16x8 (&f)[2]) {   // fragments at a0, a1 (rows r, r + 4)
      const s16x4 r0 = tr16(a0), r1 = tr16(a0 + 512), r2 = tr16(a1), r3 = tr16(a1 + 512);
      f[0] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
      f[1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    bf16x8 ta[kNP][2], tb[kNP][2];
#pragma unroll
    for (int i = 0; i < kNP; ++i) {
      tr_read(sb + i * kTB + offA0, sb + i * kTB + offA1, ta[i]);
      tr_read(sb + i * kTB + offB0, sb + i * kTB + offB1, tb[i]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const bf16x8 av[kNP] = {ta[0][u], ta[1][u], ta[2][u]};
        const bf16x8 bv[kNP] = {tb[0][v], tb[1][v], tb[2][v]};
        acc[u][v] = mma6(av, bv, acc[u][v]);
      }
  }

  // D[co = 4*grp + e][k = li] of each (u, v) fragment
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + (cf0 + u) * 16 + 4 * grp + e;
        const int k = k0 + (kf0 + v) * 16 + li;
        const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                          static_cast<int64_t>(co) * K + k;
        if (!GATHER || k < K) out[o] = acc[u][v][e];
      }
}

// The 128 co x 128 k form (Cs % 128 == 0, Co % 128 == 0): each wave computes 4 x 4 fragments (64 co x
// 64 k) instead of 2 x 2, halving the LDS fragment bytes per MFMA (the 64 x 64 form reads 512 B of
// LDS per MFMA and is LDS-bound). Each operand's [32 pixel][128 channel] step tile is kept as two
// [32][64] sub-tiles (128-byte pitch: the bank pattern of the 64 x 64 form).
constexpr int kTB2 = 2 * kTB;              // one operand piece: two [32][64] sub-tiles
constexpr int kSB2 = 2 * kNP * kTB2;       // dy pieces 0..2 | x pieces 0..2

// NB = 2: double-buffered tiles (96 KB, one workgroup per CU, one barrier per step); NB = 1: one tile
// (48 KB, two workgroups per CU hide each other's staging and barriers; two barriers per step)
template <int NB>
__global__ __launch_bounds__(256, NB == 1 ? 2 : 1) void k_cf32_wgrad2(const float* __restrict__ x, const float* __restrict__ dy,
                                                     ConvF32Geo g, int64_t rg, int64_t per_split,
                                                     float* __restrict__ out, int64_t split_stride,
                                                     int64_t group_stride) {
  extern __shared__ __attribute__((aligned(16))) char dlds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = g.KH * g.KW * g.Cs;
  const int nkb = K / 128;
  const int kb = blockIdx.x % nkb, cb = blockIdx.x / nkb;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int k0 = kb * 128, co0 = cb * 128;
  const int tap = k0 / g.Cs, c0 = k0 - tap * g.Cs;
  const int ti = tap / g.KW, tj = tap - ti * g.KW;
  const int64_t mbeg = static_cast<int64_t>(gi) * rg + static_cast<int64_t>(sp) * per_split;
  int64_t mend = mbeg + per_split;
  if (mend > static_cast<int64_t>(gi + 1) * rg) mend = static_cast<int64_t>(gi + 1) * rg;
  const int steps = mend > mbeg ? static_cast<int>((mend - mbeg + 31) / 32) : 0;
  const FastDiv fWo = make_fastdiv(g.Wo), fHo = make_fastdiv(g.Ho);

  // staging: thread t owns rows (t >> 4) and (t >> 4) + 16, channels 4 (t & 15) .. +3 of both sub-tiles
  const int srow = threadIdx.x >> 4, sch = threadIdx.x & 15;
  float4 rd[2][2], rx[2][2];   // [row half][sub-tile]
  auto load = [&](int s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t m = mbeg + static_cast<int64_t>(s) * 32 + srow + 16 * h;
      const bool mv = m < mend;
      const int64_t mm = mv ? m : 0;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      uint32_t t, uwo, un, uho;   // m < 2^31 (checked by the host)
      fdivmod(static_cast<uint32_t>(mm), fWo, t, uwo);
      fdivmod(t, fHo, un, uho);
      const int wo = static_cast<int>(uwo), ho = static_cast<int>(uho);
      const int64_t n = un;
      const int hi = ho * g.sh - g.ph + ti * g.dh, wi = wo * g.sw - g.pw + tj * g.dw;
      const bool ok = mv && hi >= 0 && hi < g.Hs && wi >= 0 && wi < g.Ws;
      const float* xp = x + ((n * g.Hs + (ok ? hi : 0)) * g.Ws + (ok ? wi : 0)) * g.Cs + c0 + sch * 4;
      const float* dp = dy + mm * g.Co + co0 + sch * 4;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float4 d = *reinterpret_cast<const float4*>(dp + 64 * b);
        const float4 v = *reinterpret_cast<const float4*>(xp + 64 * b);
        rd[h][b] = mv ? d : z;
        rx[h][b] = ok ? v : z;
      }
    }
  };
  auto stage = [&](int slot) {
    char* base = dlds + slot * kSB2;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int row = srow + 16 * h;
        const int off = b * kTB + row * 128 + ((sch ^ (4 * tr_swz(row))) * 8);
        uint32_t p0[kNP], p1[kNP];
        split2(rd[h][b].x, rd[h][b].y, p0);
        split2(rd[h][b].z, rd[h][b].w, p1);
#pragma unroll
        for (int i = 0; i < kNP; ++i) *reinterpret_cast<uint2*>(base + i * kTB2 + off) = make_uint2(p0[i], p1[i]);
        split2(rx[h][b].x, rx[h][b].y, p0);
        split2(rx[h][b].z, rx[h][b].w, p1);
#pragma unroll
        for (int i = 0; i < kNP; ++i)
          *reinterpret_cast<uint2*>(base + (kNP + i) * kTB2 + off) = make_uint2(p0[i], p1[i]);
      }
  };

  // wave (a, b): co sub-tile a = wave >> 1 (fragments 4a .. 4a + 3), k sub-tile b = wave & 1
  const int sa = wave >> 1, sbk = wave & 1;
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr)dlds));
  // fragment k (columns 16 k .. 16 k + 15) of a sub-tile: 8-byte unit 4 k + p of row 8 grp + q, stored
  // at unit (4 k + p) ^ 4 tr_swz(row) (rows + 4 share the swizzle)
  const int trow = 8 * grp + q, tsw = tr_swz(trow);
  uint32_t offA[4], offB[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    offA[k] = sa * kTB + trow * 128 + ((4 * (k ^ tsw) + p) * 8);
    offB[k] = kNP * kTB2 + sbk * kTB + trow * 128 + ((4 * (k ^ tsw) + p) * 8);
  }

  if (steps > 0) load(0);
  for (int s = 0; s < steps; ++s) {
    if (NB == 1 && s > 0) __syncthreads();   // every wave has read step s - 1's tile
    stage(NB == 1 ? 0 : (s & 1));
    if (s + 1 < steps) load(s + 1);
    __syncthreads();
    const uint32_t sb = lds0 + (NB == 1 ? 0 : (s & 1)) * kSB2;
    // fragments at a0, a1 (rows r and r + 4 each): the compiler builtin, so the 24 reads of a step are
    // in flight together (no LDS-DMA runs in this kernel: the waits it places cost nothing)
    auto tr_read = [&](uint32_t a0, uint32_t a1, bf16x8 (&f)[2]) {
      const s16x4 r0 = tr16(a0), r1 = tr16(a0 + 512), r2 = tr16(a1), r3 = tr16(a1 + 512);
      f[0] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
      f[1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    bf16x8 ta[kNP][4], tb[kNP][4];
#pragma unroll
    for (int i = 0; i < kNP; ++i) {
      const uint32_t pb = sb + i * kTB2;
      bf16x8 t0[2], t1[2];
      tr_read(pb + offA[0], pb + offA[1], t0);
      tr_read(pb + offA[2], pb + offA[3], t1);
      ta[i][0] = t0[0]; ta[i][1] = t0[1]; ta[i][2] = t1[0]; ta[i][3] = t1[1];
      tr_read(pb + offB[0], pb + offB[1], t0);
      tr_read(pb + offB[2], pb + offB[3], t1);
      tb[i][0] = t0[0]; tb[i][1] = t0[1]; tb[i][2] = t1[0]; tb[i][3] = t1[1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const bf16x8 av[kNP] = {ta[0][u], ta[1][u], ta[2][u]};
        const bf16x8 bv[kNP] = {tb[0][v], tb[1][v], tb[2][v]};
        acc[u][v] = mma6(av, bv, acc[u][v]);
      }
  }

#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + (4 * sa + u) * 16 + 4 * grp + e;
        const int k = k0 + (4 * sbk + v) * 16 + li;
        const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                          static_cast<int64_t>(co) * K + k;
        out[o] = acc[u][v][e];
      }
}

// ---------------------------------------------------------------------------------------------
// weight split (once per step): W [R][T][C] fp32 -> W_hi, W_lo [R][T][C] and Wt_hi, Wt_lo [C][T][R]
// bf16, 64 x 64 tiles of one tap through LDS (padded pitch)

constexpr int kWJobs = 64;
struct WJob {
  const float* w;
  uint16_t* pieces;    // [3][R][ld]
  uint16_t* tpieces;   // nullable: [3][C][T][R] (no transposed copy)
  int R, T, C;
  int ld;              // row pitch of the pieces (elements)
  int tile0;
};
struct WTable {
  WJob j[kWJobs];
  int n;
};

__global__ __launch_bounds__(256) void k_wsplit(WTable t) {
  __shared__ uint16_t tp[kNP][64][66];   // the tile's pieces, [c][r] order
  int ji = 0;
  while (ji + 1 < t.n && static_cast<int>(blockIdx.x) >= t.j[ji + 1].tile0) ++ji;
  const WJob jb = t.j[ji];
  const int tr = (jb.R + 63) / 64, tc = (jb.C + 63) / 64;
  const int l = blockIdx.x - jb.tile0;
  const int tap = l / (tr * tc);
  const int rem = l - tap * tr * tc;
  const int r0 = (rem / tc) * 64, c0 = (rem % tc) * 64;
  const int lc = threadIdx.x & 63, lr = threadIdx.x >> 6;
  for (int rr = lr; rr < 64; rr += 4) {
    const int r = r0 + rr, c = c0 + lc;
    uint16_t pc[kNP] = {};
    if (r < jb.R && c < jb.C) {
      const int64_t o = (static_cast<int64_t>(r) * jb.T + tap) * jb.C + c;
      const int64_t od = static_cast<int64_t>(r) * jb.ld + tap * jb.C + c;
      const int64_t stride = static_cast<int64_t>(jb.R) * jb.ld;
      float v = jb.w[o];
#pragma unroll
      for (int i = 0; i < kNP; ++i) {
        pc[i] = f_to_bf16(v);
        v -= bf16_to_f(pc[i]);
        jb.pieces[i * stride + od] = pc[i];
      }
    }
#pragma unroll
    for (int i = 0; i < kNP; ++i) tp[i][lc][rr] = pc[i];
  }
  if (jb.tpieces == nullptr) return;
  __syncthreads();
  const int64_t tstride = static_cast<int64_t>(jb.R) * jb.T * jb.C;
  for (int cc = lr; cc < 64; cc += 4) {
    const int c = c0 + cc, r = r0 + lc;
    if (c < jb.C && r < jb.R) {
      const int64_t o = (static_cast<int64_t>(c) * jb.T + tap) * jb.R + r;
#pragma unroll
      for (int i = 0; i < kNP; ++i) jb.tpieces[i * tstride + o] = tp[i][cc][lc];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// classifier (fp32 or bf16 operands, fp32 accumulation, one rounding) and global average pool
// (fp32), VALU: the classifier is ~0.1 GFLOP per step, far below a GEMM tile's worth of work

// element loads / stores of the classifier's operand type (float, or bf16 as uint16_t)
__device__ __forceinline__ float lin_ld(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float lin_ld(const uint16_t* p, int64_t i) { return bf16_to_f(p[i]); }
__device__ __forceinline__ void lin_st(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void lin_st(uint16_t* p, int64_t i, float v) { p[i] = f_to_bf16(v); }

// logits[r][o] = Σ_f x[r][f] w[o][f] + b[o]: one wave per row, O <= 64 outputs kept in registers
constexpr int kLinMaxO = 16;
// y[row][o]: one wave per row, the lanes over f, 8 f-columns per lane in flight (x and w loads issue
// back to back instead of one dependent round trip per column)
template <typename T>
__global__ __launch_bounds__(256) void k_linear_fwd(const T* __restrict__ x, const T* __restrict__ w,
                                                    const T* __restrict__ b, int R, int F, int O, T* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + static_cast<int64_t>(row) * F;
  for (int o0 = 0; o0 < O; o0 += kLinMaxO) {
    float acc[kLinMaxO];
#pragma unroll
    for (int o = 0; o < kLinMaxO; ++o) acc[o] = 0.f;
    for (int f0 = 0; f0 < F; f0 += 512) {
      float xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int f = f0 + u * 64 + lane;
        xv[u] = f < F ? lin_ld(xr, f) : 0.f;
      }
#pragma unroll
      for (int o = 0; o < kLinMaxO; ++o) {
        if (o0 + o < O) {
          const T* wr = w + static_cast<int64_t>(o0 + o) * F;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int f = f0 + u * 64 + lane;
            acc[o] = fmaf(xv[u], f < F ? lin_ld(wr, f) : 0.f, acc[o]);
          }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < kLinMaxO; ++o) {
      float v = acc[o];
#pragma unroll
      for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
      if (lane == 0 && o0 + o < O) lin_st(y, static_cast<int64_t>(row) * O + o0 + o, v + (b ? lin_ld(b, o0 + o) : 0.f));
    }
  }
}
template <typename T>
__global__ __launch_bounds__(256) void k_linear_dgrad(const T* __restrict__ dl, const T* __restrict__ w, int R, int F,
                                                      int O, T* __restrict__ dx) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= static_cast<int64_t>(R) * F) return;
  const int64_t r = t / F;
  const int f = static_cast<int>(t - r * F);
  float a = 0.f;
  for (int o = 0; o < O; ++o) a = fmaf(lin_ld(dl, r * O + o), lin_ld(w, static_cast<int64_t>(o) * F + f), a);
  lin_st(dx, t, a);
}
// per-worker dW_g[o][f] = Σ_{r in g} dl[r][o] x[r][f] and db_g[o] = Σ_{r in g} dl[r][o], written straight
// into worker g's exchange row (element type ODT: fp32 / bf16 / fp16)
template <typename T>
__global__ __launch_bounds__(256) void k_linear_wgrad(const T* __restrict__ x, const T* __restrict__ dl, int rg, int F,
                                                      int O, void* __restrict__ out, int odt, int64_t row_stride,
                                                      int64_t off_w, int64_t off_b) {
  __shared__ float red[3][kLinMaxO][64];
  const int g = blockIdx.y;
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + lane;
  const T* xg = x + static_cast<int64_t>(g) * rg * F;
  const T* dg = dl + static_cast<int64_t>(g) * rg * O;
  const int64_t og = static_cast<int64_t>(g) * row_stride;
  for (int o0 = 0; o0 < O; o0 += kLinMaxO) {
    float acc[kLinMaxO];
#pragma unroll
    for (int o = 0; o < kLinMaxO; ++o) acc[o] = 0.f;
    if (f < F) {
#pragma unroll 4
      for (int r = q; r < rg; r += 4) {
        const float xv = lin_ld(xg, static_cast<int64_t>(r) * F + f);
#pragma unroll
        for (int o = 0; o < kLinMaxO; ++o)
          if (o0 + o < O) acc[o] = fmaf(lin_ld(dg, static_cast<int64_t>(r) * O + o0 + o), xv, acc[o]);
      }
    }
    if (q > 0) {
#pragma unroll
      for (int o = 0; o < kLinMaxO; ++o) red[q - 1][o][lane] = acc[o];
    }
    __syncthreads();
    if (q == 0 && f < F) {
#pragma unroll
      for (int o = 0; o < kLinMaxO; ++o)
        if (o0 + o < O)
          store_one(out, odt, og + off_w + static_cast<int64_t>(o0 + o) * F + f,
                    ((acc[o] + red[0][o][lane]) + red[1][o][lane]) + red[2][o][lane]);
    }
    __syncthreads();
  }
  if (off_b >= 0 && blockIdx.x == 0 && threadIdx.x < O) {
    float s = 0.f;
    for (int r = 0; r < rg; ++r) s += lin_ld(dg, static_cast<int64_t>(r) * O + threadIdx.x);
    store_one(out, odt, og + off_b + threadIdx.x, s);
  }
}
// db_g[o] for a wide head (the ImageNet classifier's 1000 outputs): one thread per output, the rows of
// the worker read coalesced across the threads
template <typename T>
__global__ __launch_bounds__(256) void k_linear_bias_grad(const T* __restrict__ dl, int rg, int O, void* __restrict__ out,
                                                          int odt, int64_t row_stride, int64_t off_b) {
  const int g = blockIdx.y;
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= O) return;
  const T* dg = dl + static_cast<int64_t>(g) * rg * O;
  float s = 0.f;
  for (int r = 0; r < rg; ++r) s += lin_ld(dg, static_cast<int64_t>(r) * O + o);
  store_one(out, odt, static_cast<int64_t>(g) * row_stride + off_b + o, s);
}
// ---- bf16 classifier with 16-byte operand loads (F % 8 == 0, O <= kLinV) ------------------------
// The step's classifier is [2000 x 2048] x [2048 x 10]: ~0.1 GFLOP and 8 MB of activations, so it is
// an HBM stream, not a GEMM: each lane holds 8 consecutive features of a row (one 16-byte load), the
// weight rows are staged in LDS once per workgroup, and the O dot products are reduced across the wave.
constexpr int kLinV = 16;        // outputs per launch pass (O <= kLinV)
constexpr int kLinRows = 8;      // rows per workgroup (2 per wave)

__device__ __forceinline__ void unpack_bf16x8(const uint4 u, float (&v)[8]) {
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}

// y[r][o] = Σ_f x[r][f] w[o][f] + b[o]; LDS: w [O][F] bf16 (<= 16 x 4096 x 2 = 128 KB). Each wave's two
// rows are loaded (4 x 16 B per lane and row per 2048 features) before the weight staging barrier, so the
// HBM latency of x overlaps the weight's L2 reads.
__global__ __launch_bounds__(256) void k_linear_fwd_v(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                      const uint16_t* __restrict__ b, int R, int F, int O,
                                                      uint16_t* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) uint16_t wl[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fv = F / 8;
  const int r0 = blockIdx.x * kLinRows + wave * 2;
  float acc[2][kLinV];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int o = 0; o < kLinV; ++o) acc[i][o] = 0.f;
  for (int c0 = 0; c0 < fv; c0 += 256) {
    uint4 xr[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + u * 64 + lane;
        xr[i][u] = (r0 + i < R && c < fv) ? reinterpret_cast<const uint4*>(x + static_cast<int64_t>(r0 + i) * F)[c]
                                          : make_uint4(0u, 0u, 0u, 0u);
      }
    if (c0 == 0) {   // uniform over the workgroup
      const int nv = O * fv;
      for (int e = threadIdx.x; e < nv; e += 256)
        reinterpret_cast<uint4*>(wl)[e] = reinterpret_cast<const uint4*>(w)[e];
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * 64 + lane;
      if (c >= fv) break;
      float xv[2][8];
      unpack_bf16x8(xr[0][u], xv[0]);
      unpack_bf16x8(xr[1][u], xv[1]);
#pragma unroll
      for (int o = 0; o < kLinV; ++o) {
        if (o < O) {
          float wv[8];
          unpack_bf16x8(reinterpret_cast<const uint4*>(wl + o * F)[c], wv);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            acc[0][o] = fmaf(xv[0][k], wv[k], acc[0][o]);
            acc[1][o] = fmaf(xv[1][k], wv[k], acc[1][o]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int o = 0; o < kLinV; ++o) {
      if (o < O) {
        float v = acc[i][o];
#pragma unroll
        for (int s2 = 32; s2 >= 1; s2 >>= 1) v += __shfl_xor(v, s2);
        if (lane == o && r0 + i < R) y[static_cast<int64_t>(r0 + i) * O + o] = f_to_bf16(v + (b ? bf16_to_f(b[o]) : 0.f));
      }
    }
}

// dx[r][f .. f + 8] = Σ_o dl[r][o] w[o][f .. f + 8]: one 16-byte output per thread
__global__ __launch_bounds__(256) void k_linear_dgrad_v(const uint16_t* __restrict__ dl, const uint16_t* __restrict__ w,
                                                        int R, int F, int O, uint16_t* __restrict__ dx) {
  const int fv = F / 8;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= static_cast<int64_t>(R) * fv) return;
  const int64_t r = t / fv;
  const int c = static_cast<int>(t - r * fv);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int o = 0; o < O; ++o) {
    const float d = bf16_to_f(dl[r * O + o]);
    float wv[8];
    unpack_bf16x8(reinterpret_cast<const uint4*>(w + static_cast<int64_t>(o) * F)[c], wv);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fmaf(d, wv[k], a[k]);
  }
  reinterpret_cast<uint4*>(dx)[t] = make_uint4(pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]),
                                               pack_bf16x2(a[4], a[5]), pack_bf16x2(a[6], a[7]));
}

// per-worker dW_g[o][f] = Σ_{r in g} dl[r][o] x[r][f], db_g[o] = Σ_{r in g} dl[r][o] into worker g's exchange
// row. Workgroup (64 features, worker g): lane = feature chunk (8 x 8 features) + 8 x row lane (8 per wave, 32
// in all), four rows' loads in flight per lane; dl of the worker staged in LDS as fp32; the row lanes
// reduced by shuffles inside the wave, then across the 4 waves through LDS.
constexpr int kWgF = 64;
__global__ __launch_bounds__(256) void k_linear_wgrad_v(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dl,
                                                        int rg, int F, int O, void* __restrict__ out, int odt,
                                                        int64_t row_stride, int64_t off_w, int64_t off_b) {
  extern __shared__ __attribute__((aligned(16))) float dls[];   // [rg][O] then [4][kLinV][8][8] partials
  const int g = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ch = lane & 7, rl = wave * 8 + (lane >> 3);          // feature chunk, row lane (0..31)
  const int f0 = blockIdx.x * kWgF + ch * 8;
  const uint16_t* dg = dl + static_cast<int64_t>(g) * rg * O;
  const uint16_t* xg = x + static_cast<int64_t>(g) * rg * F + f0;
  const bool fok = f0 < F;
  uint4 xr[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {   // the first four rows' loads before the staging barrier
    const int r = rl + 32 * u;
    xr[u] = (fok && r < rg) ? *reinterpret_cast<const uint4*>(xg + static_cast<int64_t>(r) * F) : make_uint4(0u, 0u, 0u, 0u);
  }
  for (int e = threadIdx.x; e < rg * O; e += 256) dls[e] = bf16_to_f(dg[e]);
  __syncthreads();
  float acc[kLinV][8];
#pragma unroll
  for (int o = 0; o < kLinV; ++o)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[o][k] = 0.f;
  for (int r0 = 0; r0 < rg; r0 += 128) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + rl + 32 * u;
      if (r < rg) {
        float xv[8];
        unpack_bf16x8(xr[u], xv);
#pragma unroll
        for (int o = 0; o < kLinV; ++o) {
          if (o < O) {
            const float d = dls[r * O + o];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[o][k] = fmaf(d, xv[k], acc[o][k]);
          }
        }
      }
    }
    if (r0 + 128 < rg) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + 128 + rl + 32 * u;
        xr[u] = (fok && r < rg) ? *reinterpret_cast<const uint4*>(xg + static_cast<int64_t>(r) * F)
                                : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  float* red = dls + rg * O;
#pragma unroll
  for (int o = 0; o < kLinV; ++o)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = acc[o][k];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      acc[o][k] = v;
    }
  if ((lane >> 3) == 0) {
#pragma unroll
    for (int o = 0; o < kLinV; ++o)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[((wave * kLinV + o) * 8 + ch) * 8 + k] = acc[o][k];
  }
  __syncthreads();
  const int64_t og = static_cast<int64_t>(g) * row_stride;
  for (int e = threadIdx.x; e < O * kWgF; e += 256) {
    const int o = e / kWgF, q = e - o * kWgF, c2 = q / 8, k = q - c2 * 8;
    const int f = blockIdx.x * kWgF + q;
    if (f < F) {
      float v = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) v += red[((w2 * kLinV + o) * 8 + c2) * 8 + k];
      store_one(out, odt, og + off_w + static_cast<int64_t>(o) * F + f, v);
    }
  }
  if (off_b >= 0 && blockIdx.x == 0 && threadIdx.x < O) {
    float sb = 0.f;
    for (int r = 0; r < rg; ++r) sb += dls[r * O + threadIdx.x];
    store_one(out, odt, og + off_b + threadIdx.x, sb);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_avgpool_fwd(const T* __restrict__ x, int N, int HW, int C, T* __restrict__ y) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= static_cast<int64_t>(N) * C) return;
  const int64_t n = t / C;
  const int c = static_cast<int>(t - n * C);
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += lin_ld(x, (n * HW + p) * C + c);
  lin_st(y, t, s / static_cast<float>(HW));
}
template <typename T>
__global__ __launch_bounds__(256) void k_avgpool_bwd(const T* __restrict__ dy, int N, int HW, int C, T* __restrict__ dx) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= static_cast<int64_t>(N) * HW * C) return;
  const int c = static_cast<int>(t % C);
  const int64_t n = t / (static_cast<int64_t>(HW) * C);
  lin_st(dx, t, lin_ld(dy, n * C + c) / static_cast<float>(HW));
}

unsigned blocks_for(int64_t items) { return static_cast<unsigned>((items + 255) / 256); }

}  // namespace

bool conv_f32_supported(const ConvF32Geo& g) { return g.Co % 64 == 0 && g.Cs > 0 && g.Co > 0; }

// the LDS-staged kernel's preconditions: 32-channel k-steps, a tap mask of <= 32 bits, 32-bit element
// offsets into the source, unit dilation for the transposed (data-gradient) form
bool conv_f32_lds_ok(const ConvF32Geo& g, bool dgrad) {
  return g.Cs % 32 == 0 && g.KH * g.KW <= 32 && (!dgrad || (g.dh == 1 && g.dw == 1)) &&
         static_cast<int64_t>(g.N) * g.Hs * g.Ws * g.Cs < (int64_t{1} << 31);
}

int conv_f32_ksplit(const ConvF32Geo& g, bool dgrad) {
  // below 400 PM = 2 tiles (two workgroups per CU: ~512 slots), split-K up to 400+ workgroups, each split
  // at least 8 k-steps; the slabs cost 2 x S x M x Co x 4 bytes of traffic. Measured on the ResNet-50
  // CIFAR shapes (scripts/bench_conv_f32.py, profiles/r4): e.g. 512 ch 3x3 at 1x1 px 0.32 -> 0.08 ms
  // with S = 4; 500 tiles and more run best unsplit.
  const int csh = dgrad ? g.sh : 1, csw = dgrad ? g.sw : 1;
  const int64_t Mc = static_cast<int64_t>(g.N) * ((g.Ho + csh - 1) / csh) * ((g.Wo + csw - 1) / csw);
  const int64_t tiles = ((Mc + 127) / 128) * (g.Co / 64) * csh * csw;   // PM = 2 tiles
  const int taps = dgrad ? ((g.KH + csh - 1) / csh) * ((g.KW + csw - 1) / csw) : g.KH * g.KW;
  const int steps = taps * (g.Cs / 32);
  int S = 1;
  while (S < 8 && tiles * S < 400 && steps / (2 * S) >= 8) S *= 2;
  return S;
}

void conv_f32(const float* src, const uint16_t* w3, const ConvF32Geo& g, bool dgrad, float* out, const float* add,
              int pm, hipStream_t stream, int ksplit, float* part) {
  if (static_cast<int64_t>(g.N) * g.Ho * g.Wo <= 0) return;
  if (ksplit > 1 && part != nullptr && conv_f32_lds_ok(g, dgrad)) {
    // PM = 4 tiles, split-K into the slabs of `part`, then one summing pass (+ add)
    if (pm <= 0 || pm == 13) {
      if (dgrad) launch_conv_lds<2, 2, true>(src, w3, g, part, nullptr, ksplit, stream);
      else launch_conv_lds<2, 2, false>(src, w3, g, part, nullptr, ksplit, stream);
    } else if (pm == 15) {
      if (dgrad) launch_conv_lds<4, 3, true>(src, w3, g, part, nullptr, ksplit, stream);
      else launch_conv_lds<4, 3, false>(src, w3, g, part, nullptr, ksplit, stream);
    } else {
      if (dgrad) launch_conv_lds<4, 2, true>(src, w3, g, part, nullptr, ksplit, stream);
      else launch_conv_lds<4, 2, false>(src, w3, g, part, nullptr, ksplit, stream);
    }
    const int64_t slab = static_cast<int64_t>(g.N) * g.Ho * g.Wo * g.Co;
    int64_t blocks = (slab / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_cf32_ksum, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, part, ksplit, slab, out,
                       add);
    return;
  }
  // automatic: PM = 2 with a 2-deep ring (57 KB of LDS: two workgroups per CU hide each other's barriers
  // and load waits) -- 10-25 % under PM = 4 / one workgroup per CU on the larger ResNet-50 layers
  // (profiles/r4/bench_conv_f32.log); the few-tile layers take it with split-K (conv_f32_ksplit)
  if (pm <= 0) pm = 13;
  if (pm > 10 && conv_f32_lds_ok(g, dgrad)) {   // the LDS-staged kernel
    if (dgrad) {
      if (pm == 15) launch_conv_lds<4, 3, true>(src, w3, g, out, add, 1, stream);
      else if (pm >= 14) launch_conv_lds<4, 2, true>(src, w3, g, out, add, 1, stream);
      else if (pm == 12) launch_conv_lds<2, 3, true>(src, w3, g, out, add, 1, stream);
      else if (pm == 13) launch_conv_lds<2, 2, true>(src, w3, g, out, add, 1, stream);
      else launch_conv_lds<1, 3, true>(src, w3, g, out, add, 1, stream);
    } else {
      if (pm == 15) launch_conv_lds<4, 3, false>(src, w3, g, out, add, 1, stream);
      else if (pm >= 14) launch_conv_lds<4, 2, false>(src, w3, g, out, add, 1, stream);
      else if (pm == 12) launch_conv_lds<2, 3, false>(src, w3, g, out, add, 1, stream);
      else if (pm == 13) launch_conv_lds<2, 2, false>(src, w3, g, out, add, 1, stream);
      else launch_conv_lds<1, 3, false>(src, w3, g, out, add, 1, stream);
    }
    return;
  }
  if (pm > 10) pm -= 10;
  if (dgrad) {
    if (pm >= 4) launch_conv<4, true>(src, w3, g, out, add, stream);
    else if (pm == 2) launch_conv<2, true>(src, w3, g, out, add, stream);
    else launch_conv<1, true>(src, w3, g, out, add, stream);
  } else {
    if (pm >= 4) launch_conv<4, false>(src, w3, g, out, add, stream);
    else if (pm == 2) launch_conv<2, false>(src, w3, g, out, add, stream);
    else launch_conv<1, false>(src, w3, g, out, add, stream);
  }
}

bool wgrad_f32_supported(const ConvF32Geo& g) { return g.Cs > 0 && g.Co % 64 == 0; }
bool wgrad_f32_wide(const ConvF32Geo& g) { return g.Cs % 128 == 0 && g.Co % 128 == 0; }

void wgrad_f32(const float* x, const float* dy, const ConvF32Geo& g, int groups, int64_t rg, int splits, float* out,
               int64_t split_stride, int64_t group_stride, hipStream_t stream, int variant) {
  const int K = g.KH * g.KW * g.Cs;
  if (splits < 1) splits = 1;
  const int64_t per_split = (rg + splits - 1) / splits;
  // automatic: the single-buffered 128 x 128 form (two workgroups per CU) wherever it applies -- 25-30 %
  // under the double-buffered one on every ResNet-50 CIFAR shape (profiles/r4/bench_conv_f32.log)
  if (variant == 0) variant = wgrad_f32_wide(g) ? 2 : 3;
  if (variant == 1 || variant == 2) {
    static bool once = (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cf32_wgrad2<2>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kSB2),
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cf32_wgrad2<1>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, kSB2),
                        true);
    (void)once;
    const dim3 grid2((K / 128) * (g.Co / 128), groups, splits);
    if (variant == 1)
      hipLaunchKernelGGL(k_cf32_wgrad2<2>, grid2, dim3(256), 2 * kSB2, stream, x, dy, g, rg, per_split, out,
                         split_stride, group_stride);
    else
      hipLaunchKernelGGL(k_cf32_wgrad2<1>, grid2, dim3(256), kSB2, stream, x, dy, g, rg, per_split, out,
                         split_stride, group_stride);
    return;
  }
  const dim3 grid(((K + 63) / 64) * (g.Co / 64), groups, splits);
  if (g.Cs % 64 != 0)
    hipLaunchKernelGGL(k_cf32_wgrad<true>, grid, dim3(256), 0, stream, x, dy, g, rg, per_split, out, split_stride,
                       group_stride);
  else
    hipLaunchKernelGGL(k_cf32_wgrad<false>, grid, dim3(256), 0, stream, x, dy, g, rg, per_split, out, split_stride,
                       group_stride);
}

void wsplit_multi(const WSplitJob* jobs, int count, hipStream_t stream) {
  for (int b = 0; b < count; b += kWJobs) {
    WTable t{};
    int tiles = 0;
    t.n = count - b < kWJobs ? count - b : kWJobs;
    for (int i = 0; i < t.n; ++i) {
      const WSplitJob& s = jobs[b + i];
      t.j[i] = WJob{s.w, s.pieces, s.tpieces, s.R, s.T, s.C, s.ld > 0 ? s.ld : s.T * s.C, tiles};
      tiles += s.T * ((s.R + 63) / 64) * ((s.C + 63) / 64);
    }
    if (tiles > 0) hipLaunchKernelGGL(k_wsplit, dim3(tiles), dim3(256), 0, stream, t);
  }
}

namespace {
// Wide bf16 classifier heads (O > kLinV outputs, e.g. ImageNet's 1000 classes) are GEMMs: they run on
// gemm_nt.hip (and the 1x1 weight-gradient kernel) with the output dimension padded to Op, a multiple
// of 64. Once per step one launch writes wp [Op][F] (rows >= O zero: the forward's B operand) and
// wpt [F][Op] (columns >= O zero: the data gradient's B operand) from w [O][F], through a 64 x 64 LDS
// tile (row pitch 72: the column reads of the transpose spread over the banks).
constexpr int kHT = 64;

__device__ __forceinline__ uint4 pack8_u16(const uint16_t (&e)[8]) {
  return make_uint4(e[0] | (static_cast<uint32_t>(e[1]) << 16), e[2] | (static_cast<uint32_t>(e[3]) << 16),
                    e[4] | (static_cast<uint32_t>(e[5]) << 16), e[6] | (static_cast<uint32_t>(e[7]) << 16));
}

__global__ __launch_bounds__(256) void k_head_weights(const uint16_t* __restrict__ w, int O, int F, int Op,
                                                      uint16_t* __restrict__ wp, uint16_t* __restrict__ wpt) {
  __shared__ __attribute__((aligned(16))) uint16_t t[kHT][kHT + 8];
  const int f0 = blockIdx.x * kHT, o0 = blockIdx.y * kHT;
  for (int i = threadIdx.x; i < kHT * 8; i += 256) {
    const int r = i / 8, cv = (i % 8) * 8;
    const int o = o0 + r;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (o < O) v = *reinterpret_cast<const uint4*>(w + static_cast<int64_t>(o) * F + f0 + cv);
    *reinterpret_cast<uint4*>(wp + static_cast<int64_t>(o) * F + f0 + cv) = v;
    *reinterpret_cast<uint4*>(&t[r][cv]) = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHT * 8; i += 256) {
    const int fr = i / 8, ov = (i % 8) * 8;
    uint16_t e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = t[ov + k][fr];
    *reinterpret_cast<uint4*>(wpt + static_cast<int64_t>(f0 + fr) * Op + o0 + ov) = pack8_u16(e);
  }
}

// bf16 rows re-pitched: dst[r][c] = src[r][c] (+ bias[c], added in fp32, one rounding) for c < min(a, b),
// 0 for a <= c < b (the padded head's logits cropped, its logit gradient padded)
__global__ __launch_bounds__(256) void k_repitch(const uint16_t* __restrict__ src, int a, uint16_t* __restrict__ dst,
                                                 int b, int64_t R, const uint16_t* __restrict__ bias) {
  const int nv = b / 8, ncp = a < b ? a : b;
  const int64_t items = R * nv;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < items;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = i / nv;
    const int c = static_cast<int>(i - r * nv) * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (c < ncp) {
      v = *reinterpret_cast<const uint4*>(src + r * a + c);
      if (bias) {
        const uint4 bv = *reinterpret_cast<const uint4*>(bias + c);
        const uint32_t xs[4] = {v.x, v.y, v.z, v.w}, bs[4] = {bv.x, bv.y, bv.z, bv.w};
        uint16_t e[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          e[2 * k] = f_to_bf16(__uint_as_float(xs[k] << 16) + __uint_as_float(bs[k] << 16));
          e[2 * k + 1] = f_to_bf16(__uint_as_float(xs[k] & 0xffff0000u) + __uint_as_float(bs[k] & 0xffff0000u));
        }
        v = pack8_u16(e);
      }
    }
    *reinterpret_cast<uint4*>(dst + r * b + c) = v;
  }
}
}  // namespace

void head_weights_bf16(const uint16_t* w, int O, int F, int Op, uint16_t* wp, uint16_t* wpt, hipStream_t stream) {
  if (O <= 0 || F <= 0) return;
  hipLaunchKernelGGL(k_head_weights, dim3(F / kHT, Op / kHT), dim3(256), 0, stream, w, O, F, Op, wp, wpt);
}

void repitch_bf16(const uint16_t* src, int a, uint16_t* dst, int b, int64_t R, const uint16_t* bias,
                  hipStream_t stream) {
  const int64_t items = R * (b / 8);
  if (items <= 0) return;
  int64_t blocks = (items + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_repitch, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, src, a, dst, b, R, bias);
}

void linear_f32_fwd(const float* x, const float* w, const float* b, int R, int F, int O, float* y, hipStream_t stream) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_linear_fwd<float>, dim3((R + 3) / 4), dim3(256), 0, stream, x, w, b, R, F, O, y);
}

void linear_f32_dgrad(const float* dl, const float* w, int R, int F, int O, float* dx, hipStream_t stream) {
  const int64_t items = static_cast<int64_t>(R) * F;
  if (items <= 0) return;
  hipLaunchKernelGGL(k_linear_dgrad<float>, dim3(blocks_for(items)), dim3(256), 0, stream, dl, w, R, F, O, dx);
}

void linear_f32_wgrad(const float* x, const float* dl, int groups, int rg, int F, int O, float* out, int64_t row_stride,
                      int64_t off_w, int64_t off_b, hipStream_t stream) {
  if (groups <= 0 || F <= 0) return;
  hipLaunchKernelGGL(k_linear_wgrad<float>, dim3((F + 63) / 64, groups), dim3(256), 0, stream, x, dl, rg, F, O,
                     static_cast<void*>(out), static_cast<int>(kF32), row_stride, off_w, off_b);
}

// the vectorised kernels' limits: F % 8, O <= kLinV, the staged weight / gradient rows in LDS
bool linear_bf16_vec(int R, int F, int O, int rg) {
  (void)R;
  return F % 8 == 0 && O >= 1 && O <= kLinV && static_cast<int64_t>(O) * F * 2 <= 128 * 1024 &&
         (rg <= 0 || (static_cast<int64_t>(rg) * O + 4 * kLinV * kWgF) * 4 <= 128 * 1024);
}

namespace {
template <typename K>
void allow_lin_lds(K* k, size_t bytes) {
  if (bytes > 64 * 1024) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
}
}  // namespace

void linear_bf16_fwd(const uint16_t* x, const uint16_t* w, const uint16_t* b, int R, int F, int O, uint16_t* y,
                     hipStream_t stream) {
  if (R <= 0) return;
  if (linear_bf16_vec(R, F, O, 0)) {
    const size_t lds = static_cast<size_t>(O) * F * 2;
    allow_lin_lds(k_linear_fwd_v, lds);
    hipLaunchKernelGGL(k_linear_fwd_v, dim3((R + kLinRows - 1) / kLinRows), dim3(256), lds, stream, x, w, b, R, F, O, y);
    return;
  }
  hipLaunchKernelGGL(k_linear_fwd<uint16_t>, dim3((R + 3) / 4), dim3(256), 0, stream, x, w, b, R, F, O, y);
}

void linear_bf16_dgrad(const uint16_t* dl, const uint16_t* w, int R, int F, int O, uint16_t* dx, hipStream_t stream) {
  const int64_t items = static_cast<int64_t>(R) * F;
  if (items <= 0) return;
  if (F % 8 == 0) {
    hipLaunchKernelGGL(k_linear_dgrad_v, dim3(blocks_for(items / 8)), dim3(256), 0, stream, dl, w, R, F, O, dx);
    return;
  }
  hipLaunchKernelGGL(k_linear_dgrad<uint16_t>, dim3(blocks_for(items)), dim3(256), 0, stream, dl, w, R, F, O, dx);
}

void linear_bias_grad(const void* dl, bool dl_f32, int groups, int rg, int O, void* out, int odt, int64_t row_stride,
                      int64_t off_b, hipStream_t stream) {
  const dim3 grid((O + 255) / 256, groups);
  if (dl_f32)
    hipLaunchKernelGGL(k_linear_bias_grad<float>, grid, dim3(256), 0, stream, static_cast<const float*>(dl), rg, O, out,
                       odt, row_stride, off_b);
  else
    hipLaunchKernelGGL(k_linear_bias_grad<uint16_t>, grid, dim3(256), 0, stream, static_cast<const uint16_t*>(dl), rg,
                       O, out, odt, row_stride, off_b);
}

void linear_bf16_wgrad(const uint16_t* x, const uint16_t* dl, int groups, int rg, int F, int O, void* out, int odt,
                       int64_t row_stride, int64_t off_w, int64_t off_b, hipStream_t stream) {
  if (groups <= 0 || F <= 0) return;
  if (linear_bf16_vec(rg * groups, F, O, rg)) {
    const size_t lds = (static_cast<size_t>(rg) * O + 4 * kLinV * kWgF) * 4;
    allow_lin_lds(k_linear_wgrad_v, lds);
    hipLaunchKernelGGL(k_linear_wgrad_v, dim3((F + kWgF - 1) / kWgF, groups), dim3(256), lds, stream, x, dl, rg, F, O, out,
                       odt, row_stride, off_w, off_b);
    return;
  }
  hipLaunchKernelGGL(k_linear_wgrad<uint16_t>, dim3((F + 63) / 64, groups), dim3(256), 0, stream, x, dl, rg, F, O, out,
                     odt, row_stride, off_w, off_b);
}

void avgpool_f32_fwd(const float* x, int N, int HW, int C, float* y, hipStream_t stream) {
  const int64_t items = static_cast<int64_t>(N) * C;
  if (items <= 0) return;
  hipLaunchKernelGGL(k_avgpool_fwd<float>, dim3(blocks_for(items)), dim3(256), 0, stream, x, N, HW, C, y);
}

void avgpool_f32_bwd(const float* dy, int N, int HW, int C, float* dx, hipStream_t stream) {
  const int64_t items = static_cast<int64_t>(N) * HW * C;
  if (items <= 0) return;
  hipLaunchKernelGGL(k_avgpool_bwd<float>, dim3(blocks_for(items)), dim3(256), 0, stream, dy, N, HW, C, dx);
}

void avgpool_bf16_fwd(const uint16_t* x, int N, int HW, int C, uint16_t* y, hipStream_t stream) {
  const int64_t items = static_cast<int64_t>(N) * C;
  if (items <= 0) return;
  hipLaunchKernelGGL(k_avgpool_fwd<uint16_t>, dim3(blocks_for(items)), dim3(256), 0, stream, x, N, HW, C, y);
}

void avgpool_bf16_bwd(const uint16_t* dy, int N, int HW, int C, uint16_t* dx, hipStream_t stream) {
  const int64_t items = static_cast<int64_t>(N) * HW * C;
  if (items <= 0) return;
  hipLaunchKernelGGL(k_avgpool_bwd<uint16_t>, dim3(blocks_for(items)), dim3(256), 0, stream, dy, N, HW, C, dx);
}

}  // namespace gpu
}  // namespace garfield
