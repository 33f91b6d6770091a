// Halo-staged 3x3 / stride-1 / pad-1 convolution on MFMA (NHWC, bf16 in, fp32 accumulate), gfx950.
//
// The implicit-GEMM kernel of iconv_nhwc.hip stages, for every one of the nine taps, the shifted
// 64-channel input tile of its output pixels: the same input bytes travel L2 -> LDS nine times
// (a 256-pixel x 64-channel tile: 9 x 32 KB per 64-channel block, plus 9 x 8 KB of weights), and the
// one-stage-ahead ring of its 256-pixel variant leaves the load latency exposed. Measured on the
// CIFAR ResNet-18 step this is 26 % of the bf16 MFMA peak (profiles/r3/configs/rocprof_r18_krum_f2.txt).
//
// Here a workgroup's output tile is TR WHOLE image rows (TP = TR * W <= BM = 64 * PMF pixels; any
// width: 224 of 256 pixels at W = 56, so the ImageNet widths 56 / 28 / 14 / 7 run here too), and its
// input is staged ONCE per 64-channel block as a zero-padded halo: per image segment of the tile,
// (rows + 2) x (W + 2) pixels (a 32-wide image: 10 x 34 pixels for 256 outputs, 1.33x instead of
// 9x). The nine taps then read their B fragments from the halo at a uniform shift (i * (W + 2) + j),
// and only the weight tap tiles stream through a 3-stage global_load_lds ring. Tiles spanning
// several small images (8x8, 4x4) stage one padded image per segment, so image borders are zeros
// in LDS and no tap needs a mask.
//
//   y[m, co] = Σ_{i, j, ci} x[n, h + i - 1, w + j - 1, ci] · W[co, i, j, ci]   (+ add[m, co])
//
// GEMM view as in iconv_nhwc.hip: A = weight rows (co), B = input pixels, v_mfma_f32_16x16x32_bf16,
// wave tile 16*PMF pixels x 64 channels, 4 waves stacked over pixels (workgroup 64*PMF x 64).
// LDS images are 128-byte rows (one pixel's or one channel's 64 bf16) with the 16-byte chunk
// index XOR-swizzled by (row & 7) on the global side (glds writes lane-linear), so a fragment read
// (16 rows x one chunk) touches every bank once on consecutive rows.
//
// The data gradient of this convolution is the same kernel on dy with the flipped, transposed
// weight Wd[ci][i'][j'][co] = W[co][2-i'][2-j'][ci] (refreshed once per step for every layer by
// transpose_multi with taps = 9), padding 1 again.
#include <cstdlib>

#include "bn_gpu.hpp"
#include "bn_stats.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

using lds_ptr = __attribute__((address_space(3))) void*;

__device__ __attribute__((aligned(16))) uint4 g_c3_zero[8];   // 128 zero bytes: padded pixels

struct Halo {
  int TR;    // output rows per tile: the most whole rows with TR * W <= BM that tile the images evenly
  int TP;    // output pixels per tile: TR * W (= BM for power-of-two widths; 224 of 256 at W = 56)
  int TRI;   // output rows per image segment: min(TR, H)
  int SW;    // staged columns: W + 2
  int SEGP;  // staged pixels per segment: (TRI + 2) * SW
  int NPIX;  // staged pixels per tile: (TR / TRI) * SEGP
  int nu;    // halo glds instructions per wave: ceil(NPIX / 32) <= NU
  // magic-number divisors of the per-tile index arithmetic (a runtime integer division is ~20 VALU
  // instructions, a 64-bit one far more; the prologue of a 256-pixel tile did ~40 of them)
  FastDiv fSEGP, fSW, fTRI, fWo, fHo, fW, fH;
};

constexpr int EPI_PLAIN = 0, EPI_ADD = 1, EPI_STATS = 2;

// Output of one wave's 16*PMF-pixel x 64-channel tile (pixels mw + 16 r + fr): D[co = 4 fq + e][pixel fr]
// of every fragment is 4 consecutive channels of one pixel (one 8-byte store); EPI_ADD adds add (the
// other gradient branch), EPI_STATS writes the wave's per-worker statistics tile (bn_stats.hpp).
template <int PMF, int EPI>
__device__ __forceinline__ void conv_epilogue(const f32x4 (&acc)[PMF][4], int mw, int M, int Cout, int co0, uint16_t* y,
                                              const uint16_t* add, float* __restrict__ stats, int64_t rg,
                                              const uint8_t* __restrict__ amask) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  float vs[PMF][4][4];   // the stored (bf16-rounded) values, for the statistics
#pragma unroll
  for (int r = 0; r < PMF; ++r) {
    const int m = mw + r * 16 + fr;
    const int64_t rowoff = static_cast<int64_t>(m < M ? m : 0) * Cout;
    RowMask<4> rm;   // amask: add counts only where the (BatchNorm ReLU) bit is set
    if constexpr (EPI == EPI_ADD)
      if (m < M) rm.load(amask, rowoff + co0);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t off = rowoff + co0 + c * 16 + fq * 4;
      float v[4] = {acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]};
      if constexpr (EPI == EPI_ADD) {
        if (m < M) add_bf16x4(v, add, rm.nib(c, fq), off);
      }
      uint2 o;
      o.x = static_cast<uint32_t>(f_to_bf16(v[0])) | (static_cast<uint32_t>(f_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f_to_bf16(v[2])) | (static_cast<uint32_t>(f_to_bf16(v[3])) << 16);
      if (m < M) *reinterpret_cast<uint2*>(y + off) = o;
      if constexpr (EPI == EPI_STATS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) vs[r][c][i] = bf16_round(v[i]);
      }
    }
  }
  if constexpr (EPI == EPI_STATS) {
    if (mw < M) wave_stats<PMF, 4>(vs, mw, M, rg, Cout, co0, stats);
  }
}

// EPI_STATS: the per-worker (rg pixels) statistics of the stored bf16 outputs for the BatchNorm that
// consumes y, one statistics tile per wave (16 * PMF pixels, bn_stats.hpp), so its forward skips the
// partial-sum pass over y.
template <int PMF, int NU, int EPI>
__global__ __launch_bounds__(256) void k_conv3x3(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                 Im2col g, Halo hp, int Cout, uint16_t* y, const uint16_t* add,
                                                 float* __restrict__ stats, int64_t rg, const uint8_t* amask) {
  constexpr int NSW = 3;               // weight ring stages
  constexpr int BM = 64 * PMF;         // output pixels per workgroup
  constexpr int XB = NU * 4096;        // halo bytes (NU glds rounds of 4 waves x 8 pixels)
  constexpr int WB = 64 * 128;         // one weight tap tile: 64 co x 64 ci
  __shared__ __attribute__((aligned(16))) char lds[XB + NSW * WB];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int M = g.N * g.Ho * g.Wo;
  const int st = g.sh;                 // 1, or 2 (a downsampling convolution)
  const int R0 = blockIdx.x * hp.TR;   // first output (global) row of the tile
  const int m0 = blockIdx.x * hp.TP;
  const int mlim = m0 + hp.TP < M ? m0 + hp.TP : M;   // pixels past TP (a non-power-of-two width) are idle
  const int co0 = blockIdx.y * 64;
  const int lc = lane & 7;             // this lane's 16-byte slot of a staged row

  // halo sources, computed once: element offset of (pixel, logical chunk) or -1 for a zero pixel.
  // Staged row r of segment seg is input row st * h0 - 1 + r of the segment's image (h0 its first
  // output row), staged column c input column c - 1.
  int soff[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int p = (u * 4 + wave) * 8 + (lane >> 3);
    const int seg = static_cast<int>(fdiv(static_cast<uint32_t>(p), hp.fSEGP));
    const int rem = p - seg * hp.SEGP;
    const int r = static_cast<int>(fdiv(static_cast<uint32_t>(rem), hp.fSW)), c = rem - r * hp.SW;
    const int orow = R0 + seg * hp.TRI;                            // the segment's first output row
    const int n = static_cast<int>(fdiv(static_cast<uint32_t>(orow), hp.fHo));
    const int hl = (orow - n * g.Ho) * st - 1 + r;                 // input row inside the image
    const bool ok = p < hp.NPIX && n < g.N && hl >= 0 && hl < g.H && c >= 1 && c <= g.W;
    soff[u] = ok ? ((n * g.H + hl) * g.W + c - 1) * g.C + (lc ^ (p & 7)) * 8 : -1;
  }
  const uint64_t az = reinterpret_cast<uint64_t>(reinterpret_cast<const uint16_t*>(g_c3_zero) + lc * 8);

  // weight tap tile sources: rows (wave*2 + u)*8 + lane/8 of the 64-row tile
  const int K = 9 * g.C;
  const uint16_t* wsrc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = (wave * 2 + u) * 8 + (lane >> 3);
    wsrc[u] = w + static_cast<int64_t>(co0 + row) * K + (lc ^ (row & 7)) * 8;
  }

  auto issue_halo = [&](int cb) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (u < hp.nu) {
        const uint64_t ax = reinterpret_cast<uint64_t>(x + soff[u] + cb * 64);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(soff[u] >= 0 ? ax : az),
                                         (lds_ptr)(lds + (u * 4 + wave) * 1024), 16, 0, 0);
      }
    }
  };
  auto issue_w = [&](int s, int slot) {
    const int cb = s / 9, tap = s - (s / 9) * 9;
    const int off = tap * g.C + cb * 64;
    char* base = lds + XB + slot * WB;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_global_load_lds(wsrc[u] + off, (lds_ptr)(base + (wave * 2 + u) * 1024), 16, 0, 0);
  };

  // this lane's B rows: staged pixel of tap (0, 0) for each pixel fragment
  const int fr = lane & 15, fq = lane >> 4;
  int sp0[PMF];
#pragma unroll
  for (int r = 0; r < PMF; ++r) {
    const int ml = (wave * PMF + r) * 16 + fr;
    const int t = static_cast<int>(fdiv(static_cast<uint32_t>(ml), hp.fWo)), col = ml - t * g.Wo;
    const int seg = static_cast<int>(fdiv(static_cast<uint32_t>(t), hp.fTRI));
    sp0[r] = ml < hp.TP ? seg * hp.SEGP + (t - seg * hp.TRI) * st * hp.SW + col * st : 0;
  }

  f32x4 acc[PMF][4];
#pragma unroll
  for (int r = 0; r < PMF; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ncb = g.C / 64;
  const int steps = ncb * 9;
  issue_halo(0);
#pragma unroll
  for (int s0 = 0; s0 < NSW - 1; ++s0)
    if (s0 < steps) issue_w(s0, s0);

  int tap = 0, cb = 0;
  for (int s = 0; s < steps; ++s) {
    if (tap == 0 || s + 1 >= steps) {
      // a new halo (issued after the ring loads in flight), or the last stage: drain
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // W(s + 1) may stay in flight
    }
    __builtin_amdgcn_s_barrier();
    if (s + NSW - 1 < steps) issue_w(s + NSW - 1, (s + NSW - 1) % NSW);
    const char* wb = lds + XB + (s % NSW) * WB;
    const int ti = tap / 3;
    const int toff = ti * hp.SW + (tap - ti * 3);
    // both 32-channel halves' fragments are read up front: the second half's reads are in flight
    // while the first half's MFMAs run
    bf16x8 a[2][4], b[2][PMF];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = c * 16 + fr;
        a[ks][c] = *reinterpret_cast<const bf16x8*>(wb + row * 128 + (((ks * 4 + fq) ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int r = 0; r < PMF; ++r) {
        const int sp = sp0[r] + toff;
        b[ks][r] = *reinterpret_cast<const bf16x8*>(lds + sp * 128 + (((ks * 4 + fq) ^ (sp & 7)) * 16));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int r = 0; r < PMF; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks][c], b[ks][r], acc[r][c], 0, 0, 0);
    // every wave's reads of this ring slot (and of the halo) retire before the next barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (++tap == 9) {
      tap = 0;
      if (++cb < ncb) {
        __builtin_amdgcn_s_barrier();   // the halo is refilled only once every wave is done with it
        issue_halo(cb);
      }
    }
  }

  conv_epilogue<PMF, EPI>(acc, m0 + wave * PMF * 16, mlim, Cout, co0, y, add, stats, rg, amask);
}

// 64 input channels (one halo block per tile: ResNet layer1-type layers). The one-shot kernel above
// stages a 43 KB halo and nine weight taps per 256-pixel tile and computes for only nine k-steps,
// so every tile pays the full load latency. Here a persistent workgroup keeps its 64-channel output
// block's whole weight (9 taps x 64 x 64, 72 KB) resident in LDS, double-buffers the halo (2 x 44 KB:
// the 160 KB of LDS exactly), and walks tiles blockIdx.x, + gridDim.x, ...: the next tile's halo
// streams in while the nine taps of the current one run.
constexpr int kNuRes = 11;   // 256-pixel tiles of 32- or 16-wide images: 340 / 324 halo pixels

template <int EPI>
__global__ __launch_bounds__(256) void k_conv3x3_res(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                     Im2col g, Halo hp, int Cout, int tiles, uint16_t* y,
                                                     const uint16_t* add, float* __restrict__ stats, int64_t rg,
                                                     const uint8_t* amask) {
  constexpr int PMF = 4, BM = 256, NU = kNuRes;
  constexpr int XB = NU * 4096;
  constexpr int WB = 9 * 64 * 128;
  __shared__ __attribute__((aligned(16))) char lds[WB + 2 * XB];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int M = g.N * g.H * g.W;
  const int rows = g.N * g.H;
  const int co0 = blockIdx.y * 64;
  const int lc = lane & 7;
  const uint64_t az = reinterpret_cast<uint64_t>(reinterpret_cast<const uint16_t*>(g_c3_zero) + lc * 8);

  // resident weight: tap t rows co0 .. co0 + 63 at lds + t * 8 KB (18 glds per lane)
#pragma unroll
  for (int u = 0; u < 18; ++u) {
    const int tap = u >> 1;
    const int row = ((u & 1) * 4 + wave) * 8 + (lane >> 3);
    __builtin_amdgcn_global_load_lds(w + static_cast<int64_t>(co0 + row) * (9 * 64) + tap * 64 + (lc ^ (row & 7)) * 8,
                                     (lds_ptr)(lds + tap * 8192 + ((u & 1) * 4 + wave) * 1024), 16, 0, 0);
  }
  // halo pixel decomposition of this lane's glds rows (tile-independent)
  int hrow[NU], hcol[NU], hsw[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int p = (u * 4 + wave) * 8 + (lane >> 3);
    const int seg = static_cast<int>(fdiv(static_cast<uint32_t>(p), hp.fSEGP));
    const int rem = p - seg * hp.SEGP;
    const int r = static_cast<int>(fdiv(static_cast<uint32_t>(rem), hp.fSW));
    const int c = rem - r * hp.SW;
    const bool ok = u < hp.nu && p < hp.NPIX && c >= 1 && c <= g.W;
    hrow[u] = ok ? (seg * hp.TRI + r - 1) : -(1 << 28);
    hcol[u] = (c - 1) * 64 + ((lc ^ (p & 7)) * 8);
    hsw[u] = r - 1;
  }
  auto issue_halo = [&](int tile, int buf) {
    const int R0 = tile * hp.TR;
    const int h0 = R0 - static_cast<int>(fdiv(static_cast<uint32_t>(R0), hp.fH)) * g.H;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (u < hp.nu) {
        const int gr = R0 + hrow[u];
        const int hl = h0 + hsw[u];
        const bool ok = hrow[u] > -(1 << 27) && gr < rows && hl >= 0 && hl < g.H;
        const uint64_t a = reinterpret_cast<uint64_t>(x + static_cast<int64_t>(gr) * g.W * 64 + hcol[u]);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? a : az),
                                         (lds_ptr)(lds + WB + buf * XB + (u * 4 + wave) * 1024), 16, 0, 0);
      }
    }
  };

  const int fr = lane & 15, fq = lane >> 4;
  int sp0[PMF];
#pragma unroll
  for (int r = 0; r < PMF; ++r) {
    const int ml = (wave * PMF + r) * 16 + fr;
    const int t = static_cast<int>(fdiv(static_cast<uint32_t>(ml), hp.fW)), col = ml - t * g.W;
    const int seg = static_cast<int>(fdiv(static_cast<uint32_t>(t), hp.fTRI));
    sp0[r] = ml < hp.TP ? seg * hp.SEGP + (t - seg * hp.TRI) * hp.SW + col : 0;
  }

  int tile = blockIdx.x;
  if (tile < tiles) issue_halo(tile, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int it = 0; tile < tiles; ++it, tile += gridDim.x) {
    const int buf = it & 1;
    if (tile + static_cast<int>(gridDim.x) < tiles) issue_halo(tile + gridDim.x, buf ^ 1);
    const char* hb = lds + WB + buf * XB;
    f32x4 acc[PMF][4];
#pragma unroll
    for (int r = 0; r < PMF; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 18 k-steps (tap, 32-channel half); the fragments of step s + 1 are read from LDS while the
    // MFMAs of step s run (one wave per SIMD: nothing else hides the LDS latency)
    auto frags = [&](int st, bf16x8 (&a)[4], bf16x8 (&b)[PMF]) {
      const int tap = st >> 1, ks = st & 1;
      const char* wb = lds + tap * 8192;
      const int ti = tap / 3;
      const int toff = ti * hp.SW + (tap - ti * 3);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = c * 16 + fr;
        a[c] = *reinterpret_cast<const bf16x8*>(wb + row * 128 + (((ks * 4 + fq) ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int r = 0; r < PMF; ++r) {
        const int sp = sp0[r] + toff;
        b[r] = *reinterpret_cast<const bf16x8*>(hb + sp * 128 + (((ks * 4 + fq) ^ (sp & 7)) * 16));
      }
    };
    auto mma = [&](const bf16x8 (&a)[4], const bf16x8 (&b)[PMF]) {
#pragma unroll
      for (int r = 0; r < PMF; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[r], acc[r][c], 0, 0, 0);
    };
    bf16x8 a0[4], b0[PMF], a1[4], b1[PMF];
    frags(0, a0, b0);
#pragma unroll 1
    for (int st = 0; st < 18; st += 2) {
      frags(st + 1, a1, b1);
      mma(a0, b0);
      if (st + 2 < 18) frags(st + 2, a0, b0);
      mma(a1, b1);
    }
    const int mt = tile * hp.TP;
    conv_epilogue<PMF, EPI>(acc, mt + wave * PMF * 16, mt + hp.TP < M ? mt + hp.TP : M, Cout, co0, y, add, stats,
                            rg, amask);
    // the next halo has landed and every wave is done with this one before it is refilled. The
    // epilogue's 16 output stores (PMF x 4 global_store_dwordx2, issued after the halo loads) may stay
    // in flight: waiting for them too exposed the store latency once per tile. A ragged tile (the
    // last one, or every tile of a TP < BM width) may branch around stores, so it drains everything.
    if (hp.TP == BM && mt + BM <= M) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

// tile geometry for PMF pixel fragments per wave; false when the shape does not fit
bool plan(const Im2col& g, int pmf, int nu_max, Halo& hp) {
  // output tiles of TR whole output rows; stride st stages ((TRI - 1) * st + 3) input rows x
  // ((Wo - 1) * st + 3) input columns per image segment
  const int st = g.sh;
  const int BM = 64 * pmf;
  if (g.Wo > BM) return false;
  // the most whole output rows per tile that still tile the images evenly (TR | Ho, or Ho | TR for tiles
  // of several small images): W = 32 -> 8 rows (256 px), 56 -> 4 (224), 28 -> 7 (196), 7 -> 35 (245)
  hp.TR = 0;
  for (int tr = BM / g.Wo; tr >= 1 && hp.TR == 0; --tr)
    if ((tr <= g.Ho && g.Ho % tr == 0) || (tr > g.Ho && tr % g.Ho == 0)) hp.TR = tr;
  if (hp.TR == 0) return false;
  hp.TP = hp.TR * g.Wo;
  if (4 * hp.TP < 3 * BM) return false;   // under 75 % of the tile's MFMA work would be used
  hp.TRI = hp.TR < g.Ho ? hp.TR : g.Ho;
  hp.SW = (g.Wo - 1) * st + 3;
  hp.SEGP = ((hp.TRI - 1) * st + 3) * hp.SW;
  hp.NPIX = (hp.TR / hp.TRI) * hp.SEGP;
  hp.nu = (hp.NPIX + 31) / 32;
  hp.fSEGP = make_fastdiv(static_cast<uint32_t>(hp.SEGP));
  hp.fSW = make_fastdiv(static_cast<uint32_t>(hp.SW));
  hp.fTRI = make_fastdiv(static_cast<uint32_t>(hp.TRI));
  hp.fWo = make_fastdiv(static_cast<uint32_t>(g.Wo));
  hp.fHo = make_fastdiv(static_cast<uint32_t>(g.Ho));
  hp.fW = make_fastdiv(static_cast<uint32_t>(g.W));
  hp.fH = make_fastdiv(static_cast<uint32_t>(g.H));
  return hp.nu <= nu_max && static_cast<int64_t>(g.N) * g.H * g.W < (int64_t{1} << 31);
}

template <int PMF, int NU>
void launch(const uint16_t* x, const uint16_t* w, const Im2col& g, const Halo& hp, int Cout, uint16_t* y,
            const uint16_t* add, float* stats, int64_t rg, hipStream_t stream, const uint8_t* amask) {
  const int tiles = (g.N * g.Ho + hp.TR - 1) / hp.TR;
  const dim3 grid(tiles, Cout / 64);
  if (add)
    hipLaunchKernelGGL((k_conv3x3<PMF, NU, EPI_ADD>), grid, dim3(256), 0, stream, x, w, g, hp, Cout, y, add, stats,
                       rg, amask);
  else if (stats)
    hipLaunchKernelGGL((k_conv3x3<PMF, NU, EPI_STATS>), grid, dim3(256), 0, stream, x, w, g, hp, Cout, y, add, stats,
                       rg, nullptr);
  else
    hipLaunchKernelGGL((k_conv3x3<PMF, NU, EPI_PLAIN>), grid, dim3(256), 0, stream, x, w, g, hp, Cout, y, add, stats,
                       rg, nullptr);
}

constexpr int kNuBig = 14;    // PMF 4: 14 x 4 KB halo + 3 x 8 KB ring = 80 KB (two workgroups per CU)
constexpr int kNuSmall = 10;  // PMF 2: 40 + 24 = 64 KB

// ---------------------------------------------------------------------------------------------
// Per-worker weight gradient of the same convolutions, halo-staged:
//
//   dW_g[co, (i, j, ci)] = Σ_{m in worker g} dy[m, co] · x[n, h + i - 1, w + j - 1, ci]
//
// A workgroup owns one (64 co, 64 ci) block of ALL nine taps for one worker (and one pixel split of
// it) and walks that worker's pixels in tiles of 128 (whole rows, as in the forward): per tile the dy
// tile [128 px x 64 co] and the input halo [(rows + 2) x (W + 2) px x 64 ci] are staged ONCE, and each
// 32-pixel k-step feeds the nine taps' MFMAs from the same dy fragments (the implicit kernel of
// iconv_nhwc.hip stages one shifted input tile per tap row and re-reads dy per kernel row).
// Both operands are reduced over pixels, so fragments are read transposed (ds_read_b64_tr_b16:
// lane 4q+p of a 16-lane group addresses pixel row 8*grp + 4h + q, channels 16f + 4p .. +3). The
// staged 128-byte rows carry their 16-byte chunks XOR-swizzled by bits 1 and 3 of the row, which makes
// those reads conflict-free on consecutive rows. Wave tile (WL 1, the default): all 4 co fragments x one
// ci fragment x 9 taps, so each transposed read of the halo feeds four MFMAs instead of two (26 instead
// of 40 fragment reads per 36 MFMAs: the kernel is bound by its LDS reads, not its MFMAs); WL 0 (2 co x
// 2 ci) was 15-20 % slower per call on every ResNet-18 layer, bit-identical (profiles/r6/wgrad3x3/).
__device__ __forceinline__ int tr_swz(int row) { return (((row >> 3) & 1) << 2) | (((row >> 1) & 1) << 1); }

typedef short s16x4 __attribute__((ext_vector_type(4)));

// ds_read_b64_tr_b16 through the compiler builtin (no LDS-DMA is in flight at the reads of this
// kernel, so the vmcnt(0) the compiler puts in front of it costs nothing; the compiler then also
// tracks the returned registers: inline-asm reads raced with co-resident workgroups' timing)
__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)((lds_ptr)p));
}

template <int NU, bool OUT_BF16, int WL = 1>
__global__ __launch_bounds__(256, 2) void k_wgrad3x3(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                  Im2col g, Halo hp, int Cout, int64_t rg, int tiles_per_split,
                                                  void* out, int64_t split_stride, int64_t group_stride) {
  constexpr int TPC = 128;              // output pixels per tile at most (hp.TP: whole rows)
  constexpr int DB = TPC * 128;         // dy tile bytes
  __shared__ __attribute__((aligned(16))) char lds[DB + NU * 4096];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ncb = g.C / 64;
  const int cb = blockIdx.x % ncb, ob = blockIdx.x / ncb;
  const int c0 = cb * 64, co0 = ob * 64;
  const int gi = blockIdx.y, sp = blockIdx.z;
  const int K = 9 * g.C;
  const int rows = g.N * g.H;
  const int64_t pbeg = static_cast<int64_t>(gi) * rg;       // the worker's first pixel (an image start)
  const int64_t pend = pbeg + rg;
  const int ntiles = static_cast<int>((rg + hp.TP - 1) / hp.TP);
  const FastDiv fW = hp.fW;
  const int t0 = sp * tiles_per_split;
  const int t1 = t0 + tiles_per_split < ntiles ? t0 + tiles_per_split : ntiles;
  const int lc = lane & 7;
  const uint64_t az = reinterpret_cast<uint64_t>(reinterpret_cast<const uint16_t*>(g_c3_zero) + lc * 8);

  // halo pixel decomposition of this lane's glds rows (tile-independent)
  int hrow[NU], hcol[NU], hsw[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int p = (u * 4 + wave) * 8 + (lane >> 3);
    const int seg = static_cast<int>(fdiv(static_cast<uint32_t>(p), hp.fSEGP));
    const int rem = p - seg * hp.SEGP;
    const int r = static_cast<int>(fdiv(static_cast<uint32_t>(rem), hp.fSW));
    const int c = rem - r * hp.SW;
    const bool ok = u < hp.nu && p < hp.NPIX && c >= 1 && c <= g.W;
    hrow[u] = ok ? (seg * hp.TRI + r - 1) : -(1 << 28);   // input row relative to the tile's first row
    hcol[u] = (c - 1) * g.C + c0 + ((lc ^ tr_swz(p)) * 8);
    hsw[u] = r - 1;                                        // row shift inside the segment's image
  }

  // transposed-read addresses: lane (grp, q, p) of pixel rows 8*grp + 4h + q of each 32-pixel step
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  constexpr int NCF = WL == 0 ? 2 : 4, NKF = WL == 0 ? 2 : 1;   // co x ci fragments per wave
  const int cf0 = WL == 0 ? 2 * (wave >> 1) : 0, kf0 = WL == 0 ? 2 * (wave & 1) : wave;

  f32x4 acc[9][NCF][NKF];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int a = 0; a < NCF; ++a)
#pragma unroll
      for (int b = 0; b < NKF; ++b) acc[t][a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int tile = t0; tile < t1; ++tile) {
    const int64_t P0 = pbeg + static_cast<int64_t>(tile) * hp.TP;   // first pixel of the tile
    const int64_t Pend = P0 + hp.TP < pend ? P0 + hp.TP : pend;
    const int R0 = static_cast<int>(fdiv(static_cast<uint32_t>(P0), hp.fW));   // P0 < 2^31 (host check)
    const int h0 = R0 - static_cast<int>(fdiv(static_cast<uint32_t>(R0), hp.fH)) * g.H;
    // dy tile: 128 pixels x 8 chunks, 4 glds per lane (pixels past TP: zero rows)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = (u * 4 + wave) * 8 + (lane >> 3);
      const int64_t P = P0 + m;
      const uint64_t a = reinterpret_cast<uint64_t>(dy + P * Cout + co0 + ((lc ^ tr_swz(m)) * 8));
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(P < Pend ? a : az),
                                       (lds_ptr)(lds + (u * 4 + wave) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (u < hp.nu) {
        const int gr = R0 + hrow[u];
        const int hl = h0 + hsw[u];
        const bool ok = hrow[u] > -(1 << 27) && gr < rows && hl >= 0 && hl < g.H;
        const uint64_t a = reinterpret_cast<uint64_t>(x + static_cast<int64_t>(gr) * g.W * g.C + hcol[u]);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ok ? a : az),
                                         (lds_ptr)(lds + DB + (u * 4 + wave) * 1024), 16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // (a runtime loop: unrolled, the compiler hoists every tap's fragment address out of the tile
    // loop and spills)
#pragma unroll 1
    for (int c = 0; c < 4; ++c) {
      int hp0[2];   // halo pixel of tap (0, 0) for tile pixel 32*c + 8*grp + 4*h + q
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = 32 * c + 8 * grp + 4 * h + q;
        uint32_t t, col;
        fdivmod(static_cast<uint32_t>(m), fW, t, col);
        const int seg = static_cast<int>(fdiv(t, hp.fTRI));
        // a pixel past TP has a zero dy row; it reads halo pixel 0 (finite) so 0 x stale LDS cannot be NaN
        hp0[h] = m < hp.TP ? seg * hp.SEGP + (static_cast<int>(t) - seg * hp.TRI) * hp.SW + static_cast<int>(col) : 0;
      }
      // A = dyᵀ fragments of co fragments cf0 .. cf0 + NCF - 1: dy rows 32c + 8grp + 4h + q
      s16x4 ra[2 * NCF];
#pragma unroll
      for (int u = 0; u < NCF; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int m = 32 * c + 8 * grp + 4 * h + q;
          const int ch = 2 * (cf0 + u) + (pp >> 1);
          ra[2 * u + h] = tr_read(lds + m * 128 + ((ch ^ tr_swz(m)) * 16) + (pp & 1) * 8);
        }
      bf16x8 a[NCF];
#pragma unroll
      for (int u = 0; u < NCF; ++u)
        a[u] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ra[2 * u], ra[2 * u + 1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * hp.SW + (tap % 3);
        s16x4 rb[2 * NKF];
#pragma unroll
        for (int v = 0; v < NKF; ++v)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int s = hp0[h] + toff;
            const int ch = 2 * (kf0 + v) + (pp >> 1);
            rb[2 * v + h] = tr_read(lds + DB + s * 128 + ((ch ^ tr_swz(s)) * 16) + (pp & 1) * 8);
          }
#pragma unroll
        for (int v = 0; v < NKF; ++v) {
          const bf16x8 b = __builtin_bit_cast(bf16x8,
                                              __builtin_shufflevector(rb[2 * v], rb[2 * v + 1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int u = 0; u < NCF; ++u)
            acc[tap][u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b, acc[tap][u][v], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_s_barrier();   // every wave is done with the tile before it is refilled
  }

  // D[co = 16 (cf0 + u) + 4 grp + e][ci = 16 (kf0 + v) + li] of every tap
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int u = 0; u < NCF; ++u)
#pragma unroll
      for (int v = 0; v < NKF; ++v)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + (cf0 + u) * 16 + 4 * grp + e;
          const int64_t o = static_cast<int64_t>(sp) * split_stride + static_cast<int64_t>(gi) * group_stride +
                            static_cast<int64_t>(co) * K + tap * g.C + c0 + (kf0 + v) * 16 + li;
          if constexpr (OUT_BF16) static_cast<uint16_t*>(out)[o] = f_to_bf16(acc[tap][u][v][e]);
          else static_cast<float*>(out)[o] = acc[tap][u][v][e];
        }
}

constexpr int kNuWgrad = 10;   // 16 KB dy tile + 40 KB halo: two workgroups per CU

}  // namespace

bool wgrad3x3_fits(const Im2col& g, int Cout, int64_t rg) {
  Halo hp;
  return g.sh == 1 && g.sw == 1 && conv3x3_pick(g, Cout) != 0 && plan(g, 2, kNuWgrad, hp) && rg > 0 &&
         rg % (static_cast<int64_t>(g.H) * g.W) == 0;
}

bool wgrad3x3_nhwc(const uint16_t* x, const uint16_t* dy, const Im2col& g, int Cout, int groups, int64_t rg,
                   int splits, void* out, bool out_bf16, int64_t split_stride, int64_t group_stride,
                   hipStream_t stream) {
  Halo hp;
  if (!wgrad3x3_fits(g, Cout, rg) || !plan(g, 2, kNuWgrad, hp)) return false;
  const int ntiles = static_cast<int>((rg + hp.TP - 1) / hp.TP);
  if (splits < 1) splits = 1;
  const int per = (ntiles + splits - 1) / splits;
  const dim3 grid((g.C / 64) * (Cout / 64), groups, splits);
  if (out_bf16)
    hipLaunchKernelGGL((k_wgrad3x3<kNuWgrad, true>), grid, dim3(256), 0, stream, x, dy, g, hp, Cout, rg, per, out,
                       split_stride, group_stride);
  else
    hipLaunchKernelGGL((k_wgrad3x3<kNuWgrad, false>), grid, dim3(256), 0, stream, x, dy, g, hp, Cout, rg, per, out,
                       split_stride, group_stride);
  return true;
}

int conv3x3_pick(const Im2col& g, int Cout) {
  if (g.KH != 3 || g.KW != 3 || g.ph != 1 || g.pw != 1 || g.dh != 1 || g.dw != 1 || g.C % 64 || Cout % 64)
    return 0;
  Halo hp;
  // stride 2 stays on the implicit-GEMM kernel: a halo-staged stride-2 variant measured 222 vs 176 us
  // per ResNet-18 downsampling layer (one 16-pixel fragment per wave re-reads four weight fragments per
  // MFMA pair, and the stride-2 B rows hit 2-way bank conflicts) and was removed
  if (g.sh != 1 || g.sw != 1 || g.Ho != g.H || g.Wo != g.W) return 0;
  if (plan(g, 4, kNuBig, hp)) return 4;
  if (plan(g, 2, kNuSmall, hp)) return 2;
  return 0;
}

namespace {
int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

bool conv3x3_nhwc(const uint16_t* x, const uint16_t* w, const Im2col& g, int Cout, uint16_t* y, const uint16_t* add,
                  int pmf, hipStream_t stream, float* stats, int64_t rg, const uint8_t* add_mask) {
  if (pmf <= 0) pmf = conv3x3_pick(g, Cout);
  if (!add) add_mask = nullptr;
  if (stats && (add || rg < 16 * pmf)) return false;
  Halo hp;
  // the statistics epilogue indexes its tiles by 16 * PMF-pixel wave ranges: whole tiles only
  if (stats && !(plan(g, pmf, pmf == 4 ? kNuBig : kNuSmall, hp) && hp.TP == 64 * pmf)) return false;
  if (pmf == 4 && g.C == 64 && conv3x3_pick(g, Cout) == 4 && plan(g, 4, kNuRes, hp)) {
    const int tiles = (g.N * g.H + hp.TR - 1) / hp.TR;
    int gx = cu_count() / (Cout / 64);   // (the tile rows above are re-planned for the resident halo)
    gx = gx < 1 ? 1 : (gx > tiles ? tiles : gx);
    const dim3 grid(gx, Cout / 64);
    if (add)
      hipLaunchKernelGGL((k_conv3x3_res<EPI_ADD>), grid, dim3(256), 0, stream, x, w, g, hp, Cout, tiles, y, add, stats,
                         rg, add_mask);
    else if (stats)
      hipLaunchKernelGGL((k_conv3x3_res<EPI_STATS>), grid, dim3(256), 0, stream, x, w, g, hp, Cout, tiles, y, add,
                         stats, rg, nullptr);
    else
      hipLaunchKernelGGL((k_conv3x3_res<EPI_PLAIN>), grid, dim3(256), 0, stream, x, w, g, hp, Cout, tiles, y, add,
                         stats, rg, nullptr);
    return true;
  }
  const int pick = conv3x3_pick(g, Cout);
  const bool s1 = g.sh == 1;
  if (pmf == 4 && pick && s1 && plan(g, 4, kNuBig, hp)) {
    launch<4, kNuBig>(x, w, g, hp, Cout, y, add, stats, rg, stream, add_mask);
    return true;
  }
  if (pmf == 2 && pick && s1 && plan(g, 2, kNuSmall, hp)) {
    launch<2, kNuSmall>(x, w, g, hp, Cout, y, add, stats, rg, stream, add_mask);
    return true;
  }
  return false;
}

}  // namespace gpu
}  // namespace garfield
