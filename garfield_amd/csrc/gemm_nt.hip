// Row-major "NT" GEMMs for the grouped step's 1x1 convolutions, on MFMA (bf16 in, fp32
// accumulate, bf16 out), gfx950, with the producer-side BatchNorm statistics fused in.
//
//   C[M, N] = A[M, K] · B[N, K]ᵀ  (+ add[M, N])
//
// Forward of a 1x1 stride-1 convolution: A = the NHWC activation rows [pixels, Cin],
// B = the weight [Cout, Cin]. Data gradient: A = dy rows [pixels, Cout], B = the
// transposed weight [Cin, Cout]; ``add`` folds in the residual branch's gradient.
//
// The step's 1x1 GEMMs are skinny (M = 2k..128k pixels, N, K = 64..2048) and mostly
// memory-bound; hipBLASLt measured 1.5-2.5x the compulsory-byte time on them with a
// ~10 µs floor per call (scripts/bench_1x1.py), and its epilogue cannot produce the
// per-WORKER BatchNorm statistics the next layer needs. Two kernels:
//
// * k_gemm_ws (K <= 256, the big-M layers): weight-stationary and persistent. A
//   workgroup loads its [BN, K] weight slice into LDS ONCE and then streams row tiles
//   [BM, K] through a 2-slot global_load_lds ring (tile t+1 in flight while tile t is
//   multiplied and written). Each of the 4 waves owns RW rows x 64 channels, so its
//   epilogue is wave-private: the bf16 tile goes through the wave's own XOR-swizzled LDS
//   slice and leaves as whole 128-B row lines (16 B per lane), with no workgroup barrier.
//   Workgroups streaming the same row tiles (different N slices) share an XCD (L2).
// * k_gemm_nt (any K % 64): a K-loop over 64-deep steps staged by global_load_lds in an
//   NS-deep ring, XCD-aware tile order, whole-tile LDS epilogue.
//
// v_mfma_f32_16x16x32_bf16 takes the WEIGHT as the MFMA A operand, so the accumulator's
// lane holds 4 consecutive output channels of one pixel, and the 16 lanes of a DPP row
// hold one channel quad for 16 pixels. EPI_STATS therefore reduces the per-channel
// statistics of the STORED bf16 values in registers: a 4-step DPP row reduction gives
// Σy over the wave's rows, then Σ(y - ȳ)² around that sub-tile mean (count-free pairs,
// no cancellation whatever |mean| / std). Each wave's RW-row sub-tile is one statistics
// tile (split in two slots where it straddles a worker boundary); ``bn_finalize_tiles``
// merges a worker's tiles with Chan's parallel-variance update, so the BatchNorm forward
// runs only its apply pass.
//
// Statistics layout: stats[T][E][slot][q][N] floats, q = {n, Σy, Σ(y - ȳ)²}: stats tile T covers
// rows [T*H, (T+1)*H) (H <= rows per worker, so at most two workers: slot 0 the first, slot 1
// the next); its E entries (e.g. the waves that share it) each cover a subset of those rows and
// carry their own count.
#include "bn_gpu.hpp"
#include "bn_stats.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
int kernel_variant(const char* name);   // bindings.cpp: A/B switches of kernel forms (0: default)
namespace {

using lds_ptr = __attribute__((address_space(3))) void*;

// LDS-DMA of 16 bytes per lane (lane i -> lds_dst + 16 i) issued from inline asm: hipcc does not see it,
// so it neither counts it nor, as it does for __builtin_amdgcn_global_load_lds, waits vmcnt(0) for it
// before an unrelated ds_write it cannot prove disjoint (k_gemm_ws's epilogue slice: that wait drained
// the next row tile's prefetch every tile). The caller waits for it with counted vmcnt. lds_dst: the
// wave-uniform LDS byte address; M0 is written and restored in the same statement.
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
// 8 bytes per lane by inline asm (for k_gemm_ws's addend: hipcc neither counts nor waits for it;
// the caller waits with a counted vmcnt, then pins the registers with an empty "+v" statement)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 ld8_asm(const void* p) {
  u32x2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(lds_ptr)(p);
}
__device__ __attribute__((aligned(16))) uint4 g_gemm_zero[8];

struct GemmPro {         // BatchNorm prologue of A (see pro_chunk); sc == nullptr: none
  const float* sc;       // [G][K] scale
  const float* sh;       // [G][K] shift
  FastDiv frg;           // rows per worker
  int G;
  const uint8_t* amask;  // EPI_ADD: add is masked by this 1-bit-per-element mask (BatchNorm ReLU bits); nullptr: not
};  // 128 zero bytes: source of padded rows

constexpr int EPI_PLAIN = 0, EPI_ADD = 1, EPI_STATS = 2;
// EPI_SPLIT: split-K (blockIdx.y = split ky of gridDim.y): the workgroup reduces K range
// [ky K / S, (ky + 1) K / S) and stores its fp32 accumulators to ws[ky][M][N]; k_split_sum adds the
// S slabs (+ add) into C. For the latency-bound small-M x N, long-K problems (ResNet-50 CIFAR
// layer3 / layer4 1x1 and small-image GEMMs: 250-250 workgroups walking 16-32 k-steps each).
constexpr int EPI_SPLIT = 3;

// BatchNorm prologue (PRO): A holds the PRE-BatchNorm activation of the layer before; each staged
// 16-byte chunk (8 channels of one row) becomes bf16(max(x * scale[g][c] + shift[g][c], 0)) in LDS
// before any wave reads it, g = row / rg (the row's worker). The lane that staged a chunk by
// LDS-DMA transforms exactly that chunk (its own completed load), then one barrier publishes the
// tile: the normalised activation is never written to HBM. Scale / shift come from an LDS table
// filled once per workgroup (dynamic LDS).
__device__ __forceinline__ void pro_chunk(char* p, const float* sc, const float* sh) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  const float4 s0 = *reinterpret_cast<const float4*>(sc), s1 = *reinterpret_cast<const float4*>(sc + 4);
  const float4 h0 = *reinterpret_cast<const float4*>(sh), h1 = *reinterpret_cast<const float4*>(sh + 4);
  const float a[8] = {__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                      __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u),
                      __uint_as_float(v.z << 16), __uint_as_float(v.z & 0xffff0000u),
                      __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xffff0000u)};
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
  float y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) y[i] = fmaxf(fmaf(a[i], sv[i], hv[i]), 0.f);
  *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]),
                                            pack_bf16x2(y[4], y[5]), pack_bf16x2(y[6], y[7]));
}

// ---------------------------------------------------------------------------------------------
// K-loop kernel

// KG > 1 (in-workgroup split-K): KG groups of 4 waves (256 * KG threads) walk consecutive quarters
// (halves) of the K range over their own LDS rings, so each SIMD holds KG waves to hide the ring's
// latency with, and each group makes 1 / KG of the serial k-steps. The groups' fp32 accumulators
// are summed in group order through LDS (deterministic) and group 0 runs the epilogue. For the
// latency-bound small-M problems (ResNet-50 CIFAR layer3 / layer4: ~250 workgroups, 16-32 k-steps
// each at one wave per SIMD), without the split-K slabs' second launch and fp32 HBM round trip.
// The ring then lives in dynamic LDS (> 64 KB).
template <int WPM, int WPN, int WM, int WN, int NS, int EPI, bool PRO, int KG = 1>
__global__ __launch_bounds__(256 * KG) void k_gemm_nt(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                      int M, int N, int K, uint16_t* __restrict__ C,
                                                      const uint16_t* __restrict__ add, float* __restrict__ stats,
                                                      int64_t rg, GemmPro pro) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(KG == 1 || (!PRO && EPI != EPI_SPLIT), "in-workgroup split-K: plain / add / statistics epilogues");
  constexpr int BM = 16 * WPM * WM, BN = 16 * WPN * WN;
  constexpr int AB = BM * 128, BB = BN * 128, SB = AB + BB;
  constexpr int AI = BM / 32, BI = BN / 32;     // glds instructions per wave per stage
  constexpr int PER = AI + BI;
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tiles are whole 8-row glds blocks per wave");
  static_assert(KG == 1 || (KG - 1) * 4 * WPM * WPN * 1024 <= KG * NS * SB, "the group sums fit the rings");
  __shared__ __attribute__((aligned(16))) char lds_s[KG == 1 ? NS * SB : 16];
  extern __shared__ __attribute__((aligned(16))) char lds_d[];
  char* const lds = KG == 1 ? lds_s : lds_d;

  const int lane = threadIdx.x & 63;
  const int wave = (threadIdx.x >> 6) & 3;
  const int kg = KG == 1 ? 0 : static_cast<int>(threadIdx.x >> 8);   // K group
  const int tiles_n = N / BN;
  const int nt = gridDim.x;
  const int b = blockIdx.x;
  // XCD-aware numbering: block b runs on XCD b % 8; consecutive tile ids (the N blocks
  // of one M block) get blocks of the same residue
  const int t = (nt % 8 == 0) ? (b % 8) * (nt / 8) + b / 8 : b;
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lrow = lane >> 3, lchunk = lane & 7;

  // split-K: this workgroup's K range
  const int KS = EPI == EPI_SPLIT ? K / static_cast<int>(gridDim.y) : K;
  const int kbase = EPI == EPI_SPLIT ? static_cast<int>(blockIdx.y) * KS : 0;
  const uint16_t* asrc[AI];
  bool av[AI];
#pragma unroll
  for (int u = 0; u < AI; ++u) {
    const int row = (wave * AI + u) * 8 + lrow;
    av[u] = m0 + row < M;
    asrc[u] = A + static_cast<int64_t>(av[u] ? m0 + row : 0) * K + kbase + (lchunk ^ lrow) * 8;
  }
  const uint16_t* bsrc[BI];
#pragma unroll
  for (int u = 0; u < BI; ++u) {
    const int row = (wave * BI + u) * 8 + lrow;
    bsrc[u] = B + static_cast<int64_t>(n0 + row) * K + kbase + (lchunk ^ lrow) * 8;
  }
  const uint64_t az = reinterpret_cast<uint64_t>(reinterpret_cast<const uint16_t*>(g_gemm_zero) + lchunk * 8);
  const int steps = KS / 64 / KG;                // (K / 64) % KG == 0: every group makes the same k-steps
  const int kstep0 = kg * steps;                 // this group's first k-step
  char* const ring = lds + kg * NS * SB;

  // PRO: the [2][K] scale and shift of the tile's (at most two) workers: rows of worker g0 use entry 0
  extern __shared__ __attribute__((aligned(16))) float ptab[];
  uint32_t pg0 = 0;
  if constexpr (PRO) {
    pg0 = fdiv(static_cast<uint32_t>(m0), pro.frg);
    const uint32_t pg1 = pg0 + 1 < static_cast<uint32_t>(pro.G) ? pg0 + 1 : pg0;
    for (int i = threadIdx.x; i < K; i += 256) {
      ptab[i] = pro.sc[static_cast<int64_t>(pg0) * K + i];
      ptab[K + i] = pro.sc[static_cast<int64_t>(pg1) * K + i];
      ptab[2 * K + i] = pro.sh[static_cast<int64_t>(pg0) * K + i];
      ptab[3 * K + i] = pro.sh[static_cast<int64_t>(pg1) * K + i];
    }
    __syncthreads();   // the table is read by every lane's transforms
  }

  auto issue = [&](int s, int slot) {
    char* base = ring + slot * SB;
    const int k0 = (kstep0 + s) * 64;
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const uint64_t a = reinterpret_cast<uint64_t>(asrc[u] + k0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(av[u] ? a : az),
                                       (lds_ptr)(base + (wave * AI + u) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < BI; ++u)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(bsrc[u] + k0), (lds_ptr)(base + AB + (wave * BI + u) * 1024), 16, 0, 0);
  };

  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[WPM][WPN];
#pragma unroll
  for (int r = 0; r < WPM; ++r)
#pragma unroll
    for (int c = 0; c < WPN; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);

  // stage st has landed (for this lane) when at most (stages issued after it) x PER loads are outstanding
  auto wait_landed = [&](int st, int issued) {
    const int after = issued - 1 - st;
    if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // PRO: this lane's own landed chunks of stage st (published by the barrier at the top of its k-step)
  auto pro_stage = [&](int st) {
    char* sb = lds + (st % NS) * SB;
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const int row = (wave * AI + u) * 8 + lrow;
      if (av[u]) {
        const int sel = fdiv(static_cast<uint32_t>(m0 + row), pro.frg) != pg0 ? 1 : 0;
        const int ch = st * 64 + (lchunk ^ lrow) * 8;
        pro_chunk(sb + (wave * AI + u) * 1024 + lane * 16, ptab + sel * K + ch, ptab + (2 + sel) * K + ch);
      }
    }
  };
  if constexpr (PRO) {
    if (steps > 0) {
      wait_landed(0, steps < NS - 1 ? steps : NS - 1);
      pro_stage(0);
    }
  }

  for (int s = 0; s < steps; ++s) {
    const int issued = s + NS - 1 < steps ? s + NS - 1 : steps;   // stages issued before this k-step
    if constexpr (PRO) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // stage s was transformed last k-step
    else wait_landed(s, issued);
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    const char* base = ring + (s % NS) * SB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = (ks * 4 + fq) ^ (fr & 7);
      bf16x8 wf[WPN], xf[WPM];
#pragma unroll
      for (int c = 0; c < WPN; ++c)
        wf[c] = *reinterpret_cast<const bf16x8*>(base + AB + ((wn * WPN + c) * 16 + fr) * 128 + chunk * 16);
#pragma unroll
      for (int r = 0; r < WPM; ++r)
        xf[r] = *reinterpret_cast<const bf16x8*>(base + ((wm * WPM + r) * 16 + fr) * 128 + chunk * 16);
#pragma unroll
      for (int r = 0; r < WPM; ++r)
#pragma unroll
        for (int c = 0; c < WPN; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[r], acc[r][c], 0, 0, 0);
    }
    // every wave's fragment reads of this slot retire before the barrier that lets it be refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (PRO) {   // the next stage, while the other waves still multiply this one
      if (s + 1 < steps) {
        wait_landed(s + 1, s + NS < steps ? s + NS : steps);
        pro_stage(s + 1);
      }
    }
  }

  if constexpr (EPI == EPI_SPLIT) {   // fp32 partial sums straight from the registers (C is the slab array)
    float* ws = reinterpret_cast<float*>(C) + static_cast<int64_t>(blockIdx.y) * M * N;
#pragma unroll
    for (int r = 0; r < WPM; ++r) {
      const int m = m0 + (wm * WPM + r) * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int c = 0; c < WPN; ++c)
        *reinterpret_cast<f32x4*>(ws + static_cast<int64_t>(m) * N + n0 + (wn * WPN + c) * 16 + 4 * fq) = acc[r][c];
    }
    return;
  }
  // ---- epilogue. The fragments hold 4 channels of one pixel per lane; the tile goes through
  // LDS (bf16, padded row pitch) and leaves as 16-byte-per-lane row segments (whole 128-B
  // lines per 8 lanes). Statistics come from the registers (wave_stats).
  constexpr int TP = BN * 2 + 16;                       // LDS row pitch (bytes)
  constexpr int CPR = BN / 8;                           // 16-byte chunks per tile row
  constexpr int RL = 256 * KG / CPR;                    // tile rows per pass of the workgroup
  static_assert(BM * TP <= NS * SB, "epilogue tile fits the ring");
  __syncthreads();                                      // every wave's last ring reads are done
  if constexpr (KG > 1) {   // the groups' accumulators, summed in group order into group 0's
    constexpr int WB = WPM * WPN * 1024;                // bytes of one wave's accumulators
    if (kg > 0) {
#pragma unroll
      for (int r = 0; r < WPM; ++r)
#pragma unroll
        for (int c = 0; c < WPN; ++c)
          *reinterpret_cast<f32x4*>(lds + ((kg - 1) * 4 + wave) * WB + ((r * WPN + c) * 64 + lane) * 16) = acc[r][c];
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int q = 1; q < KG; ++q)
#pragma unroll
        for (int r = 0; r < WPM; ++r)
#pragma unroll
          for (int c = 0; c < WPN; ++c) {
            const f32x4 o = *reinterpret_cast<const f32x4*>(lds + ((q - 1) * 4 + wave) * WB + ((r * WPN + c) * 64 + lane) * 16);
            acc[r][c][0] += o[0];
            acc[r][c][1] += o[1];
            acc[r][c][2] += o[2];
            acc[r][c][3] += o[3];
          }
    }
    __syncthreads();                                    // the sums are read before the tile reuses the LDS
  }
  if (kg == 0) {
    const int mwl = wm * 16 * WPM;                      // first tile row of this wave
    const int nwl = wn * 16 * WPN + 4 * fq;             // first tile channel of this lane (c = 0)
    float vs[WPM][WPN][4];
#pragma unroll
    for (int r = 0; r < WPM; ++r) {
      const int m = m0 + mwl + r * 16 + fr;
      RowMask<WPN> rm;
      if constexpr (EPI == EPI_ADD)
        if (m < M) rm.load(pro.amask, static_cast<int64_t>(m) * N + n0 + wn * 16 * WPN);
#pragma unroll
      for (int c = 0; c < WPN; ++c) {
        float v[4] = {acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]};
        if constexpr (EPI == EPI_ADD) {                 // one rounding: the sum is formed in fp32
          if (m < M) add_bf16x4(v, add, rm.nib(c, fq), static_cast<int64_t>(m) * N + n0 + nwl + c * 16);
        }
        uint2 o;
        o.x = static_cast<uint32_t>(f_to_bf16(v[0])) | (static_cast<uint32_t>(f_to_bf16(v[1])) << 16);
        o.y = static_cast<uint32_t>(f_to_bf16(v[2])) | (static_cast<uint32_t>(f_to_bf16(v[3])) << 16);
        *reinterpret_cast<uint2*>(lds + (mwl + r * 16 + fr) * TP + (nwl + c * 16) * 2) = o;
        if constexpr (EPI == EPI_STATS) {
          vs[r][c][0] = bf16_to_f(o.x & 0xffffu);
          vs[r][c][1] = bf16_to_f(o.x >> 16);
          vs[r][c][2] = bf16_to_f(o.y & 0xffffu);
          vs[r][c][3] = bf16_to_f(o.y >> 16);
        }
      }
    }
    if constexpr (EPI == EPI_STATS)
      if (m0 + mwl < M) wave_stats<WPM, WPN>(vs, m0 + mwl, M, rg, N, n0 + wn * 16 * WPN, stats);
  }
  __syncthreads();
  const int ck = static_cast<int>(threadIdx.x) % CPR, rl = static_cast<int>(threadIdx.x) / CPR;
  const int rows = M - m0 < BM ? M - m0 : BM;
  for (int rr = rl; rr < rows; rr += RL) {
    const uint4 v = *reinterpret_cast<const uint4*>(lds + rr * TP + ck * 16);
    *reinterpret_cast<uint4*>(C + static_cast<int64_t>(m0 + rr) * N + n0 + ck * 8) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Weight-stationary persistent kernel (K = 64 * KB <= 256)
//
// LDS: [KB][BN][128 B] weights | 2 x [KB][BM][128 B] row-tile ring | 4 x [RW][128 B] wave slices.
// The row tiles are dealt in CHUNKS of `per` consecutive tiles: block b streams N slice
// tn = (b / 8) % tiles_n and chunks p, p + P, ... with p = b % 8 + 8 * (b / (8 * tiles_n)), so
// the tiles_n blocks that read the same row tiles have equal b % 8 (one XCD under the
// round-robin placement; a speed choice only). Tile t + 1 is in flight while tile t is
// multiplied and written.
// EPI_STATS: each wave accumulates, over the whole chunk, the shifted sums Σ(y - s), Σ(y - s)²
// of its stored bf16 values per channel in registers (s: the wave's first stored row of the
// chunk), and reduces them over the 16 lanes of a DPP row only when the chunk (or the worker)
// ends: one statistics tile per chunk (H = per * BM rows), one entry per wave row (E = WM).
template <int BN, int RW, int KB, int EPI, bool PRO>
__global__ __launch_bounds__(256) void k_gemm_ws(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                 int M, int N, uint16_t* __restrict__ C,
                                                 const uint16_t* __restrict__ add, float* __restrict__ stats,
                                                 int64_t rg, int tiles_m, int P, int per, int nchunks, GemmPro pro) {
  constexpr int WN = BN / 64, WM = 4 / WN, BM = WM * RW, WPM = RW / 16, K = KB * 64;
  static_assert(WN * WM == 4 && RW % 16 == 0 && BM % 32 == 0, "4 waves of RW x 64");
  constexpr int BB = BN * K * 2, AB = BM * K * 2, EB = RW * 128;
  constexpr int AI = BM * KB / 32, BI = BN * KB / 32;   // glds per wave: a row tile / the weights
  __shared__ __attribute__((aligned(16))) char lds[BB + 2 * AB + 4 * EB];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_n = N / BN;
  const int b = blockIdx.x;
  const int tn = (b >> 3) % tiles_n;
  const int p = (b & 7) + 8 * (b / (8 * tiles_n));
  if (p >= nchunks) return;                             // whole workgroup: before any barrier
  const int n0 = tn * BN;
  const int lrow = lane >> 3, lchunk = lane & 7;
  char* const el = lds + BB + 2 * AB + wave * EB;
  // PRO: every worker's scale and shift ([2][G][K], dynamic LDS), filled before the first barrier
  extern __shared__ __attribute__((aligned(16))) float ptab[];
  if constexpr (PRO) {
    const int n = pro.G * K;
    for (int i = threadIdx.x; i < n; i += 256) {
      ptab[i] = pro.sc[i];
      ptab[n + i] = pro.sh[i];
    }
    __syncthreads();   // the table is read by every lane's transforms
  }

#pragma unroll
  for (int u = 0; u < BI; ++u) {
    const int q = wave * BI + u, kb = q / (BN / 8), rb = q - kb * (BN / 8);
    const uint16_t* src = B + static_cast<int64_t>(n0 + rb * 8 + lrow) * K + kb * 64 + (lchunk ^ lrow) * 8;
    glds16_asm(src, __builtin_amdgcn_readfirstlane(lds_addr(lds + kb * BN * 128 + rb * 1024)));
  }
  const uint16_t* az = reinterpret_cast<const uint16_t*>(g_gemm_zero) + lchunk * 8;
  auto issue = [&](int tm, int slot) {
    const int m0 = tm * BM;
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const int q = wave * AI + u, kb = q / (BM / 8), rb = q - kb * (BM / 8);
      const int row = m0 + rb * 8 + lrow;
      const uint16_t* src = row < M ? A + static_cast<int64_t>(row) * K + kb * 64 + (lchunk ^ lrow) * 8 : az;
      glds16_asm(src, __builtin_amdgcn_readfirstlane(lds_addr(lds + BB + slot * AB + kb * BM * 128 + rb * 1024)));
    }
  };

  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int nc = n0 + wn * 64;

  // statistics state of this wave (EPI_STATS)
  float sh[4][4] = {}, sd[4][4], sq[4][4];
  int cs = 0, cnt = 0;
  bool have_shift = false;
  int64_t gb = 0, c1 = 0;
  auto reset = [&]() {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) sd[c][i] = sq[c][i] = 0.f;
    cnt = 0;
  };
  auto flush = [&](int T) {
    const float n = static_cast<float>(cnt);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sd[c][i] = row16_sum(sd[c][i]);
        sq[c][i] = row16_sum(sq[c][i]);
      }
    if (fr == 0) {
      float* ps = stats + ((static_cast<int64_t>(T) * WM + wm) * 2 + cs) * 3 * N + nc + 4 * fq;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float sy[4], m2[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sy[i] = sd[c][i] + n * sh[c][i];
          m2[i] = cnt > 0 ? fmaxf(sq[c][i] - sd[c][i] * sd[c][i] / n, 0.f) : 0.f;
        }
        *reinterpret_cast<float4*>(ps + c * 16) = make_float4(n, n, n, n);
        *reinterpret_cast<float4*>(ps + N + c * 16) = make_float4(sy[0], sy[1], sy[2], sy[3]);
        *reinterpret_cast<float4*>(ps + 2 * N + c * 16) = make_float4(m2[0], m2[1], m2[2], m2[3]);
      }
    }
    reset();
  };
  // rows [mlo, mhi) of this wave's tile rows r0 + r*16 + fr join the current slot's sums
  auto accumulate = [&](const uint32_t (&pk)[WPM][4][2], int r0, int64_t mlo, int64_t mhi) {
    const int64_t a = r0 > mlo ? r0 : mlo;
    const int64_t z = r0 + RW < mhi ? r0 + RW : mhi;
    if (z <= a) return;
    cnt += static_cast<int>(z - a);
    const bool full = a == r0 && z == r0 + RW;
#pragma unroll
    for (int r = 0; r < WPM; ++r) {
      const int m = r0 + r * 16 + fr;
      const float w = (full || (m >= mlo && m < mhi)) ? 1.f : 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t h = pk[r][c][i >> 1];
          const float y = bf16_to_f((i & 1) ? (h >> 16) : (h & 0xffffu));
          const float d = (y - sh[c][i]) * w;
          sd[c][i] += d;
          sq[c][i] = fmaf(d, d, sq[c][i]);
        }
    }
  };

  // PRO: this lane's own landed chunks of tile t in slot sl (published by the next loop-top barrier)
  auto pro_tile = [&](int t, int sl) {
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const int q = wave * AI + u, kb = q / (BM / 8), rb = q - kb * (BM / 8);
      const int row = t * BM + rb * 8 + lrow;
      if (row < M) {
        const int g = static_cast<int>(fdiv(static_cast<uint32_t>(row), pro.frg));
        const int ch = kb * 64 + (lchunk ^ lrow) * 8;
        pro_chunk(lds + BB + sl * AB + kb * BM * 128 + rb * 1024 + lane * 16, ptab + g * K + ch,
                  ptab + pro.G * K + g * K + ch);
      }
    }
  };

  int T = p, tm = p * per;
  issue(tm, 0);
  int slot = 0;
  if constexpr (PRO) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pro_tile(tm, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (EPI == EPI_STATS) {
    reset();
    const int64_t c0 = static_cast<int64_t>(T) * per * BM;
    c1 = c0 + static_cast<int64_t>(per) * BM < M ? c0 + static_cast<int64_t>(per) * BM : M;
    gb = (c0 / rg + 1) * rg;
    cs = 0;
    have_shift = false;
  }
  bool first = true;
  while (true) {
    // this tile's rows (and the weights) have landed for every wave; every wave is done
    // reading the other slot (the previous tile), which is refilled next. The LDS-DMA is inline asm
    // (glds16_asm), so these waits are the only ones for it: after the first tile, the previous
    // epilogue's RW / 8 row stores (issued after this tile's loads and counted with them, in issue
    // order) stay in flight (ab_gemm_ws.py: bit-identical, ImageNet-size statistics GEMMs 20-30 %
    // faster than with the builtin, whose tracking drained the prefetch before every epilogue)
    if (!first) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RW / 8) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    first = false;
    __builtin_amdgcn_s_barrier();
    int T2 = T, tm2 = tm + 1;
    const int cend = (T + 1) * per < tiles_m ? (T + 1) * per : tiles_m;
    if (tm2 >= cend) {
      T2 = T + P;
      tm2 = T2 * per;
    }
    const bool more = T2 < nchunks;
    // EPI_ADD: this tile's addend (and mask bits) loaded BEFORE the next tile's LDS-DMA, by inline asm,
    // and waited for by count below: the DMA issued after them stays in flight through the epilogue
    u32x2 av[WPM][4], mv[WPM];
    if constexpr (EPI == EPI_ADD) {
#pragma unroll
      for (int r = 0; r < WPM; ++r) {
        const int m = tm * BM + wm * RW + r * 16 + fr;
        const int64_t e = static_cast<int64_t>(m < M ? m : 0) * N + nc;   // rows past M: any valid row
        // unconditional (a branch around an asm load makes hipcc copy its register before it lands):
        // without a mask the addend's own first bytes stand in, and are ignored
        mv[r] = ld8_asm(pro.amask ? static_cast<const void*>(pro.amask + (e >> 3)) : static_cast<const void*>(add + e));
#pragma unroll
        for (int c = 0; c < 4; ++c) av[r][c] = ld8_asm(add + e + c * 16 + 4 * fq);
      }
    }
    if (more) issue(tm2, slot ^ 1);
    f32x4 acc[WPM][4];
#pragma unroll
    for (int r = 0; r < WPM; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* as = lds + BB + slot * AB;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int chunk = (ks * 4 + fq) ^ (fr & 7);
        bf16x8 wf[4], xf[WPM];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          wf[c] = *reinterpret_cast<const bf16x8*>(lds + kb * BN * 128 + (wn * 64 + c * 16 + fr) * 128 + chunk * 16);
#pragma unroll
        for (int r = 0; r < WPM; ++r)
          xf[r] = *reinterpret_cast<const bf16x8*>(as + kb * BM * 128 + (wm * RW + r * 16 + fr) * 128 + chunk * 16);
#pragma unroll
        for (int r = 0; r < WPM; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[r], acc[r][c], 0, 0, 0);
      }

    // ---- wave-private epilogue: rows r0 .. r0 + RW, channels nc .. nc + 64
    const int r0 = tm * BM + wm * RW;
    if constexpr (EPI == EPI_ADD) {   // the addend loads: only the next tile's AI DMA ops are younger
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int r = 0; r < WPM; ++r) {
        asm volatile("" : "+v"(mv[r]));
#pragma unroll
        for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(av[r][c]));
      }
    }
    uint32_t pk[WPM][4][2];
#pragma unroll
    for (int r = 0; r < WPM; ++r) {
      const int rr = r * 16 + fr;
      RowMask<4> rm;
      if constexpr (EPI == EPI_ADD) {
        rm.w[0] = pro.amask ? mv[r].x : 0xffffffffu;
        rm.w[1] = pro.amask ? mv[r].y : 0xffffffffu;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float v[4] = {acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]};
        if constexpr (EPI == EPI_ADD) {
          const uint32_t keep = rm.nib(c, fq);
          v[0] += (keep & 1u) ? bf16_to_f(av[r][c].x & 0xffffu) : 0.f;
          v[1] += (keep & 2u) ? bf16_to_f(av[r][c].x >> 16) : 0.f;
          v[2] += (keep & 4u) ? bf16_to_f(av[r][c].y & 0xffffu) : 0.f;
          v[3] += (keep & 8u) ? bf16_to_f(av[r][c].y >> 16) : 0.f;
        }
        pk[r][c][0] = pack_bf16x2(v[0], v[1]);
        pk[r][c][1] = pack_bf16x2(v[2], v[3]);
        const int ch16 = (c * 2 + (fq >> 1)) ^ (rr & 7);                // swizzled 16-B chunk of the row
        *reinterpret_cast<uint2*>(el + rr * 128 + ch16 * 16 + (fq & 1) * 8) = make_uint2(pk[r][c][0], pk[r][c][1]);
      }
    }
    // LDS accesses of one wave execute in order: the slice written above is read back
    // whole-line by the same wave (compiler ordering pinned by the clobber)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < RW / 8; ++it) {
      const int rr = it * 8 + lrow;
      const uint4 v = *reinterpret_cast<const uint4*>(el + rr * 128 + ((lchunk ^ (rr & 7)) * 16));
      if (r0 + rr < M) *reinterpret_cast<uint4*>(C + static_cast<int64_t>(r0 + rr) * N + nc + lchunk * 8) = v;
    }

    if constexpr (EPI == EPI_STATS) {
      if (!have_shift && r0 < M) {                      // the wave's first stored row of the chunk
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t h = pk[0][c][i >> 1];
            const float y = bf16_to_f((i & 1) ? (h >> 16) : (h & 0xffffu));
            sh[c][i] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y), 0x150,
                                                                             0xF, 0xF, false));   // row_newbcast:0
          }
        have_shift = true;
      }
      if (cs == 0) {
        const int64_t hi0 = gb < c1 ? gb : c1;
        accumulate(pk, r0, static_cast<int64_t>(T) * per * BM, hi0);
        if (gb < c1 && r0 + RW > gb) {                  // the worker boundary falls in this tile
          flush(T);
          cs = 1;
        }
      }
      if (cs == 1) accumulate(pk, r0, gb, c1);
      if (T2 != T || !more) {                           // chunk ends: its last slot
        flush(T);
        if (gb < c1 && cs == 0) {                       // a straddling chunk whose second worker's
          cs = 1;                                       // rows this wave never held: n = 0 entry
          flush(T);
        }
        if (more) {
          const int64_t c0 = static_cast<int64_t>(T2) * per * BM;
          c1 = c0 + static_cast<int64_t>(per) * BM < M ? c0 + static_cast<int64_t>(per) * BM : M;
          gb = (c0 / rg + 1) * rg;
          cs = 0;
          have_shift = false;
        }
      }
    }
    if (!more) break;
    if constexpr (PRO) {   // the next tile, while the other waves still finish this one
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pro_tile(tm2, slot ^ 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    T = T2;
    tm = tm2;
    slot ^= 1;
  }
}

// Merge of one worker's tile statistics (Chan et al.): 16 channels x 64 lanes per workgroup,
// each lane folding every 64th (tile, entry) of the worker (four loads in flight before they are
// used), the 64 lane partials merged by a fixed-order tree in LDS (deterministic).
constexpr int kMergeCh = 16, kMergeLanes = 64;

__device__ __forceinline__ void chan_merge(float& n, float& mu, float& m2, float nb, float mub, float m2b) {
  if (nb <= 0.f) return;
  const float nn = n + nb;
  const float d = mub - mu;
  mu += d * (nb / nn);
  m2 += m2b + d * d * (n * nb / nn);
  n = nn;
}

__global__ __launch_bounds__(kMergeCh * kMergeLanes) void k_finalize_tiles(
    const float* __restrict__ stats, int H, int E, int64_t M, int64_t rg, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ mean, float* __restrict__ istd,
    float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float sn[kMergeLanes][kMergeCh], smu[kMergeLanes][kMergeCh], sm2[kMergeLanes][kMergeCh];
  const int tc = threadIdx.x % kMergeCh, lane = threadIdx.x / kMergeCh;
  const int c = blockIdx.x * kMergeCh + tc;
  const int g = blockIdx.y;
  const int64_t g0 = static_cast<int64_t>(g) * rg, g1 = g0 + rg < M ? g0 + rg : M;
  const int64_t t_lo = g0 / H, t_hi = (g1 - 1) / H;
  const int nent = static_cast<int>((t_hi - t_lo + 1) * E);   // (tile, entry) pairs of this worker
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C) {
    for (int i0 = lane; i0 < nent; i0 += kMergeLanes * 4) {   // 32-bit index math (no 64-bit divisions)
      float sv[4], qv[4], nv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * kMergeLanes;
        nv[u] = 0.f;
        sv[u] = qv[u] = 0.f;
        if (i < nent) {
          const int q = i / E;
          const int64_t t = t_lo + q, e = i - q * E;
          const int slot = t * H < g0 ? 1 : 0;          // the tile started in the previous worker
          const float* p = stats + ((t * E + e) * 2 + slot) * 3 * C + c;
          nv[u] = p[0];
          sv[u] = p[C];
          qv[u] = p[2 * C];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) chan_merge(n, mu, m2, nv[u], nv[u] > 0.f ? sv[u] / nv[u] : 0.f, qv[u]);
    }
  }
  sn[lane][tc] = n;
  smu[lane][tc] = mu;
  sm2[lane][tc] = m2;
  __syncthreads();
#pragma unroll
  for (int h = kMergeLanes / 2; h >= 1; h >>= 1) {
    if (lane < h) {
      float a = sn[lane][tc], b = smu[lane][tc], q = sm2[lane][tc];
      chan_merge(a, b, q, sn[lane + h][tc], smu[lane + h][tc], sm2[lane + h][tc]);
      sn[lane][tc] = a;
      smu[lane][tc] = b;
      sm2[lane][tc] = q;
    }
    __syncthreads();
  }
  if (lane != 0 || c >= C) return;
  const float N0 = sn[0][tc], MU = smu[0][tc], M2 = sm2[0][tc];
  float var = N0 > 0.f ? M2 / N0 : 0.f;
  var = var > 0.f ? var : 0.f;
  const float is = rsqrtf(var + eps);
  const int64_t gc = static_cast<int64_t>(g) * C + c;
  mean[gc] = MU;
  istd[gc] = is;
  const float sc = (gamma ? gamma[c] : 1.f) * is;
  scale[gc] = sc;
  shift[gc] = (beta ? beta[c] : 0.f) - MU * sc;
}

// C[i] = bf16(Σ_s ws[s][i] (+ add[i], masked by amask when given)), 8 elements per thread
template <bool ADD>
__global__ __launch_bounds__(256) void k_split_sum(const float* __restrict__ ws, int S, int64_t n8,
                                                   uint16_t* __restrict__ C, const uint16_t* __restrict__ add,
                                                   const uint8_t* __restrict__ amask) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  float v[8];
  const float4 a0 = reinterpret_cast<const float4*>(ws)[2 * i], a1 = reinterpret_cast<const float4*>(ws)[2 * i + 1];
  v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
  for (int s = 1; s < S; ++s) {
    const float4* p = reinterpret_cast<const float4*>(ws + static_cast<int64_t>(s) * n8 * 8) + 2 * i;
    const float4 b0 = p[0], b1 = p[1];
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  if constexpr (ADD) {
    const uint4 u = reinterpret_cast<const uint4*>(add)[i];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    const uint32_t keep = amask ? static_cast<uint32_t>(amask[i]) : 0xffu;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] += ((keep >> e) & 1u) ? bf16_to_f((e & 1) ? (w[e >> 1] >> 16) : (w[e >> 1] & 0xffffu)) : 0.f;
  }
  reinterpret_cast<uint4*>(C)[i] = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                              pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}

template <int WPM, int WPN, int WM, int WN, int NS>
void launch_split(const uint16_t* A, const uint16_t* B, int M, int N, int K, uint16_t* C, const uint16_t* add,
                  const uint8_t* amask, float* ws, int S, hipStream_t stream) {
  constexpr int BM = 16 * WPM * WM, BN = 16 * WPN * WN;
  const dim3 grid(((M + BM - 1) / BM) * (N / BN), S);
  hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_SPLIT, false>), grid, dim3(256), 0, stream, A, B, M, N, K,
                     reinterpret_cast<uint16_t*>(ws), nullptr, nullptr, int64_t{0}, GemmPro{});
  const int64_t n8 = static_cast<int64_t>(M) * N / 8;
  const dim3 g2(static_cast<unsigned>((n8 + 255) / 256));
  if (add) hipLaunchKernelGGL((k_split_sum<true>), g2, dim3(256), 0, stream, ws, S, n8, C, add, amask);
  else hipLaunchKernelGGL((k_split_sum<false>), g2, dim3(256), 0, stream, ws, S, n8, C, add, amask);
}

template <int WPM, int WPN, int WM, int WN, int NS, int KG = 1>
void launch_cfg(const uint16_t* A, const uint16_t* B, int M, int N, int K, uint16_t* C, const uint16_t* add,
                float* stats, int64_t rg, hipStream_t stream, const GemmPro& pro) {
  constexpr int BM = 16 * WPM * WM, BN = 16 * WPN * WN;
  const dim3 grid(((M + BM - 1) / BM) * (N / BN));
  if constexpr (KG > 1) {   // in-workgroup split-K: 256 * KG threads, the KG rings in dynamic LDS
    constexpr int lds = KG * NS * (BM + BN) * 128;
    static_assert(lds <= 160 * 1024, "LDS");
    static bool once = (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_STATS, false, KG>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, lds),
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_ADD, false, KG>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, lds),
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_PLAIN, false, KG>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, lds),
                        true);
    (void)once;
    if (stats)
      hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_STATS, false, KG>), grid, dim3(256 * KG), lds, stream, A, B,
                         M, N, K, C, add, stats, rg, pro);
    else if (add)
      hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_ADD, false, KG>), grid, dim3(256 * KG), lds, stream, A, B,
                         M, N, K, C, add, stats, rg, pro);
    else
      hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_PLAIN, false, KG>), grid, dim3(256 * KG), lds, stream, A, B,
                         M, N, K, C, add, stats, rg, pro);
    return;
  }
  if (pro.sc) {   // forward of a 1x1 convolution over a pre-BatchNorm input (plain or statistics epilogue)
    const size_t tab = static_cast<size_t>(4) * K * sizeof(float);
    if (stats)
      hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_STATS, true>), grid, dim3(256), tab, stream, A, B, M, N,
                         K, C, add, stats, rg, pro);
    else
      hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_PLAIN, true>), grid, dim3(256), tab, stream, A, B, M, N,
                         K, C, add, stats, rg, pro);
    return;
  }
  if (stats)
    hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_STATS, false>), grid, dim3(256), 0, stream, A, B, M, N, K,
                       C, add, stats, rg, pro);
  else if (add)
    hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_ADD, false>), grid, dim3(256), 0, stream, A, B, M, N, K, C,
                       add, stats, rg, pro);
  else
    hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_PLAIN, false>), grid, dim3(256), 0, stream, A, B, M, N, K,
                       C, add, stats, rg, pro);
}

constexpr int ws_bm(int BN, int RW) { return (4 / (BN / 64)) * RW; }
constexpr int ws_lds(int BN, int RW, int KB) { return BN * KB * 128 + 2 * ws_bm(BN, RW) * KB * 128 + 4 * RW * 128; }
constexpr int ws_occ(int lds) { return (160 * 1024) / lds >= 2 ? 2 : 1; }

// Chunking of a weight-stationary launch: P persistent blocks per N slice (a multiple of 8),
// chunks of `per` row tiles; with statistics (rg > 0) a chunk spans at most rg rows.
struct WsPlan {
  int P, per, nchunks, tiles_m, bm;
};
WsPlan ws_plan(int BN, int RW, int KB, int64_t M, int N, int64_t rg) {
  WsPlan w{};
  w.bm = ws_bm(BN, RW);
  w.tiles_m = static_cast<int>((M + w.bm - 1) / w.bm);
  const int tiles_n = N / BN;
  const int P0 = (256 * ws_occ(ws_lds(BN, RW, KB)) + tiles_n - 1) / tiles_n;
  w.per = (w.tiles_m + P0 - 1) / P0;
  if (rg > 0) {
    const int cap = static_cast<int>(rg / w.bm);
    w.per = w.per < cap ? w.per : cap;
  }
  if (w.per < 1) w.per = 1;
  w.nchunks = (w.tiles_m + w.per - 1) / w.per;
  const int P = w.nchunks < P0 ? w.nchunks : P0;
  w.P = (P + 7) / 8 * 8;
  return w;
}

template <int BN, int RW, int KB>
void launch_ws(const uint16_t* A, const uint16_t* B, int M, int N, uint16_t* C, const uint16_t* add, float* stats,
               int64_t rg, hipStream_t stream, const GemmPro& pro) {
  static_assert(ws_lds(BN, RW, KB) <= 160 * 1024, "LDS");
  const WsPlan w = ws_plan(BN, RW, KB, M, N, stats ? rg : 0);
  const dim3 grid(w.P * (N / BN));
  if (pro.sc) {
    const size_t tab = static_cast<size_t>(2) * pro.G * KB * 64 * sizeof(float);
    if (stats)
      hipLaunchKernelGGL((k_gemm_ws<BN, RW, KB, EPI_STATS, true>), grid, dim3(256), tab, stream, A, B, M, N, C, add,
                         stats, rg, w.tiles_m, w.P, w.per, w.nchunks, pro);
    else
      hipLaunchKernelGGL((k_gemm_ws<BN, RW, KB, EPI_PLAIN, true>), grid, dim3(256), tab, stream, A, B, M, N, C, add,
                         stats, rg, w.tiles_m, w.P, w.per, w.nchunks, pro);
    return;
  }
  if (stats)
    hipLaunchKernelGGL((k_gemm_ws<BN, RW, KB, EPI_STATS, false>), grid, dim3(256), 0, stream, A, B, M, N, C, add, stats,
                       rg, w.tiles_m, w.P, w.per, w.nchunks, pro);
  else if (add)
    hipLaunchKernelGGL((k_gemm_ws<BN, RW, KB, EPI_ADD, false>), grid, dim3(256), 0, stream, A, B, M, N, C, add, stats,
                       rg, w.tiles_m, w.P, w.per, w.nchunks, pro);
  else
    hipLaunchKernelGGL((k_gemm_ws<BN, RW, KB, EPI_PLAIN, false>), grid, dim3(256), 0, stream, A, B, M, N, C, add, stats,
                       rg, w.tiles_m, w.P, w.per, w.nchunks, pro);
}

template <int BN, int RW>
void launch_ws_k(int K, const uint16_t* A, const uint16_t* B, int M, int N, uint16_t* C, const uint16_t* add,
                 float* stats, int64_t rg, hipStream_t stream, const GemmPro& pro) {
  switch (K) {
    case 64: launch_ws<BN, RW, 1>(A, B, M, N, C, add, stats, rg, stream, pro); break;
    case 128: launch_ws<BN, RW, 2>(A, B, M, N, C, add, stats, rg, stream, pro); break;
    default:
      if constexpr (BN <= 128 && ws_lds(BN, RW, 4) <= 160 * 1024)
        launch_ws<BN, RW, 4>(A, B, M, N, C, add, stats, rg, stream, pro);
      break;
  }
}

// tile configurations: K-loop {BM, BN, stats rows} 0..8, weight-stationary {BN, RW} 9..14
constexpr int kNumNt = 9;
constexpr int kCfgBM[] = {128, 256, 64, 64, 64, 128, 128, 64, 32};
constexpr int kCfgBN[] = {128, 64, 128, 256, 64, 256, 128, 64, 256};
constexpr int kCfgSR[] = {64, 64, 32, 64, 32, 64, 64, 32, 32};
constexpr int kWsBN[] = {256, 256, 128, 128, 64, 64};
constexpr int kWsRW[] = {32, 64, 16, 32, 16, 32};
constexpr int kNumBase = kNumNt + 6;
constexpr int kSplits[] = {2, 4};                       // split-K variants of the K-loop configurations
constexpr int kNumSplit = kNumBase + 2 * kNumNt;        // first in-workgroup split-K configuration
// in-workgroup split-K variants (k_gemm_nt KG): {K-loop configuration, K groups}
constexpr int kKgBase[] = {7, 7, 4, 2, 8};
constexpr int kKgK[] = {2, 4, 2, 2, 2};
constexpr int kNumCfg = kNumSplit + 5;
// configuration -> (K-loop configuration, splits, K groups); 1 / 1 for the base configurations
inline int split_of(int cfg) { return cfg >= kNumBase && cfg < kNumSplit ? kSplits[(cfg - kNumBase) / kNumNt] : 1; }
inline int kg_of(int cfg) { return cfg >= kNumSplit && cfg < kNumCfg ? kKgK[cfg - kNumSplit] : 1; }
inline int base_of(int cfg) {
  if (cfg >= kNumSplit) return kKgBase[cfg - kNumSplit];
  return cfg >= kNumBase ? (cfg - kNumBase) % kNumNt : cfg;
}

bool ws_fits(int i, int K) {
  const int kb = K / 64;
  if (K % 64 || kb < 1 || kb > 4 || kb == 3) return false;
  if (kWsBN[i] * K * 2 > 64 * 1024) return false;     // the weight slice stays <= 64 KB of LDS
  return ws_lds(kWsBN[i], kWsRW[i], kb) <= 160 * 1024;
}

// ---------------------------------------------------------------------------------------------
// Transposes of many bf16 matrices in one launch: dst_j [C_j, R_j] = src_j [R_j, C_j]ᵀ (the
// data-gradient GEMMs' B = Wᵀ of every 1x1 convolution, refreshed once per step). 64 x 64 tiles
// through LDS (padded pitch), 16-byte loads and stores; R_j, C_j multiples of 8.
// taps > 1: src is [R][taps][C] and dst [C][taps][R] with the taps reversed, dst[c][T-1-t][r] =
// src[r][t][c]: the flipped, transposed weight of a k x k convolution's data gradient.
struct TJob {
  const uint16_t* src;
  uint16_t* dst;
  int R, C;
  int taps;
  int tile0;               // first tile of this job in the launch
};
constexpr int kTJobs = 40;
struct TTable {
  TJob j[kTJobs];
  int n;
};

__global__ __launch_bounds__(256) void k_transpose_multi(TTable t) {
  __shared__ uint16_t tile[64][64 + 8];
  int ji = 0;
  while (ji + 1 < t.n && static_cast<int>(blockIdx.x) >= t.j[ji + 1].tile0) ++ji;
  const TJob jb = t.j[ji];
  const int tcol = (jb.C + 63) / 64;
  const int per_tap = ((jb.R + 63) / 64) * tcol;
  const int tap = (blockIdx.x - jb.tile0) / per_tap;
  const int tl = blockIdx.x - jb.tile0 - tap * per_tap;
  const int r0 = (tl / tcol) * 64, c0 = (tl % tcol) * 64;
  const int64_t sld = static_cast<int64_t>(jb.taps) * jb.C, dld = static_cast<int64_t>(jb.taps) * jb.R;
  const uint16_t* src = jb.src + static_cast<int64_t>(tap) * jb.C;
  uint16_t* dst = jb.dst + static_cast<int64_t>(jb.taps - 1 - tap) * jb.R;
  const int lr = threadIdx.x >> 3, lc = (threadIdx.x & 7) * 8;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int r = r0 + lr + 32 * k, c = c0 + lc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < jb.R && c < jb.C) v = *reinterpret_cast<const uint4*>(src + r * sld + c);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[lr + 32 * k][lc + 2 * e] = static_cast<uint16_t>(w[e] & 0xffffu);
      tile[lr + 32 * k][lc + 2 * e + 1] = static_cast<uint16_t>(w[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = c0 + lr + 32 * k, r = r0 + lc;     // dst row c, columns r .. r + 8
    if (c < jb.C && r < jb.R) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = static_cast<uint32_t>(tile[lc + 2 * e][lr + 32 * k]) |
               (static_cast<uint32_t>(tile[lc + 2 * e + 1][lr + 32 * k]) << 16);
      *reinterpret_cast<uint4*>(dst + c * dld + r) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

}  // namespace

void transpose_multi(const uint16_t* const* srcs, uint16_t* const* dsts, const int* R, const int* C, int count,
                     hipStream_t stream, const int* taps) {
  for (int b = 0; b < count; b += kTJobs) {
    TTable t{};
    int tiles = 0;
    t.n = count - b < kTJobs ? count - b : kTJobs;
    for (int i = 0; i < t.n; ++i) {
      const int tp = taps ? taps[b + i] : 1;
      t.j[i] = TJob{srcs[b + i], dsts[b + i], R[b + i], C[b + i], tp, tiles};
      tiles += tp * ((R[b + i] + 63) / 64) * ((C[b + i] + 63) / 64);
    }
    if (tiles > 0) hipLaunchKernelGGL(k_transpose_multi, dim3(tiles), dim3(256), 0, stream, t);
  }
}

int gemm_nt_num_cfg() { return kNumCfg; }

// The BatchNorm-prologue form of configuration cfg: its LDS (ring + scale / shift table) fits, and a
// K-loop tile spans at most two workers (BM <= rows per worker)
bool gemm_nt_pro_ok(int cfg, int K, int64_t prg, int groups) {
  if (cfg < 0 || cfg >= kNumBase || prg <= 0 || prg >= (int64_t{1} << 31)) return false;
  if (cfg < kNumNt) return kCfgBM[cfg] <= prg && static_cast<int64_t>(4) * K * 4 <= 32 * 1024;
  const int i = cfg - kNumNt;
  const int64_t tab = static_cast<int64_t>(2) * groups * K * 4;   // dynamic LDS: <= 64 KB without an attribute
  return ws_fits(i, K) && tab <= 64 * 1024 && ws_lds(kWsBN[i], kWsRW[i], K / 64) + tab <= 160 * 1024;
}

bool gemm_nt_valid(int cfg, int N, int K) {
  if (cfg < 0 || cfg >= kNumCfg || K % 64 || K <= 0) return false;
  if (cfg >= kNumSplit) return K % (64 * kg_of(cfg)) == 0 && N % kCfgBN[base_of(cfg)] == 0;
  if (cfg >= kNumBase) return K % (64 * split_of(cfg)) == 0 && N % kCfgBN[base_of(cfg)] == 0 && N % 8 == 0;
  if (cfg < kNumNt) return N % kCfgBN[cfg] == 0;
  return N % kWsBN[cfg - kNumNt] == 0 && ws_fits(cfg - kNumNt, K);
}

int gemm_nt_splits(int cfg) { return cfg >= 0 && cfg < kNumCfg ? split_of(cfg) : 1; }

int gemm_nt_tile_m(int cfg) {
  if (cfg >= kNumBase && cfg < kNumCfg) return kCfgBM[base_of(cfg)];
  if (cfg >= 0 && cfg < kNumNt) return kCfgBM[cfg];
  if (cfg >= kNumNt && cfg < kNumCfg) return (4 / (kWsBN[cfg - kNumNt] / 64)) * kWsRW[cfg - kNumNt];
  return 0;
}
int gemm_nt_tile_n(int cfg) {
  if (cfg >= kNumBase && cfg < kNumCfg) return kCfgBN[base_of(cfg)];
  if (cfg >= 0 && cfg < kNumNt) return kCfgBN[cfg];
  if (cfg >= kNumNt && cfg < kNumCfg) return kWsBN[cfg - kNumNt];
  return 0;
}
int gemm_nt_stats_rows(int cfg) {
  if (cfg >= kNumSplit && cfg < kNumCfg) return kCfgSR[base_of(cfg)];   // in-workgroup split-K: as its base
  if (cfg >= kNumBase) return 1 << 30;   // split-K forms have no statistics epilogue
  if (cfg >= 0 && cfg < kNumNt) return kCfgSR[cfg];
  if (cfg >= kNumNt && cfg < kNumCfg) return ws_bm(kWsBN[cfg - kNumNt], kWsRW[cfg - kNumNt]);
  return 0;
}

void gemm_nt_stats_geometry(int cfg, int64_t M, int N, int K, int64_t rg, int64_t* H, int* E) {
  if ((cfg >= 0 && cfg < kNumNt) || (cfg >= kNumSplit && cfg < kNumCfg)) {
    *H = kCfgSR[base_of(cfg)];
    *E = 1;
    return;
  }
  const int i = cfg - kNumNt;
  const WsPlan w = ws_plan(kWsBN[i], kWsRW[i], K / 64, M, N, rg);
  *H = static_cast<int64_t>(w.per) * w.bm;
  *E = 4 / (kWsBN[i] / 64);
}

int gemm_nt_pick(int64_t M, int N, int K, int64_t rg_limit) {
  // K <= 256: the weight-stationary kernel, widest weight slice, then the row height whose
  // LDS admits two workgroups per CU where there is one
  if (K <= 256) {
    int best = -1, best_occ = 0;
    for (int i = 0; i < 6; ++i) {
      const int cfg = kNumNt + i;
      if (!gemm_nt_valid(cfg, N, K) || (rg_limit > 0 && ws_bm(kWsBN[i], kWsRW[i]) > rg_limit)) continue;
      if (best >= 0 && kWsBN[i] < kWsBN[best - kNumNt]) break;
      const int occ = (160 * 1024) / ws_lds(kWsBN[i], kWsRW[i], K / 64) >= 2 ? 2 : 1;
      if (best < 0 || occ > best_occ || (occ == best_occ && kWsRW[i] > kWsRW[best - kNumNt] && M >= 32000)) {
        best = cfg;
        best_occ = occ;
      }
    }
    if (best >= 0) return best;
  }
  // K-loop: largest tile that still gives >= 512 workgroups (2 per CU); BN never above N;
  // with statistics a wave's stats tile must not span more than two workers
  static const int order[] = {5, 0, 1, 3, 2, 4};
  int best = -1;
  int64_t best_wg = -1;
  for (int cfg : order) {
    const int bm = kCfgBM[cfg], bn = kCfgBN[cfg];
    if (N % bn != 0 || (rg_limit > 0 && kCfgSR[cfg] > rg_limit)) continue;
    const int64_t wg = ((M + bm - 1) / bm) * (N / bn);
    if (wg >= 512) return cfg;
    if (wg > best_wg) { best_wg = wg; best = cfg; }
  }
  return best;
}

void gemm_nt(const uint16_t* A, const uint16_t* B, int M, int N, int K, uint16_t* C, const uint16_t* add,
             float* stats, int64_t rg, int cfg, hipStream_t stream, const float* pro_scale, const float* pro_shift,
             int64_t pro_rg, int pro_groups, float* split_ws, const uint8_t* add_mask) {
  if (M <= 0) return;
  if (cfg >= kNumSplit) {   // in-workgroup split-K (no prologue)
    GemmPro pk{};
    pk.amask = add ? add_mask : nullptr;
    switch (cfg - kNumSplit) {
      case 0: launch_cfg<2, 2, 2, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream, pk); break;
      case 1: launch_cfg<2, 2, 2, 2, 2, 4>(A, B, M, N, K, C, add, stats, rg, stream, pk); break;
      case 2: launch_cfg<2, 2, 2, 2, 4, 2>(A, B, M, N, K, C, add, stats, rg, stream, pk); break;
      case 3: launch_cfg<2, 4, 2, 2, 3, 2>(A, B, M, N, K, C, add, stats, rg, stream, pk); break;
      default: launch_cfg<2, 4, 1, 4, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream, pk); break;
    }
    return;
  }
  if (cfg >= kNumBase) {   // split-K (no statistics, no prologue; the caller provides the fp32 slabs)
    const int S = split_of(cfg);
    switch (base_of(cfg)) {
      case 0: launch_split<4, 4, 2, 2, 2>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 6: launch_split<4, 4, 2, 2, 3>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 7: launch_split<2, 2, 2, 2, 2>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 8: launch_split<2, 4, 1, 4, 2>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 1: launch_split<4, 4, 4, 1, 2>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 2: launch_split<2, 4, 2, 2, 3>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 3: launch_split<4, 4, 1, 4, 2>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      case 4: launch_split<2, 2, 2, 2, 4>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
      default: launch_split<4, 8, 2, 2, 2>(A, B, M, N, K, C, add, add_mask, split_ws, S, stream); break;
    }
    return;
  }
  GemmPro pro{};
  pro.amask = add ? add_mask : nullptr;
  if (pro_scale) {
    pro.sc = pro_scale;
    pro.sh = pro_shift;
    pro.frg = make_fastdiv(static_cast<uint32_t>(pro_rg));
    pro.G = pro_groups;
  }
  switch (cfg) {
    case 0: launch_cfg<4, 4, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 6: launch_cfg<4, 4, 2, 2, 3>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 7: launch_cfg<2, 2, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 8: launch_cfg<2, 4, 1, 4, 2>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 1: launch_cfg<4, 4, 4, 1, 2>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 2: launch_cfg<2, 4, 2, 2, 3>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 3: launch_cfg<4, 4, 1, 4, 2>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 4: launch_cfg<2, 2, 2, 2, 4>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 5: launch_cfg<4, 8, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream, pro); break;
    case 9: launch_ws_k<256, 32>(K, A, B, M, N, C, add, stats, rg, stream, pro); break;
    case 10: launch_ws_k<256, 64>(K, A, B, M, N, C, add, stats, rg, stream, pro); break;
    case 11: launch_ws_k<128, 16>(K, A, B, M, N, C, add, stats, rg, stream, pro); break;
    case 12: launch_ws_k<128, 32>(K, A, B, M, N, C, add, stats, rg, stream, pro); break;
    case 13: launch_ws_k<64, 16>(K, A, B, M, N, C, add, stats, rg, stream, pro); break;
    default: launch_ws_k<64, 32>(K, A, B, M, N, C, add, stats, rg, stream, pro); break;
  }
}

void bn_finalize_tiles(const float* stats, int64_t H, int E, int64_t M, int64_t rg, int groups, int C,
                       const float* gamma, const float* beta, float eps, float* mean, float* istd, float* scale,
                       float* shift, hipStream_t stream) {
  const dim3 grid((C + kMergeCh - 1) / kMergeCh, groups);
  hipLaunchKernelGGL(k_finalize_tiles, grid, dim3(kMergeCh * kMergeLanes), 0, stream, stats, static_cast<int>(H), E, M,
                     rg, C, gamma, beta, eps, mean, istd, scale, shift);
}

}  // namespace gpu
}  // namespace garfield
