// Bulyan's coordinate-wise tail for n <= 64 gradients (every dtype).
//
// Input: the t x n selection matrix W of bulyan_select (row k = uniform weights
// 1/(m-k) over the set S_k chosen at step k). Output per coordinate: the mean of
// the beta values closest to the median of the t selection means
// (reference: py_bulyan/bulyan.cu:227-243, 256-322).
//
// The previous form gathered every mean from scratch: sum_k |S_k| ~ t*m LDS reads
// and FMAs per coordinate (1,764 at n = 64, f = 3). Consecutive sets differ by a
// few gradients, so here the means are built INCREMENTALLY: each set S_k is a
// 64-bit mask (kept in LDS, read as wave-uniform SGPRs), the running sum adds
// S_k \ S_{k-1} and subtracts S_{k-1} \ S_k with scalar bit loops (about m + 2t
// LDS reads). A coordinate whose running sum turns non-finite (inf - inf) is
// recomputed exactly with direct per-set sums (divergent, rare).
//
// The t means are sorted with an odd-even merge network in registers; the beta
// closest to the median form a window [a, a + beta) of the sorted values, whose
// start a is found from the e = t - beta smallest and largest values (no second
// sort by distance, unlike the generic closest_mean).
#pragma once
#include <cstdlib>
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
namespace coord {
using namespace dev;

// fp32 <-> order-preserving int32 key (NaN already mapped to +inf): integer
// min/max need no NaN canonicalisation of their inputs, unlike fminf/fmaxf
__device__ __forceinline__ int f32_key(float f) {
  const int b = __float_as_int(f);
  return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float key_f32(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }

template <int NP>
__device__ __forceinline__ void oem_sort_i32(int (&v)[NP]) {
#pragma unroll
  for (int p = 1; p < NP; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < NP; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k; ++i) {
          if (i + j + k < NP && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const int a = v[i + j], b = v[i + j + k];
            v[i + j] = min(a, b);
            v[i + j + k] = max(a, b);
          }
        }
      }
    }
  }
}

// volatile read of a __shared__ object through an LDS-typed pointer (a generic volatile
// pointer would become a system-coherent FLAT load)
template <typename T>
__device__ __forceinline__ T lds_volatile(const T& x) {
  typedef __attribute__((address_space(3))) const volatile T lds_t;
  return *(lds_t*)(&x);
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

constexpr int kTailTile = 256;
constexpr int kTailMaxExcluded = 16;  // e = t - beta <= 16 (host checks; larger e: generic kernel)

template <int DT, int NP, bool DIRECT>
__global__ __launch_bounds__(256) void k_bulyan_tail(RowTable rows, int n, int64_t d, int beta,
                                                     const float* __restrict__ W, int t, void* out, int out_dt) {
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  constexpr int CPR = kTailTile * ESZ / 16;  // 16-byte chunks per tile row
  __shared__ __align__(16) unsigned char tile[64 * kTailTile * ESZ];
  __shared__ uint64_t smask[NP];
  __shared__ float sscale[NP];
  for (int k = threadIdx.x; k < t && !DIRECT; k += blockDim.x) {
    uint64_t m = 0;
    float sc = 0.f;
    for (int j = 0; j < n; ++j) {
      const float w = W[k * n + j];
      if (w != 0.f) { m |= 1ull << j; sc = w; }
    }
    smask[k] = m;
    sscale[k] = sc;
  }
  __syncthreads();
  const int e = t - beta;  // values left out of the window
  const float inv_beta = 1.f / static_cast<float>(beta);
  const int64_t ntiles = d / kTailTile;
  auto at = [&](int j, int col) -> float {
    if constexpr (DT == kF32) return reinterpret_cast<const float*>(tile)[j * kTailTile + col];
    else return cvt16<DT>(reinterpret_cast<const uint16_t*>(tile)[j * kTailTile + col]);
  };
  for (int64_t tb = blockIdx.x; tb < ntiles + 1; tb += gridDim.x) {
    const int64_t x0 = tb * kTailTile;
    const int width = static_cast<int>(tb < ntiles ? kTailTile : d - x0);  // last tile: the d % 256 tail
    if (width <= 0) break;
    if (width == kTailTile) {
      for (int c = threadIdx.x; c < n * CPR; c += blockDim.x) {
        const int i = c / CPR, k = c % CPR;
        *reinterpret_cast<uint4*>(tile + (i * kTailTile) * ESZ + k * 16) =
            *reinterpret_cast<const uint4*>(static_cast<const char*>(rows.p[i]) + x0 * ESZ + k * 16);
      }
    } else {
      for (int c = threadIdx.x; c < n * kTailTile; c += blockDim.x) {  // columns >= width repeat column 0
        const int i = c / kTailTile, k = c % kTailTile;
        const int64_t xs = k < width ? x0 + k : x0;
        if constexpr (DT == kF32) reinterpret_cast<float*>(tile)[i * kTailTile + k] = load_one<DT>(rows.p[i], xs);
        else reinterpret_cast<uint16_t*>(tile)[i * kTailTile + k] = static_cast<const uint16_t*>(rows.p[i])[xs];
      }
    }
    __syncthreads();
    const int col = threadIdx.x;
    const int tt = opaque_uniform(t), ee = opaque_uniform(e), bb = opaque_uniform(beta);
    float v[NP];
    float r = 0.f;
    uint64_t prev = 0;
    bool exact = true;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      if constexpr (DIRECT) {  // averaged median: the rows themselves (NaN -> +inf)
        v[k] = k < tt ? sanitize_inf(at(k, col)) : kInf;
        continue;
      }
      if (k < tt) {  // uniform
        // volatile LDS reads: the per-set mask and scale are tile-invariant, and hoisting
        // all t of them out of the tile loop would pin 2t SGPRs + t VGPRs (spills)
        const uint64_t cur = uniform64(lds_volatile(smask[k]));
        uint64_t add = cur & ~prev, rem = prev & ~cur;
#pragma clang loop unroll(disable)
        while (add) { r += at(__builtin_ctzll(add), col); add &= add - 1; }
#pragma clang loop unroll(disable)
        while (rem) { r -= at(__builtin_ctzll(rem), col); rem &= rem - 1; }
        prev = cur;
        exact = exact && isfinite(r);
        v[k] = r * lds_volatile(sscale[k]);
      } else {
        v[k] = kInf;
      }
    }
    if (!DIRECT && !exact) {  // inf / NaN inputs: direct per-set sums (sanitised like the generic path)
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        if (k < tt) {
          uint64_t m = uniform64(lds_volatile(smask[k]));
          float s = 0.f;
#pragma clang loop unroll(disable)
          while (m) { s += at(__builtin_ctzll(m), col); m &= m - 1; }
          v[k] = sanitize_inf(s * lds_volatile(sscale[k]));
        }
      }
    }
    int key[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) key[k] = f32_key(sanitize_inf(v[k]));
    oem_sort_i32<NP>(key);
#pragma unroll
    for (int k = 0; k < NP; ++k) v[k] = key_f32(key[k]);
    const float med = pick_sel(v, tt / 2);
    // window start a = #{s < e : v[s] is farther from med than v[s + beta]} (monotone in s);
    // v[s + beta] for s < e comes from a barrel shift by the uniform beta (static indices only)
    float u[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) u[i] = v[i];
#pragma unroll
    for (int b = NP / 2; b >= 1; b >>= 1) {
      if (bb & b) {
#pragma unroll
        for (int i = 0; i + b < NP; ++i) u[i] = u[i + b];
      }
    }
    int a = 0;
#pragma unroll
    for (int s = 0; s < kTailMaxExcluded; ++s) {
      if (s < ee) a += !(sanitize_inf(med - v[s]) <= sanitize_inf(u[s] - med));
    }
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) acc += (i >= a && i < a + bb) ? v[i] : 0.f;
    if (col < width) store_one(out, out_dt, x0 + col, acc * inv_beta);
    __syncthreads();
  }
}

// grid cap of the tail kernels (grid-stride over coordinate groups); GARFIELD_TAIL_GRID overrides
inline int64_t tail_grid_cap(int64_t dflt) {
  static const int64_t env = [] {
    const char* e = std::getenv("GARFIELD_TAIL_GRID");
    const long v = e ? std::atol(e) : 0;
    return static_cast<int64_t>(v > 0 ? v : 0);
  }();
  return env > 0 ? env : dflt;
}

// W == nullptr: averaged median of the n rows themselves (t = n)
template <int DT, int NP>
void launch_bulyan_tail(const RowTable& rows, int n, int64_t d, int beta, const float* W, int t, void* out,
                        int out_dt, hipStream_t s) {
  int64_t g = d / kTailTile + 1;
  const int64_t cap = tail_grid_cap(4096);
  if (g > cap) g = cap;
  if (W == nullptr)
    hipLaunchKernelGGL((k_bulyan_tail<DT, NP, true>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, rows, n, d,
                       beta, W, n, out, out_dt);
  else
    hipLaunchKernelGGL((k_bulyan_tail<DT, NP, false>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, rows, n, d,
                       beta, W, t, out, out_dt);
}

// ---------------------------------------------------------------------------
// bf16 / fp16 gradients: the t selection means on MFMA.
//
// The means are a GEMM: C[t x coords] = S[t x n] . G[n x coords] with S the 0/1
// selection matrix (exact in bf16/fp16; the 1/(m-k) scale is applied in fp32
// afterwards). One wave owns 64 coordinates: it stages the [n x 64] gradient
// tile in its own LDS region with 16-byte loads (no workgroup barrier), reads
// the B fragments with ds_read_b64_tr_b16 (the hardware transpose: gradient rows
// are contiguous along coordinates, the MFMA wants 8 consecutive rows per lane),
// and runs MB x 2 x KS v_mfma_f32_32x32x16 with the S fragments held in
// registers for the whole kernel. A v_permlane32_swap then leaves every lane
// with all t means of ONE coordinate (lane = coordinate), which it sorts in
// registers as above. Coordinates whose means are not all finite (an inf/NaN
// input also turns 0 * inf into NaN inside the MFMA) are recomputed exactly with
// direct per-set sums from the same LDS tile.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

constexpr int kMfmaTailPitch = 144;  // bytes per LDS tile row: 64 coordinates x 2 B + 16 B (bank spread)

template <int DT>
__device__ __forceinline__ f32x16_t mfma32x32x16(s16x8_t a, s16x8_t b, f32x16_t c) {
  if constexpr (DT == kBF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
}

// odd-even merge sort on floats (no NaN: callers map NaN to +inf first)
template <int NP>
__device__ __forceinline__ void oem_sort_f32(float (&v)[NP]) {
#pragma unroll
  for (int p = 1; p < NP; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < NP; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k; ++i) {
          if (i + j + k < NP && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const float a = v[i + j], b = v[i + j + k];
            v[i + j] = __builtin_fminf(a, b);
            v[i + j + k] = __builtin_fmaxf(a, b);
          }
        }
      }
    }
  }
}

// Sorted means -> mean of the beta closest to the median (window [a, a + beta)).
// The runtime positions read (the median t / 2 and the excluded highs beta ..
// t - 1) must be >= P0 = wm_p0(NP) (host-checked: t / 2 >= P0, beta >= P0): the
// sorted values from P0 up are spilled to this wave's LDS scratch `ks` ((NP - P0)
// x 64 floats, [position / 4][lane][position % 4]) with static b128 stores and read
// back at uniform addresses -- no select chains over the register array. The e
// lowest stay in registers (static indices). EXACT: inputs may hold +-inf (NaN
// already mapped to +inf), so distances are sanitised like the reference's.
constexpr int wm_p0(int np) { return (np / 4) & ~3; }

template <int NP, bool EXACT>
__device__ __forceinline__ float window_mean(float (&v)[NP], int tt, int bb, float inv_beta, float* ks, int lane) {
  constexpr int P0 = wm_p0(NP);
  constexpr int SMAX = NP < kTailMaxExcluded ? NP : kTailMaxExcluded;
  static_assert(P0 <= kTailMaxExcluded, "window_mean layout");
  oem_sort_f32<NP>(v);
#pragma unroll
  for (int i = P0; i < NP; i += 4)
    *reinterpret_cast<float4*>(ks + (i - P0) * 64 + lane * 4) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
  asm volatile("" ::: "memory");
  const float* kl = ks + lane * 4;
  auto at = [&](int p) { return kl[((p - P0) >> 2) * 256 + (p & 3)]; };
  const float med = at(tt / 2);
  const int ee = tt - bb;
  int a = 0;
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    if (s < ee) {  // uniform
      const float lo = v[s], hi = at(bb + s);
      a += EXACT ? !(sanitize_inf(med - lo) <= sanitize_inf(hi - med)) : !(med - lo <= hi - med);
    }
  }
  const int lim = a + bb;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) acc += ((i >= SMAX || i >= a) && i < lim) ? v[i] : 0.f;
  asm volatile("" ::: "memory");  // the scratch is the next group's tile
  return acc * inv_beta;
}

// One 64-coordinate group of the KR gradient rows: KR * 8 16-byte chunks, KR / 8 per lane.
// Loads are unconditional (rows >= n point at row 0; zeroed when stored) and global, so
// all of them are in flight at once; the next group's loads are issued before the current
// group's compute (register double buffer).
template <int KR>
struct TileRegs {
  static constexpr int NC = KR / 8;
  u32x4 v[NC];
};

template <int KR>
__device__ __forceinline__ void tile_load(TileRegs<KR>& r, const void* const* sptr, int64_t x0, int lane, int nn) {
  typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
#pragma unroll
  for (int c = 0; c < TileRegs<KR>::NC; ++c) {
    const int idx = c * 64 + lane, row = idx >> 3, ch = idx & 7;
    if (c * 8 < nn)  // uniform: chunks of padding rows only are not loaded (tile_store zeroes them)
      r.v[c] = *(g_u32x4*)(static_cast<const char*>(sptr[row]) + x0 * 2 + ch * 16);
  }
}

template <int KR>
__device__ __forceinline__ void tile_store(unsigned char* tile, const TileRegs<KR>& r, int nn, int lane) {
  const u32x4 zero = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int c = 0; c < TileRegs<KR>::NC; ++c) {
    const int idx = c * 64 + lane, row = idx >> 3, ch = idx & 7;
    *reinterpret_cast<u32x4*>(tile + row * kMfmaTailPitch + ch * 16) = row < nn ? r.v[c] : zero;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local LDS hand-off
}

template <int DT, int KR>
__device__ __forceinline__ void stage_tile(unsigned char* tile, const void* const* sptr, int nn, int64_t x0, int lane) {
  TileRegs<KR> r;
  tile_load<KR>(r, sptr, x0, lane, nn);
  tile_store<KR>(tile, r, nn, lane);
}

constexpr int kTailBadSlots = 32;  // per-wave list of 64-coordinate groups needing the exact path

// One wave per 64-coordinate group (grid-stride). NP = padded set count (8 .. 64),
// KS = 16-row MFMA k-steps (KR = 16 KS >= n). The t set sums of the group come from
// v_mfma_f32_32x32x16 (A = the 0/1 set masks in LDS, B = the gradient tile read with
// ds_read_b64_tr_b16), scaled to means and padded with +inf rows, sorted
// in registers (window_mean). Groups with a non-finite sum are listed and redone by
// the exact pass; the partial last group (d % 64) is done there too.
template <int DT, int NP, int KS>
__global__ __launch_bounds__(256, 2) void k_bulyan_tail_mfma(RowTable rows, int n, int64_t ngroups, int last_width,
                                                             int beta, const float* __restrict__ W, int t, void* out,
                                                             int out_dt) {
  constexpr int MB = NP > 32 ? 2 : 1;   // 32-row MFMA blocks of sets
  constexpr int KR = 16 * KS;           // gradient rows (padded)
  constexpr int KRP = KR + 8;           // sA pitch: 16-byte fragment reads of 8 consecutive lanes hit distinct banks
  constexpr int P0 = wm_p0(NP);
  // per-wave LDS: the gradient tile, then (once its MFMA reads are done) the sorted-means scratch
  constexpr int WAVE_LDS = KR * kMfmaTailPitch > (NP - P0) * 256 ? KR * kMfmaTailPitch : (NP - P0) * 256;
  __shared__ __align__(16) unsigned char tiles[4][WAVE_LDS];
  __shared__ __align__(16) uint16_t sA[32 * MB * KRP];
  __shared__ const void* sptr[KR];
  __shared__ uint64_t smask[NP];
  __shared__ __align__(16) float sscale[NP];
  __shared__ __align__(16) float spad[NP];  // 0 for the t real means, +inf for the padding
  __shared__ int64_t sbad[4][kTailBadSlots];
  __shared__ int sbadn[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  {  // set tables: one W row per wave iteration (n <= 64 = lanes), masks by ballot
    const uint16_t one = DT == kBF16 ? 0x3F80 : 0x3C00;
    for (int k = wave; k < 32 * MB; k += 4) {
      const float w = (k < t && lane < n) ? W[k * n + lane] : 0.f;
      const uint64_t m = __builtin_amdgcn_ballot_w64(w != 0.f);
      if (lane < KR) sA[k * KRP + lane] = w != 0.f ? one : 0;
      if (k < NP) {
        const int first = m ? __builtin_ctzll(m) : 0;
        const float sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), first));
        if (lane == 0) {
          smask[k] = m;
          sscale[k] = m ? sc : 0.f;
          spad[k] = k < t ? 0.f : kInf;
        }
      }
    }
  }
  for (int j = threadIdx.x; j < KR; j += blockDim.x) sptr[j] = rows.p[j < n ? j : 0];
  if (threadIdx.x < 4) sbadn[threadIdx.x] = 0;
  __syncthreads();
  unsigned char* tile = tiles[wave];
  float* ks = reinterpret_cast<float*>(tile);
  // ds_read_b64_tr_b16 addressing: group g = lane / 16 reads rows 8 (g >> 1) + q and
  // columns 16 (g & 1) + 4 p .. + 3 (lane = 16 g + 4 q + p); lane i of the group gets column i
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int tr_off = (8 * (g >> 1) + q) * kMfmaTailPitch + (16 * (g & 1) + 4 * p) * 2;
  const int a_off = (lane & 31) * KRP + 8 * (lane >> 5);
  const float inv_beta = 1.f / static_cast<float>(beta);
  bool overflow = false;
  const int64_t gstep = static_cast<int64_t>(gridDim.x) * 4;
  const int64_t gfirst = static_cast<int64_t>(blockIdx.x) * 4 + wave;
  TileRegs<KR> pre;
  if (gfirst < ngroups) tile_load<KR>(pre, sptr, gfirst * 64, lane, n);
  for (int64_t gi = gfirst; gi < ngroups; gi += gstep) {
    // the LDS tables (sA, scales, pads) are re-read every group: no hoisting into registers
    asm volatile("" ::: "memory");
    const int64_t x0 = gi * 64;
    const int nn = opaque_uniform(n), tt = opaque_uniform(t), bb = opaque_uniform(beta);
    tile_store<KR>(tile, pre, nn, lane);
    if (gi + gstep < ngroups) tile_load<KR>(pre, sptr, (gi + gstep) * 64, lane, nn);  // flies during this group
    f32x16_t acc[MB][2];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[mb][nb][i] = 0.f;
#pragma unroll
    for (int ks_ = 0; ks_ < KS; ++ks_) {
      s16x8_t afrag[MB];  // S[32 mb + (l & 31)][16 ks + 8 (l >> 5) + 0..7]
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        afrag[mb] = *reinterpret_cast<const s16x8_t*>(&sA[a_off + 32 * mb * KRP + 16 * ks_]);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
        const unsigned char* base = tile + ks_ * 16 * kMfmaTailPitch + nb * 64 + tr_off;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 4 * kMfmaTailPitch));
        const s16x8_t bfrag = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][nb] = mfma32x32x16<DT>(afrag[mb], bfrag, acc[mb][nb]);
      }
    }
    // lane = coordinate: swap the halves so each lane holds the NP set sums of x0 + lane
    float v[NP];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k0 = 32 * mb + (i & 3) + 8 * (i >> 2);
        if (k0 < NP) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[mb][0][i]),
                                                           __float_as_uint(acc[mb][1][i]), false, false);
          v[k0] = __uint_as_float(sw[0]);
          v[k0 + 4] = __uint_as_float(sw[1]);
        }
      }
    // chk stays 0 unless a sum is inf / NaN (x * 0 is NaN exactly then): such groups
    // go to the exact pass. mean = sum * scale (+ inf on the padding rows, whose sums are 0)
    float chk = 0.f;
#pragma unroll
    for (int k = 0; k < NP; k += 4) {
      if (k % 8 == 0) asm volatile("" ::: "memory");  // scale / pad reads in chunks (registers)
      const f32x4_t sc = *reinterpret_cast<const f32x4_t*>(&sscale[k]);
      const f32x4_t pd = *reinterpret_cast<const f32x4_t*>(&spad[k]);
      const float scv[4] = {sc[0], sc[1], sc[2], sc[3]}, pdv[4] = {pd[0], pd[1], pd[2], pd[3]};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        chk = __builtin_fmaf(v[k + c], 0.f, chk);
        v[k + c] = __builtin_fmaf(v[k + c], scv[c], pdv[c]);
      }
    }
    if (__builtin_amdgcn_ballot_w64(chk != 0.f)) {  // exact pass later (out of this loop's registers)
      const int slot = sbadn[wave];
      if (slot < kTailBadSlots) {
        if (lane == 0) sbad[wave][slot] = gi;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) sbadn[wave] = slot + 1;
      } else {
        overflow = true;
      }
    }
    store_one(out, out_dt, x0 + lane, window_mean<NP, false>(v, tt, bb, inv_beta, ks, lane));
  }
  // exact pass: groups whose MFMA sums were not all finite (inf/NaN inputs), recomputed
  // with direct per-set sums from the LDS tile (after an overflow of the list: every
  // group of this wave); then the partial last group (last_width < 64 coordinates),
  // which is block 0 / wave 0's
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int nbad = overflow ? 0 : sbadn[wave];
  bool partial_pending = last_width > 0 && gfirst == 0;
  int64_t gi = overflow ? gfirst : 0;
  for (int b = 0;; ++b) {
    int64_t gcur;
    int width = 64;
    if (overflow ? gi < ngroups : b < nbad) {
      gcur = overflow ? gi : sbad[wave][b];
      if (overflow) gi += gstep;
    } else if (partial_pending) {
      gcur = ngroups;
      width = last_width;
      partial_pending = false;
    } else {
      break;
    }
    const int64_t x0 = gcur * 64;
    const int nn = opaque_uniform(n), tt = opaque_uniform(t), bb = opaque_uniform(beta);
    if (width == 64) {
      stage_tile<DT, KR>(tile, sptr, nn, x0, lane);
    } else {  // partial group: per-column loads, columns >= width repeat the first
      const int64_t xs = x0 + (lane < width ? lane : 0);
      for (int j = 0; j < KR; ++j)
        reinterpret_cast<uint16_t*>(tile)[j * (kMfmaTailPitch / 2) + lane] =
            j < nn ? static_cast<const uint16_t*>(sptr[j])[xs] : 0;
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    const uint16_t* col = reinterpret_cast<const uint16_t*>(tile) + lane;
    float v[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      v[k] = kInf;
      if (k < tt) {
        uint64_t m = uniform64(lds_volatile(smask[k]));
        float s = 0.f;
#pragma clang loop unroll(disable)
        while (m) {
          s += cvt16<DT>(col[__builtin_ctzll(m) * (kMfmaTailPitch / 2)]);
          m &= m - 1;
        }
        v[k] = sanitize_inf(s * lds_volatile(sscale[k]));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tile reads done before the scratch is written
    // every listed group is rewritten: its MFMA sums may be NaN (0 * inf from a row outside
    // every set) while all its set means are finite
    const float r = window_mean<NP, true>(v, tt, bb, inv_beta, ks, lane);
    if (lane < width) store_one(out, out_dt, x0 + lane, r);
  }
}

template <int DT, int NP>
void launch_tail_mfma_ks(int ks, const RowTable& rows, int n, int64_t groups, int last_width, int beta,
                         const float* W, int t, void* out, int out_dt, hipStream_t s) {
  int64_t g = (groups + 3) / 4;
  const int64_t cap = tail_grid_cap(4096);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  const dim3 grid(static_cast<unsigned>(g)), block(256);
#define GARFIELD_TAIL_MFMA(KS)                                                                                   \
  hipLaunchKernelGGL((k_bulyan_tail_mfma<DT, NP, KS>), grid, block, 0, s, rows, n, groups, last_width, beta, W, t, \
                     out, out_dt)
  switch (ks) {
    case 1: GARFIELD_TAIL_MFMA(1); break;
    case 2: GARFIELD_TAIL_MFMA(2); break;
    case 3: GARFIELD_TAIL_MFMA(3); break;
    default: GARFIELD_TAIL_MFMA(4); break;
  }
#undef GARFIELD_TAIL_MFMA
}

// bf16/fp16, n <= 64, t <= 64, e = t - beta <= 16: the MFMA tail (every coordinate,
// the d % 64 tail in its exact pass); otherwise false (generic kernels)
template <int DT>
bool launch_bulyan_tail_mfma(const RowTable& rows, int n, int64_t d, int beta, const float* W, int t, void* out,
                             int out_dt, hipStream_t s) {
  if (DT == kF32 || n > 64 || t > 64 || t < 1 || beta < 1 || t - beta > kTailMaxExcluded || W == nullptr) return false;
  const int np = t <= 8 ? 8 : (t <= 16 ? 16 : (t <= 32 ? 32 : 64));
  if (t / 2 < wm_p0(np) || beta < wm_p0(np)) return false;   // window_mean's spilled positions
  const int64_t groups = d / 64;
  const int last = static_cast<int>(d - groups * 64);
  const int ks = (n + 15) / 16;
  switch (np) {
    case 8: launch_tail_mfma_ks<DT, 8>(ks, rows, n, groups, last, beta, W, t, out, out_dt, s); break;
    case 16: launch_tail_mfma_ks<DT, 16>(ks, rows, n, groups, last, beta, W, t, out, out_dt, s); break;
    case 32: launch_tail_mfma_ks<DT, 32>(ks, rows, n, groups, last, beta, W, t, out, out_dt, s); break;
    default: launch_tail_mfma_ks<DT, 64>(ks, rows, n, groups, last, beta, W, t, out, out_dt, s); break;
  }
  return true;
}

// fp32, n <= 64, t <= 64, e = t - beta <= 16: the register kernel of gar_tail_f32.hip; otherwise false
// (generic kernels)
bool launch_bulyan_tail_f32(const RowTable& rows, int n, int64_t d, int beta, const float* W, int t, void* out,
                            int out_dt, hipStream_t s);

}  // namespace coord
}  // namespace gpu
}  // namespace garfield
