// Coordinate-wise rules on bf16 / fp16 gradients with PACKED 16-bit sort keys.
//
// A bf16 (or fp16) value maps to a signed 16-bit key that orders exactly like
// the value (sign-magnitude -> two's complement: flip the magnitude bits of the
// negatives; 2 VALU ops per 32-bit word with v_pk_ashrrev_i16 + v_bitop3_b32),
// so one v_pk_min_i16 / v_pk_max_i16 pair is a compare-exchange of TWO
// coordinates at once: half the VALU work of an fp32 sorting network, and no
// fp32 conversion before the sort. Each lane owns 2P consecutive coordinates
// (P words per row, 4P-byte loads), rows are sorted with Batcher's odd-even
// merge network (fewer comparators than bitonic: 19/63/191/543 for 8/16/32/64
// rows) entirely in registers.
//
// Non-finite inputs: rows >= n are padded with the largest FINITE key, so after
// the sort a lane whose smallest key is <= key(-inf) or whose largest key is
// >= key(+inf) holds a NaN/inf; only such (rare) lanes take the exact fp32
// per-coordinate path of gar_coord.hpp (NaN -> +inf / finite-only median), so
// results never depend on the fast path's assumptions.
//
// Reference semantics: median.cu:60-83 (finite-only lower median),
// bulyan.cu:227-243 / deprecated_native native.cpp:714-747 (averaged median),
// plus the trimmed mean (not in the reference).
#pragma once
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
namespace coord {
using namespace dev;

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int DT> struct Key16 {
  // bf16: +inf 0x7F80, largest finite 0x7F7F, key(-inf) = 0xFF80 ^ 0x7FFF
  static constexpr int kPosInf = DT == kBF16 ? 0x7F80 : 0x7C00;
  static constexpr int kMaxFinite = DT == kBF16 ? 0x7F7F : 0x7BFF;
  static constexpr int kNegInf = DT == kBF16 ? static_cast<short>(0x807F) : static_cast<short>(0x83FF);
};

__device__ __forceinline__ uint32_t to_key(uint32_t w) {
  // negative halves: flip the 15 magnitude bits (-> monotone signed 16-bit key); involution
  const s16x2 x = __builtin_bit_cast(s16x2, w);
  const s16x2 s = x >> (s16x2){15, 15};
  return w ^ (__builtin_bit_cast(uint32_t, s) & 0x7fff7fffu);
}

__device__ __forceinline__ void cmpx(uint32_t& a, uint32_t& b) {
  const s16x2 x = __builtin_bit_cast(s16x2, a), y = __builtin_bit_cast(s16x2, b);
  a = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
  b = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}

// Batcher odd-even merge sort (ascending), fully unrolled: compile-time indices only.
template <int NP, int P>
__device__ __forceinline__ void oem_sort(uint32_t (&v)[NP][P]) {
#pragma unroll
  for (int p = 1; p < NP; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < NP; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k; ++i) {
          if (i + j + k < NP && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
#pragma unroll
            for (int q = 0; q < P; ++q) cmpx(v[i + j][q], v[i + j + k][q]);
          }
        }
      }
    }
  }
}

// value of half h of a key word as fp32
template <int DT>
__device__ __forceinline__ float key_val(uint32_t keyword, int h) {
  const uint32_t w = to_key(keyword);  // involution: back to the raw 16-bit patterns
  if constexpr (DT == kBF16) return __uint_as_float(h ? (w & 0xffff0000u) : (w << 16));
  else return f16_to_f(h ? (w >> 16) : (w & 0xffffu));
}

// v[idx][q] for a wave-uniform runtime idx (scalar branch tree, gar_device.hpp).
template <int NP, int P>
__device__ __forceinline__ uint32_t pick_word(const uint32_t (&v)[NP][P], int q, int idx) {
  uint32_t col[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) col[i] = v[i][q];
  return pick_uniform(col, idx);  // idx is wave-uniform at every call site
}

template <int DT, int NP, int P, int MODE>
__device__ __forceinline__ void coord16_fast(const uint32_t (&v)[NP][P], const uint32_t (&first)[P], int n, int f,
                                             int beta, uint64_t seed, uint64_t thr, int64_t x,
                                             float (&res)[2 * P]) {
  if constexpr (MODE == kMedian || MODE == kCondense) {
    const int mid = n / 2;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const uint32_t w = pick_word<NP, P>(v, q, mid);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float med = key_val<DT>(w, h);
        if constexpr (MODE == kCondense) {
          const uint32_t draw = mix_hash(seed, static_cast<uint64_t>(x + 2 * q + h));
          const uint32_t raw = first[q];
          const float f0 = DT == kBF16 ? __uint_as_float(h ? (raw & 0xffff0000u) : (raw << 16))
                                       : f16_to_f(h ? (raw >> 16) : (raw & 0xffffu));
          med = (static_cast<uint64_t>(draw) < thr) ? med : f0;
        }
        res[2 * q + h] = med;
      }
    }
  } else if constexpr (MODE == kTrimmedMean) {
    const float inv = 1.f / static_cast<float>(n - 2 * f);
#pragma unroll
    for (int q = 0; q < P; ++q) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        if (i >= f && i < n - f) {  // uniform
          s0 += key_val<DT>(v[i][q], 0);
          s1 += key_val<DT>(v[i][q], 1);
        }
      }
      res[2 * q] = s0 * inv;
      res[2 * q + 1] = s1 * inv;
    }
  } else {  // kAveragedMedian: mean of the beta values closest to the median (ties -> smaller value)
    const int mid = n / 2;
    const float inv = 1.f / static_cast<float>(beta);
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const uint32_t mw = pick_word<NP, P>(v, q, mid);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float m = key_val<DT>(mw, h);
        // sorted values: the beta closest form a window [s, s + beta); s = first s with
        // m - v[s] <= v[s + beta] - m (monotone in s)
        int s = 0;
#pragma unroll
        for (int i = 0; i + 1 < NP; ++i) {
          if (i < n - beta) {  // uniform
            const float lo = key_val<DT>(v[i][q], h);
            const float hi = key_val<DT>(pick_word<NP, P>(v, q, i + beta), h);
            s += !((m - lo) <= (hi - m));
          }
        }
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          if (i < n) {
            const float val = key_val<DT>(v[i][q], h);
            acc += (i >= s && i < s + beta) ? val : 0.f;
          }
        }
        res[2 * q + h] = acc * inv;
      }
    }
  }
}

// Exact per-coordinate path for the rare coordinates holding a NaN / inf (and the
// d % 2P tail): rank counting, O(n^2) scalar loads from cache, a handful of
// registers, so it does not inflate the fast path's register allocation.
// Semantics of gar_coord.hpp's fp32 networks: median = finite-only lower median
// (0 if none); trimmed mean / averaged median sort NaN as +inf; averaged median
// orders by (|v - med|, v).
template <int DT, int MODE>
__device__ __forceinline__ float coord16_rank(const RowTable& rows, int n, int f, int beta, uint64_t seed,
                                              uint64_t thr, int64_t x) {
  if constexpr (MODE == kMedian || MODE == kCondense) {
    int cnt = 0;
    for (int j = 0; j < n; ++j) cnt += isfinite(load_one<DT>(rows.p[j], x));
    float med = 0.f;
    const int r = cnt / 2;
    for (int i = 0; i < n && cnt; ++i) {
      const float vi = load_one<DT>(rows.p[i], x);
      if (!isfinite(vi)) continue;
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const float vj = load_one<DT>(rows.p[j], x);
        rank += isfinite(vj) && (vj < vi || (vj == vi && j < i));
      }
      if (rank == r) { med = vi; break; }
    }
    if constexpr (MODE == kCondense) {
      const uint32_t draw = mix_hash(seed, static_cast<uint64_t>(x));
      if (!(static_cast<uint64_t>(draw) < thr)) med = load_one<DT>(rows.p[0], x);
    }
    return med;
  } else if constexpr (MODE == kTrimmedMean) {
    float acc = 0.f;
    for (int i = 0; i < n; ++i) {
      const float vi = sanitize_inf(load_one<DT>(rows.p[i], x));
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const float vj = sanitize_inf(load_one<DT>(rows.p[j], x));
        rank += vj < vi || (vj == vi && j < i);
      }
      if (rank >= f && rank < n - f) acc += vi;
    }
    return acc / static_cast<float>(n - 2 * f);
  } else {  // kAveragedMedian
    float m = 0.f;
    for (int i = 0; i < n; ++i) {
      const float vi = sanitize_inf(load_one<DT>(rows.p[i], x));
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const float vj = sanitize_inf(load_one<DT>(rows.p[j], x));
        rank += vj < vi || (vj == vi && j < i);
      }
      if (rank == n / 2) { m = vi; break; }
    }
    float acc = 0.f;
    for (int i = 0; i < n; ++i) {
      const float vi = sanitize_inf(load_one<DT>(rows.p[i], x));
      const float ki = sanitize_inf(fabsf(vi - m));
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const float vj = sanitize_inf(load_one<DT>(rows.p[j], x));
        const float kj = sanitize_inf(fabsf(vj - m));
        rank += kj < ki || (kj == ki && (vj < vi || (vj == vi && j < i)));
      }
      if (rank < beta) acc += vi;
    }
    return acc / static_cast<float>(beta);
  }
}

template <int DT, int NP, int P, int MODE>
__global__ __launch_bounds__(256) void k_coord16(RowTable rows, int n, int64_t d, int f, int beta, uint64_t seed,
                                                 uint64_t thr, void* out, int out_dt) {
  constexpr int VEC = 2 * P;
  using K = Key16<DT>;
  const uint32_t pad = (static_cast<uint32_t>(K::kMaxFinite) << 16) | static_cast<uint32_t>(K::kMaxFinite);
  const int64_t dv = (d / VEC) * VEC;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * VEC;
  for (int64_t x = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * VEC; x < dv; x += stride) {
    uint32_t v[NP][P];
    // branch-free gather: every row load is issued back to back (rows >= n re-read
    // row 0 and are replaced by the pad key), one wait for all of them
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const uint16_t* src = static_cast<const uint16_t*>(rows.p[i < n ? i : 0]) + x;
      if constexpr (P == 4) {
        const u32x4 a = *reinterpret_cast<const u32x4*>(src);
        v[i][0] = a[0]; v[i][1 % P] = a[1]; v[i][2 % P] = a[2]; v[i][3 % P] = a[3];
      } else if constexpr (P == 2) {
        const u32x2 a = *reinterpret_cast<const u32x2*>(src);
        v[i][0] = a[0]; v[i][1 % P] = a[1];
      } else {
        v[i][0] = *reinterpret_cast<const uint32_t*>(src);
      }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int q = 0; q < P; ++q) v[i][q] = (i < n) ? v[i][q] : pad;
    uint32_t first[P];
#pragma unroll
    for (int q = 0; q < P; ++q) first[q] = v[0][q];
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int q = 0; q < P; ++q) v[i][q] = to_key(v[i][q]);
    oem_sort<NP, P>(v);
    bool bad = false;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const s16x2 lo = __builtin_bit_cast(s16x2, v[0][q]);
      const s16x2 hi = __builtin_bit_cast(s16x2, v[NP - 1][q]);
      bad |= (lo.x <= K::kNegInf) | (lo.y <= K::kNegInf) | (hi.x >= K::kPosInf) | (hi.y >= K::kPosInf);
    }
    float res[VEC];
    if (!bad) {
      coord16_fast<DT, NP, P, MODE>(v, first, opaque_uniform(n), opaque_uniform(f), opaque_uniform(beta), seed, thr,
                                    x, res);
    } else {  // a NaN / inf among this lane's coordinates: exact fp32 per-coordinate path
#pragma unroll
      for (int c = 0; c < VEC; ++c) res[c] = coord16_rank<DT, MODE>(rows, n, f, beta, seed, thr, x + c);
    }
    store_vec<VEC>(out, out_dt, x, res);
  }
  if (blockIdx.x == 0) {
    for (int64_t x = dv + threadIdx.x; x < d; x += blockDim.x)
      store_one(out, out_dt, x, coord16_rank<DT, MODE>(rows, n, f, beta, seed, thr, x));
  }
}

template <int NP> struct Coord16Words { static constexpr int P = NP <= 16 ? 4 : (NP == 32 ? 2 : 1); };

template <int MODE> constexpr bool coord16_mode() {
  return MODE == kMedian || MODE == kTrimmedMean || MODE == kCondense;  // averaged median: gar_bulyan_tail.hpp
}

template <int DT, int NP, int MODE>
void launch_coord16(const RowTable& rows, int n, int64_t d, int f, int beta, uint64_t seed, uint64_t thr, void* out,
                    int out_dt, hipStream_t s) {
  constexpr int P = Coord16Words<NP>::P;
  int64_t g = (d / (2 * P) + 255) / 256;
  const int64_t cap = coord16_grid_cap(NP);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  hipLaunchKernelGGL((k_coord16<DT, NP, P, MODE>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, rows, n, d, f,
                     beta, seed, thr, out, out_dt);
}

}  // namespace coord
}  // namespace gpu
}  // namespace garfield
