// Device-side helpers shared by the gfx950 aggregation kernels (dtype
// conversion, vector loads/stores, wave reductions, register sorting networks).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cfloat>
#include "gar_gpu.hpp"

namespace garfield {
namespace gpu {
namespace dev {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr float kInf = __builtin_huge_valf();

// ---------------------------------------------------------------------------
// dtype helpers

__device__ __forceinline__ float bf16_to_f(uint32_t u16) { return __uint_as_float(u16 << 16); }
__device__ __forceinline__ float f16_to_f(uint32_t u16) {
  return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(u16)));
}
// fp32 -> bf16 round-to-nearest-even on the gfx950 converter (v_cvt_pk_bf16_f32), one
// instruction instead of the integer rounding sequence; NaN stays a (quiet) NaN.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
// two floats -> packed bf16 pair (a in the low half), one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}
__device__ __forceinline__ uint16_t f_to_f16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}

template <int DT> __device__ __forceinline__ float cvt16(uint32_t u) {
  return DT == kBF16 ? bf16_to_f(u) : f16_to_f(u);
}

// Load VEC consecutive elements (16-, 8-, 4- or 2-byte vector loads) as fp32.
template <int DT, int VEC>
__device__ __forceinline__ void load_vec(const void* base, int64_t x, float (&v)[VEC]) {
  if constexpr (DT == kF32) {
    const float* p = static_cast<const float*>(base) + x;
    if constexpr (VEC == 8) {
      float4 a = *reinterpret_cast<const float4*>(p);
      float4 b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else if constexpr (VEC == 4) {
      float4 a = *reinterpret_cast<const float4*>(p);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else if constexpr (VEC == 2) {
      float2 a = *reinterpret_cast<const float2*>(p);
      v[0] = a.x; v[1] = a.y;
    } else {
      v[0] = *p;
    }
  } else {
    const uint16_t* p = static_cast<const uint16_t*>(base) + x;
    if constexpr (VEC == 8) {
      uint4 a = *reinterpret_cast<const uint4*>(p);
      uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) { v[2 * i] = cvt16<DT>(w[i] & 0xffffu); v[2 * i + 1] = cvt16<DT>(w[i] >> 16); }
    } else if constexpr (VEC == 4) {
      uint2 a = *reinterpret_cast<const uint2*>(p);
      v[0] = cvt16<DT>(a.x & 0xffffu); v[1] = cvt16<DT>(a.x >> 16);
      v[2] = cvt16<DT>(a.y & 0xffffu); v[3] = cvt16<DT>(a.y >> 16);
    } else if constexpr (VEC == 2) {
      uint32_t a = *reinterpret_cast<const uint32_t*>(p);
      v[0] = cvt16<DT>(a & 0xffffu); v[1] = cvt16<DT>(a >> 16);
    } else {
      v[0] = cvt16<DT>(*p);
    }
  }
}

template <int DT> __device__ __forceinline__ float load_one(const void* base, int64_t x) {
  if constexpr (DT == kF32) return static_cast<const float*>(base)[x];
  else return cvt16<DT>(static_cast<const uint16_t*>(base)[x]);
}

__device__ __forceinline__ void store_one(void* out, int out_dt, int64_t x, float v) {
  if (out_dt == kF32) static_cast<float*>(out)[x] = v;
  else if (out_dt == kBF16) static_cast<uint16_t*>(out)[x] = f_to_bf16(v);
  else static_cast<uint16_t*>(out)[x] = f_to_f16(v);
}

template <int VEC>
__device__ __forceinline__ void store_vec(void* out, int out_dt, int64_t x, const float (&v)[VEC]) {
  if (out_dt == kF32) {
    float* p = static_cast<float*>(out) + x;
    if constexpr (VEC % 4 == 0) {
#pragma unroll
      for (int i = 0; i < VEC; i += 4)
        *reinterpret_cast<float4*>(p + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) p[i] = v[i];
    }
  } else {
    uint16_t* p = static_cast<uint16_t*>(out) + x;
    uint16_t h[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] = out_dt == kBF16 ? f_to_bf16(v[i]) : f_to_f16(v[i]);
    if constexpr (VEC == 8) {
      uint4 w;
      w.x = h[0] | (uint32_t(h[1]) << 16); w.y = h[2] | (uint32_t(h[3]) << 16);
      w.z = h[4] | (uint32_t(h[5]) << 16); w.w = h[6] | (uint32_t(h[7]) << 16);
      *reinterpret_cast<uint4*>(p) = w;
    } else if constexpr (VEC == 4) {
      uint2 w;
      w.x = h[0] | (uint32_t(h[1]) << 16); w.y = h[2] | (uint32_t(h[3]) << 16);
      *reinterpret_cast<uint2*>(p) = w;
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) p[i] = h[i];
    }
  }
}

__device__ __forceinline__ float sanitize_inf(float v) {
  return (v == v) ? v : kInf;  // NaN -> +inf (total order for sorting)
}

// A wave-uniform int re-materialised inside a loop body (volatile asm: never
// hoisted). Comparisons of unrolled static indices against a loop-invariant
// uniform bound otherwise become NP hoisted 64-bit lane masks per bound, which
// spill the SGPR file into VGPR lanes.
__device__ __forceinline__ int opaque_uniform(int v) {
  int r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(v));
  return r;
}

// v[idx] of a register array for a WAVE-UNIFORM runtime idx: a binary tree of
// scalar branches ending in one static register read (no select chain, no
// dynamically indexed — scratch-backed — array).
template <int LO, int HI, class T, int N>
__device__ __forceinline__ T pick_uniform_rec(const T (&v)[N], int idx) {
  if constexpr (HI - LO == 1) {
    T r = v[LO];
    asm volatile("" : "+v"(r));
    return r;
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (idx < MID) return pick_uniform_rec<LO, MID, T, N>(v, idx);
    return pick_uniform_rec<MID, HI, T, N>(v, idx);
  }
}
template <class T, int N>
__device__ __forceinline__ T pick_uniform(const T (&v)[N], int idx) {
  return pick_uniform_rec<0, N, T, N>(v, idx);
}

// v[idx] for any runtime idx as a v_cndmask chain; the empty asm keeps each operand
// opaque (otherwise instcombine re-forms ONE dynamically indexed load, which pins
// the whole array in scratch). Pass an opaque_uniform() idx inside loops.
template <class T, int N>
__device__ __forceinline__ T pick_sel(const T (&v)[N], int idx) {
  T r = v[0];
  asm("" : "+v"(r));
#pragma unroll
  for (int i = 1; i < N; ++i) {
    T t = v[i];
    asm("" : "+v"(t));
    r = (i == idx) ? t : r;
  }
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int score_rank(const float* s, int n, int i) {
  const float si = sanitize_inf(s[i]);
  int rank = 0;
  for (int j = 0; j < n; ++j) {
    const float sj = sanitize_inf(s[j]);
    rank += (sj < si) || (sj == si && j < i);
  }
  return rank;
}

template <int NP, int VEC>
__device__ __forceinline__ void bitonic_sort(float (&v)[NP][VEC]) {
#pragma unroll
  for (int k = 2; k <= NP; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
#pragma unroll
          for (int c = 0; c < VEC; ++c) {
            const float a = v[i][c], b = v[l][c];
            const float lo = fminf(a, b), hi = fmaxf(a, b);
            v[i][c] = up ? lo : hi;
            v[l][c] = up ? hi : lo;
          }
        }
      }
    }
  }
}

// Sort (key, value) pairs by (key, value) ascending.
template <int NP, int VEC>
__device__ __forceinline__ void bitonic_sort_pairs(float (&key)[NP][VEC], float (&val)[NP][VEC]) {
#pragma unroll
  for (int k = 2; k <= NP; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
#pragma unroll
          for (int c = 0; c < VEC; ++c) {
            const float ka = key[i][c], kb = key[l][c], va = val[i][c], vb = val[l][c];
            const bool gt = (ka > kb) || (ka == kb && va > vb);
            const bool sw = up ? gt : !gt;
            key[i][c] = sw ? kb : ka; key[l][c] = sw ? ka : kb;
            val[i][c] = sw ? vb : va; val[l][c] = sw ? va : vb;
          }
        }
      }
    }
  }
}

// Select element idx (runtime, uniform or not) from a sorted column.
template <int NP, int VEC>
__device__ __forceinline__ float pick(const float (&v)[NP][VEC], int c, int idx) {
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) r = (i == idx) ? v[i][c] : r;
  return r;
}

// Mean of the beta values closest to v[mid] (ties broken by value), v sorted.
template <int NP, int VEC>
__device__ __forceinline__ void closest_mean(float (&v)[NP][VEC], const int (&mid)[VEC], int beta,
                                             float (&res)[VEC]) {
  float key[NP][VEC];
  float med[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) med[c] = pick<NP, VEC>(v, c, mid[c]);
#pragma unroll
  for (int i = 0; i < NP; ++i)
#pragma unroll
    for (int c = 0; c < VEC; ++c) key[i][c] = sanitize_inf(fabsf(v[i][c] - med[c]));
  bitonic_sort_pairs<NP, VEC>(key, v);
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) s += (i < beta) ? v[i][c] : 0.f;
    res[c] = s / static_cast<float>(beta);
  }
}

template <template <int> class F, typename... A>
void by_dtype(int dt, A&&... a) {
  if (dt == kF32) F<kF32>::run(a...);
  else if (dt == kBF16) F<kBF16>::run(a...);
  else F<kF16>::run(a...);
}


// Division by a run-time constant d >= 1 without the ~30-instruction integer division sequence
// (Granlund-Montgomery with a 33-bit multiplier): q = (umulhi(n, m) + n) >> l, exact for n < 2^31.
// Pixel decompositions in the k-loops of the implicit-GEMM kernels (m -> n, h, w) use it.
struct FastDiv {
  uint32_t d, m, l;
};
__host__ __device__ inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((1ull << (32 + l)) / d) - (1ull << 32) + 1;
  return FastDiv{d, static_cast<uint32_t>(m), l};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.l; }
// q = n / d, r = n - q d
__device__ __forceinline__ void fdivmod(uint32_t n, const FastDiv& f, uint32_t& q, uint32_t& r) {
  q = fdiv(n, f);
  r = n - q * f.d;
}

}  // namespace dev
}  // namespace gpu
}  // namespace garfield
