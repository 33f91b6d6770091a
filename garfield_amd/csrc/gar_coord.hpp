// Coordinate-wise rule kernels (register bitonic networks), instantiated per
// mode in gar_coord_m*.hip so the 90 variants compile in parallel.
#pragma once
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
namespace coord {
using namespace dev;

// ---------------------------------------------------------------------------
// Coordinate-wise rules: each lane holds NP x VEC values in registers and runs
// a fully unrolled bitonic network per coordinate (constant register indices
// only: no scratch). Rows >= n are padded with +inf.

template <int DT, int NP, int VEC, int MODE>
__device__ __forceinline__ void coord_body(const RowTable& rows, int n, int f, int beta, const float* sW,
                                           int t, uint64_t seed, uint64_t thr, int64_t x, float (&res)[VEC],
                                           bool vector_path) {
  float v[NP][VEC];
  float first[VEC];
  if constexpr (MODE == kBulyanTail) {
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int c = 0; c < VEC; ++c) v[k][c] = 0.f;
    for (int j = 0; j < n; ++j) {
      float g[VEC];
      if (vector_path) load_vec<DT, VEC>(rows.p[j], x, g);
      else { g[0] = load_one<DT>(rows.p[j], x); }
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        if (k < t) {
          const float w = sW[k * n + j];
#pragma unroll
          for (int c = 0; c < VEC; ++c) v[k][c] += w * g[c];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int c = 0; c < VEC; ++c) v[k][c] = (k < t) ? sanitize_inf(v[k][c]) : kInf;
  } else {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (i < n) {
        if (vector_path) load_vec<DT, VEC>(rows.p[i], x, v[i]);
        else v[i][0] = load_one<DT>(rows.p[i], x);
      } else {
#pragma unroll
        for (int c = 0; c < VEC; ++c) v[i][c] = kInf;
      }
    }
  }

  if constexpr (MODE == kAverageNan) {
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      float s = 0.f;
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const bool ok = (i < n) && isfinite(v[i][c]);
        s += ok ? v[i][c] : 0.f;
        cnt += ok;
      }
      res[c] = cnt ? s / static_cast<float>(cnt) : 0.f;
    }
    return;
  }

  if constexpr (MODE == kCondense) {
#pragma unroll
    for (int c = 0; c < VEC; ++c) first[c] = v[0][c];
  }

  int cnt[VEC];
  if constexpr (MODE == kMedian || MODE == kCondense) {
    // finite-only median: non-finite values pushed to +inf and not counted
#pragma unroll
    for (int c = 0; c < VEC; ++c) cnt[c] = 0;
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int c = 0; c < VEC; ++c) {
        const bool ok = (i < n) && isfinite(v[i][c]);
        cnt[c] += ok;
        v[i][c] = ok ? v[i][c] : kInf;
      }
  } else if constexpr (MODE != kBulyanTail) {
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int c = 0; c < VEC; ++c) v[i][c] = sanitize_inf(v[i][c]);
  }

  bitonic_sort<NP, VEC>(v);

  if constexpr (MODE == kMedian || MODE == kCondense) {
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      float med = cnt[c] ? pick<NP, VEC>(v, c, cnt[c] / 2) : 0.f;
      if constexpr (MODE == kCondense) {
        const uint32_t draw = mix_hash(seed, static_cast<uint64_t>(x + c));
        med = (static_cast<uint64_t>(draw) < thr) ? med : first[c];
      }
      res[c] = med;
    }
  } else if constexpr (MODE == kTrimmedMean) {
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NP; ++i) s += (i >= f && i < n - f) ? v[i][c] : 0.f;
      res[c] = s / static_cast<float>(n - 2 * f);
    }
  } else {  // kAveragedMedian, kBulyanTail
    const int len = (MODE == kBulyanTail) ? t : n;
    int mid[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) mid[c] = len / 2;
    closest_mean<NP, VEC>(v, mid, beta, res);
  }
}

template <int DT, int NP, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_coordwise(RowTable rows, int n, int64_t d, int f, int beta,
                                                   const float* __restrict__ W, int t, uint64_t seed,
                                                   uint64_t thr, void* out, int out_dt) {
  __shared__ float sW[(MODE == kBulyanTail) ? (NP * kMaxRows) : 1];
  if constexpr (MODE == kBulyanTail) {
    for (int e = threadIdx.x; e < t * n; e += blockDim.x) sW[e] = W[e];
    __syncthreads();
  }
  const int64_t dv = (d / VEC) * VEC;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * VEC;
  for (int64_t x = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * VEC; x < dv; x += stride) {
    float res[VEC];
    coord_body<DT, NP, VEC, MODE>(rows, n, f, beta, sW, t, seed, thr, x, res, true);
    store_vec<VEC>(out, out_dt, x, res);
  }
  if (blockIdx.x == 0) {
    for (int64_t x = dv + threadIdx.x; x < d; x += blockDim.x) {
      float res[1];
      coord_body<DT, NP, 1, MODE>(rows, n, f, beta, sW, t, seed, thr, x, res, false);
      store_one(out, out_dt, x, res[0]);
    }
  }
}

template <int DT, int NP, int VEC, int MODE>
void launch_coord(const RowTable& rows, int n, int64_t d, int f, int beta, const float* W, int t, uint64_t seed,
                  uint64_t thr, void* out, int out_dt, hipStream_t s) {
  int64_t g = (d / VEC + 255) / 256;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL((k_coordwise<DT, NP, VEC, MODE>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, rows, n, d,
                     f, beta, W, t, seed, thr, out, out_dt);
}

template <int DT, int MODE>
void coord_np(int np, const RowTable& rows, int n, int64_t d, int f, int beta, const float* W, int t, uint64_t seed,
              uint64_t thr, void* out, int out_dt, hipStream_t s) {
  switch (np) {
    case 8: launch_coord<DT, 8, 8, MODE>(rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s); break;
    case 16: launch_coord<DT, 16, 4, MODE>(rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s); break;
    case 32: launch_coord<DT, 32, 2, MODE>(rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s); break;
    case 64: launch_coord<DT, 64, 1, MODE>(rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s); break;
    default: launch_coord<DT, 128, 1, MODE>(rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s); break;
  }
}

inline int np_for(int k) { return k <= 8 ? 8 : (k <= 16 ? 16 : (k <= 32 ? 32 : (k <= 64 ? 64 : 128))); }

template <int MODE> struct ByDtype {
  template <int DT> struct F {
    static void run(int np, const RowTable& rows, int n, int64_t d, int f, int beta, const float* W, int t,
                    uint64_t seed, uint64_t thr, void* out, int out_dt, hipStream_t s) {
      coord_np<DT, MODE>(np, rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s);
    }
  };
};

template <int MODE>
void coord_mode(int dt, int np, const RowTable& rows, int n, int64_t d, int f, int beta, const float* W,
                int t, uint64_t seed, uint64_t thr, void* out, int out_dt, hipStream_t s);

}  // namespace coord
}  // namespace gpu
}  // namespace garfield
