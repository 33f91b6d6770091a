// Coordinate-wise rule kernels (register bitonic networks), instantiated per
// mode in gar_coord_m*.hip so the 90 variants compile in parallel.
#pragma once
#include <cstdlib>
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
namespace coord {
using namespace dev;

// ---------------------------------------------------------------------------
// Coordinate-wise rules: each lane holds NP x VEC values in registers and runs
// a fully unrolled bitonic network per coordinate (constant register indices
// only: no scratch). Rows >= n are padded with +inf.

// Row loaders: `load(i, g)` fills g[VEC] with row i's values at the current coordinate(s).
template <int DT, int VEC>
struct DirectLoader {  // straight from HBM: VEC consecutive coordinates per lane (8/16-byte loads)
  const RowTable& rows;
  int64_t x;
  bool vector_path;
  __device__ __forceinline__ void operator()(int i, float (&g)[VEC]) const {
    if (vector_path) load_vec<DT, VEC>(rows.p[i], x, g);
    else g[0] = load_one<DT>(rows.p[i], x);
  }
};

template <int DT>
struct LdsLoader {  // from an LDS tile [row][TILE coords] staged with 16-byte loads
  const void* tile;
  int pitch;  // elements per tile row
  int col;
  __device__ __forceinline__ void operator()(int i, float (&g)[1]) const {
    if constexpr (DT == kF32) g[0] = static_cast<const float*>(tile)[i * pitch + col];
    else g[0] = cvt16<DT>(static_cast<const uint16_t*>(tile)[i * pitch + col]);
  }
};

// W is read with wave-uniform indices straight from global memory: scalar loads
// (s_load) into SGPRs, shared by the 64 lanes — not one LDS read per lane and FMA.
template <int DT, int NP, int VEC, int MODE, class Loader>
__device__ __forceinline__ void coord_gather(const Loader& load, int n, const float* __restrict__ W, int t,
                                             float (&v)[NP][VEC]) {
  if constexpr (MODE == kBulyanTail) {
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int c = 0; c < VEC; ++c) v[k][c] = 0.f;
    for (int j = 0; j < n; ++j) {
      float g[VEC];
      load(j, g);
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        if (k < t) {
          const float w = W[k * n + j];  // uniform index: scalar load
          if (w != 0.f) {                // uniform branch: W rows are sparse (m - k non-zeros)
#pragma unroll
            for (int c = 0; c < VEC; ++c) v[k][c] += w * g[c];
          }
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
        load(i, v[i]);
      } else {
#pragma unroll
        for (int c = 0; c < VEC; ++c) v[i][c] = kInf;
      }
    }
  }
}

template <int NP, int VEC, int MODE>
__device__ __forceinline__ void coord_reduce(float (&v)[NP][VEC], int n, int f, int beta, int t,
                                             uint64_t seed, uint64_t thr, int64_t x, float (&res)[VEC]) {
  float first[VEC];
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

template <int DT, int NP, int VEC, int MODE, class Loader>
__device__ __forceinline__ void coord_body(const Loader& load, int n, int f, int beta, const float* __restrict__ W,
                                           int t, uint64_t seed, uint64_t thr, int64_t x, float (&res)[VEC]) {
  float v[NP][VEC];
  coord_gather<DT, NP, VEC, MODE>(load, n, W, t, v);
  coord_reduce<NP, VEC, MODE>(v, n, f, beta, t, seed, thr, x, res);
}

template <int DT, int NP, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_coordwise(RowTable rows, int n, int64_t d, int f, int beta,
                                                   const float* __restrict__ W, int t, uint64_t seed,
                                                   uint64_t thr, void* out, int out_dt) {
  const int64_t dv = (d / VEC) * VEC;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * VEC;
  for (int64_t x = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * VEC; x < dv; x += stride) {
    float res[VEC];
    coord_body<DT, NP, VEC, MODE>(DirectLoader<DT, VEC>{rows, x, true}, n, f, beta, W, t, seed, thr, x, res);
    store_vec<VEC>(out, out_dt, x, res);
  }
  if (blockIdx.x == 0) {
    for (int64_t x = dv + threadIdx.x; x < d; x += blockDim.x) {
      float res[1];
      coord_body<DT, NP, 1, MODE>(DirectLoader<DT, 1>{rows, x, false}, n, f, beta, W, t, seed, thr, x, res);
      store_one(out, out_dt, x, res[0]);
    }
  }
}

// knobs: GARFIELD_COORD16=0 disables the packed 16-bit-key kernels (A/B runs);
// GARFIELD_COORD16_GRID caps their grid (grid-stride loop beyond it)
inline bool coord16_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("GARFIELD_COORD16");
    return !(e && e[0] == '0');
  }();
  return on;
}
inline bool coord_mfma_tail_enabled() {  // GARFIELD_MFMA_TAIL=0: Bulyan tail without MFMA (A/B runs)
  static const bool on = [] {
    const char* e = std::getenv("GARFIELD_MFMA_TAIL");
    return !(e && e[0] == '0');
  }();
  return on;
}
// Grid cap of the packed 16-bit coordinate kernels (grid-stride loop). Measured at d = 23.5M
// bf16 (profiles/r2/coord16_grid_sweep.log): small sets (NP <= 16, 8 coordinates per lane) are
// fastest with one pass per lane (cap 16384: median n=8 0.080 vs 0.084 ms at 4096); large sets
// with 4096 (n=64 0.611 vs 0.634 ms at 16384). GARFIELD_COORD16_GRID overrides both.
inline int64_t coord16_grid_cap(int np) {
  static const int64_t env = [] {
    const char* e = std::getenv("GARFIELD_COORD16_GRID");
    const long v = e ? std::atol(e) : 0;
    return static_cast<int64_t>(v > 0 ? v : 0);
  }();
  if (env > 0) return env;
  return np <= 16 ? 16384 : 4096;
}

}  // namespace coord
}  // namespace gpu
}  // namespace garfield

#include "gar_coord16.hpp"
#include "gar_bulyan_tail.hpp"

namespace garfield {
namespace gpu {
namespace coord {

// Large n (NP >= 32): one lane per coordinate would issue n 2-byte loads; instead
// a workgroup stages a [n x 256-coordinate] tile through LDS with 16-byte loads
// (each row segment is 512 B / 1 KB contiguous), then every lane reads its
// column (conflict-free: consecutive lanes, consecutive elements).
constexpr int kCoordTile = 256;

template <int DT, int NP, int MODE>
__global__ __launch_bounds__(256) void k_coordwise_lds(RowTable rows, int n, int64_t d, int f, int beta,
                                                       const float* __restrict__ W, int t, uint64_t seed,
                                                       uint64_t thr, void* out, int out_dt) {
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  constexpr int CPR = kCoordTile * ESZ / 16;  // 16-byte chunks per tile row
  __shared__ __align__(16) unsigned char tile[NP * kCoordTile * ESZ];
  // Bulyan tail: W [t][n] compacted once per workgroup into per-row index lists
  // (uniform trip counts, one LDS read per selected gradient) + the row scale.
  __shared__ uint8_t sel[(MODE == kBulyanTail) ? NP * NP : 1];
  __shared__ int selcnt[(MODE == kBulyanTail) ? NP : 1];
  __shared__ float selscale[(MODE == kBulyanTail) ? NP : 1];
  if constexpr (MODE == kBulyanTail) {
    for (int k = threadIdx.x; k < t; k += blockDim.x) {
      int c = 0;
      float sc = 0.f;
      for (int j = 0; j < n; ++j) {
        const float w = W[k * n + j];
        if (w != 0.f) { sel[k * NP + c] = static_cast<uint8_t>(j); ++c; sc = w; }
      }
      selcnt[k] = c;
      selscale[k] = sc;  // uniform weights 1/(m-k) per row
    }
    __syncthreads();
  }
  const int64_t ntiles = d / kCoordTile;
  const int nrows = (MODE == kBulyanTail) ? n : (n < NP ? n : NP);
  for (int64_t tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
    const int64_t x0 = tb * kCoordTile;
    for (int c = threadIdx.x; c < nrows * CPR; c += blockDim.x) {
      const int i = c / CPR, k = c % CPR;
      const uint4 val = *reinterpret_cast<const uint4*>(static_cast<const char*>(rows.p[i]) + x0 * ESZ + k * 16);
      *reinterpret_cast<uint4*>(tile + (i * kCoordTile) * ESZ + k * 16) = val;
    }
    __syncthreads();
    const int col = threadIdx.x;
    float res[1];
    if constexpr (MODE == kBulyanTail) {
      const LdsLoader<DT> load{tile, kCoordTile, col};
      float v[NP][1];
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        float acc = 0.f;
        if (k < t) {
          const int cnt = selcnt[k];
          for (int c = 0; c < cnt; ++c) {
            float g[1];
            load(sel[k * NP + c], g);
            acc += g[0];
          }
          acc = sanitize_inf(acc * selscale[k]);
        } else {
          acc = kInf;
        }
        v[k][0] = acc;
      }
      coord_reduce<NP, 1, MODE>(v, n, f, beta, t, seed, thr, x0 + col, res);
    } else {
      coord_body<DT, NP, 1, MODE>(LdsLoader<DT>{tile, kCoordTile, col}, n, f, beta, W, t, seed, thr, x0 + col, res);
    }
    store_one(out, out_dt, x0 + col, res[0]);
    __syncthreads();
  }
  if (blockIdx.x == 0) {
    for (int64_t x = ntiles * kCoordTile + threadIdx.x; x < d; x += blockDim.x) {
      float res[1];
      coord_body<DT, NP, 1, MODE>(DirectLoader<DT, 1>{rows, x, false}, n, f, beta, W, t, seed, thr, x, res);
      store_one(out, out_dt, x, res[0]);
    }
  }
}

template <int DT, int NP, int VEC, int MODE>
void launch_coord(const RowTable& rows, int n, int64_t d, int f, int beta, const float* W, int t, uint64_t seed,
                  uint64_t thr, void* out, int out_dt, hipStream_t s) {
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  if constexpr (DT != kF32 && coord16_mode<MODE>()) {
    if (coord16_enabled()) {
      launch_coord16<DT, NP, MODE>(rows, n, d, f, beta, seed, thr, out, out_dt, s);
      return;
    }
  }
  if constexpr (MODE == kBulyanTail && DT != kF32) {
    if (n <= 64 && coord16_enabled() && coord_mfma_tail_enabled() &&
        launch_bulyan_tail_mfma<DT>(rows, n, d, beta, W, t, out, out_dt, s))
      return;
  }
  if constexpr (MODE == kBulyanTail && DT == kF32) {
    if (n <= 64 && coord16_enabled() && launch_bulyan_tail_f32(rows, n, d, beta, W, t, out, out_dt, s)) return;
  }
  if constexpr ((MODE == kBulyanTail || MODE == kAveragedMedian) && NP <= 64) {
    const int tt = MODE == kBulyanTail ? t : n;
    if (n <= 64 && tt - beta <= kTailMaxExcluded && coord16_enabled()) {
      launch_bulyan_tail<DT, NP>(rows, n, d, beta, MODE == kBulyanTail ? W : nullptr, t, out, out_dt, s);
      return;
    }
  }
  // LDS-staged path: NP >= 32, tile <= 64 KB, and (Bulyan tail) all n rows fit the NP-row tile
  if constexpr (NP >= 32 && NP * kCoordTile * ESZ <= 65536) {
    if (MODE != kBulyanTail || n <= NP) {
      int64_t g = d / kCoordTile;
      if (g < 1) g = 1;
      if (g > 2048) g = 2048;
      hipLaunchKernelGGL((k_coordwise_lds<DT, NP, MODE>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, rows, n,
                         d, f, beta, W, t, seed, thr, out, out_dt);
      return;
    }
  }
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
