// Shared (host + device) definitions of the Garfield-MI355X native layer.
//
// The reference keeps one dispatch header per backend
// (pytorch_impl/libs/native/include/aggregator.hpp:76-135) and passes gradient
// lists as a device pointer array uploaded with a synchronous cudaMemcpy per
// call (include/cudarray.cu.hpp:60-79). Here a gradient set is always described
// by a RowTable passed BY VALUE as a kernel argument: no allocation, no copy,
// and the launch stays hipGraph-capturable.
#pragma once
#include <cstdint>

namespace garfield {

// Largest number of gradients a single RowTable addresses (1 KiB of kernarg).
constexpr int kMaxRows = 128;
// Largest gradient set of the large-n kernels (gar_large.hip: one [n, ld] matrix, LDS radix select).
constexpr int kLargeRows = 1024;

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kF64 = 3 };

inline int dtype_size(int dt) { return dt == kF32 ? 4 : (dt == kF64 ? 8 : 2); }

struct RowTable {
  const void* p[kMaxRows];
};

// Coordinate-wise aggregation modes (gar_coord kernel family).
enum CoordMode : int {
  kMedian = 0,          // finite-only median, upper median (native py_median semantics)
  kTrimmedMean = 1,     // drop f lowest and f highest, mean of the rest (new rule)
  kAveragedMedian = 2,  // mean of the beta values closest to the median (TF MeaMed)
  kAverageNan = 3,      // mean of the finite values (TF average-nan)
  kCondense = 4,        // Bernoulli(p) mask: median where 1, gradients[0] where 0
  kBulyanTail = 5,      // v = W g (t rows), then averaged-median with beta = t - 2f
};

// Counter-based hash used by Condense on CPU and GPU alike, so both sides draw
// the same Bernoulli mask for a given (seed, coordinate).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t mix_hash(uint64_t seed, uint64_t x) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + x + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<uint32_t>(z >> 32);
}

// p in (0, 1]  ->  threshold on a uniform 32-bit draw (draw < thr  <=>  keep median)
inline uint64_t bernoulli_threshold(double p) {
  if (p >= 1.0) return 0x100000000ull;
  if (p <= 0.0) return 0;
  return static_cast<uint64_t>(p * 4294967296.0);
}

}  // namespace garfield
