// CPU implementations of every aggregation rule (float / double), used by the
// gloo / CPU configuration and as a second, independent implementation for the
// GPU kernels' tests. Semantics (tie-breaking, non-finite policy) are the ones
// documented in docs/GAR_SEMANTICS.md and are shared with the HIP kernels.
//
// Reference counterparts: py_krum/krum.cpp:50-118, py_bulyan/bulyan.cpp:53-193,
// py_median/median.cpp:42-77, py_brute/brute.cpp:47-113,
// TF deprecated_native/native.cpp:714-782 (averaged-median, average-nan).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace garfield {
namespace cpu {

template <class T>
struct Rows {
  std::vector<const T*> p;
  size_t n = 0;
  size_t d = 0;
};

// D[i*n + j] = ||g_i - g_j||^2 (double accumulation, fixed chunk order);
// non-finite -> +inf, diagonal -> +inf.
template <class T> std::vector<double> pairwise_sqdist(const Rows<T>& r);

// Selections (operate on the distance matrix, n x n).
std::vector<float> krum_weights(const std::vector<double>& D, size_t n, size_t f, size_t m,
                                std::vector<double>* scores = nullptr);
std::vector<float> bulyan_weights(const std::vector<double>& D, size_t n, size_t f, size_t m, size_t t);
std::vector<float> brute_weights(const std::vector<double>& D, size_t n, size_t f);
std::vector<float> aksel_weights(const std::vector<double>& dists, size_t n, size_t c);

// out = Σ_j w[j] g_j (accumulated in double)
template <class T> void combine(const Rows<T>& r, const std::vector<float>& w, T* out);

// Coordinate-wise rule (mode: garfield::CoordMode); W/t only for kBulyanTail.
template <class T>
void coordwise(const Rows<T>& r, int mode, size_t f, size_t beta, const std::vector<float>& W, size_t t,
               uint64_t seed, uint64_t threshold, T* out);

// dist_j = ||g_j - center||^2
template <class T> std::vector<double> sqdist_to(const Rows<T>& r, const T* center);

}  // namespace cpu
}  // namespace garfield
