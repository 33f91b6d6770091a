// Instantiation of the coordinate-wise kernels for mode kAveragedMedian.
#include "gar_coord.hpp"

namespace garfield {
namespace gpu {
namespace coord {

template <>
void coord_mode<kAveragedMedian>(int dt, int np, const RowTable& rows, int n, int64_t d, int f, int beta,
                       const float* W, int t, uint64_t seed, uint64_t thr, void* out, int out_dt,
                       hipStream_t s) {
  by_dtype<ByDtype<kAveragedMedian>::F>(dt, np, rows, n, d, f, beta, W, t, seed, thr, out, out_dt, s);
}

}  // namespace coord
}  // namespace gpu
}  // namespace garfield
