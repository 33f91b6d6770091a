// Dispatcher of the coordinate-wise rules.
#include "gar_coord.hpp"

namespace garfield {
namespace gpu {

namespace coord {
template <> void coord_mode<kMedian>(int, int, const RowTable&, int, int64_t, int, int, const float*, int,
                               uint64_t, uint64_t, void*, int, hipStream_t);
template <> void coord_mode<kTrimmedMean>(int, int, const RowTable&, int, int64_t, int, int, const float*, int,
                               uint64_t, uint64_t, void*, int, hipStream_t);
template <> void coord_mode<kAveragedMedian>(int, int, const RowTable&, int, int64_t, int, int, const float*, int,
                               uint64_t, uint64_t, void*, int, hipStream_t);
template <> void coord_mode<kAverageNan>(int, int, const RowTable&, int, int64_t, int, int, const float*, int,
                               uint64_t, uint64_t, void*, int, hipStream_t);
template <> void coord_mode<kCondense>(int, int, const RowTable&, int, int64_t, int, int, const float*, int,
                               uint64_t, uint64_t, void*, int, hipStream_t);
template <> void coord_mode<kBulyanTail>(int, int, const RowTable&, int, int64_t, int, int, const float*, int,
                               uint64_t, uint64_t, void*, int, hipStream_t);
}  // namespace coord

int coordwise_max_rows() { return kMaxRows; }

void coordwise(const RowTable& rows, int n, int64_t d, int dt, int mode, int f, int beta, const float* W, int t,
               uint64_t seed, uint64_t threshold, void* out, int out_dt, hipStream_t stream) {
  const int k = (mode == kBulyanTail) ? t : n;
  const int np = coord::np_for(k);
  switch (mode) {
    case kMedian: coord::coord_mode<kMedian>(dt, np, rows, n, d, f, beta, W, t, seed, threshold, out, out_dt, stream); break;
    case kTrimmedMean: coord::coord_mode<kTrimmedMean>(dt, np, rows, n, d, f, beta, W, t, seed, threshold, out, out_dt, stream); break;
    case kAveragedMedian: coord::coord_mode<kAveragedMedian>(dt, np, rows, n, d, f, beta, W, t, seed, threshold, out, out_dt, stream); break;
    case kAverageNan: coord::coord_mode<kAverageNan>(dt, np, rows, n, d, f, beta, W, t, seed, threshold, out, out_dt, stream); break;
    case kCondense: coord::coord_mode<kCondense>(dt, np, rows, n, d, f, beta, W, t, seed, threshold, out, out_dt, stream); break;
    default: coord::coord_mode<kBulyanTail>(dt, np, rows, n, d, f, beta, W, t, seed, threshold, out, out_dt, stream); break;
  }
}

}  // namespace gpu
}  // namespace garfield
