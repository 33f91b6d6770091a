// Aggregation kernels for LARGE gradient sets (128 < n <= kLargeRows), gfx950.
//
// The main GAR kernels (gar_coord*.hpp, gar_gram.hip, gar_combine.hip) keep a worker's
// values in registers / sorting networks sized for n <= kMaxRows = 128 and address rows
// through a pointer table. The reference's gar_bench sweeps n up to 512
// (pytorch_impl/applications/benchmarks/gar_bench.py:41-58); here such sets arrive as
// one [n, ld] matrix (row stride ld) and run on:
//
// * k_large_combine: out[j] = Σ_i w[i] x[i, j] (fp32 accumulation over the non-zero
//   weights, compacted in LDS), the combine step of Krum / Multi-Krum / Brute / Aksel;
// * k_large_coord: coordinate-wise order statistics by LDS RADIX SELECT. A workgroup
//   stages a tile of 32 coordinates x n rows as order-preserving 32-bit keys in LDS
//   (n <= 1024: 128 KiB) and finds the k-th smallest key of each coordinate in eight
//   4-bit passes (8 lanes per coordinate, LDS histograms), without sorting:
//     median          value of rank cnt/2 among the finite values (0 if none);
//     trimmed-mean    mean of ranks [f, n - f) (NaN counted as +inf): two selects and
//                     one scan (Σ strictly between the two thresholds + tie copies);
//     averaged-median mean of the beta values closest to the median (rank n/2, NaN as
//                     +inf), ties in value order: a select on |x - med| keys computed
//                     on the fly, then one scan.
//   Semantics are those of ops/gar.py's vectorised PyTorch versions (_torch_coord).
// * k_large_near + k_large_select: Multi-Krum / Bulyan SELECTION from the fp32 Gram [n, n], on
//   device (no host round trip; reference semantics of ops/reference.py krum_weights /
//   bulyan_weights, distances in fp64):
//     k_large_near    one workgroup per row i: D[i, j] = g_ii + g_jj - 2 g_ij (fp64; +inf on the
//                     diagonal and where non-finite, else clamped at 0), bitonic-sorted as
//                     (value, index) pairs in LDS; the q-th pair is row i's neighbourhood
//                     threshold (j near i iff (D_ij, j) <= it) and Σ_j near D_ij its Krum score;
//     k_large_select  one workgroup: `rounds` selection rounds on the scores held in LDS; each
//                     round ranks every row by (score, index) (NaN as +inf) in one O(n) pass per
//                     lane, writes W[k] = 1/mk on the mk best, removes the best (score = FLT_MAX)
//                     and subtracts its distance from the rows it is near (Bulyan's P column).
#include <cfloat>
#include "gar_device.hpp"
#include "gar_gpu.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kTC = 32;                  // coordinates per workgroup
constexpr int kLanes = 8;                // lanes per coordinate
constexpr int kLT = kTC * kLanes;        // 256 threads
constexpr uint32_t kMaxKey = 0xffffffffu;

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int DT>
__device__ __forceinline__ float load1(const void* p, int64_t off) {
  if constexpr (DT == kF32) return static_cast<const float*>(p)[off];
  else return cvt16<DT>(static_cast<const uint16_t*>(p)[off]);
}

template <int DT>
__device__ __forceinline__ void store1(void* p, int64_t off, float v) {
  if constexpr (DT == kF32) static_cast<float*>(p)[off] = v;
  else if constexpr (DT == kBF16) static_cast<uint16_t*>(p)[off] = f_to_bf16(v);
  else static_cast<uint16_t*>(p)[off] = f_to_f16(v);
}

// ---------------------------------------------------------------------------

template <int DT>
__global__ __launch_bounds__(256) void k_large_combine(const void* __restrict__ x, int n, int64_t d, int64_t ld,
                                                       const float* __restrict__ w, void* __restrict__ out) {
  __shared__ int sel[kLargeRows];
  __shared__ float ws[kLargeRows];
  __shared__ int cnt;
  if (threadIdx.x == 0) {
    int c = 0;
    for (int i = 0; i < n; ++i)
      if (w[i] != 0.f) { sel[c] = i; ws[c] = w[i]; ++c; }
    cnt = c;
  }
  __syncthreads();
  const int m = cnt;
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < d;
       j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float acc = 0.f;
    for (int t = 0; t < m; ++t) acc += ws[t] * load1<DT>(x, static_cast<int64_t>(sel[t]) * ld + j);
    store1<DT>(out, j, acc);
  }
}

// ---------------------------------------------------------------------------

constexpr int MODE_MEDIAN = 0, MODE_TRIMMED = 1, MODE_AVGMED = 2;

// k-th smallest (0-based) of the keys produced by key_of(row) for this lane's coordinate.
// passes = 4 for keys of 16-bit values (bf16 / fp16 widened to fp32): their low 16 key bits
// are all 0 (positive) or all 1 (negative), so only the top 16 bits need selecting.
template <typename KeyOf>
__device__ uint32_t radix_select(int n, int k, int c, int lane8, uint32_t (*hist)[16], KeyOf key_of, int passes) {
  uint32_t prefix = 0, mask = 0;
  int kk = k;
#pragma unroll 1
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = 28 - 4 * pass;
    hist[c][lane8] = 0;          // 8 lanes clear the coordinate's 16 bins
    hist[c][lane8 + 8] = 0;
    __syncthreads();
    for (int i = lane8; i < n; i += kLanes) {
      const uint32_t key = key_of(i);
      if ((key & mask) == prefix) atomicAdd(&hist[c][(key >> shift) & 15u], 1u);
    }
    __syncthreads();
    int cum = 0, digit = 15;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int h = static_cast<int>(hist[c][b]);
      if (cum + h > kk) { digit = b; break; }
      cum += h;
    }
    kk -= cum;
    prefix |= static_cast<uint32_t>(digit) << shift;
    mask |= 15u << shift;
    __syncthreads();
  }
  if (passes == 4) prefix |= (prefix & 0x80000000u) ? 0u : 0xffffu;
  return prefix;
}

template <int DT, int MODE>
__global__ __launch_bounds__(kLT) void k_large_coord(const void* __restrict__ x, int n, int64_t d, int64_t ld, int f,
                                                     int beta, void* __restrict__ out) {
  __shared__ uint32_t keys[kLargeRows][kTC];
  __shared__ uint32_t hist[kTC][16];
  __shared__ float red[3][kLanes][kTC];
  __shared__ int redi[2][kLanes][kTC];
  const int c = threadIdx.x % kTC, lane8 = threadIdx.x / kTC;
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * kTC;
  const int64_t j = j0 + c;
  const bool valid = j < d;
  // stage keys (threads of one row read consecutive coordinates)
  for (int i = lane8; i < n; i += kLanes) {
    float v = valid ? load1<DT>(x, static_cast<int64_t>(i) * ld + j) : 0.f;
    uint32_t k;
    if constexpr (MODE == MODE_MEDIAN) k = __builtin_isfinite(v) ? fkey(v) : kMaxKey;
    else k = __builtin_isnan(v) ? fkey(__builtin_huge_valf()) : fkey(v);
    keys[i][c] = k;
  }
  __syncthreads();
  auto plain = [&](int i) { return keys[i][c]; };
  constexpr int PP = DT == kF32 ? 8 : 4;     // radix passes over the (widened) input values
  float result = 0.f;
  if constexpr (MODE == MODE_MEDIAN) {
    int cnt = 0;
    for (int i = lane8; i < n; i += kLanes) cnt += keys[i][c] != kMaxKey;
    redi[0][lane8][c] = cnt;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int l = 0; l < kLanes; ++l) tot += redi[0][l][c];
    const int k = tot / 2 < n - 1 ? tot / 2 : n - 1;
    const uint32_t key = radix_select(n, k, c, lane8, hist, plain, PP);
    result = tot > 0 ? kval(key) : 0.f;
  } else if constexpr (MODE == MODE_TRIMMED) {
    const uint32_t klo = radix_select(n, f, c, lane8, hist, plain, PP);
    const uint32_t khi = radix_select(n, n - f - 1, c, lane8, hist, plain, PP);
    float s = 0.f;
    int le_lo = 0, lt_hi = 0;
    for (int i = lane8; i < n; i += kLanes) {
      const uint32_t k = keys[i][c];
      if (k > klo && k < khi) s += kval(k);
      le_lo += k <= klo;
      lt_hi += k < khi;
    }
    red[0][lane8][c] = s;
    redi[0][lane8][c] = le_lo;
    redi[1][lane8][c] = lt_hi;
    __syncthreads();
    float S = 0.f;
    int LE = 0, LT = 0;
#pragma unroll
    for (int l = 0; l < kLanes; ++l) { S += red[0][l][c]; LE += redi[0][l][c]; LT += redi[1][l][c]; }
    const float vlo = kval(klo), vhi = kval(khi);
    const int keep = n - 2 * f;
    float total;
    if (klo == khi) {
      total = static_cast<float>(keep) * vlo;
    } else {
      const int clo = (LE < n - f ? LE : n - f) - f;
      const int chi = (n - f) - (LT > f ? LT : f);
      total = S;
      if (clo > 0) total += static_cast<float>(clo) * vlo;
      if (chi > 0) total += static_cast<float>(chi) * vhi;
    }
    result = total / static_cast<float>(keep);
  } else {  // MODE_AVGMED
    const float med = kval(radix_select(n, n / 2, c, lane8, hist, plain, PP));
    auto dist = [&](int i) {
      const float a = __builtin_fabsf(kval(keys[i][c]) - med);
      return __builtin_isnan(a) ? fkey(__builtin_huge_valf()) : fkey(a);
    };
    const uint32_t tk = radix_select(n, beta - 1, c, lane8, hist, dist, 8);
    float s = 0.f, slo = 0.f, shi = 0.f;
    int lt = 0, clo = 0, chi = 0;
    for (int i = lane8; i < n; i += kLanes) {
      const uint32_t dk = dist(i);
      const float v = kval(keys[i][c]);
      if (dk < tk) { s += v; ++lt; }
      else if (dk == tk) {
        if (v <= med) { slo += v; ++clo; }
        else { shi += v; ++chi; }
      }
    }
    red[0][lane8][c] = s;
    red[1][lane8][c] = slo;
    red[2][lane8][c] = shi;
    redi[0][lane8][c] = lt;
    redi[1][lane8][c] = clo | (chi << 16);
    __syncthreads();
    float S = 0.f, SL = 0.f, SH = 0.f;
    int LT = 0, CL = 0, CH = 0;
#pragma unroll
    for (int l = 0; l < kLanes; ++l) {
      S += red[0][l][c]; SL += red[1][l][c]; SH += red[2][l][c];
      LT += redi[0][l][c];
      CL += redi[1][l][c] & 0xffff;
      CH += redi[1][l][c] >> 16;
    }
    // the ties at distance t are taken in value order: low side first (equal values assumed per side)
    const int r = beta - LT;
    const int a = r < CL ? r : CL;
    float total = S;
    if (a > 0) total += SL * (static_cast<float>(a) / static_cast<float>(CL));
    if (r - a > 0 && CH > 0) total += SH * (static_cast<float>(r - a) / static_cast<float>(CH));
    result = total / static_cast<float>(beta);
  }
  if (valid && lane8 == 0) store1<DT>(out, j, result);
}

template <int DT>
void launch_coord(const void* x, int n, int64_t d, int64_t ld, int mode, int f, int beta, void* out,
                  hipStream_t stream) {
  const dim3 grid(static_cast<unsigned>((d + kTC - 1) / kTC));
  if (mode == MODE_MEDIAN) hipLaunchKernelGGL((k_large_coord<DT, MODE_MEDIAN>), grid, dim3(kLT), 0, stream, x, n, d, ld, f, beta, out);
  else if (mode == MODE_TRIMMED) hipLaunchKernelGGL((k_large_coord<DT, MODE_TRIMMED>), grid, dim3(kLT), 0, stream, x, n, d, ld, f, beta, out);
  else hipLaunchKernelGGL((k_large_coord<DT, MODE_AVGMED>), grid, dim3(kLT), 0, stream, x, n, d, ld, f, beta, out);
}

constexpr int kSelThreads = 1024;   // = kLargeRows: one lane per row

__device__ __forceinline__ double lg_dist(const float* __restrict__ g, int64_t ld, int i, int j) {
  if (i == j) return INFINITY;
  const double d = static_cast<double>(g[i * ld + i]) + static_cast<double>(g[j * ld + j]) -
                   2.0 * static_cast<double>(g[i * ld + j]);
  return isfinite(d) ? fmax(d, 0.0) : INFINITY;
}

__device__ __forceinline__ bool pair_less(double a, int ia, double b, int ib) {
  return a < b || (a == b && ia < ib);
}

__global__ __launch_bounds__(kSelThreads) void k_large_near(const float* __restrict__ g, int64_t ld, int n, int q,
                                                            double* __restrict__ thr_val, int* __restrict__ thr_idx,
                                                            double* __restrict__ nearsum) {
  __shared__ double val[kSelThreads];
  __shared__ double row[kSelThreads];
  __shared__ int idx[kSelThreads];
  const int i = blockIdx.x, t = threadIdx.x;
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  if (t < np2) {
    const double d = t < n ? lg_dist(g, ld, i, t) : INFINITY;
    val[t] = d;
    idx[t] = t;   // padding sorts after every real entry (index >= n)
    row[t] = d;
  }
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (t < np2) {
        const int p = t ^ j;
        if (p > t) {
          const bool up = (t & k) == 0;
          const bool sw = up ? pair_less(val[p], idx[p], val[t], idx[t]) : pair_less(val[t], idx[t], val[p], idx[p]);
          if (sw) {
            const double tv = val[t];
            val[t] = val[p];
            val[p] = tv;
            const int ti = idx[t];
            idx[t] = idx[p];
            idx[p] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  if (t == 0) {
    const double tv = val[q - 1];
    const int ti = idx[q - 1];
    double s = 0.0;
    for (int j = 0; j < n; ++j)
      if (!pair_less(tv, ti, row[j], j)) s += row[j];   // (D_ij, j) <= threshold: j is near i
    thr_val[i] = tv;
    thr_idx[i] = ti;
    nearsum[i] = s;
  }
}

__global__ __launch_bounds__(kSelThreads) void k_large_select(const float* __restrict__ g, int64_t ld, int n, int m,
                                                              int rounds, int shrink,
                                                              const double* __restrict__ thr_val,
                                                              const int* __restrict__ thr_idx,
                                                              const double* __restrict__ nearsum,
                                                              float* __restrict__ W) {
  __shared__ double sc[kSelThreads];
  __shared__ int best;
  const int i = threadIdx.x;
  const bool mine = i < n;
  double tv = 0.0;
  int ti = 0;
  if (mine) {
    sc[i] = nearsum[i];
    tv = thr_val[i];
    ti = thr_idx[i];
  }
  for (int k = 0; k < rounds; ++k) {
    __syncthreads();
    const int mk = shrink ? (m - k > 1 ? m - k : 1) : m;
    if (mine) {
      const double vi = isnan(sc[i]) ? INFINITY : sc[i];
      int r = 0;
      for (int j = 0; j < n; ++j) {
        const double vj = isnan(sc[j]) ? INFINITY : sc[j];
        r += pair_less(vj, j, vi, i);
      }
      W[static_cast<int64_t>(k) * n + i] = r < mk ? 1.0f / static_cast<float>(mk) : 0.0f;
      if (r == 0) best = i;
    }
    __syncthreads();
    const int b = best;
    if (mine) {
      if (i == b) {
        sc[i] = static_cast<double>(FLT_MAX);
      } else {
        const double dib = lg_dist(g, ld, i, b);
        if (!pair_less(tv, ti, dib, b)) sc[i] -= dib;   // b is among row i's q nearest: P[i, b]
      }
    }
  }
}

}  // namespace

void large_select(const float* gram, int64_t ld, int n, int f, int m, int rounds, bool shrink, double* thr_val,
                  int* thr_idx, double* nearsum, float* W, hipStream_t stream) {
  const int q = n - f - 2;
  hipLaunchKernelGGL(k_large_near, dim3(n), dim3(kSelThreads), 0, stream, gram, ld, n, q, thr_val, thr_idx, nearsum);
  hipLaunchKernelGGL(k_large_select, dim3(1), dim3(kSelThreads), 0, stream, gram, ld, n, m, rounds, shrink ? 1 : 0,
                     thr_val, thr_idx, nearsum, W);
}

void large_combine(const void* x, int dt, int n, int64_t d, int64_t ld, const float* w, void* out, hipStream_t stream) {
  if (d <= 0) return;
  int64_t blocks = (d + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  const dim3 grid(static_cast<unsigned>(blocks));
  if (dt == kF32) hipLaunchKernelGGL(k_large_combine<kF32>, grid, dim3(256), 0, stream, x, n, d, ld, w, out);
  else if (dt == kBF16) hipLaunchKernelGGL(k_large_combine<kBF16>, grid, dim3(256), 0, stream, x, n, d, ld, w, out);
  else hipLaunchKernelGGL(k_large_combine<kF16>, grid, dim3(256), 0, stream, x, n, d, ld, w, out);
}

void large_coord(const void* x, int dt, int n, int64_t d, int64_t ld, int mode, int f, int beta, void* out,
                 hipStream_t stream) {
  if (d <= 0) return;
  if (dt == kF32) launch_coord<kF32>(x, n, d, ld, mode, f, beta, out, stream);
  else if (dt == kBF16) launch_coord<kBF16>(x, n, d, ld, mode, f, beta, out, stream);
  else launch_coord<kF16>(x, n, d, ld, mode, f, beta, out, stream);
}

}  // namespace gpu
}  // namespace garfield
