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


// ---------------------------------------------------------------------------
// Gram matrix of a large set on MFMA (the selections' distances): G = X Xᵀ for n <= kLargeRows
// rows. The n x n output is cut into 64 x 64 tiles (4 x 4 blocks of 16 rows); workgroup
// (split s, tile pair (I, J), I <= J) multiplies rows I*64.. by rows J*64.. over the coordinate
// chunk of split s, each lane holding the same 64-byte slices of its A and B rows as MFMA operands
// (a common k permutation of both operands is free for a dot product, as in gar_gram.hip's n <= 128
// kernel), 4 waves over the chunk, combined in LDS. The split partials are summed in a fixed order
// by k_large_gram_reduce, which writes both triangles.
constexpr int kGT = 64;                  // tile rows
constexpr int kGTB = kGT / 16;           // 16-row blocks per tile side

__device__ __forceinline__ void tri_pair(int p, int T, int& I, int& J) {
  I = 0;
  while (p >= T - I) { p -= T - I; ++I; }
  J = I + p;
}

template <int DT>
__global__ __launch_bounds__(256) void k_large_gram_tile(const void* __restrict__ x, int n, int64_t d, int64_t ld,
                                                         int T, int64_t chunk, float* __restrict__ slabs) {
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  constexpr int KSPAN = 256 / ESZ;   // elements per row per wave step
  constexpr int QSPAN = KSPAN / 4;   // elements per lane per wave step
  __shared__ float red[kGTB * kGTB * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int split = blockIdx.x;
  int I, J;
  tri_pair(static_cast<int>(blockIdx.y), T, I, J);
  const int64_t d_main = (d / KSPAN) * KSPAN;
  const int64_t start = static_cast<int64_t>(split) * chunk;
  int64_t end = start + chunk;
  if (end > d_main) end = d_main;
  const char* base = static_cast<const char*>(x);
  const char* ap[kGTB];
  const char* bp[kGTB];
  bool av[kGTB], bv[kGTB];
#pragma unroll
  for (int a = 0; a < kGTB; ++a) {
    const int ra = I * kGT + a * 16 + r16, rb = J * kGT + a * 16 + r16;
    av[a] = ra < n;
    bv[a] = rb < n;
    ap[a] = base + static_cast<int64_t>(av[a] ? ra : 0) * ld * ESZ;
    bp[a] = base + static_cast<int64_t>(bv[a] ? rb : 0) * ld * ESZ;
  }
  f32x4 acc[kGTB][kGTB];
#pragma unroll
  for (int a = 0; a < kGTB; ++a)
#pragma unroll
    for (int b = 0; b < kGTB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t k = start + static_cast<int64_t>(wave) * KSPAN; k < end; k += 4 * KSPAN) {
    const int64_t off = (k + static_cast<int64_t>(q) * QSPAN) * ESZ;
    uint4 ua[kGTB][4], ub[kGTB][4];
#pragma unroll
    for (int a = 0; a < kGTB; ++a)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        ua[a][s4] = av[a] ? *reinterpret_cast<const uint4*>(ap[a] + off + 16 * s4) : make_uint4(0u, 0u, 0u, 0u);
        ub[a][s4] = bv[a] ? *reinterpret_cast<const uint4*>(bp[a] + off + 16 * s4) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
    for (int a = 0; a < kGTB; ++a)
#pragma unroll
      for (int b = 0; b < kGTB; ++b)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          if constexpr (DT == kBF16) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ua[a][s4]),
                                                                __builtin_bit_cast(bf16x8, ub[b][s4]), acc[a][b], 0, 0, 0);
          } else if constexpr (DT == kF16) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ua[a][s4]),
                                                               __builtin_bit_cast(f16x8, ub[b][s4]), acc[a][b], 0, 0, 0);
          } else {
            const float4 xa = __builtin_bit_cast(float4, ua[a][s4]);
            const float4 xb = __builtin_bit_cast(float4, ub[b][s4]);
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.x, xb.x, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.y, xb.y, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.z, xb.z, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.w, xb.w, acc[a][b], 0, 0, 0);
          }
        }
  }
  // 4 waves combined in LDS in a fixed order; C/D map: row = 4 (lane >> 4) + reg, column = lane & 15
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int a = 0; a < kGTB; ++a)
#pragma unroll
        for (int b = 0; b < kGTB; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int idx = (a * 16 + q * 4 + r) * kGT + b * 16 + r16;
            red[idx] = (w == 0 ? 0.f : red[idx]) + acc[a][b][r];
          }
    }
    __syncthreads();
  }
  if (split == 0 && d_main < d) {   // the < KSPAN trailing coordinates
    for (int e = threadIdx.x; e < kGT * kGT; e += 256) {
      const int i = I * kGT + e / kGT, j = J * kGT + e % kGT;
      if (i < n && j < n) {
        float sum = 0.f;
        for (int64_t c = d_main; c < d; ++c)
          sum += load1<DT>(x, static_cast<int64_t>(i) * ld + c) * load1<DT>(x, static_cast<int64_t>(j) * ld + c);
        red[e] += sum;
      }
    }
    __syncthreads();
  }
  float* slab = slabs + (static_cast<int64_t>(blockIdx.y) * gridDim.x + split) * (kGT * kGT);
  for (int e = threadIdx.x; e < kGT * kGT; e += 256) slab[e] = red[e];
}

// Σ over the splits (fixed order) of tile pair blockIdx.y, written to both triangles of gram [n, n].
__global__ __launch_bounds__(256) void k_large_gram_reduce(const float* __restrict__ slabs, int splits, int T, int n,
                                                           float* __restrict__ gram) {
  int I, J;
  tri_pair(static_cast<int>(blockIdx.y), T, I, J);
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kGT * kGT) return;
  const float* sp = slabs + static_cast<int64_t>(blockIdx.y) * splits * (kGT * kGT) + e;
  float sum = 0.f;
  for (int s2 = 0; s2 < splits; ++s2) sum += sp[static_cast<int64_t>(s2) * (kGT * kGT)];
  const int i = I * kGT + e / kGT, j = J * kGT + e % kGT;
  if (i < n && j < n) {
    gram[static_cast<int64_t>(i) * n + j] = sum;
    gram[static_cast<int64_t>(j) * n + i] = sum;
  }
}

// ---------------------------------------------------------------------------
// V = W · X on MFMA (Bulyan's t selection means of every coordinate): W [t, n] fp32 (rows of weights
// 1/mk), X [n, d] (row stride ld, bf16 / fp16 / fp32), V [t, d] fp32 (row stride ldv). fp32 MFMA
// (v_mfma_f32_16x16x4_f32) on X widened exactly to fp32, so V is the fp32 product of the reference.
// Workgroup tile: 64 rows of W x 256 coordinates, 16-deep k-steps staged in LDS (X widened to fp32
// on the way in); wave w owns coordinates [64 w, 64 w + 64) as 4 x 4 16x16 fragments.
constexpr int kWxT = 64, kWxC = 256, kWxK = 16, kWxXP = kWxC + 8, kWxWP = kWxK + 1;

template <int DT>
__global__ __launch_bounds__(256) void k_large_wx(const float* __restrict__ W, int t, int n, const void* __restrict__ x,
                                                  int64_t d, int64_t ld, float* __restrict__ V, int64_t ldv) {
  __shared__ float xs[kWxK * kWxXP];
  __shared__ float wsm[kWxT * kWxWP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * kWxC;
  const int t0 = blockIdx.y * kWxT;
  // staging roles: X row xr = tid / 16, 16 coordinates from xc = (tid % 16) * 16; W row wr = tid / 4, 4 k
  const int xr = threadIdx.x >> 4, xc = (threadIdx.x & 15) * 16;
  const int wr = threadIdx.x >> 2, wk = (threadIdx.x & 3) * 4;
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < n; k0 += kWxK) {
    {   // X tile [16 rows][256 coordinates] -> fp32 LDS
      const int row = k0 + xr;
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t c = c0 + xc + i;
        v[i] = (row < n && c < d) ? load1<DT>(x, static_cast<int64_t>(row) * ld + c) : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 16; i += 4)
        *reinterpret_cast<float4*>(&xs[xr * kWxXP + xc + i]) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    }
    {   // W tile [64 rows][16 k]
      const int row = t0 + wr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + wk + i;
        wsm[wr * kWxWP + wk + i] = (row < t && k < n) ? W[static_cast<int64_t>(row) * n + k] : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kWxK; kk += 4) {
      float av[4], bv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) av[a] = wsm[(a * 16 + r16) * kWxWP + kk + kq];
#pragma unroll
      for (int b = 0; b < 4; ++b) bv[b] = xs[(kk + kq) * kWxXP + wave * 64 + b * 16 + r16];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = t0 + a * 16 + kq * 4 + r;
        const int64_t c = c0 + wave * 64 + b * 16 + r16;
        if (row < t && c < d) V[static_cast<int64_t>(row) * ldv + c] = acc[a][b][r];
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


int large_gram_tiles(int n) { const int T = (n + kGT - 1) / kGT; return T * (T + 1) / 2; }

int large_gram_splits(int n, int64_t d, int dt) {
  const int64_t kspan = 256 / (dt == kF32 ? 4 : 2);
  const int64_t steps = d / kspan;
  const int pairs = large_gram_tiles(n);
  int64_t s = (1024 + pairs - 1) / pairs;   // ~1024 workgroups in all
  const int64_t maxs = steps / 32;          // >= 8 steps per wave
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  return static_cast<int>(s);
}

int64_t large_gram_slab_floats(int n, int64_t d, int dt) {
  return static_cast<int64_t>(large_gram_tiles(n)) * large_gram_splits(n, d, dt) * kGT * kGT;
}

namespace {
template <int DT> struct GramTiles {
  static void run(const void* x, int n, int64_t d, int64_t ld, float* slabs, float* gram, hipStream_t stream) {
    constexpr int64_t kspan = 256 / (DT == kF32 ? 4 : 2);
    const int T = (n + kGT - 1) / kGT;
    const int pairs = T * (T + 1) / 2;
    const int splits = large_gram_splits(n, d, DT);
    const int64_t steps = d / kspan;
    const int64_t per = (steps + splits - 1) / splits;
    const int64_t chunk = (per < 1 ? 1 : per) * kspan;
    hipLaunchKernelGGL((k_large_gram_tile<DT>), dim3(splits, pairs), dim3(256), 0, stream, x, n, d, ld, T, chunk,
                       slabs);
    hipLaunchKernelGGL(k_large_gram_reduce, dim3((kGT * kGT + 255) / 256, pairs), dim3(256), 0, stream, slabs, splits,
                       T, n, gram);
  }
};
template <int DT> struct Wx {
  static void run(const float* W, int t, int n, const void* x, int64_t d, int64_t ld, float* V, int64_t ldv,
                  hipStream_t stream) {
    const dim3 grid(static_cast<unsigned>((d + kWxC - 1) / kWxC), (t + kWxT - 1) / kWxT);
    hipLaunchKernelGGL((k_large_wx<DT>), grid, dim3(256), 0, stream, W, t, n, x, d, ld, V, ldv);
  }
};
}  // namespace

void large_gram(const void* x, int dt, int n, int64_t d, int64_t ld, float* slabs, float* gram, hipStream_t stream) {
  if (n <= 0) return;
  by_dtype<GramTiles>(dt, x, n, d, ld, slabs, gram, stream);
}

void large_wx(const float* W, int t, int n, const void* x, int dt, int64_t d, int64_t ld, float* V, int64_t ldv,
              hipStream_t stream) {
  if (t <= 0 || d <= 0) return;
  by_dtype<Wx>(dt, W, t, n, x, d, ld, V, ldv, stream);
}
}  // namespace gpu
}  // namespace garfield
