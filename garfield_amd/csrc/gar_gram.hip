// CDNA4 (gfx950 / MI355X) kernels for Byzantine-resilient gradient aggregation.
//
// What the reference does (pytorch_impl/libs/native):
//   K1/K1b  one squared_difference launch + one cub::DeviceReduce::Sum per PAIR
//           (n(n-1) launches, krum.cu:90-99), then a D2H copy + host sort,
//   K2      selection_average over a device pointer array (operations.cu.hpp:57-64),
//   K3-K8   Bulyan on a t x d intermediate (bulyan.cu:256-322, n <= 23),
//   K9      median with a per-thread n-array in shared memory (median.cu:60-83).
// What this file does instead:
//   gram      one split-K MFMA Gram kernel G·Gᵀ over the n x d gradient set
//             (bf16/fp16: v_mfma_f32_16x16x32_{bf16,f16}; fp32: v_mfma_f32_16x16x4_f32),
//             each wave streaming 256 contiguous bytes per row per step, 4-wave LDS
//             combine, deterministic fixed-order slab reduction;
//   select    Krum / Bulyan / Brute selection inside ONE workgroup on the device
//             (rank counting over an LDS distance matrix, no sort, no host copy);
//   combine   weighted row combine with 16-byte loads, optionally fused with the
//             SGD(momentum, weight-decay, nesterov) update of fp32 master weights;
//   coordwise register bitonic sorting networks (NP = 8..128 rows, VEC coordinates
//             per lane) for median / trimmed-mean / averaged-median / Condense /
//             average-nan, and the Bulyan tail fused with its W·G selection (no t x d
//             intermediate).
#include <cstdlib>

#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

// ---------------------------------------------------------------------------
// Gram: partial G·Gᵀ per split-K chunk on MFMA.
//
// Lane l of a wave owns row (16a + (l & 15)) of every 16-row block a and the
// contiguous 64-byte slice [q*QSPAN, (q+1)*QSPAN) (q = l >> 4) of the wave's
// 256-byte K step. A Gram entry sums over k, so the same k permutation on the
// A and B operands is free: the fragment a lane loads for block a is at once
// its A operand (rows of block a) and its B operand (columns of block a).

template <int DT, int NB>
__global__ __launch_bounds__(256) void k_gram_partial(RowTable rows, int n, int64_t d,
                                                     int64_t chunk, float* __restrict__ slabs) {
  constexpr int NPAIR = NB * (NB + 1) / 2;
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  constexpr int KSPAN = 256 / ESZ;   // elements per row per wave step
  constexpr int QSPAN = KSPAN / 4;   // elements per lane per wave step
  __shared__ float red[NPAIR * 256];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int64_t d_main = (d / KSPAN) * KSPAN;
  const int64_t start = static_cast<int64_t>(blockIdx.x) * chunk;
  int64_t end = start + chunk;
  if (end > d_main) end = d_main;

  const char* rp[NB];
  bool rv[NB];
#pragma unroll
  for (int a = 0; a < NB; ++a) {
    const int row = a * 16 + r16;
    rv[a] = row < n;
    rp[a] = rv[a] ? static_cast<const char*>(rows.p[row]) : nullptr;
  }

  f32x4 acc[NPAIR];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int64_t k = start + static_cast<int64_t>(wave) * KSPAN; k < end; k += 4 * KSPAN) {
    const int64_t off = (k + static_cast<int64_t>(q) * QSPAN) * ESZ;
    uint4 u[NB][4];
#pragma unroll
    for (int a = 0; a < NB; ++a) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (rv[a]) u[a][s] = *reinterpret_cast<const uint4*>(rp[a] + off + 16 * s);
        else u[a][s] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    int p = 0;
#pragma unroll
    for (int a = 0; a < NB; ++a) {
#pragma unroll
      for (int b = a; b < NB; ++b) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if constexpr (DT == kBF16) {
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, u[a][s]), __builtin_bit_cast(bf16x8, u[b][s]), acc[p], 0, 0, 0);
          } else if constexpr (DT == kF16) {
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                __builtin_bit_cast(f16x8, u[a][s]), __builtin_bit_cast(f16x8, u[b][s]), acc[p], 0, 0, 0);
          } else {
            const float4 xa = __builtin_bit_cast(float4, u[a][s]);
            const float4 xb = __builtin_bit_cast(float4, u[b][s]);
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.x, xb.x, acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.y, xb.y, acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.z, xb.z, acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.w, xb.w, acc[p], 0, 0, 0);
          }
        }
        ++p;
      }
    }
  }

  // Combine the 4 waves in LDS, wave by wave (fixed order => deterministic).
  // C/D map of the 16x16 MFMA: column = lane & 15, row = 4 * (lane >> 4) + reg.
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int idx = p * 256 + (q * 4 + r) * 16 + r16;
          red[idx] = (w == 0 ? 0.f : red[idx]) + acc[p][r];
        }
      }
    }
    __syncthreads();
  }

  // Tail (< KSPAN trailing coordinates): scalar, done by workgroup 0 only.
  if (blockIdx.x == 0 && d_main < d) {
    for (int e = threadIdx.x; e < NPAIR * 256; e += 256) {
      int p = e >> 8, a = 0;
      while (p >= NB - a) { p -= NB - a; ++a; }
      const int b = a + p;
      const int i = a * 16 + ((e >> 4) & 15);
      const int j = b * 16 + (e & 15);
      if (i < n && j < n) {
        float s = 0.f;
        for (int64_t x = d_main; x < d; ++x) s += load_one<DT>(rows.p[i], x) * load_one<DT>(rows.p[j], x);
        red[e] += s;
      }
    }
    __syncthreads();
  }

  float* slab = slabs + static_cast<int64_t>(blockIdx.x) * (NPAIR * 256);
  for (int e = threadIdx.x; e < NPAIR * 256; e += 256) slab[e] = red[e];
}

// Stage 1 of the slab reduction: block (bx, r) sums, for 64 entries, the slabs
// g = r, r + R, r + 2R, ... (split over its 4 waves in a fixed order) into part[r].
// Spreads the ~1024-slab reduction over ceil(E/64) x R workgroups instead of a
// handful of latency-bound ones.
__global__ __launch_bounds__(256) void k_gram_reduce_stage1(const float* __restrict__ slabs, int nslab, int E,
                                                            int R, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int r = blockIdx.y;
  __shared__ float acc[4][64];
  float s = 0.f;
  if (e < E)
    for (int g = r + R * wave; g < nslab; g += 4 * R) s += slabs[static_cast<int64_t>(g) * E + e];
  acc[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < E) part[static_cast<int64_t>(r) * E + e] = ((acc[0][lane] + acc[1][lane]) + acc[2][lane]) + acc[3][lane];
}

// Fixed-order reduction of the split-K slabs into the symmetric np x np Gram.
__global__ __launch_bounds__(256) void k_gram_reduce(const float* __restrict__ slabs, int nslab,
                                                     int nb, float* __restrict__ gram) {
  const int npair = nb * (nb + 1) / 2;
  const int E = npair * 256;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  __shared__ float part[4][64];
  float s = 0.f;
  if (e < E)
    for (int g = wave; g < nslab; g += 4) s += slabs[static_cast<int64_t>(g) * E + e];
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < E) {
    const float tot = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    int p = e >> 8, a = 0;
    while (p >= nb - a) { p -= nb - a; ++a; }
    const int b = a + p;
    const int i = a * 16 + ((e >> 4) & 15);
    const int j = b * 16 + (e & 15);
    const int np = nb * 16;
    gram[i * np + j] = tot;
    gram[j * np + i] = tot;
  }
}

// ---------------------------------------------------------------------------
// Selection kernels: one workgroup of 1024 threads (16 waves). Row i of the
// distance matrix is handled by wave (i % 16); each lane owns columns
// (lane, lane + 64). Ranks are counted, not sorted: rank(i,j) = #{k != i :
// (D_ik, k) < (D_ij, j)}, which gives a strict total order, hence the same
// selection on every rank of a data-parallel job and on the CPU oracle.

// D (pitch n+1) from the Gram; diagonal = +inf, non-finite = +inf, clamped at 0.
__device__ void fill_distances(const float* __restrict__ gram, int np, int n, float* D) {
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    const int i = e / n, j = e % n;
    float v;
    if (i == j) {
      v = kInf;
    } else {
      v = gram[i * np + i] + gram[j * np + j] - 2.f * gram[i * np + j];
      if (!isfinite(v)) v = kInf;
      v = fmaxf(v, 0.f);
    }
    D[i * (n + 1) + j] = v;
  }
}

// Krum score of row i (sum of the q smallest off-diagonal distances); when
// keep != nullptr, also reports whether column j is among the q nearest.
__device__ float row_score(const float* D, int n, int i, int q, int lane, bool keep[2]) {
  const float* row = D + i * (n + 1);
  float contrib = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int j = lane + 64 * c;
    keep[c] = false;
    if (j < n && j != i) {
      const float dj = row[j];
      int rank = 0;
      for (int k = 0; k < n; ++k) {
        const float dk = row[k];
        rank += (k != i) && (dk < dj || (dk == dj && k < j));
      }
      if (rank < q) { contrib += dj; keep[c] = true; }
    }
  }
  return wave_sum(contrib);
}

__global__ __launch_bounds__(1024) void k_krum_select(const float* __restrict__ gram, int np, int n,
                                                      int f, int m, float* __restrict__ weights,
                                                      int* __restrict__ order, float* __restrict__ scores) {
  extern __shared__ float lds[];
  // workgroup b selects problem b of a batch (the layer-wise GAR: one Gram per parameter segment)
  gram += static_cast<int64_t>(blockIdx.x) * np * np;
  weights += static_cast<int64_t>(blockIdx.x) * n;
  order += static_cast<int64_t>(blockIdx.x) * n;
  scores += static_cast<int64_t>(blockIdx.x) * n;
  float* D = lds;                    // n * (n + 1)
  float* S = lds + n * (n + 1);      // n
  fill_distances(gram, np, n, D);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = n - f - 2;
  for (int i = wave; i < n; i += 16) {
    bool keep[2];
    const float s = row_score(D, n, i, q, lane, keep);
    if (lane == 0) S[i] = s;
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i < n) {
    const int r = score_rank(S, n, i);
    weights[i] = r < m ? 1.f / static_cast<float>(m) : 0.f;
    order[r] = i;
    scores[i] = S[i];
  }
}

__global__ __launch_bounds__(1024) void k_bulyan_select(const float* __restrict__ gram, int np, int n,
                                                        int f, int m, int t, float* __restrict__ W) {
  extern __shared__ float lds[];
  // workgroup b selects problem b of a batch (the layer-wise GAR: one Gram per parameter segment)
  gram += static_cast<int64_t>(blockIdx.x) * np * np;
  W += static_cast<int64_t>(blockIdx.x) * t * n;
  float* D = lds;                    // n * (n + 1); becomes the pruned distances
  float* S = lds + n * (n + 1);      // n scores
  __shared__ int best;
  fill_distances(gram, np, n, D);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = n - f - 2;
  bool keep[8][2];  // rows handled by this wave: wave, wave + 16, ... (n <= 128)
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int i = wave + 16 * r;
    keep[r][0] = keep[r][1] = false;
    if (i < n) {
      const float s = row_score(D, n, i, q, lane, keep[r]);
      if (lane == 0) S[i] = s;
    }
  }
  __syncthreads();
  // Prune: keep only each row's q nearest (native py_bulyan/bulyan.cpp:118-129).
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int i = wave + 16 * r;
    if (i < n) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = lane + 64 * c;
        if (j < n && j != i && !keep[r][c]) D[i * (n + 1) + j] = 0.f;
      }
    }
  }
  __syncthreads();
  // t selection steps; each rank count is split over G lanes of one wave (G = 16 for
  // n <= 64, 8 for n <= 128) and summed with a 16/8-lane butterfly, so a step costs
  // n / G LDS reads per lane instead of a serial pass over all n scores
  const int G = n <= 64 ? 16 : 8;
  const int i = threadIdx.x / G, c = threadIdx.x % G;
  for (int k = 0; k < t; ++k) {
    int mk = m - k;
    if (mk < 1) mk = 1;
    int r = 0;
    if (i < n) {
      const float si = sanitize_inf(S[i]);
      for (int j = c; j < n; j += G) {
        const float sj = sanitize_inf(S[j]);
        r += (sj < si) || (sj == si && j < i);
      }
    }
    for (int o = G / 2; o >= 1; o >>= 1) r += __shfl_xor(r, o, G);
    if (i < n && c == 0) {
      W[k * n + i] = r < mk ? 1.f / static_cast<float>(mk) : 0.f;
      if (r == 0) best = i;
    }
    __syncthreads();
    const int id = best;
    if (i < n && c == 0) S[i] = i == id ? FLT_MAX : S[i] - D[i * (n + 1) + id];
    __syncthreads();
  }
}

// Brute: smallest-diameter subset of size k = n - f among C(n, k), enumerated
// as k-bit masks in increasing numeric order (combinatorial number system).
__device__ __forceinline__ unsigned long long binom(int a, int b) {
  if (b < 0 || b > a) return 0ull;
  if (b > a - b) b = a - b;
  unsigned long long r = 1;
  for (int i = 1; i <= b; ++i) r = r * static_cast<unsigned long long>(a - b + i) / static_cast<unsigned long long>(i);
  return r;
}

__global__ __launch_bounds__(256) void k_brute_search(const float* __restrict__ gram, int np, int n, int k,
                                                      unsigned long long total, unsigned long long per,
                                                      unsigned long long* __restrict__ best) {
  __shared__ float D[64 * 65];
  __shared__ unsigned long long wbest[4];
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    const int i = e / n, j = e % n;
    float v = gram[i * np + i] + gram[j * np + j] - 2.f * gram[i * np + j];
    if (!isfinite(v)) v = FLT_MAX;
    D[i * 65 + j] = fmaxf(v, 0.f);
  }
  __syncthreads();
  unsigned long long my = ~0ull;
  const unsigned long long tid = static_cast<unsigned long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const unsigned long long r0 = tid * per;
  if (r0 < total) {
    // Unrank r0.
    unsigned long long r = r0, mask = 0ull;
    int kk = k;
    for (int i = n - 1; i >= 0 && kk > 0; --i) {
      const unsigned long long c = binom(i, kk);
      if (c <= r) { mask |= 1ull << i; r -= c; --kk; }
    }
    unsigned long long r1 = r0 + per;
    if (r1 > total) r1 = total;
    for (unsigned long long rank = r0; rank < r1; ++rank) {
      float diam = 0.f;
      unsigned long long mi = mask;
      while (mi) {
        const int i = __builtin_ctzll(mi);
        mi &= mi - 1ull;
        unsigned long long mj = mi;
        while (mj) {
          const int j = __builtin_ctzll(mj);
          mj &= mj - 1ull;
          diam = fmaxf(diam, D[i * 65 + j]);
        }
      }
      const unsigned long long key = (static_cast<unsigned long long>(__float_as_uint(diam)) << 32) | rank;
      if (key < my) my = key;
      // Gosper: next k-bit mask in numeric order.
      const unsigned long long c = mask & (~mask + 1ull);
      const unsigned long long rr = mask + c;
      mask = (((rr ^ mask) >> 2) / c) | rr;
    }
  }
  // wave min then block min then one atomic per block (order-independent => deterministic)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(my, o, 64);
    my = other < my ? other : my;
  }
  if ((threadIdx.x & 63) == 0) wbest[threadIdx.x >> 6] = my;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = wbest[0];
    for (int w = 1; w < 4; ++w) b = wbest[w] < b ? wbest[w] : b;
    atomicMin(best, b);
  }
}

__global__ void k_brute_init(unsigned long long* best) { *best = ~0ull; }

__global__ void k_brute_finalize(const unsigned long long* __restrict__ best, int n, int k,
                                 float* __restrict__ weights) {
  __shared__ unsigned long long mask;
  if (threadIdx.x == 0) {
    unsigned long long r = (*best) & 0xffffffffull, msk = 0ull;
    int kk = k;
    for (int i = n - 1; i >= 0 && kk > 0; --i) {
      const unsigned long long c = binom(i, kk);
      if (c <= r) { msk |= 1ull << i; r -= c; --kk; }
    }
    mask = msk;
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i < n) weights[i] = ((mask >> i) & 1ull) ? 1.f / static_cast<float>(k) : 0.f;
}

}  // namespace

// ---------------------------------------------------------------------------
// Gram

int gram_nb(int n) { return n <= 16 ? 1 : (n <= 32 ? 2 : (n <= 64 ? 4 : 8)); }
int gram_padded(int n) { return 16 * gram_nb(n); }
int64_t gram_slab_floats(int n) { const int nb = gram_nb(n); return static_cast<int64_t>(nb * (nb + 1) / 2) * 256; }

int gram_grid(int64_t d, int dt, int n) {
  (void)n;
  const int64_t kspan = 256 / (dt == kF32 ? 4 : 2);
  const int64_t steps = d / kspan;         // wave steps over the whole vector
  int64_t g = steps / 32;                  // >= 8 steps per wave
  if (g < 1) g = 1;
  static const int64_t cap = [] {   // tuning knob: split-K workgroup cap
    const char* e = std::getenv("GARFIELD_GRAM_MAXGRID");
    const long v = e ? std::atol(e) : 0;
    return static_cast<int64_t>(v > 0 ? v : 1024);
  }();
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

namespace {
template <int DT, int NB>
void launch_gram_partial(const RowTable& rows, int n, int64_t d, int grid, float* slabs, hipStream_t s) {
  constexpr int64_t kspan = 256 / (DT == kF32 ? 4 : 2);
  const int64_t steps = d / kspan;
  const int64_t per = (steps + grid - 1) / grid;
  const int64_t chunk = (per < 1 ? 1 : per) * kspan;
  hipLaunchKernelGGL((k_gram_partial<DT, NB>), dim3(grid), dim3(256), 0, s, rows, n, d, chunk, slabs);
}
template <int DT> struct GramPartial {
  static void run(const RowTable& rows, int n, int64_t d, int grid, float* slabs, hipStream_t s) {
    switch (gram_nb(n)) {
      case 1: launch_gram_partial<DT, 1>(rows, n, d, grid, slabs, s); break;
      case 2: launch_gram_partial<DT, 2>(rows, n, d, grid, slabs, s); break;
      case 4: launch_gram_partial<DT, 4>(rows, n, d, grid, slabs, s); break;
      default: launch_gram_partial<DT, 8>(rows, n, d, grid, slabs, s); break;
    }
  }
};
}  // namespace

void gram(const RowTable& rows, int n, int64_t d, int dt, float* slabs, int grid, float* gram_out,
          hipStream_t stream) {
  by_dtype<GramPartial>(dt, rows, n, d, grid, slabs, stream);
  const int nb = gram_nb(n);
  const int E = nb * (nb + 1) / 2 * 256;
  if (grid > 2 * kGramReduceGroups) {
    // two-stage deterministic reduction: grid slabs -> kGramReduceGroups partials -> gram
    float* part = slabs + static_cast<int64_t>(grid) * E;
    hipLaunchKernelGGL(k_gram_reduce_stage1, dim3((E + 63) / 64, kGramReduceGroups), dim3(256), 0, stream, slabs,
                       grid, E, kGramReduceGroups, part);
    hipLaunchKernelGGL(k_gram_reduce, dim3((E + 63) / 64), dim3(256), 0, stream, part, kGramReduceGroups, nb,
                       gram_out);
  } else {
    hipLaunchKernelGGL(k_gram_reduce, dim3((E + 63) / 64), dim3(256), 0, stream, slabs, grid, nb, gram_out);
  }
}

// ---------------------------------------------------------------------------
// Selection

static size_t select_lds_bytes(int n) { return static_cast<size_t>(n * (n + 1) + n) * sizeof(float); }

static void allow_big_lds(const void* fn) {
  // 128 x 129 fp32 distance matrix + scores = 66.6 KB > the 64 KB default
  // (n <= 128). Ask for 96 KB: the static __shared__ of the kernel counts against the 160 KB too.
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) != hipSuccess)
    (void)hipGetLastError();  // never leave a sticky error for the framework to trip over
}

void krum_select(const float* gram_in, int np, int n, int f, int m, float* weights, int* order, float* scores,
                 hipStream_t stream, int batch) {
  static bool once = (allow_big_lds(reinterpret_cast<const void*>(&k_krum_select)), true);
  (void)once;
  hipLaunchKernelGGL(k_krum_select, dim3(batch), dim3(1024), select_lds_bytes(n), stream, gram_in, np, n, f, m,
                     weights, order, scores);
}

void bulyan_select(const float* gram_in, int np, int n, int f, int m, int t, float* W, hipStream_t stream, int batch) {
  static bool once = (allow_big_lds(reinterpret_cast<const void*>(&k_bulyan_select)), true);
  (void)once;
  hipLaunchKernelGGL(k_bulyan_select, dim3(batch), dim3(1024), select_lds_bytes(n), stream, gram_in, np, n, f, m, t,
                     W);
}

static unsigned long long host_binom(int a, int b) {
  if (b < 0 || b > a) return 0ull;
  if (b > a - b) b = a - b;
  unsigned long long r = 1;
  for (int i = 1; i <= b; ++i) r = r * static_cast<unsigned long long>(a - b + i) / static_cast<unsigned long long>(i);
  return r;
}

void brute_select(const float* gram_in, int np, int n, int f, unsigned long long* best, float* weights,
                  hipStream_t stream) {
  const int k = n - f;
  const unsigned long long total = host_binom(n, k);
  const unsigned long long threads_max = 256ull * 2048ull;
  unsigned long long per = (total + threads_max - 1) / threads_max;
  if (per < 1) per = 1;
  const unsigned long long threads = (total + per - 1) / per;
  const unsigned int blocks = static_cast<unsigned int>((threads + 255) / 256);
  hipLaunchKernelGGL(k_brute_init, dim3(1), dim3(1), 0, stream, best);
  hipLaunchKernelGGL(k_brute_search, dim3(blocks), dim3(256), 0, stream, gram_in, np, n, k, total, per, best);
  hipLaunchKernelGGL(k_brute_finalize, dim3(1), dim3(64), 0, stream, best, n, k, weights);
}

}  // namespace gpu
}  // namespace garfield
