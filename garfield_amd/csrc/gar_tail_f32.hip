// Bulyan's tail on fp32 gradients (coordinate-wise closest-to-median mean of the t selected set
// means), its own translation unit: declared in gar_bulyan_tail.hpp, launched by launch_coord.
#include "gar_coord.hpp"

namespace garfield {
namespace gpu {
namespace coord {

// ---------------------------------------------------------------------------
// fp32 gradients: one lane per coordinate, the n gradient values of a 64-coordinate group in
// registers (loaded for the next group while this one computes). Set k's mean is the sum of its
// selected rows times the set's scale, in row order: Σ_j s_kj x_j with the 0/1 selection s_kj read
// from an LDS table (broadcast 16-byte reads: one FMA per row and set; a 0 x x_j term adds +0, the
// same sum as skipping the row) -- or, in a 64-coordinate group holding an inf / NaN (0 x inf would be
// NaN), with the set's bit mask as a select per row, so a value outside the set never reaches it (as
// the generic path's exact pass). The means are parked in the wave's LDS rows and read back into
// registers for window_mean's sort and window. Branch-free over the rows (rows >= n read row 0 under
// a zero weight). (The generic LDS-tile kernel stages 256 columns per workgroup between barriers and
// ran the fp32 rule at 0.8-1.0 TB/s.)
template <int NP, int NR>
__global__ __launch_bounds__(256) void k_bulyan_tail_f32(RowTable rows, int n, int64_t d, int beta,
                                                        const float* __restrict__ W, int t, void* out, int out_dt) {
  __shared__ __align__(16) float scratch[4][NP * 64];   // per wave: the set means [k][lane], then the spill
  __shared__ const float* sptr[NR];
  __shared__ uint64_t smask[NP];
  __shared__ float sscale[NP];
  __shared__ __align__(16) float sel[NP][NR];          // 0/1 selection table
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int k = wave; k < NP; k += 4) {   // set tables: one W row per wave iteration, masks by ballot
    const float w = (k < t && lane < n) ? W[k * n + lane] : 0.f;
    const uint64_t m = __builtin_amdgcn_ballot_w64(w != 0.f);
    const int first = m ? __builtin_ctzll(m) : 0;
    const float sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), first));
    if (lane == 0) {
      smask[k] = m;
      sscale[k] = m ? sc : 0.f;
    }
  }
  for (int j = threadIdx.x; j < NR; j += blockDim.x) sptr[j] = static_cast<const float*>(rows.p[j < n ? j : 0]);
  __syncthreads();
  for (int i = threadIdx.x; i < NP * NR; i += blockDim.x)
    sel[i / NR][i % NR] = (smask[i / NR] >> (i % NR)) & 1u ? 1.f : 0.f;
  __syncthreads();
  float* ks = scratch[wave];
  const float inv_beta = 1.f / static_cast<float>(beta);
  const int64_t ngroups = (d + 63) / 64;
  const int64_t gstep = static_cast<int64_t>(gridDim.x) * 4;
  const int64_t gfirst = static_cast<int64_t>(blockIdx.x) * 4 + wave;
  float nxt[NR];
  auto load = [&](int64_t gi) {
    const int64_t x = gi * 64 + lane;
    const int64_t xs = x < d ? x : d - 1;
#pragma unroll
    for (int j = 0; j < NR; ++j) nxt[j] = sptr[j][xs];
  };
  if (gfirst < ngroups) load(gfirst);
  for (int64_t gi = gfirst; gi < ngroups; gi += gstep) {
    float v[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) v[j] = nxt[j];
    if (gi + gstep < ngroups) load(gi + gstep);   // in flight during this group
    const int tt = opaque_uniform(t), bb = opaque_uniform(beta);
    bool fin = true;
#pragma unroll
    for (int j = 0; j < NR; ++j) fin = fin && isfinite(v[j]);
    if (__builtin_amdgcn_ballot_w64(!fin) == 0) {   // uniform: every value of the group finite
#pragma unroll 1
      for (int k = 0; k < tt; ++k) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < NR; j += 4) {
          const float4 w = *reinterpret_cast<const float4*>(&sel[k][j]);
          acc = fmaf(w.x, v[j], acc);
          acc = fmaf(w.y, v[j + 1], acc);
          acc = fmaf(w.z, v[j + 2], acc);
          acc = fmaf(w.w, v[j + 3], acc);
        }
        ks[k * 64 + lane] = sanitize_inf(acc * lds_volatile(sscale[k]));
      }
    } else {
#pragma unroll 1
      for (int k = 0; k < tt; ++k) {
        const uint64_t m = uniform64(lds_volatile(smask[k]));
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < NR; ++j) acc += ((m >> j) & 1u) ? v[j] : 0.f;
        ks[k * 64 + lane] = sanitize_inf(acc * lds_volatile(sscale[k]));
      }
    }
    float mean[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) mean[k] = k < tt ? ks[k * 64 + lane] : kInf;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read back before window_mean reuses the rows
    const float r = window_mean<NP, true>(mean, tt, bb, inv_beta, ks, lane);
    const int64_t x = gi * 64 + lane;
    if (x < d) store_one(out, out_dt, x, r);
  }
}

template <int NP>
void launch_tail_f32_nr(int nr, const RowTable& rows, int n, int64_t d, int beta, const float* W, int t, void* out,
                        int out_dt, hipStream_t s) {
  int64_t g = ((d + 63) / 64 + 3) / 4;
  const int64_t cap = tail_grid_cap(2048);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
#define GARFIELD_TAIL_F32(NRV)                                                                                     \
  hipLaunchKernelGGL((k_bulyan_tail_f32<NP, NRV>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, rows, n, d, beta, \
                     W, t, out, out_dt)
  switch (nr) {
    case 16: GARFIELD_TAIL_F32(16); break;
    case 32: GARFIELD_TAIL_F32(32); break;
    default: GARFIELD_TAIL_F32(64); break;
  }
#undef GARFIELD_TAIL_F32
}

// fp32, n <= 64, t <= 64, e = t - beta <= 16 (window_mean's layout, as the MFMA tail): the register
// kernel; otherwise false (generic kernels)
bool launch_bulyan_tail_f32(const RowTable& rows, int n, int64_t d, int beta, const float* W, int t, void* out,
                                   int out_dt, hipStream_t s) {
  if (n > 64 || t > 64 || t < 1 || beta < 1 || t - beta > kTailMaxExcluded || W == nullptr || d < 1) return false;
  const int np = t <= 8 ? 8 : (t <= 16 ? 16 : (t <= 32 ? 32 : 64));
  if (t / 2 < wm_p0(np) || beta < wm_p0(np)) return false;
  const int nr = n <= 16 ? 16 : (n <= 32 ? 32 : 64);
  switch (np) {
    case 8: launch_tail_f32_nr<8>(nr, rows, n, d, beta, W, t, out, out_dt, s); break;
    case 16: launch_tail_f32_nr<16>(nr, rows, n, d, beta, W, t, out, out_dt, s); break;
    case 32: launch_tail_f32_nr<32>(nr, rows, n, d, beta, W, t, out, out_dt, s); break;
    default: launch_tail_f32_nr<64>(nr, rows, n, d, beta, W, t, out, out_dt, s); break;
  }
  return true;
}

}  // namespace coord
}  // namespace gpu
}  // namespace garfield
