// Layer-wise robust aggregation on gfx950: the GAR applied to every parameter segment of the
// flat [n, d] gradient rows in a handful of launches instead of one Gram / selection / combine
// per parameter tensor.
//
// Reference semantics: pytorch_impl/applications/Garfield_CC/trainer.py:100,125 (--layerwise:
// the rule runs on each layer's gradient slice separately). A ResNet-50 has 161 parameter
// tensors, so a per-tensor loop is ~480 launches with tiny grids; here:
//
//   lw_gram         one split-K MFMA Gram launch over a JOB table (each job a coordinate range
//                   inside one segment) writing a partial [np, np] slab per job, then one
//                   fixed-order segmented reduction into gram[L][np][np];
//   krum_select     the existing one-workgroup selection, batched: workgroup s selects segment s
//                   (bulyan_select likewise: W [L][t][n]);
//   lw_bulyan_tail  Bulyan's tail per coordinate with its segment's W [t][n] (the t selection
//                   means, then their averaged median: the flat tail's per-coordinate code);
//   lw_combine_sgd  one launch: job j combines its coordinates with its segment's weights and
//                   applies the fused SGD update (the same per-element arithmetic as k_combine +
//                   k_combine_sgd: 8-wide groups from the segment start, 4 rows per step, a scalar
//                   tail), so the result is bitwise that of the per-segment path.
//
// Segment boundaries are arbitrary element offsets (a BatchNorm bias of 64, a 9408-element
// stem): 16-byte loads where a group is aligned, element loads where it is not.
#include <cstdlib>

#include "gar_coord.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

// GARFIELD_LW_TAIL_MFMA=0: the scalar per-coordinate tail (A/B switch)
bool lw_tail_mfma_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("GARFIELD_LW_TAIL_MFMA");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// ---------------------------------------------------------------------------------------------
// Segmented Gram partials: the k_gram_partial scheme (gar_gram.hip) over [start, end) of one
// job; pieces straddling the range ends are masked element by element.
template <int DT, int NB>
__global__ __launch_bounds__(256) void k_lw_gram_partial(RowTable rows, int n, const int64_t* __restrict__ jobs,
                                                         float* __restrict__ slabs) {
  constexpr int NPAIR = NB * (NB + 1) / 2;
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  constexpr int KSPAN = 256 / ESZ;   // elements per row per wave step
  constexpr int QSPAN = KSPAN / 4;   // elements per lane per wave step
  constexpr int PE = 16 / ESZ;       // elements per 16-byte piece
  __shared__ float red[NPAIR * 256];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int64_t a = jobs[3 * blockIdx.x], b = jobs[3 * blockIdx.x + 1];
  const int64_t base = a - (a % PE);                  // piece-aligned start

  const char* rp[NB];
  bool rv[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = i * 16 + r16;
    rv[i] = row < n;
    rp[i] = rv[i] ? static_cast<const char*>(rows.p[row]) : nullptr;
  }
  f32x4 acc[NPAIR];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int64_t k = base + static_cast<int64_t>(wave) * KSPAN; k < b; k += 4 * KSPAN) {
    uint4 u[NB][4];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int64_t e0 = k + static_cast<int64_t>(q) * QSPAN + PE * s;   // first element of the piece
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (rv[i]) {
          const bool aligned = (reinterpret_cast<uintptr_t>(rp[i] + e0 * ESZ) & 15) == 0;
          if (e0 >= a && e0 + PE <= b && aligned) {
            v = *reinterpret_cast<const uint4*>(rp[i] + e0 * ESZ);
          } else if (e0 + PE > a && e0 < b) {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < PE; ++e) {
              const int64_t x = e0 + e;
              if (x >= a && x < b) {
                if constexpr (ESZ == 4) {
                  w[e] = *reinterpret_cast<const uint32_t*>(rp[i] + x * 4);
                } else {
                  const uint32_t h = *reinterpret_cast<const uint16_t*>(rp[i] + x * 2);
                  w[e >> 1] |= (e & 1) ? (h << 16) : h;
                }
              }
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
        u[i][s] = v;
      }
    }
    int p = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
#pragma unroll
      for (int j = i; j < NB; ++j) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if constexpr (DT == kBF16) {
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, u[i][s]),
                                                             __builtin_bit_cast(bf16x8, u[j][s]), acc[p], 0, 0, 0);
          } else if constexpr (DT == kF16) {
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, u[i][s]),
                                                            __builtin_bit_cast(f16x8, u[j][s]), acc[p], 0, 0, 0);
          } else {
            const float4 xa = __builtin_bit_cast(float4, u[i][s]);
            const float4 xb = __builtin_bit_cast(float4, u[j][s]);
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
  // the 4 waves in LDS, in a fixed order (deterministic); C/D map: col = lane & 15, row = 4q + reg
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int p = 0; p < NPAIR; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int idx = p * 256 + (q * 4 + r) * 16 + r16;
          red[idx] = (w == 0 ? 0.f : red[idx]) + acc[p][r];
        }
    }
    __syncthreads();
  }
  float* slab = slabs + static_cast<int64_t>(blockIdx.x) * (NPAIR * 256);
  for (int e = threadIdx.x; e < NPAIR * 256; e += 256) slab[e] = red[e];
}

// gram[s] (symmetric np x np) = Σ over the jobs of segment s of their slabs, in job order.
__global__ __launch_bounds__(256) void k_lw_gram_reduce(const float* __restrict__ slabs, const int* __restrict__ seg_lo,
                                                        int nb, float* __restrict__ gram) {
  const int npair = nb * (nb + 1) / 2;
  const int E = npair * 256;
  const int s = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float tot = 0.f;
  for (int j = seg_lo[s]; j < seg_lo[s + 1]; ++j) tot += slabs[static_cast<int64_t>(j) * E + e];
  int p = e >> 8, ia = 0;
  while (p >= nb - ia) { p -= nb - ia; ++ia; }
  const int ib = ia + p;
  const int i = ia * 16 + ((e >> 4) & 15);
  const int jj = ib * 16 + (e & 15);
  const int np = nb * 16;
  float* g = gram + static_cast<int64_t>(s) * np * np;
  g[i * np + jj] = tot;
  g[jj * np + i] = tot;
}

// ---------------------------------------------------------------------------------------------
// Segmented combine + SGD

template <int DT>
__device__ __forceinline__ void load8_any(const void* row, int64_t x, float (&v)[8]) {
  constexpr int ESZ = (DT == kF32) ? 4 : 2;
  if ((reinterpret_cast<uintptr_t>(static_cast<const char*>(row) + x * ESZ) & 15) == 0) {
    load_vec<DT, 8>(row, x, v);
  } else {
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = load_one<DT>(row, x + c);
  }
}

// k_combine's arithmetic (gar_combine.hip gather_weighted), loads of any alignment
template <int DT>
__device__ __forceinline__ void gather8(const RowTable& rows, const int* sel, const float* wsel, int cnt, int64_t x,
                                        float (&acc)[8]) {
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
  int j = 0;
  for (; j + 4 <= cnt; j += 4) {
    float v0[8], v1[8], v2[8], v3[8];
    load8_any<DT>(rows.p[sel[j]], x, v0);
    load8_any<DT>(rows.p[sel[j + 1]], x, v1);
    load8_any<DT>(rows.p[sel[j + 2]], x, v2);
    load8_any<DT>(rows.p[sel[j + 3]], x, v3);
    const float w0 = wsel[j], w1 = wsel[j + 1], w2 = wsel[j + 2], w3 = wsel[j + 3];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] += w0 * v0[c] + w1 * v1[c] + w2 * v2[c] + w3 * v3[c];
  }
  for (; j < cnt; ++j) {
    float v[8];
    load8_any<DT>(rows.p[sel[j]], x, v);
    const float w = wsel[j];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] += w * v[c];
  }
}

// one element with gather8's arithmetic (4 rows per step): a group's elements that a job boundary
// splits (a shard edge inside an 8-wide group) get the bits the 8-wide path would give them
template <int DT>
__device__ __forceinline__ float gather1_grouped(const RowTable& rows, const int* sel, const float* wsel, int cnt,
                                                 int64_t x) {
  float acc = 0.f;
  int j = 0;
  for (; j + 4 <= cnt; j += 4) {
    const float v0 = load_one<DT>(rows.p[sel[j]], x), v1 = load_one<DT>(rows.p[sel[j + 1]], x);
    const float v2 = load_one<DT>(rows.p[sel[j + 2]], x), v3 = load_one<DT>(rows.p[sel[j + 3]], x);
    const float w0 = wsel[j], w1 = wsel[j + 1], w2 = wsel[j + 2], w3 = wsel[j + 3];
    acc += w0 * v0 + w1 * v1 + w2 * v2 + w3 * v3;
  }
  for (; j < cnt; ++j) acc += wsel[j] * load_one<DT>(rows.p[sel[j]], x);
  return acc;
}

__device__ __forceinline__ void sgd_one(float g, float& p, float& buf, const SgdArgs& a) {
  if (a.weight_decay != 0.f) g += a.weight_decay * p;
  if (a.momentum != 0.f) {
    buf = a.first_step ? g : a.momentum * buf + (1.f - a.dampening) * g;
    g = a.nesterov ? g + a.momentum * buf : buf;
  }
  p -= a.lr * g;
}

// jobs: (start, end, segment) in LOCAL coordinates of the rows / param / mom / shadow; base: the
// global (flat-vector) coordinate of local 0 (a sharded bucket's owned range), seg_off global.
template <int DT>
__global__ __launch_bounds__(256) void k_lw_combine_sgd(RowTable rows, int n, const int64_t* __restrict__ jobs,
                                                        const float* __restrict__ weights, float* __restrict__ param,
                                                        float* __restrict__ mom, void* __restrict__ shadow,
                                                        int shadow_dt, SgdArgs args, const int64_t* __restrict__ seg_off,
                                                        int64_t base) {
  __shared__ int sel[kMaxRows];
  __shared__ float wsel[kMaxRows];
  __shared__ int cnt_s;
  const int64_t a = jobs[3 * blockIdx.x], b = jobs[3 * blockIdx.x + 1];
  const int s = static_cast<int>(jobs[3 * blockIdx.x + 2]);
  const int64_t s0 = seg_off[s] - base, s1 = seg_off[s + 1] - base;   // local segment bounds
  if (threadIdx.x == 0) {
    int c = 0;
    for (int j = 0; j < n; ++j) {
      const float w = weights[static_cast<int64_t>(s) * n + j];
      if (w != 0.f) { sel[c] = j; wsel[c] = w; ++c; }
    }
    cnt_s = c;
  }
  __syncthreads();
  const int cnt = cnt_s;
  auto update = [&](int64_t x, float g) {
    float p = param[x];
    float bf = (args.momentum != 0.f && !args.first_step) ? mom[x] : 0.f;
    sgd_one(g, p, bf, args);
    param[x] = p;
    if (shadow) store_one(shadow, shadow_dt, x, p);
    if (args.momentum != 0.f) mom[x] = bf;
  };
  // 8-wide groups counted from the SEGMENT start (as a per-segment combine sees them); the
  // segment's last (s1 - s0) % 8 elements are its scalar tail
  const int64_t sv = s0 + ((s1 - s0) & ~static_cast<int64_t>(7));
  const int64_t va = s0 + ((a - s0 + 7) & ~static_cast<int64_t>(7));        // first whole group in [a, b)
  const int64_t ve_max = b < sv ? b : sv;
  const int64_t ve = va + ((ve_max > va ? ve_max - va : 0) & ~static_cast<int64_t>(7));   // end of whole groups
  auto tail_one = [&](int64_t x) {
    float g = 0.f;
    for (int j = 0; j < cnt; ++j) g += wsel[j] * load_one<DT>(rows.p[sel[j]], x);
    return g;
  };
  for (int64_t x = a + threadIdx.x; x < (va < b ? va : b); x += 256)        // a split group's head
    update(x, x < sv ? gather1_grouped<DT>(rows, sel, wsel, cnt, x) : tail_one(x));
  for (int64_t x = va + static_cast<int64_t>(threadIdx.x) * 8; x < ve; x += 256 * 8) {
    float acc[8];
    gather8<DT>(rows, sel, wsel, cnt, x, acc);
#pragma unroll
    for (int c = 0; c < 8; ++c) update(x + c, acc[c]);
  }
  for (int64_t x = (ve > a ? ve : a) + threadIdx.x; x < b; x += 256) {
    if (x < va) continue;
    // a split group's rest, or the segment tail
    update(x, x < sv ? gather1_grouped<DT>(rows, sel, wsel, cnt, x) : tail_one(x));
  }
}

// Layer-wise Bulyan's tail: job j's coordinates get the flat tail (coord_body<kBulyanTail>: the
// t selection means with the segment's W [t][n], read by uniform scalar loads, then the averaged
// median of the t means, beta = t - 2f) -- the per-coordinate arithmetic of k_coordwise. Grid
// (jobs, kLwTailSub): the kLwTailSub workgroups of a job interleave its coordinates.
constexpr int kLwTailSub = 8;

template <int DT, int NP>
__global__ __launch_bounds__(256) void k_lw_bulyan_tail(RowTable rows, int n, const int64_t* __restrict__ jobs,
                                                        const float* __restrict__ W, int t, int beta,
                                                        float* __restrict__ out) {
  const int64_t a = jobs[3 * blockIdx.x], b = jobs[3 * blockIdx.x + 1];
  const float* Ws = W + jobs[3 * blockIdx.x + 2] * static_cast<int64_t>(t) * n;
  for (int64_t x = a + blockIdx.y * 256 + threadIdx.x; x < b; x += 256 * kLwTailSub) {
    float res[1];
    coord::coord_body<DT, NP, 1, kBulyanTail>(coord::DirectLoader<DT, 1>{rows, x, false}, n, 0, beta, Ws, t, 0, 0,
                                              x, res);
    out[x] = res[0];
  }
}

// The same tail on MFMA (coord::k_bulyan_tail_mfma's scheme, per job): a workgroup builds its job's
// segment set tables, then each wave takes whole 64-coordinate groups of the job ([64 q, 64 q + 64)
// inside [a, b): v_mfma_f32_32x32x16 set sums, register-sorted window mean); groups with a
// non-finite sum and the job's partial head / tail groups (a group that a segment boundary cuts)
// take the exact per-set sums. Job boundaries are segment boundaries or multiples of 64 (the
// engines split jobs at global multiples of LW_JOB, shards are whole 64-blocks), so which
// coordinates take the MFMA sums does not depend on how the vector is sharded.
template <int DT, int NP, int KS>
__global__ __launch_bounds__(256, 2) void k_lw_bulyan_tail_mfma(RowTable rows, int n, const int64_t* __restrict__ jobs,
                                                                const float* __restrict__ Wall, int t, int beta,
                                                                float* __restrict__ out) {
  using namespace coord;
  constexpr int MB = NP > 32 ? 2 : 1;
  constexpr int KR = 16 * KS;
  constexpr int KRP = KR + 8;
  constexpr int P0 = wm_p0(NP);
  constexpr int WAVE_LDS = KR * kMfmaTailPitch > (NP - P0) * 256 ? KR * kMfmaTailPitch : (NP - P0) * 256;
  __shared__ __align__(16) unsigned char tiles[4][WAVE_LDS];
  __shared__ __align__(16) uint16_t sA[32 * MB * KRP];
  __shared__ const void* sptr[KR];
  __shared__ uint64_t smask[NP];
  __shared__ __align__(16) float sscale[NP];
  __shared__ __align__(16) float spad[NP];
  __shared__ int64_t sbad[4][kTailBadSlots];
  __shared__ int sbadn[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t a = jobs[3 * blockIdx.x], b = jobs[3 * blockIdx.x + 1];
  const float* W = Wall + jobs[3 * blockIdx.x + 2] * static_cast<int64_t>(t) * n;
  // a workgroup with no whole group of the job and no partial range to do leaves before the tables
  if ((a + 63) / 64 + static_cast<int64_t>(blockIdx.y) * 4 >= b / 64 && (blockIdx.y != 0 || (a % 64 == 0 && b % 64 == 0)))
    return;
  {
    const uint16_t one = DT == kBF16 ? 0x3F80 : 0x3C00;
    for (int k = wave; k < 32 * MB; k += 4) {
      const float w = (k < t && lane < n) ? W[k * n + lane] : 0.f;
      const uint64_t m = __builtin_amdgcn_ballot_w64(w != 0.f);
      if (lane < KR) sA[k * KRP + lane] = w != 0.f ? one : 0;
      if (k < NP) {
        const int first = m ? __builtin_ctzll(m) : 0;
        const float sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), first));
        if (lane == 0) {
          smask[k] = m;
          sscale[k] = m ? sc : 0.f;
          spad[k] = k < t ? 0.f : kInf;
        }
      }
    }
  }
  for (int j = threadIdx.x; j < KR; j += blockDim.x) sptr[j] = rows.p[j < n ? j : 0];
  if (threadIdx.x < 4) sbadn[threadIdx.x] = 0;
  __syncthreads();
  unsigned char* tile = tiles[wave];
  float* ks = reinterpret_cast<float*>(tile);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int tr_off = (8 * (g >> 1) + q) * kMfmaTailPitch + (16 * (g & 1) + 4 * p) * 2;
  const int a_off = (lane & 31) * KRP + 8 * (lane >> 5);
  const float inv_beta = 1.f / static_cast<float>(beta);
  bool overflow = false;
  const int64_t q0 = (a + 63) / 64, q1 = b / 64;      // whole groups [q0, q1)
  const int64_t gstep = static_cast<int64_t>(gridDim.y) * 4;
  const int64_t gfirst = q0 + static_cast<int64_t>(blockIdx.y) * 4 + wave;
  TileRegs<KR> pre;
  if (gfirst < q1) tile_load<KR>(pre, sptr, gfirst * 64, lane, n);
  for (int64_t gi = gfirst; gi < q1; gi += gstep) {
    asm volatile("" ::: "memory");
    const int64_t x0 = gi * 64;
    const int nn = opaque_uniform(n), tt = opaque_uniform(t), bb = opaque_uniform(beta);
    tile_store<KR>(tile, pre, nn, lane);
    if (gi + gstep < q1) tile_load<KR>(pre, sptr, (gi + gstep) * 64, lane, nn);
    f32x16_t acc[MB][2];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[mb][nb][i] = 0.f;
#pragma unroll
    for (int ks_ = 0; ks_ < KS; ++ks_) {
      s16x8_t afrag[MB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        afrag[mb] = *reinterpret_cast<const s16x8_t*>(&sA[a_off + 32 * mb * KRP + 16 * ks_]);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
        const unsigned char* base = tile + ks_ * 16 * kMfmaTailPitch + nb * 64 + tr_off;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 4 * kMfmaTailPitch));
        const s16x8_t bfrag = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][nb] = mfma32x32x16<DT>(afrag[mb], bfrag, acc[mb][nb]);
      }
    }
    float v[NP];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k0 = 32 * mb + (i & 3) + 8 * (i >> 2);
        if (k0 < NP) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[mb][0][i]),
                                                           __float_as_uint(acc[mb][1][i]), false, false);
          v[k0] = __uint_as_float(sw[0]);
          v[k0 + 4] = __uint_as_float(sw[1]);
        }
      }
    float chk = 0.f;
#pragma unroll
    for (int k = 0; k < NP; k += 4) {
      if (k % 8 == 0) asm volatile("" ::: "memory");
      const f32x4_t sc = *reinterpret_cast<const f32x4_t*>(&sscale[k]);
      const f32x4_t pd = *reinterpret_cast<const f32x4_t*>(&spad[k]);
      const float scv[4] = {sc[0], sc[1], sc[2], sc[3]}, pdv[4] = {pd[0], pd[1], pd[2], pd[3]};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        chk = __builtin_fmaf(v[k + c], 0.f, chk);
        v[k + c] = __builtin_fmaf(v[k + c], scv[c], pdv[c]);
      }
    }
    if (__builtin_amdgcn_ballot_w64(chk != 0.f)) {
      const int slot = sbadn[wave];
      if (slot < kTailBadSlots) {
        if (lane == 0) sbad[wave][slot] = gi;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) sbadn[wave] = slot + 1;
      } else {
        overflow = true;
      }
    }
    out[x0 + lane] = window_mean<NP, false>(v, tt, bb, inv_beta, ks, lane);
  }
  // exact pass: listed groups (every group of this wave after a list overflow), then the job's
  // partial groups: [a, 64 q0) and [64 q1, b), or [a, b) inside one group (block y 0, waves 0 / 1)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int nbad = overflow ? 0 : sbadn[wave];
  int64_t ps = 0, pe = 0;   // this wave's partial range
  if (blockIdx.y == 0) {
    if (q0 > q1) {
      if (wave == 0) { ps = a; pe = b; }
    } else if (wave == 0 && a < q0 * 64) {
      ps = a; pe = q0 * 64;
    } else if (wave == 1 && q1 * 64 < b) {
      ps = q1 * 64; pe = b;
    }
  }
  bool partial_pending = pe > ps;
  int64_t gi = overflow ? gfirst : 0;
  for (int bi = 0;; ++bi) {
    int64_t xs;
    int width = 64;
    if (overflow ? gi < q1 : bi < nbad) {
      xs = (overflow ? gi : sbad[wave][bi]) * 64;
      if (overflow) gi += gstep;
    } else if (partial_pending) {
      xs = ps;
      width = static_cast<int>(pe - ps);
      partial_pending = false;
    } else {
      break;
    }
    const int nn = opaque_uniform(n), tt = opaque_uniform(t), bb = opaque_uniform(beta);
    if (width == 64 && (xs & 63) == 0) {
      stage_tile<DT, KR>(tile, sptr, nn, xs, lane);
    } else {   // per-column loads; columns >= width repeat the first
      const int64_t xl = xs + (lane < width ? lane : 0);
      for (int j = 0; j < KR; ++j)
        reinterpret_cast<uint16_t*>(tile)[j * (kMfmaTailPitch / 2) + lane] =
            j < nn ? static_cast<const uint16_t*>(sptr[j])[xl] : 0;
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    const uint16_t* col = reinterpret_cast<const uint16_t*>(tile) + lane;
    float v[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      v[k] = kInf;
      if (k < tt) {
        uint64_t m = uniform64(lds_volatile(smask[k]));
        float sm = 0.f;
#pragma clang loop unroll(disable)
        while (m) {
          sm += cvt16<DT>(col[__builtin_ctzll(m) * (kMfmaTailPitch / 2)]);
          m &= m - 1;
        }
        v[k] = sanitize_inf(sm * lds_volatile(sscale[k]));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float r = window_mean<NP, true>(v, tt, bb, inv_beta, ks, lane);
    if (lane < width) out[xs + lane] = r;
  }
}

// the MFMA tail's limits (coord::launch_bulyan_tail_mfma): bf16 / fp16, n <= 64, t - beta <= 16,
// window_mean's register positions
inline bool lw_tail_mfma_ok(int dt, int n, int t, int beta) {
  if (dt == kF32 || n > 64 || t > 64 || t < 1 || beta < 1 || t - beta > coord::kTailMaxExcluded) return false;
  const int np = coord::np_for(t);
  return t / 2 >= coord::wm_p0(np) && beta >= coord::wm_p0(np);
}

constexpr int kLwTailMfmaSub = 16;   // workgroups per job (a 32768-coordinate job = 512 groups)

template <int DT, int NP>
void launch_lw_tail_mfma(int ks, const RowTable& rows, int n, const int64_t* jobs, int njobs, const float* W, int t,
                         int beta, float* out, hipStream_t s) {
  const dim3 grid(njobs, kLwTailMfmaSub);
#define GARFIELD_LW_TAIL(KS) \
  hipLaunchKernelGGL((k_lw_bulyan_tail_mfma<DT, NP, KS>), grid, dim3(256), 0, s, rows, n, jobs, W, t, beta, out)
  switch (ks) {
    case 1: GARFIELD_LW_TAIL(1); break;
    case 2: GARFIELD_LW_TAIL(2); break;
    case 3: GARFIELD_LW_TAIL(3); break;
    default: GARFIELD_LW_TAIL(4); break;
  }
#undef GARFIELD_LW_TAIL
}

template <int DT> struct LwBulyan {
  static void run(const RowTable& rows, int n, const int64_t* jobs, int njobs, const float* W, int t, int beta,
                  float* out, hipStream_t s) {
    if constexpr (DT != kF32) {
      if (lw_tail_mfma_ok(DT, n, t, beta) && lw_tail_mfma_enabled()) {
        const int ks = (n + 15) / 16;
        switch (coord::np_for(t)) {
          case 8: launch_lw_tail_mfma<DT, 8>(ks, rows, n, jobs, njobs, W, t, beta, out, s); break;
          case 16: launch_lw_tail_mfma<DT, 16>(ks, rows, n, jobs, njobs, W, t, beta, out, s); break;
          case 32: launch_lw_tail_mfma<DT, 32>(ks, rows, n, jobs, njobs, W, t, beta, out, s); break;
          default: launch_lw_tail_mfma<DT, 64>(ks, rows, n, jobs, njobs, W, t, beta, out, s); break;
        }
        return;
      }
    }
    const dim3 grid(njobs, kLwTailSub);
    switch (coord::np_for(t)) {
      case 8: hipLaunchKernelGGL((k_lw_bulyan_tail<DT, 8>), grid, dim3(256), 0, s, rows, n, jobs, W, t, beta, out); break;
      case 16: hipLaunchKernelGGL((k_lw_bulyan_tail<DT, 16>), grid, dim3(256), 0, s, rows, n, jobs, W, t, beta, out); break;
      case 32: hipLaunchKernelGGL((k_lw_bulyan_tail<DT, 32>), grid, dim3(256), 0, s, rows, n, jobs, W, t, beta, out); break;
      default: hipLaunchKernelGGL((k_lw_bulyan_tail<DT, 64>), grid, dim3(256), 0, s, rows, n, jobs, W, t, beta, out); break;
    }
  }
};

template <int DT, int NB>
void launch_lw_gram(const RowTable& rows, int n, const int64_t* jobs, int njobs, float* slabs, hipStream_t s) {
  hipLaunchKernelGGL((k_lw_gram_partial<DT, NB>), dim3(njobs), dim3(256), 0, s, rows, n, jobs, slabs);
}
template <int DT> struct LwGram {
  static void run(const RowTable& rows, int n, const int64_t* jobs, int njobs, float* slabs, hipStream_t s) {
    switch (gram_nb(n)) {
      case 1: launch_lw_gram<DT, 1>(rows, n, jobs, njobs, slabs, s); break;
      case 2: launch_lw_gram<DT, 2>(rows, n, jobs, njobs, slabs, s); break;
      case 4: launch_lw_gram<DT, 4>(rows, n, jobs, njobs, slabs, s); break;
      default: launch_lw_gram<DT, 8>(rows, n, jobs, njobs, slabs, s); break;
    }
  }
};
template <int DT> struct LwCombine {
  static void run(const RowTable& rows, int n, const int64_t* jobs, int njobs, const float* w, float* param,
                  float* mom, void* shadow, int shadow_dt, SgdArgs a, const int64_t* seg_off, int64_t base,
                  hipStream_t s) {
    hipLaunchKernelGGL(k_lw_combine_sgd<DT>, dim3(njobs), dim3(256), 0, s, rows, n, jobs, w, param, mom, shadow,
                       shadow_dt, a, seg_off, base);
  }
};

}  // namespace

void lw_gram(const RowTable& rows, int n, int dt, const int64_t* jobs, int njobs, const int* seg_lo, int L,
             float* slabs, float* gram, hipStream_t stream) {
  if (njobs <= 0 || L <= 0) return;
  by_dtype<LwGram>(dt, rows, n, jobs, njobs, slabs, stream);
  const int nb = gram_nb(n);
  const int E = nb * (nb + 1) / 2 * 256;
  hipLaunchKernelGGL(k_lw_gram_reduce, dim3((E + 255) / 256, L), dim3(256), 0, stream, slabs, seg_lo, nb, gram);
}

void lw_bulyan_tail(const RowTable& rows, int n, int dt, const int64_t* jobs, int njobs, const float* W, int t,
                    int beta, float* out, hipStream_t stream) {
  if (njobs <= 0 || t <= 0) return;
  by_dtype<LwBulyan>(dt, rows, n, jobs, njobs, W, t, beta, out, stream);
}

void lw_combine_sgd(const RowTable& rows, int n, int dt, const int64_t* jobs, int njobs, const float* weights,
                    float* param, float* momentum_buf, void* shadow, int shadow_dt, SgdArgs args,
                    const int64_t* seg_off, int64_t base, hipStream_t stream) {
  if (njobs <= 0) return;
  by_dtype<LwCombine>(dt, rows, n, jobs, njobs, weights, param, momentum_buf, shadow, shadow_dt, args, seg_off, base,
                      stream);
}

}  // namespace gpu
}  // namespace garfield
