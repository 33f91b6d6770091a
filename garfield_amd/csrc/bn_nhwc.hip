// Worker-grouped BatchNorm (+ residual add) (+ ReLU) for NHWC activations, gfx950.
//
// The engine runs its k logical workers as ONE batched forward/backward
// (garfield_amd/parallel/grouped.py): the activations of all workers are one
// [R, C] NHWC matrix with R = k * Rg rows (Rg = B*H*W rows per worker), and
// BatchNorm must still use per-WORKER batch statistics, exactly as if each
// worker ran alone. The reference runs one worker per process
// (pytorch_impl/libs/garfieldpp/worker.py:77-96) and its nets use
// nn.BatchNorm2d + F.relu (+ residual add): three to four kernels per layer per
// worker (MIOpenBatchNormFwdTrainSpatial, relu, add; and their backward).
// Here one layer costs three launches FOR ALL k WORKERS, forward and backward:
//
//   forward : partial (sum, sum of squares) per (worker, channel, row chunk)
//             -> finalize (mean, 1/std, scale/shift per worker and channel)
//             -> apply  y = relu(x*scale + shift [+ residual])      (bf16x8 I/O);
//                its first workgroup also replays the k sequential running-stat
//                updates of k independent workers
//   backward: partial (Σdz, Σdz·(x-μ)) with dz = dy·[y > 0] (the ReLU test reads a
//             one-bit-per-element mask written by the forward apply, not y)
//             -> finalize (dγ, dβ per worker, written STRAIGHT into each
//                worker's row of the gradient exchange buffer; apply coefficients)
//             -> apply  dx = γ/σ·(dz - dβ/M - x̂·dγ/M)   [+ dres = dz]
//
// Launch boundaries order the stages (no inter-workgroup hand-off inside a
// launch); every reduction runs in a fixed order, so results are deterministic.
#include <cstdlib>
#include <type_traits>

#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kThreads = 256;

struct Geo {
  int64_t rg;      // rows per group (worker)
  int groups;
  int C;
  int cb;          // channels per workgroup in the partial kernels (multiple of 8)
  int tch;         // threads across channels = cb / 8
  int rp;          // row lanes = 256 / tch
  int chunks;      // row chunks per group
  int64_t rows_per_chunk;
};

Geo geometry(int64_t rg, int groups, int C) {
  Geo g{};
  g.rg = rg;
  g.groups = groups;
  g.C = C;
  g.cb = C < 512 ? C : 512;
  g.tch = g.cb / 8;
  g.rp = kThreads / g.tch;
  if (g.rp < 1) g.rp = 1;
  // enough row chunks to give the partial kernel ~1024 workgroups, each at least 4 row passes
  const int ncb = (C + g.cb - 1) / g.cb;
  const int64_t wg = static_cast<int64_t>(groups) * ncb;
  constexpr int64_t target = 1024;   // total partial-pass workgroups
  int64_t want = (target + wg - 1) / wg;
  int64_t maxc = (rg + 4 * g.rp - 1) / (4 * g.rp);
  int64_t c = want < maxc ? want : maxc;
  if (c < 1) c = 1;
  if (c > kBnMaxChunks) c = kBnMaxChunks;
  g.rows_per_chunk = (rg + c - 1) / c;
  g.chunks = static_cast<int>((rg + g.rows_per_chunk - 1) / g.rows_per_chunk);
  return g;
}

template <int DT>
__device__ __forceinline__ void load8(const void* p, int64_t off, float (&v)[8]) {
  load_vec<DT, 8>(p, off, v);
}

// bit of the ReLU mask: the STORED value is > 0 (what a y > 0 test reads back)
template <int DT>
__device__ __forceinline__ bool stored_pos(float o) {
  if constexpr (DT == kF32) return o > 0.f;
  else return f_to_bf16(o) != 0;
}

__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// dz = dy masked by the forward ReLU. RM: 0 none, 1 y > 0, 2 the bit mask, 3 the stored value of
// bf16(x * scale + shift) > 0 (a BatchNorm whose normalised output was never written)
template <int RM, int DT>
__device__ __forceinline__ void relu_mask8(float (&d)[8], const float (&a)[8], const void* y, const uint8_t* mask,
                                           int64_t off, const float (&sc)[8], const float (&sf)[8]) {
  if constexpr (RM == 1) {
    float yy[8];
    load8<DT>(y, off, yy);
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = yy[i] > 0.f ? d[i] : 0.f;
  } else if constexpr (RM == 2) {
    const uint32_t mb = mask[off >> 3];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = (mb >> i) & 1u ? d[i] : 0.f;
  } else if constexpr (RM == 3) {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = stored_pos<DT>(fmaxf(fmaf(a[i], sc[i], sf[i]), 0.f)) ? d[i] : 0.f;
  }
}

// 8 channels of one row as stored: packed bf16 (one uint4) or fp32 (two float4)
struct F8 {
  float4 a, b;
};
template <int DT>
using Raw8 = typename std::conditional<DT == kF32, F8, uint4>::type;

template <int DT>
__device__ __forceinline__ Raw8<DT> ld_raw8(const void* p, int64_t off) {
  if constexpr (DT == kF32) {
    const float* f = static_cast<const float*>(p) + off;
    return F8{*reinterpret_cast<const float4*>(f), *reinterpret_cast<const float4*>(f + 4)};
  } else {
    return *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + off);
  }
}

template <int DT>
__device__ __forceinline__ void st_raw8(void* p, int64_t off, const Raw8<DT>& r) {
  if constexpr (DT == kF32) {
    float* f = static_cast<float*>(p) + off;
    *reinterpret_cast<float4*>(f) = r.a;
    *reinterpret_cast<float4*>(f + 4) = r.b;
  } else {
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + off) = r;
  }
}

__device__ __forceinline__ void unpack8(const uint4 u, float (&v)[8]) {
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ void unpack8(const F8& u, float (&v)[8]) {
  v[0] = u.a.x; v[1] = u.a.y; v[2] = u.a.z; v[3] = u.a.w;
  v[4] = u.b.x; v[5] = u.b.y; v[6] = u.b.z; v[7] = u.b.w;
}

// Partial per-(group, channel) sums over one row chunk.
//   forward : s = Σ (x - shift), q = Σ (x - shift)^2  with shift = x[first row of the group]
//             (shifted sums: no catastrophic cancellation when |mean| >> std)
//   backward: s = Σ dz, q = Σ dz (x - mean)
// RM: ReLU mask source of the backward: 0 none, 1 the bf16 output y (> 0), 2 the
// forward's bit mask (one byte per 8 channels: 1/16 of y's bytes).
template <bool BWD, int RM, int DT>
__global__ __launch_bounds__(kThreads) void k_partial(const void* __restrict__ x, const void* __restrict__ dy,
                                                     const void* __restrict__ y, const uint8_t* __restrict__ mask,
                                                     const float* __restrict__ mean, Geo geo,
                                                     float* __restrict__ part, const float* __restrict__ rsc,
                                                     const float* __restrict__ rsh) {
  __shared__ __attribute__((aligned(16))) float red[2][kThreads * 8];
  const int C = geo.C;
  const int tc = threadIdx.x % geo.tch;
  const int tr = threadIdx.x / geo.tch;
  const int chunk = blockIdx.x;
  const int cbk = blockIdx.y;
  const int g = blockIdx.z;
  const int c0 = cbk * geo.cb + tc * 8;
  const bool lane_ok = tr < geo.rp;
  const bool active = lane_ok && (c0 < C);
  const int64_t base = static_cast<int64_t>(g) * geo.rg;
  const int64_t r0 = static_cast<int64_t>(chunk) * geo.rows_per_chunk;
  int64_t r1 = r0 + geo.rows_per_chunk;
  if (r1 > geo.rg) r1 = geo.rg;
  float s[8], q[8], sh[8], rs[8] = {}, rf[8] = {};
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; q[i] = 0.f; sh[i] = 0.f; }
  if (active) {
    if constexpr (BWD) load8f(mean + static_cast<int64_t>(g) * C + c0, sh);
    else load8<DT>(x, base * C + c0, sh);
    if constexpr (RM == 3) {
      load8f(rsc + static_cast<int64_t>(g) * C + c0, rs);
      load8f(rsh + static_cast<int64_t>(g) * C + c0, rf);
    }
    int64_t r = r0 + tr;
    // two rows in flight per lane, unpacked as loaded (hipcc keeps this loop's loads in one batch but
    // serialises a four-row raw batch, checked in the ISA). One loop for every form: the sums of a
    // shortcut BatchNorm fed dy + ReLU bits (RM 2) and of one fed the written dres (RM 0) agree bit for bit
    // (the ResLink path, tests/test_grouped_gpu.py::test_lazy_residual_*)
    for (; r + geo.rp < r1; r += 2 * geo.rp) {
      const int64_t o0 = (base + r) * C + c0, o1 = o0 + static_cast<int64_t>(geo.rp) * C;
      float a0[8], a1[8];
      load8<DT>(x, o0, a0);
      load8<DT>(x, o1, a1);
      if constexpr (BWD) {
        float d0[8], d1[8];
        load8<DT>(dy, o0, d0);
        load8<DT>(dy, o1, d1);
        relu_mask8<RM, DT>(d0, a0, y, mask, o0, rs, rf);
        relu_mask8<RM, DT>(d1, a1, y, mask, o1, rs, rf);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s[i] += d0[i] + d1[i];
          q[i] += d0[i] * (a0[i] - sh[i]) + d1[i] * (a1[i] - sh[i]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float e0 = a0[i] - sh[i], e1 = a1[i] - sh[i];
          s[i] += e0 + e1;
          q[i] += e0 * e0 + e1 * e1;
        }
      }
    }
    for (; r < r1; r += geo.rp) {
      const int64_t o0 = (base + r) * C + c0;
      float a0[8];
      load8<DT>(x, o0, a0);
      if constexpr (BWD) {
        float d0[8];
        load8<DT>(dy, o0, d0);
        relu_mask8<RM, DT>(d0, a0, y, mask, o0, rs, rf);
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[i] += d0[i]; q[i] += d0[i] * (a0[i] - sh[i]); }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float e = a0[i] - sh[i]; s[i] += e; q[i] += e * e; }
      }
    }
  }
  // reduce the row lanes through LDS: red[.][lane_row * cb + channel]
  if (lane_ok) {
    float* p0 = &red[0][tr * geo.cb + tc * 8];
    float* p1 = &red[1][tr * geo.cb + tc * 8];
    *reinterpret_cast<float4*>(p0) = make_float4(s[0], s[1], s[2], s[3]);
    *reinterpret_cast<float4*>(p0 + 4) = make_float4(s[4], s[5], s[6], s[7]);
    *reinterpret_cast<float4*>(p1) = make_float4(q[0], q[1], q[2], q[3]);
    *reinterpret_cast<float4*>(p1 + 4) = make_float4(q[4], q[5], q[6], q[7]);
  }
  __syncthreads();
  // row lanes summed by all threads: nparts = 256 / cb threads per channel (cb < 256), each over
  // every nparts-th lane row, then the parts (in the free tail of red) by one thread per channel
  const int nparts = geo.cb < kThreads ? kThreads / geo.cb : 1;
  if (nparts > 1) {
    const int c = threadIdx.x % geo.cb, pt = threadIdx.x / geo.cb;
    float a = 0.f, b = 0.f;
    for (int t = pt; t < geo.rp; t += nparts) { a += red[0][t * geo.cb + c]; b += red[1][t * geo.cb + c]; }
    __syncthreads();
    if (pt < nparts) {   // (256 % cb threads left over when cb does not divide 256)
      red[0][pt * geo.cb + c] = a;
      red[1][pt * geo.cb + c] = b;
    }
    __syncthreads();
  }
  const int rows = nparts > 1 ? nparts : geo.rp;
  for (int c = threadIdx.x; c < geo.cb; c += kThreads) {
    const int cc = cbk * geo.cb + c;
    if (cc >= C) continue;
    float a = 0.f, b = 0.f;
    for (int t = 0; t < rows; ++t) { a += red[0][t * geo.cb + c]; b += red[1][t * geo.cb + c]; }
    const int64_t o = (static_cast<int64_t>(g) * geo.chunks + chunk) * 2 * C;
    part[o + cc] = a;
    part[o + C + cc] = b;
  }
}

// Finalize workgroups: FC channels x 256 / FC chunk lanes for ONE group (blockIdx.y),
// every chunk load issued before it is consumed (the chunk sums are a
// latency-bound gather otherwise), lanes reduced through LDS in a fixed order.
// Finalize: 16 channels x 16 chunk lanes per workgroup: a chunk lane's loads (<= 8 per array for up to
// 128 chunks) are one batch, so the pass costs one memory latency instead of four with 64 x 4
// (bf16 ResNet-50 step -0.02 ms, fp32 -0.05 ms: profiles/r4/bn_fin/)
constexpr int kFin = 16;

template <int FC>
struct Fin {
  static constexpr int Ch = FC, Lanes = kThreads / FC;
};

template <int FC>
__device__ __forceinline__ void chunk_sums(const float* __restrict__ part, const Geo& geo, int g, int c, float* sred,
                                           float* qred, float& S, float& Q) {
  const int tc = threadIdx.x % Fin<FC>::Ch, lane = threadIdx.x / Fin<FC>::Ch;
  const int C = geo.C;
  float s = 0.f, q = 0.f;
  if (c < C) {
    for (int ch0 = lane; ch0 < geo.chunks; ch0 += Fin<FC>::Lanes * 8) {
      float a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int ch = ch0 + Fin<FC>::Lanes * u;
        const int64_t o = (static_cast<int64_t>(g) * geo.chunks + ch) * 2 * C;
        a[u] = ch < geo.chunks ? part[o + c] : 0.f;
        b[u] = ch < geo.chunks ? part[o + C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { s += a[u]; q += b[u]; }
    }
  }
  sred[lane * Fin<FC>::Ch + tc] = s;
  qred[lane * Fin<FC>::Ch + tc] = q;
  __syncthreads();
  S = 0.f;
  Q = 0.f;
#pragma unroll
  for (int l = 0; l < Fin<FC>::Lanes; ++l) { S += sred[l * Fin<FC>::Ch + tc]; Q += qred[l * Fin<FC>::Ch + tc]; }
}

// Forward finalize of one (group, 64-channel block): mean, 1/std, scale, shift.
template <int DT, int FC>
__global__ __launch_bounds__(kThreads) void k_fwd_finalize(const float* __restrict__ part, const void* __restrict__ x,
                                                          Geo geo, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          float* __restrict__ mean, float* __restrict__ istd,
                                                          float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float sred[kThreads], qred[kThreads];
  const int C = geo.C;
  const int g = blockIdx.y;
  const int c = blockIdx.x * FC + threadIdx.x % FC;
  float S, Q;
  chunk_sums<FC>(part, geo, g, c, sred, qred, S, Q);
  if (threadIdx.x >= FC || c >= C) return;
  const float M = static_cast<float>(geo.rg);
  const float sh = load_one<DT>(x, static_cast<int64_t>(g) * geo.rg * C + c);
  const float m1 = S / M;
  float var = Q / M - m1 * m1;
  var = var > 0.f ? var : 0.f;
  const float mu = sh + m1;
  const float is = rsqrtf(var + eps);
  const int64_t gc = static_cast<int64_t>(g) * C + c;
  mean[gc] = mu;
  istd[gc] = is;
  const float sc = (gamma ? gamma[c] : 1.f) * is;
  scale[gc] = sc;
  shift[gc] = (beta ? beta[c] : 0.f) - mu * sc;
}

// Running statistics: the k sequential updates of k independent workers, in
// worker order (run by the first workgroup of the apply pass).
__device__ __forceinline__ void running_update(const float* __restrict__ mean, const float* __restrict__ istd,
                                               int groups, int C, int64_t rg, float eps, float momentum,
                                               float* __restrict__ run_mean, float* __restrict__ run_var) {
  const float M = static_cast<float>(rg);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float rm = run_mean[c], rv = run_var[c];
    for (int g = 0; g < groups; ++g) {
      const float is = istd[static_cast<int64_t>(g) * C + c];
      float var = 1.f / (is * is) - eps;
      var = var > 0.f ? var : 0.f;
      const float unb = rg > 1 ? var * M / (M - 1.f) : var;
      rm = (1.f - momentum) * rm + momentum * mean[static_cast<int64_t>(g) * C + c];
      rv = (1.f - momentum) * rv + momentum * unb;
    }
    run_mean[c] = rm;
    run_var[c] = rv;
  }
}

// Elementwise passes over [R, C]: each workgroup owns kApplyIters x rp rows.
constexpr int kApplyIters = 4;

struct RunStats {
  const float* mean;
  const float* istd;
  float* run_mean;
  float* run_var;
  float eps;
  float momentum;
  int groups;
  // RES: the residual is a PRE-BatchNorm activation whose own per-worker scale / shift ([groups][C])
  // is applied here (a projection shortcut's BatchNorm folded into this apply pass); nullptr: plain add
  const float* res_sc;
  const float* res_sh;
};

template <bool RES, bool RELU, int DT>
__global__ __launch_bounds__(kThreads) void k_fwd_apply(const void* __restrict__ x, const void* __restrict__ res,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       int64_t rg, int64_t R, int C, int tch, int rp,
                                                       void* __restrict__ y, uint8_t* __restrict__ mask,
                                                       RunStats rs) {
  if (blockIdx.x == 0 && rs.run_mean)
    running_update(rs.mean, rs.istd, rs.groups, C, rg, rs.eps, rs.momentum, rs.run_mean, rs.run_var);
  const int tr = threadIdx.x / tch;
  if (tr >= rp) return;
  const int nv = C / 8;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * rp * kApplyIters;
  // one channel group per thread (C <= 8 * tch): its scale / shift are loaded once per worker
  // instead of once per row (they were 4x the row's own bytes in load instructions)
  const bool fixed = nv <= tch;
  int gl = -1;
  float sc[8], sf[8], rsc[8], rsf[8];
  const bool raff = RES && rs.res_sc != nullptr;
  if (fixed && row0 + static_cast<int64_t>(kApplyIters) * rp <= R && rp * kApplyIters <= rg) {
    // every row of the workgroup exists and it spans at most two workers: all of this thread's
    // loads are issued before the first use (kApplyIters rows in flight, not one)
    const int v = threadIdx.x % tch;
    if (v >= nv) return;
    const int c = v * 8;
    const int g0 = static_cast<int>(row0 / rg);
    const int64_t gb = static_cast<int64_t>(g0 + 1) * rg;   // the next worker's first row
    Raw8<DT> xr[kApplyIters], rr[kApplyIters];
#pragma unroll
    for (int it = 0; it < kApplyIters; ++it) {
      const int64_t off = (row0 + static_cast<int64_t>(it) * rp + tr) * C + c;
      xr[it] = ld_raw8<DT>(x, off);
      if constexpr (RES) rr[it] = ld_raw8<DT>(res, off);
    }
#pragma unroll
    for (int it = 0; it < kApplyIters; ++it) {
      const int64_t row = row0 + static_cast<int64_t>(it) * rp + tr;
      const int g = g0 + (row >= gb ? 1 : 0);
      if (g != gl) {
        load8f(scale + static_cast<int64_t>(g) * C + c, sc);
        load8f(shift + static_cast<int64_t>(g) * C + c, sf);
        if (raff) {
          load8f(rs.res_sc + static_cast<int64_t>(g) * C + c, rsc);
          load8f(rs.res_sh + static_cast<int64_t>(g) * C + c, rsf);
        }
        gl = g;
      }
      const int64_t off = row * C + c;
      float a[8], o[8];
      unpack8(xr[it], a);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = a[i] * sc[i] + sf[i];
      if constexpr (RES) {
        float r[8];
        unpack8(rr[it], r);
        if (raff) {
#pragma unroll
          for (int i = 0; i < 8; ++i) r[i] = r[i] * rsc[i] + rsf[i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += r[i];
      }
      if constexpr (RELU) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = o[i] > 0.f ? o[i] : 0.f;
        if (mask) {
          uint32_t bits = 0;
#pragma unroll
          for (int i = 0; i < 8; ++i) bits |= (stored_pos<DT>(o[i]) ? 1u : 0u) << i;
          mask[off >> 3] = static_cast<uint8_t>(bits);
        }
      }
      store_vec<8>(y, DT, off, o);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < kApplyIters; ++it) {
    const int64_t row = row0 + static_cast<int64_t>(it) * rp + tr;
    if (row >= R) break;
    const int g = static_cast<int>(row / rg);
    for (int v = threadIdx.x % tch; v < nv; v += tch) {
      const int c = v * 8;
      const int64_t off = row * C + c;
      float a[8];
      load8<DT>(x, off, a);
      if (!fixed || g != gl) {
        load8f(scale + static_cast<int64_t>(g) * C + c, sc);
        load8f(shift + static_cast<int64_t>(g) * C + c, sf);
        if (raff) {
          load8f(rs.res_sc + static_cast<int64_t>(g) * C + c, rsc);
          load8f(rs.res_sh + static_cast<int64_t>(g) * C + c, rsf);
        }
        gl = g;
      }
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = a[i] * sc[i] + sf[i];
      if constexpr (RES) {
        float r[8];
        load8<DT>(res, off, r);
        if (raff) {
#pragma unroll
          for (int i = 0; i < 8; ++i) r[i] = r[i] * rsc[i] + rsf[i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += r[i];
      }
      if constexpr (RELU) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = o[i] > 0.f ? o[i] : 0.f;
        if (mask) {  // bit i: the STORED value is > 0, exactly what a y > 0 test reads back
          uint32_t bits = 0;
#pragma unroll
          for (int i = 0; i < 8; ++i) bits |= (stored_pos<DT>(o[i]) ? 1u : 0u) << i;
          mask[off >> 3] = static_cast<uint8_t>(bits);
        }
      }
      store_vec<8>(y, DT, off, o);
    }
  }
}

// Backward finalize of one (group, 64-channel block): dγ, dβ -> exchange rows;
// apply coefficients.
template <int FC>
__device__ __forceinline__ void bwd_finalize_body(const float* __restrict__ part, const Geo& geo,
                                                  const float* __restrict__ gamma, const float* __restrict__ istd,
                                                  float* __restrict__ coef, void* grow, int grow_dt,
                                                  int64_t row_stride, int64_t off_gamma, int64_t off_beta,
                                                  float* sred, float* qred) {
  const int C = geo.C;
  const int g = blockIdx.y;
  const int c = blockIdx.x * FC + threadIdx.x % FC;
  float A, B;
  chunk_sums<FC>(part, geo, g, c, sred, qred, A, B);
  if (threadIdx.x >= FC || c >= C) return;
  const float M = static_cast<float>(geo.rg);
  const int64_t gc = static_cast<int64_t>(g) * C + c;
  const float is = istd[gc];
  const float dgamma = B * is;
  const float dbeta = A;
  if (grow) {
    if (off_gamma >= 0) store_one(grow, grow_dt, static_cast<int64_t>(g) * row_stride + off_gamma + c, dgamma);
    if (off_beta >= 0) store_one(grow, grow_dt, static_cast<int64_t>(g) * row_stride + off_beta + c, dbeta);
  }
  const int64_t o3 = static_cast<int64_t>(g) * 3 * C;
  coef[o3 + c] = (gamma ? gamma[c] : 1.f) * is;  // a
  coef[o3 + C + c] = dbeta / M;                 // b
  coef[o3 + 2 * C + c] = dgamma / M * is;       // c  (x̂·dγ/M = (x-μ)·c)
}

template <int FC>
__global__ __launch_bounds__(kThreads) void k_bwd_finalize(const float* __restrict__ part, Geo geo,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ istd,
                                                          float* __restrict__ coef, void* grow, int grow_dt,
                                                          int64_t row_stride, int64_t off_gamma, int64_t off_beta) {
  __shared__ float sred[kThreads], qred[kThreads];
  bwd_finalize_body<FC>(part, geo, gamma, istd, coef, grow, grow_dt, row_stride, off_gamma, off_beta, sred, qred);
}

// the two BatchNorms of a dual backward in one launch (blockIdx.z: 0 = a, 1 = b)
struct FinJob {
  const float* part;
  const float* gamma;
  const float* istd;
  float* coef;
  int64_t off_gamma, off_beta;
};
template <int FC>
__global__ __launch_bounds__(kThreads) void k_bwd_finalize_dual(FinJob ja, FinJob jb, Geo geo, void* grow, int grow_dt,
                                                               int64_t row_stride) {
  __shared__ float sred[kThreads], qred[kThreads];
  const FinJob& j = blockIdx.z ? jb : ja;
  bwd_finalize_body<FC>(j.part, geo, j.gamma, j.istd, j.coef, grow, grow_dt, row_stride, j.off_gamma, j.off_beta,
                        sred, qred);
}

template <int RM, bool RES_OUT, int DT>
__global__ __launch_bounds__(kThreads) void k_bwd_apply(const void* __restrict__ x, const void* __restrict__ dy,
                                                       const void* __restrict__ y, const uint8_t* __restrict__ mask,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ coef, int64_t rg, int64_t R, int C,
                                                       int tch, int rp, void* __restrict__ dx,
                                                       void* __restrict__ dres, const float* __restrict__ rsc,
                                                       const float* __restrict__ rsh) {
  const int tr = threadIdx.x / tch;
  if (tr >= rp) return;
  const int nv = C / 8;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * rp * kApplyIters;
  const bool fixed = nv <= tch;   // one channel group per thread: coefficients once per worker
  int gl = -1;
  float mu[8], ca[8], cb[8], cc[8], rs[8] = {}, rf[8] = {};
  if (fixed && RM != 1 && row0 + static_cast<int64_t>(kApplyIters) * rp <= R && rp * kApplyIters <= rg) {
    // whole rows, at most two workers: every load of the thread issued before the first use
    const int v = threadIdx.x % tch;
    if (v >= nv) return;
    const int c = v * 8;
    const int g0 = static_cast<int>(row0 / rg);
    const int64_t gb = static_cast<int64_t>(g0 + 1) * rg;
    Raw8<DT> xr[kApplyIters], dr[kApplyIters];
    uint32_t mb[kApplyIters];
#pragma unroll
    for (int it = 0; it < kApplyIters; ++it) {
      const int64_t off = (row0 + static_cast<int64_t>(it) * rp + tr) * C + c;
      xr[it] = ld_raw8<DT>(x, off);
      dr[it] = ld_raw8<DT>(dy, off);
      if constexpr (RM == 2) mb[it] = mask[off >> 3];
    }
#pragma unroll
    for (int it = 0; it < kApplyIters; ++it) {
      const int64_t row = row0 + static_cast<int64_t>(it) * rp + tr;
      const int g = g0 + (row >= gb ? 1 : 0);
      if (g != gl) {
        const float* cg = coef + static_cast<int64_t>(g) * 3 * C;
        load8f(mean + static_cast<int64_t>(g) * C + c, mu);
        load8f(cg + c, ca);
        load8f(cg + C + c, cb);
        load8f(cg + 2 * C + c, cc);
        if constexpr (RM == 3) {
          load8f(rsc + static_cast<int64_t>(g) * C + c, rs);
          load8f(rsh + static_cast<int64_t>(g) * C + c, rf);
        }
        gl = g;
      }
      const int64_t off = row * C + c;
      float a[8], d[8];
      unpack8(xr[it], a);
      unpack8(dr[it], d);
      if constexpr (RM == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = (mb[it] >> i) & 1u ? d[i] : 0.f;
      } else if constexpr (RM == 3) {
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = stored_pos<DT>(fmaxf(fmaf(a[i], rs[i], rf[i]), 0.f)) ? d[i] : 0.f;
      }
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = ca[i] * (d[i] - cb[i] - (a[i] - mu[i]) * cc[i]);
      store_vec<8>(dx, DT, off, o);
      if constexpr (RES_OUT) store_vec<8>(dres, DT, off, d);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < kApplyIters; ++it) {
    const int64_t row = row0 + static_cast<int64_t>(it) * rp + tr;
    if (row >= R) break;
    const int g = static_cast<int>(row / rg);
    const float* cg = coef + static_cast<int64_t>(g) * 3 * C;
    for (int v = threadIdx.x % tch; v < nv; v += tch) {
      const int c = v * 8;
      const int64_t off = row * C + c;
      float a[8], d[8];
      load8<DT>(x, off, a);
      load8<DT>(dy, off, d);
      if (!fixed || g != gl) {
        load8f(mean + static_cast<int64_t>(g) * C + c, mu);
        load8f(cg + c, ca);
        load8f(cg + C + c, cb);
        load8f(cg + 2 * C + c, cc);
        if constexpr (RM == 3) {
          load8f(rsc + static_cast<int64_t>(g) * C + c, rs);
          load8f(rsh + static_cast<int64_t>(g) * C + c, rf);
        }
        gl = g;
      }
      relu_mask8<RM, DT>(d, a, y, mask, off, rs, rf);
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = ca[i] * (d[i] - cb[i] - (a[i] - mu[i]) * cc[i]);
      store_vec<8>(dx, DT, off, o);
      if constexpr (RES_OUT) store_vec<8>(dres, DT, off, d);
    }
  }
}

// Dual backward of a projection block's last BatchNorm and its folded shortcut BatchNorm: both see
// the same dz = dy · [ReLU bit] (RM 2, or RM 0 without a ReLU), so one pass reads dy and the mask once
// for the two statistics (Σdz is shared: part_a and part_b get the same s, q_a = Σdz(x_a - μ_a),
// q_b = Σdz(x_b - μ_b)), and one apply pass writes both data gradients.
template <int RM, int DT>
__global__ __launch_bounds__(kThreads) void k_partial_dual(const void* __restrict__ xa, const void* __restrict__ xb,
                                                          const void* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          const float* __restrict__ mean_a,
                                                          const float* __restrict__ mean_b, Geo geo,
                                                          float* __restrict__ part_a, float* __restrict__ part_b) {
  static_assert(RM == 0 || RM == 2, "dz is dy or dy under the bit mask");
  __shared__ __attribute__((aligned(16))) float red[3][kThreads * 8];
  const int C = geo.C;
  const int tc = threadIdx.x % geo.tch;
  const int tr = threadIdx.x / geo.tch;
  const int chunk = blockIdx.x, cbk = blockIdx.y, g = blockIdx.z;
  const int c0 = cbk * geo.cb + tc * 8;
  const bool lane_ok = tr < geo.rp;
  const bool active = lane_ok && (c0 < C);
  const int64_t base = static_cast<int64_t>(g) * geo.rg;
  const int64_t r0 = static_cast<int64_t>(chunk) * geo.rows_per_chunk;
  int64_t r1 = r0 + geo.rows_per_chunk;
  if (r1 > geo.rg) r1 = geo.rg;
  float s[8], qa[8], qb[8], ma[8], mb[8], dum[8] = {};
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; qa[i] = 0.f; qb[i] = 0.f; ma[i] = 0.f; mb[i] = 0.f; }
  if (active) {
    load8f(mean_a + static_cast<int64_t>(g) * C + c0, ma);
    load8f(mean_b + static_cast<int64_t>(g) * C + c0, mb);
    int64_t r = r0 + tr;
    for (; r + geo.rp < r1; r += 2 * geo.rp) {
      const int64_t o0 = (base + r) * C + c0, o1 = o0 + static_cast<int64_t>(geo.rp) * C;
      float a0[8], a1[8], b0[8], b1[8], d0[8], d1[8];
      load8<DT>(xa, o0, a0);
      load8<DT>(xa, o1, a1);
      load8<DT>(xb, o0, b0);
      load8<DT>(xb, o1, b1);
      load8<DT>(dy, o0, d0);
      load8<DT>(dy, o1, d1);
      relu_mask8<RM, DT>(d0, a0, nullptr, mask, o0, dum, dum);
      relu_mask8<RM, DT>(d1, a1, nullptr, mask, o1, dum, dum);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] += d0[i] + d1[i];
        qa[i] += d0[i] * (a0[i] - ma[i]) + d1[i] * (a1[i] - ma[i]);
        qb[i] += d0[i] * (b0[i] - mb[i]) + d1[i] * (b1[i] - mb[i]);
      }
    }
    for (; r < r1; r += geo.rp) {
      const int64_t o0 = (base + r) * C + c0;
      float a0[8], b0[8], d0[8];
      load8<DT>(xa, o0, a0);
      load8<DT>(xb, o0, b0);
      load8<DT>(dy, o0, d0);
      relu_mask8<RM, DT>(d0, a0, nullptr, mask, o0, dum, dum);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += d0[i]; qa[i] += d0[i] * (a0[i] - ma[i]); qb[i] += d0[i] * (b0[i] - mb[i]); }
    }
  }
  if (lane_ok) {
    float* p0 = &red[0][tr * geo.cb + tc * 8];
    float* p1 = &red[1][tr * geo.cb + tc * 8];
    float* p2 = &red[2][tr * geo.cb + tc * 8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { p0[i] = s[i]; p1[i] = qa[i]; p2[i] = qb[i]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < geo.cb; c += kThreads) {
    const int cc = cbk * geo.cb + c;
    if (cc >= C) continue;
    float a = 0.f, b = 0.f, e = 0.f;
    for (int t = 0; t < geo.rp; ++t) { a += red[0][t * geo.cb + c]; b += red[1][t * geo.cb + c]; e += red[2][t * geo.cb + c]; }
    const int64_t o = (static_cast<int64_t>(g) * geo.chunks + chunk) * 2 * C;
    part_a[o + cc] = a;
    part_a[o + C + cc] = b;
    part_b[o + cc] = a;
    part_b[o + C + cc] = e;
  }
}

template <int RM, int DT>
__global__ __launch_bounds__(kThreads) void k_bwd_apply_dual(const void* __restrict__ xa, const void* __restrict__ xb,
                                                            const void* __restrict__ dy,
                                                            const uint8_t* __restrict__ mask,
                                                            const float* __restrict__ mean_a,
                                                            const float* __restrict__ mean_b,
                                                            const float* __restrict__ coef_a,
                                                            const float* __restrict__ coef_b, int64_t rg, int64_t R,
                                                            int C, int tch, int rp, void* __restrict__ dxa,
                                                            void* __restrict__ dxb) {
  const int tr = threadIdx.x / tch;
  if (tr >= rp) return;
  const int nv = C / 8;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * rp * kApplyIters;
  const bool fixed = nv <= tch;   // one channel group per thread: its coefficients once per worker
  int gl = -1;
  float dum[8] = {}, mua[8], mub[8], caa[8], cba[8], cca[8], cab[8], cbb[8], ccb[8];
  for (int it = 0; it < kApplyIters; ++it) {
    const int64_t row = row0 + static_cast<int64_t>(it) * rp + tr;
    if (row >= R) break;
    const int g = static_cast<int>(row / rg);
    const float* ga = coef_a + static_cast<int64_t>(g) * 3 * C;
    const float* gb = coef_b + static_cast<int64_t>(g) * 3 * C;
    for (int v = threadIdx.x % tch; v < nv; v += tch) {
      const int c = v * 8;
      const int64_t off = row * C + c;
      float a[8], b[8], d[8];
      load8<DT>(xa, off, a);
      load8<DT>(xb, off, b);
      load8<DT>(dy, off, d);
      if (!fixed || g != gl) {
        load8f(mean_a + static_cast<int64_t>(g) * C + c, mua);
        load8f(mean_b + static_cast<int64_t>(g) * C + c, mub);
        load8f(ga + c, caa);
        load8f(ga + C + c, cba);
        load8f(ga + 2 * C + c, cca);
        load8f(gb + c, cab);
        load8f(gb + C + c, cbb);
        load8f(gb + 2 * C + c, ccb);
        gl = g;
      }
      relu_mask8<RM, DT>(d, a, nullptr, mask, off, dum, dum);
      float oa[8], ob[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        oa[i] = caa[i] * (d[i] - cba[i] - (a[i] - mua[i]) * cca[i]);
        ob[i] = cab[i] * (d[i] - cbb[i] - (b[i] - mub[i]) * ccb[i]);
      }
      store_vec<8>(dxa, DT, off, oa);
      store_vec<8>(dxb, DT, off, ob);
    }
  }
}

void apply_geometry(int C, int* tch, int* rp) {
  int t = C / 8;
  if (t > kThreads) t = kThreads;
  *tch = t;
  *rp = kThreads / t;
}

dim3 apply_grid(int64_t R, int rp) {
  const int64_t rows_per_wg = static_cast<int64_t>(rp) * kApplyIters;
  return dim3(static_cast<unsigned>((R + rows_per_wg - 1) / rows_per_wg));
}

// ---------------------------------------------------------------------------
// Small layers (<= kSmallRows rows per worker: CIFAR layer3/layer4, 250-1000 rows):
// the three-launch pipeline above is launch-bound there (~5 µs per dependent kernel
// for a few MB of data), so ONE workgroup per (worker, 64 channels) does the whole
// layer: the statistics pass, the finalize (LDS), and the apply pass over the same
// (L2-resident) rows. No inter-workgroup hand-off; the running statistics are
// replayed by k_running (one tiny launch, or batched for many layers by the caller).
constexpr int kSmallRows = 1024;
constexpr int kSmallThreads = 1024;             // CH = 32: 16 waves per workgroup to hide the load latency
// Channels per workgroup CH with T threads: a layer of C channels and k workers runs C / CH x k
// workgroups. One CU streams only ~24 GB/s (10 B/cycle), so the 64 workgroups of CH = 32 on a 256-channel
// layer leave three quarters of the chip idle; CH = 8 (T = 256) runs four times as many, each a quarter
// of the bytes (bn_small_ch(), GARFIELD_BN_SMALL_CH).
template <int CH, int T>
struct SmallGeo {
  static constexpr int Vec = CH / 8;                       // 16-byte vectors per row
  static constexpr int Lanes = T / Vec;                    // row lanes
  static constexpr int Split = T / CH;                     // first-stage reduction splits per channel
  static constexpr int It = kSmallRows / Lanes;            // rows per thread, held in registers
  static_assert(kSmallRows % Lanes == 0 && Lanes % Split == 0, "small-layer rows must tile the row lanes");
};
template <int CH>
constexpr int small_threads() { return CH == 8 ? 256 : (CH == 16 ? 512 : kSmallThreads); }

// (channel group, worker) of this workgroup: the workgroups that share a 128-byte row segment (8 / CH
// consecutive channel groups of one worker) get consecutive ids within one XCD's share of the grid
// (blocks are dealt to the 8 XCDs round-robin), so each segment is fetched into one L2 only
__device__ __forceinline__ void small_block(int& cg, int& g) {
  const int ncg = gridDim.x, total = gridDim.x * gridDim.y;
  const int b = blockIdx.x + blockIdx.y * ncg;
  const int w = (total % 8 == 0) ? (b % 8) * (total / 8) + b / 8 : b;
  g = w / ncg;
  cg = w - g * ncg;
}

// Sums red[k][lane][c] over the row lanes for both k; result in red[k][0][c].
template <int CH, int T, int L>
__device__ __forceinline__ void small_reduce(float (&red)[2][L][CH]) {
  constexpr int kSmallCh = CH, kSmallSplit = SmallGeo<CH, T>::Split;
  const int c = threadIdx.x % kSmallCh, part = threadIdx.x / kSmallCh;
  constexpr int per = SmallGeo<CH, T>::Lanes / kSmallSplit;
  float a = 0.f, b = 0.f;
#pragma unroll 8
  for (int t = 0; t < per; ++t) { a += red[0][part * per + t][c]; b += red[1][part * per + t][c]; }
  __syncthreads();
  red[0][part][c] = a;
  red[1][part][c] = b;
  __syncthreads();
  if (threadIdx.x < kSmallCh) {
    a = 0.f; b = 0.f;
#pragma unroll
    for (int t = 0; t < kSmallSplit; ++t) { a += red[0][t][c]; b += red[1][t][c]; }
    red[0][0][c] = a;
    red[1][0][c] = b;
  }
  __syncthreads();
}


// dz = dy where the forward output y > 0 (RM 1) / its mask bit is set (RM 2), else 0
__device__ __forceinline__ uint4 keep_pos(uint4 d, const uint4 yy) {
  // bf16 > 0: sign bit clear and non-zero
  auto keep = [](uint32_t dv, uint32_t yv) {
    const uint32_t lo = ((yv & 0x8000u) == 0 && (yv & 0x7fffu) != 0) ? 0x0000ffffu : 0u;
    const uint32_t hi = ((yv & 0x80000000u) == 0 && (yv & 0x7fff0000u) != 0) ? 0xffff0000u : 0u;
    return dv & (lo | hi);
  };
  d.x = keep(d.x, yy.x); d.y = keep(d.y, yy.y); d.z = keep(d.z, yy.z); d.w = keep(d.w, yy.w);
  return d;
}
__device__ __forceinline__ F8 keep_pos(F8 d, const F8& yy) {
  d.a.x = yy.a.x > 0.f ? d.a.x : 0.f; d.a.y = yy.a.y > 0.f ? d.a.y : 0.f;
  d.a.z = yy.a.z > 0.f ? d.a.z : 0.f; d.a.w = yy.a.w > 0.f ? d.a.w : 0.f;
  d.b.x = yy.b.x > 0.f ? d.b.x : 0.f; d.b.y = yy.b.y > 0.f ? d.b.y : 0.f;
  d.b.z = yy.b.z > 0.f ? d.b.z : 0.f; d.b.w = yy.b.w > 0.f ? d.b.w : 0.f;
  return d;
}
__device__ __forceinline__ uint4 keep_bits(uint4 d, uint32_t mb) {
  auto keep = [](uint32_t dv, uint32_t m2) {
    return dv & (((m2 & 1u) ? 0x0000ffffu : 0u) | ((m2 & 2u) ? 0xffff0000u : 0u));
  };
  d.x = keep(d.x, mb); d.y = keep(d.y, mb >> 2); d.z = keep(d.z, mb >> 4); d.w = keep(d.w, mb >> 6);
  return d;
}
__device__ __forceinline__ F8 keep_bits(F8 d, uint32_t mb) {
  d.a.x = (mb & 1u) ? d.a.x : 0.f; d.a.y = (mb & 2u) ? d.a.y : 0.f;
  d.a.z = (mb & 4u) ? d.a.z : 0.f; d.a.w = (mb & 8u) ? d.a.w : 0.f;
  d.b.x = (mb & 16u) ? d.b.x : 0.f; d.b.y = (mb & 32u) ? d.b.y : 0.f;
  d.b.z = (mb & 64u) ? d.b.z : 0.f; d.b.w = (mb & 128u) ? d.b.w : 0.f;
  return d;
}

// RM 3: dz = dy where the never-written normalised value bf16(x * scale + shift) is > 0
template <int DT>
__device__ __forceinline__ Raw8<DT> keep_affine(Raw8<DT> d, const Raw8<DT>& xr, const float (&sc)[8],
                                                const float (&sf)[8]) {
  float a[8];
  unpack8(xr, a);
  if constexpr (DT == kF32) {
    float dd[8];
    unpack8(d, dd);
#pragma unroll
    for (int i = 0; i < 8; ++i) dd[i] = stored_pos<DT>(fmaxf(fmaf(a[i], sc[i], sf[i]), 0.f)) ? dd[i] : 0.f;
    return F8{make_float4(dd[0], dd[1], dd[2], dd[3]), make_float4(dd[4], dd[5], dd[6], dd[7])};
  } else {
    uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (!stored_pos<DT>(fmaxf(fmaf(a[i], sc[i], sf[i]), 0.f))) w[i >> 1] &= (i & 1) ? 0x0000ffffu : 0xffff0000u;
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Each thread keeps its (<= kSmallIt) rows of 8 channels in registers as stored (packed
// bf16 or fp32), so the apply pass does not re-read x (or dy) from memory.
template <int CH, bool RES, bool RELU, int DT, int T = small_threads<CH>()>
__global__ __launch_bounds__(T) void k_bn_fwd_small(const void* __restrict__ x,
                                                          const void* __restrict__ res, int64_t rg, int C,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          float* __restrict__ mean, float* __restrict__ istd,
                                                          float* __restrict__ scale, float* __restrict__ shift,
                                                          void* __restrict__ y, uint8_t* __restrict__ mask,
                                                          const float* __restrict__ res_sc,
                                                          const float* __restrict__ res_sh) {
  constexpr int kSmallCh = CH, kSmallVec = SmallGeo<CH, T>::Vec, kSmallLanes = SmallGeo<CH, T>::Lanes,
                kSmallIt = SmallGeo<CH, T>::It;
  __shared__ float red[2][kSmallLanes][kSmallCh];
  __shared__ float lsc[kSmallCh], lsh[kSmallCh];
  const int tc = threadIdx.x % kSmallVec, tr = threadIdx.x / kSmallVec;
  int cg, g;
  small_block(cg, g);
  const int c0 = cg * kSmallCh + tc * 8;
  const bool act = c0 < C;
  const int64_t base = static_cast<int64_t>(g) * rg;
  float s[8], q[8], sh[8];
  Raw8<DT> xr[kSmallIt];
  // the finalize thread's operands, loaded now instead of after the reduction (off its critical path)
  float fg = 1.f, fb = 0.f, fx0 = 0.f;
  if (threadIdx.x < kSmallCh && cg * kSmallCh + static_cast<int>(threadIdx.x) < C) {
    const int c = cg * kSmallCh + threadIdx.x;
    fg = gamma ? gamma[c] : 1.f;
    fb = beta ? beta[c] : 0.f;
    fx0 = load_one<DT>(x, base * C + c);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; q[i] = 0.f; sh[i] = 0.f; }
  if (act) {
    load8<DT>(x, base * C + c0, sh);   // shifted sums (see k_partial)
#pragma unroll
    for (int it = 0; it < kSmallIt; ++it) {
      const int64_t r = tr + it * kSmallLanes;
      if (r < rg) xr[it] = ld_raw8<DT>(x, (base + r) * C + c0);
    }
#pragma unroll
    for (int it = 0; it < kSmallIt; ++it) {
      if (tr + it * kSmallLanes < rg) {
        float a[8];
        unpack8(xr[it], a);
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float e = a[i] - sh[i]; s[i] += e; q[i] += e * e; }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[0][tr][tc * 8 + i] = s[i]; red[1][tr][tc * 8 + i] = q[i]; }
  __syncthreads();
  small_reduce<CH, T, kSmallLanes>(red);
  if (threadIdx.x < kSmallCh) {
    const int c = cg * kSmallCh + threadIdx.x;
    const float S = red[0][0][threadIdx.x], Q = red[1][0][threadIdx.x];
    float sc = 0.f, sf = 0.f;
    if (c < C) {
      const float M = static_cast<float>(rg);
      const float m1 = S / M;
      float var = Q / M - m1 * m1;
      var = var > 0.f ? var : 0.f;
      const float mu = fx0 + m1;
      const float is = rsqrtf(var + eps);
      const int64_t gc = static_cast<int64_t>(g) * C + c;
      mean[gc] = mu;
      istd[gc] = is;
      sc = fg * is;
      sf = fb - mu * sc;
      scale[gc] = sc;
      shift[gc] = sf;
    }
    lsc[threadIdx.x] = sc;
    lsh[threadIdx.x] = sf;
  }
  __syncthreads();
  if (!act || y == nullptr) return;   // y null: statistics only (the consumer applies scale / shift itself)
  float sc[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sc[i] = lsc[tc * 8 + i]; sf[i] = lsh[tc * 8 + i]; }
#pragma unroll
  for (int it = 0; it < kSmallIt; ++it) {
    const int64_t r = tr + it * kSmallLanes;
    if (r >= rg) break;
    const int64_t off = (base + r) * C + c0;
    float a[8], o[8];
    unpack8(xr[it], a);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = a[i] * sc[i] + sf[i];
    if constexpr (RES) {
      float rr[8];
      load8<DT>(res, off, rr);
      if (res_sc) {   // a pre-BatchNorm residual: its BatchNorm's scale / shift applied here
        float ra[8], rb[8];
        load8f(res_sc + static_cast<int64_t>(g) * C + c0, ra);
        load8f(res_sh + static_cast<int64_t>(g) * C + c0, rb);
#pragma unroll
        for (int i = 0; i < 8; ++i) rr[i] = rr[i] * ra[i] + rb[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] += rr[i];
    }
    if constexpr (RELU) {
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = o[i] > 0.f ? o[i] : 0.f;
      if (mask) {
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) bits |= (stored_pos<DT>(o[i]) ? 1u : 0u) << i;
        mask[off >> 3] = static_cast<uint8_t>(bits);
      }
    }
    store_vec<8>(y, DT, off, o);
  }
}

template <int CH, int RM, bool RES_OUT, int DT, int T = small_threads<CH>()>
__global__ __launch_bounds__(T) void k_bn_bwd_small(
    const void* __restrict__ x, const void* __restrict__ dy, const void* __restrict__ y,
    const uint8_t* __restrict__ mask, int64_t rg, int C, const float* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ istd, void* __restrict__ dx,
    void* __restrict__ dres, void* grow, int grow_dt, int64_t row_stride, int64_t off_gamma, int64_t off_beta,
    const float* __restrict__ rsc, const float* __restrict__ rsh) {
  constexpr int kSmallCh = CH, kSmallVec = SmallGeo<CH, T>::Vec, kSmallLanes = SmallGeo<CH, T>::Lanes,
                kSmallIt = SmallGeo<CH, T>::It;
  __shared__ float red[2][kSmallLanes][kSmallCh];
  __shared__ float la[kSmallCh], lb[kSmallCh], lc[kSmallCh];
  const int tc = threadIdx.x % kSmallVec, tr = threadIdx.x / kSmallVec;
  int cg, g;
  small_block(cg, g);
  const int c0 = cg * kSmallCh + tc * 8;
  const bool act = c0 < C;
  const int64_t base = static_cast<int64_t>(g) * rg;
  // dz = dy masked by the forward ReLU, kept as stored in registers with x
  Raw8<DT> xr[kSmallIt], dr[kSmallIt];
  float A[8], B[8], mu[8], rs[8] = {}, rf[8] = {};
  float fis = 0.f, fg = 1.f;   // the finalize thread's operands, loaded before the reduction
  if (threadIdx.x < kSmallCh && cg * kSmallCh + static_cast<int>(threadIdx.x) < C) {
    const int c = cg * kSmallCh + threadIdx.x;
    fis = istd[static_cast<int64_t>(g) * C + c];
    fg = gamma ? gamma[c] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { A[i] = 0.f; B[i] = 0.f; mu[i] = 0.f; }
  if (act) {
    load8f(mean + static_cast<int64_t>(g) * C + c0, mu);
    if constexpr (RM == 3) {
      load8f(rsc + static_cast<int64_t>(g) * C + c0, rs);
      load8f(rsh + static_cast<int64_t>(g) * C + c0, rf);
    }
#pragma unroll
    for (int it = 0; it < kSmallIt; ++it) {
      const int64_t r = tr + it * kSmallLanes;
      if (r < rg) {
        const int64_t off = (base + r) * C + c0;
        xr[it] = ld_raw8<DT>(x, off);
        Raw8<DT> d = ld_raw8<DT>(dy, off);
        if constexpr (RM == 1) d = keep_pos(d, ld_raw8<DT>(y, off));
        else if constexpr (RM == 2) d = keep_bits(d, mask[off >> 3]);
        else if constexpr (RM == 3) d = keep_affine<DT>(d, xr[it], rs, rf);
        dr[it] = d;
      }
    }
#pragma unroll
    for (int it = 0; it < kSmallIt; ++it) {
      if (tr + it * kSmallLanes < rg) {
        float a[8], d[8];
        unpack8(xr[it], a);
        unpack8(dr[it], d);
#pragma unroll
        for (int i = 0; i < 8; ++i) { A[i] += d[i]; B[i] += d[i] * (a[i] - mu[i]); }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[0][tr][tc * 8 + i] = A[i]; red[1][tr][tc * 8 + i] = B[i]; }
  __syncthreads();
  small_reduce<CH, T, kSmallLanes>(red);
  if (threadIdx.x < kSmallCh) {
    const int c = cg * kSmallCh + threadIdx.x;
    const float SA = red[0][0][threadIdx.x], SB = red[1][0][threadIdx.x];
    float ca = 0.f, cb = 0.f, cc = 0.f;
    if (c < C) {
      const float M = static_cast<float>(rg);
      const float is = fis;
      const float dgamma = SB * is, dbeta = SA;
      if (grow) {
        if (off_gamma >= 0) store_one(grow, grow_dt, static_cast<int64_t>(g) * row_stride + off_gamma + c, dgamma);
        if (off_beta >= 0) store_one(grow, grow_dt, static_cast<int64_t>(g) * row_stride + off_beta + c, dbeta);
      }
      ca = fg * is;
      cb = dbeta / M;
      cc = dgamma / M * is;
    }
    la[threadIdx.x] = ca;
    lb[threadIdx.x] = cb;
    lc[threadIdx.x] = cc;
  }
  __syncthreads();
  if (!act) return;
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { ca[i] = la[tc * 8 + i]; cb[i] = lb[tc * 8 + i]; cc[i] = lc[tc * 8 + i]; }
#pragma unroll
  for (int it = 0; it < kSmallIt; ++it) {
    const int64_t r = tr + it * kSmallLanes;
    if (r >= rg) break;
    const int64_t off = (base + r) * C + c0;
    float a[8], d[8], o[8];
    unpack8(xr[it], a);
    unpack8(dr[it], d);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = ca[i] * (d[i] - cb[i] - (a[i] - mu[i]) * cc[i]);
    store_vec<8>(dx, DT, off, o);
    if constexpr (RES_OUT) st_raw8<DT>(dres, off, dr[it]);
  }
}

// Dual form of the above for a projection block's last BatchNorm (a) and its folded shortcut BatchNorm
// (b), which share dz: x_a, x_b and dz rows held in registers, Σdz shared, both finalizes in the same
// workgroup, both data gradients from one read of dy and the mask.
template <int CH, int RM, int DT, int T = small_threads<CH>()>
__global__ __launch_bounds__(T) void k_bn_bwd_small_dual(
    const void* __restrict__ xa, const void* __restrict__ xb, const void* __restrict__ dy,
    const uint8_t* __restrict__ mask, int64_t rg, int C, const float* __restrict__ gamma_a,
    const float* __restrict__ mean_a, const float* __restrict__ istd_a, const float* __restrict__ gamma_b,
    const float* __restrict__ mean_b, const float* __restrict__ istd_b, void* __restrict__ dxa,
    void* __restrict__ dxb, void* grow, int grow_dt, int64_t row_stride, int64_t oga, int64_t oba, int64_t ogb,
    int64_t obb) {
  static_assert(RM == 0 || RM == 2, "dz is dy or dy under the bit mask");
  constexpr int kSmallCh = CH, kSmallVec = SmallGeo<CH, T>::Vec, kSmallLanes = SmallGeo<CH, T>::Lanes,
                kSmallIt = SmallGeo<CH, T>::It;
  __shared__ float red[2][kSmallLanes][kSmallCh];
  __shared__ float sA[kSmallCh], la[2][kSmallCh], lb[2][kSmallCh], lc[2][kSmallCh];
  const int tc = threadIdx.x % kSmallVec, tr = threadIdx.x / kSmallVec;
  int cg, g;
  small_block(cg, g);
  const int c0 = cg * kSmallCh + tc * 8;
  const bool act = c0 < C;
  const int64_t base = static_cast<int64_t>(g) * rg;
  Raw8<DT> xra[kSmallIt], xrb[kSmallIt], dr[kSmallIt];
  float A[8], Ba[8], Bb[8], mua[8], mub[8];
  float fis[2] = {0.f, 0.f}, fg[2] = {1.f, 1.f};   // the finalize thread's operands, loaded up front
  if (threadIdx.x < kSmallCh && cg * kSmallCh + static_cast<int>(threadIdx.x) < C) {
    const int c = cg * kSmallCh + threadIdx.x;
    fis[0] = istd_a[static_cast<int64_t>(g) * C + c];
    fis[1] = istd_b[static_cast<int64_t>(g) * C + c];
    fg[0] = gamma_a ? gamma_a[c] : 1.f;
    fg[1] = gamma_b ? gamma_b[c] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { A[i] = 0.f; Ba[i] = 0.f; Bb[i] = 0.f; mua[i] = 0.f; mub[i] = 0.f; }
  if (act) {
    load8f(mean_a + static_cast<int64_t>(g) * C + c0, mua);
    load8f(mean_b + static_cast<int64_t>(g) * C + c0, mub);
#pragma unroll
    for (int it = 0; it < kSmallIt; ++it) {
      const int64_t r = tr + it * kSmallLanes;
      if (r < rg) {
        const int64_t off = (base + r) * C + c0;
        xra[it] = ld_raw8<DT>(xa, off);
        xrb[it] = ld_raw8<DT>(xb, off);
        Raw8<DT> d = ld_raw8<DT>(dy, off);
        if constexpr (RM == 2) d = keep_bits(d, mask[off >> 3]);
        dr[it] = d;
      }
    }
#pragma unroll
    for (int it = 0; it < kSmallIt; ++it) {
      if (tr + it * kSmallLanes < rg) {
        float a[8], b[8], d[8];
        unpack8(xra[it], a);
        unpack8(xrb[it], b);
        unpack8(dr[it], d);
#pragma unroll
        for (int i = 0; i < 8; ++i) { A[i] += d[i]; Ba[i] += d[i] * (a[i] - mua[i]); Bb[i] += d[i] * (b[i] - mub[i]); }
      }
    }
  }
  // Σdz and Σdz(x_a - μ_a), then Σdz(x_b - μ_b) (in red[1] again)
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[0][tr][tc * 8 + i] = A[i]; red[1][tr][tc * 8 + i] = Ba[i]; }
  __syncthreads();
  small_reduce<CH, T, kSmallLanes>(red);
  float SA = 0.f, SBa = 0.f;
  if (threadIdx.x < kSmallCh) { SA = red[0][0][threadIdx.x]; SBa = red[1][0][threadIdx.x]; }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[0][tr][tc * 8 + i] = 0.f; red[1][tr][tc * 8 + i] = Bb[i]; }
  __syncthreads();
  small_reduce<CH, T, kSmallLanes>(red);
  if (threadIdx.x < kSmallCh) {
    const int c = cg * kSmallCh + threadIdx.x;
    const float SBb = red[1][0][threadIdx.x];
    const float M = static_cast<float>(rg);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float ca = 0.f, cb = 0.f, cc = 0.f;
      if (c < C) {
        const float is = fis[k];
        const float dgamma = (k == 0 ? SBa : SBb) * is, dbeta = SA;
        const int64_t og = k == 0 ? oga : ogb, ob = k == 0 ? oba : obb;
        if (grow) {
          if (og >= 0) store_one(grow, grow_dt, static_cast<int64_t>(g) * row_stride + og + c, dgamma);
          if (ob >= 0) store_one(grow, grow_dt, static_cast<int64_t>(g) * row_stride + ob + c, dbeta);
        }
        ca = fg[k] * is;
        cb = dbeta / M;
        cc = dgamma / M * is;
      }
      la[k][threadIdx.x] = ca;
      lb[k][threadIdx.x] = cb;
      lc[k][threadIdx.x] = cc;
    }
  }
  __syncthreads();
  if (!act) return;
  float caa[8], cba[8], cca[8], cab[8], cbb[8], ccb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    caa[i] = la[0][tc * 8 + i]; cba[i] = lb[0][tc * 8 + i]; cca[i] = lc[0][tc * 8 + i];
    cab[i] = la[1][tc * 8 + i]; cbb[i] = lb[1][tc * 8 + i]; ccb[i] = lc[1][tc * 8 + i];
  }
#pragma unroll
  for (int it = 0; it < kSmallIt; ++it) {
    const int64_t r = tr + it * kSmallLanes;
    if (r >= rg) break;
    const int64_t off = (base + r) * C + c0;
    float a[8], b[8], d[8], oa[8], ob[8];
    unpack8(xra[it], a);
    unpack8(xrb[it], b);
    unpack8(dr[it], d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      oa[i] = caa[i] * (d[i] - cba[i] - (a[i] - mua[i]) * cca[i]);
      ob[i] = cab[i] * (d[i] - cbb[i] - (b[i] - mub[i]) * ccb[i]);
    }
    store_vec<8>(dxa, DT, off, oa);
    store_vec<8>(dxb, DT, off, ob);
  }
}

// Running statistics of up to kRunJobs layers in one launch (blockIdx.y = layer).
__global__ __launch_bounds__(kThreads) void k_running(RunJobs jobs) {
  const RunJob& j = jobs.j[blockIdx.y];
  const float M = static_cast<float>(j.rg);
  for (int c = blockIdx.x * kThreads + threadIdx.x; c < j.C; c += gridDim.x * kThreads) {
    float rm = j.run_mean[c], rv = j.run_var[c];
    for (int g = 0; g < j.groups; ++g) {
      const float is = j.istd[static_cast<int64_t>(g) * j.C + c];
      float var = 1.f / (is * is) - j.eps;
      var = var > 0.f ? var : 0.f;
      const float unb = j.rg > 1 ? var * M / (M - 1.f) : var;
      rm = (1.f - j.momentum) * rm + j.momentum * j.mean[static_cast<int64_t>(g) * j.C + c];
      rv = (1.f - j.momentum) * rv + j.momentum * unb;
    }
    j.run_mean[c] = rm;
    j.run_var[c] = rv;
  }
}

template <int CH, int DT>
void launch_fwd_small(const void* x, const void* res, int64_t rg, int groups, int C, const float* gamma,
                      const float* beta, float eps, float* mean, float* istd, float* scale, float* shift, void* y,
                      bool relu, uint8_t* mask, hipStream_t stream, const float* res_sc, const float* res_sh) {
  const dim3 sgrid((C + CH - 1) / CH, groups);
  if (res) {
    if (relu) hipLaunchKernelGGL((k_bn_fwd_small<CH, true, true, DT>), sgrid, dim3(small_threads<CH>()), 0, stream, x, res, rg, C, gamma, beta, eps, mean, istd, scale, shift, y, mask, res_sc, res_sh);
    else hipLaunchKernelGGL((k_bn_fwd_small<CH, true, false, DT>), sgrid, dim3(small_threads<CH>()), 0, stream, x, res, rg, C, gamma, beta, eps, mean, istd, scale, shift, y, nullptr, res_sc, res_sh);
  } else {
    if (relu) hipLaunchKernelGGL((k_bn_fwd_small<CH, false, true, DT>), sgrid, dim3(small_threads<CH>()), 0, stream, x, res, rg, C, gamma, beta, eps, mean, istd, scale, shift, y, mask, res_sc, res_sh);
    else hipLaunchKernelGGL((k_bn_fwd_small<CH, false, false, DT>), sgrid, dim3(small_threads<CH>()), 0, stream, x, res, rg, C, gamma, beta, eps, mean, istd, scale, shift, y, nullptr, res_sc, res_sh);
  }
}

template <int CH, int DT>
void launch_bwd_small(const void* x, const void* dy, const void* y, const uint8_t* mask, int64_t rg,
                      int groups, int C, const float* gamma, const float* mean, const float* istd, void* dx,
                      void* dres, void* grow, int grow_dt, int64_t row_stride, int64_t off_gamma, int64_t off_beta,
                      int rm, hipStream_t stream, const float* rsc, const float* rsh) {
  const dim3 sgrid((C + CH - 1) / CH, groups);
#define GARFIELD_BWD_SMALL(RMV, RESV)                                                                           \
  hipLaunchKernelGGL((k_bn_bwd_small<CH, RMV, RESV, DT>), sgrid, dim3(small_threads<CH>()), 0, stream, x, dy, y, mask, rg, C, \
                     gamma, mean, istd, dx, dres, grow, grow_dt, row_stride, off_gamma, off_beta, rsc, rsh)
  if (rm == 3) { if (dres) GARFIELD_BWD_SMALL(3, true); else GARFIELD_BWD_SMALL(3, false); }
  else if (rm == 2) { if (dres) GARFIELD_BWD_SMALL(2, true); else GARFIELD_BWD_SMALL(2, false); }
  else if (rm == 1) { if (dres) GARFIELD_BWD_SMALL(1, true); else GARFIELD_BWD_SMALL(1, false); }
  else { if (dres) GARFIELD_BWD_SMALL(0, true); else GARFIELD_BWD_SMALL(0, false); }
#undef GARFIELD_BWD_SMALL
}

template <int DT>
void forward_dt(const void* x, const void* res, int64_t rg, int groups, int C, const float* gamma,
                const float* beta, float eps, float momentum, float* run_mean, float* run_var, float* part,
                float* mean, float* istd, float* scale, float* shift, void* y, bool relu, uint8_t* mask,
                bool defer_running, hipStream_t stream, const float* tile_stats, int64_t tile_m, int tile_e,
                const float* res_sc, const float* res_sh) {
  if (rg <= kSmallRows && tile_stats == nullptr) {
    switch (small_ch_for(C, groups)) {
      case 8: launch_fwd_small<8, DT>(x, res, rg, groups, C, gamma, beta, eps, mean, istd, scale, shift, y, relu, mask, stream, res_sc, res_sh); break;
      case 16: launch_fwd_small<16, DT>(x, res, rg, groups, C, gamma, beta, eps, mean, istd, scale, shift, y, relu, mask, stream, res_sc, res_sh); break;
      default: launch_fwd_small<32, DT>(x, res, rg, groups, C, gamma, beta, eps, mean, istd, scale, shift, y, relu, mask, stream, res_sc, res_sh); break;
    }
    if (run_mean && !defer_running) {
      RunJobs jobs{};
      jobs.j[0] = RunJob{mean, istd, run_mean, run_var, rg, C, groups, eps, momentum};
      jobs.n = 1;
      bn_running_update(jobs, stream);
    }
    return;
  }
  if (tile_stats) {   // statistics from the producing GEMM's epilogue (gemm_nt.hip): no partial pass
    bn_finalize_tiles(tile_stats, tile_m, tile_e, rg * groups, rg, groups, C, gamma, beta, eps, mean, istd, scale,
                      shift, stream);
  } else {
    const Geo g = geometry(rg, groups, C);
    const int ncb = (C + g.cb - 1) / g.cb;
    hipLaunchKernelGGL((k_partial<false, 0, DT>), dim3(g.chunks, ncb, groups), dim3(kThreads), 0, stream, x, nullptr,
                       nullptr, nullptr, nullptr, g, part, nullptr, nullptr);
    hipLaunchKernelGGL((k_fwd_finalize<DT, kFin>), dim3((C + kFin - 1) / kFin, groups), dim3(kThreads), 0, stream, part,
                       x, g, gamma, beta, eps, mean, istd, scale, shift);
  }
  if (y == nullptr) {   // statistics only: the running statistics without the apply pass's first workgroup
    if (run_mean && !defer_running) {
      RunJobs jobs{};
      jobs.j[0] = RunJob{mean, istd, run_mean, run_var, rg, C, groups, eps, momentum};
      jobs.n = 1;
      bn_running_update(jobs, stream);
    }
    return;
  }
  const RunStats rs{mean, istd, run_mean, run_var, eps, momentum, groups, res_sc, res_sh};
  int tch, rp;
  apply_geometry(C, &tch, &rp);
  const int64_t R = rg * groups;
  const dim3 grid = apply_grid(R, rp);
  if (res) {
    if (relu) hipLaunchKernelGGL((k_fwd_apply<true, true, DT>), grid, dim3(kThreads), 0, stream, x, res, scale, shift, rg, R, C, tch, rp, y, mask, rs);
    else hipLaunchKernelGGL((k_fwd_apply<true, false, DT>), grid, dim3(kThreads), 0, stream, x, res, scale, shift, rg, R, C, tch, rp, y, nullptr, rs);
  } else {
    if (relu) hipLaunchKernelGGL((k_fwd_apply<false, true, DT>), grid, dim3(kThreads), 0, stream, x, res, scale, shift, rg, R, C, tch, rp, y, mask, rs);
    else hipLaunchKernelGGL((k_fwd_apply<false, false, DT>), grid, dim3(kThreads), 0, stream, x, res, scale, shift, rg, R, C, tch, rp, y, nullptr, rs);
  }
}

template <int DT>
void backward_dt(const void* x, const void* dy, const void* y, const uint8_t* mask, int64_t rg, int groups,
                 int C, const float* gamma, const float* mean, const float* istd, float* part, float* coef, void* dx,
                 void* dres, void* grow, int grow_dt, int64_t row_stride, int64_t off_gamma, int64_t off_beta,
                 hipStream_t stream, const float* rsc, const float* rsh) {
  const int rm = mask ? 2 : (y ? 1 : (rsc ? 3 : 0));
  if (rg <= kSmallRows) {
    switch (small_ch_for(C, groups)) {
      case 8: launch_bwd_small<8, DT>(x, dy, y, mask, rg, groups, C, gamma, mean, istd, dx, dres, grow, grow_dt, row_stride, off_gamma, off_beta, rm, stream, rsc, rsh); break;
      case 16: launch_bwd_small<16, DT>(x, dy, y, mask, rg, groups, C, gamma, mean, istd, dx, dres, grow, grow_dt, row_stride, off_gamma, off_beta, rm, stream, rsc, rsh); break;
      default: launch_bwd_small<32, DT>(x, dy, y, mask, rg, groups, C, gamma, mean, istd, dx, dres, grow, grow_dt, row_stride, off_gamma, off_beta, rm, stream, rsc, rsh); break;
    }
    return;
  }
  const Geo g = geometry(rg, groups, C);
  const int ncb = (C + g.cb - 1) / g.cb;
  const dim3 pgrid(g.chunks, ncb, groups);
#define GARFIELD_PARTIAL(RMV) \
  hipLaunchKernelGGL((k_partial<true, RMV, DT>), pgrid, dim3(kThreads), 0, stream, x, dy, y, mask, mean, g, part, rsc, rsh)
  if (rm == 3) GARFIELD_PARTIAL(3);
  else if (rm == 2) GARFIELD_PARTIAL(2);
  else if (rm == 1) GARFIELD_PARTIAL(1);
  else GARFIELD_PARTIAL(0);
#undef GARFIELD_PARTIAL
  hipLaunchKernelGGL(k_bwd_finalize<kFin>, dim3((C + kFin - 1) / kFin, groups), dim3(kThreads), 0, stream, part, g,
                     gamma, istd, coef, grow, grow_dt, row_stride, off_gamma, off_beta);
  int tch, rp;
  apply_geometry(C, &tch, &rp);
  const int64_t R = rg * groups;
  const dim3 grid = apply_grid(R, rp);
#define GARFIELD_BWD_APPLY(RMV, RESV) \
  hipLaunchKernelGGL((k_bwd_apply<RMV, RESV, DT>), grid, dim3(kThreads), 0, stream, x, dy, y, mask, mean, coef, rg, R, C, tch, rp, dx, dres, rsc, rsh)
  if (rm == 3) { if (dres) GARFIELD_BWD_APPLY(3, true); else GARFIELD_BWD_APPLY(3, false); }
  else if (rm == 2) { if (dres) GARFIELD_BWD_APPLY(2, true); else GARFIELD_BWD_APPLY(2, false); }
  else if (rm == 1) { if (dres) GARFIELD_BWD_APPLY(1, true); else GARFIELD_BWD_APPLY(1, false); }
  else { if (dres) GARFIELD_BWD_APPLY(0, true); else GARFIELD_BWD_APPLY(0, false); }
#undef GARFIELD_BWD_APPLY
}

template <int DT>
void backward_dual_dt(const void* xa, const void* xb, const void* dy, const uint8_t* mask, int64_t rg, int groups,
                      int C, const float* gamma_a, const float* gamma_b, const float* mean_a, const float* istd_a,
                      const float* mean_b, const float* istd_b, float* part_a, float* part_b, float* coef_a,
                      float* coef_b, void* dxa, void* dxb, void* grow, int grow_dt, int64_t row_stride,
                      int64_t og_a, int64_t ob_a, int64_t og_b, int64_t ob_b, hipStream_t stream) {
  const Geo g = geometry(rg, groups, C);
  const int ncb = (C + g.cb - 1) / g.cb;
  const dim3 pgrid(g.chunks, ncb, groups);
  if (mask)
    hipLaunchKernelGGL((k_partial_dual<2, DT>), pgrid, dim3(kThreads), 0, stream, xa, xb, dy, mask, mean_a, mean_b, g,
                       part_a, part_b);
  else
    hipLaunchKernelGGL((k_partial_dual<0, DT>), pgrid, dim3(kThreads), 0, stream, xa, xb, dy, mask, mean_a, mean_b, g,
                       part_a, part_b);
  const dim3 fgrid((C + kFin - 1) / kFin, groups, 2);
  hipLaunchKernelGGL(k_bwd_finalize_dual<kFin>, fgrid, dim3(kThreads), 0, stream,
                     FinJob{part_a, gamma_a, istd_a, coef_a, og_a, ob_a}, FinJob{part_b, gamma_b, istd_b, coef_b, og_b, ob_b},
                     g, grow, grow_dt, row_stride);
  int tch, rp;
  apply_geometry(C, &tch, &rp);
  const int64_t R = rg * groups;
  const dim3 grid = apply_grid(R, rp);
  if (mask)
    hipLaunchKernelGGL((k_bwd_apply_dual<2, DT>), grid, dim3(kThreads), 0, stream, xa, xb, dy, mask, mean_a, mean_b,
                       coef_a, coef_b, rg, R, C, tch, rp, dxa, dxb);
  else
    hipLaunchKernelGGL((k_bwd_apply_dual<0, DT>), grid, dim3(kThreads), 0, stream, xa, xb, dy, mask, mean_a, mean_b,
                       coef_a, coef_b, rg, R, C, tch, rp, dxa, dxb);
}

}  // namespace

int64_t bn_part_floats(int64_t rg, int groups, int C) {
  const Geo g = geometry(rg, groups, C);
  return static_cast<int64_t>(groups) * g.chunks * 2 * C;
}

void bn_forward(const void* x, const void* res, int64_t rg, int groups, int C, const float* gamma,
                const float* beta, float eps, float momentum, float* run_mean, float* run_var, float* part,
                float* mean, float* istd, float* scale, float* shift, void* y, bool relu, uint8_t* mask,
                bool defer_running, hipStream_t stream, const float* tile_stats, int64_t tile_m,
                int tile_e, int dt, const float* res_sc, const float* res_sh) {
  if (dt == kF32)
    forward_dt<kF32>(x, res, rg, groups, C, gamma, beta, eps, momentum, run_mean, run_var, part, mean, istd, scale,
                     shift, y, relu, mask, defer_running, stream, tile_stats, tile_m, tile_e, res_sc,
                     res_sh);
  else
    forward_dt<kBF16>(x, res, rg, groups, C, gamma, beta, eps, momentum, run_mean, run_var, part, mean, istd, scale,
                      shift, y, relu, mask, defer_running, stream, tile_stats, tile_m, tile_e, res_sc,
                     res_sh);
}

void bn_backward(const void* x, const void* dy, const void* y, const uint8_t* mask, int64_t rg, int groups,
                 int C, const float* gamma, const float* mean, const float* istd, float* part, float* coef, void* dx,
                 void* dres, void* grow, int grow_dt, int64_t row_stride, int64_t off_gamma, int64_t off_beta,
                 hipStream_t stream, int dt, const float* rsc, const float* rsh) {
  if (dt == kF32)
    backward_dt<kF32>(x, dy, y, mask, rg, groups, C, gamma, mean, istd, part, coef, dx, dres, grow, grow_dt, row_stride,
                      off_gamma, off_beta, stream, rsc, rsh);
  else
    backward_dt<kBF16>(x, dy, y, mask, rg, groups, C, gamma, mean, istd, part, coef, dx, dres, grow, grow_dt,
                       row_stride, off_gamma, off_beta, stream, rsc, rsh);
}

void bn_backward_dual(const void* xa, const void* xb, const void* dy, const uint8_t* mask, int64_t rg, int groups,
                      int C, const float* gamma_a, const float* gamma_b, const float* mean_a, const float* istd_a,
                      const float* mean_b, const float* istd_b, float* part_a, float* part_b, float* coef_a,
                      float* coef_b, void* dxa, void* dxb, void* grow, int grow_dt, int64_t row_stride,
                      int64_t og_a, int64_t ob_a, int64_t og_b, int64_t ob_b, hipStream_t stream, int dt) {
  if (rg <= kSmallRows) {   // the single-kernel small path, both BatchNorms in one workgroup
    const int ch = small_ch_for(C, groups);
    const int rm = mask ? 2 : 0;
#define GARFIELD_DUAL_SMALL(CHV, RMV, DTV)                                                                          \
  hipLaunchKernelGGL((k_bn_bwd_small_dual<CHV, RMV, DTV>), dim3((C + CHV - 1) / CHV, groups),                       \
                     dim3(small_threads<CHV>()), 0, stream, xa, xb, dy, mask, rg, C, gamma_a, mean_a, istd_a, gamma_b, \
                     mean_b, istd_b, dxa, dxb, grow, grow_dt, row_stride, og_a, ob_a, og_b, ob_b)
#define GARFIELD_DUAL_SMALL_RM(CHV, DTV) \
  if (rm == 2) GARFIELD_DUAL_SMALL(CHV, 2, DTV); else GARFIELD_DUAL_SMALL(CHV, 0, DTV)
    if (dt == kF32) {
      if (ch == 8) { GARFIELD_DUAL_SMALL_RM(8, kF32); }
      else if (ch == 16) { GARFIELD_DUAL_SMALL_RM(16, kF32); }
      else { GARFIELD_DUAL_SMALL_RM(32, kF32); }
    } else {
      if (ch == 8) { GARFIELD_DUAL_SMALL_RM(8, kBF16); }
      else if (ch == 16) { GARFIELD_DUAL_SMALL_RM(16, kBF16); }
      else { GARFIELD_DUAL_SMALL_RM(32, kBF16); }
    }
#undef GARFIELD_DUAL_SMALL_RM
#undef GARFIELD_DUAL_SMALL
    return;
  }
  if (dt == kF32)
    backward_dual_dt<kF32>(xa, xb, dy, mask, rg, groups, C, gamma_a, gamma_b, mean_a, istd_a, mean_b, istd_b, part_a,
                           part_b, coef_a, coef_b, dxa, dxb, grow, grow_dt, row_stride, og_a, ob_a, og_b, ob_b, stream);
  else
    backward_dual_dt<kBF16>(xa, xb, dy, mask, rg, groups, C, gamma_a, gamma_b, mean_a, istd_a, mean_b, istd_b, part_a,
                            part_b, coef_a, coef_b, dxa, dxb, grow, grow_dt, row_stride, og_a, ob_a, og_b, ob_b,
                            stream);
}

void bn_running_update(const RunJobs& jobs, hipStream_t stream) {
  if (jobs.n <= 0) return;
  int cmax = 0;
  for (int i = 0; i < jobs.n; ++i) cmax = jobs.j[i].C > cmax ? jobs.j[i].C : cmax;
  const dim3 grid((cmax + kThreads - 1) / kThreads, jobs.n);
  hipLaunchKernelGGL(k_running, grid, dim3(kThreads), 0, stream, jobs);
}

bool bn_small(int64_t rg) { return rg <= kSmallRows; }

namespace {
int g_small_ch = -1;
}
int bn_small_ch() {
  if (g_small_ch < 0) {
    const char* e = std::getenv("GARFIELD_BN_SMALL_CH");
    const int v = e ? std::atoi(e) : 0;
    g_small_ch = (v == 8 || v == 16 || v == 32) ? v : 0;
  }
  return g_small_ch;
}
void set_bn_small_ch(int ch) { g_small_ch = (ch == 8 || ch == 16 || ch == 32) ? ch : 0; }
// 0 (automatic): the widest CH whose grid has >= 256 workgroups (one per CU), else 8. ResNet-50 CIFAR,
// 8 workers: 256-channel layers run CH = 8 (9.8 -> 7.2 µs forward), 1024 / 2048-channel ones CH = 32
// (18.4 vs 21.4 µs with CH = 8) (profiles/r5/bn_small_ch/)
int small_ch_for(int C, int groups) {
  const int forced = bn_small_ch();
  if (forced) return forced;
  for (int ch : {32, 16})
    if (static_cast<int64_t>((C + ch - 1) / ch) * groups >= 256) return ch;
  return 8;
}

}  // namespace gpu
}  // namespace garfield
