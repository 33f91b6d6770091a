// Weighted combine (+ fused SGD) and Aksel distance kernels for gfx950.
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

// ---------------------------------------------------------------------------
// Weighted combine. The selected rows (non-zero weights) are compacted in LDS
// first, so unselected gradients are never read, and 4 row loads are kept in
// flight per lane.

template <int DT>
__device__ __forceinline__ void gather_weighted(const RowTable& rows, const int* sel, const float* wsel,
                                                int cnt, int64_t x, float (&acc)[8]) {
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
  int j = 0;
  for (; j + 4 <= cnt; j += 4) {
    float v0[8], v1[8], v2[8], v3[8];
    load_vec<DT, 8>(rows.p[sel[j]], x, v0);
    load_vec<DT, 8>(rows.p[sel[j + 1]], x, v1);
    load_vec<DT, 8>(rows.p[sel[j + 2]], x, v2);
    load_vec<DT, 8>(rows.p[sel[j + 3]], x, v3);
    const float w0 = wsel[j], w1 = wsel[j + 1], w2 = wsel[j + 2], w3 = wsel[j + 3];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] += w0 * v0[c] + w1 * v1[c] + w2 * v2[c] + w3 * v3[c];
  }
  for (; j < cnt; ++j) {
    float v[8];
    load_vec<DT, 8>(rows.p[sel[j]], x, v);
    const float w = wsel[j];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] += w * v[c];
  }
}

template <int DT>
__device__ __forceinline__ float gather_weighted_one(const RowTable& rows, const int* sel, const float* wsel,
                                                     int cnt, int64_t x) {
  float a = 0.f;
  for (int j = 0; j < cnt; ++j) a += wsel[j] * load_one<DT>(rows.p[sel[j]], x);
  return a;
}

__device__ int compact_selection(const float* __restrict__ weights, int n, int* sel, float* wsel) {
  __shared__ int cnt;
  if (threadIdx.x == 0) {
    int c = 0;
    for (int j = 0; j < n; ++j) {
      const float w = weights[j];
      if (w != 0.f) { sel[c] = j; wsel[c] = w; ++c; }
    }
    cnt = c;
  }
  __syncthreads();
  return cnt;
}

template <int DT>
__global__ __launch_bounds__(256) void k_combine(RowTable rows, int n, int64_t d,
                                                 const float* __restrict__ weights, void* out, int out_dt) {
  __shared__ int sel[kMaxRows];
  __shared__ float wsel[kMaxRows];
  const int cnt = compact_selection(weights, n, sel, wsel);
  const int64_t dv = d & ~static_cast<int64_t>(7);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * 8;
  for (int64_t x = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 8; x < dv; x += stride) {
    float acc[8];
    gather_weighted<DT>(rows, sel, wsel, cnt, x, acc);
    store_vec<8>(out, out_dt, x, acc);
  }
  if (blockIdx.x == 0)
    for (int64_t x = dv + threadIdx.x; x < d; x += blockDim.x)
      store_one(out, out_dt, x, gather_weighted_one<DT>(rows, sel, wsel, cnt, x));
}

// ---------------------------------------------------------------------------
// Colluding attacks on the exchanged rows (lie / empire, runtime/attacks.py semantics): rows 0..P-1
// of the table are the colluders' honest estimates, rows P..P+T-1 the Byzantine rows, which still hold
// their own honest gradient g_t. With E_t = {g_t} + the P estimates (k = P + 1 rows):
//   lie    g_t <- mean(E_t) + z * std_unbiased(E_t)
//   empire g_t <- -eps * mean(E_t)
// One pass reads the estimates once for every target (per coordinate: their sum, then the sum of
// squared deviations from their mean in a second pass over the same L2-resident lines), so the
// estimates are never materialised in fp32 (the ATen form stacked k fp32 copies of every row).
// var(E_t) = (Q + P (m_p - m_t)^2 + (g_t - m_t)^2) / (k - 1), Q = Σ_p (v_p - m_p)^2.
template <int DT>
__global__ __launch_bounds__(256) void k_collude(RowTable rows, int P, int T, int64_t d, int empire, float param) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * 8;
  const float k = static_cast<float>(P + 1);
  for (int64_t x = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 8; x < d; x += stride) {
    const int nv = d - x >= 8 ? 8 : static_cast<int>(d - x);
    float s1[8], q[8], mp[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { s1[c] = 0.f; q[c] = 0.f; }
    for (int j = 0; j < P; ++j) {
      float v[8];
      if (nv == 8) load_vec<DT, 8>(rows.p[j], x, v);
      else
        for (int c = 0; c < 8; ++c) v[c] = c < nv ? load_one<DT>(rows.p[j], x + c) : 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) s1[c] += v[c];
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) mp[c] = P > 0 ? s1[c] / static_cast<float>(P) : 0.f;
    if (!empire) {
      for (int j = 0; j < P; ++j) {
        float v[8];
        if (nv == 8) load_vec<DT, 8>(rows.p[j], x, v);
        else
          for (int c = 0; c < 8; ++c) v[c] = c < nv ? load_one<DT>(rows.p[j], x + c) : 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) { const float e = v[c] - mp[c]; q[c] = fmaf(e, e, q[c]); }
      }
    }
    for (int t = 0; t < T; ++t) {
      void* row = const_cast<void*>(rows.p[P + t]);
      float g[8], o[8];
      if (nv == 8) load_vec<DT, 8>(row, x, g);
      else
        for (int c = 0; c < 8; ++c) g[c] = c < nv ? load_one<DT>(row, x + c) : 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float m = (s1[c] + g[c]) / k;
        if (empire) {
          o[c] = -param * m;
        } else {
          const float dm = mp[c] - m, dg = g[c] - m;
          const float var = P > 0 ? (q[c] + static_cast<float>(P) * dm * dm + dg * dg) / (k - 1.f) : 0.f;
          o[c] = m + param * sqrtf(var > 0.f ? var : 0.f);
        }
      }
      if (nv == 8) store_vec<8>(row, DT, x, o);
      else
        for (int c = 0; c < nv; ++c) store_one(row, DT, x + c, o[c]);
    }
  }
}

template <int DT> struct Collude {
  static void run(const RowTable& rows, int P, int T, int64_t d, int empire, float param, hipStream_t s) {
    int64_t blocks = (d / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((k_collude<DT>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, rows, P, T, d, empire,
                       param);
  }
};

__device__ __forceinline__ float sgd_apply(float g, float& p, float& buf, const SgdArgs& a) {
  if (a.weight_decay != 0.f) g += a.weight_decay * p;
  if (a.momentum != 0.f) {
    buf = a.first_step ? g : a.momentum * buf + (1.f - a.dampening) * g;
    g = a.nesterov ? g + a.momentum * buf : buf;
  }
  p -= a.lr * g;
  return g;
}

template <int DT>
__global__ __launch_bounds__(256) void k_combine_sgd(RowTable rows, int n, int64_t d,
                                                     const float* __restrict__ weights, float* __restrict__ param,
                                                     float* __restrict__ mom, float* __restrict__ grad_out,
                                                     void* __restrict__ shadow, int shadow_dt, SgdArgs args) {
  __shared__ int sel[kMaxRows];
  __shared__ float wsel[kMaxRows];
  const int cnt = compact_selection(weights, n, sel, wsel);
  const int64_t dv = d & ~static_cast<int64_t>(7);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * 8;
  for (int64_t x = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 8; x < dv; x += stride) {
    float acc[8];
    gather_weighted<DT>(rows, sel, wsel, cnt, x, acc);
    if (grad_out) store_vec<8>(grad_out, kF32, x, acc);
    float4 p0 = *reinterpret_cast<float4*>(param + x), p1 = *reinterpret_cast<float4*>(param + x + 4);
    float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    float bv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (args.momentum != 0.f && !args.first_step) {
      float4 b0 = *reinterpret_cast<float4*>(mom + x), b1 = *reinterpret_cast<float4*>(mom + x + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) sgd_apply(acc[c], pv[c], bv[c], args);
    *reinterpret_cast<float4*>(param + x) = make_float4(pv[0], pv[1], pv[2], pv[3]);
    *reinterpret_cast<float4*>(param + x + 4) = make_float4(pv[4], pv[5], pv[6], pv[7]);
    if (shadow) store_vec<8>(shadow, shadow_dt, x, pv);
    if (args.momentum != 0.f) {
      *reinterpret_cast<float4*>(mom + x) = make_float4(bv[0], bv[1], bv[2], bv[3]);
      *reinterpret_cast<float4*>(mom + x + 4) = make_float4(bv[4], bv[5], bv[6], bv[7]);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t x = dv + threadIdx.x; x < d; x += blockDim.x) {
      const float g = gather_weighted_one<DT>(rows, sel, wsel, cnt, x);
      if (grad_out) grad_out[x] = g;
      float p = param[x];
      float b = (args.momentum != 0.f && !args.first_step) ? mom[x] : 0.f;
      sgd_apply(g, p, b, args);
      param[x] = p;
      if (shadow) store_one(shadow, shadow_dt, x, p);
      if (args.momentum != 0.f) mom[x] = b;
    }
  }
}

// ---------------------------------------------------------------------------
// Aksel: partial squared distances to a centre, NP row accumulators per lane.

template <int DT, int NP>
__global__ __launch_bounds__(256) void k_sqdist_partial(RowTable rows, int n, int64_t d,
                                                        const float* __restrict__ center, int64_t chunk,
                                                        float* __restrict__ slabs) {
  __shared__ float red[4][NP];
  float acc[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) acc[j] = 0.f;
  const int64_t start = static_cast<int64_t>(blockIdx.x) * chunk;
  int64_t end = start + chunk;
  if (end > d) end = d;
  const int64_t dv_end = start + ((end - start) / 4) * 4;  // chunk is a multiple of 4 except at d
  for (int64_t x = start + threadIdx.x * 4; x < dv_end; x += blockDim.x * 4) {
    const float4 cc = *reinterpret_cast<const float4*>(center + x);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if (j < n) {
        float g[4];
        load_vec<DT, 4>(rows.p[j], x, g);
        const float a = g[0] - cc.x, b = g[1] - cc.y, c = g[2] - cc.z, e = g[3] - cc.w;
        acc[j] += a * a + b * b + c * c + e * e;
      }
    }
  }
  for (int64_t x = dv_end + threadIdx.x; x < end; x += blockDim.x) {
    const float cc = center[x];
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if (j < n) { const float a = load_one<DT>(rows.p[j], x) - cc; acc[j] += a * a; }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const float s = wave_sum(acc[j]);
    if (lane == 0) red[wave][j] = s;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += blockDim.x)
    slabs[static_cast<int64_t>(blockIdx.x) * n + j] = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
}

__global__ __launch_bounds__(128) void k_aksel_select(const float* __restrict__ slabs, int grid, int n, int c,
                                                      float* __restrict__ weights, float* __restrict__ dists) {
  __shared__ float S[kMaxRows];
  const int i = threadIdx.x;
  if (i < n) {
    float s = 0.f;
    for (int g = 0; g < grid; ++g) s += slabs[static_cast<int64_t>(g) * n + i];
    if (!isfinite(s)) s = kInf;
    S[i] = s;
  }
  __syncthreads();
  if (i < n) {
    const int r = score_rank(S, n, i);
    weights[i] = r < c ? 1.f / static_cast<float>(c) : 0.f;
    dists[i] = S[i];
  }
}

int np_for(int k) { return k <= 8 ? 8 : (k <= 16 ? 16 : (k <= 32 ? 32 : (k <= 64 ? 64 : 128))); }

int combine_grid(int64_t d) {
  int64_t g = (d / 8 + 255) / 256;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return static_cast<int>(g);
}

}  // namespace

// ---------------------------------------------------------------------------
// Combine

namespace {
template <int DT> struct Combine {
  static void run(const RowTable& rows, int n, int64_t d, const float* w, void* out, int out_dt, hipStream_t s) {
    hipLaunchKernelGGL(k_combine<DT>, dim3(combine_grid(d)), dim3(256), 0, s, rows, n, d, w, out, out_dt);
  }
};
template <int DT> struct CombineSgd {
  static void run(const RowTable& rows, int n, int64_t d, const float* w, float* param, float* mom,
                  float* gout, void* shadow, int shadow_dt, SgdArgs a, hipStream_t s) {
    hipLaunchKernelGGL(k_combine_sgd<DT>, dim3(combine_grid(d)), dim3(256), 0, s, rows, n, d, w, param, mom, gout,
                       shadow, shadow_dt, a);
  }
};
}  // namespace

void combine(const RowTable& rows, int n, int64_t d, int dt, const float* weights, void* out, int out_dt,
             hipStream_t stream) {
  by_dtype<Combine>(dt, rows, n, d, weights, out, out_dt, stream);
}

void combine_sgd(const RowTable& rows, int n, int64_t d, int dt, const float* weights, float* param,
                 float* momentum_buf, float* grad_out, void* shadow, int shadow_dt, SgdArgs args,
                 hipStream_t stream) {
  by_dtype<CombineSgd>(dt, rows, n, d, weights, param, momentum_buf, grad_out, shadow, shadow_dt, args, stream);
}

// ---------------------------------------------------------------------------
// Aksel

int sqdist_grid(int64_t d) {
  int64_t g = d / (256 * 4 * 8);
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return static_cast<int>(g);
}

namespace {
template <int DT, int NP>
void launch_sqdist(const RowTable& rows, int n, int64_t d, const float* c, float* slabs, int grid, hipStream_t s) {
  int64_t chunk = (d + grid - 1) / grid;
  chunk = ((chunk + 3) / 4) * 4;
  hipLaunchKernelGGL((k_sqdist_partial<DT, NP>), dim3(grid), dim3(256), 0, s, rows, n, d, c, chunk, slabs);
}
template <int DT> struct Sqdist {
  static void run(const RowTable& rows, int n, int64_t d, const float* c, float* slabs, int grid, hipStream_t s) {
    switch (np_for(n)) {
      case 8: launch_sqdist<DT, 8>(rows, n, d, c, slabs, grid, s); break;
      case 16: launch_sqdist<DT, 16>(rows, n, d, c, slabs, grid, s); break;
      case 32: launch_sqdist<DT, 32>(rows, n, d, c, slabs, grid, s); break;
      case 64: launch_sqdist<DT, 64>(rows, n, d, c, slabs, grid, s); break;
      default: launch_sqdist<DT, 128>(rows, n, d, c, slabs, grid, s); break;
    }
  }
};
}  // namespace

void sqdist_partial(const RowTable& rows, int n, int64_t d, int dt, const float* center, float* slabs, int grid,
                    hipStream_t stream) {
  by_dtype<Sqdist>(dt, rows, n, d, center, slabs, grid, stream);
}

void collude(const RowTable& rows, int P, int T, int64_t d, int dt, bool empire, float param, hipStream_t stream) {
  if (T <= 0 || d <= 0) return;
  by_dtype<Collude>(dt, rows, P, T, d, empire ? 1 : 0, param, stream);
}

void aksel_select(const float* slabs, int grid, int n, int c, float* weights, float* dists, hipStream_t stream) {
  hipLaunchKernelGGL(k_aksel_select, dim3(1), dim3(128), 0, stream, slabs, grid, n, c, weights, dists);
}

}  // namespace gpu
}  // namespace garfield
