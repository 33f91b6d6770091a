// Fused per-worker cross-entropy for the grouped step (gfx950).
//
// The grouped pass (garfield_amd/parallel/grouped.py) needs each logical worker's
// mean loss, exactly what the reference computes per worker process
// (pytorch_impl/libs/garfieldpp/worker.py:77-96: loss_fn(output, target) then
// backward). Through ATen that is a bf16->fp32 cast, log-softmax, NLL, a per-worker
// mean and, in the backward, fills, NLL/log-softmax backward and casts: ~12 launches
// for a [2000, 10] matrix. Here the forward is ONE launch (one workgroup per worker,
// one row per thread) that also leaves d(loss_g)/d(logits) behind, and the backward
// is one elementwise scale by the upstream per-worker gradient.
#include "gar_device.hpp"
#include "loss_gpu.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kXentThreads = 256;

template <int DT>
__device__ __forceinline__ float ld(const void* p, int64_t i) {
  if constexpr (DT == kF32) return static_cast<const float*>(p)[i];
  else return bf16_to_f(static_cast<const uint16_t*>(p)[i]);
}

template <int DT>
__device__ __forceinline__ void st(void* p, int64_t i, float v) {
  if constexpr (DT == kF32) static_cast<float*>(p)[i] = v;
  else static_cast<uint16_t*>(p)[i] = f_to_bf16(v);
}

template <int DT>
__global__ __launch_bounds__(kXentThreads) void k_xent_fwd(const void* __restrict__ logits,
                                                           const int64_t* __restrict__ labels, int64_t rows, int nc,
                                                           float* __restrict__ loss, void* __restrict__ dl) {
  __shared__ float wsum[kXentThreads / 64];
  const int g = blockIdx.x;
  const float inv = 1.f / static_cast<float>(rows);
  float acc = 0.f;
  for (int64_t t = threadIdx.x; t < rows; t += kXentThreads) {
    const int64_t r = static_cast<int64_t>(g) * rows + t;
    const int64_t o = r * nc;
    const int64_t lab = labels[r];
    const bool ok = lab >= 0 && lab < nc;
    float z[kXentMaxClasses];
    float m = -INFINITY, zl = 0.f;
#pragma unroll
    for (int c = 0; c < kXentMaxClasses; ++c) {
      if (c < nc) {
        z[c] = ld<DT>(logits, o + c);
        m = fmaxf(m, z[c]);
        if (c == lab) zl = z[c];
      }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kXentMaxClasses; ++c) {
      if (c < nc) {
        z[c] = __expf(z[c] - m);
        s += z[c];
      }
    }
    const float is = 1.f / s;
#pragma unroll
    for (int c = 0; c < kXentMaxClasses; ++c) {
      if (c < nc) {
        const bool hit = ok && c == lab;
        st<DT>(dl, o + c, (z[c] * is - (hit ? 1.f : 0.f)) * inv);
      }
    }
    // logsumexp(z) - z_label = m + log(s) - z_label
    acc += ok ? (m + __logf(s) - zl) : __int_as_float(0x7fc00000);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kXentThreads / 64; ++w) t += wsum[w];
    loss[g] = t * inv;
  }
}

template <int DT>
__global__ __launch_bounds__(kXentThreads) void k_xent_bwd(const void* __restrict__ dl,
                                                           const float* __restrict__ go, int64_t rows, int nc,
                                                           int64_t total, void* __restrict__ dx) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kXentThreads + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * kXentThreads) {
    const int64_t g = i / (rows * nc);
    st<DT>(dx, i, ld<DT>(dl, i) * go[g]);
  }
}

// nc > kXentMaxClasses (an ImageNet head): one wave per row, the lanes over the classes in three
// passes over the row's (L1 / L2-resident) logits: max, Σ exp, then d(loss)/d(logits); the row's loss
// goes to rowloss and k_xent_rowsum reduces each worker's rows in a fixed order (deterministic)
template <int DT>
__global__ __launch_bounds__(kXentThreads) void k_xent_rows_wide(const void* __restrict__ logits,
                                                                 const int64_t* __restrict__ labels, int64_t total,
                                                                 int64_t rows, int nc, float* __restrict__ rowloss,
                                                                 void* __restrict__ dl) {
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * (kXentThreads / 64) + (threadIdx.x >> 6);
  if (r >= total) return;
  const int64_t o = r * nc;
  const int64_t lab = labels[r];
  const bool ok = lab >= 0 && lab < nc;
  const float inv = 1.f / static_cast<float>(rows);
  float m = -INFINITY;
  for (int c = lane; c < nc; c += 64) m = fmaxf(m, ld<DT>(logits, o + c));
#pragma unroll
  for (int sft = 32; sft >= 1; sft >>= 1) m = fmaxf(m, __shfl_xor(m, sft));
  float sum = 0.f;
  for (int c = lane; c < nc; c += 64) sum += __expf(ld<DT>(logits, o + c) - m);
  sum = wave_sum(sum);
  const float is = 1.f / sum;
  for (int c = lane; c < nc; c += 64) {
    const float pr = __expf(ld<DT>(logits, o + c) - m) * is;
    st<DT>(dl, o + c, (pr - ((ok && c == lab) ? 1.f : 0.f)) * inv);
  }
  if (lane == 0) rowloss[r] = ok ? (m + __logf(sum) - ld<DT>(logits, o + lab)) : __int_as_float(0x7fc00000);
}

// loss[g] = mean of worker g's row losses (one workgroup per worker)
__global__ __launch_bounds__(kXentThreads) void k_xent_rowsum(const float* __restrict__ rowloss, int64_t rows,
                                                              float* __restrict__ loss) {
  __shared__ float wsum[kXentThreads / 64];
  const int g = blockIdx.x;
  float acc = 0.f;
  for (int64_t t = threadIdx.x; t < rows; t += kXentThreads) acc += rowloss[static_cast<int64_t>(g) * rows + t];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kXentThreads / 64; ++w) t += wsum[w];
    loss[g] = t / static_cast<float>(rows);
  }
}

// out[0] = mean of n fp32 values (the step's reported loss over the workers), fixed order
__global__ __launch_bounds__(kXentThreads) void k_mean_f32(const float* __restrict__ x, int64_t n,
                                                           float* __restrict__ out) {
  __shared__ float wsum[kXentThreads / 64];
  float acc = 0.f;
  for (int64_t t = threadIdx.x; t < n; t += kXentThreads) acc += x[t];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kXentThreads / 64; ++w) t += wsum[w];
    out[0] = t / static_cast<float>(n);
  }
}

}  // namespace

void mean_f32(const float* x, int64_t n, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_mean_f32, dim3(1), dim3(kXentThreads), 0, stream, x, n, out);
}

void xent_forward(const void* logits, int dt, const int64_t* labels, int64_t rows, int groups, int nc,
                  float* loss, void* dlogits, hipStream_t stream, float* rowloss) {
  if (nc > kXentMaxClasses) {
    const int64_t total = rows * groups;
    const dim3 grid(static_cast<unsigned>((total + kXentThreads / 64 - 1) / (kXentThreads / 64)));
    if (dt == kF32)
      hipLaunchKernelGGL(k_xent_rows_wide<kF32>, grid, dim3(kXentThreads), 0, stream, logits, labels, total, rows, nc,
                         rowloss, dlogits);
    else
      hipLaunchKernelGGL(k_xent_rows_wide<kBF16>, grid, dim3(kXentThreads), 0, stream, logits, labels, total, rows, nc,
                         rowloss, dlogits);
    hipLaunchKernelGGL(k_xent_rowsum, dim3(groups), dim3(kXentThreads), 0, stream, rowloss, rows, loss);
    return;
  }
  if (dt == kF32)
    hipLaunchKernelGGL(k_xent_fwd<kF32>, dim3(groups), dim3(kXentThreads), 0, stream, logits, labels, rows, nc, loss,
                       dlogits);
  else
    hipLaunchKernelGGL(k_xent_fwd<kBF16>, dim3(groups), dim3(kXentThreads), 0, stream, logits, labels, rows, nc, loss,
                       dlogits);
}

void xent_backward(const void* dlogits, int dt, const float* grad_loss, int64_t rows, int groups, int nc, void* dx,
                   hipStream_t stream) {
  const int64_t total = rows * groups * nc;
  int64_t blocks = (total + kXentThreads - 1) / kXentThreads;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  if (dt == kF32)
    hipLaunchKernelGGL(k_xent_bwd<kF32>, dim3(static_cast<unsigned>(blocks)), dim3(kXentThreads), 0, stream, dlogits,
                       grad_loss, rows, nc, total, dx);
  else
    hipLaunchKernelGGL(k_xent_bwd<kBF16>, dim3(static_cast<unsigned>(blocks)), dim3(kXentThreads), 0, stream, dlogits,
                       grad_loss, rows, nc, total, dx);
}

}  // namespace gpu
}  // namespace garfield
