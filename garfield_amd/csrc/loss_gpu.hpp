// Host-side launchers of the fused per-worker cross-entropy (loss_xent.hip).
// Asynchronous on the given stream, no allocation: HIP-graph capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace garfield {
namespace gpu {

constexpr int kXentMaxClasses = 64;

// logits: [groups * rows, nc] (dt: kBF16 or kF32), labels: [groups * rows] int64.
// loss[g] = mean over worker g's rows of (logsumexp(z) - z[label]);
// dlogits (same dtype as logits) = (softmax(z) - onehot(label)) / rows.
// nc > kXentMaxClasses: the wide form (one wave per row), which needs rowloss: [groups * rows] fp32 scratch.
void xent_forward(const void* logits, int dt, const int64_t* labels, int64_t rows, int groups, int nc,
                  float* loss, void* dlogits, hipStream_t stream, float* rowloss = nullptr);

// out[0] = mean of x[0 .. n) (fp32, fixed summation order)
void mean_f32(const float* x, int64_t n, float* out, hipStream_t stream);

// dx[r, :] = dlogits[r, :] * grad_loss[r / rows]
void xent_backward(const void* dlogits, int dt, const float* grad_loss, int64_t rows, int groups, int nc, void* dx,
                   hipStream_t stream);

}  // namespace gpu
}  // namespace garfield
