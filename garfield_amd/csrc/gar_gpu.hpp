// Host-side launchers of the CDNA4 (gfx950) robust-aggregation kernels.
//
// Every launcher is asynchronous on the given stream, allocates nothing and
// never synchronises, so a caller may capture it into a hipGraph
// (contrast: the reference's cudaMalloc + cudaMemcpy + cudaStreamSynchronize
// inside every call, pytorch_impl/libs/native/py_krum/krum.cu:77-154).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "gar_common.hpp"

namespace garfield {
namespace gpu {

// ---- Gram matrix (pairwise distances as G·Gᵀ on MFMA) ----------------------
int gram_nb(int n);                          // 16-row blocks: 1, 2, 4 or 8
int gram_padded(int n);                      // 16 * gram_nb(n)
int gram_grid(int64_t d, int dt, int n);     // split-K workgroups
int64_t gram_slab_floats(int n);             // floats per split-K slab
constexpr int kGramReduceGroups = 16;        // stage-1 partials of the slab reduction
// slabs: [grid + kGramReduceGroups][slab_floats] workspace; gram: [np][np] fp32 output
void gram(const RowTable& rows, int n, int64_t d, int dt, float* slabs, int grid,
          float* gram, hipStream_t stream);

// ---- Selection (one workgroup, on device, no host round-trip) --------------
// weights[n] (fp32), order[n] (gradient ids by increasing score), scores[n]
// batch > 1: `batch` independent problems, gram [batch][np][np] -> weights/order/scores [batch][n]
void krum_select(const float* gram, int np, int n, int f, int m, float* weights,
                 int* order, float* scores, hipStream_t stream, int batch = 1);

// W[t][n]: row k = uniform weights of the (m-k) best-scoring gradients at step k
// batch > 1: gram [batch][np][np] -> W [batch][t][n]
void bulyan_select(const float* gram, int np, int n, int f, int m, int t, float* W,
                   hipStream_t stream, int batch = 1);
// best: one uint64 (initialised here), weights[n]
void brute_select(const float* gram, int np, int n, int f, unsigned long long* best,
                  float* weights, hipStream_t stream);

// ---- Weighted combine  out = Σ_j w_j g_j  (optionally fused SGD update) -----
void combine(const RowTable& rows, int n, int64_t d, int dt, const float* weights,
             void* out, int out_dt, hipStream_t stream);

struct SgdArgs {
  float lr;
  float momentum;
  float dampening;
  float weight_decay;
  int nesterov;
  int first_step;  // momentum buffer initialised to the gradient (torch.optim.SGD)
};
// shadow (optional): low-precision copy of the updated parameters (bf16/f16
// working weights of the forward/backward), written in the same pass.
void combine_sgd(const RowTable& rows, int n, int64_t d, int dt, const float* weights,
                 float* param, float* momentum_buf, float* grad_out, void* shadow, int shadow_dt,
                 SgdArgs args, hipStream_t stream);

// ---- Layer-wise GAR: the rule on every parameter segment of the flat rows ----
// jobs: [njobs][3] int64 (start, end, segment) coordinate ranges, each inside one segment, in
// segment order; seg_lo: [L + 1] int32, the first job of each segment (seg_lo[L] = njobs).
// lw_gram: gram [L][np][np] = per-segment G·Gᵀ (slabs: [njobs][gram_slab_floats(n)] workspace).
void lw_gram(const RowTable& rows, int n, int dt, const int64_t* jobs, int njobs, const int* seg_lo, int L,
             float* slabs, float* gram, hipStream_t stream);
// lw_bulyan_tail: out[x] (fp32) for every coordinate x of the jobs (LOCAL coordinates) = Bulyan's
// tail with x's segment's W[s] [t][n]: the averaged median (beta) of the t selection means
void lw_bulyan_tail(const RowTable& rows, int n, int dt, const int64_t* jobs, int njobs, const float* W, int t,
                    int beta, float* out, hipStream_t stream);
// lw_combine_sgd: per coordinate of segment s, g = Σ_j weights[s][j] row_j, then the SGD update
// of param / momentum (and the shadow copy), as combine_sgd does with one weight vector.
// jobs in LOCAL coordinates of rows / param / momentum / shadow, base = the global coordinate of
// local 0 (a sharded bucket's owned range); seg_off: [L + 1] int64 global segment offsets.
void lw_combine_sgd(const RowTable& rows, int n, int dt, const int64_t* jobs, int njobs, const float* weights,
                    float* param, float* momentum_buf, void* shadow, int shadow_dt, SgdArgs args,
                    const int64_t* seg_off, int64_t base, hipStream_t stream);

// ---- Coordinate-wise rules (median, trimmed mean, MeaMed, ...) -------------
// W/t are only read for kBulyanTail; seed/threshold only for kCondense.
void coordwise(const RowTable& rows, int n, int64_t d, int dt, int mode, int f, int beta,
               const float* W, int t, uint64_t seed, uint64_t threshold, void* out,
               int out_dt, hipStream_t stream);
int coordwise_max_rows();

// ---- Large gradient sets (kMaxRows < n <= kLargeRows), one [n, ld] matrix (gar_large.hip) ----
// out[j] = Σ_i w[i] x[i, j] (out in x's dtype); mode 0 median, 1 trimmed-mean(f), 2 averaged-median(beta).
void large_combine(const void* x, int dt, int n, int64_t d, int64_t ld, const float* w, void* out, hipStream_t stream);
// fp32 Gram [n, n] of the [n, d] rows x (row stride ld) on MFMA: split-K 64 x 64 tiles into
// large_gram_slab_floats(n, d, dt) floats of slabs, then a fixed-order reduction (n <= kLargeRows)
int64_t large_gram_slab_floats(int n, int64_t d, int dt);
void large_gram(const void* x, int dt, int n, int64_t d, int64_t ld, float* slabs, float* gram, hipStream_t stream);
// V [t, d] (row stride ldv) = W [t, n] fp32 · x [n, d] (row stride ld) on fp32 MFMA
void large_wx(const float* W, int t, int n, const void* x, int dt, int64_t d, int64_t ld, float* V, int64_t ldv,
              hipStream_t stream);
// Multi-Krum (rounds 1, W [1][n] = 1/m on the m best scores) / Bulyan (rounds t, shrink: W [t][n] with
// 1/max(m - k, 1) in round k) selection from an fp32 Gram [n][ld] (n <= kLargeRows, 1 <= n - f - 2);
// thr_val / thr_idx / nearsum: [n] workspaces.
void large_select(const float* gram, int64_t ld, int n, int f, int m, int rounds, bool shrink, double* thr_val,
                  int* thr_idx, double* nearsum, float* W, hipStream_t stream);
void large_coord(const void* x, int dt, int n, int64_t d, int64_t ld, int mode, int f, int beta, void* out,
                 hipStream_t stream);

// ---- Aksel: squared distances of every gradient to a centre vector ---------
int sqdist_grid(int64_t d);
void sqdist_partial(const RowTable& rows, int n, int64_t d, int dt, const float* center,
                    float* slabs, int grid, hipStream_t stream);
// Colluding attacks (runtime/attacks.py lie / empire) in place on the exchanged rows: rows 0..P-1 the
// colluders' estimates, rows P..P+T-1 the Byzantine rows (holding their honest gradient); param = z
// (lie) or eps (empire)
void collude(const RowTable& rows, int P, int T, int64_t d, int dt, bool empire, float param, hipStream_t stream);
void aksel_select(const float* slabs, int grid, int n, int c, float* weights, float* dists,
                  hipStream_t stream);

// ---- Split-K partial sums -> exchange rows (gar_flatten.hip) -----------------
// out[g * ostride + r * opitch + c] = Σ_s part[s * ss + g * gs + r * ipitch + c] (cast to odt),
// r < R, c < Cc, g < G.
void split_reduce(const float* part, int S, int G, int64_t R, int64_t Cc, int64_t ipitch, int64_t opitch, int64_t ss,
                  int64_t gs, void* out, int odt, int64_t ostride, hipStream_t stream);

// The same for many (part, out) pairs in one launch (up to kMaxSplitJobs per launch).
struct SplitJob {
  const float* part;
  void* out;
  int64_t R, Cc, ipitch, opitch, ss, gs, ostride;
  int S, G, odt, vec;
};
constexpr int kMaxSplitJobs = 32;   // kernarg budget: 32 x 80 B
void split_reduce_multi(const SplitJob* jobs, int count, hipStream_t stream);

// ---- Multi-tensor flatten + cast (per-parameter grads -> exchange row) -----
constexpr int kMaxFlatTensors = 96;  // tensors per launch (kernarg budget); more => several launches
int flatten_cast(const void* const* srcs, const int* src_dts, const int64_t* numels, const int64_t* offsets,
                 int count, void* dst, int out_dt, hipStream_t stream);

// ---- Stream signal: 1-thread kernel storing `value` (system-scope release) ----
void signal_set(void* p, uint64_t value, hipStream_t stream);
// host stub of the signal kernel (identifies its nodes in a captured graph)
const void* signal_kernel();
// counter signals: k_signal_add (+1, release) and a bounded device-side wait (>= target)
const void* signal_add_kernel();
void signal_add(void* p, hipStream_t stream);
void wait_geq(const void* p, uint64_t target, uint64_t timeout_us, void* err, hipStream_t stream);

}  // namespace gpu
}  // namespace garfield
