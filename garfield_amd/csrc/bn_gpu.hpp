// Host-side launchers of the worker-grouped NHWC kernels: BatchNorm(+residual)
// (+ReLU) (bn_nhwc.hip) and the im2col gather of the per-worker weight-gradient
// GEMMs. Asynchronous on the given stream, no allocation, no synchronisation:
// HIP-graph capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace garfield {
namespace gpu {

constexpr int kBnMaxChunks = 64;  // row chunks per (group, channel block) in the partial-sum pass

// Floats of the partial-sum workspace for `groups` groups of `rg` rows and C channels.
int64_t bn_part_floats(int64_t rg, int groups, int C);

// x, res, y: [groups * rg, C] bf16 (NHWC rows). gamma/beta/run_*: [C] fp32 (nullable).
// mean, istd, scale, shift: [groups, C] fp32 outputs (saved for the backward).
// Running-statistics replay of one or more layers (the k sequential updates of k workers).
struct RunJob {
  const float* mean;
  const float* istd;
  float* run_mean;
  float* run_var;
  int64_t rg;
  int C;
  int groups;
  float eps;
  float momentum;
};
constexpr int kRunJobs = 48;
struct RunJobs {
  RunJob j[kRunJobs];
  int n;
};
// Backward of a projection block's last BatchNorm (a) and its folded shortcut BatchNorm (b), which share
// dz = dy · [mask bit] (mask nullptr: dz = dy): one statistics pass and one apply pass read dy / mask once.
// (the single-kernel small path: one workgroup per (worker, channel group) for both).
void bn_backward_dual(const void* xa, const void* xb, const void* dy, const uint8_t* mask, int64_t rg, int groups,
                      int C, const float* gamma_a, const float* gamma_b, const float* mean_a, const float* istd_a,
                      const float* mean_b, const float* istd_b, float* part_a, float* part_b, float* coef_a,
                      float* coef_b, void* dxa, void* dxb, void* grow, int grow_dt, int64_t row_stride,
                      int64_t og_a, int64_t ob_a, int64_t og_b, int64_t ob_b, hipStream_t stream, int dt);
void bn_running_update(const RunJobs& jobs, hipStream_t stream);
// True when a layer of rg rows per worker takes the single-kernel small-layer path.
bool bn_small(int64_t rg);
// channels per workgroup of the single-kernel small-layer BatchNorm: 8, 16 or 32 forced
// (GARFIELD_BN_SMALL_CH), 0 automatic (small_ch_for)
int bn_small_ch();
void set_bn_small_ch(int ch);
int small_ch_for(int C, int groups);

// defer_running (small-layer path, and any layer with y null): skip the running-statistics replay; the
// caller batches it with bn_running_update. y null: statistics and scale / shift only, no apply pass (the
// consumer applies the BatchNorm + ReLU while staging its input: gemm_nt / iwgrad prologues).
// dt: the activations' dtype (kBF16, or kF32 for the reference-precision step)
void bn_forward(const void* x, const void* res, int64_t rg, int groups, int C, const float* gamma,
                const float* beta, float eps, float momentum, float* run_mean, float* run_var, float* part,
                float* mean, float* istd, float* scale, float* shift, void* y, bool relu, uint8_t* mask,
                bool defer_running, hipStream_t stream, const float* tile_stats = nullptr, int64_t tile_m = 0,
                int tile_e = 1, int dt = 1, const float* res_scale = nullptr, const float* res_shift = nullptr);
// res_scale / res_shift ([groups][C] fp32): res is a PRE-BatchNorm activation, added as res * res_scale + res_shift
// (its own BatchNorm, a projection shortcut's, folded into this one's apply pass)

// Fresh batches (data_aug.hip): out[r] (bf16 channels_last [R, C, H, W]) = normalise(random crop
// (pad) + random horizontal flip of uint8 NHWC image src[idx[r]]); the crop/flip of row r is a hash
// of (seed, step, r). C <= 4.
struct AugNorm {
  float mean[4];
  float inv_std[4];
};
// idx null: row r samples image hash(seed, step, r) % nsrc; lab_out (nullable) receives lab_src[image].
void augment_gather(const uint8_t* src, int64_t nsrc, const int64_t* idx, const int64_t* lab_src, int64_t* lab_out,
                    int64_t R, int H, int W, int C, int pad, bool flip,
                    uint64_t seed, uint64_t step, const AugNorm& nrm, void* out, hipStream_t stream, int out_dt = 1);

// ResNet stem (stem_nhwc.hip): the convolution of 3-channel NHWC images into 64 channels on MFMA,
// without a patch matrix; kind kStem7x7: 7x7 / stride 2 / padding 3 (K = 147 taps x channels, padded
// KP = 160), kStem3x3: the CIFAR ResNet-18 3x3 / stride 1 / padding 1 (K = 27, KP = 32).
// split: the fp32 form — x / y fp32, w = the weight's three bf16 pieces [3][64][KP].
constexpr int kStem7x7 = 0, kStem3x3 = 1;
int stem_k(int kind);
int stem_kp(int kind);
bool stem_supported(int H, int W, int kind = kStem7x7);
// w: the zero-padded [64][KP] matrix (split: its three pieces), or (wpitch = K, bf16 only) the
// channels_last [64][KH][KW][3] weight itself
void stem_fwd(const void* x, const uint16_t* w, bool split, int N, int H, int W, void* y, hipStream_t stream,
              int wpitch = 160, int kind = kStem7x7, uint16_t* scratch = nullptr, float* stats = nullptr);
// bf16 elements of the scratch stem_fwd takes for its channel-padded weight (0: none used)
int stem_fwd_scratch(int kind);
// statistics tiles (of 256 output pixels, gemm_nt.hip's layout, E = 1) the bf16 stem forward writes for
// the consuming BatchNorm, 0 when the geometry has none (tiles must hold whole images' pixels)
int64_t stem_fwd_stat_tiles(int N, int H, int W, int kind);
// per-worker weight gradients: part fp32 [slices][groups][64][K] (sum over slices = dW of the worker);
// split: x / dy fp32
void stem_wgrad(const void* x, const void* dy, int N, int H, int W, int groups, int slices, float* part, bool split,
                hipStream_t stream, int kind = kStem7x7);

// Row-major NT GEMM on MFMA (gemm_nt.hip): C[M, N] = A[M, K] · B[N, K]ᵀ (+ add), bf16; K % 64 == 0,
// N a multiple of the configuration's tile width. stats (nullable): per-stats-tile, per-worker (rg rows)
// BatchNorm statistics of C, [ceil(M / SR)][2][2][N] floats (SR = gemm_nt_stats_rows(cfg)), merged by
// bn_finalize_tiles. Configurations 0..8 stream K through an LDS ring; 9..14 keep the weight slice
// resident in LDS and stream row tiles through a persistent workgroup (K <= 256).
// pro_scale / pro_shift [pro_groups][K] (nullable, no `add`): the BatchNorm prologue -- A is the
// pre-BatchNorm activation (pro_rg rows per worker) and each element is used as
// bf16(max(a * scale + shift, 0)) (gemm_nt_pro_ok(cfg, ...) must hold)
void gemm_nt(const uint16_t* A, const uint16_t* B, int M, int N, int K, uint16_t* C, const uint16_t* add,
             float* stats, int64_t rg, int cfg, hipStream_t stream, const float* pro_scale = nullptr,
             const float* pro_shift = nullptr, int64_t pro_rg = 0, int pro_groups = 0, float* split_ws = nullptr,
             const uint8_t* add_mask = nullptr);
bool gemm_nt_pro_ok(int cfg, int K, int64_t prg, int groups);
// split-K factor of a configuration (1: none); a split configuration needs split_ws = S x M x N floats
int gemm_nt_splits(int cfg);
// Configuration for an M x N x K problem (-1: none fits); rg_limit > 0: stats tiles <= rg_limit rows.
int gemm_nt_pick(int64_t M, int N, int K, int64_t rg_limit);
int gemm_nt_num_cfg();
bool gemm_nt_valid(int cfg, int N, int K);
int gemm_nt_tile_m(int cfg);
int gemm_nt_tile_n(int cfg);
int gemm_nt_stats_rows(int cfg);
// statistics tiles of an M x N x K launch of cfg with rg-row workers: H rows, E entries each
// (stats buffer: ceil(M / H) * E * 6 * N floats)
void gemm_nt_stats_geometry(int cfg, int64_t M, int N, int K, int64_t rg, int64_t* H, int* E);
// dst_i [C_i, R_i] = src_i [R_i, C_i]ᵀ for bf16 matrices (R_i, C_i multiples of 8), in one launch per 40;
// taps[i] > 1: src_i is [R][taps][C], dst_i [C][taps][R] with the taps reversed (the flipped transposed
// weight of a k x k convolution's data gradient)
void transpose_multi(const uint16_t* const* srcs, uint16_t* const* dsts, const int* R, const int* C, int count,
                     hipStream_t stream, const int* taps = nullptr);
void bn_finalize_tiles(const float* stats, int64_t H, int E, int64_t M, int64_t rg, int groups, int C,
                       const float* gamma, const float* beta, float eps, float* mean, float* istd, float* scale,
                       float* shift, hipStream_t stream);

// mask (nullable, relu only): bit (r*C + c) of the byte array = y[r, c] > 0, for the backward.
// ReLU source of the backward: mask when given, else y (nullable) > 0. dres (nullable) receives dz.
// grow (nullable): exchange buffer; group g's dγ[c] goes to grow[g*row_stride + off_gamma + c]
// (dβ likewise at off_beta; a negative offset skips it), cast to grow_dt.
// coef: [groups, 3, C] fp32 workspace.
void bn_backward(const void* x, const void* dy, const void* y, const uint8_t* mask, int64_t rg, int groups,
                 int C,
                 const float* gamma, const float* mean, const float* istd, float* part, float* coef, void* dx,
                 void* dres, void* grow, int grow_dt, int64_t row_stride, int64_t off_gamma, int64_t off_beta,
                 hipStream_t stream, int dt = 1, const float* rsc = nullptr, const float* rsh = nullptr);
// (rsc / rsh [groups, C], nullable: the ReLU test of a BatchNorm whose normalised output was never
// written -- its consumer applied it while staging its input -- recomputes it as bf16(x * rsc + rsh) > 0.)

// NHWC im2col (bf16): col[(n*Ho + ho)*Wo + wo][(i*KW + j)*C + c] = x[n][ho*sh - ph + i*dh][wo*sw - pw + j*dw][c]
// (0 outside the image). col: [N*Ho*Wo, ldc] with ldc >= KH*KW*C; columns past KH*KW*C are zeroed
// (GEMM-friendly padding of the 3-channel stem).
struct Im2col {
  int N, H, W, C, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo;
  int ldc;
};
void im2col_nhwc(const uint16_t* x, const Im2col& g, uint16_t* col, hipStream_t stream);

// The adjoint gather: dx[n][hi][wi][c] = Σ_{taps (i, j) hitting (hi, wi)} dcol[(n*Ho + ho)*Wo + wo][(i*KW + j)*C + c]
// (fp32 accumulation, every element written once: no atomics, deterministic).
// Implicit-GEMM convolution on MFMA (iconv_nhwc.hip): y[m, co] = Σ x-patch · w[co, (i, j, ci)]
// (+ add[m, co]); C % 32 == 0, Cout % 64 == 0; pm = pixel fragments per wave (0: auto).
// transpose_w (C % 64 == 0): w is the forward weight [C][KH][KW][Cout] of the convolution whose data
// gradient this computes (flipped taps, swapped channel roles).
void iconv_nhwc(const uint16_t* x, const uint16_t* w, const Im2col& g, int Cout, uint16_t* y, const uint16_t* add,
                int pm, bool transpose_w, hipStream_t stream);
// Halo-staged 3x3 / stride-1 / pad-1 convolution (conv3x3_nhwc.hip): same contract as iconv_nhwc
// without transpose_w; C % 64 == 0, Cout % 64 == 0, tiles of whole image rows. conv3x3_pick returns
// the pixel fragments per wave (4 or 2) it would use, 0 when the shape does not fit; conv3x3_nhwc
// returns false (and launches nothing) in that case. pmf <= 0: auto.
int conv3x3_pick(const Im2col& g, int Cout);
// 3x3 / stride-1 / pad-1 convolutions on images of at most 2x2 pixels as dense GEMMs (sconv_nhwc.hip):
// per step, every such layer's W [Cout, 3, 3, Cin] -> Wbig [P*Cout, P*Cin] and Wbigᵀ in one launch
// (P = H * W), and the fold of the dense weight gradient [S, G, P*Cout, P*Cin] (fp32) onto the taps.
struct ScExpandJob {
  const uint16_t* w;
  uint16_t* big;
  uint16_t* bigT;
  int cout, cin, H, W;
};
constexpr int kScMaxJobs = 32;
struct ScExpandJobs {
  ScExpandJob job[kScMaxJobs];
  int64_t start[kScMaxJobs + 1];   // prefix sums of the 8-element units of each job's Wbig
  int count;
};
void sc_expand(const ScExpandJobs& jobs, hipStream_t stream);
void sc_fold(const float* slab, int S, int G, int H, int W, int cout, int cin, void* out, bool out_bf16,
             int64_t gstride, hipStream_t stream);

// Data gradient of a stride-2 convolution (iconv_nhwc.hip, k_iconv_lds S2): four parity classes of
// dx, each a stride-1 correlation of dy with its sub-kernel; no dcol matrix, no col2im. g: the
// forward geometry seen from dy (H, W, C = dy's; Ho, Wo = dx's, even; sh = sw = 2); w: the forward
// channels_last weight [C, Cout, KH, KW]; add: folded into dx.
bool dgrad_s2_ok(const Im2col& g, int Cout);
void dgrad_s2_nhwc(const uint16_t* dy, const uint16_t* w, const Im2col& g, int Cout, uint16_t* dx, const uint16_t* add,
                   int pm, hipStream_t stream);
// stats (nullable, no add): per-worker (rg pixels) BatchNorm statistics of y for bn_finalize_tiles, one
// statistics tile of 16 * pmf pixels per wave (H = 16 * pmf, E = 1: ceil(M / H) * 6 * Cout floats).
bool conv3x3_nhwc(const uint16_t* x, const uint16_t* w, const Im2col& g, int Cout, uint16_t* y, const uint16_t* add,
                  int pmf, hipStream_t stream, float* stats = nullptr, int64_t rg = 0,
                  const uint8_t* add_mask = nullptr);   // add_mask: add counts where its bit is set (1 bit / element)
// Halo-staged per-worker weight gradient of the same 3x3 convolutions (conv3x3_nhwc.hip), same
// contract as iwgrad_nhwc; splits cut each worker's 128-pixel tiles into contiguous ranges (an empty
// range writes a zero slab). wgrad3x3_fits: the shape fits (rg whole images); otherwise
// wgrad3x3_nhwc launches nothing and returns false.
bool wgrad3x3_fits(const Im2col& g, int Cout, int64_t rg);
bool wgrad3x3_nhwc(const uint16_t* x, const uint16_t* dy, const Im2col& g, int Cout, int groups, int64_t rg,
                   int splits, void* out, bool out_bf16, int64_t split_stride, int64_t group_stride,
                   hipStream_t stream);
// Max pooling over NHWC bf16 (C % 8 == 0); idx: the window tap of each output maximum
// (one byte per output element), consumed by the gather backward.
void maxpool_fwd_nhwc(const void* x, const Im2col& g, void* y, uint8_t* idx, hipStream_t stream, int dt = 1);
void maxpool_bwd_nhwc(const void* dy, const uint8_t* idx, const Im2col& g, void* dx, hipStream_t stream, int dt = 1);
// Per-worker implicit weight gradient (iconv_nhwc.hip): out[s][g][co][k] (fp32 partial slab s of
// worker g, or bf16 when out_bf16, e.g. straight into the exchange rows) = Σ over the s-th of `splits`
// pixel ranges of worker g of dy[m, co] · patch(x)[m, k]; C % 64 == 0, Cout % 64 == 0, x / dy 16-B aligned.
// Taps per workgroup of iwgrad_nhwc for a kh x kw kernel over C input channels (3x3: the three
// taps of a kernel row share each staged dy tile, GARFIELD_IWGRAD_ROW; 1x1: up to four 64-channel
// input blocks share it, GARFIELD_IWGRAD_1X1_NT).
int iwgrad_taps_per_block(int kw, int kh = 3, int C = 0, int Cout = 0);
// pro_scale / pro_shift [groups][C] (nullable; 1x1 / stride 1 / no padding only): x is a pre-BatchNorm
// activation used as bf16(max(x * scale + shift, 0)) of the workgroup's worker
void iwgrad_nhwc(const uint16_t* x, const uint16_t* dy, const Im2col& g, int Cout, int groups, int64_t rg,
                 int splits, void* out, bool out_bf16, int64_t split_stride, int64_t group_stride, hipStream_t stream,
                 const float* pro_scale = nullptr, const float* pro_shift = nullptr);
// accumulate: dx += col2im(dcol) instead of dx = col2im(dcol).
void col2im_nhwc(const uint16_t* dcol, const Im2col& g, uint16_t* dx, bool accumulate, hipStream_t stream);

}  // namespace gpu
}  // namespace garfield
