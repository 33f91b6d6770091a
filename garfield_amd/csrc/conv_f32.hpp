// Host-side launchers of the fp32 (reference-precision) grouped-step kernels (conv_f32.hip):
// NHWC convolutions on split-bf16 MFMA (three bf16 pieces per fp32 operand, the six products of
// order <= 2, fp32 accumulation), the per-step weight split, and the classifier / average-pool
// kernels. Asynchronous, no allocation, HIP-graph capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace garfield {
namespace gpu {

// Geometry of one convolution: source activation [N][Hs][Ws][Cs], output [N][Ho][Wo][Co], and the
// FORWARD convolution's kernel / stride / padding / dilation. For a data gradient the source is dy
// (Hs, Ws, Cs = the forward's Ho, Wo, Cout) and the output dx (Ho, Wo, Co = the forward's H, W, Cin).
struct ConvF32Geo {
  int N, Hs, Ws, Cs, Ho, Wo, Co;
  int KH, KW, sh, sw, ph, pw, dh, dw;
};

// Cs % 32 == 0, Co % 64 == 0
bool conv_f32_supported(const ConvF32Geo& g);
bool conv_f32_lds_ok(const ConvF32Geo& g, bool dgrad);
// split-K factor of the automatic choice (1: none); ksplit > 1 needs a `part` workspace of
// ksplit x N x Ho x Wo x Co floats
int conv_f32_ksplit(const ConvF32Geo& g, bool dgrad);
// out[m, co] (+= add, read from `add`) of the forward (w3: the pieces [3][Co][KH][KW][Cs]) or, with
// dgrad, of the data gradient (w3: the transposed pieces [3][Co = Cin][KH][KW][Cs = Cout], any stride).
void conv_f32(const float* src, const uint16_t* w3, const ConvF32Geo& g, bool dgrad, float* out, const float* add,
              int pm, hipStream_t stream, int ksplit = 1, float* part = nullptr);
// Cs % 64 == 0, Co % 64 == 0 (g: the forward geometry)
bool wgrad_f32_supported(const ConvF32Geo& g);
// the 128 x 128-tile weight gradient takes this layer (Cs % 128 == 0, Co % 128 == 0): 4x fewer tiles
bool wgrad_f32_wide(const ConvF32Geo& g);
// out[s][grp][co][k] (fp32) = Σ over the s-th of `splits` ranges of worker grp's rg output pixels of
// dy[m, co] · patch(x)[m, k]; element offset s * split_stride + grp * group_stride + co * K + k.
// variant: 0 automatic, 1 / 2 the 128 x 128 form double- / single-buffered (wgrad_f32_wide shapes), 3 the
// 64 x 64 form
void wgrad_f32(const float* x, const float* dy, const ConvF32Geo& g, int groups, int64_t rg, int splits, float* out,
               int64_t split_stride, int64_t group_stride, hipStream_t stream, int variant = 0);

struct WSplitJob {
  const float* w;      // [R][T][C] fp32 (a channels_last weight: R = Cout, T = KH*KW, C = Cin)
  uint16_t* pieces;    // [3][R][ld] bf16: w0 = bf16(w), w1 = bf16(w - w0), w2 = bf16(w - w0 - w1)
  uint16_t* tpieces;   // nullable: [3][C][T][R] the transposed pieces (the data gradient's weight)
  int R, T, C;
  int ld;              // row pitch of the pieces in elements (0: T * C; e.g. 160 for the padded stem)
};
void wsplit_multi(const WSplitJob* jobs, int count, hipStream_t stream);

// classifier: y[R][O] = x[R][F] · w[O][F]ᵀ + b; dx = dl · w; per-worker dW / db into rows
void linear_f32_fwd(const float* x, const float* w, const float* b, int R, int F, int O, float* y, hipStream_t stream);
void linear_f32_dgrad(const float* dl, const float* w, int R, int F, int O, float* dx, hipStream_t stream);
void linear_f32_wgrad(const float* x, const float* dl, int groups, int rg, int F, int O, float* out, int64_t row_stride,
                      int64_t off_w, int64_t off_b, hipStream_t stream);
// bf16 classifier (fp32 accumulation, one rounding); the weight gradient is written in the exchange
// rows' element type odt (gar_device.hpp dtype codes)
void linear_bf16_fwd(const uint16_t* x, const uint16_t* w, const uint16_t* b, int R, int F, int O, uint16_t* y,
                     hipStream_t stream);
void linear_bf16_dgrad(const uint16_t* dl, const uint16_t* w, int R, int F, int O, uint16_t* dx, hipStream_t stream);
// db_g[o] = Σ_{r in worker g} dl[r][o] (dl bf16 or fp32), into worker g's exchange row at off_b
void linear_bias_grad(const void* dl, bool dl_f32, int groups, int rg, int O, void* out, int odt, int64_t row_stride,
                      int64_t off_b, hipStream_t stream);
void linear_bf16_wgrad(const uint16_t* x, const uint16_t* dl, int groups, int rg, int F, int O, void* out, int odt,
                       int64_t row_stride, int64_t off_w, int64_t off_b, hipStream_t stream);
// wide bf16 heads on gemm_nt (output dimension padded to Op, a multiple of 64; F % 64 == 0): wp [Op][F]
// and wpt [F][Op] from w [O][F], zero-padded; and bf16 rows re-pitched [R][a] -> [R][b] (cropped, or
// zero-padded; + bias on the copied columns; a, b multiples of 8)
void head_weights_bf16(const uint16_t* w, int O, int F, int Op, uint16_t* wp, uint16_t* wpt, hipStream_t stream);
void repitch_bf16(const uint16_t* src, int a, uint16_t* dst, int b, int64_t R, const uint16_t* bias, hipStream_t stream);
void avgpool_bf16_fwd(const uint16_t* x, int N, int HW, int C, uint16_t* y, hipStream_t stream);
void avgpool_bf16_bwd(const uint16_t* dy, int N, int HW, int C, uint16_t* dx, hipStream_t stream);
void avgpool_f32_fwd(const float* x, int N, int HW, int C, float* y, hipStream_t stream);
void avgpool_f32_bwd(const float* dy, int N, int HW, int C, float* dx, hipStream_t stream);

}  // namespace gpu
}  // namespace garfield
