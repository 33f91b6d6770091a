// Per-worker BatchNorm statistics of an MFMA tile, reduced in registers in a GEMM / convolution
// epilogue (gemm_nt.hip, conv3x3_nhwc.hip). The accumulator of v_mfma_f32_16x16x32_bf16 with the
// weight as the A operand holds 4 consecutive output channels of one pixel per lane, and the 16
// lanes of a DPP row one channel quad for 16 pixels: a 4-step DPP row reduction gives Σy over a
// wave's rows, then Σ(y - ȳ)² around that sub-tile mean (count-free pairs, no cancellation).
// Layout: stats[T][E][slot][q][N] floats, q = {n, Σy, Σ(y - ȳ)²}; stats tile T covers rows
// [T*H, (T+1)*H) (H <= rows per worker, so at most two workers: slot 0 the first, slot 1 the
// next), merged per worker by bn_finalize_tiles.
#pragma once
#include <hip/hip_runtime.h>

#include "gar_device.hpp"

namespace garfield {
namespace gpu {
namespace dev {

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sum over the 16 lanes of a DPP row, returned in every lane of the row.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
  return v;
}

__device__ __forceinline__ float bf16_round(float x) { return bf16_to_f(f_to_bf16(x)); }

// Statistics of one wave's sub-tile: rows r0 + r*16 + fr (r < WPM), channels chb + c*16 + 4*fq + i.
// v: the stored (bf16-rounded) values. Writes stats[((t*2 + slot)*2 + {0: Σy, 1: Σ(y-ȳ)²})*N + ch]
// for t = r0 / (16*WPM); slot 1 holds the rows past the first worker boundary inside the tile.
template <int WPM, int WPN>
__device__ __forceinline__ void wave_stats(const float (&v)[WPM][WPN][4], int64_t r0, int64_t M, int64_t rg, int N,
                                           int chb, float* __restrict__ stats) {
  constexpr int RW = 16 * WPM;
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int64_t t = r0 / RW;
  const int64_t end = r0 + RW < M ? r0 + RW : M;
  const int64_t gb = (r0 / rg + 1) * rg;
  const int split = static_cast<int>((gb < end ? gb : end) - r0);   // rows of slot 0
  const int rows = static_cast<int>(end - r0);
  const int nslot = split < rows ? 2 : 1;
  for (int slot = 0; slot < nslot; ++slot) {
    const int lo = slot ? split : 0, hi = slot ? rows : split;
    const float cnt = static_cast<float>(hi - lo);
    float s[WPN][4], q[WPN][4];
#pragma unroll
    for (int c = 0; c < WPN; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a = 0.f;
#pragma unroll
        for (int r = 0; r < WPM; ++r) {
          const int rr = r * 16 + fr;
          a += (rr >= lo && rr < hi) ? v[r][c][i] : 0.f;
        }
        s[c][i] = row16_sum(a);
      }
#pragma unroll
    for (int c = 0; c < WPN; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float mu = s[c][i] / cnt;
        float a = 0.f;
#pragma unroll
        for (int r = 0; r < WPM; ++r) {
          const int rr = r * 16 + fr;
          const float d = v[r][c][i] - mu;
          a += (rr >= lo && rr < hi) ? d * d : 0.f;
        }
        q[c][i] = row16_sum(a);
      }
    if (fr == 0) {
      float* ps = stats + ((t * 2 + slot) * 3) * N + chb + 4 * fq;
#pragma unroll
      for (int c = 0; c < WPN; ++c) {
        *reinterpret_cast<float4*>(ps + c * 16) = make_float4(cnt, cnt, cnt, cnt);
        *reinterpret_cast<float4*>(ps + N + c * 16) = make_float4(s[c][0], s[c][1], s[c][2], s[c][3]);
        *reinterpret_cast<float4*>(ps + 2 * N + c * 16) = make_float4(q[c][0], q[c][1], q[c][2], q[c][3]);
      }
    }
  }
}

// v[0..3] += add[e .. e + 4), term i kept where bit i of keep is set
__device__ __forceinline__ void add_bf16x4(float (&v)[4], const uint16_t* __restrict__ add, uint32_t keep, int64_t e) {
  const uint2 a = *reinterpret_cast<const uint2*>(add + e);
  v[0] += (keep & 1u) ? bf16_to_f(a.x & 0xffffu) : 0.f;
  v[1] += (keep & 2u) ? bf16_to_f(a.x >> 16) : 0.f;
  v[2] += (keep & 4u) ? bf16_to_f(a.y & 0xffffu) : 0.f;
  v[3] += (keep & 8u) ? bf16_to_f(a.y >> 16) : 0.f;
}

// EPI_ADD with amask (the residual gradient dres = dy · [y > 0] of a BatchNorm + ReLU, read from dy and
// the forward's ReLU bits instead of a materialised dres): the mask bits of a lane's row over the
// wave's 16 * NG channels from element e (a multiple of 16 * NG) in ONE load of 2 * NG bytes; all ones
// without a mask
template <int NG>
struct RowMask {
  uint32_t w[NG / 2];
  __device__ __forceinline__ void load(const uint8_t* __restrict__ amask, int64_t e) {
    static_assert(NG == 2 || NG == 4 || NG == 8, "2, 4 or 8 channel groups of 16");
    if (!amask) {
#pragma unroll
      for (int i = 0; i < NG / 2; ++i) w[i] = 0xffffffffu;
      return;
    }
    const uint8_t* p = amask + (e >> 3);
    if constexpr (NG == 2) {
      w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (NG == 4) {
      const uint2 u = *reinterpret_cast<const uint2*>(p);
      w[0] = u.x; w[1] = u.y;
    } else {
      const uint4 u = *reinterpret_cast<const uint4*>(p);
      w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
    }
  }
  // bits of channel group c's 4 channels at 4 * fq (byte 2c + fq / 2, nibble fq % 2)
  __device__ __forceinline__ uint32_t nib(int c, int fq) const {
    const int b = 2 * c + (fq >> 1);
    return (w[b >> 2] >> ((b & 3) * 8 + (fq & 1) * 4)) & 0xfu;
  }
};

}  // namespace dev
}  // namespace gpu
}  // namespace garfield
