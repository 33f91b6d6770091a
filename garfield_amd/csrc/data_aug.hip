// Fresh training batches on the device, one launch per step (gfx950).
//
// The reference feeds every worker from a torch DataLoader over CIFAR-10 with
// RandomCrop(32, padding=4) + RandomHorizontalFlip + Normalize
// (pytorch_impl/libs/garfieldpp/datasets.py:99-140), i.e. host-side PIL work
// per image per step. Here the dataset lives in HBM as uint8 NHWC images and ONE
// kernel builds the whole grouped batch of all k logical workers: it gathers
// image idx[r], applies a random crop offset (zero padding) and a random
// horizontal flip drawn from a counter-based hash of (seed, step, r) — no RNG
// state, no extra launches, the same batch for the same (seed, step) — then
// normalises and writes bf16 (fp32 for the reference-precision step) straight into the grouped
// channels_last input.
// One thread per output pixel (C <= 4 channels: the uint8 pixel is one load).
#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

template <int DT>
__global__ __launch_bounds__(256) void k_augment_gather(const uint8_t* __restrict__ src, int64_t nsrc,
                                                        const int64_t* __restrict__ idx,
                                                        const int64_t* __restrict__ lab_src,
                                                        int64_t* __restrict__ lab_out, int64_t R, int H, int W, int C, int pad, int flip,
                                                        uint64_t key, AugNorm nrm, void* __restrict__ out) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t HW = static_cast<int64_t>(H) * W;
  if (p >= R * HW) return;
  const int64_t r = p / HW;
  const int pix = static_cast<int>(p - r * HW);
  const int h = pix / W, w = pix - (pix / W) * W;
  const uint32_t u = mix32(key ^ (static_cast<uint64_t>(r) * 0x9e3779b97f4a7c15ull));
  const int span = 2 * pad + 1;
  const int oy = pad ? static_cast<int>(u % span) - pad : 0;
  const int ox = pad ? static_cast<int>((u >> 8) % span) - pad : 0;
  const bool fl = flip && ((u >> 20) & 1u);
  const int hs = h + oy;
  const int ws = (fl ? W - 1 - w : w) + ox;
  const bool in = hs >= 0 && hs < H && ws >= 0 && ws < W;
  int64_t img;
  if (idx) {
    img = idx[r];
    img = img < 0 ? 0 : (img >= nsrc ? nsrc - 1 : img);   // never read outside the dataset
  } else {  // sampling with replacement from the same counter-based hash
    const uint64_t h = (static_cast<uint64_t>(mix32(key + 0x51ed270b27a3b9c1ull * (r + 1))) << 32) |
                       mix32(~key ^ (static_cast<uint64_t>(r) * 0xbf58476d1ce4e5b9ull));
    img = static_cast<int64_t>(h % static_cast<uint64_t>(nsrc));
  }
  if (lab_out && pix == 0) lab_out[r] = lab_src[img];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c >= C) break;
    // padded pixels are black before normalisation (RandomCrop pads the image, then Normalize)
    const float raw = in ? static_cast<float>(src[((img * H + hs) * W + ws) * C + c]) * (1.f / 255.f) : 0.f;
    const float v = (raw - nrm.mean[c]) * nrm.inv_std[c];
    if constexpr (DT == kF32) static_cast<float*>(out)[p * C + c] = v;
    else static_cast<uint16_t*>(out)[p * C + c] = f_to_bf16(v);
  }
}

}  // namespace

void augment_gather(const uint8_t* src, int64_t nsrc, const int64_t* idx, const int64_t* lab_src, int64_t* lab_out,
                    int64_t R, int H, int W, int C, int pad, bool flip,
                    uint64_t seed, uint64_t step, const AugNorm& nrm, void* out, hipStream_t stream, int out_dt) {
  const int64_t total = R * H * W;
  if (total <= 0) return;
  const uint64_t key = seed * 0xd1b54a32d192ed03ull + step * 0x2545f4914f6cdd1dull + 0x632be59bd9b4e019ull;
  const dim3 grid(static_cast<unsigned>((total + 255) / 256));
  if (out_dt == kF32)
    hipLaunchKernelGGL(k_augment_gather<kF32>, grid, dim3(256), 0, stream, src, nsrc, idx, lab_src, lab_out, R, H, W, C,
                       pad, flip ? 1 : 0, key, nrm, out);
  else
    hipLaunchKernelGGL(k_augment_gather<kBF16>, grid, dim3(256), 0, stream, src, nsrc, idx, lab_src, lab_out, R, H, W, C,
                       pad, flip ? 1 : 0, key, nrm, out);
}

}  // namespace gpu
}  // namespace garfield
