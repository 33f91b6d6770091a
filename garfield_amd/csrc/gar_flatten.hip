// Multi-tensor flatten + cast: scatter-free copy of a model's per-parameter
// gradients (fp32 / bf16 / fp16 per tensor, each its own allocation) into one row
// of the gradient exchange buffer (bf16 / fp16 / fp32), in ONE launch.
//
// Reference counterpart: `torch.cat([p.grad.view(-1) ...]).to("cpu")` in
// garfieldpp/worker.py:93-94 (one concat kernel + a D2H copy per worker per step).
// Here the row stays on the device, the cast is fused, and no intermediate fp32
// flat vector is materialised.
#include <vector>
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

constexpr int kChunk = 4096;  // elements per workgroup (256 threads x 16)

struct FlatTable {
  const void* src[kMaxFlatTensors];
  int64_t numel[kMaxFlatTensors];
  int64_t dst_off[kMaxFlatTensors];
  int32_t chunk_start[kMaxFlatTensors + 1];  // prefix sum of chunks per tensor
  int8_t src_dt[kMaxFlatTensors];            // kF32 / kBF16 / kF16 per source tensor
  int count;
};

template <int ODT>
__device__ __forceinline__ void store8(void* dst, int64_t x, const float (&v)[8]) {
  store_vec<8>(dst, ODT, x, v);
}

template <int SDT, int ODT>
__device__ __forceinline__ void copy_chunk(const void* __restrict__ src, void* __restrict__ dst, int64_t off,
                                           int64_t c0, int64_t c1) {
  // 8-element vectors: 2×16 B (fp32) or 16 B (16-bit) loads, both need a 16 B aligned source
  const bool vec = ((off & 7) == 0) && ((reinterpret_cast<uintptr_t>(src) & 15) == 0);
  if (vec) {
    const int64_t v_end = c0 + ((c1 - c0) / 8) * 8;
    for (int64_t x = c0 + threadIdx.x * 8; x < v_end; x += 256 * 8) {
      float v[8];
      load_vec<SDT, 8>(src, x, v);
      store8<ODT>(dst, off + x, v);
    }
    for (int64_t x = v_end + threadIdx.x; x < c1; x += 256) store_one(dst, ODT, off + x, load_one<SDT>(src, x));
  } else {
    for (int64_t x = c0 + threadIdx.x; x < c1; x += 256) store_one(dst, ODT, off + x, load_one<SDT>(src, x));
  }
}

template <int ODT>
__global__ __launch_bounds__(256) void k_flatten_cast(FlatTable t, void* __restrict__ dst) {
  const int b = blockIdx.x;
  // which tensor does this chunk belong to (uniform linear scan over <= 96 entries)
  int ti = 0;
  while (ti + 1 < t.count && t.chunk_start[ti + 1] <= b) ++ti;
  const int64_t c0 = static_cast<int64_t>(b - t.chunk_start[ti]) * kChunk;
  const int64_t numel = t.numel[ti];
  const int64_t off = t.dst_off[ti];
  int64_t c1 = c0 + kChunk;
  if (c1 > numel) c1 = numel;
  switch (t.src_dt[ti]) {
    case kBF16: copy_chunk<kBF16, ODT>(t.src[ti], dst, off, c0, c1); break;
    case kF16: copy_chunk<kF16, ODT>(t.src[ti], dst, off, c0, c1); break;
    default: copy_chunk<kF32, ODT>(t.src[ti], dst, off, c0, c1); break;
  }
}

}  // namespace

int flatten_cast(const void* const* srcs, const int* src_dts, const int64_t* numels, const int64_t* offsets,
                 int count, void* dst, int out_dt, hipStream_t stream) {
  int launched = 0;
  for (int base = 0; base < count; base += kMaxFlatTensors) {
    FlatTable t{};
    int c = count - base;
    if (c > kMaxFlatTensors) c = kMaxFlatTensors;
    t.count = c;
    int32_t chunks = 0;
    for (int i = 0; i < c; ++i) {
      t.src[i] = srcs[base + i];
      t.src_dt[i] = static_cast<int8_t>(src_dts[base + i]);
      t.numel[i] = numels[base + i];
      t.dst_off[i] = offsets[base + i];
      t.chunk_start[i] = chunks;
      chunks += static_cast<int32_t>((numels[base + i] + kChunk - 1) / kChunk);
    }
    t.chunk_start[c] = chunks;
    if (chunks == 0) continue;
    if (out_dt == kBF16) hipLaunchKernelGGL(k_flatten_cast<kBF16>, dim3(chunks), dim3(256), 0, stream, t, dst);
    else if (out_dt == kF16) hipLaunchKernelGGL(k_flatten_cast<kF16>, dim3(chunks), dim3(256), 0, stream, t, dst);
    else hipLaunchKernelGGL(k_flatten_cast<kF32>, dim3(chunks), dim3(256), 0, stream, t, dst);
    ++launched;
  }
  return launched;
}

}  // namespace gpu
}  // namespace garfield

// ---------------------------------------------------------------------------
// Split-K partial sums -> exchange rows: out[g * ostride + r * opitch + c] =
// cast(Σ_s part[s * ss + g * gs + r * ipitch + c]), r < R, c < Cc, for the per-worker weight
// gradients computed in S pixel splits (grouped step). One launch replaces an ATen reduction +
// a cast/scatter (and, with ipitch > Cc, the crop of padded GEMM columns); 4 fp32 per lane
// when everything is 16-byte aligned.
namespace garfield {
namespace gpu {
namespace {

template <int ODT, bool VEC>
__global__ __launch_bounds__(256) void k_split_reduce(const float* __restrict__ part, int S, int G, int64_t R,
                                                      int64_t Cc, int64_t ipitch, int64_t opitch, int64_t ss,
                                                      int64_t gs, void* __restrict__ out, int64_t ostride) {
  constexpr int V = VEC ? 4 : 1;
  const int64_t cv = (Cc + V - 1) / V;
  const int64_t per = R * cv;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= per * G) return;
  const int g = static_cast<int>(t / per);
  const int64_t rem = t - static_cast<int64_t>(g) * per;
  const int64_t r = rem / cv;
  const int64_t c = (rem - r * cv) * V;
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;
  const float* p = part + static_cast<int64_t>(g) * gs + r * ipitch + c;
  for (int s = 0; s < S; ++s) {
    if constexpr (VEC) {
      const float4 a = *reinterpret_cast<const float4*>(p + static_cast<int64_t>(s) * ss);
      acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    } else {
      acc[0] += p[static_cast<int64_t>(s) * ss];
    }
  }
  const int64_t o = static_cast<int64_t>(g) * ostride + r * opitch + c;
#pragma unroll
  for (int v = 0; v < V; ++v) dev::store_one(out, ODT, o + v, acc[v]);
}

}  // namespace

void split_reduce(const float* part, int S, int G, int64_t R, int64_t Cc, int64_t ipitch, int64_t opitch, int64_t ss,
                  int64_t gs, void* out, int odt, int64_t ostride, hipStream_t stream) {
  const bool vec = Cc % 4 == 0 && ipitch % 4 == 0 && ss % 4 == 0 && gs % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(part) % 16 == 0;
  const int64_t work = (vec ? Cc / 4 : Cc) * R * G;
  if (work <= 0) return;
  const dim3 grid(static_cast<unsigned>((work + 255) / 256));
#define GARFIELD_SPLIT(ODT)                                                                                     \
  if (vec) hipLaunchKernelGGL((k_split_reduce<ODT, true>), grid, dim3(256), 0, stream, part, S, G, R, Cc, ipitch, \
                              opitch, ss, gs, out, ostride);                                                      \
  else hipLaunchKernelGGL((k_split_reduce<ODT, false>), grid, dim3(256), 0, stream, part, S, G, R, Cc, ipitch,    \
                          opitch, ss, gs, out, ostride)
  if (odt == kBF16) { GARFIELD_SPLIT(kBF16); }
  else if (odt == kF16) { GARFIELD_SPLIT(kF16); }
  else { GARFIELD_SPLIT(kF32); }
#undef GARFIELD_SPLIT
}

}  // namespace gpu
}  // namespace garfield

// ---------------------------------------------------------------------------
// Many split-K reductions in ONE launch (the grouped backward queues one per layer and
// runs them all after the last layer): block b finds its job through the prefix sum of
// blocks per job, then does what k_split_reduce does for 256 x V elements of it.
namespace garfield {
namespace gpu {
namespace {

struct SplitTable {
  SplitJob job[kMaxSplitJobs];
  int32_t blk0[kMaxSplitJobs + 1];
  dev::FastDiv fper[kMaxSplitJobs], fcv[kMaxSplitJobs];   // the element decomposition without divisions
  int count;
};

__global__ __launch_bounds__(256) void k_split_reduce_multi(SplitTable t) {
  int j = 0;
  while (j + 1 < t.count && static_cast<int>(blockIdx.x) >= t.blk0[j + 1]) ++j;
  const SplitJob& J = t.job[j];
  const int V = J.vec ? 4 : 1;
  const uint32_t cv = t.fcv[j].d, per = t.fper[j].d;   // (Cc / V) per row, R rows per group: < 2^31 (host)
  const uint32_t tid = (blockIdx.x - t.blk0[j]) * blockDim.x + threadIdx.x;
  if (tid >= per * static_cast<uint32_t>(J.G)) return;
  const uint32_t g = dev::fdiv(tid, t.fper[j]);
  const uint32_t rem = tid - g * per;
  const uint32_t r = dev::fdiv(rem, t.fcv[j]);
  const int64_t c = static_cast<int64_t>(rem - r * cv) * V;
  const float* p = J.part + static_cast<int64_t>(g) * J.gs + r * J.ipitch + c;
  const int64_t o = static_cast<int64_t>(g) * J.ostride + r * J.opitch + c;
  if (J.vec) {
    // unrolled: the S slab loads are independent and issue back to back (a rolled loop waits on
    // each one: at S = 64-128 slabs that latency chain dominated the launch)
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int s = 0; s < J.S; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(p + static_cast<int64_t>(s) * J.ss);
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    if (J.vec == 2) {   // fp32 rows, 16-byte aligned: one vector store
      *reinterpret_cast<float4*>(static_cast<float*>(J.out) + o) = acc;
    } else {
      dev::store_one(J.out, J.odt, o, acc.x);
      dev::store_one(J.out, J.odt, o + 1, acc.y);
      dev::store_one(J.out, J.odt, o + 2, acc.z);
      dev::store_one(J.out, J.odt, o + 3, acc.w);
    }
  } else {
    float acc = 0.f;
#pragma unroll 8
    for (int s = 0; s < J.S; ++s) acc += p[static_cast<int64_t>(s) * J.ss];
    dev::store_one(J.out, J.odt, o, acc);
  }
}

}  // namespace

void split_reduce_multi(const SplitJob* jobs, int count, hipStream_t stream) {
  // the batched kernel decomposes its element index in 32 bits: a job of 2^31 or more vector
  // elements (or a launch of 2^31 threads) runs alone on the 64-bit kernel instead
  constexpr int64_t kLim = (int64_t{1} << 31) - 256;
  std::vector<SplitJob> small;
  small.reserve(count);
  for (int i = 0; i < count; ++i) {
    const SplitJob& J = jobs[i];
    const int64_t work = J.Cc * J.R * J.G;     // >= the vector-element count
    if (work >= kLim - 512) split_reduce(J.part, J.S, J.G, J.R, J.Cc, J.ipitch, J.opitch, J.ss, J.gs, J.out, J.odt,
                                   J.ostride, stream);
    else small.push_back(J);
  }
  jobs = small.data();
  count = static_cast<int>(small.size());
  for (int base = 0; base < count; base += kMaxSplitJobs) {
    SplitTable t{};
    t.count = count - base < kMaxSplitJobs ? count - base : kMaxSplitJobs;
    int64_t blocks = 0;
    for (int i = 0; i < t.count; ++i) {
      SplitJob J = jobs[base + i];
      J.vec = (J.Cc % 4 == 0 && J.ipitch % 4 == 0 && J.ss % 4 == 0 && J.gs % 4 == 0 &&
               reinterpret_cast<uintptr_t>(J.part) % 16 == 0) ? 1 : 0;
      if (J.vec && J.odt == kF32 && J.opitch % 4 == 0 && J.ostride % 4 == 0 &&
          reinterpret_cast<uintptr_t>(J.out) % 16 == 0)
        J.vec = 2;
      t.job[i] = J;
      const int64_t cvh = J.vec ? J.Cc / 4 : J.Cc;
      const int64_t nb = (cvh * J.R * J.G + 255) / 256;
      if ((blocks + nb) * 256 >= kLim) {     // this job starts the next launch
        t.count = i;
        break;
      }
      t.blk0[i] = static_cast<int32_t>(blocks);
      t.fcv[i] = dev::make_fastdiv(static_cast<uint32_t>(cvh));
      t.fper[i] = dev::make_fastdiv(static_cast<uint32_t>(cvh * J.R));
      blocks += nb;
    }
    if (t.count == 0) continue;   // unreachable: every job alone is below the limit
    t.blk0[t.count] = static_cast<int32_t>(blocks);
    if (blocks > 0) hipLaunchKernelGGL(k_split_reduce_multi, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, t);
    base -= kMaxSplitJobs - t.count;   // resume after the last job launched
  }
}

}  // namespace gpu
}  // namespace garfield
