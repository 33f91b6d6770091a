// Row-major "NT" GEMM for the grouped step's 1x1 convolutions, on MFMA (bf16 in, fp32
// accumulate, bf16 out), gfx950, with the producer-side BatchNorm statistics fused in.
//
//   C[M, N] = A[M, K] · B[N, K]ᵀ  (+ add[M, N])
//
// Forward of a 1x1 stride-1 convolution: A = the NHWC activation rows [pixels, Cin],
// B = the weight [Cout, Cin]. Data gradient: A = dy rows [pixels, Cout], B = the
// transposed weight [Cin, Cout]; ``add`` folds in the residual branch's gradient.
//
// Why not hipBLASLt: the step's 1x1 GEMMs are skinny (M = 2k..128k pixels, N, K =
// 64..2048) and memory-bound; hipBLASLt measured 2.2x the compulsory-byte time on
// them, with a ~10 µs floor per call (scripts/bench_1x1.py), and its epilogue cannot
// produce the per-WORKER BatchNorm statistics that the next layer needs, so a
// separate pass re-read every output (bn_nhwc.hip k_partial). Here:
//
// * workgroup tile BM pixels x BN channels (4 waves, WM x WN, each 16*WPM x 16*WPN),
//   64-deep k-steps staged global -> LDS by global_load_lds (16 B per lane, no VGPR
//   round trip) in an NS-deep ring, chunk index XOR-swizzled by (row & 7) on the
//   global side so the 16-row fragment reads hit 8 different bank groups;
// * v_mfma_f32_16x16x32_bf16 with the WEIGHT as the MFMA A operand, so D's lane holds
//   4 consecutive output channels of one pixel: one 8-byte store per fragment;
// * tiles are numbered XCD-aware (the N blocks of one M block run on the same XCD
//   and share its L2 copy of the A rows);
// * EPI_STATS: every tile also emits, per channel and per worker group its rows
//   belong to (a tile spans <= 2 groups: BM <= rows per worker), the count-free pair
//   (Σ y, Σ (y - ȳ_tile)²) of the STORED bf16 values. ``bn_finalize_tiles`` merges
//   the tiles of a worker with Chan's parallel-variance update (no cancellation,
//   whatever |mean| / std), so the BatchNorm forward only runs its apply pass.
#include "bn_gpu.hpp"
#include "gar_device.hpp"

namespace garfield {
namespace gpu {
using namespace dev;
namespace {

using lds_ptr = __attribute__((address_space(3))) void*;
__device__ __attribute__((aligned(16))) uint4 g_gemm_zero[8];  // 128 zero bytes: source of padded rows

constexpr int EPI_PLAIN = 0, EPI_ADD = 1, EPI_STATS = 2;

template <int WPM, int WPN, int WM, int WN, int NS, int EPI>
__global__ __launch_bounds__(256) void k_gemm_nt(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                 int M, int N, int K, uint16_t* __restrict__ C,
                                                 const uint16_t* __restrict__ add, float* __restrict__ stats,
                                                 int64_t rg) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  constexpr int BM = 16 * WPM * WM, BN = 16 * WPN * WN;
  constexpr int AB = BM * 128, BB = BN * 128, SB = AB + BB;
  constexpr int AI = BM / 32, BI = BN / 32;     // glds instructions per wave per stage
  constexpr int PER = AI + BI;
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tiles are whole 8-row glds blocks per wave");
  __shared__ __attribute__((aligned(16))) char lds[NS * SB];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tiles_n = N / BN;
  const int nt = gridDim.x;
  const int b = blockIdx.x;
  // XCD-aware numbering: block b runs on XCD b % 8; consecutive tile ids (the N blocks
  // of one M block) get blocks of the same residue
  const int t = (nt % 8 == 0) ? (b % 8) * (nt / 8) + b / 8 : b;
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lrow = lane >> 3, lchunk = lane & 7;

  const uint16_t* asrc[AI];
  bool av[AI];
#pragma unroll
  for (int u = 0; u < AI; ++u) {
    const int row = (wave * AI + u) * 8 + lrow;
    av[u] = m0 + row < M;
    asrc[u] = A + static_cast<int64_t>(av[u] ? m0 + row : 0) * K + (lchunk ^ lrow) * 8;
  }
  const uint16_t* bsrc[BI];
#pragma unroll
  for (int u = 0; u < BI; ++u) {
    const int row = (wave * BI + u) * 8 + lrow;
    bsrc[u] = B + static_cast<int64_t>(n0 + row) * K + (lchunk ^ lrow) * 8;
  }
  const uint64_t az = reinterpret_cast<uint64_t>(reinterpret_cast<const uint16_t*>(g_gemm_zero) + lchunk * 8);
  const int steps = K / 64;

  auto issue = [&](int s, int slot) {
    char* base = lds + slot * SB;
    const int k0 = s * 64;
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const uint64_t a = reinterpret_cast<uint64_t>(asrc[u] + k0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(av[u] ? a : az),
                                       (lds_ptr)(base + (wave * AI + u) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < BI; ++u)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(bsrc[u] + k0), (lds_ptr)(base + AB + (wave * BI + u) * 1024), 16, 0, 0);
  };

  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[WPM][WPN];
#pragma unroll
  for (int r = 0; r < WPM; ++r)
#pragma unroll
    for (int c = 0; c < WPN; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < steps) issue(s0, s0);

  for (int s = 0; s < steps; ++s) {
    // stage s has landed when at most (stages issued after it) x PER loads are outstanding
    const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < steps) issue(s + NS - 1, (s + NS - 1) % NS);
    const char* base = lds + (s % NS) * SB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = (ks * 4 + fq) ^ (fr & 7);
      bf16x8 wf[WPN], xf[WPM];
#pragma unroll
      for (int c = 0; c < WPN; ++c)
        wf[c] = *reinterpret_cast<const bf16x8*>(base + AB + ((wn * WPN + c) * 16 + fr) * 128 + chunk * 16);
#pragma unroll
      for (int r = 0; r < WPM; ++r)
        xf[r] = *reinterpret_cast<const bf16x8*>(base + ((wm * WPM + r) * 16 + fr) * 128 + chunk * 16);
#pragma unroll
      for (int r = 0; r < WPM; ++r)
#pragma unroll
        for (int c = 0; c < WPN; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[r], acc[r][c], 0, 0, 0);
    }
    // every wave's fragment reads of this slot retire before the barrier that lets it be refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // ---- epilogue. The fragments hold 4 channels of one pixel per lane; written straight
  // to global memory that is 16 rows x 32 B per store instruction. Instead the tile goes
  // through LDS (bf16, padded row pitch) and leaves as 16-byte-per-lane row segments
  // (whole 128-B lines per 8 lanes); the statistics are read back from the same image.
  constexpr int TP = BN * 2 + 16;                       // LDS row pitch (bytes)
  constexpr int CPR = BN / 8;                           // 16-byte chunks per tile row
  constexpr int RL = 256 / CPR;                         // tile rows per pass of the workgroup
  static_assert(BM * TP + 2 * 256 * 8 * 4 + 2 * BN * 4 <= NS * SB, "epilogue tile fits the ring");
  __syncthreads();                                      // every wave's last ring reads are done
  {
    const int mwl = wm * 16 * WPM;                      // first tile row of this wave
    const int nwl = wn * 16 * WPN + 4 * fq;             // first tile channel of this lane (c = 0)
#pragma unroll
    for (int r = 0; r < WPM; ++r) {
      const int m = m0 + mwl + r * 16 + fr;
#pragma unroll
      for (int c = 0; c < WPN; ++c) {
        float v[4] = {acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]};
        if constexpr (EPI == EPI_ADD) {                 // one rounding: the sum is formed in fp32
          if (m < M) {
            const uint2 a = *reinterpret_cast<const uint2*>(add + static_cast<int64_t>(m) * N + n0 + nwl + c * 16);
            v[0] += bf16_to_f(a.x & 0xffffu);
            v[1] += bf16_to_f(a.x >> 16);
            v[2] += bf16_to_f(a.y & 0xffffu);
            v[3] += bf16_to_f(a.y >> 16);
          }
        }
        uint2 o;
        o.x = static_cast<uint32_t>(f_to_bf16(v[0])) | (static_cast<uint32_t>(f_to_bf16(v[1])) << 16);
        o.y = static_cast<uint32_t>(f_to_bf16(v[2])) | (static_cast<uint32_t>(f_to_bf16(v[3])) << 16);
        *reinterpret_cast<uint2*>(lds + (mwl + r * 16 + fr) * TP + (nwl + c * 16) * 2) = o;
      }
    }
  }
  __syncthreads();
  const int ck = threadIdx.x % CPR, rl = threadIdx.x / CPR;
  const int rows = M - m0 < BM ? M - m0 : BM;
  float s0[8], s1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s0[i] = 0.f; s1[i] = 0.f; }
  // worker groups of this tile (statistics): rows [m0, mb) -> slot 0, [mb, m0 + rows) -> slot 1
  const int64_t gb = EPI == EPI_STATS ? (static_cast<int64_t>(m0) / rg + 1) * rg : 0;
  const int rb = EPI == EPI_STATS ? (gb - m0 < rows ? static_cast<int>(gb - m0) : rows) : rows;
  for (int rr = rl; rr < rows; rr += RL) {
    const uint4 v = *reinterpret_cast<const uint4*>(lds + rr * TP + ck * 16);
    *reinterpret_cast<uint4*>(C + static_cast<int64_t>(m0 + rr) * N + n0 + ck * 8) = v;
    if constexpr (EPI == EPI_STATS) {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const bool lo = rr < rb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = bf16_to_f(w[i] & 0xffffu), b = bf16_to_f(w[i] >> 16);
        s0[2 * i] += lo ? a : 0.f;
        s0[2 * i + 1] += lo ? b : 0.f;
        s1[2 * i] += lo ? 0.f : a;
        s1[2 * i + 1] += lo ? 0.f : b;
      }
    }
  }

  if constexpr (EPI == EPI_STATS) {
    // per-(slot, channel) totals over the RL row lanes: red[slot][rl][channel]
    float* red = reinterpret_cast<float*>(lds + BM * TP);
    float* mean = red + 2 * RL * BN;                    // [2][BN]
    const float cnt0 = static_cast<float>(rb), cnt1 = static_cast<float>(rows - rb);
    auto reduce = [&](float (&x0)[8], float (&x1)[8], int which) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        red[(0 * RL + rl) * BN + ck * 8 + i] = x0[i];
        red[(1 * RL + rl) * BN + ck * 8 + i] = x1[i];
      }
      __syncthreads();
      for (int i = threadIdx.x; i < 2 * BN; i += 256) {
        const int slot = i / BN, ch = i - slot * BN;
        float t = 0.f;
        for (int l = 0; l < RL; ++l) t += red[(slot * RL + l) * BN + ch];
        const float cnt = slot ? cnt1 : cnt0;
        if (which == 0) mean[i] = cnt > 0.f ? t / cnt : 0.f;
        if (cnt > 0.f) stats[((static_cast<int64_t>(tm) * 2 + slot) * 2 + which) * N + n0 + ch] = t;
      }
      __syncthreads();
    };
    reduce(s0, s1, 0);
    float mu0[8], mu1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mu0[i] = mean[ck * 8 + i];
      mu1[i] = mean[BN + ck * 8 + i];
      s0[i] = 0.f;
      s1[i] = 0.f;
    }
    for (int rr = rl; rr < rows; rr += RL) {
      const uint4 v = *reinterpret_cast<const uint4*>(lds + rr * TP + ck * 16);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const bool lo = rr < rb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float x = bf16_to_f(h ? (w[i] >> 16) : (w[i] & 0xffffu));
          const float d0 = x - mu0[2 * i + h], d1 = x - mu1[2 * i + h];
          s0[2 * i + h] += lo ? d0 * d0 : 0.f;
          s1[2 * i + h] += lo ? 0.f : d1 * d1;
        }
      }
    }
    reduce(s0, s1, 1);
  }
}

// Merge of one worker's tile statistics (Chan et al.): 64 channels x 16 tile lanes per
// workgroup, each lane folding every 16th tile of the worker (all its loads issued
// before they are used), the 16 lane partials merged in a fixed order through LDS.
constexpr int kMergeCh = 64, kMergeLanes = 16;

__device__ __forceinline__ void chan_merge(float& n, float& mu, float& m2, float nb, float mub, float m2b) {
  if (nb <= 0.f) return;
  const float nn = n + nb;
  const float d = mub - mu;
  mu += d * (nb / nn);
  m2 += m2b + d * d * (n * nb / nn);
  n = nn;
}

__global__ __launch_bounds__(kMergeCh * kMergeLanes) void k_finalize_tiles(
    const float* __restrict__ stats, int BM, int64_t M, int64_t rg, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ mean, float* __restrict__ istd,
    float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float sn[kMergeLanes][kMergeCh], smu[kMergeLanes][kMergeCh], sm2[kMergeLanes][kMergeCh];
  const int tc = threadIdx.x % kMergeCh, lane = threadIdx.x / kMergeCh;
  const int c = blockIdx.x * kMergeCh + tc;
  const int g = blockIdx.y;
  const int64_t g0 = static_cast<int64_t>(g) * rg, g1 = g0 + rg < M ? g0 + rg : M;
  const int64_t t_lo = g0 / BM, t_hi = (g1 - 1) / BM;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C) {
    for (int64_t t0 = t_lo + lane; t0 <= t_hi; t0 += kMergeLanes * 4) {
      float sv[4], qv[4], nv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t t = t0 + static_cast<int64_t>(u) * kMergeLanes;
        nv[u] = 0.f;
        sv[u] = qv[u] = 0.f;
        if (t <= t_hi) {
          const int64_t lo = t * BM > g0 ? t * BM : g0;
          const int64_t hi = (t + 1) * BM < g1 ? (t + 1) * BM : g1;
          const int slot = t * BM < g0 ? 1 : 0;   // the tile started in the previous worker
          nv[u] = static_cast<float>(hi - lo);
          sv[u] = stats[((t * 2 + slot) * 2 + 0) * C + c];
          qv[u] = stats[((t * 2 + slot) * 2 + 1) * C + c];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) chan_merge(n, mu, m2, nv[u], nv[u] > 0.f ? sv[u] / nv[u] : 0.f, qv[u]);
    }
  }
  sn[lane][tc] = n;
  smu[lane][tc] = mu;
  sm2[lane][tc] = m2;
  __syncthreads();
  if (lane != 0 || c >= C) return;
  float N0 = sn[0][tc], MU = smu[0][tc], M2 = sm2[0][tc];
  for (int l = 1; l < kMergeLanes; ++l) chan_merge(N0, MU, M2, sn[l][tc], smu[l][tc], sm2[l][tc]);
  float var = N0 > 0.f ? M2 / N0 : 0.f;
  var = var > 0.f ? var : 0.f;
  const float is = rsqrtf(var + eps);
  const int64_t gc = static_cast<int64_t>(g) * C + c;
  mean[gc] = MU;
  istd[gc] = is;
  const float sc = (gamma ? gamma[c] : 1.f) * is;
  scale[gc] = sc;
  shift[gc] = (beta ? beta[c] : 0.f) - MU * sc;
}

template <int WPM, int WPN, int WM, int WN, int NS>
void launch_cfg(const uint16_t* A, const uint16_t* B, int M, int N, int K, uint16_t* C, const uint16_t* add,
                float* stats, int64_t rg, hipStream_t stream) {
  constexpr int BM = 16 * WPM * WM, BN = 16 * WPN * WN;
  const dim3 grid(((M + BM - 1) / BM) * (N / BN));
  if (stats)
    hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_STATS>), grid, dim3(256), 0, stream, A, B, M, N, K, C,
                       add, stats, rg);
  else if (add)
    hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_ADD>), grid, dim3(256), 0, stream, A, B, M, N, K, C,
                       add, stats, rg);
  else
    hipLaunchKernelGGL((k_gemm_nt<WPM, WPN, WM, WN, NS, EPI_PLAIN>), grid, dim3(256), 0, stream, A, B, M, N, K, C,
                       add, stats, rg);
}

// tile configurations: {BM, BN}
constexpr int kCfgBM[] = {128, 256, 64, 64, 64, 128, 128, 64, 32};
constexpr int kCfgBN[] = {128, 64, 128, 256, 64, 256, 128, 64, 256};
constexpr int kNumCfg = 9;

}  // namespace

int gemm_nt_tile_m(int cfg) { return (cfg >= 0 && cfg < kNumCfg) ? kCfgBM[cfg] : 0; }
int gemm_nt_tile_n(int cfg) { return (cfg >= 0 && cfg < kNumCfg) ? kCfgBN[cfg] : 0; }

int gemm_nt_pick(int64_t M, int N, int K, int64_t rg_limit) {
  // largest tile that still gives >= 512 workgroups (2 per CU); BN never above N;
  // with statistics a tile must not span more than two workers (BM <= rows per worker)
  static const int order[] = {5, 0, 1, 3, 2, 4};
  int best = -1;
  int64_t best_wg = -1;
  for (int cfg : order) {
    const int bm = kCfgBM[cfg], bn = kCfgBN[cfg];
    if (N % bn != 0 || (rg_limit > 0 && bm > rg_limit)) continue;
    const int64_t wg = ((M + bm - 1) / bm) * (N / bn);
    if (wg >= 512) return cfg;
    if (wg > best_wg) { best_wg = wg; best = cfg; }
  }
  (void)K;
  return best;
}

void gemm_nt(const uint16_t* A, const uint16_t* B, int M, int N, int K, uint16_t* C, const uint16_t* add,
             float* stats, int64_t rg, int cfg, hipStream_t stream) {
  if (M <= 0) return;
  switch (cfg) {
    case 0: launch_cfg<4, 4, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 6: launch_cfg<4, 4, 2, 2, 3>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 7: launch_cfg<2, 2, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 8: launch_cfg<2, 4, 1, 4, 2>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 1: launch_cfg<4, 4, 4, 1, 2>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 2: launch_cfg<2, 4, 2, 2, 3>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 3: launch_cfg<4, 4, 1, 4, 2>(A, B, M, N, K, C, add, stats, rg, stream); break;
    case 4: launch_cfg<2, 2, 2, 2, 4>(A, B, M, N, K, C, add, stats, rg, stream); break;
    default: launch_cfg<4, 8, 2, 2, 2>(A, B, M, N, K, C, add, stats, rg, stream); break;
  }
}

void bn_finalize_tiles(const float* stats, int BM, int64_t M, int64_t rg, int groups, int C, const float* gamma,
                       const float* beta, float eps, float* mean, float* istd, float* scale, float* shift,
                       hipStream_t stream) {
  const dim3 grid((C + kMergeCh - 1) / kMergeCh, groups);
  hipLaunchKernelGGL(k_finalize_tiles, grid, dim3(kMergeCh * kMergeLanes), 0, stream, stats, BM, M, rg, C, gamma,
                     beta, eps, mean, istd, scale, shift);
}

}  // namespace gpu
}  // namespace garfield
