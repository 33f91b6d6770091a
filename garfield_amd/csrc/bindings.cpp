// Python bindings of the Garfield-MI355X native layer (module garfield_amd._C).
//
// Reference counterpart: the per-rule pybind modules py_krum/py_bulyan/py_median/
// py_brute (e.g. py_krum/rule.cpp:43-62) plus the dtype/device dispatcher
// include/aggregator.hpp:76-135. Here one module exposes the building blocks
// (Gram, selection, combine, coordinate-wise, fused SGD) on both devices; the
// Python layer (garfield_amd/ops/gar.py) composes them into rules.
#include <map>
#include <mutex>
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "bn_gpu.hpp"
#include "conv_f32.hpp"
#include "gar_common.hpp"
#include "gar_cpu.hpp"
#include "gar_gpu.hpp"
#include "loss_gpu.hpp"
#include "mailbox.hpp"
#include "threadpool.hpp"

namespace py = pybind11;
using garfield::RowTable;

namespace {

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return garfield::kF32;
    case at::kBFloat16: return garfield::kBF16;
    case at::kHalf: return garfield::kF16;
    case at::kDouble: return garfield::kF64;
    default: TORCH_CHECK(false, "garfield: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

// A validated set of n gradient rows of length d on one device.
struct RowSet {
  RowTable table{};
  int n = 0;
  int64_t d = 0;
  int dt = 0;
  at::Device device{at::kCPU};
  at::ScalarType st = at::kFloat;
};

void check_row(const at::Tensor& t, const RowSet& rs, bool gpu) {
  TORCH_CHECK(t.device() == rs.device, "garfield: all gradients must be on the same device");
  TORCH_CHECK(t.scalar_type() == rs.st, "garfield: all gradients must have the same dtype");
  if (gpu)
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
                "garfield: gradient rows must be 16-byte aligned on the GPU path");
}

RowSet rows_from_list(const std::vector<at::Tensor>& rows, bool gpu) {
  TORCH_CHECK(!rows.empty(), "garfield: expected a non-empty list of gradients");
  TORCH_CHECK(static_cast<int>(rows.size()) <= garfield::kMaxRows, "garfield: at most ", garfield::kMaxRows,
              " gradients per call, got ", rows.size());
  RowSet rs;
  rs.n = static_cast<int>(rows.size());
  rs.device = rows[0].device();
  rs.st = rows[0].scalar_type();
  rs.dt = dtype_code(rows[0]);
  rs.d = rows[0].numel();
  for (int i = 0; i < rs.n; ++i) {
    const auto& t = rows[i];
    TORCH_CHECK(t.is_contiguous(), "garfield: gradient ", i, " is not contiguous");
    TORCH_CHECK(t.numel() == rs.d, "garfield: gradient ", i, " has ", t.numel(), " elements, expected ", rs.d);
    check_row(t, rs, gpu);
    rs.table.p[i] = t.data_ptr();
  }
  return rs;
}

RowSet rows_from_2d(const at::Tensor& G, bool gpu) {
  TORCH_CHECK(G.dim() == 2, "garfield: expected a 2-D [n, d] gradient buffer");
  TORCH_CHECK(G.size(0) >= 1 && G.size(0) <= garfield::kMaxRows, "garfield: 1 <= n <= ", garfield::kMaxRows);
  TORCH_CHECK(G.stride(1) == 1, "garfield: gradient rows must be contiguous");
  RowSet rs;
  rs.n = static_cast<int>(G.size(0));
  rs.d = G.size(1);
  rs.device = G.device();
  rs.st = G.scalar_type();
  rs.dt = dtype_code(G);
  const int64_t esz = G.element_size();
  const char* base = static_cast<const char*>(G.data_ptr());
  for (int i = 0; i < rs.n; ++i) rs.table.p[i] = base + static_cast<int64_t>(i) * G.stride(0) * esz;
  if (gpu)
    for (int i = 0; i < rs.n; ++i)
      TORCH_CHECK(reinterpret_cast<uintptr_t>(rs.table.p[i]) % 16 == 0,
                  "garfield: gradient rows must be 16-byte aligned on the GPU path (pad the row stride)");
  return rs;
}

template <class T>
garfield::cpu::Rows<T> cpu_rows(const RowSet& rs) {
  TORCH_CHECK(rs.device.is_cpu(), "garfield: CPU path called with device tensors");
  garfield::cpu::Rows<T> r;
  r.n = static_cast<size_t>(rs.n);
  r.d = static_cast<size_t>(rs.d);
  for (int i = 0; i < rs.n; ++i) r.p.push_back(static_cast<const T*>(rs.table.p[i]));
  return r;
}

void check_gpu(const RowSet& rs) {
  TORCH_CHECK(rs.device.is_cuda(), "garfield: GPU path called with host tensors");
  TORCH_CHECK(rs.dt != garfield::kF64, "garfield: fp64 is not supported by the MFMA kernels");
}

hipStream_t stream_of(const at::Device& dev) { return c10::hip::getCurrentHIPStream(dev.index()).stream(); }

float* fptr(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous(), "garfield: expected a contiguous fp32 tensor");
  return t.data_ptr<float>();
}

// ------------------------------------------------------------------ GPU ----

void g_gram(const RowSet& rs, const at::Tensor& slabs, const at::Tensor& gram) {
  check_gpu(rs);
  c10::hip::HIPGuard guard(rs.device.index());
  const int grid = garfield::gpu::gram_grid(rs.d, rs.dt, rs.n);
  TORCH_CHECK(slabs.numel() >= (grid + garfield::gpu::kGramReduceGroups) * garfield::gpu::gram_slab_floats(rs.n),
              "garfield: gram slab workspace too small");
  const int np = garfield::gpu::gram_padded(rs.n);
  TORCH_CHECK(gram.numel() >= np * np, "garfield: gram output too small");
  garfield::gpu::gram(rs.table, rs.n, rs.d, rs.dt, fptr(slabs), grid, fptr(gram), stream_of(rs.device));
}

void g_combine(const RowSet& rs, const at::Tensor& weights, const at::Tensor& out) {
  check_gpu(rs);
  c10::hip::HIPGuard guard(rs.device.index());
  TORCH_CHECK(out.is_contiguous() && out.numel() == rs.d, "garfield: combine output shape mismatch");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "garfield: output must be 16-byte aligned");
  garfield::gpu::combine(rs.table, rs.n, rs.d, rs.dt, fptr(weights), out.data_ptr(), dtype_code(out),
                         stream_of(rs.device));
}

void g_combine_sgd(const RowSet& rs, const at::Tensor& weights, const at::Tensor& param, const at::Tensor& mom,
                   const c10::optional<at::Tensor>& grad_out, const c10::optional<at::Tensor>& shadow, double lr,
                   double momentum, double dampening, double weight_decay, bool nesterov, bool first_step) {
  check_gpu(rs);
  c10::hip::HIPGuard guard(rs.device.index());
  TORCH_CHECK(param.numel() == rs.d && mom.numel() == rs.d, "garfield: parameter/momentum size mismatch");
  float* g = nullptr;
  if (grad_out.has_value() && grad_out->defined()) {
    TORCH_CHECK(grad_out->numel() == rs.d, "garfield: grad_out size mismatch");
    g = fptr(*grad_out);
  }
  void* sh = nullptr;
  int sh_dt = garfield::kBF16;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->is_cuda() && shadow->device() == param.device() && shadow->is_contiguous(),
                "garfield: shadow must be a contiguous tensor on the parameters' device");
    TORCH_CHECK(shadow->numel() >= rs.d, "garfield: shadow too small");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(shadow->data_ptr()) % 16 == 0, "garfield: shadow must be 16-byte aligned");
    sh_dt = dtype_code(*shadow);
    TORCH_CHECK(sh_dt == garfield::kBF16 || sh_dt == garfield::kF16 || sh_dt == garfield::kF32,
                "garfield: shadow dtype must be bf16, fp16 or fp32");
    sh = shadow->data_ptr();
  }
  garfield::gpu::SgdArgs a{static_cast<float>(lr), static_cast<float>(momentum), static_cast<float>(dampening),
                           static_cast<float>(weight_decay), nesterov ? 1 : 0, first_step ? 1 : 0};
  garfield::gpu::combine_sgd(rs.table, rs.n, rs.d, rs.dt, fptr(weights), fptr(param), fptr(mom), g, sh, sh_dt, a,
                             stream_of(rs.device));
}

// GARFIELD_AVGMED_TAIL=0: averaged median on its direct window kernel
bool averaged_median_as_tail() {
  static const bool on = [] {
    const char* e = std::getenv("GARFIELD_AVGMED_TAIL");
    return !(e && e[0] == '0');
  }();
  return on;
}

// n x n fp32 identity on a device, made once per (device, n) and kept (a persistent tensor:
// the aggregation runs outside graph capture)
const at::Tensor& identity_rows(int n, const at::Device& dev) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, at::Tensor> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair(static_cast<int>(dev.index()), n);
  auto it = cache.find(key);
  if (it == cache.end())
    it = cache.emplace(key, at::eye(n, at::TensorOptions().dtype(at::kFloat).device(dev))).first;
  return it->second;
}

void g_coordwise(const RowSet& rs, int mode, int f, int beta, const c10::optional<at::Tensor>& W, int t,
                 uint64_t seed, double p, const at::Tensor& out) {
  check_gpu(rs);
  c10::hip::HIPGuard guard(rs.device.index());
  TORCH_CHECK(out.is_contiguous() && out.numel() == rs.d, "garfield: coordwise output shape mismatch");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "garfield: output must be 16-byte aligned");
  const float* w = nullptr;
  if (mode == garfield::kBulyanTail) {
    TORCH_CHECK(W.has_value() && W->numel() >= t * rs.n, "garfield: Bulyan tail needs W[t, n]");
    TORCH_CHECK(t >= 1 && t <= garfield::kMaxRows, "garfield: invalid t");
    w = fptr(*W);
  } else if (mode == garfield::kAveragedMedian && rs.dt != garfield::kF32 && rs.n <= 64 && averaged_median_as_tail()) {
    // the averaged median of the rows IS Bulyan's tail with W = I (t = n): the MFMA tail kernel
    // (set "means" = the rows themselves, exact) is ~1.5x faster than the direct window kernel
    // at n = 64 (profiles/r2/gar_bench_avgmed_tail.jsonl)
    const at::Tensor& eye = identity_rows(rs.n, rs.device);
    garfield::gpu::coordwise(rs.table, rs.n, rs.d, rs.dt, garfield::kBulyanTail, f, beta, eye.data_ptr<float>(),
                             rs.n, seed, garfield::bernoulli_threshold(p), out.data_ptr(), dtype_code(out),
                             stream_of(rs.device));
    return;
  }
  garfield::gpu::coordwise(rs.table, rs.n, rs.d, rs.dt, mode, f, beta, w, t, seed,
                           garfield::bernoulli_threshold(p), out.data_ptr(), dtype_code(out), stream_of(rs.device));
}

void g_sqdist(const RowSet& rs, const at::Tensor& center, const at::Tensor& slabs) {
  check_gpu(rs);
  c10::hip::HIPGuard guard(rs.device.index());
  TORCH_CHECK(center.numel() == rs.d, "garfield: centre size mismatch");
  const int grid = garfield::gpu::sqdist_grid(rs.d);
  TORCH_CHECK(slabs.numel() >= static_cast<int64_t>(grid) * rs.n, "garfield: sqdist workspace too small");
  garfield::gpu::sqdist_partial(rs.table, rs.n, rs.d, rs.dt, fptr(center), fptr(slabs), grid, stream_of(rs.device));
}

// ------------------------------------------------------------------ CPU ----

template <class F>
auto cpu_dispatch(const RowSet& rs, F&& f) {
  if (rs.dt == garfield::kF64) return f(cpu_rows<double>(rs), double{});
  TORCH_CHECK(rs.dt == garfield::kF32, "garfield: CPU path supports fp32/fp64 (convert bf16/fp16 first)");
  return f(cpu_rows<float>(rs), float{});
}

at::Tensor dist_tensor(const std::vector<double>& D, int64_t n) {
  auto t = at::empty({n, n}, at::TensorOptions().dtype(at::kDouble));
  std::copy(D.begin(), D.end(), t.data_ptr<double>());
  return t;
}

at::Tensor weights_tensor(const std::vector<float>& w, std::vector<int64_t> shape) {
  auto t = at::empty(shape, at::TensorOptions().dtype(at::kFloat));
  std::copy(w.begin(), w.end(), t.data_ptr<float>());
  return t;
}

std::vector<double> dist_from(const at::Tensor& D) {
  auto c = D.to(at::kDouble).contiguous().cpu();
  return std::vector<double>(c.data_ptr<double>(), c.data_ptr<double>() + c.numel());
}

std::vector<float> floats_from(const at::Tensor& W) {
  auto c = W.to(at::kFloat).contiguous().cpu();
  return std::vector<float>(c.data_ptr<float>(), c.data_ptr<float>() + c.numel());
}

at::Tensor c_pairwise(const RowSet& rs) {
  return cpu_dispatch(rs, [&](auto r, auto) { return dist_tensor(garfield::cpu::pairwise_sqdist(r), rs.n); });
}

at::Tensor c_combine(const RowSet& rs, const at::Tensor& weights) {
  auto w = floats_from(weights);
  TORCH_CHECK(static_cast<int>(w.size()) == rs.n, "garfield: weights size mismatch");
  auto out = at::empty({rs.d}, at::TensorOptions().dtype(rs.st));
  cpu_dispatch(rs, [&](auto r, auto z) {
    using T = decltype(z);
    garfield::cpu::combine<T>(r, w, out.data_ptr<T>());
    return 0;
  });
  return out;
}

at::Tensor c_coordwise(const RowSet& rs, int mode, int f, int beta, const c10::optional<at::Tensor>& W, int t,
                       uint64_t seed, double p) {
  std::vector<float> w;
  if (mode == garfield::kBulyanTail) {
    TORCH_CHECK(W.has_value(), "garfield: Bulyan tail needs W");
    w = floats_from(*W);
    TORCH_CHECK(static_cast<int64_t>(w.size()) >= static_cast<int64_t>(t) * rs.n, "garfield: W too small");
  }
  auto out = at::empty({rs.d}, at::TensorOptions().dtype(rs.st));
  cpu_dispatch(rs, [&](auto r, auto z) {
    using T = decltype(z);
    garfield::cpu::coordwise<T>(r, mode, static_cast<size_t>(f), static_cast<size_t>(beta), w,
                                static_cast<size_t>(t), seed, garfield::bernoulli_threshold(p), out.data_ptr<T>());
    return 0;
  });
  return out;
}

at::Tensor c_sqdist(const RowSet& rs, const at::Tensor& center) {
  auto c = center.to(rs.st).contiguous();
  TORCH_CHECK(c.numel() == rs.d, "garfield: centre size mismatch");
  return cpu_dispatch(rs, [&](auto r, auto z) {
    using T = decltype(z);
    auto v = garfield::cpu::sqdist_to<T>(r, c.data_ptr<T>());
    auto t = at::empty({rs.n}, at::TensorOptions().dtype(at::kDouble));
    std::copy(v.begin(), v.end(), t.data_ptr<double>());
    return t;
  });
}

// ------------------------------------------------- worker-grouped layers ----
// Every shape, dtype, device and alignment the kernels assume is checked here,
// on the host, before anything is launched.

void check_bf16_rows(const at::Tensor& t, const at::Device& dev, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.device() == dev && t.scalar_type() == at::kBFloat16,
              "garfield: ", what, " must be a bf16 tensor on ", dev);
  TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), "garfield: ", what, " must be a contiguous [rows, C] matrix");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "garfield: ", what, " must be 16-byte aligned");
}

// Activation rows of the grouped layers: bf16, or fp32 for the reference-precision step; every
// tensor of one call must share x's dtype. Returns the dtype code.
int check_act_rows(const at::Tensor& t, const at::Device& dev, const char* what, int want = -1) {
  TORCH_CHECK(t.is_cuda() && t.device() == dev &&
                  (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat),
              "garfield: ", what, " must be a bf16 or fp32 tensor on ", dev);
  TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), "garfield: ", what, " must be a contiguous [rows, C] matrix");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "garfield: ", what, " must be 16-byte aligned");
  const int dt = t.scalar_type() == at::kFloat ? garfield::kF32 : garfield::kBF16;
  TORCH_CHECK(want < 0 || dt == want, "garfield: ", what, " must have x's dtype");
  return dt;
}

const uint16_t* u16(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* u16_mut(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

float* opt_vec(const c10::optional<at::Tensor>& t, int64_t numel, const at::Device& dev, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->device() == dev && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == numel,
              "garfield: ", what, " must be a contiguous fp32 tensor of ", numel, " elements on ", dev);
  return t->data_ptr<float>();
}

float* ws_vec(const at::Tensor& t, int64_t numel, const at::Device& dev, const char* what) {
  TORCH_CHECK(t.device() == dev && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() >= numel,
              "garfield: ", what, " must be a contiguous fp32 tensor of >= ", numel, " elements on ", dev);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "garfield: ", what, " must be 16-byte aligned");
  return t.data_ptr<float>();
}

int64_t bn_groups(const at::Tensor& x, int64_t groups) {
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(groups >= 1 && R > 0 && R % groups == 0, "garfield bn: ", R, " rows do not split into ", groups,
              " equal worker groups");
  TORCH_CHECK(C > 0 && C % 8 == 0, "garfield bn: the channel count must be a positive multiple of 8, got ", C);
  return R / groups;
}

// One bit per element of the [R, C] rows (C % 8 == 0 by check_bf16_rows): a uint8 tensor of R*C/8 bytes.
void check_relu_mask(const at::Tensor& mask, const at::Tensor& x) {
  TORCH_CHECK(mask.device() == x.device() && mask.scalar_type() == at::kByte && mask.is_contiguous() &&
                  mask.numel() * 8 == x.numel(),
              "garfield bn: the ReLU mask must be a contiguous uint8 tensor of numel(x) / 8 bytes on x's device");
}

void g_bn_forward(const at::Tensor& x, const c10::optional<at::Tensor>& res, int64_t groups,
                  const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta, double eps,
                  double momentum, const c10::optional<at::Tensor>& run_mean,
                  const c10::optional<at::Tensor>& run_var, const at::Tensor& part, const at::Tensor& mean,
                  const at::Tensor& istd, const at::Tensor& scale, const at::Tensor& shift,
                  const c10::optional<at::Tensor>& y, bool relu, const c10::optional<at::Tensor>& mask,
                  bool defer_running,
                  const c10::optional<at::Tensor>& tile_stats, int64_t tile_m, int64_t tile_e,
                  const c10::optional<at::Tensor>& res_scale, const c10::optional<at::Tensor>& res_shift) {
  const auto dev = x.device();
  const int dt = check_act_rows(x, dev, "x");
  void* yp = nullptr;
  if (y.has_value() && y->defined()) {
    check_act_rows(*y, dev, "y", dt);
    TORCH_CHECK(y->sizes() == x.sizes(), "garfield bn: y must have x's shape");
    yp = y->data_ptr();
  }
  uint8_t* mp = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(yp != nullptr, "garfield bn: a ReLU mask comes with the apply pass (y)");
    TORCH_CHECK(relu, "garfield bn: a ReLU mask needs relu=True");
    check_relu_mask(*mask, x);
    mp = static_cast<uint8_t*>(mask->data_ptr());
  }
  const int64_t rg = bn_groups(x, groups);
  const int64_t C = x.size(1);
  const void* r = nullptr;
  if (res.has_value() && res->defined()) {
    check_act_rows(*res, dev, "res", dt);
    TORCH_CHECK(res->sizes() == x.sizes(), "garfield bn: the residual must have x's shape");
    r = res->data_ptr();
  }
  const int G = static_cast<int>(groups);
  float* pw = ws_vec(part, garfield::gpu::bn_part_floats(rg, G, static_cast<int>(C)), dev, "part");
  float* m = ws_vec(mean, groups * C, dev, "mean");
  float* is = ws_vec(istd, groups * C, dev, "istd");
  float* sc = ws_vec(scale, groups * C, dev, "scale");
  float* sh = ws_vec(shift, groups * C, dev, "shift");
  const float* g = opt_vec(gamma, C, dev, "gamma");
  const float* b = opt_vec(beta, C, dev, "beta");
  float* rm = opt_vec(run_mean, C, dev, "running_mean");
  float* rv = opt_vec(run_var, C, dev, "running_var");
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "garfield bn: pass both running statistics or neither");
  const float* ts = nullptr;
  if (tile_stats.has_value() && tile_stats->defined()) {
    TORCH_CHECK(tile_m > 0 && tile_m <= rg, "garfield bn: tile statistics need 0 < tile_m <= rows per worker");
    TORCH_CHECK(tile_e >= 1, "garfield bn: tile_e must be >= 1");
    const int64_t tiles = (x.size(0) + tile_m - 1) / tile_m;
    ts = ws_vec(*tile_stats, tiles * tile_e * 6 * C, dev, "tile_stats");
  }
  const float* rsc = opt_vec(res_scale, groups * C, dev, "res_scale");
  const float* rsh = opt_vec(res_shift, groups * C, dev, "res_shift");
  TORCH_CHECK((rsc == nullptr) == (rsh == nullptr), "garfield bn: pass both res_scale and res_shift or neither");
  TORCH_CHECK(rsc == nullptr || (r != nullptr && yp != nullptr), "garfield bn: res_scale needs res and y");
  TORCH_CHECK(rsc == nullptr || (reinterpret_cast<uintptr_t>(rsc) % 16 == 0 && reinterpret_cast<uintptr_t>(rsh) % 16 == 0),
              "garfield bn: res_scale / res_shift must be 16-byte aligned");
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::bn_forward(x.data_ptr(), r, rg, G, static_cast<int>(C), g, b, static_cast<float>(eps),
                            static_cast<float>(momentum), rm, rv, pw, m, is, sc, sh, yp, relu, mp,
                            defer_running, stream_of(dev), ts, tile_m, static_cast<int>(tile_e), dt, rsc, rsh);
}

// Backward of a projection block's last BatchNorm (a) and its folded shortcut BatchNorm (b) sharing dz
// (every shape: the small layers on the single-kernel dual path, the others on one statistics + one apply pass).
void g_bn_backward_dual(const at::Tensor& xa, const at::Tensor& xb, const at::Tensor& dy,
                        const c10::optional<at::Tensor>& mask, int64_t groups, const c10::optional<at::Tensor>& gamma_a,
                        const c10::optional<at::Tensor>& gamma_b, const at::Tensor& mean_a, const at::Tensor& istd_a,
                        const at::Tensor& mean_b, const at::Tensor& istd_b, const at::Tensor& part_a,
                        const at::Tensor& part_b, const at::Tensor& coef_a, const at::Tensor& coef_b,
                        const at::Tensor& dxa, const at::Tensor& dxb, const c10::optional<at::Tensor>& grow,
                        int64_t row_stride, int64_t og_a, int64_t ob_a, int64_t og_b, int64_t ob_b) {
  const auto dev = xa.device();
  const int dt = check_act_rows(xa, dev, "xa");
  for (const at::Tensor* t : {&xb, &dy, &dxa, &dxb}) {
    check_act_rows(*t, dev, "dual operand", dt);
    TORCH_CHECK(t->sizes() == xa.sizes(), "garfield bn dual: operands must have xa's shape");
  }
  const int64_t rg = bn_groups(xa, groups);
  const int64_t C = xa.size(1);
  {
    const uint8_t* mp = nullptr;
    if (mask.has_value() && mask->defined()) {
      check_relu_mask(*mask, xa);
      mp = static_cast<const uint8_t*>(mask->data_ptr());
    }
    const int G = static_cast<int>(groups);
    const int64_t pn = garfield::gpu::bn_part_floats(rg, G, static_cast<int>(C));
    float* pa = ws_vec(part_a, pn, dev, "part_a");
    float* pb = ws_vec(part_b, pn, dev, "part_b");
    float* ca = ws_vec(coef_a, 3 * groups * C, dev, "coef_a");
    float* cb = ws_vec(coef_b, 3 * groups * C, dev, "coef_b");
    void* gp = nullptr;
    int gdt = garfield::kF32;
    if (grow.has_value() && grow->defined()) {
      TORCH_CHECK(grow->device() == dev && grow->is_contiguous(), "garfield bn dual: grow must be contiguous");
      gdt = dtype_code(*grow);
      TORCH_CHECK(gdt != garfield::kF64, "garfield bn dual: grow must be fp32, bf16 or fp16");
      for (int64_t off : {og_a, ob_a, og_b, ob_b})
        if (off >= 0)
          TORCH_CHECK(row_stride >= 0 && (groups - 1) * row_stride + off + C <= grow->numel(),
                      "garfield bn dual: grow offset ", off, " out of bounds");
      gp = grow->data_ptr();
    }
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::bn_backward_dual(
        xa.data_ptr(), xb.data_ptr(), dy.data_ptr(), mp, rg, G, static_cast<int>(C), opt_vec(gamma_a, C, dev, "gamma_a"),
        opt_vec(gamma_b, C, dev, "gamma_b"), ws_vec(mean_a, groups * C, dev, "mean_a"),
        ws_vec(istd_a, groups * C, dev, "istd_a"), ws_vec(mean_b, groups * C, dev, "mean_b"),
        ws_vec(istd_b, groups * C, dev, "istd_b"), pa, pb, ca, cb, dxa.data_ptr(), dxb.data_ptr(), gp, gdt, row_stride,
        og_a, ob_a, og_b, ob_b, stream_of(dev), dt);
  }
}

}  // namespace

namespace garfield {
namespace gpu {
// Experiment switches of kernel forms under measurement (A/B runs set them; 0 is the default form).
static std::map<std::string, int>& variant_table() {
  static std::map<std::string, int> m;
  return m;
}
int kernel_variant(const char* name) {
  const auto& m = variant_table();
  const auto it = m.find(name);
  return it == m.end() ? 0 : it->second;
}
}  // namespace gpu
}  // namespace garfield

namespace {
int xent_dtype(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 2, "gpu_xent: ", what, " must be a contiguous 2-D GPU tensor");
  if (t.scalar_type() == at::kFloat) return garfield::kF32;
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "gpu_xent: ", what, " must be fp32 or bf16");
  return garfield::kBF16;
}

void g_xent_forward(const at::Tensor& logits, const at::Tensor& labels, int64_t groups, const at::Tensor& loss,
                    const at::Tensor& dlogits) {
  const int dt = xent_dtype(logits, "logits");
  TORCH_CHECK(xent_dtype(dlogits, "dlogits") == dt && dlogits.sizes() == logits.sizes(), "gpu_xent: dlogits shape/dtype");
  const int64_t N = logits.size(0), nc = logits.size(1);
  TORCH_CHECK(groups > 0 && N % groups == 0, "gpu_xent: rows not divisible into groups");
  TORCH_CHECK(nc >= 1, "gpu_xent: at least one class");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == N,
              "gpu_xent: labels must be a contiguous int64 GPU tensor of N entries");
  TORCH_CHECK(loss.is_cuda() && loss.scalar_type() == at::kFloat && loss.is_contiguous() && loss.numel() == groups,
              "gpu_xent: loss must be a contiguous fp32 GPU tensor of `groups` entries");
  const auto dev = logits.device();
  TORCH_CHECK(labels.device() == dev && loss.device() == dev && dlogits.device() == dev, "gpu_xent: one device");
  c10::hip::HIPGuard guard(dev.index());
  at::Tensor rowloss;   // wide heads: per-row losses (caching allocator: graph-capture safe)
  if (nc > garfield::gpu::kXentMaxClasses) rowloss = at::empty({N}, logits.options().dtype(at::kFloat));
  garfield::gpu::xent_forward(logits.data_ptr(), dt, labels.data_ptr<int64_t>(), N / groups, static_cast<int>(groups),
                              static_cast<int>(nc), loss.data_ptr<float>(), dlogits.data_ptr(), stream_of(dev),
                              rowloss.defined() ? rowloss.data_ptr<float>() : nullptr);
}

at::Tensor g_mean_f32(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.numel() >= 1,
              "gpu_mean_f32: a non-empty contiguous fp32 GPU tensor");
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor out = at::empty({}, x.options());
  garfield::gpu::mean_f32(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), stream_of(x.device()));
  return out;
}

void g_xent_backward(const at::Tensor& dlogits, const at::Tensor& grad_loss, int64_t groups, const at::Tensor& dx) {
  const int dt = xent_dtype(dlogits, "dlogits");
  TORCH_CHECK(xent_dtype(dx, "dx") == dt && dx.sizes() == dlogits.sizes(), "gpu_xent: dx shape/dtype");
  const int64_t N = dlogits.size(0), nc = dlogits.size(1);
  TORCH_CHECK(groups > 0 && N % groups == 0, "gpu_xent: rows not divisible into groups");
  TORCH_CHECK(grad_loss.is_cuda() && grad_loss.scalar_type() == at::kFloat && grad_loss.is_contiguous() &&
                  grad_loss.numel() == groups, "gpu_xent: grad_loss must be a contiguous fp32 GPU tensor of `groups`");
  const auto dev = dlogits.device();
  TORCH_CHECK(grad_loss.device() == dev && dx.device() == dev, "gpu_xent: one device");
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::xent_backward(dlogits.data_ptr(), dt, grad_loss.data_ptr<float>(), N / groups,
                               static_cast<int>(groups), static_cast<int>(nc), dx.data_ptr(), stream_of(dev));
}

void g_bn_running_update(const std::vector<py::tuple>& jobs) {
  garfield::gpu::RunJobs rj{};
  c10::Device dev = c10::Device(c10::kCPU);
  size_t i = 0;
  auto flush = [&]() {
    if (rj.n == 0) return;
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::bn_running_update(rj, stream_of(dev));
    rj.n = 0;
  };
  for (; i < jobs.size(); ++i) {
    const auto& t = jobs[i];
    TORCH_CHECK(t.size() == 7, "gpu_bn_running_update: each job is (mean, istd, running_mean, running_var, rg, eps, "
                "momentum)");
    auto mean = t[0].cast<at::Tensor>(), istd = t[1].cast<at::Tensor>();
    auto rm = t[2].cast<at::Tensor>(), rv = t[3].cast<at::Tensor>();
    const int64_t rg = t[4].cast<int64_t>();
    if (i == 0) dev = mean.device();
    TORCH_CHECK(mean.device() == dev && mean.is_cuda(), "gpu_bn_running_update: all jobs on one device");
    const int64_t C = rm.numel();
    TORCH_CHECK(C > 0 && mean.numel() % C == 0 && istd.numel() == mean.numel() && rv.numel() == C, "gpu_bn_running_update: shapes");
    float* pm = ws_vec(mean, mean.numel(), dev, "mean");
    float* pi = ws_vec(istd, istd.numel(), dev, "istd");
    float* prm = ws_vec(rm, C, dev, "running_mean");
    float* prv = ws_vec(rv, C, dev, "running_var");
    rj.j[rj.n++] = garfield::gpu::RunJob{pm, pi, prm, prv, rg, static_cast<int>(C),
                                         static_cast<int>(mean.numel() / C), static_cast<float>(t[5].cast<double>()),
                                         static_cast<float>(t[6].cast<double>())};
    if (rj.n == garfield::gpu::kRunJobs) flush();
  }
  flush();
}

void g_bn_backward(const at::Tensor& x, const at::Tensor& dy, const c10::optional<at::Tensor>& y, int64_t groups,
                   const c10::optional<at::Tensor>& gamma, const at::Tensor& mean, const at::Tensor& istd,
                   const at::Tensor& part, const at::Tensor& coef, const at::Tensor& dx,
                   const c10::optional<at::Tensor>& dres, const c10::optional<at::Tensor>& grow, int64_t row_stride,
                   int64_t off_gamma, int64_t off_beta, const c10::optional<at::Tensor>& rscale,
                   const c10::optional<at::Tensor>& rshift) {
  const auto dev = x.device();
  const int dt = check_act_rows(x, dev, "x");
  check_act_rows(dy, dev, "dy", dt);
  check_act_rows(dx, dev, "dx", dt);
  TORCH_CHECK(dy.sizes() == x.sizes() && dx.sizes() == x.sizes(), "garfield bn: dy/dx must have x's shape");
  const int64_t rg = bn_groups(x, groups);
  const int64_t C = x.size(1);
  const void* yp = nullptr;
  const uint8_t* mp = nullptr;
  if (y.has_value() && y->defined()) {
    if (y->scalar_type() == at::kByte) {   // the forward's ReLU bit mask
      check_relu_mask(*y, x);
      mp = static_cast<const uint8_t*>(y->data_ptr());
    } else {
      check_act_rows(*y, dev, "y", dt);
      TORCH_CHECK(y->sizes() == x.sizes(), "garfield bn: y must have x's shape");
      yp = y->data_ptr();
    }
  }
  void* dr = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_act_rows(*dres, dev, "dres", dt);
    TORCH_CHECK(dres->sizes() == x.sizes(), "garfield bn: dres must have x's shape");
    dr = dres->data_ptr();
  }
  const int G = static_cast<int>(groups);
  float* pw = ws_vec(part, garfield::gpu::bn_part_floats(rg, G, static_cast<int>(C)), dev, "part");
  float* cw = ws_vec(coef, 3 * groups * C, dev, "coef");
  const float* m = ws_vec(mean, groups * C, dev, "mean");
  const float* is = ws_vec(istd, groups * C, dev, "istd");
  const float* g = opt_vec(gamma, C, dev, "gamma");
  void* gp = nullptr;
  int gdt = garfield::kF32;
  if (grow.has_value() && grow->defined()) {
    TORCH_CHECK(grow->device() == dev && grow->is_contiguous(), "garfield bn: grow must be contiguous on ", dev);
    gdt = dtype_code(*grow);
    TORCH_CHECK(gdt != garfield::kF64, "garfield bn: grow must be fp32, bf16 or fp16");
    TORCH_CHECK(row_stride >= 0 && off_gamma >= -1 && off_beta >= -1, "garfield bn: invalid grow offsets");
    for (int64_t off : {off_gamma, off_beta})
      if (off >= 0)
        TORCH_CHECK((groups - 1) * row_stride + off + C <= grow->numel(), "garfield bn: grow offset ", off,
                    " + ", groups, " rows of stride ", row_stride, " is out of bounds (", grow->numel(), ")");
    gp = grow->data_ptr();
  }
  const float* rs = opt_vec(rscale, groups * C, dev, "relu scale");
  const float* rf = opt_vec(rshift, groups * C, dev, "relu shift");
  TORCH_CHECK((rs == nullptr) == (rf == nullptr), "garfield bn: pass both the ReLU scale and shift or neither");
  TORCH_CHECK(rs == nullptr || (yp == nullptr && mp == nullptr),
              "garfield bn: the ReLU test from (scale, shift) replaces y / the mask");
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::bn_backward(x.data_ptr(), dy.data_ptr(), yp, mp, rg, G, static_cast<int>(C), g, m, is, pw, cw,
                             dx.data_ptr(), dr, gp, gdt, row_stride, off_gamma, off_beta, stream_of(dev), dt, rs, rf);
}

garfield::gpu::Im2col conv_geometry(const at::Tensor& x, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph,
                                    int64_t pw, int64_t dh, int64_t dw, bool allow_f32 = false) {
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kBFloat16 || (allow_f32 && x.scalar_type() == at::kFloat)) &&
                  x.dim() == 4,
              "garfield im2col: x must be a 4-D bf16", allow_f32 ? " or fp32" : "", " device tensor");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "garfield im2col: x must be channels_last");
  TORCH_CHECK(kh >= 1 && kw >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0 && dh >= 1 && dw >= 1,
              "garfield im2col: invalid kernel geometry");
  garfield::gpu::Im2col g{};
  g.N = static_cast<int>(x.size(0));
  g.C = static_cast<int>(x.size(1));
  g.H = static_cast<int>(x.size(2));
  g.W = static_cast<int>(x.size(3));
  g.KH = static_cast<int>(kh); g.KW = static_cast<int>(kw);
  g.sh = static_cast<int>(sh); g.sw = static_cast<int>(sw);
  g.ph = static_cast<int>(ph); g.pw = static_cast<int>(pw);
  g.dh = static_cast<int>(dh); g.dw = static_cast<int>(dw);
  g.Ho = static_cast<int>((x.size(2) + 2 * ph - dh * (kh - 1) - 1) / sh + 1);
  g.Wo = static_cast<int>((x.size(3) + 2 * pw - dw * (kw - 1) - 1) / sw + 1);
  TORCH_CHECK(g.Ho >= 1 && g.Wo >= 1, "garfield im2col: empty output");
  TORCH_CHECK(x.numel() <= INT32_MAX && static_cast<int64_t>(g.N) * g.Ho * g.Wo <= INT32_MAX,
              "garfield im2col: problem too large for 32-bit pixel indexing");
  TORCH_CHECK(kh * kw * g.C <= INT32_MAX / 256, "garfield im2col: kernel too large");
  return g;
}

void check_col(const at::Tensor& col, const at::Tensor& x, garfield::gpu::Im2col& g) {
  const int64_t rows = static_cast<int64_t>(g.N) * g.Ho * g.Wo;
  const int64_t K = static_cast<int64_t>(g.KH) * g.KW * g.C;
  TORCH_CHECK(col.device() == x.device() && col.scalar_type() == at::kBFloat16 && col.is_contiguous() &&
                  col.dim() == 2 && col.size(0) == rows && col.size(1) >= K && col.size(1) <= INT32_MAX / 256,
              "garfield im2col: col must be a contiguous bf16 [", rows, ", >= ", K, "] tensor on x's device");
  g.ldc = static_cast<int>(col.size(1));
  if (g.C % 8 == 0)
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(col.data_ptr()) % 16 == 0,
                "garfield im2col: x and col must be 16-byte aligned");
}

void g_im2col(const at::Tensor& x, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
              int64_t dh, int64_t dw, const at::Tensor& col) {
  auto g = conv_geometry(x, kh, kw, sh, sw, ph, pw, dh, dw);
  check_col(col, x, g);
  c10::hip::HIPGuard guard(x.device().index());
  garfield::gpu::im2col_nhwc(u16(x), g, u16_mut(col), stream_of(x.device()));
}

// dx: the (channels_last, bf16) input-shaped output; dcol: [N*Ho*Wo, ldc] bf16
void g_col2im(const at::Tensor& dcol, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
              int64_t dh, int64_t dw, const at::Tensor& dx, bool accumulate) {
  auto g = conv_geometry(dx, kh, kw, sh, sw, ph, pw, dh, dw);
  check_col(dcol, dx, g);
  c10::hip::HIPGuard guard(dx.device().index());
  garfield::gpu::col2im_nhwc(u16(dcol), g, u16_mut(dx), accumulate, stream_of(dx.device()));
}

// Small-image 3x3 convolutions as dense GEMMs (sconv_nhwc.hip): the per-step weight expansion of every
// such layer (one launch) and the fold of a dense weight gradient onto the nine taps.
void g_sc_expand(const std::vector<at::Tensor>& ws, const std::vector<int64_t>& hs, const std::vector<int64_t>& wds,
                 const std::vector<at::Tensor>& bigs, const std::vector<at::Tensor>& bigTs) {
  const size_t n = ws.size();
  TORCH_CHECK(hs.size() == n && wds.size() == n && bigs.size() == n && bigTs.size() == n,
              "gpu_sc_expand: one H, W, Wbig and Wbigᵀ per weight");
  if (n == 0) return;
  c10::hip::HIPGuard guard(ws[0].device().index());
  garfield::gpu::ScExpandJobs jobs{};
  auto flush = [&]() {
    if (jobs.count) garfield::gpu::sc_expand(jobs, stream_of(ws[0].device()));
    jobs = garfield::gpu::ScExpandJobs{};
  };
  for (size_t k = 0; k < n; ++k) {
    const auto& w = ws[k];
    const int64_t H = hs[k], W = wds[k];
    TORCH_CHECK(w.is_cuda() && w.device() == ws[0].device() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 &&
                    w.size(2) == 3 && w.size(3) == 3 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_sc_expand: weights must be channels_last bf16 [Cout, Cin, 3, 3] on one device");
    const int64_t co = w.size(0), ci = w.size(1), P = H * W;
    TORCH_CHECK(H >= 1 && H <= 2 && W >= 1 && W <= 2 && ci % 8 == 0 && co % 8 == 0,
                "gpu_sc_expand: H, W in {1, 2}, Cin % 8 == 0, Cout % 8 == 0");
    for (const auto* t : {&bigs[k], &bigTs[k]})
      TORCH_CHECK(t->device() == w.device() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                      t->numel() == P * co * P * ci,
                  "gpu_sc_expand: Wbig / Wbigᵀ must be contiguous bf16 of ", P * co, " x ", P * ci, " elements");
    TORCH_CHECK(bigs[k].dim() == 2 && bigs[k].size(0) == P * co && bigTs[k].dim() == 2 && bigTs[k].size(0) == P * ci,
                "gpu_sc_expand: Wbig is [P*Cout, P*Cin], Wbigᵀ [P*Cin, P*Cout]");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(bigs[k].data_ptr()) % 16 == 0,
                "gpu_sc_expand: 16-byte aligned weight and Wbig");
    if (jobs.count == garfield::gpu::kScMaxJobs) flush();
    auto& J = jobs.job[jobs.count];
    J.w = u16(w);
    J.big = u16_mut(bigs[k]);
    J.bigT = u16_mut(bigTs[k]);
    J.cout = static_cast<int>(co);
    J.cin = static_cast<int>(ci);
    J.H = static_cast<int>(H);
    J.W = static_cast<int>(W);
    jobs.start[jobs.count + 1] = jobs.start[jobs.count] + P * co * P * ci / 8;
    ++jobs.count;
  }
  flush();
}

void g_sc_fold(const at::Tensor& slab, int64_t H, int64_t W, const at::Tensor& out) {
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.dim() == 4 && slab.is_contiguous(),
              "gpu_sc_fold: slab must be a contiguous fp32 [S, G, P*Cout, P*Cin] device tensor");
  TORCH_CHECK(out.device() == slab.device() && (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat) &&
                  out.dim() == 3 && out.stride(2) == 1 && out.stride(1) == out.size(2),
              "gpu_sc_fold: out must be a bf16 / fp32 [G, Cout, 9*Cin] view with dense rows");
  const int64_t P = H * W, S = slab.size(0), G = slab.size(1), co = out.size(1), ci = out.size(2) / 9;
  TORCH_CHECK(H >= 1 && H <= 2 && W >= 1 && W <= 2 && out.size(2) == 9 * ci && ci % 8 == 0 && out.size(0) == G &&
                  slab.size(2) == P * co && slab.size(3) == P * ci,
              "gpu_sc_fold: shapes do not match (slab [S, G, P*Cout, P*Cin], out [G, Cout, 9*Cin])");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 && (out.stride(0) * out.element_size()) % 16 == 0,
              "gpu_sc_fold: out rows must be 16-byte aligned");
  c10::hip::HIPGuard guard(slab.device().index());
  garfield::gpu::sc_fold(slab.data_ptr<float>(), static_cast<int>(S), static_cast<int>(G), static_cast<int>(H),
                         static_cast<int>(W), static_cast<int>(co), static_cast<int>(ci), out.data_ptr(),
                         out.scalar_type() == at::kBFloat16, out.stride(0), stream_of(slab.device()));
}

// Data gradient of a stride-2 convolution on the parity-class kernel (iconv_nhwc.hip):
// dx (+)= conv_transpose(dy, w); dy/dx/add channels_last bf16, w the channels_last forward weight.
garfield::gpu::Im2col s2_geometry(const at::Tensor& dy, const at::Tensor& dx, int64_t kh, int64_t kw, int64_t ph,
                                  int64_t pw) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dx.is_cuda() && dx.device() == dy.device() &&
                  dx.scalar_type() == at::kBFloat16 && dx.dim() == 4 && dx.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dx.size(0) == dy.size(0),
              "gpu_dgrad_s2: dy and dx must be channels_last bf16 device tensors of one batch");
  garfield::gpu::Im2col g{};
  g.N = static_cast<int>(dy.size(0));
  g.C = static_cast<int>(dy.size(1));
  g.H = static_cast<int>(dy.size(2));
  g.W = static_cast<int>(dy.size(3));
  g.Ho = static_cast<int>(dx.size(2));
  g.Wo = static_cast<int>(dx.size(3));
  g.KH = static_cast<int>(kh); g.KW = static_cast<int>(kw);
  g.sh = g.sw = 2;
  g.ph = static_cast<int>(ph); g.pw = static_cast<int>(pw);
  g.dh = g.dw = 1;
  return g;
}

bool g_dgrad_s2_ok(const at::Tensor& dy, const at::Tensor& dx, int64_t kh, int64_t kw, int64_t ph, int64_t pw) {
  return garfield::gpu::dgrad_s2_ok(s2_geometry(dy, dx, kh, kw, ph, pw), static_cast<int>(dx.size(1)));
}

void g_dgrad_s2(const at::Tensor& dy, const at::Tensor& w, int64_t kh, int64_t kw, int64_t ph, int64_t pw,
                const at::Tensor& dx, const c10::optional<at::Tensor>& add, int64_t pm) {
  auto g = s2_geometry(dy, dx, kh, kw, ph, pw);
  const int64_t cout = dx.size(1);
  TORCH_CHECK(garfield::gpu::dgrad_s2_ok(g, static_cast<int>(cout)),
              "gpu_dgrad_s2: needs a stride-2 geometry with even dx sides, C % 64 == 0, Cout % 64 == 0, k <= 3, pad <= 1");
  TORCH_CHECK(w.device() == dy.device() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == g.C &&
                  w.size(1) == cout && w.size(2) == kh && w.size(3) == kw && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gpu_dgrad_s2: w must be the channels_last bf16 forward weight [", g.C, ", ", cout, ", ", kh, ", ", kw, "]");
  const uint16_t* ap = nullptr;
  if (add.has_value()) {
    const auto& a = *add;
    TORCH_CHECK(a.device() == dx.device() && a.scalar_type() == at::kBFloat16 && a.sizes() == dx.sizes() &&
                    a.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_dgrad_s2: add must be a channels_last bf16 tensor shaped like dx");
    ap = u16(a);
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dx.data_ptr()) % 8 == 0 &&
                  (ap == nullptr || reinterpret_cast<uintptr_t>(ap) % 8 == 0),
              "gpu_dgrad_s2: dy and w must be 16-byte aligned, dx and add 8-byte aligned");
  TORCH_CHECK(dy.numel() < INT32_MAX && static_cast<int64_t>(g.N) * g.Ho * g.Wo < INT32_MAX, "gpu_dgrad_s2: tensor too large");
  c10::hip::HIPGuard guard(dy.device().index());
  garfield::gpu::dgrad_s2_nhwc(u16(dy), u16(w), g, static_cast<int>(cout), u16_mut(dx), ap, static_cast<int>(pm),
                               stream_of(dy.device()));
}

// Implicit-GEMM convolution: y = conv(x, w) (+ add); x/y/add channels_last bf16, w the
// [Cout, KH, KW, C]-ordered weight (a channels_last 4-D weight or its [Cout, K] matrix).
bool g_iconv(const at::Tensor& x, const at::Tensor& w, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph,
             int64_t pw, int64_t dh, int64_t dw, const at::Tensor& y, const c10::optional<at::Tensor>& add,
             int64_t pm, bool transpose_w, const c10::optional<at::Tensor>& stats, int64_t rg,
             const c10::optional<at::Tensor>& add_mask) {
  auto g = conv_geometry(x, kh, kw, sh, sw, ph, pw, dh, dw);
  TORCH_CHECK(g.C % 32 == 0, "gpu_iconv: input channels must be a multiple of 32 (got ", g.C, ")");
  TORCH_CHECK(y.is_cuda() && y.device() == x.device() && y.scalar_type() == at::kBFloat16 && y.dim() == 4 &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gpu_iconv: y must be a channels_last bf16 tensor on x's device");
  const int64_t cout = y.size(1);
  TORCH_CHECK(cout % 64 == 0, "gpu_iconv: output channels must be a multiple of 64 (got ", cout, ")");
  TORCH_CHECK(y.size(0) == g.N && y.size(2) == g.Ho && y.size(3) == g.Wo, "gpu_iconv: y must be [", g.N, ", Cout, ",
              g.Ho, ", ", g.Wo, "]");
  const int64_t K = static_cast<int64_t>(g.KH) * g.KW * g.C;
  TORCH_CHECK(w.device() == x.device() && w.scalar_type() == at::kBFloat16 && w.numel() == cout * K,
              "gpu_iconv: w must be a bf16 weight of ", cout, " x ", K, " elements on x's device");
  if (transpose_w) {
    TORCH_CHECK(g.C % 64 == 0, "gpu_iconv: transpose_w needs C % 64 == 0");
    TORCH_CHECK(w.dim() == 4 && w.size(0) == g.C && w.size(1) == cout && w.size(2) == g.KH && w.size(3) == g.KW &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_iconv: with transpose_w, w must be the channels_last forward weight [C, Cout, KH, KW]");
  } else if (w.dim() == 4) {
    TORCH_CHECK(w.size(0) == cout && w.size(1) == g.C && w.size(2) == g.KH && w.size(3) == g.KW &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_iconv: a 4-D weight must be channels_last [Cout, C, KH, KW]");
  } else {
    TORCH_CHECK(w.dim() == 2 && w.size(0) == cout && w.is_contiguous(), "gpu_iconv: a 2-D weight must be [Cout, K]");
  }
  const uint16_t* ap = nullptr;
  if (add.has_value()) {
    const auto& a = *add;
    TORCH_CHECK(a.device() == x.device() && a.scalar_type() == at::kBFloat16 && a.sizes() == y.sizes() &&
                    a.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_iconv: add must be a channels_last bf16 tensor shaped like y");
    ap = u16(a);
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0 &&
                  (ap == nullptr || reinterpret_cast<uintptr_t>(ap) % 8 == 0),
              "gpu_iconv: x and w must be 16-byte aligned, y and add 8-byte aligned");
  TORCH_CHECK(static_cast<int64_t>(g.N) * g.H * g.W * g.C < INT32_MAX && static_cast<int64_t>(g.N) * g.Ho * g.Wo < INT32_MAX,
              "gpu_iconv: tensor too large");
  float* sp = nullptr;
  if (stats.has_value()) {
    const auto& st = *stats;
    const int pmf = pm == 22 || pm == 24 ? static_cast<int>(pm - 20) : garfield::gpu::conv3x3_pick(g, static_cast<int>(cout));
    TORCH_CHECK(!transpose_w && !add.has_value() && pmf > 0 && (pm == 0 || pm == 22 || pm == 24),
                "gpu_iconv: stats need the halo-staged 3x3 kernel (no add, no transpose_w)");
    const int64_t M = static_cast<int64_t>(g.N) * g.Ho * g.Wo;
    const int64_t H = 16 * pmf;
    TORCH_CHECK(rg >= H && M % rg == 0, "gpu_iconv: stats need rg >= ", H, " rows per worker dividing ", M);
    TORCH_CHECK(st.is_cuda() && st.device() == x.device() && st.scalar_type() == at::kFloat && st.is_contiguous() &&
                    st.numel() >= (M + H - 1) / H * 6 * cout,
                "gpu_iconv: stats must be a contiguous fp32 tensor of ", (M + H - 1) / H * 6 * cout, " floats");
    sp = st.data_ptr<float>();
  }
  c10::hip::HIPGuard guard(x.device().index());
  if (sp) {
    TORCH_CHECK(garfield::gpu::conv3x3_nhwc(u16(x), u16(w), g, static_cast<int>(cout), u16_mut(y), nullptr,
                                            pm == 0 ? 0 : static_cast<int>(pm - 20), stream_of(x.device()), sp, rg),
                "gpu_iconv: the halo-staged kernel refused the statistics launch");
    return true;
  }
  static const bool c3 = [] {
    const char* e = std::getenv("GARFIELD_CONV3X3");
    return !(e && e[0] == '0');
  }();
  if (add_mask.has_value() && add_mask->defined()) {
    // add masked by a 1-bit-per-element mask (a BatchNorm's ReLU bits): the halo-staged kernel only;
    // false (nothing launched) when it does not take this launch, the caller then materialises
    const auto& mk = *add_mask;
    TORCH_CHECK(ap != nullptr, "gpu_iconv: add_mask needs add");
    TORCH_CHECK(mk.is_cuda() && mk.device() == x.device() && mk.scalar_type() == at::kByte && mk.is_contiguous() &&
                    mk.numel() * 8 == y.numel(),
                "gpu_iconv: add_mask must be a contiguous uint8 bit mask of y.numel() / 8 bytes");
    TORCH_CHECK(y.data_ptr() != ap, "gpu_iconv: with add_mask, y must not alias add");
    if (transpose_w || !(pm == 0 || pm == 22 || pm == 24) || !c3 ||
        garfield::gpu::conv3x3_pick(g, static_cast<int>(cout)) == 0)
      return false;
    return garfield::gpu::conv3x3_nhwc(u16(x), u16(w), g, static_cast<int>(cout), u16_mut(y), ap,
                                       pm == 0 ? 0 : static_cast<int>(pm - 20), stream_of(x.device()), nullptr, 0,
                                       mk.data_ptr<uint8_t>());
  }
  // pm 0 (auto): the halo-staged 3x3 kernel whenever it fits (GARFIELD_CONV3X3=0 disables it);
  // pm 22 / 24: force it with 2 / 4 pixel fragments per wave; 1..14: the implicit-GEMM kernel
  if (!transpose_w && (pm == 22 || pm == 24)) {
    TORCH_CHECK(garfield::gpu::conv3x3_pick(g, static_cast<int>(cout)) != 0 &&
                    garfield::gpu::conv3x3_nhwc(u16(x), u16(w), g, static_cast<int>(cout), u16_mut(y), ap,
                                                static_cast<int>(pm - 20), stream_of(x.device())),
                "gpu_iconv: pm ", pm, " (halo-staged 3x3 kernel) does not fit this shape");
    return true;
  }
  if (!transpose_w && pm == 0 && c3 &&
      garfield::gpu::conv3x3_nhwc(u16(x), u16(w), g, static_cast<int>(cout), u16_mut(y), ap, 0,
                                  stream_of(x.device())))
    return true;
  garfield::gpu::iconv_nhwc(u16(x), u16(w), g, static_cast<int>(cout), u16_mut(y), ap, static_cast<int>(pm),
                            transpose_w, stream_of(x.device()));
  return true;
}

int64_t g_conv3x3_pick(int64_t n, int64_t h, int64_t w, int64_t c, int64_t cout) {
  garfield::gpu::Im2col g{static_cast<int>(n), static_cast<int>(h), static_cast<int>(w), static_cast<int>(c), 3, 3,
                          1, 1, 1, 1, 1, 1, static_cast<int>(h), static_cast<int>(w), 0};
  return garfield::gpu::conv3x3_pick(g, static_cast<int>(cout));
}

// Row-major NT GEMM (gemm_nt.hip): c = a · bᵀ (+ add); a [M, K], b [N, K], c/add [M, N], all contiguous
// bf16 rows; stats (fp32, [ceil(M / BM)][2][2][N]): fused per-worker (rg rows) BatchNorm statistics.
void g_gemm_nt(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, const c10::optional<at::Tensor>& add,
               const c10::optional<at::Tensor>& stats, int64_t rg, int64_t cfg,
               const c10::optional<at::Tensor>& pro_scale, const c10::optional<at::Tensor>& pro_shift,
               int64_t pro_groups, const c10::optional<at::Tensor>& add_mask) {
  const auto dev = a.device();
  auto chk = [&](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.device() == dev && t.scalar_type() == at::kBFloat16 && t.dim() == 2 &&
                    t.stride(1) == 1 && t.stride(0) == t.size(1),
                "gpu_gemm_nt: ", what, " must be contiguous 2-D bf16 rows on a's device");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "gpu_gemm_nt: ", what, " must be 16-byte aligned");
  };
  chk(a, "a");
  chk(b, "b");
  chk(c, "c");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && c.size(0) == M && c.size(1) == N, "gpu_gemm_nt: shapes a [M, K], b [N, K], c [M, N]");
  TORCH_CHECK(K % 64 == 0 && K > 0, "gpu_gemm_nt: K must be a positive multiple of 64 (got ", K, ")");
  TORCH_CHECK(M * std::max(K, N) < INT32_MAX, "gpu_gemm_nt: too large");
  const uint16_t* ap = nullptr;
  if (add.has_value() && add->defined()) {
    chk(*add, "add");
    TORCH_CHECK(add->sizes() == c.sizes(), "gpu_gemm_nt: add must be shaped like c");
    ap = u16(*add);
  }
  float* sp = nullptr;
  const bool want_stats = stats.has_value() && stats->defined();
  if (want_stats) {
    TORCH_CHECK(ap == nullptr, "gpu_gemm_nt: statistics and add are exclusive");
    TORCH_CHECK(rg > 0 && M % rg == 0, "gpu_gemm_nt: statistics need M to split into rg-row workers");
  }
  if (cfg < 0) cfg = garfield::gpu::gemm_nt_pick(M, static_cast<int>(N), static_cast<int>(K), want_stats ? rg : 0);
  TORCH_CHECK(garfield::gpu::gemm_nt_valid(static_cast<int>(cfg), static_cast<int>(N), static_cast<int>(K)),
              "gpu_gemm_nt: no tile configuration ", cfg, " for N = ", N, ", K = ", K);
  if (want_stats) {
    const int sr = garfield::gpu::gemm_nt_stats_rows(static_cast<int>(cfg));
    TORCH_CHECK(sr <= rg, "gpu_gemm_nt: statistics tile of ", sr, " rows spans more than two workers of ", rg, " rows");
    int64_t H = 0;
    int E = 0;
    garfield::gpu::gemm_nt_stats_geometry(static_cast<int>(cfg), M, static_cast<int>(N), static_cast<int>(K), rg, &H, &E);
    sp = ws_vec(*stats, ((M + H - 1) / H) * E * 6 * N, dev, "stats");
  }
  const float* psc = nullptr;
  const float* psh = nullptr;
  int64_t prg = 0;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(ap == nullptr, "gpu_gemm_nt: the BatchNorm prologue and add are exclusive");
    TORCH_CHECK(pro_groups >= 1 && M % pro_groups == 0, "gpu_gemm_nt: the prologue needs M to split into ",
                pro_groups, " workers");
    prg = M / pro_groups;
    psc = opt_vec(pro_scale, pro_groups * K, dev, "pro_scale");
    psh = opt_vec(pro_shift, pro_groups * K, dev, "pro_shift");
    TORCH_CHECK(psh != nullptr, "gpu_gemm_nt: pro_shift missing");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(psc) % 16 == 0 && reinterpret_cast<uintptr_t>(psh) % 16 == 0,
                "gpu_gemm_nt: pro_scale / pro_shift must be 16-byte aligned");
    TORCH_CHECK(garfield::gpu::gemm_nt_pro_ok(static_cast<int>(cfg), static_cast<int>(K), prg,
                                              static_cast<int>(pro_groups)),
                "gpu_gemm_nt: configuration ", cfg, " has no BatchNorm-prologue form for K = ", K, ", ", prg,
                " rows per worker");
  }
  const uint8_t* mp = nullptr;
  if (add_mask.has_value() && add_mask->defined()) {
    TORCH_CHECK(ap != nullptr, "gpu_gemm_nt: add_mask needs add");
    TORCH_CHECK(add_mask->is_cuda() && add_mask->device() == dev && add_mask->scalar_type() == at::kByte &&
                    add_mask->is_contiguous() && add_mask->numel() * 8 == M * N,
                "gpu_gemm_nt: add_mask must be a contiguous uint8 bit mask of M * N / 8 bytes on a's device");
    mp = add_mask->data_ptr<uint8_t>();
  }
  const int S = garfield::gpu::gemm_nt_splits(static_cast<int>(cfg));
  at::Tensor slabs;
  if (S > 1) {   // split-K: fp32 slabs from the caching allocator (graph-capture safe), summed into c
    TORCH_CHECK(!want_stats && psc == nullptr, "gpu_gemm_nt: split-K configurations have no statistics / prologue");
    slabs = at::empty({S, M, N}, a.options().dtype(at::kFloat));
  }
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::gemm_nt(u16(a), u16(b), static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), u16_mut(c),
                         ap, sp, rg, static_cast<int>(cfg), stream_of(dev), psc, psh, prg,
                         static_cast<int>(pro_groups), S > 1 ? slabs.data_ptr<float>() : nullptr, mp);
}

// Transposes of many bf16 matrices in one launch: dsts[i] = srcs[i]ᵀ (2-D, contiguous, 16-B aligned,
// both dims multiples of 8). A 4-D pair is a k x k convolution weight: src the channels_last
// [Cout, Cin, KH, KW] weight, dst the channels_last [Cin, Cout, KH, KW] flipped transpose
// dst[ci, co, i, j] = src[co, ci, KH-1-i, KW-1-j] (its data gradient's weight).
void g_transpose_multi(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "gpu_transpose_multi: one dst per src");
  if (srcs.empty()) return;
  std::vector<const uint16_t*> sp;
  std::vector<uint16_t*> dp;
  std::vector<int> R, C, T;
  const auto dev = srcs[0].device();
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& a = srcs[i];
    const auto& b = dsts[i];
    TORCH_CHECK(a.is_cuda() && a.device() == dev && a.scalar_type() == at::kBFloat16 && b.device() == dev &&
                    b.scalar_type() == at::kBFloat16 && a.dim() == b.dim() && b.size(0) == a.size(1) &&
                    b.size(1) == a.size(0),
                "gpu_transpose_multi: src [R, C(, KH, KW)] and dst [C, R(, KH, KW)] bf16 on one device");
    if (a.dim() == 2) {
      TORCH_CHECK(a.is_contiguous() && b.is_contiguous(), "gpu_transpose_multi: 2-D matrices must be contiguous");
      T.push_back(1);
    } else {
      TORCH_CHECK(a.dim() == 4 && a.size(2) == b.size(2) && a.size(3) == b.size(3) &&
                      a.is_contiguous(at::MemoryFormat::ChannelsLast) && b.is_contiguous(at::MemoryFormat::ChannelsLast),
                  "gpu_transpose_multi: 4-D weights must be channels_last [Cout, Cin, KH, KW] -> [Cin, Cout, KH, KW]");
      T.push_back(static_cast<int>(a.size(2) * a.size(3)));
    }
    TORCH_CHECK(a.size(0) % 8 == 0 && a.size(1) % 8 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
                "gpu_transpose_multi: dims multiples of 8, 16-byte aligned");
    sp.push_back(u16(a));
    dp.push_back(u16_mut(b));
    R.push_back(static_cast<int>(a.size(0)));
    C.push_back(static_cast<int>(a.size(1)));
  }
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::transpose_multi(sp.data(), dp.data(), R.data(), C.data(), static_cast<int>(sp.size()),
                                 stream_of(dev), T.data());
}

// Layer-wise GAR building blocks (gar_layerwise.hip)
void g_lw_gram(const RowSet& rs, const at::Tensor& jobs, const at::Tensor& seg_lo, const at::Tensor& slabs,
               const at::Tensor& gram) {
  check_gpu(rs);
  TORCH_CHECK(jobs.device() == rs.device && jobs.scalar_type() == at::kLong && jobs.dim() == 2 && jobs.size(1) == 3 &&
                  jobs.is_contiguous(), "gpu_lw_gram: jobs must be a contiguous int64 [J, 3] tensor on the rows' device");
  TORCH_CHECK(seg_lo.device() == rs.device && seg_lo.scalar_type() == at::kInt && seg_lo.dim() == 1 &&
                  seg_lo.is_contiguous() && seg_lo.numel() >= 2,
              "gpu_lw_gram: seg_lo must be a contiguous int32 [L + 1] tensor on the rows' device");
  const int J = static_cast<int>(jobs.size(0)), L = static_cast<int>(seg_lo.numel() - 1);
  const int np = garfield::gpu::gram_padded(rs.n);
  TORCH_CHECK(slabs.numel() >= static_cast<int64_t>(J) * garfield::gpu::gram_slab_floats(rs.n),
              "gpu_lw_gram: slab workspace too small");
  TORCH_CHECK(gram.numel() >= static_cast<int64_t>(L) * np * np, "gpu_lw_gram: gram output too small");
  c10::hip::HIPGuard guard(rs.device.index());
  garfield::gpu::lw_gram(rs.table, rs.n, rs.dt, jobs.data_ptr<int64_t>(), J, seg_lo.data_ptr<int>(), L, fptr(slabs),
                         fptr(gram), stream_of(rs.device));
}

void g_lw_combine_sgd(const RowSet& rs, const at::Tensor& jobs, const at::Tensor& seg_off, int64_t base,
                      const at::Tensor& weights, const at::Tensor& param, const at::Tensor& mom,
                      const c10::optional<at::Tensor>& shadow, double lr, double momentum, double dampening,
                      double weight_decay, bool nesterov, bool first_step) {
  check_gpu(rs);
  TORCH_CHECK(jobs.device() == rs.device && jobs.scalar_type() == at::kLong && jobs.dim() == 2 && jobs.size(1) == 3 &&
                  jobs.is_contiguous(), "gpu_lw_combine_sgd: jobs must be a contiguous int64 [J, 3] tensor");
  TORCH_CHECK(seg_off.device() == rs.device && seg_off.scalar_type() == at::kLong && seg_off.is_contiguous(),
              "gpu_lw_combine_sgd: seg_off must be a contiguous int64 [L + 1] tensor");
  const int64_t L = seg_off.numel() - 1;
  TORCH_CHECK(weights.numel() >= L * rs.n, "gpu_lw_combine_sgd: weights must be [L, n]");
  TORCH_CHECK(param.numel() >= rs.d && mom.numel() >= rs.d, "gpu_lw_combine_sgd: parameter/momentum too small");
  void* sh = nullptr;
  int sh_dt = garfield::kBF16;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->is_cuda() && shadow->device() == rs.device && shadow->is_contiguous() && shadow->numel() >= rs.d,
                "gpu_lw_combine_sgd: shadow must be a contiguous tensor of >= d elements on the rows' device");
    sh_dt = dtype_code(*shadow);
    sh = shadow->data_ptr();
  }
  garfield::gpu::SgdArgs a{static_cast<float>(lr), static_cast<float>(momentum), static_cast<float>(dampening),
                           static_cast<float>(weight_decay), nesterov ? 1 : 0, first_step ? 1 : 0};
  c10::hip::HIPGuard guard(rs.device.index());
  garfield::gpu::lw_combine_sgd(rs.table, rs.n, rs.dt, jobs.data_ptr<int64_t>(), static_cast<int>(jobs.size(0)),
                                fptr(weights), fptr(param), fptr(mom), sh, sh_dt, a, seg_off.data_ptr<int64_t>(), base,
                                stream_of(rs.device));
}

void g_lw_bulyan_tail(const RowSet& rs, const at::Tensor& jobs, const at::Tensor& W, int64_t t, int64_t beta,
                      const at::Tensor& out) {
  check_gpu(rs);
  TORCH_CHECK(jobs.device() == rs.device && jobs.scalar_type() == at::kLong && jobs.dim() == 2 && jobs.size(1) == 3 &&
                  jobs.is_contiguous(), "gpu_lw_bulyan_tail: jobs must be a contiguous int64 [J, 3] tensor");
  TORCH_CHECK(t >= 1 && t <= 64 && beta >= 1 && beta <= t, "gpu_lw_bulyan_tail: 1 <= beta <= t <= 64");
  TORCH_CHECK(W.device() == rs.device && W.scalar_type() == at::kFloat && W.is_contiguous() &&
                  W.numel() % (t * rs.n) == 0, "gpu_lw_bulyan_tail: W must be a contiguous fp32 [L, t, n] tensor");
  TORCH_CHECK(out.device() == rs.device && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() >= rs.d,
              "gpu_lw_bulyan_tail: out must be a contiguous fp32 vector of >= d elements");
  c10::hip::HIPGuard guard(rs.device.index());
  garfield::gpu::lw_bulyan_tail(rs.table, rs.n, rs.dt, jobs.data_ptr<int64_t>(), static_cast<int>(jobs.size(0)),
                                fptr(W), static_cast<int>(t), static_cast<int>(beta), out.data_ptr<float>(),
                                stream_of(rs.device));
}

// Large gradient sets: x an [n, d] GPU matrix (unit column stride, row stride ld, 16-bit or fp32).
int large_dtype(const at::Tensor& x, const at::Tensor& out) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1 && x.size(0) >= 1 &&
                  x.size(0) <= garfield::kLargeRows,
              "garfield large: x must be an [n, d] GPU matrix with unit column stride, 1 <= n <= ", garfield::kLargeRows);
  TORCH_CHECK(out.device() == x.device() && out.scalar_type() == x.scalar_type() && out.is_contiguous() &&
                  out.numel() == x.size(1),
              "garfield large: out must be a contiguous [d] tensor of x's dtype on x's device");
  return dtype_code(x);
}

void g_large_combine(const at::Tensor& x, const at::Tensor& w, const at::Tensor& out) {
  const int dt = large_dtype(x, out);
  TORCH_CHECK(w.device() == x.device() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == x.size(0),
              "gpu_large_combine: w must be a contiguous fp32 [n] tensor on x's device");
  c10::hip::HIPGuard guard(x.device().index());
  garfield::gpu::large_combine(x.data_ptr(), dt, static_cast<int>(x.size(0)), x.size(1), x.stride(0),
                               w.data_ptr<float>(), out.data_ptr(), stream_of(x.device()));
}

void g_large_gram(const at::Tensor& x, const at::Tensor& slabs, const at::Tensor& gram) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1 && x.size(0) <= garfield::kLargeRows,
              "gpu_large_gram: x must be a GPU [n, d] matrix with unit column stride, n <= ", garfield::kLargeRows);
  const int dt = dtype_code(x);
  TORCH_CHECK(dt != garfield::kF64, "gpu_large_gram: x must be fp32, bf16 or fp16");
  const int64_t n = x.size(0), d = x.size(1);
  const int esz = dt == garfield::kF32 ? 4 : 2;
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && (x.stride(0) * esz) % 16 == 0,
              "gpu_large_gram: rows must be 16-byte aligned");
  TORCH_CHECK(gram.device() == x.device() && gram.scalar_type() == at::kFloat && gram.is_contiguous() &&
                  gram.numel() == n * n, "gpu_large_gram: gram must be a contiguous fp32 [n, n] tensor");
  ws_vec(slabs, garfield::gpu::large_gram_slab_floats(static_cast<int>(n), d, dt), x.device(), "slabs");
  c10::hip::HIPGuard guard(x.device().index());
  garfield::gpu::large_gram(x.data_ptr(), dt, static_cast<int>(n), d, x.stride(0), slabs.data_ptr<float>(),
                            gram.data_ptr<float>(), stream_of(x.device()));
}

void g_large_wx(const at::Tensor& W, const at::Tensor& x, const at::Tensor& V) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "gpu_large_wx: x must be a GPU [n, d] matrix");
  const int dt = dtype_code(x);
  TORCH_CHECK(dt != garfield::kF64, "gpu_large_wx: x must be fp32, bf16 or fp16");
  const int64_t n = x.size(0), d = x.size(1);
  TORCH_CHECK(W.device() == x.device() && W.scalar_type() == at::kFloat && W.is_contiguous() && W.dim() == 2 &&
                  W.size(1) == n, "gpu_large_wx: W must be a contiguous fp32 [t, n] tensor");
  const int64_t t = W.size(0);
  TORCH_CHECK(V.device() == x.device() && V.scalar_type() == at::kFloat && V.dim() == 2 && V.size(0) == t &&
                  V.size(1) == d && V.stride(1) == 1, "gpu_large_wx: V must be an fp32 [t, d] matrix (unit column stride)");
  c10::hip::HIPGuard guard(x.device().index());
  garfield::gpu::large_wx(W.data_ptr<float>(), static_cast<int>(t), static_cast<int>(n), x.data_ptr(), dt, d,
                          x.stride(0), V.data_ptr<float>(), V.stride(0), stream_of(x.device()));
}

void g_large_coord(const at::Tensor& x, int64_t mode, int64_t f, int64_t beta, const at::Tensor& out) {
  const int dt = large_dtype(x, out);
  const int64_t n = x.size(0);
  TORCH_CHECK(mode >= 0 && mode <= 2, "gpu_large_coord: mode 0 median, 1 trimmed-mean, 2 averaged-median");
  TORCH_CHECK(mode != 1 || (f >= 0 && 2 * f < n), "gpu_large_coord: trimmed-mean needs 0 <= 2f < n");
  TORCH_CHECK(mode != 2 || (beta >= 1 && beta <= n), "gpu_large_coord: averaged-median needs 1 <= beta <= n");
  c10::hip::HIPGuard guard(x.device().index());
  garfield::gpu::large_coord(x.data_ptr(), dt, static_cast<int>(n), x.size(1), x.stride(0), static_cast<int>(mode),
                             static_cast<int>(f), static_cast<int>(beta), out.data_ptr(), stream_of(x.device()));
}

void g_large_select(const at::Tensor& gram, int64_t f, int64_t m, int64_t rounds, bool shrink, const at::Tensor& W) {
  TORCH_CHECK(gram.is_cuda() && gram.scalar_type() == at::kFloat && gram.dim() == 2 && gram.size(0) == gram.size(1) &&
                  gram.stride(1) == 1 && gram.size(0) <= garfield::kLargeRows,
              "gpu_large_select: gram must be an fp32 [n, n] GPU matrix (unit column stride), n <= ", garfield::kLargeRows);
  const int64_t n = gram.size(0);
  TORCH_CHECK(f >= 0 && n - f - 2 >= 1 && m >= 1 && m <= n && rounds >= 1 && rounds <= n,
              "gpu_large_select: needs n - f - 2 >= 1, 1 <= m <= n, 1 <= rounds <= n");
  TORCH_CHECK(W.device() == gram.device() && W.scalar_type() == at::kFloat && W.is_contiguous() &&
                  W.numel() == rounds * n, "gpu_large_select: W must be a contiguous fp32 [rounds, n] tensor");
  c10::hip::HIPGuard guard(gram.device().index());
  auto dopt = gram.options().dtype(at::kDouble);
  at::Tensor tv = at::empty({n}, dopt), ns = at::empty({n}, dopt), ti = at::empty({n}, gram.options().dtype(at::kInt));
  garfield::gpu::large_select(gram.data_ptr<float>(), gram.stride(0), static_cast<int>(n), static_cast<int>(f),
                              static_cast<int>(m), static_cast<int>(rounds), shrink, tv.data_ptr<double>(),
                              ti.data_ptr<int>(), ns.data_ptr<double>(), W.data_ptr<float>(), stream_of(gram.device()));
}

// Split-K slabs -> strided per-group output: part fp32 [S, G, ...] and out [G, ...] (fp32 / bf16 /
// fp16) may have any slab / group strides and one row pitch each (the last dim contiguous, the
// dims between it and the group dim dense), e.g. a padded GEMM result cropped into exchange rows.
garfield::gpu::SplitJob split_job(const at::Tensor& part, const at::Tensor& out) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() >= 3,
              "gpu_split_reduce: part must be an fp32 [S, G, ...] GPU tensor");
  TORCH_CHECK(out.device() == part.device() && out.dim() == part.dim() - 1 && out.size(0) == part.size(1),
              "gpu_split_reduce: out must be [G, ...] on part's device");
  const int64_t D = part.dim();
  for (int64_t k = 2; k < D; ++k)
    TORCH_CHECK(part.size(k) == out.size(k - 1), "gpu_split_reduce: part and out shapes differ");
  const int64_t Cc = part.size(D - 1);
  TORCH_CHECK(part.stride(D - 1) == 1 && out.stride(D - 2) == 1, "gpu_split_reduce: the last dim must be contiguous");
  int64_t R = 1, ipitch = Cc, opitch = Cc;
  if (D >= 4) {
    ipitch = part.stride(D - 2);
    opitch = out.stride(D - 3);
    // dims [2, D-2) must be dense over the row pitch
    int64_t ai = ipitch, ao = opitch;
    for (int64_t k = D - 2; k >= 2; --k) {
      TORCH_CHECK(part.stride(k) == ai && out.stride(k - 1) == ao, "gpu_split_reduce: outer inner dims must be dense");
      ai *= part.size(k);
      ao *= part.size(k);
      R *= part.size(k);
    }
    TORCH_CHECK(ipitch >= Cc && opitch >= Cc, "gpu_split_reduce: row pitch below the row length");
  }
  const int odt = dtype_code(out);
  TORCH_CHECK(odt != garfield::kF64, "gpu_split_reduce: out must be fp32, bf16 or fp16");
  garfield::gpu::SplitJob j{};
  j.part = part.data_ptr<float>();
  j.out = out.data_ptr();
  j.R = R;
  j.Cc = Cc;
  j.ipitch = ipitch;
  j.opitch = opitch;
  j.ss = part.stride(0);
  j.gs = part.stride(1);
  j.ostride = out.stride(0);
  j.S = static_cast<int>(part.size(0));
  j.G = static_cast<int>(part.size(1));
  j.odt = odt;
  return j;
}

// Split-K slabs -> strided per-group output: part fp32 [S, G, ...] and out [G, ...] (fp32 / bf16 /
// fp16) may have any slab / group strides and one row pitch each (the last dim contiguous, the
// dims between it and the group dim dense), e.g. a padded GEMM result cropped into exchange rows.
void g_split_reduce(const at::Tensor& part, const at::Tensor& out) {
  const auto j = split_job(part, out);
  c10::hip::HIPGuard guard(part.device().index());
  garfield::gpu::split_reduce(j.part, j.S, j.G, j.R, j.Cc, j.ipitch, j.opitch, j.ss, j.gs, j.out, j.odt, j.ostride,
                              stream_of(part.device()));
}

// Many of them in one launch (the grouped backward's per-layer split-K sums).
void g_split_reduce_multi(const std::vector<at::Tensor>& parts, const std::vector<at::Tensor>& outs) {
  TORCH_CHECK(parts.size() == outs.size(), "gpu_split_reduce_multi: one out per part");
  if (parts.empty()) return;
  std::vector<garfield::gpu::SplitJob> jobs;
  jobs.reserve(parts.size());
  for (size_t i = 0; i < parts.size(); ++i) {
    TORCH_CHECK(parts[i].device() == parts[0].device(), "gpu_split_reduce_multi: one device");
    jobs.push_back(split_job(parts[i], outs[i]));
  }
  c10::hip::HIPGuard guard(parts[0].device().index());
  garfield::gpu::split_reduce_multi(jobs.data(), static_cast<int>(jobs.size()), stream_of(parts[0].device()));
}

// Fresh grouped batch: out [R, C, H, W] bf16 channels_last from uint8 NHWC images src[idx[r]].
void g_augment_gather(const at::Tensor& src, const c10::optional<at::Tensor>& idx_opt, int64_t seed, int64_t step,
                      const std::vector<double>& mean, const std::vector<double>& std, const at::Tensor& out,
                      int64_t pad, bool flip, const c10::optional<at::Tensor>& labels,
                      const c10::optional<at::Tensor>& labels_out) {
  const auto dev = src.device();
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.dim() == 4 && src.is_contiguous(),
              "gpu_augment_gather: src must be a contiguous uint8 [N, H, W, C] GPU tensor");
  const int64_t H = src.size(1), W = src.size(2), C = src.size(3);
  TORCH_CHECK(C >= 1 && C <= 4, "gpu_augment_gather: 1..4 channels");
  const int64_t R = out.size(0);
  const int64_t* ip = nullptr;
  if (idx_opt.has_value() && idx_opt->defined()) {
    const auto& idx = *idx_opt;
    TORCH_CHECK(idx.device() == dev && idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous() &&
                    idx.size(0) == R,
                "gpu_augment_gather: idx must be a contiguous int64 [len(out)] vector on src's device");
    ip = idx.data_ptr<int64_t>();
  }
  const int64_t* lp = nullptr;
  int64_t* lo = nullptr;
  if (labels_out.has_value() && labels_out->defined()) {
    TORCH_CHECK(labels.has_value() && labels->defined() && labels->device() == dev &&
                    labels->scalar_type() == at::kLong && labels->is_contiguous() && labels->numel() == src.size(0),
                "gpu_augment_gather: labels must be a contiguous int64 [N] tensor on src's device");
    TORCH_CHECK(labels_out->device() == dev && labels_out->scalar_type() == at::kLong && labels_out->is_contiguous() &&
                    labels_out->numel() == R,
                "gpu_augment_gather: labels_out must be a contiguous int64 [len(out)] tensor");
    lp = labels->data_ptr<int64_t>();
    lo = labels_out->data_ptr<int64_t>();
  }
  TORCH_CHECK(out.device() == dev && (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat) &&
                  out.dim() == 4 &&
                  out.size(1) == C && out.size(2) == H && out.size(3) == W &&
                  out.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gpu_augment_gather: out must be a channels_last bf16 or fp32 [len(idx), C, H, W] tensor");
  TORCH_CHECK(static_cast<int64_t>(mean.size()) == C && static_cast<int64_t>(std.size()) == C,
              "gpu_augment_gather: one mean / std per channel");
  TORCH_CHECK(pad >= 0 && pad < H && pad < W, "gpu_augment_gather: invalid padding");
  garfield::gpu::AugNorm n{};
  for (int64_t c = 0; c < C; ++c) {
    TORCH_CHECK(std[c] > 0, "gpu_augment_gather: std must be positive");
    n.mean[c] = static_cast<float>(mean[c]);
    n.inv_std[c] = static_cast<float>(1.0 / std[c]);
  }
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::augment_gather(src.data_ptr<uint8_t>(), src.size(0), ip, lp, lo, R, static_cast<int>(H),
                                static_cast<int>(W), static_cast<int>(C), static_cast<int>(pad), flip,
                                static_cast<uint64_t>(seed), static_cast<uint64_t>(step), n, out.data_ptr(),
                                stream_of(dev), dtype_code(out));
}

// Per-worker implicit weight gradient. out: fp32 [splits, groups, Cout, K] (contiguous partial
// slabs) or, with splits == 1, a bf16 [groups, Cout, K] view whose rows are contiguous (any group
// stride: the exchange rows).
// ------------------------------------------- fp32 (reference-precision) step ----

void check_f32_cl(const at::Tensor& t, const at::Device& dev, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.device() == dev && t.scalar_type() == at::kFloat && t.dim() == 4 &&
                  t.is_contiguous(at::MemoryFormat::ChannelsLast) && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "garfield conv_f32: ", what, " must be a 16-byte aligned channels_last fp32 4-D tensor on ", dev);
  TORCH_CHECK(t.numel() < INT32_MAX, "garfield conv_f32: ", what, " is too large");
}

int64_t conv_out(int64_t in, int64_t k, int64_t s, int64_t p, int64_t d) { return (in + 2 * p - d * (k - 1) - 1) / s + 1; }

// out = conv(src) (forward: w [Co][kh][kw][Cs] split) or the data gradient of a convolution with this
// geometry (dgrad: src = dy, out = dx, w = Wt [Co = Cin][kh][kw][Cs = Cout] split); (+ add)
void g_conv_f32(const at::Tensor& src, const at::Tensor& w3, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool dgrad, const at::Tensor& out,
                const c10::optional<at::Tensor>& add, int64_t pm, int64_t ksplit) {
  const auto dev = src.device();
  check_f32_cl(src, dev, "src");
  check_f32_cl(out, dev, "out");
  TORCH_CHECK(kh >= 1 && kw >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0 && dh >= 1 && dw >= 1,
              "gpu_conv_f32: invalid kernel geometry");
  garfield::gpu::ConvF32Geo g{};
  g.N = static_cast<int>(src.size(0));
  g.Cs = static_cast<int>(src.size(1));
  g.Hs = static_cast<int>(src.size(2));
  g.Ws = static_cast<int>(src.size(3));
  g.Co = static_cast<int>(out.size(1));
  g.Ho = static_cast<int>(out.size(2));
  g.Wo = static_cast<int>(out.size(3));
  g.KH = static_cast<int>(kh); g.KW = static_cast<int>(kw);
  g.sh = static_cast<int>(sh); g.sw = static_cast<int>(sw);
  g.ph = static_cast<int>(ph); g.pw = static_cast<int>(pw);
  g.dh = static_cast<int>(dh); g.dw = static_cast<int>(dw);
  TORCH_CHECK(out.size(0) == g.N, "gpu_conv_f32: src and out must hold the same images");
  if (dgrad) {
    TORCH_CHECK(conv_out(g.Ho, kh, sh, ph, dh) == g.Hs && conv_out(g.Wo, kw, sw, pw, dw) == g.Ws,
                "gpu_conv_f32: dy [", g.Hs, "x", g.Ws, "] is not the forward output of dx [", g.Ho, "x", g.Wo, "]");
  } else {
    TORCH_CHECK(conv_out(g.Hs, kh, sh, ph, dh) == g.Ho && conv_out(g.Ws, kw, sw, pw, dw) == g.Wo,
                "gpu_conv_f32: out [", g.Ho, "x", g.Wo, "] is not the forward output of src [", g.Hs, "x", g.Ws, "]");
  }
  TORCH_CHECK(garfield::gpu::conv_f32_supported(g), "gpu_conv_f32: needs Co % 64 == 0 (got ", g.Co, ")");
  TORCH_CHECK(g.Cs % 32 == 0 || !dgrad, "gpu_conv_f32: a data gradient needs Cs % 32 == 0");
  // Cs % 32 != 0 (gathered k): weight rows of the flattened (tap, channel) index padded to a multiple of 32
  const int64_t kr = kh * kw * g.Cs;
  const int64_t wn = static_cast<int64_t>(g.Co) * (g.Cs % 32 ? (kr + 31) / 32 * 32 : kr);
  TORCH_CHECK(w3.device() == dev && w3.scalar_type() == at::kBFloat16 && w3.is_contiguous() && w3.numel() == 3 * wn &&
                  reinterpret_cast<uintptr_t>(w3.data_ptr()) % 16 == 0,
              "gpu_conv_f32: w must be the contiguous bf16 pieces [3, Co, K] (", 3 * wn, " elements)");
  const float* ap = nullptr;
  if (add.has_value() && add->defined()) {
    check_f32_cl(*add, dev, "add");
    TORCH_CHECK(add->sizes() == out.sizes(), "gpu_conv_f32: add must have out's shape");
    ap = add->data_ptr<float>();
  }
  c10::hip::HIPGuard guard(dev.index());
  // split-K: automatic with the automatic kernel choice (pm <= 0, ksplit 0), or forced (ksplit > 1)
  int S = ksplit > 0 ? static_cast<int>(ksplit) : (pm <= 0 ? garfield::gpu::conv_f32_ksplit(g, dgrad) : 1);
  if (!garfield::gpu::conv_f32_lds_ok(g, dgrad)) S = 1;
  at::Tensor part;
  if (S > 1) part = at::empty({S * out.numel()}, out.options().memory_format(at::MemoryFormat::Contiguous));
  garfield::gpu::conv_f32(src.data_ptr<float>(), reinterpret_cast<const uint16_t*>(w3.data_ptr()), g, dgrad,
                          out.data_ptr<float>(), ap, static_cast<int>(pm), stream_of(dev), S,
                          S > 1 ? part.data_ptr<float>() : nullptr);
}

// per-worker weight gradients of a convolution (forward geometry from x, dy): out fp32
// [splits, groups, Cout, K] contiguous, or (splits == 1) a [groups, Cout, K] view with contiguous rows
void g_wgrad_f32(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph,
                 int64_t pw, int64_t dh, int64_t dw, int64_t groups, const at::Tensor& out, int64_t splits,
                 int64_t variant) {
  const auto dev = x.device();
  check_f32_cl(x, dev, "x");
  check_f32_cl(dy, dev, "dy");
  garfield::gpu::ConvF32Geo g{};
  g.N = static_cast<int>(x.size(0));
  g.Cs = static_cast<int>(x.size(1));
  g.Hs = static_cast<int>(x.size(2));
  g.Ws = static_cast<int>(x.size(3));
  g.Co = static_cast<int>(dy.size(1));
  g.Ho = static_cast<int>(dy.size(2));
  g.Wo = static_cast<int>(dy.size(3));
  g.KH = static_cast<int>(kh); g.KW = static_cast<int>(kw);
  g.sh = static_cast<int>(sh); g.sw = static_cast<int>(sw);
  g.ph = static_cast<int>(ph); g.pw = static_cast<int>(pw);
  g.dh = static_cast<int>(dh); g.dw = static_cast<int>(dw);
  TORCH_CHECK(dy.size(0) == g.N && conv_out(g.Hs, kh, sh, ph, dh) == g.Ho && conv_out(g.Ws, kw, sw, pw, dw) == g.Wo,
              "gpu_wgrad_f32: dy is not the forward output of x");
  TORCH_CHECK(garfield::gpu::wgrad_f32_supported(g), "gpu_wgrad_f32: needs Cout % 64 == 0");
  TORCH_CHECK(dy.numel() / g.Co < (int64_t{1} << 31), "gpu_wgrad_f32: more than 2^31 output pixels");
  const int64_t M = static_cast<int64_t>(g.N) * g.Ho * g.Wo;
  TORCH_CHECK(groups >= 1 && M % groups == 0, "gpu_wgrad_f32: ", M, " output pixels do not split into ", groups,
              " workers");
  TORCH_CHECK(splits >= 1 && splits <= 64, "gpu_wgrad_f32: splits must be in [1, 64]");
  const int64_t K = static_cast<int64_t>(kh) * kw * g.Cs, cout = g.Co;
  TORCH_CHECK(out.device() == dev && out.scalar_type() == at::kFloat, "gpu_wgrad_f32: out must be fp32 on x's device");
  int64_t ss = 0, gs = 0;
  if (out.dim() == 4) {
    TORCH_CHECK(out.is_contiguous() && out.size(0) == splits && out.size(1) == groups && out.size(2) == cout &&
                    out.size(3) == K,
                "gpu_wgrad_f32: a 4-D out must be contiguous [splits, groups, Cout, K]");
    ss = groups * cout * K;
    gs = cout * K;
  } else {
    TORCH_CHECK(splits == 1 && out.dim() == 3 && out.size(0) == groups && out.size(1) == cout && out.size(2) == K &&
                    out.stride(2) == 1 && out.stride(1) == K && out.stride(0) >= cout * K,
                "gpu_wgrad_f32: a 3-D out must be a [groups, Cout, K] view with contiguous rows (splits == 1)");
    gs = out.stride(0);
  }
  c10::hip::HIPGuard guard(dev.index());
  TORCH_CHECK(variant >= 0 && variant <= 3 && ((variant != 1 && variant != 2) || garfield::gpu::wgrad_f32_wide(g)),
              "gpu_wgrad_f32: variant 0 auto, 1/2 the 128x128 form (Cin, Cout % 128 == 0), 3 the 64x64 form");
  garfield::gpu::wgrad_f32(x.data_ptr<float>(), dy.data_ptr<float>(), g, static_cast<int>(groups), M / groups,
                           static_cast<int>(splits), out.data_ptr<float>(), ss, gs, stream_of(dev),
                           static_cast<int>(variant));
}

// jobs: (w fp32 [R, T, C] memory order, pieces bf16 [3, R, ld], tpieces [3, C, T, R] or None, R, T, C, ld)
void g_wsplit_multi(const std::vector<py::tuple>& jobs) {
  if (jobs.empty()) return;
  std::vector<garfield::gpu::WSplitJob> js;
  js.reserve(jobs.size());
  c10::Device dev = jobs[0][0].cast<at::Tensor>().device();
  for (const auto& t : jobs) {
    TORCH_CHECK(t.size() == 7, "gpu_wsplit_multi: each job is (w, pieces, tpieces, R, T, C, ld)");
    auto w = t[0].cast<at::Tensor>(), pc = t[1].cast<at::Tensor>();
    const int64_t R = t[3].cast<int64_t>(), T = t[4].cast<int64_t>(), C = t[5].cast<int64_t>(), ld = t[6].cast<int64_t>();
    TORCH_CHECK(w.is_cuda() && w.device() == dev && w.scalar_type() == at::kFloat && w.numel() == R * T * C,
                "gpu_wsplit_multi: w must be an fp32 tensor of R*T*C elements on one device");
    TORCH_CHECK(w.is_contiguous() || w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_wsplit_multi: w must be dense (memory order [R][T][C])");
    const int64_t rows = ld > 0 ? ld : T * C;
    TORCH_CHECK(ld == 0 || ld >= T * C, "gpu_wsplit_multi: ld < T*C");
    TORCH_CHECK(pc.device() == dev && pc.scalar_type() == at::kBFloat16 && pc.is_contiguous() &&
                    pc.numel() == 3 * R * rows,
                "gpu_wsplit_multi: pieces must be a contiguous bf16 [3, R, ld] tensor");
    uint16_t* tp = nullptr;
    if (!t[2].is_none()) {
      auto a = t[2].cast<at::Tensor>();
      TORCH_CHECK(a.device() == dev && a.scalar_type() == at::kBFloat16 && a.is_contiguous() &&
                      a.numel() == 3 * R * T * C,
                  "gpu_wsplit_multi: tpieces must be a contiguous bf16 [3, C, T, R] tensor");
      tp = reinterpret_cast<uint16_t*>(a.data_ptr());
    }
    js.push_back(garfield::gpu::WSplitJob{w.data_ptr<float>(), reinterpret_cast<uint16_t*>(pc.data_ptr()), tp,
                                           static_cast<int>(R), static_cast<int>(T), static_cast<int>(C),
                                           static_cast<int>(ld)});
  }
  c10::hip::HIPGuard guard(dev.index());
  garfield::gpu::wsplit_multi(js.data(), static_cast<int>(js.size()), stream_of(dev));
}

void check_f32_mat(const at::Tensor& t, const at::Device& dev, int64_t r, int64_t c, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.device() == dev && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                  t.numel() == r * c,
              "garfield linear_f32: ", what, " must be a contiguous fp32 [", r, ", ", c, "] tensor on ", dev);
}

void g_iwgrad(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph,
              int64_t pw, int64_t dh, int64_t dw, int64_t groups, const at::Tensor& out, int64_t splits,
              const c10::optional<at::Tensor>& pro_scale, const c10::optional<at::Tensor>& pro_shift) {
  auto g = conv_geometry(x, kh, kw, sh, sw, ph, pw, dh, dw);
  TORCH_CHECK(g.C % 64 == 0, "gpu_iwgrad: input channels must be a multiple of 64 (got ", g.C, ")");
  TORCH_CHECK(dy.is_cuda() && dy.device() == x.device() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.size(0) == g.N && dy.size(2) == g.Ho &&
                  dy.size(3) == g.Wo,
              "gpu_iwgrad: dy must be a channels_last bf16 [", g.N, ", Cout, ", g.Ho, ", ", g.Wo, "] tensor");
  const int64_t cout = dy.size(1);
  TORCH_CHECK(cout % 64 == 0, "gpu_iwgrad: output channels must be a multiple of 64 (got ", cout, ")");
  const int64_t M = static_cast<int64_t>(g.N) * g.Ho * g.Wo;
  TORCH_CHECK(groups >= 1 && M % groups == 0, "gpu_iwgrad: ", M, " output pixels do not split into ", groups,
              " workers");
  TORCH_CHECK(M < INT32_MAX && static_cast<int64_t>(g.N) * g.H * g.W * g.C < INT32_MAX,
              "gpu_iwgrad: tensor too large");
  TORCH_CHECK(splits >= 1 && splits <= 64, "gpu_iwgrad: splits must be in [1, 64]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0,
              "gpu_iwgrad: x and dy must be 16-byte aligned");
  const int64_t K = static_cast<int64_t>(g.KH) * g.KW * g.C;
  TORCH_CHECK(out.device() == x.device(), "gpu_iwgrad: out must be on x's device");
  bool bf16 = false;
  int64_t ss = 0, gs = 0;
  if (out.scalar_type() == at::kFloat) {
    TORCH_CHECK(out.is_contiguous() && out.dim() == 4 && out.size(0) == splits && out.size(1) == groups &&
                    out.size(2) == cout && out.size(3) == K,
                "gpu_iwgrad: an fp32 out must be contiguous [splits, groups, Cout, K]");
    ss = groups * cout * K;
    gs = cout * K;
  } else {
    TORCH_CHECK(out.scalar_type() == at::kBFloat16 && splits == 1 && out.dim() == 3 && out.size(0) == groups &&
                    out.size(1) == cout && out.size(2) == K && out.stride(2) == 1 && out.stride(1) == K &&
                    out.stride(0) >= cout * K,
                "gpu_iwgrad: a bf16 out must be a [groups, Cout, K] view with contiguous rows (splits == 1)");
    bf16 = true;
    gs = out.stride(0);
  }
  const float* psc = opt_vec(pro_scale, groups * g.C, x.device(), "pro_scale");
  const float* psh = opt_vec(pro_shift, groups * g.C, x.device(), "pro_shift");
  TORCH_CHECK((psc == nullptr) == (psh == nullptr), "gpu_iwgrad: pass both pro_scale and pro_shift or neither");
  c10::hip::HIPGuard guard(x.device().index());
  if (psc) {   // the BatchNorm prologue: 1x1 / stride 1 / no padding (no padding pixel to keep at zero)
    TORCH_CHECK(kh == 1 && kw == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0,
                "gpu_iwgrad: the BatchNorm prologue takes 1x1 stride-1 unpadded convolutions only");
    garfield::gpu::iwgrad_nhwc(u16(x), u16(dy), g, static_cast<int>(cout), static_cast<int>(groups), M / groups,
                               static_cast<int>(splits), out.data_ptr(), bf16, ss, gs, stream_of(x.device()), psc, psh);
    return;
  }
  // the halo-staged 3x3 kernel whenever it fits
  if (garfield::gpu::wgrad3x3_nhwc(u16(x), u16(dy), g, static_cast<int>(cout), static_cast<int>(groups),
                                         M / groups, static_cast<int>(splits), out.data_ptr(), bf16, ss, gs,
                                         stream_of(x.device())))
    return;
  garfield::gpu::iwgrad_nhwc(u16(x), u16(dy), g, static_cast<int>(cout), static_cast<int>(groups), M / groups,
                             static_cast<int>(splits), out.data_ptr(), bf16, ss, gs, stream_of(x.device()));
}

bool g_wgrad3x3_fits(int64_t n, int64_t h, int64_t w, int64_t c, int64_t cout, int64_t groups) {
  garfield::gpu::Im2col g{static_cast<int>(n), static_cast<int>(h), static_cast<int>(w), static_cast<int>(c), 3, 3,
                          1, 1, 1, 1, 1, 1, static_cast<int>(h), static_cast<int>(w), 0};
  if (groups < 1 || n % groups) return false;
  return garfield::gpu::wgrad3x3_fits(g, static_cast<int>(cout), n / groups * h * w);
}

garfield::gpu::Im2col pool_geometry(const at::Tensor& x, const at::Tensor& y, const at::Tensor& idx, int64_t k,
                                    int64_t s, int64_t p) {
  auto g = conv_geometry(x, k, k, s, s, p, p, 1, 1, true);
  TORCH_CHECK(g.C % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "garfield maxpool: channels must be a multiple of 8 and x 16-byte aligned");
  TORCH_CHECK(y.device() == x.device() && y.scalar_type() == x.scalar_type() && y.dim() == 4 && y.size(0) == g.N &&
                  y.size(1) == g.C && y.size(2) == g.Ho && y.size(3) == g.Wo &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast) && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "garfield maxpool: y must be a channels_last [", g.N, ", ", g.C, ", ", g.Ho, ", ", g.Wo, "] tensor of x's dtype");
  TORCH_CHECK(idx.device() == x.device() && idx.scalar_type() == at::kByte && idx.numel() == y.numel() &&
                  idx.is_contiguous() && reinterpret_cast<uintptr_t>(idx.data_ptr()) % 8 == 0 && k * k <= 256,
              "garfield maxpool: idx must be a contiguous uint8 tensor of y's element count");
  return g;
}

void g_maxpool_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t p, const at::Tensor& y, const at::Tensor& idx) {
  auto g = pool_geometry(x, y, idx, k, s, p);
  c10::hip::HIPGuard guard(x.device().index());
  garfield::gpu::maxpool_fwd_nhwc(x.data_ptr(), g, y.data_ptr(), static_cast<uint8_t*>(idx.data_ptr()),
                                  stream_of(x.device()), dtype_code(x));
}

void g_maxpool_bwd(const at::Tensor& dy, const at::Tensor& idx, int64_t k, int64_t s, int64_t p, const at::Tensor& dx) {
  auto g = pool_geometry(dx, dy, idx, k, s, p);
  c10::hip::HIPGuard guard(dx.device().index());
  garfield::gpu::maxpool_bwd_nhwc(dy.data_ptr(), static_cast<const uint8_t*>(idx.data_ptr()), g, dx.data_ptr(),
                                  stream_of(dx.device()), dtype_code(dx));
}

int g_flatten_cast_at(const std::vector<at::Tensor>& srcs, const std::vector<int64_t>& offsets,
                      const at::Tensor& dst) {
  TORCH_CHECK(srcs.size() == offsets.size(), "flatten_cast_at: one offset per source tensor");
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "flatten_cast_at: dst must be a contiguous device tensor");
  const int odt = dtype_code(dst);
  TORCH_CHECK(odt != garfield::kF64, "flatten_cast_at: dst must be fp32, bf16 or fp16");
  if (srcs.empty()) return 0;
  c10::hip::HIPGuard guard(dst.device().index());
  std::vector<const void*> ptrs;
  std::vector<int> dts;
  std::vector<int64_t> numels, offs;
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& t = srcs[i];
    const auto st = t.scalar_type();
    TORCH_CHECK((st == at::kFloat || st == at::kBFloat16 || st == at::kHalf) && t.device() == dst.device(),
                "flatten_cast_at: fp32/bf16/fp16 sources on dst's device");
    TORCH_CHECK(t.is_non_overlapping_and_dense(), "flatten_cast_at: sources must be dense");
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] + t.numel() <= dst.numel(), "flatten_cast_at: source ", i,
                " at offset ", offsets[i], " overruns dst (", dst.numel(), " elements)");
    ptrs.push_back(t.data_ptr());
    dts.push_back(dtype_code(t));
    numels.push_back(t.numel());
    offs.push_back(offsets[i]);
  }
  return garfield::gpu::flatten_cast(ptrs.data(), dts.data(), numels.data(), offs.data(),
                                     static_cast<int>(ptrs.size()), dst.data_ptr(), odt, stream_of(dst.device()));
}

// Register a function under `name` for both a 2-D buffer and a list of rows.
template <class Fn2d, class FnList>
void def_rows(py::module& m, const char* name, Fn2d&& f2d, FnList&& flist, const char* doc) {
  m.def(name, std::forward<Fn2d>(f2d), doc);
  m.def(name, std::forward<FnList>(flist), doc);
}

}  // namespace

// Stream-ordered signals for waiting on a point INSIDE a captured HIP graph
// (hipEventRecordExternal is rejected during capture on ROCm 7, and torch refuses
// Event(external=True) there). A 1-thread kernel captured in the graph stores 1 to an
// 8-byte signal word (system-scope release, a vector store); another stream waits
// with hipStreamWaitValue64 (a command-processor wait: no spinning kernel) and
// re-arms the word with hipStreamWriteValue64.
int64_t signal_alloc(int64_t count) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, static_cast<size_t>(8 * count), hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  (void)hipMemset(p, 0, static_cast<size_t>(8 * count));
  (void)hipDeviceSynchronize();
  return reinterpret_cast<int64_t>(p);
}
void signal_free(int64_t p) { (void)hipFree(reinterpret_cast<void*>(p)); }
bool signal_wait_supported(int64_t device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, static_cast<int>(device)) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return v != 0;
}
void signal_set(int64_t p, int64_t value, int64_t stream) {
  garfield::gpu::signal_set(reinterpret_cast<void*>(p), static_cast<uint64_t>(value),
                            reinterpret_cast<hipStream_t>(stream));
  TORCH_CHECK(hipGetLastError() == hipSuccess, "garfield: signal_set launch failed");
}
void stream_wait_value(int64_t stream, int64_t p, int64_t value) {
  TORCH_CHECK(hipStreamWaitValue64(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<void*>(p),
                                   static_cast<uint64_t>(value), hipStreamWaitValueGte,
                                   0xFFFFFFFFFFFFFFFFull) == hipSuccess,
              "garfield: hipStreamWaitValue64 failed");
}
void stream_write_value(int64_t stream, int64_t p, int64_t value) {
  TORCH_CHECK(hipStreamWriteValue64(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<void*>(p),
                                    static_cast<uint64_t>(value), 0) == hipSuccess,
              "garfield: hipStreamWriteValue64 failed");
}

// Events recorded / waited for at points INSIDE a captured HIP graph. Capture puts a
// 1-thread marker kernel (k_signal_set on a per-mark word) at each point; after
// capture (torch CUDAGraph(keep_graph=True)) the marker nodes are found in the raw
// hipGraph_t and an event-record node is added behind each (another stream then
// waits with hipStreamWaitEvent: an ordinary barrier packet, not a CP value poll),
// or an event-wait node in front of the marker's dependents (the graph's later
// kernels wait for work of another stream, e.g. a weight all-gather).
// flags: 0 default (system-scope release on record), 1 device-scope release, 2 no system fence
int64_t event_create(int64_t scope) {
  hipEvent_t e = nullptr;
  unsigned flags = hipEventDisableTiming;
  if (scope == 1) flags |= hipEventReleaseToDevice;
  if (scope == 2) flags |= hipEventDisableSystemFence;
  TORCH_CHECK(hipEventCreateWithFlags(&e, flags) == hipSuccess, "garfield: hipEventCreate failed");
  return reinterpret_cast<int64_t>(e);
}
void event_destroy(int64_t e) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e)); }
void event_record(int64_t e, int64_t stream) {
  TORCH_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(e), reinterpret_cast<hipStream_t>(stream)) == hipSuccess,
              "garfield: hipEventRecord failed");
}
void event_wait(int64_t stream, int64_t e) {
  TORCH_CHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<hipEvent_t>(e), 0) ==
                  hipSuccess,
              "garfield: hipStreamWaitEvent failed");
}

namespace {
// marker nodes of the graph in insertion order, with the signal word each one stores to
std::vector<std::pair<hipGraphNode_t, int64_t>> marker_nodes(hipGraph_t g) {
  size_t count = 0;
  TORCH_CHECK(hipGraphGetNodes(g, nullptr, &count) == hipSuccess, "garfield: hipGraphGetNodes failed");
  std::vector<hipGraphNode_t> nodes(count);
  TORCH_CHECK(hipGraphGetNodes(g, nodes.data(), &count) == hipSuccess, "garfield: hipGraphGetNodes failed");
  std::vector<std::pair<hipGraphNode_t, int64_t>> out;
  const void* fn = garfield::gpu::signal_kernel();
  for (auto nd : nodes) {
    hipGraphNodeType ty;
    if (hipGraphNodeGetType(nd, &ty) != hipSuccess || ty != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams kp{};
    if (hipGraphKernelNodeGetParams(nd, &kp) != hipSuccess || kp.func != fn) continue;
    int64_t word = -1;   // -1: arguments not retrievable, matched by order
    if (kp.kernelParams != nullptr && kp.kernelParams[0] != nullptr)
      word = reinterpret_cast<int64_t>(*static_cast<unsigned long long* const*>(kp.kernelParams[0]));
    out.emplace_back(nd, word);
  }
  (void)hipGetLastError();
  return out;
}

hipGraphNode_t find_marker(const std::vector<std::pair<hipGraphNode_t, int64_t>>& marks, int64_t word, size_t i) {
  for (const auto& m : marks)
    if (m.second == word) return m.first;
  const bool by_order = !marks.empty() && marks[0].second == -1;
  TORCH_CHECK(by_order && i < marks.size(), "garfield: marker kernel for signal word ", word,
              " not found in the captured graph");
  return marks[i].first;
}
}  // namespace

std::vector<hipGraphNode_t> dependents_of(hipGraphNode_t nd) {
  size_t n = 0;
  TORCH_CHECK(hipGraphNodeGetDependentNodes(nd, nullptr, &n) == hipSuccess, "garfield: dependents query failed");
  std::vector<hipGraphNode_t> deps(n);
  if (n) TORCH_CHECK(hipGraphNodeGetDependentNodes(nd, deps.data(), &n) == hipSuccess,
                     "garfield: dependents query failed");
  return deps;
}

// Put `node` between `mk` and mk's former dependents (the chain stays linear).
void splice_after(hipGraph_t g, hipGraphNode_t mk, hipGraphNode_t node, const std::vector<hipGraphNode_t>& deps) {
  for (auto d : deps) {
    TORCH_CHECK(hipGraphRemoveDependencies(g, &mk, &d, 1) == hipSuccess, "garfield: hipGraphRemoveDependencies failed");
    TORCH_CHECK(hipGraphAddDependencies(g, &node, &d, 1) == hipSuccess, "garfield: hipGraphAddDependencies failed");
  }
}

int64_t graph_attach_record_events(int64_t graph, const std::vector<int64_t>& words,
                                   const std::vector<int64_t>& events, bool inline_) {
  TORCH_CHECK(words.size() == events.size(), "garfield: one event per marker");
  auto g = reinterpret_cast<hipGraph_t>(graph);
  const auto marks = marker_nodes(g);
  for (size_t i = 0; i < words.size(); ++i) {
    hipGraphNode_t dep = find_marker(marks, words[i], i);
    const auto after = inline_ ? dependents_of(dep) : std::vector<hipGraphNode_t>{};
    hipGraphNode_t node = nullptr;
    TORCH_CHECK(hipGraphAddEventRecordNode(&node, g, &dep, 1, reinterpret_cast<hipEvent_t>(events[i])) == hipSuccess,
                "garfield: hipGraphAddEventRecordNode failed");
    splice_after(g, dep, node, after);
  }
  return static_cast<int64_t>(marks.size());
}

int64_t graph_attach_wait_events(int64_t graph, const std::vector<int64_t>& words,
                                 const std::vector<int64_t>& events, bool inline_) {
  TORCH_CHECK(words.size() == events.size(), "garfield: one event per marker");
  auto g = reinterpret_cast<hipGraph_t>(graph);
  const auto marks = marker_nodes(g);
  for (size_t i = 0; i < words.size(); ++i) {
    hipGraphNode_t mk = find_marker(marks, words[i], i);
    const auto deps = dependents_of(mk);
    hipGraphNode_t w = nullptr;
    if (inline_) {   // marker -> wait -> the marker's former dependents
      TORCH_CHECK(hipGraphAddEventWaitNode(&w, g, &mk, 1, reinterpret_cast<hipEvent_t>(events[i])) == hipSuccess,
                  "garfield: hipGraphAddEventWaitNode failed");
      splice_after(g, mk, w, deps);
      continue;
    }
    TORCH_CHECK(hipGraphAddEventWaitNode(&w, g, nullptr, 0, reinterpret_cast<hipEvent_t>(events[i])) == hipSuccess,
                "garfield: hipGraphAddEventWaitNode failed");
    for (auto d : deps)
      TORCH_CHECK(hipGraphAddDependencies(g, &w, &d, 1) == hipSuccess, "garfield: hipGraphAddDependencies failed");
  }
  return static_cast<int64_t>(marks.size());
}

namespace garfield {
namespace rccl {
bool load(const std::string& path);
void all_to_all(int64_t comm, const void* send, void* recv, size_t count, int dtype, hipStream_t stream);
void all_gather(int64_t comm, const void* send, void* recv, size_t count, int dtype, hipStream_t stream);
void all_reduce_sum(int64_t comm, const void* send, void* recv, size_t count, int dtype, hipStream_t stream);
void exchange(int64_t comm, const int64_t* ptr, const int64_t* count, const int64_t* peer, int64_t nsend,
              int64_t nops, int dtype, hipStream_t stream);
}  // namespace rccl
}  // namespace garfield

namespace {
int nccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return 9;
    case at::kFloat: return 7;
    case at::kHalf: return 6;
    case at::kDouble: return 8;
    case at::kLong: return 4;
    case at::kInt: return 2;
    default: TORCH_CHECK(false, "garfield rccl: unsupported dtype ", t.scalar_type());
  }
  return -1;
}
void rccl_check(const at::Tensor& a, const at::Tensor& b, int64_t need_b) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.device() == b.device(), "garfield rccl: GPU tensors on one device");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous(), "garfield rccl: contiguous tensors");
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "garfield rccl: one dtype");
  TORCH_CHECK(b.numel() == need_b, "garfield rccl: output has ", b.numel(), " elements, expected ", need_b);
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("rccl_load", &garfield::rccl::load, py::arg("path"),
        "Bind torch's librccl instance (dlopen RTLD_NOLOAD) for the direct collectives; False if not found");
  m.def("rccl_all_to_all", [](int64_t comm, const at::Tensor& send, const at::Tensor& recv, int64_t world,
                              int64_t stream) {
    rccl_check(send, recv, send.numel());
    TORCH_CHECK(send.numel() % world == 0, "garfield rccl: all_to_all input not divisible by world");
    garfield::rccl::all_to_all(comm, send.data_ptr(), recv.data_ptr(), static_cast<size_t>(send.numel() / world),
                               nccl_dtype(send), reinterpret_cast<hipStream_t>(stream));
  }, py::arg("comm"), py::arg("send"), py::arg("recv"), py::arg("world"), py::arg("stream"),
     "ncclAllToAll on `stream` (no cross-stream events): chunk r of send goes to rank r, chunk r of recv comes "
     "from rank r");
  m.def("rccl_all_gather", [](int64_t comm, const at::Tensor& send, const at::Tensor& recv, int64_t world,
                              int64_t stream) {
    TORCH_CHECK(send.is_cuda() && recv.is_cuda() && recv.is_contiguous() && send.is_contiguous(),
                "garfield rccl: contiguous GPU tensors");
    TORCH_CHECK(recv.numel() == send.numel() * world && send.scalar_type() == recv.scalar_type(),
                "garfield rccl: all_gather output must be world x input");
    garfield::rccl::all_gather(comm, send.data_ptr(), recv.data_ptr(), static_cast<size_t>(send.numel()),
                               nccl_dtype(send), reinterpret_cast<hipStream_t>(stream));
  }, py::arg("comm"), py::arg("send"), py::arg("recv"), py::arg("world"), py::arg("stream"),
     "ncclAllGather on `stream` (in place when send is recv's own rank block)");
  m.def("rccl_all_reduce_sum", [](int64_t comm, const at::Tensor& send, const at::Tensor& recv, int64_t stream) {
    rccl_check(send, recv, send.numel());
    garfield::rccl::all_reduce_sum(comm, send.data_ptr(), recv.data_ptr(), static_cast<size_t>(send.numel()),
                                   nccl_dtype(send), reinterpret_cast<hipStream_t>(stream));
  }, py::arg("comm"), py::arg("send"), py::arg("recv"), py::arg("stream"), "ncclAllReduce(sum) on `stream`");
  m.def("rccl_exchange", [](int64_t comm, const std::vector<at::Tensor>& sends, const std::vector<int64_t>& to,
                            const std::vector<at::Tensor>& recvs, const std::vector<int64_t>& from, int64_t world,
                            int64_t stream) {
    TORCH_CHECK(sends.size() == to.size() && recvs.size() == from.size(), "garfield rccl: one peer per buffer");
    TORCH_CHECK(!sends.empty() || !recvs.empty(), "garfield rccl: empty exchange");
    const at::Tensor& ref = sends.empty() ? recvs[0] : sends[0];
    std::vector<int64_t> ptr, cnt, peer;
    auto add = [&](const at::Tensor& t, int64_t p) {
      TORCH_CHECK(t.is_cuda() && t.device() == ref.device() && t.is_contiguous() && t.scalar_type() == ref.scalar_type(),
                  "garfield rccl: contiguous GPU buffers of one dtype on one device");
      TORCH_CHECK(p >= 0 && p < world, "garfield rccl: peer ", p, " outside the world of ", world);
      ptr.push_back(reinterpret_cast<int64_t>(t.data_ptr()));
      cnt.push_back(t.numel());
      peer.push_back(p);
    };
    for (size_t i = 0; i < sends.size(); ++i) add(sends[i], to[i]);
    for (size_t i = 0; i < recvs.size(); ++i) add(recvs[i], from[i]);
    garfield::rccl::exchange(comm, ptr.data(), cnt.data(), peer.data(), static_cast<int64_t>(sends.size()),
                             static_cast<int64_t>(ptr.size()), nccl_dtype(ref), reinterpret_cast<hipStream_t>(stream));
  }, py::arg("comm"), py::arg("sends"), py::arg("to"), py::arg("recvs"), py::arg("from_"), py::arg("world"),
     py::arg("stream"),
     "One ncclGroup of ncclSend(sends[i] -> to[i]) and ncclRecv(recvs[i] <- from_[i]) on `stream`; transfers "
     "between one pair of ranks match in issue order");
  m.def("event_create", &event_create, py::arg("scope") = 1,
        "HIP event (no timing); scope 0: system-scope release on record (HIP default), 1: device-scope "
        "release (enough for other streams of this device), 2: no system fence");
  m.def("event_destroy", &event_destroy);
  m.def("event_record", &event_record, py::arg("event"), py::arg("stream"));
  m.def("event_wait", &event_wait, py::arg("stream"), py::arg("event"));
  m.def("graph_attach_record_events", &graph_attach_record_events, py::arg("graph"), py::arg("words"),
        py::arg("events"), py::arg("inline_") = true,
        "Add an event-record node behind each marker kernel (signal word words[i]) of a captured, not yet "
        "instantiated graph; returns the number of marker nodes found");
  m.def("graph_attach_wait_events", &graph_attach_wait_events, py::arg("graph"), py::arg("words"),
        py::arg("events"), py::arg("inline_") = true,
        "Make the nodes that follow each marker kernel (signal word words[i]) wait for events[i] (event-wait "
        "node); returns the number of marker nodes found");
  m.def("signal_add", [](int64_t p, int64_t stream) {
    garfield::gpu::signal_add(reinterpret_cast<void*>(p), reinterpret_cast<hipStream_t>(stream));
    TORCH_CHECK(hipGetLastError() == hipSuccess, "garfield: signal_add launch failed");
  }, py::arg("ptr"), py::arg("stream"), "1-lane kernel: counter word += 1 (system-scope release)");
  m.def("wait_geq", [](int64_t p, int64_t target, int64_t timeout_us, int64_t err, int64_t stream) {
    garfield::gpu::wait_geq(reinterpret_cast<const void*>(p), static_cast<uint64_t>(target),
                            static_cast<uint64_t>(timeout_us), reinterpret_cast<void*>(err),
                            reinterpret_cast<hipStream_t>(stream));
    TORCH_CHECK(hipGetLastError() == hipSuccess, "garfield: wait_geq launch failed");
  }, py::arg("ptr"), py::arg("target"), py::arg("timeout_us"), py::arg("err"), py::arg("stream"),
     "1-lane kernel on `stream`: wait until the counter word >= target (bounded by timeout_us; a miss "
     "increments err[0])");
  m.def("signal_alloc", &signal_alloc, py::arg("count"));
  m.def("signal_free", &signal_free);
  m.def("signal_wait_supported", &signal_wait_supported, py::arg("device"));
  m.def("signal_set", &signal_set, py::arg("ptr"), py::arg("value"), py::arg("stream"));
  m.def("stream_wait_value", &stream_wait_value, py::arg("stream"), py::arg("ptr"), py::arg("value"));
  m.def("stream_write_value", &stream_write_value, py::arg("stream"), py::arg("ptr"), py::arg("value"));
  m.doc() = "Garfield-MI355X native robust-aggregation kernels (gfx950 HIP + C++ thread pool)";
  m.attr("MAX_ROWS") = garfield::kMaxRows;
  m.attr("MODE_MEDIAN") = static_cast<int>(garfield::kMedian);
  m.attr("MODE_TRIMMED_MEAN") = static_cast<int>(garfield::kTrimmedMean);
  m.attr("MODE_AVERAGED_MEDIAN") = static_cast<int>(garfield::kAveragedMedian);
  m.attr("MODE_AVERAGE_NAN") = static_cast<int>(garfield::kAverageNan);
  m.attr("MODE_CONDENSE") = static_cast<int>(garfield::kCondense);
  m.attr("MODE_BULYAN_TAIL") = static_cast<int>(garfield::kBulyanTail);

  // sizing helpers
  m.def("gram_padded", &garfield::gpu::gram_padded);
  m.def("gram_grid", [](int64_t d, const at::Tensor& like, int n) { return garfield::gpu::gram_grid(d, dtype_code(like), n); });
  m.def("gram_slab_floats", &garfield::gpu::gram_slab_floats);
  m.attr("GRAM_REDUCE_GROUPS") = garfield::gpu::kGramReduceGroups;
  m.def("sqdist_grid", &garfield::gpu::sqdist_grid);

  // GPU building blocks (asynchronous on the current stream)
  def_rows(m, "gpu_gram",
           [](const at::Tensor& G, const at::Tensor& s, const at::Tensor& g) { g_gram(rows_from_2d(G, true), s, g); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& s, const at::Tensor& g) { g_gram(rows_from_list(L, true), s, g); },
           "Split-K MFMA Gram matrix G·Gᵀ (fp32 [np, np])");
  m.def("gpu_krum_select", [](const at::Tensor& gram, int n, int f, int mm, const at::Tensor& w, const at::Tensor& order,
                              const at::Tensor& scores, int batch) {
    c10::hip::HIPGuard guard(gram.device().index());
    TORCH_CHECK(order.scalar_type() == at::kInt, "order must be int32");
    TORCH_CHECK(batch >= 1, "batch must be >= 1");
    const int np = garfield::gpu::gram_padded(n);
    TORCH_CHECK(gram.numel() >= static_cast<int64_t>(batch) * np * np && w.numel() >= static_cast<int64_t>(batch) * n &&
                    order.numel() >= static_cast<int64_t>(batch) * n && scores.numel() >= static_cast<int64_t>(batch) * n,
                "gpu_krum_select: buffers too small for the batch");
    garfield::gpu::krum_select(fptr(gram), np, n, f, mm, fptr(w), order.data_ptr<int>(), fptr(scores),
                               stream_of(gram.device()), batch);
  }, py::arg("gram"), py::arg("n"), py::arg("f"), py::arg("m"), py::arg("weights"), py::arg("order"),
     py::arg("scores"), py::arg("batch") = 1,
     "Multi-Krum selection weights on device; batch > 1: gram [batch, np, np] -> weights [batch, n]");
  def_rows(m, "gpu_lw_gram",
           [](const at::Tensor& G, const at::Tensor& jobs, const at::Tensor& seg_lo, const at::Tensor& slabs,
              const at::Tensor& gram) { g_lw_gram(rows_from_2d(G, true), jobs, seg_lo, slabs, gram); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& jobs, const at::Tensor& seg_lo, const at::Tensor& slabs,
              const at::Tensor& gram) { g_lw_gram(rows_from_list(L, true), jobs, seg_lo, slabs, gram); },
           "Per-segment MFMA Gram matrices of the rows: gram [L, np, np]; jobs [J, 3] int64 (start, end, segment) "
           "ranges inside one segment each, in segment order; seg_lo [L + 1] int32 first job per segment");
  def_rows(m, "gpu_lw_bulyan_tail",
           [](const at::Tensor& G, const at::Tensor& jobs, const at::Tensor& W, int64_t t, int64_t beta,
              const at::Tensor& out) { g_lw_bulyan_tail(rows_from_2d(G, true), jobs, W, t, beta, out); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& jobs, const at::Tensor& W, int64_t t, int64_t beta,
              const at::Tensor& out) { g_lw_bulyan_tail(rows_from_list(L, true), jobs, W, t, beta, out); },
           "Layer-wise Bulyan's tail: out[x] = the averaged median (beta) of the t selection means of x's "
           "segment (W [L, t, n] fp32, jobs (start, end, segment) in local coordinates)");
  def_rows(m, "gpu_lw_combine_sgd",
           [](const at::Tensor& G, const at::Tensor& jobs, const at::Tensor& seg_off, int64_t base, const at::Tensor& w,
              const at::Tensor& p, const at::Tensor& mom, const c10::optional<at::Tensor>& sh, double lr, double mo,
              double da, double wd, bool ne, bool first) {
             g_lw_combine_sgd(rows_from_2d(G, true), jobs, seg_off, base, w, p, mom, sh, lr, mo, da, wd, ne, first);
           },
           [](const std::vector<at::Tensor>& L, const at::Tensor& jobs, const at::Tensor& seg_off, int64_t base,
              const at::Tensor& w, const at::Tensor& p, const at::Tensor& mom, const c10::optional<at::Tensor>& sh,
              double lr, double mo, double da, double wd, bool ne, bool first) {
             g_lw_combine_sgd(rows_from_list(L, true), jobs, seg_off, base, w, p, mom, sh, lr, mo, da, wd, ne, first);
           },
           "Per-segment weighted combine of the rows (weights [L, n]) fused with the SGD update; args (rows, jobs "
           "(local coordinates), seg_off (global), base (global coordinate of local 0), weights, param, mom, "
           "shadow|None, lr, momentum, dampening, weight_decay, nesterov, first_step)");
  m.def("gpu_bulyan_select", [](const at::Tensor& gram, int n, int f, int mm, int t, const at::Tensor& W, int batch) {
    c10::hip::HIPGuard guard(gram.device().index());
    TORCH_CHECK(batch >= 1, "batch must be >= 1");
    const int np = garfield::gpu::gram_padded(n);
    TORCH_CHECK(W.numel() >= static_cast<int64_t>(batch) * t * n && gram.numel() >= static_cast<int64_t>(batch) * np * np,
                "gpu_bulyan_select: buffers too small for the batch");
    garfield::gpu::bulyan_select(fptr(gram), np, n, f, mm, t, fptr(W), stream_of(gram.device()), batch);
  }, py::arg("gram"), py::arg("n"), py::arg("f"), py::arg("m"), py::arg("t"), py::arg("W"), py::arg("batch") = 1,
     "Bulyan's t selection steps on device: W [t, n]; batch > 1: gram [batch, np, np] -> W [batch, t, n]");
  m.def("gpu_brute_select", [](const at::Tensor& gram, int n, int f, const at::Tensor& best, const at::Tensor& w) {
    c10::hip::HIPGuard guard(gram.device().index());
    TORCH_CHECK(n <= 64, "brute: n must be <= 64");
    TORCH_CHECK(best.scalar_type() == at::kLong && best.numel() >= 1, "best must be an int64 tensor");
    garfield::gpu::brute_select(fptr(gram), garfield::gpu::gram_padded(n), n, f,
                                reinterpret_cast<unsigned long long*>(best.data_ptr<int64_t>()), fptr(w), stream_of(gram.device()));
  });
  m.def("gpu_aksel_select", [](const at::Tensor& slabs, int n, int c, const at::Tensor& w, const at::Tensor& dists) {
    c10::hip::HIPGuard guard(slabs.device().index());
    const int grid = static_cast<int>(slabs.numel() / n);
    garfield::gpu::aksel_select(fptr(slabs), grid, n, c, fptr(w), fptr(dists), stream_of(slabs.device()));
  });
  def_rows(m, "gpu_combine",
           [](const at::Tensor& G, const at::Tensor& w, const at::Tensor& o) { g_combine(rows_from_2d(G, true), w, o); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& w, const at::Tensor& o) { g_combine(rows_from_list(L, true), w, o); },
           "out = Σ_j w_j g_j");
  def_rows(m, "gpu_combine_sgd",
           [](const at::Tensor& G, const at::Tensor& w, const at::Tensor& p, const at::Tensor& b,
              const c10::optional<at::Tensor>& go, const c10::optional<at::Tensor>& sh, double lr, double mo, double da,
              double wd, bool ne, bool first) {
             g_combine_sgd(rows_from_2d(G, true), w, p, b, go, sh, lr, mo, da, wd, ne, first);
           },
           [](const std::vector<at::Tensor>& L, const at::Tensor& w, const at::Tensor& p, const at::Tensor& b,
              const c10::optional<at::Tensor>& go, const c10::optional<at::Tensor>& sh, double lr, double mo, double da,
              double wd, bool ne, bool first) {
             g_combine_sgd(rows_from_list(L, true), w, p, b, go, sh, lr, mo, da, wd, ne, first);
           },
           "Fused robust combine + SGD(momentum, dampening, weight decay, nesterov) on fp32 master weights; "
           "args (G, w, param, mom, grad_out|None, shadow|None, lr, momentum, dampening, weight_decay, nesterov, "
           "first_step); shadow receives a bf16/fp16 copy of the updated parameters");
  def_rows(m, "gpu_coordwise",
           [](const at::Tensor& G, int mode, int f, int beta, const c10::optional<at::Tensor>& W, int t, uint64_t seed,
              double p, const at::Tensor& o) { g_coordwise(rows_from_2d(G, true), mode, f, beta, W, t, seed, p, o); },
           [](const std::vector<at::Tensor>& L, int mode, int f, int beta, const c10::optional<at::Tensor>& W, int t,
              uint64_t seed, double p, const at::Tensor& o) { g_coordwise(rows_from_list(L, true), mode, f, beta, W, t, seed, p, o); },
           "Coordinate-wise rule (median / trimmed mean / averaged median / average-nan / condense / Bulyan tail)");
  def_rows(m, "gpu_sqdist",
           [](const at::Tensor& G, const at::Tensor& c, const at::Tensor& s) { g_sqdist(rows_from_2d(G, true), c, s); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& c, const at::Tensor& s) { g_sqdist(rows_from_list(L, true), c, s); },
           "Partial squared distances of every row to a centre (split-K slabs [grid, n])");

  m.def("gpu_flatten_cast", [](const std::vector<at::Tensor>& srcs, const at::Tensor& dst) {
    TORCH_CHECK(!srcs.empty(), "flatten_cast: empty tensor list");
    TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "flatten_cast: dst must be a contiguous device tensor");
    c10::hip::HIPGuard guard(dst.device().index());
    std::vector<const void*> ptrs;
    std::vector<int> dts;
    std::vector<int64_t> numels, offs;
    int64_t pos = 0;
    for (const auto& t : srcs) {
      const auto st = t.scalar_type();
      TORCH_CHECK((st == at::kFloat || st == at::kBFloat16 || st == at::kHalf) && t.device() == dst.device(),
                  "flatten_cast: fp32/bf16/fp16 sources on dst's device");
      TORCH_CHECK(t.is_non_overlapping_and_dense(), "flatten_cast: sources must be dense");
      ptrs.push_back(t.data_ptr());
      dts.push_back(dtype_code(t));
      numels.push_back(t.numel());
      offs.push_back(pos);
      pos += t.numel();
    }
    TORCH_CHECK(pos <= dst.numel(), "flatten_cast: destination too small (", dst.numel(), " < ", pos, ")");
    return garfield::gpu::flatten_cast(ptrs.data(), dts.data(), numels.data(), offs.data(),
                                       static_cast<int>(ptrs.size()), dst.data_ptr(), dtype_code(dst),
                                       stream_of(dst.device()));
  }, "Copy a list of dense fp32/bf16/fp16 tensors (memory order) back to back into dst, casting to dst's dtype");

  m.def("gpu_flatten_cast_at", &g_flatten_cast_at,
        "Copy dense fp32/bf16/fp16 tensors (memory order) into dst at explicit element offsets, casting to dst's dtype");

  // worker-grouped NHWC layers (bn_nhwc.hip, im2col_nhwc.hip)
  m.def("bn_part_floats", [](int64_t rg, int groups, int C) { return garfield::gpu::bn_part_floats(rg, groups, C); });
  m.def("gpu_bn_forward", &g_bn_forward,
        "Per-worker BatchNorm(+residual)(+ReLU) forward on [k*Rg, C] bf16 rows; args (x, res|None, groups, gamma, "
        "beta, eps, momentum, running_mean|None, running_var|None, part, mean, istd, scale, shift, y, relu, "
        "mask=None); mask: uint8 [numel/8] ReLU bit mask written for the backward; res_scale / res_shift "
        "([groups, C] fp32): res is a pre-BatchNorm activation added as res * res_scale + res_shift (a projection "
        "shortcut's BatchNorm folded into this apply pass)",
        py::arg("x"), py::arg("res"), py::arg("groups"), py::arg("gamma"), py::arg("beta"), py::arg("eps"),
        py::arg("momentum"), py::arg("running_mean"), py::arg("running_var"), py::arg("part"), py::arg("mean"),
        py::arg("istd"), py::arg("scale"), py::arg("shift"), py::arg("y"), py::arg("relu"),
        py::arg("mask") = py::none(), py::arg("defer_running") = false, py::arg("tile_stats") = py::none(),
        py::arg("tile_m") = 0, py::arg("tile_e") = 1, py::arg("res_scale") = py::none(),
        py::arg("res_shift") = py::none());
  m.def("gpu_bn_backward_dual", &g_bn_backward_dual,
        "Backward of a BatchNorm (a) and a folded shortcut BatchNorm (b) sharing dz = dy under mask: one statistics "
        "pass and one apply pass (or one single-kernel workgroup per channel group on small layers) read dy and the "
        "mask once",
        py::arg("xa"), py::arg("xb"), py::arg("dy"), py::arg("mask"), py::arg("groups"), py::arg("gamma_a"),
        py::arg("gamma_b"), py::arg("mean_a"), py::arg("istd_a"), py::arg("mean_b"), py::arg("istd_b"),
        py::arg("part_a"), py::arg("part_b"), py::arg("coef_a"), py::arg("coef_b"), py::arg("dxa"), py::arg("dxb"),
        py::arg("grow"), py::arg("row_stride"), py::arg("og_a"), py::arg("ob_a"), py::arg("og_b"), py::arg("ob_b"));
  m.def("bn_small", [](int64_t rg) { return garfield::gpu::bn_small(rg); },
        "True when rg rows per worker take the single-kernel BatchNorm path (whose running statistics "
        "can be deferred to gpu_bn_running_update)");
  m.def("gpu_bn_running_update", &g_bn_running_update,
        "Replay the per-worker running-statistics updates of several layers in one launch; args (jobs) with "
        "jobs = [(mean, istd, running_mean, running_var, rows_per_worker, eps, momentum), ...]");
  m.def("gpu_mean_f32", &g_mean_f32, py::arg("x"),
        "0-d fp32 mean of a contiguous fp32 GPU tensor (one workgroup, fixed summation order)");
  m.def("gpu_xent_forward", &g_xent_forward,
        "Per-worker mean cross-entropy of [groups*rows, nc] logits (nc <= 64: one thread per row; wider: one wave "
        "per row) and d(loss_g)/d(logits); args "
        "(logits, labels, groups, loss[groups] fp32, dlogits like logits)");
  m.def("gpu_xent_backward", &g_xent_backward,
        "dx = dlogits scaled row-wise by the upstream per-worker loss gradient; args (dlogits, grad_loss, groups, dx)");
  m.def("gpu_bn_backward", &g_bn_backward,
        "Per-worker BatchNorm backward; writes dγ/dβ of worker g to grow[g*row_stride + off_(gamma|beta) + c]; "
        "args (x, dy, y|mask|None, groups, gamma, mean, istd, part, coef, dx, dres|None, grow|None, row_stride, "
        "off_gamma, off_beta, relu_scale=None, relu_shift=None); the ReLU test reads y > 0 (bf16), "
        "the forward's uint8 bit mask, or recomputes bf16(x * relu_scale + relu_shift) > 0",
        py::arg("x"), py::arg("dy"), py::arg("y"), py::arg("groups"), py::arg("gamma"), py::arg("mean"),
        py::arg("istd"), py::arg("part"), py::arg("coef"), py::arg("dx"), py::arg("dres"), py::arg("grow"),
        py::arg("row_stride"), py::arg("off_gamma"), py::arg("off_beta"), py::arg("relu_scale") = py::none(),
        py::arg("relu_shift") = py::none());
  m.def("gpu_im2col", &g_im2col, "NHWC im2col of a channels_last bf16 tensor into col [N*Ho*Wo, ldc >= KH*KW*C] "
        "(pad columns zeroed); args (x, kh, kw, sh, sw, ph, pw, dh, dw, col)");
  m.def("gpu_col2im", &g_col2im, "Adjoint of gpu_im2col (gather, deterministic): dx = col2im(dcol); args "
        "(dcol, kh, kw, sh, sw, ph, pw, dh, dw, dx, accumulate=False); accumulate adds into dx",
        py::arg("dcol"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dh"), py::arg("dw"), py::arg("dx"), py::arg("accumulate") = false);

  m.attr("LARGE_ROWS") = garfield::kLargeRows;
  m.def("large_gram_slab_floats", [](int64_t n, int64_t d, const at::Tensor& like) {
    return garfield::gpu::large_gram_slab_floats(static_cast<int>(n), d, dtype_code(like));
  }, py::arg("n"), py::arg("d"), py::arg("like"), "Workspace floats gpu_large_gram needs for n rows of d elements "
     "of like's dtype");
  m.def("gpu_large_gram", &g_large_gram, py::arg("x"), py::arg("slabs"), py::arg("gram"),
        "fp32 Gram [n, n] of the [n, d] rows x (n <= LARGE_ROWS) on MFMA: split-K 64 x 64 tiles, fixed-order sums");
  m.def("gpu_large_wx", &g_large_wx, py::arg("W"), py::arg("x"), py::arg("V"),
        "V [t, d] = W [t, n] fp32 · x [n, d] on fp32 MFMA (Bulyan's selection means)");
  m.def("gpu_collude", [](const std::vector<at::Tensor>& rows, int64_t peers, bool empire, double param) {
    RowSet rs = rows_from_list(rows, true);
    TORCH_CHECK(rs.device.is_cuda(), "gpu_collude: GPU rows");
    TORCH_CHECK(peers >= 0 && peers < rs.n, "gpu_collude: 0 <= peers < number of rows");
    TORCH_CHECK(rs.dt != garfield::kF64, "gpu_collude: fp32, bf16 or fp16 rows");
    c10::hip::HIPGuard guard(rs.device.index());
    garfield::gpu::collude(rs.table, static_cast<int>(peers), rs.n - static_cast<int>(peers), rs.d, rs.dt, empire,
                           static_cast<float>(param), stream_of(rs.device));
  }, py::arg("rows"), py::arg("peers"), py::arg("empire"), py::arg("param"),
     "Colluding attacks in place on exchanged rows: rows[:peers] are the estimates, rows[peers:] the Byzantine rows "
     "(their honest gradient in, mean + z * std (lie) or -eps * mean (empire) of {own row} + estimates out)");
  m.def("gpu_large_combine", &g_large_combine,
        "out = w · x for an [n, d] gradient matrix with n <= LARGE_ROWS (fp32 accumulation); args (x, w, out)");
  m.def("gpu_large_select", &g_large_select, py::arg("gram"), py::arg("f"), py::arg("m"), py::arg("rounds"),
        py::arg("shrink"), py::arg("W"),
        "Multi-Krum (rounds=1, shrink=False) / Bulyan (rounds=t, shrink=True) selection weights W [rounds, n] "
        "from an fp32 Gram of n <= LARGE_ROWS rows, on device (fp64 distances)");
  m.def("gpu_large_coord", &g_large_coord,
        "Coordinate-wise rule on an [n, d] gradient matrix with n <= LARGE_ROWS by LDS radix select; "
        "args (x, mode 0 median | 1 trimmed-mean | 2 averaged-median, f, beta, out)");
  m.def("iwgrad_taps_per_block",
        [](int64_t kw, int64_t kh, int64_t c, int64_t cout) {
          return garfield::gpu::iwgrad_taps_per_block(static_cast<int>(kw), static_cast<int>(kh), static_cast<int>(c),
                                                      static_cast<int>(cout));
        },
        py::arg("kw"), py::arg("kh") = 3, py::arg("c") = 0, py::arg("cout") = 0,
        "Taps (1x1: 64-channel input blocks x 64-channel output blocks / 64x64 tiles) per workgroup gpu_iwgrad uses "
        "for a kh x kw kernel over c input and cout output channels");
  m.def("gpu_split_reduce_multi", &g_split_reduce_multi,
        "gpu_split_reduce for many (part, out) pairs in one launch; args (parts, outs)");
  m.def("gpu_split_reduce", &g_split_reduce,
        "out[g] = Σ_s part[s, g] (fp32 accumulation, one launch; out may be strided exchange rows); args (part, out)");
  m.def("gpu_augment_gather", &g_augment_gather,
        "Fresh batch in one launch: out[r] = normalise(random crop (pad) + flip of uint8 NHWC image src[idx[r]]), "
        "bf16 channels_last; crop/flip per row from a hash of (seed, step, r); idx None: the image index is drawn "
        "from the same hash; labels_out[r] = labels[image]; args (src, idx, seed, step, mean, std, out, pad=4, "
        "flip=True, labels=None, labels_out=None)",
        py::arg("src"), py::arg("idx"), py::arg("seed"), py::arg("step"), py::arg("mean"), py::arg("std"),
        py::arg("out"), py::arg("pad") = 4, py::arg("flip") = true, py::arg("labels") = py::none(),
        py::arg("labels_out") = py::none());
  m.def("gpu_gemm_nt", &g_gemm_nt,
        "Row-major NT GEMM on MFMA: c = a · bᵀ (+ add); args (a [M,K], b [N,K], c [M,N], add=None, stats=None, "
        "rg=0, cfg=-1); stats: fp32 per-worker BatchNorm statistics of c, laid out as gemm_nt_stats_geometry "
        "says (gpu_bn_forward's tile_stats / tile_m / tile_e); pro_scale / pro_shift [pro_groups, K] fp32: a is a "
        "pre-BatchNorm activation used as bf16(max(a * scale + shift, 0)) of its row's worker (the BatchNorm + ReLU "
        "fused into the staging of a); add_mask [M * N / 8] uint8: add counts only where its bit is set (a "
        "BatchNorm's ReLU bits: add = dy gives the residual gradient without materialising it)",
        py::arg("a"), py::arg("b"), py::arg("c"), py::arg("add") = py::none(), py::arg("stats") = py::none(),
        py::arg("rg") = 0, py::arg("cfg") = -1, py::arg("pro_scale") = py::none(), py::arg("pro_shift") = py::none(),
        py::arg("pro_groups") = 0, py::arg("add_mask") = py::none());
  m.def("bn_small_ch", &garfield::gpu::bn_small_ch,
        "Forced channels per workgroup of the single-kernel small-layer BatchNorm (GARFIELD_BN_SMALL_CH: 8, 16, 32; 0 automatic)");
  m.def("set_bn_small_ch", &garfield::gpu::set_bn_small_ch, py::arg("ch"),
        "Force the small-layer BatchNorm's channels per workgroup (8, 16 or 32; 0 automatic) for later launches");
  m.def("gemm_nt_pro_ok", [](int64_t cfg, int64_t K, int64_t prg, int64_t groups) {
    return garfield::gpu::gemm_nt_pro_ok(static_cast<int>(cfg), static_cast<int>(K), prg, static_cast<int>(groups));
  }, py::arg("cfg"), py::arg("K"), py::arg("rows_per_worker"), py::arg("groups"),
     "Whether gpu_gemm_nt configuration cfg has a BatchNorm-prologue form for this shape");
  m.def("gemm_nt_pick", [](int64_t M, int64_t N, int64_t K, int64_t rg_limit) {
    return garfield::gpu::gemm_nt_pick(M, static_cast<int>(N), static_cast<int>(K), rg_limit);
  }, "Tile configuration gpu_gemm_nt picks for M x N x K (rg_limit > 0: stats rows <= rg_limit); -1 if none");
  m.def("gemm_nt_tile", [](int64_t cfg) {
    return std::make_pair(garfield::gpu::gemm_nt_tile_m(static_cast<int>(cfg)),
                          garfield::gpu::gemm_nt_tile_n(static_cast<int>(cfg)));
  }, "(BM, BN) of a gpu_gemm_nt tile configuration");
  m.def("gpu_transpose_multi", &g_transpose_multi,
        "dsts[i] = srcs[i]ᵀ for 2-D bf16 matrices (dims multiples of 8), one launch per 40 matrices",
        py::arg("srcs"), py::arg("dsts"));
  m.def("_set_kernel_variant", [](const std::string& name, int64_t v) {
    garfield::gpu::variant_table()[name] = static_cast<int>(v);
  }, py::arg("name"), py::arg("value"), "Experiment switch of a kernel form under measurement (0: default)");
  m.def("gemm_nt_num_cfg", &garfield::gpu::gemm_nt_num_cfg, "Number of gpu_gemm_nt tile configurations");
  m.def("gemm_nt_splits", &garfield::gpu::gemm_nt_splits, py::arg("cfg"),
        "Split-K factor of a gpu_gemm_nt configuration (1: none)");
  m.def("gemm_nt_valid", [](int64_t cfg, int64_t N, int64_t K) {
    return garfield::gpu::gemm_nt_valid(static_cast<int>(cfg), static_cast<int>(N), static_cast<int>(K));
  }, "Whether configuration cfg runs an N x K weight");
  m.def("gemm_nt_stats_rows", [](int64_t cfg) { return garfield::gpu::gemm_nt_stats_rows(static_cast<int>(cfg)); },
        "Least rows per worker that configuration cfg's fused statistics need");
  m.def("gemm_nt_stats_geometry", [](int64_t cfg, int64_t M, int64_t N, int64_t K, int64_t rg) {
    int64_t H = 0;
    int E = 0;
    garfield::gpu::gemm_nt_stats_geometry(static_cast<int>(cfg), M, static_cast<int>(N), static_cast<int>(K), rg, &H, &E);
    return std::make_tuple(H, E, ((M + H - 1) / H) * E * 6 * N);
  }, "(H, E, floats): statistics tiles of H rows with E entries each (gpu_bn_forward's tile_m, tile_e) and the "
     "stats buffer size of a gpu_gemm_nt launch with fused statistics");
  m.def("gpu_iconv", &g_iconv, "Implicit-GEMM NHWC convolution on MFMA: y = conv(x, w) (+ add); args (x, w, kh, kw, "
        "sh, sw, ph, pw, dh, dw, y, add=None, pm=0, transpose_w=False); x/y/add channels_last bf16, C % 32 == 0, "
        "Cout % 64 == 0; transpose_w: w is the forward weight [C, Cout, KH, KW] whose flipped transpose is applied "
        "(the data gradient of that convolution); add_mask [y.numel() / 8] uint8: add counts where its bit is set "
        "(halo-staged 3x3 kernel only, y a separate tensor). Returns False when nothing was launched (add_mask on a "
        "shape the halo kernel does not take)",
        py::arg("x"), py::arg("w"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"), py::arg("ph"),
        py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("y"), py::arg("add") = py::none(), py::arg("pm") = 0,
        py::arg("transpose_w") = false, py::arg("stats") = py::none(), py::arg("rg") = 0,
        py::arg("add_mask") = py::none());
  m.def("conv3x3_stats_rows", [](int64_t n, int64_t h, int64_t w, int64_t c, int64_t cout) -> int64_t {
          return 16 * g_conv3x3_pick(n, h, w, c, cout);
        }, py::arg("n"), py::arg("h"), py::arg("w"), py::arg("c"), py::arg("cout"),
        "Rows per statistics tile of the halo-staged 3x3 kernel's BatchNorm-statistics epilogue (0: no fit); "
        "the stats buffer holds ceil(M / rows) * 6 * Cout floats (E = 1)");

  m.def("gpu_sc_expand", &g_sc_expand, py::arg("weights"), py::arg("hs"), py::arg("ws"), py::arg("bigs"),
        py::arg("bigTs"), "Per-step expansion of 3x3 weights for images of at most 2x2 pixels: Wbig[(p', co), (p, ci)] "
        "= W[co, h - h' + 1, w - w' + 1, ci] (0 off the kernel) and its transpose, every layer in one launch");
  m.def("gpu_sc_fold", &g_sc_fold, py::arg("slab"), py::arg("h"), py::arg("w"), py::arg("out"),
        "Fold a dense small-image weight gradient (fp32 [S, G, P*Cout, P*Cin]) onto the nine taps: out[g, co, "
        "(i, j, ci)] = Σ_s Σ over the pixel pairs of tap (i, j)");
  m.def("gpu_dgrad_s2", &g_dgrad_s2, "Data gradient of a stride-2 convolution on MFMA without a dcol matrix: dx = "
        "conv_transpose(dy, w) (+ add, in place of add when given; dx may be add); args (dy, w, kh, kw, ph, pw, dx, "
        "add=None, pm=0); w the channels_last forward weight [C, Cout, KH, KW]", py::arg("dy"), py::arg("w"),
        py::arg("kh"), py::arg("kw"), py::arg("ph"), py::arg("pw"), py::arg("dx"), py::arg("add") = py::none(),
        py::arg("pm") = 0);
  m.def("dgrad_s2_ok", &g_dgrad_s2_ok, py::arg("dy"), py::arg("dx"), py::arg("kh"), py::arg("kw"), py::arg("ph"),
        py::arg("pw"), "True when gpu_dgrad_s2 takes this geometry");
  m.def("conv3x3_pick", &g_conv3x3_pick, py::arg("n"), py::arg("h"), py::arg("w"), py::arg("c"), py::arg("cout"),
        "Pixel fragments per wave the halo-staged 3x3 kernel uses for this NHWC shape (0: it does not fit)");
  m.def("wgrad3x3_fits", &g_wgrad3x3_fits, py::arg("n"), py::arg("h"), py::arg("w"), py::arg("c"), py::arg("cout"),
        py::arg("groups"), "True when gpu_iwgrad of this 3x3 / stride-1 / pad-1 shape runs the halo-staged kernel");
  m.def("gpu_iwgrad", &g_iwgrad, "Per-worker implicit-GEMM weight gradient on MFMA: out[s, g] = Σ over pixel "
        "split s of worker g of dyᵀ · patches(x); args (x, dy, kh, kw, sh, sw, ph, pw, dh, dw, groups, out, splits, "
        "pro_scale=None, pro_shift=None); pro_*: [groups, C] BatchNorm prologue of x (1x1 only)",
        py::arg("x"), py::arg("dy"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"), py::arg("ph"),
        py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("groups"), py::arg("out"), py::arg("splits"),
        py::arg("pro_scale") = py::none(), py::arg("pro_shift") = py::none());
  m.def("gpu_conv_f32", &g_conv_f32, py::arg("src"), py::arg("w"), py::arg("kh"), py::arg("kw"),
        py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("dgrad"),
        py::arg("out"), py::arg("add") = py::none(), py::arg("pm") = 0, py::arg("ksplit") = 0,
        "fp32 NHWC implicit-GEMM convolution (forward, or with dgrad the data gradient of a convolution of this "
        "geometry, any stride) on split-bf16 MFMA (three bf16 pieces per operand, the six products of order <= 2, "
        "fp32 accumulation); w: the weight's pieces [3, Co, K]; pm 0: automatic kernel choice (split-K included "
        "unless ksplit is given), ksplit > 1: that many k-splits summed by a second pass");
  m.def("conv_f32_supported", [](int64_t cs, int64_t co) {
    garfield::gpu::ConvF32Geo g{};
    g.Cs = static_cast<int>(cs);
    g.Co = static_cast<int>(co);
    return garfield::gpu::conv_f32_supported(g);
  }, py::arg("cs"), py::arg("co"));
  m.def("gpu_wgrad_f32", &g_wgrad_f32, py::arg("x"), py::arg("dy"), py::arg("kh"), py::arg("kw"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("groups"), py::arg("out"),
        py::arg("splits"), py::arg("variant") = 0,
        "Per-worker fp32 weight gradient on split-bf16 MFMA (variant: 0 auto, 1 / 2 the 128x128 tile double- / "
        "single-buffered, 3 the 64x64 tile)");
  m.def("gpu_wsplit_multi", &g_wsplit_multi, "Per-step weight split of many fp32 weights: W -> its three bf16 "
        "pieces (row pitch ld) and, optionally, the channel-transposed pieces of the data gradient");
  m.def("gpu_linear_f32_fwd", [](const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                                 const at::Tensor& y) {
    const auto dev = x.device();
    const int64_t R = x.size(0), F = x.size(1), O = w.size(0);
    check_f32_mat(x, dev, R, F, "x");
    check_f32_mat(w, dev, O, F, "w");
    check_f32_mat(y, dev, R, O, "y");
    const float* bp = nullptr;
    if (b.has_value() && b->defined()) {
      check_f32_mat(*b, dev, 1, O, "b");
      bp = b->data_ptr<float>();
    }
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_f32_fwd(x.data_ptr<float>(), w.data_ptr<float>(), bp, static_cast<int>(R),
                                  static_cast<int>(F), static_cast<int>(O), y.data_ptr<float>(), stream_of(dev));
  }, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("y"), "fp32 classifier forward y = x wᵀ + b");
  m.def("gpu_linear_f32_dgrad", [](const at::Tensor& dl, const at::Tensor& w, const at::Tensor& dx) {
    const auto dev = dl.device();
    const int64_t R = dl.size(0), O = dl.size(1), F = w.size(1);
    check_f32_mat(dl, dev, R, O, "dl");
    check_f32_mat(w, dev, O, F, "w");
    check_f32_mat(dx, dev, R, F, "dx");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_f32_dgrad(dl.data_ptr<float>(), w.data_ptr<float>(), static_cast<int>(R),
                                    static_cast<int>(F), static_cast<int>(O), dx.data_ptr<float>(), stream_of(dev));
  }, py::arg("dl"), py::arg("w"), py::arg("dx"), "fp32 classifier data gradient dx = dl w");
  m.def("gpu_linear_f32_wgrad", [](const at::Tensor& x, const at::Tensor& dl, int64_t groups, const at::Tensor& rows,
                                   int64_t row_stride, int64_t off_w, int64_t off_b) {
    const auto dev = x.device();
    const int64_t R = x.size(0), F = x.size(1), O = dl.size(1);
    check_f32_mat(x, dev, R, F, "x");
    check_f32_mat(dl, dev, R, O, "dl");
    TORCH_CHECK(groups >= 1 && R % groups == 0, "gpu_linear_f32_wgrad: rows do not split into groups");
    TORCH_CHECK(rows.is_cuda() && rows.device() == dev && rows.scalar_type() == at::kFloat && rows.is_contiguous(),
                "gpu_linear_f32_wgrad: rows must be a contiguous fp32 exchange buffer");
    TORCH_CHECK(off_w >= 0 && row_stride >= 0 && (groups - 1) * row_stride + off_w + O * F <= rows.numel() &&
                    (off_b < 0 || (groups - 1) * row_stride + off_b + O <= rows.numel()),
                "gpu_linear_f32_wgrad: row offsets out of bounds");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_f32_wgrad(x.data_ptr<float>(), dl.data_ptr<float>(), static_cast<int>(groups),
                                    static_cast<int>(R / groups), static_cast<int>(F), static_cast<int>(O),
                                    rows.data_ptr<float>(), row_stride, off_w, off_b, stream_of(dev));
  }, py::arg("x"), py::arg("dl"), py::arg("groups"), py::arg("rows"), py::arg("row_stride"), py::arg("off_w"),
     py::arg("off_b"), "Per-worker fp32 classifier dW / db written into the exchange rows");
  auto check_bf16_mat = [](const at::Tensor& t, const at::Device& dev, int64_t r, int64_t c, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.device() == dev && t.scalar_type() == at::kBFloat16 && t.is_contiguous() &&
                    t.numel() == r * c,
                "garfield linear_bf16: ", what, " must be a contiguous bf16 [", r, ", ", c, "] tensor on ", dev);
  };
  m.def("gpu_linear_bf16_fwd", [check_bf16_mat](const at::Tensor& x, const at::Tensor& w,
                                                const c10::optional<at::Tensor>& b, const at::Tensor& y) {
    const auto dev = x.device();
    const int64_t R = x.size(0), F = x.size(1), O = w.size(0);
    check_bf16_mat(x, dev, R, F, "x");
    check_bf16_mat(w, dev, O, F, "w");
    check_bf16_mat(y, dev, R, O, "y");
    const uint16_t* bp = nullptr;
    if (b.has_value() && b->defined()) {
      check_bf16_mat(*b, dev, 1, O, "b");
      bp = reinterpret_cast<const uint16_t*>(b->data_ptr());
    }
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_bf16_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(w.data_ptr()), bp, static_cast<int>(R),
                                   static_cast<int>(F), static_cast<int>(O), reinterpret_cast<uint16_t*>(y.data_ptr()),
                                   stream_of(dev));
  }, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("y"),
     "bf16 classifier forward y = x wᵀ + b (fp32 accumulation, one rounding)");
  m.def("gpu_head_weights", [check_bf16_mat](const at::Tensor& w, const at::Tensor& wp, const at::Tensor& wpt) {
    const auto dev = w.device();
    TORCH_CHECK(w.dim() == 2 && wp.dim() == 2, "gpu_head_weights: 2-D weights");
    const int64_t O = w.size(0), F = w.size(1), Op = wp.size(0);
    TORCH_CHECK(F % 64 == 0 && Op % 64 == 0 && Op >= O && O > 0, "gpu_head_weights: F and Op multiples of 64, Op >= O");
    check_bf16_mat(w, dev, O, F, "w");
    check_bf16_mat(wp, dev, Op, F, "wp");
    check_bf16_mat(wpt, dev, F, Op, "wpt");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "gpu_head_weights: w must be 16-byte aligned");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::head_weights_bf16(reinterpret_cast<const uint16_t*>(w.data_ptr()), static_cast<int>(O),
                                     static_cast<int>(F), static_cast<int>(Op), reinterpret_cast<uint16_t*>(wp.data_ptr()),
                                     reinterpret_cast<uint16_t*>(wpt.data_ptr()), stream_of(dev));
  }, py::arg("w"), py::arg("wp"), py::arg("wpt"),
     "Padded copies of a wide head's weight: wp [Op, F] (zero rows) and wpt [F, Op] (zero columns)");
  m.def("gpu_repitch", [check_bf16_mat](const at::Tensor& src, const at::Tensor& dst, const c10::optional<at::Tensor>& b) {
    const auto dev = src.device();
    TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.size(0) == dst.size(0), "gpu_repitch: [R, a] -> [R, b]");
    const int64_t R = src.size(0), a = src.size(1), bb = dst.size(1);
    TORCH_CHECK(a % 8 == 0 && bb % 8 == 0, "gpu_repitch: row lengths must be multiples of 8");
    check_bf16_mat(src, dev, R, a, "src");
    check_bf16_mat(dst, dev, R, bb, "dst");
    const uint16_t* bp = nullptr;
    if (b.has_value() && b->defined()) {
      check_bf16_mat(*b, dev, 1, std::min(a, bb), "b");
      bp = reinterpret_cast<const uint16_t*>(b->data_ptr());
      TORCH_CHECK(reinterpret_cast<uintptr_t>(bp) % 16 == 0, "gpu_repitch: b must be 16-byte aligned");
    }
    TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
                "gpu_repitch: src and dst must be 16-byte aligned");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::repitch_bf16(reinterpret_cast<const uint16_t*>(src.data_ptr()), static_cast<int>(a),
                                reinterpret_cast<uint16_t*>(dst.data_ptr()), static_cast<int>(bb), R, bp, stream_of(dev));
  }, py::arg("src"), py::arg("dst"), py::arg("b"),
     "bf16 rows [R, a] -> [R, b]: cropped or zero-padded, + b on the copied columns");
  m.def("gpu_linear_bf16_dgrad", [check_bf16_mat](const at::Tensor& dl, const at::Tensor& w, const at::Tensor& dx) {
    const auto dev = dl.device();
    const int64_t R = dl.size(0), O = dl.size(1), F = w.size(1);
    check_bf16_mat(dl, dev, R, O, "dl");
    check_bf16_mat(w, dev, O, F, "w");
    check_bf16_mat(dx, dev, R, F, "dx");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_bf16_dgrad(reinterpret_cast<const uint16_t*>(dl.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(w.data_ptr()), static_cast<int>(R),
                                     static_cast<int>(F), static_cast<int>(O), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                                     stream_of(dev));
  }, py::arg("dl"), py::arg("w"), py::arg("dx"), "bf16 classifier data gradient dx = dl w");
  m.def("gpu_linear_bf16_wgrad", [check_bf16_mat](const at::Tensor& x, const at::Tensor& dl, int64_t groups,
                                                  const at::Tensor& rows, int64_t row_stride, int64_t off_w,
                                                  int64_t off_b) {
    const auto dev = x.device();
    const int64_t R = x.size(0), F = x.size(1), O = dl.size(1);
    check_bf16_mat(x, dev, R, F, "x");
    check_bf16_mat(dl, dev, R, O, "dl");
    TORCH_CHECK(groups >= 1 && R % groups == 0, "gpu_linear_bf16_wgrad: rows do not split into groups");
    TORCH_CHECK(rows.is_cuda() && rows.device() == dev && rows.is_contiguous() &&
                    (rows.scalar_type() == at::kFloat || rows.scalar_type() == at::kBFloat16 ||
                     rows.scalar_type() == at::kHalf),
                "gpu_linear_bf16_wgrad: rows must be a contiguous fp32 / bf16 / fp16 exchange buffer");
    TORCH_CHECK(off_w >= 0 && row_stride >= 0 && (groups - 1) * row_stride + off_w + O * F <= rows.numel() &&
                    (off_b < 0 || (groups - 1) * row_stride + off_b + O <= rows.numel()),
                "gpu_linear_bf16_wgrad: row offsets out of bounds");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_bf16_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(dl.data_ptr()), static_cast<int>(groups),
                                     static_cast<int>(R / groups), static_cast<int>(F), static_cast<int>(O),
                                     rows.data_ptr(), dtype_code(rows), row_stride, off_w, off_b, stream_of(dev));
  }, py::arg("x"), py::arg("dl"), py::arg("groups"), py::arg("rows"), py::arg("row_stride"), py::arg("off_w"),
     py::arg("off_b"), "Per-worker bf16 classifier dW / db (fp32 sums, one rounding) written into the exchange rows");
  m.def("gpu_linear_bias_grad", [](const at::Tensor& dl, int64_t groups, const at::Tensor& rows, int64_t row_stride,
                                    int64_t off_b) {
    const auto dev = dl.device();
    TORCH_CHECK(dl.is_cuda() && dl.dim() == 2 && dl.is_contiguous() &&
                    (dl.scalar_type() == at::kBFloat16 || dl.scalar_type() == at::kFloat),
                "gpu_linear_bias_grad: dl must be a contiguous 2-D bf16 / fp32 GPU tensor");
    const int64_t R = dl.size(0), O = dl.size(1);
    TORCH_CHECK(groups >= 1 && R % groups == 0, "gpu_linear_bias_grad: rows do not split into groups");
    TORCH_CHECK(rows.is_cuda() && rows.device() == dev && rows.is_contiguous() &&
                    (rows.scalar_type() == at::kFloat || rows.scalar_type() == at::kBFloat16 ||
                     rows.scalar_type() == at::kHalf),
                "gpu_linear_bias_grad: rows must be a contiguous fp32 / bf16 / fp16 exchange buffer");
    TORCH_CHECK(off_b >= 0 && row_stride >= 0 && (groups - 1) * row_stride + off_b + O <= rows.numel(),
                "gpu_linear_bias_grad: row offsets out of bounds");
    c10::hip::HIPGuard guard(dev.index());
    garfield::gpu::linear_bias_grad(dl.data_ptr(), dl.scalar_type() == at::kFloat, static_cast<int>(groups),
                                    static_cast<int>(R / groups), static_cast<int>(O), rows.data_ptr(),
                                    dtype_code(rows), row_stride, off_b, stream_of(dev));
  }, py::arg("dl"), py::arg("groups"), py::arg("rows"), py::arg("row_stride"), py::arg("off_b"),
     "Per-worker classifier bias gradient db_g[o] = sum of worker g's dl rows (fp32 sums), written into the exchange rows");
  m.def("gpu_avgpool_f32", [](const at::Tensor& x, const at::Tensor& y, bool backward) {
    // forward: x [N, C, H, W] channels_last -> y [N, C]; backward: x = dy [N, C] -> y = dx [N, C, H, W]
    const at::Tensor& big = backward ? y : x;
    const at::Tensor& small = backward ? x : y;
    const auto dev = big.device();
    if (big.scalar_type() == at::kBFloat16) {   // the bf16 step
      TORCH_CHECK(big.is_cuda() && big.dim() == 4 && big.is_contiguous(at::MemoryFormat::ChannelsLast),
                  "gpu_avgpool: the activation must be a channels_last 4-D tensor");
      const int64_t N = big.size(0), C = big.size(1), HW = big.size(2) * big.size(3);
      TORCH_CHECK(small.is_cuda() && small.device() == dev && small.scalar_type() == at::kBFloat16 &&
                      small.is_contiguous() && small.numel() == N * C,
                  "gpu_avgpool: the pooled tensor must be a contiguous bf16 [N, C] tensor");
      c10::hip::HIPGuard guard(dev.index());
      auto xp = reinterpret_cast<const uint16_t*>(x.data_ptr());
      auto yp = reinterpret_cast<uint16_t*>(y.data_ptr());
      if (backward)
        garfield::gpu::avgpool_bf16_bwd(xp, static_cast<int>(N), static_cast<int>(HW), static_cast<int>(C), yp,
                                        stream_of(dev));
      else
        garfield::gpu::avgpool_bf16_fwd(xp, static_cast<int>(N), static_cast<int>(HW), static_cast<int>(C), yp,
                                        stream_of(dev));
      return;
    }
    check_f32_cl(big, dev, "activation");
    const int64_t N = big.size(0), C = big.size(1), HW = big.size(2) * big.size(3);
    check_f32_mat(small, dev, N, C, "pooled");
    c10::hip::HIPGuard guard(dev.index());
    if (backward)
      garfield::gpu::avgpool_f32_bwd(x.data_ptr<float>(), static_cast<int>(N), static_cast<int>(HW),
                                     static_cast<int>(C), y.data_ptr<float>(), stream_of(dev));
    else
      garfield::gpu::avgpool_f32_fwd(x.data_ptr<float>(), static_cast<int>(N), static_cast<int>(HW),
                                     static_cast<int>(C), y.data_ptr<float>(), stream_of(dev));
  }, py::arg("x"), py::arg("y"), py::arg("backward"), "fp32 / bf16 NHWC global average pool (forward / backward)");
  m.def("stem_fwd_stat_tiles", [](int64_t n, int64_t h, int64_t w, int64_t kind) {
    return garfield::gpu::stem_fwd_stat_tiles(static_cast<int>(n), static_cast<int>(h), static_cast<int>(w),
                                              static_cast<int>(kind));
  }, py::arg("n"), py::arg("h"), py::arg("w"), py::arg("kind") = 0,
        "Statistics tiles (256 output pixels each) the bf16 stem forward writes for its BatchNorm (0: none)");
  m.def("stem_supported", [](int64_t h, int64_t w, int64_t kind) {
          return garfield::gpu::stem_supported(static_cast<int>(h), static_cast<int>(w), static_cast<int>(kind));
        }, py::arg("h"), py::arg("w"), py::arg("kind") = 0,
        "True when the implicit stem kernels (3 -> 64 channels; kind 0: 7x7/2 pad 3, 1: 3x3/1 pad 1) handle H x W images");
  m.def("stem_k", &garfield::gpu::stem_k, py::arg("kind") = 0, "taps x channels of the stem kind (147 / 27)");
  m.def("stem_kp", &garfield::gpu::stem_kp, py::arg("kind") = 0, "K padded to whole 32-wide k-steps (160 / 32)");
  m.def("gpu_stem_fwd", [](const at::Tensor& x, const at::Tensor& wm, const at::Tensor& y, int64_t kind,
                            const c10::optional<at::Tensor>& stats) {
    const bool split = x.scalar_type() == at::kFloat;
    const int kd = static_cast<int>(kind);
    const int K = garfield::gpu::stem_k(kd), KP = garfield::gpu::stem_kp(kd);
    const int64_t kh = kd == garfield::gpu::kStem3x3 ? 3 : 7, st = kd == garfield::gpu::kStem3x3 ? 1 : 2,
                  pd = kd == garfield::gpu::kStem3x3 ? 1 : 3;
    TORCH_CHECK(x.is_cuda() && (split || x.scalar_type() == at::kBFloat16) && x.dim() == 4 && x.size(1) == 3 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_stem_fwd: x must be a channels_last bf16 or fp32 [N, 3, H, W] tensor");
    const bool raw = !split && wm.numel() == 64 * K;   // the channels_last weight itself (padded in LDS)
    TORCH_CHECK(wm.device() == x.device() && wm.scalar_type() == at::kBFloat16 &&
                    (raw ? (wm.dim() == 4 && wm.size(2) == kh && wm.is_contiguous(at::MemoryFormat::ChannelsLast))
                         : wm.is_contiguous()) &&
                    (raw || wm.numel() == (split ? 3 : 1) * 64 * KP),
                "gpu_stem_fwd: w must be the contiguous zero-padded [64, ", KP, "] bf16 matrix, the channels_last bf16 "
                "[64, 3, ", kh, ", ", kh, "] weight (bf16 x), or (fp32 x) the pieces [3, 64, ", KP, "]");
    const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
    TORCH_CHECK(garfield::gpu::stem_supported(static_cast<int>(H), static_cast<int>(W), kd), "gpu_stem_fwd: unsupported size");
    const int64_t Ho = (H + 2 * pd - kh) / st + 1, Wo = (W + 2 * pd - kh) / st + 1;
    TORCH_CHECK(y.device() == x.device() && y.scalar_type() == x.scalar_type() && y.dim() == 4 && y.size(0) == N &&
                    y.size(1) == 64 && y.size(2) == Ho && y.size(3) == Wo &&
                    y.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_stem_fwd: y must be a channels_last [N, 64, Ho, Wo] tensor of x's dtype");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(wm.data_ptr()) % 16 == 0, "gpu_stem_fwd: w must be 16-byte aligned");
    c10::hip::HIPGuard guard(x.device().index());
    // the channel-padded weight of the bf16 7x7 form: scratch from the caching allocator (graph-pool safe)
    const int sc = split ? 0 : garfield::gpu::stem_fwd_scratch(kd);
    at::Tensor scratch = sc > 0 ? at::empty({sc}, wm.options()) : at::Tensor();
    float* sp = nullptr;
    if (stats.has_value() && stats->defined()) {
      const int64_t tiles = garfield::gpu::stem_fwd_stat_tiles(static_cast<int>(N), static_cast<int>(H),
                                                               static_cast<int>(W), kd);
      TORCH_CHECK(!split && tiles > 0, "gpu_stem_fwd: no statistics tiles for this geometry / dtype");
      TORCH_CHECK(stats->is_cuda() && stats->device() == x.device() && stats->scalar_type() == at::kFloat &&
                      stats->is_contiguous() && stats->numel() >= tiles * 2 * 3 * 64,
                  "gpu_stem_fwd: stats must be a contiguous fp32 tensor of >= ", tiles * 2 * 3 * 64, " elements");
      sp = stats->data_ptr<float>();
    }
    garfield::gpu::stem_fwd(x.data_ptr(), reinterpret_cast<const uint16_t*>(wm.data_ptr()), split,
                            static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), y.data_ptr(),
                            stream_of(x.device()), raw ? K : KP, kd,
                            sc > 0 ? reinterpret_cast<uint16_t*>(scratch.data_ptr()) : nullptr, sp);
  }, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("kind") = 0, py::arg("stats") = py::none(),
     "Implicit-GEMM ResNet stem forward (3 -> 64; kind 0: 7x7/2 pad 3, 1: 3x3/1 pad 1); fp32 x: split-bf16 MFMA on "
     "the weight's pieces");
  m.def("gpu_stem_wgrad", [](const at::Tensor& x, const at::Tensor& dy, int64_t groups, const at::Tensor& part,
                             int64_t kind) {
    const bool split = x.scalar_type() == at::kFloat;
    const int kd = static_cast<int>(kind);
    const int K = garfield::gpu::stem_k(kd);
    const int64_t kh = kd == garfield::gpu::kStem3x3 ? 3 : 7, st = kd == garfield::gpu::kStem3x3 ? 1 : 2,
                  pd = kd == garfield::gpu::kStem3x3 ? 1 : 3;
    TORCH_CHECK(x.is_cuda() && (split || x.scalar_type() == at::kBFloat16) && x.dim() == 4 && x.size(1) == 3 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_stem_wgrad: x must be a channels_last bf16 or fp32 [N, 3, H, W] tensor");
    const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
    const int64_t Ho = (H + 2 * pd - kh) / st + 1, Wo = (W + 2 * pd - kh) / st + 1;
    TORCH_CHECK(dy.device() == x.device() && dy.scalar_type() == x.scalar_type() && dy.dim() == 4 && dy.size(0) == N &&
                    dy.size(1) == 64 && dy.size(2) == Ho && dy.size(3) == Wo &&
                    dy.is_contiguous(at::MemoryFormat::ChannelsLast),
                "gpu_stem_wgrad: dy must be a channels_last [N, 64, Ho, Wo] tensor of x's dtype");
    TORCH_CHECK(groups >= 1 && N % groups == 0, "gpu_stem_wgrad: images not divisible into groups");
    TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 4 &&
                    part.size(1) == groups && part.size(2) == 64 && part.size(3) == K,
                "gpu_stem_wgrad: part must be a contiguous fp32 [slices, groups, 64, ", K, "] tensor");
    TORCH_CHECK(garfield::gpu::stem_supported(static_cast<int>(H), static_cast<int>(W), kd), "gpu_stem_wgrad: unsupported size");
    c10::hip::HIPGuard guard(x.device().index());
    garfield::gpu::stem_wgrad(x.data_ptr(), dy.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                              static_cast<int>(W), static_cast<int>(groups), static_cast<int>(part.size(0)),
                              part.data_ptr<float>(), split, stream_of(x.device()), kd);
  }, py::arg("x"), py::arg("dy"), py::arg("groups"), py::arg("part"), py::arg("kind") = 0,
     "Implicit ResNet-stem weight gradient per worker: part[s, g] = slice s of worker g's dW [64, K] (bf16 or "
     "fp32 x / dy; kind as gpu_stem_fwd)");
  m.def("gpu_maxpool_fwd", &g_maxpool_fwd, "NHWC bf16 max pooling (k x k, stride s, padding p) keeping the "
        "argmax tap per element; args (x, k, s, p, y, idx)");
  m.def("gpu_maxpool_bwd", &g_maxpool_bwd, "Max-pooling backward as a gather; args (dy, idx, k, s, p, dx)");

  // CPU building blocks (thread pool)
  def_rows(m, "cpu_pairwise",
           [](const at::Tensor& G) { return c_pairwise(rows_from_2d(G, false)); },
           [](const std::vector<at::Tensor>& L) { return c_pairwise(rows_from_list(L, false)); },
           "Pairwise squared distances (fp64 [n, n], +inf diagonal / non-finite)");
  def_rows(m, "cpu_combine",
           [](const at::Tensor& G, const at::Tensor& w) { return c_combine(rows_from_2d(G, false), w); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& w) { return c_combine(rows_from_list(L, false), w); },
           "out = Σ_j w_j g_j");
  def_rows(m, "cpu_coordwise",
           [](const at::Tensor& G, int mode, int f, int beta, const c10::optional<at::Tensor>& W, int t, uint64_t seed, double p) {
             return c_coordwise(rows_from_2d(G, false), mode, f, beta, W, t, seed, p);
           },
           [](const std::vector<at::Tensor>& L, int mode, int f, int beta, const c10::optional<at::Tensor>& W, int t,
              uint64_t seed, double p) { return c_coordwise(rows_from_list(L, false), mode, f, beta, W, t, seed, p); },
           "Coordinate-wise rule on the CPU");
  def_rows(m, "cpu_sqdist",
           [](const at::Tensor& G, const at::Tensor& c) { return c_sqdist(rows_from_2d(G, false), c); },
           [](const std::vector<at::Tensor>& L, const at::Tensor& c) { return c_sqdist(rows_from_list(L, false), c); },
           "Squared distance of every row to a centre (fp64 [n])");
  m.def("cpu_krum_weights", [](const at::Tensor& D, int f, int mm) {
    const int64_t n = D.size(0);
    std::vector<double> scores;
    auto w = garfield::cpu::krum_weights(dist_from(D), n, f, mm, &scores);
    auto s = at::empty({n}, at::TensorOptions().dtype(at::kDouble));
    std::copy(scores.begin(), scores.end(), s.data_ptr<double>());
    return py::make_tuple(weights_tensor(w, {n}), s);
  });
  m.def("cpu_bulyan_weights", [](const at::Tensor& D, int f, int mm, int t) {
    const int64_t n = D.size(0);
    return weights_tensor(garfield::cpu::bulyan_weights(dist_from(D), n, f, mm, t), {t, n});
  });
  m.def("cpu_brute_weights", [](const at::Tensor& D, int f) {
    const int64_t n = D.size(0);
    return weights_tensor(garfield::cpu::brute_weights(dist_from(D), n, f), {n});
  });
  m.def("cpu_aksel_weights", [](const at::Tensor& dists, int c) {
    const int64_t n = dists.numel();
    return weights_tensor(garfield::cpu::aksel_weights(dist_from(dists), n, c), {n});
  });
  m.def("cpu_num_threads", [] { return garfield::cpu::pool().size(); });

  garfield::mailbox::bind(m);
}
