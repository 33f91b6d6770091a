#include "gar_cpu.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <mutex>
#include <numeric>
#include <stdexcept>

#include "gar_common.hpp"
#include "threadpool.hpp"

namespace garfield {
namespace cpu {

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

inline double nan_to_inf(double v) { return v == v ? v : kInf; }

// Strict total order (value with NaN as +inf, index): the order every rank and
// every backend uses, so selections are identical everywhere.
inline bool key_less(double a, size_t ia, double b, size_t ib) {
  a = nan_to_inf(a);
  b = nan_to_inf(b);
  return a < b || (a == b && ia < ib);
}

}  // namespace

template <class T>
std::vector<double> pairwise_sqdist(const Rows<T>& r) {
  const size_t n = r.n, d = r.d;
  const size_t npairs = n * (n - 1) / 2;
  const size_t nchunks = default_chunks(d);
  std::vector<double> partial(nchunks * npairs, 0.0);
  parallel_for(0, d, nchunks, [&](size_t c, size_t lo, size_t hi) {
    double* out = partial.data() + c * npairs;
    size_t k = 0;
    for (size_t i = 0; i + 1 < n; ++i) {
      const T* a = r.p[i];
      for (size_t j = i + 1; j < n; ++j, ++k) {
        const T* b = r.p[j];
        double s = 0.0;
        for (size_t x = lo; x < hi; ++x) {
          const double v = static_cast<double>(a[x]) - static_cast<double>(b[x]);
          s += v * v;
        }
        out[k] = s;
      }
    }
  });
  std::vector<double> D(n * n, kInf);
  size_t k = 0;
  for (size_t i = 0; i + 1 < n; ++i) {
    for (size_t j = i + 1; j < n; ++j, ++k) {
      double s = 0.0;
      for (size_t c = 0; c < nchunks; ++c) s += partial[c * npairs + k];
      if (!std::isfinite(s)) s = kInf;
      D[i * n + j] = s;
      D[j * n + i] = s;
    }
  }
  return D;
}

// Per-row nearest set: ids of the q smallest off-diagonal distances by (D, j).
static std::vector<size_t> nearest(const std::vector<double>& D, size_t n, size_t i, size_t q) {
  std::vector<size_t> ids;
  ids.reserve(n - 1);
  for (size_t j = 0; j < n; ++j)
    if (j != i) ids.push_back(j);
  std::sort(ids.begin(), ids.end(),
            [&](size_t a, size_t b) { return key_less(D[i * n + a], a, D[i * n + b], b); });
  if (ids.size() > q) ids.resize(q);
  return ids;
}

static std::vector<size_t> rank_order(const std::vector<double>& s) {
  std::vector<size_t> order(s.size());
  std::iota(order.begin(), order.end(), size_t{0});
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return key_less(s[a], a, s[b], b); });
  return order;
}

std::vector<float> krum_weights(const std::vector<double>& D, size_t n, size_t f, size_t m,
                                std::vector<double>* scores_out) {
  if (n < 2 * f + 3) throw std::invalid_argument("krum: n must be >= 2f + 3");
  const size_t q = n - f - 2;
  std::vector<double> scores(n, 0.0);
  for (size_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (size_t j : nearest(D, n, i, q)) s += D[i * n + j];
    scores[i] = s;
  }
  const auto order = rank_order(scores);
  std::vector<float> w(n, 0.f);
  for (size_t r = 0; r < m && r < n; ++r) w[order[r]] = 1.f / static_cast<float>(m);
  if (scores_out) *scores_out = scores;
  return w;
}

std::vector<float> bulyan_weights(const std::vector<double>& D, size_t n, size_t f, size_t m, size_t t) {
  const size_t q = n - f - 2;
  std::vector<double> scores(n, 0.0);
  std::vector<double> P(n * n, 0.0);  // pruned distances: only each row's q nearest survive
  for (size_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (size_t j : nearest(D, n, i, q)) {
      s += D[i * n + j];
      P[i * n + j] = D[i * n + j];
    }
    scores[i] = s;
  }
  std::vector<float> W(t * n, 0.f);
  for (size_t k = 0; k < t; ++k) {
    const size_t mk = (m > k) ? m - k : 1;
    const auto order = rank_order(scores);
    for (size_t r = 0; r < mk && r < n; ++r) W[k * n + order[r]] = 1.f / static_cast<float>(mk);
    const size_t id = order[0];
    for (size_t i = 0; i < n; ++i)
      if (i != id) scores[i] -= P[i * n + id];
    scores[id] = static_cast<double>(FLT_MAX);
  }
  return W;
}

static unsigned long long binom(size_t a, size_t b) {
  if (b > a) return 0ull;
  if (b > a - b) b = a - b;
  unsigned long long r = 1;
  for (size_t i = 1; i <= b; ++i) r = r * static_cast<unsigned long long>(a - b + i) / i;
  return r;
}

static unsigned long long unrank_mask(unsigned long long r, size_t n, size_t k) {
  unsigned long long mask = 0ull;
  for (size_t ii = n; ii-- > 0 && k > 0;) {
    const unsigned long long c = binom(ii, k);
    if (c <= r) {
      mask |= 1ull << ii;
      r -= c;
      --k;
    }
  }
  return mask;
}

std::vector<float> brute_weights(const std::vector<double>& D, size_t n, size_t f) {
  if (n > 64) throw std::invalid_argument("brute: n must be <= 64");
  const size_t k = n - f;
  const unsigned long long total = binom(n, k);
  // distances as fp32 (non-finite -> FLT_MAX), exactly as the device search
  std::vector<float> Df(n * n);
  for (size_t e = 0; e < n * n; ++e) {
    const double v = D[e];
    Df[e] = std::isfinite(v) ? static_cast<float>(std::max(v, 0.0)) : FLT_MAX;
  }
  const size_t nchunks = static_cast<size_t>(std::min<unsigned long long>(total, 256ull));
  std::vector<std::pair<float, unsigned long long>> best(nchunks, {FLT_MAX, ~0ull});
  parallel_for(0, static_cast<size_t>(total), nchunks, [&](size_t c, size_t lo, size_t hi) {
    unsigned long long mask = unrank_mask(lo, n, k);
    std::pair<float, unsigned long long> b{std::numeric_limits<float>::infinity(), ~0ull};
    for (size_t rank = lo; rank < hi; ++rank) {
      float diam = 0.f;
      for (unsigned long long mi = mask; mi;) {
        const int i = __builtin_ctzll(mi);
        mi &= mi - 1ull;
        for (unsigned long long mj = mi; mj;) {
          const int j = __builtin_ctzll(mj);
          mj &= mj - 1ull;
          diam = std::max(diam, Df[static_cast<size_t>(i) * n + static_cast<size_t>(j)]);
        }
      }
      if (diam < b.first || (diam == b.first && rank < b.second)) b = {diam, rank};
      const unsigned long long cc = mask & (~mask + 1ull);
      const unsigned long long rr = mask + cc;
      mask = (((rr ^ mask) >> 2) / cc) | rr;
    }
    best[c] = b;
  });
  auto b = best[0];
  for (auto& x : best)
    if (x.first < b.first || (x.first == b.first && x.second < b.second)) b = x;
  const unsigned long long mask = unrank_mask(b.second, n, k);
  std::vector<float> w(n, 0.f);
  for (size_t i = 0; i < n; ++i)
    if ((mask >> i) & 1ull) w[i] = 1.f / static_cast<float>(k);
  return w;
}

std::vector<float> aksel_weights(const std::vector<double>& dists, size_t n, size_t c) {
  const auto order = rank_order(dists);
  std::vector<float> w(n, 0.f);
  for (size_t r = 0; r < c && r < n; ++r) w[order[r]] = 1.f / static_cast<float>(c);
  return w;
}

template <class T>
void combine(const Rows<T>& r, const std::vector<float>& w, T* out) {
  std::vector<size_t> sel;
  for (size_t j = 0; j < r.n; ++j)
    if (w[j] != 0.f) sel.push_back(j);
  parallel_for(0, r.d, default_chunks(r.d), [&](size_t, size_t lo, size_t hi) {
    for (size_t x = lo; x < hi; ++x) {
      double s = 0.0;
      for (size_t j : sel) s += static_cast<double>(w[j]) * static_cast<double>(r.p[j][x]);
      out[x] = static_cast<T>(s);
    }
  });
}

// Mean of the beta values of v closest to the median v[len/2] of the sorted v;
// ties broken by value (the GPU network's (key, value) order).
static double closest_mean(std::vector<double>& v, size_t len, size_t beta) {
  std::sort(v.begin(), v.begin() + static_cast<long>(len));
  const double med = v[len / 2];
  std::vector<std::pair<double, double>> kv(len);
  for (size_t i = 0; i < len; ++i) kv[i] = {nan_to_inf(std::fabs(v[i] - med)), v[i]};
  std::sort(kv.begin(), kv.end());
  double s = 0.0;
  for (size_t i = 0; i < beta && i < len; ++i) s += kv[i].second;
  return s / static_cast<double>(beta);
}

template <class T>
void coordwise(const Rows<T>& r, int mode, size_t f, size_t beta, const std::vector<float>& W, size_t t,
               uint64_t seed, uint64_t threshold, T* out) {
  const size_t n = r.n;
  parallel_for(0, r.d, default_chunks(r.d, 1024), [&](size_t, size_t lo, size_t hi) {
    std::vector<double> v(std::max(n, t) + 1);
    for (size_t x = lo; x < hi; ++x) {
      double res = 0.0;
      switch (mode) {
        case kAverageNan: {
          double s = 0.0;
          size_t c = 0;
          for (size_t i = 0; i < n; ++i) {
            const double a = static_cast<double>(r.p[i][x]);
            if (std::isfinite(a)) { s += a; ++c; }
          }
          res = c ? s / static_cast<double>(c) : 0.0;
          break;
        }
        case kMedian:
        case kCondense: {
          size_t c = 0;
          for (size_t i = 0; i < n; ++i) {
            const double a = static_cast<double>(r.p[i][x]);
            if (std::isfinite(a)) v[c++] = a;
          }
          if (c) {
            std::nth_element(v.begin(), v.begin() + static_cast<long>(c / 2), v.begin() + static_cast<long>(c));
            res = v[c / 2];
          }
          if (mode == kCondense) {
            const uint32_t draw = mix_hash(seed, static_cast<uint64_t>(x));
            if (!(static_cast<uint64_t>(draw) < threshold)) res = static_cast<double>(r.p[0][x]);
          }
          break;
        }
        case kTrimmedMean: {
          for (size_t i = 0; i < n; ++i) v[i] = nan_to_inf(static_cast<double>(r.p[i][x]));
          std::sort(v.begin(), v.begin() + static_cast<long>(n));
          double s = 0.0;
          for (size_t i = f; i < n - f; ++i) s += v[i];
          res = s / static_cast<double>(n - 2 * f);
          break;
        }
        case kAveragedMedian: {
          for (size_t i = 0; i < n; ++i) v[i] = nan_to_inf(static_cast<double>(r.p[i][x]));
          res = closest_mean(v, n, beta);
          break;
        }
        case kBulyanTail: {
          for (size_t k = 0; k < t; ++k) {
            double s = 0.0;
            for (size_t j = 0; j < n; ++j) {
              const float w = W[k * n + j];
              if (w != 0.f) s += static_cast<double>(w) * static_cast<double>(r.p[j][x]);
            }
            v[k] = nan_to_inf(s);
          }
          res = closest_mean(v, t, beta);
          break;
        }
        default:
          throw std::invalid_argument("coordwise: unknown mode");
      }
      out[x] = static_cast<T>(res);
    }
  });
}

template <class T>
std::vector<double> sqdist_to(const Rows<T>& r, const T* center) {
  const size_t n = r.n;
  const size_t nchunks = default_chunks(r.d);
  std::vector<double> partial(nchunks * n, 0.0);
  parallel_for(0, r.d, nchunks, [&](size_t c, size_t lo, size_t hi) {
    for (size_t j = 0; j < n; ++j) {
      double s = 0.0;
      for (size_t x = lo; x < hi; ++x) {
        const double a = static_cast<double>(r.p[j][x]) - static_cast<double>(center[x]);
        s += a * a;
      }
      partial[c * n + j] = s;
    }
  });
  std::vector<double> out(n, 0.0);
  for (size_t j = 0; j < n; ++j) {
    double s = 0.0;
    for (size_t c = 0; c < nchunks; ++c) s += partial[c * n + j];
    out[j] = std::isfinite(s) ? s : kInf;
  }
  return out;
}

#define GARFIELD_INSTANTIATE(T)                                                                          \
  template std::vector<double> pairwise_sqdist<T>(const Rows<T>&);                                       \
  template void combine<T>(const Rows<T>&, const std::vector<float>&, T*);                               \
  template void coordwise<T>(const Rows<T>&, int, size_t, size_t, const std::vector<float>&, size_t,     \
                             uint64_t, uint64_t, T*);                                                    \
  template std::vector<double> sqdist_to<T>(const Rows<T>&, const T*);

GARFIELD_INSTANTIATE(float)
GARFIELD_INSTANTIATE(double)
#undef GARFIELD_INSTANTIATE

}  // namespace cpu
}  // namespace garfield
