#include "shares.hpp"

#include <algorithm>
#include <cmath>

namespace bsc {

std::vector<i64> quantize(const std::vector<double>& v, int precision) {
  double s = std::pow(10.0, precision);
  std::vector<i64> r(v.size());
  for (size_t i = 0; i < v.size(); ++i) r[i] = i64(v[i] * s);  // C++ conversion truncates like Go
  return r;
}

std::vector<double> dequantize(const std::vector<i64>& v, int precision) {
  double s = std::pow(10.0, precision);
  std::vector<double> r(v.size());
  for (size_t i = 0; i < v.size(); ++i) r[i] = double(v[i]) / s;
  return r;
}

std::vector<i64> chunk_stops(i64 d, i64 poly) {
  std::vector<i64> s;
  for (i64 i = 0; i < d; i += poly) s.push_back(std::min(i + poly, d));
  return s;
}

std::vector<i64> share_xs(i64 total) {
  std::vector<i64> xs(static_cast<size_t>(total));
  for (i64 i = 0; i < total; ++i) xs[size_t(i)] = i - 10;
  return xs;
}

i64 poly_eval(const i64* c, int n, i64 x) {
  // Horner in wrapping int64 (exact whenever the result fits)
  u64 acc = 0;
  for (int k = n - 1; k >= 0; --k) acc = acc * u64(x) + u64(c[k]);
  return i64(acc);
}

std::vector<i64> poly_quotient(const i64* c, int n, i64 x) {
  std::vector<i64> q(static_cast<size_t>(std::max(n - 1, 0)));
  u64 carry = 0;
  for (int k = n - 1; k >= 1; --k) {
    carry = carry * u64(x) + u64(c[k]);
    q[size_t(k - 1)] = i64(carry);
  }
  return q;
}

// divide a signed 128-bit value by a small signed divisor; returns false if not exact
static bool div_exact(i128 a, i64 d, i128* q) {
  if (d == 0) return false;
  i128 qq = a / d;
  if (qq * d != a) return false;
  *q = qq;
  return true;
}

bool recover_exact(const std::vector<i64>& xs, const std::vector<i64>& ys, int deg, std::vector<i64>* out) {
  int n = deg + 1;
  if (int(xs.size()) < n || xs.size() != ys.size()) return false;
  // choose the n nodes of smallest |x| (keeps divided differences small)
  std::vector<size_t> idx(xs.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
    i64 ax = xs[a] < 0 ? -xs[a] : xs[a], bx = xs[b] < 0 ? -xs[b] : xs[b];
    return ax < bx || (ax == bx && xs[a] < xs[b]);
  });
  std::vector<i128> nx(static_cast<size_t>(n)), dd(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) { nx[size_t(i)] = xs[idx[size_t(i)]]; dd[size_t(i)] = ys[idx[size_t(i)]]; }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (nx[size_t(i)] == nx[size_t(j)]) return false;
  // divided differences in place: dd[k] = f[x0..xk]
  for (int lvl = 1; lvl < n; ++lvl)
    for (int k = n - 1; k >= lvl; --k) {
      i128 q;
      if (!div_exact(dd[size_t(k)] - dd[size_t(k - 1)], i64(nx[size_t(k)] - nx[size_t(k - lvl)]), &q)) return false;
      dd[size_t(k)] = q;
    }
  // Newton -> monomial: p = dd[n-1]; p = p*(X - x_k) + dd[k]
  std::vector<i128> c(static_cast<size_t>(n), 0);
  c[0] = dd[size_t(n - 1)];
  int cur = 0;
  for (int k = n - 2; k >= 0; --k) {
    // c(X) = c(X) * (X - x_k) + dd[k]
    for (int j = cur + 1; j >= 1; --j) c[size_t(j)] = c[size_t(j - 1)] - nx[size_t(k)] * c[size_t(j)];
    c[0] = -nx[size_t(k)] * c[0] + dd[size_t(k)];
    ++cur;
  }
  std::vector<i64> res(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    if (c[size_t(i)] > i128(INT64_MAX) || c[size_t(i)] < i128(INT64_MIN)) return false;
    res[size_t(i)] = i64(c[size_t(i)]);
  }
  // consistency check on every point (exact, 128-bit)
  for (size_t p = 0; p < xs.size(); ++p) {
    i128 acc = 0;
    for (int k = n - 1; k >= 0; --k) acc = acc * xs[p] + res[size_t(k)];
    if (acc != i128(ys[p])) return false;
  }
  *out = res;
  return true;
}

std::vector<i64> recover_lstsq(const std::vector<i64>& xs, const std::vector<i64>& ys, int deg) {
  int m = int(xs.size()), n = deg + 1;
  std::vector<double> A(static_cast<size_t>(m * n)), b(static_cast<size_t>(m));
  for (int i = 0; i < m; ++i) {
    double p = 1;
    for (int j = 0; j < n; ++j) { A[size_t(i * n + j)] = p; p *= double(xs[size_t(i)]); }
    b[size_t(i)] = double(ys[size_t(i)]);
  }
  // Householder QR
  for (int k = 0; k < n && k < m; ++k) {
    double norm = 0;
    for (int i = k; i < m; ++i) norm += A[size_t(i * n + k)] * A[size_t(i * n + k)];
    norm = std::sqrt(norm);
    if (norm == 0) continue;
    double alpha = A[size_t(k * n + k)] > 0 ? -norm : norm;
    std::vector<double> v(static_cast<size_t>(m), 0);
    for (int i = k; i < m; ++i) v[size_t(i)] = A[size_t(i * n + k)];
    v[size_t(k)] -= alpha;
    double vn = 0;
    for (int i = k; i < m; ++i) vn += v[size_t(i)] * v[size_t(i)];
    if (vn == 0) continue;
    for (int j = k; j < n; ++j) {
      double s = 0;
      for (int i = k; i < m; ++i) s += v[size_t(i)] * A[size_t(i * n + j)];
      s = 2 * s / vn;
      for (int i = k; i < m; ++i) A[size_t(i * n + j)] -= s * v[size_t(i)];
    }
    double s = 0;
    for (int i = k; i < m; ++i) s += v[size_t(i)] * b[size_t(i)];
    s = 2 * s / vn;
    for (int i = k; i < m; ++i) b[size_t(i)] -= s * v[size_t(i)];
  }
  std::vector<double> x(static_cast<size_t>(n), 0);
  for (int i = n - 1; i >= 0; --i) {
    double s = b[size_t(i)];
    for (int j = i + 1; j < n; ++j) s -= A[size_t(i * n + j)] * x[size_t(j)];
    double d = A[size_t(i * n + i)];
    x[size_t(i)] = d != 0 ? s / d : 0;
  }
  std::vector<i64> r(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) r[size_t(i)] = i64(std::round(x[size_t(i)]));
  return r;
}

G1 commit(const std::vector<i64>& coeffs, const std::vector<G1>& pk, size_t offset) {
  G1 acc = G1::infinity();
  for (size_t i = 0; i < coeffs.size(); ++i) {
    if (offset + i >= pk.size()) fail("commit: key too short");
    if (coeffs[i]) acc = acc.add(pk[offset + i].mul_i64(coeffs[i]));
  }
  return acc;
}

std::vector<G1> witness_bases(const std::vector<G1>& pk, i64 d, i64 poly, i64 total) {
  auto stops = chunk_stops(d, poly);
  auto xs = share_xs(total);
  size_t J = size_t(poly - 1);
  std::vector<G1> out(stops.size() * size_t(total) * J, G1::infinity());
  i64 prev = 0;
  for (size_t k = 0; k < stops.size(); ++k) {
    i64 L = stops[k] - prev;
    for (size_t s = 0; s < size_t(total); ++s) {
      G1 b = G1::infinity();
      for (i64 j = 1; j < L; ++j) {  // B_{j,x}
        b = (j == 1) ? pk[size_t(prev)] : b.mul_i64(xs[s]).add(pk[size_t(prev + j - 1)]);
        out[(k * size_t(total) + s) * J + size_t(j - 1)] = b;
      }
    }
    prev = stops[k];
  }
  return out;
}

SharePackage make_shares(const std::vector<i64>& c, const std::vector<G1>& pk, i64 poly, i64 total) {
  SharePackage sp;
  auto stops = chunk_stops(i64(c.size()), poly);
  auto xs = share_xs(total);
  sp.commitment = G1::infinity();
  i64 prev = 0;
  for (i64 stop : stops) {
    int L = int(stop - prev);
    std::vector<i64> chunk(c.begin() + prev, c.begin() + stop);
    G1 cc = commit(chunk, pk, size_t(prev));
    sp.chunk_commit.push_back(cc);
    sp.commitment = sp.commitment.add(cc);
    for (i64 x : xs) {
      sp.ys.push_back(poly_eval(chunk.data(), L, x));
      // exact quotient in 128-bit (|q| < 2^63 * 10^9 * 10 fits), committed mod Order
      G1 w = G1::infinity();
      i128 carry = 0;
      for (int k = L - 1; k >= 1; --k) {
        carry = carry * x + chunk[size_t(k)];
        if (carry != 0) {
          u128 mag = carry < 0 ? u128(-carry) : u128(carry);
          U256 m;
          m.w[0] = u64(mag);
          m.w[1] = u64(mag >> 64);
          G1 t = pk[size_t(prev + k - 1)].mul(m);
          w = w.add(carry < 0 ? t.neg() : t);
        }
      }
      sp.witnesses.push_back(w);
    }
    prev = stop;
  }
  return sp;
}

}  // namespace bsc
