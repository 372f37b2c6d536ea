#include "pairing.hpp"

namespace bsc {
namespace {

Fp2 fp2_from_fp(const U256& a) {
  Fp2 r;
  r.y = a;  // value x*i + y
  return r;
}
Fp2 conj(const Fp2& a) {
  Fp2 r = a;
  Fp().neg(r.x, a.x);
  return r;
}
// a * xi, xi = i + 3:  (x i + y)(i + 3) = (3x + y) i + (3y - x)
Fp2 mul_xi(const Fp2& a) {
  const MontField& F = Fp();
  Fp2 r;
  U256 t;
  F.add(t, a.x, a.x);
  F.add(t, t, a.x);
  F.add(r.x, t, a.y);
  F.add(t, a.y, a.y);
  F.add(t, t, a.y);
  F.sub(r.y, t, a.x);
  return r;
}
Fp2 fp2_pow(Fp2 a, const U256& e) {
  Fp2 r = Fp2::one();
  for (int i = e.bitlen() - 1; i >= 0; --i) {
    r = r.sqr();
    if (e.bit(i)) r = r.mul(a);
  }
  return r;
}
U256 div_small(const U256& a, u64 d) {  // a / d (exact division assumed by callers)
  U256 q;
  unsigned __int128 rem = 0;
  for (int i = 3; i >= 0; --i) {
    unsigned __int128 cur = (rem << 64) | a.w[i];
    q.w[i] = u64(cur / d);
    rem = cur % d;
  }
  return q;
}

struct Consts {
  Fp2 xi_pow[6];    // gamma^k, gamma = xi^((p-1)/6): Frobenius on w^k
  std::vector<int> hard_bits;   // (p^4 - p^2 + 1) / n, MSB first
  std::vector<int> loop_bits;   // 6u + 2, MSB first
  Consts() {
    U256 pm1;
    sub_u256(pm1, PRIME(), U256::from_u64(1));
    Fp2 xi;
    xi.x = Fp().one;
    xi.y = Fp().to_mont(U256::from_u64(3));
    const Fp2 g = fp2_pow(xi, div_small(pm1, 6));
    xi_pow[0] = Fp2::one();
    for (int k = 1; k < 6; ++k) xi_pow[k] = xi_pow[k - 1].mul(g);
    // hard part exponent, derived offline from p and n with exact integer arithmetic
    static const char* hard_hex =
        "2d48f5d6a28b7f3deeed3f421b94baf5c71111e8a7e1753b6eacb8ab9cf04ee448640d2cffe43f648a280f64fd3f8f33"
        "0ac0991f1134eb9e52f955e46c3bfc48a6b42c01710a2869419b140b103cccf38d21e80343adbacb5f95a4f039bf9611";
    for (const char* c = hard_hex; *c; ++c) {
      const int v = (*c >= 'a') ? (*c - 'a' + 10) : (*c - '0');
      for (int b = 3; b >= 0; --b) hard_bits.push_back((v >> b) & 1);
    }
    while (!hard_bits.empty() && hard_bits.front() == 0) hard_bits.erase(hard_bits.begin());
    const unsigned __int128 u = 6518589491078791937ull;
    const unsigned __int128 L = 6 * u + 2;
    for (int b = 127; b >= 0; --b) {
      const int bit = int((L >> b) & 1);
      if (loop_bits.empty() && !bit) continue;
      loop_bits.push_back(bit);
    }
  }
};
const Consts& K() {
  static const Consts k;
  return k;
}

// line through the twisted points, evaluated at P: yP + (-l xP) w + (l xT - yT) w^3
Fp12 line(const Fp2& lam, const Fp2& xT, const Fp2& yT, const U256& xP, const U256& yP) {
  Fp12 r;
  r.c[0] = fp2_from_fp(yP);
  r.c[1] = lam.mul_fp(xP).neg();
  r.c[3] = lam.mul(xT).sub(yT);
  return r;
}

Fp12 miller(const U256& xP, const U256& yP, const Fp2& xQ, const Fp2& yQ) {
  const Consts& k = K();
  Fp12 f = Fp12::one();
  Fp2 xT = xQ, yT = yQ;
  const MontField& F = Fp();
  (void)F;
  auto add_step = [&](const Fp2& xR, const Fp2& yR) {
    const Fp2 dx = xR.sub(xT);
    if (dx.is_zero()) {
      // T = -R (vertical line: lies in a proper subfield, killed by the final exponentiation)
      // or T = R (never happens on the loop for points of prime order n)
      xT = Fp2::zero();
      yT = Fp2::zero();
      return;
    }
    const Fp2 lam = yR.sub(yT).mul(dx.inv());
    f = f.mul(line(lam, xT, yT, xP, yP));
    const Fp2 x3 = lam.sqr().sub(xT).sub(xR);
    yT = lam.mul(xT.sub(x3)).sub(yT);
    xT = x3;
  };
  for (size_t i = 1; i < k.loop_bits.size(); ++i) {
    // doubling: lambda = 3 x^2 / (2 y)
    const Fp2 x2 = xT.sqr();
    const Fp2 lam = x2.add(x2).add(x2).mul(yT.add(yT).inv());
    f = f.sqr().mul(line(lam, xT, yT, xP, yP));
    const Fp2 x3 = lam.sqr().sub(xT).sub(xT);
    yT = lam.mul(xT.sub(x3)).sub(yT);
    xT = x3;
    if (k.loop_bits[i]) add_step(xQ, yQ);
  }
  // Q1 = pi(Q), Q2 = -pi^2(Q) on the twist: x -> conj(x) g^2, y -> conj(y) g^3
  const Fp2 x1 = conj(xQ).mul(k.xi_pow[2]), y1 = conj(yQ).mul(k.xi_pow[3]);
  const Fp2 x2 = conj(x1).mul(k.xi_pow[2]), y2 = conj(y1).mul(k.xi_pow[3]).neg();
  add_step(x1, y1);
  add_step(x2, y2);
  return f;
}

Fp12 final_exp_slow(const Fp12& f) {
  Fp12 a = f.conj6().mul(f.inv());   // f^(p^6 - 1)
  a = a.frob().frob().mul(a);         // ^(p^2 + 1)
  Fp12 r = a;
  const auto& hb = K().hard_bits;
  for (size_t i = 1; i < hb.size(); ++i) {
    r = r.sqr();
    if (hb[i]) r = r.mul(a);
  }
  return r;
}

}  // namespace

Fp12 Fp12::one() {
  Fp12 r;
  r.c[0] = Fp2::one();
  return r;
}
bool Fp12::operator==(const Fp12& o) const {
  for (int k = 0; k < 6; ++k)
    if (!(c[k] == o.c[k])) return false;
  return true;
}
bool Fp12::is_one() const { return *this == one(); }

Fp12 Fp12::mul(const Fp12& o) const {
  Fp2 acc[11];
  for (int i = 0; i < 6; ++i) {
    if (c[i].is_zero()) continue;
    for (int j = 0; j < 6; ++j) {
      if (o.c[j].is_zero()) continue;
      acc[i + j] = acc[i + j].add(c[i].mul(o.c[j]));
    }
  }
  Fp12 r;
  for (int k = 0; k < 6; ++k) r.c[k] = acc[k];
  for (int k = 6; k < 11; ++k) r.c[k - 6] = r.c[k - 6].add(mul_xi(acc[k]));  // w^6 = xi
  return r;
}

Fp12 Fp12::conj6() const {
  Fp12 r = *this;
  for (int k = 1; k < 6; k += 2) r.c[k] = c[k].neg();
  return r;
}

Fp12 Fp12::inv() const {
  // N = f * conj6(f) lies in Fp6 = Fp2[v], v = w^2, v^3 = xi
  const Fp12 cj = conj6();
  const Fp12 N = mul(cj);
  const Fp2 a0 = N.c[0], a1 = N.c[2], a2 = N.c[4];
  const Fp2 t0 = a0.sqr().sub(mul_xi(a1.mul(a2)));
  const Fp2 t1 = mul_xi(a2.sqr()).sub(a0.mul(a1));
  const Fp2 t2 = a1.sqr().sub(a0.mul(a2));
  const Fp2 d = a0.mul(t0).add(mul_xi(a2.mul(t1).add(a1.mul(t2))));
  const Fp2 di = d.inv();
  Fp12 ninv;
  ninv.c[0] = t0.mul(di);
  ninv.c[2] = t1.mul(di);
  ninv.c[4] = t2.mul(di);
  return cj.mul(ninv);
}

Fp12 Fp12::frob() const {
  Fp12 r;
  for (int k = 0; k < 6; ++k) r.c[k] = conj(c[k]).mul(K().xi_pow[k]);
  return r;
}

Fp12 Fp12::pow(const U256& e) const {
  Fp12 r = one();
  for (int i = e.bitlen() - 1; i >= 0; --i) {
    r = r.sqr();
    if (e.bit(i)) r = r.mul(*this);
  }
  return r;
}

Fp12 multi_pairing(const std::vector<G1>& Ps, const std::vector<G2>& Qs) {
  if (Ps.size() != Qs.size()) fail("multi_pairing: size mismatch");
  Fp12 f = Fp12::one();
  for (size_t i = 0; i < Ps.size(); ++i) {
    if (Ps[i].is_inf() || Qs[i].is_inf()) continue;
    U256 xP, yP;
    Ps[i].to_affine(xP, yP);
    Fp2 xQ, yQ;
    Qs[i].to_affine(xQ, yQ);
    f = f.mul(miller(xP, yP, xQ, yQ));
  }
  return final_exp_u(f);
}

Fp12 pairing(const G1& P, const G2& Q) { return multi_pairing({P}, {Q}); }

Fp12 Fp12::sqr() const {
  Fp2 acc[11];
  for (int i = 0; i < 6; ++i) {
    if (c[i].is_zero()) continue;
    acc[2 * i] = acc[2 * i].add(c[i].sqr());
    for (int j = i + 1; j < 6; ++j) {
      if (c[j].is_zero()) continue;
      const Fp2 t = c[i].mul(c[j]);
      acc[i + j] = acc[i + j].add(t.add(t));
    }
  }
  Fp12 r;
  for (int k = 0; k < 6; ++k) r.c[k] = acc[k];
  for (int k = 6; k < 11; ++k) r.c[k - 6] = r.c[k - 6].add(mul_xi(acc[k]));
  return r;
}

namespace {
// f * (c0 + c1 w + c3 w^3) with c0 in Fp: the shape of every Miller-loop line (18 products, not 36)
Fp12 mul_line(const Fp12& f, const U256& c0, const Fp2& c1, const Fp2& c3) {
  Fp2 acc[9];
  for (int i = 0; i < 6; ++i) {
    acc[i] = acc[i].add(f.c[i].mul_fp(c0));
    acc[i + 1] = acc[i + 1].add(f.c[i].mul(c1));
    acc[i + 3] = acc[i + 3].add(f.c[i].mul(c3));
  }
  Fp12 r;
  for (int k = 0; k < 6; ++k) r.c[k] = acc[k];
  for (int k = 6; k < 9; ++k) r.c[k - 6] = r.c[k - 6].add(mul_xi(acc[k]));
  return r;
}

// x^u, u = 6518589491078791937 (the BN parameter; 63 bits)
Fp12 pow_u(const Fp12& x) {
  const u64 u = 6518589491078791937ull;
  Fp12 r = x;
  for (int b = 61; b >= 0; --b) {
    r = r.sqr();
    if ((u >> b) & 1) r = r.mul(x);
  }
  return r;
}
}  // namespace

Fp12 final_exp_generic(const Fp12& f) { return final_exp_slow(f); }

// f^((p^12 - 1) / n).  Easy part f^((p^6 - 1)(p^2 + 1)) leaves the cyclotomic subgroup, where the
// inverse is the p^6 conjugate; the hard part (p^4 - p^2 + 1)/n = l3 p^3 + l2 p^2 + l1 p + l0 with
// l3 = 1, l2 = 6u^2 + 1, l1 = -36u^3 - 18u^2 - 12u + 1, l0 = -36u^3 - 30u^2 - 18u - 2 is evaluated as
// y0 y1^2 y2^6 y3^12 y4^18 y5^30 y6^36 (Scott, Benger, Charlemagne, Dominguez Perez, Kachisa 2009):
// 3 exponentiations by u instead of a 760-bit square-and-multiply.
Fp12 final_exp_u(const Fp12& f) {
  Fp12 a = f.conj6().mul(f.inv());
  a = a.frob().frob().mul(a);
  const Fp12 fu = pow_u(a), fu2 = pow_u(fu), fu3 = pow_u(fu2);
  const Fp12 ap = a.frob(), ap2 = ap.frob(), ap3 = ap2.frob();
  const Fp12 y0 = ap.mul(ap2).mul(ap3);
  const Fp12 y1 = a.conj6();
  const Fp12 y2 = fu2.frob().frob();
  const Fp12 y3 = fu.frob().conj6();
  const Fp12 y4 = fu.mul(fu2.frob()).conj6();
  const Fp12 y5 = fu2.conj6();
  const Fp12 y6 = fu3.mul(fu3.frob()).conj6();
  Fp12 t0 = y6.sqr().mul(y4).mul(y5);
  Fp12 t1 = y3.mul(y5).mul(t0);
  t0 = t0.mul(y2);
  t1 = t1.sqr().mul(t0);
  t1 = t1.sqr();
  t0 = t1.mul(y1);
  t1 = t1.mul(y0);
  t0 = t0.sqr();
  return t0.mul(t1);
}

G2Prepared g2_prepare(const G2& Q) {
  G2Prepared pr;
  if (Q.is_inf()) { pr.inf = true; return pr; }
  const Consts& k = K();
  Fp2 xQ, yQ;
  Q.to_affine(xQ, yQ);
  Fp2 xT = xQ, yT = yQ;
  auto add_step = [&](const Fp2& xR, const Fp2& yR) {
    const Fp2 dx = xR.sub(xT);
    if (dx.is_zero()) {   // vertical line (T = -R): a subfield element, dropped like in miller()
      pr.lines.push_back({Fp2::zero(), Fp2::zero(), true});
      xT = Fp2::zero();
      yT = Fp2::zero();
      return;
    }
    const Fp2 lam = yR.sub(yT).mul(dx.inv());
    pr.lines.push_back({lam, lam.mul(xT).sub(yT), false});
    const Fp2 x3 = lam.sqr().sub(xT).sub(xR);
    yT = lam.mul(xT.sub(x3)).sub(yT);
    xT = x3;
  };
  for (size_t i = 1; i < k.loop_bits.size(); ++i) {
    const Fp2 x2 = xT.sqr();
    const Fp2 lam = x2.add(x2).add(x2).mul(yT.add(yT).inv());
    pr.lines.push_back({lam, lam.mul(xT).sub(yT), false});
    const Fp2 x3 = lam.sqr().sub(xT).sub(xT);
    yT = lam.mul(xT.sub(x3)).sub(yT);
    xT = x3;
    if (k.loop_bits[i]) add_step(xQ, yQ);
  }
  const Fp2 x1 = conj(xQ).mul(k.xi_pow[2]), y1 = conj(yQ).mul(k.xi_pow[3]);
  const Fp2 x2 = conj(x1).mul(k.xi_pow[2]), y2 = conj(y1).mul(k.xi_pow[3]).neg();
  add_step(x1, y1);
  add_step(x2, y2);
  return pr;
}

Fp12 miller_prepared(const std::vector<G1>& Ps, const std::vector<const G2Prepared*>& Qs) {
  if (Ps.size() != Qs.size()) fail("miller_prepared: size mismatch");
  const Consts& k = K();
  struct Pair { U256 xP, yP; const G2Prepared* q; };
  std::vector<Pair> pairs;
  for (size_t i = 0; i < Ps.size(); ++i) {
    if (Ps[i].is_inf() || Qs[i]->inf) continue;
    Pair p;
    Ps[i].to_affine(p.xP, p.yP);
    p.q = Qs[i];
    pairs.push_back(p);
  }
  Fp12 f = Fp12::one();
  size_t li = 0;
  auto apply = [&](size_t idx) {
    for (const Pair& p : pairs) {
      const auto& L = p.q->lines[idx];
      if (L.skip) continue;
      f = mul_line(f, p.yP, L.lam.mul_fp(p.xP).neg(), L.mu);
    }
  };
  for (size_t i = 1; i < k.loop_bits.size(); ++i) {
    if (i > 1) f = f.sqr();
    apply(li++);
    if (k.loop_bits[i]) apply(li++);
  }
  apply(li++);
  apply(li++);
  return f;
}

bool multi_pairing_is_one(const std::vector<G1>& Ps, const std::vector<const G2Prepared*>& Qs) {
  return final_exp_u(miller_prepared(Ps, Qs)).is_one();
}

bool verify_secret(const G1& commitment, const G1& witness, const G2& g2_0, const G2& g2_1, i64 x, i64 y,
                   const G1& y_base) {
  // e(C, G2) == e(W, sG2 - xG2) * e(B, G2)^y  <=>  e(C - yB, G2) * e(-W, sG2 - xG2) == 1
  const G1 lhs1 = commitment.add(y_base.mul_i64(y).neg());
  const G2 xg2 = x >= 0 ? G2::generator().mul(U256::from_u64(u64(x)))
                        : G2::generator().mul(U256::from_u64(u64(-x))).neg();
  const G2 rhs2 = g2_1.add(xg2.neg());
  return multi_pairing({lhs1, witness.neg()}, {g2_0, rhs2}).is_one();
}

}  // namespace bsc
