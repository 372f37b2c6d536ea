// Optimal ate pairing on the Go x/crypto / kyber BN256 curve (e: G1 x G2 -> GT subset Fp12).
//
// The reference defines verifySecret (DistSys/kyber.go:650-673), a KZG evaluation check
//   e(C, g2) == e(W, s*g2 - x*g2) * e(g1, g2)^y
// over kyber's pairing (lib/dedis/kyber/pairing/bn256/optate.go:119-268).  It is never called on the
// protocol's main path (miners trust the witnesses), but it is part of the API: this host module
// provides it for batched audits.  Only pairing *equalities* are observable through that API, so
// any non-degenerate bilinear pairing of the same groups answers identically; GT elements are not
// marshalled.
//
// Tower: Fp12 = Fp2[w] / (w^6 - xi), xi = i + 3, so the sextic twist E'(Fp2): y^2 = x^3 + 3/xi maps
// into E(Fp12) by psi(x', y') = (x' w^2, y' w^3).  Frobenius: (sum c_k w^k)^p = sum conj(c_k) g^k w^k
// with g = xi^((p-1)/6), computed at start-up instead of hard-coding tables.
#pragma once
#include "bn256.hpp"

namespace bsc {

struct Fp12 {
  Fp2 c[6];  // value sum c[k] * w^k
  static Fp12 one();
  bool is_one() const;
  bool operator==(const Fp12& o) const;
  Fp12 mul(const Fp12& o) const;
  Fp12 sqr() const;           // 21 Fp2 products (symmetric schoolbook) instead of 36
  Fp12 inv() const;
  Fp12 frob() const;          // x -> x^p
  Fp12 conj6() const;         // x -> x^(p^6)
  Fp12 pow(const U256& e) const;
};

// Miller loop + final exponentiation.  Infinity on either side gives 1.
Fp12 pairing(const G1& P, const G2& Q);
// prod_i e(P_i, Q_i) with one shared final exponentiation
Fp12 multi_pairing(const std::vector<G1>& Ps, const std::vector<G2>& Qs);
// Fixed G2 point with its Miller-loop line coefficients precomputed once (affine, so every
// inversion happens here): the loop over a prepared point is one Fp12 squaring per bit plus a sparse
// line product per step -- no inversions and no G2 arithmetic.  The KZG audit pairs against the three
// fixed points G2, s*G2 and g2key[0], so they are prepared once per run.
struct G2Prepared {
  struct Line { Fp2 lam, mu; bool skip; };   // l(P) = yP - lam xP w + mu w^3,  mu = lam xT - yT
  std::vector<Line> lines;
  bool inf = false;
};
G2Prepared g2_prepare(const G2& Q);
// prod_i e(P_i, Q_i) == 1 over prepared points: shared Fp12 squarings across the pairs and the
// final exponentiation's hard part by the BN parameter u (Scott et al., 3 exponentiations by u).
bool multi_pairing_is_one(const std::vector<G1>& Ps, const std::vector<const G2Prepared*>& Qs);
Fp12 final_exp_u(const Fp12& f);     // exposed for the equality test against the generic exponent
Fp12 final_exp_generic(const Fp12& f);
Fp12 miller_prepared(const std::vector<G1>& Ps, const std::vector<const G2Prepared*>& Qs);
// kyber.go:650-673 -- commitment C = f(s) G1, witness W = q(s) G1 with q = (f - y)/(X - x),
// g2key[0] = G2, g2key[1] = s G2:   e(C, G2) == e(W, sG2 - xG2) * e(y_base, G2)^y.
// The reference uses y_base = minerG1key[0] = G1, which is only consistent for chunk 0: chunk k is
// committed on PK[10k..] (C = s^(10k) f(s) G1, and likewise W), so its check needs
// y_base = PK_G1[10k] (quirk Q9, docs/QUIRKS.md).
bool verify_secret(const G1& commitment, const G1& witness, const G2& g2_0, const G2& g2_1, i64 x, i64 y,
                   const G1& y_base);

}  // namespace bsc
