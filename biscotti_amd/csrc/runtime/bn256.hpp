// BN256 (the Go x/crypto "bn256" curve used by kyber: y^2 = x^3 + 3 over GF(p),
// p = 36u^4+36u^3+24u^2+6u+1, u = 6518589491078791937) -- host reference implementation.
//
// Reference semantics reproduced here (not translated):
//   * field constants             lib/dedis/kyber/pairing/bn256/constants.go:13-56
//   * G1 generator (1, -2)        lib/dedis/kyber/pairing/bn256/curve.go:16-21
//   * G2 generator / twist        lib/dedis/kyber/pairing/bn256/twist.go:14-30
//   * G1 marshal: 64 B affine, big-endian, Montgomery-decoded; infinity = 64 zero bytes
//                                 lib/dedis/kyber/pairing/bn256/point.go:109-166
//   * G2 marshal: 0x01||x.x||x.y||y.x||y.y (129 B); infinity = single 0x00 byte
//                                 lib/dedis/kyber/pairing/bn256/point.go:280-330
//   * scalars: mod.Int mod Order, 32-byte big-endian marshal (group/mod/int.go:314-357)
//   * Schnorr over G1 with a blake2xb challenge (DistSys/kyber.go:873-933)
//
// Representation: 4 x 64-bit little-endian limbs, Montgomery form with R = 2^256.
// The device kernels (csrc/kernels/bn256_dev.h) use 8 x 32-bit limbs of the same
// Montgomery representation, so affine coordinates can be copied between them verbatim.
#pragma once
#include "common.hpp"

namespace bsc {

struct U256 {
  u64 w[4] = {0, 0, 0, 0};  // little-endian limbs
  bool is_zero() const { return (w[0] | w[1] | w[2] | w[3]) == 0; }
  bool operator==(const U256& o) const {
    return w[0] == o.w[0] && w[1] == o.w[1] && w[2] == o.w[2] && w[3] == o.w[3];
  }
  bool operator!=(const U256& o) const { return !(*this == o); }
  static U256 from_be(const u8* p);
  void to_be(u8* p) const;
  static U256 from_u64(u64 v) { U256 r; r.w[0] = v; return r; }
  int bitlen() const;
  bool bit(int i) const { return (w[i >> 6] >> (i & 63)) & 1; }
};

int cmp(const U256& a, const U256& b);
// r = a + b, returns carry
u64 add_u256(U256& r, const U256& a, const U256& b);
// r = a - b, returns borrow
u64 sub_u256(U256& r, const U256& a, const U256& b);

// Montgomery arithmetic modulo a fixed 256-bit odd modulus.
struct MontField {
  U256 m;    // modulus
  u64 inv;   // -m^{-1} mod 2^64
  U256 r2;   // R^2 mod m
  U256 one;  // R mod m
  explicit MontField(const U256& mod);
  void add(U256& r, const U256& a, const U256& b) const;
  void sub(U256& r, const U256& a, const U256& b) const;
  void neg(U256& r, const U256& a) const;
  void mul(U256& r, const U256& a, const U256& b) const;  // Montgomery product a*b/R
  void sqr(U256& r, const U256& a) const { mul(r, a, a); }
  U256 to_mont(const U256& a) const;   // a*R mod m  (a may be >= m: it is reduced)
  U256 from_mont(const U256& a) const;
  void inv_mont(U256& r, const U256& a) const;  // Montgomery inverse via Fermat
  void pow_mont(U256& r, const U256& a, const U256& e) const;
  U256 reduce(const U256& a) const;  // a mod m (a < 2^256)
};

const MontField& Fp();  // base field
const MontField& Fr();  // scalar field (group order)
const U256& ORDER();
const U256& PRIME();

// ------------------------------------------------------------------ scalars (plain, not Montgomery)
struct Scalar {
  U256 v;  // canonical value in [0, Order)
  static Scalar from_i64(i64 x);
  static Scalar from_u256(const U256& x);  // reduced mod Order
  static Scalar from_be(const Bytes& b);   // 32 B, must be < Order
  Bytes to_be() const;
  Scalar add(const Scalar& o) const;
  Scalar sub(const Scalar& o) const;
  Scalar mul(const Scalar& o) const;
  bool operator==(const Scalar& o) const { return v == o.v; }
};

// ------------------------------------------------------------------ G1
struct G1 {
  U256 x, y, z;  // Jacobian, Montgomery; z == 0 <=> infinity
  static G1 infinity();
  static G1 generator();
  static G1 from_affine_mont(const U256& ax, const U256& ay);  // (0,0) -> infinity
  bool is_inf() const { return z.is_zero(); }
  G1 dbl() const;
  G1 add(const G1& o) const;
  G1 add_affine(const U256& ax, const U256& ay) const;  // mixed addition, (ax, ay) != infinity
  G1 neg() const;
  G1 mul(const U256& k) const;       // k taken as an integer (any 256-bit value)
  G1 mul_i64(i64 k) const;            // signed small scalar: |k|*P, negated if k<0
  void to_affine(U256& ax, U256& ay) const;  // Montgomery affine; infinity -> (0, 0)
  Bytes marshal() const;              // 64 B, kyber format
  static G1 unmarshal(const Bytes& b);  // throws on malformed / not on curve
  bool on_curve() const;
  bool equals(const G1& o) const;
};

// Fixed-base table for the generator (Schnorr nonces, key generation): 33 signed 8-bit windows x
// 128 affine multiples, so k*G costs <= 33 mixed additions and no doublings.
struct G1GenTable {
  std::vector<U256> tx, ty;  // entry w*128 + (d-1) = d * 256^w * G, affine Montgomery
  G1GenTable();
  G1 mul(const U256& k) const;
};
const G1GenTable& gen_table();
// Kyber marshals of many points with ONE field inversion (Montgomery's trick).
std::vector<Bytes> g1_marshal_batch(const std::vector<G1>& pts);

// ------------------------------------------------------------------ Fp2 / G2
struct Fp2 {
  U256 x, y;  // value x*i + y, i^2 = -1 (kyber gfP2 convention)
  static Fp2 zero() { return Fp2{}; }
  static Fp2 one();
  bool is_zero() const { return x.is_zero() && y.is_zero(); }
  bool operator==(const Fp2& o) const { return x == o.x && y == o.y; }
  Fp2 add(const Fp2& o) const;
  Fp2 sub(const Fp2& o) const;
  Fp2 neg() const;
  Fp2 mul(const Fp2& o) const;
  Fp2 sqr() const;
  Fp2 mul_fp(const U256& s) const;
  Fp2 inv() const;
};

struct G2 {
  Fp2 x, y, z;  // Jacobian over Fp2 on y^2 = x^3 + 3/xi, xi = i + 3
  static G2 infinity();
  static G2 generator();
  bool is_inf() const { return z.is_zero(); }
  G2 dbl() const;
  G2 add(const G2& o) const;
  G2 neg() const;
  G2 mul(const U256& k) const;
  void to_affine(Fp2& ax, Fp2& ay) const;
  Bytes marshal() const;                 // 129 B or [0x00] for infinity
  static G2 unmarshal(const Bytes& b);
  bool on_curve() const;
  bool equals(const G2& o) const;
};
const Fp2& twist_b();

// ------------------------------------------------------------------ Schnorr (kyber.go:873-933)
// Signature bytes = marshal(c) || marshal(r), 64 B. nonce: 32 B of entropy (the reference draws
// it from crypto/rand); pass deterministic bytes for reproducible runs.
// Batched signing pieces: nonce scalar + commitment point, then the response from T's marshal.
std::pair<Scalar, G1> schnorr_nonce(const Bytes& nonce_entropy);
Bytes schnorr_finish(const Bytes& message, const Scalar& sk, const Scalar& v, const Bytes& t_marshal);
Bytes schnorr_sign(const Bytes& message, const Scalar& sk, const Bytes& nonce_entropy);
bool schnorr_verify(const Bytes& message, const G1& pk, const Bytes& sig);
Scalar hash_schnorr(const Bytes& message, const G1& T);
// kyber Scalar().Pick(stream): rejection-sample 32 B big-endian values in (0, Order).
Scalar pick_scalar_from_xof(struct Blake2Xb& xof);

}  // namespace bsc
