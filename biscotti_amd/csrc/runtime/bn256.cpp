#include "bn256.hpp"

#include "hash.hpp"

namespace bsc {

// ------------------------------------------------------------------ U256 helpers
U256 U256::from_be(const u8* p) {
  U256 r;
  for (int i = 0; i < 4; ++i) r.w[3 - i] = load_be64(p + 8 * i);
  return r;
}
void U256::to_be(u8* p) const {
  for (int i = 0; i < 4; ++i) store_be64(p + 8 * i, w[3 - i]);
}
int U256::bitlen() const {
  for (int i = 3; i >= 0; --i)
    if (w[i]) return 64 * i + 64 - __builtin_clzll(w[i]);
  return 0;
}
int cmp(const U256& a, const U256& b) {
  for (int i = 3; i >= 0; --i) {
    if (a.w[i] < b.w[i]) return -1;
    if (a.w[i] > b.w[i]) return 1;
  }
  return 0;
}
u64 add_u256(U256& r, const U256& a, const U256& b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += u128(a.w[i]) + b.w[i];
    r.w[i] = u64(c);
    c >>= 64;
  }
  return u64(c);
}
u64 sub_u256(U256& r, const U256& a, const U256& b) {
  u64 borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = u128(a.w[i]) - b.w[i] - borrow;
    r.w[i] = u64(d);
    borrow = u64(d >> 64) & 1;
  }
  return borrow;
}

static U256 hex256(const char* s) {
  // big-endian hex string, 64 chars
  U256 r;
  for (int i = 0; i < 64; ++i) {
    char c = s[i];
    u64 v = (c <= '9') ? u64(c - '0') : u64((c | 32) - 'a' + 10);
    int limb = (63 - i) / 16, sh = ((63 - i) % 16) * 4;
    r.w[limb] |= v << sh;
  }
  return r;
}

// ------------------------------------------------------------------ MontField
MontField::MontField(const U256& mod) : m(mod) {
  // inv = -m^{-1} mod 2^64 by Newton iteration
  u64 x = 1;
  for (int i = 0; i < 7; ++i) x *= 2 - m.w[0] * x;
  inv = ~x + 1;
  // one = 2^256 mod m ; r2 = 2^512 mod m computed by doubling
  U256 t;  // t = 1
  t.w[0] = 1;
  for (int i = 0; i < 512; ++i) {
    u64 c = add_u256(t, t, t);
    U256 s;
    if (c || cmp(t, m) >= 0) { sub_u256(s, t, m); t = s; }
    if (i == 255) one = t;
  }
  r2 = t;
}

void MontField::add(U256& r, const U256& a, const U256& b) const {
  U256 s;
  u64 c = add_u256(s, a, b);
  if (c || cmp(s, m) >= 0) sub_u256(s, s, m);
  r = s;
}
void MontField::sub(U256& r, const U256& a, const U256& b) const {
  U256 s;
  if (sub_u256(s, a, b)) add_u256(s, s, m);
  r = s;
}
void MontField::neg(U256& r, const U256& a) const {
  if (a.is_zero()) { r = a; return; }
  sub_u256(r, m, a);
}
void MontField::mul(U256& r, const U256& a, const U256& b) const {
  u64 t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c = u128(t[j]) + u128(a.w[j]) * b.w[i] + (c >> 64);
      t[j] = u64(c);
    }
    c = u128(t[4]) + (c >> 64);
    t[4] = u64(c);
    t[5] = u64(c >> 64);
    u64 mm = t[0] * inv;
    c = u128(t[0]) + u128(mm) * m.w[0];
    for (int j = 1; j < 4; ++j) {
      c = u128(t[j]) + u128(mm) * m.w[j] + (c >> 64);
      t[j - 1] = u64(c);
    }
    c = u128(t[4]) + (c >> 64);
    t[3] = u64(c);
    t[4] = t[5] + u64(c >> 64);
  }
  U256 s;
  s.w[0] = t[0]; s.w[1] = t[1]; s.w[2] = t[2]; s.w[3] = t[3];
  if (t[4] || cmp(s, m) >= 0) sub_u256(s, s, m);
  r = s;
}
U256 MontField::reduce(const U256& a) const {
  U256 s = a;
  while (cmp(s, m) >= 0) sub_u256(s, s, m);
  return s;
}
U256 MontField::to_mont(const U256& a) const {
  U256 r;
  mul(r, reduce(a), r2);
  return r;
}
U256 MontField::from_mont(const U256& a) const {
  U256 r, one1;
  one1.w[0] = 1;
  mul(r, a, one1);
  return r;
}
void MontField::pow_mont(U256& r, const U256& a, const U256& e) const {
  U256 acc = one;
  for (int i = e.bitlen() - 1; i >= 0; --i) {
    mul(acc, acc, acc);
    if (e.bit(i)) mul(acc, acc, a);
  }
  r = acc;
}
void MontField::inv_mont(U256& r, const U256& a) const {
  U256 e;
  U256 two;
  two.w[0] = 2;
  sub_u256(e, m, two);
  pow_mont(r, a, e);
}

static const U256 kP = hex256("8fb501e34aa387f9aa6fecb86184dc21ee5b88d120b5b59e185cac6c5e089667");

const U256& PRIME() { return kP; }
const U256& ORDER() {
  // Order = 65000549695646603732796438742359905742570406053903786389881062969044166799969
  static const U256 o = [] {
    // decimal -> U256
    const char* s = "65000549695646603732796438742359905742570406053903786389881062969044166799969";
    U256 r;
    for (const char* c = s; *c; ++c) {
      // r = r*10 + d
      u128 carry = u64(*c - '0');
      for (int i = 0; i < 4; ++i) {
        u128 v = u128(r.w[i]) * 10 + carry;
        r.w[i] = u64(v);
        carry = v >> 64;
      }
    }
    return r;
  }();
  return o;
}
const MontField& Fp() {
  static const MontField f([] {
    const char* s = "65000549695646603732796438742359905742825358107623003571877145026864184071783";
    U256 r;
    for (const char* c = s; *c; ++c) {
      u128 carry = u64(*c - '0');
      for (int i = 0; i < 4; ++i) {
        u128 v = u128(r.w[i]) * 10 + carry;
        r.w[i] = u64(v);
        carry = v >> 64;
      }
    }
    if (r != kP) fail("bn256: prime constant mismatch");
    return r;
  }());
  return f;
}
const MontField& Fr() {
  static const MontField f(ORDER());
  return f;
}

// ------------------------------------------------------------------ Scalar
Scalar Scalar::from_u256(const U256& x) { Scalar s; s.v = Fr().reduce(x); return s; }
Scalar Scalar::from_i64(i64 x) {
  Scalar s;
  if (x >= 0) { s.v.w[0] = u64(x); return s; }
  U256 mag;
  mag.w[0] = u64(0) - u64(x);
  sub_u256(s.v, ORDER(), mag);
  return s;
}
Scalar Scalar::from_be(const Bytes& b) {
  if (b.size() != 32) fail("scalar: wrong size buffer");
  Scalar s;
  s.v = U256::from_be(b.data());
  if (cmp(s.v, ORDER()) >= 0) fail("scalar: value out of range");
  return s;
}
Bytes Scalar::to_be() const { Bytes b(32); v.to_be(b.data()); return b; }
Scalar Scalar::add(const Scalar& o) const { Scalar r; Fr().add(r.v, v, o.v); return r; }
Scalar Scalar::sub(const Scalar& o) const { Scalar r; Fr().sub(r.v, v, o.v); return r; }
Scalar Scalar::mul(const Scalar& o) const {
  Scalar r;
  U256 t;
  Fr().mul(t, v, o.v);        // v*o/R
  Fr().mul(r.v, t, Fr().r2);  // * R^2 / R = v*o
  return r;
}

// ------------------------------------------------------------------ G1
static U256 mont_small(u64 v) { return Fp().to_mont(U256::from_u64(v)); }

G1 G1::infinity() { G1 p; p.y = Fp().one; return p; }
G1 G1::generator() {
  G1 g;
  g.x = Fp().one;
  Fp().neg(g.y, mont_small(2));
  g.z = Fp().one;
  return g;
}
G1 G1::from_affine_mont(const U256& ax, const U256& ay) {
  if (ax.is_zero() && ay.is_zero()) return infinity();
  G1 p; p.x = ax; p.y = ay; p.z = Fp().one;
  return p;
}

G1 G1::dbl() const {
  const MontField& F = Fp();
  if (is_inf()) return *this;
  U256 A, B, C, D, E, Fv, t;
  F.sqr(A, x);
  F.sqr(B, y);
  F.sqr(C, B);
  F.add(t, x, B); F.sqr(t, t); F.sub(t, t, A); F.sub(t, t, C); F.add(D, t, t);
  F.add(E, A, A); F.add(E, E, A);
  F.sqr(Fv, E);
  G1 r;
  F.sub(r.x, Fv, D); F.sub(r.x, r.x, D);
  U256 c8; F.add(c8, C, C); F.add(c8, c8, c8); F.add(c8, c8, c8);
  F.sub(t, D, r.x); F.mul(t, E, t); F.sub(r.y, t, c8);
  F.mul(t, y, z); F.add(r.z, t, t);
  return r;
}

G1 G1::add(const G1& o) const {
  const MontField& F = Fp();
  if (is_inf()) return o;
  if (o.is_inf()) return *this;
  U256 z1z1, z2z2, u1, u2, s1, s2, h, i, j, r, v, t;
  F.sqr(z1z1, z);
  F.sqr(z2z2, o.z);
  F.mul(u1, x, z2z2);
  F.mul(u2, o.x, z1z1);
  F.mul(t, o.z, z2z2); F.mul(s1, y, t);
  F.mul(t, z, z1z1); F.mul(s2, o.y, t);
  F.sub(h, u2, u1);
  F.sub(r, s2, s1);
  if (h.is_zero()) {
    if (r.is_zero()) return dbl();
    return infinity();
  }
  F.add(i, h, h); F.sqr(i, i);
  F.mul(j, h, i);
  F.add(r, r, r);
  F.mul(v, u1, i);
  G1 out;
  F.sqr(out.x, r); F.sub(out.x, out.x, j); F.sub(out.x, out.x, v); F.sub(out.x, out.x, v);
  F.sub(t, v, out.x); F.mul(t, r, t);
  U256 s1j; F.mul(s1j, s1, j); F.add(s1j, s1j, s1j);
  F.sub(out.y, t, s1j);
  F.add(t, z, o.z); F.sqr(t, t); F.sub(t, t, z1z1); F.sub(t, t, z2z2); F.mul(out.z, t, h);
  return out;
}

// madd-2007-bl (a = 0) with the exceptional cases handled: P == Q doubles, P == -Q -> infinity
G1 G1::add_affine(const U256& ax, const U256& ay) const {
  const MontField& F = Fp();
  if (is_inf()) return from_affine_mont(ax, ay);
  U256 z1z1, u2, s2, h, hh, i, j, r, v, t;
  F.sqr(z1z1, z);
  F.mul(u2, ax, z1z1);
  F.mul(t, z, z1z1); F.mul(s2, ay, t);
  F.sub(h, u2, x);
  F.sub(r, s2, y);
  if (h.is_zero()) {
    if (r.is_zero()) return dbl();
    return infinity();
  }
  F.sqr(hh, h);
  F.add(i, hh, hh); F.add(i, i, i);
  F.mul(j, h, i);
  F.add(r, r, r);
  F.mul(v, x, i);
  G1 out;
  F.sqr(out.x, r); F.sub(out.x, out.x, j); F.sub(out.x, out.x, v); F.sub(out.x, out.x, v);
  F.sub(t, v, out.x); F.mul(t, r, t);
  U256 yj; F.mul(yj, y, j); F.add(yj, yj, yj);
  F.sub(out.y, t, yj);
  F.add(t, z, h); F.sqr(t, t); F.sub(t, t, z1z1); F.sub(out.z, t, hh);
  return out;
}

std::vector<Bytes> g1_marshal_batch(const std::vector<G1>& pts) {
  const MontField& F = Fp();
  const size_t n = pts.size();
  std::vector<U256> pre(n);
  U256 acc = F.one;
  for (size_t i = 0; i < n; ++i) {
    pre[i] = acc;
    if (!pts[i].is_inf()) F.mul(acc, acc, pts[i].z);
  }
  U256 inv;
  F.inv_mont(inv, acc);
  std::vector<Bytes> out(n, Bytes(64, 0));
  for (size_t k = n; k-- > 0;) {
    if (pts[k].is_inf()) continue;
    U256 zi, zi2, zi3, ax, ay;
    F.mul(zi, inv, pre[k]);
    F.mul(inv, inv, pts[k].z);
    F.sqr(zi2, zi);
    F.mul(zi3, zi2, zi);
    F.mul(ax, pts[k].x, zi2);
    F.mul(ay, pts[k].y, zi3);
    F.from_mont(ax).to_be(out[k].data());
    F.from_mont(ay).to_be(out[k].data() + 32);
  }
  return out;
}

G1 G1::neg() const {
  G1 r = *this;
  Fp().neg(r.y, y);
  return r;
}

G1 G1::mul(const U256& k) const {
  G1 acc = infinity();
  for (int i = k.bitlen() - 1; i >= 0; --i) {
    acc = acc.dbl();
    if (k.bit(i)) acc = acc.add(*this);
  }
  return acc;
}

G1 G1::mul_i64(i64 k) const {
  if (k == 0) return infinity();
  u64 mag = k < 0 ? u64(0) - u64(k) : u64(k);
  G1 r = mul(U256::from_u64(mag));
  return k < 0 ? r.neg() : r;
}

void G1::to_affine(U256& ax, U256& ay) const {
  const MontField& F = Fp();
  if (is_inf()) { ax = U256(); ay = U256(); return; }
  U256 zi, zi2, zi3;
  F.inv_mont(zi, z);
  F.sqr(zi2, zi);
  F.mul(zi3, zi2, zi);
  F.mul(ax, x, zi2);
  F.mul(ay, y, zi3);
}

Bytes G1::marshal() const {
  Bytes out(64, 0);
  if (is_inf()) return out;
  U256 ax, ay;
  to_affine(ax, ay);
  Fp().from_mont(ax).to_be(out.data());
  Fp().from_mont(ay).to_be(out.data() + 32);
  return out;
}

bool G1::on_curve() const {
  if (is_inf()) return true;
  const MontField& F = Fp();
  U256 ax, ay, y2, x3;
  to_affine(ax, ay);
  F.sqr(y2, ay);
  F.sqr(x3, ax); F.mul(x3, x3, ax); F.add(x3, x3, mont_small(3));
  return y2 == x3;
}

G1 G1::unmarshal(const Bytes& b) {
  if (b.size() < 64) fail("bn256.G1: not enough data");
  U256 x = U256::from_be(b.data()), y = U256::from_be(b.data() + 32);
  if (x.is_zero() && y.is_zero()) return infinity();
  G1 p = from_affine_mont(Fp().to_mont(x), Fp().to_mont(y));
  if (!p.on_curve()) fail("bn256.G1: malformed point");
  return p;
}

bool G1::equals(const G1& o) const { return marshal() == o.marshal(); }

G1GenTable::G1GenTable() {
  constexpr int NWIN = 33, E = 128;
  tx.resize(NWIN * E);
  ty.resize(NWIN * E);
  const MontField& F = Fp();
  G1 base = G1::generator();
  std::vector<G1> row(E);
  for (int w = 0; w < NWIN; ++w) {
    row[0] = base;
    for (int d = 1; d < E; ++d) row[d] = row[d - 1].add(base);
    // one inversion per window (Montgomery's trick); multiples of G are never infinity here
    std::vector<U256> pre(E);
    U256 acc = F.one;
    for (int d = 0; d < E; ++d) { pre[d] = acc; F.mul(acc, acc, row[d].z); }
    U256 inv;
    F.inv_mont(inv, acc);
    for (int d = E - 1; d >= 0; --d) {
      U256 zi, zi2, zi3;
      F.mul(zi, inv, pre[d]);
      F.mul(inv, inv, row[d].z);
      F.sqr(zi2, zi);
      F.mul(zi3, zi2, zi);
      F.mul(tx[w * E + d], row[d].x, zi2);
      F.mul(ty[w * E + d], row[d].y, zi3);
    }
    for (int i = 0; i < 8; ++i) base = base.dbl();
  }
}
G1 G1GenTable::mul(const U256& k) const {
  // signed radix-256 digits in [-127, 128]
  G1 acc = G1::infinity();
  int carry = 0;
  for (int w = 0; w < 33; ++w) {
    int d = carry + (w < 32 ? int((k.w[w / 8] >> ((w % 8) * 8)) & 0xFF) : 0);
    if (d > 128) { d -= 256; carry = 1; } else { carry = 0; }
    if (d == 0) continue;
    const int ad = d < 0 ? -d : d;
    const U256& x = tx[w * 128 + ad - 1];
    if (d > 0) {
      acc = acc.add_affine(x, ty[w * 128 + ad - 1]);
    } else {
      U256 ny;
      Fp().neg(ny, ty[w * 128 + ad - 1]);
      acc = acc.add_affine(x, ny);
    }
  }
  return acc;
}
const G1GenTable& gen_table() {
  static const G1GenTable t;
  return t;
}

// ------------------------------------------------------------------ Fp2
Fp2 Fp2::one() { Fp2 r; r.y = Fp().one; return r; }
Fp2 Fp2::add(const Fp2& o) const { Fp2 r; Fp().add(r.x, x, o.x); Fp().add(r.y, y, o.y); return r; }
Fp2 Fp2::sub(const Fp2& o) const { Fp2 r; Fp().sub(r.x, x, o.x); Fp().sub(r.y, y, o.y); return r; }
Fp2 Fp2::neg() const { Fp2 r; Fp().neg(r.x, x); Fp().neg(r.y, y); return r; }
Fp2 Fp2::mul(const Fp2& o) const {
  // (x i + y)(ox i + oy) = (x oy + y ox) i + (y oy - x ox)
  // Karatsuba: x oy + y ox = (x + y)(ox + oy) - x ox - y oy  (3 products)
  const MontField& F = Fp();
  U256 c, d, s1, s2, m;
  F.mul(c, y, o.y); F.mul(d, x, o.x);
  F.add(s1, x, y); F.add(s2, o.x, o.y);
  F.mul(m, s1, s2);
  Fp2 r;
  F.sub(m, m, c);
  F.sub(r.x, m, d);
  F.sub(r.y, c, d);
  return r;
}
Fp2 Fp2::sqr() const {
  // (x i + y)^2 = 2xy i + (y + x)(y - x)  (2 products)
  const MontField& F = Fp();
  U256 a, b, t;
  F.add(a, y, x); F.sub(b, y, x);
  Fp2 r;
  F.mul(r.y, a, b);
  F.mul(t, x, y);
  F.add(r.x, t, t);
  return r;
}
Fp2 Fp2::mul_fp(const U256& s) const { Fp2 r; Fp().mul(r.x, x, s); Fp().mul(r.y, y, s); return r; }
Fp2 Fp2::inv() const {
  const MontField& F = Fp();
  U256 n, t, ni;
  F.sqr(n, x); F.sqr(t, y); F.add(n, n, t);
  F.inv_mont(ni, n);
  Fp2 r;
  F.neg(r.x, x); F.mul(r.x, r.x, ni);
  F.mul(r.y, y, ni);
  return r;
}

static U256 limbs(u64 a, u64 b, u64 c, u64 d) { U256 r; r.w[0] = a; r.w[1] = b; r.w[2] = c; r.w[3] = d; return r; }

const Fp2& twist_b() {
  static const Fp2 b = [] {
    Fp2 r;
    r.x = limbs(0x75046774386b8d71, 0x5bd0854a46d36cf8, 0x664327a1d41c8414, 0x96c9abb932eeb2f);
    r.y = limbs(0xb94f760fb4c5ee14, 0xdae9f8f24c3b6eb4, 0x77a675d2e52f4fe4, 0x736f31b09116c66b);
    // Self-check: twistB = 3 / xi with xi = i + 3.
    Fp2 xi; xi.x = Fp().one; xi.y = mont_small(3);
    Fp2 three; three.y = mont_small(3);
    Fp2 chk = three.mul(xi.inv());
    if (!(chk == r)) fail("bn256: twistB constant mismatch");
    return r;
  }();
  return b;
}

// ------------------------------------------------------------------ G2
G2 G2::infinity() { G2 p; p.y = Fp2::one(); return p; }
G2 G2::generator() {
  G2 g;
  g.x.x = limbs(0x402c4ab7139e1404, 0xce1c368a183d85a4, 0xd67cf9a6cb8d3983, 0x3cf246bbc2a9fbe8);
  g.x.y = limbs(0x88f9f11da7cdc184, 0x18293f95d69509d3, 0xb5ce0c55a735d5a1, 0x15134189bfd45a0);
  g.y.x = limbs(0xbfac7d731e9e87a2, 0xa50bb8007962e441, 0xafe910a4e8270556, 0x5075c5429d69159a);
  g.y.y = limbs(0xc2e07c1463ea9e56, 0xee4442052072ebd2, 0x561a519486036937, 0x5bd9394cc0d2cce);
  g.z = Fp2::one();
  return g;
}
G2 G2::dbl() const {
  if (is_inf()) return *this;
  Fp2 A = x.sqr(), B = y.sqr(), C = B.sqr();
  Fp2 t = x.add(B).sqr().sub(A).sub(C);
  Fp2 D = t.add(t);
  Fp2 E = A.add(A).add(A);
  Fp2 Fv = E.sqr();
  G2 r;
  r.x = Fv.sub(D).sub(D);
  Fp2 c8 = C.add(C); c8 = c8.add(c8); c8 = c8.add(c8);
  r.y = E.mul(D.sub(r.x)).sub(c8);
  Fp2 yz = y.mul(z);
  r.z = yz.add(yz);
  return r;
}
G2 G2::add(const G2& o) const {
  if (is_inf()) return o;
  if (o.is_inf()) return *this;
  Fp2 z1z1 = z.sqr(), z2z2 = o.z.sqr();
  Fp2 u1 = x.mul(z2z2), u2 = o.x.mul(z1z1);
  Fp2 s1 = y.mul(o.z).mul(z2z2), s2 = o.y.mul(z).mul(z1z1);
  Fp2 h = u2.sub(u1), r = s2.sub(s1);
  if (h.is_zero()) {
    if (r.is_zero()) return dbl();
    return infinity();
  }
  Fp2 i = h.add(h).sqr();
  Fp2 j = h.mul(i);
  r = r.add(r);
  Fp2 v = u1.mul(i);
  G2 out;
  out.x = r.sqr().sub(j).sub(v).sub(v);
  Fp2 s1j = s1.mul(j);
  out.y = r.mul(v.sub(out.x)).sub(s1j.add(s1j));
  out.z = z.add(o.z).sqr().sub(z1z1).sub(z2z2).mul(h);
  return out;
}
G2 G2::neg() const { G2 r = *this; r.y = y.neg(); return r; }
G2 G2::mul(const U256& k) const {
  G2 acc = infinity();
  for (int i = k.bitlen() - 1; i >= 0; --i) {
    acc = acc.dbl();
    if (k.bit(i)) acc = acc.add(*this);
  }
  return acc;
}
void G2::to_affine(Fp2& ax, Fp2& ay) const {
  if (is_inf()) { ax = Fp2(); ay = Fp2(); return; }
  Fp2 zi = z.inv(), zi2 = zi.sqr(), zi3 = zi2.mul(zi);
  ax = x.mul(zi2);
  ay = y.mul(zi3);
}
Bytes G2::marshal() const {
  if (is_inf()) return Bytes(1, 0);
  Fp2 ax, ay;
  to_affine(ax, ay);
  Bytes out(129, 0);
  out[0] = 1;
  Fp().from_mont(ax.x).to_be(out.data() + 1);
  Fp().from_mont(ax.y).to_be(out.data() + 33);
  Fp().from_mont(ay.x).to_be(out.data() + 65);
  Fp().from_mont(ay.y).to_be(out.data() + 97);
  return out;
}
bool G2::on_curve() const {
  if (is_inf()) return true;
  Fp2 ax, ay;
  to_affine(ax, ay);
  return ay.sqr() == ax.sqr().mul(ax).add(twist_b());
}
G2 G2::unmarshal(const Bytes& b) {
  if (!b.empty() && b[0] == 0) return infinity();
  if (b.empty() || b[0] != 1) fail("bn256.G2: malformed point");
  if (b.size() < 129) fail("bn256.G2: not enough data");
  G2 p;
  p.x.x = Fp().to_mont(U256::from_be(b.data() + 1));
  p.x.y = Fp().to_mont(U256::from_be(b.data() + 33));
  p.y.x = Fp().to_mont(U256::from_be(b.data() + 65));
  p.y.y = Fp().to_mont(U256::from_be(b.data() + 97));
  p.z = Fp2::one();
  if (!p.on_curve()) fail("bn256.G2: malformed point");
  return p;
}
bool G2::equals(const G2& o) const { return marshal() == o.marshal(); }

// ------------------------------------------------------------------ Schnorr
Scalar pick_scalar_from_xof(Blake2Xb& xof) {
  for (;;) {
    u8 buf[32];
    xof.read(buf, 32);
    U256 v = U256::from_be(buf);
    if (!v.is_zero() && cmp(v, ORDER()) < 0) { Scalar s; s.v = v; return s; }
  }
}

Scalar hash_schnorr(const Bytes& message, const G1& T) {
  Blake2Xb xof(T.marshal());
  xof.write(message);
  return pick_scalar_from_xof(xof);
}

std::pair<Scalar, G1> schnorr_nonce(const Bytes& nonce_entropy) {
  Blake2Xb nx(nonce_entropy);
  Scalar v = pick_scalar_from_xof(nx);
  return {v, gen_table().mul(v.v)};
}

Bytes schnorr_finish(const Bytes& message, const Scalar& sk, const Scalar& v, const Bytes& t_marshal) {
  Blake2Xb xof(t_marshal);
  xof.write(message);
  Scalar c = pick_scalar_from_xof(xof);
  Scalar r = v.sub(sk.mul(c));
  Bytes out = c.to_be();
  Bytes rb = r.to_be();
  out.insert(out.end(), rb.begin(), rb.end());
  return out;
}

Bytes schnorr_sign(const Bytes& message, const Scalar& sk, const Bytes& nonce_entropy) {
  Blake2Xb nx(nonce_entropy);
  Scalar v = pick_scalar_from_xof(nx);
  G1 T = gen_table().mul(v.v);
  Scalar c = hash_schnorr(message, T);
  Scalar r = v.sub(sk.mul(c));
  Bytes out = c.to_be();
  Bytes rb = r.to_be();
  out.insert(out.end(), rb.begin(), rb.end());
  return out;
}

bool schnorr_verify(const Bytes& message, const G1& pk, const Bytes& sig) {
  if (sig.size() != 64) return false;
  U256 c = U256::from_be(sig.data()), r = U256::from_be(sig.data() + 32);
  if (cmp(c, ORDER()) >= 0 || cmp(r, ORDER()) >= 0) return false;
  G1 T = gen_table().mul(r).add(pk.mul(c));
  Scalar c2 = hash_schnorr(message, T);
  return c2.v == c;
}

}  // namespace bsc
