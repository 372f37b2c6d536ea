#include "vrf.hpp"

#include "hash.hpp"

#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>

namespace bsc {
namespace {

// ---------------------------------------------------------------- GF(2^255-19), radix 2^51
struct Fe { u64 v[5]; };
constexpr u64 MASK51 = (u64(1) << 51) - 1;

Fe fe_zero() { return Fe{{0, 0, 0, 0, 0}}; }
Fe fe_one() { return Fe{{1, 0, 0, 0, 0}}; }

Fe fe_carry(Fe a) {
  for (int k = 0; k < 2; ++k) {
    u64 c;
    c = a.v[0] >> 51; a.v[0] &= MASK51; a.v[1] += c;
    c = a.v[1] >> 51; a.v[1] &= MASK51; a.v[2] += c;
    c = a.v[2] >> 51; a.v[2] &= MASK51; a.v[3] += c;
    c = a.v[3] >> 51; a.v[3] &= MASK51; a.v[4] += c;
    c = a.v[4] >> 51; a.v[4] &= MASK51; a.v[0] += c * 19;
  }
  return a;
}
// one carry pass: inputs with limbs < 2^52 give limbs < 2^51 + 2^2 (limb 0 < 2^51 + 19*2^2)
inline Fe fe_carry1(Fe a) {
  u64 c;
  c = a.v[0] >> 51; a.v[0] &= MASK51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= MASK51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= MASK51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= MASK51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= MASK51; a.v[0] += c * 19;
  return a;
}
Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
  return fe_carry1(r);
}
Fe fe_sub(const Fe& a, const Fe& b) {
  // add 4p to keep limbs positive
  static const u64 p4[5] = {0x1FFFFFFFFFFFB4ULL * 1, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
                            0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
  Fe r;
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + p4[i] - b.v[i];
  return fe_carry1(r);
}
Fe fe_neg(const Fe& a) { return fe_sub(fe_zero(), a); }
Fe fe_mul(const Fe& a, const Fe& b) {
  u128 t[5];
  const u64 *x = a.v, *y = b.v;
  u64 y19[5];
  for (int i = 0; i < 5; ++i) y19[i] = y[i] * 19;
  t[0] = u128(x[0]) * y[0] + u128(x[1]) * y19[4] + u128(x[2]) * y19[3] + u128(x[3]) * y19[2] + u128(x[4]) * y19[1];
  t[1] = u128(x[0]) * y[1] + u128(x[1]) * y[0] + u128(x[2]) * y19[4] + u128(x[3]) * y19[3] + u128(x[4]) * y19[2];
  t[2] = u128(x[0]) * y[2] + u128(x[1]) * y[1] + u128(x[2]) * y[0] + u128(x[3]) * y19[4] + u128(x[4]) * y19[3];
  t[3] = u128(x[0]) * y[3] + u128(x[1]) * y[2] + u128(x[2]) * y[1] + u128(x[3]) * y[0] + u128(x[4]) * y19[4];
  t[4] = u128(x[0]) * y[4] + u128(x[1]) * y[3] + u128(x[2]) * y[2] + u128(x[3]) * y[1] + u128(x[4]) * y[0];
  Fe r;
  u128 c = 0;
  for (int i = 0; i < 5; ++i) {
    t[i] += c;
    r.v[i] = u64(t[i]) & MASK51;
    c = t[i] >> 51;
  }
  // every limb is < 2^51 here; the wrap-around term only needs one more carry (limb 0 -> limb 1)
  // to give limbs < 2^51 + 2^13, which is all fe_add / fe_sub / fe_mul assume of their inputs
  r.v[0] += u64(c) * 19;
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= MASK51;
  return r;
}
Fe fe_sq(const Fe& a) {
  const u64* x = a.v;
  const u64 d0 = 2 * x[0], d1 = 2 * x[1], d2 = 2 * x[2], d3_19 = 2 * 19 * x[3], x4_19 = 19 * x[4], x3_19 = 19 * x[3];
  u128 t[5];
  t[0] = u128(x[0]) * x[0] + u128(d1) * x4_19 + u128(d2) * x3_19;
  t[1] = u128(d0) * x[1] + u128(d2) * x4_19 + u128(x[3]) * x3_19;
  t[2] = u128(d0) * x[2] + u128(x[1]) * x[1] + u128(d3_19) * x[4];
  t[3] = u128(d0) * x[3] + u128(d1) * x[2] + u128(x[4]) * x4_19;
  t[4] = u128(d0) * x[4] + u128(d1) * x[3] + u128(x[2]) * x[2];
  Fe r;
  u128 c = 0;
  for (int i = 0; i < 5; ++i) {
    t[i] += c;
    r.v[i] = u64(t[i]) & MASK51;
    c = t[i] >> 51;
  }
  // every limb is < 2^51 here; the wrap-around term only needs one more carry (limb 0 -> limb 1)
  // to give limbs < 2^51 + 2^13, which is all fe_add / fe_sub / fe_mul assume of their inputs
  r.v[0] += u64(c) * 19;
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= MASK51;
  return r;
}
Fe fe_sqn(Fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// canonical 32-byte little-endian encoding
void fe_tobytes(u8 out[32], Fe a) {
  a = fe_carry(a);
  // subtract p if a >= p: compute a + 19 and check bit 255
  u64 q = (a.v[0] + 19) >> 51;
  q = (a.v[1] + q) >> 51;
  q = (a.v[2] + q) >> 51;
  q = (a.v[3] + q) >> 51;
  q = (a.v[4] + q) >> 51;
  a.v[0] += 19 * q;
  u64 c;
  c = a.v[0] >> 51; a.v[0] &= MASK51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= MASK51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= MASK51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= MASK51; a.v[4] += c;
  a.v[4] &= MASK51;
  u8 buf[40] = {0};
  // pack 255 bits
  u128 acc = 0;
  int bits = 0, o = 0;
  for (int i = 0; i < 5; ++i) {
    acc |= u128(a.v[i]) << bits;
    bits += 51;
    while (bits >= 8) { buf[o++] = u8(acc); acc >>= 8; bits -= 8; }
  }
  if (bits > 0) buf[o++] = u8(acc);
  memcpy(out, buf, 32);
}
Fe fe_frombytes(const u8 in[32]) {
  u8 b[32];
  memcpy(b, in, 32);
  b[31] &= 0x7f;
  Fe r;
  u64 w[4];
  for (int i = 0; i < 4; ++i) w[i] = load_le64(b + 8 * i);
  r.v[0] = w[0] & MASK51;
  r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  r.v[4] = (w[3] >> 12) & MASK51;
  return r;
}
bool fe_eq(const Fe& a, const Fe& b) {
  u8 x[32], y[32];
  fe_tobytes(x, a); fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}
bool fe_iszero(const Fe& a) { return fe_eq(a, fe_zero()); }
bool fe_isneg(const Fe& a) { u8 x[32]; fe_tobytes(x, a); return x[0] & 1; }
Fe fe_pow(const Fe& a, const u8 e_le[32]) {
  Fe r = fe_one();
  for (int i = 255; i >= 0; --i) {
    r = fe_sq(r);
    if ((e_le[i >> 3] >> (i & 7)) & 1) r = fe_mul(r, a);
  }
  return r;
}
// z^(p-2), addition chain: 254 squarings + 11 multiplications
Fe fe_invert(const Fe& z) {
  Fe t0 = fe_sq(z);
  Fe t1 = fe_sqn(t0, 2);
  t1 = fe_mul(z, t1);
  t0 = fe_mul(t0, t1);
  Fe t2 = fe_sq(t0);
  t1 = fe_mul(t1, t2);
  t2 = fe_sqn(t1, 5);
  t1 = fe_mul(t2, t1);
  t2 = fe_sqn(t1, 10);
  t2 = fe_mul(t2, t1);
  Fe t3 = fe_sqn(t2, 20);
  t2 = fe_mul(t3, t2);
  t2 = fe_sqn(t2, 10);
  t1 = fe_mul(t2, t1);
  t2 = fe_sqn(t1, 50);
  t2 = fe_mul(t2, t1);
  t3 = fe_sqn(t2, 100);
  t2 = fe_mul(t3, t2);
  t2 = fe_sqn(t2, 50);
  t1 = fe_mul(t2, t1);
  t1 = fe_sqn(t1, 5);
  return fe_mul(t1, t0);
}
// z^((p-5)/8) = z^(2^252 - 3)
Fe fe_pow22523(const Fe& z) {
  Fe t0 = fe_sq(z);
  Fe t1 = fe_sqn(t0, 2);
  t1 = fe_mul(z, t1);
  t0 = fe_mul(t0, t1);
  t0 = fe_sq(t0);
  t0 = fe_mul(t1, t0);
  t1 = fe_sqn(t0, 5);
  t0 = fe_mul(t1, t0);
  t1 = fe_sqn(t0, 10);
  t1 = fe_mul(t1, t0);
  Fe t2 = fe_sqn(t1, 20);
  t1 = fe_mul(t2, t1);
  t1 = fe_sqn(t1, 10);
  t0 = fe_mul(t1, t0);
  t1 = fe_sqn(t0, 50);
  t1 = fe_mul(t1, t0);
  t2 = fe_sqn(t1, 100);
  t1 = fe_mul(t2, t1);
  t1 = fe_sqn(t1, 50);
  t0 = fe_mul(t1, t0);
  t0 = fe_sqn(t0, 2);
  return fe_mul(t0, z);
}
Fe fe_from_dec(const char* s) {
  u64 w[4] = {0, 0, 0, 0};
  for (const char* c = s; *c; ++c) {
    u128 carry = u64(*c - '0');
    for (int i = 0; i < 4; ++i) {
      u128 v = u128(w[i]) * 10 + carry;
      w[i] = u64(v);
      carry = v >> 64;
    }
  }
  u8 b[32];
  for (int i = 0; i < 4; ++i) store_le64(b + 8 * i, w[i]);
  return fe_frombytes(b);
}

const Fe& D() { static const Fe d = fe_from_dec("37095705934669439343138083508754565189542113879843219016388785533085940283555"); return d; }
const Fe& D2() { static const Fe d2 = fe_add(D(), D()); return d2; }
const Fe& SQRTM1() { static const Fe s = fe_from_dec("19681161376707505956807079304988542015446066515923890162744021073123829784752"); return s; }

// ---------------------------------------------------------------- points (extended coordinates)
struct Ge { Fe X, Y, Z, T; };
Ge ge_identity() { return Ge{fe_zero(), fe_one(), fe_one(), fe_zero()}; }
Ge ge_add(const Ge& p, const Ge& q) {
  Fe A = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  Fe B = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  Fe C = fe_mul(fe_mul(p.T, D2()), q.T);
  Fe Dd = fe_mul(fe_add(p.Z, p.Z), q.Z);
  Fe E = fe_sub(B, A), F = fe_sub(Dd, C), G = fe_add(Dd, C), H = fe_add(B, A);
  return Ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
Ge ge_neg(const Ge& p) { return Ge{fe_neg(p.X), p.Y, p.Z, fe_neg(p.T)}; }
// dbl-2008-hwcd for a = -1: 4M + 4S (vs 9M for the unified addition)
Ge ge_dbl(const Ge& p) {
  Fe A = fe_sq(p.X), Bv = fe_sq(p.Y);
  Fe zz = fe_sq(p.Z);
  Fe C = fe_add(zz, zz);
  Fe Dd = fe_neg(A);
  Fe E = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), A), Bv);
  Fe G = fe_add(Dd, Bv), F = fe_sub(G, C), H = fe_sub(Dd, Bv);
  return Ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
// doubling whose result feeds another doubling: T is never read, skip its multiplication
Ge ge_dbl_noT(const Ge& p) {
  Fe A = fe_sq(p.X), Bv = fe_sq(p.Y);
  Fe zz = fe_sq(p.Z);
  Fe C = fe_add(zz, zz);
  Fe Dd = fe_neg(A);
  Fe E = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), A), Bv);
  Fe G = fe_add(Dd, Bv), F = fe_sub(G, C), H = fe_sub(Dd, Bv);
  return Ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_zero()};
}
// "cached" form of a table entry: (Y+X, Y-X, 2Z, 2dT) -> an addition costs 8M instead of 10M
struct GeCached { Fe YpX, YmX, Z2, T2d; };
GeCached ge_cache(const Ge& p) {
  return GeCached{fe_add(p.Y, p.X), fe_sub(p.Y, p.X), fe_add(p.Z, p.Z), fe_mul(p.T, D2())};
}
GeCached ge_cached_neg(const GeCached& c) { return GeCached{c.YmX, c.YpX, c.Z2, fe_neg(c.T2d)}; }
Ge ge_add_cached(const Ge& p, const GeCached& q) {
  Fe A = fe_mul(fe_sub(p.Y, p.X), q.YmX);
  Fe B = fe_mul(fe_add(p.Y, p.X), q.YpX);
  Fe C = fe_mul(p.T, q.T2d);
  Fe Dd = fe_mul(p.Z, q.Z2);
  Fe E = fe_sub(B, A), F = fe_sub(Dd, C), G = fe_add(Dd, C), H = fe_add(B, A);
  return Ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
// scalar (32-byte LE, < 2^255) -> 64 signed radix-16 digits in [-8, 8)
void signed_digits(int8_t e[64], const u8 k[32]) {
  for (int i = 0; i < 32; ++i) {
    e[2 * i] = int8_t(k[i] & 15);
    e[2 * i + 1] = int8_t(k[i] >> 4);
  }
  int carry = 0;
  for (int i = 0; i < 63; ++i) {
    e[i] = int8_t(e[i] + carry);
    carry = (e[i] + 8) >> 4;
    e[i] = int8_t(e[i] - (carry << 4));
  }
  e[63] = int8_t(e[63] + carry);
}
// variable-base: table of 1P..8P in cached form, 4 doublings (3 without T) + 1 cached add per digit
Ge ge_mul(const Ge& p, const u8 k[32]) {
  GeCached tbl[8];  // tbl[i] = (i+1) P
  tbl[0] = ge_cache(p);
  Ge acc = ge_dbl(p);
  tbl[1] = ge_cache(acc);
  for (int i = 2; i < 8; ++i) {
    acc = ge_add_cached(acc, tbl[0]);
    tbl[i] = ge_cache(acc);
  }
  int8_t e[64];
  signed_digits(e, k);
  Ge r = ge_identity();
  for (int w = 63; w >= 0; --w) {
    if (w != 63) { r = ge_dbl_noT(r); r = ge_dbl_noT(r); r = ge_dbl_noT(r); r = ge_dbl(r); }
    const int d = e[w];
    if (d > 0) r = ge_add_cached(r, tbl[d - 1]);
    else if (d < 0) r = ge_add_cached(r, ge_cached_neg(tbl[-d - 1]));
  }
  return r;
}
Ge ge_base() {
  static const Ge b = [] {
    Fe x = fe_from_dec("15112221349535400772501151409588531511454012693041857206046113283949847762202");
    Fe y = fe_from_dec("46316835694926478169428394003475163141307993866256225615783033603165251855960");
    return Ge{x, y, fe_one(), fe_mul(x, y)};
  }();
  return b;
}
// fixed-base table for B: 64 signed radix-16 windows x 8 cached multiples (d * 16^w * B, d = 1..8)
struct BaseTable {
  std::vector<GeCached> t;
  BaseTable() {
    t.resize(64 * 8);
    Ge base = ge_base();
    for (int w = 0; w < 64; ++w) {
      Ge acc = base;
      for (int d = 0; d < 8; ++d) {
        t[w * 8 + d] = ge_cache(acc);
        acc = ge_add_cached(acc, t[w * 8]);
      }
      for (int i = 0; i < 4; ++i) base = ge_dbl(base);
    }
  }
};
const BaseTable& base_table() {
  static const BaseTable bt;
  return bt;
}
// no doublings at all: one cached addition per non-zero digit
Ge ge_mul_base(const u8 k[32]) {
  const BaseTable& bt = base_table();
  int8_t e[64];
  signed_digits(e, k);
  Ge r = ge_identity();
  for (int w = 0; w < 64; ++w) {
    const int d = e[w];
    if (d > 0) r = ge_add_cached(r, bt.t[w * 8 + d - 1]);
    else if (d < 0) r = ge_add_cached(r, ge_cached_neg(bt.t[w * 8 - d - 1]));
  }
  return r;
}
Bytes ge_tobytes(const Ge& p) {
  Fe zi = fe_invert(p.Z);
  Fe x = fe_mul(p.X, zi), y = fe_mul(p.Y, zi);
  Bytes out(32);
  fe_tobytes(out.data(), y);
  if (fe_isneg(x)) out[31] |= 0x80;
  return out;
}
// encode several points with ONE field inversion (Montgomery's trick)
void ge_tobytes_batch(const Ge* const* pts, int n, Bytes* out) {
  Fe pre[8];
  Fe acc = fe_one();
  for (int i = 0; i < n; ++i) { pre[i] = acc; acc = fe_mul(acc, pts[i]->Z); }
  Fe inv = fe_invert(acc);
  for (int i = n - 1; i >= 0; --i) {
    Fe zi = fe_mul(inv, pre[i]);
    inv = fe_mul(inv, pts[i]->Z);
    Fe x = fe_mul(pts[i]->X, zi), y = fe_mul(pts[i]->Y, zi);
    out[i].assign(32, 0);
    fe_tobytes(out[i].data(), y);
    if (fe_isneg(x)) out[i][31] |= 0x80;
  }
}
bool ge_frombytes(Ge& out, const u8 in[32]) {
  // RFC 8032 5.1.3: reject non-canonical y
  u8 b[32];
  memcpy(b, in, 32);
  int sign = b[31] >> 7;
  b[31] &= 0x7f;
  Fe y = fe_frombytes(b);
  u8 chk[32];
  fe_tobytes(chk, y);
  if (memcmp(chk, b, 32) != 0) return false;
  Fe y2 = fe_sq(y);
  Fe u = fe_sub(y2, fe_one());
  Fe v = fe_add(fe_mul(D(), y2), fe_one());
  Fe v3 = fe_mul(fe_sq(v), v);
  Fe v7 = fe_mul(fe_sq(v3), v);
  Fe x = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  Fe vx2 = fe_mul(v, fe_sq(x));
  if (!fe_eq(vx2, u)) {
    if (fe_eq(vx2, fe_neg(u))) x = fe_mul(x, SQRTM1());
    else return false;
  }
  if (fe_iszero(x) && sign) return false;
  if (int(fe_isneg(x)) != sign) x = fe_neg(x);
  out = Ge{x, y, fe_one(), fe_mul(x, y)};
  return true;
}
bool ge_is_identity(const Ge& p) { return fe_iszero(p.X) && fe_eq(p.Y, p.Z); }

// ---------------------------------------------------------------- scalars mod L
// L = 2^252 + 27742317777372353535851937790883648493 as 4 LE limbs
const u64 Lw[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0000000000000000ULL, 0x1000000000000000ULL};
bool ge_L(const u64 r[4]) {
  for (int i = 3; i >= 0; --i) {
    if (r[i] > Lw[i]) return true;
    if (r[i] < Lw[i]) return false;
  }
  return true;
}
void subL(u64 r[4]) {
  u64 br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = u128(r[i]) - Lw[i] - br;
    r[i] = u64(d);
    br = u64(d >> 64) & 1;
  }
}
// reduce an arbitrary little-endian byte string mod L (bitwise long division)
void sc_reduce(u8 out[32], const u8* in, size_t n) {
  u64 r[4] = {0, 0, 0, 0};
  for (size_t bi = n * 8; bi-- > 0;) {
    u64 bit = (in[bi >> 3] >> (bi & 7)) & 1;
    // r = 2r + bit
    u64 c = bit;
    for (int i = 0; i < 4; ++i) {
      u64 nc = r[i] >> 63;
      r[i] = (r[i] << 1) | c;
      c = nc;
    }
    if (ge_L(r)) subL(r);
  }
  for (int i = 0; i < 4; ++i) store_le64(out + 8 * i, r[i]);
}
// out = (a + b*c) mod L ; all little-endian, a,b 32B, c given as cLen bytes
void sc_muladd(u8 out[32], const u8 a[32], const u8* b, size_t blen, const u8 c[32]) {
  // schoolbook product into 96 bytes, then add a, then reduce
  u64 prod[12] = {0};
  u64 bw[4] = {0, 0, 0, 0}, cw[4];
  u8 bb[32] = {0};
  memcpy(bb, b, blen);
  for (int i = 0; i < 4; ++i) { bw[i] = load_le64(bb + 8 * i); cw[i] = load_le64(c + 8 * i); }
  for (int i = 0; i < 4; ++i) {
    u128 carry = 0;
    for (int j = 0; j < 4; ++j) {
      u128 v = u128(bw[i]) * cw[j] + prod[i + j] + carry;
      prod[i + j] = u64(v);
      carry = v >> 64;
    }
    prod[i + 4] += u64(carry);
  }
  u128 carry = 0;
  for (int i = 0; i < 12; ++i) {
    u128 v = u128(prod[i]) + (i < 4 ? load_le64(a + 8 * i) : 0) + carry;
    prod[i] = u64(v);
    carry = v >> 64;
  }
  u8 buf[96];
  for (int i = 0; i < 12; ++i) store_le64(buf + 8 * i, prod[i]);
  sc_reduce(out, buf, 96);
}

void clamp_secret(const Bytes& seed, u8 x[32], u8 prefix[32]) {
  Bytes h = Sha512::digest(seed);
  memcpy(x, h.data(), 32);
  x[0] &= 248;
  x[31] &= 127;
  x[31] |= 64;
  memcpy(prefix, h.data() + 32, 32);
}

const u8 SUITE = 0x03;

Ge encode_to_curve(const Bytes& pk, const Bytes& alpha) {
  for (int ctr = 0; ctr < 256; ++ctr) {
    Sha512 h;
    u8 pre[2] = {SUITE, 0x01};
    h.update(pre, 2);
    h.update(pk);
    h.update(alpha);
    u8 tail[2] = {u8(ctr), 0x00};
    h.update(tail, 2);
    u8 dig[64];
    h.final(dig);
    Ge H;
    if (ge_frombytes(H, dig)) {
      H = ge_dbl(ge_dbl(ge_dbl(H)));  // cofactor 8
      return H;
    }
  }
  fail("ecvrf: encode_to_curve failed");
}

Bytes challenge_str(const Bytes& Y, const Bytes& H, const Bytes& G, const Bytes& U, const Bytes& V) {
  Sha512 h;
  u8 pre[2] = {SUITE, 0x02};
  h.update(pre, 2);
  for (const Bytes* p : {&Y, &H, &G, &U, &V}) h.update(*p);
  u8 z = 0;
  h.update(&z, 1);
  u8 dig[64];
  h.final(dig);
  return Bytes(dig, dig + 16);
}

}  // namespace

// the scalar field code for vrf_ifma.cpp (per-lane encodings and constants of the batched path)
namespace vrf_detail {
void fe51_tobytes(u8 out[32], const u64 v[5]) {
  Fe a;
  memcpy(a.v, v, sizeof(a.v));
  fe_tobytes(out, a);
}
void fe51_frombytes(u64 v[5], const u8 in[32]) {
  const Fe a = fe_frombytes(in);
  memcpy(v, a.v, sizeof(a.v));
}
void fe51_consts(u64 d[5], u64 sqrtm1[5]) {
  memcpy(d, D().v, 5 * sizeof(u64));
  memcpy(sqrtm1, SQRTM1().v, 5 * sizeof(u64));
}
// the fixed-base table of B: entry (w, d) = (d + 1) * 16^w * B in cached form, 4 elements of 5 limbs
const u64* base_table_limbs() {
  static_assert(sizeof(GeCached) == 20 * sizeof(u64), "cached point layout");
  return reinterpret_cast<const u64*>(base_table().t.data());
}
void sc_reduce64(u8 out[32], const u8 in[64]) { sc_reduce(out, in, 64); }
void sc_muladd16(u8 out[32], const u8 k[32], const u8 c16[16], const u8 x[32]) { sc_muladd(out, k, c16, 16, x); }
Bytes challenge(const Bytes& Y, const Bytes& H, const Bytes& G, const Bytes& U, const Bytes& V) {
  return challenge_str(Y, H, G, U, V);
}
}  // namespace vrf_detail

Bytes ed25519_public_from_seed(const Bytes& seed32) {
  if (seed32.size() != 32) fail("ed25519: seed must be 32 bytes");
  u8 x[32], prefix[32];
  clamp_secret(seed32, x, prefix);
  return ge_tobytes(ge_mul_base(x));
}

VrfKey VrfKey::from_seed(const Bytes& seed32) {
  if (seed32.size() != 32) fail("ed25519: seed must be 32 bytes");
  VrfKey k;
  k.seed = seed32;
  clamp_secret(seed32, k.x, k.prefix);
  k.pk = ge_tobytes(ge_mul_base(k.x));
  return k;
}

const VrfKey& VrfKey::cached(const Bytes& seed32) {
  static std::mutex mu;
  static std::unordered_map<std::string, std::unique_ptr<VrfKey>> cache;
  std::string key(seed32.begin(), seed32.end());
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return *it->second;
  }
  auto k = std::make_unique<VrfKey>(from_seed(seed32));
  std::lock_guard<std::mutex> lk(mu);
  auto& slot = cache[key];
  if (!slot) slot = std::move(k);
  return *slot;
}

Bytes vrf_proof_to_hash(const Bytes& pi) {
  if (pi.size() != 80) fail("ecvrf: bad proof length");
  Ge G;
  if (!ge_frombytes(G, pi.data())) fail("ecvrf: bad gamma");
  G = ge_dbl(ge_dbl(ge_dbl(G)));
  Sha512 h;
  u8 pre[2] = {SUITE, 0x03};
  h.update(pre, 2);
  h.update(ge_tobytes(G));
  u8 z = 0;
  h.update(&z, 1);
  Bytes out(64);
  h.final(out.data());
  return out;
}

[[maybe_unused]] static Bytes gamma_to_hash(const Ge& Gamma) {
  Ge G8 = ge_dbl(ge_dbl(ge_dbl(Gamma)));
  Sha512 h;
  u8 pre[2] = {SUITE, 0x03};
  h.update(pre, 2);
  h.update(ge_tobytes(G8));
  u8 z = 0;
  h.update(&z, 1);
  Bytes out(64);
  h.final(out.data());
  return out;
}

namespace {
struct Staged {  // one proof between the output phase and the proof phase
  Ge H, Gamma;
  Bytes hstr;
};
}  // namespace

Bytes vrf_output(const VrfKey& key, const Bytes& alpha, VrfStage* stage) {
  auto st = std::make_shared<Staged>();
  st->H = encode_to_curve(key.pk, alpha);
  st->hstr = ge_tobytes(st->H);
  st->Gamma = ge_mul(st->H, key.x);
  Ge G8 = ge_dbl(ge_dbl(ge_dbl(st->Gamma)));
  Sha512 bh;
  u8 pre[2] = {SUITE, 0x03};
  bh.update(pre, 2);
  bh.update(ge_tobytes(G8));
  u8 z = 0;
  bh.update(&z, 1);
  Bytes beta(64);
  bh.final(beta.data());
  stage->st = st;
  return beta;
}

Bytes vrf_beta(const VrfKey& key, const Bytes& alpha) {
  const Ge H = encode_to_curve(key.pk, alpha);
  const Ge G8 = ge_dbl(ge_dbl(ge_dbl(ge_mul(H, key.x))));
  Sha512 bh;
  u8 pre[2] = {SUITE, 0x03};
  bh.update(pre, 2);
  bh.update(ge_tobytes(G8));
  u8 z = 0;
  bh.update(&z, 1);
  Bytes beta(64);
  bh.final(beta.data());
  return beta;
}

Bytes vrf_base_table_bytes() {
  const BaseTable& bt = base_table();
  Bytes out(bt.t.size() * 128);
  for (size_t i = 0; i < bt.t.size(); ++i) {
    const GeCached& c = bt.t[i];
    const Fe* f[4] = {&c.YpX, &c.YmX, &c.Z2, &c.T2d};
    for (int j = 0; j < 4; ++j) fe_tobytes(out.data() + 128 * i + 32 * j, *f[j]);
  }
  return out;
}

Bytes vrf_finish(const VrfKey& key, const VrfStage& stage) {
  const Staged& st = *static_cast<const Staged*>(stage.st.get());
  const u8* x = key.x;
  Sha512 kh;
  kh.update(key.prefix, 32);
  kh.update(st.hstr);
  u8 kd[64];
  kh.final(kd);
  u8 k[32];
  sc_reduce(k, kd, 64);
  // Gamma, k*B and k*H share one inversion
  Ge U = ge_mul_base(k), V = ge_mul(st.H, k);
  const Ge* pts[3] = {&st.Gamma, &U, &V};
  Bytes enc[3];
  ge_tobytes_batch(pts, 3, enc);
  Bytes c = challenge_str(key.pk, st.hstr, enc[0], enc[1], enc[2]);
  u8 s[32];
  sc_muladd(s, k, c.data(), 16, x);
  Bytes pi = enc[0];
  pi.insert(pi.end(), c.begin(), c.end());
  pi.insert(pi.end(), s, s + 32);
  return pi;
}

std::pair<Bytes, Bytes> vrf_prove(const VrfKey& key, const Bytes& alpha) {
  VrfStage stage;
  Bytes beta = vrf_output(key, alpha, &stage);
  return {beta, vrf_finish(key, stage)};
}

bool vrf_verify(const Bytes& pk, const Bytes& alpha, const Bytes& pi, Bytes* beta) {
  if (pk.size() != 32 || pi.size() != 80) return false;
  Ge Y, Gamma;
  if (!ge_frombytes(Y, pk.data())) return false;
  if (!ge_frombytes(Gamma, pi.data())) return false;
  u8 c[32] = {0}, s[32];
  memcpy(c, pi.data() + 32, 16);
  memcpy(s, pi.data() + 48, 32);
  u64 sw[4];
  for (int i = 0; i < 4; ++i) sw[i] = load_le64(s + 8 * i);
  if (ge_L(sw)) return false;
  Ge H = encode_to_curve(pk, alpha);
  Ge U = ge_add(ge_mul_base(s), ge_neg(ge_mul(Y, c)));
  Ge V = ge_add(ge_mul(H, s), ge_neg(ge_mul(Gamma, c)));
  Bytes c2 = challenge_str(pk, ge_tobytes(H), Bytes(pi.begin(), pi.begin() + 32), ge_tobytes(U), ge_tobytes(V));
  if (memcmp(c2.data(), c, 16) != 0) return false;
  if (beta) *beta = vrf_proof_to_hash(pi);
  return true;
}

}  // namespace bsc
