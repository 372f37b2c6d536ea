// Eight VRF outputs at once: Edwards25519 arithmetic on AVX-512 IFMA lanes (vrf.hpp vrf_beta_batch).
//
// The round's noiser lottery waits for every peer's VRF output of the new block (~100 variable-base scalar
// multiplications x*H, one per peer, H = encode_to_curve(pk, block hash)): on the host, because one output is a
// few thousand dependent field multiplications -- a latency chain the GPU runs far slower than a CPU core.  This
// file runs eight of them side by side in the 8 x 64-bit lanes of AVX-512, each field multiplication a 5 x 5
// limb product on the 52-bit multiply-accumulate units (vpmadd52luq / vpmadd52huq), so a core gives ~4x the
// outputs per second of the scalar radix-2^51 code (vrf.cpp), which stays the path on CPUs without IFMA.
//
// Field elements use vrf.cpp's representation, 5 limbs of radix 2^51 (one lane per output).  madd52 reads only
// the low 52 bits of its inputs, so every multiplication input must have limbs < 2^52; the invariants below keep
// them there:
//   - f_mul / f_sq outputs: limbs 1..4 < 2^51 + 2^10, limb 0 < 2^51 + 2^15;
//   - f_add / f_sub outputs (one parallel carry pass): the same bounds;
//   - f_sub adds 4p first (limb-wise >= any operand above), so no limb goes negative.
// Products: a_i * b_j < 2^104 splits into lo (bits 0..51, weight 2^(51(i+j))) and hi (bits 52..103, weight
// 2^(51(i+j)+52) = 2 * 2^(51(i+j+1))); column k = lo_k + 2 hi_{k-1} < 15 * 2^52; columns 5..9 wrap with 19
// (2^255 = 19 mod p): r_k = c_k + 19 c_{k+5} < 2^61, then one parallel carry pass.
//
// Only the functions marked IFMA use AVX-512: they run after vrf_beta_batch_supported() (cpuid) says so.
// Every result is compared against the scalar path in tests/test_vrf_batch.py.
#include <immintrin.h>

#include <cstring>

#include "hash.hpp"
#include "vrf.hpp"

namespace bsc {
namespace vrf_detail {
void fe51_tobytes(u8 out[32], const u64 v[5]);
void fe51_frombytes(u64 v[5], const u8 in[32]);
void fe51_consts(u64 d[5], u64 sqrtm1[5]);
const u64* base_table_limbs();
void sc_reduce64(u8 out[32], const u8 in[64]);
void sc_muladd16(u8 out[32], const u8 k[32], const u8 c16[16], const u8 x[32]);
Bytes challenge(const Bytes& Y, const Bytes& H, const Bytes& G, const Bytes& U, const Bytes& V);
}  // namespace vrf_detail

namespace {

#define IFMA __attribute__((target("avx512f,avx512ifma"))) inline
using V = __m512i;
constexpr u64 M51 = (u64(1) << 51) - 1;

struct F {
  V l[5];
};
struct P {  // extended coordinates
  F X, Y, Z, T;
};
struct C {  // cached: (Y+X, Y-X, 2Z, 2dT)
  F YpX, YmX, Z2, T2d;
};

IFMA V vz() { return _mm512_setzero_si512(); }
IFMA V v1(u64 x) { return _mm512_set1_epi64((long long)x); }

IFMA F f_zero() {
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = vz();
  return r;
}
IFMA F f_one() {
  F r = f_zero();
  r.l[0] = v1(1);
  return r;
}

// one parallel carry pass over limbs < 2^63: limb k keeps its low 51 bits plus the carry of limb k-1
IFMA F f_carry(const F& a) {
  const V m = v1(M51);
  V t[5];
  for (int k = 0; k < 5; ++k) t[k] = _mm512_srli_epi64(a.l[k], 51);
  F r;
  r.l[0] = _mm512_madd52lo_epu64(_mm512_and_si512(a.l[0], m), t[4], v1(19));   // t4 * 19 < 2^52
  for (int k = 1; k < 5; ++k) r.l[k] = _mm512_add_epi64(_mm512_and_si512(a.l[k], m), t[k - 1]);
  return r;
}

IFMA F f_add(const F& a, const F& b) {
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = _mm512_add_epi64(a.l[k], b.l[k]);
  return f_carry(r);
}

IFMA F f_sub(const F& a, const F& b) {
  static constexpr u64 P4_0 = 0x1FFFFFFFFFFFB4ULL, P4_K = 0x1FFFFFFFFFFFFCULL;   // 4p
  F r;
  for (int k = 0; k < 5; ++k)
    r.l[k] = _mm512_sub_epi64(_mm512_add_epi64(a.l[k], v1(k == 0 ? P4_0 : P4_K)), b.l[k]);
  return f_carry(r);
}

IFMA F f_neg(const F& a) { return f_sub(f_zero(), a); }

IFMA V mul19(V x) {   // 19 x = 16 x + 2 x + x (x < 2^57)
  return _mm512_add_epi64(_mm512_add_epi64(_mm512_slli_epi64(x, 4), _mm512_slli_epi64(x, 1)), x);
}

// columns lo[0..8], hi[0..8] of a 5 x 5 limb product -> reduced element
IFMA F f_reduce(const V lo[9], const V hi[9]) {
  V c[10];
  c[0] = lo[0];
  for (int k = 1; k < 9; ++k) c[k] = _mm512_add_epi64(lo[k], _mm512_add_epi64(hi[k - 1], hi[k - 1]));
  c[9] = _mm512_add_epi64(hi[8], hi[8]);
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = _mm512_add_epi64(c[k], mul19(c[k + 5]));
  return f_carry(r);
}

IFMA F f_mul(const F& a, const F& b) {
  V lo[9], hi[9];
  for (int k = 0; k < 9; ++k) lo[k] = hi[k] = vz();
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) {
      lo[i + j] = _mm512_madd52lo_epu64(lo[i + j], a.l[i], b.l[j]);
      hi[i + j] = _mm512_madd52hi_epu64(hi[i + j], a.l[i], b.l[j]);
    }
  return f_reduce(lo, hi);
}

IFMA F f_sq(const F& a) {
  // the 10 cross products once, doubled: 15 products instead of 25
  V lo[9], hi[9], xlo[9], xhi[9];
  for (int k = 0; k < 9; ++k) lo[k] = hi[k] = xlo[k] = xhi[k] = vz();
  for (int i = 0; i < 5; ++i) {
    lo[2 * i] = _mm512_madd52lo_epu64(lo[2 * i], a.l[i], a.l[i]);
    hi[2 * i] = _mm512_madd52hi_epu64(hi[2 * i], a.l[i], a.l[i]);
    for (int j = i + 1; j < 5; ++j) {
      xlo[i + j] = _mm512_madd52lo_epu64(xlo[i + j], a.l[i], a.l[j]);
      xhi[i + j] = _mm512_madd52hi_epu64(xhi[i + j], a.l[i], a.l[j]);
    }
  }
  for (int k = 0; k < 9; ++k) {
    lo[k] = _mm512_add_epi64(lo[k], _mm512_add_epi64(xlo[k], xlo[k]));
    hi[k] = _mm512_add_epi64(hi[k], _mm512_add_epi64(xhi[k], xhi[k]));
  }
  return f_reduce(lo, hi);
}

IFMA F f_sqn(F a, int n) {
  for (int i = 0; i < n; ++i) a = f_sq(a);
  return a;
}

IFMA F f_blend(__mmask8 m, const F& a, const F& b) {   // lanes of m from b
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = _mm512_mask_blend_epi64(m, a.l[k], b.l[k]);
  return r;
}

// z^(p-2) and z^((p-5)/8): the scalar code's addition chains
IFMA F f_invert(const F& z) {
  F t0 = f_sq(z);
  F t1 = f_sqn(t0, 2);
  t1 = f_mul(z, t1);
  t0 = f_mul(t0, t1);
  F t2 = f_sq(t0);
  t1 = f_mul(t1, t2);
  t2 = f_sqn(t1, 5);
  t1 = f_mul(t2, t1);
  t2 = f_sqn(t1, 10);
  t2 = f_mul(t2, t1);
  F t3 = f_sqn(t2, 20);
  t2 = f_mul(t3, t2);
  t2 = f_sqn(t2, 10);
  t1 = f_mul(t2, t1);
  t2 = f_sqn(t1, 50);
  t2 = f_mul(t2, t1);
  t3 = f_sqn(t2, 100);
  t2 = f_mul(t3, t2);
  t2 = f_sqn(t2, 50);
  t1 = f_mul(t2, t1);
  t1 = f_sqn(t1, 5);
  return f_mul(t1, t0);
}

IFMA F f_pow22523(const F& z) {
  F t0 = f_sq(z);
  F t1 = f_sqn(t0, 2);
  t1 = f_mul(z, t1);
  t0 = f_mul(t0, t1);
  t0 = f_sq(t0);
  t0 = f_mul(t1, t0);
  t1 = f_sqn(t0, 5);
  t0 = f_mul(t1, t0);
  t1 = f_sqn(t0, 10);
  t1 = f_mul(t1, t0);
  F t2 = f_sqn(t1, 20);
  t1 = f_mul(t2, t1);
  t1 = f_sqn(t1, 10);
  t0 = f_mul(t1, t0);
  t1 = f_sqn(t0, 50);
  t1 = f_mul(t1, t0);
  t2 = f_sqn(t1, 100);
  t1 = f_mul(t2, t1);
  t1 = f_sqn(t1, 50);
  t0 = f_mul(t1, t0);
  t0 = f_sqn(t0, 2);
  return f_mul(t0, z);
}

// lanes <-> per-lane limbs (scalar radix-2^51 elements)
IFMA F f_gather(const u64 (*v)[5]) {
  alignas(64) u64 t[5][8];
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 5; ++k) t[k][i] = v[i][k];
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = _mm512_load_si512(t[k]);
  return r;
}
IFMA void f_scatter(const F& a, u64 (*v)[5]) {
  alignas(64) u64 t[5][8];
  for (int k = 0; k < 5; ++k) _mm512_store_si512(t[k], a.l[k]);
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 5; ++k) v[i][k] = t[k][i];
}
IFMA void f_tobytes(const F& a, u8 out[8][32]) {
  u64 v[8][5];
  f_scatter(a, v);
  for (int i = 0; i < 8; ++i) vrf_detail::fe51_tobytes(out[i], v[i]);
}

// ---------------------------------------------------------------- points (the scalar code's formulas)
IFMA P p_dbl(const P& p) {
  F A = f_sq(p.X), B = f_sq(p.Y);
  F zz = f_sq(p.Z);
  F Cc = f_add(zz, zz);
  F D = f_neg(A);
  F E = f_sub(f_sub(f_sq(f_add(p.X, p.Y)), A), B);
  F G = f_add(D, B), Fv = f_sub(G, Cc), H = f_sub(D, B);
  return P{f_mul(E, Fv), f_mul(G, H), f_mul(Fv, G), f_mul(E, H)};
}
IFMA P p_dbl_noT(const P& p) {   // the result feeds another doubling: T is never read
  F A = f_sq(p.X), B = f_sq(p.Y);
  F zz = f_sq(p.Z);
  F Cc = f_add(zz, zz);
  F D = f_neg(A);
  F E = f_sub(f_sub(f_sq(f_add(p.X, p.Y)), A), B);
  F G = f_add(D, B), Fv = f_sub(G, Cc), H = f_sub(D, B);
  return P{f_mul(E, Fv), f_mul(G, H), f_mul(Fv, G), f_zero()};
}
IFMA C p_cache(const P& p, const F& d2) {
  return C{f_add(p.Y, p.X), f_sub(p.Y, p.X), f_add(p.Z, p.Z), f_mul(p.T, d2)};
}
IFMA P p_add_cached(const P& p, const C& q) {
  F A = f_mul(f_sub(p.Y, p.X), q.YmX);
  F B = f_mul(f_add(p.Y, p.X), q.YpX);
  F Cc = f_mul(p.T, q.T2d);
  F D = f_mul(p.Z, q.Z2);
  F E = f_sub(B, A), Fv = f_sub(D, Cc), G = f_add(D, Cc), H = f_add(B, A);
  return P{f_mul(E, Fv), f_mul(G, H), f_mul(Fv, G), f_mul(E, H)};
}

// x_lane * P_lane: signed radix-16 digits (e[w][lane] in [-8, 8]), a per-lane table of 1P..8P selected by
// masked blends (lanes hold different points and digits), 4 doublings + 1 cached addition per digit
IFMA P p_mul(const P& p, const int64_t e[64][8], const F& d2) {
  C tbl[8];
  tbl[0] = p_cache(p, d2);
  P acc = p_dbl(p);
  tbl[1] = p_cache(acc, d2);
  for (int i = 2; i < 8; ++i) {
    acc = p_add_cached(acc, tbl[0]);
    tbl[i] = p_cache(acc, d2);
  }
  const F one = f_one();
  F two = f_zero();
  two.l[0] = v1(2);
  P r{f_zero(), one, one, f_zero()};
  for (int w = 63; w >= 0; --w) {
    if (w != 63) {
      r = p_dbl_noT(r);
      r = p_dbl_noT(r);
      r = p_dbl_noT(r);
      r = p_dbl(r);
    }
    const V d = _mm512_loadu_si512(e[w]);
    const V ad = _mm512_abs_epi64(d);
    C s{one, one, two, f_zero()};   // the identity (digit 0)
    for (int k = 0; k < 8; ++k) {
      const __mmask8 m = _mm512_cmpeq_epi64_mask(ad, v1(u64(k + 1)));
      if (!m) continue;
      s.YpX = f_blend(m, s.YpX, tbl[k].YpX);
      s.YmX = f_blend(m, s.YmX, tbl[k].YmX);
      s.Z2 = f_blend(m, s.Z2, tbl[k].Z2);
      s.T2d = f_blend(m, s.T2d, tbl[k].T2d);
    }
    const __mmask8 neg = _mm512_cmplt_epi64_mask(d, vz());
    if (neg) {
      const F ypx = s.YpX;
      s.YpX = f_blend(neg, s.YpX, s.YmX);
      s.YmX = f_blend(neg, s.YmX, ypx);
      s.T2d = f_blend(neg, s.T2d, f_neg(s.T2d));
    }
    r = p_add_cached(r, s);
  }
  return r;
}

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

const u8 SUITE = 0x03;

IFMA F f_bcast(const u64 v[5]) {
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = v1(v[k]);
  return r;
}

// ECVRF encode_to_curve (try-and-increment) of 8 (pk, alpha) pairs: each round hashes the pending lanes at their
// counters, decompresses all 8 candidates side by side, and retires the lanes whose candidate is a point
IFMA bool encode8(const VrfKey* const* keys, int n, const Bytes& alpha, const F& d, const F& sqrtm1, P& H) {
  int ctr[8] = {0};
  bool done[8];
  for (int i = 0; i < 8; ++i) done[i] = i >= n;
  u64 yv[8][5];
  u8 sign[8] = {0};
  u64 ox[8][5], oy[8][5];
  for (int i = 0; i < 8; ++i) {   // unused lanes: y = 1 (x = 0), any valid point
    memset(ox[i], 0, sizeof(ox[i]));
    memset(oy[i], 0, sizeof(oy[i]));
    oy[i][0] = 1;
  }
  for (int round = 0; round < 256; ++round) {
    bool any = false;
    bool canon[8] = {false};
    for (int i = 0; i < 8; ++i) {
      memset(yv[i], 0, sizeof(yv[i]));
      yv[i][0] = 1;
      if (done[i]) continue;
      any = true;
      Sha512 h;
      u8 pre[2] = {SUITE, 0x01};
      h.update(pre, 2);
      h.update(keys[i]->pk);
      h.update(alpha);
      u8 tail[2] = {u8(ctr[i]), 0x00};
      h.update(tail, 2);
      u8 dig[64];
      h.final(dig);
      sign[i] = dig[31] >> 7;
      u8 b[32];
      memcpy(b, dig, 32);
      b[31] &= 0x7f;
      vrf_detail::fe51_frombytes(yv[i], b);
      u8 chk[32];
      vrf_detail::fe51_tobytes(chk, yv[i]);
      canon[i] = memcmp(chk, b, 32) == 0;   // RFC 8032 5.1.3: a non-canonical y is no point
    }
    if (!any) break;
    const F y = f_gather(yv);
    const F y2 = f_sq(y);
    const F u = f_sub(y2, f_one());
    const F v = f_add(f_mul(d, y2), f_one());
    const F v3 = f_mul(f_sq(v), v);
    const F v7 = f_mul(f_sq(v3), v);
    F x = f_mul(f_mul(u, v3), f_pow22523(f_mul(u, v7)));
    const F vx2 = f_mul(v, f_sq(x));
    const F xr = f_mul(x, sqrtm1);
    u8 bvx2[8][32], bu[8][32], bnu[8][32];
    f_tobytes(vx2, bvx2);
    f_tobytes(u, bu);
    f_tobytes(f_neg(u), bnu);
    __mmask8 rot = 0;
    bool ok[8] = {false};
    for (int i = 0; i < 8; ++i) {
      if (done[i] || !canon[i]) continue;
      if (memcmp(bvx2[i], bu[i], 32) == 0) ok[i] = true;
      else if (memcmp(bvx2[i], bnu[i], 32) == 0) { ok[i] = true; rot |= __mmask8(1u << i); }
    }
    x = f_blend(rot, x, xr);
    u8 bx[8][32];
    f_tobytes(x, bx);
    const F nx = f_neg(x);
    u64 xv[8][5], nxv[8][5];
    f_scatter(x, xv);
    f_scatter(nx, nxv);
    for (int i = 0; i < 8; ++i) {
      if (done[i]) continue;
      bool zero = true;
      for (int k = 0; k < 32; ++k) zero = zero && bx[i][k] == 0;
      if (ok[i] && zero && sign[i]) ok[i] = false;
      if (!ok[i]) {
        ++ctr[i];
        if (ctr[i] > 255) return false;
        continue;
      }
      memcpy(ox[i], (bx[i][0] & 1) != sign[i] ? nxv[i] : xv[i], sizeof(ox[i]));
      memcpy(oy[i], yv[i], sizeof(oy[i]));
      done[i] = true;
    }
  }
  for (int i = 0; i < 8; ++i)
    if (!done[i]) return false;
  const F X = f_gather(ox), Y = f_gather(oy);
  P h{X, Y, f_one(), f_mul(X, Y)};
  H = p_dbl(p_dbl(p_dbl(h)));   // cofactor 8
  return true;
}

IFMA bool beta8(const VrfKey* const* keys, int n, const Bytes& alpha, Bytes* out) {
  u64 dv[5], sv[5];
  vrf_detail::fe51_consts(dv, sv);
  const F d = f_bcast(dv), sqrtm1 = f_bcast(sv);
  const F d2 = f_add(d, d);
  P H;
  if (!encode8(keys, n, alpha, d, sqrtm1, H)) return false;
  alignas(64) int64_t e[64][8];
  for (int i = 0; i < 8; ++i) {
    int8_t dg[64];
    if (i < n) signed_digits(dg, keys[i]->x);
    else memset(dg, 0, sizeof(dg));
    for (int w = 0; w < 64; ++w) e[w][i] = dg[w];
  }
  P G = p_mul(H, e, d2);
  G = p_dbl(p_dbl(p_dbl(G)));   // cofactor 8
  const F zi = f_invert(G.Z);
  u8 bx[8][32], by[8][32];
  f_tobytes(f_mul(G.X, zi), bx);
  f_tobytes(f_mul(G.Y, zi), by);
  for (int i = 0; i < n; ++i) {
    if (bx[i][0] & 1) by[i][31] |= 0x80;
    Sha512 bh;
    u8 pre[2] = {SUITE, 0x03};
    bh.update(pre, 2);
    bh.update(by[i], 32);
    u8 z = 0;
    bh.update(&z, 1);
    out[i].assign(64, 0);
    bh.final(out[i].data());
  }
  return true;
}

// k * B with the resident fixed-base table of B (64 signed radix-16 windows x 8 cached multiples): no
// doublings, one cached addition per window, each lane's entry selected by masked blends of broadcast entries
IFMA F f_bcast_limbs(const u64* v) {
  F r;
  for (int k = 0; k < 5; ++k) r.l[k] = v1(v[k]);
  return r;
}
IFMA P p_mul_base(const int64_t e[64][8]) {
  const u64* bt = vrf_detail::base_table_limbs();   // [512][4][5]
  const F one = f_one();
  F two = f_zero();
  two.l[0] = v1(2);
  P r{f_zero(), one, one, f_zero()};
  for (int w = 0; w < 64; ++w) {
    const V d = _mm512_loadu_si512(e[w]);
    const V ad = _mm512_abs_epi64(d);
    C s{one, one, two, f_zero()};
    for (int k = 0; k < 8; ++k) {
      const __mmask8 m = _mm512_cmpeq_epi64_mask(ad, v1(u64(k + 1)));
      if (!m) continue;
      const u64* t = bt + (size_t)(w * 8 + k) * 20;
      s.YpX = f_blend(m, s.YpX, f_bcast_limbs(t));
      s.YmX = f_blend(m, s.YmX, f_bcast_limbs(t + 5));
      s.Z2 = f_blend(m, s.Z2, f_bcast_limbs(t + 10));
      s.T2d = f_blend(m, s.T2d, f_bcast_limbs(t + 15));
    }
    const __mmask8 neg = _mm512_cmplt_epi64_mask(d, vz());
    if (neg) {
      const F ypx = s.YpX;
      s.YpX = f_blend(neg, s.YpX, s.YmX);
      s.YmX = f_blend(neg, s.YmX, ypx);
      s.T2d = f_blend(neg, s.T2d, f_neg(s.T2d));
    }
    r = p_add_cached(r, s);
  }
  return r;
}

// the RFC 8032 encodings of k points per lane (y with the sign of x in bit 255), one vector inversion
IFMA void p_encode(const P* const* pts, int k, u8 (*out)[8][32]) {
  F pre[4];
  F acc = f_one();
  for (int j = 0; j < k; ++j) {
    pre[j] = acc;
    acc = f_mul(acc, pts[j]->Z);
  }
  F inv = f_invert(acc);
  for (int j = k - 1; j >= 0; --j) {
    const F zi = f_mul(inv, pre[j]);
    inv = f_mul(inv, pts[j]->Z);
    u8 bx[8][32];
    f_tobytes(f_mul(pts[j]->X, zi), bx);
    f_tobytes(f_mul(pts[j]->Y, zi), out[j]);
    for (int i = 0; i < 8; ++i)
      if (bx[i][0] & 1) out[j][i][31] |= 0x80;
  }
}

IFMA void digits8(const u8 (*sc)[32], int n, int64_t e[64][8]) {
  for (int i = 0; i < 8; ++i) {
    int8_t dg[64];
    if (i < n) signed_digits(dg, sc[i]);
    else memset(dg, 0, sizeof(dg));
    for (int w = 0; w < 64; ++w) e[w][i] = dg[w];
  }
}

// ECVRF prove (vrf.cpp vrf_output + vrf_finish) for up to 8 keys: H, Gamma = x*H, k*B and k*H as lane vectors
IFMA bool prove8(const VrfKey* const* keys, int n, const Bytes& alpha, Bytes* beta, Bytes* pi) {
  u64 dv[5], sv[5];
  vrf_detail::fe51_consts(dv, sv);
  const F d = f_bcast(dv), sqrtm1 = f_bcast(sv);
  const F d2 = f_add(d, d);
  P H;
  if (!encode8(keys, n, alpha, d, sqrtm1, H)) return false;
  u8 hb[1][8][32];
  const P* hp[1] = {&H};
  p_encode(hp, 1, hb);
  u8 xs[8][32], ks[8][32];
  for (int i = 0; i < 8; ++i) {
    memset(xs[i], 0, 32);
    memset(ks[i], 0, 32);
    if (i >= n) continue;
    memcpy(xs[i], keys[i]->x, 32);
    Sha512 kh;   // nonce k = SHA-512(prefix || encode(H)) mod L (vrf_finish)
    kh.update(keys[i]->prefix, 32);
    kh.update(hb[0][i], 32);
    u8 kd[64];
    kh.final(kd);
    vrf_detail::sc_reduce64(ks[i], kd);
  }
  alignas(64) int64_t ex[64][8], ek[64][8];
  digits8(xs, n, ex);
  digits8(ks, n, ek);
  const P G = p_mul(H, ex, d2);
  const P Vp = p_mul(H, ek, d2);
  const P Up = p_mul_base(ek);
  const P G8 = p_dbl(p_dbl(p_dbl(G)));
  u8 enc[4][8][32];
  const P* pts[4] = {&G, &Up, &Vp, &G8};
  p_encode(pts, 4, enc);
  for (int i = 0; i < n; ++i) {
    Sha512 bh;
    u8 pre[2] = {SUITE, 0x03};
    bh.update(pre, 2);
    bh.update(enc[3][i], 32);
    u8 z = 0;
    bh.update(&z, 1);
    beta[i].assign(64, 0);
    bh.final(beta[i].data());
    const Bytes e0(enc[0][i], enc[0][i] + 32);
    const Bytes c = vrf_detail::challenge(keys[i]->pk, Bytes(hb[0][i], hb[0][i] + 32), e0,
                                          Bytes(enc[1][i], enc[1][i] + 32), Bytes(enc[2][i], enc[2][i] + 32));
    u8 s[32];
    vrf_detail::sc_muladd16(s, ks[i], c.data(), xs[i]);
    pi[i] = e0;
    pi[i].insert(pi[i].end(), c.begin(), c.end());
    pi[i].insert(pi[i].end(), s, s + 32);
  }
  return true;
}

}  // namespace

void vrf_prove_batch(const VrfKey* const* keys, int n, const Bytes& alpha, Bytes* beta, Bytes* pi) {
  for (int off = 0; off < n; off += 8) {
    const int m = n - off < 8 ? n - off : 8;
    if (!vrf_beta_batch_supported() || !prove8(keys + off, m, alpha, beta + off, pi + off))
      for (int i = 0; i < m; ++i) {
        auto r = vrf_prove(*keys[off + i], alpha);
        beta[off + i] = std::move(r.first);
        pi[off + i] = std::move(r.second);
      }
  }
}

bool vrf_beta_batch_supported() {
  static const bool ok = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512ifma");
  }();
  return ok;
}

void vrf_beta_batch(const VrfKey* const* keys, int n, const Bytes& alpha, Bytes* out) {
  for (int off = 0; off < n; off += 8) {
    const int m = n - off < 8 ? n - off : 8;
    if (!vrf_beta_batch_supported() || !beta8(keys + off, m, alpha, out + off))
      for (int i = 0; i < m; ++i) out[off + i] = vrf_beta(*keys[off + i], alpha);
  }
}

}  // namespace bsc
