// EXPERIMENT (not built): 9 x 29-bit-limb Montgomery arithmetic for the fixed-base MSM loops,
// with scripts/isa/msm_bn29_experiment.hip (msm.hip using it; tables stored as R29 coordinates).
// Bit-exact (tests/test_gpu_bn256.py: 16/16 passed with it), but SLOWER on MI355X: the share MSM
// for 62 rows took 1.32 ms against 1.10 ms for the 8 x 32-bit FIPS multiplier of bn256_dev.h
// (profiles/msm_bn29_ab.json).  Instruction counts barely differ (~240 vs ~286 per product: the
// carry-free columns still need 64-bit shifts and adds, and every add/sub needs a carry pass plus
// two reductions per point addition), so the lazy-reduction bookkeeping eats the gain.  Kept as
// the record of that measurement.
// BN256 base field in 9 x 29-bit limbs (Montgomery, R = 2^261) for the fixed-base MSM loops.
//
// Why a second representation: a product of two 29-bit limbs is < 2^58, so a whole product column
// (9 a*b terms + 9 m*p terms + the carry) fits one 64-bit accumulator.  A column is then a chain
// of plain v_mad_u64_u32 -- no carry flag, no high word, nothing that pins the order -- against
// one v_mad_u64_u32 + one v_addc per term in the 8 x 32-bit FIPS multiplier (bn256_dev.h).
// Additions are limb adds plus one carry pass (no borrow chains through VCC).
//
// Values are kept *lazily reduced*: every limb normalised (< 2^29, the top limb holds bits
// 232..260) but the value only bounded, not < p.  Since R / p = 57, a Montgomery product of inputs
// below A p and B p is below (A B / 57 + 1) p; the point formulas below track those bounds (see
// jac29_add_aff) and reduce two coordinates per addition with a quotient estimate from the top
// limb, so nothing ever leaves [0, 2^261).
//
// Tables: the fixed-base tables store affine points as canonical R29 values (x * 2^261 mod p)
// packed into 8 x 32-bit words (k_fb_table converts on write); to_r256 turns a result back into
// the 8 x 32-bit R = 2^256 form every other kernel uses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bn256_dev.h"

namespace bn29 {

constexpr uint32_t M29 = (1u << 29) - 1;
constexpr uint32_t NINV29 = 0x1f17daa9u;   // -p^-1 mod 2^29

__device__ __constant__ static const uint32_t P29[9] = {0x1e089667u, 0x02e56362u, 0x0d6d6786u, 0x1711a241u,
                                                        0x0dc21ee5u, 0x165c30c2u, 0x1fe6a9bfu, 0x1c695470u,
                                                        0x008fb501u};
// 4p and 8p with 2^30 borrowed into limbs 0..7 (every limb >= 2^30 - 2 > any normalised limb): the
// minuend-side constants of a borrow-free limb subtraction
__device__ __constant__ static const uint32_t D4[9] = {0x5822599cu, 0x4b958d89u, 0x55b59e16u, 0x5c468903u,
                                                       0x57087b94u, 0x5970c307u, 0x5f9aa6fcu, 0x51a551c1u,
                                                       0x023ed405u};
__device__ __constant__ static const uint32_t D8[9] = {0x5044b338u, 0x572b1b15u, 0x4b6b3c2eu, 0x588d1209u,
                                                       0x4e10f72bu, 0x52e18611u, 0x5f354dfbu, 0x434aa385u,
                                                       0x047da80du};
__device__ __constant__ static const uint32_t ONE29[9] = {0x10168311u, 0x1aecdef8u, 0x02a3f324u, 0x1d12df6fu,
                                                          0x0fc71ed9u, 0x057924b5u, 0x05a43451u, 0x0c8c32d7u,
                                                          0x0000b294u};
__device__ __constant__ static const uint32_t K256[9] = {0x01f76999u, 0x1d1a9c9du, 0x12929879u, 0x08ee5dbeu,
                                                         0x123de11au, 0x09a3cf3du, 0x00195640u, 0x0396ab8fu,
                                                         0x00704afeu};   // 2^256 mod p
__device__ __constant__ static const uint32_t K266[9] = {0x02d06220u, 0x1d9bdf10u, 0x147e649au, 0x025bede2u,
                                                         0x18e3db3du, 0x0f2496afu, 0x14868a25u, 0x11865ae5u,
                                                         0x0016528cu};   // 2^266 mod p

struct f29 {
  uint32_t v[9];
};

__device__ __forceinline__ f29 f29_const(const uint32_t* c) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = c[i];
  return r;
}

// carry pass: limbs 0..7 to 29 bits, the top limb keeps the rest
__device__ __forceinline__ void f29_carry(f29& r) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.v[i + 1] += r.v[i] >> 29;
    r.v[i] &= M29;
  }
}

__device__ __forceinline__ f29 f29_add(const f29& a, const f29& b) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
  f29_carry(r);
  return r;
}

// a + 4p - b (b < 3.5 p) and a + 8p - b (b < 7.5 p): no limb goes negative
__device__ __forceinline__ f29 f29_sub4(const f29& a, const f29& b) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + D4[i] - b.v[i];
  f29_carry(r);
  return r;
}
__device__ __forceinline__ f29 f29_sub8(const f29& a, const f29& b) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + D8[i] - b.v[i];
  f29_carry(r);
  return r;
}

// Montgomery reduction of the 17 product columns (each < 2^61.2): m*p terms added column by
// column (column + carry + 9 * 2^58 < 2^63)
__device__ __forceinline__ f29 f29_redc(const unsigned long long* ab) {
  uint32_t m[9];
  f29 r;
  unsigned long long t = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    t += ab[i];
#pragma unroll
    for (int j = 0; j < i; ++j) t += (unsigned long long)m[j] * P29[i - j];
    m[i] = ((uint32_t)t * NINV29) & M29;
    t += (unsigned long long)m[i] * P29[0];
    t >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
    t += ab[i];
#pragma unroll
    for (int j = i - 8; j < 9; ++j) t += (unsigned long long)m[j] * P29[i - j];
    r.v[i - 9] = (uint32_t)t & M29;
    t >>= 29;
  }
  r.v[8] = (uint32_t)t;
  return r;
}

// a^2 / 2^261: the 36 cross products once, doubled through 2 a_i (< 2^30; a column is <= 4 cross
// terms < 2^59 plus one square < 2^58), so 45 products instead of 81
__device__ __forceinline__ f29 f29_sqr(const f29& a) {
  unsigned long long ab[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) ab[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t a2 = a.v[i] << 1;
    ab[2 * i] += (unsigned long long)a.v[i] * a.v[i];
#pragma unroll
    for (int j = i + 1; j < 9; ++j) ab[i + j] += (unsigned long long)a2 * a.v[j];
  }
  return f29_redc(ab);
}

// Montgomery product a b / 2^261 (mod p).  The 17 columns of a*b are independent sums (< 9 * 2^58):
// they are formed first, so the scheduler can interleave those 81 v_mad_u64_u32 freely; the
// reduction then walks the columns once, adding m*p terms (column + carry + 9 * 2^58 < 2^63).
__device__ __forceinline__ f29 f29_mul(const f29& a, const f29& b) {
  unsigned long long ab[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) ab[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < 9; ++j) ab[i + j] += (unsigned long long)a.v[i] * b.v[j];
  }
  return f29_redc(ab);
}

// a - q p with q = floor(a_8 / (p_8 + 1)) <= a / p: the result is in [0, p + 2^238)
__device__ __forceinline__ f29 f29_reduce(const f29& a) {
  const uint32_t q = a.v[8] / (0x008fb501u + 1u);
  f29 r;
  long long s = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    s += (long long)a.v[i] - (long long)((unsigned long long)q * P29[i]);
    r.v[i] = (uint32_t)s & M29;
    s >>= 29;   // arithmetic: the borrow
  }
  r.v[8] = (uint32_t)(r.v[8] | ((uint32_t)s << 29));   // the final value is non-negative and < 2^261
  return r;
}

__device__ __forceinline__ bool f29_eq_limbs(const f29& a, const uint32_t* c) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) o |= a.v[i] ^ c[i];
  return o == 0;
}
// a == 0 (mod p) for a normalised a < 57 p
__device__ __forceinline__ bool f29_is_zero_mod(const f29& a) {
  const f29 r = f29_reduce(a);
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) z |= r.v[i];
  return z == 0 || f29_eq_limbs(r, P29);
}

// packed 8 x 32-bit little-endian words (value < 2^256) -> 29-bit limbs
__device__ __forceinline__ f29 f29_unpack(const uint32_t* w) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int off = 29 * i, wi = off >> 5, sh = off & 31;
    const unsigned long long lo = w[wi];
    const unsigned long long hi = (wi + 1 < 8) ? w[wi + 1] : 0ull;
    r.v[i] = (uint32_t)(((hi << 32) | lo) >> sh) & (i < 8 ? M29 : 0xffffffffu);
  }
  return r;
}
// canonical value (< p < 2^256) -> packed words
__device__ __forceinline__ void f29_pack(uint32_t* w, const f29& a) {
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int off = 29 * i, wi = off >> 5, sh = off & 31;
    w[wi] |= a.v[i] << sh;
    if (wi + 1 < 8 && sh > 3) w[wi + 1] |= a.v[i] >> (32 - sh);
  }
}
// fully reduced value in [0, p)
__device__ __forceinline__ f29 f29_canon(const f29& a) {
  f29 r = f29_reduce(a);
  // r < p + 2^238: subtract p once if r >= p
  f29 s;
  long long c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c += (long long)r.v[i] - (long long)P29[i];
    s.v[i] = (uint32_t)c & M29;
    c >>= 29;
  }
  const bool ge = c >= 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = ge ? s.v[i] : r.v[i];
  return r;
}

// R29 value -> R256 Montgomery value (bn::fp, canonical): a * 2^256 / 2^261
__device__ __forceinline__ bn::fp to_r256(const f29& a) {
  const f29 c = f29_canon(f29_mul(a, f29_const(K256)));
  bn::fp r;
  f29_pack(r.v, c);
  return r;
}
// R256 Montgomery value (canonical bn::fp) -> R29: a * 2^266 / 2^261
__device__ __forceinline__ f29 from_r256(const bn::fp& a) { return f29_mul(f29_unpack(a.v), f29_const(K266)); }

// ------------------------------------------------------------------ points
struct jac29 {
  f29 x, y, z;
  bool inf;
};

__device__ __forceinline__ jac29 jac29_inf() {
  jac29 r;
  r.inf = true;
  r.x = f29_const(ONE29);
  r.y = r.x;
  r.z = r.x;
  return r;
}

// table entry (canonical R29 x, y packed in 16 words; y == 0 <=> infinity) -> limbs
struct aff29 {
  f29 x, y;
};
__device__ __forceinline__ aff29 ld_aff29(const uint32_t* p) {
  aff29 q;
  q.x = f29_unpack(p);
  q.y = f29_unpack(p + 8);
  return q;
}
// -y for a canonical y (< p): p - y, or 0 for 0
__device__ __forceinline__ f29 f29_neg_canon(const f29& y) {
  f29 r;
  long long c = 0;
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    z |= y.v[i];
    c += (long long)P29[i] - (long long)y.v[i];
    r.v[i] = (uint32_t)c & M29;
    c >>= 29;
  }
  if (z == 0) return y;
  return r;
}

// the rare equal-x case of an addition, through the 8 x 32-bit formulas
__device__ __noinline__ jac29 jac29_dbl_slow(const jac29& p) {
  bn::jac q;
  q.x = to_r256(p.x);
  q.y = to_r256(p.y);
  q.z = to_r256(p.z);
  q = bn::jac_dbl(q);
  jac29 r;
  r.inf = bn::jac_is_inf(q);
  r.x = from_r256(q.x);
  r.y = from_r256(q.y);
  r.z = from_r256(q.z);
  if (!r.inf) {
    r.x = f29_reduce(r.x);
    r.y = f29_reduce(r.y);
  }
  return r;
}

// acc + q (q affine, canonical coordinates, not infinity).  madd-2007-bl with Z3 = 2 Z1 H.
// Bounds (units of p, inputs X1, Y1 < 1.01 (reduced), Z1 < 2.44; mul(A, B) < A B / 57 + 1):
//   z1z1 1.11  u2 1.02  t 1.05  s2 1.02  h = u2 + 4p - X1 5.02  rr 5.02  hh 1.45  i = 4 hh 5.8
//   j 1.52  r = 2 rr 10.04  v 1.11  r^2 2.77  w = j + 2 v 3.74  X3 = r^2 + 8p - w 10.8 -> reduce
//   d = v + 4p - X3 5.12  a = r d 1.91  b = 2 Y1 j 2.06  Y3 = a + 4p - b 5.91 -> reduce
//   Z3 = 2 Z1 h 2.43.
__device__ __forceinline__ jac29 jac29_add_aff(const jac29& p, const aff29& q) {
  if (p.inf) {
    jac29 r;
    r.inf = false;
    r.x = q.x;
    r.y = q.y;
    r.z = f29_const(ONE29);
    return r;
  }
  const f29 z1z1 = f29_sqr(p.z);
  const f29 u2 = f29_mul(q.x, z1z1);
  const f29 s2 = f29_mul(q.y, f29_mul(p.z, z1z1));
  const f29 h = f29_sub4(u2, p.x);
  const f29 rr = f29_sub4(s2, p.y);
  // h == 0 (mod p) only when the x's agree: screen on limb 0 of the multiples 0..5 p, then check
  const uint32_t h0 = h.v[0];
  if (h0 == 0u || h0 == 0x1e089667u || h0 == 0x1c112cceu || h0 == 0x1a19c335u || h0 == 0x1822599cu ||
      h0 == 0x162af003u) {
    if (f29_is_zero_mod(h)) {
      if (f29_is_zero_mod(rr)) return jac29_dbl_slow(p);
      return jac29_inf();
    }
  }
  const f29 hh = f29_sqr(h);
  f29 i4 = f29_add(hh, hh);
  i4 = f29_add(i4, i4);
  const f29 j = f29_mul(h, i4);
  const f29 r = f29_add(rr, rr);
  const f29 v = f29_mul(p.x, i4);
  jac29 o;
  o.inf = false;
  const f29 w = f29_add(j, f29_add(v, v));
  o.x = f29_reduce(f29_sub8(f29_sqr(r), w));
  const f29 b = f29_mul(p.y, j);
  o.y = f29_reduce(f29_sub4(f29_mul(r, f29_sub4(v, o.x)), f29_add(b, b)));
  const f29 zh = f29_mul(p.z, h);
  o.z = f29_add(zh, zh);
  return o;
}

// R29 Jacobian -> R256 Jacobian for the kernels downstream (infinity: z = 0)
__device__ __forceinline__ bn::jac to_jac256(const jac29& p) {
  if (p.inf) return bn::jac_inf();
  bn::jac r;
  r.x = to_r256(p.x);
  r.y = to_r256(p.y);
  r.z = to_r256(p.z);
  return r;
}

}  // namespace bn29
