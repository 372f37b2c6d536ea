// BN256 G1 arithmetic for CDNA4 (gfx950).
//
// Field elements: 8 x 32-bit little-endian limbs in Montgomery form (R = 2^256), the same
// representation the host runtime uses with 4 x 64-bit limbs, so affine tables produced on the
// host can be consumed verbatim.  Products use FIPS Montgomery with v_mad_u64_u32 carry chains,
// adds/subs explicit VCC carry chains (bn256_fp_asm.h); p > 2^255, so every add/sub reduces fully.
//
// Curve: y^2 = x^3 + 3 (a = 0), Jacobian coordinates, infinity <=> Z == 0.
// Affine table points use (0, 0) for infinity (y == 0 never occurs on this prime-order curve).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bn256_fp_asm.h"

namespace bn {

struct fp {
  uint32_t v[8];
};

__device__ __constant__ static const uint32_t P[8] = {0x5e089667u, 0x185cac6cu, 0x20b5b59eu, 0xee5b88d1u,
                                                       0x6184dc21u, 0xaa6fecb8u, 0x4aa387f9u, 0x8fb501e3u};
__device__ __constant__ static const uint32_t ONE[8] = {0xa1f76999u, 0xe7a35393u, 0xdf4a4a61u, 0x11a4772eu,
                                                         0x9e7b23deu, 0x55901347u, 0xb55c7806u, 0x704afe1cu};
static constexpr uint32_t NINV = 0x7f17daa9u;

__device__ __forceinline__ fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = 0;
  return r;
}
__device__ __forceinline__ fp fp_one() {
  fp r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = ONE[i];
  return r;
}
__device__ __forceinline__ bool fp_is_zero(const fp& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i];
  return o == 0;
}
__device__ __forceinline__ bool fp_eq(const fp& a, const fp& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// r = a - p if (carry || a >= p) else a
__device__ __forceinline__ fp fp_reduce_once(const uint32_t* t, uint32_t carry) {
  fp r;
  reduce256(r.v, t, carry);
  return r;
}

__device__ __forceinline__ fp fp_add(const fp& a, const fp& b) {
  uint32_t t[8];
  const uint32_t cy = add256(t, a.v, b.v);
  return fp_reduce_once(t, cy);
}

__device__ __forceinline__ fp fp_sub(const fp& a, const fp& b) {
  fp r;
  sub256_mod(r.v, a.v, b.v);
  return r;
}

__device__ __forceinline__ fp fp_neg(const fp& a) {
  fp r;
  neg256_raw(r.v, a.v);
  const bool z = fp_is_zero(a);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = z ? 0u : r.v[i];
  return r;
}

__device__ __forceinline__ fp fp_dbl(const fp& a) { return fp_add(a, a); }

// Montgomery product a*b/R mod p: finely integrated product scanning (FIPS).  Column k of
// a*b and of m*p accumulate together in a 96-bit (acc:hi) register triple; each limb product is
// one v_mad_u64_u32 with carry-out plus one v_addc (see mac()).  1.40x the CIOS throughput on
// MI355X (scripts/isa/fpmul_bench.hip: 110.8 vs 79.1 Gmul/s), bit-identical results.
__device__ __forceinline__ fp fp_mul(const fp& a, const fp& b) {
  uint32_t m[8], u[8];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) mac2(acc, hi, a.v[j], b.v[i - j], m[j], P[i - j]);
    mac(acc, hi, a.v[i], b.v[0]);
    m[i] = (uint32_t)acc * NINV;
    mac(acc, hi, m[i], P[0]);
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 15; ++i) {
#pragma unroll
    for (int j = i - 7; j < 8; ++j) mac2(acc, hi, a.v[j], b.v[i - j], m[j], P[i - j]);
    u[i - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  u[7] = (uint32_t)acc;
  return fp_reduce_once(u, (uint32_t)(acc >> 32));
}

__device__ __forceinline__ fp fp_sqr(const fp& a) { return fp_mul(a, a); }

// a^(p-2) (Fermat inverse); a == 0 -> 0
__device__ inline fp fp_inv(const fp& a) {
  // exponent p - 2, scanned from the top bit
  const uint32_t E[8] = {0x5e089665u, 0x185cac6cu, 0x20b5b59eu, 0xee5b88d1u,
                         0x6184dc21u, 0xaa6fecb8u, 0x4aa387f9u, 0x8fb501e3u};
  fp r = fp_one();
  for (int w = 7; w >= 0; --w) {
    const uint32_t e = E[w];
    for (int b = 31; b >= 0; --b) {
      r = fp_sqr(r);
      if ((e >> b) & 1u) r = fp_mul(r, a);
    }
  }
  return r;
}

// from Montgomery: a * 1 / R
__device__ __forceinline__ fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.v[0] = 1;
  return fp_mul(a, one);
}

// ------------------------------------------------------------------ points
struct jac {
  fp x, y, z;
};
struct aff {
  fp x, y;  // (0,0) = infinity
};

__device__ __forceinline__ jac jac_inf() {
  jac r;
  r.x = fp_zero();
  r.y = fp_one();
  r.z = fp_zero();
  return r;
}
__device__ __forceinline__ bool jac_is_inf(const jac& p) { return fp_is_zero(p.z); }
__device__ __forceinline__ bool aff_is_inf(const aff& q) { return fp_is_zero(q.y); }

// dbl-2009-l
__device__ inline jac jac_dbl(const jac& p) {
  if (jac_is_inf(p)) return p;
  fp A = fp_sqr(p.x);
  fp B = fp_sqr(p.y);
  fp C = fp_sqr(B);
  fp t = fp_sqr(fp_add(p.x, B));
  t = fp_sub(fp_sub(t, A), C);
  fp D = fp_dbl(t);
  fp E = fp_add(fp_dbl(A), A);
  fp F = fp_sqr(E);
  jac r;
  r.x = fp_sub(F, fp_dbl(D));
  fp c8 = fp_dbl(fp_dbl(fp_dbl(C)));
  r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), c8);
  r.z = fp_dbl(fp_mul(p.y, p.z));
  return r;
}

// add-2007-bl, complete for the special cases (P==Q, P==-Q, infinities)
__device__ __forceinline__ jac jac_add(const jac& p, const jac& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  fp z1z1 = fp_sqr(p.z);
  fp z2z2 = fp_sqr(q.z);
  fp u1 = fp_mul(p.x, z2z2);
  fp u2 = fp_mul(q.x, z1z1);
  fp s1 = fp_mul(p.y, fp_mul(q.z, z2z2));
  fp s2 = fp_mul(q.y, fp_mul(p.z, z1z1));
  fp h = fp_sub(u2, u1);
  fp r = fp_sub(s2, s1);
  if (fp_is_zero(h)) {
    if (fp_is_zero(r)) return jac_dbl(p);
    return jac_inf();
  }
  fp i = fp_sqr(fp_dbl(h));
  fp j = fp_mul(h, i);
  r = fp_dbl(r);
  fp v = fp_mul(u1, i);
  jac o;
  o.x = fp_sub(fp_sub(fp_sub(fp_sqr(r), j), v), v);
  o.y = fp_sub(fp_mul(r, fp_sub(v, o.x)), fp_dbl(fp_mul(s1, j)));
  fp zz = fp_sqr(fp_add(p.z, q.z));
  o.z = fp_mul(fp_sub(fp_sub(zz, z1z1), z2z2), h);
  return o;
}

// madd-2007-bl: Jacobian + affine (Z2 = 1), complete for the special cases
__device__ inline jac jac_add_aff(const jac& p, const aff& q) {
  if (aff_is_inf(q)) return p;
  if (jac_is_inf(p)) {
    jac r;
    r.x = q.x;
    r.y = q.y;
    r.z = fp_one();
    return r;
  }
  fp z1z1 = fp_sqr(p.z);
  fp u2 = fp_mul(q.x, z1z1);
  fp s2 = fp_mul(q.y, fp_mul(p.z, z1z1));
  fp h = fp_sub(u2, p.x);
  fp r = fp_sub(s2, p.y);
  if (fp_is_zero(h)) {
    if (fp_is_zero(r)) return jac_dbl(p);
    return jac_inf();
  }
  fp hh = fp_sqr(h);
  fp i = fp_dbl(fp_dbl(hh));
  fp j = fp_mul(h, i);
  r = fp_dbl(r);
  fp v = fp_mul(p.x, i);
  jac o;
  o.x = fp_sub(fp_sub(fp_sub(fp_sqr(r), j), v), v);
  o.y = fp_sub(fp_mul(r, fp_sub(v, o.x)), fp_dbl(fp_mul(p.y, j)));
  fp zh = fp_sqr(fp_add(p.z, h));
  o.z = fp_sub(fp_sub(zh, z1z1), hh);
  return o;
}

__device__ __forceinline__ aff aff_neg(const aff& q) {
  aff r;
  r.x = q.x;
  r.y = fp_neg(q.y);
  return r;
}

__device__ __forceinline__ jac jac_neg(const jac& p) {
  jac r = p;
  r.y = fp_neg(p.y);
  return r;
}

// small signed scalar multiple (|k| < 2^31) by double-and-add
__device__ inline jac jac_mul_small(const jac& p, int k) {
  unsigned m = k < 0 ? unsigned(-k) : unsigned(k);
  jac acc = jac_inf();
  for (int b = 31; b >= 0; --b) {
    acc = jac_dbl(acc);
    if ((m >> b) & 1u) acc = jac_add(acc, p);
  }
  return k < 0 ? jac_neg(acc) : acc;
}

// Jacobian -> affine (Montgomery); infinity -> (0,0)
__device__ inline aff jac_to_aff(const jac& p) {
  aff r;
  if (jac_is_inf(p)) {
    r.x = fp_zero();
    r.y = fp_zero();
    return r;
  }
  fp zi = fp_inv(p.z);
  fp zi2 = fp_sqr(zi);
  r.x = fp_mul(p.x, zi2);
  r.y = fp_mul(p.y, fp_mul(zi2, zi));
  return r;
}

// ------------------------------------------------------------------ global memory helpers
__device__ __forceinline__ fp ld_fp(const uint32_t* p) {
  fp r;
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}
__device__ __forceinline__ void st_fp(uint32_t* p, const fp& a) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  q[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
__device__ __forceinline__ jac ld_jac(const uint32_t* p) {
  jac r;
  r.x = ld_fp(p);
  r.y = ld_fp(p + 8);
  r.z = ld_fp(p + 16);
  return r;
}
__device__ __forceinline__ void st_jac(uint32_t* p, const jac& a) {
  st_fp(p, a.x);
  st_fp(p + 8, a.y);
  st_fp(p + 16, a.z);
}
__device__ __forceinline__ aff ld_aff(const uint32_t* p) {
  aff r;
  r.x = ld_fp(p);
  r.y = ld_fp(p + 8);
  return r;
}
__device__ __forceinline__ void st_aff(uint32_t* p, const aff& a) {
  st_fp(p, a.x);
  st_fp(p + 8, a.y);
}

}  // namespace bn
