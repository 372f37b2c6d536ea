// ECVRF-EDWARDS25519-SHA512-TAI proofs (RFC 9381) on gfx950 -- the VRF proofs the protocol
// computes but never consumes: the roles proof of getVRFRoles (quirk Q7) and the proof half of every
// worker's noiser VRF (vrf.go:54-100; the lottery reads only the 64-byte output, which the host
// computes on the critical path).  The host runtime (runtime/vrf.cpp) is the bit-exact oracle.
//
// Latency, not throughput, is what matters: a round submits ~200 proofs (a few waves on a 1024-SIMD
// chip) and the last round's proofs must finish before a timed run ends.  A proof's work is therefore
// split over the three waves of a workgroup (16 proofs per workgroup), wave-uniform roles, LDS hand-off:
//   phase 1  hash to curve, try-and-increment: 12 counters per proof tried at once (3 waves x 4 lanes);
//            the smallest counter that decodes wins (the RFC's choice), so one round almost always ends it
//   phase 2  wave 0: cofactor, the signed radix-16 table of H (global scratch) -> Gamma = x*H
//            wave 1: cofactor, encode(H) (one inversion), nonce k = SHA512(prefix || H) mod L  -> V = k*H
//            wave 2: U = k*B over the resident fixed-base table, 4 lanes per proof x 16 windows each
//   phase 4  wave 0: the three encodings with one inversion, the challenge hash, s = k + c x mod L
// The critical path is one variable-base multiplication plus two inversions (~3.2k field products)
// instead of the serial ~6.6k of a thread-per-proof design.  Hot loops are kept rolled so a wave's loop
// body fits the instruction cache (the unrolled thread-per-proof kernel streamed ~0.5 MB of code).
//
// Field elements: 10 unsigned 32-bit limbs in radix 2^25.5 (26, 25, 26, ... bits).  A product is
// 100 32x32->64 multiply-adds (v_mad_u64_u32) into 64-bit column sums, then one carry chain; the
// wrap-around 2^255 = 19 is folded into the multiplicands (19 g_j), and the odd-odd products carry
// an extra factor 2 (2^26 * 2^25 = 2^51 = 2 * 2^50.5...).  Limbs stay non-negative: subtraction adds
// 4p first.  Bounds: carried limbs are < 2^26 + 2^9, so a column sum is < 2^62.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BSC_PRIO_FLAG bsc_prio_on_vrf
#include "wave_prio.h"
BSC_PRIO_SETTER(bsc_wave_prio_vrf)

namespace {

__constant__ static const unsigned long long K512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull,
};
__constant__ static const unsigned long long H512[8] = {
    0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
    0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull,
};

__device__ __forceinline__ unsigned long long rotr64(unsigned long long x, int n) { return (x >> n) | (x << (64 - n)); }

struct Sha512 {
  unsigned long long h[8];
  uint8_t buf[128];
  int blen;
  unsigned long long total;
};

__device__ void sha_compress(Sha512& s) {
  unsigned long long w[80];
  for (int i = 0; i < 16; ++i) {
    unsigned long long v = 0;
    for (int b = 0; b < 8; ++b) v = (v << 8) | s.buf[8 * i + b];
    w[i] = v;
  }
  for (int i = 16; i < 80; ++i) {
    const unsigned long long s0 = rotr64(w[i - 15], 1) ^ rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    const unsigned long long s1 = rotr64(w[i - 2], 19) ^ rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  unsigned long long a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
  for (int i = 0; i < 80; ++i) {
    const unsigned long long S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    const unsigned long long ch = (e & f) ^ (~e & g);
    const unsigned long long t1 = h + S1 + ch + K512[i] + w[i];
    const unsigned long long S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    const unsigned long long mj = (a & b) ^ (a & c) ^ (b & c);
    const unsigned long long t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d; s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}
__device__ void sha_init(Sha512& s) {
  for (int i = 0; i < 8; ++i) s.h[i] = H512[i];
  s.blen = 0;
  s.total = 0;
}
__device__ void sha_byte(Sha512& s, uint8_t v) {
  s.buf[s.blen++] = v;
  s.total += 1;
  if (s.blen == 128) {
    sha_compress(s);
    s.blen = 0;
  }
}
__device__ void sha_bytes(Sha512& s, const uint8_t* p, int n) {
  for (int i = 0; i < n; ++i) sha_byte(s, p[i]);
}
__device__ void sha_words(Sha512& s, const uint32_t* w, int nw) {   // little-endian words as bytes
  for (int i = 0; i < nw; ++i)
    for (int b = 0; b < 4; ++b) sha_byte(s, (uint8_t)(w[i] >> (8 * b)));
}
__device__ void sha_final(Sha512& s, uint8_t out[64]) {
  const unsigned long long bits = s.total * 8;
  sha_byte(s, 0x80);
  while (s.blen != 112) sha_byte(s, 0);
  for (int b = 0; b < 8; ++b) sha_byte(s, 0);          // high 64 bits of the 128-bit length
  for (int b = 7; b >= 0; --b) sha_byte(s, (uint8_t)(bits >> (8 * b)));
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(s.h[i] >> (56 - 8 * b));
}

// ---------------------------------------------------------------- GF(2^255 - 19)
struct fe { uint32_t v[10]; };
__device__ __forceinline__ constexpr int fw(int i) { return (i & 1) ? 25 : 26; }

__device__ __forceinline__ fe fe_small(uint32_t a) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = 0;
  r.v[0] = a;
  return r;
}
__device__ __forceinline__ void fe_carry(fe& r) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t c = r.v[i] >> fw(i);
    r.v[i] &= (1u << fw(i)) - 1;
    if (i < 9) r.v[i + 1] += c;
    else r.v[0] += 19 * c;
  }
}
__device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i];
  fe_carry(r);
  return r;
}
__device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  fe r;   // a + 4p - b
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t p4 = i == 0 ? 0x0FFFFFB4u : ((i & 1) ? 0x07FFFFFCu : 0x0FFFFFFCu);
    r.v[i] = a.v[i] + p4 - b.v[i];
  }
  fe_carry(r);
  return r;
}
__device__ __forceinline__ fe fe_neg(const fe& a) { return fe_sub(fe_small(0), a); }

__device__ fe fe_mul(const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    g19[i] = 19 * g.v[i];
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  unsigned long long h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      h[(i + j) % 10] += (unsigned long long)a * b;
    }
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned long long c = h[i] >> fw(i);
    h[i] &= (1ull << fw(i)) - 1;
    if (i < 9) h[i + 1] += c;
    else h[0] += 19 * c;
  }
  const unsigned long long c = h[0] >> 26;
  h[0] &= (1ull << 26) - 1;
  h[1] += c;
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = (uint32_t)h[i];
  return r;
}
// f^2 with the 45 symmetric cross products taken once (doubled): 55 limb products instead of fe_mul's 100.
// Same radix conventions as fe_mul: an odd-odd limb pair carries a factor 2 (25-bit limbs), a wrap past
// limb 9 a factor 19; every partial product stays below 2^60 and every column below 2^64.
__device__ fe fe_sq(const fe& f) {
  uint32_t f19[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) f19[i] = 19 * f.v[i];
  unsigned long long h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // the diagonal term (i, i)
    const uint32_t ad = (i & 1) ? 2 * f.v[i] : f.v[i];
    const uint32_t bd = (2 * i >= 10) ? f19[i] : f.v[i];
    h[(2 * i) % 10] += (unsigned long long)ad * bd;
#pragma unroll
    for (int j = i + 1; j < 10; ++j) {   // (i, j) and (j, i) together
      const uint32_t a = ((i & 1) && (j & 1)) ? 4 * f.v[i] : 2 * f.v[i];
      const uint32_t b = (i + j >= 10) ? f19[j] : f.v[j];
      h[(i + j) % 10] += (unsigned long long)a * b;
    }
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned long long c = h[i] >> fw(i);
    h[i] &= (1ull << fw(i)) - 1;
    if (i < 9) h[i + 1] += c;
    else h[0] += 19 * c;
  }
  const unsigned long long c = h[0] >> 26;
  h[0] &= (1ull << 26) - 1;
  h[1] += c;
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = (uint32_t)h[i];
  return r;
}
__device__ fe fe_sqn(fe a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// canonical little-endian 255-bit value as 8 words
__device__ void fe_tobytes(uint32_t out[8], fe a) {
  fe_carry(a);
  fe_carry(a);
  uint32_t q = (a.v[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (a.v[i] + q) >> fw(i);
  a.v[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t c = a.v[i] >> fw(i);
    a.v[i] &= (1u << fw(i)) - 1;
    a.v[i + 1] += c;
  }
  a.v[9] &= (1u << 25) - 1;
  unsigned long long acc = 0;
  int bits = 0, o = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    acc |= (unsigned long long)a.v[i] << bits;
    bits += fw(i);
    if (bits >= 32) {
      out[o++] = (uint32_t)acc;
      acc >>= 32;
      bits -= 32;
    }
  }
  out[7] = (uint32_t)acc;
}
__device__ fe fe_frombytes(const uint32_t w[8]) {   // bit 255 ignored
  fe r;
  int off = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int wi = off >> 5, sh = off & 31;
    const unsigned long long lo = w[wi], hi = wi + 1 < 8 ? w[wi + 1] : 0u;
    r.v[i] = (uint32_t)(((hi << 32) | lo) >> sh) & ((1u << fw(i)) - 1);
    off += fw(i);
  }
  return r;
}
__device__ bool fe_eq(const fe& a, const fe& b) {
  uint32_t x[8], y[8];
  fe_tobytes(x, a);
  fe_tobytes(y, b);
  uint32_t o = 0;
  for (int i = 0; i < 8; ++i) o |= x[i] ^ y[i];
  return o == 0;
}
__device__ bool fe_isneg(const fe& a) {
  uint32_t x[8];
  fe_tobytes(x, a);
  return x[0] & 1;
}
__device__ bool fe_iszero(const fe& a) { return fe_eq(a, fe_small(0)); }
__device__ fe fe_invert(const fe& z) {   // z^(p-2)
  fe t0 = fe_sq(z);
  fe t1 = fe_sqn(t0, 2);
  t1 = fe_mul(z, t1);
  t0 = fe_mul(t0, t1);
  fe t2 = fe_sq(t0);
  t1 = fe_mul(t1, t2);
  t2 = fe_sqn(t1, 5);
  t1 = fe_mul(t2, t1);
  t2 = fe_sqn(t1, 10);
  t2 = fe_mul(t2, t1);
  fe t3 = fe_sqn(t2, 20);
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
__device__ fe fe_pow22523(const fe& z) {   // z^((p-5)/8)
  fe t0 = fe_sq(z);
  fe t1 = fe_sqn(t0, 2);
  t1 = fe_mul(z, t1);
  t0 = fe_mul(t0, t1);
  t0 = fe_sq(t0);
  t0 = fe_mul(t1, t0);
  t1 = fe_sqn(t0, 5);
  t0 = fe_mul(t1, t0);
  t1 = fe_sqn(t0, 10);
  t1 = fe_mul(t1, t0);
  fe t2 = fe_sqn(t1, 20);
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

__constant__ static const uint32_t C_D[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                                             0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
__constant__ static const uint32_t C_D2[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                                              0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
__constant__ static const uint32_t C_SQRTM1[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                                                  0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
__device__ __forceinline__ fe fe_const(const uint32_t* c) {
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = c[i];
  return fe_frombytes(w);
}

// ---------------------------------------------------------------- edwards25519 points
struct ge { fe X, Y, Z, T; };
struct gc { fe YpX, YmX, Z2, T2d; };   // cached form: an addition is 8 products

__device__ ge ge_identity() { return ge{fe_small(0), fe_small(1), fe_small(1), fe_small(0)}; }
__device__ gc ge_cache(const ge& p, const fe& d2) {
  return gc{fe_add(p.Y, p.X), fe_sub(p.Y, p.X), fe_add(p.Z, p.Z), fe_mul(p.T, d2)};
}
__device__ ge ge_add_cached(const ge& p, const gc& q) {
  const fe A = fe_mul(fe_sub(p.Y, p.X), q.YmX);
  const fe B = fe_mul(fe_add(p.Y, p.X), q.YpX);
  const fe C = fe_mul(p.T, q.T2d);
  const fe D = fe_mul(p.Z, q.Z2);
  const fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
__device__ ge ge_dbl(const ge& p, bool withT) {   // dbl-2008-hwcd, a = -1
  const fe A = fe_sq(p.X), B = fe_sq(p.Y);
  const fe zz = fe_sq(p.Z);
  const fe C = fe_add(zz, zz);
  const fe D = fe_neg(A);
  const fe E = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), A), B);
  const fe G = fe_add(D, B), F = fe_sub(G, C), H = fe_sub(D, B);
  return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), withT ? fe_mul(E, H) : fe_small(0)};
}
__device__ gc gc_neg(const gc& c) { return gc{c.YmX, c.YpX, c.Z2, fe_neg(c.T2d)}; }

__device__ void st_fe(uint32_t* p, const fe& a) {
  for (int i = 0; i < 10; ++i) p[i] = a.v[i];
}
__device__ fe ld_fe(const uint32_t* p) {
  fe r;
  for (int i = 0; i < 10; ++i) r.v[i] = p[i];
  return r;
}
__device__ void st_gc(uint32_t* p, const gc& c) {
  st_fe(p, c.YpX); st_fe(p + 10, c.YmX); st_fe(p + 20, c.Z2); st_fe(p + 30, c.T2d);
}
__device__ gc ld_gc(const uint32_t* p) { return gc{ld_fe(p), ld_fe(p + 10), ld_fe(p + 20), ld_fe(p + 30)}; }

// scalar (8 LE words, < 2^255) -> 64 signed radix-16 digits in [-8, 8)
__device__ void signed_digits(int8_t e[64], const uint32_t k[8]) {
  for (int i = 0; i < 64; ++i) e[i] = (int8_t)((k[i >> 3] >> (4 * (i & 7))) & 15);
  int carry = 0;
  for (int i = 0; i < 63; ++i) {
    e[i] = (int8_t)(e[i] + carry);
    carry = (e[i] + 8) >> 4;
    e[i] = (int8_t)(e[i] - (carry << 4));
  }
  e[63] = (int8_t)(e[63] + carry);
}
// k * P with P's table (1P..8P, cached) already in `tbl` (global scratch of this thread)
// not inlined: waves 0 and 1 of a workgroup run this one copy (x H and k H) from the instruction cache
__device__ __attribute__((noinline)) ge ge_mul_tbl(const uint32_t* tbl, const uint32_t k[8]) {
  int8_t e[64];
  signed_digits(e, k);
  ge r = ge_identity();
#pragma unroll 1
  for (int w = 63; w >= 0; --w) {
    if (w != 63) {
#pragma unroll 1
      for (int j = 0; j < 4; ++j) r = ge_dbl(r, j == 3);
    }
    const int d = e[w];
    if (d > 0) r = ge_add_cached(r, ld_gc(tbl + (d - 1) * 40));
    else if (d < 0) r = ge_add_cached(r, gc_neg(ld_gc(tbl + (-d - 1) * 40)));
  }
  return r;
}
// fixed base: btab[w * 8 + d - 1] = d * 16^w * B in cached form, 4 canonical fe encodings (32 words)
__device__ gc ld_btab(const uint32_t* btab, int idx) {
  const uint32_t* p = btab + idx * 32;
  uint32_t w[8];
  gc c;
  for (int i = 0; i < 8; ++i) w[i] = p[i];
  c.YpX = fe_frombytes(w);
  for (int i = 0; i < 8; ++i) w[i] = p[8 + i];
  c.YmX = fe_frombytes(w);
  for (int i = 0; i < 8; ++i) w[i] = p[16 + i];
  c.Z2 = fe_frombytes(w);
  for (int i = 0; i < 8; ++i) w[i] = p[24 + i];
  c.T2d = fe_frombytes(w);
  return c;
}
__device__ ge ge_mul_base(const uint32_t* btab, const uint32_t k[8]) {
  int8_t e[64];
  signed_digits(e, k);
  ge r = ge_identity();
  for (int w = 0; w < 64; ++w) {
    const int d = e[w];
    if (d > 0) r = ge_add_cached(r, ld_btab(btab, w * 8 + d - 1));
    else if (d < 0) r = ge_add_cached(r, gc_neg(ld_btab(btab, w * 8 - d - 1)));
  }
  return r;
}
// RFC 8032 5.1.3 decoding (non-canonical y rejected)
__device__ bool ge_frombytes(ge& out, const uint8_t in[32], const fe& d) {
  uint32_t w[8];
  for (int i = 0; i < 8; ++i)
    w[i] = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) | ((uint32_t)in[4 * i + 2] << 16) |
           ((uint32_t)in[4 * i + 3] << 24);
  const int sign = w[7] >> 31;
  w[7] &= 0x7fffffffu;
  const fe y = fe_frombytes(w);
  uint32_t chk[8];
  fe_tobytes(chk, y);
  uint32_t o = 0;
  for (int i = 0; i < 8; ++i) o |= chk[i] ^ w[i];
  if (o) return false;
  const fe y2 = fe_sq(y);
  const fe u = fe_sub(y2, fe_small(1));
  const fe v = fe_add(fe_mul(d, y2), fe_small(1));
  const fe v3 = fe_mul(fe_sq(v), v);
  const fe v7 = fe_mul(fe_sq(v3), v);
  fe x = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  const fe vx2 = fe_mul(v, fe_sq(x));
  if (!fe_eq(vx2, u)) {
    if (fe_eq(vx2, fe_neg(u))) x = fe_mul(x, fe_const(C_SQRTM1));
    else return false;
  }
  if (fe_iszero(x) && sign) return false;
  if ((int)fe_isneg(x) != sign) x = fe_neg(x);
  out = ge{x, y, fe_small(1), fe_mul(x, y)};
  return true;
}
__device__ void enc_affine(uint32_t out[8], const fe& x, const fe& y) {
  fe_tobytes(out, y);
  if (fe_isneg(x)) out[7] |= 0x80000000u;
}

// ---------------------------------------------------------------- scalars mod L
__constant__ static const unsigned long long C_L[4] = {0x5812631a5cf5d3edull, 0x14def9dea2f79cd6ull, 0ull,
                                                       0x1000000000000000ull};
// r = (little-endian byte string of `nbits` bits, given as 32-bit words) mod L, bitwise
__device__ void sc_reduce_words(uint32_t out[8], const uint32_t* in, int nbits) {
  unsigned long long r[4] = {0, 0, 0, 0};
  for (int bi = nbits - 1; bi >= 0; --bi) {
    unsigned long long c = (in[bi >> 5] >> (bi & 31)) & 1u;
    for (int i = 0; i < 4; ++i) {
      const unsigned long long nc = r[i] >> 63;
      r[i] = (r[i] << 1) | c;
      c = nc;
    }
    bool ge_l = true;
    for (int i = 3; i >= 0; --i) {
      if (r[i] != C_L[i]) {
        ge_l = r[i] > C_L[i];
        break;
      }
    }
    if (ge_l) {
      unsigned long long br = 0;
      for (int i = 0; i < 4; ++i) {
        const unsigned long long li = C_L[i] + br;
        const unsigned long long nb = (li < br) || (r[i] < li);
        r[i] -= li;
        br = nb;
      }
    }
  }
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = (uint32_t)r[i];
    out[2 * i + 1] = (uint32_t)(r[i] >> 32);
  }
}

constexpr uint8_t SUITE = 0x03;



// r = (256-bit little-endian value given as 8 words) * 2^32 + w, reduced mod L (r < L on entry).
// L = 2^252 + delta: q = X >> 252 over-estimates floor(X / L) by at most one, so X - q L lies in
// (-L, L) and one conditional add of L finishes the step.
__device__ void sc_step(unsigned long long r[4], uint32_t w) {
  typedef unsigned __int128 u128;
  unsigned long long x[5];
  x[0] = (r[0] << 32) | w;
  x[1] = (r[1] << 32) | (r[0] >> 32);
  x[2] = (r[2] << 32) | (r[1] >> 32);
  x[3] = (r[3] << 32) | (r[2] >> 32);
  x[4] = r[3] >> 32;
  const unsigned long long q = (x[4] << 4) | (x[3] >> 60);   // X >> 252 (< 2^37)
  // X - q L, five limbs, two's complement
  unsigned long long borrow = 0, carry = 0;
  for (int i = 0; i < 5; ++i) {
    const u128 m = (u128)q * (i < 4 ? C_L[i] : 0ull) + carry;
    carry = (unsigned long long)(m >> 64);
    const unsigned long long lo = (unsigned long long)m;
    const unsigned long long d = x[i] - lo - borrow;
    borrow = (x[i] < lo) || (x[i] - lo < borrow);
    x[i] = d;
  }
  if ((long long)x[4] < 0) {   // negative: add L back
    unsigned long long c = 0;
    for (int i = 0; i < 4; ++i) {
      const u128 sum = (u128)x[i] + C_L[i] + c;
      x[i] = (unsigned long long)sum;
      c = (unsigned long long)(sum >> 64);
    }
  }
  for (int i = 0; i < 4; ++i) r[i] = x[i];
}
// out = (little-endian words in[0..nw)) mod L, most significant word first
__device__ void sc_reduce_fast(uint32_t out[8], const uint32_t* in, int nw) {
  unsigned long long r[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (int i = nw - 1; i >= 0; --i) sc_step(r, in[i]);
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = (uint32_t)r[i];
    out[2 * i + 1] = (uint32_t)(r[i] >> 32);
  }
}

constexpr int VP = 16;     // proofs per workgroup
constexpr int VTRY = 12;   // hash-to-curve counters tried at once per proof (3 waves x 4 lanes)

__device__ __forceinline__ void st_ge(uint32_t* p, const ge& a) {
  st_fe(p, a.X); st_fe(p + 10, a.Y); st_fe(p + 20, a.Z); st_fe(p + 30, a.T);
}
__device__ __forceinline__ ge ld_ge(const uint32_t* p) { return ge{ld_fe(p), ld_fe(p + 10), ld_fe(p + 20), ld_fe(p + 30)}; }
__device__ __forceinline__ uint32_t le_word(const uint8_t* d, int i) {
  return (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) | ((uint32_t)d[4 * i + 3] << 24);
}

}  // namespace

// keys: [nkeys][24] words = x (clamped secret, 8 LE words), prefix (8), pk encoding (8);
// key_idx / alpha_idx: [n]; alphas: [nalpha][alpha_len] bytes; btab: [512][32] words;
// scratch: [n][320] words (the table of H of each proof); pi: [n][80] bytes; beta: [n][64] or null.
// Grid: ceil(n / 16) workgroups of 192 threads (3 waves); thread (wave w, lane l) works on proof
// 16 * blockIdx.x + (l & 15) with sub-lane q = l >> 4.
extern "C" __global__ void __launch_bounds__(192) k_vrf_prove(const uint32_t* __restrict__ keys,
                                                             const int* __restrict__ key_idx,
                                                             const uint8_t* __restrict__ alphas,
                                                             const int* __restrict__ alpha_idx, int alpha_len, int n,
                                                             const uint32_t* __restrict__ btab, uint32_t* scratch,
                                                             uint8_t* __restrict__ pi, uint8_t* __restrict__ beta,
                                                             int urgent) {
  // a batch of rounds' proofs nothing reads fills the issue slots the round's kernels leave (priority 0); the
  // run's final flush is what the run's end waits for (urgent: highest priority -- at 0 or 1 it ran ~2x
  // longer under the share MSMs, drain 0.9 -> 1.9 ms)
  if (urgent) BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  __shared__ int s_ok[VTRY][VP];          // phase 1: counter j of proof p decoded
  __shared__ int s_win[VP];               // the winning counter slot (-1: none yet)
  __shared__ uint32_t s_h[VP][20];        // decoded H (affine x, y) of the winner
  __shared__ uint32_t s_k[VP][8];         // nonce k
  __shared__ uint32_t s_hstr[VP][8];      // encode(8 H)
  __shared__ uint32_t s_gamma[VP][40];    // Gamma (wave 0)
  __shared__ uint32_t s_v[VP][40];        // V (wave 1)
  __shared__ uint32_t s_u[4][VP][40];     // U partial sums over 16 windows each (wave 2)
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int p = l & 15, q = l >> 4;
  const int t = blockIdx.x * VP + p;
  const bool valid = t < n;
  const int tt = valid ? t : 0;
  const uint32_t* key = keys + (long long)key_idx[tt] * 24;
  const uint8_t* alpha = alphas + (long long)alpha_idx[tt] * alpha_len;
  uint32_t pk[8];
  for (int i = 0; i < 8; ++i) pk[i] = key[16 + i];
  const fe d = fe_const(C_D), d2 = fe_const(C_D2);
  // ---------------- phase 1: H = encode_to_curve_try_and_increment(pk, alpha), 12 counters at once
  const int slot = w * 4 + q;
  if (threadIdx.x < VP) s_win[threadIdx.x] = -1;
  for (int base = 0; base < 256; base += VTRY) {
    const int ctr = base + slot;
    ge cand;
    bool ok = false;
    __syncthreads();
    if (valid && s_win[p] < 0 && ctr < 256) {
      Sha512 sh;
      sha_init(sh);
      sha_byte(sh, SUITE);
      sha_byte(sh, 0x01);
      sha_words(sh, pk, 8);
      sha_bytes(sh, alpha, alpha_len);
      sha_byte(sh, (uint8_t)ctr);
      sha_byte(sh, 0x00);
      uint8_t dig[64];
      sha_final(sh, dig);
      ok = ge_frombytes(cand, dig, d);
    }
    s_ok[slot][p] = ok ? 1 : 0;
    __syncthreads();
    if (ok && s_win[p] < 0) {
      int first = slot;
      for (int j = 0; j < slot; ++j)
        if (s_ok[j][p]) { first = j; break; }
      if (first == slot) {   // the smallest decoding counter of this proof: publish H
        st_fe(&s_h[p][0], cand.X);
        st_fe(&s_h[p][10], cand.Y);
      }
    }
    __syncthreads();
    if (threadIdx.x < VP) {
      int first = -1;
      for (int j = 0; j < VTRY && first < 0; ++j)
        if (s_ok[j][threadIdx.x]) first = j;
      if (first >= 0 && s_win[threadIdx.x] < 0) s_win[threadIdx.x] = base + first;
    }
    __syncthreads();
    const int pending = (threadIdx.x < VP && blockIdx.x * VP + threadIdx.x < n && s_win[threadIdx.x] < 0) ? 1 : 0;
    if (!__syncthreads_or(pending)) break;
  }
  const bool have = valid && s_win[p] >= 0;   // probability 2^-256 of no valid counter: the host marks
  //                                             an all-zero proof as failed
  ge H;
  if (have) {
    const fe hx = ld_fe(&s_h[p][0]), hy = ld_fe(&s_h[p][10]);
    H = ge{hx, hy, fe_small(1), fe_mul(hx, hy)};
  }
  uint32_t* tbl = scratch + (long long)tt * 320;
  // ---------------- phase 2: the table of 8H (wave 0), the nonce (wave 1)
  if (have && q == 0 && w <= 1) {
    H = ge_dbl(ge_dbl(ge_dbl(H, false), false), true);   // cofactor 8
    if (w == 0) {
      const gc c1 = ge_cache(H, d2);
      st_gc(tbl, c1);
      ge acc = ge_dbl(H, true);
      st_gc(tbl + 40, ge_cache(acc, d2));
#pragma unroll 1
      for (int i = 2; i < 8; ++i) {
        acc = ge_add_cached(acc, c1);
        st_gc(tbl + 40 * i, ge_cache(acc, d2));
      }
    } else {
      const fe hzi = fe_invert(H.Z);
      uint32_t hstr[8];
      enc_affine(hstr, fe_mul(H.X, hzi), fe_mul(H.Y, hzi));
      Sha512 sh;
      sha_init(sh);
      uint32_t prefix[8];
      for (int i = 0; i < 8; ++i) prefix[i] = key[8 + i];
      sha_words(sh, prefix, 8);
      sha_words(sh, hstr, 8);
      uint8_t dig[64];
      sha_final(sh, dig);
      uint32_t dw[16];
      for (int i = 0; i < 16; ++i) dw[i] = le_word(dig, i);
      uint32_t k[8];
      sc_reduce_fast(k, dw, 16);
      for (int i = 0; i < 8; ++i) {
        s_k[p][i] = k[i];
        s_hstr[p][i] = hstr[i];
      }
    }
  }
  __syncthreads();   // the table (global, workgroup-visible after the barrier) and k are ready
  // ---------------- phase 3: Gamma = x H (wave 0) | V = k H (wave 1) | U = k B (wave 2, 4 lanes per proof)
  if (have && w == 0 && q == 0) {
    uint32_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = key[i];
    st_ge(&s_gamma[p][0], ge_mul_tbl(tbl, x));
  } else if (have && w == 1 && q == 0) {
    uint32_t k[8];
    for (int i = 0; i < 8; ++i) k[i] = s_k[p][i];
    st_ge(&s_v[p][0], ge_mul_tbl(tbl, k));
  } else if (have && w == 2) {
    uint32_t k[8];
    for (int i = 0; i < 8; ++i) k[i] = s_k[p][i];
    int8_t e[64];
    signed_digits(e, k);
    ge r = ge_identity();
#pragma unroll 1
    for (int wi = 16 * q; wi < 16 * q + 16; ++wi) {
      const int dg = e[wi];
      if (dg > 0) r = ge_add_cached(r, ld_btab(btab, wi * 8 + dg - 1));
      else if (dg < 0) r = ge_add_cached(r, gc_neg(ld_btab(btab, wi * 8 - dg - 1)));
    }
    st_ge(&s_u[q][p][0], r);
  }
  __syncthreads();
  // ---------------- phase 4: encodings, challenge, s (wave 0, one lane per proof)
  if (!(have && w == 0 && q == 0)) return;
  const ge Gamma = ld_ge(&s_gamma[p][0]);
  const ge V = ld_ge(&s_v[p][0]);
  ge U = ld_ge(&s_u[0][p][0]);
#pragma unroll 1
  for (int j = 1; j < 4; ++j) U = ge_add_cached(U, ge_cache(ld_ge(&s_u[j][p][0]), d2));
  uint32_t k[8], hstr[8], x[8];
  for (int i = 0; i < 8; ++i) {
    k[i] = s_k[p][i];
    hstr[i] = s_hstr[p][i];
    x[i] = key[i];
  }
  const fe zgu = fe_mul(Gamma.Z, U.Z);
  const fe inv = fe_invert(fe_mul(zgu, V.Z));
  const fe ziV = fe_mul(inv, zgu);
  const fe inv2 = fe_mul(inv, V.Z);          // 1 / (Zg Zu)
  const fe ziU = fe_mul(inv2, Gamma.Z);
  const fe ziG = fe_mul(inv2, U.Z);
  uint32_t eg[8], eu[8], ev[8];
  enc_affine(eg, fe_mul(Gamma.X, ziG), fe_mul(Gamma.Y, ziG));
  enc_affine(eu, fe_mul(U.X, ziU), fe_mul(U.Y, ziU));
  enc_affine(ev, fe_mul(V.X, ziV), fe_mul(V.Y, ziV));
  // c = SHA512(suite || 0x02 || Y || H || Gamma || U || V || 0x00)[0..16]
  uint8_t cdig[64];
  {
    Sha512 sh;
    sha_init(sh);
    sha_byte(sh, SUITE);
    sha_byte(sh, 0x02);
    sha_words(sh, pk, 8);
    sha_words(sh, hstr, 8);
    sha_words(sh, eg, 8);
    sha_words(sh, eu, 8);
    sha_words(sh, ev, 8);
    sha_byte(sh, 0x00);
    sha_final(sh, cdig);
  }
  // s = (k + c x) mod L: 128 x 256-bit product plus k
  uint32_t cw[4];
  for (int i = 0; i < 4; ++i) cw[i] = le_word(cdig, i);
  uint32_t prod[13];
  for (int i = 0; i < 13; ++i) prod[i] = 0;
  for (int i = 0; i < 4; ++i) {
    unsigned long long carry = 0;
    for (int j = 0; j < 8; ++j) {
      const unsigned long long v = (unsigned long long)cw[i] * x[j] + prod[i + j] + carry;
      prod[i + j] = (uint32_t)v;
      carry = v >> 32;
    }
    for (int j = i + 8; carry && j < 13; ++j) {
      const unsigned long long v = (unsigned long long)prod[j] + carry;
      prod[j] = (uint32_t)v;
      carry = v >> 32;
    }
  }
  {
    unsigned long long carry = 0;
    for (int i = 0; i < 13; ++i) {
      const unsigned long long v = (unsigned long long)prod[i] + (i < 8 ? k[i] : 0u) + carry;
      prod[i] = (uint32_t)v;
      carry = v >> 32;
    }
  }
  uint32_t sc[8];
  sc_reduce_fast(sc, prod, 13);
  // pi = Gamma (32) || c (16) || s (32)
  uint8_t* o = pi + (long long)t * 80;
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 4; ++b) o[4 * i + b] = (uint8_t)(eg[i] >> (8 * b));
  for (int i = 0; i < 16; ++i) o[32 + i] = cdig[i];
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 4; ++b) o[48 + 4 * i + b] = (uint8_t)(sc[i] >> (8 * b));
  if (beta != nullptr) {   // beta = SHA512(suite || 0x03 || encode(8 Gamma) || 0x00)
    const ge G8 = ge_dbl(ge_dbl(ge_dbl(Gamma, false), false), true);
    const fe zi = fe_invert(G8.Z);
    uint32_t e8[8];
    enc_affine(e8, fe_mul(G8.X, zi), fe_mul(G8.Y, zi));
    Sha512 sh;
    sha_init(sh);
    sha_byte(sh, SUITE);
    sha_byte(sh, 0x03);
    sha_words(sh, e8, 8);
    sha_byte(sh, 0x00);
    sha_final(sh, beta + (long long)t * 64);
  }
}

// urgent != 0: the run's end waits for these proofs (highest wave priority)
extern "C" int bsc_vrf_prove_p(const uint32_t* keys, const int* key_idx, const uint8_t* alphas, const int* alpha_idx,
                               int alpha_len, int n, const uint32_t* btab, uint32_t* scratch, uint8_t* pi,
                               uint8_t* beta, int urgent, void* stream) {
  if (n <= 0) return 0;
  if (alpha_len < 0 || alpha_len > 1024) return -1;
  hipLaunchKernelGGL(k_vrf_prove, dim3((n + VP - 1) / VP), dim3(192), 0, (hipStream_t)stream, keys, key_idx, alphas,
                     alpha_idx, alpha_len, n, btab, scratch, pi, beta, urgent);
  return (int)hipGetLastError();
}

extern "C" int bsc_vrf_prove(const uint32_t* keys, const int* key_idx, const uint8_t* alphas, const int* alpha_idx,
                             int alpha_len, int n, const uint32_t* btab, uint32_t* scratch, uint8_t* pi, uint8_t* beta,
                             void* stream) {
  return bsc_vrf_prove_p(keys, key_idx, alphas, alpha_idx, alpha_len, n, btab, scratch, pi, beta, 0, stream);
}
