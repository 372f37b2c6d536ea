#include "hash.hpp"

#include <immintrin.h>

namespace bsc {

// ---------------------------------------------------------------- SHA-256
static const u32 K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static inline u32 rotr32(u32 x, int n) { return (x >> n) | (x << (32 - n)); }

Sha256::Sha256() {
  static const u32 iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(h, iv, sizeof(h));
}

// ---- SHA-NI (x86 SHA extensions): the ledger hashes ~75 KB of gob per block, 5-8x faster than
// the portable rounds.  Runtime-dispatched, so the portable path stays the fallback.
__attribute__((target("sha,sse4.1,ssse3"))) static void sha256_ni_blocks(u32 state[8], const u8* data, size_t nblocks) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i tmp = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&state[0]));
  __m128i st1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&state[4]));
  tmp = _mm_shuffle_epi32(tmp, 0xB1);          // CDAB
  st1 = _mm_shuffle_epi32(st1, 0x1B);          // EFGH
  __m128i st0 = _mm_alignr_epi8(tmp, st1, 8);  // ABEF
  st1 = _mm_blend_epi16(st1, tmp, 0xF0);       // CDGH
  for (; nblocks > 0; --nblocks, data += 64) {
    const __m128i abef = st0, cdgh = st1;
    __m128i w[16];
    for (int g = 0; g < 16; ++g) {
      if (g < 4) {
        w[g] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * g)), MASK);
      } else {
        __m128i t = _mm_add_epi32(_mm_sha256msg1_epu32(w[g - 4], w[g - 3]), _mm_alignr_epi8(w[g - 1], w[g - 2], 4));
        w[g] = _mm_sha256msg2_epu32(t, w[g - 1]);
      }
      __m128i msg = _mm_add_epi32(w[g], _mm_loadu_si128(reinterpret_cast<const __m128i*>(&K256[4 * g])));
      st1 = _mm_sha256rnds2_epu32(st1, st0, msg);
      msg = _mm_shuffle_epi32(msg, 0x0E);
      st0 = _mm_sha256rnds2_epu32(st0, st1, msg);
    }
    st0 = _mm_add_epi32(st0, abef);
    st1 = _mm_add_epi32(st1, cdgh);
  }
  tmp = _mm_shuffle_epi32(st0, 0x1B);        // FEBA
  st1 = _mm_shuffle_epi32(st1, 0xB1);        // DCHG
  st0 = _mm_blend_epi16(tmp, st1, 0xF0);     // DCBA
  st1 = _mm_alignr_epi8(st1, tmp, 8);        // HGFE
  _mm_storeu_si128(reinterpret_cast<__m128i*>(&state[0]), st0);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(&state[4]), st1);
}

static bool have_sha_ni() {
  static const bool ok = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
  }();
  return ok;
}

void Sha256::block(const u8* p) {
  if (have_sha_ni()) {
    sha256_ni_blocks(h, p, 1);
    return;
  }
  u32 w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (u32(p[4 * i]) << 24) | (u32(p[4 * i + 1]) << 16) | (u32(p[4 * i + 2]) << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    u32 s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    u32 s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    u32 S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    u32 ch = (e & f) ^ (~e & g);
    u32 t1 = hh + S1 + ch + K256[i] + w[i];
    u32 S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    u32 mj = (a & b) ^ (a & c) ^ (b & c);
    u32 t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void Sha256::update(const u8* p, size_t n) {
  total += n;
  if (blen > 0 && blen + n >= 64) {   // complete the buffered block first
    const size_t take = 64 - blen;
    memcpy(buf + blen, p, take);
    block(buf);
    blen = 0;
    p += take;
    n -= take;
  }
  if (blen == 0 && n >= 64 && have_sha_ni()) {  // then whole blocks straight from the input, in one call
    // (a block hash's input starts with 42 bytes of hash + timestamp, so the ~75 KB of gob behind them
    // would otherwise go block by block through the buffer: one state load / shuffle / store per 64 bytes)
    const size_t nb = n / 64;
    sha256_ni_blocks(h, p, nb);
    p += nb * 64;
    n -= nb * 64;
  }
  while (n > 0) {
    size_t take = std::min(n, size_t(64) - blen);
    memcpy(buf + blen, p, take);
    blen += take; p += take; n -= take;
    if (blen == 64) { block(buf); blen = 0; }
  }
}

void Sha256::final(u8 out[32]) {
  u64 bits = total * 8;
  u8 pad = 0x80;
  update(&pad, 1);
  u8 z = 0;
  while (blen != 56) update(&z, 1);
  u8 len[8];
  store_be64(len, bits);
  update(len, 8);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = u8(h[i] >> 24); out[4 * i + 1] = u8(h[i] >> 16);
    out[4 * i + 2] = u8(h[i] >> 8); out[4 * i + 3] = u8(h[i]);
  }
}

Bytes Sha256::digest(const u8* p, size_t n) {
  Sha256 s; s.update(p, n);
  Bytes o(32); s.final(o.data());
  return o;
}

// ---------------------------------------------------------------- SHA-512
static const u64 K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static inline u64 rotr64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }

Sha512::Sha512() {
  static const u64 iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(h, iv, sizeof(h));
}

void Sha512::block(const u8* p) {
  u64 w[80];
  for (int i = 0; i < 16; ++i) w[i] = load_be64(p + 8 * i);
  for (int i = 16; i < 80; ++i) {
    u64 s0 = rotr64(w[i - 15], 1) ^ rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    u64 s1 = rotr64(w[i - 2], 19) ^ rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  u64 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 80; ++i) {
    u64 S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    u64 ch = (e & f) ^ (~e & g);
    u64 t1 = hh + S1 + ch + K512[i] + w[i];
    u64 S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    u64 mj = (a & b) ^ (a & c) ^ (b & c);
    u64 t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void Sha512::update(const u8* p, size_t n) {
  total += n;
  while (n > 0) {
    size_t take = std::min(n, size_t(128) - blen);
    memcpy(buf + blen, p, take);
    blen += take; p += take; n -= take;
    if (blen == 128) { block(buf); blen = 0; }
  }
}

void Sha512::final(u8 out[64]) {
  u64 bits = total * 8;
  u8 pad = 0x80;
  update(&pad, 1);
  u8 z = 0;
  while (blen != 112) update(&z, 1);
  u8 len[16] = {0};
  store_be64(len + 8, bits);
  update(len, 16);
  for (int i = 0; i < 8; ++i) store_be64(out + 8 * i, h[i]);
}

Bytes Sha512::digest(const u8* p, size_t n) {
  Sha512 s; s.update(p, n);
  Bytes o(64); s.final(o.data());
  return o;
}

// ---------------------------------------------------------------- BLAKE2b
static const u64 B2IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const u8 SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

void Blake2b::init_param(const u8 param[64], const u8* key, size_t keylen) {
  for (int i = 0; i < 8; ++i) h[i] = B2IV[i] ^ load_le64(param + 8 * i);
  outlen = param[0];
  t[0] = t[1] = 0;
  blen = 0;
  if (keylen > 0) {
    u8 blk[128] = {0};
    memcpy(blk, key, keylen);
    update(blk, 128);
  }
}

void Blake2b::init(size_t olen, const u8* key, size_t keylen) {
  u8 p[64] = {0};
  p[0] = u8(olen); p[1] = u8(keylen); p[2] = 1; p[3] = 1;
  init_param(p, key, keylen);
}

void Blake2b::compress(const u8* blk, bool last) {
  u64 m[16], v[16];
  for (int i = 0; i < 16; ++i) m[i] = load_le64(blk + 8 * i);
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = B2IV[i]; }
  v[12] ^= t[0]; v[13] ^= t[1];
  if (last) v[14] = ~v[14];
#define B2G(a, b, c, d, x, y)                     \
  v[a] = v[a] + v[b] + x; v[d] = rotr64(v[d] ^ v[a], 32); \
  v[c] = v[c] + v[d];     v[b] = rotr64(v[b] ^ v[c], 24); \
  v[a] = v[a] + v[b] + y; v[d] = rotr64(v[d] ^ v[a], 16); \
  v[c] = v[c] + v[d];     v[b] = rotr64(v[b] ^ v[c], 63);
  for (int r = 0; r < 12; ++r) {
    const u8* s = SIGMA[r];
    B2G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    B2G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    B2G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    B2G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    B2G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    B2G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    B2G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    B2G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
#undef B2G
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

void Blake2b::update(const u8* p, size_t n) {
  while (n > 0) {
    if (blen == 128) {  // only compress a full buffer once more input arrives
      t[0] += 128;
      if (t[0] < 128) t[1]++;
      compress(buf, false);
      blen = 0;
    }
    size_t take = std::min(n, size_t(128) - blen);
    memcpy(buf + blen, p, take);
    blen += take; p += take; n -= take;
  }
}

void Blake2b::final(u8* out) {
  t[0] += blen;
  if (t[0] < blen) t[1]++;
  memset(buf + blen, 0, 128 - blen);
  compress(buf, true);
  u8 full[64];
  for (int i = 0; i < 8; ++i) store_le64(full + 8 * i, h[i]);
  memcpy(out, full, outlen);
}

// ---------------------------------------------------------------- BLAKE2Xb
static const u32 XOF_UNKNOWN = 0xFFFFFFFFu;

Blake2Xb::Blake2Xb(const Bytes& seed) {
  size_t k = std::min(seed.size(), size_t(64));
  u8 p[64] = {0};
  p[0] = 64; p[1] = u8(k); p[2] = 1; p[3] = 1;
  // XOF digest length (bytes 12..15) = 2^32-1 for "unknown length".
  p[12] = p[13] = p[14] = p[15] = 0xFF;
  root.init_param(p, seed.data(), k);
  if (seed.size() > 64) root.update(seed.data() + 64, seed.size() - 64);
}

void Blake2Xb::write(const u8* p, size_t n) {
  if (reading) fail("blake2xb: write after read");
  root.update(p, n);
}

void Blake2Xb::read(u8* out, size_t n) {
  if (!reading) {
    root.final(rootdig);
    reading = true;
    offset = 64;  // no buffered output yet
  }
  while (n > 0) {
    if (offset == 64) {
      u8 p[64] = {0};
      p[0] = 64;  // digest length of each output node (the stream length is unbounded)
      p[4] = 64;  // leaf length
      u32 no = node_offset++;
      p[8] = u8(no); p[9] = u8(no >> 8); p[10] = u8(no >> 16); p[11] = u8(no >> 24);
      p[12] = p[13] = p[14] = p[15] = 0xFF;  // XOF length
      p[17] = 64;  // inner length
      Blake2b b;
      b.init_param(p, nullptr, 0);
      b.update(rootdig, 64);
      b.final(block);
      offset = 0;
    }
    size_t take = std::min(n, size_t(64) - offset);
    memcpy(out, block + offset, take);
    out += take; n -= take; offset += take;
  }
  (void)XOF_UNKNOWN;
}

}  // namespace bsc
