// Hash primitives used by the ledger and the crypto layer:
//   SHA-256  -- block hash (reference DistSys/block.go:23-28) and lottery re-hash (DistSys/vrf.go:77,134)
//   SHA-512  -- Ed25519 / ECVRF (replacement for the coniks VRF, DistSys/vrf.go:3-5)
//   BLAKE2b  -- with full parameter block, and the BLAKE2Xb XOF that kyber's bn256 suite
//               exposes as suite.XOF (lib/dedis/kyber/xof/blake2xb/blake.go), used by the
//               Schnorr challenge (DistSys/kyber.go:928-933).
#pragma once
#include "common.hpp"

namespace bsc {

struct Sha256 {
  u32 h[8];
  u8 buf[64];
  size_t blen = 0;
  u64 total = 0;
  Sha256();
  void update(const u8* p, size_t n);
  void update(const Bytes& b) { update(b.data(), b.size()); }
  void final(u8 out[32]);
  static Bytes digest(const u8* p, size_t n);
  static Bytes digest(const Bytes& b) { return digest(b.data(), b.size()); }
 private:
  void block(const u8* p);
};

struct Sha512 {
  u64 h[8];
  u8 buf[128];
  size_t blen = 0;
  u64 total = 0;
  Sha512();
  void update(const u8* p, size_t n);
  void update(const Bytes& b) { update(b.data(), b.size()); }
  void final(u8 out[64]);
  static Bytes digest(const u8* p, size_t n);
  static Bytes digest(const Bytes& b) { return digest(b.data(), b.size()); }
 private:
  void block(const u8* p);
};

// BLAKE2b with an explicit 64-byte parameter block (RFC 7693 + BLAKE2 spec section 2.8).
struct Blake2b {
  u64 h[8];
  u64 t[2] = {0, 0};
  u8 buf[128];
  size_t blen = 0;
  size_t outlen = 64;
  // param: 64-byte parameter block; key may be empty.
  void init_param(const u8 param[64], const u8* key, size_t keylen);
  void init(size_t outlen, const u8* key = nullptr, size_t keylen = 0);
  void update(const u8* p, size_t n);
  void final(u8* out);  // writes outlen bytes
 private:
  void compress(const u8* blk, bool last);
};

// BLAKE2Xb XOF with unknown output length, as golang.org/x/crypto/blake2b.NewXOF(0, key)
// wrapped by kyber's blake2xb.New(seed): seed[0:64] is the key, seed[64:] is absorbed.
struct Blake2Xb {
  Blake2b root;
  u8 rootdig[64];
  u8 block[64];
  size_t offset = 0;
  u32 node_offset = 0;
  bool reading = false;
  explicit Blake2Xb(const Bytes& seed);
  void write(const u8* p, size_t n);
  void write(const Bytes& b) { write(b.data(), b.size()); }
  void read(u8* out, size_t n);
};

}  // namespace bsc
