// Verifiable random function over Edwards25519.
//
// The reference draws committee roles from a coniks-go Edwards25519 VRF
// (DistSys/vrf.go:3-5,16-32; the library is fetched by `go get`, not vendored).  Its exact byte
// format cannot be reproduced offline, so this runtime implements the standardised
// ECVRF-EDWARDS25519-SHA512-TAI construction (RFC 9381): an Edwards25519 VRF with the same
// properties (uniqueness, pseudorandomness, public verifiability), 80-byte proofs and a
// 64-byte output.  Lottery code consumes only the output bytes, exactly like
// getVRFNoisers (DistSys/vrf.go:54-100).
#pragma once
#include <memory>

#include "common.hpp"

namespace bsc {

struct VrfKey {
  Bytes seed;        // 32-byte secret seed
  Bytes pk;          // 32-byte encoded public key
  uint8_t x[32];     // clamped secret scalar (SHA-512(seed)[0:32])
  uint8_t prefix[32];  // nonce prefix (SHA-512(seed)[32:64])
  static VrfKey from_seed(const Bytes& seed32);
  // process-wide cache: keys are derived once per seed (peers prove every round)
  static const VrfKey& cached(const Bytes& seed32);
};

// Returns (beta = 64-byte output, pi = 80-byte proof).
std::pair<Bytes, Bytes> vrf_prove(const VrfKey& key, const Bytes& alpha);

// The same proof in two phases.  The output beta needs only H = encode_to_curve(pk, alpha) and
// Gamma = x*H -- half of the scalar multiplications -- so a caller that consumes beta (the noiser
// lottery) can proceed while the proof itself (k*B, k*H, challenge, response) is finished.
struct VrfStage {
  std::shared_ptr<void> st;
};
Bytes vrf_output(const VrfKey& key, const Bytes& alpha, VrfStage* stage);
Bytes vrf_finish(const VrfKey& key, const VrfStage& stage);
// The output alone (no proof, no encoding of H): the noiser lottery's input when the proofs are
// produced elsewhere (kernels/vrf.hip).
Bytes vrf_beta(const VrfKey& key, const Bytes& alpha);
// vrf_beta of n keys (same alpha) eight at a time on AVX-512 IFMA lanes (vrf_ifma.cpp); CPUs without IFMA
// (vrf_beta_batch_supported() false) take vrf_beta per key.  out: n outputs.
bool vrf_beta_batch_supported();
void vrf_beta_batch(const VrfKey* const* keys, int n, const Bytes& alpha, Bytes* out);
// (beta, pi) of n keys (same alpha), the variable- and fixed-base multiplications eight at a time on AVX-512
// IFMA lanes; byte-identical to vrf_prove (which CPUs without IFMA take per key).
void vrf_prove_batch(const VrfKey* const* keys, int n, const Bytes& alpha, Bytes* beta, Bytes* pi);
// The fixed-base table of B (64 signed radix-16 windows x 8 multiples, cached form) as 512 x 4
// canonical 32-byte field encodings (Y+X, Y-X, 2Z, 2dT): the device prover's k*B table.
Bytes vrf_base_table_bytes();
// Returns true and fills beta on success.
bool vrf_verify(const Bytes& pk, const Bytes& alpha, const Bytes& pi, Bytes* beta);
Bytes vrf_proof_to_hash(const Bytes& pi);

// Plain Ed25519 public-key derivation (RFC 8032), exposed for tests.
Bytes ed25519_public_from_seed(const Bytes& seed32);

}  // namespace bsc
