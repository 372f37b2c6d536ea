// Secret sharing with polynomial commitments -- exact host reference.
//
// Reference (DistSys/kyber.go):
//   updateFloatToInt  :698-710  int64(x * 10^precision), truncation toward zero
//   makePolynomialMap :712-743  chunks [i, min(i+POLY_SIZE, d)) keyed by their stop index
//   createShareAndWitness :579-646  x = i - 10, y = p(x), witness = commit((p(X)-y)/(X-x))
//   extractMinerSecret :205-242  miner m gets shares [m*S, (m+1)*S), S = ceil(total/miners)
//   aggregateSecret    :244-287  sums of Y, witnesses and commitments
//   recoverSecret      :809-857  float64 QR least squares on a Vandermonde matrix, rounded
//
// This implementation is exact: y and the quotient are computed in integer arithmetic and the
// aggregate polynomial is recovered by Newton divided differences in 128-bit integers on ten
// nodes, then checked against every remaining share (a Byzantine/corrupt share is detected
// instead of being silently least-squared).  It equals the reference whenever the reference's
// float64 arithmetic is exact (|x^i * c_i| < 2^53), and is correct beyond that range too.
// The witness is computed as sum_j c_j * B_{j,x} with the fixed witness bases
//   B_{1,x} = PK[0],  B_{j+1,x} = x * B_{j,x} + PK[j]     (so sum_j c_j B_{j,x} == commit(q_x)),
// which is the same group element as the reference's commit(quotient).
#pragma once
#include "bn256.hpp"
#include "common.hpp"

namespace bsc {

std::vector<i64> quantize(const std::vector<double>& v, int precision);
std::vector<double> dequantize(const std::vector<i64>& v, int precision);
// chunk stop indices (sorted): e.g. d=25, poly=10 -> {10, 20, 25}
std::vector<i64> chunk_stops(i64 d, i64 poly);
std::vector<i64> share_xs(i64 total_shares);  // x = i - 10 (kyber.go:588, pointToHashVal)

i64 poly_eval(const i64* c, int n, i64 x);
// quotient of (p(X) - p(x)) / (X - x), length n-1 (synthetic division)
std::vector<i64> poly_quotient(const i64* c, int n, i64 x);

// Exact recovery of a degree-(deg) integer polynomial from (x, y) points.
// Returns false (and leaves out untouched) when the points are inconsistent.
bool recover_exact(const std::vector<i64>& xs, const std::vector<i64>& ys, int deg, std::vector<i64>* out);
// Reference-style float64 least squares (Householder QR), rounded to nearest.
std::vector<i64> recover_lstsq(const std::vector<i64>& xs, const std::vector<i64>& ys, int deg);

// Commitment key in Montgomery affine coordinates (what the device kernels consume).
G1 commit(const std::vector<i64>& coeffs, const std::vector<G1>& pk, size_t offset);

// Full host-side share generation for one update (CPU path / tests):
struct SharePackage {
  G1 commitment;                       // commit(all coefficients)
  std::vector<G1> chunk_commit;        // [nchunks]
  std::vector<i64> ys;                 // [nchunks * total_shares]
  std::vector<G1> witnesses;           // [nchunks * total_shares]
};
SharePackage make_shares(const std::vector<i64>& coeffs, const std::vector<G1>& pk, i64 poly,
                         i64 total_shares);
// Witness bases B_{j,x} for all chunks: [nchunks][total_shares][poly-1]
std::vector<G1> witness_bases(const std::vector<G1>& pk, i64 d, i64 poly, i64 total_shares);

}  // namespace bsc
