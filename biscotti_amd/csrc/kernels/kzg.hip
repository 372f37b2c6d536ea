// Batched KZG evaluation audit (K13): verifySecret (DistSys/kyber.go:650-673) for every
// (chunk k, share point j) of a round's aggregate in ONE pairing-product check.
//
// The reference's check of one share is
//     e(C_k, g2_0) == e(W_kj, g2_1 - x_j G2) * e(B_k, g2_0)^y_kj
// (B_k = G1 in the reference's literal form, PK[poly*k] for a chunk-consistent check: quirk Q9).
// With independent random 64-bit weights r_kj all of them hold (up to a 2^-64 soundness error)
// iff
//     e(L1, g2_0) * e(-A, g2_1) * e(L2, G2) == 1,
//     L1 = sum_k (R_k C_k - Z_k B_k),  R_k = sum_j r_kj,  Z_k = sum_j r_kj y_kj  (exact, 192-bit),
//     A  = sum_kj r_kj W_kj,           L2 = sum_kj x_j r_kj W_kj.
// The G1 side -- nch*npts + 2*nch variable-base scalar multiplications and their sum -- is this
// file; the three-pairing product (fixed, prepared G2 points) is host work on a native thread
// (runtime/pairing.cpp), overlapped with the next round.
//
// MI355X mapping: one thread per scalar multiplication, 64-thread blocks (one wave, ~280 blocks
// for the MNIST aggregate so every CU gets work), binary double-and-add over the scalar's actual
// bit length (no table: the bases change every round), then a wave-level LDS tree of Jacobian
// additions per output and a one-block second pass over the block partials.  Scalars are
// shifted in registers (no dynamically indexed private arrays, so nothing spills to scratch).
#include <hip/hip_runtime.h>

#include "bn256_dev.h"

using namespace bn;

namespace {

constexpr int KZ_THREADS = 64;

// r = splitmix64(seed + (idx + 1) * golden) | 1 -- the host oracle (bindings.cpp kzg_r) matches
__device__ __forceinline__ unsigned long long kzg_r(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (z ^ (z >> 31)) | 1ull;
}

// dbl-2009-l, force-inlined here (bn::jac_dbl is a call: its frame would live in scratch)
__device__ __forceinline__ jac kz_dbl(const jac& p) {
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
  return r;   // infinity (z = 0) stays infinity: z' = 2 y z = 0
}

// k * P for a 192-bit unsigned k = (k2:k1:k0), left to right over its bit length
__device__ __forceinline__ jac jac_mul_192(const jac& p, unsigned long long k0, unsigned long long k1, unsigned long long k2) {
  int nbits;
  if (k2) nbits = 192 - __clzll(k2);
  else if (k1) nbits = 128 - __clzll(k1);
  else if (k0) nbits = 64 - __clzll(k0);
  else return jac_inf();
  // left-align the top bit at position 191
  int sh = 192 - nbits;
  while (sh >= 64) { k2 = k1; k1 = k0; k0 = 0; sh -= 64; }
  if (sh) {
    k2 = (k2 << sh) | (k1 >> (64 - sh));
    k1 = (k1 << sh) | (k0 >> (64 - sh));
    k0 <<= sh;
  }
  jac acc = p;   // the top bit
  k2 = (k2 << 1) | (k1 >> 63); k1 = (k1 << 1) | (k0 >> 63); k0 <<= 1;
  for (int b = 1; b < nbits; ++b) {
    acc = kz_dbl(acc);
    if (k2 >> 63) acc = jac_add(acc, p);
    k2 = (k2 << 1) | (k1 >> 63); k1 = (k1 << 1) | (k0 >> 63); k0 <<= 1;
  }
  return acc;
}

// same with an affine base (mixed additions: 11 products instead of 16)
__device__ __forceinline__ jac aff_mul_192(const aff& q, unsigned long long k0, unsigned long long k1, unsigned long long k2) {
  if (aff_is_inf(q)) return jac_inf();
  int nbits;
  if (k2) nbits = 192 - __clzll(k2);
  else if (k1) nbits = 128 - __clzll(k1);
  else if (k0) nbits = 64 - __clzll(k0);
  else return jac_inf();
  int sh = 192 - nbits;
  while (sh >= 64) { k2 = k1; k1 = k0; k0 = 0; sh -= 64; }
  if (sh) {
    k2 = (k2 << sh) | (k1 >> (64 - sh));
    k1 = (k1 << sh) | (k0 >> (64 - sh));
    k0 <<= sh;
  }
  jac acc;
  acc.x = q.x;
  acc.y = q.y;
  acc.z = fp_one();
  k2 = (k2 << 1) | (k1 >> 63); k1 = (k1 << 1) | (k0 >> 63); k0 <<= 1;
  for (int b = 1; b < nbits; ++b) {
    acc = kz_dbl(acc);
    if (k2 >> 63) acc = jac_add_aff(acc, q);
    k2 = (k2 << 1) | (k1 >> 63); k1 = (k1 << 1) | (k0 >> 63); k0 <<= 1;
  }
  return acc;
}

// sum of one Jacobian point per lane of the block, result valid in lane 0
__device__ __forceinline__ jac block_sum(jac v, uint32_t* lds) {
  const int t = threadIdx.x;
  for (int s = KZ_THREADS / 2; s > 0; s >>= 1) {
    if (t >= s && t < 2 * s) st_jac(lds + (t - s) * 24, v);
    __syncthreads();
    if (t < s) v = jac_add(v, ld_jac(lds + t * 24));
    __syncthreads();
  }
  return v;
}

}  // namespace

// Threads [0, nch*npts): witness terms of (k, j) -> A += r W, L2 += x_j r W.
// Threads [nch*npts, +nch): R_k C_k -> L1.   Threads [nch*npts + nch, +nch): -Z_k B_k -> L1.
// wsum row of (k, j): (j / spm) * nch * spm + k * spm + j % spm (the miners' witness sums as the
// engine lays them out: contributing-miner-major, then chunk, then the miner's share slots).
// partial: [gridDim.x][3][24] Jacobian (L1, A, L2).
extern "C" __global__ void __launch_bounds__(KZ_THREADS) k_kzg_rlc(
    const uint32_t* __restrict__ csum, const uint32_t* __restrict__ wsum, const long long* __restrict__ ys,
    const int* __restrict__ xs, int nch, int npts, int spm, const uint32_t* __restrict__ bases, int base_stride,
    int nch_round, unsigned long long seed, uint32_t* __restrict__ partial) {
  __shared__ uint32_t lds[KZ_THREADS * 24];
  const long long g = (long long)blockIdx.x * KZ_THREADS + threadIdx.x;
  const long long nw = (long long)nch * npts;
  jac l1 = jac_inf(), a = jac_inf(), l2 = jac_inf();
  if (g < nw) {
    const int k = (int)(g / npts), j = (int)(g % npts);
    const unsigned long long r = kzg_r(seed, (unsigned long long)g);
    const long long row = (long long)(j / spm) * nch * spm + (long long)k * spm + j % spm;
    const jac w = ld_jac(wsum + row * 24);
    a = jac_mul_192(w, r, 0, 0);
    const int x = xs[(long long)(k / nch_round) * npts + j];
    const unsigned ax = x < 0 ? unsigned(-x) : unsigned(x);
    l2 = jac_mul_192(a, ax, 0, 0);
    if (x < 0) l2 = jac_neg(l2);
  } else if (g < nw + nch) {
    const int k = (int)(g - nw);
    unsigned long long lo = 0, hi = 0;
    for (int j = 0; j < npts; ++j) {
      const unsigned long long r = kzg_r(seed, (unsigned long long)k * npts + j);
      lo += r;
      hi += lo < r;
    }
    l1 = jac_mul_192(ld_jac(csum + (long long)k * 24), lo, hi, 0);
  } else if (g < nw + 2 * nch) {
    const int k = (int)(g - nw - nch);
    // Z = sum_j r_kj * y_kj, two's complement over 192 bits
    unsigned long long z0 = 0, z1 = 0, z2 = 0;
    for (int j = 0; j < npts; ++j) {
      const unsigned long long r = kzg_r(seed, (unsigned long long)k * npts + j);
      const long long y = ys[(long long)k * npts + j];
      const unsigned long long m = y < 0 ? 0ull - (unsigned long long)y : (unsigned long long)y;
      unsigned long long p0 = r * m, p1 = __umul64hi(r, m), p2 = 0;
      if (y < 0) {   // negate the 192-bit product
        p0 = ~p0; p1 = ~p1; p2 = ~0ull;
        p0 += 1;
        const unsigned long long c0 = p0 == 0;
        p1 += c0;
        p2 += (c0 && p1 == 0);
      }
      z0 += p0;
      const unsigned long long c0 = z0 < p0;
      const unsigned long long t1 = z1 + p1;
      const unsigned long long c1 = t1 < z1;
      z1 = t1 + c0;
      const unsigned long long c1b = z1 < c0;
      z2 += p2 + c1 + c1b;
    }
    const bool neg = z2 >> 63;
    if (neg) {
      z0 = ~z0; z1 = ~z1; z2 = ~z2;
      z0 += 1;
      const unsigned long long c0 = z0 == 0;
      z1 += c0;
      z2 += (c0 && z1 == 0);
    }
    const aff b = ld_aff(bases + (long long)(k % nch_round) * base_stride * 16);
    l1 = aff_mul_192(b, z0, z1, z2);
    if (!neg) l1 = jac_neg(l1);   // the term is -Z_k B_k
  }
  l1 = block_sum(l1, lds);
  a = block_sum(a, lds);
  l2 = block_sum(l2, lds);
  if (threadIdx.x == 0) {
    uint32_t* o = partial + (long long)blockIdx.x * 72;
    st_jac(o, l1);
    st_jac(o + 24, a);
    st_jac(o + 48, l2);
  }
}

// out[3][24] = sum over the nb block partials (one block)
extern "C" __global__ void __launch_bounds__(KZ_THREADS) k_kzg_reduce(const uint32_t* __restrict__ partial, int nb,
                                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[KZ_THREADS * 24];
  for (int s = 0; s < 3; ++s) {
    jac v = jac_inf();
    for (int i = threadIdx.x; i < nb; i += KZ_THREADS) v = jac_add(v, ld_jac(partial + (long long)i * 72 + s * 24));
    v = block_sum(v, lds);
    if (threadIdx.x == 0) st_jac(out + s * 24, v);
  }
}

// csum [nch][24], wsum [nch*npts][24] (layout above), ys int64 [nch][npts], xs int32 [nch/nch_round][npts],
// bases affine [*][16] read at (k % nch_round) * base_stride (0: one base for every chunk, the
// literal check).  Several rounds' aggregates stack as nch = rounds * nch_round chunks (witness
// sums pre-permuted to (chunk, point) order, spm = npts): the sums then cover all of them,
// one random weight per (round, chunk, point), and one launch serves the whole batch;
// partial scratch [blocks][72] (blocks = bsc_kzg_blocks), out [3][24] = (L1, A, L2).
extern "C" int bsc_kzg_blocks(int nch, int npts) {
  const long long n = (long long)nch * npts + 2LL * nch;
  return (int)((n + KZ_THREADS - 1) / KZ_THREADS);
}

extern "C" int bsc_kzg_rlc(const uint32_t* csum, const uint32_t* wsum, const long long* ys, const int* xs, int nch,
                           int npts, int spm, const uint32_t* bases, int base_stride, int nch_round,
                           unsigned long long seed, uint32_t* partial, uint32_t* out, void* stream) {
  if (nch <= 0 || npts <= 0) return 0;
  if (spm <= 0 || npts % spm != 0 || base_stride < 0 || npts > 4096 || nch_round <= 0 || nch % nch_round != 0)
    return -1;
  const int nb = bsc_kzg_blocks(nch, npts);
  hipLaunchKernelGGL(k_kzg_rlc, dim3(nb), dim3(KZ_THREADS), 0, (hipStream_t)stream, csum, wsum, ys, xs, nch, npts, spm,
                     bases, base_stride, nch_round, seed, partial);
  hipLaunchKernelGGL(k_kzg_reduce, dim3(1), dim3(KZ_THREADS), 0, (hipStream_t)stream, partial, nb, out);
  return (int)hipGetLastError();
}
