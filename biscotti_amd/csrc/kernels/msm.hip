// Batched fixed-base multi-scalar multiplication on BN256 G1 for Biscotti's secure aggregation.
//
// Reference hot loop: createCommitment / createShareAndWitness (DistSys/kyber.go:533-646),
// ~180k Go big.Int double-and-add scalar multiplications per worker per round.
//
// MI355X design:
//  * Commitment-key points PK[i] and witness bases B_{j,x} (B_1=PK[0], B_{j+1}=x*B_j+PK[j]) are
//    fixed for the run, so each gets a signed-window table resident in HBM:
//        T[base][w][k-1] = k * 2^(8w) * base,  k = 1..128, w = 0..NW-1     (affine, Montgomery)
//    A scalar |c| < 2^64 is recoded into signed 8-bit digits (d in [-127, 128]); every non-zero
//    digit costs one mixed (Jacobian + affine) addition and one 64-byte table read.
//  * One thread per output point.  Threads of one (worker, chunk) group -- 21 witness lanes and
//    the chunk-commitment lane -- consume the SAME scalar c_j at step j, so digit control flow is
//    uniform inside a group, and the 21 witness lanes read 21 adjacent table points (1344 B
//    contiguous, table layout [chunk][j][w][k][x][16]).
//  * The share values y = p(x) (kyber.go:598-605, exact int64 Horner) are fused into the same
//    kernel.  Full-vector commitment = sum of chunk commitments (PK slices are consecutive).
//  * Blocks are remapped XCD-contiguously (chunk-major order), so one chunk's table lines are
//    pulled into a single XCD's L2.
#include <hip/hip_ext.h>

#include <vector>

#include "bn256_dev.h"
#define BSC_PRIO_FLAG bsc_prio_on_msm
#include "wave_prio.h"
BSC_PRIO_SETTER(bsc_wave_prio_msm)

using namespace bn;

namespace {

constexpr int TBL_ENTRIES = 128;  // entries of an 8-bit signed window

// Window plan of every fixed-base table: window 0 is B0 bits wide (2^(B0-1) entries: signed digits
// |d| <= 2^(B0-1)), windows 1..NW-1 are 8 bits (128 entries).  Per base the entries are laid out
// window 0 first, then 128 per further window; entry (w, |d|) of a base is entry index
//   w == 0 ? |d| - 1 : E0 + (w - 1) * 128 + |d| - 1,   E0 = 2^(B0-1).
// A wide first window turns the typical quantised update coefficient (|q| < 2^13) into ONE mixed
// addition instead of two: HBM is spent (tens of GB of tables) to halve the MSM arithmetic.
__device__ __forceinline__ int win_bits(int w, int B0) { return w ? 8 : B0; }
__device__ __forceinline__ int win_entry(int w, int ad, int E0) { return (w ? E0 + (w - 1) * TBL_ENTRIES : 0) + ad - 1; }
// next signed digit of width `bits` from (m, carry); digits lie in (-2^(bits-1), 2^(bits-1)]
__device__ __forceinline__ int recode(unsigned long long& m, int& carry, int bits) {
  int dg = (int)(m & ((1ull << bits) - 1)) + carry;
  m >>= bits;
  if (dg > (1 << (bits - 1))) {
    dg -= 1 << bits;
    carry = 1;
  } else {
    carry = 0;
  }
  return dg;
}

__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  // bijective: blocks that share an XCD (bid % 8) get a contiguous logical range
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = bid % 8, idx = bid / 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace

// ------------------------------------------------------------------ test kernels
extern "C" __global__ void __launch_bounds__(256) k_fp_mul(const uint32_t* a, const uint32_t* b, uint32_t* out, int n, int op) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp x = ld_fp(a + 8 * i), y = ld_fp(b + 8 * i), r;
  switch (op) {
    case 0: r = fp_mul(x, y); break;
    case 1: r = fp_add(x, y); break;
    case 2: r = fp_sub(x, y); break;
    case 3: r = fp_inv(x); break;
    default: r = fp_from_mont(x); break;
  }
  st_fp(out + 8 * i, r);
}

// op 0: jac(a)+jac(b) ; 1: jac(a)+aff(b) ; 2: dbl(jac(a)) ; 3: small mul a*k
extern "C" __global__ void __launch_bounds__(256) k_point_op(const uint32_t* a_aff, const uint32_t* b_aff, const int* ks, uint32_t* out,
                                      int n, int op) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  aff A = ld_aff(a_aff + 16 * i), Bq = ld_aff(b_aff + 16 * i);
  jac a = jac_inf();
  if (!aff_is_inf(A)) { a.x = A.x; a.y = A.y; a.z = fp_one(); }
  jac b = jac_inf();
  if (!aff_is_inf(Bq)) { b.x = Bq.x; b.y = Bq.y; b.z = fp_one(); }
  jac r;
  switch (op) {
    case 0: r = jac_add(jac_dbl(a), b); break;  // non-trivial Z on the left operand
    case 1: r = jac_add_aff(jac_dbl(a), Bq); break;
    case 2: r = jac_dbl(a); break;
    default: r = jac_mul_small(a, ks[i]); break;
  }
  st_jac(out + 24 * i, r);
}

// ------------------------------------------------------------------ witness bases
// out: Jacobian [nchunks][J][T][24], J = poly-1.  Short chunks leave trailing bases = infinity.
extern "C" __global__ void __launch_bounds__(128) k_witness_bases(const uint32_t* pk_aff, int d, int poly, int T, uint32_t* out) {
  const int nchunks = (d + poly - 1) / poly;
  const int J = poly - 1;
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nchunks * T) return;
  const int k = g / T, s = g % T;
  const int prev = k * poly;
  const int L = min(poly, d - prev);
  const int x = s - 10;  // kyber.go:588
  jac b = jac_inf();
  for (int j = 1; j <= J; ++j) {
    if (j < L) {
      aff pk = ld_aff(pk_aff + 16 * (prev + j - 1));
      if (j == 1) {
        b = jac_add_aff(jac_inf(), pk);
      } else {
        b = jac_add_aff(jac_mul_small(b, x), pk);
      }
      st_jac(out + 24 * (((size_t)k * J + (j - 1)) * T + s), b);
    } else {
      st_jac(out + 24 * (((size_t)k * J + (j - 1)) * T + s), jac_inf());
    }
  }
}

// ------------------------------------------------------------------ fixed-base tables
// Thread per (base b, run): a run is 128 consecutive entries of one window -- window 0 has
// E0/128 runs, every 8-bit window one.  Run r of window w holds (128 r + k) * 2^shift_w * base,
// k = 1..128, shift_0 = 0, shift_w = B0 + 8 (w - 1).  Base index b = outer * inner + in; entry e
// of base b is stored at table + 16 * (outer * s_outer + e * s_e + in * s_in).
// scratch: per thread 128 x 32 u32 (Jacobian + exclusive prefix product of the Z's).
extern "C" __global__ void __launch_bounds__(64) k_fb_table(const uint32_t* bases, int bases_are_jac, int b0, int nb,
                                                           int inner, int B0, int NW, long long s_outer,
                                                           long long s_e, long long s_in, uint32_t* table,
                                                           uint32_t* scratch) {
  const int E0 = 1 << (B0 - 1);
  const int R0 = E0 / TBL_ENTRIES;
  const int runs = R0 + NW - 1;
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)nb * runs) return;
  const int bl = (int)(g / runs), run = (int)(g % runs);
  const int b = b0 + bl;
  const int w = run < R0 ? 0 : run - R0 + 1;
  const int r = run < R0 ? run : 0;
  const int shift = w ? B0 + 8 * (w - 1) : 0;
  const int e0 = w ? E0 + (w - 1) * TBL_ENTRIES : r * TBL_ENTRIES;
  jac P;
  if (bases_are_jac) {
    P = ld_jac(bases + 24 * (size_t)b);
  } else {
    aff a = ld_aff(bases + 16 * (size_t)b);
    P = jac_add_aff(jac_inf(), a);
  }
  for (int i = 0; i < shift; ++i) P = jac_dbl(P);
  uint32_t* sc = scratch + (size_t)g * TBL_ENTRIES * 32;
  jac acc = r ? jac_mul_small(P, r * TBL_ENTRIES + 1) : P;
  fp prod = fp_one();
  for (int k = 0; k < TBL_ENTRIES; ++k) {
    st_jac(sc + 32 * k, acc);
    st_fp(sc + 32 * k + 24, prod);  // exclusive prefix product of the non-zero Z's before k
    if (!jac_is_inf(acc)) prod = fp_mul(prod, acc.z);
    acc = jac_add(acc, P);
  }
  fp inv = fp_inv(prod);  // Montgomery's trick: one inversion per run
  const int outer = b / inner, in = b % inner;
  uint32_t* dst0 = table + 16 * ((long long)outer * s_outer + (long long)e0 * s_e + (long long)in * s_in);
  for (int k = TBL_ENTRIES - 1; k >= 0; --k) {
    jac pt = ld_jac(sc + 32 * k);
    aff o;
    if (jac_is_inf(pt)) {
      o.x = fp_zero();
      o.y = fp_zero();
    } else {
      fp zi = fp_mul(inv, ld_fp(sc + 32 * k + 24));  // 1 / z_k
      inv = fp_mul(inv, pt.z);
      fp zi2 = fp_sqr(zi);
      o.x = fp_mul(pt.x, zi2);
      o.y = fp_mul(pt.y, fp_mul(zi2, zi));
    }
    st_aff(dst0 + 16 * ((long long)k * s_e), o);
  }
}

// ------------------------------------------------------------------ fused shares + commitments
// coeffs: int64 [*, d] (row stride d); rows: worker rows to process.
// tbl_pk: [d][PB][16]; tbl_wb: [nchunks][J][PB][T][16]; PB = E0 + (NW-1)*128 entries per base.
// out_pts: Jacobian [nrows][nchunks][S][24] with S = T+1 (slots 0..T-1 witnesses, slot T the chunk
// commitment) or S = 1 (commit_only == 1: chunk commitments only).  commit_only == 2: witnesses and
// share values only -- slot T is left untouched (the caller has the chunk commitments already), so a
// group is T lanes instead of T+1 and no wave runs the commitment lane's extra c_0 addition.
// out_y: int64 [nrows][nchunks][T].
// The row list comes from device memory (rows) or from the kernel's argument block (RowArg, <= ROWARG_MAX
// rows): the speculative MSM is launched the moment its rows are known, with no upload in front of it.
#define ROWARG_MAX 248
struct RowArg {
  int r[ROWARG_MAX];
};
struct RowsPtr {
  const int* p;
  __device__ __forceinline__ int operator[](int i) const { return p[i]; }
};
struct RowsArg {
  const RowArg* a;
  __device__ __forceinline__ int operator[](int i) const { return a->r[i]; }
};

template <class Rows>
__device__ __forceinline__ void shares_msm_body(const long long* coeffs, int d, Rows rows, int nrows,
                                                const uint32_t* tbl_pk, const uint32_t* tbl_wb, int poly, int T,
                                                int B0, int NW, int commit_only, const int* alive,
                                                const int* compact, int group_rows, uint32_t* out_pts,
                                                long long* out_y) {
  const int nchunks = (d + poly - 1) / poly;
  // the pre-step's commitment MSM (commit_only == 1) one class below the speculative MSM: both run side by side,
  // the speculative one gates the recovery and the commitments are read only at the block build; after the
  // fence fix this measured better (200 rounds: p50 0.711 vs 0.769 ms, profiles/r5/prio2; before it, worse)
  if (commit_only == 1) BSC_SET_PRIO(BSC_PRIO_AHEAD);
  else BSC_SET_PRIO(BSC_PRIO_SPEC);
  const int S = commit_only == 1 ? 1 : T + 1;   // output slots per (row, chunk)
  const int SL = commit_only == 2 ? T : S;      // lanes per (row, chunk)
  // compact (optional): [count, row...] -- only the listed rows are computed, packed densely over the
  // grid (a rejected row costs no SIMD lanes); the grid is sized for nrows, the surplus exits at once
  const int neff = compact != nullptr ? compact[0] : nrows;
  const long long total = (long long)neff * nchunks * SL;
  // group_rows G > 0: rows are taken G at a time in list order (the speculative rows arrive sorted
  // by their arrival at the leader), chunk-major inside a group, and the XCD remap is applied per
  // 64-block super-block -- so work proceeds through the row list in dispatch order (rows the
  // selection drops later are skipped when reached) while each XCD still shares a chunk's table
  // lines across the group's rows.  G = 0: one group of every row, remapped over the whole grid.
  int lb;
  if (group_rows > 0) {
    const int SB = 64;
    const int q = blockIdx.x / SB, j = blockIdx.x % SB;
    const int sbn = min(SB, (int)gridDim.x - q * SB);
    lb = q * SB + xcd_remap(j, sbn);
  } else {
    lb = xcd_remap(blockIdx.x, gridDim.x);
  }
  const long long g = (long long)lb * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const int G = group_rows > 0 ? min(group_rows, neff) : neff;
  const long long per_group = (long long)G * nchunks * SL;
  const int gq = (int)(g / per_group);
  const int r0 = gq * G, gr = min(G, neff - r0);
  const long long gg = g - (long long)gq * per_group;
  // chunk-major inside the group: consecutive groups of SL lanes share a chunk (and its table lines)
  const int slot = (int)(gg % SL);
  const long long grp = gg / SL;
  const int pos = r0 + (int)(grp % gr);
  const int r = compact != nullptr ? compact[1 + pos] : pos;
  const int k = (int)(grp / gr);
  // late cancellation of speculative work: rows the verifiers rejected (flag cleared by
  // k_set_alive on the critical-path stream while this kernel runs) are skipped from then on;
  // their outputs are never read.  A stale read only costs the work.
  if (alive != nullptr && __hip_atomic_load(alive + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  const int row = rows[r];
  const int prev = k * poly;
  const int L = min(poly, d - prev);
  const bool is_commit = commit_only == 1 || slot == T;
  const int J = poly - 1;
  const long long* c = coeffs + (size_t)row * d + prev;

  const int E0 = 1 << (B0 - 1);
  const size_t PB = (size_t)E0 + (size_t)(NW - 1) * TBL_ENTRIES;
  const size_t pk_base_stride = PB * 16;
  const size_t wb_j_stride = PB * T * 16;
  const uint32_t* wb_chunk = tbl_wb + (size_t)k * J * wb_j_stride;

  jac acc = jac_inf();
  // commitment uses c_0..c_{L-1} on PK[prev..]; witness uses c_1..c_{L-1} on B_{1..L-1, x}
  for (int j = is_commit ? 0 : 1; j < L; ++j) {
    const long long cj = c[j];
    if (cj == 0) continue;
    const bool neg = cj < 0;
    unsigned long long m = neg ? 0ull - (unsigned long long)cj : (unsigned long long)cj;
    const uint32_t* tb;
    size_t estride;
    if (is_commit) {
      tb = tbl_pk + (size_t)(prev + j) * pk_base_stride;
      estride = 16;
    } else {
      tb = wb_chunk + (size_t)(j - 1) * wb_j_stride + (size_t)slot * 16;
      estride = (size_t)T * 16;
    }
    int carry = 0;
    for (int w = 0; w < NW && (m != 0 || carry != 0); ++w) {
      const int dg = recode(m, carry, win_bits(w, B0));
      if (dg == 0) continue;
      const int ad = dg < 0 ? -dg : dg;
      aff q = ld_aff(tb + (size_t)win_entry(w, ad, E0) * estride);
      if ((dg < 0) != neg) q = aff_neg(q);
      acc = jac_add_aff(acc, q);
    }
  }
  const size_t o = ((size_t)r * nchunks + k) * S + slot;
  st_jac(out_pts + 24 * o, acc);
  if (!is_commit && out_y != nullptr) {
    // y = p(x) exact int64 Horner (kyber.go:598-605 evaluates the same value in float64)
    const long long x = slot - 10;
    unsigned long long y = 0;
    for (int j = L - 1; j >= 0; --j) y = y * (unsigned long long)x + (unsigned long long)c[j];
    out_y[((size_t)r * nchunks + k) * T + slot] = (long long)y;
  }
}

extern "C" __global__ void __launch_bounds__(256) k_shares_msm(
    const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk, const uint32_t* tbl_wb,
    int poly, int T, int B0, int NW, int commit_only, const int* alive, const int* compact, int group_rows,
    uint32_t* out_pts, long long* out_y) {
  shares_msm_body(coeffs, d, RowsPtr{rows}, nrows, tbl_pk, tbl_wb, poly, T, B0, NW, commit_only, alive, compact,
                  group_rows, out_pts, out_y);
}

extern "C" __global__ void __launch_bounds__(256) k_shares_msm_ka(
    const long long* coeffs, int d, RowArg rows, int nrows, const uint32_t* tbl_pk, const uint32_t* tbl_wb,
    int poly, int T, int B0, int NW, int commit_only, const int* alive, int group_rows, uint32_t* out_pts,
    long long* out_y) {
  shares_msm_body(coeffs, d, RowsArg{&rows}, nrows, tbl_pk, tbl_wb, poly, T, B0, NW, commit_only, alive, nullptr,
                  group_rows, out_pts, out_y);
}

// ------------------------------------------------------------------ full-vector commitments
// C_row = sum_i c_i PK[i] for whole rows (the commit phase: commitUpdate, kyber.go:533-559).
// One 256-thread block per (row, 1024-coefficient slab):
//   1. signed 8-bit digit decomposition of the slab into an LDS work list of NONZERO digits
//      (table entry index | sign bit) -- lanes holding different coefficients would otherwise
//      diverge on their different digit counts;
//   2. every lane consumes the list round-robin (uniform mixed additions, no divergence);
//   3. LDS tree over the 256 partial sums (the list's LDS is reused).
// out_partial: Jacobian [nrows][nslab][24]; bsc_commit_rows finishes with a per-row segment sum.
#define COMMIT_CB 1024
extern "C" __global__ void __launch_bounds__(256) k_commit_rows(const long long* coeffs, int d, const int* rows,
                                                               int nrows, const uint32_t* tbl_pk, int B0, int NW,
                                                               uint32_t* out_partial) {
  __shared__ uint32_t lds[9 * COMMIT_CB];  // >= 256 * 24 for the reduction
  __shared__ int cnt;
  const int nslab = (d + COMMIT_CB - 1) / COMMIT_CB;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int r = b / nslab, slab = b % nslab;
  if (r >= nrows) return;  // uniform per block
  const long long* c = coeffs + (size_t)rows[r] * d;
  const int c0 = slab * COMMIT_CB, c1 = min(d, c0 + COMMIT_CB);
  const int E0 = 1 << (B0 - 1);
  const size_t PB = (size_t)E0 + (size_t)(NW - 1) * TBL_ENTRIES;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (int i = c0 + (int)threadIdx.x; i < c1; i += 256) {
    const long long cj = c[i];
    if (cj == 0) continue;
    const bool neg = cj < 0;
    unsigned long long m = neg ? 0ull - (unsigned long long)cj : (unsigned long long)cj;
    int carry = 0;
    for (int w = 0; w < NW && (m != 0 || carry != 0); ++w) {
      const int dg = recode(m, carry, win_bits(w, B0));
      if (dg == 0) continue;
      const int ad = dg < 0 ? -dg : dg;
      uint32_t e = (uint32_t)((size_t)i * PB + win_entry(w, ad, E0));
      if ((dg < 0) != neg) e |= 0x80000000u;
      lds[atomicAdd(&cnt, 1)] = e;
    }
  }
  __syncthreads();
  const int n = cnt;
  jac acc = jac_inf();
  // software pipeline: the next table point is in flight while the current one is added
  int k = threadIdx.x;
  uint32_t e = k < n ? lds[k] : 0u;
  aff q = ld_aff(tbl_pk + (size_t)(e & 0x7FFFFFFFu) * 16);
  while (k < n) {
    const int kn = k + 256;
    const uint32_t en = kn < n ? lds[kn] : 0u;
    const aff qn = ld_aff(tbl_pk + (size_t)(en & 0x7FFFFFFFu) * 16);
    acc = jac_add_aff(acc, (e >> 31) ? aff_neg(q) : q);
    k = kn;
    e = en;
    q = qn;
  }
  __syncthreads();
  st_jac(lds + threadIdx.x * 24, acc);
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      st_jac(lds + threadIdx.x * 24, jac_add(ld_jac(lds + threadIdx.x * 24), ld_jac(lds + (threadIdx.x + s) * 24)));
    __syncthreads();
  }
  if (threadIdx.x == 0) st_jac(out_partial + 24 * (size_t)b, ld_jac(lds));
}

// ------------------------------------------------------------------ aggregate commitment audit
// verifyCommitment (kyber.go:564-577) applied to the secure aggregate: by additive homomorphism
// the miners' summed chunk commitments sum_w C_k(q_w) must equal the commitment of the recovered
// chunk C_k(sum_w q_w).  One 64-lane block per chunk: lane j < L adds c_j * PK[prev + j] from the
// fixed-base tables, an LDS tree sums the lanes, then lane m compares the result projectively
// (X1 Z2^2 == X2 Z1^2, Y1 Z2^3 == Y2 Z1^3: no inversion) with miner m's sum.
// coeffs: int64 [nch][poly] (recovered); csum: Jacobian [nm][nch][24]; ok: int32 [nm][nch].
__device__ __forceinline__ bool jac_equal(const jac& p, const jac& q) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  const fp z1s = fp_sqr(p.z), z2s = fp_sqr(q.z);
  if (!fp_eq(fp_mul(p.x, z2s), fp_mul(q.x, z1s))) return false;
  return fp_eq(fp_mul(p.y, fp_mul(z2s, q.z)), fp_mul(q.y, fp_mul(z1s, p.z)));
}

// affine + affine -> Jacobian (mmadd-2007-bl, Z1 = Z2 = 1: 4M + 2S), complete for the special cases
__device__ __forceinline__ jac aff_add_aff(const aff& p, const aff& q) {
  if (aff_is_inf(p)) return jac_add_aff(jac_inf(), q);
  if (aff_is_inf(q)) return jac_add_aff(jac_inf(), p);
  const fp h = fp_sub(q.x, p.x);
  fp r = fp_sub(q.y, p.y);
  if (fp_is_zero(h)) {
    if (fp_is_zero(r)) return jac_dbl(jac_add_aff(jac_inf(), p));
    return jac_inf();
  }
  const fp hh = fp_sqr(h);
  const fp i = fp_dbl(fp_dbl(hh));
  const fp j = fp_mul(h, i);
  r = fp_dbl(r);
  const fp v = fp_mul(p.x, i);
  jac o;
  o.x = fp_sub(fp_sub(fp_sub(fp_sqr(r), j), v), v);
  o.y = fp_sub(fp_mul(r, fp_sub(v, o.x)), fp_dbl(fp_mul(p.y, j)));
  o.z = fp_dbl(h);
  return o;
}

// One wave per chunk.  The check sits on the round's critical path (the host commits the block only
// after it), and it is a latency chain, so it is built to be short:
//   1. signed digits of every coefficient (one lane per coefficient);
//   2. the NONZERO digits (typically one per coefficient with the 14-bit first window) are compacted
//      into an LDS list, so ~10 points, not 64 lanes, enter the sum;
//   3. lane i adds points 2i and 2i+1 affine + affine (6 products instead of a Jacobian addition's
//      16), then a tree over the ceil(n/2) partial sums (log2 levels, not 6);
//   4. lane m < nm compares the total projectively with miner m's sum.
extern "C" __global__ void __launch_bounds__(64) k_chunk_check(const long long* coeffs, int d, int poly,
                                                              const uint32_t* tbl_pk, int B0, int NW,
                                                              const uint32_t* csum, int nm, int nch, int* ok,
                                                              int* h_ok, int low) {
  if (low) BSC_SET_PRIO(BSC_PRIO_AHEAD);   // bsc_set_side_prio: below the speculative MSM
  else BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  __shared__ uint32_t sh[64 * 24];
  __shared__ int dig[16][9];      // signed digit of (coefficient j, window w); NW <= 9 (bsc_chunk_check)
  __shared__ uint32_t items[16 * 9];   // nonzero digits: table entry | sign bit
  __shared__ int cnt;
  const int k = blockIdx.x, t = threadIdx.x;
  const int prev = k * poly, L = min(poly, d - prev);
  const int E0 = 1 << (B0 - 1);
  const size_t PB = (size_t)E0 + (size_t)(NW - 1) * TBL_ENTRIES;
  if (t == 0) cnt = 0;
  if (t < 16) {
    for (int w = 0; w < 9; ++w) dig[t][w] = 0;
    if (t < L) {
      const long long cj = coeffs[(size_t)k * poly + t];
      const bool neg = cj < 0;
      unsigned long long m = neg ? 0ull - (unsigned long long)cj : (unsigned long long)cj;
      int carry = 0;
      for (int w = 0; w < NW && (m != 0 || carry != 0); ++w) {
        const int dg = recode(m, carry, win_bits(w, B0));
        dig[t][w] = neg ? -dg : dg;
      }
    }
  }
  __syncthreads();
  for (int e = t; e < L * 9; e += 64) {
    const int j = e / 9, w = e % 9;
    const int dg = w < NW ? dig[j][w] : 0;
    if (dg == 0) continue;
    const int ad = dg < 0 ? -dg : dg;
    const uint32_t ent = (uint32_t)((size_t)(prev + j) * PB + win_entry(w, ad, E0));
    items[atomicAdd(&cnt, 1)] = ent | (dg < 0 ? 0x80000000u : 0u);
  }
  __syncthreads();
  const int n = cnt, m = (n + 1) / 2;
  jac v = jac_inf();
  if (t < m) {
    const uint32_t e1 = items[2 * t];
    aff q1 = ld_aff(tbl_pk + (size_t)(e1 & 0x7FFFFFFFu) * 16);
    if (e1 >> 31) q1 = aff_neg(q1);
    if (2 * t + 1 < n) {
      const uint32_t e2 = items[2 * t + 1];
      aff q2 = ld_aff(tbl_pk + (size_t)(e2 & 0x7FFFFFFFu) * 16);
      if (e2 >> 31) q2 = aff_neg(q2);
      v = aff_add_aff(q1, q2);
    } else {
      v = jac_add_aff(jac_inf(), q1);
    }
  }
  st_jac(sh + t * 24, v);
  __syncthreads();
  int p2 = 1;
  while (p2 < m) p2 <<= 1;
  for (int s = p2 >> 1; s > 0; s >>= 1) {
    if (t < s) st_jac(sh + t * 24, jac_add(ld_jac(sh + t * 24), ld_jac(sh + (t + s) * 24)));
    __syncthreads();
  }
  if (t < nm) {
    const int v = jac_equal(ld_jac(sh), ld_jac(csum + 24 * ((size_t)t * nch + k))) ? 1 : 0;
    ok[(size_t)t * nch + k] = v;
    // pinned host mirror: read after the kernel's completion event (its end-of-kernel release makes it visible;
    // no per-block system fence), no read-back copy
    if (h_ok != nullptr) h_ok[(size_t)t * nch + k] = v;
  }
}

// ------------------------------------------------------------------ reductions
// out[i] = sum_{r < nrows} pts[(rows[r] * ncols_in + cols[i]) * 24]   (cols == nullptr: cols[i] = i)
// One thread per output column; used for miner-side share aggregation (aggregateSecret).
extern "C" __global__ void __launch_bounds__(128) k_sum_rows(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols,
                                      int ncols, uint32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncols) return;
  const int col = cols ? cols[i] : i;
  jac acc = jac_inf();
  for (int r = 0; r < nrows; ++r) {
    const int row = rows ? rows[r] : r;
    acc = jac_add(acc, ld_jac(pts + 24 * ((size_t)row * ncols_in + col)));
  }
  st_jac(out + 24 * (size_t)i, acc);
}

// Two-level version: block = 32 columns x 8 row groups; each thread sums every 8th row of its
// column, then an LDS tree over the 8 partials.  8x the parallelism of k_sum_rows, and the column
// list may concatenate several miners' slots (one launch per rank).
// row_mask (optional, indexed by input row, or by position r in `rows` when mask_by_pos): rows whose
// flag is 0 are left out -- the device-side selection of the approved workers' shares, decided by the
// verification kernels on the GPU.
extern "C" __global__ void __launch_bounds__(256) k_sum_rows2(const uint32_t* pts, int ncols_in, const int* rows,
                                                             int nrows, const int* cols, int ncols,
                                                             const int* row_mask, int mask_by_pos, uint32_t* out) {
  if (mask_by_pos) BSC_SET_PRIO(BSC_PRIO_AHEAD);   // the early commitment sums; witness sums stay background
  // 16 columns x 16 row lanes per block: each lane's serial chain is nrows/16 additions, then a
  // 4-level LDS tree (the sums sit on the round's critical path: latency, not throughput, matters)
  __shared__ uint32_t sh[16][16][24];
  const int cx = threadIdx.x & 15, ry = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + cx;
  jac acc = jac_inf();
  if (i < ncols && ry < nrows) {
    const int col = cols ? cols[i] : i;
    // software pipeline: load row r + 16 while adding row r
    int row = rows ? rows[ry] : ry;
    jac cur = ld_jac(pts + 24 * ((size_t)row * ncols_in + col));
    for (int r = ry; r < nrows; r += 16) {
      const int rn = r + 16 < nrows ? r + 16 : r;
      const int rown = rows ? rows[rn] : rn;
      const jac nxt = ld_jac(pts + 24 * ((size_t)rown * ncols_in + col));
      if (row_mask == nullptr || row_mask[mask_by_pos ? r : row] != 0) acc = jac_add(acc, cur);
      cur = nxt;
      row = rown;
    }
  }
  st_jac(&sh[ry][cx][0], acc);
  __syncthreads();
  for (int s2 = 8; s2 > 0; s2 >>= 1) {
    if (ry < s2) st_jac(&sh[ry][cx][0], jac_add(ld_jac(&sh[ry][cx][0]), ld_jac(&sh[ry + s2][cx][0])));
    __syncthreads();
  }
  if (ry == 0 && i < ncols) st_jac(out + 24 * (size_t)i, ld_jac(&sh[0][cx][0]));
}

// Throughput form of the masked column sums, for sums nothing in the round waits for (the miners' witness sums:
// per rank, read only by the KZG audit when it is on): one lane per output column adds the kept rows in order.
// k_sum_rows2's 16-lane LDS tree buys latency with 15 more Jacobian additions per column -- ~30 % of the witness
// sums' VALU work, issued while the share MSMs (VALU-bound) run beside them.  Background priority (class 0).
extern "C" __global__ void __launch_bounds__(256) k_sum_cols_serial(const uint32_t* pts, int ncols_in, int nrows,
                                                                   const int* cols, int ncols, const int* row_mask,
                                                                   uint32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncols) return;
  const int col = cols != nullptr ? cols[i] : i;
  jac acc = jac_inf();
  bool any = false;
  for (int r = 0; r < nrows; ++r) {
    if (row_mask != nullptr && row_mask[r] == 0) continue;
    const jac p = ld_jac(pts + 24 * ((size_t)r * ncols_in + col));
    acc = any ? jac_add(acc, p) : p;
    any = true;
  }
  st_jac(out + 24 * (size_t)i, acc);
}

// Sum of a strided segment per group: out[g] = sum_{k<n} pts[(g*n + k)*stride + off], one block
// per group, LDS tree.  Used for the full commitment = sum of chunk commitments.
extern "C" __global__ void __launch_bounds__(256) k_segment_sum(const uint32_t* pts, int n, int stride, int off,
                                                               uint32_t* out, uint32_t* hout, int low) {
  // the full commitments: the round's block build waits for them (a latency chain) -- or, bsc_set_side_prio, below
  // the speculative MSM they run beside (the next block build is a round away)
  if (low) BSC_SET_PRIO(BSC_PRIO_AHEAD);
  else BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  __shared__ uint32_t sh[256 * 24];
  const int g = blockIdx.x;
  jac acc = jac_inf();
  for (int k = threadIdx.x; k < n; k += blockDim.x)
    acc = jac_add(acc, ld_jac(pts + 24 * ((size_t)(g * (size_t)n + k) * stride + off)));
  st_jac(sh + threadIdx.x * 24, acc);
  __syncthreads();
  // tree only over the lanes that hold partial sums (n is typically 8 slabs: 3 levels, not 8)
  int top = 1;
  while (top < n && top < (int)blockDim.x) top <<= 1;
  for (int s = top / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      jac a = ld_jac(sh + threadIdx.x * 24), b = ld_jac(sh + (threadIdx.x + s) * 24);
      st_jac(sh + threadIdx.x * 24, jac_add(a, b));
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const jac r = ld_jac(sh);
    st_jac(out + 24 * (size_t)g, r);
    // pinned host mirror (the commitments' read-back without a copy), read after the kernel's event
    if (hout != nullptr) st_jac(hout + 24 * (size_t)g, r);
  }
}

// Jacobian -> kyber marshal (64 B: big-endian affine x || y, Montgomery-decoded; infinity = 0s)
extern "C" __global__ void __launch_bounds__(64) k_marshal(const uint32_t* pts, int n, uint8_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  aff a = jac_to_aff(ld_jac(pts + 24 * (size_t)i));
  uint8_t* o = out + 64 * (size_t)i;
  if (aff_is_inf(a)) {
    for (int t = 0; t < 64; ++t) o[t] = 0;
    return;
  }
  fp x = fp_from_mont(a.x), y = fp_from_mont(a.y);
  for (int l = 0; l < 8; ++l) {
    const uint32_t vx = x.v[7 - l], vy = y.v[7 - l];
    for (int b = 0; b < 4; ++b) {
      o[4 * l + b] = (uint8_t)(vx >> (24 - 8 * b));
      o[32 + 4 * l + b] = (uint8_t)(vy >> (24 - 8 * b));
    }
  }
}

// Jacobian -> affine (Montgomery) [n][16]
extern "C" __global__ void __launch_bounds__(64) k_to_affine(const uint32_t* pts, int n, uint32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_aff(out + 16 * (size_t)i, jac_to_aff(ld_jac(pts + 24 * (size_t)i)));
}

// ------------------------------------------------------------------ C ABI launchers
// (same translation unit as the kernels: no relocatable device code needed)
static inline int blocks_for(long long n, int bs) { return (int)((n + bs - 1) / bs); }

extern "C" int bsc_fp_op(const uint32_t* a, const uint32_t* b, uint32_t* out, int n, int op, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_fp_mul, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, a, b, out, n, op);
  return (int)hipGetLastError();
}

extern "C" int bsc_point_op(const uint32_t* a, const uint32_t* b, const int* ks, uint32_t* out, int n, int op,
                            void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_point_op, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, a, b, ks, out, n, op);
  return (int)hipGetLastError();
}

extern "C" int bsc_witness_bases(const uint32_t* pk_aff, int d, int poly, int T, uint32_t* out, void* stream) {
  const int nchunks = (d + poly - 1) / poly;
  const long long n = (long long)nchunks * T;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_witness_bases, dim3(blocks_for(n, 128)), dim3(128), 0, (hipStream_t)stream, pk_aff, d, poly,
                     T, out);
  return (int)hipGetLastError();
}

extern "C" int bsc_fb_table(const uint32_t* bases, int bases_are_jac, int b0, int nb, int inner, int B0, int NW,
                            long long s_outer, long long s_e, long long s_in, uint32_t* table, uint32_t* scratch,
                            void* stream) {
  if (B0 < 8 || B0 > 20 || NW < 1) return -1;
  const long long runs = (1ll << (B0 - 1)) / TBL_ENTRIES + NW - 1;
  const long long n = (long long)nb * runs;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_fb_table, dim3(blocks_for(n, 64)), dim3(64), 0, (hipStream_t)stream, bases, bases_are_jac, b0,
                     nb, inner, B0, NW, s_outer, s_e, s_in, table, scratch);
  return (int)hipGetLastError();
}

extern "C" int bsc_shares_msm(const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk,
                              const uint32_t* tbl_wb, int poly, int T, int B0, int NW, int commit_only,
                              const int* alive, const int* compact, int group_rows, uint32_t* out_pts,
                              long long* out_y, void* stream) {
  if (B0 < 8 || B0 > 20 || B0 + 8 * (NW - 1) < 65) return -1;  // every int64 scalar must be covered
  if (commit_only < 0 || commit_only > 2) return -1;
  const int nchunks = (d + poly - 1) / poly;
  const int SL = commit_only == 1 ? 1 : commit_only == 2 ? T : T + 1;
  const long long n = (long long)nrows * nchunks * SL;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_shares_msm, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, coeffs, d, rows,
                     nrows, tbl_pk, tbl_wb, poly, T, B0, NW, commit_only, alive, compact, group_rows, out_pts,
                     out_y);
  return (int)hipGetLastError();
}

// rows_host: n <= ROWARG_MAX row indices (host memory), passed by value in the kernel's arguments
extern "C" int bsc_shares_msm_ka(const long long* coeffs, int d, const int* rows_host, int nrows, const uint32_t* tbl_pk,
                                 const uint32_t* tbl_wb, int poly, int T, int B0, int NW, int commit_only,
                                 const int* alive, int group_rows, uint32_t* out_pts, long long* out_y, void* stream) {
  if (B0 < 8 || B0 > 20 || B0 + 8 * (NW - 1) < 65) return -1;
  if (commit_only < 0 || commit_only > 2 || nrows > ROWARG_MAX || nrows < 0) return -1;
  const int nchunks = (d + poly - 1) / poly;
  const int SL = commit_only == 1 ? 1 : commit_only == 2 ? T : T + 1;
  const long long n = (long long)nrows * nchunks * SL;
  if (n <= 0) return 0;
  RowArg ra;
  for (int i = 0; i < nrows; ++i) ra.r[i] = rows_host[i];
  hipLaunchKernelGGL(k_shares_msm_ka, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, coeffs, d, ra,
                     nrows, tbl_pk, tbl_wb, poly, T, B0, NW, commit_only, alive, group_rows, out_pts, out_y);
  return (int)hipGetLastError();
}

// compact = [count, r0, r1, ...]: the rows r with alive[r] != 0, ascending (one block, n <= 4096)
extern "C" __global__ void __launch_bounds__(1024) k_alive_compact(const int* alive, int n, int* compact) {
  __shared__ int cnt[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int lo = t * per, hi = min(n, lo + per);
  int c = 0;
  for (int r = lo; r < hi; ++r) c += alive[r] != 0;
  cnt[t] = c;
  __syncthreads();
  // inclusive scan over the 1024 per-thread counts (Hillis-Steele)
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = t >= o ? cnt[t - o] : 0;
    __syncthreads();
    cnt[t] += v;
    __syncthreads();
  }
  int w = cnt[t] - c;
  for (int r = lo; r < hi; ++r)
    if (alive[r] != 0) compact[1 + w++] = r;
  if (t == 1023) compact[0] = cnt[1023];
}

extern "C" int bsc_alive_compact(const int* alive, int n, int* compact, void* stream) {
  if (n < 0 || n > 4096) return -1;
  hipLaunchKernelGGL(k_alive_compact, dim3(1), dim3(1024), 0, (hipStream_t)stream, alive, n, compact);
  return (int)hipGetLastError();
}

// alive[map[j]] = accept[j] for every verified update j with a speculative row (map[j] >= 0):
// agent-scope stores, read by a k_shares_msm still running on another stream.
// alive[i] = accept[src[i]] for every speculative row i (src[i] < 0: the row is no candidate of the
// selection -- e.g. a peer the pre-step computed that turned out not to be a worker -- and is dropped).
// Device-scope stores: a share MSM still running on another stream skips the rows cleared here.
extern "C" __global__ void k_set_alive(const int* accept, const int* src, int n, int* alive) {
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int j = src[i];
  __hip_atomic_store(alive + i, (j >= 0 && accept[j]) ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

extern "C" int bsc_set_alive(const int* accept, const int* src, int n, int* alive, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_set_alive, dim3(blocks_for(n, 64)), dim3(64), 0, (hipStream_t)stream, accept, src, n, alive);
  return (int)hipGetLastError();
}

extern "C" int bsc_sum_rows(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols, int ncols,
                            uint32_t* out, void* stream) {
  if (ncols <= 0) return 0;
  hipLaunchKernelGGL(k_sum_rows, dim3(blocks_for(ncols, 128)), dim3(128), 0, (hipStream_t)stream, pts, ncols_in,
                     rows, nrows, cols, ncols, out);
  return (int)hipGetLastError();
}

extern "C" int bsc_sum_rows2(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols,
                             int ncols, const int* row_mask, uint32_t* out, void* stream) {
  if (ncols <= 0) return 0;
  hipLaunchKernelGGL(k_sum_rows2, dim3(blocks_for(ncols, 16)), dim3(256), 0, (hipStream_t)stream, pts, ncols_in,
                     rows, nrows, cols, ncols, row_mask, 0, out);
  return (int)hipGetLastError();
}

static int g_wit_tree = 0;   // bsc_set_witness_tree(1): the witness sums in the LDS-tree form (A/Bs)
extern "C" int bsc_set_witness_tree(int on) {
  g_wit_tree = on ? 1 : 0;
  return 0;
}

extern "C" int bsc_sum_cols_serial(const uint32_t* pts, int ncols_in, int nrows, const int* cols, int ncols,
                                   const int* row_mask, uint32_t* out, void* stream) {
  if (ncols <= 0) return 0;
  if (g_wit_tree) return bsc_sum_rows2(pts, ncols_in, nullptr, nrows, cols, ncols, row_mask, out, stream);
  hipLaunchKernelGGL(k_sum_cols_serial, dim3(blocks_for(ncols, 256)), dim3(256), 0, (hipStream_t)stream, pts, ncols_in,
                     nrows, cols, ncols, row_mask, out);
  return (int)hipGetLastError();
}

// the same with row_mask indexed by the position in `rows` (a mask over a row list, e.g. the speculative
// MSM's alive flags applied to the pre-step's per-peer chunk commitments)
extern "C" int bsc_sum_rows2_pos(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols,
                                 int ncols, const int* row_mask, uint32_t* out, void* stream) {
  if (ncols <= 0) return 0;
  hipLaunchKernelGGL(k_sum_rows2, dim3(blocks_for(ncols, 16)), dim3(256), 0, (hipStream_t)stream, pts, ncols_in,
                     rows, nrows, cols, ncols, row_mask, 1, out);
  return (int)hipGetLastError();
}

extern "C" int bsc_commit_rows(const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk,
                               int B0, int NW, uint32_t* partial, uint32_t* out, void* stream) {
  if (nrows <= 0) return 0;
  if (B0 < 8 || B0 > 20 || B0 + 8 * (NW - 1) < 65 || NW > 9) return -1;
  const long long PB = (1ll << (B0 - 1)) + (long long)(NW - 1) * TBL_ENTRIES;
  if ((long long)d * PB >= (1ll << 31)) return -1;
  const int nslab = (d + COMMIT_CB - 1) / COMMIT_CB;
  hipLaunchKernelGGL(k_commit_rows, dim3(nrows * nslab), dim3(256), 0, (hipStream_t)stream, coeffs, d, rows, nrows,
                     tbl_pk, B0, NW, partial);
  hipLaunchKernelGGL(k_segment_sum, dim3(nrows), dim3(256), 0, (hipStream_t)stream, partial, nslab, 1, 0, out,
                     (uint32_t*)nullptr, 0);
  return (int)hipGetLastError();
}

// the round's side reductions (the pre-step's full-commitment sums, the aggregate audit) at the critical class
// (default) or one below the speculative share MSM (1): experiments and A/Bs (RunConfig ablation side_prio_low)
static int g_side_low = 0;
extern "C" int bsc_set_side_prio(int low) {
  g_side_low = low ? 1 : 0;
  return 0;
}

// hout (nullable): pinned host mirror of out
extern "C" int bsc_segment_sum_h(const uint32_t* pts, int ngroups, int n, int stride, int off, uint32_t* out,
                                 uint32_t* hout, void* stream) {
  if (ngroups <= 0) return 0;
  hipLaunchKernelGGL(k_segment_sum, dim3(ngroups), dim3(256), 0, (hipStream_t)stream, pts, n, stride, off, out, hout,
                     g_side_low);
  return (int)hipGetLastError();
}
extern "C" int bsc_segment_sum(const uint32_t* pts, int ngroups, int n, int stride, int off, uint32_t* out,
                               void* stream) {
  return bsc_segment_sum_h(pts, ngroups, n, stride, off, out, nullptr, stream);
}

// h_ok (nullable): pinned host mirror of ok
extern "C" int bsc_chunk_check_h(const long long* coeffs, int d, int poly, const uint32_t* tbl_pk, int B0, int NW,
                                 const uint32_t* csum, int nm, int nch, int* ok, int* h_ok, void* stream) {
  if (nch <= 0 || nm <= 0) return 0;
  if (poly < 1 || poly > 16 || nm > 64 || B0 < 8 || B0 > 20 || B0 + 8 * (NW - 1) < 65 || NW > 9) return -1;
  if ((long long)nch * poly < d || (long long)(nch - 1) * poly >= d) return -1;
  hipLaunchKernelGGL(k_chunk_check, dim3(nch), dim3(64), 0, (hipStream_t)stream, coeffs, d, poly, tbl_pk, B0, NW,
                     csum, nm, nch, ok, h_ok, g_side_low);
  return (int)hipGetLastError();
}
extern "C" int bsc_chunk_check(const long long* coeffs, int d, int poly, const uint32_t* tbl_pk, int B0, int NW,
                               const uint32_t* csum, int nm, int nch, int* ok, void* stream) {
  return bsc_chunk_check_h(coeffs, d, poly, tbl_pk, B0, NW, csum, nm, nch, ok, nullptr, stream);
}

extern "C" int bsc_marshal(const uint32_t* pts, int n, uint8_t* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_marshal, dim3(blocks_for(n, 64)), dim3(64), 0, (hipStream_t)stream, pts, n, out);
  return (int)hipGetLastError();
}

extern "C" int bsc_to_affine(const uint32_t* pts, int n, uint32_t* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_to_affine, dim3(blocks_for(n, 64)), dim3(64), 0, (hipStream_t)stream, pts, n, out);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ streams
// A stream restricted to a subset of the CUs: the speculative share/commitment MSMs run there so
// the protocol's critical-path kernels (noise, Krum, aggregation) always find idle CUs -- HIP
// stream priorities only order dispatch, they do not preempt the MSM's long-lived waves.
// `skip_every` = 4 leaves every 4th CU (spread over all XCDs / shader engines) out of the mask.
extern "C" void* bsc_stream_create_cumask(int skip_every, int* ncu_used) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
  const int ncu = prop.multiProcessorCount;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  int used = 0;
  // skip_every < 0: the complement -- ONLY the CUs a stream created with -skip_every leaves free
  const int k = skip_every < 0 ? -skip_every : skip_every;
  for (int c = 0; c < ncu; ++c) {
    const bool skipped = k > 0 && c % k == k - 1;
    if (skip_every < 0 ? !skipped : skipped) continue;
    mask[c / 32] |= 1u << (c % 32);
    ++used;
  }
  hipStream_t st = nullptr;
  if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) return nullptr;
  if (ncu_used) *ncu_used = used;
  return (void*)st;
}

extern "C" int bsc_stream_destroy(void* st) { return (int)hipStreamDestroy((hipStream_t)st); }

// Small host -> device upload from pinned staging memory (utils.h2d): the bare runtime call,
// without the per-copy event bookkeeping a framework-level pinned copy adds on the host.
extern "C" int bsc_h2d_async(void* dst, const void* src, long long nbytes, void* stream) {
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyHostToDevice, (hipStream_t)stream);
}

// Device -> pinned host read-back on a stream (utils.d2h_into): the bare runtime call.
extern "C" int bsc_d2h_async(void* dst, const void* src, long long nbytes, void* stream) {
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToHost, (hipStream_t)stream);
}
