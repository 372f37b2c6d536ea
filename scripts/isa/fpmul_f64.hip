// Double-precision-FMA Montgomery multiplication for the BN256 base field on gfx950, against the
// production FIPS multiplier (8 x 32-bit limbs, v_mad_u64_u32 carry chains, bn256_dev.h):
//
//   6 limbs of 48 bits held as doubles (signed, |limb| <= 2^47 after normalisation), R = 2^288.  Every limb product
//   a*b (|a*b| < 2^96) is split exactly with two FMAs: h = fma(a, b, M) - M with M = 1.5 * 2^100 (the sum lies in
//   [2^100, 2^101), whose ulp is 2^48, so h = round(a*b / 2^48) * 2^48), l = fma(a, b, -h) (|l| <= 2^47, exact).
//   Column k (value v_k * 2^(48k)) then takes v_k += l and v_{k+1} = fma(h, 2^-48, v_{k+1}): 5 VALU per product, no
//   integer carries.  Montgomery reduction by columns (SOS): r = v_i mod 2^48 (signed, by rounding v_i / 2^48 with
//   the 1.5 * 2^52 trick), m = r * p' mod 2^48 (signed), v += m * p * 2^(48 i), the exact multiple of 2^48 left in
//   column i carries into column i + 1.  Every intermediate is an integer of magnitude < 2^53 (bounds in
//   docs/PERF.md round 5), so the result is exact: out = a * b * 2^-288 mod p, in (-1.2 p, 1.2 p) with signed limbs,
//   chainable without a conditional subtraction.
//
// Check (scripts/isa/fpmul_f64_check.py, exact integers): for 2^20 random pairs out == a b 2^-288 mod p and the FIPS
// result == a b 2^-256 mod p.
// Throughput: both multipliers chained in registers at full occupancy and at 2 waves per SIMD, as fpmul_bench.hip.
//   hipcc --offload-arch=gfx950 -O3 -I../../biscotti_amd/csrc/kernels fpmul_f64.hip -o fpmul_f64
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "bn256_dev.h"

using namespace bn;

struct f6 {
  double v[6];
};

// p in 48-bit limbs, p' = -p^-1 mod 2^48
__device__ __constant__ static const double P48[6] = {189581434066535.0, 35964808206428.0, 242038291007697.0,
                                                      187397689598340.0, 2075721435129.0, 36789.0};
static constexpr double PPRIME = 273780527585961.0;
static constexpr double TWO48 = 281474976710656.0;          // 2^48
static constexpr double INV48 = 1.0 / 281474976710656.0;    // 2^-48
static constexpr double MBIG = 1.5 * 1267650600228229401496703205376.0;   // 1.5 * 2^100
static constexpr double MRND = 6755399441055744.0;          // 1.5 * 2^52

// h = round(a b / 2^48) 2^48, l = a b - h (exact)
__device__ __forceinline__ void split_prod(double a, double b, double& h, double& l) {
  h = __fma_rn(a, b, MBIG) - MBIG;
  l = __fma_rn(a, b, -h);
}

__device__ __forceinline__ f6 fp_mul_f64(const f6& a, const f6& b) {
  double v[13];
#pragma unroll
  for (int k = 0; k < 13; ++k) v[k] = 0.0;
  // product columns
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double h, l;
      split_prod(a.v[i], b.v[j], h, l);
      v[i + j] += l;
      v[i + j + 1] = __fma_rn(h, INV48, v[i + j + 1]);
    }
  }
  // Montgomery reduction, one column at a time
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double q = __fma_rn(v[i], INV48, MRND) - MRND;   // round(v_i / 2^48)
    const double r = __fma_rn(q, -TWO48, v[i]);            // v_i mod 2^48, signed
    const double hm = __fma_rn(r, PPRIME * INV48, MRND) - MRND;
    const double m = __fma_rn(r, PPRIME, -hm * TWO48);     // r p' mod 2^48, signed
    double h0, l0;
    split_prod(m, P48[0], h0, l0);
    // v_i + m p_0 is a multiple of 2^48: its quotient carries into column i + 1
    v[i + 1] += (v[i] + l0 + h0) * INV48;
#pragma unroll
    for (int j = 1; j < 6; ++j) {
      double h, l;
      split_prod(m, P48[j], h, l);
      v[i + j] += l;
      v[i + j + 1] = __fma_rn(h, INV48, v[i + j + 1]);
    }
  }
  // signed normalisation of the result columns 6..12 into 6 limbs
  f6 o;
  double c = 0.0;
#pragma unroll
  for (int k = 6; k < 11; ++k) {
    const double t = v[k] + c;
    const double q = __fma_rn(t, INV48, MRND) - MRND;
    o.v[k - 6] = __fma_rn(q, -TWO48, t);
    c = q;
  }
  o.v[5] = __fma_rn(v[12], TWO48, v[11] + c);
  return o;
}

// 8 x 32-bit limbs (< p) -> 6 x 48-bit limbs
__device__ __forceinline__ f6 to_f6(const fp& x) {
  f6 o;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int bit = 48 * k, w = bit >> 5, s = bit & 31;
    uint64_t lo = (uint64_t)x.v[w] | ((uint64_t)(w + 1 < 8 ? x.v[w + 1] : 0u) << 32);
    o.v[k] = (double)((lo >> s) & 0xffffffffffffull);   // 48k mod 32 is 0 or 16: one 64-bit window holds the limb
  }
  return o;
}

__global__ void k_check(const fp* a, const fp* b, fp* ref, f6* outf, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ref[i] = fp_mul(a[i], b[i]);
  outf[i] = fp_mul_f64(to_f6(a[i]), to_f6(b[i]));
}

template <int V>
__global__ void __launch_bounds__(256) k_tput(fp* io, f6* iof, int reps) {
  extern __shared__ uint32_t lds_pad[];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (V == 0) {
    fp x = io[i], y = io[i + 1], z = io[i + 2], w = io[i + 3];
    for (int r = 0; r < reps; ++r) {
      x = fp_mul(x, y);
      z = fp_mul(z, w);
    }
    if (reps < 0) lds_pad[threadIdx.x] = x.v[0];
    fp o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = x.v[k] ^ z.v[k];
    io[i] = o;
  } else {
    f6 x = iof[i], y = iof[i + 1], z = iof[i + 2], w = iof[i + 3];
    for (int r = 0; r < reps; ++r) {
      x = fp_mul_f64(x, y);
      z = fp_mul_f64(z, w);
    }
    if (reps < 0) lds_pad[threadIdx.x] = (uint32_t)x.v[0];
    f6 o;
#pragma unroll
    for (int k = 0; k < 6; ++k) o.v[k] = x.v[k] + z.v[k];
    iof[i] = o;
  }
}

static void rnd_fp(fp* x, unsigned* s) {
  for (int k = 0; k < 8; ++k) {
    *s = *s * 1664525u + 1013904223u;
    x->v[k] = *s ^ (*s >> 13) * 2654435761u;
  }
  x->v[7] &= 0x7fffffffu;   // < 2^255 < p
}

int main(int argc, char** argv) {
  const int n = 1 << 20;
  fp *a, *b, *ref;
  f6* outf;
  hipMallocManaged(&a, n * sizeof(fp));
  hipMallocManaged(&b, n * sizeof(fp));
  hipMallocManaged(&ref, n * sizeof(fp));
  hipMallocManaged(&outf, n * sizeof(f6));
  unsigned s = 777;
  for (int i = 0; i < n; ++i) {
    rnd_fp(&a[i], &s);
    rnd_fp(&b[i], &s);
  }
  // edge cases: (p - 1)^2 and 0 * x
  const uint32_t Ph[8] = {0x5e089667u, 0x185cac6cu, 0x20b5b59eu, 0xee5b88d1u,
                          0x6184dc21u, 0xaa6fecb8u, 0x4aa387f9u, 0x8fb501e3u};
  for (int k = 0; k < 8; ++k) { a[0].v[k] = Ph[k]; b[0].v[k] = Ph[k]; a[1].v[k] = 0; }
  a[0].v[0] -= 1;
  b[0].v[0] -= 1;
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, a, b, ref, outf, n);
  hipDeviceSynchronize();
  // inputs, FIPS results and the f64 results (signed 48-bit limbs) for the host check (scripts/isa/fpmul_f64_check.py)
  const char* path = argc > 1 ? argv[1] : "fpmul_f64_check.bin";
  FILE* f = fopen(path, "wb");
  fwrite(a, sizeof(fp), n, f);
  fwrite(b, sizeof(fp), n, f);
  fwrite(ref, sizeof(fp), n, f);
  fwrite(outf, sizeof(f6), n, f);
  fclose(f);
  const int reps = 256;
  f6* iof;
  hipMalloc(&iof, (size_t)256 * 8 * 256 * sizeof(f6) + 4 * sizeof(f6));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, a, b, ref, outf, n);
  hipMemcpy(iof, outf, (size_t)256 * 8 * 256 * sizeof(f6) + 4 * sizeof(f6), hipMemcpyDefault);
  for (int occ = 0; occ < 2; ++occ) {
    const size_t lds = occ ? 80 * 1024 : 0;
    for (int v = 0; v < 2; ++v) {
      const int blocks = 256 * 8;
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      auto kern = v == 0 ? k_tput<0> : k_tput<1>;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, a, iof, reps);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, a, iof, reps);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double muls = 2.0 * reps * blocks * 256.0;
      printf("{\"variant\": \"%s\", \"occupancy\": \"%s\", \"ms\": %.3f, \"Gmul_per_s\": %.1f}\n",
             v ? "f64fma_48x6" : "fips_32x8", occ ? "2 waves/SIMD" : "full", ms, muls / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
