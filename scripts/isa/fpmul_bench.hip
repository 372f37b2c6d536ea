// Montgomery multiplication variants for the BN256 base field on gfx950: correctness cross-check
// and throughput.  hipcc --offload-arch=gfx950 -O3 -I../../biscotti_amd/csrc/kernels fpmul_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "bn256_dev.h"

using namespace bn;

// The previous production multiplier (CIOS, compiler-generated carries) kept as the baseline.
__device__ __forceinline__ fp fp_mul_cios(const fp& a, const fp& b) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c = (uint64_t)a.v[j] * b.v[i] + (uint64_t)t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    c = (uint64_t)t[8] + (c >> 32);
    t[8] = (uint32_t)c;
    t[9] = (uint32_t)(c >> 32);
    const uint32_t m = t[0] * NINV;
    c = (uint64_t)m * P[0] + (uint64_t)t[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      c = (uint64_t)m * P[j] + (uint64_t)t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    c = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)c;
    t[8] = t[9] + (uint32_t)(c >> 32);
  }
  return fp_reduce_once(t, t[8]);
}

__global__ void k_check(const fp* a, const fp* b, fp* r0, fp* r1, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  r0[i] = fp_mul_cios(a[i], b[i]);
  r1[i] = fp_mul(a[i], b[i]);
}

template <int V>
__global__ void __launch_bounds__(256) k_tput(fp* io, int reps) {
  extern __shared__ uint32_t lds_pad[];
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  fp x = io[i], y = io[i + 1], z = io[i + 2], w = io[i + 3];
  for (int r = 0; r < reps; ++r) {
    if (V == 0) {
      x = fp_mul_cios(x, y);
      z = fp_mul_cios(z, w);
    } else {
      x = fp_mul(x, y);
      z = fp_mul(z, w);
    }
  }
  if (reps < 0) lds_pad[threadIdx.x] = x.v[0];
  fp o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o.v[k] = x.v[k] ^ z.v[k];
  io[i] = o;
}

static const uint32_t Ph[8] = {0x5e089667u, 0x185cac6cu, 0x20b5b59eu, 0xee5b88d1u,
                               0x6184dc21u, 0xaa6fecb8u, 0x4aa387f9u, 0x8fb501e3u};

static void rnd_fp(fp* x, unsigned* s) {
  for (int k = 0; k < 8; ++k) {
    *s = *s * 1664525u + 1013904223u;
    x->v[k] = *s ^ (*s >> 13) * 2654435761u;
  }
  x->v[7] &= 0x7fffffffu;  // < 2^255 < p
  (void)Ph;
}

int main() {
  const int n = 1 << 20;
  fp *a, *b, *r0, *r1;
  hipMallocManaged(&a, n * sizeof(fp));
  hipMallocManaged(&b, n * sizeof(fp));
  hipMallocManaged(&r0, n * sizeof(fp));
  hipMallocManaged(&r1, n * sizeof(fp));
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) {
    rnd_fp(&a[i], &s);
    rnd_fp(&b[i], &s);
  }
  // edge cases
  for (int k = 0; k < 8; ++k) { a[0].v[k] = Ph[k]; b[0].v[k] = Ph[k]; }
  a[0].v[0] -= 1; b[0].v[0] -= 1;  // (p-1)^2
  for (int k = 0; k < 8; ++k) { a[1].v[k] = 0; b[1].v[k] = 0xffffffffu; }
  b[1].v[7] = 0x8fb501e3u; b[1].v[6] = 0;
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, a, b, r0, r1, n);
  hipDeviceSynchronize();
  int bad = 0;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 8; ++k) bad += r0[i].v[k] != r1[i].v[k];
  printf("{\"check\": \"fips vs cios\", \"n\": %d, \"mismatched_limbs\": %d}\n", n, bad);
  const int reps = 512;
  for (int occ = 0; occ < 2; ++occ) {
    // occ 0: full occupancy; occ 1: 80 KB LDS per 256-thread block -> 2 blocks/CU = 2 waves/SIMD
    const size_t lds = occ ? 80 * 1024 : 0;
    for (int v = 0; v < 2; ++v) {
      const int blocks = 256 * 8;
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      auto kern = v == 0 ? k_tput<0> : k_tput<1>;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, a, reps);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, a, reps);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double muls = 2.0 * reps * blocks * 256.0;
      printf("{\"variant\": \"%s\", \"occupancy\": \"%s\", \"ms\": %.3f, \"Gmul_per_s\": %.1f}\n",
             v ? "fips" : "cios", occ ? "2 waves/SIMD" : "full", ms, muls / (ms * 1e-3) / 1e9);
    }
  }
  return bad != 0;
}
