// Throughput of the integer / f64 multiply instructions a 256-bit Montgomery multiplier can be
// built from, on gfx950.  8 independent chains per lane, enough waves to fill every SIMD.
//   hipcc --offload-arch=gfx950 -O3 isa_rates.hip -o isa_rates && ./isa_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CHECK(x) (void)(x)

#define ITERS 4096
#define CH 8

__global__ void __launch_bounds__(256) k_mad64(uint64_t* out, uint32_t s) {
  uint64_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_mullo(uint32_t* out, uint32_t s) {
  uint32_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_mulhi(uint32_t* out, uint32_t s) {
  uint32_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_mul24(uint32_t* out, uint32_t s) {
  uint32_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_mad24(uint32_t* out, uint32_t s) {
  uint32_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_fma64(double* out, uint32_t s) {
  double acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + fa;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(fa));
  }
  double r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_add(uint32_t* out, uint32_t s) {
  uint32_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(acc[c]) : "v"(a) : "vcc");
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_addc(uint32_t* out, uint32_t s) {
  uint32_t acc[CH];
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double fa = 1.0 + 1e-9 * a;
  (void)fa; (void)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(a) : "vcc");
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <class K, class T>
static void run(const char* name, K kern, T* buf, int blocks, double ops_per_iter_chain) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, 1u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, (uint32_t)r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double lane_ops = 5.0 * blocks * 256.0 * ITERS * CH * ops_per_iter_chain;
  // per CU per cycle at the nominal 2.4 GHz, 256 CUs
  const double per_cu_cyc = lane_ops / (ms * 1e-3) / 256.0 / 2.4e9;
  printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"Gops\": %.1f, \"lane_ops_per_CU_cycle\": %.2f}\n", name, ms,
         lane_ops / (ms * 1e-3) / 1e9, per_cu_cyc);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  const int blocks = 256 * 8 * 4;
  void* buf;
  hipMalloc(&buf, (size_t)blocks * 256 * 8);
  run("v_mad_u64_u32", k_mad64, (uint64_t*)buf, blocks, 1.0);
  run("v_mul_lo_u32", k_mullo, (uint32_t*)buf, blocks, 1.0);
  run("v_mul_hi_u32", k_mulhi, (uint32_t*)buf, blocks, 1.0);
  run("v_mul_u32_u24", k_mul24, (uint32_t*)buf, blocks, 1.0);
  run("v_mad_u32_u24", k_mad24, (uint32_t*)buf, blocks, 1.0);
  run("v_fma_f64", k_fma64, (double*)buf, blocks, 1.0);
  run("v_add_co_u32", k_add, (uint32_t*)buf, blocks, 1.0);
  run("v_addc_co_u32 (serial vcc)", k_addc, (uint32_t*)buf, blocks, 1.0);
  hipFree(buf);
  return 0;
}
