// Host-side cost of the HIP runtime calls a round issues (launch, event record, stream wait, small pinned
// copies), and of the same work replayed as a captured hipGraph: the round's host thread is its critical
// path, so these costs decide what a fused native call can save.
//   hipcc -O2 --offload-arch=gfx950 scripts/isa/hip_api_costs.hip -o /tmp/hip_api_costs && /tmp/hip_api_costs
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int* p) {
  if (p != nullptr && threadIdx.x == 9999) p[0] = 1;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      return 1;                                                       \
    }                                                                 \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  int *d, *h;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipHostMalloc(&h, 1 << 20));
  const int N = 2000;
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, a, d);
  CK(hipStreamSynchronize(a));
  double t = now_us();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, a, d);
  double launch = (now_us() - t) / N;
  CK(hipStreamSynchronize(a));
  t = now_us();
  for (int i = 0; i < N; ++i) CK(hipEventRecord(ev, a));
  double rec = (now_us() - t) / N;
  t = now_us();
  for (int i = 0; i < N; ++i) CK(hipStreamWaitEvent(b, ev, 0));
  double wait = (now_us() - t) / N;
  CK(hipDeviceSynchronize());
  t = now_us();
  for (int i = 0; i < N; ++i) CK(hipMemcpyAsync(h, d, 64 * 1024, hipMemcpyDeviceToHost, a));
  double d2h = (now_us() - t) / N;
  CK(hipDeviceSynchronize());
  t = now_us();
  for (int i = 0; i < N; ++i) CK(hipMemcpyAsync(d, h, 1024, hipMemcpyHostToDevice, a));
  double h2d = (now_us() - t) / N;
  CK(hipDeviceSynchronize());
  // a 20-node fork/join sequence captured once, replayed
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, a, d);
  CK(hipEventRecord(ev, a));
  CK(hipStreamWaitEvent(b, ev, 0));
  for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, b, d);
  CK(hipMemcpyAsync(h, d, 64 * 1024, hipMemcpyDeviceToHost, b));
  hipEvent_t j;
  CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
  CK(hipEventRecord(j, b));
  CK(hipStreamWaitEvent(a, j, 0));
  CK(hipMemcpyAsync(h + 65536, d, 4096, hipMemcpyDeviceToHost, a));
  CK(hipStreamEndCapture(a, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, a));
  CK(hipDeviceSynchronize());
  const int M = 500;
  t = now_us();
  for (int i = 0; i < M; ++i) CK(hipGraphLaunch(ge, a));
  double glaunch = (now_us() - t) / M;
  CK(hipDeviceSynchronize());
  // the same 20 operations issued one by one
  t = now_us();
  for (int r = 0; r < M; ++r) {
    for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, a, d);
    CK(hipEventRecord(ev, a));
    CK(hipStreamWaitEvent(b, ev, 0));
    for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, b, d);
    CK(hipMemcpyAsync(h, d, 64 * 1024, hipMemcpyDeviceToHost, b));
    CK(hipEventRecord(j, b));
    CK(hipStreamWaitEvent(a, j, 0));
    CK(hipMemcpyAsync(h + 65536, d, 4096, hipMemcpyDeviceToHost, a));
  }
  double direct = (now_us() - t) / M;
  CK(hipDeviceSynchronize());
  printf("{\"launch_us\": %.2f, \"event_record_us\": %.2f, \"stream_wait_us\": %.2f, \"d2h_64KB_us\": %.2f, "
         "\"h2d_1KB_us\": %.2f, \"graph_20ops_launch_us\": %.2f, \"direct_20ops_us\": %.2f}\n",
         launch, rec, wait, d2h, h2d, glaunch, direct);
  return 0;
}
