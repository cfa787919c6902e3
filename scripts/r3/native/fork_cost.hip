// Cost on the producing stream of letting a side stream wait for a kernel:
// (a) no fork, (b) hipEventRecord after the kernel, (c) the kernel's own completion as the
// event (hipExtLaunchKernelGGL stopEvent).  Prints us per kernel for each variant.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void scale_k(float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 1.0000001f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const int iters = 400;
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t evs[iters];
  for (int i = 0; i < iters; ++i) CK(hipEventCreateWithFlags(&evs[i], hipEventDisableTiming));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int n : {1 << 16, 1 << 24}) {
    float* x;
    CK(hipMalloc(&x, n * sizeof(float)));
    CK(hipMemset(x, 0, n * sizeof(float)));
    const int grid = (n + 255) / 256;
    for (int v = 0; v < 3; ++v) {
      float best = 1e9f;
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(t0, s0));
        for (int i = 0; i < iters; ++i) {
          if (v == 2) {
            hipExtLaunchKernelGGL(scale_k, dim3(grid), dim3(256), 0, s0, nullptr, evs[i], 0, x, n);
          } else {
            hipLaunchKernelGGL(scale_k, dim3(grid), dim3(256), 0, s0, x, n);
            if (v == 1) CK(hipEventRecord(evs[i], s0));
          }
          if (v > 0) CK(hipStreamWaitEvent(s1, evs[i], 0));
        }
        CK(hipEventRecord(t1, s0));
        CK(hipEventSynchronize(t1));
        CK(hipStreamSynchronize(s1));
        float ms;
        CK(hipEventElapsedTime(&ms, t0, t1));
        if (rep > 0 && ms < best) best = ms;
      }
      printf("{\"numel\": %d, \"variant\": \"%s\", \"us_per_kernel\": %.2f}\n", n,
             v == 0 ? "no_fork" : (v == 1 ? "event_record" : "ext_launch_stop_event"), best * 1e3f / iters);
    }
    CK(hipFree(x));
  }
  return 0;
}
