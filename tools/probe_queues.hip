// Which HIP streams of one process share a hardware queue (GPU_MAX_HW_QUEUES): a one-wave spin
// kernel (~30 ms on the wall clock) on stream i, then an empty kernel on stream j; if j's kernel
// finishes while i's spin is still running they are on different queues (kernels of streams that
// share a queue run in submission order). Streams are created in the order given, the same way
// the library creates its own (hipStreamCreateWithFlags, non-blocking).
// build: hipcc --offload-arch=gfx950 -O2 tools/probe_queues.hip -o tools/probe_queues
// run:   GPU_MAX_HW_QUEUES=2 ./tools/probe_queues 6      (GPU box; prints an N x N matrix)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void spin_kernel(unsigned long long cycles, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) out[0] = 1;  // (a vector store)
}
__global__ void empty_kernel(int* out) {
  if (threadIdx.x == 0) out[1] = 2;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 6;
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  int wclk = 0;  // wall clock rate in kHz
  (void)hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);
  const unsigned long long cycles = (unsigned long long)wclk * 30ull;  // ~30 ms
  std::vector<hipStream_t> s(n);
  for (int i = 0; i < n; ++i)
    if (hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking) != hipSuccess) return 1;
  hipEvent_t e;
  (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  printf("wall clock %d kHz; row i = spinning stream, column j: 1 = j's kernel waited (same queue)\n", wclk);
  for (int i = 0; i < n; ++i) {
    printf("%2d:", i);
    for (int j = 0; j < n; ++j) {
      if (i == j) {
        printf(" -");
        continue;
      }
      hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s[i], cycles, d);
      hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s[j], d);
      (void)hipEventRecord(e, s[j]);
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      const bool done = hipEventQuery(e) == hipSuccess;
      (void)hipDeviceSynchronize();
      printf(" %d", done ? 0 : 1);
    }
    printf("\n");
  }
  (void)hipFree(d);
  return 0;
}
