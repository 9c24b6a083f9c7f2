// Host round trip of one tiny kernel launch on gfx950: launch + hipStreamSynchronize, launch +
// hipEventSynchronize, and a kernel that writes its result to coherent pinned memory polled by the
// host (no synchronise call). Median microseconds over 2000 calls each.
// usage: hipcc --offload-arch=gfx950 -O3 launch_roundtrip.hip -o /tmp/rt && /tmp/rt
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>
__global__ void tiny(volatile int* flag, int v) {
  if (threadIdx.x == 0) flag[0] = v;
}
int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* d;
  (void)hipMalloc(&d, 64);
  int* h;
  (void)hipHostMalloc(&h, 64, hipHostMallocCoherent);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  auto now = [] { return std::chrono::steady_clock::now(); };
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> t;
    for (int i = 0; i < 2200; ++i) {
      h[0] = 0;
      auto t0 = now();
      if (mode == 0) {
        tiny<<<1, 64, 0, s>>>(d, i + 1);
        (void)hipStreamSynchronize(s);
      } else if (mode == 1) {
        tiny<<<1, 64, 0, s>>>(d, i + 1);
        (void)hipEventRecord(ev, s);
        (void)hipEventSynchronize(ev);
      } else if (mode == 2) {
        tiny<<<1, 64, 0, s>>>(h, i + 1);
        while (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) != i + 1) {
        }
      } else {
        tiny<<<1, 64, 0, s>>>(h, i + 1);
        (void)hipStreamSynchronize(s);
      }
      auto t1 = now();
      if (i >= 200) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::sort(t.begin(), t.end());
    const char* names[] = {"launch + hipStreamSynchronize", "launch + event record + hipEventSynchronize",
                           "launch, poll coherent pinned flag", "launch to pinned + hipStreamSynchronize"};
    printf("%-48s median %7.2f us  p10 %7.2f  p90 %7.2f\n", names[mode], t[t.size() / 2], t[t.size() / 10],
           t[t.size() * 9 / 10]);
  }
  (void)hipStreamSynchronize(s);
  return 0;
}
