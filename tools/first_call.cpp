// Times the one-time HIP set-up steps of a first rt_render call, each on its
// own, in a fresh process (design tool: DESIGN.md §5 first call).
//   hipcc -O2 -o tools/first_call tools/first_call.cpp && tools/first_call
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

static double ms(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}
#define T(label, call)                                   \
  do {                                                   \
    auto t0 = std::chrono::steady_clock::now();          \
    hipError_t e = (call);                               \
    std::printf("%-34s %8.3f ms  %s\n", label, ms(t0), hipGetErrorString(e)); \
  } while (0)

int main() {
  int n = 0;
  T("hipGetDeviceCount (runtime init)", hipGetDeviceCount(&n));
  T("hipSetDevice(0)", hipSetDevice(0));
  void* d = nullptr;
  T("hipMalloc 16 B (first)", hipMalloc(&d, 16));
  hipStream_t s;
  T("hipStreamCreateWithFlags", hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipStream_t s2;
  T("hipStreamCreateWithFlags (2nd)", hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  T("hipEventCreate x1", hipEventCreate(&e0));
  T("hipEventCreate x1 (2nd)", hipEventCreate(&e1));
  (void)hipEventCreate(&e2);
  void* h = nullptr;
  T("hipHostMalloc 16 B", hipHostMalloc(&h, 16, hipHostMallocDefault));
  void* h2 = nullptr;
  T("hipHostMalloc 16 B (2nd)", hipHostMalloc(&h2, 16, hipHostMallocDefault));
  void* big = nullptr;
  T("hipMalloc 9.7 MB", hipMalloc(&big, 1200 * 675 * 12));
  T("hipMemsetAsync 16 B (first op)", hipMemsetAsync(d, 0, 16, s));
  T("hipStreamSynchronize", hipStreamSynchronize(s));
  T("hipMemsetAsync 16 B (2nd)", hipMemsetAsync(d, 0, 16, s));
  T("hipStreamSynchronize (2nd)", hipStreamSynchronize(s));
  T("hipEventRecord", hipEventRecord(e0, s));
  T("hipStreamSynchronize (3rd)", hipStreamSynchronize(s));
  return 0;
}
