// d2h_bench.cpp — the pieces of rt_render's gather for a C1 frame (9.72 MB):
// D2H into pinned staging, host copy pinned -> pageable (1 and 4 threads),
// and D2H straight into pageable memory.  hipcc -O2 -o /tmp/d2h tools/d2h_bench.cpp -pthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
  const size_t n = 1200ull * 675 * 3, bytes = n * 4;
  float *d, *pin;
  (void)hipMalloc(&d, bytes);
  (void)hipMemset(d, 1, bytes);
  (void)hipHostMalloc(&pin, bytes, hipHostMallocDefault);
  std::vector<float> user(n);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int rep = 0; rep < 4; ++rep) {
    double t0 = now_ms();
    (void)hipMemcpyAsync(pin, d, bytes, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    double t1 = now_ms();
    std::memcpy(user.data(), pin, bytes);
    double t2 = now_ms();
    std::vector<std::thread> th;
    for (int k = 0; k < 4; ++k)
      th.emplace_back([&, k] {
        const size_t a = n * k / 4, b = n * (k + 1) / 4;
        std::memcpy(user.data() + a, pin + a, (b - a) * 4);
      });
    for (auto& t : th) t.join();
    double t3 = now_ms();
    (void)hipMemcpyAsync(user.data(), d, bytes, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    double t4 = now_ms();
    printf("D2H pinned %.3f ms  memcpy 1 thr %.3f ms  4 thr %.3f ms  D2H pageable %.3f ms\n", t1 - t0, t2 - t1,
           t3 - t2, t4 - t3);
  }
  return 0;
}
