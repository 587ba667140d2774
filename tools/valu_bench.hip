// valu_bench.hip — fp32 VALU throughput on gfx950: v_fma_f32 vs v_pk_fma_f32.
// hipcc --offload-arch=gfx950 -O3 -o valu_bench tools/valu_bench.hip && ./valu_bench
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int ACC>
__global__ __launch_bounds__(256) void fma_scalar(float* out, float a, float b, int iters) {
  float acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_fmaf(acc[i], a, b);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ACC>
__global__ __launch_bounds__(256) void fma_packed(float* out, float a, float b, int iters) {
  f2 acc[ACC];
  const f2 va = {a, a}, vb = {b, b};
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_elementwise_fma(acc[i], va, vb);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* d;
  const int blocks = 256 * 8, threads = 256, iters = 20000;
  (void)hipMalloc(&d, blocks * threads * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipLaunchKernelGGL(fma_scalar<8>, blocks, threads, 0, 0, d, 0.999f, 1e-4f, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(fma_scalar<8>, blocks, threads, 0, 0, d, 0.999f, 1e-4f, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 8 * iters * double(blocks) * threads;
    printf("v_fma_f32    x8 acc: %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
    hipLaunchKernelGGL(fma_packed<8>, blocks, threads, 0, 0, d, 0.999f, 1e-4f, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(fma_packed<8>, blocks, threads, 0, 0, d, 0.999f, 1e-4f, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    fl = 2.0 * 16 * iters * double(blocks) * threads;
    printf("v_pk_fma_f32 x8 acc: %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
  }
  return 0;
}
