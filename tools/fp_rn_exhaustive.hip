// Exhaustive check of the kernel's correctly rounded fp32 helpers
// (raytracing-clj_amd/csrc/fp_rn.h) against the compiler's IEEE 1.0f / b
// (v_div_scale / v_div_fmas / v_div_fixup) and sqrtf: counts the inputs
// where each candidate's bits differ and prints a few.  Reciprocal
// candidates 0-2 over every positive normal b, candidate 3 (one Newton step,
// rcp_rn_normal) over 2^-126 <= b < 2^126, candidate 4 (rcp_rn, guard
// included) over all 2^32 bit patterns; sqrt_rn over all 2^32 and
// sqrt_rn_normal over 2^-96 <= x <= +inf.
//   built by raytracing-clj_amd/Makefile as lib/fp_rn_exhaustive; tests/test_gpu_fp_rn.py runs it
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

constexpr int kCand = 7;
constexpr int kKeep = 8;

__device__ __forceinline__ float ieee_rcp(float b) {
  float one = 1.0f;
  asm volatile("" : "+v"(one));   // (no constant folding into something else)
  return one / b;
}

// C0: one Newton step from v_rcp_f32: y1 = y0 + y0 (1 - b y0)
__device__ __forceinline__ float rcp_n1(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y0, 1.0f);
  return fmaf(e, y0, y0);
}
// C1: two steps
__device__ __forceinline__ float rcp_n2(float b) {
  const float y1 = rcp_n1(b);
  const float e = fmaf(-b, y1, 1.0f);
  return fmaf(e, y1, y1);
}
// C2: the v_rcp value alone
__device__ __forceinline__ float rcp_hw(float b) { return __builtin_amdgcn_rcpf(b); }
// C3-C6: the kernel's
#include "../raytracing-clj_amd/csrc/fp_rn.h"

__device__ __forceinline__ float ieee_sqrt(float x) {
  asm volatile("" : "+v"(x));
  return sqrtf(x);
}

__global__ void check(unsigned long long* bad, uint32_t* first) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t k = blockIdx.x * blockDim.x + threadIdx.x; k < (1ull << 32); k += stride) {
    const uint32_t bits = static_cast<uint32_t>(k);
    const float b = __uint_as_float(bits);
    const uint32_t ref = __float_as_uint(ieee_rcp(b)), sref = __float_as_uint(ieee_sqrt(b));
    const bool posnormal = bits >= 0x00800000u && bits < 0x7f800000u;
    const bool inner = bits >= 0x00800000u && bits < 0x7e800000u;   // 2^-126 <= b < 2^126
    const bool sq_normal = bits >= 0x0f800000u && bits <= 0x7f800000u;   // 2^-96 <= x <= +inf
    const uint32_t c[kCand] = {__float_as_uint(rcp_n1(b)), __float_as_uint(rcp_n2(b)), __float_as_uint(rcp_hw(b)),
                               __float_as_uint(rtclj::rcp_rn_normal(b)), __float_as_uint(rtclj::rcp_rn(b)),
                               __float_as_uint(rtclj::sqrt_rn(b)), __float_as_uint(rtclj::sqrt_rn_normal(b))};
    const uint32_t r[kCand] = {ref, ref, ref, ref, ref, sref, sref};
    const bool in[kCand] = {posnormal, posnormal, posnormal, inner, true, true, sq_normal};
#pragma unroll
    for (int i = 0; i < kCand; ++i) {
      if (in[i] && c[i] != r[i]) {
        const unsigned long long old = atomicAdd(&bad[i], 1ull);
        if (old < kKeep) first[i * kKeep + old] = bits;
      }
    }
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  CHECK(hipMalloc(&bad, kCand * sizeof(unsigned long long)));
  CHECK(hipMalloc(&first, kCand * kKeep * sizeof(uint32_t)));
  CHECK(hipMemset(bad, 0, kCand * sizeof(unsigned long long)));
  CHECK(hipMemset(first, 0, kCand * kKeep * sizeof(uint32_t)));
  hipLaunchKernelGGL(check, dim3(256 * 64), dim3(256), 0, 0, bad, first);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned long long hb[kCand];
  uint32_t hf[kCand * kKeep];
  CHECK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  const char* names[kCand] = {"rcp + 1 newton (positive normals)", "rcp + 2 newton (positive normals)",
                              "v_rcp_f32 alone (positive normals)", "rcp_rn_normal (2^-126 <= b < 2^126)",
                              "rcp_rn (all 2^32 patterns)", "sqrt_rn (all 2^32 patterns)",
                              "sqrt_rn_normal (2^-96 <= x <= inf)"};
  for (int i = 0; i < kCand; ++i) {
    std::printf("%-40s mismatches %llu", names[i], hb[i]);
    for (int j = 0; j < kKeep && j < static_cast<int>(hb[i]); ++j) std::printf(" %08x", hf[i * kKeep + j]);
    std::printf("\n");
  }
  CHECK(hipFree(bad));
  CHECK(hipFree(first));
  return 0;
}
