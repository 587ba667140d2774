// Correctly rounded fp32 square root and reciprocal for the kernel
// (trace_kernel.h): the same bits as the compiler's sqrtf and IEEE 1.0f / b
// for every input, in fewer VALU.  Both checked over all 2^32 inputs on
// gfx950 (tools/fp_rn_exhaustive.hip, profiles/r05/rcp/).
#pragma once
#include <hip/hip_runtime.h>

// (block markers of the ISA listing, trace_kernel.h; here for the rare branches)
#ifndef RT_MARK
#ifdef RTCLJ_ISA_MARKS
#define RT_MARK(name) asm volatile(";@@ " name)
#else
#define RT_MARK(name) ((void)0)
#endif
#endif

namespace rtclj {

// Correctly rounded sqrt, the same bits as sqrtf for every input: for
// x >= 2^-96 (every normal case here) the hardware v_sqrt_f32 corrected by
// the residuals of its neighbours -- the sequence the compiler emits for
// sqrtf, without its denormal scaling and zero/inf class fix-up (a rare
// branch keeps those for tiny, NaN and negative inputs): 16 -> 9 VALU.
// (sqrt_rn_normal: that sequence alone, for callers whose x >= 2^-96)
__device__ __forceinline__ float sqrt_rn_normal(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const int si = __builtin_bit_cast(int, s);
  const float sd = __builtin_bit_cast(float, si - 1), su = __builtin_bit_cast(float, si + 1);
  const float rd = fmaf(-sd, s, x), ru = fmaf(-su, s, x);
  float r = rd <= 0.0f ? sd : s;
  r = ru > 0.0f ? su : r;
  return r;
}
__device__ __forceinline__ float sqrt_rn(float x) {
  if (__builtin_expect(!(x >= 0x1p-96f), 0)) {
    RT_MARK("cold");
    return sqrtf(x);
  }
  return sqrt_rn_normal(x);
}

// Correctly rounded reciprocal, 11 -> 3 VALU (the division sequence is
// v_div_scale x2, v_rcp, v_div_fmas, v_div_fixup and six fmas/muls): one
// Newton step from v_rcp_f32 (1 ulp), y + y (1 - b y), the residual exact in
// an fma.  Equal to 1.0f / b for all 2^-126 <= b < 2^126, and only those:
// callers of rcp_rn_normal guarantee that range.
__device__ __forceinline__ float rcp_rn_normal(float b) {
  const float y = __builtin_amdgcn_rcpf(b);
  return fmaf(fmaf(-b, y, 1.0f), y, y);
}

// 1.0f / b for any b: the rest (zero, subnormals, |b| >= 2^126 whose
// reciprocal is subnormal, negatives, inf, NaN) through the division itself,
// a branch the kernel's inputs do not take.
__device__ __forceinline__ float rcp_rn(float b) {
  if (__builtin_expect(!(b >= 0x1p-126f && b < 0x1p126f), 0)) {
    RT_MARK("cold");
    return 1.0f / b;
  }
  return rcp_rn_normal(b);
}

}  // namespace rtclj
