// valu_cost.hip — issue cost of the VALU instructions the trace kernel's hot
// loop is made of, on gfx950: cycles per wave64 instruction per SIMD, at 1
// and at 8 resident waves per SIMD (the pipe's throughput), each op run as 8
// independent chains so that latency is hidden.  The shader clock is read
// from s_memtime against s_memrealtime (100 MHz) in the same run.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_cost tools/valu_cost.hip && /tmp/valu_cost
// Used for the VALU-pipe attribution in DESIGN.md §5 (profiles/r05/valu_cost.txt).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define V8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__device__ __forceinline__ void op8(float (&r)[8], float a, float b) {
#define ONE(i)                                                                                           \
  if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));        \
  if constexpr (OP == 4) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                     \
  if constexpr (OP == 9) asm volatile("v_sqrt_f32 %0, %0" : "+v"(r[i]));                                 \
  if constexpr (OP == 10) asm volatile("v_rcp_f32 %0, %0" : "+v"(r[i]));                                 \
  if constexpr (OP == 11) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xb" : "+v"(r[i]) : "v"(a), "v"(b)); \
  if constexpr (OP == 12) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));      \
  if constexpr (OP == 13) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));      \
  if constexpr (OP == 14) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                \
  if constexpr (OP == 15) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));   \
  if constexpr (OP == 16) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(r[i]));                            \
  if constexpr (OP == 17) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 18) asm volatile("v_lshlrev_b32 %0, 13, %0" : "+v"(r[i]));                        \
  if constexpr (OP == 20) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                \
  if constexpr (OP == 21) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));      \
  if constexpr (OP == 23) asm volatile("v_ffbl_b32 %0, %0" : "+v"(r[i]));                               \
  if constexpr (OP == 24 || OP == 69) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(a));          \
  if constexpr (OP == 25) asm volatile("v_div_fixup_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); \
  if constexpr (OP == 26) asm volatile("v_mov_b32 %0, %1" : "+v"(r[i]) : "v"(a));                       \
  if constexpr (OP == 40) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 41) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 42) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 43) asm volatile("v_lshrrev_b32 %0, 17, %0" : "+v"(r[i]));                        \
  if constexpr (OP == 44) asm volatile("v_ashrrev_i32 %0, 31, %0" : "+v"(r[i]));                        \
  if constexpr (OP == 45) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));      \
  if constexpr (OP == 46) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[60:61]" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 47) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));          \
  if constexpr (OP == 48) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 49) asm volatile("v_min_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 50) asm volatile("v_not_b32 %0, %0" : "+v"(r[i]));                                \
  if constexpr (OP == 51) asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(r[i]) : "v"(a));          \
  if constexpr (OP == 52) asm volatile("v_lshl_or_b32 %0, %0, 13, %1" : "+v"(r[i]) : "v"(a));           \
  if constexpr (OP == 53) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 54) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));       \
  if constexpr (OP == 55) asm volatile("v_max_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                   \
  if constexpr (OP == 56) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(r[i]));                            \
  if constexpr (OP == 57) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "s"(b));       \
  if constexpr (OP == 58) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(a) : "vcc"); \
  if constexpr (OP == 59) asm volatile("v_lshl_add_u32 %0, %0, 5, %1" : "+v"(r[i]) : "v"(a));          \
  if constexpr (OP == 60) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));      \
  if constexpr (OP == 61) { if (i & 1) asm volatile("v_lshlrev_b32 %0, 13, %0" : "+v"(r[i])); else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); } \
  if constexpr (OP == 62) { if (i & 1) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(r[i])); else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); } \
  if constexpr (OP == 63) { if (i & 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a)); else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); } \
  if constexpr (OP == 64) { if (i & 1) asm volatile("v_cmp_gt_f32_e64 s[60:61], %0, %1" : : "v"(r[i]), "v"(a) : "s60", "s61"); else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); } \
  if constexpr (OP == 66) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(a));     \
  if constexpr (OP == 67) { if (i & 1) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(a)); else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); } \
  if constexpr (OP == 68) { if (i & 1) asm volatile("v_cmp_gt_f32_e64 s[60:61], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[60:61]" : "+v"(r[i]) : "v"(a) : "s60", "s61"); else asm volatile("v_cmp_gt_f32_e64 s[62:63], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[62:63]" : "+v"(r[i]) : "v"(a) : "s62", "s63"); } \
  if constexpr (OP == 70) asm volatile("v_alignbit_b32 %0, %0, %1, 19" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 71) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 72) asm volatile("v_bfe_u32 %0, %0, 8, 24" : "+v"(r[i])); \
  if constexpr (OP == 73) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); \
  if constexpr (OP == 74) asm volatile("v_cvt_f32_ubyte0 %0, %0" : "+v"(r[i])); \
  if constexpr (OP == 75) asm volatile("v_ldexp_f32 %0, %0, 3" : "+v"(r[i])); \
  if constexpr (OP == 76) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 77) asm volatile("v_readfirstlane_b32 s60, %0" : : "v"(r[i]) : "s60"); \
  if constexpr (OP == 78) asm volatile("v_subrev_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 79) asm volatile("v_add_f32_e64 %0, -%0, |%1|" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 80) asm volatile("v_mul_f32_e64 %0, %0, -%1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 81) asm volatile("v_fmamk_f32 %0, %0, 0x3b03126f, %1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 82) asm volatile("v_add_f32 %0, 0x3b03126f, %0" : "+v"(r[i])); \
  if constexpr (OP == 83) asm volatile("v_mad_u32_u16 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); \
  if constexpr (OP == 84) asm volatile("v_lshlrev_b16 %0, 5, %0" : "+v"(r[i])); \
  if constexpr (OP == 85) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 86) asm volatile("v_lshlrev_b32 %0, 5, %0" : "+v"(r[i])); \
  if constexpr (OP == 87) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(r[i])); \
  if constexpr (OP == 88) asm volatile("v_cmp_class_f32_e64 s[60:61], %0, %1" : : "v"(r[i]), "v"(a) : "s60", "s61"); \
  if constexpr (OP == 89) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(r[i]) : "v"(a) : "vcc"); \
  if constexpr (OP == 90) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); \
  if constexpr (OP == 91) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 92) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r[i]) : "v"(a)); \
  if constexpr (OP == 93) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); \
  if constexpr (OP == 96) asm volatile("v_add_f32_e64 %0, %0, %2" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 97) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xb" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 98) asm volatile("v_mul_f32_e64 %0, %0, %2" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 99) asm volatile("v_add_u32_e64 %0, %0, %2" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 100) asm volatile("v_xor_b32_e64 %0, %0, %2" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 101) asm volatile("v_fma_f32 %0, %0, %1, 2.0" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 102) asm volatile("v_sub_f32_e64 %0, %2, %0" : "+v"(r[i]) : "v"(a), "s"(b)); \
  if constexpr (OP == 65) { if (i & 1) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[60:61]" : "+v"(r[i]) : "v"(a)); else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b)); }
  V8(ONE)
#undef ONE
}

// the 64-bit / packed / compare forms: 8 independent pairs
typedef float f2 __attribute__((ext_vector_type(2)));
template <int OP>
__device__ __forceinline__ void op8w(f2 (&r)[8], f2 a, f2 b) {
#define ONE(i)                                                                                              \
  if constexpr (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));        \
  if constexpr (OP == 2) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                    \
  if constexpr (OP == 3) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));                    \
  if constexpr (OP == 19) asm volatile("v_mad_u64_u32 %0, s[60:61], %1, %2, %0" : "+v"(r[i]) : "v"(a.x), "v"(b.x) : "s60", "s61");      \
  if constexpr (OP == 22) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(r[i]) : "v"(a));              \
  if constexpr (OP == 27) asm volatile("v_cmp_lt_u64_e64 s[60:61], %0, %1" : : "v"(r[i]), "v"(a) : "s60", "s61"); \
  if constexpr (OP == 28) asm volatile("v_cmp_gt_f32_e64 s[60:61], %0, %1" : : "v"(r[i].x), "v"(a.x) : "s60", "s61"); \
  if constexpr (OP == 29) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" : : "v"(r[i].x), "v"(a.x) : "vcc");  \
  if constexpr (OP == 30) asm volatile("v_mov_b64 %0, %1" : "+v"(r[i]) : "v"(a));
  V8(ONE)
#undef ONE
}

constexpr bool wide(int op) { return op == 1 || op == 2 || op == 3 || op == 19 || op == 22 || (op >= 27 && op <= 30); }

template <int OP>
__global__ __launch_bounds__(256) void bench(float* out, float a0, float b0, int iters, unsigned long long* clk) {
  asm volatile("s_mov_b64 vcc, -1\n\ts_mov_b64 s[60:61], -1" ::: "vcc", "s60", "s61");
  if constexpr (OP == 69) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n\ts_nop 4" : : "v"(a0), "v"(b0) : "vcc");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  float s = 0.0f;
  if constexpr (wide(OP)) {
    f2 r[8];
    const f2 a = {a0, a0 + 1.0f}, b = {b0, b0};
    for (int i = 0; i < 8; ++i) r[i] = f2{threadIdx.x * 1e-3f + i, 1.0f + i};
    for (int it = 0; it < iters; ++it) {
      op8w<OP>(r, a, b);
      op8w<OP>(r, a, b);
      op8w<OP>(r, a, b);
      op8w<OP>(r, a, b);
    }
    for (int i = 0; i < 8; ++i) s += r[i].x + r[i].y;
  } else {
    float r[8];
    for (int i = 0; i < 8; ++i) r[i] = threadIdx.x * 1e-3f + i + 1.0f;
    for (int it = 0; it < iters; ++it) {
      op8<OP>(r, a0, b0);
      op8<OP>(r, a0, b0);
      op8<OP>(r, a0, b0);
      op8<OP>(r, a0, b0);
    }
    for (int i = 0; i < 8; ++i) s += r[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

static const char* name(int op) {
  switch (op) {
    case 0: return "v_fma_f32";
    case 1: return "v_pk_fma_f32";
    case 2: return "v_pk_add_f32";
    case 3: return "v_pk_mul_f32";
    case 4: return "v_add_f32";
    case 9: return "v_sqrt_f32";
    case 10: return "v_rcp_f32";
    case 11: return "v_bitop3_b32";
    case 12: return "v_perm_b32";
    case 13: return "v_max3_f32";
    case 14: return "v_mul_lo_u32";
    case 15: return "v_mad_u32_u24";
    case 16: return "v_cvt_f32_u32";
    case 17: return "v_xor_b32";
    case 18: return "v_lshlrev_b32";
    case 19: return "v_mad_u64_u32";
    case 20: return "v_mul_hi_u32";
    case 21: return "v_med3_f32";
    case 22: return "v_lshl_add_u64";
    case 23: return "v_ffbl_b32";
    case 24: return "v_cndmask_b32 (vcc)";
    case 25: return "v_div_fixup_f32";
    case 26: return "v_mov_b32";
    case 27: return "v_cmp_lt_u64_e64 (sgpr)";
    case 28: return "v_cmp_gt_f32_e64 (sgpr)";
    case 29: return "v_cmp_gt_f32_e32 (vcc)";
    case 30: return "v_mov_b64";
    case 40: return "v_add_u32";
    case 41: return "v_sub_u32";
    case 42: return "v_and_b32";
    case 43: return "v_lshrrev_b32";
    case 44: return "v_ashrrev_i32";
    case 45: return "v_add3_u32";
    case 46: return "v_cndmask_b32_e64 (sgpr)";
    case 47: return "v_fmac_f32";
    case 48: return "v_mul_f32";
    case 49: return "v_min_f32";
    case 50: return "v_not_b32";
    case 51: return "v_mbcnt_lo_u32_b32";
    case 52: return "v_lshl_or_b32";
    case 53: return "v_sub_f32";
    case 54: return "v_or3_b32";
    case 55: return "v_max_f32";
    case 56: return "v_cvt_u32_f32";
    case 57: return "v_fma_f32 (sgpr operand)";
    case 58: return "v_cmp_e32 + v_cndmask_e32 (pair)";
    case 59: return "v_lshl_add_u32";
    case 60: return "v_xad_u32";
    case 61: return "fma / lshlrev alternating";
    case 62: return "fma / cvt_f32_u32 alternating";
    case 63: return "fma / add_u32 alternating";
    case 64: return "fma / cmp_e64 alternating";
    case 65: return "fma / cndmask_e64 alternating";
    case 66: return "v_cndmask_b32_e64 (vcc)";
    case 67: return "fma / cndmask_e32 (vcc) alternating";
    case 68: return "cmp_e64 + cndmask_e64 (2 sgpr pairs)";
    case 69: return "v_cndmask_e32 (vcc from v_cmp)";
    case 96: return "v_add_f32 (sgpr operand)";
    case 97: return "v_bitop3_b32 (sgpr operand)";
    case 98: return "v_mul_f32 (sgpr operand)";
    case 99: return "v_add_u32 (sgpr operand)";
    case 100: return "v_xor_b32 (sgpr operand)";
    case 101: return "v_fma_f32 (inline const)";
    case 102: return "v_sub_f32 (sgpr operand)";

    case 70: return "v_alignbit_b32";
    case 71: return "v_lshlrev_b32 (vgpr amount)";
    case 72: return "v_bfe_u32";
    case 73: return "v_bfi_b32";
    case 74: return "v_cvt_f32_ubyte0";
    case 75: return "v_ldexp_f32";
    case 76: return "v_or_b32";
    case 77: return "v_readfirstlane_b32";
    case 78: return "v_subrev_f32";
    case 79: return "v_add_f32_e64 (neg/abs)";
    case 80: return "v_mul_f32_e64 (neg)";
    case 81: return "v_fmamk_f32 (literal)";
    case 82: return "v_add_f32 (literal)";
    case 83: return "v_mad_u32_u16";
    case 84: return "v_lshlrev_b16";
    case 85: return "v_mul_u32_u24";
    case 86: return "v_lshlrev_b32 (imm 5)";
    case 87: return "v_lshrrev_b32 (imm 8)";
    case 88: return "v_cmp_class_f32_e64";
    case 89: return "v_sub_co_u32";
    case 90: return "v_med3_i32";
    case 91: return "v_min_u32";
    case 92: return "v_max_i32";
    case 93: return "v_and_or_b32";
    case 94: return "v_xor3_b32";

  }
  return "?";
}

template <int OP>
static void run(float* d, unsigned long long* clk, int cus) {
  const int iters = 4000;
  double cyc_per[2] = {0, 0};
  double mhz = 0;
  for (int wi = 0; wi < 2; ++wi) {
    const int waves_per_simd = wi == 0 ? 1 : 8;
    const int blocks = cus * waves_per_simd;   // 256 threads = one wave per SIMD
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(bench<OP>, blocks, 256, 0, 0, d, 0.999f, 1e-4f, iters, clk);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    unsigned long long h[2];
    (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    const double f = h[1] ? static_cast<double>(h[0]) / static_cast<double>(h[1]) * 100.0 : 2400.0;   // MHz
    if (wi == 1) mhz = f;
    const double insts_per_simd = static_cast<double>(waves_per_simd) * iters * 32.0;
    cyc_per[wi] = best * 1e-3 * f * 1e6 / insts_per_simd;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  printf("%-26s 1 wave/SIMD %6.2f cyc   8 waves/SIMD %6.2f cyc   (shader clock %.0f MHz)\n", name(OP), cyc_per[0],
         cyc_per[1], mhz);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  float* d;
  unsigned long long* clk;
  (void)hipMalloc(&d, static_cast<size_t>(cus) * 8 * 256 * sizeof(float));
  (void)hipMalloc(&clk, 2 * sizeof(unsigned long long));
  printf("# %s, %d CUs: cycles per wave64 instruction per SIMD (8 independent chains)\n", p.gcnArchName, cus);
  run<0>(d, clk, cus);
  run<0>(d, clk, cus);
  run<96>(d, clk, cus);
  run<97>(d, clk, cus);
  run<98>(d, clk, cus);
  run<99>(d, clk, cus);
  run<100>(d, clk, cus);
  run<101>(d, clk, cus);
  run<102>(d, clk, cus);
  if (getenv("VALU_COST_NEW_ONLY")) return 0;
  run<1>(d, clk, cus);
  run<2>(d, clk, cus);
  run<3>(d, clk, cus);
  run<4>(d, clk, cus);
  run<9>(d, clk, cus);
  run<10>(d, clk, cus);
  run<11>(d, clk, cus);
  run<12>(d, clk, cus);
  run<13>(d, clk, cus);
  run<14>(d, clk, cus);
  run<15>(d, clk, cus);
  run<16>(d, clk, cus);
  run<17>(d, clk, cus);
  run<18>(d, clk, cus);
  run<19>(d, clk, cus);
  run<20>(d, clk, cus);
  run<21>(d, clk, cus);
  run<22>(d, clk, cus);
  run<23>(d, clk, cus);
  run<24>(d, clk, cus);
  run<25>(d, clk, cus);
  run<26>(d, clk, cus);
  run<27>(d, clk, cus);
  run<28>(d, clk, cus);
  run<29>(d, clk, cus);
  run<30>(d, clk, cus);
  run<40>(d, clk, cus);
  run<41>(d, clk, cus);
  run<42>(d, clk, cus);
  run<43>(d, clk, cus);
  run<44>(d, clk, cus);
  run<45>(d, clk, cus);
  run<46>(d, clk, cus);
  run<47>(d, clk, cus);
  run<48>(d, clk, cus);
  run<49>(d, clk, cus);
  run<50>(d, clk, cus);
  run<51>(d, clk, cus);
  run<52>(d, clk, cus);
  run<53>(d, clk, cus);
  run<54>(d, clk, cus);
  run<55>(d, clk, cus);
  run<56>(d, clk, cus);
  run<57>(d, clk, cus);
  run<58>(d, clk, cus);
  run<59>(d, clk, cus);
  run<60>(d, clk, cus);
  run<61>(d, clk, cus);
  run<62>(d, clk, cus);
  run<63>(d, clk, cus);
  run<64>(d, clk, cus);
  run<65>(d, clk, cus);
  run<66>(d, clk, cus);
  run<67>(d, clk, cus);
  run<68>(d, clk, cus);
  run<69>(d, clk, cus);
  run<70>(d, clk, cus);
  run<71>(d, clk, cus);
  run<72>(d, clk, cus);
  run<73>(d, clk, cus);
  run<74>(d, clk, cus);
  run<75>(d, clk, cus);
  run<76>(d, clk, cus);
  run<77>(d, clk, cus);
  run<78>(d, clk, cus);
  run<79>(d, clk, cus);
  run<80>(d, clk, cus);
  run<81>(d, clk, cus);
  run<82>(d, clk, cus);
  run<83>(d, clk, cus);
  run<84>(d, clk, cus);
  run<85>(d, clk, cus);
  run<86>(d, clk, cus);
  run<87>(d, clk, cus);
  run<88>(d, clk, cus);
  run<89>(d, clk, cus);
  run<90>(d, clk, cus);
  run<91>(d, clk, cus);
  run<92>(d, clk, cus);
  run<93>(d, clk, cus);

  return 0;
}
