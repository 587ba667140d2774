// op_cost.hip — measured issue cost of the VALU instruction kinds the trace
// kernel's loop is made of (gfx950): cycles per wave-instruction per SIMD at
// a given number of resident waves per SIMD.  8 independent chains per lane,
// each instruction written as inline asm so the compiler keeps exactly that
// opcode.  hipcc --offload-arch=gfx950 -O3 -o /tmp/op_cost tools/op_cost.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
#define BODY(OPSTR)                                                             \
  for (int it = 0; it < iters; ++it) {                                          \
    _Pragma("unroll") for (int i = 0; i < CHAINS; ++i) { unsigned t_; asm volatile(OPSTR : "+v"(v[i]), "=&v"(t_) : "v"(b) : "vcc", "s40", "s41"); } \
  }

template <int OP>
__global__ __launch_bounds__(256) void op_loop(unsigned* out, unsigned b, int iters) {
  unsigned v[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) v[i] = threadIdx.x * 7u + i;
  if constexpr (OP == 0) BODY("v_max_i32 %0, %0, %2")
  if constexpr (OP == 1) BODY("v_min_i32 %0, %0, %2")
  if constexpr (OP == 2) BODY("v_max_u32 %0, %0, %2")
  if constexpr (OP == 3) BODY("v_max3_i32 %0, %0, %2, %0")
  if constexpr (OP == 4) BODY("v_min3_i32 %0, %0, %2, %0")
  if constexpr (OP == 5) BODY("v_min_f32 %0, %0, %2")
  if constexpr (OP == 6) BODY("v_max_f32_e64 %0, %0, %2")
  if constexpr (OP == 7) BODY("v_sub_f32 %0, %0, %2")
  if constexpr (OP == 8) BODY("v_sub_u32 %0, %0, %2")
  if constexpr (OP == 9) BODY("v_or_b32 %0, %0, %2")
  if constexpr (OP == 10) BODY("v_ashrrev_i32 %0, 13, %0")
  if constexpr (OP == 11) BODY("v_lshlrev_b32 %0, %2, %0")
  if constexpr (OP == 12) BODY("v_lshlrev_b32_e64 %0, 13, %0")
  if constexpr (OP == 13) BODY("v_add3_u32 %0, %0, %2, %0")
  if constexpr (OP == 14) BODY("v_mad_u32_u24 %0, %0, %2, %0")
  if constexpr (OP == 15) BODY("v_cvt_f32_i32 %0, %0")
  if constexpr (OP == 16) BODY("v_fmac_f32 %0, %0, %2")
  if constexpr (OP == 17) BODY("v_mul_f32_e64 %0, %0, %2")
  if constexpr (OP == 18) BODY("v_maximum3_f32 %0, %0, %2, %0")
  if constexpr (OP == 19) BODY("v_med3_i32 %0, %0, %2, %0")
  if constexpr (OP == 20) BODY("v_not_b32 %0, %0")
  if constexpr (OP == 21) BODY("v_cndmask_b32 %0, %0, %2, vcc")
  if constexpr (OP == 22) BODY("v_cmp_lt_f32_e64 s[40:41], %0, %2")
  if constexpr (OP == 23) BODY("v_cmp_lt_f32 vcc, %0, %2")
  if constexpr (OP == 24) BODY("v_readfirstlane_b32 s40, %0")
  if constexpr (OP == 25) BODY("v_lshlrev_b32 %1, 13, %0\n\tv_xor_b32 %0, %0, %1")
  if constexpr (OP == 26) BODY("v_add_f32 %0, %0, %2\n\tv_max_f32 %0, %0, %2")
  if constexpr (OP == 27) BODY("v_fma_f32 %0, %0, %2, %0\n\tv_fma_f32 %0, %0, %2, %0")
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// packed f32 (64-bit register pairs)
template <int OP>
__global__ __launch_bounds__(256) void op_loop64(unsigned* out, unsigned b, int iters) {
  unsigned long long v[CHAINS];
  const unsigned long long bb = b * 0x100000001ull;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) v[i] = (threadIdx.x * 7u + i) * 0x100000001ull;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) {
      if constexpr (OP == 6) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(v[i]) : "v"(bb));
      if constexpr (OP == 7) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[i]) : "v"(bb));
      if constexpr (OP == 8) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(bb));
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) s += static_cast<unsigned>(v[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the compare + cndmask pair (VOPC writes vcc, then a select)
__global__ __launch_bounds__(256) void op_cmpsel(unsigned* out, unsigned b, int iters) {
  unsigned v[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) v[i] = threadIdx.x * 7u + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i)
      asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(b) : "vcc");
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 64-bit product (v_mad_u64_u32)
__global__ __launch_bounds__(256) void op_mad64(unsigned* out, unsigned b, int iters) {
  unsigned long long v[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) v[i] = threadIdx.x * 7u + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(v[i]) : "v"(b) : "vcc");
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) s += static_cast<unsigned>(v[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned* d;
  (void)hipMalloc(&d, 256 * 8 * 1024 * sizeof(unsigned));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"v_max_i32",
"v_min_i32",
"v_max_u32",
"v_max3_i32",
"v_min3_i32",
"v_min_f32",
"v_max_f32_e64",
"v_sub_f32",
"v_sub_u32",
"v_or_b32",
"v_ashrrev_i32",
"v_lshlrev_b32_vreg",
"v_lshlrev_b32_e64",
"v_add3_u32",
"v_mad_u32_u24",
"v_cvt_f32_i32",
"v_fmac_f32",
"v_mul_f32_e64",
"v_maximum3_f32",
"v_med3_i32",
"v_not_b32",
"v_cndmask_b32(vcc)",
"v_cmp_lt_f32 (s pair)",
"v_cmp_lt_f32 (vcc)",
"v_readfirstlane",
"xorshift13 (lsl+xor)",
"mix fast+slow (add,max)",
"v_fma_f32 x2"};
  const void* fns[] = {(void*)op_loop<0>, (void*)op_loop<1>, (void*)op_loop<2>, (void*)op_loop<3>, (void*)op_loop<4>, (void*)op_loop<5>, (void*)op_loop<6>, (void*)op_loop<7>, (void*)op_loop<8>, (void*)op_loop<9>, (void*)op_loop<10>, (void*)op_loop<11>, (void*)op_loop<12>, (void*)op_loop<13>, (void*)op_loop<14>, (void*)op_loop<15>, (void*)op_loop<16>, (void*)op_loop<17>, (void*)op_loop<18>, (void*)op_loop<19>, (void*)op_loop<20>, (void*)op_loop<21>, (void*)op_loop<22>, (void*)op_loop<23>, (void*)op_loop<24>, (void*)op_loop<25>, (void*)op_loop<26>, (void*)op_loop<27>};
  const int nops = 28, cmpsel = -1;
  const int iters = 20000;
  int clk_khz = 0;
  (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  printf("CUs %d, clock attr %.0f MHz\n", cus, clk_khz / 1e3);
  for (int wps : {5, 8}) {
    const int blocks = cus * wps;   // 4 waves per block = 1 per SIMD
    for (int k = 0; k < nops; ++k) {
      float ms = 0;
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(reinterpret_cast<void (*)(unsigned*, unsigned, int)>(const_cast<void*>(fns[k])),
                           blocks, 256, 0, 0, d, 3u, iters);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(reinterpret_cast<void (*)(unsigned*, unsigned, int)>(const_cast<void*>(fns[k])),
                           blocks, 256, 0, 0, d, 3u, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
      }
      const double insts_per_simd = double(wps) * iters * CHAINS * (k >= nops - 3 ? 2 : 1);
      const double ns_per_inst = ms * 1e6 / insts_per_simd;
      printf("waves/SIMD %d  %-26s %.3f ms  %.3f ns per wave-inst per SIMD (= %.2f cyc at 2.4 GHz)\n", wps,
             names[k], ms, ns_per_inst, ns_per_inst * 2.4);
    }
  }
  return 0;
}
