// trace_kernel.h — the device side of the per-pixel render loop: the kernel
// arguments, the RNG and arithmetic helpers, and the trace_kernel template
// (shared by trace.hip, the product library, and trace_diag.hip, the
// diagnostic library's A/B and statistics instantiations).
//
// Replaces, for one launch, the reference's
//   compute-pixel spp loop            src/raytracing.clj:141-155
//   ray-color (recursive)             src/raytracing.clj:45-58
//   hit-anything (closest-hit scan)   src/raytracing.clj:33-43
//   sphere ::hit-fn                   src/hittable.clj:7-31
//   lambertian / metal / dielectric   src/material.clj:13-46
//   vec3a math, rand samplers         src/vec3a.clj:56-101
//
// Execution shape (MI355X / CDNA4), DESIGN.md §3:
//   * one 256-thread workgroup owns an 8x8 pixel tile and every
//     (pixel, sample) pair of it: the *sample pool*.  A lane runs one path
//     at a time; when it ends (sky / absorbed / depth) the lane hands in its
//     colour and takes the next pair from an LDS counter, so no lane idles
//     until the pool is empty; then a wave down to its last few paths hands
//     them to its sibling waves' idle lanes (drain compaction) and leaves;
//   * a launch's last tiles are shared with helper workgroups dispatched in
//     its tail (tile sharing), and launches of few tiles split their samples;
//   * ray-color's recursion becomes a throughput accumulator T (stackless);
//   * the closest hit comes from a BVH in LDS (default) or, in the fallback
//     and diagnostic variants, a linear scan of the sphere table (LDS or the
//     scalar cache); either way it is the hit the reference's linear scan
//     returns, bit for bit;
//   * per-lane xorshift32 RNG, seeded per (seed, pixel, sample) by a hash;
//   * a finished sample's colour is added to its pixel's fixed-point sum in
//     LDS (u64, 2^-24 units): integer addition, so the total does not depend
//     on the order in which samples finish, and nothing goes through HBM but
//     the scene and the framebuffer, written once per pixel (fp32 RGB).
//
// Arithmetic contract (fp32; mirrored op-for-op by the oracle's fp32 mode,
// oracle/rt_oracle.cpp, so GPU and CPU agree bit-for-bit): every fused
// multiply-add is an explicit fmaf, the file is compiled with
// -ffp-contract=off, division and sqrt are IEEE correctly rounded (HIP's
// default), normalisations multiply by one correctly rounded reciprocal
// (d * (1/|d|), (p - C) * (1/r)), no transcendental function is used, and a
// pixel is RN(RN(float(sum of fix24(sample colour))) * 2^-24 / spp).
// See DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "bvh.h"
#include "fp_rn.h"
#include "rt_internal.h"

namespace rtclj {

struct alignas(16) KArgs {
  const float4* geo;   // n_pad: cx, cy, cz, -r*r   (hit test)
  const struct Pair* geo2;  // n_pad/2: the same, two bodies interleaved per Pair
  const float4* sph;   // n: cx, cy, cz, 1/r    (hit record)
  const float4* mat;   // n: albedo rgb, fuzz | refraction index (dielectric: x = 1/eta)
  const int* kind;     // n: material kind
  float* out;          // rows_out x width x 3
  unsigned long long* counters;  // NULL or [segments, samples]
  unsigned long long* dbg;       // stats build only: event counters (rt_debug_stats)
  unsigned long long* dbgw;      // stats build only: per wave {t_start, t_end, hw_id, xcc_id}
  float cam[18];       // center, p00, du, dv, disk_u, disk_v
  int defocus;
  int n;
  int n_pad;           // geo entries: n rounded up to 4, plus 4 never-hit pads
  int width;
  int rows_out;
  int row_begin, row_tile, tile_first, tile_step;
  // BVH traversal: blob = nodes | pairs | pidx (the LDS image)
  const float4* bvh_blob;
  int bvh_blob_f4;       // blob size in float4
  int bvh_off_pairs;     // byte offsets inside the blob
  int bvh_off_pidx;
  int big_pair0;         // the big bodies' leaves (bvh.cpp): pairs [big_pair0, + n_big_leaves x leaf pairs)
  int n_big_leaves;
  int bvh_stack;         // stack entries per lane (stack_entries: tree depth, or + 2 for tree 0)
  float bvh_c[3], bvh_r; // bounding sphere of the tree's bodies
  const int* tile_order;   // nullable: tile order (longest first) -> tile
  unsigned* tile_cost;     // nullable: per tile, its workgroups' durations added (s_memrealtime ticks) to half the history
  // Work units: the first n_whole tiles of the order are one
  // workgroup each, every later tile is `split` workgroups, one contiguous
  // sample range each, whose integer pixel sums go to part[split index]
  // (finalize_kernel adds them up)
  unsigned long long* part;  // [rows_out][width][3]: the split tiles' integer sums (atomics; zero between launches)
  int tiles_x;               // 8 x 8 tiles per tile row
  int n_whole, split;        // uniform splits: unit v >= n_whole is split v % split of order position v / split
  // cost-balanced splits (nullable): unit n_whole + u is samples [k * spp / s,
  // (k + 1) * spp / s) of tile x, with y = k | s << 8 (x < 0: no unit); the
  // plan_kernel of the previous launch of the shape made it from the record
  const int2* unit_tab;
  // n / d as the high half of n * m, m = ceil(2^64 / d) (magic64; m = 0 for
  // d = 1: n itself), exact for every 32-bit n: the kernel's loop divides
  // nothing, so no division has its reciprocal set-up hoisted into loop
  // registers (the pool's j / npx magic is made once per workgroup)
  uint64_t rt_magic;         // d = row_tile
  int spp, sample_begin, max_depth;
  int realm;             // RT_FLAG_REALM semantics (uniform)
  int sampler;           // RT_SAMPLER_* bits: the loop-free samplers (uniform)
  uint32_t key;
  // Tile sharing.  Workgroups [0, n_units) run the units
  // (dispatch positions); the grid's last workgroups are helpers,
  // dispatched once every unit has been, i.e. into the launch's tail.  The
  // sample pool [0, P) of a published whole tile is handed out from
  // word[tile] = (epoch << 48) | (helpers << 32) | next (epoch: the
  // launch's, 16 bits, so that a word left by an earlier launch on the
  // stream is never taken for this one's; the owner entries are cleared
  // when it wraps): every wave of its owner and of each
  // helper that joins it claims batches of kShareBatch samples until the
  // pool is spent, so they finish together.  Owners publish their tile in owner[unit %
  // n_owner]; a helper looks at a window of those and joins the tile with
  // the most unclaimed samples (at least steal_min).  A shared tile's pixel
  // sums meet in sum[tile] (u64 atomics, zero between uses); whoever brings
  // done[tile] to P converts them.  word NULL: no sharing.
  unsigned long long* word;      // per tile
  unsigned* done;                // per tile
  unsigned long long* sum;       // per tile: NPX x 3
  int* owner;                    // n_owner: tiles being run (-1: none)
  unsigned long long* stealc;    // [helpers that got samples, samples they claimed] (rt_steal_stats)
  int n_owner;
  int n_units;
  int share_from;                // units before this one never share (they end long before the launch's tail)
  int steal_min;
  int batch_max;                 // a wave's largest claim on a shared tile (0: by the pool)
  int lds_batch_max;             // ... on an unshared pool (from the workgroup's LDS counter; >= 64)
  unsigned epoch;                // this launch's (per stream, 1 .. 65535)
  // Drain compaction: a wave whose batches are spent and
  // which holds at most `compact` paths posts them to its siblings through
  // its traversal stack's LDS and leaves (0: off; <= mb_paths)
  int compact;
  int mb_paths;   // paths a post holds: as many as the wave's stack slice has room for (<= 32)
  // Path export (split launches).  xq non-NULL: a wave whose
  // batches are spent and which holds at most `compact` paths writes them to
  // xq as 64-byte records (xq_n[0] counts them) and leaves, so that its
  // workgroup's slot is free as soon as its pool is spent; the sweep launch
  // that follows (trace_kernel<..., SWEEP>) runs the records to their ends,
  // its waves claiming 64 at a time from xq_n[1], and adds their colours to
  // part[].  A record: origin, direction, throughput, RNG state, the pixel
  // (compacted row x width + column), depth left, the body it leaves.
  uint4* xq;
  unsigned* xq_n;
};

// ---------------------------------------------------------------- RNG ----
// xorshift32 (Marsaglia 13/17/5); a uniform double of the reference
// (clojure.core/rand, vec3a.clj:71-72) becomes the top 24 bits / 2^24,
// i.e. a float in [0, 1) on a 2^-24 grid.
__device__ __forceinline__ float rng_uniform(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return static_cast<float>(s >> 8) * 0x1p-24f;
}

// xi - 0.5 (compute-pixel's jitter, raytracing.clj:145-146), exact in fp32
__device__ __forceinline__ float rng_centered(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return fmaf(static_cast<float>(s >> 8), 0x1p-24f, -0.5f);
}

// rand-double -1 1 = -1 + 2*xi (vec3a.clj:71-72): exact in fp32, so one fma
// of the 24-bit integer gives the same bits as the mirror's 2*xi - 1.
__device__ __forceinline__ float rng_sym(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return fmaf(static_cast<float>(s >> 8), 0x1p-23f, -1.0f);
}

// ISA block markers: in a listing built with -DRTCLJ_ISA_MARKS (make isa-marks,
// tools/isa_blocks.py) each names the block of the kernel the lines after it
// belong to ("cold": a rare branch); the shipped and diagnostic builds contain
// none.  (Defined in fp_rn.h, included above.)

// stats builds: count one event per wave (by its first active lane)
__device__ __forceinline__ void wave_event(uint64_t& c) {
  const uint64_t ex = __builtin_amdgcn_read_exec();
  if ((threadIdx.x & 63) == static_cast<unsigned>(__ffsll(static_cast<long long>(ex)) - 1)) ++c;
}

// vec3a/random-unit-vec3 (vec3a.clj:74-79): rejection in [-1,1)^3 with
// 0 < |v|^2 <= 1 (1e-160 underflows to 0 in fp32), then v / |v|.
// (A software-pipelined form -- the next trip's states made while this
// trip's |v|^2 is tested -- measured 1.9 % slower on C1: the speculative
// trip's VALU costs more than the overlap saves; profiles/r04/kernel_b/.)
template <bool STATS = false>
__device__ __forceinline__ void random_unit(uint32_t& s, float& x, float& y, float& z, uint64_t* trips = nullptr,
                                            uint64_t* flops = nullptr) {
  float l2;
  // (the trip loop tests only |v|^2 <= 1, one compare a trip; v = 0, which
  // needs three draws of exactly 2^23, is sent back to the loop after it)
  do {
    do {
      if constexpr (STATS) {
        wave_event(*trips);
        *flops += 11;   // 3 x (2 xi - 1) + |v|^2
      }
      x = rng_sym(s);
      y = rng_sym(s);
      z = rng_sym(s);
      l2 = fmaf(z, z, fmaf(y, y, x * x));
    } while (!(l2 <= 1.0f));
    asm volatile("" : "+v"(l2));   // (keeps the two loops apart: one test a trip)
  } while (__builtin_expect(!(l2 > 0.0f), 0));
  // contract: v * (1/|v|); the components are multiples of 2^-23, so
  // 2^-46 <= l2 <= 1 and |v| lies in rcp_rn_normal's range
  const float il = rcp_rn_normal(sqrt_rn_normal(l2));
  if constexpr (STATS) *flops += 5;
  x = x * il;
  y = y * il;
  z = z * il;
}

// ---- Loop-free samplers (RT_FLAG_DIRECT_SAMPLERS) ----
enum { RT_SAMPLER_SPHERE = 1, RT_SAMPLER_DISK = 2 };   // KArgs::sampler bits
// The same distributions as vec3a/random-unit-vec3 (uniform on the unit
// sphere) and vec3a/random-in-unit-disk (uniform in the unit disk), drawn
// with a fixed number of draws instead of a rejection loop, so a wave no
// longer pays for its slowest lane's trips.  Fixed fp32 op sequences with no
// hardware transcendental (the oracle's MODE_MIRROR32 | ORACLE_DIRECT restates
// them op for op):
//   sphere (Archimedes): z = 2 xi1 - 1, r = sqrt(1 - z^2), phi = 2 pi xi2;
//   disk: r = sqrt(xi1), phi = 2 pi xi2;
// (cos phi, sin phi) from the 24-bit integer of xi2: the nearest quarter turn
// q, the rest as theta in [-pi/4, pi/4) by Taylor polynomials to theta^9 /
// theta^8 (|error| < 3e-8), rotated by q.
__device__ __forceinline__ uint32_t rng_u24(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s >> 8;
}
__device__ __forceinline__ void turn24(uint32_t u, float r, float& x, float& y) {
  const int f = static_cast<int>(u << 10) >> 10;             // the low 22 bits, signed: [-2^21, 2^21)
  const uint32_t q = (u + 0x200000u) >> 22;                  // nearest quarter turn (mod 4 below)
  const float th = static_cast<float>(f) * 0x1.921fb6p-22f;  // f * RN(2 pi / 2^24): |th| <= pi/4
  const float t2 = th * th;
  float ps = fmaf(t2, 0x1.71de3ap-19f, -0x1.a01a02p-13f);    // 1/9!, -1/7!
  ps = fmaf(t2, ps, 0x1.111112p-7f);                         // 1/5!
  ps = fmaf(t2, ps, -0x1.555556p-3f);                        // -1/3!
  const float sn = fmaf(th * t2, ps, th);
  float pc = fmaf(t2, 0x1.a01a02p-16f, -0x1.6c16c2p-10f);    // 1/8!, -1/6!
  pc = fmaf(t2, pc, 0x1.555556p-5f);                         // 1/4!
  pc = fmaf(t2, pc, -0.5f);
  const float cs = fmaf(t2, pc, 1.0f);
  // q quarter turns: (cs, sn) -> (-sn, cs) -> (-cs, -sn) -> (sn, -cs); the
  // signs ride on r (x = (+-r) * a: the same bits as -(r * a))
  const bool sw = (q & 1u) != 0;
  const float a = sw ? sn : cs, b = sw ? cs : sn;
  const float rx = __uint_as_float(__float_as_uint(r) ^ (((q + 1u) & 2u) << 30));
  const float ry = __uint_as_float(__float_as_uint(r) ^ ((q & 2u) << 30));
  x = rx * a;
  y = ry * b;
}
template <bool STATS = false>
__device__ __forceinline__ void sphere_direct(uint32_t& s, float& x, float& y, float& z, uint64_t* trips = nullptr,
                                              uint64_t* flops = nullptr) {
  if constexpr (STATS) {
    wave_event(*trips);
    *flops += 24;   // 2 xi - 1, 1 - z^2, sqrt, th, polynomials (17), 2 x r * a
  }
  z = rng_sym(s);
  // 1 - z^2 in one rounding; z is a multiple of 2^-23 in [-1, 1), so the
  // operand is 0 or >= 2^-22: sqrt_rn_normal's range, 0 included (sqrt 0 = 0
  // and both neighbour residuals fail their tests)
  const float r = sqrt_rn_normal(fmaf(-z, z, 1.0f));
  turn24(rng_u24(s), r, x, y);
}
template <bool STATS = false>
__device__ __forceinline__ void disk_direct(uint32_t& s, float& x, float& y, uint64_t* trips = nullptr,
                                            uint64_t* flops = nullptr) {
  if constexpr (STATS) {
    wave_event(*trips);
    *flops += 22;
  }
  // xi1 is 0 or >= 2^-24: sqrt_rn_normal's range, 0 included
  const float r = sqrt_rn_normal(rng_uniform(s));
  turn24(rng_u24(s), r, x, y);
}

// A sample's colour channel in the pixel's fixed-point sum: c * 2^24
// converted by v_cvt_u32_f32 (toward zero; NaN and c <= 0 give 0, c >= 256
// gives 2^32 - 1).  The sums are integers, so any completion order gives
// the same total (oracle: fix24).
__device__ __forceinline__ uint32_t fix24(float c) {
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(c * 0x1p24f));
  return r;
}

// n / d by the host's 64-bit magic m (KArgs)
__device__ __forceinline__ int div_magic(int n, uint64_t m) {
  return m ? static_cast<int>(__umul64hi(static_cast<uint64_t>(static_cast<uint32_t>(n)), m)) : n;
}

// stats build only: shader-clock stamp (s_memtime, drains lgkm; diagnostic)
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), off);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), off);
    const uint64_t o = (static_cast<uint64_t>(hi) << 32) | lo;
    v = o > v ? o : v;
  }
  return v;
}

// Cross-workgroup words of the stealing protocol: only
// ever touched by agent-scope atomics (read-modify-write, executed coherently
// for every XCD; a plain or sc1 load could hit a stale line in the reader's
// XCD L2), and a returned value is waited on before the next one is issued.
__device__ __forceinline__ unsigned long long xread64(unsigned long long* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int xread32(int* p) {
  return __hip_atomic_fetch_add(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A helper's look at the owner table and tile words only guides its choice
// (its join is an RMW on the word, whose returned value decides): relaxed
// agent-scope loads (global_load sc1), a read with no write-back, suffice.
__device__ __forceinline__ unsigned long long xload64(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int xload32(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ bool xcas64(unsigned long long* p, unsigned long long& expect, unsigned long long v) {
  return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}
// a wave's smallest claim on a shared tile (2 samples per lane: fixed
// batches of 64 cost 1 % at one GPU, of 256 lose the balance at the tail;
// profiles/r03/share_ab.txt)
constexpr int kShareBatch = 128;
// Drain compaction's mailbox: a donor wave writes its paths into its own
// slice of the traversal stack ([entry][lane], dead between iterations):
// word f * P + p (field f of path p, P paths per post) at entry row
// (f * P + p) / W, word (f * P + p) % W of the wave's W = 16 x sizeof(entry)
// words in that row.  P = as many as the slice holds, 13 fields each (C1's
// depth-9 u16 stack: 22, its u8 one in variant 22: 11; at most 32).
constexpr int kMbFields = 13;
// stats builds / RTCLJ_TIMELINE: waves recorded per launch (dispatch slot order)
constexpr int kDbgWaves = 1 << 17;
__device__ __forceinline__ unsigned word_epoch(unsigned long long w) { return static_cast<unsigned>(w >> 48); }
__device__ __forceinline__ int word_helpers(unsigned long long w) { return static_cast<int>((w >> 32) & 0xffffu); }
// a workgroup-uniform value read from LDS, moved to a scalar register (an LDS
// read lands in a VGPR, and everything derived from it would stay there)
__device__ __forceinline__ int sgpr(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long sgpr64(unsigned long long v) {
  return (static_cast<unsigned long long>(static_cast<unsigned>(sgpr(static_cast<int>(v >> 32)))) << 32) |
         static_cast<unsigned>(sgpr(static_cast<int>(v)));
}

// A pointer to the kernel's arguments the compiler cannot see through: the
// loads made through it stay where they are written.  The unit loop reads its
// set-up and epilogue arguments this way, so they are re-loaded per unit
// instead of being hoisted out of the loop and kept live in SGPRs across the
// hot loop (which spilled SGPRs into VGPR lanes: 76 -> 102 VGPRs).
typedef const struct KArgs __attribute__((address_space(4)))* KArgsP;
__device__ __forceinline__ KArgsP kargs_opaque() {
  KArgsP p = (KArgsP)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// ------------------------------------------------------------- kernel ----
enum { SRC_LDS = 1, SRC_SCALAR = 2 };
enum { SCAN_SIMPLE = 0, SCAN_GROUP4 = 1, SCAN_PK4 = 2, SCAN_BVH = 3, SCAN_BVHWW = 4, SCAN_BVHQ = 5, SCAN_BVHO = 6,
       SCAN_BVHS = 7 /* sorted_kernel: 4-body leaves, 8 x 16 tiles, 512 threads */,
       SCAN_BVHQ7 = 8 /* BVHQ in a compact LDS image: seven workgroups per CU (variant 22) */ };
// the traversal variants (BVHQ: ordered traversal of the 4-body-leaf tree)
constexpr bool is_bvh_scan(int scan) { return (scan >= SCAN_BVH && scan <= SCAN_BVHO) || scan == SCAN_BVHQ7; }
// the 4-body-leaf ordered traversals: BVHQ, and BVHQ7 = the same walk with
// a compact LDS image (u8 stack of node indices, u32 pixel sums, an 8-byte
// pixel table): 23.0 KB for C1, seven workgroups per CU
constexpr bool is_q(int scan) { return scan == SCAN_BVHQ || scan == SCAN_BVHQ7; }
// body pairs per leaf of the tree a traversal variant walks
constexpr int leaf_pairs(int scan) { return scan == SCAN_BVHO ? 4 : is_q(scan) ? 2 : 1; }

// two bodies side by side for packed fp32 math (v_pk_*_f32: one IEEE op per half)
typedef float f2 __attribute__((ext_vector_type(2)));
// LDS (address space 3) pointers: 32-bit addresses, ds_read with immediate offsets
typedef const char __attribute__((address_space(3)))* LdsC;
typedef const f2 __attribute__((address_space(3)))* LdsF2;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef const f4v __attribute__((address_space(3)))* LdsF4;
typedef const long long __attribute__((address_space(3)))* LdsI64;
__device__ __forceinline__ unsigned lds_addr(const void* p) { return static_cast<unsigned>((uintptr_t)(LdsC)p); }
struct alignas(16) Pair {
  f2 x, y, z, w;   // centres and -r^2 of bodies 2p and 2p+1
};
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// v_fma_f32 in its three-address (VOP3) form: the compiler's v_fmac_f32 needs
// a v_mov copy when the addend stays live (a loop-invariant plane offset)
__device__ __forceinline__ float fma3(float a, float b, float c) {
  float r;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ f2 bc_lo(f2 v) { return __builtin_shufflevector(v, v, 0, 0); }
__device__ __forceinline__ f2 bc_hi(f2 v) { return __builtin_shufflevector(v, v, 1, 1); }

// BVH node as the kernel reads it (= rtclj::BvhNode, bvh.h): per axis the
// (child0, child1) pairs (min, max, min); a ray's (near, far) planes are the
// pairs at index s, s + 1 with s = 1 if 1/u < 0, else 0
struct alignas(16) KNode {
  f2 x[3], y[3], z[3];
  int c0, c1;
};
static_assert(sizeof(KNode) == 80, "KNode layout");

// The pool tile: 8 x 8 pixels.  (The 8-body-leaf traversal ran 8 x 4 tiles
// while its 256-thread workgroups were LDS-bound at 5 per CU; in 512-thread
// workgroups, 3 per CU by registers, the 8 x 8 pool's longer workgroup
// lifetimes were worth 1 %: C4 4.95 vs 4.99 s, profiles/r05/c4_tile/.  C4
// now runs the compact 4-body image in 16-wave workgroups, variant 26.)
constexpr int kTile = 8;
// the 4-body tree's leaf record in LDS: two pairs and their index pairs
constexpr int kLeafRecBytes = 80;
constexpr int kPoolPx = kTile * kTile;
constexpr int tile_rows(int scan) { return scan == SCAN_BVHS ? 16 : kTile; }

// Waves per SIMD the register allocator must leave room for: seven for the
// compact image (72 VGPRs; 23.0 KB of LDS fits 7 workgroups per CU), six
// for the 4-body traversal (80 VGPRs; 26.6 KB) and for the 8-body-leaf one
// (8-wave workgroups, 3 per CU by registers; 34.4 KB of LDS each).
// Without the bound the unit loop's longer-lived uniform values (SGPRs at
// their limit, copied into VGPRs) take it to ~100 VGPRs and four waves; with
// it, a few of them spill to scratch outside the hot loop.  The compact
// image's 16-wave workgroups (variant 26, C4) ask for 8: 64 VGPRs and 16
// bytes of scratch under the default scheduler, 62 and none under the
// register-pressure trackers it is compiled with (trace_w16.hip).  HIP passes
// __launch_bounds__'s second argument on as amdgpu_waves_per_eu: a count of
// waves per SIMD, whatever the workgroup's size.  The 8-body-leaf kernel asks
// for 3 (a register budget of 168): it allocates 75 VGPRs either way, and
// the schedule made under 3 is C4's faster one -- 4.996 vs 5.019 s with 6
// asked, same box (profiles/r05/launch_bound/).
constexpr int min_waves(int scan, bool stats, int nw = 4) {
  return stats ? 1 : scan == SCAN_BVHQ ? 6 : scan == SCAN_BVHQ7 ? (nw == 16 ? 8 : 7) : scan == SCAN_BVHO ? 3 : 1;
}

// The diagnostic scans (SCAN_SIMPLE, SCAN_PK4: the linear scans of the A/B
// variants 1-3, 8-10), defined in trace_diag.hip: the product library never
// instantiates them.
template <int SRC, int SCAN, class F>
__device__ void diag_scan(const struct KArgs& a, const float4* s_geo, float ox, float oy, float oz, float ux,
                          float uy, float uz, F&& consider);

// NW waves per workgroup (4; 8 or 16 for trees whose large LDS image more
// waves share: C4's 1000-body tree as the compact 4-body image, two 16-wave
// workgroups = 8 waves per SIMD, where 4-wave workgroups fit 3 per CU)
// THT: the pool's tile rows (0: tile_rows(SCAN); variant 28 runs 22's
// compact image on 8 x 4-pixel pools, for launches of few 8 x 8 tiles)
template <int SRC, int SCAN, bool STATS = false, int NW = 4, int THT = 0, bool SWEEP = false>
__global__ __launch_bounds__(64 * NW, min_waves(SCAN, STATS, NW)) void trace_kernel(const KArgs a) {
  constexpr int NT = 64 * NW;   // threads
  // The sample pool: the workgroup's 8 x 8 pixels x spp samples are the
  // indices j in [0, npx * spp), sample-major (j -> pixel j % npx, sample
  // j / npx: the lanes ending paths together add into different pixels'
  // sums).  A lane whose path ends takes the next index from an LDS counter
  // (one ds_add per wave event, then an mbcnt prefix).  The colour sums are
  // integers per pixel and channel in LDS (u64, ds_add_u64; the compact
  // variants: u32 with counted wraps, below): order-free.
  //
  // The workgroup's unit: a whole tile (owner) or one sample split of a
  // tile, or -- a helper -- a share of another workgroup's tile (DESIGN.md
  // §3.1).  Each wave runs its samples from a batch of consecutive pool
  // indices it claimed: from s_pool_next, or for a shared tile from the
  // tile's word.
  __shared__ int s_pool_next;
  __shared__ int s_cnt;               // samples this workgroup claimed (shared tiles)
  __shared__ int s_join;              // helpers the owner's claims saw (> 0: the tile was shared)
  __shared__ int s_unit[2];           // a helper's tile and first index
  __shared__ unsigned long long s_best;
  __shared__ unsigned long long s_segs;   // the workgroup's segments (counters)
  __shared__ int s_last;
  // drain compaction: per wave the paths it posted and how many were taken;
  // the waves still in the hot loop
  __shared__ int s_mb_post[NW], s_mb_take[NW], s_alive, s_mb_avail;
  // per wave: post when down to this many paths (0: posted once already; -1: off)
  __shared__ int s_mb_lim[NW];
  constexpr int TH = THT ? THT : tile_rows(SCAN);   // tile rows
  constexpr int NPX = kTile * TH;       // pool pixels
  // the pool's pixel sums: u32 in the compact variants (the host runs them
  // only when a sample's colour is <= 1 per channel and spp < 65536: a
  // sample adds at most 2^24 per channel, so a channel's sum wraps past 2^32
  // at most spp / 256 < 256 times, and the wraps are counted in a byte per
  // channel, s_carry, when spp > 255), u64 otherwise
  using AccT = std::conditional_t<SCAN == SCAN_BVHQ7, unsigned, unsigned long long>;
  __shared__ AccT s_acc[NPX * 3];
  uint64_t st_iter = 0, st_lanes = 0, st_sph = 0, st_blk = 0, st_blk_lanes = 0;
  uint64_t st_trav = 0, st_trav_lanes = 0;   // BVH: wave-level traversal iterations, lanes in them
  uint64_t st_leafw = 0, st_consw = 0;        // BVH: wave-level leaf passes, exact-test passes
  uint64_t st_ball = 0, st_disk = 0;          // wave-level rejection-loop trips (random-unit, disk)
  uint64_t st_fl = 0;                         // executed fp32 flops of this lane (fma = 2)
  uint64_t st_fresh = 0, st_fresh_lanes = 0;  // wave-level camera-sample blocks, lanes in them
  uint64_t st_diel = 0, st_diel_lanes = 0;    // wave-level dielectric blocks, lanes in them
  uint64_t st_lm = 0, st_lm_lanes = 0;        // wave-level lambertian/metal blocks, lanes in them
  // wave-level events of the loop's bookkeeping: colour sums
  // added, refills, batch claims, drain-phase checks (batches spent)
  uint64_t st_sums = 0, st_refill = 0, st_claim = 0, st_drain = 0;
  uint64_t st_c_cam = 0, st_c_scan = 0, st_c_shade = 0, st_c_acc = 0, st_ts = 0;  // clock split
  uint64_t st_t0 = 0;
  if (STATS || a.tile_cost || a.dbgw) st_t0 = __builtin_amdgcn_s_memrealtime();
  extern __shared__ __attribute__((aligned(16))) float4 s_geo[];
  const int n = a.n;
  const int lane = threadIdx.x & 63;
  const int unit = static_cast<int>(blockIdx.x);
  // (set-up and epilogue arguments through an opaque pointer: re-loaded
  // where used, not kept in SGPRs across the hot loop)
  const KArgsP ka = kargs_opaque();
  const bool own = SWEEP || unit < ka->n_units;
  // the sweep: the records the launch before wrote; workgroup u starts on
  // records [u * NT, (u + 1) * NT)
  int xpool = 0;
  if constexpr (SWEEP) {
    xpool = static_cast<int>(__hip_atomic_load(&ka->xq_n[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (unit * NT >= xpool) return;
  }
  // samples of whole tile t (its in-image pixels x spp)
  auto tile_pool = [&](KArgsP kp, int t) {
    const int ty = t / kp->tiles_x, tx = t - ty * kp->tiles_x;
    const int w = max(0, min(kTile, kp->width - tx * kTile)), h = max(0, min(TH, kp->rows_out - ty * TH));
    return kp->spp > 0 && kp->max_depth > 0 ? w * h * kp->spp : 0;
  };
  if (!own) {
    // ---- a helper: pick a tile still running, join it ----
    if (!ka->word) return;
    if (threadIdx.x == 0) {
      s_best = 0ull;
      s_unit[0] = -1;
    }
    __syncthreads();
    // each thread looks at 2 owner entries of a window of 512 that starts at
    // a per-helper offset (atomic reads: entries change as owners start
    // tiles); key = (unclaimed << 32) | tile, the most unclaimed wins
    const int M = ka->n_owner;
    const int w0 = static_cast<int>(mix32(static_cast<uint32_t>(unit)) % static_cast<uint32_t>(M));
    unsigned long long key = 0;
    for (int i = 0; i < (512 + NT - 1) / NT; ++i) {
      int w = w0 + static_cast<int>(threadIdx.x) + NT * i;
      w = w >= M ? w - M : w;
      w = w >= M ? w % M : w;
      const int t = xload32(&ka->owner[w]);
      if (t >= 0) {
        const unsigned long long wd = xload64(&ka->word[t]);
        const int fr = word_epoch(wd) == ka->epoch ? tile_pool(ka, t) - static_cast<int>(static_cast<unsigned>(wd)) : 0;
        const unsigned long long k2 = (static_cast<unsigned long long>(fr) << 32) | static_cast<unsigned>(t);
        key = (fr >= ka->steal_min && k2 > key) ? k2 : key;
      }
    }
    key = wave_max_u64(key);
    if (lane == 0 && key) __hip_atomic_fetch_max(&s_best, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    const unsigned long long best_key = sgpr64(s_best);
    if (best_key == 0) return;   // nothing worth joining in the window
    if (threadIdx.x == 0) {
      // join: one atomic counts the helper in and claims its lanes' first indices
      const int t = static_cast<int>(static_cast<unsigned>(best_key));
      const int P = tile_pool(ka, t);
      const unsigned long long wd = __hip_atomic_fetch_add(&ka->word[t], (1ull << 32) + NT, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
      const int g = static_cast<int>(static_cast<unsigned>(wd));
      if (word_epoch(wd) == ka->epoch && g < P) {   // (another epoch: a spent word of an earlier launch)
        const int got = min(P - g, NT);
        __hip_atomic_fetch_add(&ka->stealc[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&ka->stealc[1], static_cast<unsigned long long>(got), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        s_unit[0] = t;
        s_unit[1] = g;
        s_cnt = got;
      }
    }
    __syncthreads();
    if (sgpr(s_unit[0]) < 0) return;   // spent meanwhile
  }
  // the scene image (a thief only once it has samples to run)
  if constexpr (SRC == SRC_LDS) {
    if constexpr (is_q(SCAN)) {
      // the 4-body tree's inner-child refs (node byte offsets in the blob)
      // become LDS addresses as they are copied: a node step then reads its
      // child refs at ref + 72 and its planes at ref + the ray's plane
      // offsets, with no base added (float4 4 of each 80-byte node holds
      // c0, c1 in .z, .w; leaf refs are negative and stay)
      // The leaves are laid out as records: a leaf's four bodies as float4s
      // (cx, cy, cz, -r^2) and their indices (16 B) side by side, 80 B, so a
      // leaf pass and its exact passes read everything from one address; a
      // leaf ref ~p (p = its first pair, even) becomes ~(the record's LDS address).
      const int nb0 = static_cast<int>(lds_addr(s_geo));
      const int nodes_f4 = a.bvh_off_pairs >> 4;
      const int pairs_f4 = (a.bvh_off_pidx - a.bvh_off_pairs) >> 4;   // 2 per pair
      const int rec0 = nb0 + (nodes_f4 << 4);
      for (int i = threadIdx.x; i < a.bvh_blob_f4; i += NT) {
        float4 v = a.bvh_blob[i];
        int d = i;
        if (i < nodes_f4) {
          if (i % 5 == 4) {
            const int r0 = __float_as_int(v.z), r1 = __float_as_int(v.w);
            // (the compact variant's inner refs: node indices, for its u8 stack)
            const int in0 = SCAN == SCAN_BVHQ7 ? r0 / 80 : r0 + nb0, in1 = SCAN == SCAN_BVHQ7 ? r1 / 80 : r1 + nb0;
            v.z = __int_as_float(r0 >= 0 ? in0 : ~(rec0 + (~r0 >> 1) * kLeafRecBytes));
            v.w = __int_as_float(r1 >= 0 ? in1 : ~(rec0 + (~r1 >> 1) * kLeafRecBytes));
          }
        } else if (i < nodes_f4 + pairs_f4) {   // pair k / 2, half k % 2
          const int k = i - nodes_f4, pr = k >> 1;
          // (per-body float4s: half 0 holds the pair's x and y, half 1 z and w)
          float* rb = reinterpret_cast<float*>(s_geo) + 4 * (nodes_f4 + (pr >> 1) * 5 + (pr & 1) * 2) + 2 * (k & 1);
          rb[0] = v.x;
          rb[4] = v.y;
          rb[1] = v.z;
          rb[5] = v.w;
          continue;
        } else {                                 // the indices of pairs 2k, 2k + 1
          d = nodes_f4 + (i - nodes_f4 - pairs_f4) * 5 + 4;
        }
        s_geo[d] = v;
      }
    } else if constexpr (is_bvh_scan(SCAN)) {
      for (int i = threadIdx.x; i < a.bvh_blob_f4; i += NT) s_geo[i] = a.bvh_blob[i];
    } else {
      const float4* src = SCAN == SCAN_PK4 ? reinterpret_cast<const float4*>(a.geo2) : a.geo;
      for (int i = threadIdx.x; i < a.n_pad; i += NT) s_geo[i] = src[i];
    }
  }
  uint32_t segs = 0;
  if (STATS || ka->tile_cost) st_t0 = __builtin_amdgcn_s_memrealtime();
  // BVH traversal stack: bvh_stack node refs per lane, [entry][lane] (no bank conflicts)
  // (u8 entries for the 8-body-leaf traversal, whose trees the host caps at
  // 256 nodes: with its u16 body indices this keeps a 1000-body scene's
  // image under the 32 KB that 5 workgroups per CU allow)
  using StackT = std::conditional_t<SCAN == SCAN_BVHO || SCAN == SCAN_BVHQ7, unsigned char, unsigned short>;
  StackT* s_stack = reinterpret_cast<StackT*>(
      reinterpret_cast<char*>(s_geo) + (SRC == SRC_LDS ? ka->bvh_blob_f4 * 16 : 0));

  // the unit: a whole tile or one sample split of a tile at the order's end
  // (own), or a stolen sample range [first, s_lim) of a whole tile
  int tile = 0, split_ix = 0, first = 0, nsplit = 1;
  bool split = false;
  if constexpr (SWEEP) {
    first = unit * NT;
  } else if (own) {
    int pos = unit;
    split = unit >= ka->n_whole;
    if (split && ka->unit_tab) {   // a cost-balanced split
      const int2 u = ka->unit_tab[unit - ka->n_whole];
      if (u.x < 0) return;   // (the plan used fewer units than the grid has)
      tile = u.x;
      split_ix = u.y & 255;
      nsplit = u.y >> 8;
    } else {
      if (split) {
        const int v = unit - ka->n_whole;
        const int t = v / ka->split;
        pos = ka->n_whole + t;
        split_ix = v - t * ka->split;
        nsplit = ka->split;
      }
      tile = ka->tile_order ? ka->tile_order[pos] : pos;
    }
  } else {
    tile = sgpr(s_unit[0]);
    first = sgpr(s_unit[1]);
  }
  const int tby = tile / ka->tiles_x, tbx = tile - tby * ka->tiles_x;
  // the tile's in-image part, vw x vh pixels; pool pixel q at (q % vw, q / vw)
  const int qx0 = tbx * kTile, qy0 = tby * TH;
  const int vw = max(0, min(kTile, ka->width - qx0));
  const int vh = max(0, min(TH, ka->rows_out - qy0));
  const int npx = vw * vh;

  // compacted output row -> global image row (interleaved row tiles)
  auto image_row = [&](int r) {
    if (a.tile_step > 0) {
      const int t = div_magic(r, a.rt_magic);
      return a.row_begin + (a.tile_first + t * a.tile_step) * a.row_tile + (r - t * a.row_tile);
    }
    return a.row_begin + r;
  };
  auto pixel_key = [&](int x, int y) {
    return mix32(a.key ^ mix32(static_cast<uint32_t>(y) * static_cast<uint32_t>(a.width) + static_cast<uint32_t>(x)));
  };
  const float cx = a.cam[0], cy = a.cam[1], cz = a.cam[2];

  // the unit's samples [k0, k0 + cnt) of each pixel
  const int k0 = split ? static_cast<int>(static_cast<int64_t>(split_ix) * ka->spp / nsplit) : 0;
  const int cnt = split ? static_cast<int>(static_cast<int64_t>(split_ix + 1) * ka->spp / nsplit) - k0 : ka->spp;
  // pool index j -> (pixel q = j % npx, sample k0 + j / npx); the next free
  // index is `base`.  j / npx by a 64-bit magic (exact for every 32-bit j);
  // q / vw by multiply-high (exact: q < 64, vw <= 8)
  const int pool = SWEEP ? xpool : (cnt > 0 && ka->max_depth > 0) ? npx * cnt : 0;
  const uint32_t mag_vw = vw > 0 ? 0xffffffffu / static_cast<uint32_t>(vw) + 1u : 0u;
  const uint32_t mag16_vw = vw > 0 ? (65536u + static_cast<uint32_t>(vw) - 1u) / static_cast<uint32_t>(vw) : 0u;
  const uint64_t npx_magic = npx > 1 ? ~0ull / static_cast<uint64_t>(npx) + 1ull : 0ull;
  // the unit's LDS state.  The owner of a whole tile of more than 512
  // samples shares it: the tile's word with this launch's epoch, its lanes'
  // first 256 indices claimed and no helper, then its owner entry.  (No
  // order is needed between the two: a helper that reads the word before it
  // lands sees another epoch and leaves it alone.  done[tile] is 0 already:
  // zeroed at allocation and by the workgroup that completes a shared tile.)
  // Only the units dispatched in the launch's last rounds (unit >= share_from)
  // publish: an earlier unit ends while later ones still start, so no helper
  // would ever join it, and its claims would all be HBM atomics (C4: ~60 per
  // tile, 3 GB of WRITE_SIZE per launch when every unit published).
  const bool shared_tile = !SWEEP && ka->word && !split && (!own || (pool > 512 && unit >= ka->share_from));
  // where the waves claim their batches: the shared tile's word, else (NULL)
  // the workgroup's s_pool_next
  unsigned long long* const src = shared_tile ? ka->word + tile : nullptr;
  // (batch_max 0: by the pool, 1/48 of it, 128 .. 1024)
  const int kc_batch_max = ka->batch_max > 0 ? ka->batch_max : min(1024, max(kShareBatch, (pool / 48) & ~63));
  if (threadIdx.x == 0) {
    if (own && shared_tile) {
      __hip_atomic_exchange(&ka->word[tile], (static_cast<unsigned long long>(ka->epoch) << 48) | static_cast<unsigned long long>(NT),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(&ka->owner[unit % ka->n_owner], tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_cnt = NT;
    }
    s_join = own ? 0 : 1;
    s_segs = 0ull;
    s_pool_next = NT;
    s_alive = NW;
    s_mb_avail = 0;   // (posted, not yet taken: a hint for the waves' exits to the step)
  }
  if (threadIdx.x < NW) {
    s_mb_post[threadIdx.x] = 0;
    s_mb_take[threadIdx.x] = 0;
    s_mb_lim[threadIdx.x] = ka->compact > 0 ? ka->compact : -1;
  }
  if (threadIdx.x < NPX * 3) s_acc[threadIdx.x] = 0;
  // the tile's pixel table (4-body-leaf traversal): per pool pixel its RNG
  // key and coordinates, so a camera sample costs one LDS read instead of
  // the index arithmetic and two hashes (the 8-body-leaf traversal, whose
  // workgroups are register-bound, computes them instead)
  constexpr bool kPixelTable = is_q(SCAN) && !SWEEP;
  // (the compact variant: the keys alone, 4 bytes a pixel, and the image row
  // of each of the tile's rows as a float; a pixel's column is q mod vw)
  constexpr bool kCompactPx = SCAN == SCAN_BVHQ7;
  __shared__ std::conditional_t<kCompactPx, uint32_t, float4> s_px[kPixelTable ? NPX : 1];
  __shared__ float s_prow[kCompactPx ? TH : 1];
  if constexpr (kPixelTable) {
    const int t = static_cast<int>(threadIdx.x);
    if (t < npx) {
      const int qy = vw == 1 ? t : static_cast<int>(__umulhi(static_cast<uint32_t>(t), mag_vw));
      const int px = qx0 + (t - qy * vw);
      const int gy = image_row(qy0 + qy);
      if constexpr (kCompactPx) {
        s_px[t] = pixel_key(px, gy);
        if (px == qx0) s_prow[qy] = static_cast<float>(gy);
      } else {
        s_px[t] = make_float4(__uint_as_float(pixel_key(px, gy)), static_cast<float>(px), static_cast<float>(gy), 0.0f);
      }
    }
  }
  // The compact variant's u32 pixel sums, when a pixel may get more than 255
  // samples (spp > 255): a sum's wraps past 2^32 counted per channel in a
  // byte of s_carry (a sample adds less than 2^32, so at most one wrap; with
  // every colour <= 1 per channel a channel wraps at most spp / 256 < 256
  // times for spp < 65536, compact_ok): its total is carry * 2^32 + sum.
  __shared__ uint32_t s_carry[kCompactPx ? NPX * 3 / 4 : 1];
  if constexpr (kCompactPx) {
    if (threadIdx.x < NPX * 3 / 4) s_carry[threadIdx.x] = 0u;
  }
  __syncthreads();
  // the wave's batch [wb, we) of pool indices (wave-uniform; empty at first:
  // the lanes start on first + threadIdx.x)
  int wb = 0, we = 0;
  int j = first + static_cast<int>(threadIdx.x), q = 0, k = 0;
  bool active = j < pool;
  // With compaction (kCompact, below) j is the lane's whole state in the
  // loop: j >= 0 a sample not started yet (pool index j), -1 a path in
  // progress, -2 no path, -3 a path taken out of the loop to the
  // compaction step; the loop carries no flag (one live across the step
  // would be a VGPR 0/1 tested every iteration)
  if (!active) j = -2;

  // path state
  uint32_t st = 0;
  float ox = 0, oy = 0, oz = 0, dx = 0, dy = 0, dz = 0;
  float tr = 1, tg = 1, tb = 1;
  int rem = 0;
  int last = -1;   // body the current ray leaves (-1: camera ray)
  bool fresh = true;


  // Drain compaction keeps every lane of a wave in the loop
  // once its batches are spent (a lane without a path skips the body; the
  // step after it may give it a path a sibling wave posted); the wave leaves
  // when none of its lanes has one
  constexpr bool kCompact = is_bvh_scan(SCAN);
  const int wv = static_cast<int>(threadIdx.x >> 6);
  auto mb_word = [&](int d, int f, int p, int P) -> uint32_t* {
    constexpr int SZ = static_cast<int>(sizeof(StackT));
    constexpr int W = 16 * SZ;   // words per stack row per wave
    const int i = f * P + p;
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_stack) + (i / W) * NT * SZ + d * 64 * SZ +
                                       (i % W) * 4);
  };
  auto lds_load = [](int* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); };
  // Once the wave's batches are spent (wave-uniform): with no path left it
  // counts itself out of s_alive, or with a few it posts them (unless it has
  // posted once before) and counts itself out; a wave that stays takes what
  // the siblings posted into its free lanes.  Each post lands before its
  // wave counts out, so a wave still counted in sees it; the last wave out
  // finds every sibling gone -- it takes what is left, keeps its own paths,
  // and counts itself back in.
  auto compact_step = [&]() {
    RT_MARK("compact_step");
    // (the wave index in an SGPR here: its slots' addresses rebuilt in this
    // cold step, not held in a VGPR -- at 72 VGPRs one was spilled to scratch)
    const int wu = static_cast<int>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    const int P = kargs_opaque()->mb_paths;
    const int leader = static_cast<int>(__builtin_amdgcn_readfirstlane(lane));
    const uint64_t live = __ballot(active);
    const int left = static_cast<int>(__popcll(live));
    bool out = false;   // counted out, and the last wave to do so
    bool post = false;
    if constexpr (!SWEEP) {
      // path export (KArgs::xq): the wave's paths out to HBM records, for
      // the sweep launch; the wave leaves
      uint4* const xq = kargs_opaque()->xq;
      if (xq) {
        if (left > 0) {
          int base = 0;
          if (lane == leader) base = static_cast<int>(atomicAdd(&kargs_opaque()->xq_n[0], static_cast<unsigned>(left)));
          base = __builtin_amdgcn_readlane(base, leader);
          const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(live >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(live), 0u)));
          if (active) {
            // the pixel: compacted row x width + column (q / vw as the camera sample's multiply-high)
            const int qy = static_cast<int>(__umul24(static_cast<uint32_t>(q), mag16_vw) >> 16);
            const int pix = (qy0 + qy) * kargs_opaque()->width + qx0 + (q - qy * vw);
            uint4* r = xq + 4 * static_cast<size_t>(base + rank);
            r[0] = make_uint4(__float_as_uint(ox), __float_as_uint(oy), __float_as_uint(oz), __float_as_uint(dx));
            r[1] = make_uint4(__float_as_uint(dy), __float_as_uint(dz), __float_as_uint(tr), __float_as_uint(tg));
            r[2] = make_uint4(__float_as_uint(tb), st, static_cast<uint32_t>(pix), static_cast<uint32_t>(rem));
            reinterpret_cast<uint32_t*>(r + 3)[0] = static_cast<uint32_t>(last);
          }
        }
        if (lane == leader) atomicAdd(&s_alive, -1);
        active = false;
        j = -2;
        return;
      }
    }
    if (left > 0 && left <= sgpr(lds_load(&s_mb_lim[wu]))) {
      post = sgpr(lds_load(&s_alive)) > 1;
      // posting now; or alone (no sibling will ever take them): not again
      if (lane == leader) __hip_atomic_store(&s_mb_lim[wu], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (left == 0 || post) {
      if (post) {
        const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(live >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(live), 0u)));
        if (active) {
          *mb_word(wu, 0, rank, P) = __float_as_uint(ox);
          *mb_word(wu, 1, rank, P) = __float_as_uint(oy);
          *mb_word(wu, 2, rank, P) = __float_as_uint(oz);
          *mb_word(wu, 3, rank, P) = __float_as_uint(dx);
          *mb_word(wu, 4, rank, P) = __float_as_uint(dy);
          *mb_word(wu, 5, rank, P) = __float_as_uint(dz);
          *mb_word(wu, 6, rank, P) = __float_as_uint(tr);
          *mb_word(wu, 7, rank, P) = __float_as_uint(tg);
          *mb_word(wu, 8, rank, P) = __float_as_uint(tb);
          *mb_word(wu, 9, rank, P) = st;
          *mb_word(wu, 10, rank, P) = static_cast<uint32_t>(q);
          *mb_word(wu, 11, rank, P) = static_cast<uint32_t>(rem);
          *mb_word(wu, 12, rank, P) = static_cast<uint32_t>(last);
        }
      }
      int old = 0;
      if (lane == leader) {
        if (post) {
          __hip_atomic_store(&s_mb_post[wu], left, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          atomicAdd(&s_mb_avail, left);
        }
        old = __hip_atomic_fetch_add(&s_alive, -1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        // the last one out withdraws its post (no sibling is left to take any of it)
        if (post && old <= 1) {
          __hip_atomic_store(&s_mb_post[wu], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          atomicAdd(&s_mb_avail, -left);
        }
      }
      old = __builtin_amdgcn_readlane(old, leader);
      if (old > 1) {
        active = false;   // (a post's paths are the siblings' now)
        j = -2;
        return;
      }
      out = true;
    }
    // free lanes take the siblings' posts, in rank order
    uint64_t freem = ~live;
    bool took = false;
#pragma unroll 1
    for (int d = 0; d < NW && freem; ++d) {
      if (d == wu) continue;
      const int posted = sgpr(lds_load(&s_mb_post[d]));
      if (posted <= sgpr(lds_load(&s_mb_take[d]))) continue;
      const int want = static_cast<int>(__popcll(freem));
      int t0 = 0;
      if (lane == leader) t0 = atomicAdd(&s_mb_take[d], want);
      t0 = __builtin_amdgcn_readlane(t0, leader);
      const int got = min(want, posted - t0);
      if (got <= 0) continue;
      if (lane == leader) atomicAdd(&s_mb_avail, -got);
      const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(freem >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(freem), 0u)));
      const bool mine = ((freem >> lane) & 1ull) && rank < got;
      if (mine) {
        const int p = t0 + rank;
        ox = __uint_as_float(*mb_word(d, 0, p, P));
        oy = __uint_as_float(*mb_word(d, 1, p, P));
        oz = __uint_as_float(*mb_word(d, 2, p, P));
        dx = __uint_as_float(*mb_word(d, 3, p, P));
        dy = __uint_as_float(*mb_word(d, 4, p, P));
        dz = __uint_as_float(*mb_word(d, 5, p, P));
        tr = __uint_as_float(*mb_word(d, 6, p, P));
        tg = __uint_as_float(*mb_word(d, 7, p, P));
        tb = __uint_as_float(*mb_word(d, 8, p, P));
        st = *mb_word(d, 9, p, P);
        q = static_cast<int>(*mb_word(d, 10, p, P));
        rem = static_cast<int>(*mb_word(d, 11, p, P));
        last = static_cast<int>(*mb_word(d, 12, p, P));
        active = true;
        fresh = false;
        j = -1;
      }
      freem &= ~__ballot(mine);
      took = true;
    }
    // the last wave out stays in the loop if it has paths
    if (out && (took || left > 0) && lane == leader) atomicAdd(&s_alive, 1);
  };
  // one segment of the wave's active lanes' paths, then their refill (with
  // compaction, j's states above; `active` and `fresh` are only the step's and
  // the other variants')
  auto iteration = [&]() {
    bool done = false;
    if constexpr (STATS) st_ts = stamp();
    if constexpr (STATS) {  // counted once per wave event, by its first active lane
      const uint64_t ex = __builtin_amdgcn_read_exec();
      if (lane == __ffsll(static_cast<long long>(ex)) - 1) {
        ++st_iter;
        st_lanes += __popcll(ex);
      }
    }
    RT_MARK("iteration");
    if (kCompact ? j >= 0 : fresh) {
      RT_MARK("camera");
      if constexpr (SWEEP) {   // a record of the launch before: the path as it left its wave
        const uint4* r = kargs_opaque()->xq + 4 * static_cast<size_t>(j);
        const uint4 r0 = r[0], r1 = r[1], r2 = r[2];
        const uint32_t r3 = reinterpret_cast<const uint32_t*>(r + 3)[0];
        ox = __uint_as_float(r0.x);
        oy = __uint_as_float(r0.y);
        oz = __uint_as_float(r0.z);
        dx = __uint_as_float(r0.w);
        dy = __uint_as_float(r1.x);
        dz = __uint_as_float(r1.y);
        tr = __uint_as_float(r1.z);
        tg = __uint_as_float(r1.w);
        tb = __uint_as_float(r2.x);
        st = r2.y;
        q = static_cast<int>(r2.z);
        rem = static_cast<int>(r2.w);
        last = static_cast<int>(r3);
        fresh = false;
        j = -1;
      } else {
      if constexpr (STATS) {
        const uint64_t ex = __builtin_amdgcn_read_exec();
        if (lane == __ffsll(static_cast<long long>(ex)) - 1) {
          ++st_fresh;
          st_fresh_lanes += __popcll(ex);
        }
      }
      // pool index -> (pixel, sample), sample-major: the lanes ending paths
      // together add into different pixels' sums
      k = div_magic(j, npx_magic);
      q = j - k * npx;
      uint32_t pk;
      float fpx, fgy;
      if constexpr (kPixelTable && kCompactPx) {
        pk = s_px[q];
        // q / vw as (q * ceil(2^16 / vw)) >> 16: exact for q < 64, vw <= 8, vw = 1 included
        const int qy = static_cast<int>(__umul24(static_cast<uint32_t>(q), mag16_vw) >> 16);
        fpx = static_cast<float>(qx0 + (q - qy * vw));
        fgy = s_prow[qy];
      } else if constexpr (kPixelTable) {   // the pixel's key and coordinates from the tile's table
        const float4 pt = s_px[q];
        pk = __float_as_uint(pt.x);
        fpx = pt.y;
        fgy = pt.z;
      } else {
        const int qy = vw == 1 ? q : static_cast<int>(__umulhi(static_cast<uint32_t>(q), mag_vw));
        const int px = qx0 + (q - qy * vw);
        const int gy = image_row(qy0 + qy);
        pk = pixel_key(px, gy);
        fpx = static_cast<float>(px);
        fgy = static_cast<float>(gy);
      }
      // ---- compute-pixel, one sample (raytracing.clj:144-151) ----
      st = mix32(pk + static_cast<uint32_t>(a.sample_begin + k0 + k) * 0x9e3779b9u);
      if (st == 0) st = 0x6d2b79f5u;
      // xi - 0.5 is exact in fp32: one fma of the 24-bit integer, the same bits
      const float fx = fpx + rng_centered(st);
      const float fy = fgy + rng_centered(st);
      const float sx = fmaf(a.cam[9], fy, fmaf(a.cam[6], fx, a.cam[3]));
      const float sy = fmaf(a.cam[10], fy, fmaf(a.cam[7], fx, a.cam[4]));
      const float sz = fmaf(a.cam[11], fy, fmaf(a.cam[8], fx, a.cam[5]));
      if (a.defocus) {
        // defocus-disk-sample + random-in-unit-disk (raytracing.clj:89-93, vec3a.clj:81-86)
        float qx, qy2;
        if (a.sampler & RT_SAMPLER_DISK) {
          disk_direct<STATS>(st, qx, qy2, &st_disk, &st_fl);
          RT_MARK("camera");
        } else {
          RT_MARK("rejection_disk");
          do {
            if constexpr (STATS) {
              wave_event(st_disk);
              st_fl += 7;   // 2 x (2 xi - 1) + |q|^2
            }
            qx = rng_sym(st);
            qy2 = rng_sym(st);
          } while (!(fmaf(qy2, qy2, qx * qx) < 1.0f));
        }
        if constexpr (STATS) st_fl += 12;
        ox = fmaf(a.cam[15], qy2, fmaf(a.cam[12], qx, cx));
        oy = fmaf(a.cam[16], qy2, fmaf(a.cam[13], qx, cy));
        oz = fmaf(a.cam[17], qy2, fmaf(a.cam[14], qx, cz));
      } else {
        ox = cx;
        oy = cy;
        oz = cz;
      }
      if constexpr (STATS) st_fl += 21;   // jitter 2 x (fma + add), sample point 3 x 2 fma, d = s - o
      dx = sx - ox;
      dy = sy - oy;
      dz = sz - oz;
      tr = tg = tb = 1.0f;
      rem = a.max_depth;
      last = -1;
      fresh = false;
      if constexpr (kCompact) j = -1;
      }
    }


    if constexpr (STATS) {
      const uint64_t t = stamp();
      st_c_cam += t - st_ts;
      st_ts = t;
    }
    // ---- one ray-color level: hit-anything over all bodies ----
    RT_MARK("setup");
    --rem;
    ++segs;
    // |d| and 1/|d| (vec3a/unit as d * (1/|d|)), both correctly rounded; one
    // range test for the pair: a finite |d|^2 >= 2^-96 puts |d| in
    // [2^-48, 2^64), inside rcp_rn_normal's range
    const float len2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    float len, il;
    if (__builtin_expect(len2 >= 0x1p-96f && len2 <= 0x1.fffffep127f, 1)) {
      len = sqrt_rn_normal(len2);
      il = rcp_rn_normal(len);
    } else {
      RT_MARK("cold");
      len = sqrt_rn(len2);
      il = rcp_rn(len);
    }
    float ux = dx * il, uy = dy * il, uz = dz * il;
    const float tmin = 1e-3f * len;                           // t-min 1e-3 in |d| units (:48)
    if constexpr (STATS) st_fl += 11;                         // |d|, 1/|d|, u, t-min
    float best_t = INFINITY;
    int best = -1;
    // the candidate block: roots, root choice, strict closest test.  The body
    // the ray is leaving gets sq = |h| (exact arithmetic has c = 0 there:
    // the origin lies on its surface) -- the self-hit acne guard.
    auto consider = [&](float h, float disc, int s) {
      if constexpr (STATS) st_fl += 3;
      if constexpr (STATS) {
        const uint64_t ex = __builtin_amdgcn_read_exec();
        if (lane == __ffsll(static_cast<long long>(ex)) - 1) {
          ++st_blk;
          st_blk_lanes += __popcll(ex);
        }
      }
      const float sq = (s == last) ? fabsf(h) : sqrt_rn(disc);
      float t = h - sq;                 // nearer root (hittable.clj:15)
      if (!(t > tmin)) t = h + sq;      // farther root (:16-18)
      if (t > tmin && t < best_t) {     // open interval, strictly closer (:19, raytracing.clj:35-42)
        best_t = t;
        best = s;
      }
    };
    if constexpr (SCAN == SCAN_SIMPLE || SCAN == SCAN_PK4) {
      // the diagnostic scans (trace_diag.hip, librtclj_diag.so only)
      diag_scan<SRC, SCAN>(a, s_geo, ox, oy, oz, ux, uy, uz, consider);
    } else if constexpr (is_bvh_scan(SCAN)) {
      // Closest hit through the BVH (bvh.cpp), bit-identical to the scan:
      //  * each body is tested by the scan's fp32 op sequence and accepted if
      //    t is smaller, or equal with a lower index (= the scan's first-wins);
      //  * boxes are padded per ray by P = 2e-3 * D, D = |O - c| + R bounding
      //    |oc| + r of every tree body: the fp32 test never reports a point
      //    farther than 6e-4 * (|oc| + r) outside a body's box (measured,
      //    tools/pad_bound.cpp, 3x margin), so a body the scan would accept
      //    always lies in every box on its path; a box is skipped only if its
      //    padded interval misses (tmin, best_t].
      // branch-free acceptance (bitwise predicates: no exec-mask blocks)
      auto consider_tie = [&](float h, float disc, int s) {
        if constexpr (STATS) st_fl += 3;   // sqrt, h -/+ sq
        if constexpr (STATS) ++st_blk_lanes;
        const float sq = (s == last) ? fabsf(h) : sqrt_rn(disc);
        const float tn = h - sq;
        const float t = tn > tmin ? tn : h + sq;
        // (t, index) < (best_t, best) lexicographically as one 64-bit compare:
        // t > tmin > 0, so its bits order like the floats; best = -1 is the
        // largest u32 (and best_t = +inf the largest t) before any hit
        const uint64_t key = (static_cast<uint64_t>(__float_as_uint(t)) << 32) | static_cast<uint32_t>(s);
        const uint64_t bkey = (static_cast<uint64_t>(__float_as_uint(best_t)) << 32) | static_cast<uint32_t>(best);
        const bool acc = (t > tmin) & (key < bkey);
        best_t = acc ? t : best_t;
        best = acc ? s : best;
      };
      // 1) the big bodies, kept out of the tree (bvh.cpp), as leaves of their
      // own (below), 2) the tree
      const char* base = SRC == SRC_LDS ? reinterpret_cast<const char*>(s_geo)
                                        : reinterpret_cast<const char*>(a.bvh_blob);
      const KNode* nodes = reinterpret_cast<const KNode*>(base);
      const Pair* pairs = reinterpret_cast<const Pair*>(base + a.bvh_off_pairs);
      // body indices: u16 in the 8-body-leaf tree (LDS size), int elsewhere
      // (an int pair is one read with no unpacking: the 4-body leaf pass is hot)
      using PidxT = std::conditional_t<SCAN == SCAN_BVHO, ushort2, int2>;
      const PidxT* pidx = reinterpret_cast<const PidxT*>(base + a.bvh_off_pidx);
      // box tests only cull (conservatively): hardware sqrt / rcp (1 ulp) are
      // far inside the padding.  Node boxes are stored relative to the tree
      // centre c (bvh.cpp), so every slab bound is one fma:
      // (b - (o' + P)) / u = b * (1/u) - (o' + P) / u with o' = o - c; its
      // rounding (~1e-7 * D) is far inside the padding too.
      const float ecx = ox - a.bvh_c[0], ecy = oy - a.bvh_c[1], ecz = oz - a.bvh_c[2];
      const float D = __builtin_amdgcn_sqrtf(fmaf(ecz, ecz, fmaf(ecy, ecy, ecx * ecx))) + a.bvh_r;
      const float P = fmaf(2e-3f, D, 1e-6f);
      if constexpr (STATS) st_fl += 27;   // o - c, D, P, 3 rcp, 6 slab offsets
      // 1/u clamped to +-1e24 (one v_med3): with u = 0 an infinite 1/u makes
      // the fma bounds NaN and -inf, which would collapse the slab (a false
      // miss); finite, the slab of an origin inside the padded box spans
      // ~+-1e24 and one outside it lies ~1e24 away (culled) -- the u = 0
      // answers.  (u = -0 gives -inf -> -1e24: the sign still orders the planes.)
      const float rux = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(ux), -1e24f, 1e24f);
      const float ruy = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(uy), -1e24f, 1e24f);
      const float ruz = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(uz), -1e24f, 1e24f);
      // broadcast operands as halves of packed pairs (bc_lo / bc_hi: one
      // register read through op_sel for both halves, not a duplicated pair)
      f2 r_xy = {rux, ruy}, r_z = {ruz, ruz};
      // the min plane's bound b*(1/u) - (o' + P)/u, the max plane's
      // b*(1/u) - (o' - P)/u; by the sign of 1/u one is the near plane
      const float nlx = -(ecx + P) * rux, nly = -(ecy + P) * ruy, nlz = -(ecz + P) * ruz;
      const float nhx = -(ecx - P) * rux, nhy = -(ecy - P) * ruy, nhz = -(ecz - P) * ruz;
      const bool sx = rux < 0.0f, sy = ruy < 0.0f, sz = ruz < 0.0f;
      f2 nf_x = {sx ? nhx : nlx, sx ? nlx : nhx};   // (near, far) plane offsets
      f2 nf_y = {sy ? nhy : nly, sy ? nly : nhy};
      f2 nf_z = {sz ? nhz : nlz, sz ? nlz : nhz};
      // byte offsets of the (near, far) pairs of each axis inside a node
      const int offx = sx ? 8 : 0, offy = 24 + (sy ? 8 : 0), offz = 48 + (sz ? 8 : 0);
      // the ray's (near, far) plane pairs of node 0; opaque, so that a node's
      // three axis addresses are one add each from them (not the blob's base
      // added to the node first)
      f2 o_xy = {ox, oy}, o_zux = {oz, ux}, u_yz = {uy, uz};
      // a leaf: one pair (leaf size 2) or two consecutive pairs (BVHQ, leaf
      // size 4), tested packed; the acceptance is order-independent
      // (the 4-body tree in LDS: p is a leaf record's LDS address, see the copy)
      constexpr bool kLeafRec = SRC == SRC_LDS && is_q(SCAN);
      auto leaf = [&](int p) {
        RT_MARK("leaf");
        if constexpr (STATS) {
          ++st_blk;
          const uint64_t ex = __builtin_amdgcn_read_exec();
          if (lane == __ffsll(static_cast<long long>(ex)) - 1) ++st_leafw;
        }
        // (the other trees: pairs and their indices in separate arrays; an
        // 8-body leaf runs as two 4-body halves, each with its own exact
        // passes: 4 bodies' (h, disc, index) live at a time, not 8 (103 -> ~90
        // VGPRs, 4 -> 5 waves per SIMD); the acceptance is order-independent)
        constexpr int NPL = leaf_pairs(SCAN);
        constexpr int NP = NPL > 2 ? 2 : NPL;   // pairs per half
        if constexpr (kLeafRec) {
          // The 4-body record holds each body as a float4 (cx, cy, cz, -r^2) at
          // + 16 j and the four indices at + 64.  The leaf pass keeps only the
          // candidate mask; an exact pass re-reads its body (address + 2k for
          // mask bit k = 8 j) and recomputes (h, disc) with the same ops --
          // the same bits -- instead of selecting them from 12 live registers
          // with compares and v_cndmask (single-port instructions).
          unsigned pa = static_cast<unsigned>(p);
          asm volatile("" : "+v"(pa));
          auto body = [&](unsigned addr, float& h, float& c, float& disc) {
            const f4v g = *(LdsF4)(uintptr_t)addr;
            const float ocx = g.x - o_xy.x, ocy = g.y - o_xy.y, ocz = g.z - o_zux.x;
            h = fmaf(u_yz.y, ocz, fmaf(u_yz.x, ocy, o_zux.y * ocx));
            c = fmaf(ocx, ocx, fmaf(ocz, ocz, fmaf(ocy, ocy, g.w)));
            disc = fmaf(h, h, -c);
          };
          asm volatile("" : "+v"(o_xy), "+v"(o_zux), "+v"(u_yz));
          unsigned nc[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if constexpr (STATS) st_fl += 16;
            float h, c, disc;
            body(pa + 16u * j, h, c, disc);
            nc[j] = __builtin_amdgcn_bitop3_b32(__float_as_uint(disc), __float_as_uint(h), __float_as_uint(c), 0x0b);
          }
          const unsigned b01 = __builtin_amdgcn_perm(nc[1], nc[0], 0x0c0c0b09u);
          const unsigned b23 = __builtin_amdgcn_perm(nc[3], nc[2], 0x0b090c0cu);
          unsigned m = __builtin_amdgcn_bitop3_b32(b01, b23, 0x01010101u, 0xa8);
          while (m) {
            RT_MARK("exact");
            if constexpr (STATS) {
              const uint64_t ex = __builtin_amdgcn_read_exec();
              if (lane == __ffsll(static_cast<long long>(ex)) - 1) ++st_consw;
            }
            const unsigned k = __builtin_ctz(m);
            m &= m - 1;
            float h, c, disc;
            body(pa + k + k, h, c, disc);
            const int sidx = *(const int __attribute__((address_space(3)))*)(uintptr_t)(pa + 64u + (k >> 1));
            RT_MARK("exact_accept");
            consider_tie(h, disc, sidx);
          }
          RT_MARK("node");
          return;
        }
#pragma unroll
        for (int hb = 0; hb < NPL; hb += NP) {
        float hh[2 * NP], dd[2 * NP];
        int ii[2 * NP];
        unsigned nc[2 * NP];   // bit 31: body is a candidate
        // the leaf's pairs from one base address (immediate offsets for the
        // rest; indexing p + 1 let the compiler rebuild it as -c, a 2nd base)
        const Pair* const lp = pairs + p;
        const PidxT* const li = pidx + p;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          if constexpr (STATS) st_fl += 32;   // 2 bodies x (oc 3, h 5, c 6, disc 2)
          const Pair g = lp[hb + q];
          const PidxT id = li[hb + q];
          asm volatile("" : "+v"(o_xy), "+v"(o_zux), "+v"(u_yz));
          // (scalar fp32 per body, not v_pk_*: a packed op issues on one VALU
          // port only, two v_fma_f32 dual-issue -- 5.84 -> 5.45 ms on C1
          // with the node step's planes, profiles/r05/unpack/)
          f2 h, c, disc;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float ocx = g.x[e] - o_xy.x, ocy = g.y[e] - o_xy.y, ocz = g.z[e] - o_zux.x;
            h[e] = fmaf(u_yz.y, ocz, fmaf(u_yz.x, ocy, o_zux.y * ocx));
            c[e] = fmaf(ocx, ocx, fmaf(ocz, ocz, fmaf(ocy, ocy, g.w[e])));
            disc[e] = fmaf(h[e], h[e], -c[e]);
          }
          hh[2 * q] = h.x;
          hh[2 * q + 1] = h.y;
          dd[2 * q] = disc.x;
          dd[2 * q + 1] = disc.y;
          ii[2 * q] = id.x;
          ii[2 * q + 1] = id.y;
          // candidate: disc >= 0 and not (h < 0 and c >= 0), read from the sign
          // bits (disc | (h & ~c)): the same bodies as the scan's test except
          // c = -0 or h = -0 or NaN operands, whose roots the exact test
          // rejects anyway (t <= t-min or NaN)
          // (halves copied to scalars first: __builtin_bit_cast of an
          // ext_vector element read the .x half for .y here)
          const float d0 = disc.x, d1 = disc.y, h0 = h.x, h1 = h.y, k0 = c.x, k1 = c.y;
          // one v_bitop3_b32 each: LUT 0x0b = ~(s0 | (s1 & ~s2))
          nc[2 * q] = __builtin_amdgcn_bitop3_b32(__float_as_uint(d0), __float_as_uint(h0),
                                                  __float_as_uint(k0), 0x0b);
          nc[2 * q + 1] = __builtin_amdgcn_bitop3_b32(__float_as_uint(d1), __float_as_uint(h1),
                                                      __float_as_uint(k1), 0x0b);
        }
        // candidate mask: body j at bit 8j. v_perm_b32's sign selectors (9:
        // the low source's bit 31, 11: the high source's; 12: zero) gather
        // two bodies' sign bits as 0x00 / 0xff bytes per instruction, and one
        // v_bitop3 merges the halves and keeps bit 0 of each byte
        unsigned m;
        if constexpr (NP == 2) {
          const unsigned b01 = __builtin_amdgcn_perm(nc[1], nc[0], 0x0c0c0b09u);
          const unsigned b23 = __builtin_amdgcn_perm(nc[3], nc[2], 0x0b090c0cu);
          m = __builtin_amdgcn_bitop3_b32(b01, b23, 0x01010101u, 0xa8);   // (s0 | s1) & s2
        } else {
          m = __builtin_amdgcn_perm(nc[1], nc[0], 0x0c0c0b09u) & 0x0101u;
        }
        // one pass of the exact test per candidate: the wave runs it as often
        // as its lane with the most candidates needs (not once per body)
        while (m) {
          if constexpr (STATS) {
            const uint64_t ex = __builtin_amdgcn_read_exec();
            if (lane == __ffsll(static_cast<long long>(ex)) - 1) ++st_consw;
          }
          const unsigned k = __builtin_ctz(m);
          m &= m - 1;
          float h = hh[0], d = dd[0];
          int s = ii[0];
#pragma unroll
          for (int j = 1; j < 2 * NP; ++j) {
            h = k == static_cast<unsigned>(8 * j) ? hh[j] : h;
            d = k == static_cast<unsigned>(8 * j) ? dd[j] : d;
            s = k == static_cast<unsigned>(8 * j) ? ii[j] : s;
          }
          consider_tie(h, d, s);
        }
        }
      };
      // slab test of both children of node nd: entry/exit t and the cull
      // predicate "[tn, tf] meets (tmin, best_t]" (tmin < best_t always; a NaN
      // bound only makes the test pass: conservative)
      // (the near plane's t is the min of the two planes' t, bit for bit: the
      // same fma on the same operands -- no min/max orders them)
      auto node_planes = [&](int node, float& tn0, float& tn1, float& tf0, float& tf1, int& c0, int& c1) {
        if constexpr (STATS) st_fl += 24;   // 12 fma over 2 children
        // node * 80 as a 24-bit multiply (full rate; v_mul_lo_u32 is quarter rate)
        // the 4-body tree's inner-child refs are byte offsets (node * 80,
        // written by rt_scene_upload): no multiply per step
        // (BVHQ: node is the node's LDS address; BVHQ7: its index, the
        // address one multiply-add away; others: an index into nodes)
        const unsigned nof = SCAN == SCAN_BVHQ    ? static_cast<unsigned>(node)
                             : SCAN == SCAN_BVHQ7 ? __umul24(static_cast<unsigned>(node), 80u) + lds_addr(nodes)
                                                  : __umul24(static_cast<unsigned>(node), 80u);
        f2 x0, x1, y0, y1, z0, z1;   // per axis the (near, far) plane pairs of both children
        int2 ch;
        if constexpr (SRC == SRC_LDS && is_q(SCAN)) {
          // node = the node's LDS address (the refs were relocated as the
          // blob was copied): the axes one add each, the child refs at + 72
          const LdsF2 lx = (LdsF2)(uintptr_t)(nof + offx), ly = (LdsF2)(uintptr_t)(nof + offy),
                      lz = (LdsF2)(uintptr_t)(nof + offz);
          x0 = lx[0], x1 = lx[1], y0 = ly[0], y1 = ly[1], z0 = lz[0], z1 = lz[1];
          const long long c2 = *(LdsI64)(uintptr_t)(nof + 72);
          ch = make_int2(static_cast<int>(c2), static_cast<int>(c2 >> 32));
        } else {
          const char* nb = reinterpret_cast<const char*>(nodes) + nof;
          const f2* ax = reinterpret_cast<const f2*>(nb + offx);
          const f2* ay = reinterpret_cast<const f2*>(nb + offy);
          const f2* az = reinterpret_cast<const f2*>(nb + offz);
          x0 = ax[0], x1 = ax[1], y0 = ay[0], y1 = ay[1], z0 = az[0], z1 = az[1];
          ch = *reinterpret_cast<const int2*>(nb + 72);
        }
        asm volatile("" : "+v"(r_xy), "+v"(r_z), "+v"(nf_x), "+v"(nf_y), "+v"(nf_z));
        // (per child scalar v_fma_f32: dual-issued, unlike v_pk_fma_f32)
        f2 tnx, tfx, tny, tfy, tnz, tfz;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          tnx[e] = fma3(x0[e], r_xy.x, nf_x.x);
          tfx[e] = fma3(x1[e], r_xy.x, nf_x.y);
          tny[e] = fma3(y0[e], r_xy.y, nf_y.x);
          tfy[e] = fma3(y1[e], r_xy.y, nf_y.y);
          tnz[e] = fma3(z0[e], r_z.x, nf_z.x);
          tfz[e] = fma3(z1[e], r_z.x, nf_z.y);
        }
        tn0 = fmaxf(fmaxf(tnx.x, tny.x), tnz.x);
        tn1 = fmaxf(fmaxf(tnx.y, tny.y), tnz.y);
        tf0 = fminf(fminf(tfx.x, tfy.x), tfz.x);
        tf1 = fminf(fminf(tfx.y, tfy.y), tfz.y);
        c0 = ch.x;
        c1 = ch.y;
      };
      auto node_test = [&](int node, float& tn0, float& tn1, bool& hit0, bool& hit1, int& c0, int& c1) {
        float tf0, tf1;
        node_planes(node, tn0, tn1, tf0, tf1, c0, c1);
        // "[tn, tf] meets (tmin, best_t]" as max(tn, tmin) <= min(tf, best_t),
        // spelled tn <= min(tf, best_t) and tmin <= tf (tmin < best_t always):
        // a compare instead of a max per child.  Each is "not greater", so a
        // NaN bound passes (conservative).
        // (min(tf, best_t) as a bare v_min_f32: fminf would re-canonicalise
        // best_t every step; a NaN tf gives best_t, conservative)
        float tb0, tb1;
        asm("v_min_f32 %0, %1, %2" : "=v"(tb0) : "v"(tf0), "v"(best_t));
        asm("v_min_f32 %0, %1, %2" : "=v"(tb1) : "v"(tf1), "v"(best_t));
        hit0 = !(tn0 > tb0) & !(tmin > tf0);
        hit1 = !(tn1 > tb1) & !(tmin > tf1);
      };
      // the big bodies' leaves first: every lane, so a wave-uniform loop (their
      // hits, e.g. the ground, then cull the tree)
      RT_MARK("bigleaf");
      for (int b = 0; b < a.n_big_leaves; ++b) {
        if constexpr (kLeafRec)
          leaf(static_cast<int>(lds_addr(nodes)) + a.bvh_off_pairs + ((a.big_pair0 >> 1) + b) * kLeafRecBytes);
        else
          leaf(a.big_pair0 + b * leaf_pairs(SCAN));
      }
      RT_MARK("tree_setup");
      // the root: the 4-body tree's refs are LDS addresses (relocated as copied)
      int node = SRC == SRC_LDS && SCAN == SCAN_BVHQ ? static_cast<int>(lds_addr(nodes)) : 0;   // (BVHQ7: index 0)
      // the stack top as a pointer into the [entry][lane] stack: one add per
      // push / pop instead of index arithmetic
      StackT* const stk0 = s_stack + threadIdx.x;
      StackT* top = stk0;
      // a row of the stack in bytes, held in a register the compiler cannot
      // rematerialise (a literal would be moved into a VGPR on every push)
      int row_b = NT * static_cast<int>(sizeof(StackT));
      asm volatile("" : "+v"(row_b));
      bool go = true;
      while (go) {
        RT_MARK("node");
        if constexpr (STATS) {
          ++st_sph;
          const uint64_t ex = __builtin_amdgcn_read_exec();
          if (lane == __ffsll(static_cast<long long>(ex)) - 1) {
            ++st_trav;
            st_trav_lanes += __popcll(ex);
          }
        }
        float tn0, tn1;
        bool hit0, hit1;
        int c0, c1;
        node_test(node, tn0, tn1, hit0, hit1, c0, c1);
        // leaf children are tested now; a lane's first leaf shares one pass
        // with every other lane's first leaf, whichever child it is
        const bool l0 = hit0 && c0 < 0, l1 = hit1 && c1 < 0;
        if (l0 || l1) {
          leaf(l0 ? ~c0 : ~c1);
          if (l0 && l1) leaf(~c1);
        }
        // inner children: both -> the near one next, the far one pushed; one
        // -> that one; none -> pop.  The far child is written above the stack
        // top every step (a dead entry unless both were hit): no branch
        const bool i0 = hit0 && !l0, i1 = hit1 && !l1;   // (lane masks, no compares)
        const bool sw = tn1 < tn0;
        int nxt = (i0 && (!i1 || !sw)) ? c0 : c1;
        *top = static_cast<StackT>(sw ? c0 : c1);
        top = reinterpret_cast<StackT*>(reinterpret_cast<char*>(top) + ((i0 && i1) ? row_b : 0));
        if (!(i0 || i1)) {
          // pop, unconditionally: with an empty stack the top moves one row
          // below the first entry, into the blob's last bytes (a harmless
          // read), and the lane leaves -- one add and one compare, no select
          top -= NT;
          go = top >= stk0;
          nxt = *top;
        }
        node = nxt;
      }
      // the ray's origin and unit direction again from the packed copies the
      // walk used (the same values): the scalar ones are dead through it,
      // six VGPRs fewer at its peak
      RT_MARK("hit");
      ox = o_xy.x;
      oy = o_xy.y;
      oz = o_zux.x;
      ux = o_zux.y;
      uy = u_yz.x;
      uz = u_yz.y;
    } else {
      // groups of 4 bodies; the next group is loaded before the current one is
      // tested (hides the LDS / scalar-cache latency); one branch per group.
      // The table is padded to a multiple of 4 (+4) with bodies that can never
      // be candidates (-r^2 = +inf -> disc = -inf).
      // Candidate test min(disc, max(h, -c)) >= 0 admits, beyond the simple
      // form, only c == 0 & h < 0 (roots 2h and 0, rejected by t > tmin) and
      // NaN disc (t NaN, rejected): identical results.
      auto load = [&](int s) -> float4 {
        if constexpr (SRC == SRC_LDS) return s_geo[s];
        else return a.geo[s];
      };
      float4 g0 = load(0), g1 = load(1), g2 = load(2), g3 = load(3);
      for (int s = 0; s < n; s += 4) {
        const float4 n0 = load(s + 4), n1 = load(s + 5), n2 = load(s + 6), n3 = load(s + 7);
        float h[4], disc[4];
        bool cand[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float4 g = k == 0 ? g0 : k == 1 ? g1 : k == 2 ? g2 : g3;
          const float ocx = g.x - ox, ocy = g.y - oy, ocz = g.z - oz;
          h[k] = fmaf(uz, ocz, fmaf(uy, ocy, ux * ocx));
          const float c = fmaf(ocx, ocx, fmaf(ocz, ocz, fmaf(ocy, ocy, g.w)));
          disc[k] = fmaf(h[k], h[k], -c);
          cand[k] = fminf(disc[k], fmaxf(h[k], -c)) >= 0.0f;
        }
        if (cand[0] | cand[1] | cand[2] | cand[3]) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (cand[k]) consider(h[k], disc[k], s + k);
        }
        g0 = n0;
        g1 = n1;
        g2 = n2;
        g3 = n3;
      }
    }
    if constexpr (STATS && !is_bvh_scan(SCAN)) st_fl += 16ull * static_cast<uint64_t>(n);   // oc 3, h 5, c 6, disc 2
    if constexpr (STATS && !is_bvh_scan(SCAN)) {
      const uint64_t ex = __builtin_amdgcn_read_exec();
      if (lane == __ffsll(static_cast<long long>(ex)) - 1) st_sph += static_cast<uint64_t>(n);
    }

    if constexpr (STATS) {
      const uint64_t t = stamp();
      st_c_scan += t - st_ts;
      st_ts = t;
    }
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    if (best < 0) {
      // sky (raytracing.clj:55-58)
      if constexpr (STATS) st_fl += 12;
      const float sa = 0.5f * (uy + 1.0f);
      const float om = 1.0f - sa;
      cr = tr * fmaf(sa, 0.5f, om);
      cg = tg * fmaf(sa, 0.7f, om);
      cb = tb * fmaf(sa, 1.0f, om);
      done = true;
    } else if (rem == 0) {
      done = true;  // the scattered ray would get depth 0 -> black (:46-47)
    } else {
      // ---- hit record (hittable.clj:24-31, ray.clj:7-8, hit.clj:14-15) ----
      const float4 sp = a.sph[best];
      const float hx = fmaf(ux, best_t, ox);
      const float hy = fmaf(uy, best_t, oy);
      const float hz = fmaf(uz, best_t, oz);
      // outward normal (p - C) / r, as (p - C) * (1/r) with 1/r from the table
      if constexpr (STATS) st_fl += 17;   // p, n, front
      float nx = (hx - sp.x) * sp.w, ny = (hy - sp.y) * sp.w, nz = (hz - sp.z) * sp.w;
      const bool front = fmaf(dz, nz, fmaf(dy, ny, dx * nx)) < 0.0f;
      if (!front) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
      }
      const int kind = a.kind[best];
      const float4 m = a.mat[best];
      ox = hx;
      oy = hy;
      oz = hz;
      last = best;
      if (kind == RT_LAMBERTIAN || kind == RT_METAL) {
        RT_MARK("lambert_metal");
        if constexpr (STATS) {
          const uint64_t ex = __builtin_amdgcn_read_exec();
          if (lane == __ffsll(static_cast<long long>(ex)) - 1) {
            ++st_lm;
            st_lm_lanes += __popcll(ex);
          }
        }
        // one random-unit-vec3 draw for either material (the only draws of
        // the segment for these lanes): a wave loops the rejection sampler
        // once for both kinds
        float qx, qy, qz;
        if (a.sampler & RT_SAMPLER_SPHERE) {
          sphere_direct<STATS>(st, qx, qy, qz, &st_ball, &st_fl);
          RT_MARK("lambert_metal");
        } else {
          RT_MARK("rejection_sphere");
          random_unit<STATS>(st, qx, qy, qz, &st_ball, &st_fl);
        }
        if constexpr (STATS) st_fl += kind == RT_LAMBERTIAN ? 6 : 26;
        if (kind == RT_LAMBERTIAN) {
          // material.clj:13-19 + vec3a/near-zero? (vec3a.clj:88-92)
          float sx = qx + nx, sy = qy + ny, sz = qz + nz;
          // (realm.raytracing has no near-zero fallback, realm/raytracing.clj:137-143)
          if (!a.realm && fabsf(sx) < 1e-8f && fabsf(sy) < 1e-8f && fabsf(sz) < 1e-8f) {
            sx = nx;
            sy = ny;
            sz = nz;
          }
          dx = sx;
          dy = sy;
          dz = sz;
          tr *= m.x;
          tg *= m.y;
          tb *= m.z;
        } else {
          // material.clj:21-28: reflect the *un-normalised* d, add fuzz*unit
          const float k2 = 2.0f * fmaf(dz, nz, fmaf(dy, ny, dx * nx));
          const float rx0 = fmaf(-nx, k2, dx), ry0 = fmaf(-ny, k2, dy), rz0 = fmaf(-nz, k2, dz);
          const float rx = fmaf(m.w, qx, rx0), ry = fmaf(m.w, qy, ry0), rz = fmaf(m.w, qz, rz0);
          if (fmaf(rz, nz, fmaf(ry, ny, rx * nx)) > 0.0f) {
            dx = rx;
            dy = ry;
            dz = rz;
            tr *= m.x;
            tg *= m.y;
            tb *= m.z;
          } else {
            done = true;  // absorbed: scatter-fn nil -> black (:51-54)
          }
        }
      } else if (kind == RT_NONE) {
        done = true;  // no ::scatter-fn -> black (raytracing.clj:49-54)
      } else {
        // material.clj:34-46 dielectric, reflectance :30-32, refract vec3a.clj:97-101
        RT_MARK("dielectric");
        if constexpr (STATS) {
          const uint64_t ex = __builtin_amdgcn_read_exec();
          if (lane == __ffsll(static_cast<long long>(ex)) - 1) {
            ++st_diel;
            st_diel_lanes += __popcll(ex);
          }
        }
        const float ri = front ? m.x : m.w;   // 1/eta (host-divided) : eta
        const float r0 = front ? m.y : m.z;   // Schlick's r0 for that ri (host-computed, same ops)
        if constexpr (STATS) st_fl += 9;
        const float un = fmaf(uz, nz, fmaf(uy, ny, ux * nx));
        const float cosv = fminf(-un, 1.0f);
        const float sinv = sqrt_rn(fmaf(-cosv, cosv, 1.0f));
        bool refl = !(ri * sinv <= 1.0f);
        if (!refl && !a.realm) {   // (realm: no Schlick term, no draw; realm/raytracing.clj:158-177)
          const float xi = rng_uniform(st);  // drawn only when refraction is possible
          if constexpr (STATS) st_fl += 8;   // xi, x1, x2, x5, 1 - r0, fma, compare (r0: host)
          const float x1 = 1.0f - cosv;
          const float x2 = x1 * x1;
          const float x5 = x2 * x2 * x1;
          refl = fmaf(1.0f - r0, x5, r0) > xi;
        }
        if constexpr (STATS) st_fl += refl ? 7 : 22;
        if (refl) {
          const float k2 = 2.0f * un;
          dx = fmaf(-nx, k2, ux);
          dy = fmaf(-ny, k2, uy);
          dz = fmaf(-nz, k2, uz);
        } else {
          const float qx = fmaf(nx, cosv, ux) * ri;
          const float qy = fmaf(ny, cosv, uy) * ri;
          const float qz = fmaf(nz, cosv, uz) * ri;
          const float par = -sqrt_rn(fabsf(1.0f - fmaf(qz, qz, fmaf(qy, qy, qx * qx))));
          dx = fmaf(nx, par, qx);
          dy = fmaf(ny, par, qy);
          dz = fmaf(nz, par, qz);
        }
      }
    }

    if constexpr (STATS) {
      const uint64_t t = stamp();
      st_c_shade += t - st_ts;
      st_ts = t;
    }
    RT_MARK("sums");
    if (done) {   // the sample's colour into its pixel's fixed-point sum (order-free)
      if constexpr (STATS) st_fl += 3;
      if constexpr (STATS) wave_event(st_sums);
      AccT* acc = &s_acc[q * 3];
      if constexpr (SWEEP) {   // a record's path: into its pixel's split sums in HBM
        unsigned long long* pp = kargs_opaque()->part + static_cast<size_t>(q) * 3;
        const uint32_t f0 = fix24(cr), f1 = fix24(cg), f2 = fix24(cb);
        if (f0) __hip_atomic_fetch_add(pp + 0, static_cast<unsigned long long>(f0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f1) __hip_atomic_fetch_add(pp + 1, static_cast<unsigned long long>(f1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f2) __hip_atomic_fetch_add(pp + 2, static_cast<unsigned long long>(f2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (kCompactPx && sgpr(kargs_opaque()->spp) > 255) {
        // the u32 sums with their wraps counted (s_carry above)
        const uint32_t f0 = fix24(cr), f1 = fix24(cg), f2 = fix24(cb);
        const uint32_t o0 = __hip_atomic_fetch_add(acc + 0, f0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t o1 = __hip_atomic_fetch_add(acc + 1, f1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t o2 = __hip_atomic_fetch_add(acc + 2, f2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const bool w0 = o0 + f0 < o0, w1 = o1 + f1 < o1, w2 = o2 + f2 < o2;
        if (w0 | w1 | w2) {
          RT_MARK("cold");
          const int c = q * 3;
          if (w0) atomicAdd(&s_carry[c >> 2], 1u << (8 * (c & 3)));
          if (w1) atomicAdd(&s_carry[(c + 1) >> 2], 1u << (8 * ((c + 1) & 3)));
          if (w2) atomicAdd(&s_carry[(c + 2) >> 2], 1u << (8 * ((c + 2) & 3)));
        }
      } else {
        __hip_atomic_fetch_add(acc + 0, static_cast<AccT>(fix24(cr)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(acc + 1, static_cast<AccT>(fix24(cg)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(acc + 2, static_cast<AccT>(fix24(cb)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    // refill: the lanes whose paths ended take their next indices
    RT_MARK("refill");
    const uint64_t m = __ballot(done);
    if (m) {
      if constexpr (STATS) wave_event(st_refill);
      // the lanes in m take the next indices of the wave's batch, in rank
      // order; when it runs out the wave claims another: 64 indices from
      // s_pool_next, or for a shared tile 128-1024 from the tile's word
      // (whose helper count tells the owner whether the tile was shared).
      // A claim past the pool leaves the remaining lanes without one: they
      // retire, and every later claim of the wave would be past it too.
      const int need = static_cast<int>(__popcll(m));
      const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
      int nj = -1;
      for (int r0 = 0;;) {
        const int take = min(we - wb, need - r0);
        if (rank >= r0 && rank < r0 + take) nj = wb + (rank - r0);
        wb += take;
        r0 += take;
        if (r0 >= need || we >= pool) break;
        RT_MARK("claim");
        if constexpr (STATS) wave_event(st_claim);
        int g = 0;
        // a shared tile's claims shrink as its pool is spent (guided: an
        // eighth of what is left past this wave's last batch, kShareBatch ..
        // batch_max)
        // an unshared pool's the same way from its LDS counter, 64 ..
        // lds_batch_max (read where it is used: no register held for it)
        const int want = src ? max(kShareBatch, min(kc_batch_max, ((pool - we) >> 3) & ~63))
                             : max(64, min(kargs_opaque()->lds_batch_max, ((pool - we) >> 3) & ~63));
        const int leader = static_cast<int>(__builtin_amdgcn_readfirstlane(lane));
        if (lane == leader) {
          if (src) {
            const unsigned long long wd = __hip_atomic_fetch_add(src, static_cast<unsigned long long>(want),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            g = static_cast<int>(static_cast<unsigned>(wd));
            if (g < pool) atomicAdd(&s_cnt, min(pool - g, want));
            atomicMax(&s_join, word_helpers(wd));
          } else if constexpr (SWEEP) {   // records past the grid's first ones, 64 at a time
            g = static_cast<int>(atomicAdd(&kargs_opaque()->xq_n[1], 64u)) + static_cast<int>(gridDim.x) * NT;
          } else {
            g = atomicAdd(&s_pool_next, want);
          }
        }
        g = __builtin_amdgcn_readlane(g, leader);
        wb = min(g, pool);
        we = min(g + (SWEEP ? 64 : want), pool);
        if (wb >= pool) we = pool;   // spent: the lanes left over retire
      }
      RT_MARK("refill");
      if (done) {
        j = kCompact && nj < 0 ? -2 : nj;
        fresh = true;
        if (nj < 0) active = false;
      }
    }
    if constexpr (STATS) st_c_acc += stamp() - st_ts;
    RT_MARK("compaction");
    if constexpr (kCompact) {
      // spent: out to the compaction step when this wave may post its few
      // paths, or its idle lanes may take posted ones
      // (the limit and the flags from LDS: no registers held for them)
      if (wb >= pool) {
        RT_MARK("drain_check");
        if constexpr (STATS) wave_event(st_drain);
        const int lim = sgpr(lds_load(&s_mb_lim[threadIdx.x >> 6]));
        if (lim >= 0) {
          const int left = static_cast<int>(__popcll(__ballot(j >= -1)));
          // (not while a lane holds a camera sample it has not started: no
          // lane leaves the loop fresh, so that the step needs no fresh flags)
          if ((left <= lim || (left < 64 && sgpr(lds_load(&s_mb_avail)) > 0)) && __ballot(j >= 0) == 0 &&
              j == -1)
            j = -3;   // (out of the loop, the path kept)
        }
      }
    }
  };
  for (;;) {
    RT_MARK("loop");
    if constexpr (kCompact) {
      while (j >= -1) iteration();
    } else {
      while (active) iteration();
    }
    if constexpr (!kCompact) {
      break;
    } else {
      if (sgpr(lds_load(&s_mb_lim[wv])) < 0) break;   // (-1: compaction off)
      // (every lane here: the wave-level state is made the same in all)
      wb = we = pool;
      active = j == -3;   // the lanes that left the loop with a path
      if (active) j = -1;
      compact_step();
      if (__ballot(active) == 0) break;
    }
  }

  RT_MARK("epilogue");
  // ---- per-pixel mean (compute-pixel's accum / spp, raytracing.clj:155) ----
  // thread t < 3 * npx writes channel t % 3 of pool pixel t / 3: a tile row's
  // 8 pixels are 24 consecutive floats
  __syncthreads();
  const KArgsP ke = kargs_opaque();
  if constexpr (!SWEEP) {
  const int t = static_cast<int>(threadIdx.x);
  // (owner of an unshared tile: no helper joined before its pool was spent)
  const bool alone = !shared_tile || sgpr(s_join) == 0;
  auto out_index = [&](int tt) {
    const int fp = tt / 3, ch = tt - 3 * fp;
    const int qy = vw == 1 ? fp : static_cast<int>(__umulhi(static_cast<uint32_t>(fp), mag_vw));
    const int px = qx0 + (fp - qy * vw), ro = qy0 + qy;
    return (static_cast<size_t>(ro) * ke->width + px) * 3 + ch;
  };
  auto write_mean = [&](size_t e, unsigned long long sum) {
    const float tot = static_cast<float>(sum) * 0x1p-24f;   // RN(float(sum)), exact scale
    const float inv = static_cast<float>(ke->spp > 0 ? ke->spp : 1);
    // realm: pixel-scale = 1/spp, multiplied (realm/raytracing.clj:25, :276)
    ke->out[e] = ke->realm ? tot * (1.0f / inv) : tot / inv;
  };
  // channel t's integer sum (the compact variant: its wraps added back)
  auto total = [&](int tt) -> unsigned long long {
    unsigned long long v = static_cast<unsigned long long>(s_acc[tt]);
    if constexpr (kCompactPx) v += static_cast<unsigned long long>((s_carry[tt >> 2] >> (8 * (tt & 3))) & 0xffu) << 32;
    return v;
  };
  if (split) {   // one split's integer sums, added to the tile's (order-free); finalize_kernel converts them
    if (t < npx * 3) {
      const unsigned long long v = total(t);
      if (v) __hip_atomic_fetch_add(&ke->part[out_index(t)], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (alone) {   // every sample of the tile was this workgroup's
    if (t < npx * 3) write_mean(out_index(t), total(t));
  } else {
    // a shared tile (owner or helper): the integer sums
    // meet in sum[tile] (atomics: any order, the same total); the workgroup
    // whose samples complete the pool converts them and re-zeroes the slots
    unsigned long long* gs = ke->sum + static_cast<size_t>(tile) * (NPX * 3);
    if (t < npx * 3) {
      const unsigned long long v = total(t);
      if (v) __hip_atomic_fetch_add(&gs[t], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned mine = static_cast<unsigned>(s_cnt);
      const unsigned prev = __hip_atomic_fetch_add(&ke->done[tile], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev + mine == static_cast<unsigned>(pool);
      // the participant that completes the pool pairs the others' release
      // fences with an acquire before it reads (and resets) the sums
      if (prev + mine == static_cast<unsigned>(pool)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (sgpr(s_last)) {   // (every participant has added: the slots and done are free for the next use)
      if (t < npx * 3)
        write_mean(out_index(t), __hip_atomic_exchange(&gs[t], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (t == 0) __hip_atomic_exchange(&ke->done[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  if (ke->tile_cost && threadIdx.x == 0) {   // the adaptive schedule's measurement: the unit's time
    const uint64_t dt = __builtin_amdgcn_s_memrealtime() - st_t0;
    atomicAdd(&ke->tile_cost[tile], static_cast<unsigned>(dt < 0xffffffffull ? dt : 0xffffffffull));
  }
  if (ke->counters && own && threadIdx.x == 0 && pool)
    atomicAdd(&ke->counters[1], static_cast<unsigned long long>(pool));
  }   // (!SWEEP: a sweep's colours went to part[] as its paths ended)

  if constexpr (STATS) {
    if (a.dbg && st_iter) {
      atomicAdd(&a.dbg[0], static_cast<unsigned long long>(st_iter));
      atomicAdd(&a.dbg[1], static_cast<unsigned long long>(st_lanes));
    }
    if (a.dbg && st_sph) atomicAdd(&a.dbg[2], static_cast<unsigned long long>(st_sph));
    if (a.dbg && st_trav) {
      atomicAdd(&a.dbg[6], static_cast<unsigned long long>(st_trav));
      atomicAdd(&a.dbg[7], static_cast<unsigned long long>(st_trav_lanes));
    }
    if (a.dbg && (st_leafw | st_consw)) {
      atomicAdd(&a.dbg[12], static_cast<unsigned long long>(st_leafw));
      atomicAdd(&a.dbg[13], static_cast<unsigned long long>(st_consw));
    }
    if (a.dbg && (st_ball | st_disk)) {
      atomicAdd(&a.dbg[14], static_cast<unsigned long long>(st_ball));
      atomicAdd(&a.dbg[15], static_cast<unsigned long long>(st_disk));
    }
    if (a.dbg && (st_diel | st_lm)) {
      atomicAdd(&a.dbg[19], static_cast<unsigned long long>(st_diel));
      atomicAdd(&a.dbg[20], static_cast<unsigned long long>(st_diel_lanes));
      atomicAdd(&a.dbg[21], static_cast<unsigned long long>(st_lm));
      atomicAdd(&a.dbg[22], static_cast<unsigned long long>(st_lm_lanes));
    }
    if (a.dbg && st_fresh) {
      atomicAdd(&a.dbg[16], static_cast<unsigned long long>(st_fresh));
      atomicAdd(&a.dbg[17], static_cast<unsigned long long>(st_fresh_lanes));
    }
    if (a.dbg && (st_sums | st_refill | st_claim | st_drain)) {
      atomicAdd(&a.dbg[23], static_cast<unsigned long long>(st_sums));
      atomicAdd(&a.dbg[24], static_cast<unsigned long long>(st_refill));
      atomicAdd(&a.dbg[25], static_cast<unsigned long long>(st_claim));
      atomicAdd(&a.dbg[26], static_cast<unsigned long long>(st_drain));
    }
    if (a.dbg && st_blk) {
      atomicAdd(&a.dbg[3], static_cast<unsigned long long>(st_blk));
      atomicAdd(&a.dbg[4], static_cast<unsigned long long>(st_blk_lanes));
    }
    if (a.dbg && lane == 0) atomicAdd(&a.dbg[5], 1ull);
    {   // executed flops: a wave sum, one atomic
      uint64_t f = st_fl;
      for (int off = 32; off > 0; off >>= 1) {
        const uint32_t lo = __shfl_xor(static_cast<uint32_t>(f), off);
        const uint32_t hi = __shfl_xor(static_cast<uint32_t>(f >> 32), off);
        f += (static_cast<uint64_t>(hi) << 32) | lo;
      }
      if (a.dbg && lane == 0) atomicAdd(&a.dbg[18], static_cast<unsigned long long>(f));
    }
    // clock split: the lane active longest saw every iteration (max over lanes)
    const uint64_t c0 = wave_max_u64(st_c_cam), c1 = wave_max_u64(st_c_scan);
    const uint64_t c2 = wave_max_u64(st_c_shade), c3 = wave_max_u64(st_c_acc);
    if (a.dbg && lane == 0) {
      atomicAdd(&a.dbg[8], static_cast<unsigned long long>(c0));
      atomicAdd(&a.dbg[9], static_cast<unsigned long long>(c1));
      atomicAdd(&a.dbg[10], static_cast<unsigned long long>(c2));
      atomicAdd(&a.dbg[11], static_cast<unsigned long long>(c3));
    }
  }
  // wave timeline (stats variants, or any variant under RTCLJ_TIMELINE in
  // the diagnostic build; NULL otherwise: a uniform branch)
  if (a.dbgw && lane == 0) {
    // (by dispatch slot; the wave index rebuilt here, in an SGPR: held from
    // the start in a VGPR, at 72 VGPRs it was spilled to scratch)
    const size_t wid = static_cast<size_t>(unit) * NW + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wid < kDbgWaves) {
      a.dbgw[4 * wid + 0] = st_t0;
      a.dbgw[4 * wid + 1] = __builtin_amdgcn_s_memrealtime();
      a.dbgw[4 * wid + 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
      a.dbgw[4 * wid + 3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
    }
  }
  if (a.counters) {
    // the workgroup's segments (its waves' sums met in LDS) in one 64-bit
    // atomic, beside its samples (one per workgroup each: a global atomic is
    // an HBM read-modify-write)
    uint32_t v = segs;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && v) atomicAdd(&s_segs, static_cast<unsigned long long>(v));
    __syncthreads();
    if (threadIdx.x == 0 && s_segs) atomicAdd(&a.counters[0], s_segs);
  }
}

// direction-coherent waves (sorted_kernel, trace_diag.hip): its shape,
// which the host's launch code sizes
constexpr int kSortWaves = 8;
constexpr int kSortThreads = 64 * kSortWaves;
constexpr int kSortTH = 16;                       // tile rows
constexpr int kSortNPX = kTile * kSortTH;         // pool pixels
constexpr int kSortKeys = 10;                     // 0 fresh, 1..8 octants, 9 no path
constexpr int kXFields = 11;
constexpr int kXWaveWords = kXFields * 64;        // a wave's slots (u32)
constexpr size_t kXBytes = static_cast<size_t>(kSortWaves) * kXWaveWords * 4;   // 22,528


// A kernel variant (rt_set_variant; trace.hip's table, trace_diag.hip's
// diagnostic entries)
struct Variant {
  const void* fn;
  bool lds;
  bool stats;
  int scan;   // SCAN_* (the tile shape: tile_rows, unless th)
  int threads = 256;   // workgroup size
  int th = 0;          // the pool's tile rows (0: tile_rows(scan))
  const void* sweep = nullptr;   // the variant's sweep kernel (path export, KArgs::xq), or NULL
};
inline int variant_rows(const Variant& v) { return v.th ? v.th : tile_rows(v.scan); }
#define RT_K(SRC, SCAN, ST) reinterpret_cast<const void*>(&trace_kernel<SRC, SCAN, ST>)
#define RT_KW(SRC, SCAN, ST, NW) reinterpret_cast<const void*>(&trace_kernel<SRC, SCAN, ST, NW>)
#define RT_KWT(SRC, SCAN, ST, NW, TH) reinterpret_cast<const void*>(&trace_kernel<SRC, SCAN, ST, NW, TH>)
#define RT_KSW(SRC, SCAN, NW, TH) reinterpret_cast<const void*>(&trace_kernel<SRC, SCAN, false, NW, TH, true>)
// The diagnostic library's variants (trace_diag.hip): v's entry, or NULL.
const Variant* diag_variant(int v);

}  // namespace rtclj
