// trace.hip — the per-pixel render loop as one stackless gfx950 kernel.
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

// Correctly rounded sqrt, the same bits as sqrtf for every input: for
// x >= 2^-96 (every normal case here) the hardware v_sqrt_f32 corrected by
// the residuals of its neighbours -- the sequence the compiler emits for
// sqrtf, without its denormal scaling and zero/inf class fix-up (a rare
// branch keeps those for tiny, NaN and negative inputs): 16 -> 9 VALU.
__device__ __forceinline__ float sqrt_rn(float x) {
  if (__builtin_expect(!(x >= 0x1p-96f), 0)) return sqrtf(x);
  const float s = __builtin_amdgcn_sqrtf(x);
  const int si = __builtin_bit_cast(int, s);
  const float sd = __builtin_bit_cast(float, si - 1), su = __builtin_bit_cast(float, si + 1);
  const float rd = fmaf(-sd, s, x), ru = fmaf(-su, s, x);
  float r = rd <= 0.0f ? sd : s;
  r = ru > 0.0f ? su : r;
  return r;
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
  const float il = 1.0f / sqrt_rn(l2);   // contract: v * (1/|v|)
  if constexpr (STATS) *flops += 5;
  x = x * il;
  y = y * il;
  z = z * il;
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

// The pool tile: 8 x 8 pixels per 256-thread workgroup
// The pool tile: 8 pixels wide, 8 rows high -- 4 for the 8-body-leaf
// traversal, whose large-scene LDS image (C4: 1000 bodies) needs the 768 B
// that half the pixel sums give back to stay at 5 workgroups per CU
constexpr int kTile = 8;
// the 4-body tree's leaf record in LDS: two pairs and their index pairs
constexpr int kLeafRecBytes = 80;
constexpr int kPoolPx = kTile * kTile;
constexpr int tile_rows(int scan) { return scan == SCAN_BVHO ? 4 : scan == SCAN_BVHS ? 16 : kTile; }

// Waves per SIMD the register allocator must leave room for: six for the
// default traversal (80 VGPRs; its 26.5 KB LDS image fits 6 workgroups per
// CU), five for the 8-body-leaf one (C4: its LDS allows 5 workgroups per
// CU).  Without the bound the unit loop's longer-lived uniform values
// (SGPRs at their limit, copied into VGPRs) take it to ~100 VGPRs and four
// waves; with it, a few of them spill to scratch outside the hot loop.
constexpr int min_waves(int scan, bool stats) {
  return stats ? 1 : scan == SCAN_BVHQ ? 6 : scan == SCAN_BVHQ7 ? 7 : scan == SCAN_BVHO ? 5 : 1;
}

template <int SRC, int SCAN, bool STATS = false>
__global__ __launch_bounds__(256, min_waves(SCAN, STATS)) void trace_kernel(const KArgs a) {
  // The sample pool: the workgroup's 8 x 8 pixels x spp samples are the
  // indices j in [0, npx * spp), sample-major (j -> pixel j % npx, sample
  // j / npx: the lanes ending paths together add into different pixels'
  // sums).  A lane whose path ends takes the next index from an LDS counter
  // (one ds_add per wave event, then an mbcnt prefix).  The colour sums are
  // u64 per pixel and channel in LDS, added with ds_add_u64: order-free.
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
  __shared__ int s_mb_post[4], s_mb_take[4], s_alive, s_mb_avail;
  // per wave: post when down to this many paths (0: posted once already; -1: off)
  __shared__ int s_mb_lim[4];
  // A/B build only (-DRTCLJ_AB_RING): camera samples made in
  // per-wave batches into LDS rings.  Worth 2.6 % at 5 workgroups per CU,
  // but its 5 KB of LDS keep the default traversal from the sixth (§8)
#ifdef RTCLJ_AB_RING
  constexpr bool kRing = SCAN == SCAN_BVHQ && !STATS;
#else
  constexpr bool kRing = false;
#endif
  constexpr int TH = tile_rows(SCAN);   // tile rows
  constexpr int NPX = kTile * TH;       // pool pixels
  // the pool's pixel sums: u32 in the compact variant (the host runs it only
  // when a sample's colour is <= 1 per channel and spp <= 255: a sum stays
  // below 255 * 2^24 < 2^32), u64 otherwise
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
  const bool own = unit < ka->n_units;
  // samples of whole tile t (its in-image pixels x spp)
  auto tile_pool = [&](KArgsP kp, int t) {
    const int ty = t / kp->tiles_x, tx = t - ty * kp->tiles_x;
    const int w = max(0, min(kTile, kp->width - tx * kTile)), h = max(0, min(TH, kp->rows_out - ty * TH));
    return kp->spp > 0 && kp->max_depth > 0 ? w * h * kp->spp : 0;
  };
  if (!own) {
    // ---- a helper: pick a tile still running, join it ----
    if (kRing || !ka->word) return;
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
    for (int i = 0; i < 2; ++i) {
      int w = w0 + static_cast<int>(threadIdx.x) + 256 * i;
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
      const unsigned long long wd = __hip_atomic_fetch_add(&ka->word[t], (1ull << 32) + 256u, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
      const int g = static_cast<int>(static_cast<unsigned>(wd));
      if (word_epoch(wd) == ka->epoch && g < P) {   // (another epoch: a spent word of an earlier launch)
        const int got = min(P - g, 256);
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
      for (int i = threadIdx.x; i < a.bvh_blob_f4; i += 256) {
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
      for (int i = threadIdx.x; i < a.bvh_blob_f4; i += 256) s_geo[i] = a.bvh_blob[i];
    } else {
      const float4* src = SCAN == SCAN_PK4 ? reinterpret_cast<const float4*>(a.geo2) : a.geo;
      for (int i = threadIdx.x; i < a.n_pad; i += 256) s_geo[i] = src[i];
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
  int tile, split_ix = 0, first = 0, nsplit = 1;
  bool split = false;
  if (own) {
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
  const int pool = (cnt > 0 && ka->max_depth > 0) ? npx * cnt : 0;
  const uint32_t mag_vw = vw > 0 ? 0xffffffffu / static_cast<uint32_t>(vw) + 1u : 0u;
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
  const bool shared_tile = !kRing && ka->word && !split && (!own || (pool > 512 && unit >= ka->share_from));
  // where the waves claim their batches: the shared tile's word, else (NULL)
  // the workgroup's s_pool_next
  unsigned long long* const src = shared_tile ? ka->word + tile : nullptr;
  // (batch_max 0: by the pool, 1/48 of it, 128 .. 1024)
  const int kc_batch_max = ka->batch_max > 0 ? ka->batch_max : min(1024, max(kShareBatch, (pool / 48) & ~63));
  if (threadIdx.x == 0) {
    if (own && shared_tile) {
      __hip_atomic_exchange(&ka->word[tile], (static_cast<unsigned long long>(ka->epoch) << 48) | 256ull,
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(&ka->owner[unit % ka->n_owner], tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_cnt = 256;
    }
    s_join = own ? 0 : 1;
    s_segs = 0ull;
    s_pool_next = kRing ? 0 : 256;   // (the ring claims its own)
    s_alive = 4;
    s_mb_avail = 0;   // (posted, not yet taken: a hint for the waves' exits to the step)
  }
  if (threadIdx.x < 4) {
    s_mb_post[threadIdx.x] = 0;
    s_mb_take[threadIdx.x] = 0;
    s_mb_lim[threadIdx.x] = ka->compact > 0 ? ka->compact : -1;
  }
  if (threadIdx.x < NPX * 3) s_acc[threadIdx.x] = 0;
  // the tile's pixel table (4-body-leaf traversal): per pool pixel its RNG
  // key and coordinates, so a camera sample costs one LDS read instead of
  // the index arithmetic and two hashes (the 8-body-leaf traversal's LDS
  // image has no room for it: C4 keeps 5 workgroups per CU)
  constexpr bool kPixelTable = is_q(SCAN) && !kRing;
  // (the compact variant: key and (x | y << 16) in 8 bytes)
  using PxT = std::conditional_t<SCAN == SCAN_BVHQ7, uint2, float4>;
  __shared__ PxT s_px[kPixelTable ? NPX : 1];
  if constexpr (kPixelTable) {
    const int t = static_cast<int>(threadIdx.x);
    if (t < npx) {
      const int qy = vw == 1 ? t : static_cast<int>(__umulhi(static_cast<uint32_t>(t), mag_vw));
      const int px = qx0 + (t - qy * vw);
      const int gy = image_row(qy0 + qy);
      if constexpr (SCAN == SCAN_BVHQ7)
        s_px[t] = make_uint2(pixel_key(px, gy), static_cast<unsigned>(px) | (static_cast<unsigned>(gy) << 16));
      else
        s_px[t] = make_float4(__uint_as_float(pixel_key(px, gy)), static_cast<float>(px), static_cast<float>(gy), 0.0f);
    }
  }
  __syncthreads();
  // the wave's batch [wb, we) of pool indices (wave-uniform; empty at first:
  // the lanes start on first + threadIdx.x)
  int wb = 0, we = 0;
  int j = first + static_cast<int>(threadIdx.x), q = 0, k = 0;
  bool active = kRing ? true : j < pool;
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
  bool fresh = !kRing;

  // ---- camera-sample ring (A/B build -DRTCLJ_AB_RING only) ----
  // Each wave keeps up to 64 camera samples ready in LDS ([field][slot]: RNG
  // state after the sample's draws, fx, fy, the disk draws' 24-bit integers
  // with the pool pixel in the top byte of the first).  A wave whose lanes
  // need more samples than it holds makes a batch with all its lanes at once
  // (pool index -> pixel, two hashes, the jitter and the defocus-disk
  // rejection loop), so that work runs with full waves instead of with the
  // ~26 lanes that end a path in an iteration; a lane whose path ended takes
  // the next sample from the ring and sets up its camera ray.  Every sample
  // is computed with the same ops as before: the same bits.
  constexpr int kRingN = 64;
  __shared__ uint32_t s_ring[kRing ? 4 * 5 * kRingN : 1];
  uint32_t* const ring = s_ring + (kRing ? (threadIdx.x >> 6) * 5 * kRingN : 0);
  int r_head = 0, r_count = 0;   // wave-uniform: the next slot to hand out, samples held
  int r_seen = 0;                // wave-uniform: the pool counter after this wave's last batch
  auto ring_fill = [&](int need) {   // run by every lane still in the loop (wave-uniform branch)
    const uint64_t ex = __builtin_amdgcn_read_exec();
    const int nact = __popcll(ex);
    const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(ex >> 32),
                                                                __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(ex), 0u)));
    // a full batch, except near the pool's end: then only what is needed now,
    // so that no wave holds samples the workgroup's other waves could run
    // (the pool's progress as this wave last saw it: no extra LDS read)
    const int g = pool - r_seen < 4 * kRingN ? need : min(kRingN - r_count, nact);
    const int leader = __ffsll(static_cast<long long>(ex)) - 1;
    int b = 0;
    if (lane == leader) b = atomicAdd(&s_pool_next, g);
    b = __builtin_amdgcn_readlane(b, leader);
    r_seen = b + g;
    if (rank < g) {
      const int jj = b + rank;
      uint32_t e_st = 0, e_a = 0xff000000u, e_b = 0;   // pixel 0xff: the pool is empty
      float e_fx = 0.0f, e_fy = 0.0f;
      if (jj < pool) {
        // sample-major (pixel jj mod npx, sample jj / npx): a batch is one
        // sample of each of the tile's pixels, neighbouring rays, and the
        // lanes ending paths together add into different pixels' sums
        const int kk = div_magic(jj, npx_magic);
        const int qq = jj - kk * npx;
        const int qy = vw == 1 ? qq : static_cast<int>(__umulhi(static_cast<uint32_t>(qq), mag_vw));
        const int px = qx0 + (qq - qy * vw);
        const int gy = image_row(qy0 + qy);
        // ---- compute-pixel, one sample (raytracing.clj:144-151) ----
        uint32_t rs = mix32(pixel_key(px, gy) + static_cast<uint32_t>(a.sample_begin + k0 + kk) * 0x9e3779b9u);
        if (rs == 0) rs = 0x6d2b79f5u;
        e_fx = static_cast<float>(px) + rng_centered(rs);
        e_fy = static_cast<float>(gy) + rng_centered(rs);
        uint32_t ix = 0, iy = 0;
        if (a.defocus) {
          // defocus-disk-sample + random-in-unit-disk (raytracing.clj:89-93, vec3a.clj:81-86):
          // rng_sym's draws, kept as their 24-bit integers
          float qx, qy2;
          do {
            rs ^= rs << 13;
            rs ^= rs >> 17;
            rs ^= rs << 5;
            ix = rs >> 8;
            rs ^= rs << 13;
            rs ^= rs >> 17;
            rs ^= rs << 5;
            iy = rs >> 8;
            qx = fmaf(static_cast<float>(ix), 0x1p-23f, -1.0f);
            qy2 = fmaf(static_cast<float>(iy), 0x1p-23f, -1.0f);
          } while (!(fmaf(qy2, qy2, qx * qx) < 1.0f));
        }
        e_st = rs;
        e_a = ix | (static_cast<uint32_t>(qq) << 24);
        e_b = iy;
      }
      const int slot = (r_head + r_count + rank) & (kRingN - 1);
      ring[0 * kRingN + slot] = e_st;
      ring[1 * kRingN + slot] = __float_as_uint(e_fx);
      ring[2 * kRingN + slot] = __float_as_uint(e_fy);
      ring[3 * kRingN + slot] = e_a;
      ring[4 * kRingN + slot] = e_b;
    }
    r_count += g;
  };
  // the lanes in `m` (wave-uniform mask, taken: lanes with take) start their
  // next sample from the ring; a lane given no sample retires
  auto ring_take = [&](uint64_t m, bool take) {
    const int nt = __popcll(m);
    if (r_count < nt) ring_fill(nt - r_count);
    asm volatile("" ::: "memory");   // the batch's LDS writes before the reads (in order per wave)
    if (take) {
      const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
      const int slot = (r_head + rank) & (kRingN - 1);
      // all five fields in flight at once: the ray is set up unconditionally
      // (from the empty entry's zeros when the pool is done: harmless, the
      // lane retires before it traces)
      const uint32_t e0 = ring[0 * kRingN + slot], e1 = ring[1 * kRingN + slot], e2 = ring[2 * kRingN + slot];
      const uint32_t ea = ring[3 * kRingN + slot], eb = ring[4 * kRingN + slot];
      st = e0;
      const float fx = __uint_as_float(e1);
      const float fy = __uint_as_float(e2);
      q = static_cast<int>(ea >> 24);
      const float sx = fmaf(a.cam[9], fy, fmaf(a.cam[6], fx, a.cam[3]));
      const float sy = fmaf(a.cam[10], fy, fmaf(a.cam[7], fx, a.cam[4]));
      const float sz = fmaf(a.cam[11], fy, fmaf(a.cam[8], fx, a.cam[5]));
      if (a.defocus) {
        const float qx = fmaf(static_cast<float>(ea & 0xffffffu), 0x1p-23f, -1.0f);
        const float qy2 = fmaf(static_cast<float>(eb), 0x1p-23f, -1.0f);
        ox = fmaf(a.cam[15], qy2, fmaf(a.cam[12], qx, cx));
        oy = fmaf(a.cam[16], qy2, fmaf(a.cam[13], qx, cy));
        oz = fmaf(a.cam[17], qy2, fmaf(a.cam[14], qx, cz));
      } else {
        ox = cx;
        oy = cy;
        oz = cz;
      }
      dx = sx - ox;
      dy = sy - oy;
      dz = sz - oz;
      tr = tg = tb = 1.0f;
      rem = a.max_depth;
      last = -1;
      if (q == 0xff) active = false;   // the pool is done
    }
    r_head += nt;
    r_count -= nt;
  };
  if constexpr (kRing) {
    ring_take(__ballot(1), true);   // every lane's first sample
  }

  // Drain compaction keeps every lane of a wave in the loop
  // once its batches are spent (a lane without a path skips the body; the
  // step after it may give it a path a sibling wave posted); the wave leaves
  // when none of its lanes has one
#ifdef RTCLJ_AB_NOCOMPACT
  constexpr bool kCompact = false;   // (A/B build: the loop without compaction)
#else
  constexpr bool kCompact = !kRing && is_bvh_scan(SCAN);
#endif
  const int wv = static_cast<int>(threadIdx.x >> 6);
  auto mb_word = [&](int d, int f, int p, int P) -> uint32_t* {
    constexpr int SZ = static_cast<int>(sizeof(StackT));
    constexpr int W = 16 * SZ;   // words per stack row per wave
    const int i = f * P + p;
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_stack) + (i / W) * 256 * SZ + d * 64 * SZ +
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
    const int P = kargs_opaque()->mb_paths;
    const int leader = static_cast<int>(__builtin_amdgcn_readfirstlane(lane));
    const uint64_t live = __ballot(active);
    const int left = static_cast<int>(__popcll(live));
    bool out = false;   // counted out, and the last wave to do so
    bool post = false;
    if (left > 0 && left <= sgpr(lds_load(&s_mb_lim[wv]))) {
      post = sgpr(lds_load(&s_alive)) > 1;
      // posting now; or alone (no sibling will ever take them): not again
      if (lane == leader) __hip_atomic_store(&s_mb_lim[wv], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (left == 0 || post) {
      if (post) {
        const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(live >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(live), 0u)));
        if (active) {
          *mb_word(wv, 0, rank, P) = __float_as_uint(ox);
          *mb_word(wv, 1, rank, P) = __float_as_uint(oy);
          *mb_word(wv, 2, rank, P) = __float_as_uint(oz);
          *mb_word(wv, 3, rank, P) = __float_as_uint(dx);
          *mb_word(wv, 4, rank, P) = __float_as_uint(dy);
          *mb_word(wv, 5, rank, P) = __float_as_uint(dz);
          *mb_word(wv, 6, rank, P) = __float_as_uint(tr);
          *mb_word(wv, 7, rank, P) = __float_as_uint(tg);
          *mb_word(wv, 8, rank, P) = __float_as_uint(tb);
          *mb_word(wv, 9, rank, P) = st;
          *mb_word(wv, 10, rank, P) = static_cast<uint32_t>(q);
          *mb_word(wv, 11, rank, P) = static_cast<uint32_t>(rem);
          *mb_word(wv, 12, rank, P) = static_cast<uint32_t>(last);
        }
      }
      int old = 0;
      if (lane == leader) {
        if (post) {
          __hip_atomic_store(&s_mb_post[wv], left, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          atomicAdd(&s_mb_avail, left);
        }
        old = __hip_atomic_fetch_add(&s_alive, -1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        // the last one out withdraws its post (no sibling is left to take any of it)
        if (post && old <= 1) {
          __hip_atomic_store(&s_mb_post[wv], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
    for (int d = 0; d < 4 && freem; ++d) {
      if (d == wv) continue;
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
    if (kCompact ? j >= 0 : fresh) {
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
      if constexpr (kPixelTable && SCAN == SCAN_BVHQ7) {
        const uint2 pt = s_px[q];
        pk = pt.x;
        fpx = static_cast<float>(pt.y & 0xffffu);
        fgy = static_cast<float>(pt.y >> 16);
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
        do {
          if constexpr (STATS) {
            wave_event(st_disk);
            st_fl += 7;   // 2 x (2 xi - 1) + |q|^2
          }
          qx = rng_sym(st);
          qy2 = rng_sym(st);
        } while (!(fmaf(qy2, qy2, qx * qx) < 1.0f));
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


    if constexpr (STATS) {
      const uint64_t t = stamp();
      st_c_cam += t - st_ts;
      st_ts = t;
    }
    // ---- one ray-color level: hit-anything over all bodies ----
    --rem;
    ++segs;
    const float len = sqrt_rn(fmaf(dz, dz, fmaf(dy, dy, dx * dx)));
    const float il = 1.0f / len;                              // vec3a/unit as d * (1/|d|)
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
    if constexpr (SCAN == SCAN_SIMPLE) {
#pragma unroll 4
      for (int s = 0; s < n; ++s) {
        float4 g;
        if constexpr (SRC == SRC_LDS) g = s_geo[s];
        else g = a.geo[s];
        // hittable.clj:10-14 with a unit direction: a = 1, h = u.oc,
        // c = |oc|^2 - r^2 (y first: the big ground sphere cancels exactly in the fma)
        const float ocx = g.x - ox, ocy = g.y - oy, ocz = g.z - oz;
        const float h = fmaf(uz, ocz, fmaf(uy, ocy, ux * ocx));
        const float c = fmaf(ocx, ocx, fmaf(ocz, ocz, fmaf(ocy, ocy, g.w)));
        const float disc = fmaf(h, h, -c);
        // h < 0 && c >= 0: both roots <= 0 (exact in fp: sqrt(RN(h*h)) = |h|)
        if ((disc >= 0.0f) & ((h >= 0.0f) | (c < 0.0f))) consider(h, disc, s);
      }
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
            if constexpr (STATS) {
              const uint64_t ex = __builtin_amdgcn_read_exec();
              if (lane == __ffsll(static_cast<long long>(ex)) - 1) ++st_consw;
            }
            const unsigned k = __builtin_ctz(m);
            m &= m - 1;
            float h, c, disc;
            body(pa + k + k, h, c, disc);
            const int sidx = *(const int __attribute__((address_space(3)))*)(uintptr_t)(pa + 64u + (k >> 1));
            consider_tie(h, disc, sidx);
          }
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
      for (int b = 0; b < a.n_big_leaves; ++b) {
        if constexpr (kLeafRec)
          leaf(static_cast<int>(lds_addr(nodes)) + a.bvh_off_pairs + ((a.big_pair0 >> 1) + b) * kLeafRecBytes);
        else
          leaf(a.big_pair0 + b * leaf_pairs(SCAN));
      }
      if constexpr (SCAN == SCAN_BVHWW) {
        // speculative while-while (Aila & Laine 2009): a node phase in which
        // a lane that already holds a leaf keeps descending until every lane
        // holds one (or has run out of nodes), then one leaf phase in which
        // the lanes test their leaves together -- the wave no longer runs the
        // leaf test for a few lanes at every node step.  Stack entries are
        // child refs (node >= 0, leaf ~p < 0); at most depth + 2 are live.
        short* stk = reinterpret_cast<short*>(s_stack);
        int node = 0, pend = -1, sp = 0;
        for (;;) {
          while (node >= 0) {
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
            const bool sw = tn1 < tn0;   // near child first
            const int cn = sw ? c1 : c0, cf = sw ? c0 : c1;
            const bool hn = sw ? hit1 : hit0, hf = sw ? hit0 : hit1;
            int next = -1;
            if (hf) {       // far child: pushed unless it is the only way on
              if (cf < 0 && pend < 0 && !(hn && cn < 0)) pend = ~cf;
              else if (cf >= 0 && !hn) next = cf;
              else stk[(sp++) * 256 + threadIdx.x] = static_cast<short>(cf);
            }
            if (hn) {
              if (cn < 0) {
                if (pend < 0) pend = ~cn;
                else stk[(sp++) * 256 + threadIdx.x] = static_cast<short>(cn);
              } else {
                next = cn;
              }
            }
            node = next;
            if (node < 0) {
              if (pend >= 0 || sp == 0) break;       // test the leaf first / done
              const int e = stk[(--sp) * 256 + threadIdx.x];
              if (e >= 0) {
                node = e;
              } else {
                pend = ~e;
                break;
              }
            }
            if (__all(pend >= 0)) break;             // every lane holds a leaf
          }
          if (pend >= 0) {
            leaf(pend);
            pend = -1;
          }
          if (node < 0) {
            if (sp == 0) break;
            const int e = stk[(--sp) * 256 + threadIdx.x];
            if (e >= 0) node = e;
            else pend = ~e;
          }
        }
      } else {
      // the root: the 4-body tree's refs are LDS addresses (relocated as copied)
      int node = SRC == SRC_LDS && SCAN == SCAN_BVHQ ? static_cast<int>(lds_addr(nodes)) : 0;   // (BVHQ7: index 0)
      // the stack top as a pointer into the [entry][lane] stack: one add per
      // push / pop instead of index arithmetic
      StackT* const stk0 = s_stack + threadIdx.x;
      StackT* top = stk0;
      // a row of the stack in bytes, held in a register the compiler cannot
      // rematerialise (a literal would be moved into a VGPR on every push)
      int row_b = 256 * static_cast<int>(sizeof(StackT));
      asm volatile("" : "+v"(row_b));
      bool go = true;
      while (go) {
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
          top -= 256;
          go = top >= stk0;
          nxt = *top;
        }
        node = nxt;
      }
      }
      // the ray's origin and unit direction again from the packed copies the
      // walk used (the same values): the scalar ones are dead through it,
      // six VGPRs fewer at its peak
      ox = o_xy.x;
      oy = o_xy.y;
      oz = o_zux.x;
      ux = o_zux.y;
      uy = u_yz.x;
      uz = u_yz.y;
    } else if constexpr (SCAN == SCAN_PK4) {
      // As SCAN_GROUP4, but the arithmetic of two bodies runs in one packed
      // instruction (v_pk_add/mul/fma_f32: each half is the same IEEE-rounded
      // op as the scalar form, so the bits are unchanged); the group's
      // "any candidate" test is one max-reduction and one compare.
      const Pair* tab;
      if constexpr (SRC == SRC_LDS) tab = reinterpret_cast<const Pair*>(s_geo);
      else tab = a.geo2;
      const f2 ox2 = {ox, ox}, oy2 = {oy, oy}, oz2 = {oz, oz};
      const f2 ux2 = {ux, ux}, uy2 = {uy, uy}, uz2 = {uz, uz};
      Pair A = tab[0], B = tab[1];
      for (int s = 0; s < n; s += 4) {
        const Pair nA = tab[(s >> 1) + 2], nB = tab[(s >> 1) + 3];
        f2 h[2], c[2], disc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const Pair& g = j == 0 ? A : B;
          const f2 ocx = g.x - ox2, ocy = g.y - oy2, ocz = g.z - oz2;
          h[j] = fma2(uz2, ocz, fma2(uy2, ocy, ux2 * ocx));
          c[j] = fma2(ocx, ocx, fma2(ocz, ocz, fma2(ocy, ocy, g.w)));
          disc[j] = fma2(h[j], h[j], -c[j]);
        }
        const float q0 = fminf(disc[0].x, fmaxf(h[0].x, -c[0].x));
        const float q1 = fminf(disc[0].y, fmaxf(h[0].y, -c[0].y));
        const float q2 = fminf(disc[1].x, fmaxf(h[1].x, -c[1].x));
        const float q3 = fminf(disc[1].y, fmaxf(h[1].y, -c[1].y));
        if (fmaxf(fmaxf(q0, q1), fmaxf(q2, q3)) >= 0.0f) {
          if (q0 >= 0.0f) consider(h[0].x, disc[0].x, s);
          if (q1 >= 0.0f) consider(h[0].y, disc[0].y, s + 1);
          if (q2 >= 0.0f) consider(h[1].x, disc[1].x, s + 2);
          if (q3 >= 0.0f) consider(h[1].y, disc[1].y, s + 3);
        }
        A = nA;
        B = nB;
      }
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
        random_unit<STATS>(st, qx, qy, qz, &st_ball, &st_fl);
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
    if (done) {   // the sample's colour into its pixel's fixed-point sum (order-free)
      if constexpr (STATS) st_fl += 3;
      AccT* acc = &s_acc[q * 3];
      __hip_atomic_fetch_add(acc + 0, static_cast<AccT>(fix24(cr)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(acc + 1, static_cast<AccT>(fix24(cg)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(acc + 2, static_cast<AccT>(fix24(cb)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // refill: the lanes whose paths ended take their next indices
    const uint64_t m = __ballot(done);
    if constexpr (kRing) {
      if (m) ring_take(m, done);
    } else if (m) {
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
          } else {
            g = atomicAdd(&s_pool_next, want);
          }
        }
        g = __builtin_amdgcn_readlane(g, leader);
        wb = min(g, pool);
        we = min(g + want, pool);
        if (wb >= pool) we = pool;   // spent: the lanes left over retire
      }
      if (done) {
        j = kCompact && nj < 0 ? -2 : nj;
        fresh = true;
        if (nj < 0) active = false;
      }
    }
    if constexpr (STATS) st_c_acc += stamp() - st_ts;
    if constexpr (kCompact) {
      // spent: out to the compaction step when this wave may post its few
      // paths, or its idle lanes may take posted ones
      // (the limit and the flags from LDS: no registers held for them)
      if (wb >= pool) {
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

  // ---- per-pixel mean (compute-pixel's accum / spp, raytracing.clj:155) ----
  // thread t < 3 * npx writes channel t % 3 of pool pixel t / 3: a tile row's
  // 8 pixels are 24 consecutive floats
  __syncthreads();
  const KArgsP ke = kargs_opaque();
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
  if (split) {   // one split's integer sums, added to the tile's (order-free); finalize_kernel converts them
    if (t < npx * 3 && s_acc[t])
      __hip_atomic_fetch_add(&ke->part[out_index(t)], static_cast<unsigned long long>(s_acc[t]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  } else if (alone) {   // every sample of the tile was this workgroup's
    if (t < npx * 3) write_mean(out_index(t), static_cast<unsigned long long>(s_acc[t]));
  } else {
    // a shared tile (owner or helper): the integer sums
    // meet in sum[tile] (atomics: any order, the same total); the workgroup
    // whose samples complete the pool converts them and re-zeroes the slots
    unsigned long long* gs = ke->sum + static_cast<size_t>(tile) * (NPX * 3);
    if (t < npx * 3 && s_acc[t])
      __hip_atomic_fetch_add(&gs[t], static_cast<unsigned long long>(s_acc[t]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    const size_t wid = static_cast<size_t>(unit) * 4 + (threadIdx.x >> 6);   // by dispatch slot
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

// ------------------------------------------------ direction-coherent waves ----
// sorted_kernel<SORT> (variants 20 / 21; DESIGN.md §3.6, an A/B against the
// default traversal 16).  The same sample pool, traversal (the 4-body-leaf
// BVH in LDS), shading and fixed-point sums as trace_kernel, in a different
// execution shape: a 512-thread workgroup (8 waves) owns an 8 x 16-pixel
// tile, and its waves advance in lock step, one ray-color level per
// iteration.  Before every iteration the workgroup's 512 paths are dealt to
// its waves in key order -- fresh camera samples first, then the bounce
// paths by the octant of their direction (SORT; without it only the live
// paths are packed into the first waves) -- through an exchange buffer in
// LDS, so that a wave's lanes traverse the tree in similar directions
// (tools/simt_sim.cpp priced it: 59.3 against 66.5 VALU per sample for the
// shipped shape).  Paths without a path state (the pool's drain) sink to the
// last waves, which skip the iteration: the exchange is also the drain's
// compaction.  One tree copy serves 8 waves, so the exchange buffer fits
// beside it at 3 workgroups (6 waves per SIMD) per CU.
//
// Exchange buffer ([wave][field][lane] u32, 11 fields a path): a fresh
// sample is its pool index (field 0); a bounce path is origin, direction,
// throughput, RNG state and (pixel | depth left << 7 | (body left + 1) << 17).
// After the exchange a wave's traversal stack lives in its own slots of the
// buffer (it has read them before it pushes).
constexpr int kSortWaves = 8;
constexpr int kSortThreads = 64 * kSortWaves;
constexpr int kSortTH = 16;                       // tile rows
constexpr int kSortNPX = kTile * kSortTH;         // pool pixels
constexpr int kSortKeys = 10;                     // 0 fresh, 1..8 octants, 9 no path
constexpr int kXFields = 11;
constexpr int kXWaveWords = kXFields * 64;        // a wave's slots (u32)
constexpr size_t kXBytes = static_cast<size_t>(kSortWaves) * kXWaveWords * 4;   // 22,528

template <bool SORT>
__global__ __launch_bounds__(kSortThreads, 6) void sorted_kernel(const KArgs a) {
  __shared__ int s_pool_next;
  __shared__ unsigned long long s_segs;
  __shared__ unsigned long long s_acc[kSortNPX * 3];
  __shared__ float4 s_px[kSortNPX];
  __shared__ int s_cnt[kSortWaves * kSortKeys];
  extern __shared__ __attribute__((aligned(16))) float4 s_geo[];
  uint64_t st_t0 = 0;
  const int lane = threadIdx.x & 63;
  const int wv = static_cast<int>(threadIdx.x >> 6);
  const int unit = static_cast<int>(blockIdx.x);
  const KArgsP ka = kargs_opaque();
  for (int i = threadIdx.x; i < a.bvh_blob_f4; i += kSortThreads) s_geo[i] = a.bvh_blob[i];
  if (ka->tile_cost) st_t0 = __builtin_amdgcn_s_memrealtime();
  // the unit: a whole tile, or one sample split of a tile (as trace_kernel)
  int pos = unit, split_ix = 0, nsplit = 1, tile;
  const bool split = unit >= ka->n_whole;
  if (split && ka->unit_tab) {
    const int2 u = ka->unit_tab[unit - ka->n_whole];
    if (u.x < 0) return;
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
  const int tby = tile / ka->tiles_x, tbx = tile - tby * ka->tiles_x;
  const int qx0 = tbx * kTile, qy0 = tby * kSortTH;
  const int vw = max(0, min(kTile, ka->width - qx0));
  const int vh = max(0, min(kSortTH, ka->rows_out - qy0));
  const int npx = vw * vh;
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
  const int k0 = split ? static_cast<int>(static_cast<int64_t>(split_ix) * ka->spp / nsplit) : 0;
  const int cnt = split ? static_cast<int>(static_cast<int64_t>(split_ix + 1) * ka->spp / nsplit) - k0 : ka->spp;
  const int pool = (cnt > 0 && ka->max_depth > 0) ? npx * cnt : 0;
  const uint32_t mag_vw = vw > 0 ? 0xffffffffu / static_cast<uint32_t>(vw) + 1u : 0u;
  const uint64_t npx_magic = npx > 1 ? ~0ull / static_cast<uint64_t>(npx) + 1ull : 0ull;
  if (threadIdx.x == 0) {
    s_pool_next = 0;
    s_segs = 0ull;
  }
  if (threadIdx.x < kSortNPX * 3) s_acc[threadIdx.x] = 0ull;
  {
    const int t = static_cast<int>(threadIdx.x);
    if (t < npx) {
      const int qy = vw == 1 ? t : static_cast<int>(__umulhi(static_cast<uint32_t>(t), mag_vw));
      const int px = qx0 + (t - qy * vw);
      const int gy = image_row(qy0 + qy);
      s_px[t] = make_float4(__uint_as_float(pixel_key(px, gy)), static_cast<float>(px), static_cast<float>(gy), 0.0f);
    }
  }
  __syncthreads();

  uint32_t* const xw = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_geo) + a.bvh_blob_f4 * 16);
  auto xslot = [&](int slot, int f) -> uint32_t* { return xw + ((slot >> 6) * kXFields + f) * 64 + (slot & 63); };
  // j: >= 0 a fresh sample (pool index), -1 a path in progress, -2 none
  int j = -2, q = 0;
  uint32_t st = 0;
  float ox = 0, oy = 0, oz = 0, dx = 0, dy = 0, dz = 0;
  float tr = 1, tg = 1, tb = 1;
  int rem = 0, last = -1;
  bool spent = pool == 0;   // wave-uniform: the pool is handed out
  uint32_t segs = 0;
  const KNode* nodes = reinterpret_cast<const KNode*>(s_geo);
  const Pair* pairs = reinterpret_cast<const Pair*>(reinterpret_cast<const char*>(s_geo) + a.bvh_off_pairs);
  const int2* pidx = reinterpret_cast<const int2*>(reinterpret_cast<const char*>(s_geo) + a.bvh_off_pidx);
  // this wave's traversal stack: its own exchange slots, [entry][lane] u16
  unsigned short* const stk0 = reinterpret_cast<unsigned short*>(xw + wv * kXWaveWords) + lane;

  for (;;) {
    // ---- refill: lanes without a path take the next pool indices ----
    if (!spent) {
      const uint64_t m = __ballot(j == -2);
      if (m) {
        const int need = static_cast<int>(__popcll(m));
        const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
        int g = 0;
        if (lane == 0) g = atomicAdd(&s_pool_next, need);
        g = __builtin_amdgcn_readlane(g, 0);
        if (j == -2) j = g + rank < pool ? g + rank : -2;
        spent = g + need >= pool;
      }
    }
    // ---- deal the workgroup's paths to its waves in key order ----
    int key = 9;
    if (j >= 0) key = 0;
    else if (j == -1) key = SORT ? 1 + ((dx < 0.0f) ? 1 : 0) + ((dy < 0.0f) ? 2 : 0) + ((dz < 0.0f) ? 4 : 0) : 1;
    uint64_t mine = 0;
    int mycnt = 0;
#pragma unroll
    for (int k = 0; k < kSortKeys; ++k) {
      if (!SORT && k >= 2 && k < 9) continue;
      const uint64_t b = __ballot(key == k);
      mine = key == k ? b : mine;
      mycnt = lane == k ? static_cast<int>(__popcll(b)) : mycnt;
    }
    const int myrank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mine >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mine), 0u)));
    if (lane < kSortKeys) s_cnt[wv * kSortKeys + lane] = mycnt;
    __syncthreads();
    // lane k < 10: key k's count over the waves, and in the waves before this one
    int tot = 0, before = 0;
    if (lane < kSortKeys) {
#pragma unroll
      for (int w2 = 0; w2 < kSortWaves; ++w2) {
        const int c = s_cnt[w2 * kSortKeys + lane];
        tot += c;
        before += w2 < wv ? c : 0;
      }
    }
    int scan = tot;   // inclusive prefix over the keys (lanes 0..9)
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const int v = __shfl_up(scan, off);
      scan += lane >= off ? v : 0;
    }
    const int n_live = __builtin_amdgcn_readlane(scan, 8);    // keys 0..8: the paths and fresh samples
    const int n_fresh = __builtin_amdgcn_readlane(tot, 0);
    if (n_live == 0) break;   // (workgroup-uniform: every wave read the same counts)
    const int base_k = scan - tot + before;                   // lane k: this wave's first slot of key k
    const int dst = __shfl(base_k, key) + myrank;
    if (key == 0) {
      *xslot(dst, 0) = static_cast<uint32_t>(j);
    } else if (key < 9) {
      *xslot(dst, 0) = __float_as_uint(ox);
      *xslot(dst, 1) = __float_as_uint(oy);
      *xslot(dst, 2) = __float_as_uint(oz);
      *xslot(dst, 3) = __float_as_uint(dx);
      *xslot(dst, 4) = __float_as_uint(dy);
      *xslot(dst, 5) = __float_as_uint(dz);
      *xslot(dst, 6) = __float_as_uint(tr);
      *xslot(dst, 7) = __float_as_uint(tg);
      *xslot(dst, 8) = __float_as_uint(tb);
      *xslot(dst, 9) = st;
      *xslot(dst, 10) = static_cast<uint32_t>(q) | (static_cast<uint32_t>(rem) << 7) |
                        (static_cast<uint32_t>(last + 1) << 17);
    }
    __syncthreads();
    {
      const int t = static_cast<int>(threadIdx.x);
      if (t < n_fresh) {
        j = static_cast<int>(*xslot(t, 0));
      } else if (t < n_live) {
        ox = __uint_as_float(*xslot(t, 0));
        oy = __uint_as_float(*xslot(t, 1));
        oz = __uint_as_float(*xslot(t, 2));
        dx = __uint_as_float(*xslot(t, 3));
        dy = __uint_as_float(*xslot(t, 4));
        dz = __uint_as_float(*xslot(t, 5));
        tr = __uint_as_float(*xslot(t, 6));
        tg = __uint_as_float(*xslot(t, 7));
        tb = __uint_as_float(*xslot(t, 8));
        st = *xslot(t, 9);
        const uint32_t meta = *xslot(t, 10);
        q = static_cast<int>(meta & 127u);
        rem = static_cast<int>((meta >> 7) & 1023u);
        last = static_cast<int>(meta >> 17) - 1;
        j = -1;
      } else {
        j = -2;
      }
    }
    if (wv * 64 >= n_live) continue;   // (wave-uniform: no path in this wave; the barriers above)
    if (j < -1) continue;
    // ---- a fresh sample: compute-pixel's camera ray (raytracing.clj:144-151) ----
    if (j >= 0) {
      const int k = div_magic(j, npx_magic);
      q = j - k * npx;
      const float4 pt = s_px[q];
      st = mix32(__float_as_uint(pt.x) + static_cast<uint32_t>(a.sample_begin + k0 + k) * 0x9e3779b9u);
      if (st == 0) st = 0x6d2b79f5u;
      const float fx = pt.y + rng_centered(st);
      const float fy = pt.z + rng_centered(st);
      const float sx = fmaf(a.cam[9], fy, fmaf(a.cam[6], fx, a.cam[3]));
      const float sy = fmaf(a.cam[10], fy, fmaf(a.cam[7], fx, a.cam[4]));
      const float sz = fmaf(a.cam[11], fy, fmaf(a.cam[8], fx, a.cam[5]));
      if (a.defocus) {
        float qx, qy2;
        do {
          qx = rng_sym(st);
          qy2 = rng_sym(st);
        } while (!(fmaf(qy2, qy2, qx * qx) < 1.0f));
        ox = fmaf(a.cam[15], qy2, fmaf(a.cam[12], qx, cx));
        oy = fmaf(a.cam[16], qy2, fmaf(a.cam[13], qx, cy));
        oz = fmaf(a.cam[17], qy2, fmaf(a.cam[14], qx, cz));
      } else {
        ox = cx;
        oy = cy;
        oz = cz;
      }
      dx = sx - ox;
      dy = sy - oy;
      dz = sz - oz;
      tr = tg = tb = 1.0f;
      rem = a.max_depth;
      last = -1;
      j = -1;
    }
    // ---- one ray-color level (as trace_kernel's SCAN_BVHQ iteration) ----
    bool done = false;
    --rem;
    ++segs;
    const float len = sqrt_rn(fmaf(dz, dz, fmaf(dy, dy, dx * dx)));
    const float il = 1.0f / len;
    const float ux = dx * il, uy = dy * il, uz = dz * il;
    const float tmin = 1e-3f * len;
    float best_t = INFINITY;
    int best = -1;
    {
      auto consider_tie = [&](float h, float disc, int s) {
        const float sq = (s == last) ? fabsf(h) : sqrt_rn(disc);
        const float tn = h - sq;
        const float t = tn > tmin ? tn : h + sq;
        const uint64_t kk = (static_cast<uint64_t>(__float_as_uint(t)) << 32) | static_cast<uint32_t>(s);
        const uint64_t bkey = (static_cast<uint64_t>(__float_as_uint(best_t)) << 32) | static_cast<uint32_t>(best);
        const bool acc = (t > tmin) & (kk < bkey);
        best_t = acc ? t : best_t;
        best = acc ? s : best;
      };
      const float ecx = ox - a.bvh_c[0], ecy = oy - a.bvh_c[1], ecz = oz - a.bvh_c[2];
      const float D = __builtin_amdgcn_sqrtf(fmaf(ecz, ecz, fmaf(ecy, ecy, ecx * ecx))) + a.bvh_r;
      const float P = fmaf(2e-3f, D, 1e-6f);
      const float rux = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(ux), -1e24f, 1e24f);
      const float ruy = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(uy), -1e24f, 1e24f);
      const float ruz = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(uz), -1e24f, 1e24f);
      f2 r_xy = {rux, ruy}, r_z = {ruz, ruz};
      const float nlx = -(ecx + P) * rux, nly = -(ecy + P) * ruy, nlz = -(ecz + P) * ruz;
      const float nhx = -(ecx - P) * rux, nhy = -(ecy - P) * ruy, nhz = -(ecz - P) * ruz;
      const bool sx = rux < 0.0f, sy = ruy < 0.0f, sz = ruz < 0.0f;
      f2 nf_x = {sx ? nhx : nlx, sx ? nlx : nhx};
      f2 nf_y = {sy ? nhy : nly, sy ? nly : nhy};
      f2 nf_z = {sz ? nhz : nlz, sz ? nlz : nhz};
      const int offx = sx ? 8 : 0, offy = 24 + (sy ? 8 : 0), offz = 48 + (sz ? 8 : 0);
      f2 o_xy = {ox, oy}, o_zux = {oz, ux}, u_yz = {uy, uz};
      auto leaf = [&](int p) {
        float hh[4], dd[4];
        int ii[4];
        unsigned nc[4];
        const Pair* const lp = pairs + p;
        const int2* const li = pidx + p;
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const Pair g = lp[qq];
          const int2 id = li[qq];
          asm volatile("" : "+v"(o_xy), "+v"(o_zux), "+v"(u_yz));
          const f2 ocx = g.x - bc_lo(o_xy), ocy = g.y - bc_hi(o_xy), ocz = g.z - bc_lo(o_zux);
          const f2 h = fma2(bc_hi(u_yz), ocz, fma2(bc_lo(u_yz), ocy, bc_hi(o_zux) * ocx));
          const f2 c = fma2(ocx, ocx, fma2(ocz, ocz, fma2(ocy, ocy, g.w)));
          const f2 disc = fma2(h, h, -c);
          hh[2 * qq] = h.x;
          hh[2 * qq + 1] = h.y;
          dd[2 * qq] = disc.x;
          dd[2 * qq + 1] = disc.y;
          ii[2 * qq] = id.x;
          ii[2 * qq + 1] = id.y;
          const float d0 = disc.x, d1 = disc.y, h0 = h.x, h1 = h.y, c0 = c.x, c1 = c.y;
          nc[2 * qq] = __builtin_amdgcn_bitop3_b32(__float_as_uint(d0), __float_as_uint(h0), __float_as_uint(c0), 0x0b);
          nc[2 * qq + 1] = __builtin_amdgcn_bitop3_b32(__float_as_uint(d1), __float_as_uint(h1), __float_as_uint(c1), 0x0b);
        }
        const unsigned b01 = __builtin_amdgcn_perm(nc[1], nc[0], 0x0c0c0b09u);
        const unsigned b23 = __builtin_amdgcn_perm(nc[3], nc[2], 0x0b090c0cu);
        unsigned m = __builtin_amdgcn_bitop3_b32(b01, b23, 0x01010101u, 0xa8);
        while (m) {
          const unsigned k = __builtin_ctz(m);
          m &= m - 1;
          float h = hh[0], d = dd[0];
          int s = ii[0];
#pragma unroll
          for (int jj = 1; jj < 4; ++jj) {
            h = k == static_cast<unsigned>(8 * jj) ? hh[jj] : h;
            d = k == static_cast<unsigned>(8 * jj) ? dd[jj] : d;
            s = k == static_cast<unsigned>(8 * jj) ? ii[jj] : s;
          }
          consider_tie(h, d, s);
        }
      };
      auto node_test = [&](int node, float& tn0, float& tn1, bool& hit0, bool& hit1, int& c0, int& c1) {
        const char* nb = reinterpret_cast<const char*>(nodes) + static_cast<unsigned>(node);
        const f2* ax = reinterpret_cast<const f2*>(nb + offx);
        const f2* ay = reinterpret_cast<const f2*>(nb + offy);
        const f2* az = reinterpret_cast<const f2*>(nb + offz);
        const int2 ch = *reinterpret_cast<const int2*>(nb + 72);
        asm volatile("" : "+v"(r_xy), "+v"(r_z), "+v"(nf_x), "+v"(nf_y), "+v"(nf_z));
        const f2 tnx = fma2(ax[0], bc_lo(r_xy), bc_lo(nf_x)), tfx = fma2(ax[1], bc_lo(r_xy), bc_hi(nf_x));
        const f2 tny = fma2(ay[0], bc_hi(r_xy), bc_lo(nf_y)), tfy = fma2(ay[1], bc_hi(r_xy), bc_hi(nf_y));
        const f2 tnz = fma2(az[0], bc_lo(r_z), bc_lo(nf_z)), tfz = fma2(az[1], bc_lo(r_z), bc_hi(nf_z));
        tn0 = fmaxf(fmaxf(tnx.x, tny.x), tnz.x);
        tn1 = fmaxf(fmaxf(tnx.y, tny.y), tnz.y);
        const float tf0 = fminf(fminf(tfx.x, tfy.x), tfz.x);
        const float tf1 = fminf(fminf(tfx.y, tfy.y), tfz.y);
        float ntn0, ntn1;
        asm("v_max_f32 %0, %1, %2" : "=v"(ntn0) : "v"(tn0), "v"(tmin));
        asm("v_max_f32 %0, %1, %2" : "=v"(ntn1) : "v"(tn1), "v"(tmin));
        hit0 = ntn0 <= fminf(tf0, best_t);
        hit1 = ntn1 <= fminf(tf1, best_t);
        c0 = ch.x;
        c1 = ch.y;
      };
      for (int b = 0; b < a.n_big_leaves; ++b) leaf(a.big_pair0 + b * 2);
      int node = 0;
      unsigned short* top = stk0;
      bool go = true;
      while (go) {
        float tn0, tn1;
        bool hit0, hit1;
        int c0, c1;
        node_test(node, tn0, tn1, hit0, hit1, c0, c1);
        const bool l0 = hit0 && c0 < 0, l1 = hit1 && c1 < 0;
        if (l0 || l1) {
          leaf(l0 ? ~c0 : ~c1);
          if (l0 && l1) leaf(~c1);
        }
        const bool i0 = hit0 && !l0, i1 = hit1 && !l1;
        const bool sw = tn1 < tn0;
        int nxt = (i0 && (!i1 || !sw)) ? c0 : c1;
        *top = static_cast<unsigned short>(sw ? c0 : c1);
        top += (i0 && i1) ? 64 : 0;
        if (!(i0 || i1)) {
          go = top != stk0;
          top -= go ? 64 : 0;
          nxt = *top;
        }
        node = nxt;
      }
    }
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    if (best < 0) {
      const float sa = 0.5f * (uy + 1.0f);
      const float om = 1.0f - sa;
      cr = tr * fmaf(sa, 0.5f, om);
      cg = tg * fmaf(sa, 0.7f, om);
      cb = tb * fmaf(sa, 1.0f, om);
      done = true;
    } else if (rem == 0) {
      done = true;
    } else {
      const float4 sp = a.sph[best];
      const float hx = fmaf(ux, best_t, ox);
      const float hy = fmaf(uy, best_t, oy);
      const float hz = fmaf(uz, best_t, oz);
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
        float qx, qy, qz;
        random_unit<false>(st, qx, qy, qz);
        if (kind == RT_LAMBERTIAN) {
          float sx = qx + nx, sy = qy + ny, sz = qz + nz;
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
            done = true;
          }
        }
      } else if (kind == RT_NONE) {
        done = true;
      } else {
        const float ri = front ? m.x : m.w;
        const float r0 = front ? m.y : m.z;
        const float un = fmaf(uz, nz, fmaf(uy, ny, ux * nx));
        const float cosv = fminf(-un, 1.0f);
        const float sinv = sqrt_rn(fmaf(-cosv, cosv, 1.0f));
        bool refl = !(ri * sinv <= 1.0f);
        if (!refl && !a.realm) {
          const float xi = rng_uniform(st);
          const float x1 = 1.0f - cosv;
          const float x2 = x1 * x1;
          const float x5 = x2 * x2 * x1;
          refl = fmaf(1.0f - r0, x5, r0) > xi;
        }
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
    if (done) {
      unsigned long long* acc = &s_acc[q * 3];
      __hip_atomic_fetch_add(acc + 0, static_cast<unsigned long long>(fix24(cr)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(acc + 1, static_cast<unsigned long long>(fix24(cg)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(acc + 2, static_cast<unsigned long long>(fix24(cb)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      j = -2;
    }
  }

  // ---- per-pixel mean (compute-pixel's accum / spp, raytracing.clj:155) ----
  __syncthreads();
  const KArgsP ke = kargs_opaque();
  const int t = static_cast<int>(threadIdx.x);
  if (t < npx * 3) {
    const int fp = t / 3, ch = t - 3 * fp;
    const int qy = vw == 1 ? fp : static_cast<int>(__umulhi(static_cast<uint32_t>(fp), mag_vw));
    const int px = qx0 + (fp - qy * vw), ro = qy0 + qy;
    const size_t e = (static_cast<size_t>(ro) * ke->width + px) * 3 + ch;
    if (split) {
      if (s_acc[t]) __hip_atomic_fetch_add(&ke->part[e], s_acc[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const float tot = static_cast<float>(s_acc[t]) * 0x1p-24f;
      const float inv = static_cast<float>(ke->spp > 0 ? ke->spp : 1);
      ke->out[e] = ke->realm ? tot * (1.0f / inv) : tot / inv;
    }
  }
  if (ke->tile_cost && threadIdx.x == 0) {
    const uint64_t dt = __builtin_amdgcn_s_memrealtime() - st_t0;
    atomicAdd(&ke->tile_cost[tile], static_cast<unsigned>(dt < 0xffffffffull ? dt : 0xffffffffull));
  }
  if (ke->counters && threadIdx.x == 0 && pool) atomicAdd(&ke->counters[1], static_cast<unsigned long long>(pool));
  if (a.counters) {
    uint32_t v = segs;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && v) atomicAdd(&s_segs, static_cast<unsigned long long>(v));
    __syncthreads();
    if (threadIdx.x == 0 && s_segs) atomicAdd(&a.counters[0], s_segs);
  }
}

// The adaptive schedule's sort: tile indices by descending cost (a counting
// sort over 256 log-scale buckets: the top 5 bits are the cost's bit length,
// the low 3 the bits below its leading one).  One block; the order within a
// bucket is arbitrary (any order renders the same bits).  Each cost is then
// halved, so the next launch sorts by its own durations plus half of this
// history (a decayed mean: a tile's cost depends on what shared its CU;
// profiles/r02/shard_cost_decay.txt).
__device__ __forceinline__ int cost_bucket(unsigned c) {
  if (c < 8) return static_cast<int>(c);
  const int e = 31 - __clz(c);                                  // 3..31
  return ((e - 2) << 3) | static_cast<int>((c >> (e - 3)) & 7u); // monotone, < 256
}
__global__ __launch_bounds__(1024) void order_kernel(unsigned* __restrict__ cost, int* __restrict__ order,
                                                     int n) {
  __shared__ int hist[256];
  __shared__ int cursor[256];
  for (int i = threadIdx.x; i < 256; i += 1024) hist[i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 1024) atomicAdd(&hist[cost_bucket(cost[i])], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int b = 255; b >= 0; --b) {   // descending cost first
      cursor[b] = run;
      run += hist[b];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 1024) {
    const unsigned c = cost[i];
    order[atomicAdd(&cursor[cost_bucket(c)], 1)] = i;
    cost[i] = c >> 1;   // the next launch adds its durations to half of these
  }
}

// The split tiles' pixels (order positions [n_whole, n_tiles)): the sum of
// their splits' integer sums (added by the splits' atomics: exact, any
// order), then the unsplit epilogue's conversion: RN(float(sum)) * 2^-24,
// / spp (realm: * (1/spp)); the sums are zeroed for the next launch.  One
// block per split tile, thread t = tile row * 24 + x * 3 + channel.
__global__ __launch_bounds__(384) void finalize_kernel(unsigned long long* __restrict__ part,
                                                        const int* __restrict__ order, int n_whole,
                                                        int tiles_x, int tile_h, int width, int rows,
                                                        float* __restrict__ out, int spp, int realm) {
  const int pos = n_whole + static_cast<int>(blockIdx.x);
  const int tile = order ? order[pos] : pos;
  const int tby = tile / tiles_x, tbx = tile - tby * tiles_x;
  const int t = static_cast<int>(threadIdx.x);
  const int row = t / (kTile * 3), col = t - row * (kTile * 3);
  const int y = tby * tile_h + row, x3 = tbx * kTile * 3 + col;
  if (row >= tile_h || y >= rows || x3 >= width * 3) return;
  const size_t e = static_cast<size_t>(y) * width * 3 + x3;
  const unsigned long long sum = part[e];
  part[e] = 0ull;
  const float tot = static_cast<float>(sum) * 0x1p-24f;
  const float inv = static_cast<float>(spp > 0 ? spp : 1);
  out[e] = realm ? tot * (1.0f / inv) : tot / inv;
}

// rt_quantize on the device (rt_render_u8, rt_quantize_device): a channel's
// byte is the number of thresholds t[1..255] <= it (rt_internal.h), found by
// an 8-step binary search in LDS -- NaN fails every compare and gets 0, as
// rt_quantize's isnan does.  Streaming: 4 bytes read, 1 written per channel.
struct QThr {
  float t[256];
};
__global__ __launch_bounds__(256) void quantize_kernel(const float* __restrict__ lin, uint8_t* __restrict__ out,
                                                        size_t n, const QThr q) {
  __shared__ float s_t[256];
  s_t[threadIdx.x] = q.t[threadIdx.x];
  __syncthreads();
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
    const float c = lin[i];
    int b = 0;
#pragma unroll
    for (int step = 128; step > 0; step >>= 1)
      if (s_t[b + step] <= c) b += step;   // b + step <= 255
    out[i] = static_cast<uint8_t>(b);
  }
}

// Cost-balanced splits: the next split launch of the shape deals its U units
// to the tiles in proportion to their recorded cost (the decayed record
// order_kernel has just sorted and halved), so that units cost about the
// same and the launch does not end on a few long ones (a uniform split of
// C1's 8-GPU shard left units of 330-360 us against a 259 us mean in the
// launch's tail: DESIGN.md §6).  Tile at order position p gets
// s_p = min(smax, 1 + floor(cost_p (U - n) / C)) units, the U - sum s units
// left go one each to the first positions, and unit u of the plan is
// {tile, k | s << 8}: samples [k spp / s, (k + 1) spp / s).  Units the clamps
// leave over are {-1, 0}.  One block.
__global__ __launch_bounds__(1024) void plan_kernel(const unsigned* __restrict__ cost, const int* __restrict__ order,
                                                     int n, int U, int smax, int2* __restrict__ units) {
  __shared__ unsigned long long s_tot;
  __shared__ int s_part[1024];
  __shared__ int s_left;
  const int tid = static_cast<int>(threadIdx.x);
  const int per = (n + 1023) / 1024;
  const int p0 = min(n, tid * per), p1 = min(n, p0 + per);
  if (tid == 0) s_tot = 0ull;
  __syncthreads();
  unsigned long long my = 0;
  for (int p = p0; p < p1; ++p) my += cost[order[p]];
  if (my) atomicAdd(&s_tot, my);
  __syncthreads();
  const unsigned long long tot = s_tot;
  const int spare = max(0, U - n);
  auto raw = [&](int p) {
    const long long c = static_cast<long long>(cost[order[p]]);
    const long long extra = tot ? (c * spare) / static_cast<long long>(tot) : spare / max(n, 1);
    return static_cast<int>(min<long long>(smax, 1 + extra));
  };
  int sum = 0;
  for (int p = p0; p < p1; ++p) sum += raw(p);
  s_part[tid] = sum;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    for (int i = 0; i < 1024; ++i) t += s_part[i];
    s_left = max(0, U - t);
  }
  __syncthreads();
  const int left = s_left;
  auto fin = [&](int p) {
    const int r = raw(p);
    return r + ((p < left && r < smax) ? 1 : 0);
  };
  sum = 0;
  for (int p = p0; p < p1; ++p) sum += fin(p);
  __syncthreads();
  s_part[tid] = sum;
  __syncthreads();
  if (tid == 0) {   // exclusive prefix of the threads' unit counts (1024 adds)
    int run = 0;
    for (int i = 0; i < 1024; ++i) {
      const int v = s_part[i];
      s_part[i] = run;
      run += v;
    }
    s_left = run;   // units used
  }
  __syncthreads();
  int base = s_part[tid];
  for (int p = p0; p < p1; ++p) {
    const int sp = fin(p);
    const int tile = order[p];
    for (int k = 0; k < sp; ++k) units[base + k] = make_int2(tile, k | (sp << 8));
    base += sp;
  }
  for (int u = s_left + tid; u < U; u += 1024) units[u] = make_int2(-1, 0);
}

// ------------------------------------------------------------- host ------
// Kernel variants (rt_set_variant).  The product library carries the default
// traversal and its fallbacks:
//   16 BVH in LDS, 4-body leaves (two pairs)      18 BVH in LDS, 8-body leaves
//   12 BVH (2-body leaves) read from global memory: a tree too big for LDS
//    5 linear scan, grouped, table through the scalar cache: a tree too deep
//    0 = default (22 where it applies, else 16; 18 when the 4-body tree's LDS image is large)
// The diagnostic build (-DRTCLJ_DIAG, lib/librtclj_diag.so) adds the A/B and
// statistics variants:
//    1 LDS table, simple scan         2 scalar-cache table, simple scan
//    3 = 1 + stats                    4 LDS table, grouped scan (north_star's LDS-staged scan)
//    6 = 4 + stats                    7 = 5 + stats
//    8 LDS table, packed pairs        9 scalar, packed pairs   10 = 9 + stats
//   11 BVH in LDS, 2-body leaves     13 = 11 + stats
//   14 11 with a speculative while-while traversal           15 = 14 + stats
//   17 = 16 + stats                  19 = 18 + stats
//   20 / 21 direction-coherent waves (sorted_kernel)
// Both builds: 22 = 16 in a compact LDS image, seven workgroups per CU
// (the default where spp <= 255, albedos lie in [-1, 1] and the tree has
// <= 256 nodes; 16 elsewhere).
// Every variant renders the same bits.
struct Variant {
  const void* fn;
  bool lds;
  bool stats;
  int scan;   // SCAN_* (the tile shape: tile_rows)
  int threads = 256;   // workgroup size
};
constexpr int kVariants = 23;
// the tree a traversal variant walks: 0 = 2-body leaves, 1 = 4, 2 = 8
static int variant_tree(int v) { return v >= 20 ? 1 : v >= 18 ? 2 : v >= 16 ? 1 : 0; }
#define RT_K(SRC, SCAN, ST) reinterpret_cast<const void*>(&trace_kernel<SRC, SCAN, ST>)
static const Variant& variant_table(int v) {
  static const Variant none{nullptr, false, false, 0};
  static const Variant t[kVariants] = {
      {RT_K(SRC_LDS, SCAN_BVHQ, false), true, false, SCAN_BVHQ},          // 0: placeholder (resolved per scene)
#ifdef RTCLJ_DIAG
      {RT_K(SRC_LDS, SCAN_SIMPLE, false), true, false, SCAN_SIMPLE},        // 1
      {RT_K(SRC_SCALAR, SCAN_SIMPLE, false), false, false, SCAN_SIMPLE},    // 2
      {RT_K(SRC_LDS, SCAN_SIMPLE, true), true, true, SCAN_SIMPLE},          // 3
      {RT_K(SRC_LDS, SCAN_GROUP4, false), true, false, SCAN_GROUP4},        // 4
#else
      none, none, none, none,
#endif
      {RT_K(SRC_SCALAR, SCAN_GROUP4, false), false, false, SCAN_GROUP4},    // 5
#ifdef RTCLJ_DIAG
      {RT_K(SRC_LDS, SCAN_GROUP4, true), true, true, SCAN_GROUP4},          // 6
      {RT_K(SRC_SCALAR, SCAN_GROUP4, true), false, true, SCAN_GROUP4},      // 7
      {RT_K(SRC_LDS, SCAN_PK4, false), true, false, SCAN_PK4},           // 8
      {RT_K(SRC_SCALAR, SCAN_PK4, false), false, false, SCAN_PK4},       // 9
      {RT_K(SRC_SCALAR, SCAN_PK4, true), false, true, SCAN_PK4},         // 10
      {RT_K(SRC_LDS, SCAN_BVH, false), true, false, SCAN_BVH},           // 11
#else
      none, none, none, none, none, none,
#endif
      {RT_K(SRC_SCALAR, SCAN_BVH, false), false, false, SCAN_BVH},       // 12
#ifdef RTCLJ_DIAG
      {RT_K(SRC_LDS, SCAN_BVH, true), true, true, SCAN_BVH},             // 13
      {RT_K(SRC_LDS, SCAN_BVHWW, false), true, false, SCAN_BVHWW},         // 14
      {RT_K(SRC_LDS, SCAN_BVHWW, true), true, true, SCAN_BVHWW},           // 15
#else
      none, none, none,
#endif
      {RT_K(SRC_LDS, SCAN_BVHQ, false), true, false, SCAN_BVHQ},          // 16
#ifdef RTCLJ_DIAG
      {RT_K(SRC_LDS, SCAN_BVHQ, true), true, true, SCAN_BVHQ},            // 17
#else
      none,
#endif
      {RT_K(SRC_LDS, SCAN_BVHO, false), true, false, SCAN_BVHO},          // 18
#ifdef RTCLJ_DIAG
      {RT_K(SRC_LDS, SCAN_BVHO, true), true, true, SCAN_BVHO},            // 19
#else
      none,
#endif
#ifdef RTCLJ_DIAG
      // direction-coherent waves (A/B, measured slower: profiles/r04/sorted_waves/):
      // octant-sorted, and lock-step packing only
      {reinterpret_cast<const void*>(&sorted_kernel<true>), true, false, SCAN_BVHS, kSortThreads},    // 20
      {reinterpret_cast<const void*>(&sorted_kernel<false>), true, false, SCAN_BVHS, kSortThreads},   // 21
#else
      none, none,
#endif
      // 16's walk in a compact LDS image, seven workgroups per CU (the
      // default where compact_ok holds; rt_launch falls back to 16 elsewhere)
      {RT_K(SRC_LDS, SCAN_BVHQ7, false), true, false, SCAN_BVHQ7},        // 22
  };
  return (v >= 0 && v < kVariants) ? t[v] : none;
}
#undef RT_K
// selectors (rt_set_variant / rt_set_schedule): atomics, read once per launch
static std::atomic<int> g_variant{0};
// tile schedule: 0 = adaptive longest-first, 1 = dispatch order
static std::atomic<int> g_schedule{0};
// BVH build: surface-area splits (default) or median splits (RTCLJ_BVH=median, for A/B)
static const bool g_bvh_sah = [] {
  const char* e = std::getenv("RTCLJ_BVH");
  return !(e && std::strcmp(e, "median") == 0);
}();
#ifdef RTCLJ_DIAG
// diagnostic build: RTCLJ_TIMELINE=1 records every launch's wave timeline
static const bool g_timeline = [] {
  const char* e = std::getenv("RTCLJ_TIMELINE");
  return e && std::atoi(e) != 0;
}();
#endif
// stats builds: per device, u64[kDbg] event counters and the u64[4 * kDbgWaves]
// wave timeline, allocated on that device at its first stats launch
constexpr int kDbg = 32;
constexpr int kDbgDevices = 64;
static std::mutex g_dbg_mu;
static unsigned long long* g_dbg[kDbgDevices] = {};
static unsigned long long* g_dbgw[kDbgDevices] = {};

}  // namespace rtclj

using namespace rtclj;

// one BVH on the device: blob = nodes | pairs | pidx (the big bodies' leaves after the tree's)
struct DTree {
  float4* blob;
  int blob_f4, off_pairs, off_pidx, big_pair0, n_big_leaves, depth, n_nodes;
  float c[3], r;
};

// Adaptive tile schedule (rt_launch): per stream, the per-tile durations of
// the stream's last launch and the longest-first order derived from them, for
// the launch shape `key` (frame rows, tiling, grid).  The order is a
// prediction: camera, spp, seed, flags and the kernel variant may change
// between launches of one shape (progressive passes, animation, A/B) and it
// stays a good one, and it never affects the result.  A launch of another
// shape re-keys the entry (and runs in dispatch order once).  Entries are per
// stream so that nothing a stream's kernels read is written from another
// stream; a dscene serves up to kSchedStreams streams this way, launches on
// further streams run unscheduled.
// The same per-stream entry holds the split tiles' partial sums (rt_launch).
struct ScheduleKey {
  int width, rows, row_begin, row_tile, tile_first, tile_step, gx, gy;
};
struct Schedule {
  hipStream_t stream = nullptr;
  unsigned* cost = nullptr;
  int* order = nullptr;
  int cap = 0;          // tiles the buffers hold
  bool ready = false;   // order[] holds a permutation of key's tiles (stream-ordered)
  ScheduleKey key{};
  unsigned long long* part = nullptr;   // [rows][width][3] pixel sums of split tiles (zero between launches)
  size_t part_cap = 0;                  // u64 elements
  // a split launch's trace kernel was enqueued but its finalize_kernel (which
  // re-zeroes the sums) was not: the next split launch zeroes them first
  bool part_dirty = false;
  // the stealing state (KArgs word, done, sum, owner, stealc)
  unsigned long long* word = nullptr;   // per tile
  unsigned* done = nullptr;             // per tile
  unsigned long long* sum = nullptr;    // per tile x kPoolPx x 3, zero between uses
  int steal_cap = 0;                    // tiles those hold
  int* owner = nullptr;                 // KArgs n_owner entries
  int owner_cap = 0;
  unsigned long long* stealc = nullptr; // [helpers that got samples, their first samples] since rt_steal_stats
  unsigned epoch = 0;                   // launches with sharing on this stream (mod 2^16, 1 .. 65535)
  bool epoch_started = false;
  int2* units = nullptr;                // cost-balanced split plan (plan_kernel) of the next split launch
  int units_cap = 0;
  int plan_units = -1;                  // the plan's unit count (-1: none)
};
constexpr int kSchedStreams = 8;
struct ScheduleSet {
  std::mutex mu;
  int used = 0;
  Schedule s[kSchedStreams];
  static void free_entry(Schedule& e) {
    if (e.cost) (void)hipFree(e.cost);
    if (e.order) (void)hipFree(e.order);
    if (e.part) (void)hipFree(e.part);
    if (e.word) (void)hipFree(e.word);
    if (e.done) (void)hipFree(e.done);
    if (e.sum) (void)hipFree(e.sum);
    if (e.owner) (void)hipFree(e.owner);
    if (e.stealc) (void)hipFree(e.stealc);
    if (e.units) (void)hipFree(e.units);
    e = Schedule{};
  }
  void release() {
    for (int k = 0; k < used; ++k) free_entry(s[k]);
    used = 0;
  }
  // drop `stream`'s entry (its kernels have finished), keeping the others packed
  void release_stream(hipStream_t stream) {
    for (int k = 0; k < used; ++k)
      if (s[k].stream == stream) {
        free_entry(s[k]);
        if (k != used - 1) {
          s[k] = s[used - 1];
          s[used - 1] = Schedule{};
        }
        --used;
        return;
      }
  }
};

struct rt_dscene {
  int device;
  int n;
  int n_pad;
  float4* geo;
  float4* geo2;   // n_pad/2 Pairs (= n_pad float4)
  // BVHs (bvh.cpp): tree[0] 2-body leaves, tree[1] 4-body, tree[2] 8-body
  DTree tree[3];
  float4* sph;
  float4* mat;
  int* kind;
  bool unit_albedo;            // every lambertian/metal albedo channel within [-1, 1] (compact_ok)
  uint64_t uid;                // upload id (scene_uid): contexts name scenes by it, not by address
  mutable ScheduleSet sched;   // rt_launch's adaptive tile order
};
static std::atomic<uint64_t> g_scene_uid{0};
uint64_t rtclj::scene_uid(const rt_dscene* ds) { return ds ? ds->uid : 0; }

// live device scenes, for release_stream_schedules (rt_host.cpp's contexts)
static std::mutex g_scenes_mu;
static std::vector<rt_dscene*> g_scenes;

// the live scenes among `uids` (a context's list may name freed ones; a
// new scene at a freed one's address has another id)
template <class F>
static void for_live_scenes(const uint64_t* uids, int n, F f) {
  std::lock_guard<std::mutex> lk(g_scenes_mu);
  for (rt_dscene* d : g_scenes)
    if (std::find(uids, uids + n, d->uid) != uids + n) {
      std::lock_guard<std::mutex> l2(d->sched.mu);
      f(d->sched);
    }
}

void rtclj::release_stream_schedules(void* stream, const uint64_t* uids, int n) {
  for_live_scenes(uids, n, [&](ScheduleSet& set) { set.release_stream(static_cast<hipStream_t>(stream)); });
}

void rtclj::rebind_stream_schedules(void* from, void* to, const uint64_t* uids, int n) {
  for_live_scenes(uids, n, [&](ScheduleSet& set) {
    Schedule* src = nullptr;
    for (int k = 0; k < set.used; ++k) {
      if (set.s[k].stream == static_cast<hipStream_t>(to)) return;
      if (set.s[k].stream == static_cast<hipStream_t>(from)) src = &set.s[k];
    }
    if (src) src->stream = static_cast<hipStream_t>(to);
  });
}

static int hip_fail(hipError_t e, const char* what) {
  return set_error(RT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(call)                                  \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return hip_fail(_e, #call);  \
  } while (0)

extern "C" int rt_set_variant(int v) {
  clear_error();
  if (v != 0 && !variant_table(v).fn)
    return set_error(RT_E_ARG, "rt_set_variant: variant " + std::to_string(v) +
                                   " is not in this build (diagnostic variants: lib/librtclj_diag.so)");
  return g_variant.exchange(v);
}

extern "C" int rt_set_schedule(int mode) {
  clear_error();
  if (mode != 0 && mode != 1) return set_error(RT_E_ARG, "rt_set_schedule: mode must be 0 or 1");
  return g_schedule.exchange(mode);
}

extern "C" int rt_scene_upload(int device, const rt_scene* s, rt_dscene** out) {
  clear_error();
  if (!s || !out) return set_error(RT_E_ARG, "rt_scene_upload: NULL argument");
  *out = nullptr;
  if (s->n < 0 || (s->n > 0 && (!s->sphere || !s->mat_kind || !s->mat)))
    return set_error(RT_E_ARG, "rt_scene_upload: bad scene arrays");
  if (s->n > RT_MAX_SPHERES)
    return set_error(RT_E_TOO_MANY, "rt_scene_upload: " + std::to_string(s->n) +
                                        " spheres > RT_MAX_SPHERES (" +
                                        std::to_string(RT_MAX_SPHERES) + ")");
  for (int i = 0; i < s->n; ++i) {
    const int k = s->mat_kind[i];
    if (k != RT_LAMBERTIAN && k != RT_METAL && k != RT_DIELECTRIC && k != RT_NONE)
      return set_error(RT_E_MATERIAL, "rt_scene_upload: body " + std::to_string(i) +
                                          " has unsupported material kind " + std::to_string(k));
  }
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return set_error(RT_E_NODEV, "rt_scene_upload: device " + std::to_string(device) +
                                     " not available (" + std::to_string(ndev) + " visible)");
  HIP_TRY(hipSetDevice(device));
  const int n = s->n;
  const int n_pad = ((n + 3) / 4) * 4 + 4;   // grouped scan reads up to 4 past the last group
  const size_t cnt = n > 0 ? n : 1;
  // pads: -r^2 = +inf -> c = +inf, disc = -inf: never a candidate
  std::vector<float4> geo(n_pad, make_float4(0.0f, 0.0f, 0.0f, INFINITY)), sph(cnt), mat(cnt);
  std::vector<int> kind(cnt, 0);
  for (int i = 0; i < n; ++i) {
    const float* q = s->sphere + 4 * i;
    const float r = q[3];
    geo[i] = make_float4(q[0], q[1], q[2], -(r * r));
    sph[i] = make_float4(q[0], q[1], q[2], 1.0f / r);                   // 1/r for the normal
    const float* m = s->mat + 4 * i;
    mat[i] = make_float4(m[0], m[1], m[2], m[3]);
    if (s->mat_kind[i] == RT_DIELECTRIC) {   // (albedo unused)
      mat[i].x = 1.0f / m[3];                // ri of a front face: 1/eta
      // Schlick's r0 = ((1 - ri) / (1 + ri))^2 for ri = 1/eta (front face) and
      // eta (back face): the kernel's fp32 ops, done once here (IEEE division,
      // no contraction: the same bits)
      for (int f = 0; f < 2; ++f) {
        const float ri = f == 0 ? mat[i].x : m[3];
        float r0 = (1.0f - ri) / (1.0f + ri);
        r0 = r0 * r0;
        (f == 0 ? mat[i].y : mat[i].z) = r0;
      }
    }
    kind[i] = s->mat_kind[i];
  }
  // pair-interleaved copy for the packed scan: (x0 x1 y0 y1 z0 z1 w0 w1) per pair
  std::vector<float> geo2(4 * static_cast<size_t>(n_pad));
  for (int q = 0; q < n_pad / 2; ++q) {
    const float4 b0 = geo[2 * q], b1 = geo[2 * q + 1];
    float* o = &geo2[8 * static_cast<size_t>(q)];
    o[0] = b0.x; o[1] = b1.x; o[2] = b0.y; o[3] = b1.y;
    o[4] = b0.z; o[5] = b1.z; o[6] = b0.w; o[7] = b1.w;
  }
  rt_dscene* d = new rt_dscene{};
  d->uid = ++g_scene_uid;
  d->device = device;
  d->n = n;
  d->n_pad = n_pad;
  d->unit_albedo = true;
  for (int i = 0; i < n; ++i)
    if (s->mat_kind[i] == RT_LAMBERTIAN || s->mat_kind[i] == RT_METAL)
      for (int c = 0; c < 3; ++c)
        if (!(std::fabs(s->mat[4 * i + c]) <= 1.0f)) d->unit_albedo = false;
  // BVHs over the bodies (the traversal variants), the three trees built
  // concurrently on host threads (C1: 2.4 -> ~1 ms of a first rt_render)
  BvhHost bvhs[3];
  {
    std::thread th[2];
    for (int k = 1; k < 3; ++k) th[k - 1] = std::thread([&, k] { bvh_build(s->sphere, n, &bvhs[k], 2 << k, g_bvh_sah); });
    bvh_build(s->sphere, n, &bvhs[0], 2, g_bvh_sah);
    for (std::thread& t : th) t.join();
  }
  hipError_t e = hipMalloc(&d->geo, n_pad * sizeof(float4));
  // blob = nodes | pairs | pidx
  for (int k = 0; k < 3 && e == hipSuccess; ++k) {
    BvhHost& bvh = bvhs[k];
    const size_t nb = bvh.nodes.size() * sizeof(BvhNode);
    const size_t pb = bvh.pairs.size() * sizeof(float);
    // body indices: u16 for the 8-body-leaf tree (RT_MAX_SPHERES < 65535; a
    // pad's -1 -> 0xffff, never a candidate), int for the others
    const size_t isz = k == 2 ? sizeof(uint16_t) : sizeof(int);
    std::vector<uint16_t> pidx16(bvh.pidx.size());
    for (size_t i = 0; i < pidx16.size(); ++i) pidx16[i] = static_cast<uint16_t>(bvh.pidx[i]);
    const size_t ib = ((bvh.pidx.size() * isz + 15) / 16) * 16;
    std::vector<char> blob(nb + pb + ib, 0);
    if (k == 1)   // 4-body tree: inner-child refs as byte offsets (< 65536 while it fits LDS: u16 stack)
      for (BvhNode& nd : bvh.nodes)
        for (int& c : nd.child)
          if (c >= 0) c *= static_cast<int>(sizeof(BvhNode));
    std::memcpy(blob.data(), bvh.nodes.data(), nb);
    std::memcpy(blob.data() + nb, bvh.pairs.data(), pb);
    if (k == 2) std::memcpy(blob.data() + nb + pb, pidx16.data(), pidx16.size() * sizeof(uint16_t));
    else std::memcpy(blob.data() + nb + pb, bvh.pidx.data(), bvh.pidx.size() * sizeof(int));
    DTree& t = d->tree[k];
    t.blob_f4 = static_cast<int>(blob.size() / 16);
    t.off_pairs = static_cast<int>(nb);
    t.off_pidx = static_cast<int>(nb + pb);
    t.big_pair0 = bvh.big_pair0;
    t.n_big_leaves = bvh.n_big_leaves;
    t.depth = bvh.depth;
    t.n_nodes = static_cast<int>(bvh.nodes.size());
    for (int j = 0; j < 3; ++j) t.c[j] = bvh.center[j];
    t.r = bvh.radius;
    e = hipMalloc(&t.blob, blob.size());
    if (e == hipSuccess) e = hipMemcpy(t.blob, blob.data(), blob.size(), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMalloc(&d->geo2, n_pad * sizeof(float4));
  if (e == hipSuccess) e = hipMemcpy(d->geo2, geo2.data(), n_pad * sizeof(float4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&d->sph, cnt * sizeof(float4));
  if (e == hipSuccess) e = hipMalloc(&d->mat, cnt * sizeof(float4));
  if (e == hipSuccess) e = hipMalloc(&d->kind, cnt * sizeof(int));
  if (e == hipSuccess) e = hipMemcpy(d->geo, geo.data(), n_pad * sizeof(float4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d->sph, sph.data(), cnt * sizeof(float4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d->mat, mat.data(), cnt * sizeof(float4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d->kind, kind.data(), cnt * sizeof(int), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    rt_scene_free(d);
    return hip_fail(e, "rt_scene_upload");
  }
  {
    std::lock_guard<std::mutex> lk(g_scenes_mu);
    g_scenes.push_back(d);
  }
  *out = d;
  return RT_OK;
}

extern "C" int rt_scene_free(rt_dscene* d) {
  if (!d) return RT_OK;
  {
    std::lock_guard<std::mutex> lk(g_scenes_mu);
    g_scenes.erase(std::remove(g_scenes.begin(), g_scenes.end(), d), g_scenes.end());
  }
  (void)hipSetDevice(d->device);
  if (d->geo) (void)hipFree(d->geo);
  if (d->geo2) (void)hipFree(d->geo2);
  for (const DTree& t : d->tree) {
    if (t.blob) (void)hipFree(t.blob);
  }
  d->sched.release();
  if (d->sph) (void)hipFree(d->sph);
  if (d->mat) (void)hipFree(d->mat);
  if (d->kind) (void)hipFree(d->kind);
  delete d;
  return RT_OK;
}

// traversal stack bytes: u8 entries for the 8-body-leaf tree (tree[2], at
// most 256 nodes when its variant runs), u16 otherwise
static int stack_entries(const DTree& t, int tree) { return tree == 0 ? t.depth + 2 : std::max(t.depth, 1); }
static size_t stack_of(const DTree& t, int tree) {
  return static_cast<size_t>(stack_entries(t, tree)) * 256 * (tree == 2 ? 1 : 2);
}
static size_t lds_of(const DTree& t, int tree) { return static_cast<size_t>(t.blob_f4) * 16 + stack_of(t, tree); }
// variant 22 (the compact image): u8 node indices, depth rows (the dead
// far-child write goes one above the top, as in 16)
static int stack_entries_compact(const DTree& t) { return std::max(t.depth, 1); }
static size_t lds_of_compact(const DTree& t) {
  return static_cast<size_t>(t.blob_f4) * 16 + static_cast<size_t>(stack_entries_compact(t)) * 256;
}
// LDS a CU can give each of 5 workgroups (160 KB / 5), less the 4-body-leaf
// kernel's static LDS (pool counter, the 64 pixels' colour sums and pixel
// table).  (Its registers allow 6; C1's 24.0 KB image fits 6 as well.)
constexpr size_t kStaticLds = 4 + kPoolPx * 3 * 8 + kPoolPx * 16 + 12;   // (the 8-body traversal's 8x4 tile, no table: 1.8 KB less)
constexpr size_t kLds5 = 160 * 1024 / 5 - kStaticLds;

// selector -> the variant a launch on ds runs
static int resolve_variant(const rt_dscene& ds, int vsel) {
  // default: 4-body leaves, unless that tree's LDS image limits a CU below
  // 5 workgroups (160 KB / 5) and the 8-body-leaf tree's is smaller
  // (measured: 1025 bodies 12.9 vs 14.0 ms; 484: 10.8 vs 12.2)
  if (vsel == 0)
    vsel = (lds_of(ds.tree[1], 1) > kLds5 && ds.tree[2].n_nodes <= 256 &&
            lds_of(ds.tree[2], 2) < lds_of(ds.tree[1], 1)) ? 18 : 16;
  if ((vsel == 18 || vsel == 19) && ds.tree[2].n_nodes > 256) vsel -= 2;   // u8 stack: 256 nodes at most
  // u16 stack of node LDS addresses: the kernel's static LDS (< 4 KB; 8 KB
  // allowed for) plus the node region must stay below 64 KB
  if ((vsel == 16 || vsel == 17) && ds.tree[1].n_nodes * 80 + 8192 > 65535) vsel = 12;
  // the sorted kernels: the 4-body tree's byte-offset refs in a u16 stack
  // inside a wave's exchange slots, the blob beside the exchange buffer
  if ((vsel == 20 || vsel == 21) &&
      (ds.tree[1].n_nodes * 80 > 65535 || ds.tree[1].depth + 2 > kBvhStack ||
       static_cast<size_t>(ds.tree[1].blob_f4) * 16 + kXBytes > 96 * 1024))
    vsel = 16;
  if (vsel >= 11) {
    const DTree& t = ds.tree[variant_tree(vsel)];
    if (t.depth + 2 > kBvhStack) return 5;                       // tree too deep for the stack
    if (vsel != 12 && lds_of(t, variant_tree(vsel)) > 96 * 1024) vsel = 12;          // tree too big for LDS: 2-body leaves, global
    if (vsel == 12 && ds.tree[0].depth + 2 > kBvhStack) return 5;
  }
  if (vsel == 22 && ds.tree[1].n_nodes > 256) vsel = 16;   // (u8 node indices)
  return vsel;
}

// The compact variant (22) for a launch: the 4-body tree's node indices fit
// a byte, and a pixel's u32 sum cannot overflow -- every sample's colour is
// at most 1 per channel (albedos within [-1, 1]: the sky and the dielectric
// give at most 1) and a pixel gets at most spp <= 255 samples, 255 * 2^24 <
// 2^32.  The default selector runs it wherever it applies (and an explicit
// 22 too); elsewhere the launch runs 16.  Seven workgroups per CU instead of
// six, in 72 VGPRs without a spill: C1 5.90 -> 5.83 ms (profiles/r04/w7/,
// DESIGN.md §8.1).
// Its pixel table packs a pixel's image coordinates as x | y << 16: frames
// up to 65536 pixels wide and high (wider or taller ones run 16).
static bool compact_ok(const rt_dscene& ds, const rt_params& p) {
  return ds.unit_albedo && ds.tree[1].n_nodes <= 256 && p.spp <= 255 && ds.tree[1].depth + 2 <= kBvhStack &&
         p.width <= 65536 && p.height <= 65536;
}
static int launch_variant(const rt_dscene& ds, const rt_params& p) {
  const int sel = g_variant.load();
  int vsel = resolve_variant(ds, sel);
  if ((sel == 0 && vsel == 16) || vsel == 22) vsel = compact_ok(ds, p) ? 22 : 16;
  return vsel;
}

extern "C" int rt_resolve_variant(const rt_dscene* ds) { return ds ? resolve_variant(*ds, g_variant.load()) : -1; }

// dynamic LDS of a launch of variant vsel on ds
static size_t launch_lds(const rt_dscene& ds, int vsel) {
  const Variant& v = variant_table(vsel);
  if (v.scan == SCAN_BVHS) return static_cast<size_t>(ds.tree[1].blob_f4) * 16 + kXBytes;   // blob | exchange
  if (vsel == 22) return lds_of_compact(ds.tree[1]);
  if (vsel >= 11) {
    const DTree& tr = ds.tree[variant_tree(vsel)];
    return v.lds ? lds_of(tr, variant_tree(vsel)) : stack_of(tr, variant_tree(vsel));
  }
  return v.lds ? static_cast<size_t>(ds.n_pad) * sizeof(float4) : 0;
}

// Occupancy of the launch rt_launch would make for (ds, p): the HIP occupancy
// query on the kernel and dynamic LDS it would use (diagnostic, bench.py).
extern "C" int rt_launch_occupancy(const rt_dscene* ds, const rt_params* p, int* out4) {
  clear_error();
  if (!ds || !p || !out4) return set_error(RT_E_ARG, "rt_launch_occupancy: NULL argument");
  const int rows = rows_out(*p);
  if (rows <= 0 || p->width <= 0) return set_error(RT_E_ARG, "rt_launch_occupancy: empty frame");
  HIP_TRY(hipSetDevice(ds->device));
  const int vsel = launch_variant(*ds, *p);
  const void* fn = variant_table(vsel).fn;
  if (!fn) return set_error(RT_E_ARG, "rt_launch_occupancy: no kernel for variant " + std::to_string(vsel));
  const size_t lds = launch_lds(*ds, vsel);
  if (lds > 64 * 1024)
    HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  int blocks = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, variant_table(vsel).threads, lds));
  hipFuncAttributes fa{};
  HIP_TRY(hipFuncGetAttributes(&fa, fn));
  out4[0] = blocks * variant_table(vsel).threads / 256;   // (in 256-thread workgroups) per CU
  out4[1] = fa.numRegs;           // VGPRs per lane
  out4[2] = static_cast<int>(lds + fa.sharedSizeBytes);   // LDS bytes per workgroup
  out4[3] = vsel;
  return RT_OK;
}

static int dbg_buffers(int device, unsigned long long** dbg, unsigned long long** dbgw) {
  if (device < 0 || device >= kDbgDevices) return set_error(RT_E_ARG, "stats launch: device index too large");
  std::lock_guard<std::mutex> lk(g_dbg_mu);
  if (!g_dbg[device]) {
    HIP_TRY(hipMalloc(&g_dbg[device], kDbg * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(g_dbg[device], 0, kDbg * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc(&g_dbgw[device], 4 * kDbgWaves * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(g_dbgw[device], 0, 4 * kDbgWaves * sizeof(unsigned long long)));
  }
  *dbg = g_dbg[device];
  *dbgw = g_dbgw[device];
  return RT_OK;
}

// ceil(2^64 / d), 0 for d <= 1: n / d = the high half of n * m for every
// 32-bit n (m * d = 2^64 + e with e < d, so n * e < 2^64 never reaches the
// quotient)
static uint64_t magic64(int d) { return d <= 1 ? 0 : ~0ull / static_cast<uint64_t>(d) + 1ull; }

// Sample split (rt_launch): split every tile of a launch with fewer tiles
// than kSplitRounds (RTCLJ_SPLIT_ROUNDS, default 3) x (resident workgroups), into enough splits to reach that
// (at most kSplitMax).  tools/shard_time.py on C1's 1/2/4/8-GPU shards
// (profiles/r02/shard_split_rounds.txt): 3-4 rounds best (8 GPUs: 5.88x at 3,
// 5.72x at 4, 5.30x at 6, 3.96x at 16; unsplit 2.57x)
constexpr int kSplitMax = 64;

// Tile sharing, A/B knobs read at every launch:
// RTCLJ_STEAL=0 (off: the static sample split for launches of few tiles, as
// before), RTCLJ_THIEVES (helper workgroups per workgroup slot of the
// device), RTCLJ_STEAL_MIN (unclaimed samples a tile needs for a helper to join)
static int env_int(const char* name, int dflt, int lo) {
  const char* e = std::getenv(name);
  return e ? std::max(lo, std::atoi(e)) : dflt;
}
static int split_rounds() { return env_int("RTCLJ_SPLIT_ROUNDS", 3, 1); }   // (kSplitRounds above)

// workgroups device `device` holds at once for kernel fn with `lds` bytes of
// dynamic LDS (CUs x the occupancy query), cached per (device, fn, lds)
static int launch_slots(int device, const void* fn, size_t lds, int threads = 256) {
  struct Entry { int device; const void* fn; size_t lds; int slots; };
  static std::mutex mu;
  static std::vector<Entry> cache;
  std::lock_guard<std::mutex> lk(mu);
  for (const Entry& e : cache)
    if (e.device == device && e.fn == fn && e.lds == lds) return e.slots;
  int cus = 0, per = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, lds) != hipSuccess)
    return 0;
  cache.push_back({device, fn, lds, cus * per});
  return cus * per;
}

namespace rtclj {
int quantize_launch(const float* d_lin, uint8_t* d_out, size_t n, void* stream) {
  static const QThr thr = [] {
    QThr t;
    std::memcpy(t.t, quantize_thresholds(), sizeof t.t);
    return t;
  }();
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 4096);
  QThr q = thr;
  const float* in = d_lin;
  uint8_t* out = d_out;
  void* args[] = {&in, &out, &n, &q};
  return hipLaunchKernel(reinterpret_cast<const void*>(&quantize_kernel), dim3(static_cast<unsigned>(blocks)),
                         dim3(256), args, 0, static_cast<hipStream_t>(stream));
}
}  // namespace rtclj

extern "C" int rt_launch(const rt_dscene* ds, const rt_camera* c, const rt_params* p, float* d_out,
                         uint64_t* d_counters, void* hip_stream) {
  clear_error();
  if (!ds || !c || !p || !d_out) return set_error(RT_E_ARG, "rt_launch: NULL argument");
  if (p->width <= 0 || p->height <= 0 || p->spp < 0 || p->spp > RT_MAX_SPP ||
      (p->flags & ~(RT_FLAG_REALM | RT_FLAG_STREAMED)) != 0)
    return set_error(RT_E_ARG, "rt_launch: bad width/height/spp/flags");
  const int rows = rows_out(*p);
  if (rows < 0) return set_error(RT_E_ARG, "rt_launch: bad row selection");
  KArgs a{};
  a.geo = ds->geo;
  a.geo2 = reinterpret_cast<const Pair*>(ds->geo2);
  a.sph = ds->sph;
  a.mat = ds->mat;
  a.kind = ds->kind;
  a.out = d_out;
  a.counters = reinterpret_cast<unsigned long long*>(d_counters);
  std::memcpy(a.cam + 0, c->center, 12);
  std::memcpy(a.cam + 3, c->p00, 12);
  std::memcpy(a.cam + 6, c->du, 12);
  std::memcpy(a.cam + 9, c->dv, 12);
  std::memcpy(a.cam + 12, c->disk_u, 12);
  std::memcpy(a.cam + 15, c->disk_v, 12);
  a.defocus = c->defocus ? 1 : 0;
  a.n = ds->n;
  a.n_pad = ds->n_pad;
  a.width = p->width;
  a.rows_out = rows;
  a.row_begin = p->row_begin;
  a.row_tile = p->row_tile > 0 ? p->row_tile : 8;
  a.tile_first = p->tile_first;
  a.tile_step = p->tile_step;
  a.spp = p->spp;
  a.sample_begin = p->sample_begin;
  a.max_depth = p->max_depth;
  a.realm = (p->flags & RT_FLAG_REALM) ? 1 : 0;
  a.key = seed_key(p->seed);
  if (rows == 0) return RT_OK;
  HIP_TRY(hipSetDevice(ds->device));
  int vsel = launch_variant(*ds, *p);
  if (variant_table(vsel).scan == SCAN_BVHS && p->max_depth > 1023) vsel = 16;   // (a path's depth left: 10 bits in the exchange)
  const Variant& v = variant_table(vsel);
  if (!v.fn) return set_error(RT_E_ARG, "rt_launch: no kernel for variant " + std::to_string(vsel));
  const DTree& tr = ds->tree[variant_tree(vsel)];
  a.bvh_blob = tr.blob;
  a.bvh_blob_f4 = tr.blob_f4;
  a.bvh_off_pairs = tr.off_pairs;
  a.bvh_off_pidx = tr.off_pidx;
  a.big_pair0 = tr.big_pair0;
  a.n_big_leaves = tr.n_big_leaves;
  // entries per lane: the ordered traversal (trees 1, 2) holds at most depth
  // (a node on level L has L - 1 ancestors; the dead far-child write goes one
  // above them); tree 0 also serves the while-while variants (depth + 2)
  a.bvh_stack = vsel == 22 ? stack_entries_compact(tr) : stack_entries(tr, variant_tree(vsel));
  for (int k = 0; k < 3; ++k) a.bvh_c[k] = tr.c[k];
  a.bvh_r = tr.r;
  // drain compaction: a post holds as many paths as a wave's stack slice has
  // room for (RTCLJ_COMPACT: post at or below that many paths; 0 off)
  {
    const int words = a.bvh_stack * 16 * (v.scan == SCAN_BVHO || v.scan == SCAN_BVHQ7 ? 1 : 2);   // a wave's stack slice
    a.mb_paths = std::min(32, words / kMbFields);
    a.compact = is_bvh_scan(v.scan) ? std::min(a.mb_paths, env_int("RTCLJ_COMPACT", a.mb_paths, 0)) : 0;
  }
  hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  const int th = tile_rows(v.scan);   // the variant's tile rows
  const int gx = (p->width + kTile - 1) / kTile, gy = (rows + th - 1) / th;
  const dim3 block(v.threads);
  const int n_tiles = gx * gy;
  a.tiles_x = gx;
  if (v.stats) {
    const int rc = dbg_buffers(ds->device, &a.dbg, &a.dbgw);
    if (rc != RT_OK) return rc;
  }
#ifdef RTCLJ_DIAG
  else if (g_timeline) {   // wave timeline only (rt_debug_waves), no counters
    unsigned long long* unused = nullptr;
    const int rc = dbg_buffers(ds->device, &unused, &a.dbgw);
    if (rc != RT_OK) return rc;
  }
#endif
#ifdef RTCLJ_DIAG
  // (diagnostic: RTCLJ_LDS_PAD bytes of dynamic LDS added to the launch, to
  // measure the kernel at fewer workgroups per CU)
  const size_t lds = launch_lds(*ds, vsel) + static_cast<size_t>(env_int("RTCLJ_LDS_PAD", 0, 0));
#else
  const size_t lds = launch_lds(*ds, vsel);
#endif
  if (lds > 64 * 1024)
    HIP_TRY(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  // the stream's entry: adaptive schedule and split partial sums
  Schedule* sch = nullptr;
  std::unique_lock<std::mutex> sched_lock;
  {
    ScheduleSet& set = ds->sched;
    sched_lock = std::unique_lock<std::mutex>(set.mu);
    for (int k = 0; k < set.used && !sch; ++k)
      if (set.s[k].stream == stream) sch = &set.s[k];
    if (!sch && set.used < kSchedStreams) {
      sch = &set.s[set.used++];
      sch->stream = stream;
    }
  }
  // Sample split: a frame of fewer tiles than
  // kSplitRounds x the workgroups the GPU holds at once (a shard of a
  // multi-GPU frame, a small image) runs every tile as `split` workgroups,
  // one contiguous sample range each, so that the launch does not end on a
  // few whole tiles running alone (its length would be the longest tile's).
  // The integer pixel sums add up to the same bits in any grouping.
  // (The kernel also takes a whole-tile prefix of the order, n_whole; the
  // split tiles' partial sums go through finalize_kernel.)
  // (Tile sharing, below, takes the launches that are not split: a split
  // launch has about one unit per workgroup slot, all of which end together,
  // and on C1's 8-GPU shard the split is faster -- 1.05 vs 1.09-1.18 ms --
  // while sharing balances the tail of a long launch in plain order, C1
  // 6.78 -> 6.47 ms, and in the record's longest-first order costs nothing
  // (profiles/r03/share_ab.txt).  RTCLJ_STEAL=0: never share.)
  int split = 1, n_whole = n_tiles;
  const bool steal = sch && env_int("RTCLJ_STEAL", 1, 0) != 0 && !v.stats && v.scan != SCAN_BVHS;
  if (sch && p->spp > 1) {
    if (const char* e = std::getenv("RTCLJ_SPLIT")) {
      split = std::max(1, std::atoi(e));
    } else {
      const int slots = launch_slots(ds->device, v.fn, lds, v.threads);
      const int64_t want = static_cast<int64_t>(split_rounds()) * slots;
      if (slots > 0 && n_tiles < want) {
        split = static_cast<int>((want + n_tiles - 1) / n_tiles);
        // frames in flight: the next frame fills this launch's tail, so two
        // rounds of workgroups suffice (at least 2 splits: an unsplit heavy
        // tile would outlive two frames).  C1's 8-GPU shard, 2 streams:
        // 0.817 ms per frame at split 2 vs 0.87 at 3 (profiles/r03/shard_matrix_*.txt)
        if (p->flags & RT_FLAG_STREAMED)
          split = std::max(2, static_cast<int>((2 * static_cast<int64_t>(slots) + n_tiles - 1) / n_tiles));
      }
    }
    split = std::min(split, std::min(p->spp, kSplitMax));
    if (split > 1) n_whole = 0;
  }
  a.split = split;
  a.n_whole = n_whole;
  a.rt_magic = magic64(a.row_tile);
  const int64_t n_units64 = n_whole + static_cast<int64_t>(n_tiles - n_whole) * split;
  if (n_units64 > INT_MAX) return set_error(RT_E_ARG, "rt_launch: frame too large");
  const int n_units = static_cast<int>(n_units64);
  const size_t n_elems = static_cast<size_t>(rows) * p->width * 3;
  if (split > 1) {
    // the split tiles' integer sums: one u64 per channel, added to by the
    // splits, converted and zeroed by finalize_kernel
    const size_t need = n_elems;
    if (sch->part_cap < need) {   // grow: this stream's kernels may still read the old buffer
      HIP_TRY(hipStreamSynchronize(stream));
      if (sch->part) (void)hipFree(sch->part);
      sch->part = nullptr;
      sch->part_cap = 0;
      HIP_TRY(hipMalloc(&sch->part, need * sizeof(unsigned long long)));
      HIP_TRY(hipMemsetAsync(sch->part, 0, need * sizeof(unsigned long long), stream));
      sch->part_cap = need;
      sch->part_dirty = false;
    }
    if (sch->part_dirty) {   // an earlier launch failed between its trace and finalize kernels
      HIP_TRY(hipMemsetAsync(sch->part, 0, sch->part_cap * sizeof(unsigned long long), stream));
      sch->part_dirty = false;
    }
    a.part = sch->part;
  }
  // adaptive schedule: dispatch tiles longest first, by the durations the
  // previous launches of this launch shape on this scene and stream measured
  // (each launch's added to half the record before it)
  bool new_shape = false;
  if (sch) {
    ScheduleKey key{};
    key.width = a.width;
    key.rows = a.rows_out;
    key.row_begin = a.row_begin;
    key.row_tile = a.row_tile;
    key.tile_first = a.tile_first;
    key.tile_step = a.tile_step;
    key.gx = gx;
    key.gy = gy;
    if (std::memcmp(&sch->key, &key, sizeof key) != 0) {
      sch->ready = false;
      sch->key = key;
      new_shape = true;
    }
  }
  if (sch && g_schedule.load() == 0) {
    if (sch->cap < n_tiles) {   // grow: this stream's kernels may still read the old buffers
      HIP_TRY(hipStreamSynchronize(stream));
      if (sch->cost) (void)hipFree(sch->cost);
      if (sch->order) (void)hipFree(sch->order);
      sch->cost = nullptr;
      sch->order = nullptr;
      sch->cap = 0;
      sch->ready = false;
      HIP_TRY(hipMalloc(&sch->cost, n_tiles * sizeof(unsigned)));
      HIP_TRY(hipMalloc(&sch->order, n_tiles * sizeof(int)));
      sch->cap = n_tiles;
    }
    if (sch->ready) a.tile_order = sch->order;
    a.tile_cost = sch->cost;
    // a split launch in the recorded order: with RTCLJ_SPLIT_PLAN=1, the
    // cost-balanced units the previous launch of the shape planned (when it
    // planned this many).  Off by default: C1's 8-GPU shard 1.10-1.15 ms
    // against 0.99-1.02 with uniform splits, the 4-GPU one 1.93 vs 1.69
    // (profiles/r04/split_plan/; round 2's cost-sized splits lost the same
    // way): a heavy tile's many short pools each end with idle lanes.
    if (split > 1 && sch->ready && sch->plan_units == n_units - n_whole && env_int("RTCLJ_SPLIT_PLAN", 0, 0) != 0)
      a.unit_tab = sch->units;
    // the costs decay (order_kernel halves them after sorting): zeroed only
    // when this launch shape starts a new history
    if (!sch->ready) HIP_TRY(hipMemsetAsync(sch->cost, 0, n_tiles * sizeof(unsigned), stream));
  }
  // the grid: the units, then (stealing) the thieves, dispatched last, i.e.
  // as the units' slots free up in the launch's tail
  int64_t grid = n_units;
  // Sharing balances a launch whose tiles have no cost record (plain order:
  // a process's or a shape's first frame).  In the recorded longest-first
  // order the cheap tiles come last and the tail is short without it (C1
  // 5.94 ms either way), while its claims and helpers' scans are HBM atomics
  // (C1: 31 vs 11 MB per launch; profiles/r04/share_rounds/): off there
  // unless RTCLJ_SHARE_RECORDED=1.
  if (steal && split == 1 && (!a.tile_order || env_int("RTCLJ_SHARE_RECORDED", 0, 0) != 0)) {
    const int slots = std::max(1, launch_slots(ds->device, v.fn, lds, v.threads));
    const int n_owner = 2 * slots;   // owner entries: twice the resident workgroups
    // (at most 32 per slot: a tile's helper count stays below 2^16)
    grid += static_cast<int64_t>(std::min(32, env_int("RTCLJ_THIEVES", 4, 0))) * slots;
    if (grid > INT_MAX) grid = n_units;
    if (!sch->stealc) {
      HIP_TRY(hipMalloc(&sch->stealc, 2 * sizeof(unsigned long long)));
      HIP_TRY(hipMemsetAsync(sch->stealc, 0, 2 * sizeof(unsigned long long), stream));
    }
    if (sch->steal_cap < n_tiles) {   // grow: this stream's kernels may still use the old buffers
      HIP_TRY(hipStreamSynchronize(stream));
      if (sch->word) (void)hipFree(sch->word);
      if (sch->done) (void)hipFree(sch->done);
      if (sch->sum) (void)hipFree(sch->sum);
      sch->word = nullptr;
      sch->done = nullptr;
      sch->sum = nullptr;
      sch->steal_cap = 0;
      const size_t nsum = static_cast<size_t>(n_tiles) * kPoolPx * 3;
      HIP_TRY(hipMalloc(&sch->word, n_tiles * sizeof(unsigned long long)));
      HIP_TRY(hipMalloc(&sch->done, n_tiles * sizeof(unsigned)));
      HIP_TRY(hipMalloc(&sch->sum, nsum * sizeof(unsigned long long)));
      // words 0: lo = hi, nothing to steal until an owner publishes; sums
      // and done counts 0 (the kernel keeps them so between uses)
      HIP_TRY(hipMemsetAsync(sch->word, 0, n_tiles * sizeof(unsigned long long), stream));
      HIP_TRY(hipMemsetAsync(sch->done, 0, n_tiles * sizeof(unsigned), stream));
      HIP_TRY(hipMemsetAsync(sch->sum, 0, nsum * sizeof(unsigned long long), stream));
      sch->steal_cap = n_tiles;
      new_shape = true;
    }
    if (sch->owner_cap != n_owner) {
      HIP_TRY(hipStreamSynchronize(stream));
      if (sch->owner) (void)hipFree(sch->owner);
      sch->owner = nullptr;
      sch->owner_cap = 0;
      HIP_TRY(hipMalloc(&sch->owner, n_owner * sizeof(int)));
      sch->owner_cap = n_owner;
      new_shape = true;
    }
    if (!sch->epoch_started) {   // (RTCLJ_EPOCH_START: tests start a stream near the wrap)
      sch->epoch = static_cast<unsigned>(std::min(0xffff, env_int("RTCLJ_EPOCH_START", 1, 1)) - 1);
      sch->epoch_started = true;
    }
    sch->epoch = (sch->epoch + 1) & 0xffffu;
    if (sch->epoch == 0) {   // wrapped: no word or owner entry may carry the epoch's last use
      sch->epoch = 1;
      new_shape = true;
    }
    a.epoch = sch->epoch;
    // a new shape (or a wrap): no tile is being run, and no word holds this
    // launch's epoch.  (Old owner entries would only name words of other
    // epochs, but tile indices of another shape may exceed this one's; a word
    // last published 65,535 launches ago carries the epoch a wrap reuses.)
    if (new_shape) {
      HIP_TRY(hipMemsetAsync(sch->owner, 0xff, n_owner * sizeof(int), stream));
      HIP_TRY(hipMemsetAsync(sch->word, 0, n_tiles * sizeof(unsigned long long), stream));
    }
    // owners publish only in the launch's last RTCLJ_SHARE_ROUNDS rounds of
    // units (default 2; a round = the workgroups the device holds at once.
    // C4 plain order: WRITE_SIZE 2.90 GB per launch at every round, 0.44 at
    // 2, 0.60 at 3; C1's timing the same at 1, 2, 3 or every round:
    // profiles/r04/share_rounds/)
    a.share_from = static_cast<int>(std::max<int64_t>(
        0, n_units - static_cast<int64_t>(env_int("RTCLJ_SHARE_ROUNDS", 2, 0)) * slots));
    a.word = sch->word;
    a.done = sch->done;
    a.sum = sch->sum;
    a.owner = sch->owner;
    a.n_owner = n_owner;
    a.stealc = sch->stealc;
    a.steal_min = env_int("RTCLJ_STEAL_MIN", 256, 1);
    // claims of up to 1024 samples in the record's longest-first order (the
    // heavy tiles start first: fewer claims, 6.03 -> 6.00 ms on C1); in plain
    // order up to 1/48 of the tile's pool (0: the kernel's per-pool rule; C1's
    // 6,400: 128 -- helpers then need small claims to balance the tail;
    // C4's 64,000: 1024)
    a.batch_max = env_int("RTCLJ_BATCH_MAX", a.tile_order ? 1024 : 0, 0);
  }
  a.n_units = n_units;
  // a wave's claims on an unshared pool: guided (an eighth of what is left
  // past its last batch), 64 .. RTCLJ_LDS_BATCH (default 256; fixed 64-index
  // batches were round 3's: C1 5.960 -> 5.916 ms, C2 287.9 -> 286.1 ms,
  // profiles/r04/lds_batch/)
  a.lds_batch_max = std::max(64, env_int("RTCLJ_LDS_BATCH", 256, 64));
  void* args[] = {&a};
  if (split > 1) sch->part_dirty = true;   // (cleared once finalize_kernel is enqueued)
  HIP_TRY(hipLaunchKernel(v.fn, dim3(static_cast<unsigned>(grid)), block, args, lds, stream));
  if (split > 1) {
    unsigned long long* part = a.part;
    const int* order = a.tile_order;
    int nw = n_whole, tx = gx, tht = th, w = p->width, nr = rows, spp = p->spp, realm = a.realm;
    float* out = d_out;
    void* fargs[] = {&part, &order, &nw, &tx, &tht, &w, &nr, &out, &spp, &realm};
    HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(&finalize_kernel), dim3(n_tiles - n_whole), dim3(kTile * 3 * th),
                            fargs, 0, stream));
    sch->part_dirty = false;
  }
  if (a.tile_cost) {
    // the next launch's order, stream-ordered after this kernel (no host sync)
    unsigned* cost = sch->cost;
    int* order = sch->order;
    int n = n_tiles;
    void* sargs[] = {&cost, &order, &n};
    HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(&order_kernel), dim3(1), dim3(1024), sargs, 0, stream));
    sch->ready = true;
    if (split > 1 && n_whole == 0 && env_int("RTCLJ_SPLIT_PLAN", 0, 0) != 0) {
      // the next split launch's cost-balanced units, from this record
      const int U = n_units;
      if (sch->units_cap < U) {   // grow: this stream's kernels may still read the old plan
        HIP_TRY(hipStreamSynchronize(stream));
        if (sch->units) (void)hipFree(sch->units);
        sch->units = nullptr;
        sch->units_cap = 0;
        HIP_TRY(hipMalloc(&sch->units, U * sizeof(int2)));
        sch->units_cap = U;
      }
      int2* units = sch->units;
      int Uk = U, smax = std::min(p->spp, kSplitMax);
      void* pargs[] = {&cost, &order, &n, &Uk, &smax, &units};
      HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(&plan_kernel), dim3(1), dim3(1024), pargs, 0, stream));
      sch->plan_units = U;
    } else {
      sch->plan_units = -1;
    }
  }
  HIP_TRY(hipGetLastError());
  return RT_OK;
}

// A device's start-up ahead of the first render (rt.h): the context, the
// kernels' code object (loaded for the device on a function lookup), the NULL
// stream's first work (its hardware queue) and a small pageable D2H copy (the
// runtime's staging for pageable transfers, which the first frame's gather
// otherwise pays).  Each part timed on the host.
extern "C" int rt_prepare(int device, double* out_ms4) {
  clear_error();
  using Clk = std::chrono::steady_clock;
  auto ms = [](Clk::time_point a, Clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return set_error(RT_E_NODEV, "rt_prepare: device " + std::to_string(device) + " not available");
  const auto t0 = Clk::now();
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipFree(nullptr));
  const auto t1 = Clk::now();
  hipFuncAttributes fa{};
  HIP_TRY(hipFuncGetAttributes(&fa, variant_table(16).fn));
  const auto t2 = Clk::now();
  constexpr size_t kProbe = 64 * 1024;
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, kProbe));
  hipError_t e = hipMemsetAsync(d, 0, kProbe, nullptr);
  if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
  const auto t3 = Clk::now();
  std::vector<unsigned char> host(kProbe);
  if (e == hipSuccess) e = hipMemcpy(host.data(), d, kProbe, hipMemcpyDeviceToHost);
  const auto t4 = Clk::now();
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(e, "rt_prepare");
  if (out_ms4) {
    out_ms4[0] = ms(t0, t1);
    out_ms4[1] = ms(t1, t2);
    out_ms4[2] = ms(t2, t3);
    out_ms4[3] = ms(t3, t4);
  }
  return RT_OK;
}

// Stats builds read-back: sums and clears the kDbg debug counters of every
// device that ran a stats launch.
extern "C" int rt_debug_stats(uint64_t* out32) {
  clear_error();
  if (!out32) return set_error(RT_E_ARG, "rt_debug_stats: NULL");
  for (int i = 0; i < kDbg; ++i) out32[i] = 0;
  std::lock_guard<std::mutex> lk(g_dbg_mu);
  for (int d = 0; d < kDbgDevices; ++d) {
    if (!g_dbg[d]) continue;
    uint64_t v[kDbg];
    HIP_TRY(hipSetDevice(d));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(v, g_dbg[d], sizeof v, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(g_dbg[d], 0, sizeof v));
    for (int i = 0; i < kDbg; ++i) out32[i] += v[i];
  }
  return RT_OK;
}

// Steals of the launches on (ds, stream) since the last call: out2 =
// {steals, samples stolen}; waits for the stream, then clears them.
extern "C" int rt_steal_stats(const rt_dscene* ds, void* hip_stream, uint64_t* out2) {
  clear_error();
  if (!ds || !out2) return set_error(RT_E_ARG, "rt_steal_stats: NULL argument");
  out2[0] = out2[1] = 0;
  const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  std::lock_guard<std::mutex> lk(ds->sched.mu);
  for (int k = 0; k < ds->sched.used; ++k) {
    const Schedule& e = ds->sched.s[k];
    if (e.stream != stream || !e.stealc) continue;
    HIP_TRY(hipSetDevice(ds->device));
    HIP_TRY(hipStreamSynchronize(stream));
    HIP_TRY(hipMemcpy(out2, e.stealc, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(e.stealc, 0, 2 * sizeof(uint64_t)));
  }
  return RT_OK;
}

// Stats build wave timeline of `device`: up to n waves x {t_start, t_end,
// hw_id, xcc_id} (s_memrealtime ticks, 100 MHz); cleared after the copy.
extern "C" int rt_debug_waves(int device, uint64_t* out, size_t n_waves) {
  clear_error();
  if (!out) return set_error(RT_E_ARG, "rt_debug_waves: NULL");
  if (device < 0 || device >= kDbgDevices) return set_error(RT_E_ARG, "rt_debug_waves: bad device");
  std::lock_guard<std::mutex> lk(g_dbg_mu);
  if (!g_dbgw[device]) return 0;
  if (n_waves > kDbgWaves) n_waves = kDbgWaves;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, g_dbgw[device], 4 * n_waves * sizeof(uint64_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemset(g_dbgw[device], 0, 4 * kDbgWaves * sizeof(uint64_t)));
  return static_cast<int>(n_waves);
}
