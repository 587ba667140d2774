// trace.hip — the product library's gfx950 code object and host side: the
// shipped kernel's instantiations (trace_kernel.h: the default BVH walk in its
// two LDS images and its fallbacks), the schedule / split / quantise / fill
// kernels, and rt_scene_upload / rt_launch.  The A/B scans, the
// direction-coherent waves and the statistics builds live in trace_diag.hip
// (librtclj_diag.so only).  DESIGN.md §3.
#include "trace_kernel.h"

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

namespace rtclj {

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
  __shared__ int scan[256];
  const int t = static_cast<int>(threadIdx.x);
  if (t < 256) hist[t] = 0;
  __syncthreads();
  for (int i = t; i < n; i += 1024) atomicAdd(&hist[cost_bucket(cost[i])], 1);
  __syncthreads();
  // descending cost first: bucket b's first slot is the count of the buckets
  // above it (a parallel scan over the reversed histogram, 8 steps)
  if (t < 256) scan[t] = hist[255 - t];
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int v = (t < 256 && t >= off) ? scan[t - off] : 0;
    __syncthreads();
    if (t < 256) scan[t] += v;
    __syncthreads();
  }
  if (t < 256) cursor[255 - t] = scan[t] - hist[255 - t];
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

// The library's own buffer fill (zeroing the per-stream records, the split
// sums, the counters): every memset of the product path runs this kernel, in
// the library's code object, instead of the HIP runtime's blit kernel, whose
// code object a fresh process would otherwise load on its first frame.
__global__ __launch_bounds__(256) void fill_kernel(uint32_t* __restrict__ p, uint32_t v, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) p[i] = v;
}

// Several fills in one launch: the zeroings a launch of a new shape needs
// (its tile-cost record, the sharing words and owner table) as one kernel in
// front of the trace kernel instead of one small launch each.
struct FillSet {
  static constexpr int kMax = 6;
  uint32_t* p[kMax];
  uint32_t v[kMax];
  size_t n[kMax];
  int count = 0;
  void add(void* ptr, int byte_value, size_t bytes) {
    p[count] = static_cast<uint32_t*>(ptr);
    v[count] = static_cast<uint32_t>(byte_value & 0xff) * 0x01010101u;
    n[count] = bytes / 4;
    ++count;
  }
};
// A shape's first order, before any record: the tiles bottom-up
// (order[i] = n - 1 - i)
__global__ __launch_bounds__(256) void iota_rev_kernel(int* __restrict__ order, int n) {
  const int i = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  if (i < n) order[i] = n - 1 - i;
}

__global__ __launch_bounds__(256) void fill_set_kernel(const FillSet f) {
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  for (int k = 0; k < f.count; ++k)
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < f.n[k]; i += stride) f.p[k][i] = f.v[k];
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
//   22 BVH in LDS, 4-body leaves, compact image (u8 node-index stack, u32
//      pixel sums with counted wraps, 8-byte pixel table): seven workgroups
//      per CU -- the default where spp < 65536, albedos lie in [-1, 1], the
//      tree has <= 256 nodes and the frame is at most 65536 pixels wide and high
//   16 the same walk in the full image (u16 stack of node addresses, u64 sums)
//   26 22's compact image in 16-wave workgroups (one tree image per 16
//      waves, 64 VGPRs: 8 waves per SIMD): the default for scenes whose
//      4-body image is too big for 22 (C4), where 22 applies and two fit a CU
//   24 the same in 8-wave workgroups: where three of those fit and not two of 26's
//   28 22 on 8 x 4-pixel pools (whole pools for launches of few 8 x 8 tiles
//      instead of sample splits: measured slower, selected only explicitly
//      or by RTCLJ_TH4)
//   18 BVH in LDS, 8-body leaves (large scenes where 24 does not fit)
//   12 BVH (2-body leaves) read from global memory: a tree too big for LDS
//    5 linear scan, grouped, table through the scalar cache: a tree too deep
//    0 = default (22 where it applies, else 16; 26, 24, else 18, when the 4-body tree's LDS image is large)
// The diagnostic library (lib/librtclj_diag.so) adds, from trace_diag.hip, the
// A/B variants -- 1, 2 simple scan (LDS, scalar cache), 4 grouped scan in LDS
// (north_star's LDS-staged scan), 8, 9 packed pairs, 11 BVH with 2-body leaves
// in LDS, 20 / 21 direction-coherent waves (sorted_kernel) -- and the
// statistics builds 3, 6, 7, 10, 13, 17 (= 16 + stats), 19 (= 18 + stats).
// Every variant renders the same bits.
// the tree a traversal variant walks: 0 = 2-body leaves, 1 = 4, 2 = 8
const void* trace_kernel_w16();   // trace_w16.hip
static int variant_tree(int v) { return v >= 20 ? 1 : v >= 18 ? 2 : v >= 16 ? 1 : 0; }
static const Variant& variant_table(int v) {
  static const Variant none{nullptr, false, false, 0};
  static const Variant placeholder{RT_K(SRC_LDS, SCAN_BVHQ, false), true, false, SCAN_BVHQ};   // 0: resolved per scene
  static const Variant v5{RT_K(SRC_SCALAR, SCAN_GROUP4, false), false, false, SCAN_GROUP4};
  static const Variant v12{RT_K(SRC_SCALAR, SCAN_BVH, false), false, false, SCAN_BVH};
  static const Variant v16{RT_K(SRC_LDS, SCAN_BVHQ, false), true, false, SCAN_BVHQ};
  // (8-wave workgroups: one tree image for twice the waves)
  static const Variant v18{RT_KW(SRC_LDS, SCAN_BVHO, false, 8), true, false, SCAN_BVHO, 512};
  static const Variant v22{RT_K(SRC_LDS, SCAN_BVHQ7, false), true, false, SCAN_BVHQ7, 256, 0,
                           RT_KSW(SRC_LDS, SCAN_BVHQ7, 4, 0)};
  // (22's image in 8-wave workgroups: one tree image per 8 waves, for trees
  // too big for 22's 4-wave workgroups)
  static const Variant v24{RT_KW(SRC_LDS, SCAN_BVHQ7, false, 8), true, false, SCAN_BVHQ7, 512};
  // (and in 16-wave workgroups, 64 VGPRs: 8 waves per SIMD)
  // (trace_w16.hip, compiled with its own scheduler flag)
  static const Variant v26{trace_kernel_w16(), true, false, SCAN_BVHQ7, 1024};
  // (22 on 8 x 4-pixel pools: whole pools of half the pixels for launches of
  // few 8 x 8 tiles instead of sample splits; measured slower)
  static const Variant v28{RT_KWT(SRC_LDS, SCAN_BVHQ7, false, 4, 4), true, false, SCAN_BVHQ7, 256, 4};
  switch (v) {
    case 0: return placeholder;
    case 5: return v5;
    case 12: return v12;
    case 16: return v16;
    case 18: return v18;
    case 22: return v22;
    case 24: return v24;
    case 26: return v26;
    case 28: return v28;
  }
#ifdef RTCLJ_DIAG
  if (const Variant* d = diag_variant(v)) return *d;
#endif
  return none;
}
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
  // The sort of the last launch's record (order_kernel, and plan_kernel for a
  // planned split) is enqueued at the start of the next launch of the shape
  // on the stream, not behind the trace kernel: a frame's launch ends with
  // its trace kernel (a one-frame process never pays the sort), and a frame
  // loop pays it once per frame as before.  sort_plan: the plan's unit count
  // (-1: no plan).
  bool sort_pending = false;
  int sort_plan = -1;
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
  // path export (KArgs xq, xq_n): the records of a split launch's exported
  // paths, and [written, the sweep's claims] (zeroed before each launch)
  uint4* xq = nullptr;
  size_t xq_cap = 0;                    // records
  unsigned* xq_n = nullptr;
  unsigned long long xq_launches = 0;   // export launches since rt_export_stats
};
constexpr int kSchedStreams = 16;
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
    if (e.xq) (void)hipFree(e.xq);
    if (e.xq_n) (void)hipFree(e.xq_n);
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
// (threads: the workgroup's lanes, a stack row each)
static size_t stack_of(const DTree& t, int tree, int threads = 256) {
  return static_cast<size_t>(stack_entries(t, tree)) * threads * (tree == 2 ? 1 : 2);
}
static size_t lds_of(const DTree& t, int tree, int threads = 256) {
  return static_cast<size_t>(t.blob_f4) * 16 + stack_of(t, tree, threads);
}
// variant 22 (the compact image): u8 node indices, depth rows (the dead
// far-child write goes one above the top, as in 16)
static int stack_entries_compact(const DTree& t) { return std::max(t.depth, 1); }
static size_t lds_of_compact(const DTree& t, int threads) {
  return static_cast<size_t>(t.blob_f4) * 16 + static_cast<size_t>(stack_entries_compact(t)) * threads;
}
// LDS a CU can give each of 5 workgroups (160 KB / 5), less the 4-body-leaf
// kernel's static LDS (pool counter, the 64 pixels' colour sums and pixel
// table).  (Its registers allow 6; C1's 24.0 KB image fits 6 as well.)
constexpr size_t kStaticLds = 4 + kPoolPx * 3 * 8 + kPoolPx * 16 + 12;   // (the 8-body traversal: no table, 1 KB less)
constexpr size_t kLds5 = 160 * 1024 / 5 - kStaticLds;
// (variants 24 / 26's static LDS, 1.4 / 1.5 KB: the 64 pixels' u32 sums and
// keys, the wrap counts, 8 or 16 waves' compaction counters; 2 KB allowed for)
constexpr size_t kStaticLds8 = 2048;

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

// the most splits of one tile (rt_launch's sample split, below)
constexpr int kSplitMax = 64;

// The pending sort of a stream's tile-cost record (Schedule::sort_pending):
// order_kernel, and plan_kernel for a planned split; the order is ready for
// the next launch of the shape.  Returns the launches' hipError_t.
static int sort_record(Schedule* sch, int n_tiles, int spp, hipStream_t stream) {
  unsigned* cost = sch->cost;
  int* order = sch->order;
  int n = n_tiles;
  void* sargs[] = {&cost, &order, &n};
  hipError_t e = hipLaunchKernel(reinterpret_cast<const void*>(&order_kernel), dim3(1), dim3(1024), sargs, 0, stream);
  if (e != hipSuccess) return e;
  sch->ready = true;
  sch->sort_pending = false;
  sch->plan_units = -1;
  if (sch->sort_plan > 0 && sch->units_cap >= sch->sort_plan) {
    // the next split launch's cost-balanced units, from this record
    int2* units = sch->units;
    int Uk = sch->sort_plan, smax = std::min(spp, kSplitMax);
    void* pargs[] = {&cost, &order, &n, &Uk, &smax, &units};
    e = hipLaunchKernel(reinterpret_cast<const void*>(&plan_kernel), dim3(1), dim3(1024), pargs, 0, stream);
    if (e != hipSuccess) return e;
    sch->plan_units = sch->sort_plan;
  }
  return hipSuccess;
}

// the variants of the compact image (u8 node-index stack, u32 sums)
static bool compact_variant(int v) { return v == 22 || v == 24 || v == 26 || v == 28; }

// selector -> the variant a launch on ds runs
static int resolve_variant(const rt_dscene& ds, int vsel) {
  // default: 4-body leaves, unless that tree's LDS image limits a CU below
  // 5 workgroups (160 KB / 5) and the 8-body-leaf tree's is smaller
  // (measured: 1025 bodies 12.9 vs 14.0 ms; 484: 10.8 vs 12.2); each image
  // with the stack rows of its own variant's workgroup (18: 512 lanes)
  if (vsel == 0)
    vsel = (lds_of(ds.tree[1], 1) > kLds5 && ds.tree[2].n_nodes <= 256 &&
            lds_of(ds.tree[2], 2, variant_table(18).threads) < lds_of(ds.tree[1], 1)) ? 18 : 16;
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
    // (the stack rows of the variant's own workgroup size, as launch_lds)
    if (vsel != 12 && lds_of(t, variant_tree(vsel), variant_table(vsel).threads) > 96 * 1024)
      vsel = 12;   // tree too big for LDS: 2-body leaves, global
    if (vsel == 12 && ds.tree[0].depth + 2 > kBvhStack) return 5;
  }
  if (compact_variant(vsel) && ds.tree[1].n_nodes > 256) vsel = 16;   // (u8 node indices)
  return vsel;
}

// The compact variant (22) for a launch: the 4-body tree's node indices fit
// a byte, and a pixel's u32 sum with its byte of wrap counts cannot overflow
// -- every sample's colour is at most 1 per channel (albedos within [-1, 1]:
// the sky and the dielectric give at most 1), so a channel wraps at most spp /
// 256 < 256 times for spp < 65536 (none for spp <= 255, where the kernel adds
// without counting).  Its pixel table packs no coordinates above 65535 (the
// key table plus one image row per tile row).  The default selector runs it
// wherever it applies (and an explicit 22 too); elsewhere the launch runs 16.
// Seven workgroups per CU instead of six, in 72 VGPRs without a spill.
static bool compact_ok(const rt_dscene& ds, const rt_params& p) {
  return ds.unit_albedo && ds.tree[1].n_nodes <= 256 && p.spp < 65536 && ds.tree[1].depth + 2 <= kBvhStack &&
         p.width <= 65536 && p.height <= 65536;
}
static int launch_variant(const rt_dscene& ds, const rt_params& p) {
  const int sel = g_variant.load();
  int vsel = resolve_variant(ds, sel);
  if ((sel == 0 && vsel == 16) || vsel == 22) vsel = compact_ok(ds, p) ? 22 : 16;
  // A scene the default sends to the 8-body-leaf walk (its 4-body image too
  // big for five 4-wave workgroups a CU) runs 22's compact image on the
  // 4-body walk's leaf records instead, in workgroups that share one image
  // among more waves: 16-wave workgroups (26) where two fit a CU -- 8 waves
  // per SIMD in 64 VGPRs -- else 8-wave ones (24) where three fit -- 6 per
  // SIMD, as 18.  C4: 4.295 s (26) vs 4.570 (24) vs 4.931 (18), same boxes
  // (profiles/r05/c4_v26/, c4_v24/); C2's frame on 26 instead of 22: 260.4 vs
  // 251.8 ms (a pool's 32,000 samples over 1,024 lanes drain too often).
  if (sel == 0 && vsel == 18 && compact_ok(ds, p)) {
    if (lds_of_compact(ds.tree[1], 1024) + kStaticLds8 <= 160 * 1024 / 2)
      vsel = 26;
    else if (lds_of_compact(ds.tree[1], 512) + kStaticLds8 <= 160 * 1024 / 3)
      vsel = 24;
  }
  if ((vsel == 24 || vsel == 26 || vsel == 28) && !compact_ok(ds, p)) vsel = 16;
  // RTCLJ_TH4=r (A/B knob, default 0 = never): a launch of 22 with fewer
  // 8 x 8 tiles than r x the workgroups the device holds -- a shard of a
  // multi-GPU frame -- runs 28: the same image on 8 x 4-pixel pools, whole,
  // where 22 splits every tile's samples over 2-3 workgroups.  Measured at r
  // = 2 (profiles/r06/th4/): C1's 8-rank shard 1.62 ms against 0.84 with the
  // splits, the 4-rank 1.56 against 1.37 (the whole 8 x 4 pools are 1.84
  // rounds of 3,200-sample units: the last round's long units are the tail),
  // and 28 costs 5 % more per sample on the whole C1 frame (4.95 vs 4.71 ms:
  // a pool of half the pixels drains twice as often).  DESIGN.md §6.
  if (sel == 0 && vsel == 22) {
    const int ratio = env_int("RTCLJ_TH4", 0, 0);
    if (ratio > 0) {
      const int rows = rows_out(p);
      const int64_t n8 = static_cast<int64_t>((p.width + kTile - 1) / kTile) * ((rows + kTile - 1) / kTile);
      const Variant& v22 = variant_table(22);
      const int slots = launch_slots(ds.device, v22.fn, lds_of_compact(ds.tree[1], v22.threads), v22.threads);
      if (slots > 0 && n8 < static_cast<int64_t>(ratio) * slots) vsel = 28;
    }
  }
  return vsel;
}

extern "C" int rt_resolve_variant(const rt_dscene* ds) { return ds ? resolve_variant(*ds, g_variant.load()) : -1; }

// dynamic LDS of a launch of variant vsel on ds
static size_t launch_lds(const rt_dscene& ds, int vsel) {
  const Variant& v = variant_table(vsel);
  if (v.scan == SCAN_BVHS) return static_cast<size_t>(ds.tree[1].blob_f4) * 16 + kXBytes;   // blob | exchange
  if (compact_variant(vsel)) return lds_of_compact(ds.tree[1], v.threads);
  if (vsel >= 11) {
    const DTree& tr = ds.tree[variant_tree(vsel)];
    return v.lds ? lds_of(tr, variant_tree(vsel), v.threads) : stack_of(tr, variant_tree(vsel), v.threads);
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
// (kSplitMax, the most splits of a tile: defined above sort_record)

namespace rtclj {
int fill_async(void* p, int byte_value, size_t bytes, void* stream) {
  if (bytes == 0) return hipSuccess;
  if (bytes % 4 != 0) return hipErrorInvalidValue;   // (every buffer the product fills is whole words)
  uint32_t* w = static_cast<uint32_t*>(p);
  uint32_t v = static_cast<uint32_t>(byte_value & 0xff) * 0x01010101u;
  size_t n = bytes / 4;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 2048);
  void* args[] = {&w, &v, &n};
  return hipLaunchKernel(reinterpret_cast<const void*>(&fill_kernel), dim3(static_cast<unsigned>(blocks)), dim3(256),
                         args, 0, static_cast<hipStream_t>(stream));
}

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
      (p->flags & ~(RT_FLAG_REALM | RT_FLAG_STREAMED | RT_FLAG_REJECTION_SAMPLERS)) != 0)
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
  // the loop-free samplers unless the caller asks for the reference's rejection loops
  a.sampler = (p->flags & RT_FLAG_REJECTION_SAMPLERS) ? 0 : (RT_SAMPLER_SPHERE | RT_SAMPLER_DISK);
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
  a.bvh_stack = compact_variant(vsel) ? stack_entries_compact(tr) : stack_entries(tr, variant_tree(vsel));
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
  const int th = variant_rows(v);   // the variant's tile rows
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
  if (lds > 64 * 1024) {
    HIP_TRY(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    if (v.sweep) HIP_TRY(hipFuncSetAttribute(v.sweep, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  }
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
      // (28: its pools are the split's answer already; they split only when
      // fewer than RTCLJ_TH4_SPLIT_ROUNDS (1) rounds of them fill the device)
      const int rounds = vsel == 28 ? env_int("RTCLJ_TH4_SPLIT_ROUNDS", 1, 1) : split_rounds();
      const int64_t want = static_cast<int64_t>(rounds) * slots;
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
      HIP_TRY(static_cast<hipError_t>(fill_async(sch->part, 0, need * sizeof(unsigned long long), stream)));
      sch->part_cap = need;
      sch->part_dirty = false;
    }
    if (sch->part_dirty) {   // an earlier launch failed between its trace and finalize kernels
      HIP_TRY(static_cast<hipError_t>(fill_async(sch->part, 0, sch->part_cap * sizeof(unsigned long long), stream)));
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
      sch->sort_pending = false;   // (that record was another shape's)
      sch->key = key;
      new_shape = true;
    }
  }
  // the fills this launch needs before its trace kernel, as one launch
  FillSet fills;
  bool first_order = false;   // a shape's first launch in a heuristic order
  if (sch && g_schedule.load() == 0) {
    if (sch->cap < n_tiles) {   // grow: this stream's kernels may still read the old buffers
      HIP_TRY(hipStreamSynchronize(stream));
      if (sch->cost) (void)hipFree(sch->cost);
      if (sch->order) (void)hipFree(sch->order);
      sch->cost = nullptr;
      sch->order = nullptr;
      sch->cap = 0;
      sch->ready = false;
      sch->sort_pending = false;
      HIP_TRY(hipMalloc(&sch->cost, n_tiles * sizeof(unsigned)));
      HIP_TRY(hipMalloc(&sch->order, n_tiles * sizeof(int)));
      sch->cap = n_tiles;
    }
    // the previous launch's record, sorted now (stream-ordered after it)
    if (sch->sort_pending) HIP_TRY(static_cast<hipError_t>(sort_record(sch, n_tiles, p->spp, stream)));
    if (sch->ready) {
      a.tile_order = sch->order;
    } else if (env_int("RTCLJ_FIRST_ORDER", 1, 0) == 1) {
      // No record yet: the tiles bottom-up.  The reference's scenes (and
      // C1-C4) put the ground and its bodies below the sky: the expensive
      // tiles start first and the launch ends on sky tiles, where row-major
      // order ended on the ground's.  C1's first frame of a shape 5.13-5.19
      // ms against 5.25 row-major (tools/first_frame.py, 9 pairs, two
      // rounds; profiles/r06/first_order/); RTCLJ_FIRST_ORDER=0: row-major.
      // Tile sharing still balances the tail, as in plain order.
      int* order = sch->order;
      int n = n_tiles;
      void* oargs[] = {&order, &n};
      HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(&iota_rev_kernel), dim3(static_cast<unsigned>((n + 255) / 256)),
                              dim3(256), oargs, 0, stream));
      a.tile_order = sch->order;
      first_order = true;
    }
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
    if (!sch->ready) fills.add(sch->cost, 0, n_tiles * sizeof(unsigned));
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
  if (steal && split == 1 && (!a.tile_order || first_order || env_int("RTCLJ_SHARE_RECORDED", 0, 0) != 0)) {
    const int slots = std::max(1, launch_slots(ds->device, v.fn, lds, v.threads));
    const int n_owner = 2 * slots;   // owner entries: twice the resident workgroups
    // (at most 32 per slot: a tile's helper count stays below 2^16)
    grid += static_cast<int64_t>(std::min(32, env_int("RTCLJ_THIEVES", 4, 0))) * slots;
    if (grid > INT_MAX) grid = n_units;
    if (!sch->stealc) {
      HIP_TRY(hipMalloc(&sch->stealc, 2 * sizeof(unsigned long long)));
      HIP_TRY(static_cast<hipError_t>(fill_async(sch->stealc, 0, 2 * sizeof(unsigned long long), stream)));
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
      HIP_TRY(static_cast<hipError_t>(fill_async(sch->word, 0, n_tiles * sizeof(unsigned long long), stream)));
      HIP_TRY(static_cast<hipError_t>(fill_async(sch->done, 0, n_tiles * sizeof(unsigned), stream)));
      HIP_TRY(static_cast<hipError_t>(fill_async(sch->sum, 0, nsum * sizeof(unsigned long long), stream)));
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
      fills.add(sch->owner, 0xff, n_owner * sizeof(int));
      fills.add(sch->word, 0, n_tiles * sizeof(unsigned long long));
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
    a.batch_max = env_int("RTCLJ_BATCH_MAX", (a.tile_order && !first_order) ? 1024 : 0, 0);
  }
  a.n_units = n_units;
  // a wave's claims on an unshared pool: guided (an eighth of what is left
  // past its last batch), 64 .. RTCLJ_LDS_BATCH (default 256; fixed 64-index
  // batches were round 3's: C1 5.960 -> 5.916 ms, C2 287.9 -> 286.1 ms,
  // profiles/r04/lds_batch/)
  a.lds_batch_max = std::max(64, env_int("RTCLJ_LDS_BATCH", 256, 64));
  // Path export for split launches (KArgs xq; RTCLJ_EXPORT=1, A/B): a wave
  // whose batches are spent and which holds at most RTCLJ_EXPORT_LIM paths
  // (default 64: as soon as its batches are spent) writes them out and
  // leaves, so a unit's workgroup frees its slot without draining; the sweep
  // launch runs the records.  At most one record per thread of a unit.
  const bool xport = split > 1 && v.sweep && env_int("RTCLJ_EXPORT", 0, 0) != 0;
  if (xport) {
    const size_t need = static_cast<size_t>(n_units) * v.threads;
    if (sch->xq_cap < need) {   // grow: this stream's kernels may still read the old records
      HIP_TRY(hipStreamSynchronize(stream));
      if (sch->xq) (void)hipFree(sch->xq);
      sch->xq = nullptr;
      sch->xq_cap = 0;
      HIP_TRY(hipMalloc(&sch->xq, need * 4 * sizeof(uint4)));
      sch->xq_cap = need;
    }
    if (!sch->xq_n) HIP_TRY(hipMalloc(&sch->xq_n, 2 * sizeof(unsigned)));
    fills.add(sch->xq_n, 0, 2 * sizeof(unsigned));
    a.xq = sch->xq;
    a.xq_n = sch->xq_n;
    a.compact = std::min(64, env_int("RTCLJ_EXPORT_LIM", 64, 1));
    ++sch->xq_launches;
  }
  if (fills.count) {
    size_t most = 0;
    for (int k = 0; k < fills.count; ++k) most = std::max(most, fills.n[k]);
    const size_t blocks = std::max<size_t>(1, std::min<size_t>((most + 255) / 256, 2048));
    void* fa[] = {&fills};
    HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(&fill_set_kernel), dim3(static_cast<unsigned>(blocks)),
                            dim3(256), fa, 0, stream));
  }
  void* args[] = {&a};
  if (split > 1) sch->part_dirty = true;   // (cleared once finalize_kernel is enqueued)
  HIP_TRY(hipLaunchKernel(v.fn, dim3(static_cast<unsigned>(grid)), block, args, lds, stream));
  if (xport) {
    // the sweep: one workgroup per slot the device holds, each starting on
    // its own 256 records and claiming more; a workgroup past the records
    // leaves at once.  It adds into part[], so it runs before finalize_kernel.
    KArgs b = a;
    b.word = nullptr;
    b.tile_cost = nullptr;
    b.tile_order = nullptr;
    b.unit_tab = nullptr;
    b.compact = is_bvh_scan(v.scan) ? std::min(b.mb_paths, env_int("RTCLJ_COMPACT", b.mb_paths, 0)) : 0;
    const int sw = std::max(1, launch_slots(ds->device, v.sweep, lds, v.threads));
    void* bargs[] = {&b};
    HIP_TRY(hipLaunchKernel(v.sweep, dim3(static_cast<unsigned>(sw)), block, bargs, lds, stream));
  }
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
    // this record's sort, at the next launch of the shape on the stream
    // (RTCLJ_SORT_EAGER=1, A/B: right behind this launch, as before round 6;
    // within noise on every bench.py leg, profiles/r06/sort_ab/)
    sch->sort_pending = true;
    sch->ready = false;
    sch->sort_plan = -1;
    if (split > 1 && n_whole == 0 && env_int("RTCLJ_SPLIT_PLAN", 0, 0) != 0) {
      const int U = n_units;
      if (sch->units_cap < U) {   // grow: this stream's kernels may still read the old plan
        HIP_TRY(hipStreamSynchronize(stream));
        if (sch->units) (void)hipFree(sch->units);
        sch->units = nullptr;
        sch->units_cap = 0;
        HIP_TRY(hipMalloc(&sch->units, U * sizeof(int2)));
        sch->units_cap = U;
      }
      sch->sort_plan = U;
    }
    if (env_int("RTCLJ_SORT_EAGER", 0, 0) != 0) HIP_TRY(static_cast<hipError_t>(sort_record(sch, n_tiles, p->spp, stream)));
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
  hipError_t e = static_cast<hipError_t>(fill_async(d, 0, kProbe, nullptr));
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

// Path export of the split launches on (ds, stream) (diagnostic): out2 =
// {export launches since the last call, records the latest one wrote}; waits
// for the stream.
extern "C" int rt_export_stats(const rt_dscene* ds, void* hip_stream, uint64_t* out2) {
  clear_error();
  if (!ds || !out2) return set_error(RT_E_ARG, "rt_export_stats: NULL argument");
  out2[0] = out2[1] = 0;
  const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  std::lock_guard<std::mutex> lk(ds->sched.mu);
  for (int k = 0; k < ds->sched.used; ++k) {
    Schedule& e = ds->sched.s[k];
    if (e.stream != stream || !e.xq_n) continue;
    HIP_TRY(hipSetDevice(ds->device));
    HIP_TRY(hipStreamSynchronize(stream));
    unsigned n[2] = {0, 0};
    HIP_TRY(hipMemcpy(n, e.xq_n, sizeof n, hipMemcpyDeviceToHost));
    out2[0] = e.xq_launches;
    out2[1] = n[0];
    e.xq_launches = 0;
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
