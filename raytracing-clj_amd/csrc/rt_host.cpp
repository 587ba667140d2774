// rt_host.cpp — host side of the C ABI: camera set-up, quantise/PPM, error
// slot, and the multi-GPU fan-out of rt_render (one host thread per device,
// interleaved row tiles, host-side gather; no collectives).
//
// Reference anchors:
//   camera       src/raytracing.clj:105-139 (deg->rad :60-61)
//   write-color! src/raytracing.clj:19-26, PPM :172-175
//   executor     src/raytracing.clj:157-171 (2 threads, contiguous chunks —
//                here: N devices, interleaved 8-row tiles for balance)
//
// rt_render keeps, per device, the uploaded scenes (by content) and a few
// render contexts (stream, device framebuffer, pinned counters), so a
// repeated call pays neither the upload and BVH builds nor the allocations,
// and its launches reuse the stream whose adaptive tile order the previous
// call recorded.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt_internal.h"

namespace rtclj {

static thread_local std::string t_err;

int set_error(int code, const std::string& msg) {
  t_err = msg;
  return code;
}
void clear_error() { t_err.clear(); }

int rows_out(const rt_params& p) {
  if (p.row_begin < 0 || p.row_end < p.row_begin || p.row_end > p.height) return -1;
  const int span = p.row_end - p.row_begin;
  if (p.tile_step <= 0) return span;
  const int T = p.row_tile > 0 ? p.row_tile : 8;
  if (p.tile_first < 0 || p.tile_first >= p.tile_step) return -1;
  const int ntiles = (span + T - 1) / T;
  int rows = 0;
  for (int t = p.tile_first; t < ntiles; t += p.tile_step) rows += std::min(T, span - t * T);
  return rows;
}

}  // namespace rtclj

using namespace rtclj;

namespace {

struct D3 {
  double x, y, z;
};
D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 add(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
D3 mul(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
D3 divs(D3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
D3 neg(D3 a) { return {-a.x, -a.y, -a.z}; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 cross(D3 u, D3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
D3 unit(D3 v) { return divs(v, std::sqrt(dot(v, v))); }
void put(float* dst, D3 v) {
  dst[0] = static_cast<float>(v.x);
  dst[1] = static_cast<float>(v.y);
  dst[2] = static_cast<float>(v.z);
}

}  // namespace

extern "C" int rt_camera_setup(int image_width, int image_height, double vfov,
                               const double look_from[3], const double look_at[3],
                               const double vup[3], double defocus_angle, double focus_dist,
                               rt_camera* out) {
  clear_error();
  if (!look_from || !look_at || !vup || !out || image_width <= 0 || image_height <= 0)
    return set_error(RT_E_ARG, "rt_camera_setup: bad argument");
  const double pi = 3.141592653589793;  // Math/PI
  const D3 lf{look_from[0], look_from[1], look_from[2]};
  const D3 la{look_at[0], look_at[1], look_at[2]};
  const D3 up{vup[0], vup[1], vup[2]};
  const double theta = vfov * pi / 180.0;                              // deg->rad (:60-61)
  const double h = std::tan(theta / 2);                                // (:118)
  const double vh = 2.0 * h * focus_dist;                              // (:119)
  const double vw = vh * (static_cast<double>(image_width) / image_height);  // (:120)
  const D3 w = unit(sub(lf, la));                                      // (:122)
  const D3 u = unit(cross(up, w));                                     // (:123)
  const D3 v = cross(w, u);                                            // (:124)
  const D3 vu = mul(u, vw);                                            // (:127)
  const D3 vv = mul(neg(v), vh);                                       // (:128)
  const D3 du = divs(vu, image_width);                                 // (:129)
  const D3 dv = divs(vv, image_height);                                // (:130)
  const D3 ul = sub(sub(sub(lf, mul(w, focus_dist)), divs(vu, 2)), divs(vv, 2));  // (:131-134)
  const D3 p00 = add(ul, mul(add(du, dv), 0.5));                       // (:135)
  const double radius = focus_dist * std::tan((defocus_angle / 2.0) * pi / 180.0);  // (:137)
  put(out->center, lf);
  put(out->p00, p00);
  put(out->du, du);
  put(out->dv, dv);
  put(out->disk_u, mul(u, radius));
  put(out->disk_v, mul(v, radius));
  out->defocus = defocus_angle > 0 ? 1 : 0;  // (<= defocus-angle 0) -> centre (:147)
  return RT_OK;
}

// one channel's byte (color.clj write-color)
static inline uint8_t quantize1(float lin) {
  const double c = lin;
  const double g = c > 0 ? std::sqrt(c) : 0.0;              // linear->gamma (:21-22)
  const double cl = std::min(0.999, std::max(g, 0.0));      // clamp (:19), NaN -> 0 below
  const int q = static_cast<int>(256 * cl);                 // (int (* 256 ...)) (:25)
  return static_cast<uint8_t>(std::isnan(c) ? 0 : q);
}

namespace rtclj {
const float* quantize_thresholds() {
  // the byte is 0 for NaN and every float <= 0 and non-decreasing over the
  // positive floats in bit order (sqrt, min, the scale and the truncation
  // all are), so each threshold is a binary search over [+0, +inf]
  static const std::vector<float> t = [] {
    std::vector<float> v(256, -INFINITY);
    auto of = [](uint32_t b) {
      float f;
      std::memcpy(&f, &b, 4);
      return f;
    };
    for (int q = 1; q < 256; ++q) {
      uint32_t lo = 0, hi = 0x7f800000u;   // byte(lo) < q <= byte(hi) (byte(+inf) = 255)
      while (hi - lo > 1) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (quantize1(of(mid)) >= q) hi = mid;
        else lo = mid;
      }
      v[q] = of(hi);
    }
    return v;
  }();
  return t.data();
}
}  // namespace rtclj

extern "C" int rt_quantize(const float* lin, uint8_t* out, size_t n) {
  clear_error();
  if ((!lin || !out) && n) return set_error(RT_E_ARG, "rt_quantize: NULL argument");
  auto run = [lin, out](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) out[i] = quantize1(lin[i]);
  };
  // a frame of millions of channels on a few host threads (C1's 2.43 M: 4.4
  // ms on one); every channel is computed alone, so the split changes nothing
  const size_t kChunk = size_t{1} << 19;
  const int nt = static_cast<int>(std::min<size_t>(8, (n + kChunk - 1) / kChunk));
  if (nt <= 1) {
    run(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(run, n * t / nt, n * (t + 1) / nt);
    run(0, n / nt);
    for (auto& x : th) x.join();
  }
  return RT_OK;
}

extern "C" int rt_write_ppm(const char* path, const uint8_t* rgb, int width, int height) {
  clear_error();
  if (!path || !rgb || width <= 0 || height <= 0) return set_error(RT_E_ARG, "rt_write_ppm: bad argument");
  FILE* f = std::fopen(path, "wb");
  if (!f) return set_error(RT_E_IO, std::string("rt_write_ppm: cannot open ") + path);
  // "r g b\n" per pixel (raytracing.clj:172-175) from a table of the 256
  // decimal strings, each with its separator: no formatting per value (C1's
  // 810,000 pixels: 41.7 ms with a snprintf each)
  struct Dec {
    char s[4];
    int len;
  };
  static const auto* const dec = [] {
    auto* t = new Dec[256];
    for (int v = 0; v < 256; ++v) t[v].len = std::snprintf(t[v].s, sizeof t[v].s, "%d", v);
    return t;
  }();
  const std::string head = "P3\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
  bool ok = std::fwrite(head.data(), 1, head.size(), f) == head.size();
  // formatted a block of pixels at a time into a buffer that stays in cache
  // (at most "255 255 255\n", 12 bytes, a pixel)
  constexpr size_t kBlock = 16384;
  static thread_local std::unique_ptr<char[]> buf(new char[kBlock * 12]);
  const size_t npx = static_cast<size_t>(width) * height;
  for (size_t b = 0; ok && b < npx; b += kBlock) {
    const size_t e = std::min(npx, b + kBlock);
    char* o = buf.get();
    for (size_t i = b; i < e; ++i) {
      for (int c = 0; c < 3; ++c) {
        const Dec& d = dec[rgb[3 * i + c]];
        std::memcpy(o, d.s, 4);   // (the entry's 4 bytes; the separator overwrites what follows the digits)
        o += d.len;
        *o++ = c == 2 ? '\n' : ' ';
      }
    }
    const size_t nb = static_cast<size_t>(o - buf.get());
    ok = std::fwrite(buf.get(), 1, nb, f) == nb;
  }
  std::fclose(f);
  return ok ? RT_OK : set_error(RT_E_IO, std::string("rt_write_ppm: short write to ") + path);
}

extern "C" int rt_rows_out(const rt_params* p) {
  if (!p) return 0;
  const int r = rows_out(*p);
  return r < 0 ? 0 : r;
}

extern "C" int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" const char* rt_last_error(void) { return t_err.c_str(); }

extern "C" const char* rt_version(void) { return "rtclj-mi355x 0.3 (gfx950, abi 3)"; }

extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// ---- per-device scene cache (content-keyed) ---------------------------------
struct CachedScene {
  uint64_t hash = 0;
  std::vector<float> sphere, mat;
  std::vector<int> kind;
  std::shared_ptr<rt_dscene> ds;
  uint64_t last_use = 0;
};

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
  return h;
}
uint64_t scene_hash(const rt_scene& s) {
  uint64_t h = 0xcbf29ce484222325ull;
  h = fnv1a(h, &s.n, sizeof s.n);
  if (s.n > 0) {
    h = fnv1a(h, s.sphere, sizeof(float) * 4 * s.n);
    h = fnv1a(h, s.mat_kind, sizeof(int) * s.n);
    h = fnv1a(h, s.mat, sizeof(float) * 4 * s.n);
  }
  return h;
}
bool same_scene(const CachedScene& c, const rt_scene& s) {
  if (static_cast<int>(c.kind.size()) != s.n) return false;
  if (s.n == 0) return true;
  return std::memcmp(c.sphere.data(), s.sphere, sizeof(float) * 4 * s.n) == 0 &&
         std::memcmp(c.kind.data(), s.mat_kind, sizeof(int) * s.n) == 0 &&
         std::memcmp(c.mat.data(), s.mat, sizeof(float) * 4 * s.n) == 0;
}

// ---- per-device render context: stream, buffers, events ---------------------
struct Ctx {
  int device = 0;
  // the device's NULL stream: the first call of a device only (creating a
  // stream takes 5-7 ms on MI355X, tools/first_call.cpp -- most of a first
  // call's set-up).  The NULL stream synchronises with every blocking stream
  // of the device (a host application's, synchronous copies), so the next
  // call that takes this context gives it a non-blocking stream of its own
  // (take_ctx), with the tile orders recorded so far.
  bool null_stream = false;
  hipStream_t stream = nullptr;
  // e0 .. e1 the kernel, eg .. e2 the D2H (eg right behind e1 when the copy
  // is enqueued with the launch, else where finish_shard enqueues it)
  hipEvent_t e0 = nullptr, e1 = nullptr, eg = nullptr, e2 = nullptr;
  float* d_out = nullptr;
  size_t d_cap = 0;           // floats
  uint8_t* d_u8 = nullptr;    // rt_render_u8's bytes
  size_t u8_cap = 0;
  uint64_t* d_cnt = nullptr;
  uint64_t* h_cnt = nullptr;  // pinned
  std::vector<uint64_t> scenes;   // upload ids of the device scenes launched on (their per-stream schedule entries)
  void launched(const rt_dscene* ds) {
    const uint64_t id = scene_uid(ds);
    if (std::find(scenes.begin(), scenes.end(), id) == scenes.end()) scenes.push_back(id);
  }
  ~Ctx() {
    (void)hipSetDevice(device);
    if (stream || null_stream) {
      (void)hipStreamSynchronize(stream);
      // the per-stream slots of the scenes this context launched on
      release_stream_schedules(stream, scenes.data(), static_cast<int>(scenes.size()));
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (eg) (void)hipEventDestroy(eg);
    if (e2) (void)hipEventDestroy(e2);
    if (d_out) (void)hipFree(d_out);
    if (d_u8) (void)hipFree(d_u8);
    if (d_cnt) (void)hipFree(d_cnt);
    if (h_cnt) (void)hipHostFree(h_cnt);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// rt_render's fan-out threads, kept between calls: a call runs its first
// device's share on the calling thread and hands the others to idle
// workers (spawned when none is idle, up to 64, never joined: the pool lives
// as long as the process), instead of creating and joining a std::thread per
// device per call.  Tasks never wait on other pool tasks, so a queue longer
// than the idle workers only delays them.
class HostPool {
 public:
  void run(std::vector<std::function<void()>>& tasks) {
    if (tasks.empty()) return;
    struct Latch {
      std::mutex m;
      std::condition_variable cv;
      int left = 0;
    } latch;
    latch.left = static_cast<int>(tasks.size()) - 1;
    if (latch.left > 0) {
      std::lock_guard<std::mutex> lk(mu_);
      for (size_t i = 1; i < tasks.size(); ++i)
        q_.push_back([&tasks, &latch, i] {
          tasks[i]();
          std::lock_guard<std::mutex> l2(latch.m);
          if (--latch.left == 0) latch.cv.notify_all();
        });
      const int want = static_cast<int>(q_.size()) - idle_;
      for (int k = 0; k < want && workers_ < 64; ++k, ++workers_) std::thread([this] { work(); }).detach();
      cv_.notify_all();
    }
    tasks[0]();
    std::unique_lock<std::mutex> l2(latch.m);
    latch.cv.wait(l2, [&] { return latch.left == 0; });
  }

 private:
  void work() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      ++idle_;
      cv_.wait(lk, [this] { return !q_.empty(); });
      --idle_;
      std::function<void()> t = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      t();
      lk.lock();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  int idle_ = 0, workers_ = 0;
};
HostPool* g_pool = new HostPool;   // never destroyed (workers may still wait on it at exit)

constexpr int kSceneCache = 4;   // scenes kept per device (least recently used out)
// idle contexts kept per device: as many as a scene has per-stream schedule
// slots (trace.hip kSchedStreams), so RT_FLAG_SHARDS_ON_DEVICE0 with 8 shards
// and two frames in flight (rt_render_submit) keeps its 16 streams and their
// tile orders from call to call
constexpr int kFreeCtx = 16;

struct DeviceCache {
  std::mutex mu;
  std::mutex upload_mu;   // one upload at a time: concurrent misses of one scene build it once
  std::vector<CachedScene> scenes;
  std::vector<std::unique_ptr<Ctx>> free_ctx;
  // the context on the device's NULL stream, while idle (primary_made: it
  // exists, idle or in use)
  std::unique_ptr<Ctx> primary;
  bool primary_made = false;
  uint64_t tick = 0;
};
// never destroyed: HIP may already be torn down when static destructors run
std::vector<DeviceCache>* g_cache = new std::vector<DeviceCache>(64);
std::mutex g_cache_mu;

// the cached device scene of s on `device`, if there is one
bool find_scene(int device, const rt_scene* s, std::shared_ptr<rt_dscene>* out) {
  DeviceCache& dc = (*g_cache)[device];
  const uint64_t h = scene_hash(*s);
  std::lock_guard<std::mutex> lk(dc.mu);
  for (CachedScene& c : dc.scenes)
    if (c.hash == h && same_scene(c, *s)) {
      c.last_use = ++dc.tick;
      *out = c.ds;
      return true;
    }
  return false;
}

// the cached device scene of s on `device`, uploading it on a miss.  Shards
// of one call that share a device (RT_FLAG_SHARDS_ON_DEVICE0) and concurrent
// calls miss together: the first uploads under upload_mu, the others wait for
// it and then find its entry.
int get_scene(int device, const rt_scene* s, std::shared_ptr<rt_dscene>* out, bool* hit) {
  DeviceCache& dc = (*g_cache)[device];
  const uint64_t h = scene_hash(*s);
  auto lookup = [&]() {
    std::lock_guard<std::mutex> lk(dc.mu);
    for (CachedScene& c : dc.scenes)
      if (c.hash == h && same_scene(c, *s)) {
        c.last_use = ++dc.tick;
        *out = c.ds;
        *hit = true;
        return true;
      }
    return false;
  };
  if (lookup()) return RT_OK;
  std::lock_guard<std::mutex> up(dc.upload_mu);
  if (lookup()) return RT_OK;
  rt_dscene* raw = nullptr;
  const int rc = rt_scene_upload(device, s, &raw);
  if (rc != RT_OK) return rc;
  std::shared_ptr<rt_dscene> ds(raw, [](rt_dscene* d) { rt_scene_free(d); });
  CachedScene c;
  c.hash = h;
  if (s->n > 0) {
    c.sphere.assign(s->sphere, s->sphere + 4 * s->n);
    c.kind.assign(s->mat_kind, s->mat_kind + s->n);
    c.mat.assign(s->mat, s->mat + 4 * s->n);
  }
  c.ds = ds;
  std::lock_guard<std::mutex> lk(dc.mu);
  c.last_use = ++dc.tick;
  if (static_cast<int>(dc.scenes.size()) >= kSceneCache) {
    auto lru = std::min_element(dc.scenes.begin(), dc.scenes.end(),
                                [](const CachedScene& x, const CachedScene& y) { return x.last_use < y.last_use; });
    dc.scenes.erase(lru);   // freed when the last in-flight render drops it
  }
  dc.scenes.push_back(std::move(c));
  *out = ds;
  *hit = false;
  return RT_OK;
}

// A render context's stream: non-blocking, at the device's highest priority.
// The HIP runtime maps a process's streams onto a few hardware queues per
// priority level (GPU_MAX_HW_QUEUES, 4) and, once a level's queues exist,
// adds a new stream to one already in use.  A process that has run work on
// other streams (an application's own, bench.py's pipelined leg) then puts two
// frames in flight on one queue, where frame k's D2H, enqueued at
// rt_render_wait, waits behind frame k+1's kernel and the frame loop loses its
// overlap: C1 in flight 4.97 ms per frame at normal priority after bench.py's
// pipelined leg, 4.73-4.74 at high priority (or with a full CU mask, a queue
// of its own but a blocking stream), 4.69-4.72 in a fresh process either way
// (profiles/r06/inflight/).  RTCLJ_CTX_STREAM (A/B): 0 = normal priority,
// 1 = full CU mask.
hipError_t make_stream(int device, hipStream_t* s) {
  const char* v = std::getenv("RTCLJ_CTX_STREAM");
  const int kind = v ? std::atoi(v) : 2;
  if (kind == 1) {
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return e;
    std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0u);
    for (int k = 0; k < prop.multiProcessorCount; ++k) mask[k / 32] |= 1u << (k % 32);
    return hipExtStreamCreateWithCUMask(s, static_cast<uint32_t>(mask.size()), mask.data());
  }
  if (kind == 2) {
    int lo = 0, hi = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

std::unique_ptr<Ctx> take_ctx(int device) {
  DeviceCache& dc = (*g_cache)[device];
  {
    std::unique_lock<std::mutex> lk(dc.mu);
    if (!dc.primary_made) {   // the first context of the device: its NULL stream
      dc.primary_made = true;
      auto c = std::make_unique<Ctx>();
      c->device = device;
      c->null_stream = true;
      return c;
    }
    if (dc.primary) {
      // its second use: off the NULL stream, onto a non-blocking stream of its
      // own, keeping the tile orders the NULL stream's launches recorded (if
      // the stream cannot be made, the context stays on the NULL stream)
      std::unique_ptr<Ctx> c = std::move(dc.primary);
      lk.unlock();
      hipStream_t s = nullptr;
      if (hipSetDevice(device) == hipSuccess && make_stream(device, &s) == hipSuccess) {
        rebind_stream_schedules(nullptr, s, c->scenes.data(), static_cast<int>(c->scenes.size()));
        c->stream = s;
        c->null_stream = false;
      }
      return c;
    }
    if (!dc.free_ctx.empty()) {
      std::unique_ptr<Ctx> c = std::move(dc.free_ctx.back());
      dc.free_ctx.pop_back();
      return c;
    }
  }
  auto c = std::make_unique<Ctx>();
  c->device = device;
  return c;
}
void give_ctx(std::unique_ptr<Ctx> c) {
  DeviceCache& dc = (*g_cache)[c->device];
  std::lock_guard<std::mutex> lk(dc.mu);
  if (c->null_stream) dc.primary = std::move(c);
  else if (static_cast<int>(dc.free_ctx.size()) < kFreeCtx) dc.free_ctx.push_back(std::move(c));
}

struct Shard {
  int device = 0;
  rt_params p{};
  int rows = 0;
  int status = RT_OK;
  std::string err;
  uint64_t counters[2] = {0, 0};
  float ms = 0.0f, d2h_ms = 0.0f;
  // host clocks of the share, in order (rt_stats)
  double upload_ms = 0.0, setup_ms = 0.0, enqueue_ms = 0.0, wait_ms = 0.0, scatter_ms = 0.0, wall_ms = 0.0;
  double gather_ms = 0.0;   // d2h_ms (+ scatter_ms, 0: no host scatter)
  bool cached = false;
  // between start_shard and finish_shard: the share's context (its stream,
  // device buffers) and scene, held by the frame
  std::unique_ptr<Ctx> cx;
  std::shared_ptr<rt_dscene> ds;
  Clock::time_point t0;
  bool gathered = false;   // the D2H is already enqueued behind the launch
};

// The shard's compacted row tiles, D2H straight into their rows of out_rgb
// (measured on MI355X for a C1 frame: 0.46-0.52 ms, against 0.53-0.56 ms
// into pinned staging plus 0.34 ms of host copy, tools/d2h_bench.cpp).
// Several shards: tile k of the shard -> image tile shard_idx + k * nshards,
// through one strided copy, the image's last tile, if it is short, a second.
// Then the counters.  Enqueued on the context's stream.
hipError_t enqueue_gather(Shard* sh, void* out_rgb, bool u8, int rows_total, int ntiles, int nshards, int shard_idx) {
  Ctx* cx = sh->cx.get();
  const size_t nfl = static_cast<size_t>(sh->rows) * sh->p.width * 3;
  const void* src = u8 ? static_cast<const void*>(cx->d_u8) : static_cast<const void*>(cx->d_out);
  const size_t es = u8 ? 1 : sizeof(float);
  hipError_t e = hipSuccess;
  if (nfl) {
    if (nshards == 1) {
      e = hipMemcpyAsync(out_rgb, src, nfl * es, hipMemcpyDeviceToHost, cx->stream);
    } else {
      const int T = sh->p.row_tile;
      const size_t rowb = static_cast<size_t>(sh->p.width) * 3 * es;
      const int ntile = (ntiles - shard_idx + nshards - 1) / nshards;   // this shard's tiles
      const int t_last = shard_idx + (ntile - 1) * nshards;
      const bool short_last = t_last == ntiles - 1 && rows_total % T != 0;
      const int nfull = ntile - (short_last ? 1 : 0);
      if (nfull > 0)
        e = hipMemcpy2DAsync(reinterpret_cast<char*>(out_rgb) + static_cast<size_t>(shard_idx) * T * rowb,
                             static_cast<size_t>(nshards) * T * rowb, src, T * rowb, T * rowb, nfull,
                             hipMemcpyDeviceToHost, cx->stream);
      if (e == hipSuccess && short_last)
        e = hipMemcpyAsync(reinterpret_cast<char*>(out_rgb) + static_cast<size_t>(t_last) * T * rowb,
                           static_cast<const char*>(src) + static_cast<size_t>(nfull) * T * rowb,
                           static_cast<size_t>(rows_total - t_last * T) * rowb, hipMemcpyDeviceToHost, cx->stream);
    }
  }
  if (e == hipSuccess) e = hipMemcpyAsync(cx->h_cnt, cx->d_cnt, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, cx->stream);
  if (e == hipSuccess) e = hipEventRecord(cx->e2, cx->stream);
  return e;
}

// One device's share, first half: scene (cached), render context, launch
// (and the device quantiser for u8).  gather_now: the D2H into out_rgb is
// enqueued right behind the launch (rt_render); otherwise finish_shard does
// it once the device is done (rt_render_submit: a copy into pageable memory
// would hold the host until the kernel ends).  On failure sh->status is set
// and the context released.
void start_shard(const rt_scene* s, const rt_camera* c, Shard* sh, void* out_rgb, bool u8, bool gather_now,
                 int rows_total, int ntiles, int nshards, int shard_idx) {
  auto hip_fail = [&](hipError_t e, const char* what) {
    sh->status = RT_E_HIP;
    sh->err = std::string(what) + ": " + hipGetErrorString(e);
  };
  sh->t0 = Clock::now();
  int rc = RT_OK;
  // the scene: from the cache, or (a miss: upload and BVH builds, ~1-3 ms)
  // on a helper thread while this one sets up the render context, the other
  // one-time cost of a first call (stream, events, buffers)
  std::thread upload;
  std::string upload_err;   // (the error slot is per thread)
  if (!find_scene(sh->device, s, &sh->ds)) {
    upload = std::thread([&] {
      rc = get_scene(sh->device, s, &sh->ds, &sh->cached);
      if (rc != RT_OK) upload_err = rt_last_error();
    });
  } else {
    sh->cached = true;
  }
  const auto t_setup = Clock::now();
  sh->cx = take_ctx(sh->device);
  Ctx* cx = sh->cx.get();
  const size_t nfl = static_cast<size_t>(sh->rows) * sh->p.width * 3;
  hipError_t e = hipSetDevice(sh->device);
  if (e == hipSuccess && !cx->stream && !cx->null_stream) e = make_stream(sh->device, &cx->stream);
  if (e == hipSuccess && !cx->e0) e = hipEventCreate(&cx->e0);
  if (e == hipSuccess && !cx->e1) e = hipEventCreate(&cx->e1);
  if (e == hipSuccess && !cx->eg) e = hipEventCreate(&cx->eg);
  if (e == hipSuccess && !cx->e2) e = hipEventCreate(&cx->e2);
  if (e == hipSuccess && !cx->d_cnt) e = hipMalloc(&cx->d_cnt, 2 * sizeof(uint64_t));
  if (e == hipSuccess && !cx->h_cnt) e = hipHostMalloc(&cx->h_cnt, 2 * sizeof(uint64_t), hipHostMallocDefault);
  if (e == hipSuccess && cx->d_cap < nfl) {
    if (cx->d_out) (void)hipFree(cx->d_out);
    cx->d_out = nullptr;
    cx->d_cap = 0;
    e = hipMalloc(&cx->d_out, std::max<size_t>(nfl, 1) * sizeof(float));
    if (e == hipSuccess) cx->d_cap = nfl;
  }
  if (e == hipSuccess && u8 && cx->u8_cap < nfl) {
    if (cx->d_u8) (void)hipFree(cx->d_u8);
    cx->d_u8 = nullptr;
    cx->u8_cap = 0;
    e = hipMalloc(&cx->d_u8, std::max<size_t>(nfl, 1));
    if (e == hipSuccess) cx->u8_cap = nfl;
  }
  sh->setup_ms = ms_since(t_setup);
  // upload_ms: the part of the upload the call waited for after its set-up
  const auto t_up = Clock::now();
  if (upload.joinable()) upload.join();
  sh->upload_ms = ms_since(t_up);
  if (rc != RT_OK) {
    if (e == hipSuccess) give_ctx(std::move(sh->cx));
    sh->cx.reset();
    sh->status = rc;
    sh->err = upload_err;
    return;
  }
  const auto t_enq = Clock::now();
  if (e == hipSuccess) e = static_cast<hipError_t>(fill_async(cx->d_cnt, 0, 2 * sizeof(uint64_t), cx->stream));
  if (e == hipSuccess) e = hipEventRecord(cx->e0, cx->stream);
  if (e != hipSuccess) {
    hip_fail(e, "rt_render setup");
    return;
  }
  cx->launched(sh->ds.get());   // (before the launch: it may have made the stream's entry and then failed)
  rc = rt_launch(sh->ds.get(), c, &sh->p, cx->d_out, cx->d_cnt, cx->stream);
  if (rc != RT_OK) {
    sh->status = rc;
    sh->err = rt_last_error();
    return;
  }
  e = hipEventRecord(cx->e1, cx->stream);
  // (u8: the quantiser's few microseconds fall in d2h_ms when the copy
  // follows at once)
  if (e == hipSuccess && gather_now) e = hipEventRecord(cx->eg, cx->stream);
  if (e == hipSuccess && u8 && nfl) e = static_cast<hipError_t>(quantize_launch(cx->d_out, cx->d_u8, nfl, cx->stream));
  if (e == hipSuccess && gather_now) {
    e = enqueue_gather(sh, out_rgb, u8, rows_total, ntiles, nshards, shard_idx);
    sh->gathered = true;
  }
  sh->enqueue_ms = ms_since(t_enq);
  if (e != hipSuccess) hip_fail(e, "rt_render launch/gather");
}

// Second half: wait for the device (and the D2H, enqueued here if it was
// not), the share's counters and event times; the context goes back to the
// device's pool (a failed one is dropped: its stream may hold a fault).
void finish_shard(Shard* sh, void* out_rgb, bool u8, int rows_total, int ntiles, int nshards, int shard_idx) {
  Ctx* cx = sh->cx.get();
  if (sh->status == RT_OK && cx) {
    const auto t_wait = Clock::now();
    hipError_t e = hipSetDevice(sh->device);
    if (e == hipSuccess && !sh->gathered) e = hipStreamSynchronize(cx->stream);
    // (a submitted frame's copy starts now: d2h_ms times it from here, not
    // from the kernel's end, which the caller's rt_render_wait may be long after)
    if (e == hipSuccess && !sh->gathered) e = hipEventRecord(cx->eg, cx->stream);
    if (e == hipSuccess && !sh->gathered) e = enqueue_gather(sh, out_rgb, u8, rows_total, ntiles, nshards, shard_idx);
    if (e == hipSuccess) e = hipStreamSynchronize(cx->stream);
    sh->wait_ms = ms_since(t_wait);
    float d2h = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&sh->ms, cx->e0, cx->e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&d2h, cx->eg, cx->e2);
    sh->d2h_ms = d2h;
    if (e != hipSuccess) {
      sh->status = RT_E_HIP;
      sh->err = std::string("rt_render trace/gather: ") + hipGetErrorString(e);
    } else {
      sh->counters[0] = cx->h_cnt[0];
      sh->counters[1] = cx->h_cnt[1];
      sh->scatter_ms = 0.0;   // (no host scatter: the copies place the rows)
      sh->gather_ms = d2h;
    }
  } else if (cx) {
    // a failed start: wait for whatever it enqueued before the context is dropped
    (void)hipSetDevice(sh->device);
    (void)hipStreamSynchronize(cx->stream);
  }
  sh->wall_ms = ms_since(sh->t0);
  if (sh->status == RT_OK && sh->cx) give_ctx(std::move(sh->cx));
  sh->cx.reset();
  sh->ds.reset();
}

}  // namespace

extern "C" int rt_cache_clear(void) {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  int dropped = 0;
  for (DeviceCache& dc : *g_cache) {
    std::vector<CachedScene> scenes;
    std::vector<std::unique_ptr<Ctx>> ctxs;
    {
      std::lock_guard<std::mutex> l2(dc.mu);
      scenes.swap(dc.scenes);
      ctxs.swap(dc.free_ctx);
      if (dc.primary) {   // (one in use stays; it is dropped at a later clear)
        ctxs.push_back(std::move(dc.primary));
        dc.primary_made = false;
      }
    }
    dropped += static_cast<int>(scenes.size());
  }
  return dropped;
}

// A frame in flight (rt_render, or rt_render_submit .. rt_render_wait): its
// shards, each holding its device's render context until it finishes.
struct rt_frame {
  std::vector<Shard> shards;
  void* out = nullptr;
  bool u8 = false;
  int rows = 0, ntiles = 0;
  Clock::time_point t0;
};

namespace {
// The shards of a frame (argument checks as rt_render documents them).
int plan_frame(const rt_scene* s, const rt_camera* c, const rt_params* p, void* out_rgb, bool u8, size_t out_len,
               const char* who, rt_frame* f) {
  const std::string w(who);
  if (!s || !c || !p || !out_rgb) return set_error(RT_E_ARG, w + ": NULL argument");
  const bool on_dev0 = (p->flags & RT_FLAG_SHARDS_ON_DEVICE0) != 0;
  if (p->width <= 0 || p->height <= 0 || p->spp < 0 || p->spp > RT_MAX_SPP || p->n_devices < 0 ||
      (p->flags & ~(RT_FLAG_SHARDS_ON_DEVICE0 | RT_FLAG_REALM | RT_FLAG_REJECTION_SAMPLERS)) != 0 ||
      (on_dev0 && p->n_devices == 0))
    return set_error(RT_E_ARG, w + ": bad width/height/spp/flags/n_devices");
  if (p->tile_step != 0 || p->tile_first != 0)
    return set_error(RT_E_ARG, w + ": tile_first/tile_step are per-shard (rt_launch) fields");
  if (s->n < 0 || (s->n > 0 && (!s->sphere || !s->mat_kind || !s->mat)))
    return set_error(RT_E_ARG, w + ": bad scene arrays");
  const int rows = rows_out(*p);
  if (rows < 0) return set_error(RT_E_ARG, w + ": bad row range");
  const size_t need = static_cast<size_t>(rows) * p->width * 3;
  if (out_len < need)
    return set_error(RT_E_ARG, w + ": out_len " + std::to_string(out_len) + " < " + std::to_string(need));
  const int ndev_vis = rt_device_count();
  if (ndev_vis <= 0) return set_error(RT_E_NODEV, w + ": no GPU visible");
  int ndev = p->n_devices == 0 ? ndev_vis : p->n_devices;
  if (ndev > ndev_vis && !on_dev0)
    return set_error(RT_E_NODEV, w + ": n_devices " + std::to_string(ndev) + " > visible " + std::to_string(ndev_vis));
  if (ndev_vis > static_cast<int>(g_cache->size())) return set_error(RT_E_NODEV, w + ": more than 64 devices");
  const int T = p->row_tile > 0 ? p->row_tile : 8;
  const int ntiles = (rows + T - 1) / T;
  ndev = std::max(1, std::min(ndev, std::max(ntiles, 1)));
  f->shards = std::vector<Shard>(ndev);
  for (int d = 0; d < ndev; ++d) {
    Shard& sh = f->shards[d];
    sh.device = on_dev0 ? 0 : d;
    sh.p = *p;
    sh.p.flags = p->flags & (RT_FLAG_REALM | RT_FLAG_REJECTION_SAMPLERS);   // semantics travel; the fan-out flag is rt_render's
    sh.p.row_tile = T;
    if (ndev > 1) {
      sh.p.tile_first = d;
      sh.p.tile_step = ndev;
    }
    sh.rows = rows_out(sh.p);
  }
  f->out = out_rgb;
  f->u8 = u8;
  f->rows = rows;
  f->ntiles = ntiles;
  return RT_OK;
}

// run fn(d) for every shard: the first on this thread, the others on the pool
template <class F>
void for_shards(rt_frame* f, F fn) {
  const int n = static_cast<int>(f->shards.size());
  if (n == 1) {
    fn(0);
    return;
  }
  std::vector<std::function<void()>> tasks;
  for (int d = 0; d < n; ++d) tasks.emplace_back([&fn, d] { fn(d); });
  g_pool->run(tasks);
}

// the frame's statistics and status once every shard has finished
int frame_result(rt_frame* f, rt_stats* stats) {
  const int ndev = static_cast<int>(f->shards.size());
  double kms = 0, ksum = 0, ums = 0, gms = 0, d2h = 0;
  uint64_t segs = 0, smp = 0;
  int cached = 0, slowest = 0;
  for (int d = 0; d < ndev; ++d) {
    Shard& sh = f->shards[d];
    if (sh.status != RT_OK) return set_error(sh.status, "device " + std::to_string(d) + ": " + sh.err);
    if (sh.wall_ms > f->shards[slowest].wall_ms) slowest = d;
    d2h = std::max(d2h, static_cast<double>(sh.d2h_ms));
    kms = std::max(kms, static_cast<double>(sh.ms));
    ksum += sh.ms;
    ums = std::max(ums, sh.upload_ms);
    gms = std::max(gms, sh.gather_ms);
    cached += sh.cached ? 1 : 0;
    segs += sh.counters[0];
    smp += sh.counters[1];
  }
  if (stats) {
    stats->segments = segs;
    stats->samples = smp;
    stats->kernel_ms = kms;
    stats->kernel_ms_mean = ksum / ndev;
    stats->upload_ms = ums;
    stats->gather_ms = gms;
    stats->scene_cached = cached;
    stats->n_devices = ndev;
    const Shard& sl = f->shards[slowest];
    stats->setup_ms = sl.setup_ms;
    stats->enqueue_ms = sl.enqueue_ms;
    stats->wait_ms = sl.wait_ms;
    stats->scatter_ms = sl.scatter_ms;
    stats->d2h_ms = d2h;
    stats->total_ms = ms_since(f->t0);
    stats->other_ms = stats->total_ms - (sl.upload_ms + sl.setup_ms + sl.enqueue_ms + sl.wait_ms + sl.scatter_ms);
  }
  return RT_OK;
}

// rt_render and rt_render_u8: out_rgb holds floats or (u8) bytes; each
// device's share starts, gathers and finishes on its own host worker
int render(const rt_scene* s, const rt_camera* c, const rt_params* p, void* out_rgb, bool u8, size_t out_len,
           rt_stats* stats) {
  clear_error();
  rt_frame f;
  f.t0 = Clock::now();
  const int rc = plan_frame(s, c, p, out_rgb, u8, out_len, "rt_render", &f);
  if (rc != RT_OK) return rc;
  const int n = static_cast<int>(f.shards.size());
  for_shards(&f, [&](int d) {
    start_shard(s, c, &f.shards[d], out_rgb, u8, true, f.rows, f.ntiles, n, d);
    finish_shard(&f.shards[d], out_rgb, u8, f.rows, f.ntiles, n, d);
  });
  return frame_result(&f, stats);
}
}  // namespace

extern "C" int rt_render(const rt_scene* s, const rt_camera* c, const rt_params* p, float* out_rgb,
                         size_t out_len, rt_stats* stats) {
  return render(s, c, p, out_rgb, false, out_len, stats);
}

extern "C" int rt_render_u8(const rt_scene* s, const rt_camera* c, const rt_params* p, uint8_t* out_rgb8,
                            size_t out_len, rt_stats* stats) {
  return render(s, c, p, out_rgb8, true, out_len, stats);
}

namespace {
int submit(const rt_scene* s, const rt_camera* c, const rt_params* p, void* out_rgb, bool u8, size_t out_len,
           rt_frame** frame) {
  clear_error();
  if (!frame) return set_error(RT_E_ARG, "rt_render_submit: NULL frame");
  *frame = nullptr;
  auto f = std::make_unique<rt_frame>();
  f->t0 = Clock::now();
  const int rc = plan_frame(s, c, p, out_rgb, u8, out_len, "rt_render_submit", f.get());
  if (rc != RT_OK) return rc;
  const int n = static_cast<int>(f->shards.size());
  // frames in flight: two rounds of split units per launch (RT_FLAG_STREAMED)
  for (Shard& sh : f->shards) sh.p.flags |= RT_FLAG_STREAMED;
  rt_frame* fp = f.get();
  for_shards(fp, [&](int d) { start_shard(s, c, &fp->shards[d], out_rgb, u8, false, fp->rows, fp->ntiles, n, d); });
  for (int d = 0; d < n; ++d)
    if (fp->shards[d].status != RT_OK) {   // undo: wait for what did start, drop the frame
      const std::string err = "device " + std::to_string(d) + ": " + fp->shards[d].err;
      const int code = fp->shards[d].status;
      for_shards(fp, [&](int k) { finish_shard(&fp->shards[k], out_rgb, u8, fp->rows, fp->ntiles, n, k); });
      return set_error(code, err);
    }
  *frame = f.release();
  return RT_OK;
}
}  // namespace

extern "C" int rt_render_submit(const rt_scene* s, const rt_camera* c, const rt_params* p, float* out_rgb,
                                size_t out_len, rt_frame** frame) {
  return submit(s, c, p, out_rgb, false, out_len, frame);
}

extern "C" int rt_render_submit_u8(const rt_scene* s, const rt_camera* c, const rt_params* p, uint8_t* out_rgb8,
                                   size_t out_len, rt_frame** frame) {
  return submit(s, c, p, out_rgb8, true, out_len, frame);
}

extern "C" int rt_render_wait(rt_frame* frame, rt_stats* stats) {
  clear_error();
  if (!frame) return set_error(RT_E_ARG, "rt_render_wait: NULL frame");
  std::unique_ptr<rt_frame> f(frame);
  const int n = static_cast<int>(f->shards.size());
  rt_frame* fp = f.get();
  for_shards(fp, [&](int d) { finish_shard(&fp->shards[d], fp->out, fp->u8, fp->rows, fp->ntiles, n, d); });
  return frame_result(fp, stats);
}

extern "C" int rt_quantize_device(const float* d_lin, uint8_t* d_out, size_t n, void* hip_stream) {
  clear_error();
  if ((!d_lin || !d_out) && n) return set_error(RT_E_ARG, "rt_quantize_device: NULL argument");
  if (n == 0) return RT_OK;
  const hipError_t e = static_cast<hipError_t>(quantize_launch(d_lin, d_out, n, hip_stream));
  if (e != hipSuccess) return set_error(RT_E_HIP, std::string("rt_quantize_device: ") + hipGetErrorString(e));
  return RT_OK;
}
