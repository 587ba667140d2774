// rt_host.cpp — host side of the C ABI: camera set-up, quantise/PPM, error
// slot, and the multi-GPU fan-out of rt_render (one host thread per device,
// interleaved row tiles, host-side gather; no collectives).
//
// Reference anchors:
//   camera       src/raytracing.clj:105-139 (deg->rad :60-61)
//   write-color! src/raytracing.clj:19-26, PPM :172-175
//   executor     src/raytracing.clj:157-171 (2 threads, contiguous chunks —
//                here: N devices, interleaved 8-row tiles for balance)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
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

extern "C" int rt_quantize(const float* lin, uint8_t* out, size_t n) {
  clear_error();
  if ((!lin || !out) && n) return set_error(RT_E_ARG, "rt_quantize: NULL argument");
  for (size_t i = 0; i < n; ++i) {
    const double c = lin[i];
    const double g = c > 0 ? std::sqrt(c) : 0.0;              // linear->gamma (:21-22)
    const double cl = std::min(0.999, std::max(g, 0.0));      // clamp (:19), NaN -> 0 below
    const int q = static_cast<int>(256 * cl);                 // (int (* 256 ...)) (:25)
    out[i] = static_cast<uint8_t>(std::isnan(c) ? 0 : q);
  }
  return RT_OK;
}

extern "C" int rt_write_ppm(const char* path, const uint8_t* rgb, int width, int height) {
  clear_error();
  if (!path || !rgb || width <= 0 || height <= 0) return set_error(RT_E_ARG, "rt_write_ppm: bad argument");
  FILE* f = std::fopen(path, "wb");
  if (!f) return set_error(RT_E_IO, std::string("rt_write_ppm: cannot open ") + path);
  std::string buf;
  buf.reserve(static_cast<size_t>(width) * height * 12 + 32);
  buf += "P3\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
  char line[16];
  const size_t npx = static_cast<size_t>(width) * height;
  for (size_t i = 0; i < npx; ++i) {
    const int len = std::snprintf(line, sizeof line, "%d %d %d\n", rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
    buf.append(line, len);
  }
  const bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
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

extern "C" const char* rt_version(void) { return "rtclj-mi355x 0.1 (gfx950)"; }

namespace {

struct Shard {
  int device = 0;
  rt_params p{};
  int rows = 0;
  std::vector<float> host;
  int status = RT_OK;
  std::string err;
  uint64_t counters[2] = {0, 0};
  float ms = 0.0f;
};

void run_shard(const rt_scene* s, const rt_camera* c, Shard* sh) {
  auto fail = [&](int code) {
    sh->status = code;
    sh->err = rt_last_error();
  };
  auto hip_fail = [&](hipError_t e, const char* what) {
    sh->status = RT_E_HIP;
    sh->err = std::string(what) + ": " + hipGetErrorString(e);
  };
  rt_dscene* ds = nullptr;
  int rc = rt_scene_upload(sh->device, s, &ds);
  if (rc != RT_OK) return fail(rc);
  float* d_out = nullptr;
  uint64_t* d_cnt = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const size_t nfl = static_cast<size_t>(sh->rows) * sh->p.width * 3;
  hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&d_out, std::max<size_t>(nfl, 1) * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&d_cnt, 2 * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMemsetAsync(d_cnt, 0, 2 * sizeof(uint64_t), stream);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipEventRecord(e0, stream);
  if (e != hipSuccess) {
    hip_fail(e, "rt_render setup");
  } else {
    rc = rt_launch(ds, c, &sh->p, d_out, d_cnt, stream);
    if (rc != RT_OK) {
      fail(rc);
    } else {
      e = hipEventRecord(e1, stream);
      sh->host.resize(nfl);
      if (e == hipSuccess && nfl)
        e = hipMemcpyAsync(sh->host.data(), d_out, nfl * sizeof(float), hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess)
        e = hipMemcpyAsync(sh->counters, d_cnt, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e == hipSuccess) e = hipEventElapsedTime(&sh->ms, e0, e1);
      if (e != hipSuccess) hip_fail(e, "rt_render trace/gather");
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (d_out) (void)hipFree(d_out);
  if (d_cnt) (void)hipFree(d_cnt);
  if (stream) (void)hipStreamDestroy(stream);
  rt_scene_free(ds);
}

}  // namespace

extern "C" int rt_render(const rt_scene* s, const rt_camera* c, const rt_params* p, float* out_rgb,
                         size_t out_len, rt_stats* stats) {
  clear_error();
  const auto t0 = std::chrono::steady_clock::now();
  if (!s || !c || !p || !out_rgb) return set_error(RT_E_ARG, "rt_render: NULL argument");
  const bool on_dev0 = (p->flags & RT_FLAG_SHARDS_ON_DEVICE0) != 0;
  if (p->width <= 0 || p->height <= 0 || p->spp < 0 || p->n_devices < 0 ||
      (p->flags & ~(RT_FLAG_SHARDS_ON_DEVICE0 | RT_FLAG_REALM)) != 0 || (on_dev0 && p->n_devices == 0))
    return set_error(RT_E_ARG, "rt_render: bad width/height/spp/flags/n_devices");
  if (p->tile_step != 0 || p->tile_first != 0)
    return set_error(RT_E_ARG, "rt_render: tile_first/tile_step are per-shard (rt_launch) fields");
  const int rows = rows_out(*p);
  if (rows < 0) return set_error(RT_E_ARG, "rt_render: bad row range");
  const size_t need = static_cast<size_t>(rows) * p->width * 3;
  if (out_len < need)
    return set_error(RT_E_ARG, "rt_render: out_len " + std::to_string(out_len) + " < " + std::to_string(need));
  const int ndev_vis = rt_device_count();
  if (ndev_vis <= 0) return set_error(RT_E_NODEV, "rt_render: no GPU visible");
  int ndev = p->n_devices == 0 ? ndev_vis : p->n_devices;
  if (ndev > ndev_vis && !on_dev0)
    return set_error(RT_E_NODEV, "rt_render: n_devices " + std::to_string(ndev) + " > visible " +
                                     std::to_string(ndev_vis));
  const int T = p->row_tile > 0 ? p->row_tile : 8;
  const int ntiles = (rows + T - 1) / T;
  ndev = std::max(1, std::min(ndev, ntiles));

  std::vector<Shard> shards(ndev);
  for (int d = 0; d < ndev; ++d) {
    Shard& sh = shards[d];
    sh.device = on_dev0 ? 0 : d;
    sh.p = *p;
    sh.p.flags = p->flags & RT_FLAG_REALM;   // semantics travel; the fan-out flag is rt_render's
    sh.p.row_tile = T;
    if (ndev > 1) {
      sh.p.tile_first = d;
      sh.p.tile_step = ndev;
    }
    sh.rows = rows_out(sh.p);
  }
  if (ndev == 1) {
    run_shard(s, c, &shards[0]);
  } else {
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; ++d) th.emplace_back(run_shard, s, c, &shards[d]);
    for (auto& t : th) t.join();
  }
  double kms = 0;
  uint64_t segs = 0, smp = 0;
  for (int d = 0; d < ndev; ++d) {
    Shard& sh = shards[d];
    if (sh.status != RT_OK) return set_error(sh.status, "device " + std::to_string(d) + ": " + sh.err);
    // host-side gather: compacted tiles back to their image rows
    const size_t rowf = static_cast<size_t>(p->width) * 3;
    if (ndev == 1) {
      std::memcpy(out_rgb, sh.host.data(), sh.host.size() * sizeof(float));
    } else {
      int ro = 0;
      for (int t = d; t < ntiles; t += ndev) {
        const int r0 = t * T, nr = std::min(T, rows - r0);
        std::memcpy(out_rgb + static_cast<size_t>(r0) * rowf, sh.host.data() + static_cast<size_t>(ro) * rowf,
                    nr * rowf * sizeof(float));
        ro += nr;
      }
    }
    kms = std::max(kms, static_cast<double>(sh.ms));
    segs += sh.counters[0];
    smp += sh.counters[1];
  }
  if (stats) {
    stats->segments = segs;
    stats->samples = smp;
    stats->kernel_ms = kms;
    stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->n_devices = ndev;
  }
  return RT_OK;
}
