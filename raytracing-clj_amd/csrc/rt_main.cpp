// rt_main — C++ host driver mirroring `clojure -M:main [spp] [depth]`
// (src/raytracing.clj:95-177): prints the config, renders the reference's
// five-body scene at 400x225 through rt_render, writes scene.ppm.
// --realm mirrors `clojure -M:realm` (src/realm/raytracing.clj:279-359)
// instead: realm's body order, camera (no defocus, focal length
// |look-from - look-at|), height (int (/ ^double 400 ^double 16/9)) = 224 and
// RT_FLAG_REALM semantics; it writes scene-realm.ppm.  Like the reference's
// -main, whose (time ...) ends with (ppm->png "scene.ppm" "scene.png")
// (raytracing.clj:176), it then converts the PPM it wrote to a PNG beside it
// (rt_ppm_to_png; --png PATH names it, --no-png skips it), inside the timing.  The frame
// is quantised on the device (rt_render_u8: a quarter of the copy back, no
// host pass); --host-quantize takes rt_render's floats and rt_quantize
// instead (the same bytes).
//
//   rt_main [spp] [depth] [--scene reference|cover] [--realm] [--width W]
//           [--seed S] [--gpus N] [--out PATH] [--png PATH] [--no-png] [--json]
//           [--host-quantize] [--rejection-samplers]
// Defaults follow the reference: spp 100, depth 50, width 400, 16:9.
// --json: one more line, a JSON object of where this one-frame process's time
// went (the device start-up -- the HIP runtime's first rt_device_count, then
// rt_prepare's context / code object / queue / pageable staging -- on a thread
// beside the scene set-up, what the main thread waited for it; rt_render's
// rt_stats parts; quantise and file writes) -- bench.py's first_process.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <iterator>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/rt.h"

int main(int argc, char** argv) {
  int spp = 100, depth = 50, width = 400, gpus = 0, grid = 11;
  unsigned long long seed = 1;
  std::string scene = "reference", out, png;
  bool realm = false, json = false, host_quantize = false, no_png = false, rejection = false;
  int pos = 0;
  const auto t_start = std::chrono::steady_clock::now();
  auto ms_since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  // The one-time device start-up first, on its own thread, while this one
  // parses the arguments and builds the scene: the HIP runtime (the first
  // rt_device_count), then per device its context, code object, queue and
  // pageable-copy staging (rt_prepare).
  int ndev = 0;
  double device_count_ms = 0.0, prep_ms[4] = {0, 0, 0, 0};
  int gpus_arg = 0;
  // (a missing option value ends the process before the start-up thread
  // exists: no exit while that thread may be inside the HIP runtime)
  static const char* const kValued[] = {"--scene", "--width", "--seed", "--gpus", "--grid", "--out", "--png"};
  for (int i = 1; i < argc; ++i) {
    const bool valued = std::any_of(std::begin(kValued), std::end(kValued),
                                    [&](const char* f) { return std::strcmp(argv[i], f) == 0; });
    if (!valued) continue;
    if (i + 1 >= argc) {
      std::fprintf(stderr, "missing value for %s\n", argv[i]);
      return 2;
    }
    if (std::strcmp(argv[i], "--gpus") == 0) gpus_arg = std::atoi(argv[i + 1]);
    ++i;
  }
  std::thread prep([&] {
    const auto t = std::chrono::steady_clock::now();
    ndev = rt_device_count();   // the process's first HIP call: runtime start-up
    device_count_ms = ms_since(t);
    const int use = gpus_arg > 0 ? std::min(gpus_arg, ndev) : ndev;
    std::vector<std::thread> per;
    std::vector<std::vector<double>> parts(use, std::vector<double>(4, 0.0));
    for (int d = 0; d < use; ++d) per.emplace_back([&, d] { rt_prepare(d, parts[d].data()); });
    for (auto& x : per) x.join();
    for (int d = 0; d < use; ++d)
      for (int k = 0; k < 4; ++k) prep_ms[k] = std::max(prep_ms[k], parts[d][k]);
  });
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> const char* { return argv[++i]; };   // (present: checked above)
    if (a == "--scene") scene = val();
    else if (a == "--width") width = std::atoi(val());
    else if (a == "--seed") seed = std::strtoull(val(), nullptr, 10);
    else if (a == "--gpus") gpus = std::atoi(val());
    else if (a == "--grid") grid = std::atoi(val());
    else if (a == "--out") out = val();
    else if (a == "--png") png = val();
    else if (a == "--realm") realm = true;
    else if (a == "--rejection-samplers") rejection = true;   // RT_FLAG_REJECTION_SAMPLERS
    else if (a == "--json") json = true;
    else if (a == "--no-png") no_png = true;
    else if (a == "--host-quantize") host_quantize = true;
    else if (pos == 0) spp = std::atoi(argv[i]), ++pos;   // (:96)
    else if (pos == 1) depth = std::atoi(argv[i]), ++pos; // (:97)
  }
  if (out.empty()) out = realm ? "scene-realm.ppm" : "scene.ppm";
  if (png.empty() && !no_png) {   // scene.ppm -> scene.png (raytracing.clj:176)
    png = out;
    const size_t dot = png.rfind(".ppm");
    if (dot != std::string::npos && dot + 4 == png.size()) png.resize(dot);
    png += ".png";
  }
  if (no_png) png.clear();
  if (!realm) std::printf("config: {:samples-per-px %d, :max-depth %d}\n", spp, depth);  // (:98)
  // -main: (int (/ image-width 16/9)) in exact ratios (:105-107); realm: a
  // double division by Ratio.doubleValue(16/9) = 1.777777777777778
  // (realm/raytracing.clj:20-22), 400 -> 224
  const int height = realm ? static_cast<int>(width / 1.777777777777778) : width * 9 / 16;
  const int cap = RT_MAX_SPHERES;
  std::vector<float> sph(4 * cap), mat(4 * cap);
  std::vector<int> kind(cap);
  rt_camera cam{};
  int n = 0;
  if (scene == "cover") {
    n = rt_scene_cover(grid, 42, sph.data(), kind.data(), mat.data(), cap);
    const double lf[3] = {13, 2, 3}, la[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    rt_camera_setup(width, height, 20.0, lf, la, up, 0.6, 10.0, &cam);
  } else {
    n = rt_scene_reference(sph.data(), kind.data(), mat.data(), cap);
    const double lf[3] = {-2, 2, 1}, la[3] = {0, 0, -1}, up[3] = {0, 1, 0};  // (:110-115)
    if (realm) {
      // realm/raytracing.clj:307-317 lists the centre sphere before the ground
      for (int k = 0; k < 4; ++k) {
        std::swap(sph[k], sph[4 + k]);
        std::swap(mat[k], mat[4 + k]);
      }
      std::swap(kind[0], kind[1]);
      const double fl = std::sqrt(4.0 + 4.0 + 4.0);   // |look-from - look-at| (:291-292)
      rt_camera_setup(width, height, 20.0, lf, la, up, 0.0, fl, &cam);
    } else {
      rt_camera_setup(width, height, 20.0, lf, la, up, 10.0, 3.4, &cam);
    }
  }
  rt_scene s{n, sph.data(), kind.data(), mat.data()};
  const double scene_ms = ms_since(t_start);
  prep.join();   // (the device start-up ran beside the argument parsing and the scene)
  const double prep_wait_ms = ms_since(t_start) - scene_ms;
  rt_params p{};
  p.width = width;
  p.height = height;
  p.row_begin = 0;
  p.row_end = height;
  p.spp = spp;
  p.max_depth = depth;
  p.seed = seed;
  p.n_devices = gpus;
  p.flags = (realm ? RT_FLAG_REALM : 0) | (rejection ? RT_FLAG_REJECTION_SAMPLERS : 0);
  const auto t0 = std::chrono::steady_clock::now();
  const size_t nch = static_cast<size_t>(width) * height * 3;
  std::vector<uint8_t> q(nch);
  rt_stats st{};
  double render_ms = 0.0, quantize_ms = 0.0;
  if (host_quantize) {
    std::vector<float> lin(nch);
    if (rt_render(&s, &cam, &p, lin.data(), lin.size(), &st) != RT_OK) {
      std::fprintf(stderr, "rt_render failed: %s\n", rt_last_error());
      return 1;
    }
    render_ms = ms_since(t0);
    const auto t_q = std::chrono::steady_clock::now();
    rt_quantize(lin.data(), q.data(), q.size());
    quantize_ms = ms_since(t_q);
  } else {
    if (rt_render_u8(&s, &cam, &p, q.data(), q.size(), &st) != RT_OK) {
      std::fprintf(stderr, "rt_render_u8 failed: %s\n", rt_last_error());
      return 1;
    }
    render_ms = ms_since(t0);
  }
  const auto t_w = std::chrono::steady_clock::now();
  if (rt_write_ppm(out.c_str(), q.data(), width, height) != RT_OK) {
    std::fprintf(stderr, "%s\n", rt_last_error());
    return 1;
  }
  const double write_ms = ms_since(t_w);
  // (ppm->png "scene.ppm" "scene.png"): the reference reads the PPM it wrote
  // back and encodes it (ppm2png.clj:35-87); so does this, inside the timing
  const auto t_p = std::chrono::steady_clock::now();
  if (!png.empty() && rt_ppm_to_png(out.c_str(), png.c_str()) != RT_OK) {
    std::fprintf(stderr, "%s\n", rt_last_error());
    return 1;
  }
  const double png_ms = png.empty() ? 0.0 : ms_since(t_p);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf("\"Elapsed time: %.3f msecs\"\n", ms);  // (time ...) (:99)
  std::printf("bodies %d, devices %d, kernel %.3f ms, %.1f Msamples/s, %.3f segments/sample\n", n,
              st.n_devices, st.kernel_ms, st.samples / (st.kernel_ms * 1e3),
              st.samples ? double(st.segments) / st.samples : 0.0);
  if (json)
    std::printf(
        "{\"devices_visible\": %d, \"scene_ms\": %.3f, \"device_count_ms\": %.3f, \"prepare_ms\": {\"context\": %.3f, "
        "\"code_object\": %.3f, \"queue\": %.3f, \"pageable_staging\": %.3f}, \"prepare_wait_ms\": %.3f, "
        "\"render_ms\": %.3f, \"quantize\": \"%s\", "
        "\"quantize_ms\": %.3f, \"write_ms\": %.3f, \"png_ms\": %.3f, \"process_ms\": %.3f, \"rt_stats\": {\"total_ms\": %.3f, "
        "\"upload_ms\": %.3f, \"setup_ms\": %.3f, \"enqueue_ms\": %.3f, \"wait_ms\": %.3f, \"scatter_ms\": %.3f, "
        "\"other_ms\": %.3f, \"kernel_ms\": %.3f, \"d2h_ms\": %.3f, \"segments\": %llu, \"samples\": %llu, "
        "\"n_devices\": %d}}\n",
        ndev, scene_ms, device_count_ms, prep_ms[0], prep_ms[1], prep_ms[2], prep_ms[3], prep_wait_ms, render_ms,
        host_quantize ? "host" : "device", quantize_ms, write_ms, png_ms, ms_since(t_start), st.total_ms,
        st.upload_ms, st.setup_ms, st.enqueue_ms, st.wait_ms, st.scatter_ms, st.other_ms, st.kernel_ms, st.d2h_ms,
        static_cast<unsigned long long>(st.segments), static_cast<unsigned long long>(st.samples), st.n_devices);
  return 0;
}
