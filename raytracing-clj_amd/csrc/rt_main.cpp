// rt_main — C++ host driver mirroring `clojure -M:main [spp] [depth]`
// (src/raytracing.clj:95-177): prints the config, renders the reference's
// five-body scene at 400x225 through rt_render, writes scene.ppm.
//
//   rt_main [spp] [depth] [--scene reference|cover] [--width W] [--seed S]
//           [--gpus N] [--out PATH]
// Defaults follow the reference: spp 100, depth 50, width 400, 16:9.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt.h"

int main(int argc, char** argv) {
  int spp = 100, depth = 50, width = 400, gpus = 0, grid = 11;
  unsigned long long seed = 1;
  std::string scene = "reference", out = "scene.ppm";
  int pos = 0;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--scene") scene = val();
    else if (a == "--width") width = std::atoi(val());
    else if (a == "--seed") seed = std::strtoull(val(), nullptr, 10);
    else if (a == "--gpus") gpus = std::atoi(val());
    else if (a == "--grid") grid = std::atoi(val());
    else if (a == "--out") out = val();
    else if (pos == 0) spp = std::atoi(argv[i]), ++pos;   // (:96)
    else if (pos == 1) depth = std::atoi(argv[i]), ++pos; // (:97)
  }
  std::printf("config: {:samples-per-px %d, :max-depth %d}\n", spp, depth);  // (:98)
  const int height = width * 9 / 16;  // (int (/ image-width 16/9)) (:105-107)
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
    rt_camera_setup(width, height, 20.0, lf, la, up, 10.0, 3.4, &cam);
  }
  rt_scene s{n, sph.data(), kind.data(), mat.data()};
  rt_params p{};
  p.width = width;
  p.height = height;
  p.row_begin = 0;
  p.row_end = height;
  p.spp = spp;
  p.max_depth = depth;
  p.seed = seed;
  p.n_devices = gpus;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<float> lin(static_cast<size_t>(width) * height * 3);
  rt_stats st{};
  if (rt_render(&s, &cam, &p, lin.data(), lin.size(), &st) != RT_OK) {
    std::fprintf(stderr, "rt_render failed: %s\n", rt_last_error());
    return 1;
  }
  std::vector<uint8_t> q(lin.size());
  rt_quantize(lin.data(), q.data(), q.size());
  if (rt_write_ppm(out.c_str(), q.data(), width, height) != RT_OK) {
    std::fprintf(stderr, "%s\n", rt_last_error());
    return 1;
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf("\"Elapsed time: %.3f msecs\"\n", ms);  // (time ...) (:99)
  std::printf("bodies %d, devices %d, kernel %.3f ms, %.1f Msamples/s, %.3f segments/sample\n", n,
              st.n_devices, st.kernel_ms, st.samples / (st.kernel_ms * 1e3),
              st.samples ? double(st.segments) / st.samples : 0.0);
  return 0;
}
