// scenes.cpp — host-side scene builders exported through rt.h.
//   rt_scene_reference: the reference's `hittables` (src/raytracing.clj:63-78)
//   rt_scene_cover:     RTIOW §14 cover scene (not in the reference; the
//                       benchmark workload named by BASELINE.json configs[1])
#include <cmath>
#include <cstdint>
#include <vector>

#include "rt_internal.h"

namespace {

struct Body {
  float c[3], r;
  int kind;
  float m[4];
};

int emit(const std::vector<Body>& b, float* sphere, int* kind, float* mat, int cap) {
  const int n = static_cast<int>(b.size());
  if (!sphere || !kind || !mat || cap < n) return n;
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) sphere[4 * i + k] = b[i].c[k];
    sphere[4 * i + 3] = b[i].r;
    kind[i] = b[i].kind;
    for (int k = 0; k < 4; ++k) mat[4 * i + k] = b[i].m[k];
  }
  return n;
}

struct SplitMix64 {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  double unit() { return static_cast<double>(next() >> 11) * 0x1p-53; }        // [0,1)
  double range(double lo, double hi) { return lo + (hi - lo) * unit(); }
};

Body lam(double x, double y, double z, double r, double a, double b, double c) {
  return Body{{float(x), float(y), float(z)}, float(r), RT_LAMBERTIAN, {float(a), float(b), float(c), 0.0f}};
}
Body met(double x, double y, double z, double r, double a, double b, double c, double fuzz) {
  return Body{{float(x), float(y), float(z)}, float(r), RT_METAL, {float(a), float(b), float(c), float(fuzz)}};
}
Body die(double x, double y, double z, double r, double eta) {
  return Body{{float(x), float(y), float(z)}, float(r), RT_DIELECTRIC, {0.0f, 0.0f, 0.0f, float(eta)}};
}

}  // namespace

extern "C" int rt_scene_reference(float* sphere, int* kind, float* mat, int cap) {
  const std::vector<Body> b = {
      lam(0.0, -100.5, -1.0, 100.0, 0.8, 0.8, 0.0),  // ground  (:65-66)
      lam(0.0, 0.0, -1.2, 0.5, 0.1, 0.2, 0.5),       // center  (:68-69)
      die(-1.0, 0.0, -1.0, 0.5, 1.5),                // left    (:71-72)
      die(-1.0, 0.0, -1.0, 0.4, 1.00 / 1.5),         // bubble  (:74-75)
      met(1.0, 0.0, -1.0, 0.5, 0.8, 0.6, 0.2, 1.0),  // right   (:77-78)
  };
  return emit(b, sphere, kind, mat, cap);
}

extern "C" int rt_scene_cover(int grid, uint64_t seed, float* sphere, int* kind, float* mat, int cap) {
  if (grid < 0) return 0;
  SplitMix64 rng{seed};
  std::vector<Body> b;
  b.push_back(lam(0.0, -1000.0, 0.0, 1000.0, 0.5, 0.5, 0.5));
  for (int a = -grid; a < grid; ++a) {
    for (int bb = -grid; bb < grid; ++bb) {
      const double choose = rng.unit();
      const double cx = a + 0.9 * rng.unit();
      const double cz = bb + 0.9 * rng.unit();
      const double dx = cx - 4.0, dy = 0.0, dz = cz - 0.0;
      if (std::sqrt(dx * dx + dy * dy + dz * dz) <= 0.9) continue;
      if (choose < 0.8) {
        const double r1 = rng.unit() * rng.unit();
        const double g1 = rng.unit() * rng.unit();
        const double b1 = rng.unit() * rng.unit();
        b.push_back(lam(cx, 0.2, cz, 0.2, r1, g1, b1));
      } else if (choose < 0.95) {
        const double r1 = rng.range(0.5, 1.0), g1 = rng.range(0.5, 1.0), b1 = rng.range(0.5, 1.0);
        const double fuzz = rng.range(0.0, 0.5);
        b.push_back(met(cx, 0.2, cz, 0.2, r1, g1, b1, fuzz));
      } else {
        b.push_back(die(cx, 0.2, cz, 0.2, 1.5));
      }
    }
  }
  b.push_back(die(0.0, 1.0, 0.0, 1.0, 1.5));
  b.push_back(lam(-4.0, 1.0, 0.0, 1.0, 0.4, 0.2, 0.1));
  b.push_back(met(4.0, 1.0, 0.0, 1.0, 0.7, 0.6, 0.5, 0.0));
  return emit(b, sphere, kind, mat, cap);
}
