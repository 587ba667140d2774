// rt_oracle.cpp — TEST INFRASTRUCTURE ONLY. CPU restatement of the
// reference's hot path (keychera/raytracing-clj, Clojure), used as the parity
// checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
// Nothing in the product (raytracing-clj_amd/) links, loads or calls this.
//
// Two modes:
//   MODE_REF64 (0) — reference semantics in double, following the Clojure
//     line by line: recursive ray-color with attenuation applied on return,
//     un-normalised ray directions, a = |d|^2 and division by a in the sphere
//     hit, metal reflecting the un-normalised d, Math/pow in reflectance,
//     1e-160 / 1e-8 thresholds, and `rand` drawn in the reference's order.
//       src/raytracing.clj:19-58, 89-155   (quantise, hit-anything, ray-color,
//                                           defocus sample, compute-pixel)
//       src/hittable.clj:7-31             (sphere hit-fn)
//       src/material.clj:13-46            (lambertian, metal, dielectric)
//       src/vec3a.clj:56-101              (dot, unit, samplers, reflect, refract)
//       src/hit.clj:14-15, src/ray.clj:7-8
//   MODE_MIRROR32 (1) — the GPU kernel's fp32 arithmetic contract
//     (raytracing-clj_amd/csrc/trace.hip) restated op for op:
//     explicit fmaf, correctly rounded / and sqrt, normalisation by one
//     reciprocal (v * (1/|v|), (p - C) * (1/r)), unit-direction hit test,
//     stackless throughput, exact "both roots behind" pre-filter, each
//     sample's colour added to the pixel's integer sum in 2^-24 units
//     (fix24; order-free), the pixel RN(float(sum)) * 2^-24 / spp.  The GPU
//     output must equal this bit for bit.
//
//   MODE_REALM64 (3) — the reference's second namespace, realm.raytracing
//     (src/realm/raytracing.clj, `clojure -M:realm`), in double: the same
//     hit test and samplers, but lambertian without the near-zero fallback
//     (:137-143), dielectric without Schlick reflectance, i.e. no draw
//     (:160-177), an iterative ray-color that multiplies the throughput
//     forward (:205-236), and the pixel as sum * (1/spp) (:25, :276).
//     Its camera (no defocus, focal length |lookfrom - lookat|, :285-300) is
//     the caller's rt_camera.
//   MODE_REALM32 (4) — MODE_MIRROR32 with the kernel's RT_FLAG_REALM: the
//     same three semantic changes, the pixel as total * RN(1/spp).
//   mode | 0x10, | 0x20 (MODE_MIRROR32 / MODE_REALM32 only) — the kernel's
//     loop-free samplers (RT_FLAG_DIRECT_SAMPLERS: 0x10 the unit-sphere draw
//     of lambertian and metal, 0x20 the defocus disk): the same
//     distributions as vec3a.clj:74-86, a fixed number of draws.
//
// The reference's RNG is clojure.core/rand (unseeded java.util.Random,
// vec3a.clj:71-72), so no bitwise reference image exists.  Both modes draw
// from the build's keyed stream instead: xorshift32 seeded per
// (seed, pixel, sample) through the lowbias32 hash; a draw is the top 24 bits
// / 2^24.  Parity with the reference itself is therefore statistical and is
// pinned by the reference's only hot-path fixture, scene.ppm (400x225,
// 100 spp, depth 50): tests/golden/scene_ppm_stats.json, checked in
// tests/test_oracle_pinning.py.
//
// Compiled with -O2 -ffp-contract=off (see oracle/Makefile) so that neither
// mode picks up fused multiply-adds the source does not spell out.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

enum { MODE_REF64 = 0, MODE_MIRROR32 = 1, MODE_BOOK64 = 2, MODE_REALM64 = 3, MODE_REALM32 = 4 };

// MODE_BOOK64: MODE_REF64 but metal reflects unit(d) as the RTIOW book does
// (negative control: scene.ppm must reject it).
thread_local bool t_book_metal = false;
enum { LAMB = 0, METAL = 1, DIEL = 2, NONE = 3 };

// ------------------------------------------------------------ RNG (contract)
inline uint32_t mix32(uint32_t x) {  // lowbias32
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
inline uint32_t seed_key(uint64_t seed) {
  return mix32(static_cast<uint32_t>(seed) ^ mix32(static_cast<uint32_t>(seed >> 32) ^ 0x85ebca6bu));
}
inline uint32_t sample_state(uint32_t key, uint32_t pixel, uint32_t sample) {
  const uint32_t pk = mix32(key ^ mix32(pixel));
  uint32_t st = mix32(pk + sample * 0x9e3779b9u);
  return st ? st : 0x6d2b79f5u;
}
struct Rng {
  uint32_t s;
  float uf() {  // xorshift32, top 24 bits
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return static_cast<float>(s >> 8) * 0x1p-24f;
  }
  double ud() { return static_cast<double>(uf()); }  // clojure (rand) stand-in
};

// ----------------------------------------------------------- fp64 reference
struct V {
  double x, y, z;
};
inline V vadd(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V vsub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V vmul(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V vdiv(V a, double s) { return {a.x / s, a.y / s, a.z / s}; }
inline V vmulv(V a, V b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V vneg(V a) { return {-a.x, -a.y, -a.z}; }
inline double vdot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // vec3a.clj:56-58
inline double vlen2(V a) { return a.x * a.x + a.y * a.y + a.z * a.z; }      // vec3a.clj:50-51
inline V vunit(V a) { return vdiv(a, std::sqrt(vlen2(a))); }                 // vec3a.clj:69

inline double rand_double(Rng& r, double lo, double hi) { return lo + (hi - lo) * r.ud(); }  // vec3a.clj:71-72

V random_unit64(Rng& r) {  // vec3a.clj:74-79
  for (;;) {
    const double x = rand_double(r, -1.0, 1.0);
    const double y = rand_double(r, -1.0, 1.0);
    const double z = rand_double(r, -1.0, 1.0);
    const double l2 = x * x + y * y + z * z;
    if (l2 > 1e-160 && l2 <= 1.0) return vdiv(V{x, y, z}, std::sqrt(l2));
  }
}
V random_in_unit_disk64(Rng& r) {  // vec3a.clj:81-86
  for (;;) {
    const double x = rand_double(r, -1.0, 1.0);
    const double y = rand_double(r, -1.0, 1.0);
    if (x * x + y * y < 1.0) return V{x, y, 0.0};
  }
}
inline bool near_zero64(V v) {  // vec3a.clj:88-92
  return std::fabs(v.x) < 1e-8 && std::fabs(v.y) < 1e-8 && std::fabs(v.z) < 1e-8;
}
inline V reflect64(V v, V n) { return vsub(v, vmul(n, 2 * vdot(v, n))); }  // vec3a.clj:94-95
V refract64(V uv, V n, double e) {                                          // vec3a.clj:97-101
  const double c = std::min(vdot(vneg(uv), n), 1.0);
  const V perp = vmul(vadd(uv, vmul(n, c)), e);
  const V par = vmul(n, -std::sqrt(std::fabs(1.0 - vlen2(perp))));
  return vadd(perp, par);
}
double reflectance64(double cosine, double ri) {  // material.clj:30-32
  const double r0 = std::pow((1.0 - ri) / (1.0 + ri), 2);
  return r0 + (1.0 - r0) * std::pow(1.0 - cosine, 5);
}

struct Hit64 {
  double t;
  V p, n;
  bool front;
  int what;
};

// hittable.clj:9-31 (+ ray/at, hit/front-face?)
bool sphere_hit64(const double* s, V o, V d, double tmin, double tmax, Hit64* h) {
  const V c{s[0], s[1], s[2]};
  const double r = s[3];
  const V oc = vsub(c, o);
  const double a = vlen2(d);
  const double hh = vdot(d, oc);
  const double cc = vlen2(oc) - r * r;
  const double disc = hh * hh - a * cc;
  if (disc < 0.0) return false;
  const double sq = std::sqrt(disc);
  double root = (hh - sq) / a;
  if (root <= tmin || tmax <= root) root = (hh + sq) / a;
  if (root <= tmin || tmax <= root) return false;
  const V p = vadd(o, vmul(d, root));
  const V out = vdiv(vsub(p, c), r);
  const bool front = vdot(d, out) < 0;
  h->t = root;
  h->p = p;
  h->front = front;
  h->n = front ? out : vneg(out);
  return true;
}

struct Scene64 {
  int n;
  const double* sph;
  const int* kind;
  const double* mat;
};

// raytracing.clj:33-43
bool hit_anything64(const Scene64& sc, V o, V d, double tmin, double tmax, Hit64* rec,
                    uint64_t* tests) {
  bool any = false;
  double closest = tmax;
  for (int i = 0; i < sc.n; ++i) {
    Hit64 h;
    if (sphere_hit64(sc.sph + 4 * i, o, d, tmin, closest, &h)) {
      closest = h.t;
      h.what = i;
      *rec = h;
      any = true;
    }
  }
  *tests += 1;
  return any;
}

// raytracing.clj:45-58 (recursive; attenuation applied on return)
V ray_color64(const Scene64& sc, V o, V d, int depth, Rng& rng, uint64_t* segs) {
  if (depth <= 0) return V{0, 0, 0};
  Hit64 h;
  if (hit_anything64(sc, o, d, 1e-3, INFINITY, &h, segs)) {
    const double* m = sc.mat + 4 * h.what;
    const V alb{m[0], m[1], m[2]};
    V sd;
    V att;
    switch (sc.kind[h.what]) {
      case LAMB: {  // material.clj:13-19
        V s = vadd(random_unit64(rng), h.n);
        sd = near_zero64(s) ? h.n : s;
        att = alb;
        break;
      }
      case METAL: {  // material.clj:21-28
        const V refl = reflect64(t_book_metal ? vunit(d) : d, h.n);
        const V r2 = vadd(vmul(random_unit64(rng), m[3]), refl);
        if (!(vdot(r2, h.n) > 0)) return V{0, 0, 0};
        sd = r2;
        att = alb;
        break;
      }
      case NONE:  // no ::scatter-fn on the body -> black (raytracing.clj:49-54)
        return V{0, 0, 0};
      default: {  // material.clj:34-46
        const double ri = h.front ? (1.0 / m[3]) : m[3];
        const V u = vunit(d);
        const double cs = std::min(vdot(vneg(u), h.n), 1.0);
        const double sn = std::sqrt(1.0 - cs * cs);
        const bool can = ri * sn <= 1.0;
        if (!can || reflectance64(cs, ri) > rng.ud())
          sd = reflect64(u, h.n);
        else
          sd = refract64(u, h.n, ri);
        att = V{1.0, 1.0, 1.0};
        break;
      }
    }
    return vmulv(ray_color64(sc, h.p, sd, depth - 1, rng, segs), att);
  }
  const double y = vunit(d).y;
  const double a = 0.5 * (y + 1.0);
  return vadd(vmul(V{1.0, 1.0, 1.0}, 1.0 - a), vmul(V{0.5, 0.7, 1.0}, a));
}

// realm/raytracing.clj:205-236: iterative; target starts at (1,1,1) and is
// multiplied by each attenuation, then by the sky colour (:229-236)
V ray_color_realm64(const Scene64& sc, V o, V d, int depth, Rng& rng, uint64_t* segs) {
  V target{1.0, 1.0, 1.0};
  for (;;) {
    if (depth <= 0) return V{0, 0, 0};
    Hit64 h;
    if (!hit_anything64(sc, o, d, 1e-3, INFINITY, &h, segs)) {
      const double y = vunit(d).y;
      const double a = 0.5 * (y + 1.0);
      const V sky{(1.0 - a) * 1.0 + a * 0.5, (1.0 - a) * 1.0 + a * 0.7, (1.0 - a) * 1.0 + a * 1.0};
      return vmulv(target, sky);
    }
    const double* m = sc.mat + 4 * h.what;
    const V alb{m[0], m[1], m[2]};
    V sd, att;
    switch (sc.kind[h.what]) {
      case LAMB:  // :137-143, no near-zero fallback
        sd = vadd(random_unit64(rng), h.n);
        att = alb;
        break;
      case METAL: {  // :145-156
        const V refl = reflect64(d, h.n);
        const V r2 = vadd(refl, vmul(random_unit64(rng), m[3]));
        if (!(vdot(r2, h.n) > 0)) return V{0, 0, 0};
        sd = r2;
        att = alb;
        break;
      }
      case NONE:
        return V{0, 0, 0};
      default: {  // :158-177, no Schlick term and no draw
        const double ri = h.front ? (1.0 / m[3]) : m[3];
        const V u = vunit(d);
        const double cs = std::min(vdot(vneg(u), h.n), 1.0);
        const double sn = std::sqrt(1.0 - cs * cs);
        sd = ri * sn > 1.0 ? reflect64(u, h.n) : refract64(u, h.n, ri);
        att = V{1.0, 1.0, 1.0};
        break;
      }
    }
    target = vmulv(target, att);
    o = h.p;
    d = sd;
    --depth;
  }
}

// ---------------------------------------------------------- fp32 mirror ---
struct Scene32 {
  int n;
  std::vector<float> geo;  // cx cy cz -r*r
  std::vector<float> sph;  // cx cy cz r
  std::vector<float> mat;
  const int* kind;
};

// A sample colour channel in the pixel's fixed-point sum (trace.hip fix24:
// v_cvt_u32_f32 of c * 2^24 -- toward zero, NaN and c <= 0 -> 0, >= 2^32 ->
// 2^32 - 1)
inline uint32_t fix24(float c) {
  const float v = c * 0x1p24f;
  if (!(v > 0.0f)) return 0u;
  if (v >= 0x1p32f) return 0xffffffffu;
  return static_cast<uint32_t>(v);
}

void random_unit32(Rng& s, float& x, float& y, float& z) {
  float l2;
  do {
    x = 2.0f * s.uf() - 1.0f;
    y = 2.0f * s.uf() - 1.0f;
    z = 2.0f * s.uf() - 1.0f;
    l2 = std::fmaf(z, z, std::fmaf(y, y, x * x));
  } while (!(l2 > 0.0f && l2 <= 1.0f));
  const float il = 1.0f / std::sqrt(l2);
  x = x * il;
  y = y * il;
  z = z * il;
}

// The kernel's loop-free samplers (RT_FLAG_DIRECT_SAMPLERS;
// raytracing-clj_amd/csrc/trace_kernel.h turn24 / sphere_direct /
// disk_direct), op for op: the same distributions as vec3a.clj:74-86's
// rejection loops -- uniform on the unit sphere (z = 2 xi1 - 1, r = sqrt(1 -
// z^2)) and in the unit disk (r = sqrt(xi1)) -- at the angle 2 pi xi2, whose
// (cos, sin) come from the 24-bit integer of xi2: the nearest quarter turn q
// and Taylor polynomials of the rest (|theta| <= pi/4), rotated by q.
inline uint32_t u24(Rng& r) {
  r.s ^= r.s << 13;
  r.s ^= r.s >> 17;
  r.s ^= r.s << 5;
  return r.s >> 8;
}
void turn24(uint32_t u, float r, float& x, float& y) {
  const int32_t f = static_cast<int32_t>(u << 10) >> 10;       // low 22 bits, signed
  const uint32_t q = (u + 0x200000u) >> 22;                    // nearest quarter turn (mod 4)
  const float th = static_cast<float>(f) * 0x1.921fb6p-22f;    // RN(2 pi / 2^24)
  const float t2 = th * th;
  float ps = std::fmaf(t2, 0x1.71de3ap-19f, -0x1.a01a02p-13f);
  ps = std::fmaf(t2, ps, 0x1.111112p-7f);
  ps = std::fmaf(t2, ps, -0x1.555556p-3f);
  const float sn = std::fmaf(th * t2, ps, th);
  float pc = std::fmaf(t2, 0x1.a01a02p-16f, -0x1.6c16c2p-10f);
  pc = std::fmaf(t2, pc, 0x1.555556p-5f);
  pc = std::fmaf(t2, pc, -0.5f);
  const float cs = std::fmaf(t2, pc, 1.0f);
  const bool sw = (q & 1u) != 0;
  const float a = sw ? sn : cs, b = sw ? cs : sn;
  const float rx = (((q + 1u) & 2u) != 0) ? -r : r;            // x < 0 for q = 1, 2
  const float ry = ((q & 2u) != 0) ? -r : r;                   // y < 0 for q = 2, 3
  x = rx * a;
  y = ry * b;
}
void sphere_direct32(Rng& s, float& x, float& y, float& z) {
  z = 2.0f * s.uf() - 1.0f;
  const float r = std::sqrt(std::fmaf(-z, z, 1.0f));
  turn24(u24(s), r, x, y);
}
void disk_direct32(Rng& s, float& x, float& y) {
  const float r = std::sqrt(s.uf());
  turn24(u24(s), r, x, y);
}
enum { DIRECT_SPHERE = 1, DIRECT_DISK = 2 };   // the kernel's RT_SAMPLER_* bits (mode >> 4)

// one sample of the stackless kernel loop; returns colour, adds segments
void sample32(const Scene32& sc, const float* cam, bool defocus, bool realm, int direct, int px, int gy,
              uint32_t st, int max_depth, float* col, uint64_t* segs) {
  Rng rng{st};
  const float fx = static_cast<float>(px) + (rng.uf() - 0.5f);
  const float fy = static_cast<float>(gy) + (rng.uf() - 0.5f);
  const float sx = std::fmaf(cam[9], fy, std::fmaf(cam[6], fx, cam[3]));
  const float sy = std::fmaf(cam[10], fy, std::fmaf(cam[7], fx, cam[4]));
  const float sz = std::fmaf(cam[11], fy, std::fmaf(cam[8], fx, cam[5]));
  float ox, oy, oz;
  if (defocus) {
    float qx, qy;
    if (direct & DIRECT_DISK) {
      disk_direct32(rng, qx, qy);
    } else {
      do {
        qx = 2.0f * rng.uf() - 1.0f;
        qy = 2.0f * rng.uf() - 1.0f;
      } while (!(std::fmaf(qy, qy, qx * qx) < 1.0f));
    }
    ox = std::fmaf(cam[15], qy, std::fmaf(cam[12], qx, cam[0]));
    oy = std::fmaf(cam[16], qy, std::fmaf(cam[13], qx, cam[1]));
    oz = std::fmaf(cam[17], qy, std::fmaf(cam[14], qx, cam[2]));
  } else {
    ox = cam[0];
    oy = cam[1];
    oz = cam[2];
  }
  float dx = sx - ox, dy = sy - oy, dz = sz - oz;
  float tr = 1.0f, tg = 1.0f, tb = 1.0f;
  int last = -1;
  col[0] = col[1] = col[2] = 0.0f;
  for (int rem = max_depth; rem > 0;) {
    --rem;
    *segs += 1;
    const float len = std::sqrt(std::fmaf(dz, dz, std::fmaf(dy, dy, dx * dx)));
    const float il = 1.0f / len;
    const float ux = dx * il, uy = dy * il, uz = dz * il;
    const float tmin = 1e-3f * len;
    float best_t = INFINITY;
    int best = -1;
    for (int s = 0; s < sc.n; ++s) {
      const float* g = &sc.geo[4 * s];
      const float ocx = g[0] - ox, ocy = g[1] - oy, ocz = g[2] - oz;
      const float h = std::fmaf(uz, ocz, std::fmaf(uy, ocy, ux * ocx));
      const float c = std::fmaf(ocx, ocx, std::fmaf(ocz, ocz, std::fmaf(ocy, ocy, g[3])));
      const float disc = std::fmaf(h, h, -c);
      if (disc >= 0.0f && (h >= 0.0f || c < 0.0f)) {
        // the body the ray is leaving: exact arithmetic has c = 0 there
        // (origin on its surface), so sq = |h| (self-hit acne guard)
        const float sq = (s == last) ? std::fabs(h) : std::sqrt(disc);
        float t = h - sq;
        if (!(t > tmin)) t = h + sq;
        if (t > tmin && t < best_t) {
          best_t = t;
          best = s;
        }
      }
    }
    if (best < 0) {
      const float sa = 0.5f * (uy + 1.0f);
      const float om = 1.0f - sa;
      col[0] = tr * std::fmaf(sa, 0.5f, om);
      col[1] = tg * std::fmaf(sa, 0.7f, om);
      col[2] = tb * std::fmaf(sa, 1.0f, om);
      return;
    }
    if (rem == 0) return;
    const float* sp = &sc.sph[4 * best];
    const float hx = std::fmaf(ux, best_t, ox);
    const float hy = std::fmaf(uy, best_t, oy);
    const float hz = std::fmaf(uz, best_t, oz);
    const float ir = 1.0f / sp[3];
    float nx = (hx - sp[0]) * ir, ny = (hy - sp[1]) * ir, nz = (hz - sp[2]) * ir;
    const bool front = std::fmaf(dz, nz, std::fmaf(dy, ny, dx * nx)) < 0.0f;
    if (!front) {
      nx = -nx;
      ny = -ny;
      nz = -nz;
    }
    const float* m = &sc.mat[4 * best];
    ox = hx;
    oy = hy;
    oz = hz;
    last = best;
    const int kind = sc.kind[best];
    if (kind == LAMB) {
      float rx, ry, rz;
      if (direct & DIRECT_SPHERE)
        sphere_direct32(rng, rx, ry, rz);
      else
        random_unit32(rng, rx, ry, rz);
      float qx = rx + nx, qy = ry + ny, qz = rz + nz;
      if (!realm && std::fabs(qx) < 1e-8f && std::fabs(qy) < 1e-8f && std::fabs(qz) < 1e-8f) {
        qx = nx;
        qy = ny;
        qz = nz;
      }
      dx = qx;
      dy = qy;
      dz = qz;
      tr *= m[0];
      tg *= m[1];
      tb *= m[2];
    } else if (kind == METAL) {
      const float k2 = 2.0f * std::fmaf(dz, nz, std::fmaf(dy, ny, dx * nx));
      const float rx0 = std::fmaf(-nx, k2, dx), ry0 = std::fmaf(-ny, k2, dy), rz0 = std::fmaf(-nz, k2, dz);
      float qx, qy, qz;
      if (direct & DIRECT_SPHERE)
        sphere_direct32(rng, qx, qy, qz);
      else
        random_unit32(rng, qx, qy, qz);
      const float rx = std::fmaf(m[3], qx, rx0), ry = std::fmaf(m[3], qy, ry0), rz = std::fmaf(m[3], qz, rz0);
      if (!(std::fmaf(rz, nz, std::fmaf(ry, ny, rx * nx)) > 0.0f)) return;  // absorbed
      dx = rx;
      dy = ry;
      dz = rz;
      tr *= m[0];
      tg *= m[1];
      tb *= m[2];
    } else if (kind == NONE) {
      return;
    } else {
      const float ri = front ? (1.0f / m[3]) : m[3];
      const float un = std::fmaf(uz, nz, std::fmaf(uy, ny, ux * nx));
      const float cosv = std::fmin(-un, 1.0f);
      const float sinv = std::sqrt(std::fmaf(-cosv, cosv, 1.0f));
      bool refl = !(ri * sinv <= 1.0f);
      if (!refl && !realm) {
        const float xi = rng.uf();
        float r0 = (1.0f - ri) / (1.0f + ri);
        r0 = r0 * r0;
        const float x1 = 1.0f - cosv;
        const float x2 = x1 * x1;
        const float x5 = x2 * x2 * x1;
        refl = std::fmaf(1.0f - r0, x5, r0) > xi;
      }
      if (refl) {
        const float k2 = 2.0f * un;
        dx = std::fmaf(-nx, k2, ux);
        dy = std::fmaf(-ny, k2, uy);
        dz = std::fmaf(-nz, k2, uz);
      } else {
        const float qx = std::fmaf(nx, cosv, ux) * ri;
        const float qy = std::fmaf(ny, cosv, uy) * ri;
        const float qz = std::fmaf(nz, cosv, uz) * ri;
        const float par = -std::sqrt(std::fabs(1.0f - std::fmaf(qz, qz, std::fmaf(qy, qy, qx * qx))));
        dx = std::fmaf(nx, par, qx);
        dy = std::fmaf(ny, par, qy);
        dz = std::fmaf(nz, par, qz);
      }
    }
  }
}

struct Job {
  int mode;
  int direct;   // the fp32 modes' loop-free samplers (DIRECT_* bits)
  Scene64 s64;
  Scene32 s32;
  double cam64[18];
  float cam32[18];
  bool defocus;
  int width, row_begin, row_step, spp, sample_begin, max_depth;
  uint32_t key;
  float* out;
  double* out64;
};

void render_row(const Job& J, int ro, int x0, int x1, uint64_t* segs) {
  const int gy = J.row_begin + ro * J.row_step;
  t_book_metal = J.mode == MODE_BOOK64;
  const bool realm = J.mode == MODE_REALM64 || J.mode == MODE_REALM32;
  for (int px = x0; px < x1; ++px) {
    const uint32_t pixel = static_cast<uint32_t>(gy) * static_cast<uint32_t>(J.width) + static_cast<uint32_t>(px);
    const size_t o = (static_cast<size_t>(ro) * J.width + px) * 3;
    if (J.mode == MODE_REF64 || J.mode == MODE_BOOK64 || J.mode == MODE_REALM64) {
      // compute-pixel (raytracing.clj:141-155)
      const double* c = J.cam64;
      const V center{c[0], c[1], c[2]}, p00{c[3], c[4], c[5]}, du{c[6], c[7], c[8]}, dv{c[9], c[10], c[11]};
      const V disk_u{c[12], c[13], c[14]}, disk_v{c[15], c[16], c[17]};
      V acc{0, 0, 0};
      for (int k = 0; k < J.spp; ++k) {
        Rng rng{sample_state(J.key, pixel, static_cast<uint32_t>(J.sample_begin + k))};
        const double xi1 = rng.ud();
        const V ps0 = vadd(p00, vmul(du, px + (xi1 - 0.5)));
        const double xi2 = rng.ud();
        const V ps = vadd(ps0, vmul(dv, gy + (xi2 - 0.5)));
        V org = center;
        if (J.defocus) {  // defocus-disk-sample (raytracing.clj:89-93)
          const V p = random_in_unit_disk64(rng);
          org = vadd(vadd(center, vmul(disk_u, p.x)), vmul(disk_v, p.y));
        }
        const V dir = vsub(ps, org);
        acc = vadd(acc, realm ? ray_color_realm64(J.s64, org, dir, J.max_depth, rng, segs)
                              : ray_color64(J.s64, org, dir, J.max_depth, rng, segs));
      }
      // compute-pixel divides by spp (raytracing.clj:155); realm multiplies
      // by pixel-scale = 1.0 / spp (realm/raytracing.clj:25, :276)
      const V res = realm ? vmul(acc, 1.0 / static_cast<double>(J.spp)) : vdiv(acc, static_cast<double>(J.spp));
      J.out[o] = static_cast<float>(res.x);
      J.out[o + 1] = static_cast<float>(res.y);
      J.out[o + 2] = static_cast<float>(res.z);
      if (J.out64) {
        J.out64[o] = res.x;
        J.out64[o + 1] = res.y;
        J.out64[o + 2] = res.z;
      }
    } else {
      // contract: each sample's colour channel becomes fix24(c) (c * 2^24
      // toward zero, saturating; trace.hip's v_cvt_u32_f32) and the pixel
      // sums them as integers (order-free); total = RN(float(sum)) * 2^-24,
      // then / spp (realm: * RN(1/spp))
      uint64_t sr = 0, sg = 0, sb = 0;
      const uint32_t pk = mix32(J.key ^ mix32(pixel));
      for (int k = 0; k < J.spp; ++k) {
        uint32_t st = mix32(pk + static_cast<uint32_t>(J.sample_begin + k) * 0x9e3779b9u);
        if (st == 0) st = 0x6d2b79f5u;
        float col[3];
        sample32(J.s32, J.cam32, J.defocus, realm, J.direct, px, gy, st, J.max_depth, col, segs);
        sr += fix24(col[0]);
        sg += fix24(col[1]);
        sb += fix24(col[2]);
      }
      const float tr_ = static_cast<float>(sr) * 0x1p-24f;
      const float tg_ = static_cast<float>(sg) * 0x1p-24f;
      const float tb_ = static_cast<float>(sb) * 0x1p-24f;
      const float inv = static_cast<float>(J.spp);
      if (realm) {  // total * RN(1/spp)
        const float sc = 1.0f / inv;
        J.out[o] = tr_ * sc;
        J.out[o + 1] = tg_ * sc;
        J.out[o + 2] = tb_ * sc;
      } else {
        J.out[o] = tr_ / inv;
        J.out[o + 1] = tg_ / inv;
        J.out[o + 2] = tb_ / inv;
      }
    }
  }
}

}  // namespace

extern "C" {

// Render rows row_begin, row_begin+row_step, ... < row_end into out
// (compacted: rows x width x 3 fp32, and
// optionally out64 in double for MODE_REF64).  sphere/mat: n x 4 doubles,
// cam: 18 doubles (center, p00, du, dv, disk_u, disk_v).  nthreads <= 0 ->
// hardware concurrency.  counters (nullable): [segments, samples].
// oracle_render_cols: only columns [col_begin, col_end) of those rows (the
// others are left as they are in out); oracle_render: every column.
int oracle_render_cols(int mode, int n, const double* sphere, const int* kind, const double* mat,
                       const double* cam, int defocus, int width, int height, int row_begin, int row_end,
                       int row_step, int col_begin, int col_end, int spp, int sample_begin, int max_depth,
                       uint64_t seed, int nthreads, float* out, double* out64, uint64_t* counters) {
  if (width <= 0 || height <= 0 || row_begin < 0 || row_end > height || row_end < row_begin || !out ||
      row_step <= 0 || col_begin < 0 || col_end > width || col_end < col_begin ||
      (n > 0 && (!sphere || !kind || !mat)) || !cam || (mode & ~0x3f) != 0)
    return -1;
  // mode | (DIRECT_* << 4): the fp32 mirrors with the kernel's loop-free samplers
  const int direct = (mode >> 4) & (DIRECT_SPHERE | DIRECT_DISK);
  mode &= 0xf;
  if (mode < MODE_REF64 || mode > MODE_REALM32 || (direct && mode != MODE_MIRROR32 && mode != MODE_REALM32))
    return -1;
  Job J{};
  J.mode = mode;
  J.direct = direct;
  J.s64 = Scene64{n, sphere, kind, mat};
  J.s32.n = n;
  J.s32.kind = kind;
  J.s32.geo.resize(4 * static_cast<size_t>(std::max(n, 1)));
  J.s32.sph.resize(4 * static_cast<size_t>(std::max(n, 1)));
  J.s32.mat.resize(4 * static_cast<size_t>(std::max(n, 1)));
  for (int i = 0; i < n; ++i) {
    const float r = static_cast<float>(sphere[4 * i + 3]);
    for (int k = 0; k < 3; ++k) {
      J.s32.geo[4 * i + k] = static_cast<float>(sphere[4 * i + k]);
      J.s32.sph[4 * i + k] = static_cast<float>(sphere[4 * i + k]);
    }
    J.s32.geo[4 * i + 3] = -(r * r);
    J.s32.sph[4 * i + 3] = r;
    for (int k = 0; k < 4; ++k) J.s32.mat[4 * i + k] = static_cast<float>(mat[4 * i + k]);
  }
  for (int i = 0; i < 18; ++i) {
    J.cam64[i] = cam[i];
    J.cam32[i] = static_cast<float>(cam[i]);
  }
  J.defocus = defocus != 0;
  J.width = width;
  J.row_begin = row_begin;
  J.row_step = row_step;
  J.spp = spp;
  J.sample_begin = sample_begin;
  J.max_depth = max_depth;
  J.key = seed_key(seed);
  J.out = out;
  J.out64 = out64;
  const int rows = (row_end - row_begin + row_step - 1) / row_step;  // rows r0, r0+step, ... < r1
  if (spp <= 0 || max_depth <= 0) {
    // depth <= 0 -> black (raytracing.clj:46-47); spp 0 -> 0/0 in the
    // reference, defined here (and on the GPU) as 0/1 = black.
    for (int r = 0; r < rows; ++r) {
      const size_t o = (static_cast<size_t>(r) * width + col_begin) * 3, m = static_cast<size_t>(col_end - col_begin) * 3;
      std::fill(out + o, out + o + m, 0.0f);
      if (out64) std::fill(out64 + o, out64 + o + m, 0.0);
    }
    if (counters) counters[0] = counters[1] = 0;
    return 0;
  }
  // work items: 32-pixel row chunks, handed out by an atomic counter
  constexpr int CH = 32;
  const int per_row = (col_end - col_begin + CH - 1) / CH;
  const int items = rows * per_row;
  int nt = nthreads > 0 ? nthreads : static_cast<int>(std::thread::hardware_concurrency());
  nt = std::max(1, std::min(nt, std::max(items, 1)));
  std::atomic<int> next{0};
  std::vector<uint64_t> segs(nt, 0);
  auto work = [&](int tid) {
    for (int it; (it = next.fetch_add(1)) < items;) {
      const int r = it / per_row, x0 = col_begin + (it % per_row) * CH;
      render_row(J, r, x0, std::min(col_end, x0 + CH), &segs[tid]);
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& t : th) t.join();
  }
  if (counters) {
    uint64_t s = 0;
    for (auto v : segs) s += v;
    counters[0] = s;
    counters[1] = static_cast<uint64_t>(rows) * (col_end - col_begin) * spp;
  }
  return 0;
}

int oracle_render(int mode, int n, const double* sphere, const int* kind, const double* mat,
                  const double* cam, int defocus, int width, int height, int row_begin, int row_end,
                  int row_step, int spp, int sample_begin, int max_depth, uint64_t seed, int nthreads,
                  float* out, double* out64, uint64_t* counters) {
  return oracle_render_cols(mode, n, sphere, kind, mat, cam, defocus, width, height, row_begin, row_end, row_step,
                            0, width, spp, sample_begin, max_depth, seed, nthreads, out, out64, counters);
}

// ---- known-answer entry points (fp64 reference formulas) ----

// hittable.clj:9-31.  out[0..8] = hit?, t, p(3), n(3), front
int oracle_sphere_hit(const double* sphere4, const double* o, const double* d, double tmin, double tmax,
                      double* out) {
  Hit64 h{};
  const bool hit = sphere_hit64(sphere4, V{o[0], o[1], o[2]}, V{d[0], d[1], d[2]}, tmin, tmax, &h);
  out[0] = hit ? 1.0 : 0.0;
  out[1] = h.t;
  out[2] = h.p.x;
  out[3] = h.p.y;
  out[4] = h.p.z;
  out[5] = h.n.x;
  out[6] = h.n.y;
  out[7] = h.n.z;
  out[8] = h.front ? 1.0 : 0.0;
  return hit ? 1 : 0;
}

void oracle_reflect(const double* v, const double* n, double* out) {
  const V r = reflect64(V{v[0], v[1], v[2]}, V{n[0], n[1], n[2]});
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

void oracle_refract(const double* uv, const double* n, double eta, double* out) {
  const V r = refract64(V{uv[0], uv[1], uv[2]}, V{n[0], n[1], n[2]}, eta);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

double oracle_reflectance(double cosine, double ri) { return reflectance64(cosine, ri); }

// material scatter directions with the random draws injected (material.clj):
// lambertian: unit + n, n if near-zero (:13-19, vec3a.clj:88-92)
void oracle_lambertian_dir(const double* unit, const double* n, double* out) {
  const V nn{n[0], n[1], n[2]};
  const V s = vadd(V{unit[0], unit[1], unit[2]}, nn);
  const V r = near_zero64(s) ? nn : s;
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}
// metal (:21-28): returns 1 if scattered (dot > 0), 0 if absorbed
int oracle_metal_dir(const double* d, const double* n, double fuzz, const double* unit, double* out) {
  const V nn{n[0], n[1], n[2]};
  const V r = vadd(vmul(V{unit[0], unit[1], unit[2]}, fuzz), reflect64(V{d[0], d[1], d[2]}, nn));
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
  return vdot(r, nn) > 0 ? 1 : 0;
}
// dielectric (:34-46) with the uniform draw xi; returns 1 reflected, 0 refracted
int oracle_dielectric_dir(const double* d, const double* n, int front, double eta, double xi, double* out) {
  const V nn{n[0], n[1], n[2]};
  const double ri = front ? (1.0 / eta) : eta;
  const V u = vunit(V{d[0], d[1], d[2]});
  const double cs = std::min(vdot(vneg(u), nn), 1.0);
  const double sn = std::sqrt(1.0 - cs * cs);
  const bool refl = !(ri * sn <= 1.0) || reflectance64(cs, ri) > xi;
  const V r = refl ? reflect64(u, nn) : refract64(u, nn, ri);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
  return refl ? 1 : 0;
}

// write-color! (raytracing.clj:19-26) for one channel
int oracle_quantize(double c) {
  const double g = c > 0 ? std::sqrt(c) : 0.0;
  const double cl = std::min(0.999, std::max(g, 0.0));
  return static_cast<int>(256 * cl);
}

// camera, raytracing.clj:105-139, all double; out: 18 doubles
void oracle_camera(int w, int h, double vfov, const double* lf, const double* la, const double* vup,
                   double defocus_angle, double focus_dist, double* out) {
  const double pi = 3.141592653589793;
  const V LF{lf[0], lf[1], lf[2]}, LA{la[0], la[1], la[2]}, UP{vup[0], vup[1], vup[2]};
  const double theta = (vfov * pi) / 180.0;
  const double hh = std::tan(theta / 2);
  const double vh = 2.0 * hh * focus_dist;
  const double vw = vh * (static_cast<double>(w) / h);
  const V W = vunit(vsub(LF, LA));
  const V cr{UP.y * W.z - UP.z * W.y, UP.z * W.x - UP.x * W.z, UP.x * W.y - UP.y * W.x};
  const V U = vunit(cr);
  const V Vv{W.y * U.z - W.z * U.y, W.z * U.x - W.x * U.z, W.x * U.y - W.y * U.x};
  const V vu = vmul(U, vw), vv = vmul(vneg(Vv), vh);
  const V du = vdiv(vu, w), dv = vdiv(vv, h);
  const V ul = vsub(vsub(vsub(LF, vmul(W, focus_dist)), vdiv(vu, 2)), vdiv(vv, 2));
  const V p00 = vadd(ul, vmul(vadd(du, dv), 0.5));
  const double rad = focus_dist * std::tan(((defocus_angle / 2.0) * pi) / 180.0);
  const V vals[6] = {LF, p00, du, dv, vmul(U, rad), vmul(Vv, rad)};
  for (int i = 0; i < 6; ++i) {
    out[3 * i] = vals[i].x;
    out[3 * i + 1] = vals[i].y;
    out[3 * i + 2] = vals[i].z;
  }
}

// the keyed uniform stream of (seed, pixel, sample): n draws
void oracle_rng_stream(uint64_t seed, uint32_t pixel, uint32_t sample, int n, float* out) {
  Rng r{sample_state(seed_key(seed), pixel, sample)};
  for (int i = 0; i < n; ++i) out[i] = r.uf();
}

// The samplers alone: n draws from one keyed stream (seed, pixel 0, sample
// 0), consecutive. which: 0 random_unit32 (vec3a.clj:74-79's rejection loop
// in fp32), 1 sphere_direct32, 2 the disk's rejection loop (vec3a.clj:81-86),
// 3 disk_direct32.  out: n x 3 floats (the disk's z = 0).
int oracle_sampler_draws(int which, uint64_t seed, int n, float* out) {
  if (which < 0 || which > 3 || n < 0 || (n > 0 && !out)) return -1;
  Rng r{sample_state(seed_key(seed), 0, 0)};
  for (int i = 0; i < n; ++i) {
    float x = 0, y = 0, z = 0;
    switch (which) {
      case 0: random_unit32(r, x, y, z); break;
      case 1: sphere_direct32(r, x, y, z); break;
      case 2:
        do {
          x = 2.0f * r.uf() - 1.0f;
          y = 2.0f * r.uf() - 1.0f;
        } while (!(std::fmaf(y, y, x * x) < 1.0f));
        break;
      default: disk_direct32(r, x, y); break;
    }
    out[3 * i] = x;
    out[3 * i + 1] = y;
    out[3 * i + 2] = z;
  }
  return 0;
}

// turn24 for given 24-bit integers: out[2i], out[2i+1] = r (cos, sin) of 2 pi u / 2^24
void oracle_turn24(int n, const uint32_t* u, float r, float* out) {
  for (int i = 0; i < n; ++i) turn24(u[i] & 0xffffffu, r, out[2 * i], out[2 * i + 1]);
}

}  // extern "C"
