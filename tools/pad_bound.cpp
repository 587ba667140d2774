// pad_bound.cpp — how far from a sphere can the fp32 hit test (trace.hip's
// exact op sequence) report a candidate?  Drives the BVH box padding.
// For random spheres/rays it measures, over fp32 candidates with t > tmin:
//   e_disc = |disc32 - disc_exact| / max(|oc|, r)^2
//   e_pt   = distance from O + t32*u (exact) to the sphere's AABB / |oc|
// g++ -O2 -ffp-contract=off -mfma tools/pad_bound.cpp -o /tmp/pad_bound && /tmp/pad_bound
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

int main(int argc, char** argv) {
  const long trials = argc > 1 ? std::atol(argv[1]) : 40000000;
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> U(-1, 1);
  double max_edisc = 0, max_ept = 0, max_ept_abs_over_D = 0;
  long cands = 0;
  for (long it = 0; it < trials; ++it) {
    // scene-like magnitudes: centres within +-S, origin within +-S (some far), radius log-uniform
    const double S = (it % 10 == 0) ? 1000.0 : 30.0;
    float cx = float(U(g) * 30), cy = float(U(g) * 3), cz = float(U(g) * 30);
    float r = float(std::exp(std::log(0.05) + (U(g) * 0.5 + 0.5) * std::log(40.0)));
    float ox = float(U(g) * S), oy = float(U(g) * S * 0.1 + 1), oz = float(U(g) * S);
    // aim near the sphere silhouette to stress tangency
    double ax = cx - ox + U(g) * r * 1.2, ay = cy - oy + U(g) * r * 1.2, az = cz - oz + U(g) * r * 1.2;
    float dx = float(ax), dy = float(ay), dz = float(az);
    const float len = std::sqrt(std::fmaf(dz, dz, std::fmaf(dy, dy, dx * dx)));
    const float ux = dx / len, uy = dy / len, uz = dz / len;
    const float tmin = 1e-3f * len;
    const float nr2 = -(r * r);
    const float ocx = cx - ox, ocy = cy - oy, ocz = cz - oz;
    const float h = std::fmaf(uz, ocz, std::fmaf(uy, ocy, ux * ocx));
    const float c = std::fmaf(ocx, ocx, std::fmaf(ocz, ocz, std::fmaf(ocy, ocy, nr2)));
    const float disc = std::fmaf(h, h, -c);
    if (!(std::fmin(disc, std::fmax(h, -c)) >= 0.0f)) continue;
    const float sq = std::sqrt(disc);
    float t = h - sq;
    if (!(t > tmin)) t = h + sq;
    if (!(t > tmin)) continue;
    ++cands;
    // exact (long double) on the same float inputs
    long double Ux = ux, Uy = uy, Uz = uz;
    long double OCx = (long double)cx - ox, OCy = (long double)cy - oy, OCz = (long double)cz - oz;
    long double He = Ux * OCx + Uy * OCy + Uz * OCz;
    long double oc2 = OCx * OCx + OCy * OCy + OCz * OCz;
    long double Ce = oc2 - (long double)r * r;
    long double De = He * He - Ce;
    const long double scale = oc2 > (long double)r * r ? oc2 : (long double)r * r;
    const double ed = double(std::fabs((long double)disc - De) / scale);
    if (ed > max_edisc) max_edisc = ed;
    // point at t (exact arithmetic) vs the sphere's AABB
    long double px = ox + Ux * t, py = oy + Uy * t, pz = oz + Uz * t;
    auto out = [](long double p, long double lo, long double hi) -> long double {
      return p < lo ? lo - p : (p > hi ? p - hi : 0.0L);
    };
    long double ex = out(px, (long double)cx - r, (long double)cx + r);
    long double ey = out(py, (long double)cy - r, (long double)cy + r);
    long double ez = out(pz, (long double)cz - r, (long double)cz + r);
    double e = double(std::sqrt(ex * ex + ey * ey + ez * ez));
    double D = double(std::sqrt(oc2)) + r;
    if (e / D > max_ept_abs_over_D) max_ept_abs_over_D = e / D;
    if (e > max_ept) max_ept = e;
  }
  std::printf("candidates %ld\nmax |disc32-disc| / max(|oc|,r)^2 = %.3g\nmax point-outside-AABB = %.3g (abs)\n"
              "max point-outside-AABB / (|oc|+r) = %.3g\n", cands, max_edisc, max_ept, max_ept_abs_over_D);
}
