// simt_sim.cpp — design tool (not product code): a CPU model of the trace
// kernel's SIMT cost on the C1 workload, to compare ways of grouping paths
// into waves before building one on the GPU.
//
// It traces the cover scene with the kernel's semantics in fp32 (not bit
// exact: no padding, plain sqrt; the work counts are what matters) through
// the same 4-body-leaf SAH tree (bvh.cpp), and records per segment the
// traversal as the kernel runs it: node visits, and per visit the leaves
// entered and their candidate bodies.  A wave's cost for one outer iteration
// is then priced the way the hardware issues it (VALU issue
// bound, a wave pays for a block if any lane needs it):
//   outer       C_OUT per wave iteration (camera, setup, shading)
//   traversal   sum over steps i < max lanes' visits of
//               C_NODE + C_LEAF * max_lanes(leaves at i) + C_EXACT * max_lanes(cands)
// Policies:
//   wave   the shipped shape: a workgroup's 8x8-pixel pool, 4 independent
//          waves refilling from it (advanced in cost order)
//   sort   the 4 waves advance together; before every iteration the 256
//          paths are sorted by a key and dealt to the waves in that order
//   pair   (PAIR=R, NV=7 V0=6) R paths per lane, their segments walked back
//          to back in one traversal loop, then all shaded (round 6)
//   DEFER=1 (with any policy): a visit's second leaf pushed and tested as a
//          leaf-only step next (one leaf pass per step); CNODE overrides C_NODE
//
//   g++ -O2 -std=c++17 -I include tools/simt_sim.cpp raytracing-clj_amd/csrc/bvh.cpp \
//       -Lraytracing-clj_amd/lib -lrtclj -Wl,-rpath,$PWD/raytracing-clj_amd/lib -o /tmp/simt_sim
//   /tmp/simt_sim [tiles=300] [spp=100]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "../include/rt.h"
#include "../raytracing-clj_amd/csrc/bvh.h"

using namespace rtclj;
namespace rtclj { extern float g_bvh_big_ratio; }
static double g_cand = 0, g_rej = 0, g_segs = 0, g_visits = 0, g_leafs = 0;
static float g_pad = 1.0f;
static int g_big_leaves = 0;
static int g_tile_h = 8;      // workgroup pool: 8 x g_tile_h pixels (TILEH)
static int g_nw = 4;          // waves per workgroup (NW; 8 with TILEH=16: 512 threads)
static double C_XCHG = 0;     // per wave-iteration cost of the sort policies' LDS path exchange (XCHG)
static int g_exact_mode = 0;   // 0: one pass per candidate of the busiest lane; 1: one block per leaf body
static double g_disk = 0, g_ball = 0, g_both = 0;   // rejection-loop wave trips
static double g_abs = 0;   // wave iterations with a metal absorption
static double C_EXACT_B = 32;
static double C_BALL = 27, C_DISK = 21;   // one rejection-loop trip (random-unit-vec3, disk)
static int g_restart_k = 32;
static int g_pair = 2;   // policy 3: paths per lane   // policy 2: shade once this many lanes finished traversal
static int g_charge_rej = 0;   // policies 0/1: add the rejection trips to the cost (RJ=1)

// VALU wave-instructions per block (from the ISA of the default kernel,
// trace_kernel<1, 5, -3, false>); leaf and exact costs for NP body pairs per leaf
static double C_OUT = 356, C_NODE = 38, C_LEAF = 45, C_EXACT = 44, C_SORT = 60;
static void set_leaf_costs(int np) {
  C_LEAF = 20 + 12.5 * np;
  C_EXACT = 35 + 3 * (2 * np - 1);
}

static uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
struct Rng {
  uint32_t s;
  float u() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return float(s >> 8) * 0x1p-24f; }
  float sym() { return 2.0f * u() - 1.0f; }
};

struct Scene {
  int n;
  std::vector<float> sph, mat;
  std::vector<int> kind;
  BvhHost t;
};

// one segment's traversal as the kernel runs it
struct Trav {
  int disk_tries = 0, ball_tries = 0;   // rejection-loop trips of this lane's iteration
  int absorbed = 0;                     // a metal scatter went below the surface
  int big_c = 0;                 // candidate bitmask of the big bodies (their leaf pass: every segment)
  std::vector<uint8_t> leaves;   // per visit: leaves entered (0-2)
  std::vector<uint8_t> c1, c2;   // per visit: candidate bitmasks of the first / second leaf
};

struct Hit { int body; float t; };

// Start-node table (QT=1): a quadtree over the tree's x-z extent; the entry
// of a level-k cell is the deepest node whose subtree holds every body whose
// box (grown by QT_M) meets the cell's column (-2: no body).  A ray segment
// clipped to the root box whose two ends share a level-k cell can start its
// traversal there.
static int g_qt = 0, g_qt_res = 32;
static float g_qt_m = 0.1f;
static float g_qt_lo[2], g_qt_cell[2];
static std::vector<std::vector<int>> g_qt_tab;   // per level: res_k x res_k start nodes
static double g_qt_skip = 0, g_qt_start_depth = 0, g_qt_n = 0;
// QT=2: one start node per wave (the wave's lanes stay in step): a probe
// pass records each lane's segment-end cells, the wave's start is the entry
// of the finest level whose cell holds all of them
static bool g_probe = false;
static int g_probe_valid = 0, g_probe_c[4];
static int g_force_start = 0;
static double C_QT = 30;

static int g_candbit = 0;   // the body's position in its leaf (candidate bitmask)
static void body_test(const float* s, float ox, float oy, float oz, float ux, float uy, float uz,
                      float tmin, int last, Hit& best, int idx, int& cand) {
  const float ocx = s[0] - ox, ocy = s[1] - oy, ocz = s[2] - oz;
  const float h = ux * ocx + uy * ocy + uz * ocz;
  const float c = ocx * ocx + ocy * ocy + ocz * ocz - s[3] * s[3];
  const float disc = h * h - c;
  if (!(std::fmin(disc, std::fmax(h, -c)) >= 0.0f)) return;
  cand |= 1 << g_candbit;
  g_cand += 1;
  const float sq = idx == last ? std::fabs(h) : std::sqrt(disc);
  float t = h - sq;
  if (!(t > tmin)) t = h + sq;
  if (t > tmin && (t < best.t || (t == best.t && idx < best.body))) best = {idx, t};
  else if (h - std::sqrt(disc) >= best.t) g_rej += 1;   // a near root beyond the best: a t-bound filter drops it
}

static Hit trace(const Scene& S, float ox, float oy, float oz, float ux, float uy, float uz, float tmin, int last,
                 Trav* tr) {
  Hit best{-1, INFINITY};
  int bigc = 0;
  for (size_t i = 0; i < S.t.big.size(); ++i) {
    g_candbit = int(i);
    body_test(&S.sph[4 * S.t.big[i]], ox, oy, oz, ux, uy, uz, tmin, last, best, S.t.big[i], bigc);
  }
  if (tr) tr->big_c = bigc;
  const float ex = ox - S.t.center[0], ey = oy - S.t.center[1], ez = oz - S.t.center[2];
  const float D = std::sqrt(ex * ex + ey * ey + ez * ez) + S.t.radius;
  const float P = g_pad * 2e-3f * D;
  const float rx = 1.0f / (std::fabs(ux) < 1e-24f ? std::copysign(1e-24f, ux) : ux);
  const float ry = 1.0f / (std::fabs(uy) < 1e-24f ? std::copysign(1e-24f, uy) : uy);
  const float rz = 1.0f / (std::fabs(uz) < 1e-24f ? std::copysign(1e-24f, uz) : uz);
  const int np = S.t.leaf_size / 2;
  auto leaf = [&](int p, int& cand) {
    for (int q = 0; q < np; ++q)
      for (int j = 0; j < 2; ++j) {
        const int id = S.t.pidx[2 * (p + q) + j];
        if (id < 0) continue;
        g_candbit = 2 * q + j;
        body_test(&S.sph[4 * id], ox, oy, oz, ux, uy, uz, tmin, last, best, id, cand);
      }
  };
  int stack[64], sp = 0, node = 0;
  g_segs += 1;
  if (g_qt) {
    // the root box = union of node 0's children (centre-relative), padded
    const BvhNode& r = S.t.nodes[0];
    float lo[3], hi[3];
    const float* ax[3] = {r.x, r.y, r.z};
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(ax[k][0], ax[k][1]) - P;
      hi[k] = std::max(ax[k][2], ax[k][3]) + P;
    }
    const float e[3] = {ex, ey, ez}, rr[3] = {rx, ry, rz};
    float t0 = tmin, t1 = best.t;
    for (int k = 0; k < 3; ++k) {
      const float a = (lo[k] - e[k]) * rr[k], b = (hi[k] - e[k]) * rr[k];
      t0 = std::max(t0, std::min(a, b));
      t1 = std::min(t1, std::max(a, b));
    }
    if (!g_probe) g_qt_n += 1;
    if (!(t0 <= t1)) {
      if (g_probe) { g_probe_valid = 0; return best; }
      g_qt_skip += 1;
      return best;
    }
    if (!std::isfinite(t1)) t1 = t0;   // (not reached: the box is finite)
    int c0[2], c1[2];
    const float u2[2] = {ux, uz}, e2[2] = {ex, ez};
    for (int k = 0; k < 2; ++k) {
      const float a = (e2[k] + u2[k] * t0 - g_qt_lo[k]) / g_qt_cell[k];
      const float b = (e2[k] + u2[k] * t1 - g_qt_lo[k]) / g_qt_cell[k];
      c0[k] = std::clamp(int(std::floor(a)), 0, g_qt_res - 1);
      c1[k] = std::clamp(int(std::floor(b)), 0, g_qt_res - 1);
    }
    if (g_probe) {
      g_probe_valid = 1;
      g_probe_c[0] = c0[0]; g_probe_c[1] = c0[1]; g_probe_c[2] = c1[0]; g_probe_c[3] = c1[1];
      return best;
    }
    const unsigned x = unsigned(c0[0] ^ c1[0]) | unsigned(c0[1] ^ c1[1]);
    const int lvl = x ? 32 - __builtin_clz(x) : 0;
    if (g_qt == 2) {
      if (g_force_start == -2) { g_qt_skip += 1; return best; }
      node = g_force_start;
    } else if (lvl < int(g_qt_tab.size())) {
      const int res = g_qt_res >> lvl;
      const int st = g_qt_tab[lvl][(c0[1] >> lvl) * res + (c0[0] >> lvl)];
      if (st == -2) { g_qt_skip += 1; return best; }
      node = st;
    }
  }
  for (;;) {
    g_visits += 1;
    const BvhNode& nd = S.t.nodes[node];
    float tn[2], tf[2];
    bool hit[2];
    for (int c = 0; c < 2; ++c) {
      const float x0 = (nd.x[c] - P - ex) * rx, x1 = (nd.x[2 + c] + P - ex) * rx;
      const float y0 = (nd.y[c] - P - ey) * ry, y1 = (nd.y[2 + c] + P - ey) * ry;
      const float z0 = (nd.z[c] - P - ez) * rz, z1 = (nd.z[2 + c] + P - ez) * rz;
      tn[c] = std::max({std::min(x0, x1), std::min(y0, y1), std::min(z0, z1)});
      tf[c] = std::min({std::max(x0, x1), std::max(y0, y1), std::max(z0, z1)});
      hit[c] = std::max(tn[c], tmin) <= std::min(tf[c], best.t);
    }
    const int c0 = nd.child[0], c1 = nd.child[1];
    const bool l0 = hit[0] && c0 < 0, l1 = hit[1] && c1 < 0;
    int k1 = 0, k2 = 0;
    g_leafs += l0 + l1;
    if (l0 | l1) leaf(l0 ? ~c0 : ~c1, k1);
    if (l0 & l1) leaf(~c1, k2);
    if (tr) {
      tr->leaves.push_back(uint8_t(l0 + l1));
      tr->c1.push_back(uint8_t(k1));
      tr->c2.push_back(uint8_t(k2));
    }
    const bool h0 = hit[0] && !l0, h1 = hit[1] && !l1;
    if (h0 && h1) {
      const bool sw = tn[1] < tn[0];
      stack[sp++] = sw ? c0 : c1;
      node = sw ? c1 : c0;
    } else if (h0) {
      node = c0;
    } else if (h1) {
      node = c1;
    } else {
      if (sp == 0) break;
      node = stack[--sp];
    }
  }
  return best;
}

// a path in flight: the lane state of the kernel's outer loop
struct Path {
  int j = -1;          // pool index (-1: lane idle)
  Rng rng{1};
  float o[3], d[3];
  int rem = 0, last = -1;
  bool fresh = true;
};

struct Ctx {
  const Scene* S;
  rt_camera cam;
  int width, spp, depth;
};

// one outer iteration of a lane: camera (if fresh), the segment, shading.
// Returns true when the path ended (the lane takes a new pool index).
static bool step(const Ctx& C, Path& p, int px, int py, Trav& tr) {
  const Scene& S = *C.S;
  if (p.fresh) {
    const uint32_t key = mix32(1u);
    const uint32_t pk = mix32(key ^ mix32(uint32_t(py) * uint32_t(C.width) + uint32_t(px)));
    const int k = p.j % C.spp;
    p.rng.s = mix32(pk + uint32_t(k) * 0x9e3779b9u);
    if (!p.rng.s) p.rng.s = 0x6d2b79f5u;
    const float fx = float(px) + (p.rng.u() - 0.5f), fy = float(py) + (p.rng.u() - 0.5f);
    float s[3], o[3];
    for (int a = 0; a < 3; ++a) s[a] = C.cam.p00[a] + C.cam.du[a] * fx + C.cam.dv[a] * fy;
    float qx, qy;
    do { qx = p.rng.sym(); qy = p.rng.sym(); ++tr.disk_tries; } while (!(qx * qx + qy * qy < 1.0f));
    for (int a = 0; a < 3; ++a) o[a] = C.cam.center[a] + C.cam.disk_u[a] * qx + C.cam.disk_v[a] * qy;
    for (int a = 0; a < 3; ++a) { p.o[a] = o[a]; p.d[a] = s[a] - o[a]; }
    p.rem = C.depth;
    p.last = -1;
    p.fresh = false;
  }
  --p.rem;
  const float len = std::sqrt(p.d[0] * p.d[0] + p.d[1] * p.d[1] + p.d[2] * p.d[2]);
  const float u[3] = {p.d[0] / len, p.d[1] / len, p.d[2] / len};
  const Hit h = trace(S, p.o[0], p.o[1], p.o[2], u[0], u[1], u[2], 1e-3f * len, p.last, &tr);
  if (h.body < 0 || p.rem == 0) return true;
  const float* c = &S.sph[4 * h.body];
  float hp[3], n[3];
  for (int a = 0; a < 3; ++a) hp[a] = p.o[a] + u[a] * h.t;
  for (int a = 0; a < 3; ++a) n[a] = (hp[a] - c[a]) / c[3];
  const bool front = p.d[0] * n[0] + p.d[1] * n[1] + p.d[2] * n[2] < 0.0f;
  if (!front) for (float& x : n) x = -x;
  for (int a = 0; a < 3; ++a) p.o[a] = hp[a];
  p.last = h.body;
  const int kind = S.kind[h.body];
  const float* m = &S.mat[4 * h.body];
  if (kind == RT_LAMBERTIAN || kind == RT_METAL) {
    float q[3], l2;
    do { q[0] = p.rng.sym(); q[1] = p.rng.sym(); q[2] = p.rng.sym(); l2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2]; ++tr.ball_tries; }
    while (!(l2 > 0.0f && l2 <= 1.0f));
    const float il = 1.0f / std::sqrt(l2);
    for (float& x : q) x *= il;
    if (kind == RT_LAMBERTIAN) {
      for (int a = 0; a < 3; ++a) p.d[a] = q[a] + n[a];
    } else {
      const float k2 = 2.0f * (p.d[0] * n[0] + p.d[1] * n[1] + p.d[2] * n[2]);
      float r[3];
      for (int a = 0; a < 3; ++a) r[a] = p.d[a] - n[a] * k2 + m[3] * q[a];
      if (!(r[0] * n[0] + r[1] * n[1] + r[2] * n[2] > 0.0f)) {
        tr.absorbed = 1;
        return true;
      }
      for (int a = 0; a < 3; ++a) p.d[a] = r[a];
    }
  } else {
    const float ri = front ? 1.0f / m[3] : m[3];
    const float un = u[0] * n[0] + u[1] * n[1] + u[2] * n[2];
    const float cosv = std::fmin(-un, 1.0f), sinv = std::sqrt(1.0f - cosv * cosv);
    bool refl = !(ri * sinv <= 1.0f);
    if (!refl) {
      const float xi = p.rng.u();
      float r0 = (1.0f - ri) / (1.0f + ri);
      r0 *= r0;
      const float x1 = 1.0f - cosv;
      refl = r0 + (1.0f - r0) * x1 * x1 * x1 * x1 * x1 > xi;
    }
    if (refl) {
      for (int a = 0; a < 3; ++a) p.d[a] = u[a] - n[a] * 2.0f * un;
    } else {
      float q[3];
      for (int a = 0; a < 3; ++a) q[a] = (u[a] + n[a] * cosv) * ri;
      const float par = -std::sqrt(std::fabs(1.0f - (q[0] * q[0] + q[1] * q[1] + q[2] * q[2])));
      for (int a = 0; a < 3; ++a) p.d[a] = q[a] + n[a] * par;
    }
  }
  return false;
}

// wave cost of one outer iteration over the lanes' segments
static double g_leaf_passes = 0, g_exact_passes = 0;
static int g_defer = 0;
static double wave_cost0(const std::vector<const Trav*>& lanes, double* node_steps);
static double wave_cost(const std::vector<const Trav*>& lanes0, double* node_steps) {
  if (!g_defer) return wave_cost0(lanes0, node_steps);
  // the second leaf of a two-leaf visit is pushed and popped at the next step
  // as a leaf-only step (its own single pass, shared with other lanes' first leaves)
  std::vector<Trav> tt(lanes0.size());
  std::vector<const Trav*> lanes;
  for (size_t k = 0; k < lanes0.size(); ++k) {
    const Trav& a = *lanes0[k];
    Trav& t = tt[k];
    t.disk_tries = a.disk_tries; t.ball_tries = a.ball_tries; t.absorbed = a.absorbed; t.big_c = a.big_c;
    for (size_t i = 0; i < a.leaves.size(); ++i) {
      if (a.leaves[i] == 2) {
        t.leaves.push_back(1); t.c1.push_back(a.c1[i]); t.c2.push_back(0);
        t.leaves.push_back(1); t.c1.push_back(a.c2[i]); t.c2.push_back(0);
      } else {
        t.leaves.push_back(a.leaves[i]); t.c1.push_back(a.c1[i]); t.c2.push_back(a.c2[i]);
      }
    }
    lanes.push_back(&t);
  }
  return wave_cost0(lanes, node_steps);
}
static double wave_cost0(const std::vector<const Trav*>& lanes, double* node_steps) {
  if (lanes.empty()) return 0.0;
  size_t L = 0;
  int mb = 0, ob = 0, md = 0, mball = 0, mboth = 0, anyabs = 0;
  for (const Trav* t : lanes) {
    md = std::max(md, t->disk_tries);
    mball = std::max(mball, t->ball_tries);
    mboth = std::max(mboth, std::max(t->disk_tries, t->ball_tries));
    anyabs |= t->absorbed;
    L = std::max(L, t->leaves.size());
    mb = std::max(mb, __builtin_popcount(t->big_c));
    ob |= t->big_c;
  }
  auto exact = [](int maxpop, int orm) {
    return g_exact_mode == 0 ? C_EXACT * maxpop : C_EXACT_B * __builtin_popcount(orm);
  };
  g_abs += anyabs;
  g_disk += md;
  g_ball += mball;
  g_both += mboth;
  double c = C_OUT + (g_big_leaves ? g_big_leaves * C_LEAF + exact(mb, ob) : 0.0);
  if (g_charge_rej) c += C_BALL * mball + C_DISK * md;
  for (size_t i = 0; i < L; ++i) {
    int ml = 0, m1 = 0, m2 = 0, o1 = 0, o2 = 0;
    for (const Trav* t : lanes)
      if (i < t->leaves.size()) {
        ml = std::max<int>(ml, t->leaves[i]);
        m1 = std::max<int>(m1, __builtin_popcount(t->c1[i]));
        m2 = std::max<int>(m2, __builtin_popcount(t->c2[i]));
        o1 |= t->c1[i];
        o2 |= t->c2[i];
      }
    c += C_NODE + C_LEAF * ml + exact(m1, o1) + exact(m2, o2);
    g_leaf_passes += ml;
    g_exact_passes += g_exact_mode == 0 ? m1 + m2 : __builtin_popcount(o1) + __builtin_popcount(o2);
  }
  *node_steps += double(L);
  return c;
}

struct Result { double cost = 0, iters = 0, steps = 0, samples = 0, lane_steps = 0; };

// one workgroup tile (8x8 pixels at (tx, ty)) under a policy
static void run_tile(const Ctx& C, int tx, int ty, int policy, int key_mode, Result& R) {
  const int npx = 64 * g_tile_h / 8, pool = npx * C.spp;   // 8 x g_tile_h pixels
  const int NL = 64 * g_nw;
  std::vector<Path> lanes(NL);
  int next = 0;
  for (int l = 0; l < NL; ++l) lanes[l].j = next < pool ? next++ : -1;
  auto pixel = [&](int j, int& px, int& py) {
    const int q = j / C.spp;
    px = tx * 8 + q % 8;
    py = ty * g_tile_h + q / 8;
  };
  R.samples += pool;
  if (policy == 2) {
    // lane-level restart: the wave steps the traversal of its lanes until
    // g_restart_k of them (or all live ones) have finished it, then shades
    // those lanes and sets up their next segment (camera ray if the path
    // ended); the others keep their traversal state across the phase
    struct L { Trav t; size_t i = 0; bool ended = false, live = false; };
    std::vector<L> st(NL);
    auto setup = [&](int l) {   // trace lane l's next segment (shading applied at its end)
      Path& p = lanes[l];
      st[l] = L{};
      if (p.j < 0) return;
      int px, py;
      pixel(p.j, px, py);
      st[l].ended = step(C, p, px, py, st[l].t);
      st[l].live = true;
    };
    for (int l = 0; l < NL; ++l) setup(l);
    std::vector<double> wc(g_nw, 0.0);
    for (int k = 0; k < g_nw; ++k) {   // first phase: the camera rays' set-up
      int md = 0, mb = 0, ob = 0;
      for (int l = 64 * k; l < 64 * k + 64; ++l)
        if (st[l].live) {
          md = std::max(md, st[l].t.disk_tries);
          mb = std::max(mb, __builtin_popcount(st[l].t.big_c));
          ob |= st[l].t.big_c;
        }
      wc[k] += C_OUT * 0.5 + C_DISK * md + (g_big_leaves ? g_big_leaves * C_LEAF + C_EXACT * mb : 0.0);
    }
    for (;;) {
      int w = -1;
      for (int k = 0; k < g_nw; ++k) {
        bool any = false;
        for (int l = 0; l < 64; ++l) any |= st[64 * k + l].live;
        if (any && (w < 0 || wc[k] < wc[w])) w = k;
      }
      if (w < 0) break;
      L* ln = &st[64 * w];
      int nlive = 0, nready = 0;
      for (int l = 0; l < 64; ++l) {
        nlive += ln[l].live;
        nready += ln[l].live && ln[l].i >= ln[l].t.leaves.size();
      }
      const int K = std::min(g_restart_k, nlive);
      double c = 0;
      while (nready < K) {
        int ml = 0, m1 = 0, m2 = 0, trav = 0;
        for (int l = 0; l < 64; ++l) {
          L& x = ln[l];
          if (!x.live || x.i >= x.t.leaves.size()) continue;
          ++trav;
          ml = std::max<int>(ml, x.t.leaves[x.i]);
          m1 = std::max(m1, __builtin_popcount(x.t.c1[x.i]));
          m2 = std::max(m2, __builtin_popcount(x.t.c2[x.i]));
          ++x.i;
          R.lane_steps += 1;
          if (x.i >= x.t.leaves.size()) ++nready;
        }
        c += C_NODE + 4 + C_LEAF * ml + C_EXACT * (m1 + m2);   // +4: the ready-count ballot
        R.steps += 1;
        g_leaf_passes += ml;
        g_exact_passes += m1 + m2;
      }
      // shading phase of the ready lanes, then their next segments' set-up
      int mball = 0, md = 0, mb = 0, ob = 0;
      for (int l = 0; l < 64; ++l) {
        L& x = ln[l];
        if (!x.live || x.i < x.t.leaves.size()) continue;
        mball = std::max(mball, x.t.ball_tries);
        const int gl = 64 * w + l;
        if (x.ended) {
          lanes[gl] = Path{};
          lanes[gl].j = next < pool ? next++ : -1;
        }
        setup(gl);
        if (st[gl].live) {
          md = std::max(md, st[gl].t.disk_tries);
          mb = std::max(mb, __builtin_popcount(st[gl].t.big_c));
          ob |= st[gl].t.big_c;
        }
      }
      g_ball += mball;
      g_disk += md;
      c += C_OUT + C_BALL * mball + C_DISK * md + (g_big_leaves ? g_big_leaves * C_LEAF + C_EXACT * mb : 0.0);
      wc[w] += c;
      R.cost += c;
      R.iters += 1;
    }
    return;
  }
  if (policy == 3) {
    // R paths per lane (lanes [l], [l + NL]...): one loop walks the lane's
    // segments back to back, then all are shaded
    const int R2 = g_pair;
    std::vector<Path> more(NL * (R2 - 1));
    for (auto& p : more) p.j = next < pool ? next++ : -1;
    auto P = [&](int l, int r) -> Path& { return r == 0 ? lanes[l] : more[(r - 1) * NL + l]; };
    std::vector<double> wc(g_nw, 0.0);
    for (;;) {
      int w = -1;
      for (int k = 0; k < g_nw; ++k) {
        bool any = false;
        for (int l = 0; l < 64; ++l) for (int r = 0; r < R2; ++r) any |= P(64 * k + l, r).j >= 0;
        if (any && (w < 0 || wc[k] < wc[w])) w = k;
      }
      if (w < 0) break;
      std::vector<Trav> comb(64);
      std::vector<const Trav*> act;
      int nseg_max = 0;
      for (int l = 0; l < 64; ++l) {
        int ns = 0;
        for (int r = 0; r < R2; ++r) {
          Path& p = P(64 * w + l, r);
          if (p.j < 0) continue;
          int px, py;
          pixel(p.j, px, py);
          Trav t;
          const bool end = step(C, p, px, py, t);
          ++ns;
          Trav& c = comb[l];
          c.leaves.insert(c.leaves.end(), t.leaves.begin(), t.leaves.end());
          c.c1.insert(c.c1.end(), t.c1.begin(), t.c1.end());
          c.c2.insert(c.c2.end(), t.c2.begin(), t.c2.end());
          c.big_c |= t.big_c;
          R.lane_steps += t.leaves.size();
          if (end) { p = Path{}; p.j = next < pool ? next++ : -1; }
        }
        nseg_max = std::max(nseg_max, ns);
        if (ns) act.push_back(&comb[l]);
      }
      double c = wave_cost(act, &R.steps);
      // outer work (camera/setup/shading) and the big-body leaf once per path slot in use
      c += (nseg_max - 1) * (C_OUT + (g_big_leaves ? g_big_leaves * C_LEAF : 0.0));
      wc[w] += c;
      R.cost += c;
      R.iters += 1;
    }
    return;
  }
  if (policy == 0) {
    // 4 independent waves, advanced in order of accumulated cost
    std::vector<double> wc(g_nw, 0.0);
    for (;;) {
      int w = -1;
      for (int k = 0; k < g_nw; ++k) {
        bool any = false;
        for (int l = 0; l < 64; ++l) any |= lanes[64 * k + l].j >= 0;
        if (any && (w < 0 || wc[k] < wc[w])) w = k;
      }
      if (w < 0) break;
      std::vector<Trav> tr(64);
      std::vector<const Trav*> act;
      std::vector<int> done;
      if (g_qt == 2) {   // probe pass on copies: the wave's common start node
        int ref[2] = {-1, -1};
        unsigned xo = 0;
        g_probe = true;
        for (int l = 0; l < 64; ++l) {
          Path cp = lanes[64 * w + l];
          if (cp.j < 0) continue;
          int px, py;
          pixel(cp.j, px, py);
          Trav t;
          g_probe_valid = 0;
          step(C, cp, px, py, t);
          if (!g_probe_valid) continue;
          if (ref[0] < 0) { ref[0] = g_probe_c[0]; ref[1] = g_probe_c[1]; }
          xo |= unsigned(g_probe_c[0] ^ ref[0]) | unsigned(g_probe_c[2] ^ ref[0]) |
                unsigned(g_probe_c[1] ^ ref[1]) | unsigned(g_probe_c[3] ^ ref[1]);
        }
        g_probe = false;
        const int lvl = xo ? 32 - __builtin_clz(xo) : 0;
        g_force_start = 0;
        if (ref[0] >= 0 && lvl < int(g_qt_tab.size())) {
          const int res = g_qt_res >> lvl;
          g_force_start = g_qt_tab[lvl][(ref[1] >> lvl) * res + (ref[0] >> lvl)];
        }
        wc[w] += C_QT;
        R.cost += C_QT;
      }
      for (int l = 0; l < 64; ++l) {
        Path& p = lanes[64 * w + l];
        if (p.j < 0) continue;
        int px, py;
        pixel(p.j, px, py);
        if (step(C, p, px, py, tr[l])) done.push_back(l);
        act.push_back(&tr[l]);
        R.lane_steps += tr[l].leaves.size();
      }
      const double c = wave_cost(act, &R.steps);
      wc[w] += c;
      R.cost += c;
      R.iters += 1;
      for (int l : done) {
        Path& p = lanes[64 * w + l];
        p = Path{};
        p.j = next < pool ? next++ : -1;
      }
    }
  } else {
    // all 256 lanes step together; paths dealt to waves sorted by key
    for (;;) {
      std::vector<int> live;
      for (int l = 0; l < NL; ++l)
        if (lanes[l].j >= 0) live.push_back(l);
      if (live.empty()) break;
      std::vector<int> oracle_len(NL, 0);
      if (key_mode == 3)   // upper bound: the segment's own visit count (traced on a copy)
        for (int l : live) {
          Path cp = lanes[l];
          Trav t;
          int px, py;
          pixel(cp.j, px, py);
          step(C, cp, px, py, t);
          oracle_len[l] = int(t.leaves.size());
        }
      auto key = [&](const Path& p) -> int {
        if (key_mode == 3) return oracle_len[&p - lanes.data()];
        if (key_mode == 4) return 0;   // compaction only
        if (p.fresh) return 0;   // camera rays first (coherent already)
        const int oct = (p.d[0] < 0) | ((p.d[1] < 0) << 1) | ((p.d[2] < 0) << 2);
        if (key_mode == 1) return 1 + oct;
        if (key_mode == 2) return 1 + oct * 64 + ((p.last & 63));  // octant, then the body left
        return 1 + oct;
      };
      std::stable_sort(live.begin(), live.end(), [&](int a, int b) { return key(lanes[a]) < key(lanes[b]); });
      std::vector<Trav> tr(NL);
      std::vector<int> done;
      for (size_t w = 0; w * 64 < live.size(); ++w) {
        std::vector<const Trav*> act;
        for (size_t i = w * 64; i < std::min(live.size(), w * 64 + 64); ++i) {
          const int l = live[i];
          Path& p = lanes[l];
          int px, py;
          pixel(p.j, px, py);
          if (step(C, p, px, py, tr[l])) done.push_back(l);
          act.push_back(&tr[l]);
          R.lane_steps += tr[l].leaves.size();
        }
        R.cost += wave_cost(act, &R.steps) + C_SORT + C_XCHG;
        R.iters += 1;
      }
      for (int l : done) {
        lanes[l] = Path{};
        lanes[l].j = next < pool ? next++ : -1;
      }
    }
  }
}

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? std::atoi(argv[1]) : 300;
  const int spp = argc > 2 ? std::atoi(argv[2]) : 100;
  Scene S;
  S.n = rt_scene_cover(11, 42, nullptr, nullptr, nullptr, 0);
  S.sph.resize(4 * S.n);
  S.mat.resize(4 * S.n);
  S.kind.resize(S.n);
  rt_scene_cover(11, 42, S.sph.data(), S.kind.data(), S.mat.data(), S.n);
  if (std::getenv("BIG")) g_bvh_big_ratio = std::atof(std::getenv("BIG"));
  if (std::getenv("PAD")) g_pad = std::atof(std::getenv("PAD"));
  if (std::getenv("EXACT")) g_exact_mode = std::atoi(std::getenv("EXACT"));

  const int ls = std::getenv("LS") ? std::atoi(std::getenv("LS")) : 4;
  bvh_build(S.sph.data(), S.n, &S.t, ls, true);
  set_leaf_costs(ls / 2);
  g_big_leaves = S.t.n_big_leaves;
  if (std::getenv("QT")) {
    g_qt = std::atoi(std::getenv("QT"));
    if (std::getenv("QTR")) g_qt_res = std::atoi(std::getenv("QTR"));
    if (std::getenv("QTM")) g_qt_m = std::atof(std::getenv("QTM"));
    const int nn = int(S.t.nodes.size());
    std::vector<int> parent(nn, -1), depth(nn, 0);
    std::vector<int> holder(S.n, -1);
    const int np = S.t.leaf_size / 2;
    for (int i = 0; i < nn; ++i)
      for (int c = 0; c < 2; ++c) {
        const int ch = S.t.nodes[i].child[c];
        if (ch >= 0) parent[ch] = i;
        else
          for (int q = 0; q < np; ++q)
            for (int j = 0; j < 2; ++j) {
              const int id = S.t.pidx[2 * (~ch + q) + j];
              if (id >= 0) holder[id] = i;
            }
      }
    for (int i = 1; i < nn; ++i) { int d = 0; for (int k = i; k > 0; k = parent[k]) ++d; depth[i] = d; }
    auto lca = [&](int a, int b) {
      if (a < 0) return b;
      while (depth[a] > depth[b]) a = parent[a];
      while (depth[b] > depth[a]) b = parent[b];
      while (a != b) { a = parent[a]; b = parent[b]; }
      return a;
    };
    float lo[2] = {INFINITY, INFINITY}, hi[2] = {-INFINITY, -INFINITY};
    for (int i = 0; i < S.n; ++i) {
      if (holder[i] < 0) continue;
      const float* b = &S.sph[4 * i];
      lo[0] = std::min(lo[0], b[0] - b[3] - S.t.center[0]); hi[0] = std::max(hi[0], b[0] + b[3] - S.t.center[0]);
      lo[1] = std::min(lo[1], b[2] - b[3] - S.t.center[2]); hi[1] = std::max(hi[1], b[2] + b[3] - S.t.center[2]);
    }
    for (int k = 0; k < 2; ++k) {
      g_qt_lo[k] = lo[k] - g_qt_m;
      g_qt_cell[k] = (hi[k] - lo[k] + 2 * g_qt_m) / g_qt_res;
    }
    for (int res = g_qt_res, lvl = 0; res >= 1; res >>= 1, ++lvl) {
      std::vector<int> tab(res * res, -2);
      const float cw = g_qt_cell[0] * (g_qt_res / res), ch = g_qt_cell[1] * (g_qt_res / res);
      for (int i = 0; i < S.n; ++i) {
        if (holder[i] < 0) continue;
        const float* b = &S.sph[4 * i];
        const float bx0 = b[0] - b[3] - S.t.center[0] - g_qt_m, bx1 = b[0] + b[3] - S.t.center[0] + g_qt_m;
        const float bz0 = b[2] - b[3] - S.t.center[2] - g_qt_m, bz1 = b[2] + b[3] - S.t.center[2] + g_qt_m;
        const int x0 = std::max(0, int(std::floor((bx0 - g_qt_lo[0]) / cw))), x1 = std::min(res - 1, int(std::floor((bx1 - g_qt_lo[0]) / cw)));
        const int z0 = std::max(0, int(std::floor((bz0 - g_qt_lo[1]) / ch))), z1 = std::min(res - 1, int(std::floor((bz1 - g_qt_lo[1]) / ch)));
        for (int z = z0; z <= z1; ++z)
          for (int x = x0; x <= x1; ++x) {
            int& t = tab[z * res + x];
            t = lca(t == -2 ? -1 : t, holder[i]);
          }
      }
      double dsum = 0; int ne = 0;
      for (int t : tab) if (t >= 0) { dsum += depth[t]; ++ne; }
      std::printf("qt level %d (%dx%d): %d non-empty cells, mean start depth %.2f\n", lvl, res, res, ne, ne ? dsum / ne : 0.0);
      g_qt_tab.push_back(tab);
    }
  }
  std::printf("tree: %zu nodes, depth %d, big %zu\n", S.t.nodes.size(), S.t.depth, S.t.big.size());
  Ctx C{&S, {}, 1200, spp, 50};
  const double lf[3] = {13, 2, 3}, la[3] = {0, 0, 0}, vup[3] = {0, 1, 0};
  rt_camera_setup(1200, 675, 20.0, lf, la, vup, 0.6, 10.0, &C.cam);
  if (std::getenv("TILEH")) g_tile_h = std::atoi(std::getenv("TILEH"));
  if (std::getenv("NW")) g_nw = std::atoi(std::getenv("NW"));
  if (std::getenv("XCHG")) C_XCHG = std::atof(std::getenv("XCHG"));
  if (std::getenv("CSORT")) C_SORT = std::atof(std::getenv("CSORT"));
  const int gx = 1200 / 8, gy = (675 + g_tile_h - 1) / g_tile_h;
  std::vector<int> pick;
  uint32_t h = 12345;
  for (int i = 0; i < tiles; ++i) {
    h = mix32(h + 1);
    pick.push_back(int(h % uint32_t(gx * (gy - 1))));
  }
  const char* names[] = {"wave (shipped)", "sort by octant", "sort by octant+body", "sort by visits (bound)",
                         "restart (RK lanes)", "compact (no sort)", "paths per lane (PAIR)"};
  const int pol[] = {0, 1, 1, 1, 2, 1, 3}, km[] = {0, 1, 2, 3, 0, 4, 0};
  if (std::getenv("DEFER")) g_defer = std::atoi(std::getenv("DEFER"));
  if (std::getenv("CNODE")) C_NODE = std::atof(std::getenv("CNODE"));
  if (std::getenv("PAIR")) g_pair = std::atoi(std::getenv("PAIR"));
  if (std::getenv("RJ")) g_charge_rej = std::atoi(std::getenv("RJ"));
  if (std::getenv("RK")) g_restart_k = std::atoi(std::getenv("RK"));
  const int v0 = std::getenv("V0") ? std::atoi(std::getenv("V0")) : 0;
  const int nv = std::getenv("NV") ? std::atoi(std::getenv("NV")) : 4;
  for (int v = v0; v < nv; ++v) {
    if (pol[v] == 1 && std::getenv("NOSORT")) continue;
    Result R;
    g_leaf_passes = g_exact_passes = 0;
    for (int t : pick) run_tile(C, t % gx, t / gx, pol[v], km[v], R);
    std::printf("  per wave-iter: node steps %.2f leaf passes %.2f exact passes %.2f  (cost shares: outer %.2f node %.2f leaf %.2f exact %.2f)\n",
                R.steps / R.iters, g_leaf_passes / R.iters, g_exact_passes / R.iters,
                C_OUT * R.iters / R.cost, C_NODE * R.steps / R.cost, C_LEAF * g_leaf_passes / R.cost,
                C_EXACT * g_exact_passes / R.cost);
    std::printf("  rejection loops per wave-iter: disk %.2f ball %.2f (one merged loop: %.2f); absorption in %.3f of wave-iters\n",
                g_disk / R.iters, g_ball / R.iters, g_both / R.iters, g_abs / R.iters);
    g_disk = g_ball = g_both = g_abs = 0;
    if (g_qt) { std::printf("  qt: %.3f of segments skip the tree\n", g_qt_skip / g_qt_n); g_qt_skip = g_qt_n = 0; }
    std::printf("  candidates rejected by the t bound: %.3f of %.0f; per segment: %.2f node visits, %.2f leaves\n",
                g_rej / g_cand, g_cand, g_visits / g_segs, g_leafs / g_segs);
    g_rej = g_cand = g_segs = g_visits = g_leafs = 0;
    std::printf("%-22s cost/sample %8.1f  wave-iters/sample %.3f  trav steps/wave-iter %.2f  lane eff %.3f\n",
                names[v], R.cost / R.samples, R.iters / R.samples * 64, R.steps / R.iters,
                R.lane_steps / (R.steps * 64));
  }
  return 0;
}
