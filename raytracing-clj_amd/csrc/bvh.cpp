// bvh.cpp — host-side bounding-volume hierarchy over the scene's bodies, for
// the kernel's BVH traversal variant (trace.hip, SCAN_BVH).
//
// It replaces nothing in the reference: the reference's hit-anything
// (src/raytracing.clj:33-43) is a linear scan, and the traversal is built so
// that the hit it returns is the scan's, bit for bit:
//   * every body keeps its original index; the traversal accepts a closer t,
//     or an equal t of a lower index (the scan's strict `t < closest` in
//     array order picks the lowest index among equal t);
//   * the body test itself is the scan's fp32 op sequence;
//   * boxes are culled only conservatively (per-ray padding, trace.hip).
// "Big" bodies (up to kBvhBigMax bodies of radius > 4 x the median, e.g. the
// r = 1000 ground and the cover scene's three r = 1 spheres) would make the
// boxes around them loose; they are kept out of the tree and tested as extra
// leaves before every traversal (a 4-body leaf costs the wave about what one
// scalar body test did, tools/simt_sim.cpp priced the tighter tree at -15 %).
//
// Layout (device, all 16-byte aligned):
//   nodes[n_nodes]   BvhNode: child boxes as (c0, c1) float pairs for packed
//                    slab tests, per axis (min, max, min) so a ray reads its
//                    (near, far) planes without ordering them, relative to
//                    the tree centre; child refs: >= 0 node, < 0 leaf ~pair
//                    (every child is real: small trees repeat a leaf / use a
//                    pad leaf)
//   pairs[n_pairs]   two bodies per pair: x0 x1 y0 y1 z0 z1 w0 w1 (w = -r^2;
//                    a missing body has w = +inf: never a candidate); a leaf
//                    is 1 pair (leaf_size 2) or 2 consecutive pairs (4)
//   pidx[n_pairs]    original indices of the two bodies (-1 for the pad)
//   the big bodies' leaves follow the tree's in pairs / pidx (big_pair0,
//   n_big_leaves)
#include "bvh.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <numeric>

namespace rtclj {

float g_bvh_big_ratio = 4.0f;    // big-body threshold (x the median radius); tools/simt_sim.cpp

namespace {

struct Box {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void add(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
};

// exact float box of a body, rounded outward
Box body_box(const float* s) {
  Box b;
  const float r = std::fabs(s[3]);
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = std::nextafter(s[k] - r, -INFINITY);
    b.hi[k] = std::nextafter(s[k] + r, INFINITY);
  }
  return b;
}

// child c's box into node n: per axis (min, max, min) pairs (bvh.h)
void set_box(BvhNode& n, int c, const Box& b) {
  float* ax[3] = {n.x, n.y, n.z};
  for (int k = 0; k < 3; ++k) {
    ax[k][c] = b.lo[k];
    ax[k][2 + c] = b.hi[k];
    ax[k][4 + c] = b.lo[k];
  }
}

struct Builder {
  const float* sph;
  std::vector<int> prim;   // original indices, permuted during the build
  BvhHost* out;
  int max_depth = 0;

  int leaf_size = 2;       // bodies per leaf: 2, 4 or 8 (1, 2 or 4 pairs)

  int leaf(int lo, int cnt, Box* box) {
    const int p = static_cast<int>(out->pidx.size() / 2);
    for (int q = 0; q < leaf_size / 2; ++q) {
      float pair[8] = {0, 0, 0, 0, 0, 0, INFINITY, INFINITY};
      int idx[2] = {-1, -1};
      for (int j = 0; j < 2; ++j) {
        const int k = 2 * q + j;
        if (k >= cnt) break;
        const float* s = sph + 4 * prim[lo + k];
        pair[0 + j] = s[0];
        pair[2 + j] = s[1];
        pair[4 + j] = s[2];
        pair[6 + j] = -(s[3] * s[3]);
        idx[j] = prim[lo + k];
        box->add(body_box(s));
      }
      out->pairs.insert(out->pairs.end(), pair, pair + 8);
      out->pidx.push_back(idx[0]);
      out->pidx.push_back(idx[1]);
    }
    return ~p;   // < 0: leaf (its first pair)
  }

  bool sah = true;          // surface-area split (else median)

  static double area(const Box& b) {
    const double dx = double(b.hi[0]) - b.lo[0], dy = double(b.hi[1]) - b.lo[1], dz = double(b.hi[2]) - b.lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }

  // orders prim[lo, hi) and returns the split point: the surface-area
  // heuristic (cost = sum over the two sides of box area x leaf count, all
  // cut points on all three axes) while the remaining depth allows, else the
  // median of the widest centroid extent on a leaf-size boundary
  int split(int lo, int hi, int depth) {
    const int cnt = hi - lo, L = leaf_size;
    auto by_axis = [&](int axis) {
      return [this, axis](int a, int b) {
        const float ca = sph[4 * a + axis], cb = sph[4 * b + axis];
        return ca < cb || (ca == cb && a < b);
      };
    };
    // levels a median split below here would still need
    int need = 0;
    for (int leaves = (cnt + L - 1) / L; leaves > 1; leaves = (leaves + 1) / 2) ++need;
    if (sah && depth + need + 3 <= kBvhStack - 2) {
      double best = INFINITY;
      int best_axis = 0, best_i = cnt / 2;
      std::vector<int> ord(prim.begin() + lo, prim.begin() + hi);
      std::vector<double> right(cnt + 1, 0.0);
      for (int axis = 0; axis < 3; ++axis) {
        std::sort(ord.begin(), ord.end(), by_axis(axis));
        Box r;
        for (int i = cnt - 1; i >= 1; --i) {
          r.add(body_box(sph + 4 * ord[i]));
          right[i] = area(r) * ((cnt - i + L - 1) / L);
        }
        Box l;
        for (int i = 1; i < cnt; ++i) {
          l.add(body_box(sph + 4 * ord[i - 1]));
          const double c = area(l) * ((i + L - 1) / L) + right[i];
          if (c < best) {
            best = c;
            best_axis = axis;
            best_i = i;
          }
        }
      }
      std::sort(prim.begin() + lo, prim.begin() + hi, by_axis(best_axis));
      return lo + best_i;
    }
    Box cb;  // centroid bounds
    for (int i = lo; i < hi; ++i) {
      const float* s = sph + 4 * prim[i];
      for (int k = 0; k < 3; ++k) {
        cb.lo[k] = std::min(cb.lo[k], s[k]);
        cb.hi[k] = std::max(cb.hi[k], s[k]);
      }
    }
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
    // median split on a leaf-size boundary: balanced depth, full leaves
    int mid = lo + ((cnt / 2 + L / 2) / L) * L;
    if (mid <= lo) mid = lo + L;
    if (mid >= hi) mid = hi - 1;
    std::nth_element(prim.begin() + lo, prim.begin() + mid, prim.begin() + hi, by_axis(axis));
    return mid;
  }

  // returns a child ref (node index >= 0, or ~leaf) and its box
  int build(int lo, int hi, int depth, Box* box) {
    max_depth = std::max(max_depth, depth);
    const int cnt = hi - lo;
    if (cnt <= leaf_size) return leaf(lo, cnt, box);
    const int mid = split(lo, hi, depth);
    const int me = static_cast<int>(out->nodes.size());
    out->nodes.emplace_back();
    Box b0, b1;
    const int c0 = build(lo, mid, depth + 1, &b0);
    const int c1 = build(mid, hi, depth + 1, &b1);
    BvhNode& n = out->nodes[me];
    set_box(n, 0, b0);
    set_box(n, 1, b1);
    n.child[0] = c0;
    n.child[1] = c1;
    box->add(b0);
    box->add(b1);
    return me;
  }
};

}  // namespace

int bvh_build(const float* sph, int n, BvhHost* out, int leaf_size, bool sah) {
  *out = BvhHost{};
  if (leaf_size != 2 && leaf_size != 4 && leaf_size != 8) leaf_size = 2;
  out->leaf_size = leaf_size;
  // big bodies: scanned first, outside the tree
  std::vector<float> radii;
  for (int i = 0; i < n; ++i) radii.push_back(std::fabs(sph[4 * i + 3]));
  float med = 0.0f;
  if (n > 0) {
    std::vector<float> tmp = radii;
    std::nth_element(tmp.begin(), tmp.begin() + n / 2, tmp.end());
    med = tmp[n / 2];
  }
  Builder b{sph, {}, out};
  b.leaf_size = leaf_size;
  b.sah = sah;
  // non-finite bodies (no box) and the kBvhBigMax largest bodies of radius >
  // g_bvh_big_ratio x the median (the r = 1000 ground, the cover scene's three
  // r = 1 spheres: their boxes would enclose many small bodies' boxes)
  std::vector<char> is_big(n, 0);
  for (int i = 0; i < n; ++i) {
    const bool finite = std::isfinite(sph[4 * i]) && std::isfinite(sph[4 * i + 1]) &&
                        std::isfinite(sph[4 * i + 2]) && std::isfinite(sph[4 * i + 3]);
    if (!finite && out->big.size() < 64) {
      is_big[i] = 1;
      out->big.push_back(i);
    }
  }
  if (n > 8) {
    std::vector<int> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return radii[x] > radii[y]; });
    int added = 0;
    for (int i : order) {
      if (added == kBvhBigMax || !(radii[i] > g_bvh_big_ratio * med)) break;
      if (is_big[i]) continue;
      is_big[i] = 1;
      out->big.push_back(i);
      ++added;
    }
  }
  std::sort(out->big.begin(), out->big.end());
  for (int i = 0; i < n; ++i)
    if (!is_big[i]) b.prim.push_back(i);
  // bounding sphere of the tree's bodies (centre of their box, radius to the
  // farthest surface): D = |O - centre| + radius bounds |oc| + r per ray
  Box all;
  for (int i : b.prim) all.add(body_box(sph + 4 * i));
  double bc[3] = {0, 0, 0}, br = 0;
  if (!b.prim.empty()) {
    for (int k = 0; k < 3; ++k) bc[k] = 0.5 * (double(all.lo[k]) + all.hi[k]);
    for (int i : b.prim) {
      const float* s = sph + 4 * i;
      const double dx = s[0] - bc[0], dy = s[1] - bc[1], dz = s[2] - bc[2];
      br = std::max(br, std::sqrt(dx * dx + dy * dy + dz * dz) + std::fabs(s[3]));
    }
  }
  for (int k = 0; k < 3; ++k) out->center[k] = static_cast<float>(bc[k]);
  out->radius = static_cast<float>(br * (1.0 + 1e-6)) + 1e-6f;
  // root is always node 0 with two children (a leaf-only tree gets a root)
  out->nodes.emplace_back();
  const int cnt = static_cast<int>(b.prim.size());
  Box b0, b1;
  int c0 = 0, c1 = 0;
  if (cnt == 0) {
    // no tree bodies: both children are one pad-only leaf (never a candidate)
    c0 = c1 = b.leaf(0, 0, &b0);
    for (int k = 0; k < 3; ++k) b0.lo[k] = b0.hi[k] = 0.0f;
    b1 = b0;
  } else if (cnt <= leaf_size) {
    c0 = c1 = b.leaf(0, cnt, &b0);   // the same leaf twice: a repeat test never wins a tie
    b1 = b0;
  } else {
    // the root splits by the same rule as build()
    const int mid = b.split(0, cnt, 0);
    c0 = b.build(0, mid, 1, &b0);
    c1 = b.build(mid, cnt, 1, &b1);
  }
  BvhNode& root = out->nodes[0];
  set_box(root, 0, b0);
  set_box(root, 1, b1);
  root.child[0] = c0;
  root.child[1] = c1;
  // every node box relative to the centre, in double, rounded outward: the
  // kernel's slab test is then one fma per bound with a small rounding error
  for (BvhNode& nd : out->nodes) {
    float* ax[3] = {nd.x, nd.y, nd.z};
    for (int k = 0; k < 3; ++k)
      for (int c = 0; c < 2; ++c) {
        ax[k][c] = std::nextafter(static_cast<float>(double(ax[k][c]) - out->center[k]), -INFINITY);
        ax[k][2 + c] = std::nextafter(static_cast<float>(double(ax[k][2 + c]) - out->center[k]), INFINITY);
        ax[k][4 + c] = ax[k][c];
      }
  }
  out->depth = b.max_depth + 1;
  // the big bodies as leaves after the tree's (same pair layout, padded with
  // never-hit bodies): the kernel tests them with the leaf test, every segment
  out->big_pair0 = static_cast<int>(out->pidx.size() / 2);
  const int nb = static_cast<int>(out->big.size());
  b.prim.insert(b.prim.end(), out->big.begin(), out->big.end());
  for (int q = 0; q < nb; q += leaf_size) {
    Box unused;
    b.leaf(cnt + q, std::min(leaf_size, nb - q), &unused);
    ++out->n_big_leaves;
  }
  return 0;
}

}  // namespace rtclj
