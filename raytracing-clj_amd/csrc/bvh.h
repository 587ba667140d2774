// bvh.h — host BVH build for the traversal variant (see bvh.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace rtclj {

// 80 bytes: the two child boxes, per axis as the (child0, child1) float
// pairs (min, max, min), so a ray reads its (near, far) planes of an axis as
// two consecutive pairs -- at offset 0 (1/u >= 0) or 8 (1/u < 0) -- and needs
// no min/max to order them; then the child refs
struct alignas(16) BvhNode {
  float x[6], y[6], z[6];
  int child[2];   // >= 0: node, < 0: ~leaf pair index
};
static_assert(sizeof(BvhNode) == 80, "BvhNode layout");

struct BvhHost {
  std::vector<BvhNode> nodes;
  std::vector<float> pairs;   // 8 floats per leaf pair
  std::vector<int> pidx;      // 2 original indices per leaf pair (-1: pad)
  std::vector<int> big;       // bodies tested before the traversal, ascending
  int big_pair0 = 0;          // their leaves: pairs [big_pair0, + n_big_leaves x leaf pairs)
  int n_big_leaves = 0;
  float center[3] = {0, 0, 0};
  float radius = 0.0f;        // bounding sphere of the tree's bodies
  int depth = 0;              // levels of nodes on the longest root-leaf path
  int leaf_size = 2;          // bodies per leaf (2, 4 or 8: 1, 2 or 4 pairs)
};

// traversal stack entries per lane (node indices); the build keeps
// depth + 2 <= kBvhStack (surface-area splits where the depth allows, median
// splits below: depth <= ceil(log2(n/2)) + 1 = 13 for 8192 bodies)
constexpr int kBvhStack = 16;
// bodies kept out of the tree for their size (besides non-finite ones)
constexpr int kBvhBigMax = 8;

// sah: surface-area-heuristic splits (else median splits)
int bvh_build(const float* sphere, int n, BvhHost* out, int leaf_size = 2, bool sah = true);

}  // namespace rtclj
