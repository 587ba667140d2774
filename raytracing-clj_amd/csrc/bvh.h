// bvh.h — host BVH build for the traversal variant (see bvh.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace rtclj {

// 64 bytes: two child boxes in (child0, child1) float pairs + child refs
struct alignas(16) BvhNode {
  float minx[2], miny[2], minz[2];
  float maxx[2], maxy[2], maxz[2];
  int child[2];   // >= 0: node, < 0: ~leaf pair index
  int pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode layout");

struct BvhHost {
  std::vector<BvhNode> nodes;
  std::vector<float> pairs;   // 8 floats per leaf pair
  std::vector<int> pidx;      // 2 original indices per leaf pair (-1: pad)
  std::vector<int> big;       // bodies scanned before the traversal, ascending
  float center[3] = {0, 0, 0};
  float radius = 0.0f;        // bounding sphere of the tree's bodies
  int depth = 0;              // levels of nodes on the longest root-leaf path
  int leaf_size = 2;          // bodies per leaf (2: one pair, 4: two pairs)
};

int bvh_build(const float* sphere, int n, BvhHost* out, int leaf_size = 2);

// traversal stack entries per lane (node indices); trees are median-split, so
// depth <= ceil(log2(n/2)) + 1 (13 for 8192 bodies)
constexpr int kBvhStack = 16;

}  // namespace rtclj
