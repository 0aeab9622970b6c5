// bvh_build.h — BBox-tree builders for the device scene.
#pragma once

#include <stdint.h>

#include <vector>

namespace rt {

struct Box {
  double mn[3], mx[3];
};

// Binary tree over leaf objects; one object per leaf like the reference (bbox_tree.rs:10-20).
struct BuildNode {
  Box box;
  int32_t leaf;  // object index for a leaf, -1 for a branch
  int32_t lhs, rhs;
};

struct BuiltTree {
  std::vector<BuildNode> nodes;
  int32_t root = -1;  // -1: empty tree
};

// Reference rules (bvh/bbox_tree/constructor.rs:9-212): six candidate splits per node (median and
// spatial midpoint over objects sorted by bbox.min on x, y, z), score = sum of the two child boxes'
// volumes (Aabb::area, aabb.rs:81-86), first minimum wins.  The reference rescans full sorted
// arrays through HashSets (O(N^2)); this keeps per-node sorted sub-lists instead (O(N log N) for
// balanced splits) and produces the same tree (ties in the reference's unstable sort broken by index).
BuiltTree build_reference_tree(const std::vector<Box>& boxes);

// Surface-area-heuristic tree (performance option).  sweep = true: exact SAH, every centroid
// boundary on every axis (the library's choice: +2.4 % on random_scene, +2-4 % on gen_spheres);
// false: 32 centroid bins.  Objects whose box can never pass the slab test (min > max on an axis:
// the reference's negative-radius spheres, sphere.rs:54-60) are left out; every other object keeps
// its own box as its leaf box.
// weight (sweep only): per-object test cost in the split cost, sum over a side instead of its count.
BuiltTree build_sah_tree(const std::vector<Box>& boxes, bool sweep = false, const std::vector<double>* weight = nullptr);

// Max number of branch nodes on a root-to-leaf path.
int32_t tree_branch_depth(const BuiltTree& t);

// fp.rs:3-28 NaN-aware min / max, aabb.rs:18-33 surrounding_box
double fmin_nan(double a, double b);
double fmax_nan(double a, double b);
Box surrounding(const Box& a, const Box& b);

}  // namespace rt
