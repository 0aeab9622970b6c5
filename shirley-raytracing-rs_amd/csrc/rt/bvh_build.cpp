// bvh_build.cpp — reference-rule and SAH BBox-tree builders (host side of the C ABI).
#include "bvh_build.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <numeric>

namespace rt {

double fmin_nan(double a, double b) {
  if (std::isnan(a) || std::isnan(b)) return std::isnan(a) ? b : a;
  return (a < b) ? a : b;
}
double fmax_nan(double a, double b) {
  if (std::isnan(a) || std::isnan(b)) return std::isnan(a) ? b : a;
  return (a > b) ? a : b;
}
Box surrounding(const Box& a, const Box& b) {
  Box o;
  for (int k = 0; k < 3; ++k) {
    o.mn[k] = fmin_nan(a.mn[k], b.mn[k]);
    o.mx[k] = fmax_nan(a.mx[k], b.mx[k]);
  }
  return o;
}

namespace {

// f64::total_cmp
int total_cmp(double a, double b) {
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
  ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
  return (ia < ib) ? -1 : (ia > ib ? 1 : 0);
}

// Aabb::area (aabb.rs:81-86) — the volume
double volume(const Box& b) {
  double x = b.mx[0] - b.mn[0], y = b.mx[1] - b.mn[1], z = b.mx[2] - b.mn[2];
  return x * y * z;
}

struct RefBuilder {
  const std::vector<Box>& boxes;
  std::vector<BuildNode> tree;
  std::vector<char> mark;

  explicit RefBuilder(const std::vector<Box>& b) : boxes(b), mark(b.size(), 0) {}

  // bounding() over a set (aabb.rs:6-16): union is order-independent; empty -> None -> area 0.0
  double set_volume(const std::vector<int>& ord, const std::vector<char>& in_lhs, bool want_lhs) const {
    bool any = false;
    Box acc{};
    for (size_t k = 0; k < ord.size(); ++k) {
      if ((in_lhs[k] != 0) != want_lhs) continue;
      const Box& b = boxes[ord[k]];
      acc = any ? surrounding(acc, b) : b;
      any = true;
    }
    return any ? volume(acc) : 0.0;
  }

  BuildNode build(std::array<std::vector<int>, 3>& ord) {
    const size_t n = ord[0].size();
    if (n == 1) {
      BuildNode leaf;
      leaf.box = boxes[ord[0][0]];
      leaf.leaf = ord[0][0];
      leaf.lhs = leaf.rhs = -1;
      return leaf;
    }
    // split_best (constructor.rs:137-166): xmin_median, xmin_space, ymin_median, ymin_space, zmin_median, zmin_space
    int best_axis = 0;
    std::vector<char> best_flags, flags(n);
    double best_score = 0.0;
    bool have = false;
    for (int a = 0; a < 3; ++a) {
      const std::vector<int>& o = ord[a];
      for (int kind = 0; kind < 2; ++kind) {
        if (kind == 0) {
          // split_median (constructor.rs:63-79): first n/2 in order -> lhs
          for (size_t k = 0; k < n; ++k) flags[k] = (k < n / 2) ? 1 : 0;
        } else {
          // split_space (constructor.rs:81-110): first -> lhs; others lhs iff min < midpoint
          double v0 = boxes[o[0]].mn[a], vl = boxes[o[n - 1]].mn[a];
          double mid = (vl + v0) / 2.0;
          flags[0] = 1;
          for (size_t k = 1; k < n; ++k) flags[k] = (boxes[o[k]].mn[a] < mid) ? 1 : 0;
        }
        double score = set_volume(o, flags, true) + set_volume(o, flags, false);
        if (!have || total_cmp(score, best_score) < 0) {  // min_by: first minimum wins
          have = true;
          best_score = score;
          best_axis = a;
          best_flags = flags;
        }
      }
    }
    // stable partition of the three sorted lists by membership (keeps each child's order sorted)
    const std::vector<int>& bo = ord[best_axis];
    for (size_t k = 0; k < n; ++k) mark[bo[k]] = best_flags[k];
    std::array<std::vector<int>, 3> lo, hi;
    for (int a = 0; a < 3; ++a) {
      lo[a].reserve(n);
      hi[a].reserve(n);
      for (int idx : ord[a]) (mark[idx] ? lo[a] : hi[a]).push_back(idx);
      std::vector<int>().swap(ord[a]);  // free the parent's lists before recursing
    }
    BuildNode lhs = build(lo);
    BuildNode rhs = build(hi);
    // partition_nodes (constructor.rs:168-198): push lhs, push rhs, return the parent
    BuildNode parent;
    parent.box = surrounding(lhs.box, rhs.box);
    parent.leaf = -1;
    parent.lhs = (int32_t)tree.size();
    tree.push_back(lhs);
    parent.rhs = (int32_t)tree.size();
    tree.push_back(rhs);
    return parent;
  }
};

double surface(const Box& b) {
  double x = std::max(0.0, b.mx[0] - b.mn[0]);
  double y = std::max(0.0, b.mx[1] - b.mn[1]);
  double z = std::max(0.0, b.mx[2] - b.mn[2]);
  return 2.0 * (x * y + y * z + z * x);
}

// Bin of a centroid, clamped in floating point before the conversion: with extreme coordinates the
// quotient can be huge, +-inf (ext = inf) or NaN (inf / inf), and converting those to int is undefined
// (found by tools/sanitize).  NaN goes to bin 0.
inline int sah_bin(double c, double lo, double ext, int bins) {
  const double q = (c - lo) / ext * bins;
  if (!(q > 0.0)) return 0;
  return q >= bins - 1 ? bins - 1 : (int)q;
}

struct SahBuilder {
  const std::vector<Box>& boxes;
  std::vector<BuildNode> tree;
  std::vector<int> items;
  std::vector<std::array<double, 3>> cen;

  bool sweep = false;  // exact SAH over every object boundary instead of 32 centroid bins
  const std::vector<double>* weight = nullptr;  // per-object test cost (sweep only; null: 1 each)
  std::vector<int> tmp;
  std::vector<double> right_sa, right_w;
  double w(int x) const { return weight ? (*weight)[x] : 1.0; }

  explicit SahBuilder(const std::vector<Box>& b) : boxes(b) {}

  // Sort key of a centroid: a total order for std::sort (a NaN centroid — a box with NaN or opposite
  // infinite planes — sorts as +inf; ties by object index), so the comparator is a strict weak ordering.
  double ckey(int x, int a) const {
    const double v = cen[x][a];
    return v != v ? INFINITY : v;
  }
  bool before(int x, int y, int a) const {
    const double kx = ckey(x, a), ky = ckey(y, a);
    return kx < ky || (kx == ky && x < y);
  }

  // Exact sweep: per axis, the objects sorted by centroid (ties by index), every split point
  // evaluated with prefix / suffix bounding boxes; items[begin, end) left in the best axis's order.
  // Returns the split position, or -1 when no split separates anything (all centroids equal).
  int sweep_split(int begin, int end) {
    const int n = end - begin;
    double best_cost = INFINITY;
    int best_axis = -1, best_i = -1;
    right_sa.resize(n);
    right_w.resize(n);
    for (int a = 0; a < 3; ++a) {
      tmp.assign(items.begin() + begin, items.begin() + end);
      std::sort(tmp.begin(), tmp.end(), [&](int x, int y) { return before(x, y, a); });
      Box acc = boxes[tmp[n - 1]];
      double wr = 0.0;
      for (int i = n - 1; i >= 1; --i) {  // right_sa[i]: objects [i, n)
        if (i < n - 1) acc = surrounding(acc, boxes[tmp[i]]);
        right_sa[i] = surface(acc);
        wr += w(tmp[i]);
        right_w[i] = wr;
      }
      acc = boxes[tmp[0]];
      double wl = 0.0;
      for (int i = 1; i < n; ++i) {  // split before object i: left [0, i), right [i, n)
        if (i > 1) acc = surrounding(acc, boxes[tmp[i - 1]]);
        wl += w(tmp[i - 1]);
        if (ckey(tmp[i - 1], a) == ckey(tmp[i], a)) continue;  // not a separating plane
        const double cost = weight ? surface(acc) * wl + right_sa[i] * right_w[i] : surface(acc) * i + right_sa[i] * (n - i);
        if (cost < best_cost) { best_cost = cost; best_axis = a; best_i = i; }
      }
    }
    if (best_axis < 0) return -1;
    std::sort(items.begin() + begin, items.begin() + end, [&](int x, int y) { return before(x, y, best_axis); });
    return begin + best_i;
  }

  int32_t build(int begin, int end) {
    int n = end - begin;
    if (n == 1) {
      BuildNode leaf;
      leaf.box = boxes[items[begin]];
      leaf.leaf = items[begin];
      leaf.lhs = leaf.rhs = -1;
      tree.push_back(leaf);
      return (int32_t)tree.size() - 1;
    }
    if (sweep) {
      int mid = sweep_split(begin, end);
      if (mid < 0) mid = begin + n / 2;
      const int32_t self = (int32_t)tree.size();
      tree.push_back(BuildNode{});
      const int32_t l = build(begin, mid);
      const int32_t r = build(mid, end);
      tree[self].leaf = -1;
      tree[self].lhs = l;
      tree[self].rhs = r;
      tree[self].box = surrounding(tree[l].box, tree[r].box);
      return self;
    }
    double cmn[3], cmx[3];
    for (int k = 0; k < 3; ++k) { cmn[k] = INFINITY; cmx[k] = -INFINITY; }
    for (int i = begin; i < end; ++i)
      for (int k = 0; k < 3; ++k) {
        cmn[k] = std::min(cmn[k], cen[items[i]][k]);
        cmx[k] = std::max(cmx[k], cen[items[i]][k]);
      }
    constexpr int kBins = 32;
    int best_axis = -1, best_split = -1;
    double best_cost = INFINITY;
    for (int a = 0; a < 3; ++a) {
      double ext = cmx[a] - cmn[a];
      if (!(ext > 0.0)) continue;
      Box bb[kBins];
      int cnt[kBins] = {0};
      bool init[kBins] = {false};
      for (int i = begin; i < end; ++i) {
        const int b = sah_bin(cen[items[i]][a], cmn[a], ext, kBins);
        bb[b] = init[b] ? surrounding(bb[b], boxes[items[i]]) : boxes[items[i]];
        init[b] = true;
        cnt[b]++;
      }
      double right_area[kBins];
      int right_cnt[kBins];
      Box acc{};
      bool any = false;
      int c = 0;
      for (int b = kBins - 1; b > 0; --b) {
        if (init[b]) { acc = any ? surrounding(acc, bb[b]) : bb[b]; any = true; }
        c += cnt[b];
        right_area[b] = any ? surface(acc) : 0.0;
        right_cnt[b] = c;
      }
      any = false;
      c = 0;
      for (int b = 0; b < kBins - 1; ++b) {
        if (init[b]) { acc = any ? surrounding(acc, bb[b]) : bb[b]; any = true; }
        c += cnt[b];
        if (c == 0 || right_cnt[b + 1] == 0) continue;
        double cost = surface(acc) * c + right_area[b + 1] * right_cnt[b + 1];
        if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = b; }
      }
    }
    int mid;
    if (best_axis < 0) {
      mid = begin + n / 2;  // all centroids coincide: split the list
    } else {
      double ext = cmx[best_axis] - cmn[best_axis];
      auto it = std::partition(items.begin() + begin, items.begin() + end, [&](int idx) {
        const int b = sah_bin(cen[idx][best_axis], cmn[best_axis], ext, kBins);
        return b <= best_split;
      });
      mid = (int)(it - items.begin());
      if (mid == begin || mid == end) mid = begin + n / 2;
    }
    int32_t self = (int32_t)tree.size();
    tree.push_back(BuildNode{});
    int32_t l = build(begin, mid);
    int32_t r = build(mid, end);
    tree[self].leaf = -1;
    tree[self].lhs = l;
    tree[self].rhs = r;
    tree[self].box = surrounding(tree[l].box, tree[r].box);
    return self;
  }
};

}  // namespace

BuiltTree build_reference_tree(const std::vector<Box>& boxes) {
  BuiltTree out;
  if (boxes.empty()) return out;  // constructor.rs:10-12: empty -> BboxTree::default (root None)
  RefBuilder b(boxes);
  std::array<std::vector<int>, 3> ord;
  for (int a = 0; a < 3; ++a) {
    ord[a].resize(boxes.size());
    std::iota(ord[a].begin(), ord[a].end(), 0);
    // sorted_with_idx (constructor.rs:53-57): total_cmp on bbox.min[a]; ties by index
    std::sort(ord[a].begin(), ord[a].end(), [&](int x, int y) {
      int c = total_cmp(boxes[x].mn[a], boxes[y].mn[a]);
      return c < 0 || (c == 0 && x < y);
    });
  }
  b.tree.reserve(2 * boxes.size());
  BuildNode root = b.build(ord);
  out.root = (int32_t)b.tree.size();
  b.tree.push_back(root);
  out.nodes = std::move(b.tree);
  return out;
}

BuiltTree build_sah_tree(const std::vector<Box>& boxes, bool sweep, const std::vector<double>* weight) {
  BuiltTree out;
  SahBuilder b(boxes);
  b.sweep = sweep;
  b.weight = weight;
  for (int i = 0; i < (int)boxes.size(); ++i) {
    const Box& x = boxes[i];
    bool never = false;
    for (int k = 0; k < 3; ++k) never |= (x.mn[k] > x.mx[k]);  // always rejected by the slab test
    if (never) continue;
    b.items.push_back(i);
  }
  if (b.items.empty()) return out;
  b.cen.resize(boxes.size());
  for (int i : b.items)
    for (int k = 0; k < 3; ++k) b.cen[i][k] = 0.5 * (boxes[i].mn[k] + boxes[i].mx[k]);
  b.tree.reserve(2 * b.items.size());
  out.root = b.build(0, (int)b.items.size());
  out.nodes = std::move(b.tree);
  return out;
}

int32_t tree_branch_depth(const BuiltTree& t) {
  if (t.root < 0) return 0;
  int32_t best = 0;
  std::vector<std::pair<int32_t, int32_t>> st{{t.root, 0}};
  while (!st.empty()) {
    auto [n, d] = st.back();
    st.pop_back();
    const BuildNode& nd = t.nodes[n];
    if (nd.leaf >= 0) { best = std::max(best, d); continue; }
    st.push_back({nd.lhs, d + 1});
    st.push_back({nd.rhs, d + 1});
  }
  return best;
}

}  // namespace rt
