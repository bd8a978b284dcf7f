// bvh_build.cpp — host-side scene preprocessing for libmtx.
//
// * The two BVHs of a scene (mtx.h), each a binned-SAH BVH2 collapsed by
//   SAH-optimal dynamic programming (Ylitie, Karras & Laine 2017):
//   - closest hit (mtx_bvh_build): BVH2 leaves of <= 8 triangles, 4-wide
//     nodes (64 B, 8-bit quantised child boxes, sorted near-first by the
//     traversal), laid out breadth-first with the triangles reordered into
//     leaf order as {v0, e1, e2} records;
//   - occlusion / any hit (mtx_bvh_build_occlusion): BVH2 leaves of <= 3
//     triangles, compressed 8-wide nodes (80 B, children in octant-ordered
//     slots, no per-visit sort) over the closest-hit tree's records.
//   Replaces the Embree / OptiX acceleration-structure build that
//   mi.load_file performs upstream for Scene.ray_intersect / ray_test
//   (path-mis.py:69-71, restirgi.py:320,346).
// * roughplastic precompute (upstream roughplastic constructor): the
//   64-entry external transmittance table and the internal reflectance.
//
// BVH2 depth is capped at MTX_BVH_MAX_DEPTH inner levels (object-median
// splits take over when the SAH would exceed it); the wide trees are never
// deeper, which bounds the device traversal's stacks.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mtx.h"
#include "mtx_core/bsdf.h"
#include "mtx_core/geometry.h"
#include "mtx_core/microfacet.h"

void mtx_set_error(const char *fmt, ...);

namespace {

struct Box {
  float lo[3], hi[3];
  void reset() {
    for (int a = 0; a < 3; ++a) {
      lo[a] = INFINITY;
      hi[a] = -INFINITY;
    }
  }
  void grow(const Box &b) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  void grow(const float *p) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  float area() const {
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (dx < 0 || dy < 0 || dz < 0) return 0.f;
    return 2.f * (dx * dy + dy * dz + dz * dx);
  }
};

constexpr int kMaxBins = 256;  // SAH bins: Builder::bins (default 32, MTX_BVH_BINS)
constexpr float kDefaultCt = 1.f;  // SAH cost of a traversal step, in triangle tests

struct Builder {
  const float *vpos;
  const uint32_t *vidx;
  uint32_t n;
  std::vector<Box> tbox;
  std::vector<float> cen;  // 3 per tri
  std::vector<uint32_t> idx;
  std::vector<int32_t> nodes;  // 16 words per node
  std::vector<uint32_t> order; // leaf order -> input tri
  float ct = kDefaultCt;
  int n_bins = 32;
  uint32_t max_leaf2 = MTX_BVH_MAX_LEAF;  // BVH2 leaf size cap (the occlusion tree: MTX_OCC_MAX_LEAF)
  uint32_t max_depth_seen = 0;

  static int ceil_log2(uint32_t c) {
    int l = 0;
    while ((1u << l) < c) ++l;
    return l;
  }

  Box range_box(uint32_t s, uint32_t e) const {
    Box b;
    b.reset();
    for (uint32_t i = s; i < e; ++i) b.grow(tbox[idx[i]]);
    return b;
  }

  int32_t make_leaf(uint32_t s, uint32_t e) {
    uint32_t first = (uint32_t)order.size();
    for (uint32_t i = s; i < e; ++i) order.push_back(idx[i]);
    uint32_t code = (first << 3) | (e - s - 1);
    return ~(int32_t)code;
  }

  // Partition [s,e) and return the split position; uses binned SAH unless the
  // depth budget forces an object-median split. Returns 0 when a leaf is best.
  uint32_t choose_split(uint32_t s, uint32_t e, uint32_t depth) {
    const int nb = n_bins;
    const uint32_t cnt = e - s;
    Box cb;
    cb.reset();
    for (uint32_t i = s; i < e; ++i) cb.grow(&cen[3 * idx[i]]);
    int axis_big = 0;
    float ext_big = -1.f;
    for (int a = 0; a < 3; ++a) {
      float ex = cb.hi[a] - cb.lo[a];
      if (ex > ext_big) {
        ext_big = ex;
        axis_big = a;
      }
    }
    bool force_median = depth + (uint32_t)ceil_log2(cnt) >= (uint32_t)MTX_BVH_MAX_DEPTH - 2;
    if (!force_median && ext_big > 0.f) {
      float best_cost = INFINITY;
      int best_axis = -1, best_bin = -1;
      const Box pb = range_box(s, e);
      const float pa = pb.area();
      for (int a = 0; a < 3; ++a) {
        float ext = cb.hi[a] - cb.lo[a];
        if (!(ext > 0.f)) continue;
        Box bins[kMaxBins];
        uint32_t counts[kMaxBins] = {0};
        for (int b = 0; b < nb; ++b) bins[b].reset();
        const float k = (float)nb / ext;
        for (uint32_t i = s; i < e; ++i) {
          uint32_t t = idx[i];
          int b = (int)((cen[3 * t + a] - cb.lo[a]) * k);
          b = std::min(std::max(b, 0), nb - 1);
          counts[b]++;
          bins[b].grow(tbox[t]);
        }
        float right_area[kMaxBins];
        uint32_t right_cnt[kMaxBins];
        Box acc;
        acc.reset();
        uint32_t c = 0;
        for (int b = nb - 1; b > 0; --b) {
          acc.grow(bins[b]);
          c += counts[b];
          right_area[b] = acc.area();
          right_cnt[b] = c;
        }
        acc.reset();
        c = 0;
        for (int b = 0; b < nb - 1; ++b) {
          acc.grow(bins[b]);
          c += counts[b];
          if (c == 0 || right_cnt[b + 1] == 0) continue;
          float cost = ct + (acc.area() * (float)c + right_area[b + 1] * (float)right_cnt[b + 1]) / pa;
          if (cost < best_cost) {
            best_cost = cost;
            best_axis = a;
            best_bin = b;
          }
        }
      }
      if (cnt <= max_leaf2 && (best_axis < 0 || (float)cnt <= best_cost)) return 0;
      if (best_axis >= 0) {
        const float ext = cb.hi[best_axis] - cb.lo[best_axis];
        const float k = (float)nb / ext;
        uint32_t *mid = std::partition(idx.data() + s, idx.data() + e, [&](uint32_t t) {
          int b = (int)((cen[3 * t + best_axis] - cb.lo[best_axis]) * k);
          b = std::min(std::max(b, 0), nb - 1);
          return b <= best_bin;
        });
        uint32_t m = (uint32_t)(mid - idx.data());
        if (m > s && m < e) return m;
      }
    }
    if (cnt <= max_leaf2) return 0;
    // object median along the largest centroid extent (stable for ties)
    uint32_t m = s + cnt / 2;
    std::nth_element(idx.data() + s, idx.data() + m, idx.data() + e, [&](uint32_t x, uint32_t y) {
      float a = cen[3 * x + axis_big], b = cen[3 * y + axis_big];
      return a < b || (a == b && x < y);
    });
    return m;
  }

  // Conservative padding: the slab test computes t = fma(b, 1/d, -o/d) with
  // |error| <= (|o| + |b|) |1/d| 2^-23 for points inside the scene, so a pad
  // of (|x| + E) 2^-19 (E = largest |coordinate| of the scene) covers it
  // with a 10x margin and no closest hit can be culled.
  float extent = 0.f;
  void pad_box(Box &b) const {
    const float k = 1.0f / 524288.0f;  // 2^-19
    for (int a = 0; a < 3; ++a) {
      b.lo[a] -= (std::fabs(b.lo[a]) + extent) * k;
      b.hi[a] += (std::fabs(b.hi[a]) + extent) * k;
    }
  }

  void store_child_boxes(uint32_t node, const Box &b0, const Box &b1) {
    Box p0 = b0, p1 = b1;
    pad_box(p0);
    pad_box(p1);
    float *f = reinterpret_cast<float *>(&nodes[16 * node]);
    f[0] = p0.lo[0]; f[1] = p0.hi[0]; f[2] = p0.lo[1]; f[3] = p0.hi[1];
    f[4] = p1.lo[0]; f[5] = p1.hi[0]; f[6] = p1.lo[1]; f[7] = p1.hi[1];
    f[8] = p0.lo[2]; f[9] = p0.hi[2]; f[10] = p1.lo[2]; f[11] = p1.hi[2];
  }

  // Builds the subtree for [s,e) under an inner node at `depth`; returns a child ref.
  int32_t build(uint32_t s, uint32_t e, uint32_t depth) {
    uint32_t m = choose_split(s, e, depth);
    if (m == 0) return make_leaf(s, e);
    uint32_t node = (uint32_t)(nodes.size() / 16);
    nodes.resize(nodes.size() + 16, 0);
    if (depth + 1 > max_depth_seen) max_depth_seen = depth + 1;
    Box b0 = range_box(s, m), b1 = range_box(m, e);
    int32_t c0 = build(s, m, depth + 1);
    int32_t c1 = build(m, e, depth + 1);
    store_child_boxes(node, b0, b1);
    nodes[16 * node + 12] = c0;
    nodes[16 * node + 13] = c1;
    return (int32_t)node;
  }


  // ---- SAH-optimal collapse (dynamic programming over the BVH2) ----------
  // cost[n][j] = least SAH cost of representing BVH2 subtree n as at most j
  // children of a wide node (j = 1..kw); a child is either a wide inner node
  // (area * c_node + the best kw-way split of its subtree) or a leaf holding
  // the whole subtree when it has <= max_leaf_w triangles (area * c_tri *
  // count; BVH2 subtrees are contiguous in leaf order). Replaces the greedy
  // largest-area opening (Ylitie et al. 2017, wide-BVH collapse).
  static constexpr int kMaxW = 8;
  int kw = MTX_BVH_WIDTH;                 // 4 (closest hit) or 8 (occlusion)
  uint32_t max_leaf_w = MTX_BVH_MAX_LEAF;  // leaf size cap of the wide tree
  float c_node = 1.0f, c_tri = 1.0f;      // tuned on the bedroom proxy (A/B: +1.8 % vs greedy, 4-wide)
  std::vector<float> dp_cost;      // (kw + 1) per BVH2 node (index j = 1..kw)
  std::vector<uint8_t> dp_split;   // (kw + 1) per node: 0 = use j-1 slots, k = k slots left
  std::vector<uint8_t> dp_leaf;    // 1: the subtree as one leaf (j = 1)
  std::vector<uint32_t> sub_first, sub_count;
  std::vector<Box> box2;           // padded box of each BVH2 node

  Box child_box2(uint32_t node, int c) const {
    const float *f = reinterpret_cast<const float *>(&nodes[16 * (size_t)node]);
    Box b;
    if (c == 0) {
      b.lo[0] = f[0]; b.hi[0] = f[1]; b.lo[1] = f[2]; b.hi[1] = f[3]; b.lo[2] = f[8]; b.hi[2] = f[9];
    } else {
      b.lo[0] = f[4]; b.hi[0] = f[5]; b.lo[1] = f[6]; b.hi[1] = f[7]; b.lo[2] = f[10]; b.hi[2] = f[11];
    }
    return b;
  }

  void ref_info(int32_t ref, float area, float *cost, uint32_t *first, uint32_t *count) const {
    if (ref >= 0) {
      for (int j = 1; j <= kw; ++j) cost[j] = dp_cost[(kw + 1) * (size_t)ref + j];
      *first = sub_first[ref];
      *count = sub_count[ref];
    } else {
      const uint32_t code = ~(uint32_t)ref;
      *first = code >> 3;
      *count = (code & 7u) + 1u;
      for (int j = 1; j <= kw; ++j) cost[j] = area * c_tri * (float)*count;
    }
  }

  void dp_prepare() {
    const size_t n2 = nodes.size() / 16;
    dp_cost.assign((kw + 1) * n2, 0.f);
    dp_split.assign((kw + 1) * n2, 0);
    dp_leaf.assign(n2, 0);
    sub_first.assign(n2, 0);
    sub_count.assign(n2, 0);
    box2.resize(n2);
    Box root = child_box2(0, 0);
    root.grow(child_box2(0, 1));
    box2[0] = root;
    for (size_t n = 0; n < n2; ++n)  // parents precede children (preorder indices)
      for (int c = 0; c < 2; ++c) {
        const int32_t r = nodes[16 * n + 12 + c];
        if (r >= 0) box2[r] = child_box2((uint32_t)n, c);
      }
    for (size_t n = n2; n-- > 0;) {
      float cl[kMaxW + 1], cr[kMaxW + 1];
      uint32_t fl, nl, fr, nr;
      ref_info(nodes[16 * n + 12], child_box2((uint32_t)n, 0).area(), cl, &fl, &nl);
      ref_info(nodes[16 * n + 13], child_box2((uint32_t)n, 1).area(), cr, &fr, &nr);
      sub_first[n] = std::min(fl, fr);
      sub_count[n] = nl + nr;
      float dist[kMaxW + 1];
      uint8_t kbest[kMaxW + 1] = {0};
      for (int j = 2; j <= kw; ++j) {
        dist[j] = INFINITY;
        for (int k = 1; k < j; ++k) {
          const float c = cl[k] + cr[j - k];
          if (c < dist[j]) {
            dist[j] = c;
            kbest[j] = (uint8_t)k;
          }
        }
      }
      const float area = box2[n].area();
      const float c_inner = area * c_node + dist[kw];
      const float c_lf = sub_count[n] <= max_leaf_w ? area * c_tri * (float)sub_count[n] : INFINITY;
      float *Cn = &dp_cost[(kw + 1) * n];
      dp_leaf[n] = c_lf <= c_inner ? 1 : 0;
      Cn[1] = std::min(c_lf, c_inner);
      for (int j = 2; j <= kw; ++j) {
        if (dist[j] < Cn[j - 1]) {
          Cn[j] = dist[j];
          dp_split[(kw + 1) * n + j] = kbest[j];
        } else {
          Cn[j] = Cn[j - 1];
          dp_split[(kw + 1) * n + j] = 0;
        }
      }
    }
  }

  struct Child {
    int32_t ref;  // BVH2 ref (inner index or leaf code)
    Box box;      // padded fp32 box
  };

  // Children of the wide node made from BVH2 node n with j slots.
  void dp_expand(int32_t ref, int j, Box box, std::vector<Child> &out) const {
    if (ref < 0 || j == 1) {
      out.push_back({ref, box});
      return;
    }
    int k = dp_split[(kw + 1) * (size_t)ref + j];
    while (k == 0 && j > 1) {
      --j;
      k = j > 1 ? dp_split[(kw + 1) * (size_t)ref + j] : 0;
    }
    if (j == 1) {
      out.push_back({ref, box});
      return;
    }
    dp_expand(nodes[16 * (size_t)ref + 12], k, child_box2((uint32_t)ref, 0), out);
    dp_expand(nodes[16 * (size_t)ref + 13], j - k, child_box2((uint32_t)ref, 1), out);
  }

  // the wide children of BVH2 node n2 (a subtree that prefers one slot is
  // still split at its root)
  std::vector<Child> wide_children(uint32_t n2) const {
    std::vector<Child> ch;
    dp_expand((int32_t)n2, kw, box2[n2], ch);
    if (ch.size() == 1) {
      ch.clear();
      dp_expand(nodes[16 * (size_t)n2 + 12], 1, child_box2(n2, 0), ch);
      dp_expand(nodes[16 * (size_t)n2 + 13], 1, child_box2(n2, 1), ch);
    }
    return ch;
  }

  bool quant_ok = true;
  static constexpr int kEMin = -32, kEMax = 31;
  std::vector<int32_t> wnodes;  // the wide tree (16 or 20 words per node)
  uint32_t wide_depth = 0;

  // Quantisation of axis a of the children's boxes in the frame of their
  // union: origin, exponent and the conservative 8-bit bounds of each child.
  void quantise_axis(const std::vector<Child> &ch, const Box &u, int a, float *org_out, int *e_out,
                     uint32_t *qlo_out, uint32_t *qhi_out) {
    const float org = u.lo[a];
    const double ext = (double)u.hi[a] - (double)org;
    int e = kEMin;
    if (ext > 0.0) {
      int ee;
      std::frexp(ext / 255.0, &ee);
      e = std::max(kEMin, std::min(kEMax, ee));
    }
    while (e < kEMax && mtx::wide_decode(org, mtx::wide_scale((uint32_t)(e & 255)), 255u) < u.hi[a]) ++e;
    const float sc = mtx::wide_scale((uint32_t)(e & 255));
    const double dsc = std::ldexp(1.0, e);
    for (size_t k = 0; k < ch.size(); ++k) {
      double flo = std::floor(((double)ch[k].box.lo[a] - (double)org) / dsc);
      double fhi = std::ceil(((double)ch[k].box.hi[a] - (double)org) / dsc);
      uint32_t qlo = (uint32_t)std::max(0.0, std::min(255.0, flo));
      uint32_t qhi = (uint32_t)std::max(0.0, std::min(255.0, fhi));
      while (qlo > 0 && mtx::wide_decode(org, sc, qlo) > ch[k].box.lo[a]) --qlo;
      while (qhi < 255 && mtx::wide_decode(org, sc, qhi) < ch[k].box.hi[a]) ++qhi;
      if (mtx::wide_decode(org, sc, qlo) > ch[k].box.lo[a] || mtx::wide_decode(org, sc, qhi) < ch[k].box.hi[a])
        quant_ok = false;
      qlo_out[k] = qlo;
      qhi_out[k] = qhi;
    }
    *org_out = org;
    *e_out = e;
  }

  // ---- 4-wide closest-hit nodes (mtx.h) ----------------------------------
  // Depth-first collapse into wnodes, then relayout4 reorders breadth-first.
  int32_t collapse4(uint32_t node2, uint32_t depth) {
    const std::vector<Child> ch = wide_children(node2);
    const uint32_t w = (uint32_t)(wnodes.size() / 16);
    wnodes.resize(wnodes.size() + 16, 0);
    wide_depth = std::max(wide_depth, depth + 1);
    int32_t refs[MTX_BVH_WIDTH] = {0, 0, 0, 0};
    for (size_t k = 0; k < ch.size(); ++k) {
      const int32_t r = ch[k].ref;
      if (r < 0) {
        refs[k] = r;
      } else if (dp_leaf[r]) {  // the whole subtree as one leaf
        refs[k] = ~(int32_t)((sub_first[r] << 3) | (sub_count[r] - 1u));
      } else {
        refs[k] = collapse4((uint32_t)r, depth + 1);
      }
    }
    encode4(w, ch, refs);
    return (int32_t)w;
  }

  void encode4(uint32_t w, const std::vector<Child> &ch, const int32_t *refs) {
    Box u;
    u.reset();
    for (const Child &c : ch) u.grow(c.box);
    int32_t *W = &wnodes[16 * (size_t)w];
    uint32_t q[6] = {0, 0, 0, 0, 0, 0}, ebytes = 0;
    for (int a = 0; a < 3; ++a) {
      float org;
      int e;
      uint32_t qlo[kMaxW], qhi[kMaxW];
      quantise_axis(ch, u, a, &org, &e, qlo, qhi);
      for (size_t k = 0; k < ch.size(); ++k) {
        q[2 * a] |= qlo[k] << (8 * k);
        q[2 * a + 1] |= qhi[k] << (8 * k);
      }
      std::memcpy(&W[a], &org, 4);
      ebytes |= (uint32_t)(e & 255) << (8 * a);
    }
    W[3] = (int32_t)(ebytes | ((uint32_t)ch.size() << 24));
    for (int k = 0; k < MTX_BVH_WIDTH; ++k) W[4 + k] = refs[k];
    for (int k = 0; k < 6; ++k) W[8 + k] = (int32_t)q[k];
  }

  // Breadth-first layout: the inner children of a node at consecutive
  // indices (two 64-B siblings per 128-B line), a node's slots ordered inner
  // children first (each group keeps its order), and the triangles
  // re-ordered so that a node's leaf children are consecutive ranges in slot
  // order.
  void relayout4() {
    std::vector<int32_t> out(16, 0);
    std::vector<uint32_t> queue = {0}, tris;
    tris.reserve(order.size());
    for (size_t qi = 0; qi < queue.size(); ++qi) {
      const int32_t *W = &wnodes[16 * (size_t)queue[qi]];
      int slot[MTX_BVH_WIDTH], m = 0;
      for (int k = 0; k < (int)((uint32_t)W[3] >> 24); ++k)
        if (W[4 + k] >= 0) slot[m++] = k;
      for (int k = 0; k < (int)((uint32_t)W[3] >> 24); ++k) {
        bool dup = false;  // a one-triangle mesh's root holds its leaf twice
        for (int j = 0; j < k; ++j) dup = dup || W[4 + j] == W[4 + k];
        if (W[4 + k] < 0 && !dup) slot[m++] = k;
      }
      const int nch = m;
      int32_t O[16] = {W[0], W[1], W[2], (int32_t)(((uint32_t)W[3] & 0xffffffu) | ((uint32_t)nch << 24)),
                       0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int a = 0; a < 6; ++a) {
        uint32_t q = 0;
        for (int j = 0; j < nch; ++j) q |= (((uint32_t)W[8 + a] >> (8 * slot[j])) & 255u) << (8 * j);
        O[8 + a] = (int32_t)q;
      }
      for (int j = 0; j < nch; ++j) {
        const int32_t r = W[4 + slot[j]];
        if (r >= 0) {
          O[4 + j] = (int32_t)queue.size();
          queue.push_back((uint32_t)r);
        } else {
          const uint32_t code = ~(uint32_t)r, first = code >> 3, cnt = (code & 7u) + 1u;
          O[4 + j] = ~(int32_t)(((uint32_t)tris.size() << 3) | (cnt - 1u));
          for (uint32_t t = 0; t < cnt; ++t) tris.push_back(order[first + t]);
        }
      }
      out.resize(16 * queue.size(), 0);
      std::memcpy(&out[16 * qi], O, sizeof(O));
    }
    wnodes.swap(out);
    order.swap(tris);
  }

  // ---- 8-wide occlusion nodes (mtx.h) ------------------------------------
  // Slot of each child: slot s is visited at position s ^ octant(ray), so
  // the child in slot s should lie towards the corner s of the node (axis a
  // on the + side when bit a of s is set). Greedy assignment (Ylitie et al.
  // 2017, section 3.2): repeatedly the unassigned (child, slot) pair with the
  // largest dot(centroid_child - centroid_node, corner_s); ties to the
  // smaller child, then the smaller slot.
  static void assign_slots(const std::vector<Child> &ch, int slot_of[kMaxW]) {
    Box u;
    u.reset();
    for (const Child &c : ch) u.grow(c.box);
    double pc[3], cc[kMaxW][3];
    for (int a = 0; a < 3; ++a) pc[a] = 0.5 * ((double)u.lo[a] + (double)u.hi[a]);
    for (size_t i = 0; i < ch.size(); ++i)
      for (int a = 0; a < 3; ++a) cc[i][a] = 0.5 * ((double)ch[i].box.lo[a] + (double)ch[i].box.hi[a]) - pc[a];
    bool used_c[kMaxW] = {false}, used_s[kMaxW] = {false};
    for (size_t n = 0; n < ch.size(); ++n) {
      double best = -INFINITY;
      int bc = -1, bs = -1;
      for (size_t i = 0; i < ch.size(); ++i) {
        if (used_c[i]) continue;
        for (int sl = 0; sl < kMaxW; ++sl) {
          if (used_s[sl]) continue;
          double v = 0.0;
          for (int a = 0; a < 3; ++a) v += ((sl >> a) & 1) ? cc[i][a] : -cc[i][a];
          if (v > best) {
            best = v;
            bc = (int)i;
            bs = sl;
          }
        }
      }
      used_c[bc] = used_s[bs] = true;
      slot_of[bc] = bs;
    }
  }

  // Quantised child boxes of node W in slots slot_of[k] (mtx.h layout).
  void encode8(int32_t *W, const std::vector<Child> &ch, const int *slot_of) {
    Box u;
    u.reset();
    for (const Child &c : ch) u.grow(c.box);
    uint32_t q[12];
    for (int a = 0; a < 3; ++a) {  // empty slots: q_lo 255, q_hi 0
      q[4 * a + 0] = q[4 * a + 1] = 0xffffffffu;
      q[4 * a + 2] = q[4 * a + 3] = 0u;
    }
    uint32_t ebytes = 0;
    for (int a = 0; a < 3; ++a) {
      float org;
      int e;
      uint32_t qlo[kMaxW], qhi[kMaxW];
      quantise_axis(ch, u, a, &org, &e, qlo, qhi);
      for (size_t k = 0; k < ch.size(); ++k) {
        const int sl = slot_of[k], wd = sl >> 2, sh = 8 * (sl & 3);
        uint32_t &lo = q[4 * a + wd], &hi = q[4 * a + 2 + wd];
        lo = (lo & ~(255u << sh)) | (qlo[k] << sh);
        hi = (hi & ~(255u << sh)) | (qhi[k] << sh);
      }
      std::memcpy(&W[a], &org, 4);
      ebytes |= (uint32_t)(e & 255) << (8 * a);
    }
    W[3] = (int32_t)((uint32_t)W[3] | ebytes);
    for (int k = 0; k < 12; ++k) W[8 + k] = (int32_t)q[k];
  }

  // Breadth-first wide tree: node i's inner children get consecutive
  // indices (slot order) when it is laid out, its leaves' triangles
  // consecutive slots of the new leaf order.
  void collapse8() {
    const int NW = MTX_OCC_NODE_WORDS;
    std::vector<uint32_t> queue = {0}, level = {1}, tris;
    tris.reserve(order.size());
    wnodes.assign(NW, 0);
    for (size_t qi = 0; qi < queue.size(); ++qi) {
      const uint32_t n2 = queue[qi];
      std::vector<Child> ch = wide_children(n2);
      if (qi == 0 && n == 1) ch.resize(1);  // one triangle: the root's two BVH2 children are the same leaf
      wide_depth = std::max(wide_depth, level[qi]);
      int slot_of[kMaxW];
      assign_slots(ch, slot_of);
      int child_at[kMaxW];
      for (int sl = 0; sl < kMaxW; ++sl) child_at[sl] = -1;
      for (size_t k = 0; k < ch.size(); ++k) child_at[slot_of[k]] = (int)k;
      uint32_t imask = 0, meta[2] = {0, 0}, off = 0;
      const uint32_t child_base = (uint32_t)queue.size(), tri_base = (uint32_t)tris.size();
      for (int sl = 0; sl < kMaxW; ++sl) {
        const int k = child_at[sl];
        if (k < 0) continue;
        const int32_t r = ch[k].ref;
        uint32_t first = 0, cnt = 0, m;
        bool leaf = r < 0;
        if (r < 0) {
          const uint32_t code = ~(uint32_t)r;
          first = code >> 3;
          cnt = (code & 7u) + 1u;
        } else if (dp_leaf[r]) {  // the whole subtree as one leaf
          first = sub_first[r];
          cnt = sub_count[r];
          leaf = true;
        }
        if (leaf) {
          m = (((1u << cnt) - 1u) << 5) | off;
          for (uint32_t t = 0; t < cnt; ++t) tris.push_back(order[first + t]);
          off += cnt;
        } else {
          imask |= 1u << sl;
          m = 0x20u | (24u + (uint32_t)sl);
          queue.push_back((uint32_t)r);
          level.push_back(level[qi] + 1);
        }
        meta[sl >> 2] |= m << (8 * (sl & 3));
      }
      if (off > 24) quant_ok = false;  // cannot happen: <= 8 leaves of <= 3 triangles
      wnodes.resize((size_t)NW * queue.size(), 0);
      int32_t *W = &wnodes[(size_t)NW * qi];
      W[3] = (int32_t)(imask << 24);
      W[4] = (int32_t)child_base;
      W[5] = (int32_t)tri_base;
      W[6] = (int32_t)meta[0];
      W[7] = (int32_t)meta[1];
      encode8(W, ch, slot_of);
    }
    order.swap(tris);
  }

  void run() {
    for (uint32_t t = 0; t < n; ++t)
      for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a) extent = std::max(extent, std::fabs(vpos[3 * (size_t)vidx[3 * (size_t)t + k] + a]));
    tbox.resize(n);
    cen.resize(3 * (size_t)n);
    idx.resize(n);
    for (uint32_t t = 0; t < n; ++t) {
      Box b;
      b.reset();
      for (int k = 0; k < 3; ++k) b.grow(&vpos[3 * (size_t)vidx[3 * (size_t)t + k]]);
      tbox[t] = b;
      for (int a = 0; a < 3; ++a) cen[3 * (size_t)t + a] = 0.5f * (b.lo[a] + b.hi[a]);
      idx[t] = t;
    }
    order.reserve(n);
    nodes.reserve(16 * (size_t)(n / 2 + 2));
    // The root is always an inner node (index 0).
    nodes.resize(16, 0);
    max_depth_seen = 1;
    if (n == 1) {
      int32_t leaf = make_leaf(0, 1);
      Box b = tbox[0];
      store_child_boxes(0, b, b);
      nodes[12] = leaf;
      nodes[13] = leaf;
      return;
    }
    uint32_t m = choose_split(0, n, 0);
    if (m == 0) m = n / 2;
    Box b0 = range_box(0, m), b1 = range_box(m, n);
    int32_t c0 = build(0, m, 1);
    int32_t c1 = build(m, n, 1);
    store_child_boxes(0, b0, b1);
    nodes[12] = c0;
    nodes[13] = c1;
  }
};



// Build knobs (tuning experiments, tools/bvh_experiment.py): SAH traversal
// cost relative to one triangle test, bins, and the collapse's node /
// triangle costs.
void apply_knobs(Builder &b) {
  if (const char *e = getenv("MTX_BVH_CT")) b.ct = std::max(0.05f, (float)atof(e));
  if (const char *e = getenv("MTX_BVH_BINS")) b.n_bins = std::max(2, std::min(kMaxBins, atoi(e)));
  if (const char *e = getenv("MTX_BVH_CNODE")) b.c_node = (float)atof(e);
  if (const char *e = getenv("MTX_BVH_CTRI")) b.c_tri = (float)atof(e);
}

int check_order(const Builder &b, uint32_t n_tris, const char *fn, const char *stage) {
  if (b.order.size() != n_tris) {
    mtx_set_error("%s: internal error (%zu triangles %s for %u)", fn, b.order.size(), stage, n_tris);
    return MTX_E_ARG;
  }
  if (!b.quant_ok) {
    mtx_set_error("%s: child box quantisation failed (non-finite or huge coordinates?)", fn);
    return MTX_E_ARG;
  }
  return MTX_OK;
}

}  // namespace

extern "C" int mtx_bvh_build(const float *vpos, uint32_t n_verts, const uint32_t *tri_vidx, uint32_t n_tris,
                             int32_t *nodes_out, uint32_t *n_nodes_out, float *tri_geom_out, uint32_t *perm_out,
                             uint32_t *depth_out) {
  if (!vpos || !tri_vidx || !nodes_out || !n_nodes_out || !tri_geom_out || !perm_out || n_tris == 0) {
    mtx_set_error("mtx_bvh_build: null argument or empty mesh");
    return MTX_E_ARG;
  }
  if (n_tris >= (1u << 28)) {
    mtx_set_error("mtx_bvh_build: %u triangles exceed the 2^28 leaf encoding", n_tris);
    return MTX_E_ARG;
  }
  for (uint64_t i = 0; i < 3ull * n_tris; ++i)
    if (tri_vidx[i] >= n_verts) {
      mtx_set_error("mtx_bvh_build: vertex index %u out of range (%u vertices)", tri_vidx[i], n_verts);
      return MTX_E_ARG;
    }
  Builder b;
  apply_knobs(b);
  b.vpos = vpos;
  b.vidx = tri_vidx;
  b.n = n_tris;
  b.max_leaf2 = MTX_BVH_MAX_LEAF;
  b.run();
  int rc;
  if ((rc = check_order(b, n_tris, "mtx_bvh_build", "in BVH2 leaves"))) return rc;
  b.kw = MTX_BVH_WIDTH;
  b.max_leaf_w = MTX_BVH_MAX_LEAF;
  b.dp_prepare();
  b.wnodes.reserve(b.nodes.size() / 2 + 16);
  b.collapse4(0, 0);
  b.relayout4();
  if ((rc = check_order(b, n_tris, "mtx_bvh_build", "after the collapse"))) return rc;
  std::memcpy(nodes_out, b.wnodes.data(), b.wnodes.size() * sizeof(int32_t));
  *n_nodes_out = (uint32_t)(b.wnodes.size() / MTX_BVH_NODE_WORDS);
  for (uint32_t i = 0; i < n_tris; ++i) {
    uint32_t t = b.order[i];
    perm_out[i] = t;
    const float *p0 = &vpos[3 * (size_t)tri_vidx[3 * (size_t)t + 0]];
    const float *p1 = &vpos[3 * (size_t)tri_vidx[3 * (size_t)t + 1]];
    const float *p2 = &vpos[3 * (size_t)tri_vidx[3 * (size_t)t + 2]];
    float *g = &tri_geom_out[12 * (size_t)i];
    g[0] = p0[0]; g[1] = p0[1]; g[2] = p0[2]; g[3] = 0.f;
    g[4] = p1[0] - p0[0]; g[5] = p1[1] - p0[1]; g[6] = p1[2] - p0[2]; g[7] = 0.f;
    g[8] = p2[0] - p0[0]; g[9] = p2[1] - p0[1]; g[10] = p2[2] - p0[2]; g[11] = 0.f;
  }
  if (depth_out) *depth_out = b.wide_depth;
  return MTX_OK;
}

// The occlusion tree is built over the triangle records themselves: vertices
// v0, v0 + e1, v0 + e2 (fp32) give each triangle's box, and the output
// records are the input records copied bit for bit, so an any-hit query
// tests exactly the triangles a closest-hit query does (the rounding of
// v0 + e1 is far inside the boxes' padding).
extern "C" int mtx_bvh_build_occlusion(const float *tri_geom, uint32_t n_tris, int32_t *nodes_out,
                                       uint32_t *n_nodes_out, float *tri_geom_out, uint32_t *perm_out,
                                       uint32_t *depth_out) {
  if (!tri_geom || !nodes_out || !n_nodes_out || !tri_geom_out || n_tris == 0) {
    mtx_set_error("mtx_bvh_build_occlusion: null argument or empty mesh");
    return MTX_E_ARG;
  }
  if (n_tris >= (1u << 28)) {
    mtx_set_error("mtx_bvh_build_occlusion: %u triangles exceed the 2^28 leaf encoding", n_tris);
    return MTX_E_ARG;
  }
  std::vector<float> pts(9 * (size_t)n_tris);
  std::vector<uint32_t> vidx(3 * (size_t)n_tris);
  for (size_t i = 0; i < n_tris; ++i) {
    const float *g = &tri_geom[12 * i];
    for (int a = 0; a < 3; ++a) {
      pts[9 * i + a] = g[a];
      pts[9 * i + 3 + a] = g[a] + g[4 + a];
      pts[9 * i + 6 + a] = g[a] + g[8 + a];
    }
    for (int k = 0; k < 3; ++k) vidx[3 * i + k] = (uint32_t)(3 * i + k);
  }
  Builder b;
  apply_knobs(b);
  // the occlusion tree's own costs (tuning experiments): an any-hit ray
  // stops at its first hit, so the SAH's weights need not be the closest
  // hit's
  if (const char *e = getenv("MTX_OCC_CT")) b.ct = std::max(0.05f, (float)atof(e));
  if (const char *e = getenv("MTX_OCC_CNODE")) b.c_node = (float)atof(e);
  if (const char *e = getenv("MTX_OCC_CTRI")) b.c_tri = (float)atof(e);
  b.vpos = pts.data();
  b.vidx = vidx.data();
  b.n = n_tris;
  b.max_leaf2 = MTX_OCC_MAX_LEAF;
  b.run();
  int rc;
  if ((rc = check_order(b, n_tris, "mtx_bvh_build_occlusion", "in BVH2 leaves"))) return rc;
  b.kw = MTX_OCC_WIDTH;
  b.max_leaf_w = MTX_OCC_MAX_LEAF;
  b.dp_prepare();
  b.collapse8();
  if ((rc = check_order(b, n_tris, "mtx_bvh_build_occlusion", "after the collapse"))) return rc;
  std::memcpy(nodes_out, b.wnodes.data(), b.wnodes.size() * sizeof(int32_t));
  *n_nodes_out = (uint32_t)(b.wnodes.size() / MTX_OCC_NODE_WORDS);
  for (uint32_t i = 0; i < n_tris; ++i) {
    if (perm_out) perm_out[i] = b.order[i];
    std::memcpy(&tri_geom_out[12 * (size_t)i], &tri_geom[12 * (size_t)b.order[i]], 12 * sizeof(float));
  }
  if (depth_out) *depth_out = b.wide_depth;
  return MTX_OK;
}

// --------------------------------------------------------------------------
// roughplastic precompute
// --------------------------------------------------------------------------

static void gauss_legendre(int n, std::vector<double> &x, std::vector<double> &w) {
  x.resize(n);
  w.resize(n);
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5));
    for (int it = 0; it < 100; ++it) {
      double p1 = 1.0, p2 = 0.0;
      for (int j = 1; j <= n; ++j) {
        double p3 = p2;
        p2 = p1;
        p1 = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
      }
      double pp = n * (z * p1 - p2) / (z * z - 1.0);
      double z1 = z;
      z = z1 - p1 / pp;
      if (std::fabs(z - z1) < 1e-15) {
        x[i] = -z;
        w[i] = 2.0 / ((1.0 - z * z) * pp * pp);
        break;
      }
    }
  }
}

// Average Fresnel reflectance seen through the microfacet distribution
// (upstream eval_reflectance): E over visible normals of F(wi.m) G1(wo, m).
static float eval_reflectance(const mtx::Microfacet &distr, mtx::V3 wi, float eta) {
  int res = eta > 1.f ? 32 : 128;
  std::vector<double> xs, ws;
  gauss_legendre(res, xs, ws);
  float sum = 0.f;
  for (int iy = 0; iy < res; ++iy)
    for (int ix = 0; ix < res; ++ix) {
      float nx = std::fmaf((float)xs[ix], .5f, .5f), ny = std::fmaf((float)xs[iy], .5f, .5f);
      float pdf;
      mtx::V3 m = distr.sample(wi, mtx::V2{nx, ny}, &pdf);
      mtx::V3 wo = mtx::reflect_m(wi, m);
      float f = mtx::fresnel_dielectric(mtx::dot(wi, m), eta).r * distr.smith_g1(wo, m);
      if (!(f == f)) f = 0.f;
      sum += f * (float)ws[ix] * (float)ws[iy];
    }
  return sum * .25f;
}

extern "C" int mtx_roughplastic_tables(uint32_t distribution, float alpha, float eta, float *table_out,
                                       float *internal_refl_out) {
  if (!table_out || !internal_refl_out || !(alpha > 0.f) || !(eta > 0.f)) {
    mtx_set_error("mtx_roughplastic_tables: bad argument");
    return MTX_E_ARG;
  }
  mtx::Microfacet distr;
  distr.type = distribution ? mtx::MICROFACET_BECKMANN : mtx::MICROFACET_GGX;
  distr.alpha = alpha;
  const int R = MTX_ROUGH_TRANSMITTANCE_RES;
  float internal = 0.f;
  for (int i = 0; i < R; ++i) {
    float mu = std::max(1e-6f, (float)i / (float)(R - 1));
    mtx::V3 wi = mtx::V3{std::sqrt(1.f - mu * mu), 0.f, mu};
    table_out[i] = 1.f - eval_reflectance(distr, wi, eta);
    internal += eval_reflectance(distr, wi, 1.f / eta) * mu;
  }
  *internal_refl_out = internal / (float)R * 2.f;
  return MTX_OK;
}
