// geom.cc — primitive descriptors, the SAH BVH builder and the OBJ loader.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "rt/geom.h"
#include "rt/material.h"
#include "rt/scene.h"

namespace rt::geom {

bool Sphere::ToPrim(rtx_prim* o) const {
  std::memset(o, 0, sizeof *o);
  o->kind = RTX_PRIM_SPHERE;
  o->g[0] = center_.x(), o->g[1] = center_.y(), o->g[2] = center_.z(), o->g[3] = radius_;
  return true;
}

Triangle::Triangle(const core::Point3& a, const core::Point3& b, const core::Point3& c,
                   std::shared_ptr<material::Material> mat)
    : Primitive(std::move(mat)), a_(a), b_(b), c_(c) {
  // triangle.h:18-38: per-axis extent padded by (double)1e-6f
  core::Point3 mn(std::fmin(a.x(), std::fmin(b.x(), c.x())), std::fmin(a.y(), std::fmin(b.y(), c.y())),
                  std::fmin(a.z(), std::fmin(b.z(), c.z())));
  core::Point3 mx(std::fmax(a.x(), std::fmax(b.x(), c.x())), std::fmax(a.y(), std::fmax(b.y(), c.y())),
                  std::fmax(a.z(), std::fmax(b.z(), c.z())));
  const double eps = 1e-6f;
  mn += -core::Vec3(eps, eps, eps);
  mx += core::Vec3(eps, eps, eps);
  bbox_ = Aabb(mn, mx);
}

bool Triangle::ToPrim(rtx_prim* o) const {
  std::memset(o, 0, sizeof *o);
  o->kind = RTX_PRIM_TRIANGLE;
  const core::Point3* v[3] = {&a_, &b_, &c_};
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) o->g[3 * i + k] = (*v[i])[k];
  return true;
}

Aabb AxisRect::BoundingBox() const {  // rect.h:42-45, 87-89, 132-134 (+-1e-4 thickness)
  if (kind_ == RTX_PRIM_XY_RECT) return Aabb(core::Point3(a0_, b0_, k_ - 0.0001), core::Point3(a1_, b1_, k_ + 0.0001));
  if (kind_ == RTX_PRIM_XZ_RECT) return Aabb(core::Point3(a0_, k_ - 0.0001, b0_), core::Point3(a1_, k_ + 0.0001, b1_));
  return Aabb(core::Point3(k_ - 0.0001, a0_, b0_), core::Point3(k_ + 0.0001, a1_, b1_));
}

bool AxisRect::ToPrim(rtx_prim* o) const {
  std::memset(o, 0, sizeof *o);
  o->kind = kind_;
  o->g[0] = a0_, o->g[1] = a1_, o->g[2] = b0_, o->g[3] = b1_, o->g[4] = k_;
  return true;
}

// ---------------------------------------------------------------------------------------
// Binned SAH build.  Reproduces the reference's BvhNodeGPU array and prim_indices exactly
// (bvh.h:39-68,166-367): 16 bins on the longest centroid axis, cost 1 + A_L/A N_L + A_R/A
// N_R (float constants widened to double), leaf if count <= 4, degenerate centroid extent,
// no split or best_cost >= count, and the same two-ended in-place partition as libstdc++'s
// std::partition for bidirectional iterators.  Nodes are emitted in pre-order.
// ---------------------------------------------------------------------------------------
namespace {

struct SahBuilder {
  std::vector<int>& idx;
  std::vector<Aabb> bounds;
  std::vector<core::Vec3> centroids;
  std::vector<BvhNodeGPU>& out;

  static int Bin(double c, double mn, double inv) {
    int b = static_cast<int>((c - mn) * inv * 16);
    return b < 0 ? 0 : (b > 15 ? 15 : b);
  }

  // two-ended partition (libstdc++ __partition, bidirectional_iterator_tag)
  template <class Pred>
  int Partition(int first, int last, Pred pred) {
    while (true) {
      while (true) {
        if (first == last) return first;
        if (pred(idx[first])) ++first;
        else break;
      }
      --last;
      while (true) {
        if (first == last) return first;
        if (!pred(idx[last])) --last;
        else break;
      }
      std::swap(idx[first], idx[last]);
      ++first;
    }
  }

  int Emit(int start, int end) {
    const int me = (int)out.size();
    out.push_back(BvhNodeGPU{});
    Aabb box = bounds[idx[start]];
    for (int i = start + 1; i < end; i++) box = Aabb(box, bounds[idx[i]]);
    out[me].bbox = box;
    const int count = end - start;
    auto leaf = [&]() {
      out[me].isLeaf = 1, out[me].left_pIdx = (uint32_t)start, out[me].right_pCnt = (uint32_t)count;
      return me;
    };
    if (count <= 4) return leaf();
    Aabb cb(centroids[idx[start]], centroids[idx[start]]);
    for (int i = start + 1; i < end; i++) cb = Aabb(cb, centroids[idx[i]]);
    const int axis = cb.LongestAxis();
    const double mn = cb.axis_interval(axis).min_;
    const double extent = cb.axis_interval(axis).max_ - mn;
    if (extent <= 0.0) return leaf();
    const double inv = 1.0 / extent;

    int cnt[16] = {0};
    Aabb bb[16];
    for (int i = start; i < end; i++) {
      const int b = Bin(centroids[idx[i]][axis], mn, inv);
      bb[b] = cnt[b] ? Aabb(bb[b], bounds[idx[i]]) : bounds[idx[i]];
      cnt[b]++;
    }
    Aabb lb[16], rb[16];
    int lc[16], rc[16];
    {
      Aabb acc;
      int n = 0;
      for (int i = 0; i < 16; i++) {
        if (cnt[i]) acc = n ? Aabb(acc, bb[i]) : bb[i], n += cnt[i];
        lb[i] = acc, lc[i] = n;
      }
      n = 0;
      for (int i = 15; i >= 0; i--) {
        if (cnt[i]) acc = n ? Aabb(acc, bb[i]) : bb[i], n += cnt[i];
        rb[i] = acc, rc[i] = n;
      }
    }
    const double area = box.SurfaceArea();
    double best = std::numeric_limits<double>::infinity();
    int split = -1;
    for (int i = 0; i < 15; i++) {
      if (lc[i] == 0 || rc[i + 1] == 0) continue;
      const double cost = (double)1.0f + (lb[i].SurfaceArea() / area) * lc[i] * (double)1.0f +
                          (rb[i + 1].SurfaceArea() / area) * rc[i + 1] * (double)1.0f;
      if (cost < best) best = cost, split = i;
    }
    if (split < 0 || best >= (double)(count * 1.0f)) return leaf();
    const int mid =
        Partition(start, end, [&](int p) { return Bin(centroids[p][axis], mn, inv) <= split; });
    if (mid == start || mid == end) return leaf();
    const int l = Emit(start, mid);
    const int r = Emit(mid, end);
    out[me].isLeaf = 0, out[me].left_pIdx = (uint32_t)l, out[me].right_pCnt = (uint32_t)r;
    return me;
  }
};

}  // namespace

Bvh::Bvh(scene::Scene& scene) : Bvh(scene.objects_) {}

Bvh::Bvh(std::vector<std::shared_ptr<Hittable>>& objects) : primitives_(objects) { Build(); }

void BuildSah(const std::vector<Aabb>& bounds, std::vector<int>& prim_indices, std::vector<BvhNodeGPU>& nodes) {
  const int n = (int)bounds.size();
  prim_indices.resize(n);
  nodes.clear();
  if (n == 0) return;
  SahBuilder b{prim_indices, bounds, {}, nodes};
  b.centroids.resize(n);
  for (int i = 0; i < n; i++) {
    prim_indices[i] = i;
    b.centroids[i] = b.bounds[i].center();
  }
  nodes.reserve(2 * (size_t)n);
  b.Emit(0, n);
}

void Bvh::Build() {
  std::vector<Aabb> bounds(primitives_.size());
  for (size_t i = 0; i < primitives_.size(); i++) bounds[i] = primitives_[i]->BoundingBox();
  BuildSah(bounds, prim_indices_, nodes_);
}

Mesh::Mesh(const std::vector<core::Point3>& v, const std::vector<std::array<int, 3>>& f,
           std::shared_ptr<material::Material> mat) {
  tris.reserve(f.size());
  for (const auto& t : f) tris.push_back(std::make_shared<Triangle>(v[t[0]], v[t[1]], v[t[2]], mat));
}

std::shared_ptr<Mesh> load_obj(const std::string& filename, std::shared_ptr<material::Material> mat, double scale) {
  std::ifstream in(filename);
  if (!in) throw std::runtime_error("load_obj: cannot open " + filename);
  std::vector<core::Point3> v;
  std::vector<std::array<int, 3>> f;
  std::string line;
  while (std::getline(in, line)) {
    if (line.size() < 3 || line[1] != ' ') continue;
    if (line[0] == 'v') {
      char* e = nullptr;
      const float x = std::strtof(line.c_str() + 2, &e);
      const float y = std::strtof(e, &e);
      const float z = std::strtof(e, &e);
      v.emplace_back(x, y, z);
    } else if (line[0] == 'f') {
      std::istringstream ss(line.substr(2));
      std::string tok;
      int ix[4], n = 0;
      while (ss >> tok && n < 4) ix[n++] = std::atoi(tok.c_str()) - 1;  // "a", "a/b", "a//c"
      if (n == 3 && !(ss >> tok)) f.push_back({ix[0], ix[1], ix[2]});
    }
  }
  for (const auto& t : f)
    for (int k : t)
      if (k < 0 || k >= (int)v.size()) throw std::runtime_error("load_obj: face index out of range in " + filename);
  core::Vec3 centroid(0.0f, 0.0f, 0.0f);
  for (const auto& p : v) centroid += p;
  if (!v.empty()) centroid /= (double)v.size();
  for (auto& p : v) p = (p - centroid) * scale;
  return std::make_shared<Mesh>(v, f, std::move(mat));
}

}  // namespace rt::geom
