// rt/geom.h — geometry descriptors of the host API (mirrors the reference's src/geom/:
// hittable.h, aabb.h, sphere.h, triangle.h, rect.h, bvh.h, mesh.h).
//
// Objects here describe the scene; closest-hit queries run on the GPU (rtx_intersect /
// rtx_render).  The SAH BVH build is host code that reproduces the reference's layout
// byte for byte (nodes()/prim_indices(), bvh.h:134-136), which the device kernels traverse.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include "rt/core.h"
#include "rtx.h"

namespace rt::material {
class Material;
}

namespace rt::geom {

class HitRecord {  // hittable.h:18-42
 public:
  bool hit = false;
  core::Point3 p;
  core::Vec3 normal;
  std::shared_ptr<material::Material> mat;
  double t = 0;
  bool front_face = false;
  double u = 0, v = 0;
  void set_face_normal(const core::Ray& r, const core::Vec3& outward) {
    front_face = core::Dot(r.direction(), outward) < 0;
    normal = front_face ? outward : -outward;
  }
};

enum HittableType {  // hittable.h:45-49
  HITTABLE_SPHERE = 0,
  HITTABLE_TRIANGLE = 1,
  HITTABLE_SQUARE = 2,
};

class Aabb {  // aabb.h
 public:
  core::Interval x, y, z;
  Aabb() {}
  Aabb(const core::Interval& x_, const core::Interval& y_, const core::Interval& z_) : x(x_), y(y_), z(z_) {}
  Aabb(const core::Point3& a, const core::Point3& b) {
    x = a[0] <= b[0] ? core::Interval(a[0], b[0]) : core::Interval(b[0], a[0]);
    y = a[1] <= b[1] ? core::Interval(a[1], b[1]) : core::Interval(b[1], a[1]);
    z = a[2] <= b[2] ? core::Interval(a[2], b[2]) : core::Interval(b[2], a[2]);
  }
  Aabb(const Aabb& a, const Aabb& b) : x(a.x, b.x), y(a.y, b.y), z(a.z, b.z) {}
  Aabb(const Aabb& b, const core::Vec3& p)
      : x(std::min(b.x.min_, p.x()), std::max(b.x.max_, p.x())),
        y(std::min(b.y.min_, p.y()), std::max(b.y.max_, p.y())),
        z(std::min(b.z.min_, p.z()), std::max(b.z.max_, p.z())) {}
  const core::Interval& axis_interval(int n) const { return n == 1 ? y : (n == 2 ? z : x); }
  core::Vec3 min() const { return {x.min_, y.min_, z.min_}; }
  core::Vec3 max() const { return {x.max_, y.max_, z.max_}; }
  core::Vec3 center() const {
    return core::Vec3(0.5 * (x.min_ + x.max_), 0.5 * (y.min_ + y.max_), 0.5 * (z.min_ + z.max_));
  }
  int LongestAxis() const {
    const double dx = x.max_ - x.min_, dy = y.max_ - y.min_, dz = z.max_ - z.min_;
    if (dx >= dy && dx >= dz) return 0;
    return dy >= dz ? 1 : 2;
  }
  double SurfaceArea() const {
    const double dx = x.max_ - x.min_, dy = y.max_ - y.min_, dz = z.max_ - z.min_;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

class Hittable {  // hittable.h:51-62
 public:
  virtual ~Hittable() = default;
  virtual Aabb BoundingBox() const = 0;
  virtual int TypeId() const = 0;
  virtual int ObjectIndex() const = 0;
  virtual void set_object_index(int i) = 0;
  // Device primitive record (kind + geometry; material filled by the flattener).  false
  // for aggregates (Scene, Bvh).
  virtual bool ToPrim(rtx_prim* out) const { return false; }
  virtual std::shared_ptr<material::Material> GetMaterial() const { return nullptr; }
};

class Primitive : public Hittable {
 public:
  explicit Primitive(std::shared_ptr<material::Material> m) : mat_(std::move(m)) {}
  int ObjectIndex() const override { return index_; }
  void set_object_index(int i) override { index_ = i; }
  std::shared_ptr<material::Material> GetMaterial() const override { return mat_; }

 protected:
  std::shared_ptr<material::Material> mat_;
  int index_ = -1;
};

class Sphere : public Primitive {  // sphere.h:13-88
 public:
  Sphere(const core::Point3& center, double radius, std::shared_ptr<material::Material> mat)
      : Primitive(std::move(mat)), center_(center), radius_(radius) {
    core::Vec3 rv(radius, radius, radius);
    bbox_ = Aabb(core::Point3(center + rv), core::Point3(center - rv));
  }
  Aabb BoundingBox() const override { return bbox_; }
  int TypeId() const override { return HITTABLE_SPHERE; }
  bool ToPrim(rtx_prim* o) const override;
  const core::Point3& center() const { return center_; }
  double radius() const { return radius_; }

 private:
  core::Point3 center_;
  double radius_;  // raw value; the device applies fmax(0, r) like sphere.h:17
  Aabb bbox_;
};

class Triangle : public Primitive {  // triangle.h:12-111
 public:
  Triangle(const core::Point3& a, const core::Point3& b, const core::Point3& c,
           std::shared_ptr<material::Material> mat);
  Aabb BoundingBox() const override { return bbox_; }
  int TypeId() const override { return HITTABLE_TRIANGLE; }
  bool ToPrim(rtx_prim* o) const override;

 private:
  core::Point3 a_, b_, c_;
  Aabb bbox_;
};

// Axis-aligned rectangles (rect.h): all three report HITTABLE_SQUARE like the reference.
class AxisRect : public Primitive {
 public:
  AxisRect(int kind, double a0, double a1, double b0, double b1, double k, std::shared_ptr<material::Material> mat)
      : Primitive(std::move(mat)), kind_(kind), a0_(a0), a1_(a1), b0_(b0), b1_(b1), k_(k) {}
  Aabb BoundingBox() const override;
  int TypeId() const override { return HITTABLE_SQUARE; }
  bool ToPrim(rtx_prim* o) const override;

 private:
  int kind_;
  double a0_, a1_, b0_, b1_, k_;
};
class xy_rect : public AxisRect {
 public:
  xy_rect(double x0, double x1, double y0, double y1, double k, std::shared_ptr<material::Material> m)
      : AxisRect(RTX_PRIM_XY_RECT, x0, x1, y0, y1, k, std::move(m)) {}
};
class xz_rect : public AxisRect {
 public:
  xz_rect(double x0, double x1, double z0, double z1, double k, std::shared_ptr<material::Material> m)
      : AxisRect(RTX_PRIM_XZ_RECT, x0, x1, z0, z1, k, std::move(m)) {}
};
class yz_rect : public AxisRect {
 public:
  yz_rect(double y0, double y1, double z0, double z1, double k, std::shared_ptr<material::Material> m)
      : AxisRect(RTX_PRIM_YZ_RECT, y0, y1, z0, z1, k, std::move(m)) {}
};

}  // namespace rt::geom

namespace rt::scene {
class Scene;
}

namespace rt::geom {

// Bvh (bvh.h:28-136): binned-SAH build (16 bins, leaves <= 4 unless SAH stops, libstdc++
// partition order) flattened pre-order into the reference's BvhNodeGPU layout.
struct BvhNodeGPU {
  Aabb bbox;
  uint32_t left_pIdx;
  uint32_t right_pCnt;
  uint32_t isLeaf;
};

// The binned-SAH build over primitive boxes (bvh.h:166-367): nodes in pre-order and the
// leaf-order permutation.  Bvh::Build and rtx_bvh_build_host use it.
void BuildSah(const std::vector<Aabb>& bounds, std::vector<int>& prim_indices, std::vector<BvhNodeGPU>& nodes);

class Bvh : public Hittable {
 public:
  explicit Bvh(scene::Scene& scene);
  explicit Bvh(std::vector<std::shared_ptr<Hittable>>& objects);
  Aabb BoundingBox() const override { return nodes_.empty() ? Aabb() : nodes_[0].bbox; }
  int TypeId() const override { return -1; }
  int ObjectIndex() const override { return -1; }
  void set_object_index(int) override {}
  const std::vector<BvhNodeGPU>& nodes() const { return nodes_; }
  const std::vector<int>& prim_indices() const { return prim_indices_; }
  const std::vector<std::shared_ptr<Hittable>>& primitives() const { return primitives_; }

 private:
  void Build();
  std::vector<std::shared_ptr<Hittable>> primitives_;
  std::vector<int> prim_indices_;
  std::vector<BvhNodeGPU> nodes_;
};

// Mesh (mesh.h): triangle soup; the BVH is built over its triangles.
class Mesh {
 public:
  Mesh(const std::vector<core::Point3>& vertices, const std::vector<std::array<int, 3>>& indices,
       std::shared_ptr<material::Material> mat);
  std::vector<std::shared_ptr<Hittable>> tris;
};

// load_obj (load_obj.h:10-55): 'v x y z' parsed as float (tinyobjloader real_t), triangle
// faces only, vertices centred on their centroid then scaled.  Throws on I/O failure.
std::shared_ptr<Mesh> load_obj(const std::string& filename, std::shared_ptr<material::Material> mat, double scale);

}  // namespace rt::geom
