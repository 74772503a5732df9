// rtx_flatten.h — reference-side file (add as src/integrator/rtx_flatten.h of
// Luke-TS/3360-ray-tracer): flattens the reference's scene graph into the C ABI's scene
// description (include/rtx.h) for rtx_scene_create.
//
// Needs the read accessors listed in integration/accessors.txt (values only) on Sphere,
// Triangle, the three rects, the four materials and the three textures.  Uses the GPU hooks
// the reference already has: Bvh::nodes() / prim_indices() / primitives() with BvhNodeGPU
// (geom/bvh.h:20-25,134-136).  Compiled against the reference's headers by
// tests/test_integration_reference.py.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <vector>

#include "geom/bvh.h"
#include "geom/rect.h"
#include "geom/sphere.h"
#include "geom/triangle.h"
#include "material/material.h"
#include "material/texture.h"
#include "rtx.h"
#include "scene/image.h"
#include "scene/scene.h"

namespace rt::integrator {

struct RtxScene {
  std::vector<rtx_prim> prims;  // BVH leaf order (a leaf's first/count index it directly)
  std::vector<rtx_bvh_node> nodes;
  std::vector<rtx_material> mats;
  std::vector<rtx_texture> texs;
  std::vector<rtx_image> imgs;
  std::vector<std::vector<uint8_t>> texels;                   // owned RGB8 copies of the images
  std::vector<std::shared_ptr<material::Material>> mat_ptrs;  // material id -> HitRecord::mat

  rtx_scene_desc desc() const {
    rtx_scene_desc d{};
    d.prims = prims.data(), d.n_prims = (int64_t)prims.size();
    d.nodes = nodes.empty() ? nullptr : nodes.data(), d.n_nodes = (int64_t)nodes.size();
    d.materials = mats.data(), d.n_materials = (int32_t)mats.size();
    d.textures = texs.data(), d.n_textures = (int32_t)texs.size();
    d.images = imgs.data(), d.n_images = (int32_t)imgs.size();
    return d;
  }
};

namespace detail {

class Flattener {
 public:
  explicit Flattener(RtxScene& s) : s_(s) {}

  int Texture(const std::shared_ptr<material::Texture>& t) {
    if (!t) throw std::runtime_error("rtx flatten: null texture");
    auto it = tex_.find(t.get());
    if (it != tex_.end()) return it->second;
    const int id = (int)s_.texs.size();
    tex_[t.get()] = id;
    s_.texs.push_back(rtx_texture{});
    rtx_texture r{};
    r.image = -1;
    if (auto* c = dynamic_cast<const material::SolidColor*>(t.get())) {
      r.kind = RTX_TEX_SOLID;
      for (int i = 0; i < 3; i++) r.color[i] = c->albedo()[i];
    } else if (auto* k = dynamic_cast<const material::CheckerTexture*>(t.get())) {
      r.kind = RTX_TEX_CHECKER;
      r.inv_scale = k->inv_scale();
      r.even = Texture(k->even());
      r.odd = Texture(k->odd());
    } else if (auto* im = dynamic_cast<const material::ImageTexture*>(t.get())) {
      r.kind = RTX_TEX_IMAGE;
      const scene::Image& img = im->image();
      if (img.Height() > 0) {  // no data: the device returns cyan like texture.h:62
        // Image keeps its RGB8 texels (after FloatToByte, image.cc:43-73) contiguous, rows
        // top-down; PixelData(0, 0) is their start
        const uint8_t* px = img.PixelData(0, 0);
        s_.texels.emplace_back(px, px + (size_t)img.Width() * img.Height() * 3);
        r.image = (int)s_.imgs.size();
        s_.imgs.push_back(rtx_image{img.Width(), img.Height(), nullptr});
      }
    } else {
      throw std::runtime_error("rtx flatten: unsupported texture type");
    }
    s_.texs[id] = r;
    return id;
  }

  int Material(const std::shared_ptr<material::Material>& m) {
    if (!m) throw std::runtime_error("rtx flatten: primitive without material");
    auto it = mat_.find(m.get());
    if (it != mat_.end()) return it->second;
    rtx_material r{};
    if (auto* l = dynamic_cast<const material::Lambertian*>(m.get())) {
      r.kind = RTX_MAT_LAMBERTIAN;
      r.texture = Texture(l->texture());
    } else if (auto* me = dynamic_cast<const material::Metal*>(m.get())) {
      r.kind = RTX_MAT_METAL;
      for (int i = 0; i < 3; i++) r.albedo[i] = me->albedo()[i];
      r.fuzz = me->fuzz();  // clamped to <= 1 by the constructor (material.cc:78-80)
    } else if (auto* d = dynamic_cast<const material::Dielectric*>(m.get())) {
      r.kind = RTX_MAT_DIELECTRIC;
      r.ref_idx = d->ref_idx();
    } else if (auto* e = dynamic_cast<const material::DiffuseLight*>(m.get())) {
      r.kind = RTX_MAT_DIFFUSE_LIGHT;
      r.texture = Texture(e->emit());
    } else {
      throw std::runtime_error("rtx flatten: unsupported material type");
    }
    const int id = (int)s_.mats.size();
    mat_[m.get()] = id;
    s_.mats.push_back(r);
    s_.mat_ptrs.push_back(m);
    return id;
  }

  // HittableType (hittable.h:45-49) reports SQUARE for all three rects: the axis comes from
  // the concrete type.
  rtx_prim Prim(const geom::Hittable& h) {
    rtx_prim p{};
    auto set = [&p](std::initializer_list<double> g) {
      int i = 0;
      for (double v : g) p.g[i++] = v;
    };
    if (auto* s = dynamic_cast<const geom::Sphere*>(&h)) {
      p.kind = RTX_PRIM_SPHERE;
      set({s->center()[0], s->center()[1], s->center()[2], s->radius()});
      p.material = Material(s->material());
    } else if (auto* t = dynamic_cast<const geom::Triangle*>(&h)) {
      p.kind = RTX_PRIM_TRIANGLE;
      set({t->a()[0], t->a()[1], t->a()[2], t->b()[0], t->b()[1], t->b()[2], t->c()[0], t->c()[1], t->c()[2]});
      p.material = Material(t->material());
    } else if (auto* r = dynamic_cast<const geom::xy_rect*>(&h)) {
      p.kind = RTX_PRIM_XY_RECT;
      set({r->x0(), r->x1(), r->y0(), r->y1(), r->k()});
      p.material = Material(r->material());
    } else if (auto* r = dynamic_cast<const geom::xz_rect*>(&h)) {
      p.kind = RTX_PRIM_XZ_RECT;
      set({r->x0(), r->x1(), r->z0(), r->z1(), r->k()});
      p.material = Material(r->material());
    } else if (auto* r = dynamic_cast<const geom::yz_rect*>(&h)) {
      p.kind = RTX_PRIM_YZ_RECT;
      set({r->y0(), r->y1(), r->z0(), r->z1(), r->k()});
      p.material = Material(r->material());
    } else {
      throw std::runtime_error("rtx flatten: unsupported primitive (only Sphere, Triangle, xy/xz/yz_rect)");
    }
    return p;
  }

 private:
  RtxScene& s_;
  std::map<const material::Texture*, int> tex_;
  std::map<const material::Material*, int> mat_;
};

}  // namespace detail

// world = a Scene whose only object is a Bvh (main.cc:60, world_root.Add(make_shared<Bvh>(world)))
// or a Scene of primitives (the flat list Scene::Hit walks, scene.h:47-61).
inline RtxScene Flatten(const scene::Scene& world) {
  RtxScene s;
  detail::Flattener f(s);
  const auto& objs = world.Objects();
  const auto* bvh = objs.size() == 1 ? dynamic_cast<const geom::Bvh*>(objs[0].get()) : nullptr;
  if (bvh) {
    for (const geom::BvhNodeGPU& n : bvh->nodes()) {  // same pre-order layout, left child = index + 1
      rtx_bvh_node r{};
      r.lo[0] = n.bbox.x.min_, r.lo[1] = n.bbox.y.min_, r.lo[2] = n.bbox.z.min_;
      r.hi[0] = n.bbox.x.max_, r.hi[1] = n.bbox.y.max_, r.hi[2] = n.bbox.z.max_;
      r.left_first = n.left_pIdx, r.right_count = n.right_pCnt, r.is_leaf = n.isLeaf;
      s.nodes.push_back(r);
    }
    for (int k : bvh->prim_indices()) s.prims.push_back(f.Prim(*bvh->primitives()[k]));
  } else {
    for (const auto& o : objs) s.prims.push_back(f.Prim(*o));
  }
  for (size_t i = 0; i < s.imgs.size(); i++) s.imgs[i].texels = s.texels[i].data();
  return s;
}

}  // namespace rt::integrator
