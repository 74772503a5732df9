// capi_host.cc — the host-side part of include/rtx.h: scene assembly helpers and
// cameras.json presets, implemented with the C++ host API (rt::scene / rt::geom).
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

#include "rt/image.h"
#include "rt/scene.h"
#include "rtx.h"

struct rtx_host_scene {
  std::shared_ptr<rt::scene::Scene> root;
  rt::scene::FlatScene flat;
  bool bvh = false;
};

// rtx_last_error() is defined with the device part; host helpers report through it too.
extern "C" void rtx_internal_set_error(const char* msg);

namespace {
int host_fail(int code, const std::string& m) {
  rtx_internal_set_error(m.c_str());
  return code;
}
}  // namespace

namespace {
int finish(std::shared_ptr<rt::scene::Scene> root, rtx_host_scene** out) {
  auto* s = new rtx_host_scene;
  s->root = std::move(root);
  s->flat = rt::scene::Flatten(*s->root);
  s->bvh = !s->flat.nodes.empty() || (s->root->Objects().size() == 1 &&
                                       dynamic_cast<const rt::geom::Bvh*>(s->root->Objects()[0].get()));
  *out = s;
  return RTX_OK;
}
}  // namespace

extern "C" {

int rtx_host_scene_load(const char* path, const char* asset_dir, rtx_host_scene** out) {
  if (!path || !out) return host_fail(RTX_ERR_INVALID, "NULL argument");
  try {
    return finish(rt::scene::LoadSceneFile(path, asset_dir ? asset_dir : ""), out);
  } catch (const std::exception& e) {
    return host_fail(RTX_ERR_IO, e.what());
  }
}

int rtx_host_scene_recipe(const char* name, uint32_t seed, const char* asset_dir, rtx_host_scene** out) {
  if (!name || !out) return host_fail(RTX_ERR_INVALID, "NULL argument");
  try {
    return finish(rt::scene::BuildRecipe(name, seed, asset_dir ? asset_dir : ""), out);
  } catch (const std::exception& e) {
    return host_fail(RTX_ERR_IO, e.what());
  }
}

int rtx_host_scene_write(const rtx_host_scene* s, const char* path) {
  if (!s || !path) return host_fail(RTX_ERR_INVALID, "NULL argument");
  try {
    rt::scene::WriteSceneFile(s->flat, s->bvh, path);
  } catch (const std::exception& e) {
    return host_fail(RTX_ERR_IO, e.what());
  }
  return RTX_OK;
}

int rtx_host_scene_desc(const rtx_host_scene* s, rtx_scene_desc* out) {
  if (!s || !out) return host_fail(RTX_ERR_INVALID, "NULL argument");
  *out = s->flat.desc();
  return RTX_OK;
}

int rtx_host_scene_prim_indices(const rtx_host_scene* s, int32_t* out, int64_t n) {
  if (!s || !out) return host_fail(RTX_ERR_INVALID, "NULL argument");
  if (n != (int64_t)s->flat.prim_indices.size()) return host_fail(RTX_ERR_INVALID, "n != number of prim indices");
  std::memcpy(out, s->flat.prim_indices.data(), n * sizeof(int32_t));
  return RTX_OK;
}

// Hittable::BoundingBox of each primitive record, as the host classes compute it
// (sphere.h, triangle.h:18-38, rect.h:42-45,87-89,132-134): the SAH builder's input.
int rtx_prim_bounds(const rtx_prim* prims, int64_t n, double* out) {
  if ((!prims || !out) && n > 0) return host_fail(RTX_ERR_INVALID, "NULL argument");
  using rt::core::Point3;
  using rt::core::Vec3;
  for (int64_t i = 0; i < n; i++) {
    const rtx_prim& p = prims[i];
    const double* g = p.g;
    rt::geom::Aabb b;
    if (p.kind == RTX_PRIM_SPHERE) {
      const Vec3 rv(g[3], g[3], g[3]);
      const Point3 c(g[0], g[1], g[2]);
      b = rt::geom::Aabb(Point3(c + rv), Point3(c - rv));
    } else if (p.kind == RTX_PRIM_TRIANGLE) {
      Point3 mn(std::fmin(g[0], std::fmin(g[3], g[6])), std::fmin(g[1], std::fmin(g[4], g[7])),
                std::fmin(g[2], std::fmin(g[5], g[8])));
      Point3 mx(std::fmax(g[0], std::fmax(g[3], g[6])), std::fmax(g[1], std::fmax(g[4], g[7])),
                std::fmax(g[2], std::fmax(g[5], g[8])));
      const double eps = 1e-6f;
      mn += -Vec3(eps, eps, eps);
      mx += Vec3(eps, eps, eps);
      b = rt::geom::Aabb(mn, mx);
    } else if (p.kind >= RTX_PRIM_XY_RECT && p.kind <= RTX_PRIM_YZ_RECT) {
      rt::geom::AxisRect r(p.kind, g[0], g[1], g[2], g[3], g[4], nullptr);
      b = r.BoundingBox();
    } else {
      return host_fail(RTX_ERR_INVALID, "unknown primitive kind");
    }
    const double v[6] = {b.x.min_, b.y.min_, b.z.min_, b.x.max_, b.y.max_, b.z.max_};
    std::memcpy(out + 6 * i, v, sizeof v);
  }
  return RTX_OK;
}

int rtx_bvh_build_host(const double* bounds, int64_t n, rtx_bvh_node* out_nodes, int64_t* out_n_nodes,
                       uint32_t* out_prim_indices) {
  if ((!bounds && n > 0) || !out_nodes || !out_n_nodes || !out_prim_indices)
    return host_fail(RTX_ERR_INVALID, "NULL argument");
  if (n < 0 || n > 0x3FFFFFFF) return host_fail(RTX_ERR_INVALID, "primitive count out of range");
  std::vector<rt::geom::Aabb> b(n);
  for (int64_t i = 0; i < n; i++) {
    const double* q = bounds + 6 * i;
    b[i] = rt::geom::Aabb(rt::core::Interval(q[0], q[3]), rt::core::Interval(q[1], q[4]),
                          rt::core::Interval(q[2], q[5]));
  }
  std::vector<int> idx;
  std::vector<rt::geom::BvhNodeGPU> nodes;
  rt::geom::BuildSah(b, idx, nodes);
  for (size_t i = 0; i < nodes.size(); i++) {
    rtx_bvh_node& o = out_nodes[i];
    const rt::geom::Aabb& a = nodes[i].bbox;
    o.lo[0] = a.x.min_, o.lo[1] = a.y.min_, o.lo[2] = a.z.min_;
    o.hi[0] = a.x.max_, o.hi[1] = a.y.max_, o.hi[2] = a.z.max_;
    o.left_first = nodes[i].left_pIdx, o.right_count = nodes[i].right_pCnt, o.is_leaf = nodes[i].isLeaf, o.pad_ = 0;
  }
  for (int64_t i = 0; i < n; i++) out_prim_indices[i] = (uint32_t)idx[i];
  *out_n_nodes = (int64_t)nodes.size();
  return RTX_OK;
}

int rtx_host_scene_destroy(rtx_host_scene* s) {
  delete s;
  return RTX_OK;
}

int rtx_camera_config_load(const char* json_path, const char* preset, rtx_camera_config* out) {
  if (!json_path || !preset || !out) return host_fail(RTX_ERR_INVALID, "NULL argument");
  try {
    auto cams = rt::scene::loadCameras(json_path);
    auto it = cams.find(preset);
    if (it == cams.end()) return host_fail(RTX_ERR_INVALID, std::string("camera preset not found: ") + preset);
    const auto& c = it->second;
    std::memset(out, 0, sizeof *out);
    out->aspect_ratio = c.aspect_ratio, out->image_width = c.image_width;
    out->samples_per_pixel = c.samples_per_pixel, out->max_depth = c.max_depth, out->vfov = c.vfov;
    for (int i = 0; i < 3; i++) out->lookfrom[i] = c.lookfrom[i], out->lookat[i] = c.lookat[i], out->vup[i] = c.vup[i];
    out->defocus_angle = c.defocus_angle, out->focus_dist = c.focus_dist;
  } catch (const std::exception& e) {
    return host_fail(RTX_ERR_IO, e.what());
  }
  return RTX_OK;
}

}  // extern "C"

// Image::Load (scene/image.cc:16-73) as a C entry point: the texels the renderer samples, or
// (linear8) the 8-bit decode before stb's gamma step.  texels == NULL: size query.
int rtx_image_load(const char* path, int32_t linear8, int32_t* width, int32_t* height, uint8_t* texels,
                   size_t cap) {
  if (!path || !width || !height) return host_fail(RTX_ERR_INVALID, "NULL argument");
  int w = 0, h = 0;
  std::vector<uint8_t> px;
  std::string err;
  if (!rt::scene::LoadTexels(path, w, h, px, err, linear8 != 0)) return host_fail(RTX_ERR_IO, err);
  *width = w, *height = h;
  if (texels) {
    if (cap < px.size()) return host_fail(RTX_ERR_INVALID, "texel buffer too small");
    std::memcpy(texels, px.data(), px.size());
  }
  return RTX_OK;
}
