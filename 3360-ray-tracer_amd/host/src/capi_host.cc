// capi_host.cc — the host-side part of include/rtx.h: scene assembly helpers and
// cameras.json presets, implemented with the C++ host API (rt::scene / rt::geom).
#include <cstring>
#include <stdexcept>
#include <string>

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
