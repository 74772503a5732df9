// rt/scene.h — Scene, CameraConfig/cameras.json, Camera (mirrors the reference's
// src/scene/scene.h and src/scene/camera.h) plus the flattener that turns a Scene into the
// device description of include/rtx.h.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "rt/core.h"
#include "rt/geom.h"
#include "rt/material.h"
#include "rtx.h"

namespace rt::scene {

class Scene : public geom::Hittable {  // scene.h:15-74
 public:
  std::vector<std::shared_ptr<geom::Hittable>> objects_;
  Scene() = default;
  explicit Scene(std::shared_ptr<geom::Hittable> object) { Add(std::move(object)); }
  void Add(const std::shared_ptr<geom::Hittable>& object) {
    if (!object) return;
    objects_.push_back(object);
    bbox_ = geom::Aabb(bbox_, object->BoundingBox());
  }
  void Clear() {
    objects_.clear();
    bbox_ = geom::Aabb();
  }
  const std::vector<std::shared_ptr<geom::Hittable>>& Objects() const { return objects_; }
  geom::Aabb BoundingBox() const override { return bbox_; }
  int TypeId() const override { return -1; }
  int ObjectIndex() const override { return -1; }
  void set_object_index(int) override {}
  // Optional id order for materials/textures (scene files keep their ids).
  std::vector<std::shared_ptr<material::Material>> material_order;
  std::vector<std::shared_ptr<material::Texture>> texture_order;

 private:
  geom::Aabb bbox_;
};

// Flattened, device-ready description.  Supported roots (everything the reference's
// main.cc builds): a Scene of primitives (scene::Scene::Hit, linear) or a Scene holding
// exactly one Bvh.
struct FlatScene {
  std::vector<rtx_prim> prims;  // leaf order when nodes is non-empty
  std::vector<rtx_bvh_node> nodes;
  std::vector<int32_t> prim_indices;  // Bvh::prim_indices
  std::vector<rtx_material> materials;
  std::vector<rtx_texture> textures;
  std::vector<rtx_image> images;
  std::vector<std::shared_ptr<const Image>> image_refs;  // keep texels alive
  std::vector<std::shared_ptr<material::Material>> material_ptrs;
  std::vector<std::string> texture_names;  // image textures: asset name, else ""
  std::vector<rtx_prim> list_prims;        // insertion order (Bvh::primitives())
  rtx_scene_desc desc() const;
};

// .rtxs scene files (format: DESIGN.md "Scene files").  Throws std::runtime_error.
std::shared_ptr<Scene> LoadSceneFile(const std::string& path, const std::string& asset_dir);
void WriteSceneFile(const FlatScene& f, bool bvh, const std::string& path);
// The reference's scene recipes (main.cc:23-156 + SURVEY §8d): three, cornell, final,
// bunny, mixed.  seed feeds core::SeedRng before the random ones (final, mixed).
std::shared_ptr<Scene> BuildRecipe(const std::string& name, uint32_t seed, const std::string& asset_dir);
// Throws std::runtime_error for unsupported roots.
FlatScene Flatten(const Scene& root);

// ---- cameras.json (camera.h:25-67) --------------------------------------------------------
struct CameraConfig {
  double aspect_ratio = 16 / 9.0;
  int image_width = 400;
  int samples_per_pixel = 50;
  int max_depth = 10;
  double vfov = 90.0;
  core::Vec3 lookfrom = core::Point3(0, 0, 0);
  core::Vec3 lookat = core::Point3(0, 0, -1);
  core::Vec3 vup = core::Point3(0, 1, 0);
  double defocus_angle = 0.0;
  double focus_dist = 10.0;
};
// Parses one preset object of cameras.json (camelCase keys; lookfrom/lookat/vup required).
CameraConfig parseCamera(const std::string& json_object_text);
std::unordered_map<std::string, CameraConfig> loadCameras(const std::string& filename);

class Camera {  // camera.h:69-210
 public:
  double aspect_ratio_ = 1.0;
  int image_width_ = 100;
  int max_depth_ = 10;
  int samples_per_pixel_ = 10;
  double vfov_ = 90.0;
  core::Vec3 lookfrom_ = core::Point3(0, 0, 0);
  core::Vec3 lookat = core::Point3(0, 0, -1);
  core::Vec3 vup_ = core::Point3(0, 1, 0);
  double defocus_angle_ = 0;
  double focus_dist_ = 10;

  virtual ~Camera() = default;
  void SetFromConfig(const CameraConfig& cfg);
  void Initialize();  // -> rtx_camera_init (same arithmetic as camera.h:100-131)
  int get_image_height() const { return dev_.image_height; }
  int get_image_width() const { return image_width_; }
  const rtx_camera& device() const { return dev_; }

 private:
  rtx_camera dev_{};
};
class ColorCamera : public Camera {};

}  // namespace rt::scene
