// gpu_ray_integrator.h — reference-side file (add as src/integrator/gpu_ray_integrator.h of
// Luke-TS/3360-ray-tracer): a drop-in for CPURayIntegrator (cpu_ray_integrator.h:13-50) whose
// IntersectBatch runs on the MI355X through the C ABI (include/rtx.h).  With it, main.cc:190
// becomes `integrator::GpuRayIntegrator integrator(&world);` and the reference's own
// WavefrontRenderer::Render keeps its CPU shading loop (hybrid mode).
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "core/interval.h"
#include "integrator/ray_integrator.h"
#include "rtx.h"
#include "rtx_flatten.h"

namespace rt::integrator {

class GpuRayIntegrator : public RayIntegrator {
 public:
  explicit GpuRayIntegrator(const scene::Scene* world, int device = 0, int precision = RTX_PREC_PARITY)
      : flat_(Flatten(*world)), precision_(precision) {
    const rtx_scene_desc d = flat_.desc();
    if (rtx_scene_create(device, &d, &dev_) != RTX_OK)
      throw std::runtime_error(std::string("rtx_scene_create: ") + rtx_last_error());
  }
  ~GpuRayIntegrator() { rtx_scene_destroy(dev_); }  // RayIntegrator has no virtual destructor
  GpuRayIntegrator(const GpuRayIntegrator&) = delete;
  GpuRayIntegrator& operator=(const GpuRayIntegrator&) = delete;

  // cpu_ray_integrator.h:18-46: hits resized to rays.size(), interval [0.001f, +inf), rec.hit
  // set for every ray, HitRecord::mat re-attached from the material id
  void IntersectBatch(const std::vector<core::Ray>& rays, std::vector<geom::HitRecord>& hits) const override {
    hits.resize(rays.size());
    if (rays.empty()) return;
    std::vector<rtx_ray> r(rays.size());
    for (size_t i = 0; i < rays.size(); i++)
      for (int k = 0; k < 3; k++) r[i].origin[k] = rays[i].origin()[k], r[i].direction[k] = rays[i].direction()[k];
    std::vector<rtx_hit> h(rays.size());
    if (rtx_intersect(dev_, r.data(), r.size(), h.data(), RTX_SEAM_TMIN, core::kInfinity, precision_) != RTX_OK)
      throw std::runtime_error(std::string("rtx_intersect: ") + rtx_last_error());
    for (size_t i = 0; i < rays.size(); i++) {
      geom::HitRecord& o = hits[i];
      o.hit = h[i].hit != 0;
      if (!o.hit) continue;
      o.t = h[i].t;
      o.p = core::Point3(h[i].p[0], h[i].p[1], h[i].p[2]);
      o.normal = core::Vec3(h[i].normal[0], h[i].normal[1], h[i].normal[2]);
      o.front_face = h[i].front_face != 0;
      o.u = h[i].u, o.v = h[i].v;
      o.mat = flat_.mat_ptrs[h[i].material];
    }
  }

  rtx_scene* device_scene() const { return dev_; }
  const RtxScene& flat() const { return flat_; }

 private:
  RtxScene flat_;
  int precision_;
  rtx_scene* dev_ = nullptr;
};

}  // namespace rt::integrator
