// rt/integrator.h — the batch closest-hit seam (mirrors the reference's
// src/integrator/ray_integrator.h:30-37, ray_state.h, pixel_state.h, sampler.h).
#pragma once

#include <memory>
#include <vector>

#include "rt/core.h"
#include "rt/geom.h"
#include "rt/scene.h"
#include "rtx.h"

namespace rt::integrator {

struct RayState {  // ray_state.h:8-13
  core::Ray r;
  int pixel_index = 0;
  int depth = 0;
  core::Color throughput = core::Color(1, 1, 1);
};

struct PixelState {  // pixel_state.h:13-19 (the GPU keeps the same fields per pixel)
  core::Color sum, mean, m2;
  int samples = 0;
  bool converged = false;
};

class RayIntegrator {  // ray_integrator.h:30-37
 public:
  virtual ~RayIntegrator() = default;
  virtual void IntersectBatch(const std::vector<core::Ray>& rays, std::vector<geom::HitRecord>& hits) const = 0;
};

// Drop-in replacement for CPURayIntegrator (cpu_ray_integrator.h:13-50): same contract
// (hits resized to rays.size(), interval [0.001f, +inf), HitRecord::mat re-attached from
// the material id) computed by rtx_intersect on the MI355X.  Holds a non-owning pointer to
// the world like the reference; the device copy is made on construction.
class GpuRayIntegrator : public RayIntegrator {
 public:
  explicit GpuRayIntegrator(const scene::Scene* world, int device = 0, int precision = RTX_PREC_PARITY);
  ~GpuRayIntegrator() override;
  GpuRayIntegrator(const GpuRayIntegrator&) = delete;
  GpuRayIntegrator& operator=(const GpuRayIntegrator&) = delete;
  void IntersectBatch(const std::vector<core::Ray>& rays, std::vector<geom::HitRecord>& hits) const override;
  rtx_scene* device_scene() const { return dev_; }
  const scene::FlatScene& flat() const { return flat_; }
  int device() const { return device_; }
  int precision() const { return precision_; }

 private:
  const scene::Scene* world_;
  scene::FlatScene flat_;
  rtx_scene* dev_ = nullptr;
  int device_, precision_;
};

// Samplers (sampler.h): configuration of the MegaKernel renderer on the GPU.
class Sampler {
 public:
  virtual ~Sampler() = default;
  virtual int num_samples() const = 0;
};
class DefaultSampler : public Sampler {  // sampler.h:22-37
 public:
  explicit DefaultSampler(int n) : n_(n) {}
  int num_samples() const override { return n_; }

 private:
  int n_;
};
// sampler.h:44-82: per pixel until the relative error of the running sums drops below
// `threshold` (after min_samples), at most max_samples + 1 samples.
class AdaptiveSampler : public Sampler {
 public:
  AdaptiveSampler(int min_samples, int max_samples, float threshold)
      : min_samples_(min_samples), max_samples_(max_samples), threshold_(threshold) {}
  int num_samples() const override { return max_samples_; }
  int min_samples() const { return min_samples_; }
  float threshold() const { return threshold_; }

 private:
  int min_samples_, max_samples_;
  float threshold_;
};

}  // namespace rt::integrator
