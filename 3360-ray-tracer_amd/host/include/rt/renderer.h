// rt/renderer.h — WavefrontRenderer and MegaKernel (mirrors the reference's
// src/renderer/wavefront.h:22-45 and mega_kernel.h:10-59) running on the MI355X.
#pragma once

#include <cstdint>
#include <iostream>
#include <vector>

#include "rt/integrator.h"
#include "rt/scene.h"
#include "rtx.h"

namespace rt::renderer {

// Same constructor and Render() as the reference.  The integrator must be a
// GpuRayIntegrator: generation, intersection, shading, Russian roulette, adaptive sampling
// and accumulation all run on the device (rtx_render, RTX_MODE_WAVEFRONT by default).
// batch_size is accepted for source compatibility; the GPU keeps whole sample groups in
// flight instead of 16k-ray batches.  Render() writes the P3 PPM to stdout like
// wavefront.cc:238-241; framebuffer() keeps the linear values.
class WavefrontRenderer {
 public:
  WavefrontRenderer(const scene::Scene& world, const scene::Camera& cam, integrator::RayIntegrator& integrator,
                    int max_depth = 10, int max_samples = 128, int batch_size = 8192);
  void Render();
  void Render(std::ostream& out);

  ~WavefrontRenderer();
  WavefrontRenderer(const WavefrontRenderer&) = delete;
  WavefrontRenderer& operator=(const WavefrontRenderer&) = delete;

  // MI355X extensions (defaults reproduce the reference's semantics)
  // Render one frame over `devices` (the integrator's device first): interleaved row
  // stripes of `stripe_rows` rows, one host thread + stream per device, gathered into one
  // host framebuffer and one P3 output (rtx_render_multi).  The pixels are the
  // same for every device count.
  void set_devices(const std::vector<int>& devices, int stripe_rows = 8);
  void set_gpus(int n);  // devices 0 .. n-1 (the integrator's device first)
  void set_seed(uint64_t s) { params_.seed = s; }
  void set_adaptive(bool on) { params_.adaptive = on ? 1 : 0; }
  void set_mode(int mode) { params_.mode = mode; }
  void set_precision(int p) { params_.precision = p; }
  rtx_render_params& params() { return params_; }
  const std::vector<double>& framebuffer() const { return rgb_; }
  const std::vector<int32_t>& samples() const { return spp_; }
  const rtx_stats& stats() const { return stats_; }

 private:
  const scene::Scene& world;
  const scene::Camera& cam;
  integrator::RayIntegrator& integrator;
  rtx_render_params params_{};
  std::vector<double> rgb_;
  std::vector<int32_t> spp_;
  rtx_stats stats_{};
  std::vector<int> devices_;          // the frame's devices, the integrator's first (set_devices)
  std::vector<rtx_scene*> extra_;     // their device-resident copies of the scene
  int stripe_rows_ = 8;
};

// MegaKernel + DefaultSampler semantics (recursive GetPixel with the Scatter API, camera.h:
// 148-174), one GPU path per (pixel, sample).
class MegaKernel {
 public:
  MegaKernel(scene::Scene& scene, scene::Camera& camera, integrator::Sampler& sampler, int device = 0);
  void Render();
  void Render(std::ostream& out);
  void set_seed(uint64_t s) { seed_ = s; }
  const std::vector<double>& framebuffer() const { return rgb_; }

 private:
  integrator::Sampler& sampler_;
  scene::Scene& world_;
  scene::Camera& cam_;
  int device_;
  uint64_t seed_ = 1234;
  std::vector<double> rgb_;
};

// Default render parameters: reference semantics (adaptive min 16 / rel float(0.05)).
rtx_render_params DefaultParams(int spp, int max_depth);

}  // namespace rt::renderer
