// renderer.cc — GpuRayIntegrator, WavefrontRenderer and MegaKernel over the C ABI.
#include <stdexcept>

#include "rt/material.h"
#include "rt/renderer.h"

namespace rt::integrator {

namespace {
void check(int rc, const char* what) {
  if (rc != RTX_OK) throw std::runtime_error(std::string(what) + ": " + rtx_last_error());
}
}  // namespace

GpuRayIntegrator::GpuRayIntegrator(const scene::Scene* world, int device, int precision)
    : world_(world), device_(device), precision_(precision) {
  if (!world_) throw std::invalid_argument("GpuRayIntegrator: world is null");
  flat_ = scene::Flatten(*world_);
  const rtx_scene_desc d = flat_.desc();
  check(rtx_scene_create(device_, &d, &dev_), "rtx_scene_create");
}

GpuRayIntegrator::~GpuRayIntegrator() { rtx_scene_destroy(dev_); }

// cpu_ray_integrator.h:18-46 contract on the GPU: [0.001f, +inf), hit flag per record,
// HitRecord::mat re-attached from the material id.
void GpuRayIntegrator::IntersectBatch(const std::vector<core::Ray>& rays, std::vector<geom::HitRecord>& hits) const {
  hits.resize(rays.size());
  if (rays.empty()) return;
  std::vector<rtx_ray> r(rays.size());
  for (size_t i = 0; i < rays.size(); i++)
    for (int k = 0; k < 3; k++) r[i].origin[k] = rays[i].origin()[k], r[i].direction[k] = rays[i].direction()[k];
  std::vector<rtx_hit> h(rays.size());
  check(rtx_intersect(dev_, r.data(), r.size(), h.data(), RTX_SEAM_TMIN, core::kInfinity, precision_),
        "rtx_intersect");
  for (size_t i = 0; i < rays.size(); i++) {
    geom::HitRecord& o = hits[i];
    o.hit = h[i].hit != 0;
    if (!o.hit) {
      o.mat.reset();
      continue;
    }
    o.t = h[i].t;
    o.p = core::Point3(h[i].p[0], h[i].p[1], h[i].p[2]);
    o.normal = core::Vec3(h[i].normal[0], h[i].normal[1], h[i].normal[2]);
    o.front_face = h[i].front_face != 0;
    o.u = h[i].u, o.v = h[i].v;
    o.mat = flat_.material_ptrs.at(h[i].material);
  }
}

}  // namespace rt::integrator

namespace rt::renderer {

rtx_render_params DefaultParams(int spp, int max_depth) {
  rtx_render_params p{};
  p.spp = spp;
  p.max_depth = max_depth;
  p.adaptive = 1;
  p.min_spp = 16;                        // wavefront.cc:43
  p.rel_threshold = (double)0.05f;       // wavefront.cc:42 (const float)
  p.seed = 1234;
  // the persistent schedule gives the same pixels as the bounce-synchronous wavefront one
  // (same per-path RNG streams, same per-pixel accumulation order) and is the fast kernel
  p.mode = RTX_MODE_PERSISTENT;
  p.precision = RTX_PREC_PARITY;
  return p;
}

WavefrontRenderer::WavefrontRenderer(const scene::Scene& w, const scene::Camera& c, integrator::RayIntegrator& i,
                                     int max_depth, int max_samples, int /*batch_size*/)
    : world(w), cam(c), integrator(i), params_(DefaultParams(max_samples, max_depth)) {}

WavefrontRenderer::~WavefrontRenderer() {
  for (rtx_scene* s : extra_) rtx_scene_destroy(s);
}

void WavefrontRenderer::set_devices(const std::vector<int>& devices, int stripe_rows) {
  // devices[0] renders through the integrator's own scene: it must be the integrator's device
  // (a list without it would leave a listed device unused).  A device may appear more than
  // once: each entry gets its own scene copy, thread and stream (rtx_render_multi).
  auto* gpu = dynamic_cast<integrator::GpuRayIntegrator*>(&integrator);
  const int own = gpu ? gpu->device() : 0;
  if (!devices.empty() && devices[0] != own)
    throw std::invalid_argument("WavefrontRenderer::set_devices: the first device must be the integrator's (device " +
                                std::to_string(own) + ")");
  for (rtx_scene* s : extra_) rtx_scene_destroy(s);
  extra_.clear();
  devices_ = devices;
  stripe_rows_ = stripe_rows > 0 ? stripe_rows : 8;
}

void WavefrontRenderer::set_gpus(int n) {
  int count = 0;
  if (rtx_device_count(&count) != RTX_OK) throw std::runtime_error(std::string("rtx_device_count: ") + rtx_last_error());
  if (n < 1 || n > count) throw std::invalid_argument("WavefrontRenderer::set_gpus: " + std::to_string(n) +
                                                      " GPUs requested, " + std::to_string(count) + " present");
  auto* gpu = dynamic_cast<integrator::GpuRayIntegrator*>(&integrator);
  const int first = gpu ? gpu->device() : 0;
  std::vector<int> d{first};
  for (int k = 0; (int)d.size() < n; k++)
    if (k != first) d.push_back(k);
  set_devices(d, stripe_rows_);
}

void WavefrontRenderer::Render() { Render(std::cout); }

void WavefrontRenderer::Render(std::ostream& out) {
  auto* gpu = dynamic_cast<integrator::GpuRayIntegrator*>(&integrator);
  if (!gpu)
    throw std::invalid_argument(
        "WavefrontRenderer (MI355X): the integrator must be a GpuRayIntegrator; shading runs on the device");
  const rtx_camera& dc = cam.device();
  if (dc.image_width <= 0) throw std::invalid_argument("WavefrontRenderer: camera not initialised");
  rtx_render_params p = params_;
  p.x0 = p.y0 = p.w = p.h = 0;
  p.stripe_rows = 0;
  const int64_t n = (int64_t)dc.image_width * dc.image_height;
  rgb_.assign(3 * n, 0.0);
  spp_.assign(n, 0);
  // wavefront.cc:238-241: the P3 text is formatted on the device (rtx_render_p3)
  std::string bytes(rtx_p3_max_bytes(dc.image_width, dc.image_height), '\0');
  size_t len = 0;
  if (devices_.size() > 1) {  // one frame over several devices, gathered on the host
    if (extra_.empty()) {
      const rtx_scene_desc d = gpu->flat().desc();
      for (size_t k = 1; k < devices_.size(); k++) {
        rtx_scene* s = nullptr;
        if (rtx_scene_create(devices_[k], &d, &s) != RTX_OK)
          throw std::runtime_error(std::string("rtx_scene_create: ") + rtx_last_error());
        extra_.push_back(s);
      }
    }
    std::vector<rtx_scene*> all{gpu->device_scene()};
    all.insert(all.end(), extra_.begin(), extra_.end());
    p.stripe_rows = stripe_rows_, p.stripe_index = 0, p.stripe_count = 0;
    if (rtx_render_multi(all.data(), (int32_t)all.size(), &dc, &p, rgb_.data(), spp_.data(), &stats_, nullptr) !=
            RTX_OK ||
        rtx_encode_p3(all[0], rgb_.data(), dc.image_width, dc.image_height, bytes.data(), bytes.size(), &len) !=
            RTX_OK)
      throw std::runtime_error(std::string("rtx_render_multi: ") + rtx_last_error());
    out.write(bytes.data(), (std::streamsize)len);
    return;
  }
  if (rtx_render_p3(gpu->device_scene(), &dc, &p, bytes.data(), bytes.size(), &len, rgb_.data(), spp_.data(), &stats_) != RTX_OK)
    throw std::runtime_error(std::string("rtx_render_p3: ") + rtx_last_error());
  out.write(bytes.data(), (std::streamsize)len);
}

MegaKernel::MegaKernel(scene::Scene& scene, scene::Camera& camera, integrator::Sampler& sampler, int device)
    : sampler_(sampler), world_(scene), cam_(camera), device_(device) {}

void MegaKernel::Render() { Render(std::cout); }

void MegaKernel::Render(std::ostream& out) {
  cam_.Initialize();  // mega_kernel.h:16
  integrator::GpuRayIntegrator gpu(&world_, device_);
  const rtx_camera& dc = cam_.device();
  rtx_render_params p = DefaultParams(sampler_.num_samples(), cam_.max_depth_);
  p.adaptive = 0;
  if (auto* a = dynamic_cast<const integrator::AdaptiveSampler*>(&sampler_)) {
    p.adaptive = 1;
    p.min_spp = a->min_samples();
    p.rel_threshold = (double)a->threshold();
  }
  p.mode = RTX_MODE_MEGAKERNEL;
  p.seed = seed_;
  rtx_stats st{};
  rgb_.assign(3 * (size_t)dc.image_width * dc.image_height, 0.0);
  std::string bytes(rtx_p3_max_bytes(dc.image_width, dc.image_height), '\0');
  size_t len = 0;
  if (rtx_render_p3(gpu.device_scene(), &dc, &p, bytes.data(), bytes.size(), &len, rgb_.data(), nullptr, &st) != RTX_OK)
    throw std::runtime_error(std::string("rtx_render_p3: ") + rtx_last_error());
  out.write(bytes.data(), (std::streamsize)len);
}

}  // namespace rt::renderer
