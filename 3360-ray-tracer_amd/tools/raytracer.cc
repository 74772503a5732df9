// raytracer — CLI drop-in for the reference binary (main.cc:158-197):
//   raytracer [camera-preset] [--scene cornell|three|final|bunny|mixed|<file.rtxs>]
//             [--cameras cameras.json] [--spp N] [--depth N] [--seed S] [--fixed]
//             [--mode wavefront|persistent|megakernel] [--precision parity|fast]
//             [--mk-adaptive MIN:THRESHOLD] [--gpus N] > out.ppm
// --gpus N renders one frame over N GPUs (interleaved row stripes, one host thread per GPU,
// one gathered framebuffer and P3 output; identical pixels for every N); --devices 0,2,3
// names the devices (a device may repeat: several streams on one GPU).
// --mk-adaptive selects the AdaptiveSampler (sampler.h:44-82) for --mode megakernel,
// with max_samples = the preset's (or --spp) samples.
// Defaults follow main.cc: preset "default" (fallback when unknown), the Cornell box
// scene (switch(4), main.cc:178-183), WavefrontRenderer with the preset's maxDepth and
// samplesPerPixel, adaptive sampling on; "Runtime: Xs" on stderr.
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "rt/renderer.h"

using namespace rt;

int main(int argc, char** argv) {
  core::Timer clock;
  std::string preset = "default", scene_name = "cornell", cameras = "cameras.json", mode = "persistent",
              precision = "parity";
  int spp = -1, depth = -1;
  uint64_t seed = 1234;
  bool fixed = false;
  std::vector<int> devices;
  int mk_min = -1, gpus = 1;
  float mk_thr = 0.0f;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::cerr << "missing value for " << a << "\n";
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--scene") scene_name = next();
    else if (a == "--cameras") cameras = next();
    else if (a == "--spp") spp = std::atoi(next().c_str());
    else if (a == "--depth") depth = std::atoi(next().c_str());
    else if (a == "--seed") seed = std::strtoull(next().c_str(), nullptr, 10);
    else if (a == "--mode") mode = next();
    else if (a == "--precision") precision = next();
    else if (a == "--fixed") fixed = true;
    else if (a == "--gpus") gpus = std::atoi(next().c_str());
    else if (a == "--devices") {
      const std::string v = next();
      for (size_t p = 0; p < v.size();) {
        size_t q = v.find(',', p);
        if (q == std::string::npos) q = v.size();
        devices.push_back(std::atoi(v.substr(p, q - p).c_str()));
        p = q + 1;
      }
    }
    else if (a == "--mk-adaptive") {
      const std::string v = next();
      const size_t c = v.find(':');
      if (c == std::string::npos) {
        std::cerr << "--mk-adaptive expects MIN:THRESHOLD\n";
        return 2;
      }
      mk_min = std::atoi(v.substr(0, c).c_str());
      mk_thr = std::strtof(v.substr(c + 1).c_str(), nullptr);
    }
    else if (!a.empty() && a[0] != '-') preset = a;
    else {
      std::cerr << "unknown option " << a << "\n";
      return 2;
    }
  }
  try {
    if (!std::ifstream(cameras)) {
      const std::string alt = scene::ResolveAsset("../../configs/cameras.json");
      if (!alt.empty()) cameras = alt;
    }
    auto cams = scene::loadCameras(cameras);
    if (!cams.count(preset)) {  // main.cc:169-172
      std::cerr << "Camera '" << preset << "' not found. Using default.\n";
      preset = "default";
    }
    scene::ColorCamera cam;
    cam.SetFromConfig(cams[preset]);
    cam.Initialize();
    std::shared_ptr<scene::Scene> world;
    if (scene_name.size() > 5 && scene_name.substr(scene_name.size() - 5) == ".rtxs")
      world = scene::LoadSceneFile(scene_name, "");
    else
      world = scene::BuildRecipe(scene_name, 1234, "");
    const int ns = spp > 0 ? spp : cam.samples_per_pixel_;
    const int md = depth >= 0 ? depth : cam.max_depth_;
    if (mode == "megakernel") {
      integrator::DefaultSampler fixed_sampler(ns);
      integrator::AdaptiveSampler adaptive_sampler(mk_min, ns, mk_thr);
      integrator::Sampler& sampler = mk_min >= 0 ? (integrator::Sampler&)adaptive_sampler : fixed_sampler;
      cam.max_depth_ = md;
      renderer::MegaKernel r(*world, cam, sampler);
      r.set_seed(seed);
      r.Render();
    } else {
      integrator::GpuRayIntegrator integ(world.get(), devices.empty() ? 0 : devices[0],
                                         precision == "fast" ? RTX_PREC_FAST : RTX_PREC_PARITY);
      renderer::WavefrontRenderer r(*world, cam, integ, md, ns, 2 * 8192);
      r.set_seed(seed);
      r.set_adaptive(!fixed);
      r.set_precision(precision == "fast" ? RTX_PREC_FAST : RTX_PREC_PARITY);
      r.set_mode(mode == "persistent" ? RTX_MODE_PERSISTENT : RTX_MODE_WAVEFRONT);
      if (!devices.empty()) r.set_devices(devices);
      else if (gpus > 1) r.set_gpus(gpus);
      r.Render();
      std::clog << "Rays: " << r.stats().rays_total << " (" << r.stats().rays_total / (r.stats().kernel_ms * 1e3)
                << " Mrays/s device)\n";
    }
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
  std::clog << "Runtime: " << std::setprecision(2) << clock.elapsed() << "s" << std::flush;
  return 0;
}
