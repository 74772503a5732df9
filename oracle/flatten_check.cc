// flatten_check.cc — TEST INFRASTRUCTURE (tests/test_integration_reference.py): compiles the
// reference-side integration files (integration/rtx_flatten.h, gpu_ray_integrator.h) against
// a scratch copy of the reference's headers with integration/accessors.txt inserted, builds a
// .rtxs scene with the reference's own classes (ref_harness.cc's loader), flattens it with
// the integration Flatten and dumps the C-ABI arrays for comparison with the product's.
//   flatten_check <scene.rtxs> <model_dir> <out_prefix>
#define main ref_harness_main
#include "ref_harness.cc"
#undef main

#include "gpu_ray_integrator.h"
#include "rtx_flatten.h"

template <class T>
static void dump(const std::string& path, const std::vector<T>& v) {
  std::ofstream(path, std::ios::binary).write((const char*)v.data(), (std::streamsize)(v.size() * sizeof(T)));
}

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  auto S = load_scene(argv[1], argv[2]);
  rt::integrator::RtxScene f = rt::integrator::Flatten(S->world);
  const std::string out = argv[3];
  dump(out + ".prims", f.prims);
  dump(out + ".nodes", f.nodes);
  dump(out + ".mats", f.mats);
  dump(out + ".texs", f.texs);
  std::vector<int32_t> dims;
  std::vector<uint8_t> texels;
  for (size_t i = 0; i < f.imgs.size(); i++) {
    dims.push_back(f.imgs[i].width), dims.push_back(f.imgs[i].height);
    texels.insert(texels.end(), f.imgs[i].texels, f.imgs[i].texels + (size_t)f.imgs[i].width * f.imgs[i].height * 3);
  }
  dump(out + ".imgdims", dims);
  dump(out + ".texels", texels);
  // the seam class compiles against the reference's RayIntegrator (no device needed to link)
  std::printf("%zu prims %zu nodes %zu materials %zu textures %zu images; GpuRayIntegrator %zu bytes\n",
              f.prims.size(), f.nodes.size(), f.mats.size(), f.texs.size(), f.imgs.size(),
              sizeof(rt::integrator::GpuRayIntegrator));
  return 0;
}
