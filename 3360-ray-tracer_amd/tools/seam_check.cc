// seam_check — the reference's hybrid mode at its IntersectBatch seam, driven through the
// C++ host API (rt/integrator.h over include/rtx.h): a CPU loop hands batches of at most
// `batch` rays to GpuRayIntegrator::IntersectBatch exactly as WavefrontRenderer::Render does
// (wavefront.cc:89-103: queue chunks of batch_size, hits resized by the callee), and the
// HitRecords come back with HitRecord::mat re-attached.
//
//   seam_check <scene.rtxs> <rays.f64 (n x 6)> <out.f64 (n x 12)> [--batch 16384]
//              [--precision parity|fast] [--repeat R]
//
// out row: hit, t, p[3], normal[3], u, v, front_face, material (index of HitRecord::mat in
// the flattened material table; -1 on a miss).  stdout: one JSON line with the seam's
// throughput (host round trip per batch: H2D copy, kernel, D2H copy, HitRecord assembly).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <unordered_map>
#include <vector>

#include "rt/integrator.h"

using namespace rt;

int main(int argc, char** argv) {
  if (argc < 4) {
    std::cerr << "usage: seam_check <scene.rtxs> <rays.f64> <out.f64> [--batch N] [--precision parity|fast] "
                 "[--repeat R]\n";
    return 2;
  }
  size_t batch = 16384;
  int precision = RTX_PREC_PARITY, repeat = 1;
  for (int i = 4; i + 1 < argc; i += 2) {
    const std::string a = argv[i], v = argv[i + 1];
    if (a == "--batch") batch = std::strtoull(v.c_str(), nullptr, 10);
    else if (a == "--precision") precision = v == "fast" ? RTX_PREC_FAST : RTX_PREC_PARITY;
    else if (a == "--repeat") repeat = std::atoi(v.c_str());
    else {
      std::cerr << "unknown option " << a << "\n";
      return 2;
    }
  }
  try {
    auto world = scene::LoadSceneFile(argv[1], "");
    std::ifstream in(argv[2], std::ios::binary | std::ios::ate);
    if (!in) throw std::runtime_error(std::string("cannot read ") + argv[2]);
    const size_t n = (size_t)in.tellg() / (6 * sizeof(double));
    in.seekg(0);
    std::vector<double> raw(6 * n);
    in.read((char*)raw.data(), (std::streamsize)(raw.size() * sizeof(double)));
    std::vector<core::Ray> queue(n);
    for (size_t i = 0; i < n; i++)
      queue[i] = core::Ray(core::Point3(raw[6 * i], raw[6 * i + 1], raw[6 * i + 2]),
                           core::Vec3(raw[6 * i + 3], raw[6 * i + 4], raw[6 * i + 5]));

    integrator::GpuRayIntegrator integ(world.get(), 0, precision);
    std::unordered_map<const material::Material*, int> mat_index;
    for (size_t k = 0; k < integ.flat().material_ptrs.size(); k++) mat_index[integ.flat().material_ptrs[k].get()] = (int)k;

    std::vector<double> out(12 * n, 0.0);
    core::Timer clock;
    size_t batches = 0;
    for (int rep = 0; rep < repeat; rep++) {
      if (rep == 1) clock.reset(), batches = 0;  // the first pass warms the device up
      for (size_t off = 0; off < n;) {  // wavefront.cc:89-103
        const size_t cnt = std::min(batch, n - off);
        std::vector<core::Ray> br(queue.begin() + (std::ptrdiff_t)off, queue.begin() + (std::ptrdiff_t)(off + cnt));
        std::vector<geom::HitRecord> hits;
        integ.IntersectBatch(br, hits);
        batches++;
        if (rep == 0) {
          for (size_t i = 0; i < cnt; i++) {
            const geom::HitRecord& h = hits[i];
            double* o = &out[12 * (off + i)];
            if (!h.hit) {
              o[11] = -1;
              continue;
            }
            o[0] = 1, o[1] = h.t;
            for (int c = 0; c < 3; c++) o[2 + c] = h.p[c], o[5 + c] = h.normal[c];
            o[8] = h.u, o[9] = h.v, o[10] = h.front_face ? 1 : 0;
            o[11] = mat_index.at(h.mat.get());
          }
        }
        off += cnt;
      }
    }
    const double secs = clock.elapsed();
    std::ofstream(argv[3], std::ios::binary).write((const char*)out.data(), (std::streamsize)(out.size() * sizeof(double)));
    const double rays = repeat > 1 ? (double)n * (repeat - 1) : (double)n;
    std::printf("{\"rays\": %.0f, \"batches\": %zu, \"batch\": %zu, \"seconds\": %.6f, \"mrays_s\": %.3f, "
                "\"us_per_batch\": %.2f}\n",
                rays, batches, batch, secs, rays / secs / 1e6, secs / (double)batches * 1e6);
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
