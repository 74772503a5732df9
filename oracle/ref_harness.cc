// oracle/ref_harness.cc — TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Drives the reference's OWN compiled code (headers + material.cc + image.cc from
// /root/reference/src, compiled in place by oracle/Makefile into oracle/_ref/) to emit
// golden vectors into tests/golden/.  Nothing from the reference is copied into the repo.
//
// What is the reference's own code here:
//   * geometry:   geom::Sphere/Triangle/xy_rect/xz_rect/yz_rect::Hit, Aabb::Hit, Bvh (SAH build +
//                 flatten + traversal), scene::Scene::Hit                    (geom/*.h, scene/scene.h)
//   * integrator: integrator::CPURayIntegrator::IntersectBatch, RecordSample, IsConverged
//                                                                              (integrator/*.h)
//   * materials:  Lambertian/Metal/Dielectric/DiffuseLight Sample/Scatter/Emitted (material.cc)
//   * textures:   SolidColor/CheckerTexture/ImageTexture + scene::Image (stb)   (texture.h, image.cc)
//   * RNG:        core::SeedRng / RandomDouble / RandomVec3 (core/random.h, math_utils.h)
//   * output:     core::write_color                                         (core/color.h)
//
// What is restated here (the reference's versions need nlohmann/json, absent from this
// image, so camera.h / wavefront.cc are unbuildable without a stand-in, which we refuse):
//   * Camera::Initialize / GetRay                    (scene/camera.h:100-144,196-203)
//   * WavefrontRenderer::Render's loop glue           (renderer/wavefront.cc:40-242)
//   * Camera::GetPixel for megakernel mode           (scene/camera.h:148-174)
// The glue below keeps the reference's exact expression shapes where g++'s evaluation
// order decides the RNG draw order (SampleSquare: camera.h:202).
//
// Single-threaded (omp_set_num_threads(1)) + SeedRng(seed) makes the reference
// bit-reproducible (SURVEY.md §8c "Determinism").

#include "core/color.h"
#include "core/math_utils.h"
#include "core/random.h"
#include "geom/bvh.h"
#include "geom/rect.h"
#include "geom/sphere.h"
#include "geom/triangle.h"
#include "integrator/cpu_ray_integrator.h"
#include "integrator/pixel_state.h"
#include "integrator/ray_state.h"
#include "material/material.h"
#include "material/texture.h"
#include "scene/image.h"
#include "third-party/stb/stb_image.h"  // declarations only: stbi_load for the image8 command
#include "scene/scene.h"

#include <omp.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

using namespace rt;
using core::Color;
using core::Point3;
using core::Vec3;

namespace {

// ---------------------------------------------------------------------------------------
// Scene description log (the .rtxs text format, see include/rtx_scene_format.md)
// ---------------------------------------------------------------------------------------
struct SceneLog {
  std::ostringstream out;
  int ntex = 0, nmat = 0;
  void header(bool bvh) { out << "rtxscene 1\nbvh " << (bvh ? 1 : 0) << "\n"; }
  static std::string d(double x) {
    char b[64];
    std::snprintf(b, sizeof b, "%.17g", x);
    return b;
  }
  int solid(const Color& c) {
    out << "tex " << ntex << " solid " << d(c.x()) << ' ' << d(c.y()) << ' ' << d(c.z()) << "\n";
    return ntex++;
  }
  int checker(double scale, int even, int odd) {
    out << "tex " << ntex << " checker " << d(scale) << ' ' << even << ' ' << odd << "\n";
    return ntex++;
  }
  int image(const char* name) {
    out << "tex " << ntex << " image " << name << "\n";
    return ntex++;
  }
  int lambertian(int tex) {
    out << "mat " << nmat << " lambertian " << tex << "\n";
    return nmat++;
  }
  int metal(const Color& c, double fuzz) {
    out << "mat " << nmat << " metal " << d(c.x()) << ' ' << d(c.y()) << ' ' << d(c.z()) << ' '
        << d(fuzz) << "\n";
    return nmat++;
  }
  int dielectric(double ri) {
    out << "mat " << nmat << " dielectric " << d(ri) << "\n";
    return nmat++;
  }
  int light(int tex) {
    out << "mat " << nmat << " light " << tex << "\n";
    return nmat++;
  }
  void sphere(const Point3& c, double r, int m) {
    out << "sphere " << d(c.x()) << ' ' << d(c.y()) << ' ' << d(c.z()) << ' ' << d(r) << ' ' << m
        << "\n";
  }
  void rect(const char* ax, double a0, double a1, double b0, double b1, double k, int m) {
    out << "rect " << ax << ' ' << d(a0) << ' ' << d(a1) << ' ' << d(b0) << ' ' << d(b1) << ' '
        << d(k) << ' ' << m << "\n";
  }
  void obj(const char* name, double scale, int m) {
    out << "obj " << name << ' ' << d(scale) << ' ' << m << "\n";
  }
};

// Scene recipes.  They only LOG descriptions; the reference objects are built from the
// logged file by load_scene() below, so generator and loader are exercised separately.
// Random draws go through the reference's RandomDouble/RandomVec3 with the reference's
// expression shapes so g++ picks the same argument evaluation order as main.cc:99-125.
std::string recipe(const std::string& name) {
  SceneLog L;
  if (name == "three") {  // BASELINE configs[0] / SURVEY §8d C1 (no BVH)
    L.header(false);
    int g = L.lambertian(L.solid(Color(0.8, 0.8, 0.0)));
    int c = L.lambertian(L.solid(Color(0.1, 0.2, 0.5)));
    int r = L.lambertian(L.solid(Color(0.7, 0.3, 0.3)));
    L.sphere(Point3(0.0, -100.5, -1.0), 100.0, g);
    L.sphere(Point3(0.0, 0.0, -1.2), 0.5, c);
    L.sphere(Point3(1.0, 0.0, -1.0), 0.5, r);
  } else if (name == "cornell") {  // main.cc:23-61
    L.header(true);
    int red = L.lambertian(L.solid(Color(.65, .05, .05)));
    int white = L.lambertian(L.solid(Color(.73, .73, .73)));
    int green = L.lambertian(L.solid(Color(.12, .45, .15)));
    int light = L.light(L.solid(Color(15, 15, 15)));
    const double S = 10.0, eps = 0.01;
    L.rect("yz", 0, S, 0, S, S, green);
    L.rect("yz", 0, S, 0, S, 0, red);
    L.rect("xz", 0, S, 0, S, 0, white);
    L.rect("xz", 0, S, 0, S, S, white);
    L.rect("xy", 0, S, 0, S, S, white);
    L.rect("xz", 3.0, 7.0, 3.0, 7.0, S - eps, light);
    int glass = L.dielectric(1.5);
    int metal = L.metal(Color(0.85, 0.85, 0.95), 0.03);
    int diffuse = L.lambertian(L.solid(Color(0.8, 0.3, 0.1)));
    L.sphere(Point3(3.2, 1.0, 7.0), 1.0, diffuse);
    L.sphere(Point3(7.0, 1.0, 4.0), 1.0, metal);
    L.sphere(Point3(5.0, 1.0, 2.5), 1.0, glass);
  } else if (name == "final") {  // RTIOW final scene, SeedRng(1234)
    L.header(true);
    core::SeedRng(1234);
    int ground = L.lambertian(L.solid(Color(0.5, 0.5, 0.5)));
    L.sphere(Point3(0, -1000, 0), 1000, ground);
    for (int a = -11; a < 11; a++) {
      for (int b = -11; b < 11; b++) {
        auto choose_mat = core::RandomDouble();
        Point3 center(a + 0.9 * core::RandomDouble(), 0.2, b + 0.9 * core::RandomDouble());
        if ((center - Point3(4, 0.2, 0)).length() > 0.9) {
          if (choose_mat < 0.8) {
            auto albedo = core::RandomVec3() * core::RandomVec3();
            L.sphere(center, 0.2, L.lambertian(L.solid(albedo)));
          } else if (choose_mat < 0.95) {
            auto albedo = core::RandomVec3(0.5, 1);
            auto fuzz = core::RandomDouble(0, 0.5);
            L.sphere(center, 0.2, L.metal(albedo, fuzz));
          } else {
            L.sphere(center, 0.2, L.dielectric(1.5));
          }
        }
      }
    }
    L.sphere(Point3(0, 1, 0), 1.0, L.dielectric(1.5));
    L.sphere(Point3(-4, 1, 0), 1.0, L.lambertian(L.solid(Color(0.4, 0.2, 0.1))));
    L.sphere(Point3(4, 1, 0), 1.0, L.metal(Color(0.7, 0.6, 0.5), 0.0));
  } else if (name == "bunny") {  // SURVEY §8d C3 (main.cc:135-137 recipe, load_obj.h semantics)
    L.header(true);
    int red = L.lambertian(L.solid(Color(0.8, 0.1, 0.1)));
    L.obj("stanford-bunny.obj", 50.0, red);
    int ground = L.lambertian(L.solid(Color(0.5, 0.5, 0.5)));
    L.sphere(Point3(0, -1003.9, 0), 1000, ground);
  } else if (name == "mixed") {  // main.cc:72-145 Spheres(), SeedRng(1234) — SURVEY §8d C5
    L.header(true);
    core::SeedRng(1234);
    int earth_surface = L.lambertian(L.image("earthmap"));
    int m_ground = L.lambertian(L.solid(Color(0.8, 0.8, 0.0)));
    int m_center = L.lambertian(L.solid(Color(0.1, 0.2, 0.5)));
    int m_left = L.dielectric(1.50);
    int m_bubble = L.dielectric(1.00 / 1.50);
    int m_right = L.metal(Color(0.8, 0.6, 0.2), 1.0);
    L.sphere(Point3(0.0, -100.5, -1.0), 100.0, m_ground);
    L.sphere(Point3(0.0, 0.0, -1.2), 0.5, m_center);
    L.sphere(Point3(-1.0, 0.0, -1.0), 0.5, m_left);
    L.sphere(Point3(-1.0, 0.0, -1.0), 0.4, m_bubble);
    L.sphere(Point3(1.0, 0.0, -1.0), 0.5, m_right);
    int ce = L.solid(Color(0.2, 0.3, 0.1));
    int co = L.solid(Color(.9, .9, .9));
    int checker = L.checker(0.32, ce, co);
    L.sphere(Point3(0, -1000, 0), 1000, L.lambertian(checker));
    for (int a = -110; a < 110; a++) {
      for (int b = -110; b < 110; b++) {
        auto choose_mat = core::RandomDouble();
        Point3 center(a + 0.9 * core::RandomDouble(), 0.2, b + 0.9 * core::RandomDouble());
        if ((center - Point3(4, 0.2, 0)).length() > 0.9) {
          if (choose_mat < 0.2) {
            L.sphere(center, 0.2, earth_surface);
          } else if (choose_mat < 0.8) {
            auto albedo = core::RandomVec3(0, 1);
            L.sphere(center, 0.2, L.lambertian(L.solid(albedo)));
          } else if (choose_mat < 0.95) {
            auto albedo = core::RandomVec3(0.5, 1);
            auto fuzz = core::RandomDouble(0, 0.5);
            L.sphere(center, 0.2, L.metal(albedo, fuzz));
          } else {
            L.sphere(center, 0.2, L.dielectric(1.5));
          }
        }
      }
    }
    L.sphere(Point3(0, 1, 0), 1.0, L.dielectric(1.5));
    L.sphere(Point3(-4, 0, 0), 1.0, L.lambertian(L.solid(Color(0.4, 0.2, 0.1))));
    L.sphere(Point3(4, 1, 0), 1.0, L.metal(Color(0.7, 0.6, 0.5), 0.0));
  } else if (name == "one_sphere") {
    L.header(false);
    L.sphere(Point3(0.25, -0.5, -3.0), 1.25, L.lambertian(L.solid(Color(.5, .5, .5))));
  } else if (name == "one_triangle") {
    L.header(false);
    int m = L.lambertian(L.solid(Color(.5, .5, .5)));
    L.out << "tri -1.5 -1 -3 1.25 -1.25 -3.5 0.1 1.5 -2.5 " << m << "\n";
  } else if (name == "rects") {
    L.header(false);
    int m = L.lambertian(L.solid(Color(.5, .5, .5)));
    L.rect("xy", -1, 1, -1, 1, -3, m);
    L.rect("xz", -1, 1.5, -4, -2, -1.2, m);
    L.rect("yz", -0.5, 1, -4, -2, 1.1, m);
  } else {
    std::fprintf(stderr, "unknown recipe %s\n", name.c_str());
    std::exit(2);
  }
  return L.out.str();
}

// ---------------------------------------------------------------------------------------
// Loading a .rtxs file into the reference's own object model
// ---------------------------------------------------------------------------------------
struct RefScene {
  scene::Scene world;      // root handed to the integrator (objects_ or one Bvh)
  scene::Scene flat;       // primitives in file order
  std::shared_ptr<geom::Bvh> bvh;
  std::vector<std::shared_ptr<material::Texture>> tex;
  std::vector<std::shared_ptr<material::Material>> mat;
  std::map<const material::Material*, int> mat_id;
};

// OBJ semantics restated from load_obj.h:10-55 (tinyobjloader parses coordinates as
// float, real_t = float by default; faces with !=3 vertices are skipped; vertices are
// centred on their centroid then scaled).  Parity for this step is "unpinned" against
// tinyobjloader itself, which is absent.
void load_obj(const std::string& path, double scale, std::vector<Point3>& v,
              std::vector<std::array<int, 3>>& f) {
  std::ifstream in(path);
  if (!in) {
    std::fprintf(stderr, "cannot open %s\n", path.c_str());
    std::exit(2);
  }
  std::string line;
  while (std::getline(in, line)) {
    if (line.size() > 2 && line[0] == 'v' && line[1] == ' ') {
      const char* p = line.c_str() + 2;
      char* e;
      float x = std::strtof(p, &e);
      float y = std::strtof(e, &e);
      float z = std::strtof(e, &e);
      v.emplace_back(x, y, z);
    } else if (line.size() > 2 && line[0] == 'f' && line[1] == ' ') {
      std::istringstream ss(line.substr(2));
      std::vector<int> idx;
      std::string tok;
      while (ss >> tok) idx.push_back(std::atoi(tok.c_str()) - 1);
      if (idx.size() == 3) f.push_back({idx[0], idx[1], idx[2]});
    }
  }
  Vec3 centroid(0.0f, 0.0f, 0.0f);
  for (auto& p : v) centroid += p;
  centroid /= v.size();
  for (auto& p : v) {
    p = p - centroid;
    p = p * scale;
  }
}

std::unique_ptr<RefScene> load_scene(const std::string& file, const std::string& model_dir) {
  auto S = std::make_unique<RefScene>();
  std::ifstream in(file);
  if (!in) {
    std::fprintf(stderr, "cannot open %s\n", file.c_str());
    std::exit(2);
  }
  std::string line;
  bool use_bvh = false;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string kw;
    ss >> kw;
    if (kw == "bvh") {
      int b;
      ss >> b;
      use_bvh = b != 0;
    } else if (kw == "tex") {
      int id;
      std::string kind;
      ss >> id >> kind;
      if (kind == "solid") {
        double r, g, b;
        ss >> r >> g >> b;
        S->tex.push_back(std::make_shared<material::SolidColor>(Color(r, g, b)));
      } else if (kind == "checker") {
        double sc;
        int e, o;
        ss >> sc >> e >> o;
        S->tex.push_back(std::make_shared<material::CheckerTexture>(sc, S->tex[e], S->tex[o]));
      } else {  // image: the reference decodes the original JPEG with stb (image.cc:16-41)
        std::string name;
        ss >> name;
        S->tex.push_back(std::make_shared<material::ImageTexture>((name + ".jpg").c_str()));
      }
    } else if (kw == "mat") {
      int id;
      std::string kind;
      ss >> id >> kind;
      std::shared_ptr<material::Material> m;
      if (kind == "lambertian") {
        int t;
        ss >> t;
        m = std::make_shared<material::Lambertian>(S->tex[t]);
      } else if (kind == "metal") {
        double r, g, b, fz;
        ss >> r >> g >> b >> fz;
        m = std::make_shared<material::Metal>(Color(r, g, b), fz);
      } else if (kind == "dielectric") {
        double ri;
        ss >> ri;
        m = std::make_shared<material::Dielectric>(ri);
      } else {
        int t;
        ss >> t;
        m = std::make_shared<material::DiffuseLight>(S->tex[t]);
      }
      S->mat_id[m.get()] = (int)S->mat.size();
      S->mat.push_back(m);
    } else if (kw == "sphere") {
      double x, y, z, r;
      int m;
      ss >> x >> y >> z >> r >> m;
      S->flat.Add(std::make_shared<geom::Sphere>(Point3(x, y, z), r, S->mat[m]));
    } else if (kw == "tri") {
      double a[9];
      int m;
      for (double& q : a) ss >> q;
      ss >> m;
      S->flat.Add(std::make_shared<geom::Triangle>(Point3(a[0], a[1], a[2]), Point3(a[3], a[4], a[5]),
                                                   Point3(a[6], a[7], a[8]), S->mat[m]));
    } else if (kw == "rect") {
      std::string ax;
      double a0, a1, b0, b1, k;
      int m;
      ss >> ax >> a0 >> a1 >> b0 >> b1 >> k >> m;
      if (ax == "xy")
        S->flat.Add(std::make_shared<geom::xy_rect>(a0, a1, b0, b1, k, S->mat[m]));
      else if (ax == "xz")
        S->flat.Add(std::make_shared<geom::xz_rect>(a0, a1, b0, b1, k, S->mat[m]));
      else
        S->flat.Add(std::make_shared<geom::yz_rect>(a0, a1, b0, b1, k, S->mat[m]));
    } else if (kw == "obj") {
      std::string name;
      double sc;
      int m;
      ss >> name >> sc >> m;
      std::vector<Point3> v;
      std::vector<std::array<int, 3>> f;
      load_obj(model_dir + "/" + name, sc, v, f);
      for (auto& t : f)
        S->flat.Add(std::make_shared<geom::Triangle>(v[t[0]], v[t[1]], v[t[2]], S->mat[m]));
    }
  }
  if (use_bvh) {
    S->bvh = std::make_shared<geom::Bvh>(S->flat);
    S->world.Add(S->bvh);
  } else {
    for (auto& o : S->flat.objects_) S->world.Add(o);
  }
  return S;
}

// ---------------------------------------------------------------------------------------
// Camera (restated: scene/camera.h:100-144,196-203 — camera.h itself needs nlohmann/json)
// ---------------------------------------------------------------------------------------
struct Cam {
  double aspect_ratio, vfov, defocus_angle, focus_dist;
  int image_width, image_height;
  Vec3 lookfrom, lookat, vup;
  Point3 center, pixel00, du, dv;
  Vec3 u, v, w, disk_u, disk_v;

  void Initialize() {
    image_height = int(image_width / aspect_ratio);
    image_height = (image_height < 1) ? 1 : image_height;
    center = lookfrom;
    double theta = core::DegreesToRadians(vfov);
    auto h = std::tan(theta / 2);
    auto viewport_height = 2 * h * focus_dist;
    auto viewport_width = viewport_height * (double(image_width) / image_height);
    w = core::Normalize(lookfrom - lookat);
    u = core::Normalize(core::Cross(vup, w));
    v = core::Cross(w, u);
    Vec3 viewport_u = viewport_width * u;
    Vec3 viewport_v = viewport_height * -v;
    du = viewport_u / image_width;
    dv = viewport_v / image_height;
    auto upper_left = center - (focus_dist * w) - viewport_u / 2 - viewport_v / 2;
    pixel00 = upper_left + 0.5 * (du + dv);
    auto defocus_radius = focus_dist * std::tan(core::DegreesToRadians(defocus_angle / 2));
    disk_u = u * defocus_radius;
    disk_v = v * defocus_radius;
  }
  // Same expression shape as camera.h:202 so g++ evaluates the two draws in the same order.
  Vec3 SampleSquare() const {
    return Vec3(core::RandomDouble() - 0.5, core::RandomDouble() - 0.5, 0);
  }
  Point3 DiskSample() const {
    auto p = core::RandomInUnitDisk();
    return center + (p[0] * disk_u) + (p[1] * disk_v);
  }
  core::Ray GetRay(int i, int j) const {
    auto offset = SampleSquare();
    auto pixel_sample = pixel00 + ((i + offset.x()) * du) + ((j + offset.y()) * dv);
    auto origin = (defocus_angle <= 0) ? center : DiskSample();
    return core::Ray(origin, pixel_sample - origin);
  }
};

Color sky(const core::Ray& r) {  // wavefront.cc:33-38 / camera.h:171-173
  Vec3 unit = core::Normalize(r.direction());
  auto t = 0.5 * (unit.y() + 1.0);
  return (1.0 - t) * Color(1.0, 1.0, 1.0) + t * Color(0.5, 0.7, 1.0);
}

template <class T>
void write_bin(const std::string& path, const std::vector<T>& v) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::perror(path.c_str());
    std::exit(2);
  }
  std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
}
template <class T>
std::vector<T> read_bin(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) {
    std::perror(path.c_str());
    std::exit(2);
  }
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<T> v(n / sizeof(T));
  if (std::fread(v.data(), sizeof(T), v.size(), f) != v.size()) std::exit(3);
  std::fclose(f);
  return v;
}

// Wavefront render glue (wavefront.cc:40-242) around the reference's own integrator,
// materials, PixelState and write_color.  Tile = full image.  Writes:
//   <out>.ppm      the P3 text PPM exactly as Render() would print it
//   <out>.f64      linear framebuffer sum/(float)samples, doubles, row-major RGB
//   <out>.spp      samples per pixel (int32);  <out>.var  per-pixel sample variance m2/(n-1), RGB
//   <out>.stats    rays (segments submitted to IntersectBatch), primaries, samples per pixel
void render_wavefront(RefScene& S, Cam& cam, int max_depth, int max_spp, int batch, bool adaptive,
                      const std::string& out) {
  integrator::CPURayIntegrator integ(&S.world);
  // REF_PAR_SHADE=1 (timing only: scripts/calibrate_cpu.py): the shading loop runs in parallel as
  // the reference runs it; otherwise serially, the draw order fixed by SeedRng (the goldens)
  const char* pe = std::getenv("REF_PAR_SHADE");
  const bool par_shade = pe && std::atoi(pe) != 0;
  const float kRelThresh = 0.05;
  const int kMinSamples = adaptive ? 16 : (1 << 30);
  const int W = cam.image_width, H = cam.image_height, N = W * H;
  std::vector<integrator::PixelState> px(N);
  std::vector<integrator::RayState> q, nq;
  long long rays = 0, primaries = 0;
  auto finish = [&](integrator::PixelState& ps, const Color& L) {
    integrator::RecordSample(ps, L);
    if (!ps.converged && integrator::IsConverged(ps, kRelThresh, kMinSamples)) ps.converged = true;
  };
  const auto t_start = std::chrono::steady_clock::now();
  for (int s = 0; s < max_spp; ++s) {
    q.clear();
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x) {
        int idx = y * W + x;
        if (px[idx].converged) continue;
        integrator::RayState rs;
        rs.r = cam.GetRay(x, y);
        rs.pixel_index = idx;
        rs.depth = 0;
        rs.throughput = Color(1, 1, 1);
        q.push_back(rs);
      }
    primaries += (long long)q.size();
    while (!q.empty()) {
      for (size_t off = 0; off < q.size();) {
        size_t cnt = std::min((size_t)batch, q.size() - off);
        std::vector<core::Ray> br(cnt);
        for (size_t i = 0; i < cnt; ++i) br[i] = q[off + i].r;
        std::vector<geom::HitRecord> hits;
        integ.IntersectBatch(br, hits);
        rays += (long long)cnt;
        // one ray's shading (wavefront.cc:109-208); `push` takes a continuing child
        auto shade = [&](size_t i, std::vector<integrator::RayState>& push) {
          auto rs = q[off + i];
          auto& ps = px[rs.pixel_index];
          const auto& rec = hits[i];
          const auto& r = br[i];
          Color L(0, 0, 0);
          if (!rec.hit || rs.depth >= max_depth) {
            L += rs.throughput * sky(r);
            finish(ps, L);
            return;
          }
          Color em = rec.mat->Emitted(rec.u, rec.v, rec.p);
          if (!em.NearZero()) {
            L += rs.throughput * em;
            finish(ps, L);
            return;
          }
          Vec3 wo = -core::Normalize(r.direction());
          Vec3 wi;
          float pdf = 0.0f;
          Color f;
          if (!rec.mat->Sample(rec, wo, wi, pdf, f)) {
            finish(ps, L);
            return;
          }
          if (ps.converged) return;
          integrator::RayState child;
          child.r = core::Ray(rec.p, wi);
          child.pixel_index = rs.pixel_index;
          child.depth = rs.depth + 1;
          if (rec.mat->IsSpecular()) {
            child.throughput = rs.throughput * f;
          } else {
            if (pdf < 1e-6f) {
              finish(ps, L);
              return;
            }
            float cos_theta = std::max(0.0f, static_cast<float>(core::Dot(wi, rec.normal)));
            child.throughput = rs.throughput * f * cos_theta / pdf;
          }
          if (child.depth > 5) {
            double p = std::max({child.throughput.x(), child.throughput.y(), child.throughput.z()});
            p = std::clamp(p, 0.1, 0.95);
            if (core::RandomDouble() > p) {
              finish(ps, L);
              return;
            }
            child.throughput /= p;
          }
          push.push_back(child);
        };
        if (par_shade) {
          // the reference's own schedule (wavefront.cc:105-217): the shading loop under
          // `omp parallel for schedule(dynamic)`, children in thread-local queues merged in
          // thread order (a pixel has at most one ray in flight per pass, so its PixelState is
          // touched by one thread at a time); each thread draws from its own thread_local
          // generator (core/random.h), so the draw order, and the image, are not reproducible
          const int nt = omp_get_max_threads();
          std::vector<std::vector<integrator::RayState>> local(nt);
#pragma omp parallel for schedule(dynamic)
          for (int i = 0; i < (int)cnt; i++) shade((size_t)i, local[omp_get_thread_num()]);
          for (int t = 0; t < nt; t++) nq.insert(nq.end(), local[t].begin(), local[t].end());
        } else {
          for (size_t i = 0; i < cnt; ++i) shade(i, nq);
        }
        off += cnt;
      }
      q.swap(nq);
      nq.clear();
    }
  }
  const auto t_loop = std::chrono::steady_clock::now();
  std::vector<double> fb(3 * (size_t)N), var(3 * (size_t)N);
  std::vector<int> spp(N);
  std::ofstream ppm(out + ".ppm");
  ppm << "P3\n" << W << ' ' << H << "\n255\n";
  for (int i = 0; i < N; i++) {
    Color c = px[i].samples > 0 ? px[i].sum / (float)px[i].samples : Color(0, 0, 0);
    fb[3 * i] = c.x();
    fb[3 * i + 1] = c.y();
    fb[3 * i + 2] = c.z();
    spp[i] = px[i].samples;
    const Color v = integrator::Variance(px[i]);  // pixel_state.h:41-49, for the statistical parity test
    var[3 * i] = v.x();
    var[3 * i + 1] = v.y();
    var[3 * i + 2] = v.z();
    core::write_color(ppm, c);
  }
  write_bin(out + ".f64", fb);
  write_bin(out + ".var", var);
  write_bin(out + ".spp", spp);
  ppm.close();
  const auto t_end = std::chrono::steady_clock::now();
  std::ofstream st(out + ".stats");
  st << "rays " << rays << "\nprimaries " << primaries << "\n";
  // wall seconds of the pass loop (generation .. shading) and of the whole Render()
  // including the P3 write (the reference's `Runtime:` covers the latter, main.cc:196)
  st << "loop_seconds " << std::chrono::duration<double>(t_loop - t_start).count() << "\n";
  st << "render_seconds " << std::chrono::duration<double>(t_end - t_start).count() << "\n";
  st << "threads " << omp_get_max_threads() << "\n";
  st << "parallel_shading " << (par_shade ? 1 : 0) << "\n";
}

// Megakernel mode (mega_kernel.h:15-54 + DefaultSampler sampler.h:22-34 + GetPixel
// camera.h:148-174), single-threaded, pixel order row-major.  Writes <out>.f64 / .ppm.
Color get_pixel(const core::Ray& r, int depth, const geom::Hittable& world) {
  if (depth <= 0) return Color(0, 0, 0);
  geom::HitRecord rec;
  if (world.Hit(r, core::Interval(0.001, core::kInfinity), rec)) {
    core::Ray scattered;
    Color attenuation;
    Color emitted = rec.mat->Emitted(rec.u, rec.v, rec.p);
    if (rec.mat->Scatter(r, rec, attenuation, scattered))
      return emitted + attenuation * get_pixel(scattered, depth - 1, world);
    return emitted;
  }
  return sky(r);
}

void render_megakernel(RefScene& S, Cam& cam, int max_depth, int spp, const std::string& out) {
  const int W = cam.image_width, H = cam.image_height;
  std::vector<double> fb(3 * (size_t)W * H);
  std::ofstream ppm(out + ".ppm");
  ppm << "P3\n" << W << ' ' << H << "\n255\n";
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      Color pixel(0, 0, 0);
      for (int k = 0; k < spp; k++) {
        core::Ray r = cam.GetRay(x, y);
        pixel += get_pixel(r, max_depth, S.world);
      }
      pixel /= spp;
      size_t i = (size_t)y * W + x;
      fb[3 * i] = pixel.x();
      fb[3 * i + 1] = pixel.y();
      fb[3 * i + 2] = pixel.z();
      core::write_color(ppm, pixel);
    }
  write_bin(out + ".f64", fb);
}

// MegaKernel with AdaptiveSampler::SamplePixel (sampler.h:44-82), single-threaded,
// row-major.  sampler.h needs scene/camera.h (nlohmann/json, absent), so its loop is
// restated here over the reference's own GetRay / Hit / Scatter / Color / luminance.
void render_megakernel_adaptive(RefScene& S, Cam& cam, int max_depth, int min_samples, int max_samples,
                                float threshold, const std::string& out) {
  const int W = cam.image_width, H = cam.image_height;
  std::vector<double> fb(3 * (size_t)W * H);
  std::vector<int32_t> spp((size_t)W * H);
  std::ofstream ppm(out + ".ppm");
  ppm << "P3\n" << W << ' ' << H << "\n255\n";
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      Color pixel(0, 0, 0);
      Color sum = Color(0, 0, 0);
      Color sum_sq = Color(0, 0, 0);
      int samples = 0;
      while (samples <= max_samples) {
        samples++;
        core::Ray r = cam.GetRay(x, y);
        pixel += get_pixel(r, max_depth, S.world);
        sum += pixel;
        sum_sq += pixel * pixel;
        if (samples >= min_samples) {
          Color mean = sum / samples;
          double mean_luminance = core::luminance(mean);
          Color variance = (sum_sq / samples) - (mean * mean);
          double error = sqrt(core::luminance(variance) / samples);
          if ((error / (mean_luminance + 1e-3f)) < threshold) break;
        }
      }
      pixel /= samples;
      size_t i = (size_t)y * W + x;
      fb[3 * i] = pixel.x();
      fb[3 * i + 1] = pixel.y();
      fb[3 * i + 2] = pixel.z();
      spp[i] = samples;
      core::write_color(ppm, pixel);
    }
  write_bin(out + ".f64", fb);
  write_bin(out + ".spp", spp);
}

void usage() {
  std::fprintf(stderr,
               "ref_harness recipe <name> <out.rtxs>\n"
               "ref_harness rng <seed> <n>\n"
               "ref_harness bvh <scene.rtxs> <model_dir> <out_prefix>\n"
               "ref_harness hits <scene.rtxs> <model_dir> <rays.f64> <tmin> <out.f64>\n"
               "ref_harness aabb <boxes_rays.f64> <out.i32>\n"
               "ref_harness material <cases.f64> <out.f64>\n"
               "ref_harness scatter <cases.f64> <out.f64>\n"
               "ref_harness texture <cases.f64> <out.f64>\n"
               "ref_harness texels <out.ppm>\n"
               "ref_harness pixelstate <samples.f64> <out.f64>\n"
               "ref_harness render <scene.rtxs> <model_dir> <cam 14 numbers> <maxdepth> <spp> <adaptive> "
               "<seed> <out_prefix>\n"
               "ref_harness megakernel <scene.rtxs> <model_dir> <cam 14 numbers> <maxdepth> <spp> <seed> "
               "<out_prefix>\n"
               "ref_harness megakernel_adaptive <scene.rtxs> <model_dir> <cam 14 numbers> <maxdepth> <min> <max> "
               "<threshold> <seed> <out_prefix>\n");
  std::exit(2);
}

Cam parse_cam(char** a) {
  // aspect width vfov lookfrom(3) lookat(3) vup(3) defocus focus
  Cam c{};
  c.aspect_ratio = std::atof(a[0]);
  c.image_width = std::atoi(a[1]);
  c.vfov = std::atof(a[2]);
  c.lookfrom = Vec3(std::atof(a[3]), std::atof(a[4]), std::atof(a[5]));
  c.lookat = Vec3(std::atof(a[6]), std::atof(a[7]), std::atof(a[8]));
  c.vup = Vec3(std::atof(a[9]), std::atof(a[10]), std::atof(a[11]));
  c.defocus_angle = std::atof(a[12]);
  c.focus_dist = std::atof(a[13]);
  c.Initialize();
  return c;
}

}  // namespace

int main(int argc, char** argv) {
  // Single-threaded by default (bit-reproducible under SeedRng).  REF_THREADS=n runs the
  // reference's OpenMP IntersectBatch on n threads (the CPU-rate calibration): its shading
  // loop stays on the main thread, so the result is the same.
  const char* nt = std::getenv("REF_THREADS");
  omp_set_num_threads(nt ? std::max(1, std::atoi(nt)) : 1);
  if (argc < 2) usage();
  std::string cmd = argv[1];
  if (cmd == "recipe" && argc == 4) {
    std::ofstream(argv[3]) << recipe(argv[2]);
  } else if (cmd == "rng" && argc == 4) {
    core::SeedRng((unsigned)std::strtoul(argv[2], nullptr, 10));
    int n = std::atoi(argv[3]);
    for (int i = 0; i < n; i++) std::printf("%a\n", core::RandomDouble());
  } else if (cmd == "bvh" && argc == 5) {
    auto S = load_scene(argv[2], argv[3]);
    std::string out = argv[4];
    std::vector<double> boxes;
    std::vector<uint32_t> links;
    for (const auto& n : S->bvh->nodes()) {
      boxes.insert(boxes.end(), {n.bbox.x.min_, n.bbox.x.max_, n.bbox.y.min_, n.bbox.y.max_,
                                 n.bbox.z.min_, n.bbox.z.max_});
      links.insert(links.end(), {n.left_pIdx, n.right_pCnt, n.isLeaf});
    }
    write_bin(out + ".boxes.f64", boxes);
    write_bin(out + ".links.u32", links);
    std::vector<int32_t> pi(S->bvh->prim_indices().begin(), S->bvh->prim_indices().end());
    write_bin(out + ".prims.i32", pi);
  } else if (cmd == "hits" && argc == 7) {
    auto S = load_scene(argv[2], argv[3]);
    auto rays = read_bin<double>(argv[4]);
    double tmin = std::atof(argv[5]);
    size_t n = rays.size() / 6;
    // 12 doubles per ray: hit t p[3] n[3] u v front_face mat
    std::vector<double> out(12 * n, 0.0);
    for (size_t i = 0; i < n; i++) {
      core::Ray r(Point3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                  Vec3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
      geom::HitRecord rec{};
      bool ok;
      if (tmin < 0) {  // IntersectBatch seam: fixed [0.001f, inf) (cpu_ray_integrator.h:21-29)
        std::vector<core::Ray> one{r};
        std::vector<geom::HitRecord> h;
        integrator::CPURayIntegrator integ(&S->world);
        integ.IntersectBatch(one, h);
        rec = h[0];
        ok = rec.hit;
      } else {
        ok = S->world.Hit(r, core::Interval(tmin, core::kInfinity), rec);
      }
      double* o = &out[12 * i];
      o[0] = ok;
      if (ok) {
        o[1] = rec.t;
        o[2] = rec.p.x(), o[3] = rec.p.y(), o[4] = rec.p.z();
        o[5] = rec.normal.x(), o[6] = rec.normal.y(), o[7] = rec.normal.z();
        o[8] = rec.u, o[9] = rec.v;
        o[10] = rec.front_face;
        o[11] = S->mat_id[rec.mat.get()];
      }
    }
    write_bin(argv[6], out);
  } else if (cmd == "aabb" && argc == 4) {
    // per case: box(6: xmin xmax ymin ymax zmin zmax) ray(6) tmin tmax = 14 doubles
    auto c = read_bin<double>(argv[2]);
    size_t n = c.size() / 14;
    std::vector<int32_t> out(n);
    for (size_t i = 0; i < n; i++) {
      const double* q = &c[14 * i];
      geom::Aabb b(core::Interval(q[0], q[1]), core::Interval(q[2], q[3]), core::Interval(q[4], q[5]));
      core::Ray r(Point3(q[6], q[7], q[8]), Vec3(q[9], q[10], q[11]));
      out[i] = b.Hit(r, core::Interval(q[12], q[13]));
    }
    write_bin(argv[3], out);
  } else if (cmd == "material" || cmd == "scatter") {
    if (argc != 4) usage();
    // case (20 doubles): kind p0 p1 p2 p3 | normal(3) front u v p(3) | wo/r_in dir(3) | seed
    // kind: 0 lambertian(solid p0..p2) 1 metal(p0..p2, fuzz p3) 2 dielectric(ri p0) 3 light(p0..p2)
    // out (12): ok wi/dir(3) pdf f/att(3) next_draw spec org(2 spare)
    auto c = read_bin<double>(argv[2]);
    size_t n = c.size() / 20;
    std::vector<double> out(12 * n, 0.0);
    for (size_t i = 0; i < n; i++) {
      const double* q = &c[20 * i];
      std::shared_ptr<material::Material> m;
      int kind = (int)q[0];
      if (kind == 0) m = std::make_shared<material::Lambertian>(Color(q[1], q[2], q[3]));
      if (kind == 1) m = std::make_shared<material::Metal>(Color(q[1], q[2], q[3]), q[4]);
      if (kind == 2) m = std::make_shared<material::Dielectric>(q[1]);
      if (kind == 3) m = std::make_shared<material::DiffuseLight>(Color(q[1], q[2], q[3]));
      geom::HitRecord rec{};
      rec.normal = Vec3(q[5], q[6], q[7]);
      rec.front_face = q[8] != 0;
      rec.u = q[9];
      rec.v = q[10];
      rec.p = Point3(q[11], q[12], q[13]);
      rec.mat = m;
      rec.hit = true;
      Vec3 wo(q[14], q[15], q[16]);
      core::SeedRng((unsigned)q[17]);
      double* o = &out[12 * i];
      if (cmd == "material") {
        Vec3 wi(0, 0, 0);
        float pdf = -1.0f;
        Color f(0, 0, 0);
        bool ok = m->Sample(rec, wo, wi, pdf, f);
        o[0] = ok;
        o[1] = wi.x(), o[2] = wi.y(), o[3] = wi.z();
        o[4] = pdf;
        o[5] = f.x(), o[6] = f.y(), o[7] = f.z();
        o[9] = m->IsSpecular();
        Color em = m->Emitted(rec.u, rec.v, rec.p);
        o[10] = em.x();
      } else {
        core::Ray rin(rec.p, wo);
        Color att(0, 0, 0);
        core::Ray sc;
        bool ok = m->Scatter(rin, rec, att, sc);
        o[0] = ok;
        o[1] = sc.direction().x(), o[2] = sc.direction().y(), o[3] = sc.direction().z();
        o[5] = att.x(), o[6] = att.y(), o[7] = att.z();
        o[10] = sc.origin().x();
        o[11] = sc.origin().y();
      }
      o[8] = core::RandomDouble();  // pins how many draws the call consumed
    }
    write_bin(argv[3], out);
  } else if (cmd == "texture" && argc == 4) {
    // case (8): kind(0 checker 1 image) scale u v p(3) spare ; out (3)
    auto c = read_bin<double>(argv[2]);
    size_t n = c.size() / 8;
    auto checker = std::make_shared<material::CheckerTexture>(0.32, Color(0.2, 0.3, 0.1), Color(.9, .9, .9));
    auto image = std::make_shared<material::ImageTexture>("earthmap.jpg");
    auto missing = std::make_shared<material::ImageTexture>("no_such_texture.jpg");
    std::vector<double> out(3 * n);
    for (size_t i = 0; i < n; i++) {
      const double* q = &c[8 * i];
      Color v;
      Point3 p(q[4], q[5], q[6]);
      if (q[0] == 0) v = material::CheckerTexture(q[1], Color(0.2, 0.3, 0.1), Color(.9, .9, .9)).Value(q[2], q[3], p);
      else if (q[0] == 1) v = image->Value(q[2], q[3], p);
      else v = missing->Value(q[2], q[3], p);
      out[3 * i] = v.x(), out[3 * i + 1] = v.y(), out[3 * i + 2] = v.z();
    }
    write_bin(argv[3], out);
  } else if ((cmd == "image8" || cmd == "imagebytes") && argc == 4) {
    // image8: the reference's 8-bit decode (stbi_load, 3 channels; what Image::Load feeds to
    // the gamma step); imagebytes: the texels of scene::Image (stbi_loadf + FloatToByte).
    // Output: int32 width, int32 height, then width * height * 3 bytes (0 x 0 on failure).
    int32_t wh[2] = {0, 0};
    std::vector<unsigned char> bytes;
    if (cmd == "image8") {
      int n = 0;
      unsigned char* d = stbi_load(argv[2], &wh[0], &wh[1], &n, 3);
      if (d) bytes.assign(d, d + (size_t)wh[0] * wh[1] * 3), stbi_image_free(d);
      else wh[0] = wh[1] = 0;
    } else {
      scene::Image img(argv[2]);
      wh[0] = img.Width(), wh[1] = img.Height();
      if (img.Height() <= 0) wh[0] = wh[1] = 0;
      for (int y = 0; y < wh[1]; y++)
        for (int x = 0; x < wh[0]; x++) bytes.insert(bytes.end(), img.PixelData(x, y), img.PixelData(x, y) + 3);
    }
    std::ofstream o(argv[3], std::ios::binary);
    o.write((const char*)wh, sizeof wh);
    o.write((const char*)bytes.data(), (std::streamsize)bytes.size());
  } else if (cmd == "texels" && argc == 3) {
    scene::Image img("earthmap.jpg");
    std::ofstream o(argv[2], std::ios::binary);
    o << "P6\n" << img.Width() << ' ' << img.Height() << "\n255\n";
    for (int y = 0; y < img.Height(); y++)
      for (int x = 0; x < img.Width(); x++) o.write((const char*)img.PixelData(x, y), 3);
  } else if (cmd == "pixelstate" && argc == 4) {
    // input: sequences of (n, then n samples of 3 doubles) ; output per record: mean3 m2 3 sum3 conv
    auto c = read_bin<double>(argv[2]);
    std::vector<double> out;
    size_t k = 0;
    while (k < c.size()) {
      int n = (int)c[k++];
      integrator::PixelState ps;
      for (int i = 0; i < n; i++) {
        integrator::RecordSample(ps, Color(c[k], c[k + 1], c[k + 2]));
        k += 3;
        bool conv = integrator::IsConverged(ps, 0.05f, 16);
        out.insert(out.end(), {ps.mean.x(), ps.mean.y(), ps.mean.z(), ps.m2.x(), ps.m2.y(), ps.m2.z(),
                               ps.sum.x(), ps.sum.y(), ps.sum.z(), (double)conv});
      }
    }
    write_bin(argv[3], out);
  } else if (cmd == "render" && argc == 23) {
    auto S = load_scene(argv[2], argv[3]);
    Cam cam = parse_cam(argv + 4);
    // seed "random": the main thread keeps its random_device seed too, as the reference runs
    // the bunny scene (no SeedRng call on that path; random.h:14-17)
    if (std::string(argv[21]) != "random") core::SeedRng((unsigned)std::strtoul(argv[21], nullptr, 10));
    render_wavefront(*S, cam, std::atoi(argv[18]), std::atoi(argv[19]), 2 * 8192, std::atoi(argv[20]) != 0,
                     argv[22]);
  } else if (cmd == "megakernel" && argc == 22) {
    auto S = load_scene(argv[2], argv[3]);
    Cam cam = parse_cam(argv + 4);
    core::SeedRng((unsigned)std::strtoul(argv[20], nullptr, 10));
    render_megakernel(*S, cam, std::atoi(argv[18]), std::atoi(argv[19]), argv[21]);
  } else if (cmd == "megakernel_adaptive" && argc == 24) {
    auto S = load_scene(argv[2], argv[3]);
    Cam cam = parse_cam(argv + 4);
    core::SeedRng((unsigned)std::strtoul(argv[22], nullptr, 10));
    render_megakernel_adaptive(*S, cam, std::atoi(argv[18]), std::atoi(argv[19]), std::atoi(argv[20]),
                               std::strtof(argv[21], nullptr), argv[23]);
  } else {
    usage();
  }
  return 0;
}
