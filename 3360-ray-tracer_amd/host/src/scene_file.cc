// scene_file.cc — .rtxs scene files and the reference's scene recipes (main.cc).
#include <cstdio>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "rt/scene.h"

namespace rt::scene {

using core::Color;
using core::Point3;

namespace {
std::string join(const std::string& dir, const std::string& name) {
  if (name.empty() || name[0] == '/' || dir.empty()) return name;
  return dir + "/" + name;
}
}  // namespace

std::shared_ptr<Scene> LoadSceneFile(const std::string& path, const std::string& asset_dir) {
  std::ifstream in(path);
  if (!in) throw std::runtime_error("cannot open scene file " + path);
  auto root = std::make_shared<Scene>();
  Scene list;
  bool bvh = false;
  std::string line;
  int lineno = 0;
  auto bad = [&](const std::string& why) {
    throw std::runtime_error(path + ":" + std::to_string(lineno) + ": " + why);
  };
  std::vector<std::shared_ptr<material::Texture>>& tex = root->texture_order;
  std::vector<std::shared_ptr<material::Material>>& mat = root->material_order;
  auto T = [&](int i) {
    if (i < 0 || i >= (int)tex.size()) bad("texture id out of range");
    return tex[i];
  };
  auto M = [&](int i) {
    if (i < 0 || i >= (int)mat.size()) bad("material id out of range");
    return mat[i];
  };
  while (std::getline(in, line)) {
    lineno++;
    std::istringstream ss(line);
    std::string kw;
    if (!(ss >> kw) || kw[0] == '#') continue;
    if (kw == "rtxscene") continue;
    if (kw == "bvh") {
      int b = 0;
      ss >> b;
      bvh = b != 0;
    } else if (kw == "tex") {
      int id;
      std::string kind;
      ss >> id >> kind;
      if (id != (int)tex.size()) bad("texture ids must be dense and in order");
      if (kind == "solid") {
        double r, g, b;
        if (!(ss >> r >> g >> b)) bad("solid needs r g b");
        tex.push_back(std::make_shared<material::SolidColor>(Color(r, g, b)));
      } else if (kind == "checker") {
        double sc;
        int e, o;
        if (!(ss >> sc >> e >> o)) bad("checker needs scale even odd");
        tex.push_back(std::make_shared<material::CheckerTexture>(sc, T(e), T(o)));
      } else if (kind == "image") {
        std::string name;
        ss >> name;
        // an image name without extension is the reference's "<name>.jpg" (main.cc:65); names
        // are resolved against asset_dir first (RTX_ASSET_DIR / package assets after)
        if (name.find('.') == std::string::npos) name += ".jpg";
        std::string p = join(asset_dir, name);
        std::ifstream probe(p);
        tex.push_back(std::make_shared<material::ImageTexture>((probe ? p : name).c_str()));
      } else {
        bad("unknown texture kind " + kind);
      }
    } else if (kw == "mat") {
      int id;
      std::string kind;
      ss >> id >> kind;
      if (id != (int)mat.size()) bad("material ids must be dense and in order");
      if (kind == "lambertian") {
        int t;
        ss >> t;
        mat.push_back(std::make_shared<material::Lambertian>(T(t)));
      } else if (kind == "metal") {
        double r, g, b, fz;
        if (!(ss >> r >> g >> b >> fz)) bad("metal needs r g b fuzz");
        mat.push_back(std::make_shared<material::Metal>(Color(r, g, b), fz));
      } else if (kind == "dielectric") {
        double ri;
        ss >> ri;
        mat.push_back(std::make_shared<material::Dielectric>(ri));
      } else if (kind == "light") {
        int t;
        ss >> t;
        mat.push_back(std::make_shared<material::DiffuseLight>(T(t)));
      } else {
        bad("unknown material kind " + kind);
      }
    } else if (kw == "sphere") {
      double x, y, z, r;
      int m;
      if (!(ss >> x >> y >> z >> r >> m)) bad("sphere needs cx cy cz r mat");
      list.Add(std::make_shared<geom::Sphere>(Point3(x, y, z), r, M(m)));
    } else if (kw == "tri") {
      double a[9];
      int m;
      for (double& q : a)
        if (!(ss >> q)) bad("tri needs 9 coordinates");
      ss >> m;
      list.Add(std::make_shared<geom::Triangle>(Point3(a[0], a[1], a[2]), Point3(a[3], a[4], a[5]),
                                                Point3(a[6], a[7], a[8]), M(m)));
    } else if (kw == "rect") {
      std::string ax;
      double a0, a1, b0, b1, k;
      int m;
      if (!(ss >> ax >> a0 >> a1 >> b0 >> b1 >> k >> m)) bad("rect needs axis a0 a1 b0 b1 k mat");
      if (ax == "xy") list.Add(std::make_shared<geom::xy_rect>(a0, a1, b0, b1, k, M(m)));
      else if (ax == "xz") list.Add(std::make_shared<geom::xz_rect>(a0, a1, b0, b1, k, M(m)));
      else if (ax == "yz") list.Add(std::make_shared<geom::yz_rect>(a0, a1, b0, b1, k, M(m)));
      else bad("rect axis must be xy, xz or yz");
    } else if (kw == "obj") {
      std::string name;
      double sc;
      int m;
      if (!(ss >> name >> sc >> m)) bad("obj needs file scale mat");
      std::string p = join(asset_dir, name);
      std::ifstream probe(p);
      if (!probe) p = ResolveAsset(name);
      auto mesh = geom::load_obj(p, M(m), sc);
      for (auto& t : mesh->tris) list.Add(t);
    } else {
      bad("unknown keyword " + kw);
    }
  }
  if (bvh) root->Add(std::make_shared<geom::Bvh>(list));
  else
    for (auto& o : list.objects_) root->Add(o);
  return root;
}

void WriteSceneFile(const FlatScene& f, bool bvh, const std::string& path) {
  FILE* o = std::fopen(path.c_str(), "w");
  if (!o) throw std::runtime_error("cannot write " + path);
  std::fprintf(o, "rtxscene 1\nbvh %d\n", bvh ? 1 : 0);
  for (size_t i = 0; i < f.textures.size(); i++) {
    const rtx_texture& t = f.textures[i];
    if (t.kind == RTX_TEX_SOLID)
      std::fprintf(o, "tex %zu solid %.17g %.17g %.17g\n", i, t.color[0], t.color[1], t.color[2]);
    else if (t.kind == RTX_TEX_CHECKER)
      std::fprintf(o, "tex %zu checker %.17g %d %d\n", i, 1.0 / t.inv_scale, t.even, t.odd);
    else {
      std::string n = f.texture_names[i];
      const size_t slash = n.rfind('/');
      if (slash != std::string::npos) n = n.substr(slash + 1);
      const size_t dot = n.rfind('.');
      if (dot != std::string::npos) n = n.substr(0, dot);
      std::fprintf(o, "tex %zu image %s\n", i, n.c_str());
    }
  }
  for (size_t i = 0; i < f.materials.size(); i++) {
    const rtx_material& m = f.materials[i];
    switch (m.kind) {
      case RTX_MAT_LAMBERTIAN: std::fprintf(o, "mat %zu lambertian %d\n", i, m.texture); break;
      case RTX_MAT_METAL:
        std::fprintf(o, "mat %zu metal %.17g %.17g %.17g %.17g\n", i, m.albedo[0], m.albedo[1], m.albedo[2], m.fuzz);
        break;
      case RTX_MAT_DIELECTRIC: std::fprintf(o, "mat %zu dielectric %.17g\n", i, m.ref_idx); break;
      default: std::fprintf(o, "mat %zu light %d\n", i, m.texture); break;
    }
  }
  static const char* ax[] = {"", "", "xy", "xz", "yz"};
  for (const rtx_prim& p : f.list_prims) {
    if (p.kind == RTX_PRIM_SPHERE)
      std::fprintf(o, "sphere %.17g %.17g %.17g %.17g %d\n", p.g[0], p.g[1], p.g[2], p.g[3], p.material);
    else if (p.kind == RTX_PRIM_TRIANGLE) {
      std::fprintf(o, "tri");
      for (int i = 0; i < 9; i++) std::fprintf(o, " %.17g", p.g[i]);
      std::fprintf(o, " %d\n", p.material);
    } else {
      std::fprintf(o, "rect %s %.17g %.17g %.17g %.17g %.17g %d\n", ax[p.kind], p.g[0], p.g[1], p.g[2], p.g[3], p.g[4],
                   p.material);
    }
  }
  std::fclose(o);
}

// ---------------------------------------------------------------------------------------
// Recipes.  Random draws follow the reference build's evaluation order (g++ evaluates a
// call's arguments right to left): Point3 center(a + 0.9*U, 0.2, b + 0.9*U) draws the z
// term first (main.cc:102).
// ---------------------------------------------------------------------------------------
namespace {

template <class T, class... A>
std::shared_ptr<T> reg(Scene& s, A&&... a) {
  auto p = std::make_shared<T>(std::forward<A>(a)...);
  if constexpr (std::is_base_of_v<material::Material, T>) s.material_order.push_back(p);
  else s.texture_order.push_back(p);
  return p;
}
std::shared_ptr<material::Lambertian> lambert(Scene& s, const Color& c) {
  return reg<material::Lambertian>(s, std::static_pointer_cast<material::Texture>(reg<material::SolidColor>(s, c)));
}

void random_grid(Scene& root, Scene& w, int lo, int hi, bool mixed, std::shared_ptr<material::Material> earth) {
  for (int a = lo; a < hi; a++) {
    for (int b = lo; b < hi; b++) {
      const double choose_mat = core::RandomDouble();
      const double rz = core::RandomDouble();
      const double rx = core::RandomDouble();
      const Point3 center(a + 0.9 * rx, 0.2, b + 0.9 * rz);
      if ((center - Point3(4, 0.2, 0)).length() <= 0.9) continue;
      if (mixed && choose_mat < 0.2) {
        w.Add(std::make_shared<geom::Sphere>(center, 0.2, earth));
      } else if (choose_mat < 0.8) {
        Color albedo;
        if (mixed) {
          albedo = core::RandomVec3(0, 1);
        } else {
          const Color r = core::RandomVec3();  // right operand of RandomVec3() * RandomVec3()
          const Color l = core::RandomVec3();
          albedo = l * r;
        }
        w.Add(std::make_shared<geom::Sphere>(center, 0.2, lambert(root, albedo)));
      } else if (choose_mat < 0.95) {
        const Color albedo = core::RandomVec3(0.5, 1);
        const double fuzz = core::RandomDouble(0, 0.5);
        w.Add(std::make_shared<geom::Sphere>(center, 0.2, reg<material::Metal>(root, albedo, fuzz)));
      } else {
        w.Add(std::make_shared<geom::Sphere>(center, 0.2, reg<material::Dielectric>(root, 1.5)));
      }
    }
  }
}

}  // namespace

std::shared_ptr<Scene> BuildRecipe(const std::string& name, uint32_t seed, const std::string& asset_dir) {
  auto root = std::make_shared<Scene>();
  Scene w;
  Scene& R = *root;
  if (name == "three") {  // BASELINE configs[0]: flat list, no BVH
    auto g = lambert(R, Color(0.8, 0.8, 0.0));
    auto c = lambert(R, Color(0.1, 0.2, 0.5));
    auto r = lambert(R, Color(0.7, 0.3, 0.3));
    R.Add(std::make_shared<geom::Sphere>(Point3(0.0, -100.5, -1.0), 100.0, g));
    R.Add(std::make_shared<geom::Sphere>(Point3(0.0, 0.0, -1.2), 0.5, c));
    R.Add(std::make_shared<geom::Sphere>(Point3(1.0, 0.0, -1.0), 0.5, r));
    return root;
  }
  if (name == "cornell") {  // main.cc:23-61
    auto red = lambert(R, Color(.65, .05, .05));
    auto white = lambert(R, Color(.73, .73, .73));
    auto green = lambert(R, Color(.12, .45, .15));
    auto light = reg<material::DiffuseLight>(
        R, std::static_pointer_cast<material::Texture>(reg<material::SolidColor>(R, Color(15, 15, 15))));
    const double S = 10.0, eps = 0.01;
    w.Add(std::make_shared<geom::yz_rect>(0, S, 0, S, S, green));
    w.Add(std::make_shared<geom::yz_rect>(0, S, 0, S, 0, red));
    w.Add(std::make_shared<geom::xz_rect>(0, S, 0, S, 0, white));
    w.Add(std::make_shared<geom::xz_rect>(0, S, 0, S, S, white));
    w.Add(std::make_shared<geom::xy_rect>(0, S, 0, S, S, white));
    w.Add(std::make_shared<geom::xz_rect>(3.0, 7.0, 3.0, 7.0, S - eps, light));
    auto glass = reg<material::Dielectric>(R, 1.5);
    auto metal = reg<material::Metal>(R, Color(0.85, 0.85, 0.95), 0.03);
    auto diffuse = lambert(R, Color(0.8, 0.3, 0.1));
    w.Add(std::make_shared<geom::Sphere>(Point3(3.2, 1.0, 7.0), 1.0, diffuse));
    w.Add(std::make_shared<geom::Sphere>(Point3(7.0, 1.0, 4.0), 1.0, metal));
    w.Add(std::make_shared<geom::Sphere>(Point3(5.0, 1.0, 2.5), 1.0, glass));
  } else if (name == "final") {  // the RTIOW final scene, SeedRng(seed)
    core::SeedRng(seed);
    w.Add(std::make_shared<geom::Sphere>(Point3(0, -1000, 0), 1000, lambert(R, Color(0.5, 0.5, 0.5))));
    random_grid(R, w, -11, 11, false, nullptr);
    w.Add(std::make_shared<geom::Sphere>(Point3(0, 1, 0), 1.0, reg<material::Dielectric>(R, 1.5)));
    w.Add(std::make_shared<geom::Sphere>(Point3(-4, 1, 0), 1.0, lambert(R, Color(0.4, 0.2, 0.1))));
    w.Add(std::make_shared<geom::Sphere>(Point3(4, 1, 0), 1.0, reg<material::Metal>(R, Color(0.7, 0.6, 0.5), 0.0)));
  } else if (name == "bunny") {  // bunny x50 (main.cc:135-137) on a ground sphere
    auto red = lambert(R, Color(0.8, 0.1, 0.1));
    std::string p = join(asset_dir, "stanford-bunny.obj");
    std::ifstream probe(p);
    if (!probe) p = ResolveAsset("stanford-bunny.obj");
    auto mesh = geom::load_obj(p, red, 50.0);
    for (auto& t : mesh->tris) w.Add(t);
    w.Add(std::make_shared<geom::Sphere>(Point3(0, -1003.9, 0), 1000, lambert(R, Color(0.5, 0.5, 0.5))));
  } else if (name == "mixed") {  // main.cc:72-145 Spheres(), SeedRng(seed)
    core::SeedRng(seed);
    std::string tp = join(asset_dir, "earthmap.jpg");
    std::ifstream probe(tp);
    auto earth_tex = reg<material::ImageTexture>(R, (probe ? tp : std::string("earthmap.jpg")).c_str());
    auto earth = reg<material::Lambertian>(R, std::static_pointer_cast<material::Texture>(earth_tex));
    auto ground = lambert(R, Color(0.8, 0.8, 0.0));
    auto center = lambert(R, Color(0.1, 0.2, 0.5));
    auto left = reg<material::Dielectric>(R, 1.50);
    auto bubble = reg<material::Dielectric>(R, 1.00 / 1.50);
    auto right = reg<material::Metal>(R, Color(0.8, 0.6, 0.2), 1.0);
    w.Add(std::make_shared<geom::Sphere>(Point3(0.0, -100.5, -1.0), 100.0, ground));
    w.Add(std::make_shared<geom::Sphere>(Point3(0.0, 0.0, -1.2), 0.5, center));
    w.Add(std::make_shared<geom::Sphere>(Point3(-1.0, 0.0, -1.0), 0.5, left));
    w.Add(std::make_shared<geom::Sphere>(Point3(-1.0, 0.0, -1.0), 0.4, bubble));
    w.Add(std::make_shared<geom::Sphere>(Point3(1.0, 0.0, -1.0), 0.5, right));
    auto ce = reg<material::SolidColor>(R, Color(0.2, 0.3, 0.1));
    auto co = reg<material::SolidColor>(R, Color(.9, .9, .9));
    auto checker = reg<material::CheckerTexture>(R, 0.32, std::static_pointer_cast<material::Texture>(ce),
                                                 std::static_pointer_cast<material::Texture>(co));
    w.Add(std::make_shared<geom::Sphere>(Point3(0, -1000, 0), 1000,
                                         reg<material::Lambertian>(R, std::static_pointer_cast<material::Texture>(checker))));
    random_grid(R, w, -110, 110, true, earth);
    w.Add(std::make_shared<geom::Sphere>(Point3(0, 1, 0), 1.0, reg<material::Dielectric>(R, 1.5)));
    w.Add(std::make_shared<geom::Sphere>(Point3(-4, 0, 0), 1.0, lambert(R, Color(0.4, 0.2, 0.1))));
    w.Add(std::make_shared<geom::Sphere>(Point3(4, 1, 0), 1.0, reg<material::Metal>(R, Color(0.7, 0.6, 0.5), 0.0)));
  } else {
    throw std::runtime_error("unknown scene recipe '" + name + "' (three, cornell, final, bunny, mixed)");
  }
  R.Add(std::make_shared<geom::Bvh>(w));
  return root;
}

}  // namespace rt::scene
