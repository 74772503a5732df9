// scene.cc — images, asset lookup, the Scene -> device flattener, cameras.json and Camera.
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <unordered_map>

#include "rt/image.h"
#include "rt/scene.h"

#ifndef RTX_ASSET_DIR_DEFAULT
#define RTX_ASSET_DIR_DEFAULT ""
#endif

namespace rt::core {
std::mt19937& GetRng() {  // random.h:14-17 (thread-local engine)
  thread_local std::mt19937 rng(std::random_device{}());
  return rng;
}
}  // namespace rt::core

namespace rt::scene {

// ---------------------------------------------------------------------------------------
// Image / assets
// ---------------------------------------------------------------------------------------
static bool file_exists(const std::string& p) {
  std::ifstream f(p);
  return (bool)f;
}

std::string ResolveAsset(const std::string& name) {
  if (name.empty()) return name;
  if (name[0] == '/' && file_exists(name)) return name;
  if (file_exists(name)) return name;
  if (const char* env = std::getenv("RTX_ASSET_DIR")) {
    std::string p = std::string(env) + "/" + name;
    if (file_exists(p)) return p;
  }
  std::string p = std::string(RTX_ASSET_DIR_DEFAULT) + "/" + name;
  if (file_exists(p)) return p;
  return "";
}

Image::Image(const std::string& filename) {
  if (!Load(filename)) std::cerr << "ERROR: Could not load image '" << filename << "'\n";  // image.cc:11-13
}

// image.cc:16-41: the file as named, then the image directory (here $RTX_ASSET_DIR and the
// package's assets/); decoded like stbi_loadf + FloatToByte (rt/image.h).
bool Image::Load(const std::string& filename) {
  const std::string path = ResolveAsset(filename);
  if (path.empty()) return false;
  int w = 0, h = 0;
  std::vector<unsigned char> texels;
  std::string err;
  if (!LoadTexels(path, w, h, texels, err)) {
    std::cerr << "image " << path << ": " << err << "\n";
    return false;
  }
  width_ = w, height_ = h, bdata_ = std::move(texels);
  return true;
}

const unsigned char* Image::PixelData(int x, int y) const {  // image.cc:50-67
  static unsigned char magenta[3] = {255, 0, 255};
  if (bdata_.empty()) return magenta;
  x = x < 0 ? 0 : (x < width_ ? x : width_ - 1);
  y = y < 0 ? 0 : (y < height_ ? y : height_ - 1);
  return &bdata_[((size_t)y * width_ + x) * 3];
}

}  // namespace rt::scene

namespace rt::material {
ImageTexture::ImageTexture(const char* filename)
    : name_(filename ? filename : ""), image_(std::make_shared<scene::Image>(name_)) {}
}  // namespace rt::material

namespace rt::scene {

// ---------------------------------------------------------------------------------------
// Flattener
// ---------------------------------------------------------------------------------------
rtx_scene_desc FlatScene::desc() const {
  rtx_scene_desc d{};
  d.prims = prims.data();
  d.n_prims = (int64_t)prims.size();
  d.nodes = nodes.empty() ? nullptr : nodes.data();
  d.n_nodes = (int64_t)nodes.size();
  d.materials = materials.data();
  d.n_materials = (int32_t)materials.size();
  d.textures = textures.data();
  d.n_textures = (int32_t)textures.size();
  d.images = images.data();
  d.n_images = (int32_t)images.size();
  return d;
}

namespace {

struct Registry {
  FlatScene& f;
  std::unordered_map<const material::Texture*, int> tex_id;
  std::unordered_map<const material::Material*, int> mat_id;
  std::unordered_map<const Image*, int> img_id;

  int Tex(const std::shared_ptr<material::Texture>& t) {
    if (!t) throw std::runtime_error("flatten: null texture");
    auto it = tex_id.find(t.get());
    if (it != tex_id.end()) return it->second;
    const int id = (int)f.textures.size();
    tex_id[t.get()] = id;
    f.textures.push_back(rtx_texture{});
    rtx_texture r{};
    r.image = -1;
    switch (t->Kind()) {
      case material::TextureKind::kSolid: {
        auto* s = static_cast<const material::SolidColor*>(t.get());
        r.kind = RTX_TEX_SOLID;
        for (int i = 0; i < 3; i++) r.color[i] = s->albedo()[i];
        break;
      }
      case material::TextureKind::kChecker: {
        auto* c = static_cast<const material::CheckerTexture*>(t.get());
        r.kind = RTX_TEX_CHECKER;
        r.inv_scale = c->inv_scale();
        r.even = Tex(c->even());
        r.odd = Tex(c->odd());
        break;
      }
      case material::TextureKind::kImage: {
        auto* im = static_cast<const material::ImageTexture*>(t.get());
        r.kind = RTX_TEX_IMAGE;
        const Image* img = &im->image();
        if (img->Height() > 0) {
          auto jt = img_id.find(img);
          if (jt == img_id.end()) {
            const int iid = (int)f.images.size();
            img_id[img] = iid;
            rtx_image ri{img->Width(), img->Height(), img->bytes().data()};
            f.images.push_back(ri);
            f.image_refs.push_back(std::shared_ptr<const Image>(t, img));  // aliasing: keeps the texture alive
            r.image = iid;
          } else {
            r.image = jt->second;
          }
        }
        break;
      }
    }
    f.textures[id] = r;
    return id;
  }

  int Mat(const std::shared_ptr<material::Material>& m) {
    if (!m) throw std::runtime_error("flatten: primitive without material");
    auto it = mat_id.find(m.get());
    if (it != mat_id.end()) return it->second;
    const int id = (int)f.materials.size();
    mat_id[m.get()] = id;
    f.materials.push_back(rtx_material{});
    f.material_ptrs.push_back(m);
    rtx_material r{};
    r.kind = (int32_t)m->Kind();
    r.texture = -1;
    switch (m->Kind()) {
      case material::MaterialKind::kLambertian:
        r.texture = Tex(static_cast<const material::Lambertian*>(m.get())->texture());
        break;
      case material::MaterialKind::kMetal: {
        auto* mm = static_cast<const material::Metal*>(m.get());
        for (int i = 0; i < 3; i++) r.albedo[i] = mm->albedo()[i];
        r.fuzz = mm->fuzz();
        break;
      }
      case material::MaterialKind::kDielectric:
        r.ref_idx = static_cast<const material::Dielectric*>(m.get())->ref_idx();
        break;
      case material::MaterialKind::kDiffuseLight:
        r.texture = Tex(static_cast<const material::DiffuseLight*>(m.get())->texture());
        break;
    }
    f.materials[id] = r;
    return id;
  }

  rtx_prim Prim(const geom::Hittable& h) {
    rtx_prim p;
    if (!h.ToPrim(&p)) throw std::runtime_error("flatten: nested aggregate (only Scene{primitives} or Scene{Bvh})");
    p.material = Mat(h.GetMaterial());
    return p;
  }
};

}  // namespace

FlatScene Flatten(const Scene& root) {
  FlatScene f;
  Registry R{f};
  for (const auto& t : root.texture_order) R.Tex(t);
  for (const auto& m : root.material_order) R.Mat(m);
  const auto& objs = root.Objects();
  const geom::Bvh* bvh = objs.size() == 1 ? dynamic_cast<const geom::Bvh*>(objs[0].get()) : nullptr;
  if (bvh) {
    const auto& nodes = bvh->nodes();
    const auto& idx = bvh->prim_indices();
    const auto& prims = bvh->primitives();
    f.nodes.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) {
      rtx_bvh_node& n = f.nodes[i];
      n.lo[0] = nodes[i].bbox.x.min_, n.hi[0] = nodes[i].bbox.x.max_;
      n.lo[1] = nodes[i].bbox.y.min_, n.hi[1] = nodes[i].bbox.y.max_;
      n.lo[2] = nodes[i].bbox.z.min_, n.hi[2] = nodes[i].bbox.z.max_;
      n.left_first = nodes[i].left_pIdx, n.right_count = nodes[i].right_pCnt, n.is_leaf = nodes[i].isLeaf;
      n.pad_ = 0;
    }
    f.prim_indices.assign(idx.begin(), idx.end());
    f.list_prims.reserve(prims.size());
    for (const auto& p : prims) f.list_prims.push_back(R.Prim(*p));
    f.prims.reserve(idx.size());
    for (int k : idx) f.prims.push_back(f.list_prims[k]);  // leaf order: leaf (first, count) index directly
  } else {
    for (const auto& o : objs) f.prims.push_back(R.Prim(*o));
    f.list_prims = f.prims;
  }
  f.texture_names.assign(f.textures.size(), "");
  for (const auto& kv : R.tex_id)
    if (kv.first->Kind() == material::TextureKind::kImage)
      f.texture_names[kv.second] = static_cast<const material::ImageTexture*>(kv.first)->name();
  return f;
}

// ---------------------------------------------------------------------------------------
// cameras.json: a small JSON reader (objects, arrays, numbers, strings, literals).
// ---------------------------------------------------------------------------------------
namespace {

struct Json {
  enum Type { kNull, kNum, kStr, kArr, kObj, kBool } type = kNull;
  double num = 0;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;
  const Json* get(const std::string& k) const {
    for (const auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JsonParser {
  const std::string& s;
  size_t i = 0;
  [[noreturn]] void err(const char* what) {
    throw std::runtime_error(std::string("cameras.json: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
  }
  Json value() {
    ws();
    if (i >= s.size()) err("unexpected end");
    Json v;
    const char c = s[i];
    if (c == '{') {
      v.type = Json::kObj;
      i++;
      ws();
      if (s[i] == '}') return i++, v;
      while (true) {
        ws();
        Json k = value();
        if (k.type != Json::kStr) err("object key must be a string");
        ws();
        if (s[i++] != ':') err("expected ':'");
        v.obj.emplace_back(k.str, value());
        ws();
        if (s[i] == ',') { i++; continue; }
        if (s[i] == '}') { i++; break; }
        err("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.type = Json::kArr;
      i++;
      ws();
      if (s[i] == ']') return i++, v;
      while (true) {
        v.arr.push_back(value());
        ws();
        if (s[i] == ',') { i++; continue; }
        if (s[i] == ']') { i++; break; }
        err("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.type = Json::kStr;
      i++;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\' && i + 1 < s.size()) i++;
        v.str += s[i++];
      }
      if (i >= s.size()) err("unterminated string");
      i++;
    } else if (s.compare(i, 4, "true") == 0) {
      v.type = Json::kBool, v.num = 1, i += 4;
    } else if (s.compare(i, 5, "false") == 0) {
      v.type = Json::kBool, v.num = 0, i += 5;
    } else if (s.compare(i, 4, "null") == 0) {
      i += 4;
    } else {
      const char* b = s.c_str() + i;
      char* e = nullptr;
      v.type = Json::kNum;
      v.num = std::strtod(b, &e);
      if (e == b) err("bad value");
      i += (size_t)(e - b);
    }
    return v;
  }
};

Json parse_json(const std::string& text) {
  JsonParser p{text};
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.err("trailing characters");
  return v;
}

core::Vec3 required_vec(const Json& o, const char* k) {  // camera.h:48-50 (j["lookfrom"][i])
  const Json* v = o.get(k);
  if (!v || v->type != Json::kArr || v->arr.size() < 3) throw std::runtime_error(std::string("camera: missing ") + k);
  return core::Vec3(v->arr[0].num, v->arr[1].num, v->arr[2].num);
}

CameraConfig camera_from(const Json& o) {  // parseCamera (camera.h:40-56)
  CameraConfig c;
  auto num = [&](const char* k, double def) {
    const Json* v = o.get(k);
    return v && v->type == Json::kNum ? v->num : def;
  };
  c.aspect_ratio = num("aspectRatio", c.aspect_ratio);
  c.image_width = (int)num("imageWidth", c.image_width);
  c.samples_per_pixel = (int)num("samplesPerPixel", c.samples_per_pixel);
  c.max_depth = (int)num("maxDepth", c.max_depth);
  c.vfov = num("vfov", c.vfov);
  c.lookfrom = required_vec(o, "lookfrom");
  c.lookat = required_vec(o, "lookat");
  c.vup = required_vec(o, "vup");
  c.defocus_angle = num("defocusAngle", c.defocus_angle);
  c.focus_dist = num("focusDist", c.focus_dist);
  return c;
}

}  // namespace

CameraConfig parseCamera(const std::string& text) { return camera_from(parse_json(text)); }

std::unordered_map<std::string, CameraConfig> loadCameras(const std::string& filename) {
  std::ifstream in(filename);
  if (!in) throw std::runtime_error("cannot open " + filename);
  std::stringstream ss;
  ss << in.rdbuf();
  Json root = parse_json(ss.str());
  if (root.type != Json::kObj) throw std::runtime_error("cameras.json: top level must be an object");
  std::unordered_map<std::string, CameraConfig> out;
  for (const auto& kv : root.obj) out[kv.first] = camera_from(kv.second);
  return out;
}

void Camera::SetFromConfig(const CameraConfig& c) {  // camera.h:84-97
  aspect_ratio_ = c.aspect_ratio, image_width_ = c.image_width, max_depth_ = c.max_depth;
  samples_per_pixel_ = c.samples_per_pixel, vfov_ = c.vfov;
  lookfrom_ = c.lookfrom, lookat = c.lookat, vup_ = c.vup;
  defocus_angle_ = c.defocus_angle, focus_dist_ = c.focus_dist;
}

void Camera::Initialize() {
  rtx_camera_config c{};
  c.aspect_ratio = aspect_ratio_, c.image_width = image_width_, c.samples_per_pixel = samples_per_pixel_;
  c.max_depth = max_depth_, c.vfov = vfov_;
  for (int i = 0; i < 3; i++) c.lookfrom[i] = lookfrom_[i], c.lookat[i] = lookat[i], c.vup[i] = vup_[i];
  c.defocus_angle = defocus_angle_, c.focus_dist = focus_dist_;
  if (rtx_camera_init(&c, &dev_) != RTX_OK) throw std::runtime_error(rtx_last_error());
}

}  // namespace rt::scene
