// oracle/rtx_oracle.cc — TEST INFRASTRUCTURE ONLY: the CPU checker, never the product.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
// library.  The product (3360-ray-tracer_amd/, librtx.so) never links, loads or falls
// back to it.
//
// A from-scratch CPU restatement of Luke-TS/3360-ray-tracer's per-pixel path-tracing hot
// path (reference snapshot 2025-11-14).  Every function names the reference file:line it
// follows.  Arithmetic is IEEE double with the reference's float islands, evaluated in the
// reference's operation order (built with -ffp-contract=off, like the reference's x86-64
// g++ build which has no FMA).
//
// Pinning: every piece is checked against golden vectors produced by the reference's own
// compiled code (oracle/ref_harness.cc -> tests/golden/, script oracle/gen_golden.py):
// BVH node arrays, closest-hit records, material samples, textures, PixelState sequences,
// and whole seeded single-thread renders ("mt" RNG mode, byte-identical PPM and
// bit-identical linear framebuffer).  Camera::Initialize/GetRay and the Render loop glue
// are restated in the harness too (camera.h needs nlohmann/json, absent), see DESIGN.md.
//
// Two RNG modes:
//   mt      : one std::mt19937 + uniform_real_distribution<double> stream consumed in the
//             reference's sequential order (random.h:14-32; draw order SURVEY Appendix A.10)
//   philox  : counter-based Philox-4x32-10 keyed by (seed), counter (draw>>1, sample,
//             global pixel, stream); stream 0 = camera ray, stream n+1 = shading of path
//             segment n, draw restarting at 0 per stream — shared bit-for-bit with the HIP
//             kernels (3360-ray-tracer_amd/csrc/rtx_device.h Rng).

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include <omp.h>

namespace orc {

constexpr double kPi = 3.14159265358979323846;  // constants.h:11
constexpr double kInf = std::numeric_limits<double>::infinity();

// ---------------------------------------------------------------------------------------
// Vec3 (vec3.h:8-107).  a/t is (1/t)*a (vec3.h:91-93); dot and length_squared sum left to
// right.
// ---------------------------------------------------------------------------------------
struct V3 {
  double x = 0, y = 0, z = 0;
  double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator*(double t, V3 a) { return {t * a.x, t * a.y, t * a.z}; }
inline V3 operator*(V3 a, double t) { return t * a; }  // vec3.h:87-89
inline V3 operator/(V3 a, double t) { return (1.0 / t) * a; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline double len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline double len(V3 a) { return std::sqrt(len2(a)); }
inline V3 cross(V3 u, V3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
inline bool near_zero(V3 a) {  // vec3.h:50-55
  const double s = 1e-8;
  return std::fabs(a.x) < s && std::fabs(a.y) < s && std::fabs(a.z) < s;
}
inline V3 normalize(V3 v) {  // math_utils.h:93-97
  double l = len(v);
  if (l == 0.0) return {0, 0, 0};
  return v / l;
}
inline V3 reflect(V3 v, V3 n) { return v - (2.0 * dot(v, n)) * n; }  // math_utils.h:14-16
inline V3 refract(V3 uv, V3 n, double eta) {                          // math_utils.h:24-29
  double cos_theta = std::fmin(dot(-uv, n), 1.0);
  V3 perp = eta * (uv + cos_theta * n);
  V3 par = (-std::sqrt(std::fabs(1.0 - len2(perp)))) * n;
  return perp + par;
}

// ---------------------------------------------------------------------------------------
// RNG
// ---------------------------------------------------------------------------------------
struct Philox {
  // Philox-4x32-10 (Salmon et al., SC'11).  Shared definition with csrc/rtx_device.h.
  static void block(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; r++) {
      uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
      uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
      uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
      uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
      c[0] = n0;
      c[1] = (uint32_t)p1;
      c[2] = n2;
      c[3] = (uint32_t)p0;
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
  }
};

struct Rng {
  int mode = 0;  // 0 = mt, 1 = philox
  std::mt19937* mt = nullptr;
  std::uniform_real_distribution<double>* dist = nullptr;
  uint64_t seed = 0;
  uint32_t pixel = 0, sample = 0, stream = 0, draw = 0;
  void open(uint32_t s) { stream = s, draw = 0; }  // philox: start stream s at draw 0
  double next() {  // RandomDouble() (random.h:23-26)
    if (mode == 0) return (*dist)(*mt);
    uint32_t c[4] = {draw >> 1, sample, pixel, stream};
    Philox::block(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x52545831u);
    uint32_t lo = (draw & 1) ? c[2] : c[0];
    uint32_t hi = (draw & 1) ? c[3] : c[1];
    draw++;
    uint64_t bits = ((uint64_t)hi << 32) | lo;
    return (double)(bits >> 11) * 0x1p-53;
  }
  double next(double mn, double mx) { return mn + (mx - mn) * next(); }  // random.h:31-33
};

// RandomUnitVector (math_utils.h:62-70); RandomVec3(-1,1) evaluates its three Vec3
// constructor arguments right to left under g++ (z, y, x) — SURVEY Appendix A.10.
inline V3 random_unit_vector(Rng& g) {
  while (true) {
    double z = g.next(-1.0, 1.0);
    double y = g.next(-1.0, 1.0);
    double x = g.next(-1.0, 1.0);
    V3 p{x, y, z};
    double l2 = len2(p);
    if (l2 > 1e-12 && l2 <= 1.0) return p / std::sqrt(l2);
  }
}
inline V3 random_in_unit_disk(Rng& g) {  // math_utils.h:83-88 (y drawn before x)
  while (true) {
    double y = g.next(-1, 1);
    double x = g.next(-1, 1);
    V3 p{x, y, 0.0};
    if (len2(p) < 1.0) return p;
  }
}
inline V3 random_cosine_direction(Rng& g, V3 normal) {  // math_utils.h:104-123
  double r1 = g.next();
  double r2 = g.next();
  double phi = 2.0 * kPi * r1;
  double r = std::sqrt(r2);
  double x = r * std::cos(phi);
  double y = r * std::sin(phi);
  double z = std::sqrt(1.0 - r2);
  V3 w = normalize(normal);
  V3 a = (std::fabs(w.x) > 0.9) ? v3(0, 1, 0) : v3(1, 0, 0);
  V3 v = normalize(cross(w, a));
  V3 u = cross(v, w);
  return normalize(x * u + y * v + z * w);
}

// ---------------------------------------------------------------------------------------
// Interval / Aabb (interval.h, aabb.h)
// ---------------------------------------------------------------------------------------
struct Box {
  double lo[3] = {kInf, kInf, kInf}, hi[3] = {-kInf, -kInf, -kInf};
};
inline Box box_of(V3 a, V3 b) {  // aabb.h:19-23
  Box r;
  for (int i = 0; i < 3; i++) {
    if (a[i] <= b[i]) r.lo[i] = a[i], r.hi[i] = b[i];
    else r.lo[i] = b[i], r.hi[i] = a[i];
  }
  return r;
}
inline Box box_union(const Box& a, const Box& b) {  // aabb.h:26-30 via interval.h:18-21
  Box r;
  for (int i = 0; i < 3; i++) {
    r.lo[i] = std::min(a.lo[i], b.lo[i]);
    r.hi[i] = std::max(a.hi[i], b.hi[i]);
  }
  return r;
}
inline Box box_expand(const Box& b, V3 p) {  // aabb.h:33-46
  Box r;
  for (int i = 0; i < 3; i++) {
    r.lo[i] = std::min(b.lo[i], p[i]);
    r.hi[i] = std::max(b.hi[i], p[i]);
  }
  return r;
}
inline V3 box_center(const Box& b) {
  return {0.5 * (b.lo[0] + b.hi[0]), 0.5 * (b.lo[1] + b.hi[1]), 0.5 * (b.lo[2] + b.hi[2])};
}
inline int longest_axis(const Box& b) {  // aabb.h:70-78
  double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  if (dx >= dy && dx >= dz) return 0;
  if (dy >= dz) return 1;
  return 2;
}
inline double surface_area(const Box& b) {  // aabb.h:81-86
  double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}
// Aabb::Hit slab test (aabb.h:92-115): relies on 1/0 = inf and NaN compares being false.
inline bool box_hit(const Box& b, V3 o, V3 d, double tmin, double tmax) {
  for (int a = 0; a < 3; a++) {
    const double adinv = 1.0 / d[a];
    double t0 = (b.lo[a] - o[a]) * adinv;
    double t1 = (b.hi[a] - o[a]) * adinv;
    if (t0 < t1) {
      if (t0 > tmin) tmin = t0;
      if (t1 < tmax) tmax = t1;
    } else {
      if (t1 > tmin) tmin = t1;
      if (t0 < tmax) tmax = t0;
    }
    if (tmax <= tmin) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------
// Textures (texture.h:11-77) and Image (image.cc:16-73)
// ---------------------------------------------------------------------------------------
struct Image {
  int w = 0, h = 0;
  std::vector<unsigned char> bytes;  // post-FloatToByte texels (image.cc:43-48)
  const unsigned char* pixel(int x, int y) const {  // image.cc:50-61
    static unsigned char magenta[3] = {255, 0, 255};
    if (bytes.empty()) return magenta;
    x = x < 0 ? 0 : (x < w ? x : w - 1);  // Image::Clamp image.cc:63-67
    y = y < 0 ? 0 : (y < h ? y : h - 1);
    return &bytes[((size_t)y * w + x) * 3];
  }
};

enum TexKind { TEX_SOLID = 0, TEX_CHECKER = 1, TEX_IMAGE = 2 };
struct Texture {
  int kind = TEX_SOLID;
  V3 color;
  double inv_scale = 1;
  int even = -1, odd = -1;
  std::shared_ptr<Image> img;
};

struct Scene;
V3 tex_value(const Scene& S, int t, double u, double v, V3 p);

// ---------------------------------------------------------------------------------------
// Materials (material.h/.cc)
// ---------------------------------------------------------------------------------------
enum MatKind { MAT_LAMBERT = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_LIGHT = 3 };
struct Material {
  int kind = MAT_LAMBERT;
  int tex = -1;     // lambertian albedo / light emission texture
  V3 albedo;        // metal
  double fuzz = 0;  // metal (clamped <=1 at construction, material.cc:78-80)
  double ri = 1;    // dielectric ref_idx_
};

// ---------------------------------------------------------------------------------------
// Primitives
// ---------------------------------------------------------------------------------------
enum PrimKind { PRIM_SPHERE = 0, PRIM_TRI = 1, PRIM_XY = 2, PRIM_XZ = 3, PRIM_YZ = 4 };
struct Prim {
  int kind;
  int mat;
  double g[9];  // sphere: c(3) r | tri: a b c | rect: a0 a1 b0 b1 k
  Box bbox;
};

struct Hit {  // HitRecord (hittable.h:18-42); u,v start at 0 where the reference is indeterminate
  bool hit = false;
  V3 p, normal;
  int mat = -1;
  double t = 0;
  bool front_face = false;
  double u = 0, v = 0;
};

inline void set_face_normal(Hit& h, V3 d, V3 outward) {  // hittable.h:31-34
  h.front_face = dot(d, outward) < 0;
  h.normal = h.front_face ? outward : -outward;
}

Box prim_bbox(const Prim& p) {
  const double* g = p.g;
  switch (p.kind) {
    case PRIM_SPHERE: {  // sphere.h:17-21
      V3 c{g[0], g[1], g[2]};
      double r = g[3];
      V3 rv{r, r, r};
      return box_of(c + rv, c - rv);
    }
    case PRIM_TRI: {  // triangle.h:18-38
      V3 a{g[0], g[1], g[2]}, b{g[3], g[4], g[5]}, c{g[6], g[7], g[8]};
      V3 mn{std::fmin(a.x, std::fmin(b.x, c.x)), std::fmin(a.y, std::fmin(b.y, c.y)),
            std::fmin(a.z, std::fmin(b.z, c.z))};
      V3 mx{std::fmax(a.x, std::fmax(b.x, c.x)), std::fmax(a.y, std::fmax(b.y, c.y)),
            std::fmax(a.z, std::fmax(b.z, c.z))};
      const double eps = 1e-6f;
      mn = mn + (-v3(eps, eps, eps));
      mx = mx + v3(eps, eps, eps);
      return box_of(mn, mx);
    }
    case PRIM_XY:  // rect.h:42-45
      return box_of(v3(g[0], g[2], g[4] - 0.0001), v3(g[1], g[3], g[4] + 0.0001));
    case PRIM_XZ:  // rect.h:87-89
      return box_of(v3(g[0], g[4] - 0.0001, g[2]), v3(g[1], g[4] + 0.0001, g[3]));
    default:  // PRIM_YZ rect.h:132-134
      return box_of(v3(g[4] - 0.0001, g[0], g[2]), v3(g[4] + 0.0001, g[1], g[3]));
  }
}

// Sphere::Hit (sphere.h:23-55) + get_sphere_uv (sphere.h:73-79); Surrounds is strict.
bool hit_sphere(const Prim& P, V3 o, V3 d, double tmin, double tmax, Hit& rec) {
  V3 c{P.g[0], P.g[1], P.g[2]};
  double radius = std::fmax(0, P.g[3]);
  V3 oc = c - o;
  double a = len2(d);
  double h = dot(d, oc);
  double cc = len2(oc) - radius * radius;
  double disc = h * h - a * cc;
  if (disc < 0) return false;
  double sq = std::sqrt(disc);
  double root = (h - sq) / a;
  if (!(tmin < root && root < tmax)) {
    root = (h + sq) / a;
    if (!(tmin < root && root < tmax)) return false;
  }
  rec.t = root;
  rec.p = o + rec.t * d;
  V3 outward = (rec.p - c) / radius;
  set_face_normal(rec, d, outward);
  double theta = std::acos(-outward.y);
  double phi = std::atan2(-outward.z, outward.x) + kPi;
  rec.u = phi / (2 * kPi);
  rec.v = theta / kPi;
  rec.mat = P.mat;
  return true;
}

// Triangle::Hit (triangle.h:41-87): float det/inv_det/u/v/t, inclusive t range, u/v of
// the record left untouched.
bool hit_triangle(const Prim& P, V3 o, V3 d, double tmin, double tmax, Hit& rec) {
  const float kEps = 1e-6f;
  V3 A{P.g[0], P.g[1], P.g[2]}, B{P.g[3], P.g[4], P.g[5]}, C{P.g[6], P.g[7], P.g[8]};
  V3 e1 = B - A, e2 = C - A;
  V3 pvec = cross(d, e2);
  float det = dot(e1, pvec);
  if (std::fabs(det) < kEps) return false;
  float inv_det = 1.0f / det;
  V3 tvec = o - A;
  float u = dot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return false;
  V3 qvec = cross(tvec, e1);
  float v = dot(d, qvec) * inv_det;
  if (v < 0.0f || (u + v) > 1.0f) return false;
  float t = dot(e2, qvec) * inv_det;
  if (t < tmin || t > tmax) return false;
  rec.t = t;
  rec.p = o + rec.t * d;
  rec.mat = P.mat;
  set_face_normal(rec, d, normalize(cross(e1, e2)));
  return true;
}

// xy_rect/xz_rect/yz_rect::Hit (rect.h:19-40, 65-85, 109-130).
bool hit_rect(const Prim& P, V3 o, V3 d, double tmin, double tmax, Hit& rec) {
  const double *g = P.g;
  int ax, a0, a1;  // plane axis, first and second in-plane axes
  V3 n;
  if (P.kind == PRIM_XY) ax = 2, a0 = 0, a1 = 1, n = v3(0, 0, 1);
  else if (P.kind == PRIM_XZ) ax = 1, a0 = 0, a1 = 2, n = v3(0, 1, 0);
  else ax = 0, a0 = 1, a1 = 2, n = v3(1, 0, 0);
  double t = (g[4] - o[ax]) / d[ax];
  if (!(tmin < t && t < tmax)) return false;
  double x = o[a0] + t * d[a0];
  double y = o[a1] + t * d[a1];
  if (x < g[0] || x > g[1] || y < g[2] || y > g[3]) return false;
  rec.u = (x - g[0]) / (g[1] - g[0]);
  rec.v = (y - g[2]) / (g[3] - g[2]);
  rec.t = t;
  set_face_normal(rec, d, n);
  rec.mat = P.mat;
  rec.p = o + rec.t * d;
  return true;
}

inline bool hit_prim(const Prim& P, V3 o, V3 d, double tmin, double tmax, Hit& rec) {
  if (P.kind == PRIM_SPHERE) return hit_sphere(P, o, d, tmin, tmax, rec);
  if (P.kind == PRIM_TRI) return hit_triangle(P, o, d, tmin, tmax, rec);
  return hit_rect(P, o, d, tmin, tmax, rec);
}

// ---------------------------------------------------------------------------------------
// BVH: binned SAH build (bvh.h:39-68,166-344) + pre-order flatten (bvh.h:347-367) +
// stack traversal (bvh.h:71-119).
// ---------------------------------------------------------------------------------------
struct Node {
  Box bbox;
  uint32_t a = 0, b = 0, leaf = 0;  // left_pIdx, right_pCnt, isLeaf (bvh.h:20-25)
};

struct Bvh {
  std::vector<int> idx;  // prim_indices_
  std::vector<Box> pb;
  std::vector<V3> pc;
  std::vector<Node> nodes;
  int root = -1;

  struct BNode {
    Box bounds;
    int first = 0, count = 0;
    std::unique_ptr<BNode> l, r;
  };

  void build(const std::vector<Prim>& prims) {
    int n = (int)prims.size();
    if (n == 0) return;
    idx.resize(n), pb.resize(n), pc.resize(n);
    for (int i = 0; i < n; i++) {
      idx[i] = i;
      pb[i] = prims[i].bbox;
      pc[i] = box_center(pb[i]);
    }
    auto r = sah(0, n);
    nodes.reserve(2 * (size_t)n);
    root = flatten(*r);
  }

  std::unique_ptr<BNode> sah(int start, int end) {
    const int MAX_LEAF = 4, BINS = 16;
    auto node = std::make_unique<BNode>();
    Box bounds;
    for (int i = start; i < end; i++) bounds = (i == start) ? pb[idx[i]] : box_union(bounds, pb[idx[i]]);
    node->bounds = bounds;
    int count = end - start;
    if (count <= MAX_LEAF) {
      node->first = start, node->count = count;
      return node;
    }
    Box cb;
    for (int i = start; i < end; i++) {
      V3 c = pc[idx[i]];
      cb = (i == start) ? box_of(c, c) : box_expand(cb, c);
    }
    int axis = longest_axis(cb);
    double mn = cb.lo[axis], mx = cb.hi[axis];
    double extent = mx - mn;
    if (extent <= 0.0) {
      node->first = start, node->count = count;
      return node;
    }
    const double inv = 1.0 / extent;
    auto bin_of = [&](int pi) {
      int b = static_cast<int>((pc[pi][axis] - mn) * inv * BINS);
      if (b < 0) b = 0;
      if (b >= BINS) b = BINS - 1;
      return b;
    };
    int bc[BINS] = {0};
    Box bb[BINS];
    for (int i = start; i < end; i++) {
      int b = bin_of(idx[i]);
      bb[b] = bc[b] == 0 ? pb[idx[i]] : box_union(bb[b], pb[idx[i]]);
      bc[b]++;
    }
    Box lb[BINS], rb[BINS];
    int lc[BINS], rc[BINS];
    Box acc;
    int accn = 0;
    bool init = false;
    for (int i = 0; i < BINS; i++) {
      if (bc[i] > 0) {
        acc = init ? box_union(acc, bb[i]) : bb[i];
        init = true;
        accn += bc[i];
      }
      lb[i] = acc, lc[i] = accn;
    }
    init = false, accn = 0;
    for (int i = BINS - 1; i >= 0; i--) {
      if (bc[i] > 0) {
        acc = init ? box_union(acc, bb[i]) : bb[i];
        init = true;
        accn += bc[i];
      }
      rb[i] = acc, rc[i] = accn;
    }
    double best = kInf;
    int split = -1;
    double parea = surface_area(bounds);
    for (int i = 0; i < BINS - 1; i++) {
      if (lc[i] == 0 || rc[i + 1] == 0) continue;
      double cost = (double)1.0f + (surface_area(lb[i]) / parea) * lc[i] * (double)1.0f +
                    (surface_area(rb[i + 1]) / parea) * rc[i + 1] * (double)1.0f;
      if (cost < best) best = cost, split = i;
    }
    float leaf_cost = count * 1.0f;
    if (split == -1 || best >= leaf_cost) {
      node->first = start, node->count = count;
      return node;
    }
    // std::partition exactly as the reference calls it (bvh.h:317-326).
    auto mid_it = std::partition(idx.begin() + start, idx.begin() + end,
                                 [&](int pi) { return bin_of(pi) <= split; });
    int mid = (int)(mid_it - idx.begin());
    if (mid - start == 0 || end - mid == 0) {
      node->first = start, node->count = count;
      return node;
    }
    node->l = sah(start, mid);
    node->r = sah(mid, end);
    return node;
  }

  int flatten(const BNode& b) {
    int i = (int)nodes.size();
    nodes.push_back({});
    nodes[i].bbox = b.bounds;
    if (b.count > 0) {
      nodes[i].leaf = 1, nodes[i].a = b.first, nodes[i].b = b.count;
    } else {
      int l = flatten(*b.l);
      int r = flatten(*b.r);
      nodes[i].leaf = 0, nodes[i].a = l, nodes[i].b = r;
    }
    return i;
  }
};

// ---------------------------------------------------------------------------------------
// Scene (scene.h) — root is either the flat list (Scene::Hit, scene.h:47-61) or a Scene
// holding one Bvh over all primitives.
// ---------------------------------------------------------------------------------------
struct Scene {
  std::vector<Texture> tex;
  std::vector<Material> mat;
  std::vector<Prim> prims;
  bool use_bvh = false;
  Bvh bvh;
  long long node_visits = 0, prim_tests = 0;  // not thread-safe; diagnostics only

  bool hit(V3 o, V3 d, double tmin, double tmax, Hit& out) const {
    if (!use_bvh) {  // Scene::Hit over primitives
      Hit tmp;
      bool any = false;
      double closest = tmax;
      for (const Prim& p : prims)
        if (hit_prim(p, o, d, tmin, closest, tmp)) any = true, closest = tmp.t, out = tmp;
      return any;
    }
    // Scene{Bvh}: Scene::Hit -> Bvh::Hit(r, [tmin, tmax]) (bvh.h:71-119)
    if (bvh.root < 0 || bvh.nodes.empty()) return false;
    Hit tmp;
    bool any = false;
    double closest = tmax;
    int stack[64];
    int sp = 0;
    stack[sp++] = bvh.root;
    while (sp > 0) {
      const Node& nd = bvh.nodes[stack[--sp]];
      if (!box_hit(nd.bbox, o, d, tmin, closest)) continue;
      if (nd.leaf) {
        for (uint32_t i = 0; i < nd.b; i++) {
          const Prim& p = prims[bvh.idx[nd.a + i]];
          if (hit_prim(p, o, d, tmin, closest, tmp)) any = true, closest = tmp.t, out = tmp;
        }
      } else {
        stack[sp++] = (int)nd.b;
        stack[sp++] = (int)nd.a;
      }
    }
    return any;
  }
};

V3 tex_value(const Scene& S, int t, double u, double v, V3 p) {
  const Texture& T = S.tex[t];
  if (T.kind == TEX_SOLID) return T.color;
  if (T.kind == TEX_CHECKER) {  // texture.h:37-45
    int xi = int(std::floor(T.inv_scale * p.x));
    int yi = int(std::floor(T.inv_scale * p.y));
    int zi = int(std::floor(T.inv_scale * p.z));
    bool even = (xi + yi + zi) % 2 == 0;
    return tex_value(S, even ? T.even : T.odd, u, v, p);
  }
  // ImageTexture::Value (texture.h:58-73)
  if (!T.img || T.img->h <= 0) return {0, 1, 1};
  u = u < 0 ? 0 : (u > 1 ? 1 : u);
  v = 1.0 - (v < 0 ? 0 : (v > 1 ? 1 : v));
  int i = int(u * T.img->w);
  int j = int(v * T.img->h);
  const unsigned char* px = T.img->pixel(i, j);
  double s = 1.0 / 255.0;
  return {s * px[0], s * px[1], s * px[2]};
}

inline bool mat_specular(const Material& m) { return m.kind != MAT_LAMBERT; }  // IsSpecular

inline V3 mat_emitted(const Scene& S, const Material& m, double u, double v, V3 p) {
  if (m.kind == MAT_LIGHT) return tex_value(S, m.tex, u, v, p);  // material.cc:312-316
  return {0, 0, 0};                                                 // material.h:50-54
}

// Deliberate estimator changes for the statistical parity leg's power check
// (tests/test_statistical_parity.py): 0 (always, except in that check) is the reference's
// estimator; 1 scales the Lambertian BRDF by 0.98, 2 brightens the sky by 2 %, 3 drops the
// eta^2 factor of dielectric refraction (material.cc:246-253).  Set by orc_set_perturb.
static int g_perturb = 0;

inline double reflectance(double c, double ri) {  // material.cc:258-262
  double r0 = (1.0 - ri) / (1.0 + ri);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * std::pow(1.0 - c, 5.0);
}

// Material::Sample (material.cc:57-74, 117-141, 194-256, 302-310).
bool mat_sample(const Scene& S, const Material& m, const Hit& rec, V3 wo, V3& wi, float& pdf, V3& f,
                Rng& g) {
  switch (m.kind) {
    case MAT_LAMBERT: {
      wi = random_cosine_direction(g, rec.normal);
      if (dot(wi, rec.normal) <= 0) return false;
      float c = dot(rec.normal, wi);  // Lambertian::Pdf material.cc:48-55
      pdf = (c <= 0.0f) ? 0.0f : (float)(c / kPi);
      if (dot(rec.normal, wi) <= 0) f = {0, 0, 0};  // Lambertian::Eval material.cc:36-46
      else f = tex_value(S, m.tex, rec.u, rec.v, rec.p) / kPi;
      if (g_perturb == 1) f = 0.98 * f;
      return true;
    }
    case MAT_METAL: {
      wi = reflect(-wo, rec.normal);
      wi = wi + m.fuzz * random_unit_vector(g);
      wi = normalize(wi);
      if (dot(wi, rec.normal) <= 0) return false;
      pdf = 1.0f;
      f = m.albedo;
      return true;
    }
    case MAT_DIELECTRIC: {
      V3 n = rec.normal;
      double eta_i = 1.0, eta_t = m.ri;
      if (!rec.front_face) std::swap(eta_i, eta_t);
      double eta = eta_i / eta_t;
      V3 win = -normalize(wo);
      double ci = dot(win, n);
      ci = std::clamp(ci, -1.0, 1.0);
      double si = std::sqrt(std::max(0.0, 1.0 - ci * ci));
      double st = eta * si;
      pdf = 1.0f;
      if (st >= 1.0) {
        wi = reflect(win, n);
        f = {1.0, 1.0, 1.0};
        return true;
      }
      double Fr = reflectance(std::fabs(ci), m.ri);
      if (g.next() < Fr) {
        wi = reflect(win, n);
        f = {1.0, 1.0, 1.0};
        return true;
      }
      wi = refract(win, n, eta);
      double k = g_perturb == 3 ? 1.0 : eta * eta;
      f = {k, k, k};
      return true;
    }
    default:
      return false;
  }
}

// Material::Scatter (material.cc:20-34, 82-94, 148-172, 273-280) for megakernel mode.
bool mat_scatter(const Scene& S, const Material& m, V3 rin_d, const Hit& rec, V3& att, V3& so, V3& sd,
                 Rng& g) {
  switch (m.kind) {
    case MAT_LAMBERT: {
      V3 dir = rec.normal + random_unit_vector(g);
      if (near_zero(dir)) dir = rec.normal;
      so = rec.p, sd = dir;
      att = tex_value(S, m.tex, rec.u, rec.v, rec.p);
      return true;
    }
    case MAT_METAL: {
      V3 r = reflect(rin_d, rec.normal);
      r = r + m.fuzz * random_unit_vector(g);
      so = rec.p, sd = r;
      att = m.albedo;
      return dot(sd, rec.normal) > 0;
    }
    case MAT_DIELECTRIC: {
      att = {1.0, 1.0, 1.0};
      double eta = rec.front_face ? (1.0 / m.ri) : m.ri;
      V3 ud = normalize(rin_d);
      double ct = std::fmin(dot(-ud, rec.normal), 1.0);
      double stt = std::sqrt(1.0 - ct * ct);
      bool cannot = eta * stt > 1.0;
      V3 dir;
      if (cannot || reflectance(ct, eta) > g.next()) dir = reflect(ud, rec.normal);
      else dir = refract(ud, rec.normal, eta);
      so = rec.p, sd = dir;
      return true;
    }
    default:
      return false;
  }
}

// ---------------------------------------------------------------------------------------
// Camera (camera.h:25-131,134-144,196-203)
// ---------------------------------------------------------------------------------------
struct Camera {
  double aspect = 16.0 / 9.0, vfov = 90, defocus = 0, focus = 10;
  int width = 400, height = 225;
  V3 lookfrom{0, 0, 0}, lookat{0, 0, -1}, vup{0, 1, 0};
  V3 center, p00, du, dv, u, v, w, disk_u, disk_v;

  void init() {  // Camera::Initialize
    height = int(width / aspect);
    height = height < 1 ? 1 : height;
    center = lookfrom;
    double theta = vfov * (kPi / 180.0);
    double h = std::tan(theta / 2);
    double vh = 2 * h * focus;
    double vw = vh * (double(width) / height);
    w = normalize(lookfrom - lookat);
    u = normalize(cross(vup, w));
    v = cross(w, u);
    V3 vu = vw * u;
    V3 vv = vh * (-v);
    du = vu / width;
    dv = vv / height;
    V3 ul = center - (focus * w) - vu / 2 - vv / 2;
    p00 = ul + 0.5 * (du + dv);
    double rad = focus * std::tan((defocus / 2) * (kPi / 180.0));
    disk_u = rad * u;
    disk_v = rad * v;
  }
  // GetRay: SampleSquare draws the y offset first (g++ evaluates Vec3's arguments right
  // to left, camera.h:202), then the optional thin-lens disk sample.
  void get_ray(int i, int j, Rng& g, V3& o, V3& d) const {
    double oy = g.next() - 0.5;
    double ox = g.next() - 0.5;
    V3 ps = p00 + ((i + ox) * du) + ((j + oy) * dv);
    if (defocus <= 0) o = center;
    else {
      V3 p = random_in_unit_disk(g);
      o = center + (p.x * disk_u) + (p.y * disk_v);
    }
    d = ps - o;
  }
};

inline V3 sky(V3 d) {  // wavefront.cc:33-38
  V3 ud = normalize(d);
  double t = 0.5 * (ud.y + 1.0);
  const V3 c = (1.0 - t) * v3(1.0, 1.0, 1.0) + t * v3(0.5, 0.7, 1.0);
  return g_perturb == 2 ? 1.02 * c : c;
}

// ---------------------------------------------------------------------------------------
// PixelState (pixel_state.h:13-72)
// ---------------------------------------------------------------------------------------
struct PixelState {
  double sum[3] = {0, 0, 0}, mean[3] = {0, 0, 0}, m2[3] = {0, 0, 0};
  int samples = 0;
  bool converged = false;
};
inline void record_sample(PixelState& ps, V3 L) {
  ps.samples++;
  for (int c = 0; c < 3; c++) {
    double x = L[c];
    double mu = ps.mean[c];
    double delta = x - mu;
    mu += delta / ps.samples;
    double delta2 = x - mu;
    ps.mean[c] = mu;
    ps.m2[c] += delta2 * delta;
  }
  ps.sum[0] += L.x, ps.sum[1] += L.y, ps.sum[2] += L.z;
}
inline bool is_converged(const PixelState& ps, double rel, int min_spp) {
  if (ps.samples < min_spp) return false;
  for (int c = 0; c < 3; c++) {
    double var = ps.samples > 1 ? ps.m2[c] / (ps.samples - 1) : 0.0;
    double mu = std::max(std::fabs(ps.mean[c]), 1e-3);
    double sigma = std::sqrt(var);
    double err = sigma / std::sqrt(ps.samples);
    if (err / mu > rel) return false;
  }
  return true;
}

struct Params {
  int spp = 4, max_depth = 10, adaptive = 1, min_spp = 16;
  double rel = (double)0.05f;  // wavefront.cc:42 kRelThresh is a float
  int rng_mode = 1;
  uint64_t seed = 1234;
  int x0 = 0, y0 = 0, w = 0, h = 0;  // tile (philox mode); mt mode renders the whole image
  int threads = 1;
  int mk_min_samples = 0;      // megakernel AdaptiveSampler (adaptive = 1)
  double mk_threshold = 0.0;
};

struct Stats {
  long long rays = 0, primaries = 0;
};

// One path segment's shading step (wavefront.cc:109-208).  Returns true if a child ray
// continues (o,d,thr,depth updated), false if the path terminated with radiance L.
struct PathState {
  V3 o, d, thr{1, 1, 1};
  int depth = 0;
};

bool shade(const Scene& S, const Params& P, PathState& ps, const Hit& rec, bool hit, Rng& g, V3& L) {
  g.open((uint32_t)ps.depth + 1u);  // philox stream of this segment (ignored by mt)
  L = {0, 0, 0};
  if (!hit || ps.depth >= P.max_depth) {
    L = L + ps.thr * sky(ps.d);
    return false;
  }
  const Material& m = S.mat[rec.mat];
  V3 em = mat_emitted(S, m, rec.u, rec.v, rec.p);
  if (!near_zero(em)) {
    L = L + ps.thr * em;
    return false;
  }
  V3 wo = -normalize(ps.d);
  V3 wi, f;
  float pdf = 0.0f;
  if (!mat_sample(S, m, rec, wo, wi, pdf, f, g)) return false;
  PathState c;
  c.o = rec.p, c.d = wi, c.depth = ps.depth + 1;
  if (mat_specular(m)) {
    c.thr = ps.thr * f;
  } else {
    if (pdf < 1e-6f) return false;
    float cos_theta = std::max(0.0f, static_cast<float>(dot(wi, rec.normal)));
    c.thr = ((ps.thr * f) * (double)cos_theta) / (double)pdf;
  }
  if (c.depth > 5) {
    double p = std::max({c.thr.x, c.thr.y, c.thr.z});
    p = std::clamp(p, 0.1, 0.95);
    if (g.next() > p) return false;
    c.thr = c.thr / p;
  }
  ps = c;
  return true;
}

// Faithful bounce-synchronous wavefront (wavefront.cc:40-226) — whole image.  In mt mode
// the draw order is exactly the reference's single-thread order; in philox mode it must
// give the same result as render_per_pixel (order independence check).
void render_wavefront(const Scene& S, const Camera& cam, const Params& P, double* fb, int* spp_out,
                      Stats& st, double* var_out) {
  const int W = cam.width, H = cam.height, N = W * H;
  std::mt19937 mt(P.seed);
  std::uniform_real_distribution<double> dist(0.0, 1.0);
  Rng g;
  g.mode = P.rng_mode, g.mt = &mt, g.dist = &dist, g.seed = P.seed;
  std::vector<PixelState> px(N);
  struct Q {
    PathState s;
    int pix;
  };
  std::vector<Q> q, nq;
  const int min_spp = P.adaptive ? P.min_spp : (1 << 30);
  auto finish = [&](PixelState& ps, V3 L) {
    record_sample(ps, L);
    if (!ps.converged && is_converged(ps, P.rel, min_spp)) ps.converged = true;
  };
  for (int s = 0; s < P.spp; s++) {
    q.clear();
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        int idx = y * W + x;
        if (px[idx].converged) continue;
        Q e;
        g.pixel = idx, g.sample = s, g.open(0);
        cam.get_ray(x, y, g, e.s.o, e.s.d);
        e.pix = idx;
        q.push_back(e);
      }
    st.primaries += (long long)q.size();
    while (!q.empty()) {
      st.rays += (long long)q.size();
      for (Q& e : q) {
        Hit rec;
        bool hit = S.hit(e.s.o, e.s.d, (double)0.001f, kInf, rec);
        g.pixel = e.pix, g.sample = s;
        V3 L;
        if (shade(S, P, e.s, rec, hit, g, L)) {
          nq.push_back(e);
        } else {
          finish(px[e.pix], L);
        }
      }
      q.swap(nq);
      nq.clear();
    }
  }
  for (int i = 0; i < N; i++) {
    double inv = px[i].samples > 0 ? 1.0 / (double)(float)px[i].samples : 0.0;
    for (int c = 0; c < 3; c++) fb[3 * (size_t)i + c] = px[i].samples > 0 ? inv * px[i].sum[c] : 0.0;
    if (spp_out) spp_out[i] = px[i].samples;
    if (var_out)
      for (int c = 0; c < 3; c++) var_out[3 * (size_t)i + c] = px[i].samples > 1 ? px[i].m2[c] / (px[i].samples - 1) : 0.0;
  }
}

// Philox mode, per pixel: sample s of pixel p is traced to termination before sample s+1,
// which is exactly the per-pixel order the wavefront produces (one path per pixel per
// pass, wavefront.cc:57-79).  Parallel over pixels (OpenMP), result independent of the
// thread count.
void render_per_pixel(const Scene& S, const Camera& cam, const Params& P, double* fb, int* spp_out,
                      Stats& st, double* var_out) {
  const int W = cam.width;
  const int tw = P.w, th = P.h;
  const int min_spp = P.adaptive ? P.min_spp : (1 << 30);
  long long rays = 0, prim = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(P.threads) reduction(+ : rays, prim)
  for (int ty = 0; ty < th; ty++) {
    for (int tx = 0; tx < tw; tx++) {
      int x = P.x0 + tx, y = P.y0 + ty;
      int idx = y * W + x;
      PixelState ps;
      Rng g;
      g.mode = 1, g.seed = P.seed, g.pixel = idx;
      for (int s = 0; s < P.spp && !ps.converged; s++) {
        g.sample = s, g.open(0);
        PathState path;
        cam.get_ray(x, y, g, path.o, path.d);
        prim++;
        while (true) {
          Hit rec;
          bool hit = S.hit(path.o, path.d, (double)0.001f, kInf, rec);
          rays++;
          V3 L;
          if (!shade(S, P, path, rec, hit, g, L)) {
            record_sample(ps, L);
            if (!ps.converged && is_converged(ps, P.rel, min_spp)) ps.converged = true;
            break;
          }
        }
      }
      size_t o = (size_t)ty * tw + tx;
      double inv = ps.samples > 0 ? 1.0 / (double)(float)ps.samples : 0.0;
      for (int c = 0; c < 3; c++) fb[3 * o + c] = ps.samples > 0 ? inv * ps.sum[c] : 0.0;
      if (spp_out) spp_out[o] = ps.samples;
      if (var_out)
        for (int c = 0; c < 3; c++) var_out[3 * o + c] = ps.samples > 1 ? ps.m2[c] / (ps.samples - 1) : 0.0;
    }
  }
  st.rays += rays;
  st.primaries += prim;
}

// Megakernel mode (mega_kernel.h:15-54, DefaultSampler sampler.h:22-34, GetPixel
// camera.h:148-174): recursive Scatter-API path, interval [0.001, inf) in double, black at
// depth 0, no RR.  mt mode runs pixels row-major on one thread.
V3 get_pixel(const Scene& S, V3 o, V3 d, int depth, int max_depth, Rng& g, long long& rays) {
  if (depth <= 0) return {0, 0, 0};
  g.open((uint32_t)(max_depth - depth) + 1u);  // philox stream of this segment
  Hit rec;
  rays++;
  if (S.hit(o, d, 0.001, kInf, rec)) {
    const Material& m = S.mat[rec.mat];
    V3 att, so, sd;
    V3 em = mat_emitted(S, m, rec.u, rec.v, rec.p);
    if (mat_scatter(S, m, d, rec, att, so, sd, g)) return em + att * get_pixel(S, so, sd, depth - 1, max_depth, g, rays);
    return em;
  }
  return sky(d);
}

inline double luminance(V3 c) {  // color.h:35-37 (float weights)
  return 0.2126f * c.x + 0.7152f * c.y + 0.0722f * c.z;
}

void render_megakernel(const Scene& S, const Camera& cam, const Params& P, double* fb, int* spp_out, Stats& st) {
  const int W = cam.width;
  const bool mt_mode = P.rng_mode == 0;
  std::mt19937 mt(P.seed);
  std::uniform_real_distribution<double> dist(0.0, 1.0);
  long long rays = 0;
  const int tw = mt_mode ? cam.width : P.w, th = mt_mode ? cam.height : P.h;
  const int x0 = mt_mode ? 0 : P.x0, y0 = mt_mode ? 0 : P.y0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(mt_mode ? 1 : P.threads) reduction(+ : rays)
  for (int ty = 0; ty < th; ty++)
    for (int tx = 0; tx < tw; tx++) {
      int x = x0 + tx, y = y0 + ty;
      Rng g;
      g.mode = P.rng_mode, g.mt = &mt, g.dist = &dist, g.seed = P.seed, g.pixel = y * W + x;
      V3 pixel{0, 0, 0};
      int samples = 0;
      if (!P.adaptive) {  // DefaultSampler::SamplePixel (sampler.h:22-34)
        for (int k = 0; k < P.spp; k++) {
          g.sample = k, g.open(0);
          V3 o, d;
          cam.get_ray(x, y, g, o, d);
          pixel = pixel + get_pixel(S, o, d, P.max_depth, P.max_depth, g, rays);
        }
        pixel = pixel / P.spp;
        samples = P.spp;
      } else {  // AdaptiveSampler::SamplePixel (sampler.h:44-82): `pixel` is the running sum
        V3 sum{0, 0, 0}, sum_sq{0, 0, 0};
        while (samples <= P.spp) {
          g.sample = samples, g.open(0);
          samples++;
          V3 o, d;
          cam.get_ray(x, y, g, o, d);
          pixel = pixel + get_pixel(S, o, d, P.max_depth, P.max_depth, g, rays);
          sum = sum + pixel;
          sum_sq = sum_sq + pixel * pixel;
          if (samples >= P.mk_min_samples) {
            V3 mean = sum / samples;
            double mean_luminance = luminance(mean);
            V3 variance = (sum_sq / samples) - (mean * mean);
            double error = std::sqrt(luminance(variance) / samples);
            if ((error / (mean_luminance + 1e-3f)) < P.mk_threshold) break;
          }
        }
        pixel = pixel / samples;
      }
      size_t oi = (size_t)ty * tw + tx;
      fb[3 * oi] = pixel.x, fb[3 * oi + 1] = pixel.y, fb[3 * oi + 2] = pixel.z;
      if (spp_out) spp_out[oi] = samples;
    }
  st.rays += rays;
}

// ---------------------------------------------------------------------------------------
// Scene file (.rtxs) loader — independent of the product's loader.
// ---------------------------------------------------------------------------------------
bool load_ppm(const std::string& path, Image& img) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return false;
  std::string magic;
  int maxv;
  in >> magic >> img.w >> img.h >> maxv;
  in.get();
  if (magic != "P6" || maxv != 255) return false;
  img.bytes.resize((size_t)img.w * img.h * 3);
  in.read((char*)img.bytes.data(), (std::streamsize)img.bytes.size());
  return (bool)in;
}

// OBJ (load_obj.h:10-55 semantics; coordinates parsed as float like tinyobjloader).
bool load_obj(const std::string& path, double scale, int mat, std::vector<Prim>& out) {
  std::ifstream in(path);
  if (!in) return false;
  std::vector<V3> v;
  std::vector<std::array<int, 3>> f;
  std::string line;
  while (std::getline(in, line)) {
    if (line.size() > 2 && line[0] == 'v' && line[1] == ' ') {
      char* e;
      float x = std::strtof(line.c_str() + 2, &e);
      float y = std::strtof(e, &e);
      float z = std::strtof(e, &e);
      v.push_back({x, y, z});
    } else if (line.size() > 2 && line[0] == 'f' && line[1] == ' ') {
      std::istringstream ss(line.substr(2));
      std::vector<int> ix;
      std::string tok;
      while (ss >> tok) ix.push_back(std::atoi(tok.c_str()) - 1);
      if (ix.size() == 3) f.push_back({ix[0], ix[1], ix[2]});
    }
  }
  V3 c{0.0f, 0.0f, 0.0f};
  for (V3 p : v) c = c + p;
  c = c / (double)v.size();
  for (V3& p : v) {
    p = p - c;
    p = scale * p;
  }
  for (auto& t : f) {
    Prim P{};
    P.kind = PRIM_TRI, P.mat = mat;
    V3 a = v[t[0]], b = v[t[1]], cc = v[t[2]];
    double g[9] = {a.x, a.y, a.z, b.x, b.y, b.z, cc.x, cc.y, cc.z};
    std::memcpy(P.g, g, sizeof g);
    P.bbox = prim_bbox(P);
    out.push_back(P);
  }
  return true;
}

std::vector<std::string> split_dirs(const char* list) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* c = list; *c; c++) {
    if (*c == ':') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += *c;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

Scene* load_scene(const char* file, const char* asset_dir, std::string& err) {
  std::ifstream in(file);
  if (!in) {
    err = std::string("cannot open ") + file;
    return nullptr;
  }
  auto S = std::make_unique<Scene>();
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string kw;
    ss >> kw;
    if (kw == "bvh") {
      int b;
      ss >> b;
      S->use_bvh = b != 0;
    } else if (kw == "tex") {
      int id;
      std::string kind;
      ss >> id >> kind;
      Texture T;
      if (kind == "solid") {
        T.kind = TEX_SOLID;
        ss >> T.color.x >> T.color.y >> T.color.z;
      } else if (kind == "checker") {
        double sc;
        T.kind = TEX_CHECKER;
        ss >> sc >> T.even >> T.odd;
        T.inv_scale = 1.0 / sc;
      } else {
        std::string name;
        ss >> name;
        T.kind = TEX_IMAGE;
        T.img = std::make_shared<Image>();
        // texels of the reference's decode (the fixture tests/golden/textures/<name>.ppm):
        // asset_dir may list several directories separated by ':'
        bool ok = false;
        for (const std::string& dir : split_dirs(asset_dir))
          if ((ok = load_ppm(dir + "/" + name + ".ppm", *T.img))) break;
        if (!ok) T.img->w = T.img->h = 0;
      }
      S->tex.push_back(T);
    } else if (kw == "mat") {
      int id;
      std::string kind;
      ss >> id >> kind;
      Material M;
      if (kind == "lambertian") M.kind = MAT_LAMBERT, ss >> M.tex;
      else if (kind == "metal") {
        M.kind = MAT_METAL;
        double fz;
        ss >> M.albedo.x >> M.albedo.y >> M.albedo.z >> fz;
        M.fuzz = fz < 1.0 ? fz : 1.0;
      } else if (kind == "dielectric") M.kind = MAT_DIELECTRIC, ss >> M.ri;
      else M.kind = MAT_LIGHT, ss >> M.tex;
      S->mat.push_back(M);
    } else if (kw == "sphere" || kw == "tri" || kw == "rect") {
      Prim P{};
      int n = 4;
      if (kw == "sphere") P.kind = PRIM_SPHERE;
      else if (kw == "tri") P.kind = PRIM_TRI, n = 9;
      else {
        std::string ax;
        ss >> ax;
        P.kind = ax == "xy" ? PRIM_XY : (ax == "xz" ? PRIM_XZ : PRIM_YZ);
        n = 5;
      }
      for (int i = 0; i < n; i++) ss >> P.g[i];
      ss >> P.mat;
      P.bbox = prim_bbox(P);
      S->prims.push_back(P);
    } else if (kw == "obj") {
      std::string name;
      double sc;
      int m;
      ss >> name >> sc >> m;
      bool ok = false;
      for (const std::string& dir : split_dirs(asset_dir))
        if ((ok = load_obj(dir + "/" + name, sc, m, S->prims))) break;
      if (!ok) {
        err = "cannot open obj " + name;
        return nullptr;
      }
    }
  }
  if (S->use_bvh) S->bvh.build(S->prims);
  return S.release();
}

}  // namespace orc

// =======================================================================================
// C ABI for the Python tests (ctypes).  Test infrastructure only.
// =======================================================================================
using namespace orc;

extern "C" {

struct orc_camera {
  double aspect, vfov, lookfrom[3], lookat[3], vup[3], defocus, focus;
  int width;
  int height;  // out
};

struct orc_params {
  int spp, max_depth, adaptive, rng_mode;  // rng_mode 0 = mt, 1 = philox
  unsigned long long seed;
  int x0, y0, w, h;  // tile (philox per-pixel / megakernel-philox)
  int threads;
  int mode;  // 0 = wavefront (queue order), 1 = per-pixel (philox), 2 = megakernel
  // megakernel + adaptive: AdaptiveSampler(min_samples, max_samples = spp, threshold)
  int mk_min_samples;
  double mk_threshold;  // the float threshold, widened
};

static thread_local std::string g_err;
const char* orc_last_error(void) { return g_err.c_str(); }

void* orc_scene_load(const char* file, const char* asset_dir) {
  Scene* s = load_scene(file, asset_dir, g_err);
  return s;
}
void orc_scene_free(void* s) { delete (Scene*)s; }
// the power check's deliberate estimator change (g_perturb); returns the previous setting
int orc_set_perturb(int mode) {
  const int old = g_perturb;
  g_perturb = mode;
  return old;
}
int orc_scene_counts(void* sp, int* nprims, int* nnodes, int* nmats, int* ntex) {
  Scene* s = (Scene*)sp;
  *nprims = (int)s->prims.size();
  *nnodes = (int)s->bvh.nodes.size();
  *nmats = (int)s->mat.size();
  *ntex = (int)s->tex.size();
  return 0;
}
// boxes: n*6 (xmin xmax ymin ymax zmin zmax), links: n*3, prims: nprims
int orc_scene_bvh(void* sp, double* boxes, unsigned* links, int* prim_idx) {
  Scene* s = (Scene*)sp;
  for (size_t i = 0; i < s->bvh.nodes.size(); i++) {
    const Node& n = s->bvh.nodes[i];
    for (int a = 0; a < 3; a++) boxes[6 * i + 2 * a] = n.bbox.lo[a], boxes[6 * i + 2 * a + 1] = n.bbox.hi[a];
    links[3 * i] = n.a, links[3 * i + 1] = n.b, links[3 * i + 2] = n.leaf;
  }
  for (size_t i = 0; i < s->bvh.idx.size(); i++) prim_idx[i] = s->bvh.idx[i];
  return 0;
}
// out: 12 doubles per ray (hit t p3 n3 u v front mat).  tmin < 0 -> seam interval 0.001f.
int orc_intersect(void* sp, const double* rays, long long n, double tmin, double* out, int threads) {
  Scene* s = (Scene*)sp;
  double tm = tmin < 0 ? (double)0.001f : tmin;
#pragma omp parallel for num_threads(threads > 0 ? threads : 1)
  for (long long i = 0; i < n; i++) {
    V3 o{rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]}, d{rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]};
    Hit rec;
    bool ok = s->hit(o, d, tm, kInf, rec);
    double* q = out + 12 * i;
    std::memset(q, 0, 12 * sizeof(double));
    q[0] = ok;
    if (ok) {
      q[1] = rec.t, q[2] = rec.p.x, q[3] = rec.p.y, q[4] = rec.p.z;
      q[5] = rec.normal.x, q[6] = rec.normal.y, q[7] = rec.normal.z;
      q[8] = rec.u, q[9] = rec.v, q[10] = rec.front_face, q[11] = rec.mat;
    }
  }
  return 0;
}
// Every primitive whose own closest hit on the ray (hit_prim on (tmin, inf): the near root
// first, as Scene::Hit would report it) lies at exactly distance t: up to `cap` records of
// 12 doubles (the orc_intersect layout), brute force over the whole primitive list.  Returns
// how many there are.  Test hook: a fast-precision closest hit that differs from the
// parity one must be an exact t tie between distinct primitives (tests/test_gpu_parity.py).
int orc_tied_hits(void* sp, const double* ray, double tmin, double t, double* out, int cap) {
  Scene* s = (Scene*)sp;
  double tm = tmin < 0 ? (double)0.001f : tmin;
  V3 o{ray[0], ray[1], ray[2]}, d{ray[3], ray[4], ray[5]};
  int n = 0;
  for (const Prim& p : s->prims) {
    Hit rec;
    if (!hit_prim(p, o, d, tm, kInf, rec) || rec.t != t) continue;
    if (n < cap) {
      double* q = out + 12 * n;
      q[0] = 1, q[1] = rec.t, q[2] = rec.p.x, q[3] = rec.p.y, q[4] = rec.p.z;
      q[5] = rec.normal.x, q[6] = rec.normal.y, q[7] = rec.normal.z;
      q[8] = rec.u, q[9] = rec.v, q[10] = rec.front_face, q[11] = rec.mat;
    }
    n++;
  }
  return n;
}
int orc_aabb(const double* cases, long long n, int* out) {
  for (long long i = 0; i < n; i++) {
    const double* q = cases + 14 * i;
    Box b;
    for (int a = 0; a < 3; a++) b.lo[a] = q[2 * a], b.hi[a] = q[2 * a + 1];
    out[i] = box_hit(b, v3(q[6], q[7], q[8]), v3(q[9], q[10], q[11]), q[12], q[13]);
  }
  return 0;
}
// Same case/out layout as ref_harness "material"/"scatter"; rng: mt seeded per case.
int orc_material(const double* cases, long long n, double* out, int scatter) {
  Scene S;
  S.tex.resize(1);
  for (long long i = 0; i < n; i++) {
    const double* q = cases + 20 * i;
    Material m;
    int kind = (int)q[0];
    S.tex[0].kind = TEX_SOLID, S.tex[0].color = v3(q[1], q[2], q[3]);
    m.kind = kind, m.tex = 0;
    if (kind == MAT_METAL) m.albedo = v3(q[1], q[2], q[3]), m.fuzz = q[4] < 1.0 ? q[4] : 1.0;
    if (kind == MAT_DIELECTRIC) m.ri = q[1];
    Hit rec;
    rec.normal = v3(q[5], q[6], q[7]), rec.front_face = q[8] != 0, rec.u = q[9], rec.v = q[10];
    rec.p = v3(q[11], q[12], q[13]), rec.hit = true;
    V3 wo{q[14], q[15], q[16]};
    std::mt19937 mt((unsigned)q[17]);
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    Rng g;
    g.mode = 0, g.mt = &mt, g.dist = &dist;
    double* o = out + 12 * i;
    std::memset(o, 0, 12 * sizeof(double));
    if (!scatter) {
      V3 wi{0, 0, 0}, f{0, 0, 0};
      float pdf = -1.0f;
      bool ok = mat_sample(S, m, rec, wo, wi, pdf, f, g);
      o[0] = ok, o[1] = wi.x, o[2] = wi.y, o[3] = wi.z, o[4] = pdf, o[5] = f.x, o[6] = f.y, o[7] = f.z;
      o[9] = mat_specular(m);
      o[10] = mat_emitted(S, m, rec.u, rec.v, rec.p).x;
    } else {
      V3 att{0, 0, 0}, so{0, 0, 0}, sd{0, 0, 0};
      bool ok = mat_scatter(S, m, wo, rec, att, so, sd, g);
      o[0] = ok, o[1] = sd.x, o[2] = sd.y, o[3] = sd.z, o[5] = att.x, o[6] = att.y, o[7] = att.z;
      o[10] = so.x, o[11] = so.y;
    }
    o[8] = g.next();
  }
  return 0;
}
// texture cases (8 doubles): kind(0 checker, 1 image, 2 missing image) scale u v p3 spare
int orc_texture(const double* cases, long long n, const char* texel_ppm, double* out) {
  Scene S;
  S.tex.resize(5);
  S.tex[0].color = v3(0.2, 0.3, 0.1), S.tex[1].color = v3(.9, .9, .9);
  S.tex[2].kind = TEX_CHECKER, S.tex[2].even = 0, S.tex[2].odd = 1;
  S.tex[3].kind = TEX_IMAGE, S.tex[3].img = std::make_shared<Image>();
  if (!load_ppm(texel_ppm, *S.tex[3].img)) {
    g_err = "cannot load texels";
    return -1;
  }
  S.tex[4].kind = TEX_IMAGE, S.tex[4].img = std::make_shared<Image>();
  for (long long i = 0; i < n; i++) {
    const double* q = cases + 8 * i;
    int t = q[0] == 0 ? 2 : (q[0] == 1 ? 3 : 4);
    S.tex[2].inv_scale = 1.0 / q[1];
    V3 v = tex_value(S, t, q[2], q[3], v3(q[4], q[5], q[6]));
    out[3 * i] = v.x, out[3 * i + 1] = v.y, out[3 * i + 2] = v.z;
  }
  return 0;
}
int orc_pixelstate(const double* in, long long nin, double* out) {
  long long k = 0, o = 0;
  while (k < nin) {
    int n = (int)in[k++];
    PixelState ps;
    for (int i = 0; i < n; i++, k += 3) {
      record_sample(ps, v3(in[k], in[k + 1], in[k + 2]));
      bool conv = is_converged(ps, (double)0.05f, 16);
      double r[10] = {ps.mean[0], ps.mean[1], ps.mean[2], ps.m2[0], ps.m2[1],
                      ps.m2[2],   ps.sum[0],  ps.sum[1],  ps.sum[2], (double)conv};
      std::memcpy(out + o, r, sizeof r);
      o += 10;
    }
  }
  return 0;
}
int orc_camera_init(orc_camera* c, double* basis /* 21: center p00 du dv u v w */) {
  Camera cam;
  cam.aspect = c->aspect, cam.vfov = c->vfov, cam.defocus = c->defocus, cam.focus = c->focus;
  cam.width = c->width;
  cam.lookfrom = v3(c->lookfrom[0], c->lookfrom[1], c->lookfrom[2]);
  cam.lookat = v3(c->lookat[0], c->lookat[1], c->lookat[2]);
  cam.vup = v3(c->vup[0], c->vup[1], c->vup[2]);
  cam.init();
  c->height = cam.height;
  V3 vs[7] = {cam.center, cam.p00, cam.du, cam.dv, cam.u, cam.v, cam.w};
  for (int i = 0; i < 7; i++) basis[3 * i] = vs[i].x, basis[3 * i + 1] = vs[i].y, basis[3 * i + 2] = vs[i].z;
  return 0;
}
// fb: tile w*h*3 doubles (whole image in wavefront mode), spp: tile w*h ints (may be NULL)
// stats: [rays, primaries]
// orc_render_var: orc_render plus each pixel's sample variance m2/(n-1) per channel
// (pixel_state.h:41-49) in var[3 * pixel] (wavefront and per-pixel modes), for the
// statistical parity test against the reference as it runs (tests/test_statistical_parity.py)
int orc_render_var(void* sp, orc_camera* c, const orc_params* p, double* fb, int* spp, long long* stats,
                   double* var) {
  Scene* s = (Scene*)sp;
  Camera cam;
  cam.aspect = c->aspect, cam.vfov = c->vfov, cam.defocus = c->defocus, cam.focus = c->focus;
  cam.width = c->width;
  cam.lookfrom = v3(c->lookfrom[0], c->lookfrom[1], c->lookfrom[2]);
  cam.lookat = v3(c->lookat[0], c->lookat[1], c->lookat[2]);
  cam.vup = v3(c->vup[0], c->vup[1], c->vup[2]);
  cam.init();
  c->height = cam.height;
  Params P;
  P.spp = p->spp, P.max_depth = p->max_depth, P.adaptive = p->adaptive, P.rng_mode = p->rng_mode;
  P.seed = p->seed, P.threads = p->threads > 0 ? p->threads : 1;
  P.x0 = p->x0, P.y0 = p->y0, P.w = p->w > 0 ? p->w : cam.width, P.h = p->h > 0 ? p->h : cam.height;
  if (P.x0 < 0 || P.y0 < 0 || P.x0 + P.w > cam.width || P.y0 + P.h > cam.height) {
    g_err = "tile outside image";
    return -1;
  }
  Stats st;
  if (p->mode == 0) render_wavefront(*s, cam, P, fb, spp, st, var);
  else if (p->mode == 1) {
    if (P.rng_mode != 1) {
      g_err = "per-pixel mode needs philox";
      return -1;
    }
    render_per_pixel(*s, cam, P, fb, spp, st, var);
  } else {
    P.mk_min_samples = p->mk_min_samples, P.mk_threshold = p->mk_threshold;
    render_megakernel(*s, cam, P, fb, spp, st);
  }
  stats[0] = st.rays, stats[1] = st.primaries;
  return 0;
}
int orc_render(void* sp, orc_camera* c, const orc_params* p, double* fb, int* spp, long long* stats) {
  return orc_render_var(sp, c, p, fb, spp, stats, nullptr);
}
// Every sample of every pixel of the tile at fixed spp, philox per-pixel order: radiance in
// L[3 * (pixel * spp + s)], path segments in segs[pixel * spp + s].  Input of the adaptive
// schedule simulator (scripts/adaptive_sim.py), which replays RecordSample / IsConverged and the
// phase policy over these samples without a GPU.
int orc_render_samples(void* sp, orc_camera* c, const orc_params* p, double* L, unsigned short* segs) {
  Scene* s = (Scene*)sp;
  Camera cam;
  cam.aspect = c->aspect, cam.vfov = c->vfov, cam.defocus = c->defocus, cam.focus = c->focus;
  cam.width = c->width;
  cam.lookfrom = v3(c->lookfrom[0], c->lookfrom[1], c->lookfrom[2]);
  cam.lookat = v3(c->lookat[0], c->lookat[1], c->lookat[2]);
  cam.vup = v3(c->vup[0], c->vup[1], c->vup[2]);
  cam.init();
  c->height = cam.height;
  Params P;
  P.spp = p->spp, P.max_depth = p->max_depth, P.adaptive = 0, P.rng_mode = 1;
  P.seed = p->seed, P.threads = p->threads > 0 ? p->threads : 1;
  P.x0 = p->x0, P.y0 = p->y0, P.w = p->w > 0 ? p->w : cam.width, P.h = p->h > 0 ? p->h : cam.height;
  if (P.x0 < 0 || P.y0 < 0 || P.x0 + P.w > cam.width || P.y0 + P.h > cam.height) {
    g_err = "tile outside image";
    return -1;
  }
  const Scene& S = *s;
#pragma omp parallel for schedule(dynamic, 1) num_threads(P.threads)
  for (int ty = 0; ty < P.h; ty++) {
    for (int tx = 0; tx < P.w; tx++) {
      const int x = P.x0 + tx, y = P.y0 + ty;
      const size_t o = (size_t)ty * P.w + tx;
      Rng g;
      g.mode = 1, g.seed = P.seed, g.pixel = y * cam.width + x;
      for (int smp = 0; smp < P.spp; smp++) {
        g.sample = smp, g.open(0);
        PathState path;
        cam.get_ray(x, y, g, path.o, path.d);
        unsigned n = 0;
        while (true) {
          Hit rec;
          bool hit = S.hit(path.o, path.d, (double)0.001f, kInf, rec);
          n++;
          V3 Lr;
          if (!shade(S, P, path, rec, hit, g, Lr)) {
            const size_t k = o * P.spp + smp;
            L[3 * k] = Lr.x, L[3 * k + 1] = Lr.y, L[3 * k + 2] = Lr.z;
            segs[k] = (unsigned short)(n > 65535 ? 65535 : n);
            break;
          }
        }
      }
    }
  }
  return 0;
}
// Philox stream check for the GPU RNG: out[i] = RandomDouble for (seed, pixel, sample,
// stream, draw = i)
int orc_philox_stream(unsigned long long seed, unsigned pixel, unsigned sample, unsigned stream, int n,
                      double* out) {
  Rng g;
  g.mode = 1, g.seed = seed, g.pixel = pixel, g.sample = sample;
  g.open(stream);
  for (int i = 0; i < n; i++) out[i] = g.next();
  return 0;
}
int orc_philox(unsigned long long seed, unsigned pixel, unsigned sample, int n, double* out) {
  return orc_philox_stream(seed, pixel, sample, 0u, n, out);
}
// P3 PPM bytes of a linear framebuffer via write_color (color.h:18-33)
int orc_write_ppm(const double* fb, int w, int h, const char* path) {
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  std::fprintf(f, "P3\n%d %d\n255\n", w, h);
  for (long long i = 0; i < (long long)w * h; i++) {
    int b[3];
    for (int c = 0; c < 3; c++) {
      double x = fb[3 * i + c];
      x = x > 0 ? std::sqrt(x) : 0;
      x = x < 0.000 ? 0.000 : (x > 0.999 ? 0.999 : x);
      b[c] = int(256 * x);
    }
    std::fprintf(f, "%d %d %d\n", b[0], b[1], b[2]);
  }
  std::fclose(f);
  return 0;
}

}  // extern "C"
