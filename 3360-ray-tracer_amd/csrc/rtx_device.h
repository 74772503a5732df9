// rtx_device.h — device-side building blocks of the MI355X path tracer (gfx950, wave64).
//
// Every function restates a reference routine (file:line under the reference's src/) in
// the same IEEE double operation order, with the reference's float islands.  This file is
// compiled with -ffp-contract=off: no FMA contraction anywhere in the f64 path, so parity
// mode reproduces the CPU restatement (oracle/rtx_oracle.cc) bit for bit except where the
// device libm (ocml cos/sin/acos/atan2/pow) differs from glibc in the last ulp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rtx.h"

// Per-translation-unit choices.  rtx_park.hip, which compiles the PARK instantiations of
// k_persistent and nothing else, defines RTX_PARK_TU 1 before including this file; every
// other translation unit (rtx_capi.hip: the plain kernel, the frame kernels) takes the plain
// kernel's choices.  Each was picked by A/B on the scenes that run that TU's kernels (DESIGN.md
// ledger); register allocation decides which is best per kernel.  k_persistent asserts that
// its PARK instantiations come from the PARK TU only.
#ifndef RTX_PARK_TU
#define RTX_PARK_TU 0
#endif

namespace rtxd {

// Lambertian cos/sin: the restated small-argument forms (plain TU; with them the bunny's PARK
// build spills, 0 -> 56 B per lane), else the library's cos() / sin()
constexpr bool kSincosSmall = !RTX_PARK_TU;
// kind-specialised walks: the triangle test without early exits (PARK TU: bunny +3.8 %; the
// plain kernel's builds are slower with it)
constexpr bool kTriBranchless = RTX_PARK_TU;
// textured builds: a Lambertian's albedo texture looked up before the sampling (plain TU; the
// early lookup makes the generic PARK build spill more, 80 -> 128 B per lane)
constexpr bool kEarlyTex = !RTX_PARK_TU;
// lean walk: at most one leaf test per lane and loop iteration (trace4_run_step; PARK TU: bunny
// +2.8 %; the plain kernel's sphere-tree builds are slower with it)
constexpr bool kLeafStep = RTX_PARK_TU;

constexpr double kPi = 3.14159265358979323846;
constexpr double kInf = __builtin_inf();

// ---------------------------------------------------------------------------------------
// Vec3 (vec3.h:8-107): a/t == (1/t)*a, left-to-right sums.
// ---------------------------------------------------------------------------------------
struct V3 {
  double x, y, z;
};
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 operator*(double t, V3 a) { return {t * a.x, t * a.y, t * a.z}; }
__device__ __forceinline__ V3 operator/(V3 a, double t) { return (1.0 / t) * a; }
__device__ __forceinline__ double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ V3 cross(V3 u, V3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
__device__ __forceinline__ bool near_zero(V3 a) {  // vec3.h:50-55
  return fabs(a.x) < 1e-8 && fabs(a.y) < 1e-8 && fabs(a.z) < 1e-8;
}
__device__ __forceinline__ V3 normalize(V3 v) {  // math_utils.h:93-97
  double l = sqrt(len2(v));
  if (l == 0.0) return {0, 0, 0};
  return v / l;
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return v - (2.0 * dot(v, n)) * n; }  // :14-16
__device__ __forceinline__ V3 refract(V3 uv, V3 n, double eta) {                           // :24-29
  double c = fmin(dot(-uv, n), 1.0);
  V3 perp = eta * (uv + c * n);
  V3 par = (-sqrt(fabs(1.0 - len2(perp)))) * n;
  return perp + par;
}

// ---------------------------------------------------------------------------------------
// Counter-based RNG: Philox-4x32-10, key (seed_lo, seed_hi ^ 0x52545831), counter
// (draw >> 1, sample, global pixel, stream).  Stream 0 is the camera ray (GetRay); the
// shading of path segment n (n = 0 for the primary hit) is stream n + 1, and `draw`
// restarts at 0 in every stream.  Draw 2k of a stream is words 0/1 of block k, draw 2k+1
// words 2/3, as a 53-bit double.  Bit-identical to oracle/rtx_oracle.cc Rng::next (philox
// mode).  A path's numbers depend only on (seed, pixel, sample, segment, draw): results
// are independent of tiling, GPU count, queue order and scheduling.
//
// Because every stream starts block-aligned, the first block of a stream is computed once
// in converged control flow (make_rng) and serves the first two draws of every material
// branch; a later block is computed where the wave first needs it, with per-lane counters,
// so lanes at different draw positions still share one Philox evaluation.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void philox_block(uint32_t blk, uint32_t sample, uint32_t pixel, uint32_t stream,
                                             uint32_t k0, uint32_t k1, double& u0, double& u1) {
  uint32_t c0 = blk, c1 = sample, c2 = pixel, c3 = stream;
  uint32_t a = k0, b = k1;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    // one v_mad_u64_u32 per product instead of v_mul_lo_u32 + v_mul_hi_u32
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    uint32_t n0 = hi1 ^ c1 ^ a;
    uint32_t n2 = hi0 ^ c3 ^ b;
    c0 = n0, c1 = lo1, c2 = n2, c3 = lo0;
    a += 0x9E3779B9u;
    b += 0xBB67AE85u;
  }
  u0 = (double)((((uint64_t)c1 << 32) | c0) >> 11) * 0x1p-53;
  u1 = (double)((((uint64_t)c3 << 32) | c2) >> 11) * 0x1p-53;
}

struct Rng {
  uint32_t k0, k1, pixel, sample, stream, draw;
  uint32_t cblk;   // block held in (ca, cb)
  double ca, cb;   // draws 2*cblk, 2*cblk + 1
  __device__ __forceinline__ double next() {
    const uint32_t blk = draw >> 1;
    if (blk != cblk) {
      philox_block(blk, sample, pixel, stream, k0, k1, ca, cb);
      cblk = blk;
    }
    const double r = (draw & 1) ? cb : ca;
    draw++;
    return r;
  }
  __device__ __forceinline__ double next(double mn, double mx) { return mn + (mx - mn) * next(); }
};
// Opens `stream` of (pixel, sample) at draw 0 with its first block already computed.
__device__ __forceinline__ Rng make_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t stream) {
  Rng g;
  g.k0 = (uint32_t)seed;
  g.k1 = (uint32_t)(seed >> 32) ^ 0x52545831u;
  g.pixel = pixel, g.sample = sample, g.stream = stream, g.draw = 0;
  philox_block(0u, sample, pixel, stream, g.k0, g.k1, g.ca, g.cb);
  g.cblk = 0;
  return g;
}

// RandomUnitVector (math_utils.h:62-70): draws z, y, x (g++ right-to-left argument order).
__device__ __forceinline__ V3 random_unit_vector(Rng& g) {
  while (true) {
    double z = g.next(-1.0, 1.0);
    double y = g.next(-1.0, 1.0);
    double x = g.next(-1.0, 1.0);
    V3 p{x, y, z};
    double l2 = len2(p);
    if (l2 > 1e-12 && l2 <= 1.0) return p / sqrt(l2);
  }
}
__device__ __forceinline__ V3 random_in_unit_disk(Rng& g) {  // math_utils.h:83-88
  while (true) {
    double y = g.next(-1, 1);
    double x = g.next(-1, 1);
    V3 p{x, y, 0.0};
    if (len2(p) < 1.0) return p;
  }
}
// cos(phi) and sin(phi) for 0 <= phi < 2^30 with ONE shared argument reduction, bit for bit
// what the device library's cos() and sin() return there: the same operations as its
// small-argument reduction (x * 2/pi rounded to an integer quadrant, pi/2 in three parts
// with exact error terms) and its sincos kernel polynomials, then the quadrant selection and
// sign rules of cos() / sin().  The library's large-argument (Payne-Hanek) path, which the
// Lambertian angle 2*pi*r1 < 2*pi never takes, is not compiled in: its registers made the
// shading spill.  -ffp-contract=off keeps every product and sum separately rounded, as in
// the library; fma() is the library's fma.
//   kSincosSmall: cos and sin each from its own small-argument reduction (fewest live
//   registers: the plain kernel's texture-free builds lose their last spills, A/B r02
//   `ab_sincos2_*`; one shared reduction spilled more); else the library's cos() and sin().
__device__ __forceinline__ void sincos_small(double x, double& sn, double& cs) {
  // reduction: x = q * pi/2 + (hi + lo)
  const double q = rint(x * 0x1.45f306dc9c883p-1);
  const double c1 = 0x1.1a62633145c00p-54;
  const double t4 = fma(q, -0x1.921fb54442d18p+0, x);
  const double t5 = fma(q, -c1, t4);
  const double t6 = q * c1;
  const double t8 = fma(q, c1, -t6);
  const double t9 = t4 - t6;
  const double t11 = (t4 - t9) - t6;
  const double t14 = ((t9 - t5) + t11) - t8;
  const double t15 = fma(q, -0x1.b839a252049c0p-104, t14);
  const double hi = t5 + t15;
  const double lo = t15 - (hi - t5);
  const int quad = (int)q & 3;
  // kernel on [-pi/4, pi/4]
  const double x2 = hi * hi;
  const double h = x2 * 0.5;
  const double w = 1.0 - h;
  const double e = (1.0 - w) - h;
  const double x4 = x2 * x2;
  double pc = fma(x2, -0x1.907db46cc5e42p-37, 0x1.1eeb69037ab78p-29);
  pc = fma(x2, pc, -0x1.27e4fa17f65f6p-22);
  pc = fma(x2, pc, 0x1.a01a019f4ec90p-16);
  pc = fma(x2, pc, -0x1.6c16c16c16967p-10);
  pc = fma(x2, pc, 0x1.5555555555555p-5);
  const double kc = w + fma(x4, pc, fma(hi, -lo, e));
  double ps = fma(x2, 0x1.5e0b2f9a43bb8p-33, -0x1.ae600b42fdfa7p-26);
  ps = fma(x2, ps, 0x1.71de3796cde01p-19);
  ps = fma(x2, ps, -0x1.a01a019e83e5cp-13);
  ps = fma(x2, ps, 0x1.1111111110bb3p-7);
  const double hx3 = hi * -x2;
  const double ks = hi - fma(hx3, -0x1.5555555555555p-3, fma(x2, fma(hx3, ps, lo * 0.5), -lo));
  // quadrant: cos = (c, -s, -c, s), sin = (s, c, -s, -c) (x >= +0: no sign from x)
  const double c0 = (quad & 1) == 0 ? kc : -ks;
  const double s0 = (quad & 1) == 0 ? ks : kc;
  cs = quad > 1 ? -c0 : c0;
  sn = quad > 1 ? -s0 : s0;
}
template <bool SMALL = kSincosSmall>
__device__ __forceinline__ void cos_sin(double phi, double& c, double& s) {
  if constexpr (SMALL) {
    double t;
    sincos_small(phi, t, c);
    asm volatile("" : "+v"(c));
    asm volatile("" : "+v"(phi));
    sincos_small(phi, s, t);
  } else {
    c = cos(phi), s = sin(phi);
  }
}

// ---------------------------------------------------------------------------------------
// Device scene (uploaded once per device by rtx_scene_create)
// ---------------------------------------------------------------------------------------
struct DImage {
  int32_t w, h;
  const uint8_t* texels;
};

// 4-wide fast node (RTX_PREC_FAST): a binary SAH tree collapsed so every node holds up to four
// children's outward-rounded f32 boxes (SoA for the four slab tests; build_fast4).  Every leaf
// slot holds exactly one primitive: child >= 0: node index; child < 0: leaf, ~child = the
// primitive; counts[]: 1 for a leaf slot (read by no kernel: the lean walk relies on the
// one-primitive layout); an empty slot is an inverted box (lo = +inf, hi = -inf, child -1) that
// no ray enters.  128 bytes = two cache lines.
struct F4Node {
  float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4];  // axis a: lo at 32a, hi at 32a + 16 bytes
  int32_t child[4];
  uint32_t counts[2];
  uint32_t pad_[2];
};
static_assert(sizeof(F4Node) == 128, "F4Node must be two 64-byte lines");

typedef F4Node FastNode;

struct DScene {
  const rtx_bvh_node* nodes;  // parity layout, reference pre-order
  const rtx_prim* prims;      // leaf order
  const rtx_material* mats;
  const rtx_texture* texs;
  const DImage* images;
  const FastNode* f4nodes;  // 4-wide fast layout (root at 0) or nullptr
  int64_t n_prims;
  int32_t use_bvh;
  int32_t froot_leaf;  // fast BVH: the whole tree is one leaf (count in froot_count)
  int32_t froot_count;
  int32_t has_tris;  // any triangle: prim_t preloads all 80 record bytes, else the first 48
  int32_t tree_kind;  // fast BVH: the one kind of every primitive in the tree, or -1
  int32_t all_lambertian;  // every material is a Lambertian
  int32_t no_textures;     // no material reads the texture table (solid colours resolved at upload)
  int32_t n_global;   // fast BVH: primitives kept out of the tree, tested before every walk
  int32_t global[2];  // their indices into prims (see build_global_prims, rtx_capi.hip)
  const double* tri_n;  // per primitive (x, y, z, 0), a triangle's unit normal (nullptr: no triangles)
};

struct Hit {  // HitRecord (hittable.h:18-42)
  V3 p, normal;
  double t, u, v;
  int32_t mat;
  int32_t front_face;
  // Sphere u,v (acos/atan2, sphere.h:73-79) and rect u,v (rect.h) are only ever read by image
  // textures, so the shading path defers them: lazy_uv >= 0 names the primitive whose u,v
  // are still to be derived from p (same arithmetic as at hit time, hence the same values).
  int64_t lazy_uv;
};

__device__ __forceinline__ void set_face_normal(Hit& h, V3 d, V3 outward) {  // hittable.h:31-34
  h.front_face = dot(d, outward) < 0;
  h.normal = h.front_face ? outward : -outward;
}

__device__ __forceinline__ void sphere_uv(V3 outward, double& u, double& v) {  // get_sphere_uv
  double theta = acos(-outward.y);
  double phi = atan2(-outward.z, outward.x) + kPi;
  u = phi / (2 * kPi);
  v = theta / kPi;
}

// Sphere::Hit + get_sphere_uv (sphere.h:23-55,73-79)
template <bool UV = true>
__device__ __forceinline__ bool hit_sphere(const double* g, int32_t mat, V3 o, V3 d, double tmin, double tmax,
                                           Hit& rec) {
  V3 c{g[0], g[1], g[2]};
  double radius = fmax(0.0, g[3]);
  V3 oc = c - o;
  double a = len2(d);
  double h = dot(d, oc);
  double cc = len2(oc) - radius * radius;
  double disc = h * h - a * cc;
  if (disc < 0) return false;
  double sq = sqrt(disc);
  double root = (h - sq) / a;
  if (!(tmin < root && root < tmax)) {
    root = (h + sq) / a;
    if (!(tmin < root && root < tmax)) return false;
  }
  rec.t = root;
  rec.p = o + rec.t * d;
  V3 outward = (rec.p - c) / radius;
  set_face_normal(rec, d, outward);
  if (UV) sphere_uv(outward, rec.u, rec.v);
  rec.mat = mat;
  return true;
}

// Triangle edges e1 = B - A, e2 = C - A (triangle.h:45-46): the device copy of the primitive
// table stores them in place of B and C (rtx_scene_create computes the same IEEE double
// differences on the host), so the tests read them instead of subtracting.
__device__ __forceinline__ V3 tri_e1(const double* g) { return V3{g[3], g[4], g[5]}; }
__device__ __forceinline__ V3 tri_e2(const double* g) { return V3{g[6], g[7], g[8]}; }

// Triangle::Hit (triangle.h:41-87): f32 det/inv_det/u/v/t, inclusive range, u,v untouched.
__device__ __forceinline__ bool hit_triangle(const double* g, int32_t mat, V3 o, V3 d, double tmin, double tmax,
                                             Hit& rec) {
  V3 A{g[0], g[1], g[2]};
  V3 e1 = tri_e1(g), e2 = tri_e2(g);
  V3 pvec = cross(d, e2);
  float det = (float)dot(e1, pvec);
  if (fabsf(det) < 1e-6f) return false;
  float inv_det = 1.0f / det;
  V3 tvec = o - A;
  float u = (float)(dot(tvec, pvec) * (double)inv_det);
  if (u < 0.0f || u > 1.0f) return false;
  V3 qvec = cross(tvec, e1);
  float v = (float)(dot(d, qvec) * (double)inv_det);
  if (v < 0.0f || (u + v) > 1.0f) return false;
  float t = (float)(dot(e2, qvec) * (double)inv_det);
  if ((double)t < tmin || (double)t > tmax) return false;
  rec.t = (double)t;
  rec.p = o + rec.t * d;
  rec.mat = mat;
  set_face_normal(rec, d, normalize(cross(e1, e2)));
  return true;
}

// xy/xz/yz_rect::Hit (rect.h:19-40, 65-85, 109-130)
__device__ __forceinline__ bool hit_rect(int kind, const double* g, int32_t mat, V3 o, V3 d, double tmin,
                                         double tmax, Hit& rec) {
  int ax, a0, a1;
  V3 n;
  if (kind == RTX_PRIM_XY_RECT) ax = 2, a0 = 0, a1 = 1, n = v3(0, 0, 1);
  else if (kind == RTX_PRIM_XZ_RECT) ax = 1, a0 = 0, a1 = 2, n = v3(0, 1, 0);
  else ax = 0, a0 = 1, a1 = 2, n = v3(1, 0, 0);
  double t = (g[4] - comp(o, ax)) / comp(d, ax);
  if (!(tmin < t && t < tmax)) return false;
  double x = comp(o, a0) + t * comp(d, a0);
  double y = comp(o, a1) + t * comp(d, a1);
  if (x < g[0] || x > g[1] || y < g[2] || y > g[3]) return false;
  rec.u = (x - g[0]) / (g[1] - g[0]);
  rec.v = (y - g[2]) / (g[3] - g[2]);
  rec.t = t;
  set_face_normal(rec, d, n);
  rec.mat = mat;
  rec.p = o + rec.t * d;
  return true;
}

template <bool UV = true>
__device__ __forceinline__ bool hit_prim(const rtx_prim* __restrict__ P, V3 o, V3 d, double tmin, double tmax,
                                         Hit& rec) {
  const int kind = P->kind;
  const int32_t mat = P->material;
  double g[9];
  if (kind == RTX_PRIM_TRIANGLE) {
#pragma unroll
    for (int i = 0; i < 9; i++) g[i] = P->g[i];
    return hit_triangle(g, mat, o, d, tmin, tmax, rec);
  }
  if (kind == RTX_PRIM_SPHERE) {
#pragma unroll
    for (int i = 0; i < 4; i++) g[i] = P->g[i];
    return hit_sphere<UV>(g, mat, o, d, tmin, tmax, rec);
  }
#pragma unroll
  for (int i = 0; i < 5; i++) g[i] = P->g[i];
  return hit_rect(kind, g, mat, o, d, tmin, tmax, rec);
}

// Accept/reject + distance only: the same arithmetic and decisions as hit_sphere /
// hit_triangle / hit_rect up to the point where they accept, without building the record.
// Traversal keeps just (closest t, best primitive); finish_hit() rebuilds the record of the
// winner afterwards with the interval (tmin, +inf), which yields the same root/t and hence
// the identical record (sphere: the near root is re-selected iff it was accepted).
//
// The 80-byte record is fetched as five 16-byte loads issued together, before the branch on
// `kind`: one memory latency per primitive test instead of two (kind, then the geometry
// the kind selects).  The empty asm keeps the compiler from sinking the geometry loads into
// the branches.
struct PrimRec {
  int kind;
  int32_t mat;
  double g[9];
};
template <bool KIND_KNOWN = false>
__device__ __forceinline__ PrimRec load_prim(const rtx_prim* __restrict__ P, bool tris) {
  PrimRec r;
  // spheres and rects read g[0..4] (48 bytes); triangles g[0..8] (80 bytes)
  const uint4 w0 = *(const uint4*)P;
  const double2 w1 = *((const double2*)P + 1), w2 = *((const double2*)P + 2);
  double2 w3 = make_double2(0.0, 0.0), w4 = make_double2(0.0, 0.0);
  if (tris) w3 = *((const double2*)P + 3), w4 = *((const double2*)P + 4);
  // (a kind-specialised caller never reads the kind word: it is not pinned, so not loaded)
  if (!KIND_KNOWN) asm volatile("" ::"v"(w0.x));
  asm volatile("" ::"v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w2.x), "v"(w2.y), "v"(w3.x), "v"(w3.y),
               "v"(w4.x), "v"(w4.y));
  r.kind = (int)w0.x;
  r.mat = (int32_t)w0.y;
  r.g[0] = __hiloint2double((int)w0.w, (int)w0.z);
  r.g[1] = w1.x, r.g[2] = w1.y, r.g[3] = w2.x, r.g[4] = w2.y;
  r.g[5] = w3.x, r.g[6] = w3.y, r.g[7] = w4.x, r.g[8] = w4.y;
  return r;
}

// KIND >= 0: every primitive this call can see has that kind (DScene::tree_kind), so the
// other kinds' branches are compiled out.
template <int KIND = -1>
__device__ __forceinline__ PrimRec load_prim_k(const rtx_prim* __restrict__ Pp, bool tris) {
  return load_prim<(KIND >= 0)>(Pp, KIND < 0 ? tris : KIND == (int)RTX_PRIM_TRIANGLE);
}
template <int KIND = -1>
__device__ __forceinline__ bool prim_t_rec(const PrimRec& R, V3 o, V3 d, double tmin, double tmax, double& t_out,
                                           int32_t& mat_out);
template <int KIND = -1>
__device__ __forceinline__ bool prim_t(const rtx_prim* __restrict__ Pp, bool tris, V3 o, V3 d, double tmin,
                                       double tmax, double& t_out, int32_t& mat_out) {
  // the record's loads issue together, before the test's first wait (see visit_slabs)
  __builtin_amdgcn_sched_barrier(0);
  const PrimRec R = load_prim_k<KIND>(Pp, tris);
  __builtin_amdgcn_sched_barrier(0);
  return prim_t_rec<KIND>(R, o, d, tmin, tmax, t_out, mat_out);
}
// the test itself, on a record already loaded
template <int KIND>
__device__ __forceinline__ bool prim_t_rec(const PrimRec& R, V3 o, V3 d, double tmin, double tmax, double& t_out,
                                           int32_t& mat_out) {
  mat_out = R.mat;
  const PrimRec* P = &R;
  const int kind = KIND >= 0 ? KIND : P->kind;
  if (kTriBranchless && KIND >= 0 && kind == RTX_PRIM_TRIANGLE) {
    // the same operations without the early exits: every value is computed and the four
    // rejections are combined at the end (a wave's few active leaf lanes rarely all take
    // the same early exit, so the branches only add mask bookkeeping)
    const V3 A{P->g[0], P->g[1], P->g[2]};
    const V3 e1 = tri_e1(P->g), e2 = tri_e2(P->g);
    const V3 pvec = cross(d, e2);
    const float det = (float)dot(e1, pvec);
    const float inv_det = 1.0f / det;
    const V3 tvec = o - A;
    const float u = (float)(dot(tvec, pvec) * (double)inv_det);
    const V3 qvec = cross(tvec, e1);
    const float v = (float)(dot(d, qvec) * (double)inv_det);
    const float t = (float)(dot(e2, qvec) * (double)inv_det);
    const bool ok = !(fabsf(det) < 1e-6f) & !(u < 0.0f || u > 1.0f) & !(v < 0.0f || (u + v) > 1.0f) &
                    !((double)t < tmin || (double)t > tmax);
    t_out = (double)t;
    return ok;
  }
  if (kind == RTX_PRIM_TRIANGLE) {
    V3 A{P->g[0], P->g[1], P->g[2]};
    V3 e1 = tri_e1(P->g), e2 = tri_e2(P->g);
    V3 pvec = cross(d, e2);
    float det = (float)dot(e1, pvec);
    if (fabsf(det) < 1e-6f) return false;
    float inv_det = 1.0f / det;
    V3 tvec = o - A;
    float u = (float)(dot(tvec, pvec) * (double)inv_det);
    if (u < 0.0f || u > 1.0f) return false;
    V3 qvec = cross(tvec, e1);
    float v = (float)(dot(d, qvec) * (double)inv_det);
    if (v < 0.0f || (u + v) > 1.0f) return false;
    float t = (float)(dot(e2, qvec) * (double)inv_det);
    if ((double)t < tmin || (double)t > tmax) return false;
    t_out = (double)t;
    return true;
  }
  if (kind == RTX_PRIM_SPHERE) {
    V3 c{P->g[0], P->g[1], P->g[2]};
    double radius = fmax(0.0, P->g[3]);
    V3 oc = c - o;
    double a = len2(d);
    double h = dot(d, oc);
    double cc = len2(oc) - radius * radius;
    double disc = h * h - a * cc;
    if (disc < 0) return false;  // (no gain without the early exits: ledger, ab_sph_*)
    double sq = sqrt(disc);
    double root = (h - sq) / a;
    if (!(tmin < root && root < tmax)) {
      root = (h + sq) / a;
      if (!(tmin < root && root < tmax)) return false;
    }
    t_out = root;
    return true;
  }
  int ax, a0, a1;
  if (kind == RTX_PRIM_XY_RECT) ax = 2, a0 = 0, a1 = 1;
  else if (kind == RTX_PRIM_XZ_RECT) ax = 1, a0 = 0, a1 = 2;
  else ax = 0, a0 = 1, a1 = 2;
  double t = (P->g[4] - comp(o, ax)) / comp(d, ax);
  if (!(tmin < t && t < tmax)) return false;
  double x = comp(o, a0) + t * comp(d, a0);
  double y = comp(o, a1) + t * comp(d, a1);
  if (x < P->g[0] || x > P->g[1] || y < P->g[2] || y > P->g[3]) return false;
  t_out = t;
  return true;
}

__device__ __forceinline__ bool prim_t(const rtx_prim* __restrict__ P, bool tris, V3 o, V3 d, double tmin,
                                       double tmax, double& t_out) {
  int32_t m;
  return prim_t(P, tris, o, d, tmin, tmax, t_out, m);
}

// Rebuild the HitRecord of the closest primitive (see prim_t).  u, v start at 0: the
// reference leaves them stale for triangles (triangle.h:77-84).
template <bool UV = true>
__device__ __forceinline__ void finish_hit(const DScene& S, int64_t best, V3 o, V3 d, double tmin, Hit& h) {
  h.u = 0.0, h.v = 0.0;
  hit_prim<UV>(S.prims + best, o, d, tmin, kInf, h);
  h.lazy_uv = (!UV && S.prims[best].kind == RTX_PRIM_SPHERE) ? best : -1;
}

// The same record from the winner's distance t as traversal computed it (prim_t returns
// exactly the t that hit_sphere / hit_triangle / hit_rect store), without intersecting again:
// the remaining fields depend on t and the primitive only.
template <bool UV = true>
__device__ __forceinline__ void finish_hit_at(const DScene& S, int64_t best, double t, V3 o, V3 d, Hit& h) {
  const rtx_prim* __restrict__ P = S.prims + best;
  const int kind = P->kind;
  h.u = 0.0, h.v = 0.0;
  h.mat = P->material;
  h.t = t;
  h.lazy_uv = -1;
  if (kind == RTX_PRIM_SPHERE) {  // hit_sphere after the root
    const V3 c{P->g[0], P->g[1], P->g[2]};
    const double radius = fmax(0.0, P->g[3]);
    h.p = o + h.t * d;
    const V3 outward = (h.p - c) / radius;
    set_face_normal(h, d, outward);
    if (UV) sphere_uv(outward, h.u, h.v);
    else h.lazy_uv = best;
  } else if (kind == RTX_PRIM_TRIANGLE) {  // hit_triangle after t
    h.p = o + h.t * d;
    if (S.tri_n) {
      // normalize(cross(B - A, C - A)) formed at upload in the same IEEE double operations
      const double2 n01 = *(const double2*)(S.tri_n + 4 * best), n2 = *(const double2*)(S.tri_n + 4 * best + 2);
      set_face_normal(h, d, V3{n01.x, n01.y, n2.x});
    } else {
      const V3 e1 = tri_e1(P->g), e2 = tri_e2(P->g);
      set_face_normal(h, d, normalize(cross(e1, e2)));
    }
  } else {  // hit_rect after t
    int a0, a1;
    V3 n;
    if (kind == RTX_PRIM_XY_RECT) a0 = 0, a1 = 1, n = v3(0, 0, 1);
    else if (kind == RTX_PRIM_XZ_RECT) a0 = 0, a1 = 2, n = v3(0, 1, 0);
    else a0 = 1, a1 = 2, n = v3(1, 0, 0);
    if (UV) {
      const double x = comp(o, a0) + t * comp(d, a0);
      const double y = comp(o, a1) + t * comp(d, a1);
      h.u = (x - P->g[0]) / (P->g[1] - P->g[0]);
      h.v = (y - P->g[2]) / (P->g[3] - P->g[2]);
    } else {
      h.lazy_uv = best;  // x, y above are p's components (lazy_uv)
    }
    set_face_normal(h, d, n);
    h.p = o + h.t * d;
  }
}

// Aabb::Hit (aabb.h:92-115), f64, relies on IEEE 1/0 = inf and false NaN compares.
__device__ __forceinline__ bool box_hit(const double* lo, const double* hi, V3 o, V3 inv_unused, V3 d,
                                        double tmin, double tmax) {
#pragma unroll
  for (int a = 0; a < 3; a++) {
    const double adinv = 1.0 / comp(d, a);
    double t0 = (lo[a] - comp(o, a)) * adinv;
    double t1 = (hi[a] - comp(o, a)) * adinv;
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

struct Counters {
  uint32_t nodes, prims;  // lane-level node visits / primitive tests
  uint32_t wnodes, wprims;  // wave-level loop iterations (counted by the first active lane)
  uint32_t tris, sphs;      // primitive tests by kind (rects = prims - tris - sphs)
  uint32_t witers, widle;   // persistent kernel: wave loop rounds, and those with no path to trace
  uint32_t wlive;           // ... and the lanes with a path, summed over the rounds that trace
};
// Persistent kernel, counting builds only (k_persistent's counter type is CountersClk when COUNT,
// plain Counters otherwise, so the product builds' code is untouched by this): the wave's
// shader-clock cycles (s_memtime) in the loop's regions — refill (ballot, slot claim, primary
// ray), walk (closest hit, parked walks included; of which the speculative walk's leaf rounds),
// shading (hit record, BSDF, Russian roulette, radiance store) — and the lanes that shaded,
// summed over the rounds (wave-uniform: counted by lane 0 or the first active lane).
struct CountersClk : Counters {
  uint64_t t_top, t_seg, t_walk, t_leaf;  // the current round's stamps (t_walk: set by the lanes that traced)
  uint64_t cyc_refill, cyc_walk, cyc_shade, cyc_leaf;
  uint32_t wshade, lshade;
};
__device__ __forceinline__ void count_prim(Counters& c, const rtx_prim* P) {
  c.prims++;
  const int k = P->kind;
  c.tris += k == RTX_PRIM_TRIANGLE ? 1u : 0u;
  c.sphs += k == RTX_PRIM_SPHERE ? 1u : 0u;
}
// first active lane of the (possibly divergent) wave
__device__ __forceinline__ bool first_active_lane() {
  const unsigned long long m = __ballot(1);
  return (int)__lane_id() == __ffsll((long long)m) - 1;
}

// ---------------------------------------------------------------------------------------
// Parity traversal: Scene{Bvh}::Hit exactly as bvh.h:71-119 (stack, push right then left,
// f64 slab test on [tmin, closest]).  The stack lives in LDS, one column per lane:
// stack entry i of lane t at stk[i * stride + t] (consecutive lanes -> consecutive banks).
// ---------------------------------------------------------------------------------------
// Returns the index (leaf order) of the closest primitive, or -1.
template <int STACK, bool COUNT>
__device__ __forceinline__ int64_t trace_parity(const DScene& S, V3 o, V3 d, double tmin, double tmax,
                                                uint32_t* stk, int stride, Counters& cnt, double& t_best) {
  int64_t best = -1;
  double closest = tmax, t;
  if (!S.use_bvh) {  // scene::Scene::Hit linear list (scene.h:47-61)
    for (int64_t i = 0; i < S.n_prims; i++) {
      if (COUNT) count_prim(cnt, S.prims + i);
      if (prim_t(S.prims + i, S.has_tris, o, d, tmin, closest, t)) closest = t, best = i;
    }
    t_best = closest;
    return best;
  }
  int sp = 0;
  stk[0] = 0u;
  sp = 1;
  while (sp > 0) {
    const uint32_t ni = stk[(--sp) * stride];
    const rtx_bvh_node* __restrict__ nd = S.nodes + ni;
    double lo[3] = {nd->lo[0], nd->lo[1], nd->lo[2]};
    double hi[3] = {nd->hi[0], nd->hi[1], nd->hi[2]};
    const uint32_t a = nd->left_first, b = nd->right_count, leaf = nd->is_leaf;
    if (COUNT) cnt.nodes++;
    if (!box_hit(lo, hi, o, o, d, tmin, closest)) continue;
    if (leaf) {
      for (uint32_t i = 0; i < b; i++) {
        if (COUNT) count_prim(cnt, S.prims + a + i);
        if (prim_t(S.prims + a + i, S.has_tris, o, d, tmin, closest, t)) closest = t, best = (int64_t)a + i;
      }
    } else {
      if (sp + 2 > STACK) __builtin_trap();  // host sizes STACK >= tree depth + 1
      stk[(sp++) * stride] = b;
      stk[(sp++) * stride] = a;
    }
  }
  t_best = closest;
  return best;
}

// ---------------------------------------------------------------------------------------
// Fast traversal (RTX_PREC_FAST): f32 slab tests against conservatively enlarged boxes,
// nearer child first; leaves are tested with the exact f64 primitive routines above.
// Enlarged boxes accept every ray the f64 test accepts, so the set of primitives that can
// produce the closest hit is a superset of the reference's; the closest hit is the same
// except for exact-tie orderings between distinct primitives (tests/test_gpu_parity.py checks
// every differing record is such a tie).
// ---------------------------------------------------------------------------------------
// smallest float >= x (x > 0 or +inf here)
__device__ __forceinline__ float f32_round_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = __int_as_float(__float_as_int(f) + (f >= 0.0f ? 1 : -1));
  return f;
}

// Pins a value at this point of the program (no code): the compiler can neither move its
// computation across this point nor assume it equal to an earlier value (shading: shared
// slots stay single instances; traversal: slab constants are recomputed, not kept live).
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(V3& v) {
  pin(v.x);
  pin(v.y);
  pin(v.z);
}

// 4-wide fast traversal over F4Node.  The collapsed tree has exactly the binary tree's
// leaves, and every binary box that the f64 test accepts is still accepted (each F4Node slot
// carries the outward-rounded box of the binary node it replaces, and the slab test below is
// conservative), so the candidate primitive set contains the reference's and the closest
// hit is the same up to exact t ties.  Per node: four slab tests, the hit leaves' primitives
// (one per leaf slot), then the surviving internal children sorted by entry distance; the
// nearest is visited next, the others are pushed far-to-near.  The host sizes the stack from
// the exact worst-case push depth of the collapsed tree (rtx_capi.hip build_fast4).
//
// Slab test, one FMA per plane: t = fma(plane, inv, n) with n = -(o * inv) -/+ delta.
// With inv = 1/RN(d) to within one ulp (v_rcp_f32), o_f = RN(o), n0 = RN(-o_f * inv), the
// computed plane distance is
//   t_c = T (1 + e_rel) + E,  |e_rel| <= 2^-22 + 2^-24,  |E| <= |o * inv| * 2^-23 * (1 + 2^-20)
// against the exact T = (plane - o) / d.  E is absorbed by shifting n outward by
// delta = |n0| * 2^-20 (the entry plane's offset down, the exit plane's up, by the sign of
// inv), e_rel by the 1e-5 relative slack on the entry/exit distances.  An axis whose offset
// is not finite (inv = inf for a zero f32 component) is neutralised: inv = 0, n = -/+inf,
// i.e. the slab imposes no constraint — a widening, hence still conservative.
//
// Sign-selected planes: the entry plane of axis a is `lo` when inv >= 0 and `hi` otherwise,
// so each slab needs no min/max: nl is the entry offset (n0 - delta), nh the exit offset
// (n0 + delta), and the entry-plane array is picked by a per-ray byte offset into the node.
__device__ __forceinline__ void fray4_axis_signed(double o, double d, int axis, float& inv, float& nl, float& nh,
                                                  uint32_t& off) {
  // the hardware reciprocal (1 ulp; a zero or denormal d gives +-inf or a huge inverse, and
  // an axis whose offset is not finite is neutralised below)
  inv = __builtin_amdgcn_rcpf((float)d);
  const float n0 = -((float)o * inv);
  off = 32u * axis;
  if (!(fabsf(n0) < __builtin_inff())) {
    inv = 0.0f, nl = -__builtin_inff(), nh = __builtin_inff();
    return;
  }
  const float delta = fabsf(n0) * 0x1p-20f;
  nl = n0 - delta, nh = n0 + delta;
  if (inv < 0.0f) off += 16u;
}
__device__ __forceinline__ float f4c(const float4& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); }

__device__ __forceinline__ void cswap4(float& ta, int32_t& ca, float& tb, int32_t& cb) {
  const bool s = tb < ta;
  const float t = s ? tb : ta;
  tb = s ? ta : tb;
  ta = t;
  const int32_t c = s ? cb : ca;
  cb = s ? ca : cb;
  ca = c;
}

// The 1e-5 relative slack of the slab test is folded into per-ray constants instead of two
// multiplies per slot:
//   tn' = fma(plane, inv * (1 - s), nl * (1 - s)),  tf' = fma(plane, inv * (1 + s), nh * (1 + s))
// i.e. (1 -/+ s) times each plane distance (monotone, so it commutes with the min/max and
// with the clamp at 0); the extra rounding of the two products is < 2^-23 relative, far
// inside s = 1e-5, and < 2^-23 |n0| absolute, inside the outward offset delta = 2^-20 |n0|,
// so the test stays conservative.  The walk relies on build_fast4's layout guarantees: every
// leaf slot holds exactly one primitive and empty slots have an inverted box, so no per-slot
// count is read.  Node loads use a 32-bit byte offset from the (uniform) node-array base.
struct FRay4L {
  float iex, iey, iez, nex, ney, nez;  // entry planes: inverse and offset, scaled by (1 - s)
  float ixx, ixy, ixz, nxx, nxy, nxz;  // exit planes: scaled by (1 + s)
  uint32_t ox, oy, oz;                 // byte offset of the entry-plane array per axis (exit: ^ 16)
};
struct FRay4 {  // per-ray plane constants before the slack is folded in
  float ix, iy, iz, nlx, nhx, nly, nhy, nlz, nhz;
  uint32_t ox, oy, oz;  // byte offset of the entry-plane array per axis (exit plane: offset ^ 16)
};
__device__ __forceinline__ FRay4L make_fray4l(V3 o, V3 d) {
  FRay4 b;
  fray4_axis_signed(o.x, d.x, 0, b.ix, b.nlx, b.nhx, b.ox);
  fray4_axis_signed(o.y, d.y, 1, b.iy, b.nly, b.nhy, b.oy);
  fray4_axis_signed(o.z, d.z, 2, b.iz, b.nlz, b.nhz, b.oz);
  constexpr float lo = 0.99999f, hi = 1.00001f;
  FRay4L r;
  r.iex = b.ix * lo, r.iey = b.iy * lo, r.iez = b.iz * lo;
  r.nex = b.nlx * lo, r.ney = b.nly * lo, r.nez = b.nlz * lo;
  r.ixx = b.ix * hi, r.ixy = b.iy * hi, r.ixz = b.iz * hi;
  r.nxx = b.nhx * hi, r.nxy = b.nhy * hi, r.nxz = b.nhz * hi;
  r.ox = b.ox, r.oy = b.oy, r.oz = b.oz;
  return r;
}

// Resumable form of the lean traversal.  TravState is everything a lane needs to continue
// a traversal later: the stack itself stays in the lane's LDS column, and the per-ray slab
// constants are recomputed from (o, d).  trace4_run() walks until the ray is done (true) or,
// when park_at >= 0, until at most park_at lanes of the wave are still walking at the top of
// a node iteration (false: the lane is parked with its state intact).  A parked ray continues
// exactly where it stopped, so the sequence of node visits and primitive tests — and the
// result — is the same as one uninterrupted walk.
struct TravState {
  uint32_t node;
  int32_t sp;
  double closest;
  int32_t best;  // leaf-order primitive index or -1
  int32_t mat;   // its material id
  float tmax_f;  // f32_round_up(closest)
};
__device__ __forceinline__ void trav_init(TravState& ts, double tmax) {
  ts.node = 0, ts.sp = 0, ts.closest = tmax, ts.best = -1, ts.mat = -1;
  ts.tmax_f = f32_round_up(tmax);
}

// Primitives kept out of the fast tree (a box as large as the rest of the scene together,
// e.g. a ground sphere; build_global_prims) are tested by every ray right after trav_init, in
// the converged control flow of the walk's start, instead of at scattered node visits where a
// few lanes at a time would run them.  Testing a primitive earlier only tightens `closest`
// sooner, so the closest hit is unchanged (up to the order of exact t ties, as for any tree).
template <bool COUNT>
__device__ __forceinline__ void trav_globals(const DScene& S, V3 o, V3 d, double tmin, Counters& cnt, TravState& ts) {
  for (int i = 0; i < S.n_global; i++) {
    const uint32_t gi = (uint32_t)S.global[i];
    if (COUNT) {
      count_prim(cnt, S.prims + gi);
      if (first_active_lane()) cnt.wprims++;
    }
    double t;
    int32_t m;
    if (prim_t(S.prims + gi, S.has_tris, o, d, tmin, ts.closest, t, m))
      ts.closest = t, ts.best = (int32_t)gi, ts.mat = m;
  }
  if (S.n_global) ts.tmax_f = f32_round_up(ts.closest);
}

// Pieces of a lean BVH4 node visit shared by trace4_run and trace4_run_step.
// The slab tests of node `node`'s four slots: entry distances of the internal children entered
// (+inf otherwise) in tt, the child words in cc; returns the mask of leaf slots entered.
__device__ __forceinline__ uint32_t visit_slabs(const char* __restrict__ nbase, uint32_t node, const FRay4L& r,
                                                float tmax_x, float (&tt)[4], int32_t (&cc)[4]) {
  const uint32_t noff = node << 7;  // sizeof(F4Node) == 128
  // The node's seven 16-byte loads issue back to back, before the first wait.  Left to itself,
  // LLVM's scheduler interleaves them with the slab tests of the first lines to arrive (a
  // `s_waitcnt vmcnt(4)` after five loads, the last two issued behind it: two memory round
  // trips per visit).  The barriers keep the loads together: C3 +3.2 %, and the same from
  // s_setprio at these two points, which the scheduler also does not cross
  // (profiles/r06/ab/r10y_prio_c3.txt, r10z_prio_c3.txt).
  __builtin_amdgcn_sched_barrier(0);
  const int4 ch = *(const int4*)(nbase + (noff + 96u));
  const float4 ex = *(const float4*)(nbase + (noff + r.ox)), fx = *(const float4*)(nbase + (noff + (r.ox ^ 16u)));
  const float4 ey = *(const float4*)(nbase + (noff + r.oy)), fy = *(const float4*)(nbase + (noff + (r.oy ^ 16u)));
  const float4 ez = *(const float4*)(nbase + (noff + r.oz)), fz = *(const float4*)(nbase + (noff + (r.oz ^ 16u)));
  __builtin_amdgcn_sched_barrier(0);
  cc[0] = ch.x, cc[1] = ch.y, cc[2] = ch.z, cc[3] = ch.w;
  uint32_t lmask = 0;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const float tn = fmaxf(fmaxf(fmaf(f4c(ex, c), r.iex, r.nex), fmaf(f4c(ey, c), r.iey, r.ney)),
                           fmaxf(fmaf(f4c(ez, c), r.iez, r.nez), 0.0f));
    const float tf = fminf(fminf(fmaf(f4c(fx, c), r.ixx, r.nxx), fmaf(f4c(fy, c), r.ixy, r.nxy)),
                           fminf(fmaf(f4c(fz, c), r.ixz, r.nxz), tmax_x));
    const bool hit = tn <= tf;
    lmask |= (hit && cc[c] < 0) ? (1u << c) : 0u;
    tt[c] = (hit && cc[c] >= 0) ? tn : __builtin_inff();
  }
  return lmask;
}
// The primitive of leaf slot c (its child word holds ~index)
__device__ __forceinline__ uint32_t leaf_prim(const int32_t (&cc)[4], int c) {
  const int32_t c01 = (c & 1) ? cc[1] : cc[0], c23 = (c & 1) ? cc[3] : cc[2];
  return ~(uint32_t)((c & 2) ? c23 : c01);
}
// The end of a visit: after a new closest hit (shrink), the children entered beyond it are
// dropped; the rest are sorted near to far, the nearest is visited next and the others pushed
// (branchless: the sort leaves the entered children as a prefix, so the
// stores at sp are unconditional and sp advances per entered child; build_fast4 bounds sp by
// the tree's exact worst case, and the kernels give each lane STACK + 1 slots), or the stack
// is popped.  false: the stack was empty, the walk is over.
template <int STACK, typename SE = uint32_t>
__device__ __forceinline__ bool visit_next(float (&tt)[4], int32_t (&cc)[4], bool shrink, double closest,
                                           float& tmax_f, float& tmax_x, SE* stk, int stride, int& sp,
                                           uint32_t& node) {
  if (shrink) {
    tmax_f = f32_round_up(closest);
    tmax_x = tmax_f * 1.00001f;
#pragma unroll
    for (int c = 0; c < 4; c++)
      if (tt[c] > tmax_f) tt[c] = __builtin_inff();
  }
  cswap4(tt[0], cc[0], tt[1], cc[1]);
  cswap4(tt[2], cc[2], tt[3], cc[3]);
  cswap4(tt[0], cc[0], tt[2], cc[2]);
  cswap4(tt[1], cc[1], tt[3], cc[3]);
  cswap4(tt[1], cc[1], tt[2], cc[2]);
  if (tt[0] != __builtin_inff()) {
#pragma unroll
    for (int c = 3; c >= 1; c--) {
      stk[sp * stride] = (SE)cc[c];
      sp += tt[c] != __builtin_inff() ? 1 : 0;
    }
    node = (uint32_t)cc[0];
    return true;
  }
  if (sp == 0) return false;
  node = (uint32_t)stk[(--sp) * stride];
  return true;
}

// The lean walk with its leaf tests spread over loop iterations.  A node visit whose boxes
// admit L leaf slots keeps the lane on that node for max(1, L) iterations: the slab tests and
// the first leaf test in the first, one more leaf test in each further one, and the stack
// update (cull by the new closest distance, sort, push / pop) in the last.  Each lane runs the
// same node visits and primitive tests in the same order as trace4_run (same results, bit for
// bit); what changes is how a wave's lanes line up.  trace4_run gives each node iteration a
// leaf loop as long as the longest lane's (1-4 trips of ~5 active lanes on the bunny), while
// here lanes with more leaves carry them into iterations where the other lanes visit nodes,
// so a wave iteration is one node phase plus at most one leaf test.  A lane parks only
// between node visits (no leaf pending), so the parked state is the same TravState.
template <int STACK, bool COUNT, int KIND = -1>
__device__ __forceinline__ bool trace4_run_step(const DScene& S, V3 o, V3 d, double tmin, uint32_t* stk,
                                                int stride, Counters& cnt, TravState& ts, int park_at) {
  FRay4L r = make_fray4l(o, d);
  const char* __restrict__ nbase = (const char*)S.f4nodes;
  double closest = ts.closest, t;
  int32_t best = ts.best, mat_best = ts.mat, m;
  float tmax_f = ts.tmax_f;
  float tmax_x = tmax_f * 1.00001f;
  int sp = ts.sp;
  uint32_t node = ts.node;
  bool done = true, pending = false, shrink = false;
  uint32_t lmask = 0;
  float tt[4];
  int32_t cc[4];
  while (true) {
    // every lane still in the loop counts as walking, parking takes only lanes between visits
    const bool park = park_at >= 0 && __popcll(__ballot(1)) <= park_at;
    if (!pending) {
      if (park) {
        done = false;
        break;
      }
      if (COUNT) {
        cnt.nodes++;
        if (first_active_lane()) cnt.wnodes++;
      }
      lmask = visit_slabs(nbase, node, r, tmax_x, tt, cc);
      shrink = false;
      pending = true;
    }
    if (lmask) {  // one leaf slot, in slot order
      const uint32_t cur = leaf_prim(cc, __builtin_ctz(lmask));
      lmask &= lmask - 1u;
      if (COUNT) {
        count_prim(cnt, S.prims + cur);
        if (first_active_lane()) cnt.wprims++;
      }
      if (prim_t<KIND>(S.prims + cur, S.has_tris, o, d, tmin, closest, t, m))
        closest = t, best = (int32_t)cur, mat_best = m, shrink = true;
    }
    if (lmask == 0) {  // the visit is complete: stack update
      pending = false;
      if (!visit_next<STACK>(tt, cc, shrink, closest, tmax_f, tmax_x, stk, stride, sp, node)) break;
    }
  }
  ts.node = node, ts.sp = sp, ts.closest = closest, ts.best = best, ts.mat = mat_best, ts.tmax_f = tmax_f;
  return done;
}

// The speculative walk's leaf queue: kLeafQueue words per lane (a power of two >= 8); a wave
// tests queued leaves once kLeafSpecMin of its lanes hold some, or no lane can visit a node
// (r02/ab/ab_spec8_c3.txt, ab_s16spec8_c3.txt: 8 words, forcing at 24 lanes; waiting with 8
// lanes: the bunny +0.8 % over the leaf-step walk, r03/ab_spec8w_c3.txt)
constexpr uint32_t kLeafQueue = 8;
constexpr int kLeafSpecMin = 8;
// The lean walk with speculative node visits (Aila & Laine 2009, "speculative traversal"):
// a visit's leaf slots go into the lane's FIFO queue (an LDS column of kLeafQueue words) and
// the lane walks on; a wave runs leaf tests only when kLeafSpecMin lanes hold queued leaves,
// or no lane can go on (each lane's queue might overflow on the next visit, its walk is over
// or it is parking), and then every lane with a queued leaf tests one; a lane that cannot
// visit meanwhile waits.  Same result, bit for bit, as
// trace4_run: the queue keeps the primitive tests in the order of the visits that found them,
// and node visits keep their depth-first order, because an entry distance does not depend on
// the closest hit.  A visit made before earlier leaves were tested culls its children against
// a looser closest distance, so the walk may visit extra nodes and test extra primitives —
// but each such primitive lies beyond a box entry the reference walk found past its closest
// hit (f32 box entry <= the primitive's t), so it is rejected and the closest hit, winner and
// tie order are unchanged.  A lane parks only with an empty queue, between visits.  The stack
// holds 16-bit node indices (the host runs this kernel only on trees under 2^16 nodes), so
// stack and queue fit the LDS of four blocks per CU.
template <int STACK, bool COUNT, int KIND = -1, class CNT = Counters>
__device__ __forceinline__ bool trace4_run_spec(const DScene& S, V3 o, V3 d, double tmin, uint16_t* stk,
                                                uint32_t* lq, int stride, CNT& cnt, TravState& ts,
                                                int park_at) {
  constexpr uint32_t F = kLeafQueue;
  static_assert(F >= 8 && (F & (F - 1)) == 0, "leaf queue: a power of two >= 8");
  FRay4L r = make_fray4l(o, d);
  const char* __restrict__ nbase = (const char*)S.f4nodes;
  double closest = ts.closest, t;
  int32_t best = ts.best, mat_best = ts.mat, m;
  float tmax_f = ts.tmax_f;
  float tmax_x = tmax_f * 1.00001f;
  int sp = ts.sp;
  uint32_t node = ts.node;
  bool walking = true, done = true;
  uint32_t qh = 0, qn = 0;  // queue head and length
  float tt[4];
  int32_t cc[4];
  while (true) {
    const bool park = park_at >= 0 && __popcll(__ballot(1)) <= park_at;
    if (park && qn == 0) {  // walking here: a lane whose walk is over has left the loop
      done = false;
      break;
    }
    if (walking && !park && qn <= F - 4) {  // a node visit; its leaf slots are queued
      if (COUNT) {
        cnt.nodes++;
        if (first_active_lane()) cnt.wnodes++;
      }
      uint32_t lmask = visit_slabs(nbase, node, r, tmax_x, tt, cc);
      while (lmask) {
        lq[((qh + qn) & (F - 1)) * stride] = leaf_prim(cc, __builtin_ctz(lmask));
        lmask &= lmask - 1u;
        qn++;
      }
      walking = visit_next<STACK, uint16_t>(tt, cc, false, closest, tmax_f, tmax_x, stk, stride, sp, node);
    }
    const bool can_visit = walking && !park && qn <= F - 4;
    if (__ballot(can_visit) == 0 || __popcll(__ballot(qn != 0)) >= kLeafSpecMin) {
      if constexpr (std::is_same_v<CNT, CountersClk>) cnt.t_leaf = __builtin_amdgcn_s_memtime();
      if (qn != 0) {  // one queued leaf, in visit order
        const uint32_t cur = lq[qh * stride];
        qh = (qh + 1) & (F - 1), qn--;
        if (COUNT) {
          count_prim(cnt, S.prims + cur);
          if (first_active_lane()) cnt.wprims++;
        }
        if (prim_t<KIND>(S.prims + cur, S.has_tris, o, d, tmin, closest, t, m)) {
          closest = t, best = (int32_t)cur, mat_best = m;
          tmax_f = f32_round_up(closest);
          tmax_x = tmax_f * 1.00001f;
        }
      }
      if constexpr (std::is_same_v<CNT, CountersClk>)
        if (first_active_lane()) cnt.cyc_leaf += __builtin_amdgcn_s_memtime() - cnt.t_leaf;
    }
    if (!walking && qn == 0) break;
  }
  ts.node = node, ts.sp = sp, ts.closest = closest, ts.best = best, ts.mat = mat_best, ts.tmax_f = tmax_f;
  return done;
}

template <int STACK, bool COUNT, int KIND = -1>
__device__ __forceinline__ bool trace4_run(const DScene& S, V3 o, V3 d, double tmin, uint32_t* stk, int stride,
                                           Counters& cnt, TravState& ts, int park_at) {
  if (kLeafStep) return trace4_run_step<STACK, COUNT, KIND>(S, o, d, tmin, stk, stride, cnt, ts, park_at);
  FRay4L r = make_fray4l(o, d);
  const char* __restrict__ nbase = (const char*)S.f4nodes;
  double closest = ts.closest, t;
  int32_t best = ts.best, mat_best = ts.mat, m;
  float tmax_f = ts.tmax_f;
  float tmax_x = tmax_f * 1.00001f;  // exit-side clamp with the slack folded in
  int sp = ts.sp;
  uint32_t node = ts.node;
  bool done = true;
  while (true) {
    if (park_at >= 0 && __popcll(__ballot(1)) <= park_at) {
      done = false;
      break;
    }
    if (COUNT) {
      cnt.nodes++;
      if (first_active_lane()) cnt.wnodes++;
    }
    float tt[4];
    int32_t cc[4];
    uint32_t lmask = visit_slabs(nbase, node, r, tmax_x, tt, cc);
    if (lmask) {
      bool shrink = false;
      while (lmask) {  // the visit's leaf slots, in slot order
        const int c = __builtin_ctz(lmask);
        lmask &= lmask - 1u;
        const uint32_t cur = leaf_prim(cc, c);
        if (COUNT) {
          count_prim(cnt, S.prims + cur);
          if (first_active_lane()) cnt.wprims++;
        }
        if (prim_t<KIND>(S.prims + cur, S.has_tris, o, d, tmin, closest, t, m))
          closest = t, best = (int32_t)cur, mat_best = m, shrink = true;
      }
      if (shrink) {  // children entered beyond the new closest hit are dropped
        tmax_f = f32_round_up(closest);
        tmax_x = tmax_f * 1.00001f;
#pragma unroll
        for (int c = 0; c < 4; c++)
          if (tt[c] > tmax_f) tt[c] = __builtin_inff();
      }
    }
    // (visit_next without its shrink step: this loop's own layout of the same operations
    // schedules better for the plain kernel, ab_refac_*)
    if (!visit_next<STACK>(tt, cc, false, closest, tmax_f, tmax_x, stk, stride, sp, node)) break;
  }
  ts.node = node, ts.sp = sp, ts.closest = closest, ts.best = best, ts.mat = mat_best, ts.tmax_f = tmax_f;
  return done;
}

// Linear closest hit over the whole primitive list (scene::Scene::Hit, scene.h:47-61), or the
// fast BVH's single-leaf root.
__device__ __forceinline__ int64_t trace_flat(const DScene& S, V3 o, V3 d, double tmin, double tmax, Counters& cnt,
                                              bool count, double& t_best, int32_t& mat_best) {
  int64_t best = -1;
  double closest = tmax, t;
  int32_t m;
  mat_best = -1;
  const int64_t n = S.use_bvh ? S.froot_count : S.n_prims;
  for (int64_t i = 0; i < n; i++) {
    if (count) count_prim(cnt, S.prims + i);
    if (prim_t(S.prims + i, S.has_tris, o, d, tmin, closest, t, m)) closest = t, best = i, mat_best = m;
  }
  t_best = closest;
  return best;
}

template <int STACK, bool COUNT, int KIND = -1>
__device__ __forceinline__ int64_t trace_fast4_lean(const DScene& S, V3 o, V3 d, double tmin, double tmax,
                                                    uint32_t* stk, int stride, Counters& cnt, double& t_best,
                                                    int32_t& mat_best) {
  // KIND >= 0 builds run only on scenes with a fast tree (an internal root): no flat list
  if (KIND < 0 && (!S.use_bvh || S.froot_leaf)) return trace_flat(S, o, d, tmin, tmax, cnt, COUNT, t_best, mat_best);
  TravState ts;
  trav_init(ts, tmax);
  trav_globals<COUNT>(S, o, d, tmin, cnt, ts);
  trace4_run<STACK, COUNT, KIND>(S, o, d, tmin, stk, stride, cnt, ts, -1);
  t_best = ts.closest, mat_best = ts.mat;
  return ts.best;
}

// ---------------------------------------------------------------------------------------
// Textures / materials
// ---------------------------------------------------------------------------------------
// Deferred u,v for image textures: a sphere's get_sphere_uv with outward = (p - c) / r exactly
// as hit_sphere; a rect's (x - x0) / (x1 - x0), (y - y0) / (y1 - y0) (rect.h), where x and y
// are p's in-plane components (hit_rect's x = o + t d per component, the same operations as
// p = o + t d).
// (Returned by value: reference outputs of a call live in scratch memory.  A call, not
// inlined: inlined, the textured build spills 300 B per lane, ledger.)
__device__ __noinline__ double2 lazy_uv(const rtx_prim* __restrict__ P, V3 p) {
  double2 uv;
  const int kind = P->kind;
  if (kind == RTX_PRIM_SPHERE) {
    V3 c{P->g[0], P->g[1], P->g[2]};
    double radius = fmax(0.0, P->g[3]);
    sphere_uv((p - c) / radius, uv.x, uv.y);
  } else {
    const int a0 = kind == RTX_PRIM_YZ_RECT ? 1 : 0, a1 = kind == RTX_PRIM_XY_RECT ? 1 : 2;
    uv.x = (comp(p, a0) - P->g[0]) / (P->g[1] - P->g[0]);
    uv.y = (comp(p, a1) - P->g[2]) / (P->g[3] - P->g[2]);
  }
  return uv;
}

__device__ __forceinline__ V3 tex_value(const DScene& S, int32_t t, const Hit& rec) {
  double u = rec.u, v = rec.v;
  const V3 p = rec.p;
  for (int guard = 0; guard < 16; guard++) {
    const rtx_texture T = S.texs[t];
    if (T.kind == RTX_TEX_SOLID) return v3(T.color[0], T.color[1], T.color[2]);
    if (T.kind == RTX_TEX_CHECKER) {  // texture.h:37-45 (C++ % keeps the sign)
      int xi = (int)floor(T.inv_scale * p.x);
      int yi = (int)floor(T.inv_scale * p.y);
      int zi = (int)floor(T.inv_scale * p.z);
      t = ((xi + yi + zi) % 2 == 0) ? T.even : T.odd;
      continue;
    }
    // ImageTexture::Value (texture.h:58-73), Image::PixelData/Clamp (image.cc:50-67)
    if (T.image < 0) return v3(0, 1, 1);
    const DImage im = S.images[T.image];
    if (im.h <= 0) return v3(0, 1, 1);
    if (rec.lazy_uv >= 0) {
      const double2 uv = lazy_uv(S.prims + rec.lazy_uv, p);
      u = uv.x, v = uv.y;
    }
    u = u < 0 ? 0 : (u > 1 ? 1 : u);
    v = 1.0 - (v < 0 ? 0 : (v > 1 ? 1 : v));
    int i = (int)(u * im.w);
    int j = (int)(v * im.h);
    i = i < 0 ? 0 : (i < im.w ? i : im.w - 1);
    j = j < 0 ? 0 : (j < im.h ? j : im.h - 1);
    const uint8_t* px = im.texels + ((size_t)j * im.w + i) * 3;
    double s = 1.0 / 255.0;
    return v3(s * px[0], s * px[1], s * px[2]);
  }
  return v3(0, 1, 1);
}

// Albedo / emission texture of a Lambertian or DiffuseLight material.  The device copy of
// the material table (rtx_scene_create) resolves a directly attached SolidColor texture at
// upload: texture = -1 and the colour's doubles copied into the (otherwise unused) albedo
// field, so the common case costs no dependent texture-table load.
__device__ __forceinline__ V3 mat_tex(const DScene& S, const rtx_material& m, const Hit& rec) {
  if (m.texture < 0) return v3(m.albedo[0], m.albedo[1], m.albedo[2]);
  return tex_value(S, m.texture, rec);
}

// pow(x, 5.0) (material.cc:261) as a double-double product chain rounded once: the
// correctly rounded x^5, which is what glibc's pow (<= 0.52 ulp) returns except at
// near-ties.  Explicit fma() only builds the exact error terms (no contraction elsewhere).
__device__ __forceinline__ double pow5(double x) {
  const double p2 = x * x, e2 = fma(x, x, -p2);
  const double p4 = p2 * p2, e4 = fma(p2, p2, -p4) + 2.0 * (p2 * e2);
  const double p5 = p4 * x, e5 = fma(p4, x, -p5) + e4 * x;
  return p5 + e5;
}

__device__ __forceinline__ double reflectance(double c, double ri) {  // material.cc:258-262
  double r0 = (1.0 - ri) / (1.0 + ri);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * pow5(1.0 - c);
}

// Material::Scatter (material.cc:20-34, 82-94, 148-172, 273-280) — megakernel mode
__device__ __forceinline__ bool mat_scatter(const DScene& S, const rtx_material& m, V3 rin_d, const Hit& rec,
                                            V3& att, V3& sd, Rng& g) {
  if (m.kind == RTX_MAT_LAMBERTIAN) {
    V3 dir = rec.normal + random_unit_vector(g);
    if (near_zero(dir)) dir = rec.normal;
    sd = dir;
    att = mat_tex(S, m, rec);
    return true;
  }
  if (m.kind == RTX_MAT_METAL) {
    V3 r = reflect(rin_d, rec.normal);
    r = r + m.fuzz * random_unit_vector(g);
    sd = r;
    att = v3(m.albedo[0], m.albedo[1], m.albedo[2]);
    return dot(sd, rec.normal) > 0;
  }
  if (m.kind == RTX_MAT_DIELECTRIC) {
    att = v3(1.0, 1.0, 1.0);
    double eta = rec.front_face ? (1.0 / m.ref_idx) : m.ref_idx;
    V3 ud = normalize(rin_d);
    double ct = fmin(dot(-ud, rec.normal), 1.0);
    double stt = sqrt(1.0 - ct * ct);
    bool cannot = eta * stt > 1.0;
    if (cannot || reflectance(ct, eta) > g.next()) sd = reflect(ud, rec.normal);
    else sd = refract(ud, rec.normal, eta);
    return true;
  }
  return false;
}

__device__ __forceinline__ V3 mat_emitted(const DScene& S, const rtx_material& m, const Hit& rec) {
  if (m.kind == RTX_MAT_DIFFUSE_LIGHT) return mat_tex(S, m, rec);
  return v3(0, 0, 0);
}
// NOTEX: no material of the scene reads a texture table entry (DScene::no_textures: every
// Lambertian / DiffuseLight colour was resolved into the device material table), so the
// texture lookup is compiled out.
template <bool NOTEX>
__device__ __forceinline__ V3 mat_tex_t(const DScene& S, const rtx_material& m, const Hit& rec) {
  if (NOTEX) return v3(m.albedo[0], m.albedo[1], m.albedo[2]);
  return mat_tex(S, m, rec);
}
template <bool NOTEX>
__device__ __forceinline__ V3 mat_emitted_t(const DScene& S, const rtx_material& m, const Hit& rec) {
  if (m.kind == RTX_MAT_DIFFUSE_LIGHT) return mat_tex_t<NOTEX>(S, m, rec);
  return v3(0, 0, 0);
}

__device__ __forceinline__ V3 sky(V3 d) {  // wavefront.cc:33-38, camera.h:171-173
  V3 ud = normalize(d);
  double t = 0.5 * (ud.y + 1.0);
  return (1.0 - t) * v3(1.0, 1.0, 1.0) + t * v3(0.5, 0.7, 1.0);
}

// Camera::GetRay (camera.h:134-144,196-203): y offset drawn first (g++ arg order).
// NODOF: the camera has no defocus (the host checked defocus_angle <= 0), so the thin-lens
// sampling is compiled out.
template <bool NODOF = false>
__device__ __forceinline__ void get_ray(const rtx_camera& c, int i, int j, Rng& g, V3& o, V3& d) {
  double oy = g.next() - 0.5;
  double ox = g.next() - 0.5;
  V3 p00{c.pixel00[0], c.pixel00[1], c.pixel00[2]};
  V3 du{c.pixel_delta_u[0], c.pixel_delta_u[1], c.pixel_delta_u[2]};
  V3 dv{c.pixel_delta_v[0], c.pixel_delta_v[1], c.pixel_delta_v[2]};
  V3 ps = p00 + ((i + ox) * du) + ((j + oy) * dv);
  V3 center{c.center[0], c.center[1], c.center[2]};
  if (NODOF || c.defocus_angle <= 0) {
    o = center;
  } else {
    V3 p = random_in_unit_disk(g);
    V3 ddu{c.defocus_disk_u[0], c.defocus_disk_u[1], c.defocus_disk_u[2]};
    V3 ddv{c.defocus_disk_v[0], c.defocus_disk_v[1], c.defocus_disk_v[2]};
    o = center + (p.x * ddu) + (p.y * ddv);
  }
  d = ps - o;
}

// Path state between bounces (RayState, ray_state.h:8-13).  The RNG needs no state of its
// own: segment `depth` shades with stream depth + 1 (see Rng).
struct Path {
  V3 o, d, thr;
  int32_t depth;
};

// normalize (math_utils.h:93-97) returning the length as well
__device__ __forceinline__ V3 normalize_l(V3 v, double& l) {
  l = sqrt(len2(v));
  if (l == 0.0) return {0, 0, 0};
  return v / l;
}

// One shading step (wavefront.cc:109-208).  true: continue with p updated; false: path
// terminated with radiance L (RecordSample is done by the caller, in sample order).
// `m` is the hit's material (S.mats[rec.mat]; unused on a miss).
//
// The Sample() chains of the three materials (material.cc:57-74, 117-141, 194-256) are run
// in five shared slots: a wave that holds lanes of several materials executes each
// normalize / sqrt once for all of them, instead of once per material branch.  Every lane
// still performs exactly its own material's operations on its own operands, in the
// reference's order, so the results are bit-identical to one branch per material (the
// Lambertian chain is math_utils.h:104-123 RandomCosineDirection; the merge was checked bit
// for bit against the per-material form, cmp_merged_shade_bitexact.txt, before that form was
// removed):
//   slot 1 normalize   Lambertian: w = normalize(n)          Dielectric: win = normalize(d)
//   slot 2 sqrt        Lambertian: sqrt(r2)                  Dielectric: sqrt(max(0, 1 - ci^2))
//   slot 3 sqrt        Lambertian: sqrt(1 - r2)              Dielectric (refract): sqrt|1 - |perp|^2|
//   slot 4 normalize   Lambertian: normalize(cross(w, a))    Metal: normalize(reflect + fuzz * u)
//   slot 5 normalize   Lambertian: normalize(x u + y v + z w)
// The ray's unit direction is shared too: sky() on a miss and wo = -normalize(d) on a hit.
// Dielectric uses win = -normalize(wo) = normalize(normalize(d)) exactly (sign-symmetric
// rounding), and eta = 1/ri (front face) / r0 = ((1-ri)/(1+ri))^2 precomputed at upload
// in the same IEEE double operations (device material table, rtx_scene_create).
// LAMB: every material of the scene is Lambertian (DScene::all_lambertian; the bunny), so the
// metal / dielectric / emitter branches are compiled out.  Same operations for a Lambertian.
// What one shading step decided, before the path throughput is applied (shade_finish):
// the core of the step never reads the throughput, so a caller may keep it out of registers
// (the persistent kernel parks it in LDS while the lane walks the tree).
enum : int32_t {
  kShadeEmit = 0,     // terminated, L = thr * f (sky on a miss / at the depth limit, or emission)
  kShadeDead = 1,     // terminated, L = 0 (absorbed: Sample() failed, pdf < 1e-6f, DiffuseLight)
  kShadeDiffuse = 2,  // continues, thr' = ((double)ct * (thr * f)) / (double)pdf (wavefront.cc:180-185)
  kShadeSpecular = 3  // continues, thr' = thr * f (IsSpecular)
};
struct ShadeOut {
  V3 f;
  float ct, pdf;
  int32_t what;
  int32_t fsrc;  // DEFER_F: 1 f = albedo / pi (Lambertian), 2 f = albedo (Metal), read by shade_finish
};
// A copy of a pointer the compiler cannot see through: loads through it are issued where they
// are written (late), not hoisted to an earlier load of the same address and kept live.
template <class T>
__device__ __forceinline__ const T* opaque(const T* p) {
  asm volatile("" : "+v"(p));
  return p;
}

// SET_ORIGIN = false: a continuing path's new origin (the hit point) is left for the caller
// to set, so a caller that parked the hit point elsewhere keeps rec.p out of registers.
// DEFER_F (texture-free builds): the BSDF value of a Lambertian / Metal hit is the material's
// albedo (/ pi); it is read from the material table by shade_finish, at the end, instead of
// being held in registers across the direction sampling.
template <bool LAMB = false, bool NOTEX = false, bool SET_ORIGIN = true, bool DEFER_F = false>
__device__ __forceinline__ void shade_core(const DScene& S, int max_depth, Path& p, const Hit& rec, bool hit, Rng& g,
                                           const rtx_material& m, ShadeOut& so) {
  static_assert(!DEFER_F || NOTEX, "deferred BSDF values need texture-free shading");
  so.what = kShadeDead;
  so.fsrc = 0;
  double lnd;
  const V3 nd = normalize_l(p.d, lnd);  // wo = -nd (hit), sky(d) (miss)
  if (!hit || p.depth >= max_depth) {
    const double t = 0.5 * (nd.y + 1.0);  // sky() with ud = nd
    so.f = (1.0 - t) * v3(1.0, 1.0, 1.0) + t * v3(0.5, 0.7, 1.0);
    so.what = kShadeEmit;
    return;
  }
  if (!LAMB) {  // Lambertian emits nothing (Material::Emitted default, material.h:50-54)
    V3 em = mat_emitted_t<NOTEX>(S, m, rec);
    if (!near_zero(em)) {
      so.f = em;
      so.what = kShadeEmit;
      return;
    }
  }
  const int kind = LAMB ? (int)RTX_MAT_LAMBERTIAN : m.kind;
  const bool isL = kind == RTX_MAT_LAMBERTIAN, isM = kind == RTX_MAT_METAL, isG = kind == RTX_MAT_DIELECTRIC;
  if (!(isL || isM || isG)) return;  // DiffuseLight::Sample
  const V3 n = rec.normal;
  // EARLY_TEX (textured builds): a Lambertian's albedo texture is looked up here, before the
  // direction sampling, so the hit point / u,v / lazy-uv sphere are dead during the sampling
  // (only the colour is kept); the same lookup, only earlier
  V3 ftex = v3(0, 0, 0);
  if (kEarlyTex && !NOTEX && !DEFER_F && isL) ftex = mat_tex_t<NOTEX>(S, m, rec);
  double r1 = 0.0, r2 = 0.0;
  if (isL) r1 = g.next(), r2 = g.next();
  V3 ru = v3(0, 0, 0);
  if (isM) ru = random_unit_vector(g);
  // ---- slot 1: normalize
  double l1;
  V3 s1 = normalize_l(isL ? n : nd, l1);
  pin(s1);
  const V3 w = s1;
  // win = -normalize(wo): (0,0,0) negated when the direction has zero length
  const V3 win = (!isL && l1 == 0.0) ? v3(-0.0, -0.0, -0.0) : s1;
  double eta = 0.0, ci = 0.0, a2 = 0.0;
  if (isG) {
    eta = rec.front_face ? m.albedo[0] : m.ref_idx;  // eta_i / eta_t
    ci = dot(win, n);
    ci = ci < -1.0 ? -1.0 : (ci > 1.0 ? 1.0 : ci);
    a2 = fmax(0.0, 1.0 - ci * ci);
  }
  // ---- slot 2: sqrt
  double s2 = sqrt(isL ? r2 : a2);
  pin(s2);
  double x = 0.0, y = 0.0;
  if (isL) {
    const double phi = 2.0 * kPi * r1;
    double cph, sph;
    cos_sin<kSincosSmall || !LAMB>(phi, cph, sph);
    x = s2 * cph;
    y = s2 * sph;
  }
  bool g_reflect = false;
  V3 perp = v3(0, 0, 0);
  double a3 = 1.0;
  if (isG) {
    const double st = eta * s2;
    g_reflect = st >= 1.0;
    if (!g_reflect) {
      const double r0 = m.albedo[1];  // reflectance(|ci|, ref_idx): r0 = ((1-ri)/(1+ri))^2
      const double Fr = r0 + (1.0 - r0) * pow5(1.0 - fabs(ci));
      g_reflect = g.next() < Fr;
    }
    if (!g_reflect) {  // refract (math_utils.h:24-29)
      const double c = fmin(dot(-win, n), 1.0);
      perp = eta * (win + c * n);
      a3 = fabs(1.0 - len2(perp));
    }
  }
  // ---- slot 3: sqrt
  double s3 = sqrt(isL ? 1.0 - r2 : a3);
  pin(s3);
  V3 in4;
  if (isL) {
    const V3 a = (fabs(w.x) > 0.9) ? v3(0, 1, 0) : v3(1, 0, 0);
    in4 = cross(w, a);
  } else {
    in4 = reflect(nd, n);  // reflect(-wo, n)
    in4 = in4 + m.fuzz * ru;
  }
  // ---- slot 4: normalize
  double l4;
  V3 s4 = normalize_l(in4, l4);
  pin(s4);
  V3 wi;
  if (isL) {
    const V3 v = s4;
    const V3 u = cross(v, w);
    // ---- slot 5: normalize (Lambertian only)
    wi = normalize(x * u + y * v + s3 * w);
    if (dot(wi, n) <= 0) return;
    const float cf = (float)dot(n, wi);
    const float pdf = (cf <= 0.0f) ? 0.0f : (float)((double)cf / kPi);
    if (DEFER_F) so.fsrc = 1;
    else so.f = ((kEarlyTex && !NOTEX) ? ftex : mat_tex_t<NOTEX>(S, m, rec)) / kPi;
    if (pdf < 1e-6f) return;
    so.ct = fmaxf(0.0f, (float)dot(wi, n));
    so.pdf = pdf;
    so.what = kShadeDiffuse;
  } else if (isM) {
    wi = s4;
    if (dot(wi, n) <= 0) return;
    if (DEFER_F) so.fsrc = 2;
    else so.f = v3(m.albedo[0], m.albedo[1], m.albedo[2]);
    so.what = kShadeSpecular;
  } else {
    if (g_reflect) {
      wi = reflect(win, n);
      so.f = v3(1.0, 1.0, 1.0);
    } else {
      const V3 par = (-s3) * n;
      wi = perp + par;
      const double k = eta * eta;
      so.f = v3(k, k, k);
    }
    so.what = kShadeSpecular;
  }
  if (SET_ORIGIN) p.o = rec.p;
  p.d = wi, p.depth = p.depth + 1;
}

// The rest of the step: radiance of a terminated path, or the child's throughput and Russian
// roulette (wavefront.cc:189-205) with the segment's last draw.  depth = the child's depth.
__device__ __forceinline__ bool shade_finish(const ShadeOut& so, V3& thr, int32_t depth, Rng& g, V3& L,
                                             const rtx_material* m = nullptr) {
  L = v3(0, 0, 0);
  if (so.what == kShadeEmit) {
    L = L + thr * so.f;
    return false;
  }
  if (so.what == kShadeDead) return false;
  V3 f = so.f;
  if (so.fsrc) {  // DEFER_F: the texture-free BSDF value, read now (shade_core)
    const rtx_material* mp = opaque(m);
    f = v3(mp->albedo[0], mp->albedo[1], mp->albedo[2]);
    if (so.fsrc == 1) f = f / kPi;
  }
  V3 c = so.what == kShadeDiffuse ? ((double)so.ct * (thr * f)) / (double)so.pdf : thr * f;
  if (depth > 5) {
    double q = fmax(fmax(c.x, c.y), c.z);
    q = q < 0.1 ? 0.1 : (q > 0.95 ? 0.95 : q);
    if (g.next() > q) return false;
    c = c / q;
  }
  thr = c;
  return true;
}

template <bool LAMB = false, bool NOTEX = false>
__device__ __forceinline__ bool shade_merged(const DScene& S, int max_depth, Path& p, const Hit& rec, bool hit,
                                             Rng& g, V3& L, const rtx_material& m) {
  ShadeOut so;
  shade_core<LAMB, NOTEX>(S, max_depth, p, rec, hit, g, m, so);
  return shade_finish(so, p.thr, p.depth, g, L);
}

template <bool LAMB = false, bool NOTEX = false>
__device__ __forceinline__ bool shade(const DScene& S, int max_depth, Path& p, const Hit& rec, bool hit, Rng& g,
                                      V3& L, const rtx_material& m) {
  return shade_merged<LAMB, NOTEX>(S, max_depth, p, rec, hit, g, L, m);
}

__device__ __forceinline__ bool shade(const DScene& S, int max_depth, Path& p, const Hit& rec, bool hit, Rng& g,
                                      V3& L) {
  rtx_material m;
  if (hit) m = S.mats[rec.mat];
  return shade(S, max_depth, p, rec, hit, g, L, m);
}

}  // namespace rtxd
