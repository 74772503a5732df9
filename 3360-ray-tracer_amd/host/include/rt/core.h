// rt/core.h — value types of the host API (mirrors the reference's src/core/: vec3.h,
// ray.h, interval.h, constants.h, random.h, color.h, timer.h).
//
// Host-side only: scene assembly, camera set-up and output.  No per-ray compute lives
// here; rays are generated, traced and shaded on the GPU behind include/rtx.h.
#pragma once

#include <chrono>
#include <cmath>
#include <cstdint>
#include <iostream>
#include <limits>
#include <random>

namespace rt::core {

constexpr double kPi = 3.14159265358979323846;  // constants.h:11
constexpr double kInfinity = std::numeric_limits<double>::infinity();

constexpr double DegreesToRadians(double degrees) { return degrees * (kPi / 180.0); }

class Vec3 {  // vec3.h:8-61
 public:
  constexpr Vec3() : e_{0, 0, 0} {}
  constexpr Vec3(double x, double y, double z) : e_{x, y, z} {}
  constexpr double x() const { return e_[0]; }
  constexpr double y() const { return e_[1]; }
  constexpr double z() const { return e_[2]; }
  constexpr double operator[](int i) const { return e_[i]; }
  double& operator[](int i) { return e_[i]; }
  constexpr Vec3 operator-() const { return Vec3(-e_[0], -e_[1], -e_[2]); }
  Vec3& operator+=(const Vec3& v) {
    e_[0] += v.e_[0], e_[1] += v.e_[1], e_[2] += v.e_[2];
    return *this;
  }
  Vec3& operator*=(double t) {
    e_[0] *= t, e_[1] *= t, e_[2] *= t;
    return *this;
  }
  Vec3& operator/=(double t) { return *this *= (1.0 / t); }
  constexpr double length_squared() const { return e_[0] * e_[0] + e_[1] * e_[1] + e_[2] * e_[2]; }
  double length() const { return std::sqrt(length_squared()); }
  bool NearZero() const {
    return std::fabs(e_[0]) < 1e-8 && std::fabs(e_[1]) < 1e-8 && std::fabs(e_[2]) < 1e-8;
  }

 private:
  double e_[3];
};
using Point3 = Vec3;
using Color = Vec3;

inline Vec3 operator+(const Vec3& u, const Vec3& v) { return Vec3(u[0] + v[0], u[1] + v[1], u[2] + v[2]); }
inline Vec3 operator-(const Vec3& u, const Vec3& v) { return Vec3(u[0] - v[0], u[1] - v[1], u[2] - v[2]); }
inline Vec3 operator*(const Vec3& u, const Vec3& v) { return Vec3(u[0] * v[0], u[1] * v[1], u[2] * v[2]); }
inline Vec3 operator*(double t, const Vec3& v) { return Vec3(t * v[0], t * v[1], t * v[2]); }
inline Vec3 operator*(const Vec3& v, double t) { return t * v; }
inline Vec3 operator/(const Vec3& v, double t) { return (1.0 / t) * v; }
inline double Dot(const Vec3& u, const Vec3& v) { return u[0] * v[0] + u[1] * v[1] + u[2] * v[2]; }
inline Vec3 Cross(const Vec3& u, const Vec3& v) {
  return Vec3(u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]);
}
inline Vec3 Normalize(const Vec3& v) {
  double l = v.length();
  return l == 0.0 ? Vec3(0, 0, 0) : v / l;
}
inline std::ostream& operator<<(std::ostream& o, const Vec3& v) { return o << v[0] << ' ' << v[1] << ' ' << v[2]; }

class Ray {  // ray.h
 public:
  Ray() {}
  Ray(const Point3& origin, const Vec3& direction) : orig_(origin), dir_(direction) {}
  const Point3& origin() const { return orig_; }
  const Vec3& direction() const { return dir_; }
  Point3 at(double t) const { return orig_ + t * dir_; }

 private:
  Point3 orig_;
  Vec3 dir_;
};

class Interval {  // interval.h
 public:
  double min_, max_;
  Interval() : min_(+kInfinity), max_(-kInfinity) {}
  Interval(double mn, double mx) : min_(mn), max_(mx) {}
  Interval(const Interval& a, const Interval& b) : min_(std::min(a.min_, b.min_)), max_(std::max(a.max_, b.max_)) {}
  double Size() const { return max_ - min_; }
  bool Contains(double x) const { return min_ <= x && x <= max_; }
  bool Surrounds(double x) const { return min_ < x && x < max_; }
  double Clamp(double x) const { return x < min_ ? min_ : (x > max_ ? max_ : x); }
};

// ---- RNG (random.h): the host stream used by the scene recipes (main.cc) ----------------
// The renderer itself never draws from it: paths use the counter-based device stream.
std::mt19937& GetRng();
inline double RandomDouble() {
  static thread_local std::uniform_real_distribution<double> dist(0.0, 1.0);
  return dist(GetRng());
}
inline double RandomDouble(double mn, double mx) { return mn + (mx - mn) * RandomDouble(); }
inline int RandomInt(int mn, int mx) { return std::uniform_int_distribution<int>(mn, mx)(GetRng()); }
inline void SeedRng(unsigned int seed) { GetRng().seed(seed); }
// RandomVec3 as the reference build evaluates it: g++ runs Vec3's three constructor
// arguments right to left (z, then y, then x) — pinned by tests/golden/scenes.
inline Vec3 RandomVec3() {
  double z = RandomDouble(), y = RandomDouble(), x = RandomDouble();
  return Vec3(x, y, z);
}
inline Vec3 RandomVec3(double mn, double mx) {
  double z = RandomDouble(mn, mx), y = RandomDouble(mn, mx), x = RandomDouble(mn, mx);
  return Vec3(x, y, z);
}

// ---- color.h ------------------------------------------------------------------------------
inline double linear_to_gamma(double x) { return x > 0 ? std::sqrt(x) : 0; }
inline void write_color(std::ostream& out, const Color& c) {
  static const Interval intensity(0.000, 0.999);
  out << int(256 * intensity.Clamp(linear_to_gamma(c[0]))) << ' ' << int(256 * intensity.Clamp(linear_to_gamma(c[1])))
      << ' ' << int(256 * intensity.Clamp(linear_to_gamma(c[2]))) << '\n';
}
inline double luminance(const Color& c) { return 0.2126f * c.x() + 0.7152f * c.y() + 0.0722f * c.z(); }

class Timer {  // timer.h
 public:
  Timer() { reset(); }
  void reset() { t0_ = std::chrono::steady_clock::now(); }
  double elapsed() const { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count(); }

 private:
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace rt::core
