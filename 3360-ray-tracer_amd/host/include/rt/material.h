// rt/material.h — material and texture descriptors (mirrors the reference's
// src/material/material.h, texture.h and src/scene/image.h).
//
// BSDF sampling (Material::Sample / Scatter / Emitted) executes on the GPU (csrc/
// rtx_device.h mat_sample / mat_scatter / mat_emitted); these classes carry the parameters.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "rt/core.h"
#include "rtx.h"

namespace rt::scene {

// Image (scene/image.h): texels after the reference's decode (stb_image's stbi_loadf: 8-bit
// decode, gamma 2.2) and FloatToByte (image.cc:16-73), decoded by rt/image.h (JPEG, binary
// PNM).  A file that does not load -> Height() == 0 (cyan, texture.h:62).
class Image {
 public:
  Image() = default;
  explicit Image(const std::string& filename);
  bool Load(const std::string& filename);
  int Width() const { return width_; }
  int Height() const { return height_; }
  const unsigned char* PixelData(int x, int y) const;
  const std::vector<unsigned char>& bytes() const { return bdata_; }

 private:
  int width_ = 0, height_ = 0;
  std::vector<unsigned char> bdata_;
};

// Directories searched for assets (textures, models): $RTX_ASSET_DIR, then the package's
// assets/ directory (compile-time RTX_ASSET_DIR_DEFAULT).
std::string ResolveAsset(const std::string& name);

}  // namespace rt::scene

namespace rt::material {

enum class TextureKind { kSolid, kChecker, kImage };

class Texture {
 public:
  virtual ~Texture() = default;
  virtual TextureKind Kind() const = 0;
};

class SolidColor : public Texture {
 public:
  SolidColor(const core::Color& albedo) : albedo_(albedo) {}
  SolidColor(double r, double g, double b) : albedo_(r, g, b) {}
  TextureKind Kind() const override { return TextureKind::kSolid; }
  const core::Color& albedo() const { return albedo_; }

 private:
  core::Color albedo_;
};

class CheckerTexture : public Texture {
 public:
  CheckerTexture(double scale, std::shared_ptr<Texture> even, std::shared_ptr<Texture> odd)
      : inv_scale_(1.0 / scale), even_(std::move(even)), odd_(std::move(odd)) {}
  CheckerTexture(double scale, const core::Color& c1, const core::Color& c2)
      : CheckerTexture(scale, std::make_shared<SolidColor>(c1), std::make_shared<SolidColor>(c2)) {}
  TextureKind Kind() const override { return TextureKind::kChecker; }
  double inv_scale() const { return inv_scale_; }
  const std::shared_ptr<Texture>& even() const { return even_; }
  const std::shared_ptr<Texture>& odd() const { return odd_; }

 private:
  double inv_scale_;
  std::shared_ptr<Texture> even_, odd_;
};

class ImageTexture : public Texture {
 public:
  // the file name is resolved like image.cc:16-41 (as given, then the asset directories)
  explicit ImageTexture(const char* filename);
  TextureKind Kind() const override { return TextureKind::kImage; }
  const scene::Image& image() const { return *image_; }
  const std::string& name() const { return name_; }

 private:
  std::string name_;
  std::shared_ptr<scene::Image> image_;
};

enum class MaterialKind { kLambertian = RTX_MAT_LAMBERTIAN, kMetal = RTX_MAT_METAL, kDielectric = RTX_MAT_DIELECTRIC,
                          kDiffuseLight = RTX_MAT_DIFFUSE_LIGHT };

class Material {
 public:
  virtual ~Material() = default;
  virtual MaterialKind Kind() const = 0;
  // material.h:22 / material.cc:98,175,283 (Metal, Dielectric, DiffuseLight are specular)
  virtual bool IsSpecular() const { return Kind() != MaterialKind::kLambertian; }
};

class Lambertian : public Material {
 public:
  explicit Lambertian(const core::Color& albedo) : tex_(std::make_shared<SolidColor>(albedo)) {}
  explicit Lambertian(std::shared_ptr<Texture> tex) : tex_(std::move(tex)) {}
  MaterialKind Kind() const override { return MaterialKind::kLambertian; }
  const std::shared_ptr<Texture>& texture() const { return tex_; }

 private:
  std::shared_ptr<Texture> tex_;
};

class Metal : public Material {
 public:
  Metal(const core::Color& albedo, double fuzz) : albedo_(albedo), fuzz_(fuzz < 1.0 ? fuzz : 1.0) {}
  MaterialKind Kind() const override { return MaterialKind::kMetal; }
  const core::Color& albedo() const { return albedo_; }
  double fuzz() const { return fuzz_; }

 private:
  core::Color albedo_;
  double fuzz_;
};

class Dielectric : public Material {
 public:
  explicit Dielectric(double index) : ref_idx_(index) {}
  MaterialKind Kind() const override { return MaterialKind::kDielectric; }
  double ref_idx() const { return ref_idx_; }

 private:
  double ref_idx_;
};

class DiffuseLight : public Material {
 public:
  explicit DiffuseLight(std::shared_ptr<Texture> tex) : emit_(std::move(tex)) {}
  explicit DiffuseLight(const core::Color& c) : emit_(std::make_shared<SolidColor>(c)) {}
  MaterialKind Kind() const override { return MaterialKind::kDiffuseLight; }
  const std::shared_ptr<Texture>& texture() const { return emit_; }

 private:
  std::shared_ptr<Texture> emit_;
};

}  // namespace rt::material
