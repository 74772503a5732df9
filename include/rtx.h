/* include/rtx.h — C ABI of the MI355X-native path-tracing hot path (lib: librtx.so).
 *
 * This is the drop-in boundary for Luke-TS/3360-ray-tracer's per-pixel Monte Carlo path
 * tracer.  Plain C: POD structs, pointers and sizes, int status codes (RTX_OK == 0) and a
 * thread-local rtx_last_error() string.  No C++, no torch, no HIP types in the signatures.
 *
 * Reference interfaces each entry point replaces (paths under the reference's src/):
 *   rtx_intersect / rtx_intersect_device
 *       RayIntegrator::IntersectBatch(const vector<Ray>&, vector<HitRecord>&)
 *       integrator/ray_integrator.h:30-37; CPU version cpu_ray_integrator.h:18-46
 *       (interval fixed to [0.001f, +inf) there: pass tmin = RTX_SEAM_TMIN).
 *   rtx_render / rtx_render_device
 *       WavefrontRenderer(world, cam, integrator, max_depth, max_samples, batch).Render()
 *       renderer/wavefront.h:22-45, renderer/wavefront.cc:40-242 (mode RTX_MODE_WAVEFRONT);
 *       MegaKernel(scene, camera, DefaultSampler).Render()
 *       renderer/mega_kernel.h:10-59 + integrator/sampler.h:22-34 (mode RTX_MODE_MEGAKERNEL).
 *   rtx_scene_create
 *       the GPU hooks of the reference: Bvh::nodes()/prim_indices()/primitives() +
 *       BvhNodeGPU (geom/bvh.h:20-25,134-136), HittableType (geom/hittable.h:45-49).
 *   rtx_camera_init
 *       Camera::SetFromConfig + Camera::Initialize (scene/camera.h:84-131).
 *   rtx_host_scene_* (host-side scene assembly, no GPU work)
 *       scene::Scene::Add (scene/scene.h:26-33), geom::Bvh(Scene&) SAH build
 *       (geom/bvh.h:31-68,166-367), load_obj (load_obj.h:10-55), main.cc scene recipes.
 *
 * Ownership: the library copies everything it needs; it never retains caller pointers
 * past the call.  Output buffers are caller-allocated.
 * Threading: one rtx_scene per device; calls on different scenes (devices) may run
 * concurrently from different host threads; calls on one scene are serialised by the
 * caller.  Errors: every function returns RTX_OK or a negative RTX_ERR_*; the message is
 * in rtx_last_error() (thread-local).  HIP failures are reported, never swallowed; there
 * is no CPU fallback.
 */
#ifndef RTX_H_
#define RTX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 9  /* 2: rtx_stats.node_bytes; 3: rtx_stats.parked, RTX_FLAG_PARK / NO_PARK;
                              4: rtx_stats.build, RTX_FLAG_GENERIC, rtx_render_multi;
                              5: RTX_FLAG_LEAF_STEP, RTX_BUILD_SPECULATIVE; 6: rtx_stats.rays_recorded;
                              7: RTX_FLAG_ADAPT_PHASES (the adaptive tile schedule is the default),
                              rtx_stats.wave_rounds / wave_rounds_idle;
                              8: RTX_FLAG_ADAPT_TILES (the phase schedule is the default again);
                              9: the tile schedule removed (flag bit 64 reserved, ignored) */

enum {
  RTX_OK = 0,
  RTX_ERR_INVALID = -1, /* bad argument / descriptor */
  RTX_ERR_HIP = -2,     /* HIP runtime or kernel failure */
  RTX_ERR_NODEVICE = -3,
  RTX_ERR_IO = -4,      /* file not found / parse error (host scene helpers) */
  RTX_ERR_NOMEM = -5
};

/* IntersectBatch's interval minimum: float(0.001) as a double (cpu_ray_integrator.h:21). */
#define RTX_SEAM_TMIN 0.0010000000474974513

/* ---- scene description (host memory, flattened) ---------------------------------- */

/* BvhNodeGPU (geom/bvh.h:20-25): bbox in double, pre-order layout (left child = idx+1). */
typedef struct {
  double lo[3], hi[3];
  uint32_t left_first;  /* internal: left child index; leaf: first primitive (leaf order) */
  uint32_t right_count; /* internal: right child index; leaf: primitive count */
  uint32_t is_leaf;
  uint32_t pad_;
} rtx_bvh_node; /* 64 bytes */

enum { /* HittableType (geom/hittable.h:45-49) split per rect axis */
  RTX_PRIM_SPHERE = 0,   /* g: center[3], radius                  (geom/sphere.h) */
  RTX_PRIM_TRIANGLE = 1, /* g: a[3], b[3], c[3]                   (geom/triangle.h) */
  RTX_PRIM_XY_RECT = 2,  /* g: x0 x1 y0 y1 k                      (geom/rect.h:9-47) */
  RTX_PRIM_XZ_RECT = 3,  /* g: x0 x1 z0 z1 k                      (geom/rect.h:53-91) */
  RTX_PRIM_YZ_RECT = 4   /* g: y0 y1 z0 z1 k                      (geom/rect.h:97-135) */
};
typedef struct {
  int32_t kind;
  int32_t material;
  double g[9];
} rtx_prim; /* 80 bytes */

enum { RTX_TEX_SOLID = 0, RTX_TEX_CHECKER = 1, RTX_TEX_IMAGE = 2 }; /* material/texture.h */
typedef struct {
  int32_t kind;
  int32_t even, odd; /* checker children (texture ids) */
  int32_t image;     /* image id for RTX_TEX_IMAGE; -1 = no data (cyan, texture.h:62) */
  double color[3];   /* solid */
  double inv_scale;  /* checker: 1/scale */
} rtx_texture;

typedef struct {
  int32_t width, height;
  const uint8_t* texels; /* RGB8 after Image::FloatToByte (scene/image.cc:43-73), rows top-down */
} rtx_image;

enum { /* material/material.h */
  RTX_MAT_LAMBERTIAN = 0,
  RTX_MAT_METAL = 1,
  RTX_MAT_DIELECTRIC = 2,
  RTX_MAT_DIFFUSE_LIGHT = 3
};
typedef struct {
  int32_t kind;
  int32_t texture;  /* lambertian albedo / diffuse-light emission */
  double albedo[3]; /* metal */
  double fuzz;      /* metal, already clamped to <= 1 (material.cc:78-80) */
  double ref_idx;   /* dielectric */
} rtx_material;

typedef struct {
  const rtx_prim* prims; /* in BVH leaf order when nodes != NULL, else list order */
  int64_t n_prims;
  const rtx_bvh_node* nodes; /* NULL: the root is a flat list (scene::Scene::Hit) */
  int64_t n_nodes;
  const rtx_material* materials;
  int32_t n_materials;
  const rtx_texture* textures;
  int32_t n_textures;
  const rtx_image* images;
  int32_t n_images;
} rtx_scene_desc;

typedef struct rtx_scene rtx_scene; /* device-resident scene, one per device */

/* ---- rays and hit records (IntersectBatch seam) ----------------------------------- */

typedef struct {
  double origin[3];
  double direction[3]; /* not normalised (ray.h) */
} rtx_ray;             /* 48 bytes, = core::Ray */

typedef struct {
  int32_t hit;
  int32_t front_face;
  int32_t material; /* replaces HitRecord::mat (shared_ptr): index into the material table */
  int32_t pad_;
  double t;
  double p[3];
  double normal[3]; /* faces against the ray (hittable.h:31-34) */
  double u, v;      /* triangles do not write u,v (triangle.h:77-84): 0 unless stale */
} rtx_hit;          /* 88 bytes, = geom::HitRecord */

/* ---- camera ------------------------------------------------------------------------ */

typedef struct { /* CameraConfig (scene/camera.h:25-38) */
  double aspect_ratio;
  int32_t image_width;
  int32_t samples_per_pixel;
  int32_t max_depth;
  int32_t pad_;
  double vfov;
  double lookfrom[3], lookat[3], vup[3];
  double defocus_angle;
  double focus_dist;
} rtx_camera_config;

typedef struct { /* Camera after Initialize() (scene/camera.h:100-131) */
  double center[3], pixel00[3], pixel_delta_u[3], pixel_delta_v[3];
  double u[3], v[3], w[3];
  double defocus_disk_u[3], defocus_disk_v[3];
  double defocus_angle;
  int32_t image_width, image_height;
} rtx_camera;

/* ---- rendering --------------------------------------------------------------------- */

enum {
  RTX_MODE_WAVEFRONT = 0,  /* WavefrontRenderer semantics, bounce-synchronous queues */
  RTX_MODE_PERSISTENT = 1, /* same semantics, persistent kernel with per-lane refill */
  RTX_MODE_MEGAKERNEL = 2  /* MegaKernel + DefaultSampler semantics (Scatter API) */
};
enum {
  RTX_PREC_PARITY = 0, /* f64 everywhere, reference traversal order (bvh.h:71-119) */
  RTX_PREC_FAST = 1    /* conservative f32 traversal, near-child first; f64 hit + shading */
};

typedef struct {
  int32_t spp;              /* max_samples (passes) */
  int32_t max_depth;
  int32_t adaptive;         /* 1: adaptive sampling.  WAVEFRONT/PERSISTENT: the renderer's
                               PixelState test (pixel_state.h:54-72); MEGAKERNEL:
                               AdaptiveSampler(min_spp, spp, rel_threshold) (sampler.h:44-82,
                               up to spp + 1 samples); 0: fixed spp / DefaultSampler */
  int32_t min_spp;          /* adaptive: kMinSamples (wavefront.cc:43) = 16 | min_samples_ */
  double rel_threshold;     /* adaptive: kRelThresh (float 0.05, wavefront.cc:42) | threshold_ */
  uint64_t seed;            /* Philox key: results depend on (seed, pixel, sample) only */
  int32_t mode;             /* RTX_MODE_* */
  int32_t precision;        /* RTX_PREC_* */
  /* pixel subset: interleaved row stripes (stripe_rows > 0) or a rectangle */
  int32_t stripe_rows, stripe_index, stripe_count;
  int32_t x0, y0, w, h;     /* rectangle (w == 0 -> whole image) */
  int32_t samples_per_group;/* samples in flight per pixel (0 = auto) */
  int32_t flags;            /* RTX_FLAG_* */
} rtx_render_params;

enum {
  RTX_FLAG_COUNT = 1,  /* count BVH node visits / primitive tests (diagnostic build of the kernel) */
  /* RTX_MODE_PERSISTENT + RTX_PREC_FAST schedule (results are identical either way): by
     default the first such render of a scene times both on a centre tile and keeps the
     faster for the scene; these flags force one */
  RTX_FLAG_PARK = 2,   /* park long traversals and resume them in the next segment round */
  RTX_FLAG_NO_PARK = 4, /* every traversal runs to completion within its round */
  /* RTX_MODE_PERSISTENT: run the generic kernel build, without the per-scene
     specialisations (same results; for measuring what the specialisations buy) */
  RTX_FLAG_GENERIC = 8,
  /* the PARK schedule's traversal: the speculative walk (queued leaf tests) by default on
     trees of at most 65536 BVH4 nodes, the leaf-step walk on larger ones; this flag asks for
     the leaf-step walk on every tree (same results) */
  RTX_FLAG_LEAF_STEP = 16,
  /* RTX_MODE_PERSISTENT adaptive renders (samples_per_group 0): one launch per phase over a
     device-wide slot map (the default; this flag names it explicitly) */
  RTX_FLAG_ADAPT_PHASES = 32
  /* 64: reserved (ABI <= 8: the adaptive tile schedule, removed; ignored) */
};

/* rtx_stats.build: which persistent-kernel build ran (the per-scene specialisations compile
   out code paths the scene cannot reach; every build gives identical results) */
enum {
  RTX_BUILD_PARK = 1,           /* parked-traversal schedule */
  RTX_BUILD_SPHERE_TREE = 2,    /* leaf tests for spheres only (every tree primitive a sphere) */
  RTX_BUILD_TRIANGLE_TREE = 4,  /* leaf tests for triangles only */
  RTX_BUILD_LAMBERTIAN = 8,     /* shading for Lambertian materials only */
  RTX_BUILD_NO_TEXTURES = 16,   /* no texture lookups (every colour in the material table) */
  RTX_BUILD_NO_DEFOCUS = 32,    /* no thin-lens camera sampling (defocus_angle <= 0) */
  RTX_BUILD_FAST = 64,          /* RTX_PREC_FAST traversal */
  RTX_BUILD_COUNT = 128,        /* diagnostic counting build */
  RTX_BUILD_SCATTER = 256,      /* MegaKernel (Scatter API) semantics */
  RTX_BUILD_SPECULATIVE = 512   /* PARK schedule with the speculative walk (else the leaf-step walk) */
};

typedef struct {
  uint64_t rays_primary;   /* segments at depth 0 */
  uint64_t rays_total;     /* all segments handed to closest-hit (= IntersectBatch count) */
  uint64_t paths;          /* samples recorded */
  double kernel_ms;        /* device time of the render (HIP events) */
  double hot_kernel_ms;    /* device time inside the dominant (trace) kernel */
  uint64_t hot_launches;
  uint64_t node_visits;    /* with RTX_FLAG_COUNT */
  uint64_t prim_tests;     /* with RTX_FLAG_COUNT */
  uint64_t node_bytes;     /* bytes of one BVH node visit in the traversal used (64 BVH2, 128 BVH4) */
  uint64_t wave_node_iters; /* with RTX_FLAG_COUNT, fast BVH4: node-loop iterations per wave (SIMD efficiency */
  uint64_t wave_prim_iters; /*   = node_visits / (64 * wave_node_iters)); primitive-loop iterations per wave */
  uint64_t tri_tests;       /* with RTX_FLAG_COUNT: triangle / sphere tests among prim_tests (rest: rects) */
  uint64_t sphere_tests;
  uint64_t parked;          /* 1: the persistent fast schedule that parks long traversals ran */
  uint64_t build;           /* RTX_BUILD_* bits of the persistent kernel build (0: wavefront mode) */
  uint64_t rays_recorded;   /* with RTX_FLAG_COUNT: segments of the samples the pixels recorded.  Fixed spp:
                               = rays_total.  Adaptive RTX_MODE_PERSISTENT renders with automatic grouping
                               (samples_per_group 0; the tile or phase schedule) trace some samples past a
                               pixel's convergence and discard them: counted per sample.  Other adaptive
                               renders (wavefront, megakernel, explicit samples_per_group): 0 (not
                               counted).  0 without RTX_FLAG_COUNT */
  uint64_t wave_rounds;      /* with RTX_FLAG_COUNT, persistent mode: rounds of the waves' loop (refill,
                                segment), and those in which a wave had no path to trace (waiting for work) */
  uint64_t wave_rounds_idle;
  uint64_t wave_lanes_live;  /* with RTX_FLAG_COUNT, persistent mode: lanes holding a path, summed over the
                                rounds that trace (/ (64 x tracing rounds) = the rounds' lane occupancy) */
} rtx_stats;

/* ---- entry points ------------------------------------------------------------------ */

int rtx_abi_version(void);
const char* rtx_last_error(void);
int rtx_device_count(int* n);

int rtx_scene_create(int device, const rtx_scene_desc* desc, rtx_scene** out);
int rtx_scene_destroy(rtx_scene* scene);

/* Batch closest hit on [tmin, tmax); host buffers (PCIe round trip included). */
int rtx_intersect(rtx_scene* scene, const rtx_ray* rays, size_t n, rtx_hit* hits, double tmin, double tmax,
                  int32_t precision);
/* Same on device-resident buffers; stream is a hipStream_t (NULL = the scene's stream). */
int rtx_intersect_device(rtx_scene* scene, const rtx_ray* d_rays, size_t n, rtx_hit* d_hits, double tmin,
                         double tmax, int32_t precision, void* stream);

int rtx_camera_init(const rtx_camera_config* cfg, rtx_camera* out);

/* Render the pixel subset selected by params.  out_rgb: linear sum/(float)samples, double,
 * 3 per pixel, packed in subset order (rectangle row-major, or stripes in row order);
 * out_spp: samples per pixel (may be NULL).  Host buffers. */
int rtx_render(rtx_scene* scene, const rtx_camera* cam, const rtx_render_params* params, double* out_rgb,
               int32_t* out_spp, rtx_stats* stats);
/* Number of pixels rtx_render writes for these params. */
int64_t rtx_render_pixel_count(const rtx_camera* cam, const rtx_render_params* params);
/* Device-resident variant: out buffers are device pointers; asynchronous on stream. */
int rtx_render_device(rtx_scene* scene, const rtx_camera* cam, const rtx_render_params* params,
                      double* d_out_rgb, int32_t* d_out_spp, rtx_stats* stats, void* stream);

/* One frame over several devices: the image's rows are split into interleaved
 * stripes of params->stripe_rows rows (0: 8), and scenes[k] renders stripe
 * params->stripe_index + k of params->stripe_count (stripe_count <= 0: n stripes, from 0), each
 * from its own host thread on its scene's stream.  The stripes come back to the host and are
 * placed at their rows of out_rgb (W x H x 3, the whole frame; a pinned buffer receives them by
 * DMA, a pageable one through pinned staging) and out_spp (W x H, may be NULL); rows of other
 * stripes are not written, so several processes may fill one shared framebuffer.  Replaces
 * WavefrontRenderer::Render()'s one framebuffer (renderer/wavefront.cc:228-241) for G GPUs.
 * One scene per device is the intended use (rtx_scene_create on each; the same description);
 * a scene may not appear twice.  The RNG is keyed by the global pixel, so the image is
 * bit-identical for every n and split.  stats: counters summed, times = max over scenes;
 * per_scene (n entries) may be NULL. */
int rtx_render_multi(rtx_scene* const* scenes, int32_t n, const rtx_camera* cam, const rtx_render_params* params,
                     double* out_rgb, int32_t* out_spp, rtx_stats* stats, rtx_stats* per_scene);

/* ---- host-side scene assembly (C++ host library, no GPU) --------------------------- */

typedef struct rtx_host_scene rtx_host_scene;
/* Parse a .rtxs scene file (see DESIGN.md "Scene files"); image/obj paths relative to asset_dir. */
int rtx_host_scene_load(const char* path, const char* asset_dir, rtx_host_scene** out);
/* Build one of the reference's scene recipes: three, cornell, final, bunny, mixed (seeded). */
int rtx_host_scene_recipe(const char* name, uint32_t seed, const char* asset_dir, rtx_host_scene** out);
int rtx_host_scene_write(const rtx_host_scene* s, const char* path);
/* Flattened description; pointers stay valid until rtx_host_scene_destroy. */
int rtx_host_scene_desc(const rtx_host_scene* s, rtx_scene_desc* out);
/* prim_indices (Bvh::prim_indices, bvh.h:135) of the SAH build; n = n_prims. */
int rtx_host_scene_prim_indices(const rtx_host_scene* s, int32_t* out, int64_t n);
int rtx_host_scene_destroy(rtx_host_scene* s);

/* Image::Load (scene/image.cc:16-73; stb_image's stbi_loadf + FloatToByte): decode an image
   file — JPEG (sequential or progressive, 8-bit, 1/3/4 components) or binary PNM (P5/P6) — to
   the RGB8 texels image textures sample (width * height * 3 bytes, rows top-down).
   linear8 = 1: the 8-bit decode before the gamma-2.2 / FloatToByte step (stbi_load's bytes).
   texels == NULL: only *width / *height.  RTX_ERR_IO for an unreadable or unsupported file. */
int rtx_image_load(const char* path, int32_t linear8, int32_t* width, int32_t* height, uint8_t* texels,
                   size_t cap);

/* cameras.json preset -> config (parseCamera/loadCameras, scene/camera.h:40-67). */
int rtx_camera_config_load(const char* json_path, const char* preset, rtx_camera_config* out);

/* ---- BVH build (SURVEY §8f "GPU BVH build"; bvh.h:39-68,166-367) -------------------- */
/* Reference BoundingBox of each primitive (n x 6 doubles: lo xyz, hi xyz), host-side. */
int rtx_prim_bounds(const rtx_prim* prims, int64_t n, double* out_bounds);
/* Binned-SAH BVH over n primitive boxes (in the primitives' original order), built on the
   GPU.  Output is byte-identical to the host builder's (= the reference's Bvh::Build):
   out_nodes (capacity 2n) in pre-order, *out_n_nodes, out_prim_indices[n] (the permutation:
   leaf slot -> original primitive).  Host buffers; the device work is internal. */
int rtx_bvh_build(int device, const double* bounds, int64_t n, rtx_bvh_node* out_nodes, int64_t* out_n_nodes,
                  uint32_t* out_prim_indices);
/* The same build on the host (the C++ builder scene assembly uses); identical outputs. */
int rtx_bvh_build_host(const double* bounds, int64_t n, rtx_bvh_node* out_nodes, int64_t* out_n_nodes,
                       uint32_t* out_prim_indices);

/* ---- P3 PPM output encoded on the device (wavefront.cc:238-241 header + write_color,
 * core/color.h:18-33, per pixel; SURVEY §8f "on-GPU resolve + PPM output").  The bytes are
 * identical to rtx_write_ppm / the reference's Render() output. */
/* Upper bound of the P3 file size of a width x height image (header + 12 B per pixel). */
size_t rtx_p3_max_bytes(int32_t width, int32_t height);
/* Render like rtx_render and return the P3 file bytes of the rendered pixels (the tile /
   stripe subset: width x rows) in `out` (host, cap >= rtx_p3_max_bytes); *out_len = bytes.
   out_rgb (linear framebuffer) and out_spp are optional (NULL). */
int rtx_render_p3(rtx_scene* scene, const rtx_camera* cam, const rtx_render_params* params, char* out, size_t cap,
                  size_t* out_len, double* out_rgb, int32_t* out_spp, rtx_stats* stats);
/* P3 file bytes of a device-resident linear framebuffer (width x height x 3 doubles) into a
   device buffer d_out (cap >= rtx_p3_max_bytes); synchronizes `stream` to report *out_len. */
int rtx_encode_p3_device(rtx_scene* scene, const double* d_rgb, int32_t width, int32_t height, char* d_out,
                         size_t cap, size_t* out_len, void* stream);

/* P3 file bytes of a host linear framebuffer (width x height x 3 doubles), encoded on the
   scene's device (e.g. the gathered frame of rtx_render_multi); out: host, cap >=
   rtx_p3_max_bytes. */
int rtx_encode_p3(rtx_scene* scene, const double* rgb, int32_t width, int32_t height, char* out, size_t cap,
                  size_t* out_len);

/* write_color bytes (core/color.h:18-33) as a P3 PPM; rgb is a linear framebuffer (host). */
int rtx_write_ppm(const char* path, const double* rgb, int32_t width, int32_t height);

#ifdef __cplusplus
}
#endif
#endif /* RTX_H_ */
