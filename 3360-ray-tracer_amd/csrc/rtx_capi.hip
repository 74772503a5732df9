// rtx_capi.hip — C ABI (include/rtx.h) over the HIP kernels: scene upload, IntersectBatch,
// full-path render.  gfx950 only; no CPU compute path and no fallback: a missing device or a
// HIP error is returned as RTX_ERR_* with a message in rtx_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <atomic>
#include <chrono>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "rtx.h"
#include "rtx_frame_kernels.h"
#include "rtx_p3.h"
#include "rtx_scan.h"

using namespace rtxd;

// The PARK instantiations of k_persistent are compiled in rtx_park.hip (RTX_PARK_TU).
namespace rtxd {
#define RTX_PARK_EXTERN(ST, CO, SC, MP, PK)                                                                   \
  extern template __global__ void k_persistent<ST, true, CO, SC, PK, -1, false, false, false, MP>(RenderArgs, \
                                                                                              unsigned long long*);
RTX_PARK_INSTANCES(RTX_PARK_EXTERN)
#undef RTX_PARK_EXTERN
#define RTX_PARK_TRI_EXTERN(ST, MP, PK)                                                                             \
  extern template __global__ void k_persistent<ST, true, false, false, PK, RTX_PRIM_TRIANGLE, false, false, false, \
                                               MP>(RenderArgs, unsigned long long*);                              \
  extern template __global__ void k_persistent<ST, true, false, false, PK, RTX_PRIM_TRIANGLE, true, false, false,  \
                                               MP>(RenderArgs, unsigned long long*);                              \
  extern template __global__ void k_persistent<ST, true, false, false, PK, RTX_PRIM_TRIANGLE, true, true, false,   \
                                               MP>(RenderArgs, unsigned long long*);
RTX_PARK_TRI_INSTANCES(RTX_PARK_TRI_EXTERN)
#undef RTX_PARK_TRI_EXTERN
}  // namespace rtxd

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPC(expr)                                                                                   \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      return fail(RTX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_) + " (" __FILE__ ":" + \
                                   std::to_string(__LINE__) + ")");                                  \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  int reserve(size_t bytes) {
    if (bytes <= n) return RTX_OK;
    if (p) (void)hipFree(p);
    p = nullptr, n = 0;
    if (bytes == 0) return RTX_OK;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return fail(RTX_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    n = bytes;
    return RTX_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr, n = 0;
  }
  template <class T>
  T* as() const {
    return (T*)p;
  }
};

struct HostBuf {  // pinned host staging (grow-only)
  void* p = nullptr;
  size_t n = 0;
  int reserve(size_t bytes) {
    if (bytes <= n) return RTX_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr, n = 0;
    if (bytes == 0) return RTX_OK;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) return fail(RTX_ERR_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    n = bytes;
    return RTX_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr, n = 0;
  }
};

float round_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -INFINITY);
  return f;
}
float round_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, INFINITY);
  return f;
}

}  // namespace

// statistics, queue counts, then the slot counter block (8 region counters 128 B apart, [128 + 4]
// the segment buffer (0), ...)
constexpr int kSlotBlockWords = 8 * 16 + 8;
constexpr int kCounterWords = 64 + kSlotBlockWords;

// Where a render's output goes once a band of it is final (fixed-spp renders): the
// accumulate of the last sample group runs in kBands bands of the frame's pixels, and after
// each one `copy` enqueues that band's device-to-host copy on the copy stream, so the
// framebuffer crosses PCIe while the next band is still being summed.  Band edges are
// multiples of `align` pixels (whole stripes of the caller's layout).
struct BandSink {
  int64_t align;
  int (*copy)(void* ctx, int64_t p0, int64_t p1, hipStream_t cs);
  void* ctx;
  // Adaptive renders: the caller's whole-image host framebuffer as the device sees it (pinned,
  // mapped), or nullptr.  With it, the output goes to the host early, while the last phases
  // still run (copy stream), and the pixels those phases change are written into it by the
  // device at the end (k_patch_host) instead of a second whole-frame copy.
  double* host_rgb_dev = nullptr;
};
constexpr int64_t kEarlyOutDiv = 32;  // the early output once a phase holds at most npix / 32 pixels (4: C3 / C4 adaptive -0.7 %, r9j / r9k)
constexpr int kBands = 8;  // bands of the last accumulate and of the D2H copies that overlap them (ab_bands_*: 2 / 4 / 8 / 16)

// Adaptive renders in phases (render_adaptive)
// render_adaptive: the smallest phase planned while pixels remain (round 3: 2^23; with the pooled
// prediction 2^21, scripts/adaptive_sim.py and r05 r8j / r8k)
constexpr int64_t kAdaptPhaseSlots = 1 << 21;
constexpr double kAdaptMarginStep = 0.25;      // render_adaptive: batch margin 1 + step * (phase - 1) (0.5: within noise, r3y)
// Overrides of the adaptive schedules' constants (0: the default): rtx_internal_adapt_tune, a
// test and tuning hook (not in rtx.h) that forces small workspaces and floors, so the paths
// that only a large frame at a large budget reaches run on small frames too.
struct AdaptTune {
  int64_t phase_slots;  // phases: the smallest phase planned while pixels remain (kAdaptPhaseSlots)
  int phase_kcap;       // phases: the largest batch of one pixel (else from the workspace)
  int first_map;         // the uniform first pass: 1 the phase kernel (block-shared chunks), 0 the uniform-group one (< 0: default)
  double phase_mstep;    // phases: the batch margin's growth per phase (< 0: kAdaptMarginStep)
  double margin1;        // the margin of the batches after the first phase (< 0: kAdaptMargin1)
  double pool_w;         // the pooled prediction's centre weight (< 0: kAdaptPoolW; 0: not pooled)
};
static AdaptTune g_tune{0, 0, -1, -1.0, -1.0, -1.0};
// adaptive early outputs so far (renders whose output went to the host while phases still ran)
// and the pixels k_patch_host rewrote: rtx_internal_early_output_stats, a test hook
static std::atomic<long long> g_early_outputs{0}, g_early_patched{0};
// render_adaptive: the margin of the batches after the first phase, and k_adapt_plan's centre
// weight (0: each pixel's own prediction only): ranked first by scripts/adaptive_sim.py, then
// C3 adaptive +4.0 %, C2 +0.5 % against the unpooled margin 1.0 (r05 r8j / r8k)
constexpr double kAdaptMargin1 = 0.8;
constexpr double kAdaptPoolW = 8.0;
constexpr int kFirstPassMap = 1;  // the adaptive first pass runs the phase kernel (MAP 1, no slot map)
// RTX_DEBUG_HOST: host-side timestamps of a frame (render_stripes_to_host prints them, with the
// device; per thread: rtx_render_multi renders each device on a thread of its own)
static const bool g_debug_host = std::getenv("RTX_DEBUG_HOST") != nullptr;
static double host_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static thread_local double g_t_launch = 0, g_t_sync0 = 0, g_t_sync1 = 0;
struct AdaptWs {
  // lst / kl / ol: the phases' pixel lists (ping-pong: sub-pixel, samples, first slot per entry);
  // knext: the next batch per entry of the phase just traced; pk: their packed prefix sums
  // rv: each pixel's predicted convergence count at its last record (k_adapt_plan's pooling)
  DevBuf lbuf, smap, lst[2], kl[2], ol[2], knext, pk, rv, scan_tmp, ctr;  // ctr: 8 region slot counters (128 B apart), then u64 slot count, pixel count, slot map address, ..., [132] segment buffer, then the spread pixel counts (kSpreadBase)
  DevBuf segs;                                  // counting renders: each slot's path segments (u16)
  HostBuf total_h;                              // pinned copy of the next phase's slot count
  hipEvent_t ev = nullptr;                      // total_h written
  void release() {
    for (DevBuf* b : {&lbuf, &smap, &lst[0], &lst[1], &kl[0], &kl[1], &ol[0], &ol[1], &knext, &pk, &rv, &scan_tmp, &ctr,
                      &segs})
      b->release();
    total_h.release();
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
  }
};

struct rtx_scene {
  int device = 0;
  hipStream_t stream = nullptr;
  int cus = 0;
  DevBuf nodes, prims, mats, texs, images, fnodes, tri_n;
  DevBuf segs1;  // counting adaptive renders: the first phase's per-slot path segments (u16)
  std::vector<DevBuf> texels;
  DScene S{};
  int stack_parity = 32, stack_fast = 32;
  int fast_need = 0;     // exact worst-case stack depth of the lean BVH4 walk (build_fast4)
  size_t n_f4 = 0;       // F4Node count of the fast tree
  bool fast_ok = false;  // RTX_PREC_FAST available (BVH with an internal root)
  int park = -1;         // persistent fast schedule: -1 not yet timed, 0 plain kernel, 1 PARK kernel
  DevBuf calib_rgb;      // output of the schedule-timing renders
  int64_t n_nodes = 0;
  // render workspace (grow-only)
  DevBuf px_sum, px_mean, px_m2, px_samples, px_conv, lbuf, queue[2], counters, out_rgb, out_spp, rays, hits;
  DevBuf p3_scratch, p3_body;  // device P3 encoding (rtx_p3.h)
  DevBuf patch_q;              // adaptive early output: the pixels still sampling when it went
  HostBuf stage_rgb, stage_spp;  // rtx_render_multi: pinned D2H staging of this device's stripes
  HostBuf counters_h;            // timed renders: pinned copy of the statistics counters (read after the end event)
  // ev[0] / ev[1]: a timed render's start and end (rtx_stats.kernel_ms), ev[2] / ev[3]: the
  // adaptive debug timing, ev[4]: the frame and its output copy done (the host's wait)
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> evpool;
  // banded output copies (BandSink): a copy stream and its ordering events
  hipStream_t copy_stream = nullptr;
  std::vector<hipEvent_t> band_ev;
  AdaptWs aw;  // adaptive phases' workspace
  double slot_mem = -1.0;  // bytes the slot buffers may take (slot_target; -1: not yet queried)
  ~rtx_scene() {
    (void)hipSetDevice(device);
    aw.release();
    for (auto e : evpool) (void)hipEventDestroy(e);
    for (auto e : band_ev) (void)hipEventDestroy(e);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    (void)hipSetDevice(device);
    for (DevBuf* b : {&nodes, &prims, &mats, &texs, &images, &fnodes, &tri_n, &px_sum, &px_mean, &px_m2, &px_samples,
                      &px_conv, &lbuf, &queue[0], &queue[1], &counters, &out_rgb, &out_spp, &rays, &hits, &p3_scratch,
                      &p3_body, &calib_rgb, &patch_q})
      b->release();
    for (auto& t : texels) t.release();
    stage_rgb.release(), stage_spp.release();
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// Tree depth of the reference-layout BVH (pre-order, left = idx+1).
int bvh_depth(const rtx_bvh_node* n, int64_t count) {
  if (count == 0) return 0;
  std::vector<int> d(count, 0);
  int m = 1;
  for (int64_t i = 0; i < count; i++) {
    m = std::max(m, d[i] + 1);
    if (!n[i].is_leaf) {
      d[n[i].left_first] = d[i] + 1;
      d[n[i].right_count] = d[i] + 1;
    }
  }
  return m;
}

// Conservative f64 box of one primitive (fast-path leaf splitting).  Spheres: centre +-
// |r|; rects: the rectangle on its plane; triangles: the vertex box padded by 2^-19 of its
// largest extent, which covers the points the reference's float-rounded barycentric test
// accepts just outside the exact triangle (u, v, u + v within 2^-23 of the edges).
void prim_box(const rtx_prim& p, double lo[3], double hi[3]) {
  const double* g = p.g;
  if (p.kind == RTX_PRIM_SPHERE) {
    const double r = std::fabs(g[3]);
    for (int a = 0; a < 3; a++) lo[a] = g[a] - r, hi[a] = g[a] + r;
    return;
  }
  if (p.kind == RTX_PRIM_TRIANGLE) {
    double ext = 0;
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(g[a], std::min(g[3 + a], g[6 + a]));
      hi[a] = std::max(g[a], std::max(g[3 + a], g[6 + a]));
      ext = std::max(ext, hi[a] - lo[a]);
    }
    const double pad = std::ldexp(ext, -19);
    for (int a = 0; a < 3; a++) lo[a] -= pad, hi[a] += pad;
    return;
  }
  int ax, a0, a1;  // rect.h: XY (z = k), XZ (y = k), YZ (x = k)
  if (p.kind == RTX_PRIM_XY_RECT) ax = 2, a0 = 0, a1 = 1;
  else if (p.kind == RTX_PRIM_XZ_RECT) ax = 1, a0 = 0, a1 = 2;
  else ax = 0, a0 = 1, a1 = 2;
  lo[a0] = std::min(g[0], g[1]), hi[a0] = std::max(g[0], g[1]);
  lo[a1] = std::min(g[2], g[3]), hi[a1] = std::max(g[2], g[3]);
  lo[ax] = hi[ax] = g[4];
}

// BVH4 fast layout: the binary tree collapsed top-down.  Each F4Node starts from the binary
// node's two children and repeatedly opens the slot with the largest surface area until it
// holds four slots or nothing fits: an internal binary node opens into its two children, a
// leaf of 2-4 primitives into its primitives.  Every leaf slot of the result holds exactly
// ONE primitive with its own conservative box (prim_box), so the f32 slab test culls
// primitives before their f64 test and the kernel needs no per-slot counts: a leaf of
// several primitives left in a slot becomes a child F4Node of one-primitive slots (and a leaf
// of more than four, a small tree of them).  Empty slots carry an inverted box (lo = +inf,
// hi = -inf) that no ray enters.  Every slot keeps a box that contains all hits its
// primitives can report, rounded outward, so the candidate set is unchanged.
// Returns the exact worst-case traversal stack depth (trace_fast4 pushes at most
// `internal slots - 1` entries per visited node).
int build_fast4(const rtx_bvh_node* n, const rtx_prim* prims, std::vector<F4Node>& out) {
  out.clear();
  struct Slot {
    int kind;  // 0 binary node, 1 one primitive, 2 a primitive range emitted as a child node
    uint32_t id, count;  // kind 0: node; kind 1: primitive; kind 2: first primitive, count
    double lo[3], hi[3];
  };
  auto node_slot = [&](uint32_t b) {
    Slot s{0, b, 0, {}, {}};
    for (int a = 0; a < 3; a++) s.lo[a] = n[b].lo[a], s.hi[a] = n[b].hi[a];
    if (n[b].is_leaf && n[b].right_count >= 2) s.kind = 2, s.id = n[b].left_first, s.count = n[b].right_count;
    return s;
  };
  auto prim_slot = [&](uint32_t id) {
    Slot s{1, id, 1, {}, {}};
    prim_box(prims[id], s.lo, s.hi);
    return s;
  };
  auto area = [](const Slot& s) {
    const double dx = s.hi[0] - s.lo[0], dy = s.hi[1] - s.lo[1], dz = s.hi[2] - s.lo[2];
    return dx * dy + dy * dz + dz * dx;
  };
  // the slots of the child node a kind-2 range becomes: its primitives (<= 4), else four
  // contiguous sub-ranges with the union of their primitive boxes
  auto range_slots = [&](uint32_t first, uint32_t count) {
    std::vector<Slot> r;
    if (count <= 4) {
      for (uint32_t q = 0; q < count; q++) r.push_back(prim_slot(first + q));
      return r;
    }
    const uint32_t per = (count + 3) / 4;
    for (uint32_t g = first; g < first + count; g += per) {
      const uint32_t k = std::min(per, first + count - g);
      Slot sl{k == 1 ? 1 : 2, g, k, {INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
      for (uint32_t q = 0; q < k; q++) {
        double lo[3], hi[3];
        prim_box(prims[g + q], lo, hi);
        for (int a = 0; a < 3; a++) sl.lo[a] = std::min(sl.lo[a], lo[a]), sl.hi[a] = std::max(sl.hi[a], hi[a]);
      }
      r.push_back(sl);
    }
    return r;
  };
  // number of slots a slot opens into inside the current node (0: cannot open)
  auto fan = [&](const Slot& s) -> uint32_t {
    if (s.kind == 0) return n[s.id].is_leaf ? 0 : 2;
    if (s.kind == 2) return s.count <= 4 ? s.count : 0;
    return 0;
  };
  int need = 0;
  struct Item {
    std::vector<Slot> slots;
    int64_t parent_slot;
    int depth;
  };
  std::vector<Item> work;
  if (n[0].is_leaf) work.push_back({range_slots(n[0].left_first, n[0].right_count), -1, 0});
  else work.push_back({{node_slot(n[0].left_first), node_slot(n[0].right_count)}, -1, 0});
  while (!work.empty()) {
    Item it = std::move(work.back());
    work.pop_back();
    const int32_t me = (int32_t)out.size();
    if (it.parent_slot >= 0) out[it.parent_slot >> 2].child[it.parent_slot & 3] = me;
    out.push_back(F4Node{});
    std::vector<Slot>& slots = it.slots;
    while (slots.size() < 4) {
      int pick = -1;
      double best = -1.0;
      for (size_t k = 0; k < slots.size(); k++) {
        const uint32_t f = fan(slots[k]);
        if (f && slots.size() - 1 + f <= 4 && area(slots[k]) > best) best = area(slots[k]), pick = (int)k;
      }
      if (pick < 0) break;
      const Slot b = slots[pick];
      std::vector<Slot> rep;
      if (b.kind == 0) rep = {node_slot(n[b.id].left_first), node_slot(n[b.id].right_count)};
      else rep = range_slots(b.id, b.count);
      slots.erase(slots.begin() + pick);
      slots.insert(slots.begin() + pick, rep.begin(), rep.end());
    }
    int internal = 0;
    for (const Slot& sl : slots) internal += (sl.kind == 2 || (sl.kind == 0 && !n[sl.id].is_leaf)) ? 1 : 0;
    const int child_depth = it.depth + std::max(0, internal - 1);
    need = std::max(need, child_depth);
    F4Node& f = out[me];
    for (int c = 0; c < 4; c++) {
      if (c >= (int)slots.size() || (slots[c].kind == 0 && n[slots[c].id].is_leaf && n[slots[c].id].right_count == 0)) {
        f.child[c] = -1;  // empty slot: inverted box, never entered
        f.lox[c] = f.loy[c] = f.loz[c] = INFINITY;
        f.hix[c] = f.hiy[c] = f.hiz[c] = -INFINITY;
        continue;
      }
      const Slot& sl = slots[c];
      f.lox[c] = round_down(sl.lo[0]), f.loy[c] = round_down(sl.lo[1]), f.loz[c] = round_down(sl.lo[2]);
      f.hix[c] = round_up(sl.hi[0]), f.hiy[c] = round_up(sl.hi[1]), f.hiz[c] = round_up(sl.hi[2]);
      uint32_t first;
      if (sl.kind == 1) first = sl.id;
      else if (sl.kind == 0 && n[sl.id].is_leaf) first = n[sl.id].left_first;  // one-primitive binary leaf
      else continue;  // internal: patched when the child is emitted
      f.child[c] = ~(int32_t)first;
      f.counts[c >> 1] |= 1u << (16 * (c & 1));
    }
    // push in reverse so children are laid out in slot order (pre-order)
    for (int c = (int)slots.size() - 1; c >= 0; c--) {
      const Slot& sl = slots[c];
      if (sl.kind == 2) {
        work.push_back({range_slots(sl.id, sl.count), (int64_t)me * 4 + c, child_depth});
      } else if (sl.kind == 0 && !n[sl.id].is_leaf) {
        work.push_back({{node_slot(n[sl.id].left_first), node_slot(n[sl.id].right_count)}, (int64_t)me * 4 + c,
                        child_depth});
      }
    }
  }
  return need;
}

// Fast-path tree of our own: binned SAH on all three axes (32 bins)
// over the conservative primitive boxes (prim_box), split down to one primitive per leaf;
// the result uses the reference node layout (pre-order, leaf = one primitive by its index
// in the scene's prim array) so build_fast4 collapses it like the reference tree.  The
// fast path only needs the closest hit among the same primitives, which any conservative
// tree over them yields (up to exact ties), so the tree itself is free to differ.
struct SahItem {
  double lo[3], hi[3], c[3];
  uint32_t prim;
};
static double half_area(const double lo[3], const double hi[3]) {
  const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}
static int own_sah_node(std::vector<SahItem>& it, int b, int e, std::vector<rtx_bvh_node>& out) {
  const int me = (int)out.size();
  out.push_back(rtx_bvh_node{});
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = b; i < e; i++)
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], it[i].lo[a]), hi[a] = std::max(hi[a], it[i].hi[a]);
      clo[a] = std::min(clo[a], it[i].c[a]), chi[a] = std::max(chi[a], it[i].c[a]);
    }
  for (int a = 0; a < 3; a++) out[me].lo[a] = lo[a], out[me].hi[a] = hi[a];
  if (e - b == 1) {
    out[me].is_leaf = 1, out[me].left_first = it[b].prim, out[me].right_count = 1;
    return me;
  }
  constexpr int kB = 32;
  int best_axis = -1, best_plane = -1;
  double best = INFINITY;
  for (int a = 0; a < 3; a++) {
    const double ext = chi[a] - clo[a];
    if (!(ext > 0)) continue;
    int cnt[kB] = {0};
    double blo[kB][3], bhi[kB][3];
    for (int k = 0; k < kB; k++)
      for (int q = 0; q < 3; q++) blo[k][q] = INFINITY, bhi[k][q] = -INFINITY;
    const double sc = kB / ext;
    for (int i = b; i < e; i++) {
      const int k = std::min(kB - 1, std::max(0, (int)((it[i].c[a] - clo[a]) * sc)));
      cnt[k]++;
      for (int q = 0; q < 3; q++) blo[k][q] = std::min(blo[k][q], it[i].lo[q]), bhi[k][q] = std::max(bhi[k][q], it[i].hi[q]);
    }
    double rarea[kB];
    int rcnt[kB];
    double alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int n = 0;
    for (int k = kB - 1; k >= 1; k--) {
      n += cnt[k];
      for (int q = 0; q < 3; q++) alo[q] = std::min(alo[q], blo[k][q]), ahi[q] = std::max(ahi[q], bhi[k][q]);
      rcnt[k] = n, rarea[k] = n ? half_area(alo, ahi) : 0.0;
    }
    for (int q = 0; q < 3; q++) alo[q] = INFINITY, ahi[q] = -INFINITY;
    n = 0;
    for (int k = 0; k < kB - 1; k++) {
      n += cnt[k];
      for (int q = 0; q < 3; q++) alo[q] = std::min(alo[q], blo[k][q]), ahi[q] = std::max(ahi[q], bhi[k][q]);
      if (n == 0 || rcnt[k + 1] == 0) continue;
      const double cost = half_area(alo, ahi) * n + rarea[k + 1] * rcnt[k + 1];
      if (cost < best) best = cost, best_axis = a, best_plane = k;
    }
  }
  int mid;
  if (best_axis >= 0) {
    const double ext = chi[best_axis] - clo[best_axis], sc = kB / ext, c0 = clo[best_axis];
    auto m = std::partition(it.begin() + b, it.begin() + e, [&](const SahItem& x) {
      return std::min(kB - 1, std::max(0, (int)((x.c[best_axis] - c0) * sc))) <= best_plane;
    });
    mid = (int)(m - it.begin());
  } else {
    mid = (b + e) / 2;  // coincident centroids: split the list
  }
  if (mid == b || mid == e) mid = (b + e) / 2;
  const int l = own_sah_node(it, b, mid, out);
  const int r = own_sah_node(it, mid, e, out);
  out[me].is_leaf = 0, out[me].left_first = (uint32_t)l, out[me].right_count = (uint32_t)r;
  return me;
}
static void build_own_sah(const rtx_prim* prims, int64_t n, const int32_t* skip, int n_skip,
                          std::vector<rtx_bvh_node>& out) {
  std::vector<SahItem> it;
  it.reserve((size_t)n);
  for (int64_t i = 0; i < n; i++) {
    if (std::find(skip, skip + n_skip, (int32_t)i) != skip + n_skip) continue;
    SahItem x;
    prim_box(prims[i], x.lo, x.hi);
    for (int a = 0; a < 3; a++) x.c[a] = 0.5 * (x.lo[a] + x.hi[a]);
    x.prim = (uint32_t)i;
    it.push_back(x);
  }
  out.clear();
  out.reserve(2 * it.size());
  if (!it.empty()) own_sah_node(it, 0, (int)it.size(), out);
}

// Primitives the fast path tests outside its tree (DScene::global, trav_globals): up to two
// whose conservative box has at least the surface area of the union of all other
// primitives' boxes, i.e. a box that nearly every ray's walk would enter at the root anyway
// (the ground spheres of the final, bunny and mixed scenes: r = 1000 against a scene a few
// tens of units wide).  At least two primitives stay in the tree so its root is internal.
static int build_global_prims(const rtx_prim* prims, int64_t n, int32_t out[2]) {
  int k = 0;
  while (k < 2 && n - k > 2) {
    // largest remaining box, and the union of the others
    int64_t big = -1;
    double big_area = -1.0;
    for (int64_t i = 0; i < n; i++) {
      if (std::find(out, out + k, (int32_t)i) != out + k) continue;
      double lo[3], hi[3];
      prim_box(prims[i], lo, hi);
      const double a = half_area(lo, hi);
      if (a > big_area) big_area = a, big = i;
    }
    double ulo[3] = {INFINITY, INFINITY, INFINITY}, uhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; i++) {
      if (i == big || std::find(out, out + k, (int32_t)i) != out + k) continue;
      double lo[3], hi[3];
      prim_box(prims[i], lo, hi);
      for (int a = 0; a < 3; a++) ulo[a] = std::min(ulo[a], lo[a]), uhi[a] = std::max(uhi[a], hi[a]);
    }
    if (!(big >= 0 && std::isfinite(big_area) && big_area >= half_area(ulo, uhi))) break;
    out[k++] = (int32_t)big;
  }
  return k;
}

// The allowance of a scene's slot buffers (the radiance records of the samples in flight, the
// wavefront's path queues, the adaptive workspaces): half of the device memory that is free or
// already held by them, so several scenes on one device, or a smaller GPU, get smaller groups
// instead of RTX_ERR_NOMEM.  ONE allowance for all of them: a render keeps the other kinds'
// buffers (and, for an adaptive render, the radiance buffer beyond its first pass) only while
// they fit beside its own (render_device_impl releases them otherwise) and sizes its own within
// the allowance minus what those kept buffers take.  The free-memory query is made once
// per scene (the first render that sizes its slots; it costs ~0.5 ms, too much per frame):
// scenes created later see what the earlier ones took.
double slot_allowance(rtx_scene* sc) {
  if (sc->slot_mem < 0) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
      (void)hipGetLastError();
      fr = (size_t)1 << 62;
    }
    double held = (double)sc->lbuf.n + (double)sc->queue[0].n + (double)sc->queue[1].n + (double)sc->segs1.n;
    held += (double)sc->aw.lbuf.n + (double)sc->aw.smap.n + (double)sc->aw.segs.n;
    sc->slot_mem = 0.5 * ((double)fr + held);
  }
  return sc->slot_mem;
}
// Slots a render keeps in flight: `want`, within the allowance less `other` bytes the render's
// other slot buffers take.
int64_t slot_target(rtx_scene* sc, int64_t bytes_per_slot, int64_t want, double other = 0.0) {
  const double mem = std::max(0.0, slot_allowance(sc) - other);
  return std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)(mem / (double)bytes_per_slot)));
}

int pick_stack(int depth) {
  if (depth + 2 <= 32) return 32;
  if (depth + 2 <= 64) return 64;
  return -1;
}

template <class T>
int upload(DevBuf& b, const T* src, size_t n, hipStream_t s) {
  int rc = b.reserve(std::max<size_t>(n * sizeof(T), 16));
  if (rc) return rc;
  if (n) HIPC(hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, s));
  return RTX_OK;
}

int64_t subset_pixels(const rtx_camera* cam, const rtx_render_params* p, PixelMap& m, std::string& err) {
  m.W = cam->image_width, m.H = cam->image_height;
  if (m.W <= 0 || m.H <= 0) {
    err = "camera not initialised (image size <= 0)";
    return -1;
  }
  if ((int64_t)m.W * m.H > 0x7FFFFFFFll) {  // pixel indices are 32-bit on the device
    err = "image larger than 2^31 pixels";
    return -1;
  }
  if (p->stripe_rows > 0) {
    if (p->stripe_count <= 0 || p->stripe_index < 0 || p->stripe_index >= p->stripe_count) {
      err = "bad stripe_index/stripe_count";
      return -1;
    }
    m.stripes = 1, m.srows = p->stripe_rows, m.sidx = p->stripe_index, m.scount = p->stripe_count;
    int64_t rows = 0;
    for (int y = 0; y < m.H; y++)
      if ((y / m.srows) % m.scount == m.sidx) rows++;
    m.x0 = m.y0 = 0, m.w = m.W, m.h = (int)rows;
    set_map_div(m);
    return rows * (int64_t)m.W;
  }
  m.stripes = 0;
  m.x0 = p->x0, m.y0 = p->y0, m.w = p->w, m.h = p->h;
  if (m.w == 0 && m.h == 0) m.x0 = 0, m.y0 = 0, m.w = m.W, m.h = m.H;
  if (m.x0 < 0 || m.y0 < 0 || m.w < 0 || m.h < 0 || m.x0 + m.w > m.W || m.y0 + m.h > m.H) {
    err = "tile outside the image";
    return -1;
  }
  m.srows = 1, m.sidx = 0, m.scount = 1;
  set_map_div(m);
  return (int64_t)m.w * m.h;
}

template <int STACK, bool FAST>
int launch_intersect(rtx_scene* sc, const rtx_ray* d_rays, int64_t n, rtx_hit* d_hits, double tmin, double tmax,
                     hipStream_t s) {
  const int64_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL((k_intersect<STACK, FAST>), dim3((unsigned)blocks), dim3(kBlock),
                     stack_lds_bytes(STACK), s, sc->S, d_rays, n, d_hits, tmin, tmax);
  HIPC(hipGetLastError());
  return RTX_OK;
}

int persistent_grid(rtx_scene* sc, const void* fn, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  return std::max(1, per_cu) * sc->cus;
}


struct Launch {
  rtx_scene* sc;
  hipStream_t s;
  int stack;
  bool fast, count;
  int park = 0;  // persistent: 0 plain kernel, PARK kernel (parked traversals) with 1 the leaf-step, 2 the speculative walk
  bool generic = false;  // RTX_FLAG_GENERIC: no per-scene specialisation (TK, LAMB, NOTEX, NODOF)
  int map = 0;           // k_persistent MAP: 0 uniform groups, 1 an adaptive phase's slot map
  mutable uint32_t build = 0;  // RTX_BUILD_* bits of the persistent instantiation launched last
};

template <int STACK, bool FAST, bool COUNT>
int run_extend(const Launch& L, const RenderArgs& A, const PathQueue& q, const unsigned* cnt, int64_t max_items) {
  const size_t lds = stack_lds_bytes(STACK);
  const int64_t need = (max_items + kBlock - 1) / kBlock;
  const int grid = (int)std::max<int64_t>(
      1, std::min<int64_t>(need, persistent_grid(L.sc, (const void*)k_wf_extend<STACK, FAST, COUNT>, lds)));
  hipLaunchKernelGGL((k_wf_extend<STACK, FAST, COUNT>), dim3(grid), dim3(kBlock), lds, L.s, A, q, cnt);
  HIPC(hipGetLastError());
  return RTX_OK;
}

template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK, int TK, bool LAMB, bool NOTEX, bool NODOF,
          int MAP>
int run_persistent_k1(const Launch& L, const RenderArgs& A, unsigned long long* next_slot) {
  if (A.stack_slots < 1 || A.stack_slots > STACK + 1) return fail(RTX_ERR_INVALID, "bad traversal stack size");
  const size_t lds = persist_lds(A.stack_slots, spec_walk(PARK, FAST, SCATTER), block_region_kind(MAP, SCATTER)).end;
  int grid = persistent_grid(
      L.sc, (const void*)k_persistent<STACK, FAST, COUNT, SCATTER, PARK, TK, LAMB, NOTEX, NODOF, MAP>, lds);
  L.build = (PARK ? RTX_BUILD_PARK : 0u) | (PARK == 2 ? RTX_BUILD_SPECULATIVE : 0u) | (TK == (int)RTX_PRIM_SPHERE ? RTX_BUILD_SPHERE_TREE : 0u) |
            (TK == (int)RTX_PRIM_TRIANGLE ? RTX_BUILD_TRIANGLE_TREE : 0u) | (LAMB ? RTX_BUILD_LAMBERTIAN : 0u) |
            (NOTEX ? RTX_BUILD_NO_TEXTURES : 0u) | (NODOF ? RTX_BUILD_NO_DEFOCUS : 0u) |
            (FAST ? RTX_BUILD_FAST : 0u) | (COUNT ? RTX_BUILD_COUNT : 0u) | (SCATTER ? RTX_BUILD_SCATTER : 0u);
  if (std::getenv("RTX_DEBUG_LAUNCH"))
    fprintf(stderr, "rtx launch: k_persistent build 0x%x grid %d (%d blocks per CU) lds %zu B stack_slots %d\n",
            L.build, grid, grid / std::max(1, L.sc->cus), lds, A.stack_slots);
  hipLaunchKernelGGL((k_persistent<STACK, FAST, COUNT, SCATTER, PARK, TK, LAMB, NOTEX, NODOF, MAP>), dim3(grid),
                     dim3(kBlock), lds, L.s, A, next_slot);
  HIPC(hipGetLastError());
  return RTX_OK;
}
// adaptive renders draw their slots from a slot map (L.map; never with the scatter API)
template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK, int TK, bool LAMB = false, bool NOTEX = false,
          bool NODOF = false>
int run_persistent_k0(const Launch& L, const RenderArgs& A, unsigned long long* next_slot) {
  if (!SCATTER && L.map == 1)
    return run_persistent_k1<STACK, FAST, COUNT, SCATTER, PARK, TK, LAMB, NOTEX, NODOF, SCATTER ? 0 : 1>(L, A, next_slot);
  if (L.map) return fail(RTX_ERR_INVALID, "slot maps are not used with the scatter API");
  return run_persistent_k1<STACK, FAST, COUNT, SCATTER, PARK, TK, LAMB, NOTEX, NODOF, 0>(L, A, next_slot);
}
// the texture-free plain build also comes without the camera's thin-lens sampling (defocus
// off; C2 +1.0 %; the PARK build lost 2.8 % with it, ab_nodof_*)
template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK, int TK, bool LAMB = false, bool NOTEX = false>
int run_persistent_k(const Launch& L, const RenderArgs& A, unsigned long long* next_slot) {
  if (NOTEX && !PARK && A.cam.defocus_angle <= 0)
    return run_persistent_k0<STACK, FAST, COUNT, SCATTER, PARK, TK, LAMB, NOTEX, NOTEX && !PARK>(L, A, next_slot);
  return run_persistent_k0<STACK, FAST, COUNT, SCATTER, PARK, TK, LAMB, NOTEX>(L, A, next_slot);
}
// fast frames of a scene whose tree holds one kind run a build for that kind: triangles with
// the PARK schedule (the bunny), spheres with the plain one (the final and mixed scenes)
template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK>
int run_persistent(const Launch& L, const RenderArgs& A, unsigned long long* next_slot) {
  constexpr bool spec = FAST && !COUNT && !SCATTER;
  constexpr int TK = spec ? (PARK ? (int)RTX_PRIM_TRIANGLE : (int)RTX_PRIM_SPHERE) : -1;
  if (TK >= 0 && A.S.tree_kind == TK && !L.generic) {
    // the triangle (PARK) build also comes for all-Lambertian scenes (the bunny)
    if (TK == (int)RTX_PRIM_TRIANGLE && A.S.all_lambertian) {
      constexpr bool tri = TK == (int)RTX_PRIM_TRIANGLE;
      if (A.S.no_textures) return run_persistent_k<STACK, FAST, COUNT, SCATTER, PARK, TK, tri, tri>(L, A, next_slot);
      return run_persistent_k<STACK, FAST, COUNT, SCATTER, PARK, TK, tri>(L, A, next_slot);
    }
    // the sphere (plain) build also comes for scenes that read no textures (the final scene)
    if (TK == (int)RTX_PRIM_SPHERE && A.S.no_textures)
      return run_persistent_k<STACK, FAST, COUNT, SCATTER, PARK, TK, false, TK == (int)RTX_PRIM_SPHERE>(L, A,
                                                                                                       next_slot);
    return run_persistent_k<STACK, FAST, COUNT, SCATTER, PARK, TK>(L, A, next_slot);
  }
  return run_persistent_k<STACK, FAST, COUNT, SCATTER, PARK, -1>(L, A, next_slot);
}

// template dispatch helpers
template <bool FAST, bool COUNT>
int extend_s(const Launch& L, const RenderArgs& A, const PathQueue& q, const unsigned* c, int64_t n) {
  return L.stack == 32 ? run_extend<32, FAST, COUNT>(L, A, q, c, n) : run_extend<64, FAST, COUNT>(L, A, q, c, n);
}
int extend(const Launch& L, const RenderArgs& A, const PathQueue& q, const unsigned* c, int64_t n) {
  if (L.fast) return L.count ? extend_s<true, true>(L, A, q, c, n) : extend_s<true, false>(L, A, q, c, n);
  return L.count ? extend_s<false, true>(L, A, q, c, n) : extend_s<false, false>(L, A, q, c, n);
}
template <bool FAST, bool COUNT, bool SCATTER, int PARK>
int persist_s(const Launch& L, const RenderArgs& A, unsigned long long* ns) {
  return L.stack == 32 ? run_persistent<32, FAST, COUNT, SCATTER, PARK>(L, A, ns)
                       : run_persistent<64, FAST, COUNT, SCATTER, PARK>(L, A, ns);
}
template <bool SCATTER>
int persist_m(const Launch& L, const RenderArgs& A, unsigned long long* ns) {
  constexpr int kSpec = SCATTER ? 1 : 2;  // (the scatter API never runs the PARK kernel)
  if (L.fast && L.park == 2 && !SCATTER)
    return L.count ? persist_s<true, true, SCATTER, kSpec>(L, A, ns) : persist_s<true, false, SCATTER, kSpec>(L, A, ns);
  if (L.fast && L.park && !SCATTER)
    return L.count ? persist_s<true, true, SCATTER, 1>(L, A, ns) : persist_s<true, false, SCATTER, 1>(L, A, ns);
  if (L.fast)
    return L.count ? persist_s<true, true, SCATTER, 0>(L, A, ns) : persist_s<true, false, SCATTER, 0>(L, A, ns);
  return L.count ? persist_s<false, true, SCATTER, 0>(L, A, ns) : persist_s<false, false, SCATTER, 0>(L, A, ns);
}

int time_park_schedule(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, hipStream_t s);

// Bytes of an adaptive render's uniform first pass (min_spp samples of every pixel): its
// radiance records, and in counting renders their segment counts, in the scene's buffers.
double adaptive_first_bytes(int64_t npix, const rtx_render_params* prm, int budget, bool count) {
  const int K1 = std::min(std::max(1, prm->min_spp), budget);
  return (double)npix * K1 * (3 * sizeof(double) + (count ? 2 : 0));
}

// Counting renders: the persistent launch's slot counter block names the buffer its paths'
// segment counts go to (k_persistent COUNT builds read word 8 * 16 + 4 of it).
int set_segbuf(unsigned long long* ctr, uint16_t* segs, hipStream_t st) {
  const unsigned long long v = (unsigned long long)(uintptr_t)segs;
  uint32_t* w = (uint32_t*)(ctr + 8 * 16 + 4);  // (two 32-bit memsets: stream-ordered, no host staging)
  HIPC(hipMemsetD32Async((hipDeviceptr_t)w, (int)(uint32_t)v, 1, st));
  HIPC(hipMemsetD32Async((hipDeviceptr_t)(w + 1), (int)(uint32_t)(v >> 32), 1, st));
  return RTX_OK;
}
// Adaptive sampling on the persistent kernel: the reference's WavefrontRenderer::Render loop
// (wavefront.cc:57-225, always adaptive) with the same per-pixel results, on the caller's
// stream `s`.  Phase 1 traces min_spp samples of every pixel (one uniform launch) and
// k_adapt_record replays them and sizes each pixel's next batch.  After each phase, record +
// next batch sizes (k_adapt_record, k_adapt_floor); before each phase, prefix sum and slot map
// (k_adapt_expand); the host reads the next phase's slot count (one pinned word) to launch it
// or stop; every phase is a launch of its own with its own drain.
// `mark` records a hot-kernel timing event (before and after each persistent launch);
// hot_launches counts them.  The caller resolves the pixels (k_resolve).
template <class Mark, class Early>
int render_adaptive(rtx_scene* sc, const Launch& L, const RenderArgs& A, const rtx_render_params* prm,
                    const PixelSoA& px, int budget, double other, hipStream_t s, Mark mark, uint64_t& hot_launches,
                    Early early) {
  const int64_t npix = A.npix;
  const int K1 = std::min(std::max(1, prm->min_spp), budget);
  static const bool debug = std::getenv("RTX_DEBUG_ADAPT") != nullptr;  // per-phase slot counts on stderr
  const int64_t phase_slots = g_tune.phase_slots > 0 ? g_tune.phase_slots : kAdaptPhaseSlots;
  if ((int64_t)npix * K1 > 0xFFFFFFFFll) return fail(RTX_ERR_INVALID, "adaptive render: npix x min_spp above 2^32");
  AdaptWs& w = sc->aw;
  int rc;
  // the uniform first pass's radiance (and segment) records, in the scene's buffers
  const double first_bytes = adaptive_first_bytes(npix, prm, budget, L.count);
  // slots after the first phase: 24 B of radiance + 8 B of slot map each (+ 2 B of segments),
  // within the allowance less the first pass and what the render keeps of other buffers
  const int64_t cap = std::min<int64_t>(
      0xFFFFFFFFll, slot_target(sc, 32 + (L.count ? 2 : 0), 1ll << kSlotTargetLog2, first_bytes + other));
  if (npix * 4 > cap) return fail(RTX_ERR_NOMEM, "adaptive render: too many pixels for the device memory");
  int32_t kcap = (int32_t)std::min<int64_t>(budget, std::max<int64_t>(4, (cap / npix) & ~3ll));
  if (g_tune.phase_kcap > 0) kcap = std::min(kcap, g_tune.phase_kcap);
  {
    const int64_t slots = npix * (int64_t)kcap;
    if ((rc = w.lbuf.reserve(slots * 3 * sizeof(double)))) return rc;
    if (L.count && (rc = w.segs.reserve(slots * sizeof(uint16_t)))) return rc;
    if ((rc = w.smap.reserve(slots * sizeof(uint2)))) return rc;
    for (DevBuf* b : {&w.lst[0], &w.lst[1], &w.kl[0], &w.kl[1], &w.ol[0], &w.ol[1], &w.knext})
      if ((rc = b->reserve(npix * sizeof(uint32_t)))) return rc;
    if ((rc = w.pk.reserve(npix * sizeof(unsigned long long)))) return rc;
    if ((rc = w.rv.reserve(npix * sizeof(float)))) return rc;
    if ((rc = w.scan_tmp.reserve(std::max<size_t>(16, rtxscan::temp_bytes_packed(npix))))) return rc;
    if ((rc = w.ctr.reserve(kAdaptCtrWords * sizeof(unsigned long long)))) return rc;
    if ((rc = w.total_h.reserve(2 * sizeof(unsigned long long)))) return rc;
    if (!w.ev) HIPC(hipEventCreateWithFlags(&w.ev, hipEventDisableTiming));
  }
  unsigned long long* ctr = w.ctr.as<unsigned long long>();  // 8 region counters, then the slot count, ...
  // record + next batch sizes after phase g (its slots in Lph: the uniform first phase's, or the
  // phase's slot map; its `active` pixels in its list), then the next phase's prefix sum, slot
  // map, pixel list and (to the host) slot and pixel counts
  auto record = [&](int g, const double* Lph, int64_t active) -> int {
    AdaptPlan ap;
    ap.list = g == 1 ? nullptr : w.lst[g & 1].as<uint32_t>();
    ap.kcur = g == 1 ? nullptr : w.kl[g & 1].as<uint32_t>();
    ap.off = g == 1 ? nullptr : w.ol[g & 1].as<uint32_t>();
    ap.knext = w.knext.as<uint32_t>();
    ap.kuni = K1, ap.sub_n = 1, ap.sub_j = 0;
    ap.min_spp = prm->min_spp, ap.budget = budget, ap.phase = g, ap.kcap = kcap;
    // a phase of at least ~phase_slots slots while pixels remain: once few pixels are left,
    // their batches grow (up to the budget) instead of phases that are mostly launch tail
    ap.kmin = (int32_t)std::min<int64_t>(budget, (phase_slots + active - 1) / std::max<int64_t>(1, active));
    ap.rel = prm->rel_threshold;
    ap.margin_step = g_tune.phase_mstep >= 0 ? g_tune.phase_mstep : kAdaptMarginStep;
    ap.margin1 = g_tune.margin1 >= 0 ? g_tune.margin1 : kAdaptMargin1;
    ap.pool_w = (float)(g_tune.pool_w >= 0 ? g_tune.pool_w : kAdaptPoolW);
    ap.rv = w.rv.as<float>();
    ap.width = std::max(1, A.map.stripes ? A.map.W : A.map.w);  // (the render's own rows)
    ap.segs = !L.count ? nullptr : g == 1 ? sc->segs1.as<uint16_t>() : w.segs.as<uint16_t>();
    ap.rec_segs = A.counters + 9;
    ap.next_active = ctr + kSpreadBase;
    // (ap.next_active was zeroed with the phase's slot counter block, k_slot_block_init)
    const int64_t n = active;  // entries of the phase's list
    hipLaunchKernelGGL(k_adapt_record, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, px, Lph, n, npix, ap);
    HIPC(hipGetLastError());
    if (ap.pool_w > 0.0f) {
      hipLaunchKernelGGL(k_adapt_plan, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, px, n, npix, ap);
      HIPC(hipGetLastError());
    }
    hipLaunchKernelGGL(k_adapt_floor, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ap.knext, ap.list,
                       n, 1, 0, (const int32_t*)px.samples, budget, kcap, phase_slots,
                       (const unsigned long long*)ap.next_active, ctr + 8 * 16 + 1);
    HIPC(hipGetLastError());
    HIPC(rtxscan::exclusive_scan_packed(ap.knext, w.pk.as<uint64_t>(), n, w.scan_tmp.p, w.scan_tmp.n, s));
    const AdaptList next{w.lst[(g + 1) & 1].as<uint32_t>(), w.kl[(g + 1) & 1].as<uint32_t>(),
                         w.ol[(g + 1) & 1].as<uint32_t>()};
    hipLaunchKernelGGL(k_adapt_expand, dim3((unsigned)((n + kExpandPix - 1) / kExpandPix)), dim3(kBlock), 0, s,
                       (const uint32_t*)ap.knext, (const unsigned long long*)w.pk.as<unsigned long long>(), ap.list, n,
                       1, 0, (const int32_t*)px.samples, w.smap.as<uint2>(), next, ctr + 8 * 16);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(w.total_h.p, ctr + 8 * 16, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPC(hipEventRecord(w.ev, s));
    return RTX_OK;
  };
  // one persistent launch of a phase; debug: its time and segments on stderr
  // uniform: the launch's slot count (no slot map: uniform groups); 0: the slot map's, from k_adapt_expand
  auto launch = [&](int g, const Launch& Lg, const RenderArgs& Ag, uint16_t* segs, int64_t pixels,
                    uint64_t uniform = 0) -> int {
    unsigned long long seg0 = 0;
    hipLaunchKernelGGL(k_slot_block_init, dim3(1), dim3(8 * 16), 0, s, ctr, uniform ? 1 : 0,
                       (unsigned long long)uniform, 0ull);
    HIPC(hipGetLastError());
    if (debug) {
      HIPC(hipStreamSynchronize(s));
      HIPC(hipMemcpy(&seg0, A.counters, sizeof seg0, hipMemcpyDeviceToHost));
      HIPC(hipEventRecord(sc->ev[2], s));
    }
    int rc2;
    if (debug) HIPC(hipMemsetAsync(A.counters + 13, 0, 5 * sizeof(unsigned long long), s));  // (the timeline)
    if ((rc2 = mark(s))) return rc2;
    if (L.count && (rc2 = set_segbuf(ctr, segs, s))) return rc2;
    if ((rc2 = persist_m<false>(Lg, Ag, ctr))) return rc2;
    L.build = Lg.build;  // (the stats report the instantiation launched last)
    if ((rc2 = mark(s))) return rc2;
    hot_launches++;
    if (debug) {
      HIPC(hipEventRecord(sc->ev[3], s));
      HIPC(hipEventSynchronize(sc->ev[3]));
      float ms = 0;
      unsigned long long seg1 = 0;
      HIPC(hipEventElapsedTime(&ms, sc->ev[2], sc->ev[3]));
      HIPC(hipMemcpy(&seg1, A.counters, sizeof seg1, hipMemcpyDeviceToHost));
      unsigned long long tt[18] = {};
      HIPC(hipMemcpy(tt, A.counters, sizeof tt, hipMemcpyDeviceToHost));
      if (tt[13]) {  // counting build: the launch's timeline (us from the first block's start)
        const double t0 = (double)~tt[13];
        auto us = [&](unsigned long long v) { return ((double)v - t0) / 100.0; };
        fprintf(stderr, "rtx adaptive: phase %d timeline: slots used up %.1f .. %.1f us, waves end %.1f .. %.1f us\n",
                g, us(~tt[15]), us(tt[14]), us(~tt[17]), us(tt[16]));
      }
      fprintf(stderr, "rtx adaptive: phase %d: %lld pixels, launch %.3f ms, %llu segments (%.0f Mseg/s)\n", g,
              (long long)pixels, ms, seg1 - seg0, (double)(seg1 - seg0) / (ms * 1e3));
    }
    return RTX_OK;
  };
  // phase 1: min_spp samples of every pixel, one uniform launch over the whole render (the
  // scene's radiance buffer)
  if ((rc = sc->lbuf.reserve((size_t)npix * K1 * 3 * sizeof(double)))) return rc;
  if (L.count && (rc = sc->segs1.reserve((size_t)npix * K1 * sizeof(uint16_t)))) return rc;
  RenderArgs A1 = A;
  A1.L = sc->lbuf.as<double>();
  A1.conv = nullptr;
  A1.K = K1, A1.s0 = 0, A1.fK = make_fastdiv((uint32_t)K1);
  // the phase kernel without a slot map (uniform groups: slot p * K1 + k), for its block-shared
  // chunks: the first pass ends as the phases do, its last slots traced by whole blocks
  Launch L1 = L;
  const bool first_map1 = (g_tune.first_map >= 0 ? g_tune.first_map : kFirstPassMap) == 1;
  if (first_map1) L1.map = 1;
  if ((rc = launch(1, L1, A1, sc->segs1.as<uint16_t>(), npix, first_map1 ? (uint64_t)npix * (uint64_t)K1 : 0)))
    return rc;
  if ((rc = record(1, sc->lbuf.as<double>(), npix))) return rc;
  RenderArgs Ag = A;
  Ag.L = w.lbuf.as<double>();
  Ag.conv = nullptr;    // only pixels still sampling have slots
  Ag.K = 1, Ag.s0 = 0, Ag.fK = make_fastdiv(1u);  // (unused: slots from the phase's slot map)
  Launch Lg = L;
  Lg.map = 1;
  for (int g = 2;; g++) {
    // this phase's slot count, computed at the end of the previous one
    HIPC(hipEventSynchronize(w.ev));
    const unsigned long long nsl = ((const volatile unsigned long long*)w.total_h.p)[0];
    const int64_t active = (int64_t)((const volatile unsigned long long*)w.total_h.p)[1];
    if (nsl == 0) break;
    // the output once few pixels are left: every other pixel is final (phase g's list holds the
    // rest, and later phases' lists are subsets of it)
    if ((rc = early(g, active, w.lst[g & 1].as<uint32_t>()))) return rc;
    if ((rc = launch(g, Lg, Ag, w.segs.as<uint16_t>(), active))) return rc;
    if ((rc = record(g, Ag.L, active))) return rc;
  }
  return RTX_OK;
}

}  // namespace

extern "C" {

int rtx_abi_version(void) { return RTX_ABI_VERSION; }
const char* rtx_last_error(void) { return g_err.c_str(); }
void rtx_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }

int rtx_device_count(int* n) {
  if (!n) return fail(RTX_ERR_INVALID, "n is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return fail(RTX_ERR_NODEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *n = c;
  return RTX_OK;
}

int rtx_scene_create(int device, const rtx_scene_desc* d, rtx_scene** out) {
  if (!d || !out) return fail(RTX_ERR_INVALID, "NULL argument");
  *out = nullptr;
  if (d->n_prims < 0 || d->n_nodes < 0 || d->n_materials < 0 || d->n_textures < 0 || d->n_images < 0)
    return fail(RTX_ERR_INVALID, "negative counts");
  if (d->n_prims > 0 && !d->prims) return fail(RTX_ERR_INVALID, "prims is NULL");
  if (d->n_materials > 0 && !d->materials) return fail(RTX_ERR_INVALID, "materials is NULL");
  if (d->n_textures > 0 && !d->textures) return fail(RTX_ERR_INVALID, "textures is NULL");
  if (d->n_images > 0 && !d->images) return fail(RTX_ERR_INVALID, "images is NULL");
  if (d->n_nodes > 0 && !d->nodes) return fail(RTX_ERR_INVALID, "nodes is NULL");
  if (d->n_prims > 0x7FFFFFFFll) return fail(RTX_ERR_INVALID, "more than 2^31-1 primitives");
  // validate indices so kernels never read out of bounds
  for (int64_t i = 0; i < d->n_prims; i++) {
    const rtx_prim& p = d->prims[i];
    if (p.kind < RTX_PRIM_SPHERE || p.kind > RTX_PRIM_YZ_RECT) return fail(RTX_ERR_INVALID, "bad primitive kind");
    if (p.material < 0 || p.material >= d->n_materials) return fail(RTX_ERR_INVALID, "primitive material out of range");
  }
  for (int32_t i = 0; i < d->n_materials; i++) {
    const rtx_material& m = d->materials[i];
    if (m.kind < 0 || m.kind > RTX_MAT_DIFFUSE_LIGHT) return fail(RTX_ERR_INVALID, "bad material kind");
    if ((m.kind == RTX_MAT_LAMBERTIAN || m.kind == RTX_MAT_DIFFUSE_LIGHT) && (m.texture < 0 || m.texture >= d->n_textures))
      return fail(RTX_ERR_INVALID, "material texture out of range");
  }
  for (int32_t i = 0; i < d->n_textures; i++) {
    const rtx_texture& t = d->textures[i];
    // the device treats every kind other than solid / checker as an image lookup
    if (t.kind < RTX_TEX_SOLID || t.kind > RTX_TEX_IMAGE) return fail(RTX_ERR_INVALID, "bad texture kind");
    if (t.kind == RTX_TEX_CHECKER && (t.even < 0 || t.even >= d->n_textures || t.odd < 0 || t.odd >= d->n_textures))
      return fail(RTX_ERR_INVALID, "checker child out of range");
    if (t.kind == RTX_TEX_IMAGE && t.image >= d->n_images) return fail(RTX_ERR_INVALID, "image index out of range");
  }
  for (int32_t i = 0; i < d->n_images; i++) {
    const rtx_image& im = d->images[i];
    if (im.width < 0 || im.height < 0) return fail(RTX_ERR_INVALID, "negative image size");
    if ((int64_t)im.width * im.height > (1ll << 31)) return fail(RTX_ERR_INVALID, "image above 2^31 texels");
  }
  for (int64_t i = 0; i < d->n_nodes; i++) {
    const rtx_bvh_node& n = d->nodes[i];
    if (n.is_leaf) {
      if ((int64_t)n.left_first + n.right_count > d->n_prims) return fail(RTX_ERR_INVALID, "leaf range out of bounds");
    } else if (n.left_first >= d->n_nodes || n.right_count >= d->n_nodes || n.left_first <= i || n.right_count <= i) {
      return fail(RTX_ERR_INVALID, "child index out of bounds (nodes must be pre-order)");
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RTX_ERR_NODEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return fail(RTX_ERR_INVALID, "device out of range");
  auto sc = std::make_unique<rtx_scene>();
  sc->device = device;
  HIPC(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPC(hipGetDeviceProperties(&prop, device));
  sc->cus = prop.multiProcessorCount;
  HIPC(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
  for (auto& e : sc->ev) HIPC(hipEventCreate(&e));
  hipStream_t s = sc->stream;
  int rc;
  // Triangle normals for the hit records (Triangle::Hit, triangle.h:80-82: Normalize(Cross(
  // edge1, edge2))), formed here in the device's double operations and order (cross, len2,
  // sqrt, 1 / l, products; no contraction), so the table holds the very bits finish_hit_at
  // would compute per hit.
  bool any_tri = false;
  for (int64_t i = 0; i < d->n_prims && !any_tri; i++) any_tri = d->prims[i].kind == RTX_PRIM_TRIANGLE;
  if (any_tri) {
    std::vector<double> tn((size_t)d->n_prims * 4, 0.0);
    for (int64_t i = 0; i < d->n_prims; i++) {
      const rtx_prim& q = d->prims[i];
      if (q.kind != RTX_PRIM_TRIANGLE) continue;
      double e1[3], e2[3];
      for (int a = 0; a < 3; a++) e1[a] = q.g[3 + a] - q.g[a], e2[a] = q.g[6 + a] - q.g[a];
      const double c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                           e1[0] * e2[1] - e1[1] * e2[0]};
      const double l = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
      if (l == 0.0) continue;  // normalize() returns (0, 0, 0)
      const double inv = 1.0 / l;
      for (int a = 0; a < 3; a++) tn[4 * (size_t)i + a] = inv * c[a];
    }
    if ((rc = upload(sc->tri_n, tn.data(), tn.size(), s))) return rc;
    HIPC(hipStreamSynchronize(s));  // tn is a temporary
  }
  {  // device table: triangles carry A, B - A, C - A (tri_e1 / tri_e2)
    std::vector<rtx_prim> dp(d->prims, d->prims + d->n_prims);
    for (rtx_prim& q : dp)
      if (q.kind == RTX_PRIM_TRIANGLE)
        for (int a = 0; a < 3; a++) q.g[3 + a] = q.g[3 + a] - q.g[a], q.g[6 + a] = q.g[6 + a] - q.g[a];
    if ((rc = upload(sc->prims, dp.data(), dp.size(), s))) return rc;
    HIPC(hipStreamSynchronize(s));  // dp is a temporary: the copy must finish before it goes
  }
  // Device copy of the material table: a Lambertian / DiffuseLight whose texture is a
  // SolidColor carries the colour itself (texture = -1, colour in the unused albedo field),
  // so shading skips the dependent texture-table load (mat_tex, rtx_device.h).
  std::vector<rtx_material> dmats(d->materials, d->materials + d->n_materials);
  for (rtx_material& m : dmats) {
    if ((m.kind == RTX_MAT_LAMBERTIAN || m.kind == RTX_MAT_DIFFUSE_LIGHT) && m.texture >= 0 &&
        d->textures[m.texture].kind == RTX_TEX_SOLID) {
      for (int c = 0; c < 3; c++) m.albedo[c] = d->textures[m.texture].color[c];
      m.texture = -1;
    }
  }
  // Dielectric: eta on a front-face hit (eta_i / eta_t = 1 / ri) and Schlick's r0 for
  // reflectance(c, ri) (material.cc:226-262) in the unused albedo field, computed with the same
  // IEEE double operations the kernel would perform (shade_merged, rtx_device.h).
  for (rtx_material& m : dmats) {
    if (m.kind != RTX_MAT_DIELECTRIC) continue;
    const double ri = m.ref_idx;
    double r0 = (1.0 - ri) / (1.0 + ri);
    r0 = r0 * r0;
    m.albedo[0] = 1.0 / ri;
    m.albedo[1] = r0;
  }
  if ((rc = upload(sc->mats, dmats.data(), d->n_materials, s))) return rc;
  if ((rc = upload(sc->texs, d->textures, d->n_textures, s))) return rc;
  std::vector<DImage> imgs(d->n_images);
  sc->texels.resize(d->n_images);
  for (int32_t i = 0; i < d->n_images; i++) {
    const rtx_image& im = d->images[i];
    imgs[i].w = im.width, imgs[i].h = im.height, imgs[i].texels = nullptr;
    if (im.width > 0 && im.height > 0 && im.texels) {
      if ((rc = upload(sc->texels[i], im.texels, (size_t)im.width * im.height * 3, s))) return rc;
      imgs[i].texels = sc->texels[i].as<uint8_t>();
    } else {
      imgs[i].w = imgs[i].h = 0;
    }
  }
  if ((rc = upload(sc->images, imgs.data(), imgs.size(), s))) return rc;
  sc->n_nodes = d->nodes ? d->n_nodes : 0;
  std::vector<F4Node> f4;
  int32_t global[2] = {0, 0};
  int n_global = 0;
  if (d->nodes && d->n_nodes > 0) {
    if ((rc = upload(sc->nodes, d->nodes, d->n_nodes, s))) return rc;
    const int depth = bvh_depth(d->nodes, d->n_nodes);
    sc->stack_parity = pick_stack(depth);
    sc->stack_fast = sc->stack_parity;
    if (sc->stack_parity < 0) return fail(RTX_ERR_INVALID, "BVH deeper than 62 levels");
    if (!d->nodes[0].is_leaf) {
      // the fast path's tree: our own binned SAH tree over the primitives (without the global
      // ones), collapsed to BVH4 (r01: +2 % C2 / bunny, +6 % C5 over collapsing the reference's)
      std::vector<rtx_bvh_node> own;
      n_global = build_global_prims(d->prims, d->n_prims, global);
      build_own_sah(d->prims, d->n_prims, global, n_global, own);
      const int need = build_fast4(own.data(), d->prims, f4);
      sc->stack_fast = need < 0 ? -1 : (need <= 32 ? 32 : (need <= 64 ? 64 : -1));
      sc->fast_need = need;
      sc->n_f4 = f4.size();
      if (sc->stack_fast > 0 && (rc = upload(sc->fnodes, f4.data(), f4.size(), s))) return rc;
      sc->fast_ok = sc->stack_fast > 0;
    }
  }
  HIPC(hipStreamSynchronize(s));
  DScene& S = sc->S;
  S.nodes = sc->nodes.as<rtx_bvh_node>();
  S.prims = sc->prims.as<rtx_prim>();
  S.tri_n = sc->tri_n.p ? sc->tri_n.as<double>() : nullptr;
  S.mats = sc->mats.as<rtx_material>();
  S.texs = sc->texs.as<rtx_texture>();
  S.images = sc->images.as<DImage>();
  S.f4nodes = (f4.empty() || !sc->fast_ok) ? nullptr : sc->fnodes.as<FastNode>();
  S.use_bvh = (d->nodes && d->n_nodes > 0) ? 1 : 0;
  S.n_prims = S.use_bvh ? d->n_prims : d->n_prims;
  S.froot_leaf = 0, S.froot_count = 0;
  S.has_tris = 0;
  S.n_global = sc->fast_ok ? n_global : 0;
  S.all_lambertian = d->n_materials > 0 ? 1 : 0;
  for (int32_t i = 0; i < d->n_materials && S.all_lambertian; i++)
    S.all_lambertian = d->materials[i].kind == RTX_MAT_LAMBERTIAN;
  S.no_textures = 1;
  for (const rtx_material& m : dmats)
    if ((m.kind == RTX_MAT_LAMBERTIAN || m.kind == RTX_MAT_DIFFUSE_LIGHT) && m.texture >= 0) S.no_textures = 0;
  S.tree_kind = -1;
  if (sc->fast_ok && d->n_prims > 0) {  // the one kind of the tree's primitives (globals excluded)
    int k = -2;
    for (int64_t i = 0; i < d->n_prims && k != -1; i++) {
      if ((n_global > 0 && global[0] == i) || (n_global > 1 && global[1] == i)) continue;
      k = k == -2 ? d->prims[i].kind : (k == d->prims[i].kind ? k : -1);
    }
    S.tree_kind = k < 0 ? -1 : k;
  }
  S.global[0] = global[0], S.global[1] = global[1];
  for (int64_t i = 0; i < d->n_prims && !S.has_tris; i++) S.has_tris = d->prims[i].kind == RTX_PRIM_TRIANGLE;
  if (S.use_bvh && d->nodes[0].is_leaf) S.froot_leaf = 1, S.froot_count = (int32_t)d->nodes[0].right_count;
  if (!d->nodes && d->n_nodes == 0) S.use_bvh = 0;
  *out = sc.release();
  return RTX_OK;
}

int rtx_scene_destroy(rtx_scene* s) {
  delete s;
  return RTX_OK;
}

int rtx_intersect_device(rtx_scene* sc, const rtx_ray* d_rays, size_t n, rtx_hit* d_hits, double tmin, double tmax,
                         int32_t precision, void* stream) {
  if (!sc) return fail(RTX_ERR_INVALID, "scene is NULL");
  if (n == 0) return RTX_OK;
  if (!d_rays || !d_hits) return fail(RTX_ERR_INVALID, "NULL buffer");
  HIPC(hipSetDevice(sc->device));
  hipStream_t s = stream ? (hipStream_t)stream : sc->stream;
  const bool fast = precision == RTX_PREC_FAST && sc->fast_ok;
  const int st = fast ? sc->stack_fast : sc->stack_parity;
  if (fast) return st == 32 ? launch_intersect<32, true>(sc, d_rays, (int64_t)n, d_hits, tmin, tmax, s)
                            : launch_intersect<64, true>(sc, d_rays, (int64_t)n, d_hits, tmin, tmax, s);
  return st == 32 ? launch_intersect<32, false>(sc, d_rays, (int64_t)n, d_hits, tmin, tmax, s)
                  : launch_intersect<64, false>(sc, d_rays, (int64_t)n, d_hits, tmin, tmax, s);
}

int rtx_intersect(rtx_scene* sc, const rtx_ray* rays, size_t n, rtx_hit* hits, double tmin, double tmax,
                  int32_t precision) {
  if (!sc) return fail(RTX_ERR_INVALID, "scene is NULL");
  if (n == 0) return RTX_OK;
  if (!rays || !hits) return fail(RTX_ERR_INVALID, "NULL buffer");
  HIPC(hipSetDevice(sc->device));
  int rc;
  if ((rc = sc->rays.reserve(n * sizeof(rtx_ray)))) return rc;
  if ((rc = sc->hits.reserve(n * sizeof(rtx_hit)))) return rc;
  HIPC(hipMemcpyAsync(sc->rays.p, rays, n * sizeof(rtx_ray), hipMemcpyHostToDevice, sc->stream));
  if ((rc = rtx_intersect_device(sc, sc->rays.as<rtx_ray>(), n, sc->hits.as<rtx_hit>(), tmin, tmax, precision,
                                 sc->stream)))
    return rc;
  HIPC(hipMemcpyAsync(hits, sc->hits.p, n * sizeof(rtx_hit), hipMemcpyDeviceToHost, sc->stream));
  HIPC(hipStreamSynchronize(sc->stream));
  return RTX_OK;
}

// Camera::Initialize (camera.h:100-131), same operation order as the reference.
int rtx_camera_init(const rtx_camera_config* c, rtx_camera* o) {
  if (!c || !o) return fail(RTX_ERR_INVALID, "NULL argument");
  if (c->image_width <= 0 || !(c->aspect_ratio > 0)) return fail(RTX_ERR_INVALID, "bad image width / aspect ratio");
  const double kPiH = 3.14159265358979323846;
  auto sub = [](const double* a, const double* b, double* r) { for (int i = 0; i < 3; i++) r[i] = a[i] - b[i]; };
  auto scale = [](double t, const double* a, double* r) { for (int i = 0; i < 3; i++) r[i] = t * a[i]; };
  auto norm = [&](const double* a, double* r) {
    double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (l == 0.0) { r[0] = r[1] = r[2] = 0; return; }
    scale(1.0 / l, a, r);
  };
  auto cross = [](const double* u, const double* v, double* r) {
    r[0] = u[1] * v[2] - u[2] * v[1];
    r[1] = u[2] * v[0] - u[0] * v[2];
    r[2] = u[0] * v[1] - u[1] * v[0];
  };
  std::memset(o, 0, sizeof *o);
  int H = int(c->image_width / c->aspect_ratio);
  H = H < 1 ? 1 : H;
  o->image_width = c->image_width, o->image_height = H;
  for (int i = 0; i < 3; i++) o->center[i] = c->lookfrom[i];
  double theta = c->vfov * (kPiH / 180.0);
  double h = std::tan(theta / 2);
  double vh = 2 * h * c->focus_dist;
  double vw = vh * (double(c->image_width) / H);
  double t[3], vu[3], vv[3], negv[3];
  sub(c->lookfrom, c->lookat, t);
  norm(t, o->w);
  cross(c->vup, o->w, t);
  norm(t, o->u);
  cross(o->w, o->u, o->v);
  scale(vw, o->u, vu);
  for (int i = 0; i < 3; i++) negv[i] = -o->v[i];
  scale(vh, negv, vv);
  scale(1.0 / (double)c->image_width, vu, o->pixel_delta_u);
  scale(1.0 / (double)H, vv, o->pixel_delta_v);
  double fw[3], hu[3], hv[3], ul[3], sdd[3], hd[3];
  scale(c->focus_dist, o->w, fw);
  scale(1.0 / 2.0, vu, hu);
  scale(1.0 / 2.0, vv, hv);
  for (int i = 0; i < 3; i++) ul[i] = ((o->center[i] - fw[i]) - hu[i]) - hv[i];
  for (int i = 0; i < 3; i++) sdd[i] = o->pixel_delta_u[i] + o->pixel_delta_v[i];
  scale(0.5, sdd, hd);
  for (int i = 0; i < 3; i++) o->pixel00[i] = ul[i] + hd[i];
  double rad = c->focus_dist * std::tan((c->defocus_angle / 2) * (kPiH / 180.0));
  scale(rad, o->u, o->defocus_disk_u);
  scale(rad, o->v, o->defocus_disk_v);
  o->defocus_angle = c->defocus_angle;
  return RTX_OK;
}

int64_t rtx_render_pixel_count(const rtx_camera* cam, const rtx_render_params* p) {
  if (!cam || !p) return fail(RTX_ERR_INVALID, "NULL argument");
  PixelMap m;
  std::string err;
  int64_t n = subset_pixels(cam, p, m, err);
  if (n < 0) return fail(RTX_ERR_INVALID, err);
  return n;
}

static int render_device_impl(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, double* d_rgb,
                              int32_t* d_spp, rtx_stats* stats, void* stream, const BandSink* sink);
// Whether render_device_impl hands a render's output to a BandSink: fixed-spp renders
// (RecordSample's in-order sum or the megakernel's DefaultSampler) with samples to trace.
static bool sum_path_of(const rtx_render_params* prm) {
  const bool mk_adaptive = prm->adaptive && prm->mode == RTX_MODE_MEGAKERNEL;
  return !mk_adaptive && (prm->mode == RTX_MODE_MEGAKERNEL || !prm->adaptive) && prm->spp > 0;
}

int rtx_render_device(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, double* d_rgb,
                      int32_t* d_spp, rtx_stats* stats, void* stream) {
  return render_device_impl(sc, cam, prm, d_rgb, d_spp, stats, stream, nullptr);
}

static int render_device_impl(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, double* d_rgb,
                              int32_t* d_spp, rtx_stats* stats, void* stream, const BandSink* sink) {
  if (!sc || !cam || !prm || !d_rgb) return fail(RTX_ERR_INVALID, "NULL argument");
  if (prm->spp < 0 || prm->max_depth < 0) return fail(RTX_ERR_INVALID, "negative spp / max_depth");
  if (prm->mode < RTX_MODE_WAVEFRONT || prm->mode > RTX_MODE_MEGAKERNEL) return fail(RTX_ERR_INVALID, "bad mode");
  // MegaKernel + adaptive = AdaptiveSampler(min_spp, spp, rel_threshold): up to spp + 1 samples
  const bool mk_adaptive = prm->adaptive && prm->mode == RTX_MODE_MEGAKERNEL;
  if (mk_adaptive && prm->spp >= 0x7FFFFFFF) return fail(RTX_ERR_INVALID, "spp too large");
  const int budget = mk_adaptive ? prm->spp + 1 : prm->spp;
  PixelMap map;
  std::string err;
  const int64_t npix = subset_pixels(cam, prm, map, err);
  if (npix < 0) return fail(RTX_ERR_INVALID, err);
  HIPC(hipSetDevice(sc->device));
  hipStream_t s = stream ? (hipStream_t)stream : sc->stream;
  const bool fast = prm->precision == RTX_PREC_FAST && sc->fast_ok;
  Launch L{sc, s, fast ? sc->stack_fast : sc->stack_parity, fast, (prm->flags & RTX_FLAG_COUNT) != 0};
  L.generic = (prm->flags & RTX_FLAG_GENERIC) != 0;
  if (fast && prm->mode == RTX_MODE_PERSISTENT) {
    bool park;
    if (prm->flags & RTX_FLAG_PARK) park = true;
    else if (prm->flags & RTX_FLAG_NO_PARK) park = false;
    else {
      int rc;
      if (sc->park < 0 && (rc = time_park_schedule(sc, cam, prm, s))) return rc;
      park = sc->park == 1;
    }
    // the speculative walk keeps 16-bit node indices on its stack: larger trees (and renders
    // that ask for it) get the leaf-step walk
    const bool spec = sc->n_f4 <= kSpecMaxNodes && !(prm->flags & RTX_FLAG_LEAF_STEP);
    L.park = park ? (spec ? 2 : 1) : 0;
  }

  // the reference's default sampling (adaptive) on the persistent kernel: in phases
  // (render_adaptive); an explicit samples_per_group keeps uniform groups
  const bool phased = prm->mode == RTX_MODE_PERSISTENT && prm->adaptive && !mk_adaptive &&
                      prm->samples_per_group <= 0 && budget > 0 && npix > 0;
  // One allowance (slot_allowance) for all of a scene's slot buffers: the radiance buffer of
  // uniform groups and of the adaptive first pass (lbuf), the wavefront's path queues, the
  // adaptive phases' workspace (aw).  A render keeps the other kinds' buffers as long as they
  // and what it needs itself fit in the allowance, and releases them only when they do not:
  // every release and reallocation synchronises the device, and frames that alternate kinds
  // (the bench's fixed-spp line, its adaptive leg, the CPU check) would pay it every time.
  // A phased render's first pass runs in the scene's radiance buffer (lbuf) at npix x min_spp
  // slots: whatever a fixed-spp frame left there beyond that is kept like another kind's buffer.
  double other = 0.0;  // bytes of other kinds kept (phased: and lbuf beyond the first pass)
  {
    const bool wf = prm->mode == RTX_MODE_WAVEFRONT;
    const double allow = slot_allowance(sc);
    const double per_slot = phased ? 34.0 : wf ? 24.0 + 2 * 84.0 : 24.0;  // (phases: radiance, slot map, batches)
    const double want = per_slot * (double)npix * (double)std::max(1, budget);
    const double aw_bytes = (double)sc->aw.lbuf.n + (double)sc->aw.smap.n + (double)sc->aw.segs.n;
    const double queue_bytes = (double)sc->queue[0].n + (double)sc->queue[1].n;
    const double first_bytes = phased ? adaptive_first_bytes(npix, prm, budget, L.count) : 0.0;
    const double lbuf_extra = phased ? std::max(0.0, (double)sc->lbuf.n - first_bytes) : 0.0;
    other = (phased ? lbuf_extra : aw_bytes) + (wf ? 0.0 : queue_bytes);
    if (other + std::min(want, per_slot * (double)(1ll << kSlotTargetLog2)) > allow) {
      if (!phased) sc->aw.lbuf.release(), sc->aw.smap.release(), sc->aw.segs.release();
      else if (lbuf_extra > 0.0) sc->lbuf.release();  // (render_adaptive reserves the first pass's size)
      if (!wf)
        for (auto& q : sc->queue) q.release();
      other = 0.0;
    }
  }

  // samples in flight per pixel (group size K)
  int K = prm->samples_per_group;
  if (K <= 0) {
    // slots in flight: each persistent launch ends in a tail of draining lanes, so fewer,
    // larger groups pay it less often (Lbuf = 24 B per slot); the wavefront's two queues cost
    // 84 B per slot each and keep the smaller target
    const int64_t target =
        prm->mode == RTX_MODE_WAVEFRONT
            ? slot_target(sc, 3 * sizeof(double) + 2 * (9 * sizeof(double) + 3 * sizeof(uint32_t)), 1ll << 25, other)
            : slot_target(sc, 3 * sizeof(double), 1ll << kSlotTargetLog2, other);
    K = (int)std::max<int64_t>(1, std::min<int64_t>(budget > 0 ? budget : 1, target / std::max<int64_t>(1, npix)));
  }
  K = std::max(1, std::min(K, std::max(1, budget)));
  if ((int64_t)npix * K > 0xFFFFFFFFll) return fail(RTX_ERR_INVALID, "too many slots in one group (lower samples_per_group)");
  const int64_t nslots = npix * (int64_t)K;

  int rc;
  if ((rc = sc->px_sum.reserve(npix * 3 * sizeof(double)))) return rc;
  if ((rc = sc->px_mean.reserve(npix * 3 * sizeof(double)))) return rc;
  if ((rc = sc->px_m2.reserve(npix * 3 * sizeof(double)))) return rc;
  if ((rc = sc->px_samples.reserve(npix * sizeof(int32_t)))) return rc;
  if ((rc = sc->px_conv.reserve(npix))) return rc;
  if (!phased && (rc = sc->lbuf.reserve(nslots * 3 * sizeof(double)))) return rc;
  if ((rc = sc->counters.reserve(kCounterWords * sizeof(unsigned long long)))) return rc;
  const size_t qbytes = nslots * (9 * sizeof(double) + 3 * sizeof(uint32_t));
  if (prm->mode == RTX_MODE_WAVEFRONT)
    for (auto& q : sc->queue)
      if ((rc = q.reserve(qbytes))) return rc;
  // fixed spp (RecordSample's in-order sum, or the megakernel's DefaultSampler): only the
  // running sum and count matter, and the first group starts them (k_accumulate_sum `first`)
  const bool sum_path = sum_path_of(prm);
  {
    const PixelSoA pz{sc->px_sum.as<double>(), sc->px_mean.as<double>(), sc->px_m2.as<double>(),
                      sc->px_samples.as<int32_t>(), sc->px_conv.as<uint8_t>()};
    const int64_t n = std::max<int64_t>(sum_path ? 0 : npix, kCounterWords);
    hipLaunchKernelGGL(k_frame_init, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, pz, npix,
                       sum_path ? 0 : 1, sc->counters.as<unsigned long long>(), kCounterWords);
    HIPC(hipGetLastError());
    if (g_debug_host) g_t_launch = host_us();
  }
  const bool banded = sum_path && sink && npix > 0;
  const bool early_ok = phased && sink && sink->host_rgb_dev && npix > 0;
  if (banded || early_ok) {
    if (!sc->copy_stream) HIPC(hipStreamCreateWithFlags(&sc->copy_stream, hipStreamNonBlocking));
    while (sc->band_ev.size() < kBands + 1) {
      hipEvent_t e = nullptr;
      HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      sc->band_ev.push_back(e);
    }
  }
  bool resolved = false;

  unsigned long long* cnt = sc->counters.as<unsigned long long>();
  PixelSoA px{sc->px_sum.as<double>(), sc->px_mean.as<double>(), sc->px_m2.as<double>(), sc->px_samples.as<int32_t>(),
              sc->px_conv.as<uint8_t>()};
  RenderArgs A;
  A.S = sc->S;
  A.cam = *cam;
  A.map = map;
  A.seed = prm->seed;
  A.npix = npix;
  A.max_depth = prm->max_depth;
  A.scatter_api = prm->mode == RTX_MODE_MEGAKERNEL;
  A.conv = prm->adaptive ? sc->px_conv.as<uint8_t>() : nullptr;
  A.L = sc->lbuf.as<double>();
  A.counters = cnt;
  // the lean BVH4 walk stores at most fast_need + 1 stack slots (branchless pushes); the
  // parity walk gets its template bound (pick_stack: reference depth + 2)
  A.stack_slots = fast ? sc->fast_need + 1 : L.stack + 1;
  // counters[8..] : queue counts (u32) for the wavefront;
  // [64 + 16 g] the slot counters of the 8 regions, 128 bytes apart
  unsigned* qcount = (unsigned*)(cnt + 8);
  unsigned long long* next_slot = cnt + 64;
  auto make_queue = [&](DevBuf& b) {
    PathQueue q;
    double* d = b.as<double>();
    q.ox = d, q.oy = d + nslots, q.oz = d + 2 * nslots, q.dx = d + 3 * nslots, q.dy = d + 4 * nslots;
    q.dz = d + 5 * nslots, q.tx = d + 6 * nslots, q.ty = d + 7 * nslots, q.tz = d + 8 * nslots;
    q.slot = (uint32_t*)(d + 9 * nslots);
    q.meta = q.slot + nslots;
    q.hit = (int32_t*)(q.meta + nslots);
    return q;
  };
  // per-launch timing of the dominant kernel (extend / persistent) with an event pool: one
  // pair per hot launch of the whole frame (grow-only pool)
  size_t evi = 0;
  auto ev_at = [&](size_t i) -> hipEvent_t {
    while (sc->evpool.size() <= i) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      sc->evpool.push_back(e);
    }
    return sc->evpool[i];
  };
  const bool timed = stats != nullptr;
  double hot_ms = 0;
  uint64_t hot_launches = 0;
  if (timed) HIPC(hipEventRecord(sc->ev[0], s));
  const int pix_blocks = (int)((npix + kBlock - 1) / kBlock);
  const int wf_grid = std::max(1, std::min<int>(sc->cus * 16, (int)((nslots + kBlock - 1) / kBlock)));
  // Adaptive early output: once a phase holds at most npix / kEarlyOutDiv pixels, every other
  // pixel is final, so the whole output is resolved and copied to the host on the copy stream
  // while the remaining phases run; at the end the device writes only that phase's pixels into
  // the host framebuffer (k_patch_host).  (The copy engine does not need the CUs the phase
  // launches hold.)
  int64_t patch_n = -1;
  auto early = [&](int g, int64_t active, const uint32_t* list) -> int {
    (void)g;
    if (!early_ok || patch_n >= 0 || active * kEarlyOutDiv > npix) return RTX_OK;
    int rc2;
    if ((rc2 = sc->patch_q.reserve((size_t)std::max<int64_t>(1, active) * sizeof(uint32_t)))) return rc2;
    hipLaunchKernelGGL(k_resolve, dim3(pix_blocks), dim3(kBlock), 0, s, px, npix, 0, prm->spp, d_rgb, d_spp);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(sc->patch_q.p, list, (size_t)active * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    HIPC(hipEventRecord(sc->band_ev[0], s));
    HIPC(hipStreamWaitEvent(sc->copy_stream, sc->band_ev[0], 0));
    if ((rc2 = sink->copy(sink->ctx, 0, npix, sc->copy_stream))) return rc2;
    HIPC(hipEventRecord(sc->band_ev[1], sc->copy_stream));
    patch_n = active;
    g_early_outputs++, g_early_patched += active;
    return RTX_OK;
  };
  if (phased) {
    if ((rc = render_adaptive(sc, L, A, prm, px, budget, other, s, [&](hipStream_t st) -> int {
           if (timed) {
             hipEvent_t e = ev_at(evi++);
             if (!e) return fail(RTX_ERR_HIP, "hipEventCreate failed");
             HIPC(hipEventRecord(e, st));
           }
           return RTX_OK;
         }, hot_launches, early))) {
      // an error after the early output was queued: the copy into the caller's framebuffer
      // must be over before the caller gets the error (and may free or reuse the buffer)
      if (patch_n >= 0) (void)hipEventSynchronize(sc->band_ev[1]);
      return rc;
    }
    if (patch_n >= 0) {  // the early copy is done before the device patches the same framebuffer
      hipError_t e = hipStreamWaitEvent(s, sc->band_ev[1], 0);
      if (e == hipSuccess && patch_n > 0) {
        hipLaunchKernelGGL(k_patch_host, dim3((unsigned)((patch_n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, px,
                           npix, sc->patch_q.as<uint32_t>(), patch_n, map, sink->host_rgb_dev, d_rgb, d_spp);
        e = hipGetLastError();
      }
      if (e != hipSuccess) {
        (void)hipEventSynchronize(sc->band_ev[1]);
        return fail(RTX_ERR_HIP, std::string("adaptive early output: ") + hipGetErrorString(e));
      }
      resolved = true;
    }
  }
  for (int s0 = 0, Kc = 0; s0 < budget && !phased; s0 += Kc) {
    Kc = std::min(K, budget - s0);
    // adaptive with automatic grouping: nothing can converge before min_spp, afterwards
    // small groups limit the samples traced past a pixel's convergence point
    if (prm->adaptive && prm->samples_per_group <= 0)
      Kc = std::min(Kc, s0 < prm->min_spp ? prm->min_spp - s0 : 4);
    A.K = Kc;
    A.fK = make_fastdiv((uint32_t)Kc);
    A.s0 = s0;
    auto hot_begin = [&]() -> int {
      if (timed) {
        hipEvent_t e = ev_at(evi++);
        if (!e) return fail(RTX_ERR_HIP, "hipEventCreate failed");
        HIPC(hipEventRecord(e, s));
      }
      return RTX_OK;
    };
    if (prm->mode == RTX_MODE_WAVEFRONT) {
      PathQueue q[2] = {make_queue(sc->queue[0]), make_queue(sc->queue[1])};
      HIPC(hipMemsetAsync(qcount, 0, 2 * sizeof(unsigned), s));
      hipLaunchKernelGGL(k_wf_generate, dim3(wf_grid), dim3(kBlock), 0, s, A, q[0], qcount);
      HIPC(hipGetLastError());
      for (int b = 0; b <= prm->max_depth; b++) {
        const int cur = b & 1;
        HIPC(hipMemsetAsync(qcount + (cur ^ 1), 0, sizeof(unsigned), s));
        if ((rc = hot_begin())) return rc;
        if ((rc = extend(L, A, q[cur], qcount + cur, Kc * npix))) return rc;
        if ((rc = hot_begin())) return rc;
        hipLaunchKernelGGL(k_wf_shade, dim3(wf_grid), dim3(kBlock), 0, s, A, q[cur], qcount + cur, q[cur ^ 1],
                           qcount + (cur ^ 1));
        HIPC(hipGetLastError());
        hot_launches++;
      }
    } else {
      HIPC(hipMemsetAsync(next_slot, 0, 8 * 16 * sizeof(unsigned long long), s));
      if ((rc = hot_begin())) return rc;
      rc = prm->mode == RTX_MODE_MEGAKERNEL ? persist_m<true>(L, A, next_slot) : persist_m<false>(L, A, next_slot);
      if (rc) return rc;
      if ((rc = hot_begin())) return rc;
      hot_launches++;
    }
    if (mk_adaptive)
      hipLaunchKernelGGL(k_accumulate_mk_adaptive, dim3(pix_blocks), dim3(kBlock), 0, s, px, A.L, npix, Kc,
                         prm->min_spp, prm->spp, prm->rel_threshold);
    else if (sum_path) {
      // fixed spp: only sum/(float)samples reaches the output, and the in-order sum is the
      // same as RecordSample's; the Welford mean/M2 (three divisions per sample) only feed
      // IsConverged, which adaptive sampling alone consults.  The last group writes the
      // resolved output itself (k_resolve's arithmetic), in bands when a sink takes them.
      const bool last = s0 + Kc >= budget;
      AccOut out{nullptr, nullptr, -1, prm->spp};
      if (last) out = AccOut{d_rgb, d_spp, prm->mode == RTX_MODE_MEGAKERNEL ? 1 : 0, prm->spp};
      const int nb = (last && banded) ? kBands : 1;
      const int64_t align = banded ? std::max<int64_t>(1, sink->align) : 1;
      const int64_t units = (npix + align - 1) / align;
      for (int b = 0; b < nb; b++) {
        const int64_t q0 = std::min<int64_t>(npix, units * b / nb * align);
        const int64_t q1 = std::min<int64_t>(npix, units * (b + 1) / nb * align);
        if (q1 <= q0) continue;
        hipLaunchKernelGGL(k_accumulate_sum, dim3((unsigned)((q1 - q0 + kAccPix - 1) / kAccPix)), dim3(kAccWave), 0,
                           s, px, A.L, npix, Kc, q0, q1, s0 == 0 ? 1 : 0, out);
        HIPC(hipGetLastError());
        if (last && banded) {
          HIPC(hipEventRecord(sc->band_ev[b], s));
          HIPC(hipStreamWaitEvent(sc->copy_stream, sc->band_ev[b], 0));
          if ((rc = sink->copy(sink->ctx, q0, q1, sc->copy_stream))) return rc;
        }
      }
      resolved = last;
    } else
      hipLaunchKernelGGL(k_accumulate, dim3(pix_blocks), dim3(kBlock), 0, s, px, A.L, npix, Kc, prm->adaptive,
                         prm->min_spp, prm->rel_threshold);
    HIPC(hipGetLastError());
  }
  if (!resolved) {
    hipLaunchKernelGGL(k_resolve, dim3(pix_blocks), dim3(kBlock), 0, s, px, npix,
                       prm->mode == RTX_MODE_MEGAKERNEL ? (mk_adaptive ? 2 : 1) : 0, prm->spp, d_rgb, d_spp);
    HIPC(hipGetLastError());
  }
  // the render's end (rtx_stats.kernel_ms: device time of the render, its output copies not
  // included, whatever the sampling)
  if (timed) HIPC(hipEventRecord(sc->ev[1], s));
  // renders the accumulate does not band (adaptive sampling): the whole output to the sink here,
  // on the stream before the event the host waits on, so one host wait covers the frame and its copy
  if (sink && !banded && npix > 0 && patch_n < 0) {
    if ((rc = sink->copy(sink->ctx, 0, npix, s))) return rc;
  }
  if (timed) {  // the statistics come back with the frame: one wait, no blocking copy after it
    if ((rc = sc->counters_h.reserve(24 * sizeof(unsigned long long)))) return rc;
    HIPC(hipMemcpyAsync(sc->counters_h.p, cnt, 24 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPC(hipEventRecord(sc->ev[4], s));
  }
  if (banded) {  // the caller's stream owns the output again once the band copies are done
    HIPC(hipEventRecord(sc->band_ev.back(), sc->copy_stream));
    HIPC(hipStreamWaitEvent(s, sc->band_ev.back(), 0));
  }
  if (timed) {
    if (g_debug_host) g_t_sync0 = host_us();
    HIPC(hipEventSynchronize(sc->ev[4]));
    if (g_debug_host) g_t_sync1 = host_us();
    float ms = 0;
    HIPC(hipEventElapsedTime(&ms, sc->ev[0], sc->ev[1]));
    // the hot launches' event pairs are read only now: no host wait inside the frame, so the
    // accumulate / resolve launches are queued while the hot kernel still runs
    for (size_t e = 0; e + 1 < evi; e += 2) {
      float hms = 0;
      HIPC(hipEventElapsedTime(&hms, sc->evpool[e], sc->evpool[e + 1]));
      hot_ms += hms;
    }
    unsigned long long h[24];
    std::memcpy(h, sc->counters_h.p, sizeof h);
    static const bool drain_debug = std::getenv("RTX_DEBUG_DRAIN") != nullptr;
    static const bool region_debug = std::getenv("RTX_DEBUG_REGIONS") != nullptr;
    if (region_debug && (h[18] | h[19] | h[20])) {  // counting builds: the persistent loop's regions
      const double tot = (double)(h[18] + h[19] + h[20]);
      fprintf(stderr,
              "rtx regions: wave cycles refill %.4f walk %.4f shade %.4f of %.4g (leaf rounds of the speculative "
              "walk %.4f); shading rounds %llu, lanes per shading round %.2f; segments %llu\n",
              h[18] / tot, h[19] / tot, h[20] / tot, tot, h[23] / tot, (unsigned long long)h[21],
              h[21] ? (double)h[22] / h[21] : 0.0, (unsigned long long)h[0]);
    }
    if (drain_debug && h[13] && !phased) {  // counting builds: the (last) launch's timeline
      const double t0 = (double)~h[13];
      auto us = [&](unsigned long long v) { return ((double)v - t0) / 100.0; };
      fprintf(stderr, "rtx frame timeline: slots used up %.1f .. %.1f us, waves end %.1f .. %.1f us (%lld segments)\n",
              us(~h[15]), us(h[14]), us(~h[17]), us(h[16]), (long long)h[0]);
    }
    stats->wave_rounds = h[10];
    stats->wave_rounds_idle = h[11];
    stats->wave_lanes_live = h[12];
    stats->rays_total = h[0];
    stats->parked = L.park ? 1 : 0;
    stats->rays_primary = h[1];
    stats->paths = h[1];
    stats->kernel_ms = ms;
    stats->hot_kernel_ms = hot_ms;
    stats->hot_launches = hot_launches;
    stats->node_visits = h[2];
    stats->prim_tests = h[3];
    stats->wave_node_iters = h[4];
    stats->wave_prim_iters = h[5];
    stats->tri_tests = h[6];
    stats->sphere_tests = h[7];
    stats->build = prm->mode == RTX_MODE_WAVEFRONT ? 0 : L.build;
    stats->node_bytes = L.fast ? sizeof(F4Node) : sizeof(rtx_bvh_node);  // (the byte model's 4 x 32 B boxes; a QNode is 64 B)
    // segments of the recorded samples: counted per slot by the counting build in adaptive
    // phases (k_adapt_record); every sample is recorded at fixed spp; unknown otherwise
    stats->rays_recorded = !L.count ? 0 : phased ? h[9] : (prm->adaptive ? 0 : h[0]);
  }
  return RTX_OK;
}

int rtx_render(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, double* rgb, int32_t* spp,
               rtx_stats* stats) {
  if (!sc || !cam || !prm || !rgb) return fail(RTX_ERR_INVALID, "NULL argument");
  PixelMap map;
  std::string err;
  const int64_t npix = subset_pixels(cam, prm, map, err);
  if (npix < 0) return fail(RTX_ERR_INVALID, err);
  HIPC(hipSetDevice(sc->device));
  int rc;
  if ((rc = sc->out_rgb.reserve(std::max<int64_t>(1, npix) * 3 * sizeof(double)))) return rc;
  if ((rc = sc->out_spp.reserve(std::max<int64_t>(1, npix) * sizeof(int32_t)))) return rc;
  if ((rc = rtx_render_device(sc, cam, prm, sc->out_rgb.as<double>(), sc->out_spp.as<int32_t>(), stats, sc->stream)))
    return rc;
  HIPC(hipMemcpyAsync(rgb, sc->out_rgb.p, npix * 3 * sizeof(double), hipMemcpyDeviceToHost, sc->stream));
  if (spp) HIPC(hipMemcpyAsync(spp, sc->out_spp.p, npix * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
  HIPC(hipStreamSynchronize(sc->stream));
  return RTX_OK;
}

// ---- one frame over several devices (wavefront.cc:228-241's one framebuffer) ----
namespace {
// Device k renders stripe (first + k) of `count` interleaved stripes; its packed stripe rows
// come back over one D2H copy (pinned staging, or a 2D copy straight into a pinned caller
// buffer) and are placed at their rows of the whole-frame buffers.
int render_stripes_to_host(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* base, int stripe,
                           double* out_rgb, int32_t* out_spp, rtx_stats* st) {
  const double t_in = g_debug_host ? host_us() : 0.0;
  rtx_render_params q = *base;
  q.stripe_index = stripe;
  q.x0 = q.y0 = q.w = q.h = 0;
  PixelMap map;
  std::string err;
  const int64_t npix = subset_pixels(cam, &q, map, err);
  if (npix < 0) return fail(RTX_ERR_INVALID, err);
  HIPC(hipSetDevice(sc->device));
  int rc;
  if ((rc = sc->out_rgb.reserve(std::max<int64_t>(1, npix) * 3 * sizeof(double)))) return rc;
  if ((rc = sc->out_spp.reserve(std::max<int64_t>(1, npix) * sizeof(int32_t)))) return rc;
  const int64_t W = map.W, H = map.H, R = map.srows, N = map.scount;
  const int64_t nblk = (H + R - 1) / R;  // stripes of the image; ours: stripe, stripe + N, ...
  const size_t row_rgb = (size_t)W * 3 * sizeof(double), row_spp = (size_t)W * sizeof(int32_t);
  hipPointerAttribute_t at{};
  const bool pinned = hipPointerGetAttributes(&at, out_rgb) == hipSuccess && at.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // pageable memory reports an error here on some runtimes
  const int64_t full = (H / R > stripe) ? (H / R - stripe + N - 1) / N : 0;  // our stripes with R rows
  const bool direct = pinned && full > 0;  // strided DMA straight into the caller's rows
  if (!direct && (rc = sc->stage_rgb.reserve((size_t)std::max<int64_t>(1, npix) * 3 * sizeof(double)))) return rc;
  // Packed pixels [p0, p1) of this device's rows -> host.  Band edges are whole stripes
  // (align R * W), so a band is a run of our full stripes (one strided DMA) and, in the last
  // band, the short stripe at the bottom of the image.
  struct Ctx {
    rtx_scene* sc;
    double* out_rgb;
    bool direct;
    int64_t W, R, N, stripe, full;
    size_t row_rgb;
  } ctx{sc, out_rgb, direct, W, R, N, stripe, full, row_rgb};
  auto copy = [](void* c, int64_t p0, int64_t p1, hipStream_t cs) -> int {
    const Ctx& k = *(const Ctx*)c;
    const double* src = k.sc->out_rgb.as<double>();
    if (!k.direct) {
      HIPC(hipMemcpyAsync((double*)k.sc->stage_rgb.p + 3 * p0, src + 3 * p0, (size_t)(p1 - p0) * 3 * sizeof(double),
                          hipMemcpyDeviceToHost, cs));
      return RTX_OK;
    }
    const int64_t r0 = p0 / k.W, r1 = (p1 + k.W - 1) / k.W;  // packed rows
    const int64_t k0 = r0 / k.R, k1 = std::min<int64_t>(k.full, r1 / k.R);
    if (k1 > k0)
      HIPC(hipMemcpy2DAsync(k.out_rgb + (size_t)(k.stripe + k0 * k.N) * k.R * k.W * 3, (size_t)k.N * k.R * k.row_rgb,
                            src + (size_t)k0 * k.R * k.W * 3, (size_t)k.R * k.row_rgb, (size_t)k.R * k.row_rgb,
                            (size_t)(k1 - k0), hipMemcpyDeviceToHost, cs));
    const int64_t rs = std::max<int64_t>(r0, k.full * k.R);  // rows of the short last stripe
    if (r1 > rs)
      HIPC(hipMemcpyAsync(k.out_rgb + (size_t)((k.stripe + k.full * k.N) * k.R + (rs - k.full * k.R)) * k.W * 3,
                          src + (size_t)rs * k.W * 3, (size_t)(r1 - rs) * k.row_rgb, hipMemcpyDeviceToHost, cs));
    return RTX_OK;
  };
  BandSink sink{R * W, copy, &ctx};
  if (direct) {  // adaptive renders may write their last pixels straight into the caller's pinned rows
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, out_rgb, 0) == hipSuccess) sink.host_rgb_dev = (double*)dp;
    else (void)hipGetLastError();
  }
  if ((rc = render_device_impl(sc, cam, &q, sc->out_rgb.as<double>(), sc->out_spp.as<int32_t>(), st, sc->stream,
                               &sink)))
    return rc;
  if (npix == 0) return RTX_OK;
  // (renders the accumulate does not band sent the whole output to the sink at their end)
  if (out_spp) {
    if ((rc = sc->stage_spp.reserve((size_t)npix * sizeof(int32_t)))) return rc;
    HIPC(hipMemcpyAsync(sc->stage_spp.p, sc->out_spp.p, (size_t)npix * sizeof(int32_t), hipMemcpyDeviceToHost,
                        sc->stream));
  }
  HIPC(hipStreamSynchronize(sc->stream));
  int64_t r = 0;  // packed row
  for (int64_t b = stripe; b < nblk; b += N) {
    const int64_t y0 = b * R, rows = std::min<int64_t>(R, H - y0);
    if (!direct)
      std::memcpy(out_rgb + (size_t)y0 * W * 3, (const char*)sc->stage_rgb.p + (size_t)r * row_rgb,
                  (size_t)rows * row_rgb);
    if (out_spp)
      std::memcpy(out_spp + (size_t)y0 * W, (const char*)sc->stage_spp.p + (size_t)r * row_spp,
                  (size_t)rows * row_spp);
    r += rows;
  }
  if (g_debug_host) {
    static thread_local double t_prev_out = 0;  // (rtx_render_multi: one thread per device)
    const double t_out = host_us();
    fprintf(stderr,
            "rtx host: device %d: since last frame %.1f us | to first launch %.1f | launches %.1f | sync wait %.1f | "
            "after %.1f\n",
            sc->device, t_prev_out > 0 ? t_in - t_prev_out : -1.0, g_t_launch - t_in, g_t_sync0 - g_t_launch,
            g_t_sync1 - g_t_sync0, t_out - g_t_sync1);
    t_prev_out = t_out;
  }
  return RTX_OK;
}
}  // namespace

int rtx_render_multi(rtx_scene* const* scenes, int32_t n, const rtx_camera* cam, const rtx_render_params* prm,
                     double* out_rgb, int32_t* out_spp, rtx_stats* stats, rtx_stats* per_scene) {
  if (!scenes || n <= 0 || !cam || !prm || !out_rgb) return fail(RTX_ERR_INVALID, "bad argument");
  for (int32_t k = 0; k < n; k++)
    if (!scenes[k]) return fail(RTX_ERR_INVALID, "scene is NULL");
  for (int32_t j = 0; j < n; j++)
    for (int32_t k = j + 1; k < n; k++)
      if (scenes[j] == scenes[k]) return fail(RTX_ERR_INVALID, "a scene appears twice (one scene per render thread)");
  rtx_render_params base = *prm;
  if (base.stripe_rows <= 0) base.stripe_rows = 8;
  if (base.stripe_count <= 0) base.stripe_count = n, base.stripe_index = 0;
  if (base.stripe_index < 0 || base.stripe_index + n > base.stripe_count)
    return fail(RTX_ERR_INVALID, "stripes stripe_index .. stripe_index + n - 1 must lie below stripe_count");
  std::vector<int> rc(n, RTX_OK);
  std::vector<std::string> msg(n);
  std::vector<rtx_stats> st(n);
  auto work = [&](int k) {
    st[k] = rtx_stats{};
    rc[k] = render_stripes_to_host(scenes[k], cam, &base, base.stripe_index + k, out_rgb, out_spp, &st[k]);
    if (rc[k] != RTX_OK) msg[k] = g_err;  // rtx_last_error is per thread
  };
  if (n == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(n);
    for (int k = 0; k < n; k++) th.emplace_back(work, k);
    for (auto& t : th) t.join();
  }
  for (int k = 0; k < n; k++)
    if (rc[k] != RTX_OK) return fail(rc[k], "device " + std::to_string(scenes[k]->device) + ": " + msg[k]);
  if (per_scene)
    for (int k = 0; k < n; k++) per_scene[k] = st[k];
  if (stats) {
    rtx_stats a{};
    for (int k = 0; k < n; k++) {
      a.rays_primary += st[k].rays_primary, a.rays_total += st[k].rays_total, a.paths += st[k].paths;
      a.kernel_ms = std::max(a.kernel_ms, st[k].kernel_ms);
      a.hot_kernel_ms = std::max(a.hot_kernel_ms, st[k].hot_kernel_ms);
      a.hot_launches += st[k].hot_launches, a.node_visits += st[k].node_visits, a.prim_tests += st[k].prim_tests;
      a.wave_node_iters += st[k].wave_node_iters, a.wave_prim_iters += st[k].wave_prim_iters;
      a.tri_tests += st[k].tri_tests, a.sphere_tests += st[k].sphere_tests;
      a.rays_recorded += st[k].rays_recorded;
      a.wave_rounds += st[k].wave_rounds, a.wave_rounds_idle += st[k].wave_rounds_idle;
      a.wave_lanes_live += st[k].wave_lanes_live;
      a.node_bytes = st[k].node_bytes, a.parked |= st[k].parked, a.build |= st[k].build;
    }
    *stats = a;
  }
  return RTX_OK;
}

// ---- P3 output on the device (wavefront.cc:238-241, core/color.h:18-33) ----
static std::string p3_header(int64_t w, int64_t h) {
  return "P3\n" + std::to_string(w) + " " + std::to_string(h) + "\n255\n";
}

size_t rtx_p3_max_bytes(int32_t w, int32_t h) {
  if (w <= 0 || h <= 0) return 0;
  return p3_header(w, h).size() + (size_t)w * (size_t)h * rtxp3::kMaxLine;
}

// body of d_rgb into sc->p3_body; *len = body bytes
static int p3_encode(rtx_scene* sc, const double* d_rgb, int64_t npix, size_t* len, hipStream_t s) {
  if ((uint64_t)npix * rtxp3::kMaxLine > 0xFFFFFFFFull) return fail(RTX_ERR_INVALID, "P3 output above 4 GiB");
  int rc;
  if ((rc = sc->p3_scratch.reserve(rtxp3::scratch_bytes(std::max<int64_t>(1, npix))))) return rc;
  if ((rc = sc->p3_body.reserve(std::max<int64_t>(1, npix) * rtxp3::kMaxLine))) return rc;
  HIPC(rtxp3::encode_body(d_rgb, npix, sc->p3_scratch.p, (char*)sc->p3_body.p, len, s));
  return RTX_OK;
}

int rtx_encode_p3_device(rtx_scene* sc, const double* d_rgb, int32_t w, int32_t h, char* d_out, size_t cap,
                         size_t* out_len, void* stream) {
  if (!sc || !d_rgb || !d_out || !out_len || w <= 0 || h <= 0) return fail(RTX_ERR_INVALID, "bad argument");
  if (cap < rtx_p3_max_bytes(w, h)) return fail(RTX_ERR_INVALID, "output buffer below rtx_p3_max_bytes");
  HIPC(hipSetDevice(sc->device));
  hipStream_t s = stream ? (hipStream_t)stream : sc->stream;
  const std::string hd = p3_header(w, h);
  size_t body = 0;
  int rc;
  if ((rc = p3_encode(sc, d_rgb, (int64_t)w * h, &body, s))) return rc;
  HIPC(hipMemcpyAsync(d_out, hd.data(), hd.size(), hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(d_out + hd.size(), sc->p3_body.p, body, hipMemcpyDeviceToDevice, s));
  HIPC(hipStreamSynchronize(s));
  *out_len = hd.size() + body;
  return RTX_OK;
}

int rtx_encode_p3(rtx_scene* sc, const double* rgb, int32_t w, int32_t h, char* out, size_t cap, size_t* out_len) {
  if (!sc || !rgb || !out || !out_len || w <= 0 || h <= 0) return fail(RTX_ERR_INVALID, "bad argument");
  if (cap < rtx_p3_max_bytes(w, h)) return fail(RTX_ERR_INVALID, "output buffer below rtx_p3_max_bytes");
  HIPC(hipSetDevice(sc->device));
  const int64_t npix = (int64_t)w * h;
  int rc;
  if ((rc = sc->out_rgb.reserve(npix * 3 * sizeof(double)))) return rc;
  HIPC(hipMemcpyAsync(sc->out_rgb.p, rgb, npix * 3 * sizeof(double), hipMemcpyHostToDevice, sc->stream));
  const std::string hd = p3_header(w, h);
  size_t body = 0;
  if ((rc = p3_encode(sc, sc->out_rgb.as<double>(), npix, &body, sc->stream))) return rc;
  std::memcpy(out, hd.data(), hd.size());
  HIPC(hipMemcpyAsync(out + hd.size(), sc->p3_body.p, body, hipMemcpyDeviceToHost, sc->stream));
  HIPC(hipStreamSynchronize(sc->stream));
  *out_len = hd.size() + body;
  return RTX_OK;
}

int rtx_render_p3(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, char* out, size_t cap,
                  size_t* out_len, double* rgb, int32_t* spp, rtx_stats* stats) {
  if (!sc || !cam || !prm || !out || !out_len) return fail(RTX_ERR_INVALID, "NULL argument");
  PixelMap map;
  std::string err;
  const int64_t npix = subset_pixels(cam, prm, map, err);
  if (npix < 0) return fail(RTX_ERR_INVALID, err);
  const std::string hd = p3_header(map.w, map.h);
  if (cap < hd.size() + (size_t)npix * rtxp3::kMaxLine) return fail(RTX_ERR_INVALID, "output buffer below rtx_p3_max_bytes");
  HIPC(hipSetDevice(sc->device));
  int rc;
  if ((rc = sc->out_rgb.reserve(std::max<int64_t>(1, npix) * 3 * sizeof(double)))) return rc;
  if ((rc = sc->out_spp.reserve(std::max<int64_t>(1, npix) * sizeof(int32_t)))) return rc;
  if ((rc = rtx_render_device(sc, cam, prm, sc->out_rgb.as<double>(), sc->out_spp.as<int32_t>(), stats, sc->stream)))
    return rc;
  size_t body = 0;
  if ((rc = p3_encode(sc, sc->out_rgb.as<double>(), npix, &body, sc->stream))) return rc;
  std::memcpy(out, hd.data(), hd.size());
  HIPC(hipMemcpyAsync(out + hd.size(), sc->p3_body.p, body, hipMemcpyDeviceToHost, sc->stream));
  if (rgb) HIPC(hipMemcpyAsync(rgb, sc->out_rgb.p, npix * 3 * sizeof(double), hipMemcpyDeviceToHost, sc->stream));
  if (spp) HIPC(hipMemcpyAsync(spp, sc->out_spp.p, npix * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
  HIPC(hipStreamSynchronize(sc->stream));
  *out_len = hd.size() + body;
  return RTX_OK;
}

// write_color (core/color.h:10-33): sqrt gamma, clamp [0, 0.999], int(256 x).
int rtx_write_ppm(const char* path, const double* rgb, int32_t w, int32_t h) {
  if (!path || !rgb || w <= 0 || h <= 0) return fail(RTX_ERR_INVALID, "bad argument");
  FILE* f = std::fopen(path, "w");
  if (!f) return fail(RTX_ERR_IO, std::string("cannot write ") + path);
  std::fprintf(f, "P3\n%d %d\n255\n", w, h);
  for (int64_t i = 0; i < (int64_t)w * h; i++) {
    int b[3];
    for (int c = 0; c < 3; c++) {
      double x = rgb[3 * i + c];
      x = x > 0 ? std::sqrt(x) : 0;
      x = x < 0.0 ? 0.0 : (x > 0.999 ? 0.999 : x);
      b[c] = int(256 * x);
    }
    std::fprintf(f, "%d %d %d\n", b[0], b[1], b[2]);
  }
  std::fclose(f);
  return RTX_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// Self-check of the restated small-argument cos/sin (rtxd::sincos_small, used by the plain
// kernel's Lambertian sampling) against the device library's cos() and sin(): n arguments
// phi = 2*pi*u with u the reference's 53-bit uniform draws (a 64-bit mix of seed and index,
// top 53 bits), plus the ends of [0, 1) and the quadrant boundaries.  Test hook only (not in
// rtx.h): tests/test_gpu_timed.py.
namespace {
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ void k_check_sincos(int64_t n, uint64_t seed, unsigned long long* bad, double* first_bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + 64; i += (int64_t)gridDim.x * blockDim.x) {
    double u;
    if (i < n) {
      u = (double)(mix64(seed + (uint64_t)i) >> 11) * 0x1.0p-53;
    } else {  // 0, the largest draw, and 1/4, 1/2, 3/4 (and their neighbours)
      const int j = (int)(i - n);
      const double base[5] = {0.0, 1.0, 0.25, 0.5, 0.75};
      u = base[j % 5];
      const int steps = j / 5 - 6;  // -6 .. +6 draws around the point
      u += steps * 0x1.0p-53;
      if (u < 0.0 || u >= 1.0) continue;
    }
    const double phi = 2.0 * rtxd::kPi * u;
    double s, c;
    rtxd::sincos_small(phi, s, c);
    const double c0 = cos(phi), s0 = sin(phi);
    if (__double_as_longlong(c) != __double_as_longlong(c0) || __double_as_longlong(s) != __double_as_longlong(s0)) {
      if (atomicAdd(bad, 1ull) == 0) *first_bad = u;
    }
  }
}
}  // namespace

extern "C" int rtx_internal_check_sincos(int device, int64_t n, uint64_t seed, int64_t* mismatches,
                                         double* first_bad) {
  if (n < 0 || !mismatches) return fail(RTX_ERR_INVALID, "bad argument");
  HIPC(hipSetDevice(device));
  struct Owned : DevBuf {
    ~Owned() { release(); }
  } b;
  int rc;
  if ((rc = b.reserve(2 * sizeof(unsigned long long)))) return rc;
  HIPC(hipMemset(b.p, 0, 2 * sizeof(unsigned long long)));
  unsigned long long* bad = b.as<unsigned long long>();
  hipLaunchKernelGGL(k_check_sincos, dim3(1024), dim3(256), 0, nullptr, n, seed, bad, (double*)(bad + 1));
  HIPC(hipGetLastError());
  unsigned long long h[2];
  HIPC(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
  *mismatches = (int64_t)h[0];
  if (first_bad) std::memcpy(first_bad, &h[1], sizeof(double));
  return RTX_OK;
}

// Test / tuning hook (not in rtx.h): overrides of the adaptive phases' constants for the
// renders that follow in this process (0 / negative restores a default): the smallest phase,
// the largest batch of a pixel, the first pass's kernel (1 the phase kernel, 0 the uniform-group
// one) and the batch margin's growth per phase.  Results never depend on them, only the amount
// of work and the number of phases do (tests/test_gpu_timed.py runs the full budgets through
// forced small workspaces).
extern "C" int rtx_internal_adapt_tune(int64_t phase_slots, int32_t phase_kcap, int32_t first_map, double phase_mstep,
                                       double margin1, double pool_w) {
  if (phase_slots < 0 || phase_kcap < 0 || first_map > 1) return fail(RTX_ERR_INVALID, "bad tuning value");
  g_tune = AdaptTune{phase_slots, phase_kcap, first_map, phase_mstep, margin1, pool_w};
  return RTX_OK;
}

// Test hook (not in rtx.h): the launch-constant division of the kernels (FastDiv, the slot ->
// pixel and pixel -> row maps) on the host: out[i] = n[i] / d for i < cnt.
extern "C" int rtx_internal_fastdiv(uint32_t d, const uint32_t* n, int64_t cnt, uint32_t* out) {
  if ((!n || !out) && cnt > 0) return fail(RTX_ERR_INVALID, "NULL argument");
  if (d == 0) return fail(RTX_ERR_INVALID, "division by zero");
  const FastDiv f = make_fastdiv(d);
  for (int64_t i = 0; i < cnt; i++) out[i] = f.div(n[i]);
  return RTX_OK;
}

// Test hook (not in rtx.h): the image rows of stripe `index` of `count` (stripe_rows-row
// interleaved stripes) in the order the render writes them, through the same PixelMap the
// kernels use (subset_pixels, PixelMap::xy): rows[0 .. *nrows).  No device needed.
extern "C" int rtx_internal_stripe_rows(int32_t width, int32_t height, int32_t stripe_rows, int32_t index,
                                        int32_t count, int32_t* rows, int64_t* nrows) {
  if (!rows || !nrows) return fail(RTX_ERR_INVALID, "NULL argument");
  rtx_camera cam{};
  cam.image_width = width, cam.image_height = height;
  rtx_render_params prm{};
  prm.stripe_rows = stripe_rows, prm.stripe_index = index, prm.stripe_count = count;
  PixelMap m;
  std::string err;
  const int64_t n = subset_pixels(&cam, &prm, m, err);
  if (n < 0) return fail(RTX_ERR_INVALID, err);
  *nrows = m.h;
  for (int r = 0; r < m.h; r++) {
    int x, y;
    m.xy((uint32_t)r * (uint32_t)m.w, x, y);
    rows[r] = y;
  }
  return RTX_OK;
}

// Test hook (not in rtx.h): how many adaptive renders of this process sent their output to the
// host early (while phases still ran; render_device_impl `early`), and how many pixels the
// device patched afterwards (k_patch_host), summed over them.
extern "C" int rtx_internal_early_output_stats(long long* outputs, long long* patched) {
  if (!outputs || !patched) return fail(RTX_ERR_INVALID, "NULL argument");
  *outputs = g_early_outputs.load(), *patched = g_early_patched.load();
  return RTX_OK;
}

// Test hook (not in rtx.h): the persistent kernel's LDS layout (persist_lds) for a traversal
// stack of stack_slots entries per lane and a schedule (park: 0 plain, 1 PARK with the
// leaf-step walk, 2 PARK with the speculative walk; + 8: an adaptive phase launch, with its
// block-shared slot chunks):
// out[0..5] = byte offsets of the stack, throughput, hit point, leaf queue, block-wide region
// and the block's LDS size; out[6..9] = the first four regions' bytes per lane (entries x
// element size; they are lane-interleaved with stride kBlock), out[10] = the block-wide region's
// bytes (the chunk words).  tests/test_capi_exports.py checks that the regions are disjoint and
// inside the block's LDS for every stack size the host can choose.
extern "C" int rtx_internal_lds_layout(int stack_slots, int park, uint32_t* out) {
  const int block_kind = (park & 8) ? 1 : 0;
  if ((park & ~11) || stack_slots < 1 || stack_slots > 65 || (park & 3) > 2 || !out)
    return fail(RTX_ERR_INVALID, "bad argument");
  park &= 3;
  const bool spec = spec_walk(park, true, false);
  const PersistLds l = persist_lds(stack_slots, spec, block_kind);
  const uint32_t v[11] = {l.stack, l.thr, l.hitp, l.leafq, l.block, l.end, (uint32_t)stack_slots * (spec ? 2u : 4u),
                          24u, 24u, spec ? kLeafQueue * 4u : 0u, block_region_bytes(block_kind)};
  std::memcpy(out, v, sizeof v);
  return RTX_OK;
}

namespace {

// Which persistent fast schedule suits this scene: the PARK kernel wins where a few lanes
// walk long after the rest of their wave (dense meshes: the bunny, +14..18 %) and loses where
// shading dominates (sphere scenes, -5..-10 %), see DESIGN.md.  Both produce identical
// results, so the choice is timing only: the first persistent fast render of a scene renders
// a centre tile of 1/16 of its pixels with each kernel (twice each; the faster second run
// counts) and keeps the one with the higher segment rate for the scene.
// The timing renders run on the caller's stream `s`, so they are ordered after any render
// still queued there: they share the scene's scratch buffers (pixel state, Lbuf, counters).
int time_park_schedule(rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* prm, hipStream_t s) {
  rtx_render_params q = *prm;
  q.stripe_rows = q.stripe_index = q.stripe_count = 0;
  q.w = std::max(1, cam->image_width / 4), q.h = std::max(1, cam->image_height / 4);
  q.x0 = (cam->image_width - q.w) / 2, q.y0 = (cam->image_height - q.h) / 2;
  q.flags = prm->flags & ~(RTX_FLAG_COUNT | RTX_FLAG_PARK | RTX_FLAG_NO_PARK | RTX_FLAG_GENERIC);
  int rc;
  if ((rc = sc->calib_rgb.reserve((size_t)q.w * q.h * 3 * sizeof(double)))) return rc;
  double rate[2] = {0, 0};
  for (int rep = 0; rep < 2; rep++)
    for (int k = 0; k < 2; k++) {
      rtx_render_params r = q;
      r.flags |= k ? RTX_FLAG_PARK : RTX_FLAG_NO_PARK;
      rtx_stats st{};
      if ((rc = rtx_render_device(sc, cam, &r, sc->calib_rgb.as<double>(), nullptr, &st, s))) return rc;
      rate[k] = st.hot_kernel_ms > 0 ? (double)st.rays_total / st.hot_kernel_ms : 0.0;
    }
  sc->park = rate[1] > 1.02 * rate[0] ? 1 : 0;
  return RTX_OK;
}

}  // namespace
