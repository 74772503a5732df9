// rtx_kernels.h — HIP kernels of the hot path (included once, by rtx_capi.hip).
//
//   k_intersect        RayIntegrator::IntersectBatch seam (one ray per lane)
//   k_wf_generate      WavefrontRenderer primary generation (wavefront.cc:62-79)
//   k_wf_extend        closest hit for every queued path (traversal only: low VGPR count,
//                      high occupancy for the latency-bound BVH walk)
//   k_wf_shade         shading + Russian roulette + ballot-compacted child queue
//   k_persistent       persistent lanes with per-wave refill (same results as the wavefront)
//   k_accumulate       RecordSample/IsConverged in sample order (pixel_state.h:22-72)
//   k_resolve          sum/(float)samples (wavefront.cc:229-235) or pixel/N (mega_kernel)
//
// Sample bookkeeping: a render is processed in groups of K samples per pixel.  Every path
// (pixel p, sample s0+k) owns slot p*K+k of Lbuf and writes its radiance exactly once, so
// k_accumulate can replay RecordSample in sample order: the result equals the reference's
// pass-by-pass order regardless of how lanes, queues or XCDs interleave the work.
#pragma once

#include "rtx_device.h"

namespace rtxd {

constexpr int kBlock = 256;

// Tuned constants (DESIGN.md ledger: each picked by A/B, the alternatives removed).
constexpr int kTraceWaves = 4;  // min waves per SIMD for the trace kernels (<= 128 VGPRs; 3 and 5 slower)
constexpr int kSlotTargetLog2 = 29;  // persistent: up to 2^29 slots (pixel x sample) per launch (r02: 2^29 vs 2^27 C4 +4.0 %, C5 +1.3 %), capped by free memory
constexpr int kRefillMin = 24;      // persistent lanes: refill once this many lanes of a wave are idle (ab_refill2_*)
constexpr int kRefillMinPark = 16;  // the same for the PARK kernel
constexpr int kParkAt = 16;  // PARK kernel: park traversals once at most this many lanes still walk (ab_parkT_*)
#ifndef RTX_CHUNK
#define RTX_CHUNK 256
#endif
constexpr int kChunk = RTX_CHUNK;  // persistent: slots taken per atomic on a region's slot counter (ab_chunk_*)
#ifndef RTX_REFILL_SHARED
#define RTX_REFILL_SHARED 0  // > 0: the refill threshold of the block-shared chunk launches (A/B; 0: the kernel's own)
#endif
#ifndef RTX_CHUNK_SHARED
#define RTX_CHUNK_SHARED 128
#endif
constexpr int kChunkShared = RTX_CHUNK_SHARED;  // the same for the block-shared chunks (adaptive phase launches)

// Pixel subset of the image handled by one call (rectangle or interleaved row stripes).
struct PixelMap {
  int32_t W, H;
  int32_t stripes;  // 0: rectangle, 1: stripes
  int32_t x0, y0, w, h;
  int32_t srows, sidx, scount;
  // 32-bit arithmetic: the host keeps pixel counts below 2^31
  __device__ __forceinline__ void xy(uint32_t local, int& x, int& y) const {
    if (!stripes) {
      const uint32_t r = local / (uint32_t)w;
      x = x0 + (int)(local - r * (uint32_t)w);
      y = y0 + (int)r;
    } else {
      const int r = (int)(local / (uint32_t)W);
      x = (int)(local - (uint32_t)r * (uint32_t)W);
      int blk = r / srows;
      y = (blk * scount + sidx) * srows + r % srows;
    }
  }
};

struct PathQueue {  // SoA, one entry per in-flight path
  double *ox, *oy, *oz, *dx, *dy, *dz, *tx, *ty, *tz;
  uint32_t* slot;
  uint32_t* meta;  // path depth (segment index); the RNG stream is depth + 1
  int32_t* hit;    // closest primitive (leaf order) or -1, written by k_wf_extend
};

struct RenderArgs {
  DScene S;
  rtx_camera cam;
  PixelMap map;
  uint64_t seed;
  int64_t npix;         // pixels in the subset
  int32_t K;            // samples in this group
  int32_t s0;           // first sample index of the group
  int32_t max_depth;
  int32_t scatter_api;  // megakernel (Scatter/GetPixel) semantics
  const uint8_t* conv;  // per-pixel converged flag (adaptive), may be null
  double* L;            // Lbuf: 3 doubles per slot
  unsigned long long* counters;  // [0] segments [1] primaries [2] node visits [3] prim tests
  int32_t stack_slots;  // persistent kernel: traversal-stack slots per lane in LDS (the walk's exact bound + 1)
};

// Per-sample radiance of group slot (pixel p, group sample k) = slot p*K+k, channel c.
// Pixel-major: the path-end writes of neighbouring lanes (same pixel, consecutive samples)
// are contiguous.  (Sample-major [k][c][p] coalesces the accumulate's reads but scatters
// these writes: A/B r01 -2 % C2 and bunny.)
__device__ __forceinline__ void store_radiance(const RenderArgs& A, uint32_t slot, V3 L) {
  double* Lp = A.L + 3 * (uint64_t)slot;
  Lp[0] = L.x, Lp[1] = L.y, Lp[2] = L.z;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Wave-level compaction: this lane's destination among the lanes with `want` set; one
// atomicAdd per wave (ballot + popcount of the lower lanes).
__device__ __forceinline__ int64_t wave_compact(bool want, unsigned int* counter) {
  const unsigned long long mask = __ballot(want);
  if (mask == 0) return -1;
  const int leader = __ffsll((long long)mask) - 1;
  const int total = __popcll(mask);
  unsigned int base = 0;
  if ((int)lane_id() == leader) base = atomicAdd(counter, (unsigned int)total);
  base = __shfl(base, leader);
  const int rank = __popcll(mask & ((1ull << lane_id()) - 1ull));
  return want ? (int64_t)base + rank : -1;
}

// Closest primitive (leaf order) or -1; its distance in t_best.
// mat_best: the closest primitive's material id (or -1); the fast traversal keeps it from the
// primitive record it already loaded, so shading can fetch the material without first
// waiting for the record.
// LDS of a block's traversal stacks: STACK + 1 slots per lane (the branchless pushes of the
// lean walk may store one slot above the deepest entry, see trace4_run).
constexpr size_t stack_lds_bytes(int STACK) { return (size_t)(STACK + 1) * kBlock * sizeof(uint32_t); }
// The persistent kernel's LDS per block: the traversal stacks (stack_slots per lane, the walk's
// exact bound + 1), then each lane's path throughput and hit point, 3 doubles each,
// channel-major (lane-consecutive 8-byte words: conflict-free).  Shading reads the throughput
// only at its end and the hit point only as the next origin, so both stay in LDS while the
// lane walks the tree and samples the BSDF instead of occupying 12 of the 128 VGPRs a lane has
// at 4 waves per SIMD (or spilling to scratch).  The PARK kernel with the speculative walk
// (PARK = 2) keeps 16-bit stack entries and adds each lane's leaf queue, kLeafQueue 32-bit
// words, after the hit point.
//
// Every region is lane-interleaved with its own element size (2, 8 or 4 bytes), so a lane's
// words in one region are OTHER lanes' words — lanes of other waves, which run concurrently —
// in any region it overlapped.  Regions must therefore never share bytes, even where one
// lane's uses of them never overlap in time: a 6-word leaf queue laid over the hit-point
// words faulted this way in round 2 (cmp_spec6_fault.txt, ledger).  persist_lds() is the one
// statement of the layout, used by the kernel and the launch; rtx_internal_lds_layout exposes it
// to a CPU test that checks the regions are disjoint and inside the block's LDS.
struct PersistLds {
  uint32_t stack, thr, hitp, leafq, tiles, end;  // byte offsets of the regions in a block's LDS, its size
};

// ---------------------------------------------------------------------------------------
// Adaptive sampling, tile schedule (k_persistent MAP == 2; render_adaptive, rtx_capi.hip).
// After the uniform first pass (min_spp samples of every pixel, recorded by k_adapt_record),
// the pixels still sampling are cut into tiles of kTileTP consecutive pixels, ordered within
// each of the 8 slot regions by their predicted work, largest first.  ONE persistent launch
// then runs every remaining phase of every tile: a workgroup claims a tile (one atomic per
// tile), its lanes trace the tile's batch (each pixel's next samples, pixel-major), and once
// the batch's last path has ended, one wave of the SAME workgroup replays the batch into the
// pixels' statistics (RecordSample / IsConverged in sample order, lane = pixel) and lays out
// the tile's next batch in LDS.  A workgroup keeps up to kTileNT tiles in flight, so its lanes
// trace the other tiles while one waits for its batch's last paths: there is no launch drain
// between phases, and every hand-off stays inside one CU (LDS counters, workgroup-scope
// release / acquire), so no cross-XCD visibility is needed.  Largest tiles first keeps the
// launch's end short: the last tiles claimed are the cheapest.
// ---------------------------------------------------------------------------------------
constexpr int kTileTP = 8;   // most pixels per tile (the record runs one lane per pixel; TileArgs::tp)
constexpr int kTileNT = 10;  // most tiles in flight per workgroup (TileArgs::nt)
struct PixelSoA {
  double *sum, *mean, *m2;  // 3 x npix each (channel-major)
  int32_t* samples;
  uint8_t* conv;
};
// What the tile launch reads (device memory; its address is word 8 * 16 + 6 of the slot
// counter block, like the slot map's in MAP == 1 launches).
struct TileArgs {
  const uint32_t* act;     // subset pixels still sampling after the first pass, in image order
  const uint32_t* order;   // tile ids (tile t = act[t * tp ...]) in claim order, region by region
  const uint32_t* rcount;  // tiles of each of the 8 regions
  const uint32_t* knext;   // each pixel's predicted further samples (k_adapt_record of the first pass)
  const uint32_t* nact;    // the number of active pixels
  double* L;               // radiance: two batches of tp * kcap slots per (block, descriptor)
  uint16_t* segs;          // counting builds: each slot's path segments (same indexing), else null
  unsigned long long* rec_segs;  // counting builds: segments of the recorded samples
  PixelSoA px;
  int64_t npix;
  int32_t kcap;      // largest batch of one pixel
  int32_t min_spp, budget;
  int32_t kinc;      // smallest further batch of a pixel not yet converged
  int32_t max_blocks;  // blocks the radiance workspace has room for
  int32_t k1;          // act == nullptr: the launch runs the first pass too (every pixel, tiles in
                       // image order, first batch k1 = min_spp samples; order and knext unused)
  int32_t tp, nt;      // pixels per tile (<= kTileTP), tiles in flight per workgroup (<= kTileNT)
  int32_t tail_px;     // a tile with at most this many pixels left sampling gives them the rest of
                       // their budget (within kcap): no further phase chains
  int32_t split;       // a pixel's predicted samples are traced as two batches (front, back) when
                       // there are more than this many
  double rel, margin;
  double margin_step;  // the margin grows by this much with every batch of the tile
  double starve_gain;  // ... and by this much per wave of the block idle at the record (no work to claim)
};
// A tile in flight (LDS).  Its pixels' predicted samples are traced as two pipelined batches in
// two buffers: the FRONT batch (recorded next, in sample order) and the BACK batch (the samples
// that follow), both laid out at once, front first in claim order, so the block traces the back
// batch while the front's last paths finish instead of waiting for the front's record.  A
// buffer: word = (cursor << 32) | T: its T slots are claimed by adding to the cursor (an add
// returns T with it, so a claim is consistent even when it races a re-layout); rem counts its
// paths still running; slot s is sample s0[i] + (s - off[i]) of pixel pix[i], off[i] <= s <
// off[i + 1].  Only the wave holding the tile's lock (its claim, then one record at a time)
// lays out batches.
struct TileBuf {
  unsigned long long word;
  uint32_t rem, pad_;
  uint32_t off[kTileTP + 1];
  uint32_t s0[kTileTP];
  uint32_t pad2_;
};
struct TileDesc {
  TileBuf b[2];
  uint32_t state;  // 0 free, 1 being initialised, 2 in flight
  uint32_t npx, phase;
  uint32_t front;  // the front buffer (0 / 1); the other one holds the back batch
  uint32_t done;   // bit b: buffer b's batch has ended (its last path counted off), not yet recorded
  uint32_t lock;   // 1: a wave lays out this tile's batches (its claim or a record)
  uint32_t pix[kTileTP];
  uint32_t fin[kTileTP];  // 1: the pixel is finished (converged or out of budget)
};
constexpr uint32_t kTileDone = 0xFFFFFFFFu;
struct TileLds {
  uint32_t ready;      // descriptors one of whose batches has ended (their records are due)
  uint32_t exhausted;  // the claim order is used up
  uint32_t idle;       // waves of the block waiting for work (no path, nothing to claim)
  uint32_t avail;      // bit 2 j + b: buffer b of descriptor j may have unclaimed slots
  TileDesc d[kTileNT];
  // each wave's record keeps the pixels' statistics here (sum, mean, M2 by channel, pixel
  // interleaved), not in registers: the record runs inside the persistent loop, where every
  // register of the walk is taken
  double rec[kBlock / 64][9][kTileTP];
};
static_assert(sizeof(TileBuf) % 8 == 0 && sizeof(TileDesc) % 8 == 0 && sizeof(TileLds) % 8 == 0,
              "8-byte aligned tile descriptors");

// PARK: 0 the plain schedule, 1 the PARK schedule with the leaf-step walk (trace4_run_step),
// 2 the PARK schedule with the speculative walk (trace4_run_spec; trees of at most
// kSpecMaxNodes nodes, its stack entries being 16-bit)
constexpr bool spec_walk(int park, bool fast, bool scatter) { return park == 2 && fast && !scatter; }
constexpr int64_t kSpecMaxNodes = 65536;
// The slot chunks of an adaptive phase launch (MAP == 1), one word per wave of the block: a
// chunk of kChunk slots of one slot region, claimed by LDS adds to its cursor, by its wave and,
// once the slot counters are dry, by the other waves of the block too.
// word = region (3 bits) | chunk index in the region (29 bits) | cursor (32 bits)
struct ChunkLds {
  unsigned long long w[kBlock / 64];
};
// block-wide region after the per-lane ones: 0 none, 1 the chunk words (MAP == 1), 2 the tile
// schedule's descriptors (MAP == 2)
constexpr uint32_t block_region_bytes(int kind) {
  return kind == 2 ? (uint32_t)sizeof(TileLds) : kind == 1 ? (uint32_t)sizeof(ChunkLds) : 0u;
}
// which block-wide region a launch of k_persistent<..., SCATTER, ..., MAP> has
constexpr int block_region_kind(int map, bool scatter) {
  return map == 2 ? 2 : (map == 1 || (map == 0 && RTX_SHARED_CHUNKS0 && !scatter)) ? 1 : 0;
}
constexpr PersistLds persist_lds(int stack_slots, bool spec, int block_region = 0) {
  const uint32_t stack_bytes = (uint32_t)stack_slots * kBlock * (spec ? 2u : 4u);
  const uint32_t thr = (stack_bytes + 7u) & ~7u, hitp = thr + 3u * kBlock * 8u, leafq = hitp + 3u * kBlock * 8u;
  const uint32_t tl = leafq + (spec ? (uint32_t)kLeafQueue * kBlock * 4u : 0u);
  return PersistLds{0u, thr, hitp, leafq, tl, tl + block_region_bytes(block_region)};
}

template <int STACK, bool FAST, bool COUNT, int TK = -1>
__device__ __forceinline__ int64_t trace(const DScene& S, V3 o, V3 d, double tmin, double tmax, uint32_t* stk,
                                         Counters& c, double& t_best, int32_t& mat_best) {
  if (FAST) return trace_fast4_lean<STACK, COUNT, TK>(S, o, d, tmin, tmax, stk, kBlock, c, t_best, mat_best);
  const int64_t b = trace_parity<STACK, COUNT>(S, o, d, tmin, tmax, stk, kBlock, c, t_best);
  mat_best = b >= 0 ? S.prims[b].material : -1;
  return b;
}
template <int STACK, bool FAST, bool COUNT>
__device__ __forceinline__ int64_t trace(const DScene& S, V3 o, V3 d, double tmin, double tmax, uint32_t* stk,
                                         Counters& c, double& t_best) {
  int32_t m;
  return trace<STACK, FAST, COUNT>(S, o, d, tmin, tmax, stk, c, t_best, m);
}

__device__ __forceinline__ void flush_counters(const RenderArgs& A, const Counters& c, uint32_t segs,
                                               uint32_t prims, bool count) {
  if (count) {
    atomicAdd(&A.counters[2], (unsigned long long)c.nodes);
    atomicAdd(&A.counters[3], (unsigned long long)c.prims);
    atomicAdd(&A.counters[4], (unsigned long long)c.wnodes);
    atomicAdd(&A.counters[5], (unsigned long long)c.wprims);
    atomicAdd(&A.counters[6], (unsigned long long)c.tris);
    atomicAdd(&A.counters[7], (unsigned long long)c.sphs);
    if (c.witers) atomicAdd(&A.counters[10], (unsigned long long)c.witers);
    if (c.widle) atomicAdd(&A.counters[11], (unsigned long long)c.widle);
    if (c.wlive) atomicAdd(&A.counters[12], (unsigned long long)c.wlive);
  }
  if (segs) atomicAdd(&A.counters[0], (unsigned long long)segs);
  if (prims) atomicAdd(&A.counters[1], (unsigned long long)prims);
}

// ---------------------------------------------------------------------------------------
// IntersectBatch
// ---------------------------------------------------------------------------------------
template <int STACK, bool FAST>
__global__ __launch_bounds__(kBlock, kTraceWaves) void k_intersect(DScene S, const rtx_ray* __restrict__ rays,
                                                                       int64_t n, rtx_hit* __restrict__ hits,
                                                                       double tmin, double tmax) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* stk = lds + threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const rtx_ray r = rays[i];
  V3 o{r.origin[0], r.origin[1], r.origin[2]}, d{r.direction[0], r.direction[1], r.direction[2]};
  Counters c{};
  double tb;
  const int64_t best = trace<STACK, FAST, false>(S, o, d, tmin, tmax, stk, c, tb);
  rtx_hit out;
  out.pad_ = 0;
  if (best >= 0) {
    Hit h;
    finish_hit_at(S, best, tb, o, d, h);
    out.hit = 1;
    out.front_face = h.front_face, out.material = h.mat, out.t = h.t;
    out.p[0] = h.p.x, out.p[1] = h.p.y, out.p[2] = h.p.z;
    out.normal[0] = h.normal.x, out.normal[1] = h.normal.y, out.normal[2] = h.normal.z;
    out.u = h.u, out.v = h.v;
  } else {
    out.hit = 0, out.front_face = 0, out.material = -1, out.t = 0;
    out.p[0] = out.p[1] = out.p[2] = 0;
    out.normal[0] = out.normal[1] = out.normal[2] = 0;
    out.u = out.v = 0;
  }
  hits[i] = out;
}

// ---------------------------------------------------------------------------------------
// Wavefront: primary generation for every slot of active pixels
// ---------------------------------------------------------------------------------------
#ifndef RTX_PERSISTENT_ONLY  // rtx_park.hip: the persistent kernel's PARK instantiations only
__global__ __launch_bounds__(kBlock) void k_wf_generate(RenderArgs A, PathQueue q, unsigned int* count) {
  const int64_t nslots = A.npix * A.K;
  uint32_t made = 0;
  for (int64_t base = (int64_t)blockIdx.x * kBlock; base < nslots; base += (int64_t)gridDim.x * kBlock) {
    const int64_t slot = base + threadIdx.x;
    bool live = slot < nslots;
    int64_t p = live ? slot / A.K : 0;
    if (live && A.conv && A.conv[p]) live = false;
    Path P;
    if (live) {
      const int k = (int)(slot - p * A.K);
      int x, y;
      A.map.xy(p, x, y);
      Rng g = make_rng(A.seed, (uint32_t)(y * A.map.W + x), (uint32_t)(A.s0 + k), 0u);
      get_ray(A.cam, x, y, g, P.o, P.d);
      made++;
    }
    const int64_t dst = wave_compact(live, count);
    if (live) {
      q.ox[dst] = P.o.x, q.oy[dst] = P.o.y, q.oz[dst] = P.o.z;
      q.dx[dst] = P.d.x, q.dy[dst] = P.d.y, q.dz[dst] = P.d.z;
      q.tx[dst] = 1.0, q.ty[dst] = 1.0, q.tz[dst] = 1.0;
      q.slot[dst] = (uint32_t)slot;
      q.meta[dst] = 0u;  // depth 0
    }
  }
  flush_counters(A, Counters{}, 0, made, false);
}
#endif

// Closest hit for every queued path (one ray per lane, grid-stride).
template <int STACK, bool FAST, bool COUNT>
__global__ __launch_bounds__(kBlock, kTraceWaves) void k_wf_extend(RenderArgs A, PathQueue q,
                                                                       const unsigned int* count) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* stk = lds + threadIdx.x;
  const int64_t n = *count;
  Counters c{};
  uint32_t segs = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const V3 o = v3(q.ox[i], q.oy[i], q.oz[i]);
    const V3 d = v3(q.dx[i], q.dy[i], q.dz[i]);
    double tb;
    q.hit[i] = (int32_t)trace<STACK, FAST, COUNT>(A.S, o, d, (double)0.001f, kInf, stk, c, tb);
    segs++;
  }
  flush_counters(A, c, segs, 0, COUNT);
}

// Shading for every queued path + compacted child queue (wavefront.cc:109-217).
#ifndef RTX_PERSISTENT_ONLY  // rtx_park.hip: the persistent kernel's PARK instantiations only
__global__ __launch_bounds__(kBlock) void k_wf_shade(RenderArgs A, PathQueue in, const unsigned int* in_count,
                                                     PathQueue out, unsigned int* out_count) {
  const int64_t n = *in_count;
  for (int64_t base = (int64_t)blockIdx.x * kBlock; base < n; base += (int64_t)gridDim.x * kBlock) {
    const int64_t i = base + threadIdx.x;
    bool cont = false;
    Path P;
    uint32_t slot = 0;
    if (i < n) {
      P.o = v3(in.ox[i], in.oy[i], in.oz[i]);
      P.d = v3(in.dx[i], in.dy[i], in.dz[i]);
      P.thr = v3(in.tx[i], in.ty[i], in.tz[i]);
      slot = in.slot[i];
      const uint32_t meta = in.meta[i];
      P.depth = (int32_t)meta;
      const int64_t p = slot / A.K;
      const int k = (int)(slot - p * A.K);
      int x, y;
      A.map.xy(p, x, y);
      const int32_t best = in.hit[i];
      Hit h;
      if (best >= 0) finish_hit<false>(A.S, best, P.o, P.d, (double)0.001f, h);
      Rng g = make_rng(A.seed, (uint32_t)(y * A.map.W + x), (uint32_t)(A.s0 + k), (uint32_t)P.depth + 1u);
      V3 L;
      cont = shade(A.S, A.max_depth, P, h, best >= 0, g, L);
      if (!cont) {
        store_radiance(A, (uint32_t)slot, L);
      }
    }
    const int64_t dst = wave_compact(cont, out_count);
    if (cont) {
      out.ox[dst] = P.o.x, out.oy[dst] = P.o.y, out.oz[dst] = P.o.z;
      out.dx[dst] = P.d.x, out.dy[dst] = P.d.y, out.dz[dst] = P.d.z;
      out.tx[dst] = P.thr.x, out.ty[dst] = P.thr.y, out.tz[dst] = P.thr.z;
      out.slot[dst] = slot;
      out.meta[dst] = (uint32_t)P.depth;
    }
  }
}
#endif

// ---------------------------------------------------------------------------------------
// One pixel's RecordSample (pixel_state.h:22-39) over K radiance records in sample order, each
// followed by IsConverged (pixel_state.h:54-72), stopping at convergence; the statistics come
// in and go out through r.  AHEAD: the loads of the next samples kept in flight while the
// current one is replayed.  Used by k_adapt_record (a kernel of its own) and by the tile
// schedule's record inside the persistent kernel (fewer loads ahead: registers).
// ---------------------------------------------------------------------------------------
struct PixRec {
  double sum[3], mean[3], m2[3];
  int n;
  bool conv;
};
template <int AHEAD>
__device__ __forceinline__ void replay_pixel(PixRec& r, const double* __restrict__ Lp, int K, int min_spp,
                                             double rel) {
  auto record = [&](const double (&x)[3]) {
    r.n++;
    for (int c = 0; c < 3; c++) {
      double mu = r.mean[c];
      double delta = x[c] - mu;
      mu += delta / r.n;
      double delta2 = x[c] - mu;
      r.mean[c] = mu;
      r.m2[c] += delta2 * delta;
    }
    for (int c = 0; c < 3; c++) r.sum[c] += x[c];
    if (r.n >= min_spp) {
      // err / mu > rel  <=>  m2 > rel^2 (n - 1) n mu^2 up to the few ulps the exact form rounds
      // by: decided by products where the two sides differ by more than 1e-10 relative (the
      // usual case), the exact form (two divisions, two square roots) only in between; NaN
      // fails both comparisons and takes the exact form too.
      // (channels in order, the first failing one decides; unrolled, so the statistics stay in
      // registers)
      bool ok = true;
#pragma unroll
      for (int c = 0; c < 3; c++) {
        if (ok) {
          double mu = fmax(fabs(r.mean[c]), 1e-3);
          const double thr = rel * rel * ((double)(r.n - 1) * (double)r.n * (mu * mu));
          if (r.m2[c] > thr * (1.0 + 1e-10)) {
            ok = false;
          } else if (!(r.m2[c] < thr * (1.0 - 1e-10))) {
            double var = r.n > 1 ? r.m2[c] / (r.n - 1) : 0.0;
            double err = sqrt(var) / sqrt((double)r.n);
            if (err / mu > rel) ok = false;
          }
        }
      }
      r.conv = ok;
    }
  };
  double b[AHEAD][3];
  auto load = [&](int slot, int k) {
    if (k < K)
      for (int c = 0; c < 3; c++) b[slot][c] = Lp[3 * k + c];
  };
#pragma unroll
  for (int i = 0; i < AHEAD; i++) load(i, i);
  for (int k = 0; k < K && !r.conv; k += AHEAD) {
#pragma unroll
    for (int i = 0; i < AHEAD; i++) {
      if (k + i >= K || r.conv) break;
      record(b[i]);
      load(i, k + i + AHEAD);
    }
  }
}
// replay_pixel's arithmetic, in the same order, on statistics held in LDS (st[q * kTileTP]: sum
// 0-2, mean 3-5, M2 6-8, one column per pixel): the tile schedule's record inside the persistent
// loop (volatile: every step reads and writes them, none is kept in a register).
__device__ __forceinline__ void replay_pixel_lds(volatile double* st, int& n, bool& conv, const double* __restrict__ Lp,
                                                 int K, int min_spp, double rel) {
  constexpr int S = kTileTP;
  for (int k = 0; k < K && !conv; k++) {
    double x[3];
    for (int c = 0; c < 3; c++) x[c] = Lp[3 * k + c];
    n++;
    for (int c = 0; c < 3; c++) {
      double mu = st[(3 + c) * S];
      double delta = x[c] - mu;
      mu += delta / n;
      double delta2 = x[c] - mu;
      st[(3 + c) * S] = mu;
      st[(6 + c) * S] = st[(6 + c) * S] + delta2 * delta;
    }
    for (int c = 0; c < 3; c++) st[c * S] = st[c * S] + x[c];
    if (n >= min_spp) {
      bool ok = true;
#pragma unroll
      for (int c = 0; c < 3; c++) {
        if (ok) {
          const double m2 = st[(6 + c) * S];
          double mu = fmax(fabs(st[(3 + c) * S]), 1e-3);
          const double thr = rel * rel * ((double)(n - 1) * (double)n * (mu * mu));
          if (m2 > thr * (1.0 + 1e-10)) {
            ok = false;
          } else if (!(m2 < thr * (1.0 - 1e-10))) {
            double var = n > 1 ? m2 / (n - 1) : 0.0;
            double err = sqrt(var) / sqrt((double)n);
            if (err / mu > rel) ok = false;
          }
        }
      }
      conv = ok;
    }
  }
}
__device__ __forceinline__ void load_pixel(PixRec& r, const PixelSoA& px, int64_t npix, int64_t p) {
  for (int c = 0; c < 3; c++) r.sum[c] = px.sum[c * npix + p], r.mean[c] = px.mean[c * npix + p], r.m2[c] = px.m2[c * npix + p];
  r.n = px.samples[p];
  r.conv = false;
}
__device__ __forceinline__ void store_pixel(const PixRec& r, const PixelSoA& px, int64_t npix, int64_t p) {
  for (int c = 0; c < 3; c++) px.sum[c * npix + p] = r.sum[c], px.mean[c * npix + p] = r.mean[c], px.m2[c * npix + p] = r.m2[c];
  px.samples[p] = r.n;
  px.conv[p] = r.conv;
}

// ---- the tile schedule's pieces (see TileArgs) ----
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if ((int)lane_id() >= o) v += t;
  }
  return v;
}
// A pixel's predicted further samples once a batch is recorded and it is neither converged nor
// out of budget: IsConverged holds at n samples once n >= var / (rel * max(|mean|, 1e-3))^2 in
// every channel, so that many more samples (times the margin), at least kinc, within the budget
// and the workspace.  Only the amount of work depends on it, never the result: a sample traced
// past the pixel's convergence point is discarded by the record.
// (st: the pixel's statistics in the record's LDS columns, as replay_pixel_lds keeps them)
__device__ __forceinline__ uint32_t tile_next_batch(volatile const double* st, int n, const TileArgs* ta,
                                                    uint32_t phase, uint32_t idle) {
  const double rel = ta->rel;
  double need = 0.0;
  for (int c = 0; c < 3; c++) {
    const double var = n > 1 ? st[(6 + c) * kTileTP] / (n - 1) : 0.0;
    const double mu = fmax(fabs(st[(3 + c) * kTileTP]), 1e-3);
    need = fmax(need, var / (rel * rel * mu * mu));
  }
  const int left = ta->budget - n;
  const double want = (need - (double)n) * (ta->margin + ta->margin_step * (double)phase + ta->starve_gain * (double)idle);
  int k = (want < (double)left) ? (int)ceil(want) : left;  // NaN / inf: the whole budget
  k = max(k, min(ta->kinc, left));
  return (uint32_t)min(k, left);
}
// The front share of a pixel's predicted samples kt (the rest goes to the back batch).
__device__ __forceinline__ uint32_t tile_front_share(uint32_t kt, const TileArgs* ta) {
  const uint32_t f = kt > (uint32_t)ta->split ? (kt + 1u) / 2u : kt;
  return min(f, (uint32_t)ta->kcap);
}
// Slot index of the tile workspace: descriptor j of this block, buffer b, batch slot s.
__device__ __forceinline__ uint64_t tile_slot(const TileArgs* ta, int j, int b, uint32_t s) {
  return ((uint64_t)((blockIdx.x * (uint32_t)ta->nt + (uint32_t)j) * 2u + (uint32_t)b) * (uint32_t)ta->tp) *
             (uint64_t)ta->kcap + s;
}
// Lays out buffer b of descriptor j: pixel i takes k samples from sample s, and publishes it
// (wave-uniform; the whole wave; lanes >= npx pass k = 0).  A batch without slots is ended at
// once (its done bit).  Returns the batch's slot count.
__device__ __forceinline__ uint32_t tile_layout(TileLds* tl, int j, int b, int npx, uint32_t k, uint32_t s) {
  TileDesc& d = tl->d[j];
  const int i = (int)lane_id();
  const uint32_t inc = wave_incl_scan(k);
  const uint32_t T = __shfl(inc, 63);
  TileBuf& B = d.b[b];
  if (i < npx) B.off[i] = inc - k, B.s0[i] = s;
  if (i == 0) B.off[npx] = T, B.rem = T;
  // the layout (LDS) and every statistic (global) complete before the slots are claimable
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (i == 0) {
    atomicExch(&B.word, (unsigned long long)T);
    if (T) atomicOr(&tl->avail, 1u << (2 * j + b));
    else atomicOr(&d.done, 1u << b);
  }
  return T;
}
// Claims a free descriptor and the next tile in claim order (this block's region first, then
// the others) and lays out its front and back batches (wave-uniform; the whole wave).  false:
// no free descriptor, or the claim order is used up (then tl->exhausted is set).
__device__ __forceinline__ bool tile_claim(TileLds* tl, const TileArgs* ta, unsigned long long* ctr, uint32_t region,
                                           int& claimed, unsigned long long* tstat = nullptr) {
  claimed = -1;  // the descriptor claimed (its lock held: the caller runs tile_unlock)
  int j = -1;
  const int nt = ta->nt;
  if (lane_id() == 0)
    for (int q = 0; q < nt; q++)
      if (atomicCAS(&tl->d[q].state, 0u, 1u) == 0u) {
        j = q;
        break;
      }
  j = __shfl(j, 0);
  if (j < 0) return false;
  int tid = -1;
  if (lane_id() == 0) {
    for (int tries = 0; tries < 8 && tid < 0; tries++) {
      const uint32_t r = (region + tries) & 7;
      uint32_t base = 0;
      for (uint32_t q = 0; q < r; q++) base += ta->rcount[q];
      const uint32_t cnt = ta->rcount[r];
      if (cnt == 0) continue;
      const unsigned long long t = atomicAdd(ctr + 16 * r, 1ull);
      if (t < cnt) tid = ta->act ? (int)ta->order[base + (uint32_t)t] : (int)(base + (uint32_t)t);
    }
  }
  tid = __shfl(tid, 0);
  TileDesc& d = tl->d[j];
  if (tid < 0) {
    if (lane_id() == 0) {
      if (tstat && atomicExch(&tl->exhausted, 1u) == 0u) {  // (counting builds: the timeline)
        const unsigned long long t = (unsigned long long)wall_clock64();
        atomicMax(tstat + 14, t);
        atomicMax(tstat + 15, ~t);
      }
      atomicExch(&tl->exhausted, 1u);
      atomicExch(&d.state, 0u);
    }
    return false;
  }
  // the lock (released by tile_unlock): a wave still holding it found a stale ready bit
  // of the descriptor's last tile, and lets go at once
  if (lane_id() == 0)
    while (atomicCAS(&d.lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
  const uint32_t first = (uint32_t)tid * (uint32_t)ta->tp, nact = *ta->nact;
  const int n = (int)min<uint32_t>((uint32_t)ta->tp, nact - first);
  const int i = (int)lane_id();
  uint32_t p = 0, kt = 0, s = 0;
  if (i < n) {
    if (ta->act) p = ta->act[first + i], kt = ta->knext[p];
    else p = first + (uint32_t)i, kt = (uint32_t)ta->k1;
    s = (uint32_t)ta->px.samples[p];
  }
  // the first pass of a one-launch render is not split: nothing is predicted before it
  const uint32_t f = ta->act ? tile_front_share(kt, ta) : kt;
  if (i < n) d.pix[i] = p, d.fin[i] = 0u;
  if (i == 0) d.npx = (uint32_t)n, d.phase = 0, d.front = 0, d.done = 0;
  const uint32_t T = tile_layout(tl, j, 0, n, f, s);
  tile_layout(tl, j, 1, n, min(kt - f, (uint32_t)ta->kcap), s + f);
  if (i == 0) atomicExch(&d.state, 2u);  // (an active pixel always has a batch)
  claimed = j;
  return T != 0;
}
// Records the front batch of descriptor j while it has ended: replay it into the pixels'
// statistics (lane i = pixel i of the tile); the back batch becomes the front, and the samples
// predicted beyond it are laid out as the new back batch in the buffer just recorded
// (wave-uniform; the whole wave; one wave per tile at a time: it claims the front's done bit).
// (the caller holds the tile's lock; true: the tile has ended, its descriptor and lock are free)
template <bool COUNT>
__device__ __forceinline__ bool tile_record_locked(TileLds* tl, const TileArgs* ta, int j) {
  TileDesc& d = tl->d[j];
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // every lane's radiance store, before its count-off
  const int i = (int)lane_id();
  const int n = (int)d.npx;
  while (true) {
    const int fb = (int)d.front, bb = fb ^ 1;
    uint32_t old = 0;
    if (i == 0) old = atomicAnd(&d.done, ~(1u << fb));
    old = __shfl(old, 0);
    if (!(old & (1u << fb))) break;  // the front batch is still running
    if (__ballot(i < n && d.fin[i] == 0u) == 0) {
      // every pixel is finished: the tile ends once the back batch has no path running
      const bool end = (old & (1u << bb)) != 0u;
      if (i == 0) {
        if (end) {
          atomicAnd(&d.done, ~(1u << bb));
          atomicAnd(&tl->avail, ~(3u << (2 * j)));
          atomicExch(&d.lock, 0u);
          atomicExch(&d.state, 0u);
        } else {
          atomicOr(&d.done, 1u << fb);  // (empty: the back's record finds it ended)
          d.front = (uint32_t)bb;
        }
      }
      return end;
    }
    const uint32_t idle = *(volatile uint32_t*)&tl->idle;
    const bool exh = *(volatile uint32_t*)&tl->exhausted != 0u;
    uint32_t kt = 0, nrec = 0;
    bool live = false;  // the pixel is still sampling after this batch
    if (i < n && d.fin[i] == 0u) {
      const uint32_t p = d.pix[i], o0 = d.b[fb].off[i], K = d.b[fb].off[i + 1] - o0;
      const PixelSoA& px = ta->px;
      const int64_t np = ta->npix;
      volatile double* st = &tl->rec[threadIdx.x >> 6][0][i];
      int nn = px.samples[p];
      bool conv = false;
      const int n0 = nn;
      for (int c = 0; c < 3; c++)
        st[c * kTileTP] = px.sum[c * np + p], st[(3 + c) * kTileTP] = px.mean[c * np + p],
        st[(6 + c) * kTileTP] = px.m2[c * np + p];
      if (K > 0) {
        const uint64_t base = tile_slot(ta, j, fb, o0);
        replay_pixel_lds(st, nn, conv, ta->L + 3 * base, (int)K, ta->min_spp, ta->rel);
        if (COUNT) {  // the segments of the samples recorded (the rest are discarded)
          unsigned long long t = 0;
          for (int k = 0; k < nn - n0; k++) t += ta->segs[base + k];
          atomicAdd(ta->rec_segs, t);
        }
        for (int c = 0; c < 3; c++)
          px.sum[c * np + p] = st[c * kTileTP], px.mean[c * np + p] = st[(3 + c) * kTileTP],
          px.m2[c * np + p] = st[(6 + c) * kTileTP];
        px.samples[p] = nn;
        px.conv[p] = conv;
      }
      live = !conv && nn < ta->budget;
      if (live) {
        kt = tile_next_batch(st, nn, ta, d.phase, idle);
      } else {
        d.fin[i] = 1u;
      }
      nrec = (uint32_t)nn;
    }
    // few pixels left sampling, or nothing left to claim: the rest of their budget now, rather
    // than further batches of a few paths each
    if (live && (exh || (int)__popcll(__ballot(live)) <= ta->tail_px)) kt = (uint32_t)(ta->budget - (int)nrec);
    // a live pixel's back samples follow the ones just recorded (nrec == its back batch's first
    // sample); what its prediction wants beyond them goes in the new back batch
    uint32_t kb = 0, sb = 0;
    if (i < n) kb = d.b[bb].off[i + 1] - d.b[bb].off[i], sb = d.b[bb].s0[i];
    const uint32_t kn = live ? min(kt > kb ? kt - kb : 0u, (uint32_t)ta->kcap) : 0u;
    if (i == 0) d.front = (uint32_t)bb, d.phase = d.phase + 1u;
    tile_layout(tl, j, fb, n, kn, sb + kb);
  }
  return false;
}
// Releases the tile's lock.  A batch that ended meanwhile (its ready bit taken by a wave that
// found the lock held) is marked ready again, for the next wave at the top of its loop.
__device__ __forceinline__ void tile_unlock(TileLds* tl, int j) {
  TileDesc& d = tl->d[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane_id() == 0) {
    atomicExch(&d.lock, 0u);
    const uint32_t f = *(volatile uint32_t*)&d.front, dn = *(volatile uint32_t*)&d.done;
    if (dn & (1u << f)) atomicOr(&tl->ready, 1u << j);
  }
}
// Records descriptor j's ended batches unless another wave holds its lock (that wave looks
// again when it lets go).  (Wave-uniform; the whole wave.)
template <bool COUNT>
__device__ __forceinline__ void tile_record(TileLds* tl, const TileArgs* ta, int j) {
  uint32_t got = 0;
  if (lane_id() == 0) got = atomicCAS(&tl->d[j].lock, 0u, 1u) == 0u ? 1u : 0u;
  if (!__builtin_amdgcn_readfirstlane(got)) return;
  if (!tile_record_locked<COUNT>(tl, ta, j)) tile_unlock(tl, j);
}
// The wave's exit test: no tile left to claim, none in flight.
__device__ __forceinline__ bool tiles_done(const TileLds* tl) {
  bool busy = false;
#pragma unroll
  for (int q = 0; q < kTileNT; q++) busy |= ((const volatile uint32_t*)&tl->d[q].state)[0] != 0u;
  return *(const volatile uint32_t*)&tl->exhausted && !busy && *(const volatile uint32_t*)&tl->ready == 0u;
}

// ---------------------------------------------------------------------------------------
// Persistent lanes: each lane owns one path at a time and refills from a global slot
// counter in wave-sized chunks (one atomic per kChunk slots), so lanes whose path ended
// (miss, emitter, absorption, Russian roulette) are immediately given a new primary —
// the per-wave __ballot of idle lanes is the active-ray compaction.
// ---------------------------------------------------------------------------------------
// TK >= 0: every primitive in the fast tree has kind TK (the ground sphere is a global
// primitive, so the bunny's tree holds triangles, the final and mixed scenes' spheres), so
// the walk's leaf tests are compiled for that kind alone.
// Which slots the kernel draws: uniform groups (MAP = 0), slot p * K + k is sample s0 + k of
// pixel p; adaptive phases with a slot map (MAP = 1; the default adaptive render), slot i is sample
// smap[i].y of pixel smap[i].x for i below the phase's slot count, where the slot counters'
// block holds, after the 8 region counters, the slot count (next_slot[128]) and the slot map's
// address (next_slot[130]), both written by k_adapt_expand; the adaptive tile schedule (MAP =
// 2, RTX_FLAG_ADAPT_TILES, after the first pass), slots of the tiles in flight in the
// block's LDS descriptors (TileArgs at next_slot[134]).  MAP is a template parameter, not a
// kernel argument: the fixed-spp kernels run at the SGPR limit, and any extra uniform state
// there reshuffles their register allocation (a runtime switch cost the bunny's build 3.7 %, r3d).
template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK, int TK = -1, bool LAMB = false,
          bool NOTEX = false, bool NODOF = false, int MAP = 0>
__global__ __launch_bounds__(kBlock, kTraceWaves) void k_persistent(RenderArgs A, unsigned long long* next_slot) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  // the LDS layout (persist_lds: the launch sizes it the same way; the host launches PARK
  // kernels only for fast, non-scatter renders)
  constexpr bool kSpecLds = spec_walk(PARK, FAST, SCATTER);
  constexpr bool kTiles = MAP == 2;
  constexpr bool kShared = block_region_kind(MAP, SCATTER) == 1;  // block-shared slot chunks (ChunkLds)
  const PersistLds lay = persist_lds(A.stack_slots, kSpecLds, block_region_kind(MAP, SCATTER));
  char* const ldsb = (char*)lds;
  TileLds* const tl = (TileLds*)(ldsb + lay.tiles);  // (kTiles)
  const TileArgs* const ta = kTiles ? (const TileArgs*)next_slot[8 * 16 + 6] : nullptr;
  (void)tl, (void)ta;
  // counting builds: the launch's timeline (wall clock, 100 MHz): [13] ~first block start,
  // [14] last wave to find the slots (tiles: the claim order) used up, [15] ~first one, [16]
  // last wave end, [17] ~first wave end
  if (COUNT && threadIdx.x == 0) atomicMax(&A.counters[13], ~(unsigned long long)wall_clock64());
  if (kTiles) {
    if (blockIdx.x >= (uint32_t)ta->max_blocks) return;  // (the host sizes the grid within it)
    for (uint32_t w = threadIdx.x; w < sizeof(TileLds) / 4; w += kBlock) ((uint32_t*)tl)[w] = 0u;
    __syncthreads();
  }
  unsigned long long* const cw = (unsigned long long*)(ldsb + lay.tiles);  // (kShared) the chunk words
  (void)cw;
  if (kShared) {
    if (threadIdx.x < kBlock / 64) cw[threadIdx.x] = (unsigned long long)kChunkShared;  // (no chunk: cursor past any)
    __syncthreads();
  }
  uint32_t* stk = (uint32_t*)(ldsb + lay.stack) + threadIdx.x;
  uint16_t* stk16 = (uint16_t*)(ldsb + lay.stack) + threadIdx.x;  // (kSpecLds)
  (void)stk16;
  double* thr_lds = (double*)(ldsb + lay.thr) + threadIdx.x;    // [c * kBlock]
  double* hitp_lds = (double*)(ldsb + lay.hitp) + threadIdx.x;  // [c * kBlock]
  uint32_t* leafq = (uint32_t*)(ldsb + lay.leafq) + threadIdx.x;  // (kSpecLds)
  (void)leafq;
  // nothing else reads rec.p (textured builds: once the texture lookups moved before the sampling)
  constexpr bool kHitpLds = (NOTEX || RTX_EARLY_TEX) && !SCATTER;
  (void)hitp_lds;
  const uint64_t nslots = MAP == 1 ? (uint64_t)next_slot[8 * 16] : (uint64_t)A.npix * (uint64_t)A.K;
  // GetPixel uses Interval(0.001, inf) (camera.h:158); IntersectBatch uses 0.001f (cpu_ray_integrator.h:21)
  const double tmin = SCATTER ? 0.001 : (double)0.001f;
  Counters c{};
  uint32_t segs = 0, prims = 0;
  // counting builds: the lane's path segments, stored per slot when the launch's slot counter
  // block names a buffer for them (adaptive renders: the segments of the recorded samples)
  uint32_t pseg = 0;
  uint16_t* const segbuf = !COUNT ? nullptr : kTiles ? ta->segs : (uint16_t*)next_slot[8 * 16 + 4];
  (void)pseg, (void)segbuf;
  uint64_t chunk_base = 0, chunk_left = 0;  // wave-uniform
  bool exhausted = false;                   // wave-uniform
  bool dry = false;                         // (kShared) wave-uniform: the slot counters are used up
  uint32_t region = blockIdx.x & 7;         // wave-uniform
  bool has = false;
  Path P;
  P.depth = 0;
  uint32_t slot = 0;           // < nslots <= 2^32 - 1 (host check)
  uint32_t pix = 0, smp = 0;  // RNG identity of the lane's path: global pixel, sample
  // A traversal still running when at most kParkAt lanes of the wave are left walking is
  // parked (trace4_run) and resumed in the next segment round, so the wave goes on to shade
  // the finished lanes instead of idling behind a few long walks.
  // (PARK instantiation only: the host picks it per scene, see rtx_render_device.)
  constexpr bool kPark = PARK > 0 && FAST && !SCATTER;
  const bool park_ok = kPark && A.S.use_bvh && !A.S.froot_leaf;
  bool parked = false;
  bool waiting = false;  // (tile schedule: the wave is counted in tl->idle)
  TravState trs;
  while (true) {
    if constexpr (kTiles) {  // a tile whose batch has ended is recorded first (at most one per round)
      const uint32_t rdy = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&tl->ready);
      if (rdy) {
        const int j = __builtin_ctz(rdy);
        uint32_t old = 0;
        if (lane_id() == 0) old = atomicAnd(&tl->ready, ~(1u << j));
        old = __builtin_amdgcn_readfirstlane(old);
        if (old & (1u << j)) tile_record<COUNT>(tl, ta, j);
      }
    }
    // ---- refill: ballot of idle lanes, leftover of the current chunk first.  Refilling
    // only once kRefillMin lanes are idle (or the wave is empty) amortises the
    // primary-generation code over several lanes.
    const unsigned long long idle = __ballot(!has);
    bool fresh = false;
    constexpr int kRefill = kShared && RTX_REFILL_SHARED > 0 ? RTX_REFILL_SHARED : kPark ? kRefillMinPark : kRefillMin;
    if (kTiles) {
      // tile schedule: the idle lanes take slots of the block's tiles in flight (descriptor
      // order; each tile's front batch, then its back batch, laid out here once the front's
      // slots are all claimed), one LDS add per batch; when those run out, the wave claims the
      // next tile
      if (idle != 0 && (__popcll(idle) >= kRefill || idle == ~0ull)) {
        const uint32_t nidle = (uint32_t)__popcll(idle);
        const uint32_t rank = (uint32_t)__popcll(idle & ((1ull << lane_id()) - 1ull));
        uint32_t given = 0;
        // descriptors with unclaimed slots (tl->avail: a hint; each buffer's word decides)
        uint32_t av = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&tl->avail);
        while (av != 0u && given < nidle) {
          const int j = (int)(__builtin_ctz(av) >> 1);
          av &= ~(3u << (2 * j));
          TileDesc& d = tl->d[j];
          for (int h = 0; h < 2 && given < nidle; h++) {  // the front batch first
            const int b = (int)(__builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&d.front) ^ (uint32_t)h);
            const unsigned long long w = *(volatile unsigned long long*)&d.b[b].word;
            const uint32_t wc = __builtin_amdgcn_readfirstlane((uint32_t)(w >> 32));
            const uint32_t wt = __builtin_amdgcn_readfirstlane((uint32_t)w);
            uint32_t c0 = wc, T = wt;
            if (wc < wt) {
              unsigned long long old = 0;
              if (lane_id() == 0) old = atomicAdd(&d.b[b].word, (unsigned long long)(nidle - given) << 32);
              c0 = __builtin_amdgcn_readfirstlane((uint32_t)(old >> 32));
              T = __builtin_amdgcn_readfirstlane((uint32_t)old);
              if (c0 < T) {
                const uint32_t got = min(nidle - given, T - c0);
                if (!has && rank >= given && rank < given + got)
                  slot = ((uint32_t)j << 24) | ((uint32_t)b << 23) | (c0 + rank - given), fresh = true;
                given += got;
                c0 += got;
              }
            }
            if (c0 >= T && lane_id() == 0) {
              // used up: clear the hint, then set it again if a record has re-laid the buffer
              atomicAnd(&tl->avail, ~(1u << (2 * j + b)));
              const unsigned long long w2 = *(volatile unsigned long long*)&d.b[b].word;
              if ((uint32_t)(w2 >> 32) < (uint32_t)w2) atomicOr(&tl->avail, 1u << (2 * j + b));
            }
          }
        }
        if (given < nidle && !__builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&tl->exhausted))
        {  // its slots go to the next refill
          int cj;
          tile_claim(tl, ta, next_slot, region, cj, COUNT ? A.counters : nullptr);
          if (cj >= 0) tile_unlock(tl, cj);
        }
      }
    } else if (kShared) {
      // block-shared chunks: the wave takes slots from its own chunk word (an LDS add), then from
      // a fresh chunk of the slot counters (installed in its word), and once the counters are
      // dry from the chunks of the block's other waves, so a block's last slots are traced by
      // its four waves instead of by the one that happened to claim them
      if (idle != 0 && !exhausted && (__popcll(idle) >= kRefill || idle == ~0ull)) {
        const uint32_t nidle = (uint32_t)__popcll(idle);
        const uint32_t rank = (uint32_t)__popcll(idle & ((1ull << lane_id()) - 1ull));
        const int wv = (int)(threadIdx.x >> 6);
        uint32_t given = 0;
        auto take = [&](int j) {
          unsigned long long old = 0;
          if (lane_id() == 0) old = atomicAdd(&cw[j], (unsigned long long)(nidle - given));
          old = __shfl(old, 0);
          const uint32_t r = (uint32_t)(old >> 61), id = (uint32_t)(old >> 32) & 0x1FFFFFFFu, cur = (uint32_t)old;
          const uint64_t rs = ((uint64_t)r * nslots) >> 3, re = ((uint64_t)(r + 1) * nslots) >> 3;
          const uint64_t cs = rs + (uint64_t)id * kChunkShared;
          const uint32_t csz = cs < re ? (uint32_t)min<uint64_t>(kChunkShared, re - cs) : 0u;
          const uint32_t got = cur < csz ? min(nidle - given, csz - cur) : 0u;
          if (!has && rank >= given && rank < given + got) slot = (uint32_t)(cs + cur + (rank - given)), fresh = true;
          given += got;
        };
        take(wv);
        if (given < nidle && !dry) {  // a fresh chunk: this wave's region first, then the next ones
          bool ok = false;
          for (int tries = 0; tries < 8 && !ok; tries++) {
            unsigned long long b = 0;
            if (lane_id() == 0) b = atomicAdd(next_slot + 16 * region, (unsigned long long)kChunkShared);
            b = __shfl(b, 0);
            const uint64_t rs = ((uint64_t)region * nslots) >> 3, re = ((uint64_t)(region + 1) * nslots) >> 3;
            if (rs + b < re) {
              ok = true;
              if (lane_id() == 0)
                atomicExch(&cw[wv], ((unsigned long long)((region << 29) | (uint32_t)(b / kChunkShared)) << 32));
            } else {
              region = (region + 1) & 7;
            }
          }
          if (ok) take(wv);
          else dry = true;
        }
        for (int m = 1; m < kBlock / 64 && dry && given < nidle; m++) take((wv + m) & (kBlock / 64 - 1));
        if (dry && given == 0) {  // nothing left anywhere: the counters are dry and so are the block's chunks
          exhausted = true;
          if (COUNT && lane_id() == 0) {
            const unsigned long long t = (unsigned long long)wall_clock64();
            atomicMax(&A.counters[14], t);
            atomicMax(&A.counters[15], ~t);
          }
        }
      }
    } else if (idle != 0 && !exhausted && (__popcll(idle) >= kRefill || idle == ~0ull)) {
      const uint64_t nidle = (uint64_t)__popcll(idle);
      const uint64_t rank = (uint64_t)__popcll(idle & ((1ull << lane_id()) - 1ull));
      uint64_t cand = ~0ull;
      if (chunk_left >= nidle) {
        if (!has) cand = chunk_base + rank;
        chunk_base += nidle, chunk_left -= nidle;
      } else {
        // the slot range is cut into 8 contiguous regions (bands of the image), one counter
        // each; a wave drains the region of its XCD group (blockIdx % 8: blocks b and b + 8
        // share an XCD and its L2), then moves on to the next ones (load balance at the end).
        // Which wave renders a slot changes, not what it computes.
        uint64_t nb = ~0ull, ne = 0;
        for (int tries = 0; tries < 8 && nb == ~0ull; tries++) {
          unsigned long long b = 0;
          if (lane_id() == 0) b = atomicAdd(next_slot + 16 * region, (unsigned long long)kChunk);
          b = __shfl(b, 0);
          const uint64_t rs = ((uint64_t)region * nslots) >> 3, re = ((uint64_t)(region + 1) * nslots) >> 3;
          if (rs + b < re) nb = rs + b, ne = std::min<uint64_t>(rs + b + kChunk, re);
          else region = (region + 1) & 7;
        }
        if (!has) {
          if (rank < chunk_left) cand = chunk_base + rank;
          else if (nb != ~0ull && nb + (rank - chunk_left) < ne) cand = nb + (rank - chunk_left);
        }
        if (nb != ~0ull) {
          const uint64_t used = std::min<uint64_t>(nidle - chunk_left, ne - nb);
          chunk_base = nb + used, chunk_left = (ne - nb) - used;
        } else {
          chunk_left = 0, exhausted = true;
          if (COUNT && lane_id() == 0) {
            const unsigned long long t = (unsigned long long)wall_clock64();
            atomicMax(&A.counters[14], t);
            atomicMax(&A.counters[15], ~t);
          }
        }
      }
      if (cand < nslots) slot = (uint32_t)cand, fresh = true;
    }
    // ---- start the primary path of a freshly assigned slot ----
    if (fresh) {
      // The primary's inputs (camera, pixel map, group) are read from the kernel argument
      // segment here (A is the kernel's first argument, at offset 0), through a pointer the
      // compiler cannot see through, so they are not held in registers across the walk: the
      // kernel runs at the SGPR limit (generic PARK build: +4.3 %, C2 +0.7 %, C5 +-0, its
      // scratch 80 -> 16 B; the bunny's Lambertian texture-free builds lost 1.0 % (their spilled
      // SGPRs 79 -> 60, scratch 52 -> 0 B), so they keep the arguments in registers;
      // profiles/r03/ab_kernarg_refill_r4g_*).
      constexpr bool kArgsAtRefill = !(LAMB && NOTEX);
      // RTX_CAM_KARG (A/B): those builds read only the camera from the argument segment
      constexpr bool kCamAtRefill = kArgsAtRefill || RTX_CAM_KARG;
      auto kseg = __builtin_amdgcn_kernarg_segment_ptr();
      if (kCamAtRefill) asm volatile("" : "+s"(kseg));
      const RenderArgs& Ar = kArgsAtRefill ? *(const RenderArgs*)kseg : A;
      const rtx_camera& Cr = kCamAtRefill ? ((const RenderArgs*)kseg)->cam : A.cam;
      // (A must stay the kernel's first parameter: the counting builds, which every parity
      // test of the counts and the bench's counting pass run, check the argument segment
      // against the arguments and fault on a mismatch)
      if (COUNT && kArgsAtRefill && (Ar.npix != A.npix || Ar.seed != A.seed || Ar.stack_slots != A.stack_slots))
        __builtin_trap();
      // nslots < 2^32 (checked on the host): 32-bit division
      uint2 e = make_uint2(0u, 0u);
      if (MAP == 1) {  // a phase's slot map, or none: uniform groups (the adaptive first pass)
        const uint2* const sm = (const uint2*)next_slot[8 * 16 + 2];
        e = sm ? sm[slot] : make_uint2(slot / (uint32_t)Ar.K, (uint32_t)Ar.s0 + slot % (uint32_t)Ar.K);
      }
      if (kTiles) {  // slot s of buffer b of descriptor j: the last pixel i with off[i] <= s
        const TileDesc& d = tl->d[slot >> 24];
        const TileBuf& B = d.b[(slot >> 23) & 1u];
        const uint32_t s = slot & 0x7FFFFFu;
        int lo = 0, hi = (int)d.npx;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (B.off[mid] <= s) lo = mid;
          else hi = mid;
        }
        e = make_uint2(d.pix[lo], B.s0[lo] + (s - B.off[lo]));
      }
      const uint32_t p = MAP ? e.x : (uint32_t)slot / (uint32_t)Ar.K;
      if (kTiles || !(Ar.conv && Ar.conv[p])) {  // (a tile slot is always traced: its count-off ends the batch)
        const int k = MAP ? 0 : (int)((uint32_t)slot - p * (uint32_t)Ar.K);
        int x, y;
        Ar.map.xy(p, x, y);
        pix = (uint32_t)(y * Ar.map.W + x), smp = MAP ? e.y : (uint32_t)(Ar.s0 + k);
        Rng g = make_rng(A.seed, pix, smp, 0u);
        get_ray<NODOF>(Cr, x, y, g, P.o, P.d);
        thr_lds[0] = 1.0, thr_lds[kBlock] = 1.0, thr_lds[2 * kBlock] = 1.0;
        P.depth = SCATTER ? Ar.max_depth : 0;
        has = true;
        prims++;
        if (COUNT) pseg = 0;
      }
    }
    if (COUNT && lane_id() == 0) c.witers++;  // (the loop's rounds are wave-uniform: lane 0 counts)
    if (!__any(has)) {
      if (COUNT && lane_id() == 0) c.widle++;
      if (kTiles) {  // nothing to trace now: leave once no tile is left or in flight, else wait
        if (__builtin_amdgcn_readfirstlane(tiles_done(tl) ? 1u : 0u)) break;
        if (!waiting && lane_id() == 0) atomicAdd(&tl->idle, 1u);  // (records meanwhile size batches larger)
        waiting = true;
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      if (exhausted) break;
      continue;
    }
    if (kTiles && waiting) {  // work again
      if (lane_id() == 0) atomicSub(&tl->idle, 1u);
      waiting = false;
    }
    if (COUNT) {
      const uint32_t live = (uint32_t)__popcll(__ballot(has));
      if (lane_id() == 0) c.wlive += live;
    }
    if (!has) continue;
    // ---- one segment: closest hit + shading ----
    V3 L;
    bool cont;
    if (SCATTER && P.depth <= 0) {  // GetPixel: depth exhausted -> black (camera.h:149-151)
      L = v3(0, 0, 0);
      cont = false;
    } else {
      double tb;
      int32_t bmat;
      int64_t best;
      if (kPark && park_ok) {
        const int active = __popcll(__ballot(1));  // lanes tracing this round
        if (!parked) {
          trav_init(trs, kInf);
          trav_globals<COUNT>(A.S, P.o, P.d, tmin, c, trs);
        }
        // parking only when some lane of this round finishes first: every round makes progress
        const bool done =
            kSpecLds ? trace4_run_spec<STACK, COUNT, TK>(A.S, P.o, P.d, tmin, stk16, leafq, kBlock, c, trs,
                                                         active > kParkAt ? kParkAt : -1)
                     : trace4_run<STACK, COUNT, TK>(A.S, P.o, P.d, tmin, stk, kBlock, c, trs,
                                                    active > kParkAt ? kParkAt : -1);
        parked = !done;
        if (parked) continue;
        best = trs.best, tb = trs.closest, bmat = trs.mat;
      } else if (kPark) {  // no BVH, or its root is a leaf
        best = trace_flat(A.S, P.o, P.d, tmin, kInf, c, COUNT, tb, bmat);
      } else {
        best = trace<STACK, FAST, COUNT, TK>(A.S, P.o, P.d, tmin, kInf, stk, c, tb, bmat);
      }
      segs++;
      if (COUNT) pseg++;
      Hit h;
      rtx_material m;
      if (best >= 0) finish_hit_at<false>(A.S, best, tb, P.o, P.d, h);
      if (kHitpLds && best >= 0) hitp_lds[0] = h.p.x, hitp_lds[kBlock] = h.p.y, hitp_lds[2 * kBlock] = h.p.z;
      if (best >= 0) m = A.S.mats[h.mat];
      if (SCATTER) P.thr = v3(thr_lds[0], thr_lds[kBlock], thr_lds[2 * kBlock]);
      // stream of this segment: depth + 1 (GetPixel: depth counts down from max_depth)
      Rng g = make_rng(A.seed, pix, smp, SCATTER ? (uint32_t)(A.max_depth - P.depth) + 1u : (uint32_t)P.depth + 1u);
      if (SCATTER) {
        // GetPixel(r, depth) iteratively (camera.h:148-174); P.thr holds the product of the
        // attenuations, P.depth the remaining depth.  Emitters never scatter, so the
        // recursion's emitted terms reduce to the terminal one.
        if (best < 0) {
          L = P.thr * sky(P.d);
          cont = false;
        } else {
          V3 att, sd;
          if (mat_scatter(A.S, m, P.d, h, att, sd, g)) {
            P.thr = P.thr * att;
            P.o = h.p, P.d = sd;
            P.depth--;
            cont = true;
          } else {
            L = P.thr * mat_emitted(A.S, m, h);
            cont = false;
          }
        }
        if (cont) thr_lds[0] = P.thr.x, thr_lds[kBlock] = P.thr.y, thr_lds[2 * kBlock] = P.thr.z;
      } else {
        // the throughput is read from LDS only after the shading core: none of its registers
        // are live across the walk or the BSDF sampling; the material's fields are read where
        // shading uses them (a reference into the table, not a copy loaded up front and held
        // across the sampling)
        ShadeOut so;
        const rtx_material& mr = *opaque(A.S.mats + (best >= 0 ? h.mat : 0));
        shade_core<LAMB, NOTEX, !kHitpLds>(A.S, A.max_depth, P, h, best >= 0, g, mr, so);
        V3 thr = v3(thr_lds[0], thr_lds[kBlock], thr_lds[2 * kBlock]);
        cont = shade_finish(so, thr, P.depth, g, L, best >= 0 ? A.S.mats + h.mat : A.S.mats);
        if (cont) thr_lds[0] = thr.x, thr_lds[kBlock] = thr.y, thr_lds[2 * kBlock] = thr.z;
        if (kHitpLds && cont) P.o = v3(hitp_lds[0], hitp_lds[kBlock], hitp_lds[2 * kBlock]);
      }
    }
    if (!cont) {
      if (kTiles) {
        // the radiance record, then the path is counted off its tile's batch; the count-off
        // that ends the batch marks the tile for its record (by a wave of this block: the
        // workgroup-scope release orders the store before the LDS count)
        const int j = (int)(slot >> 24), b = (int)((slot >> 23) & 1u);
        const uint64_t q = tile_slot(ta, j, b, slot & 0x7FFFFFu);
        double* Lq = ta->L + 3 * q;
        Lq[0] = L.x, Lq[1] = L.y, Lq[2] = L.z;
        if (COUNT) segbuf[q] = (uint16_t)min(pseg, 65535u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (atomicSub(&tl->d[j].b[b].rem, 1u) == 1u) {
          atomicOr(&tl->d[j].done, 1u << b);
          atomicOr(&tl->ready, 1u << j);
        }
      } else {
        store_radiance(A, slot, L);
        if (COUNT && segbuf) segbuf[slot] = (uint16_t)min(pseg, 65535u);
      }
      has = false;
    }
  }
  flush_counters(A, c, segs, prims, COUNT);
  if (COUNT && lane_id() == 0) {
    const unsigned long long t = (unsigned long long)wall_clock64();
    atomicMax(&A.counters[16], t);
    atomicMax(&A.counters[17], ~t);
  }
}

// The PARK instantiations are compiled in their own translation unit (rtx_park.hip), with
// their own macro defaults (the leaf-step walk, the branchless triangle test) and scheduler
// options (Makefile PARKFLAGS; the LLVM default since the leaf-step walk, `ab_sch_c3.txt`).
// (ST: stack size, CO: counting build, SC: scatter API, MP: 0 uniform groups, 1 adaptive slot
// map, 2 adaptive tiles, PK: 1 the leaf-step walk, 2 the speculative walk; the host never
// launches the PARK kernel for the scatter API, nor maps a scatter render's slots, but its
// dispatch names those builds)
#define RTX_PARK_INSTANCES(X)                                                                                    \
  X(32, false, false, 0, 1) X(32, true, false, 0, 1) X(64, false, false, 0, 1)                                  \
  X(64, true, false, 0, 1) X(32, false, true, 0, 1) X(32, true, true, 0, 1)                                     \
  X(64, false, true, 0, 1) X(64, true, true, 0, 1) X(32, false, false, 1, 1)                                    \
  X(32, true, false, 1, 1) X(64, false, false, 1, 1) X(64, true, false, 1, 1)                                   \
  X(32, false, false, 2, 1) X(32, true, false, 2, 1) X(64, false, false, 2, 1) X(64, true, false, 2, 1)         \
  X(32, false, false, 0, 2) X(32, true, false, 0, 2) X(64, false, false, 0, 2)                                  \
  X(64, true, false, 0, 2) X(32, false, false, 1, 2) X(32, true, false, 1, 2)                                   \
  X(64, false, false, 1, 2) X(64, true, false, 1, 2)                                                            \
  X(32, false, false, 2, 2) X(32, true, false, 2, 2) X(64, false, false, 2, 2) X(64, true, false, 2, 2)
#define RTX_PARK_TRI_INSTANCES(Y)                                                                           \
  Y(32, 0, 1) Y(64, 0, 1) Y(32, 1, 1) Y(64, 1, 1) Y(32, 2, 1) Y(64, 2, 1) Y(32, 0, 2) Y(64, 0, 2) Y(32, 1, 2) \
      Y(64, 1, 2) Y(32, 2, 2) Y(64, 2, 2)
#ifndef RTX_PERSISTENT_ONLY
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
#endif

// ---------------------------------------------------------------------------------------
// RecordSample in sample order (pixel_state.h:22-39) + IsConverged (pixel_state.h:54-72)
// (PixelSoA: see the tile schedule above)
// ---------------------------------------------------------------------------------------
#ifndef RTX_PERSISTENT_ONLY  // rtx_park.hip: the persistent kernel's PARK instantiations only
__global__ __launch_bounds__(kBlock) void k_accumulate(PixelSoA px, const double* __restrict__ L, int64_t npix,
                                                       int K, int adaptive, int min_spp, double rel) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= npix) return;
  if (px.conv[p]) return;
  double sum[3], mean[3], m2[3];
  for (int c = 0; c < 3; c++) sum[c] = px.sum[c * npix + p], mean[c] = px.mean[c * npix + p], m2[c] = px.m2[c * npix + p];
  int n = px.samples[p];
  bool conv = false;
  const int need = adaptive ? min_spp : 0x7FFFFFFF;
  for (int k = 0; k < K && !conv; k++) {
    const double* x = L + 3 * (p * K + k);
    n++;
    for (int c = 0; c < 3; c++) {
      double mu = mean[c];
      double delta = x[c] - mu;
      mu += delta / n;
      double delta2 = x[c] - mu;
      mean[c] = mu;
      m2[c] += delta2 * delta;
    }
    for (int c = 0; c < 3; c++) sum[c] += x[c];
    if (n >= need) {
      bool ok = true;
      for (int c = 0; c < 3 && ok; c++) {
        double var = n > 1 ? m2[c] / (n - 1) : 0.0;
        double mu = fmax(fabs(mean[c]), 1e-3);
        double err = sqrt(var) / sqrt((double)n);
        if (err / mu > rel) ok = false;
      }
      conv = ok;
    }
  }
  for (int c = 0; c < 3; c++) px.sum[c * npix + p] = sum[c], px.mean[c * npix + p] = mean[c], px.m2[c * npix + p] = m2[c];
  px.samples[p] = n;
  px.conv[p] = conv;
}

// ---------------------------------------------------------------------------------------
// Adaptive sampling in phases (the reference's default mode: WavefrontRenderer::Render,
// wavefront.cc:42-43 kRelThresh / kMinSamples, converged pixels skipped at :68-69,
// RecordSample + IsConverged at :125-127 and pixel_state.h:22-72).
//
// Phase 1 traces the min_spp samples every pixel needs (uniform slots).  After each phase,
// k_adapt_record replays RecordSample / IsConverged over the phase's samples of every pixel in
// sample order (k_accumulate's arithmetic) and, for a pixel neither converged nor out of
// budget, sizes its next batch from its running statistics: IsConverged holds at n samples once
// sqrt(var / n) / max(|mean|, 1e-3) <= rel in every channel, i.e. n >= var / (rel mu)^2, so the
// batch is that many more samples (with a margin that grows with the phase, at least 4, a
// multiple of 4, within the budget and the workspace).  k_adapt_expand then lays out the next
// phase's slots, pixel-major, from a prefix sum of the batch sizes, each slot holding its
// (pixel, sample).  Only pixels still sampling get slots.  A sample traced past its pixel's
// convergence point is discarded here, so the result is the reference's whatever the batch
// sizes are: the prediction only decides how much work is spent and how many phases it takes.
// ---------------------------------------------------------------------------------------
struct AdaptPlan {
  const uint32_t* kcur;  // samples of sub-pixel q in the phase just traced (nullptr: kuni each)
  const uint32_t* off;   // their first slot (nullptr: the uniform first phase, p * kuni)
  uint32_t* knext;       // out: samples of q in the next phase (0: q is finished)
  int32_t kuni;
  int32_t sub_n, sub_j;  // pixel p = q * sub_n + sub_j
  int32_t min_spp, budget, phase, kcap;
  int32_t kmin;  // smallest next batch: keeps a phase with few pixels left large enough to fill the GPU
  double rel;
  double margin_step;  // the batch margin grows by this much per phase (1 + step * (phase - 1))
  const uint16_t* segs;           // counting renders: segments of each slot's path (else nullptr)
  unsigned long long* rec_segs;   // ... summed here over the samples the pixels record
  unsigned long long* active;  // the next phase's pixel count (k_adapt_expand adds; zeroed here)
  unsigned long long* next_active;  // ... counted here too (zeroed before the launch), for k_adapt_floor
};
__device__ __forceinline__ uint32_t adapt_next_batch(const double (&mean)[3], const double (&m2)[3], int n,
                                                     const AdaptPlan& ap) {
  double need = 0.0;  // samples at which IsConverged would hold with the current estimates
  for (int c = 0; c < 3; c++) {
    const double var = n > 1 ? m2[c] / (n - 1) : 0.0;
    const double mu = fmax(fabs(mean[c]), 1e-3);
    need = fmax(need, var / (ap.rel * ap.rel * mu * mu));
  }
  const int left = ap.budget - n;
  const double margin = 1.0 + ap.margin_step * (double)(ap.phase - 1);
  const double want = (need - (double)n) * margin;
  int k = (want < (double)left) ? (int)ceil(want) : left;  // NaN / inf: the whole budget
  k = max(k, min(max(4 << min(ap.phase - 1, 4), ap.kmin), left));  // at least 4, 8, ... 64 more, and kmin
  k = (k + 3) & ~3;
  return (uint32_t)min(k, min(left, ap.kcap));
}
// One lane per sub-pixel: the replay of a pixel's samples is sequential (each step divides by
// the running count), so the parallelism is across pixels, and each lane streams its own run
// of the phase's slots with the loads of the next kRecAhead samples in flight while it
// replays the current one (a lane's run is contiguous: its loads walk the same cache lines).
#ifndef RTX_REC_AHEAD
#define RTX_REC_AHEAD 8
#endif
constexpr int kRecAhead = RTX_REC_AHEAD;
__global__ __launch_bounds__(kBlock) void k_adapt_record(PixelSoA px, const double* __restrict__ L, int64_t nq,
                                                         int64_t npix, AdaptPlan ap) {
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q == 0) *ap.active = 0;  // k_adapt_expand, later on the stream, counts the next phase's pixels
  if (q >= nq) return;
  const int64_t p = q * ap.sub_n + ap.sub_j;
  const int K = ap.kcur ? (int)ap.kcur[q] : ap.kuni;
  uint32_t kn = 0;
  if (K > 0 && !px.conv[p]) {
    const double* __restrict__ Lp = L + 3 * (ap.off ? (int64_t)ap.off[q] : p * (int64_t)ap.kuni);
    PixRec r;
    load_pixel(r, px, npix, p);
    const int n0 = r.n;
    replay_pixel<kRecAhead>(r, Lp, K, ap.min_spp, ap.rel);
    if (ap.segs) {  // counting render: the segments of the samples recorded (the rest are discarded)
      const uint16_t* sg = ap.segs + (ap.off ? (int64_t)ap.off[q] : p * (int64_t)ap.kuni);
      unsigned long long t = 0;
      for (int k = 0; k < r.n - n0; k++) t += sg[k];
      atomicAdd(ap.rec_segs, t);
    }
    store_pixel(r, px, npix, p);
    if (!r.conv && r.n < ap.budget) kn = adapt_next_batch(r.mean, r.m2, r.n, ap);
  }
  ap.knext[q] = kn;
  const unsigned long long na = __popcll(__ballot(kn != 0));
  if (na && lane_id() == 0) atomicAdd(ap.next_active, na);
}
// Once the next phase's pixel count is known: every batch at least target / that count (within
// the pixel's budget and the workspace), so a phase with few pixels left is large enough to
// fill the GPU, and the pixels finish in it rather than in further phases that would be mostly
// launch drain (the last paths of a launch run with their waves nearly empty).
__global__ __launch_bounds__(kBlock) void k_adapt_floor(uint32_t* __restrict__ knext, int64_t nq, int32_t sub_n,
                                                        int32_t sub_j, const int32_t* __restrict__ samples,
                                                        int32_t budget, int32_t kcap, int64_t target,
                                                        const unsigned long long* __restrict__ next_active) {
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q >= nq) return;
  const uint32_t k = knext[q];
  if (k == 0) return;
  const unsigned long long na = *next_active;
  const int64_t kmin = (target + (int64_t)na - 1) / (int64_t)max(na, 1ull);
  const int left = budget - samples[q * sub_n + sub_j];
  int kn = (int)max<int64_t>((int64_t)k, min<int64_t>(kmin, (int64_t)left));
  kn = (kn + 3) & ~3;
  knext[q] = (uint32_t)min(kn, min(left, kcap));
}
// The next phase's slot map: sub-pixel q's batch occupies slots [off[q], off[q] + knext[q]),
// slot off[q] + k being sample samples[p] + k of pixel p.  One block per kExpandPix sub-pixels;
// its slots are a contiguous range written by all its threads (coalesced), each finding its
// sub-pixel by a search of the block's offsets in LDS.  The last sub-pixel's thread writes the
// phase's slot count.  (Few pixels per block: the pixels still sampling cluster, and a block
// over 256 of them had up to 256 x kcap slots to write while most blocks had none.)
constexpr int kExpandPix = 32;
__global__ __launch_bounds__(kBlock) void k_adapt_expand(const uint32_t* __restrict__ knext,
                                                         const uint32_t* __restrict__ off, int64_t nq, int32_t sub_n,
                                                         int32_t sub_j, const int32_t* __restrict__ samples,
                                                         uint2* __restrict__ smap,
                                                         unsigned long long* __restrict__ total) {
  __shared__ uint32_t s_off[kExpandPix], s_p[kExpandPix], s_s0[kExpandPix];
  __shared__ uint32_t s_end;
  const int t = threadIdx.x;
  const int64_t q0 = (int64_t)blockIdx.x * kExpandPix, q = q0 + t;
  const int nb = (int)min<int64_t>(kExpandPix, nq - q0);
  bool act = false;
  if (t < nb) {
    const uint32_t k = knext[q], o = off[q];
    const int64_t p = q * sub_n + sub_j;
    act = k != 0;
    s_off[t] = o, s_p[t] = (uint32_t)p, s_s0[t] = k ? (uint32_t)samples[p] : 0u;
    if (t == nb - 1) {
      s_end = o + k;
      if (q == nq - 1) total[0] = (unsigned long long)o + k, total[2] = (unsigned long long)smap;
    }
  }
  const unsigned long long nact = __popcll(__ballot(act));  // total[1]: the phase's pixels
  if (nact && lane_id() == 0) atomicAdd(total + 1, nact);
  __syncthreads();
  const uint32_t b = s_off[0], e = s_end;
  for (uint32_t i = b + t; i < e; i += kBlock) {
    int lo = 0, hi = nb;  // the last q with s_off[q] <= i (a zero batch shares its successor's offset)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_off[mid] <= i) lo = mid;
      else hi = mid;
    }
    smap[i] = make_uint2(s_p[lo], s_s0[lo] + (i - s_off[lo]));
  }
}

// ---- the tile schedule's claim order (render_adaptive): the pixels still sampling after the
// first pass, compacted in image order (flag, exclusive scan, compact), cut into tiles of
// kTileTP, each keyed by (region, predicted work descending) for a radix sort, so each region's
// tiles are claimed largest batch first.  The region of a tile is the 1/8 band of the subset's
// pixels its first pixel lies in: the same bands the first pass's slot regions cover, so a
// block keeps to its XCD group's band of the image as long as the band has tiles.
__global__ __launch_bounds__(kBlock) void k_tile_flags(const uint32_t* __restrict__ knext, int64_t npix,
                                                       uint32_t* __restrict__ flag) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p < npix) flag[p] = knext[p] != 0u ? 1u : 0u;
}
__global__ __launch_bounds__(kBlock) void k_tile_compact(const uint32_t* __restrict__ flag,
                                                         const uint32_t* __restrict__ idx, int64_t npix,
                                                         uint32_t* __restrict__ act, uint32_t* __restrict__ nact) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= npix) return;
  if (flag[p]) act[idx[p]] = (uint32_t)p;
  if (p == npix - 1) *nact = idx[p] + flag[p];
}
__global__ __launch_bounds__(kBlock) void k_tile_keys(const uint32_t* __restrict__ act,
                                                      const uint32_t* __restrict__ nact,
                                                      const uint32_t* __restrict__ knext, int64_t npix,
                                                      int64_t max_tiles, int32_t tp, uint32_t* __restrict__ keys,
                                                      uint32_t* __restrict__ vals, uint32_t* __restrict__ rcount) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= max_tiles) return;
  const int64_t first = t * tp, na = *nact;
  vals[t] = (uint32_t)t;
  if (first >= na) {
    keys[t] = 0xFFFFFFFFu;  // no such tile: sorted after every region
    return;
  }
  uint32_t work = 0;
  for (int64_t i = first; i < min<int64_t>(first + tp, na); i++) work += knext[act[i]];
  const uint32_t region = (uint32_t)min<int64_t>(7, ((int64_t)act[first] * 8) / max<int64_t>(1, npix));
  keys[t] = (region << 24) | (0xFFFFFFu - min(work, 0xFFFFFFu));
  atomicAdd(&rcount[region], 1u);
}
// The launch's TileArgs into device memory, its address into the slot counter block; with the
// first pass in the launch (a.act == nullptr), also the tile counts of the regions and the
// pixel count (tiles of every pixel in image order: rcount_fp, nact_fp).
struct RegionCounts {
  uint32_t c[8];
};
__global__ void k_tile_setup(TileArgs a, TileArgs* __restrict__ dst, unsigned long long* __restrict__ ctr,
                             RegionCounts rc, uint32_t npix_fp, uint32_t* __restrict__ tcount) {
  if (!a.act) {
    for (int r = 0; r < 8; r++) tcount[r] = rc.c[r];
    tcount[8] = npix_fp;
  }
  *dst = a;
  ctr[8 * 16 + 6] = (unsigned long long)dst;
}
#endif

// Fixed-spp accumulation: the sum RecordSample (and DefaultSampler) forms, in sample order.
// One wave per 64 consecutive pixels, whose radiance runs are one contiguous region of Lbuf
// (pixel-major slots).  Chunks of kAccChunk samples are staged through LDS: the wave reads
// each pixel's contiguous run of 3 * kAccChunk doubles with 16-byte loads (8-byte loads when
// the runs are not 16-byte aligned, i.e. K odd, or for a short last chunk), all issued before
// the first LDS store, then each lane adds its own pixel's samples in order.
// 8-sample chunks, 16 pixels per 64-lane workgroup (LDS 3.1 KB; ab_acc*), the next chunk's
// loads in flight while the current one is summed (ab_acc_pipe).
constexpr int kAccWave = 64, kAccPix = 16, kAccChunk = 8,
              kAccPitch = 3 * kAccChunk + 1;  // odd pitch: spread LDS banks
static_assert(kAccPix <= kAccWave, "one summing lane per pixel");
#ifndef RTX_PERSISTENT_ONLY  // rtx_park.hip: the persistent kernel's PARK instantiations only
// Pixels [p_begin, p_end) of the npix (one band of the frame, so the caller can copy a
// finished band to the host while the next is summed).  first: the group starts the pixels'
// sums (nothing to read).  resolve >= 0 (the last group): the pixel's output is written here,
// as k_resolve would (0: sum / (float)samples, 1: the megakernel's DefaultSampler sum / spp),
// instead of the running sum and count.
struct AccOut {
  double* rgb;
  int32_t* spp_out;
  int resolve;  // -1: keep the running sums in px; 0 / 1: write the resolved pixel
  int spp;
};
__global__ __launch_bounds__(kAccWave) void k_accumulate_sum(PixelSoA px, const double* __restrict__ L, int64_t npix,
                                                             int K, int64_t p_begin, int64_t p_end, int first,
                                                             AccOut out) {
  __shared__ double st[kAccPix * kAccPitch];
  const int t = threadIdx.x;
  const int64_t p0 = p_begin + (int64_t)blockIdx.x * kAccPix;
  const int npx = (int)std::min<int64_t>(kAccPix, p_end - p0);
  const int64_t p = p0 + t;
  const double* __restrict__ base = L + p0 * 3 * (int64_t)K;
  double sum[3] = {0, 0, 0};
  if (t < npx && !first)
    for (int c = 0; c < 3; c++) sum[c] = px.sum[c * npix + p];
  // Full chunks with 16-byte-aligned runs (K even) are software-pipelined: chunk i + 1 is
  // loaded into registers before chunk i is summed out of LDS.  Same adds, same order.
  constexpr int PP = 3 * kAccChunk / 2;  // 16-byte pieces per pixel run
  constexpr int NL = (kAccPix * PP + kAccWave - 1) / kAccWave;  // 16-byte loads per lane per chunk
  const int kfull = (K & 1) == 0 ? (K / kAccChunk) * kAccChunk : 0;
  if (kfull > 0) {
    double2 v[NL];
    auto load = [&](int k0) {
#pragma unroll
      for (int i = 0; i < NL; i++) {
        const int e = t + kAccWave * i, q = e / PP, j = e - q * PP;
        if (q < npx) v[i] = *(const double2*)(base + (int64_t)q * 3 * K + 3 * k0 + 2 * j);
      }
    };
    load(0);
    for (int k0 = 0; k0 < kfull; k0 += kAccChunk) {
#pragma unroll
      for (int i = 0; i < NL; i++) {
        const int e = t + kAccWave * i, q = e / PP, j = e - q * PP;
        if (q < npx) st[q * kAccPitch + 2 * j] = v[i].x, st[q * kAccPitch + 2 * j + 1] = v[i].y;
      }
      __syncthreads();
      if (k0 + kAccChunk < kfull) load(k0 + kAccChunk);
      if (t < npx)
#pragma unroll
        for (int k = 0; k < kAccChunk; k++)
          for (int c = 0; c < 3; c++) sum[c] += st[t * kAccPitch + 3 * k + c];
      __syncthreads();
    }
  }
  for (int k0 = kfull; k0 < K; k0 += kAccChunk) {
    const int kc = std::min(kAccChunk, K - k0);
    if (kc == kAccChunk && (K & 1) == 0) {
      constexpr int PP = 3 * kAccChunk / 2;  // 16-byte pieces per pixel run
      constexpr int NL = (kAccPix * PP + kAccWave - 1) / kAccWave;
      double2 v[NL];
#pragma unroll
      for (int i = 0; i < NL; i++) {
        const int e = t + kAccWave * i, q = e / PP, j = e - q * PP;
        if (q < npx) v[i] = *(const double2*)(base + (int64_t)q * 3 * K + 3 * k0 + 2 * j);
      }
#pragma unroll
      for (int i = 0; i < NL; i++) {
        const int e = t + kAccWave * i, q = e / PP, j = e - q * PP;
        if (q < npx) st[q * kAccPitch + 2 * j] = v[i].x, st[q * kAccPitch + 2 * j + 1] = v[i].y;
      }
    } else {
      const int run = 3 * kc, total = npx * run;
      for (int e = t; e < total; e += kAccWave) {
        const int q = e / run, j = e - q * run;
        st[q * kAccPitch + j] = base[(int64_t)q * 3 * K + 3 * k0 + j];
      }
    }
    __syncthreads();
    if (t < npx)
      for (int k = 0; k < kc; k++)
        for (int c = 0; c < 3; c++) sum[c] += st[t * kAccPitch + 3 * k + c];
    __syncthreads();
  }
  if (t < npx) {
    const int n = (first ? 0 : px.samples[p]) + K;
    if (out.resolve < 0) {
      for (int c = 0; c < 3; c++) px.sum[c * npix + p] = sum[c];
      px.samples[p] = n;
    } else {  // k_resolve's arithmetic (n > 0 here)
      const double sc = out.resolve == 1 ? 1.0 / (double)out.spp : 1.0 / (double)(float)n;
      for (int c = 0; c < 3; c++) out.rgb[3 * p + c] = sc * sum[c];
      if (out.spp_out) out.spp_out[p] = out.resolve == 1 ? out.spp : n;
    }
  }
}
#endif

// AdaptiveSampler::SamplePixel (sampler.h:44-82) replayed in sample order for the MegaKernel
// renderer.  Its quirks are kept: `pixel` is the running SUM of the samples and the mean /
// variance are taken over those running sums; luminance uses float weights (color.h:35-37);
// the loop runs while samples <= max_samples, i.e. up to max_samples + 1 samples.  State:
// px.sum = pixel, px.mean = sum, px.m2 = sum_sq, px.samples, px.conv = finished.
__device__ __forceinline__ double luminance(double x, double y, double z) {
  return (double)0.2126f * x + (double)0.7152f * y + (double)0.0722f * z;
}
#ifndef RTX_PERSISTENT_ONLY  // rtx_park.hip: the persistent kernel's PARK instantiations only
__global__ __launch_bounds__(kBlock) void k_accumulate_mk_adaptive(PixelSoA px, const double* __restrict__ L,
                                                                   int64_t npix, int K, int min_samples,
                                                                   int max_samples, double threshold) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= npix) return;
  if (px.conv[p]) return;
  double pixel[3], sum[3], sq[3];
  for (int c = 0; c < 3; c++)
    pixel[c] = px.sum[c * npix + p], sum[c] = px.mean[c * npix + p], sq[c] = px.m2[c * npix + p];
  int n = px.samples[p];
  bool done = false;
  for (int k = 0; k < K && !done; k++) {
    if (n > max_samples) {  // while (samples <= max_samples_) fails
      done = true;
      break;
    }
    n++;
    const double* x = L + 3 * (p * K + k);
    for (int c = 0; c < 3; c++) pixel[c] += x[c];
    for (int c = 0; c < 3; c++) sum[c] += pixel[c];
    for (int c = 0; c < 3; c++) sq[c] += pixel[c] * pixel[c];
    if (n >= min_samples) {
      const double inv = 1.0 / n;  // Vec3 / int is (1/t) * v
      double mean[3], var[3];
      for (int c = 0; c < 3; c++) mean[c] = inv * sum[c];
      const double mean_lum = luminance(mean[0], mean[1], mean[2]);
      for (int c = 0; c < 3; c++) var[c] = inv * sq[c] - mean[c] * mean[c];
      const double error = sqrt(luminance(var[0], var[1], var[2]) / n);
      if ((error / (mean_lum + (double)1e-3f)) < threshold) done = true;
    }
  }
  if (n > max_samples) done = true;
  for (int c = 0; c < 3; c++)
    px.sum[c * npix + p] = pixel[c], px.mean[c * npix + p] = sum[c], px.m2[c * npix + p] = sq[c];
  px.samples[p] = n;
  px.conv[p] = done ? 1 : 0;
}
#endif

// wavefront.cc:229-235: sum / (float)samples  (Vec3 operator/ is (1/t)*v); megakernel
// (mega_kernel.h + sampler.h:32,79): pixel /= num_samples (DefaultSampler) or /= samples
// (AdaptiveSampler).
#ifndef RTX_PERSISTENT_ONLY  // rtx_park.hip: the persistent kernel's PARK instantiations only
// A frame's start in one launch instead of one fill per buffer (each fill is a launch with its
// own gap): the pixel statistics (zero_px) and the statistics counters.
__global__ __launch_bounds__(kBlock) void k_frame_init(PixelSoA px, int64_t npix, int zero_px,
                                                       unsigned long long* __restrict__ counters, int nwords) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < nwords) counters[i] = 0ull;
  if (!zero_px || i >= npix) return;
  for (int c = 0; c < 3; c++) px.sum[c * npix + i] = 0.0, px.mean[c * npix + i] = 0.0, px.m2[c * npix + i] = 0.0;
  px.samples[i] = 0;
  px.conv[i] = 0;
}
// An adaptive launch's slot counter block: the 8 region counters and the next phase's pixel
// count (word 8 * 16 + 3, k_adapt_record's) zeroed, the slot count and the slot map's address
// set (set: 0 keeps them, as k_adapt_expand wrote them).
__global__ void k_slot_block_init(unsigned long long* __restrict__ ctr, int set, unsigned long long nslots,
                                  unsigned long long smap) {
  const int i = (int)threadIdx.x;
  if (i < 8 * 16) ctr[i] = 0ull;
  if (i == 0) {
    ctr[8 * 16 + 3] = 0ull;
    if (set) ctr[8 * 16] = nslots, ctr[8 * 16 + 2] = smap;
  }
}
__global__ __launch_bounds__(kBlock) void k_resolve(PixelSoA px, int64_t npix, int megakernel, int spp,
                                                    double* __restrict__ rgb, int32_t* __restrict__ spp_out) {
  // megakernel: 1 = DefaultSampler (divide by spp), 2 = AdaptiveSampler (by the pixel's count)
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= npix) return;
  const int n = px.samples[p];
  double s = 0.0;
  if (megakernel == 1) s = 1.0 / (double)spp;
  else if (megakernel == 2) s = 1.0 / (double)n;
  else if (n > 0) s = 1.0 / (double)(float)n;
  for (int c = 0; c < 3; c++) rgb[3 * p + c] = (megakernel || n > 0) ? s * px.sum[c * npix + p] : 0.0;
  if (spp_out) spp_out[p] = megakernel == 1 ? spp : n;
}
#endif

}  // namespace rtxd
