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
constexpr int kChunk = 256;  // persistent: slots taken per atomic on a region's slot counter (ab_chunk_*)

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
  uint32_t stack, thr, hitp, leafq, end;  // byte offsets of the regions in a block's LDS, its size
};
// PARK: 0 the plain schedule, 1 the PARK schedule with the leaf-step walk (trace4_run_step),
// 2 the PARK schedule with the speculative walk (trace4_run_spec; trees of at most
// kSpecMaxNodes nodes, its stack entries being 16-bit)
constexpr bool spec_walk(int park, bool fast, bool scatter) { return park == 2 && fast && !scatter; }
constexpr int64_t kSpecMaxNodes = 65536;
constexpr PersistLds persist_lds(int stack_slots, bool spec) {
  const uint32_t stack_bytes = (uint32_t)stack_slots * kBlock * (spec ? 2u : 4u);
  const uint32_t thr = stack_bytes, hitp = thr + 3u * kBlock * 8u, leafq = hitp + 3u * kBlock * 8u;
  return PersistLds{0u, thr, hitp, leafq, leafq + (spec ? (uint32_t)kLeafQueue * kBlock * 4u : 0u)};
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
// Persistent lanes: each lane owns one path at a time and refills from a global slot
// counter in wave-sized chunks (one atomic per kChunk slots), so lanes whose path ended
// (miss, emitter, absorption, Russian roulette) are immediately given a new primary —
// the per-wave __ballot of idle lanes is the active-ray compaction.
// ---------------------------------------------------------------------------------------
// TK >= 0: every primitive in the fast tree has kind TK (the ground sphere is a global
// primitive, so the bunny's tree holds triangles, the final and mixed scenes' spheres), so
// the walk's leaf tests are compiled for that kind alone.
// Which slots the kernel draws: uniform groups (MAP = false), slot p * K + k is sample s0 + k
// of pixel p; adaptive phases (render_adaptive, MAP = true), slot i is sample smap[i].y of
// pixel smap[i].x for i below the phase's slot count, where the slot counters' block holds,
// after the 8 region counters, the slot count (next_slot[128]) and the slot map's address
// (next_slot[130]), both written by k_adapt_expand.  MAP is a template parameter, not a kernel
// argument: the fixed-spp kernels run at the SGPR limit, and any extra uniform state there
// reshuffles their register allocation (a runtime switch cost the bunny's build 3.7 %, r3d).
template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK, int TK = -1, bool LAMB = false,
          bool NOTEX = false, bool NODOF = false, bool MAP = false>
__global__ __launch_bounds__(kBlock, kTraceWaves) void k_persistent(RenderArgs A, unsigned long long* next_slot) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  // the LDS layout (persist_lds: the launch sizes it the same way; the host launches PARK
  // kernels only for fast, non-scatter renders)
  constexpr bool kSpecLds = spec_walk(PARK, FAST, SCATTER);
  const PersistLds lay = persist_lds(A.stack_slots, kSpecLds);
  char* const ldsb = (char*)lds;
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
  const uint64_t nslots = MAP ? (uint64_t)next_slot[8 * 16] : (uint64_t)A.npix * (uint64_t)A.K;
  // GetPixel uses Interval(0.001, inf) (camera.h:158); IntersectBatch uses 0.001f (cpu_ray_integrator.h:21)
  const double tmin = SCATTER ? 0.001 : (double)0.001f;
  Counters c{};
  uint32_t segs = 0, prims = 0;
  // counting builds: the lane's path segments, stored per slot when the launch's slot counter
  // block names a buffer for them (adaptive renders: the segments of the recorded samples)
  uint32_t pseg = 0;
  uint16_t* const segbuf = COUNT ? (uint16_t*)next_slot[8 * 16 + 4] : nullptr;
  (void)pseg, (void)segbuf;
  uint64_t chunk_base = 0, chunk_left = 0;  // wave-uniform
  bool exhausted = false;                   // wave-uniform
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
  TravState trs;
  while (true) {
    // ---- refill: ballot of idle lanes, leftover of the current chunk first.  Refilling
    // only once kRefillMin lanes are idle (or the wave is empty) amortises the
    // primary-generation code over several lanes.
    const unsigned long long idle = __ballot(!has);
    bool fresh = false;
    constexpr int kRefill = kPark ? kRefillMinPark : kRefillMin;
    if (idle != 0 && !exhausted && (__popcll(idle) >= kRefill || idle == ~0ull)) {
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
      auto kseg = __builtin_amdgcn_kernarg_segment_ptr();
      if (kArgsAtRefill) asm volatile("" : "+s"(kseg));
      const RenderArgs& Ar = kArgsAtRefill ? *(const RenderArgs*)kseg : A;
      // nslots < 2^32 (checked on the host): 32-bit division
      uint2 e = make_uint2(0u, 0u);
      if (MAP) e = ((const uint2*)next_slot[8 * 16 + 2])[slot];
      const uint32_t p = MAP ? e.x : (uint32_t)slot / (uint32_t)Ar.K;
      if (!(Ar.conv && Ar.conv[p])) {
        const int k = MAP ? 0 : (int)((uint32_t)slot - p * (uint32_t)Ar.K);
        int x, y;
        Ar.map.xy(p, x, y);
        pix = (uint32_t)(y * Ar.map.W + x), smp = MAP ? e.y : (uint32_t)(Ar.s0 + k);
        Rng g = make_rng(A.seed, pix, smp, 0u);
        get_ray<NODOF>(Ar.cam, x, y, g, P.o, P.d);
        thr_lds[0] = 1.0, thr_lds[kBlock] = 1.0, thr_lds[2 * kBlock] = 1.0;
        P.depth = SCATTER ? Ar.max_depth : 0;
        has = true;
        prims++;
        if (COUNT) pseg = 0;
      }
    }
    if (!__any(has)) {
      if (exhausted) break;
      continue;
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
      store_radiance(A, slot, L);
      if (COUNT && segbuf) segbuf[slot] = (uint16_t)min(pseg, 65535u);
      has = false;
    }
  }
  flush_counters(A, c, segs, prims, COUNT);
}

// The PARK instantiations are compiled in their own translation unit (rtx_park.hip), with
// their own macro defaults (the leaf-step walk, the branchless triangle test) and scheduler
// options (Makefile PARKFLAGS; the LLVM default since the leaf-step walk, `ab_sch_c3.txt`).
// (ST: stack size, CO: counting build, SC: scatter API, MP: adaptive slot map, PK: 1 the
// leaf-step walk, 2 the speculative walk; the host never launches the PARK kernel for the
// scatter API, nor maps a scatter render's slots, but its dispatch names those builds)
#define RTX_PARK_INSTANCES(X)                                                                                    \
  X(32, false, false, false, 1) X(32, true, false, false, 1) X(64, false, false, false, 1)                      \
  X(64, true, false, false, 1) X(32, false, true, false, 1) X(32, true, true, false, 1)                         \
  X(64, false, true, false, 1) X(64, true, true, false, 1) X(32, false, false, true, 1)                         \
  X(32, true, false, true, 1) X(64, false, false, true, 1) X(64, true, false, true, 1)                          \
  X(32, false, false, false, 2) X(32, true, false, false, 2) X(64, false, false, false, 2)                      \
  X(64, true, false, false, 2) X(32, false, false, true, 2) X(32, true, false, true, 2)                         \
  X(64, false, false, true, 2) X(64, true, false, true, 2)
#define RTX_PARK_TRI_INSTANCES(Y) \
  Y(32, false, 1) Y(64, false, 1) Y(32, true, 1) Y(64, true, 1) Y(32, false, 2) Y(64, false, 2) Y(32, true, 2) Y(64, true, 2)
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
// ---------------------------------------------------------------------------------------
struct PixelSoA {
  double *sum, *mean, *m2;  // 3 x npix each (channel-major)
  int32_t* samples;
  uint8_t* conv;
};

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
constexpr int kRecAhead = 8;
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
    double sum[3], mean[3], m2[3];
    for (int c = 0; c < 3; c++) sum[c] = px.sum[c * npix + p], mean[c] = px.mean[c * npix + p], m2[c] = px.m2[c * npix + p];
    int n = px.samples[p];
    bool conv = false;
    // RecordSample (pixel_state.h:22-39), then IsConverged (pixel_state.h:54-72)
    auto record = [&](const double (&x)[3]) {
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
      if (n >= ap.min_spp) {
        // err / mu > rel  <=>  m2 > rel^2 (n - 1) n mu^2 up to the few ulps the exact form rounds
        // by: decided by products where the two sides differ by more than 1e-10 relative (the
        // usual case), the exact form (two divisions, two square roots) only in between; NaN
        // fails both comparisons and takes the exact form too.
        bool ok = true;
        for (int c = 0; c < 3 && ok; c++) {
          double mu = fmax(fabs(mean[c]), 1e-3);
          const double thr = ap.rel * ap.rel * ((double)(n - 1) * (double)n * (mu * mu));
          if (m2[c] > thr * (1.0 + 1e-10)) {
            ok = false;
          } else if (!(m2[c] < thr * (1.0 - 1e-10))) {
            double var = n > 1 ? m2[c] / (n - 1) : 0.0;
            double err = sqrt(var) / sqrt((double)n);
            if (err / mu > ap.rel) ok = false;
          }
        }
        conv = ok;
      }
    };
    double b[kRecAhead][3];
    auto load = [&](int slot, int k) {
      if (k < K)
        for (int c = 0; c < 3; c++) b[slot][c] = Lp[3 * k + c];
    };
#pragma unroll
    for (int i = 0; i < kRecAhead; i++) load(i, i);
    for (int k = 0; k < K && !conv; k += kRecAhead) {
#pragma unroll
      for (int i = 0; i < kRecAhead; i++) {
        if (k + i >= K || conv) break;
        record(b[i]);
        load(i, k + i + kRecAhead);
      }
    }
    if (ap.segs) {  // counting render: the segments of the samples recorded (the rest are discarded)
      const uint16_t* sg = ap.segs + (ap.off ? (int64_t)ap.off[q] : p * (int64_t)ap.kuni);
      unsigned long long t = 0;
      for (int k = 0; k < n - px.samples[p]; k++) t += sg[k];
      atomicAdd(ap.rec_segs, t);
    }
    for (int c = 0; c < 3; c++) px.sum[c * npix + p] = sum[c], px.mean[c * npix + p] = mean[c], px.m2[c * npix + p] = m2[c];
    px.samples[p] = n;
    px.conv[p] = conv;
    if (!conv && n < ap.budget) kn = adapt_next_batch(mean, m2, n, ap);
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
// slot off[q] + k being sample samples[p] + k of pixel p.  One block per 256 sub-pixels; its
// slots are a contiguous range written by all its threads (coalesced), each finding its
// sub-pixel by a search of the block's offsets in LDS.  The last sub-pixel's thread writes the
// phase's slot count.
__global__ __launch_bounds__(kBlock) void k_adapt_expand(const uint32_t* __restrict__ knext,
                                                         const uint32_t* __restrict__ off, int64_t nq, int32_t sub_n,
                                                         int32_t sub_j, const int32_t* __restrict__ samples,
                                                         uint2* __restrict__ smap,
                                                         unsigned long long* __restrict__ total) {
  __shared__ uint32_t s_off[kBlock], s_p[kBlock], s_s0[kBlock];
  __shared__ uint32_t s_end;
  const int t = threadIdx.x;
  const int64_t q0 = (int64_t)blockIdx.x * kBlock, q = q0 + t;
  const int nb = (int)min<int64_t>(kBlock, nq - q0);
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
