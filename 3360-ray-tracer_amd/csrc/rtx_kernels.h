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
constexpr int kRefillMinPark = 12;  // the same for the PARK kernel (12 vs 16: C3 adaptive +0.5 %, fixed +-0; r9f / r9g)
constexpr int kParkAt = 16;  // PARK kernel: park traversals once at most this many lanes still walk (ab_parkT_*)
// persistent: slots taken per atomic on a region's slot counter, by schedule (k_persistent
// kChunk): the plain kernel 256 (ab_chunk_*; 512 C2 -0.4 %), the PARK kernel 512 (bunny C3
// +0.7 %, profiles/r04/ab_chunk_map0_r6e_*.txt)
constexpr int kChunkPlain = 256, kChunkPark = 512;
// the same for the block-shared chunks of the adaptive phase launches (MAP 1; <= 511: ChunkLds),
// by schedule: the PARK kernel 128 (64: -0.3 %, 256: -2.1 % C3 adaptive), the plain kernel 256
// (C2 adaptive +1.0 % over 128; 64: -3.6 %) (profiles/r06/ab/ab_r10c_c3a.txt, ab_r10c_c2a.txt)
constexpr int kChunkSharedPlain = 256, kChunkSharedPark = 128;
static_assert(kChunkSharedPlain <= 511 && kChunkSharedPark <= 511, "ChunkLds keeps a chunk's size in 9 bits");

// Unsigned 32-bit division by a divisor fixed for a launch: one multiply-high, a subtract and
// two shifts (Granlund & Montgomery 1994; Hacker's Delight §10-9) instead of the ~17
// instructions of a runtime division (a float reciprocal, its corrections and three 32-bit
// multiplies, which do not pair).  For d >= 2, l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1
// and q = (t + ((n - t) >> 1)) >> (l - 1) with t = mulhi(n, m), exact for every n < 2^32;
// d = 1: m = 0 and no shifts.  tests/test_capi_exports.py checks it against the division.
struct FastDiv {
  uint32_t m, sh;  // magic; shifts: sh & 0xFF first (0 or 1), sh >> 8 second (l - 1)
  __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t t = (uint32_t)(((uint64_t)n * m) >> 32);
    return (t + ((n - t) >> (sh & 0xFFu))) >> (sh >> 8);
  }
};
inline FastDiv make_fastdiv(uint32_t d) {  // host side; d >= 1
  if (d <= 1) return FastDiv{0u, 0u};
  uint32_t l = 0;
  while (l < 32 && (1ull << l) < d) l++;
  const uint64_t m = ((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d) + 1;
  return FastDiv{(uint32_t)m, 1u | ((l - 1) << 8)};
}

// Pixel subset of the image handled by one call (rectangle or interleaved row stripes).
struct PixelMap {
  int32_t W, H;
  int32_t stripes;  // 0: rectangle, 1: stripes
  int32_t x0, y0, w, h;
  int32_t srows, sidx, scount;
  FastDiv frow, fsrows;  // division by the row length (w, or W for stripes) and by srows (set_map_div)
  // 32-bit arithmetic: the host keeps pixel counts below 2^31 (host side: rtx_internal_stripe_rows)
  // FD = false: the runtime divisions (the same quotients)
  template <bool FD = true>
  __host__ __device__ __forceinline__ void xy(uint32_t local, int& x, int& y) const {
    if (!stripes) {
      const uint32_t r = FD ? frow.div(local) : local / (uint32_t)w;
      x = x0 + (int)(local - r * (uint32_t)w);
      y = y0 + (int)r;
    } else {
      const uint32_t r = FD ? frow.div(local) : local / (uint32_t)W;
      x = (int)(local - r * (uint32_t)W);
      const uint32_t blk = FD ? fsrows.div(r) : r / (uint32_t)srows;
      y = ((int)blk * scount + sidx) * srows + (int)(r - blk * (uint32_t)srows);
    }
  }
};
inline void set_map_div(PixelMap& m) {
  const int row = m.stripes ? m.W : m.w;
  m.frow = make_fastdiv((uint32_t)(row > 1 ? row : 1));
  m.fsrows = make_fastdiv((uint32_t)(m.srows > 1 ? m.srows : 1));
}

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
  FastDiv fK;           // division by K (set with it: set_group)
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
// Stored non-temporal (global_store ... nt): the records (2.7 GB per C3 frame) stream through
// the L2 instead of displacing the scene's nodes and primitives (C3 +1.5 %, C3 adaptive +0.9 %,
// C2 +-0; profiles/r05/ab/ab_nt_records_r9c.txt).
__device__ __forceinline__ void store_radiance(const RenderArgs& A, uint32_t slot, V3 L) {
  double* Lp = A.L + 3 * (uint64_t)slot;
  __builtin_nontemporal_store(L.x, Lp), __builtin_nontemporal_store(L.y, Lp + 1), __builtin_nontemporal_store(L.z, Lp + 2);
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
  uint32_t stack, thr, hitp, leafq, block, end;  // byte offsets of the regions in a block's LDS, its size
};

// A render's per-pixel statistics (RecordSample's sum / mean / M2, the sample count, the
// converged flag), channel-major SoA.
struct PixelSoA {
  double *sum, *mean, *m2;  // 3 x npix each (channel-major)
  int32_t* samples;
  uint8_t* conv;
};

// PARK: 0 the plain schedule, 1 the PARK schedule with the leaf-step walk (trace4_run_step),
// 2 the PARK schedule with the speculative walk (trace4_run_spec; trees of at most
// kSpecMaxNodes nodes, its stack entries being 16-bit)
constexpr bool spec_walk(int park, bool fast, bool scatter) { return park == 2 && fast && !scatter; }
constexpr int64_t kSpecMaxNodes = 65536;
// The slot chunks of an adaptive phase launch (MAP == 1), one word per wave of the block: a
// chunk of up to kChunkShared slots of one slot region, claimed by LDS adds to its cursor, by its
// wave and, once the slot counters are dry, by the other waves of the block too.
// word = first slot (32 bits) | slots in the chunk (9 bits) | cursor (23 bits): a claim decodes
// its slots from the word alone (32-bit arithmetic; the region bounds are needed only to install
// a chunk).  The cursor cannot reach bit 23: a wave adds at most 64 per claim, and the claims on a
// word between two installs are bounded by the block's four chunks (at most ~6 k adds).
struct ChunkLds {
  unsigned long long w[kBlock / 64];
};
// block-wide region after the per-lane ones: 0 none, 1 the chunk words (MAP == 1)
constexpr uint32_t block_region_bytes(int kind) { return kind == 1 ? (uint32_t)sizeof(ChunkLds) : 0u; }
// which block-wide region a launch of k_persistent<..., SCATTER, ..., MAP> has
constexpr int block_region_kind(int map, bool scatter) { return map == 1 && !scatter ? 1 : 0; }
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

// counting builds of the persistent kernel: the loop's region cycles (CountersClk)
__device__ __forceinline__ void flush_clock(const RenderArgs& A, const CountersClk& c) {
  if (c.cyc_refill) atomicAdd(&A.counters[18], c.cyc_refill);
  if (c.cyc_walk) atomicAdd(&A.counters[19], c.cyc_walk);
  if (c.cyc_shade) atomicAdd(&A.counters[20], c.cyc_shade);
  if (c.wshade) atomicAdd(&A.counters[21], (unsigned long long)c.wshade);
  if (c.lshade) atomicAdd(&A.counters[22], (unsigned long long)c.lshade);
  if (c.cyc_leaf) atomicAdd(&A.counters[23], c.cyc_leaf);
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
// address (next_slot[130]), both written by k_adapt_expand.  MAP is a template parameter, not a
// kernel argument: the fixed-spp kernels run at the SGPR limit, and any extra uniform state
// there reshuffles their register allocation (a runtime switch cost the bunny's build 3.7 %, r3d).
template <int STACK, bool FAST, bool COUNT, bool SCATTER, int PARK, int TK = -1, bool LAMB = false,
          bool NOTEX = false, bool NODOF = false, int MAP = 0>
__global__ __launch_bounds__(kBlock, kTraceWaves) void k_persistent(RenderArgs A, unsigned long long* next_slot) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  // the LDS layout (persist_lds: the launch sizes it the same way; the host launches PARK
  // kernels only for fast, non-scatter renders)
  constexpr bool kSpecLds = spec_walk(PARK, FAST, SCATTER);
  constexpr bool kShared = block_region_kind(MAP, SCATTER) == 1;  // block-shared slot chunks (ChunkLds)
  // the PARK instantiations are compiled in rtx_park.hip only (its per-TU choices, rtx_device.h):
  // an implicit instantiation anywhere else is a compile error, not a silently different kernel
  static_assert((PARK > 0) == (RTX_PARK_TU != 0), "k_persistent: PARK kernels belong to rtx_park.hip");
  constexpr int kChunk = PARK ? kChunkPark : kChunkPlain;
  constexpr int kChunkShared = PARK ? kChunkSharedPark : kChunkSharedPlain;
  const PersistLds lay = persist_lds(A.stack_slots, kSpecLds, block_region_kind(MAP, SCATTER));
  char* const ldsb = (char*)lds;
  // counting builds: the launch's timeline (wall clock, 100 MHz): [13] ~first block start,
  // [14] last wave to find the slots used up, [15] ~first one, [16] last wave end, [17] ~first
  // wave end
  if (COUNT && threadIdx.x == 0) atomicMax(&A.counters[13], ~(unsigned long long)wall_clock64());
  unsigned long long* const cw = (unsigned long long*)(ldsb + lay.block);  // (kShared) the chunk words
  (void)cw;
  if (kShared) {
    if (threadIdx.x < kBlock / 64) cw[threadIdx.x] = 0ull;  // (no chunk: zero slots)
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
  constexpr bool kHitpLds = (NOTEX || kEarlyTex) && !SCATTER;
  (void)hitp_lds;
  const uint64_t nslots = MAP == 1 ? (uint64_t)next_slot[8 * 16] : (uint64_t)A.npix * (uint64_t)A.K;
  // GetPixel uses Interval(0.001, inf) (camera.h:158); IntersectBatch uses 0.001f (cpu_ray_integrator.h:21)
  const double tmin = SCATTER ? 0.001 : (double)0.001f;
  std::conditional_t<COUNT, CountersClk, Counters> c{};
  uint32_t segs = 0, prims = 0;
  // counting builds: the lane's path segments, stored per slot when the launch's slot counter
  // block names a buffer for them (adaptive renders: the segments of the recorded samples)
  uint32_t pseg = 0;
  uint16_t* const segbuf = !COUNT ? nullptr : (uint16_t*)next_slot[8 * 16 + 4];
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
  TravState trs;
  while (true) {
    // counting builds: region stamps (s_memtime, wave-uniform); t_walk is set by the lanes that
    // traced this round and read here, at the next loop top, where the wave has reconverged
    if constexpr (COUNT) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      const unsigned long long tw = __ballot(c.t_walk != 0);
      if (c.t_seg && tw) {  // the previous round traced: refill .. walk .. shading
        const uint64_t w = __shfl(c.t_walk, __ffsll((long long)tw) - 1);
        if (lane_id() == 0) c.cyc_refill += c.t_seg - c.t_top, c.cyc_walk += w - c.t_seg, c.cyc_shade += now - w;
      } else if (c.t_top && lane_id() == 0) {
        c.cyc_refill += now - c.t_top;  // (a round with nothing to trace: all refill / waiting)
      }
      c.t_top = now, c.t_seg = 0, c.t_walk = 0;
    }
    // ---- refill: ballot of idle lanes, leftover of the current chunk first.  Refilling
    // only once kRefillMin lanes are idle (or the wave is empty) amortises the
    // primary-generation code over several lanes.
    const unsigned long long idle = __ballot(!has);
    bool fresh = false;
    // (re-checked with the cheaper primary setup, FastDiv: PARK at 8 / 10, plain at 16 / 20 idle
    // lanes within +-0.4 %, r10q)
    constexpr int kRefill = kPark ? kRefillMinPark : kRefillMin;
    if (kShared) {
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
          const uint32_t cs = (uint32_t)(old >> 32), csz = ((uint32_t)old >> 23) & 0x1FFu, cur = (uint32_t)old & 0x7FFFFFu;
          const uint32_t got = cur < csz ? min(nidle - given, csz - cur) : 0u;
          if (!has && rank >= given && rank < given + got) slot = cs + cur + (rank - given), fresh = true;
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
              const uint32_t csz = (uint32_t)min<uint64_t>(kChunkShared, re - (rs + b));
              if (lane_id() == 0) atomicExch(&cw[wv], ((unsigned long long)(rs + b) << 32) | ((unsigned long long)csz << 23));
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
      constexpr bool kArgsAtRefill = !(LAMB && NOTEX);  // (also for the MAP 1 builds: -0.3 %, r10b)
      auto kseg = __builtin_amdgcn_kernarg_segment_ptr();
      if (kArgsAtRefill) asm volatile("" : "+s"(kseg));
      const RenderArgs& Ar = kArgsAtRefill ? *(const RenderArgs*)kseg : A;
      // (A must stay the kernel's first parameter: the counting builds, which every parity
      // test of the counts and the bench's counting pass run, check the argument segment
      // against the arguments and fault on a mismatch)
      if (COUNT && kArgsAtRefill && (Ar.npix != A.npix || Ar.seed != A.seed || Ar.stack_slots != A.stack_slots))
        __builtin_trap();
      // nslots < 2^32 (checked on the host): 32-bit division
      // the fixed-spp kernel (MAP 0) maps slot -> pixel -> row with the launch-constant divisions
      // (FastDiv: C2 +0.8 %, C5 +0.6 %, C3 +0.1 %, r10l); the phase kernel keeps the runtime
      // divisions (its C3 adaptive frame -0.35 % with FastDiv, register allocation; r10m)
      constexpr bool kFdMap1 = false;
      uint2 e = make_uint2(0u, 0u);
      if (MAP == 1) {  // a phase's slot map, or none: uniform groups (the adaptive first pass)
        const uint2* const sm = (const uint2*)next_slot[8 * 16 + 2];
        if (sm) {
          e = sm[slot];
        } else {
          const uint32_t q = kFdMap1 ? Ar.fK.div(slot) : slot / (uint32_t)Ar.K;
          e = make_uint2(q, (uint32_t)Ar.s0 + (slot - q * (uint32_t)Ar.K));
        }
      }
      const uint32_t p = MAP ? e.x : Ar.fK.div(slot);
      if (!(Ar.conv && Ar.conv[p])) {
        const int k = MAP ? 0 : (int)((uint32_t)slot - p * (uint32_t)Ar.K);
        int x, y;
        Ar.map.template xy<MAP == 0 || kFdMap1>(p, x, y);
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
    if (COUNT && lane_id() == 0) c.witers++;  // (the loop's rounds are wave-uniform: lane 0 counts)
    if (!__any(has)) {
      if (COUNT && lane_id() == 0) c.widle++;
      if (exhausted) break;
      continue;
    }
    if (COUNT) {
      const uint32_t live = (uint32_t)__popcll(__ballot(has));
      if (lane_id() == 0) c.wlive += live;
    }
    if constexpr (COUNT) c.t_seg = __builtin_amdgcn_s_memtime();
    if (!has) continue;
    // wave priority by phase: a wave walking (node visits, leaf tests) outranks one shading or
    // refilling, so the SIMD's issue slots go first to the walks, whose loads are the long
    // latencies (C3 +0.9 % over the load barriers alone; shading above walking, or leaf rounds
    // above or below node visits: slower; profiles/r06/ab/r10z_prio_c3.txt, r11c_c3.txt)
    __builtin_amdgcn_s_setprio(1);
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
        // (the phase launches, MAP 1, run the same thresholds: leaf rounds at 6 / 12 lanes and
        // parking at 12 / 20 lanes measured within noise on C3 adaptive, r10j)
        const bool done =
            kSpecLds ? trace4_run_spec<STACK, COUNT, TK>(A.S, P.o, P.d, tmin, stk16, leafq, kBlock, c, trs,
                                                         active > kParkAt ? kParkAt : -1)
                     : trace4_run<STACK, COUNT, TK>(A.S, P.o, P.d, tmin, stk, kBlock, c, trs,
                                                    active > kParkAt ? kParkAt : -1);
        parked = !done;
        if constexpr (COUNT) c.t_walk = __builtin_amdgcn_s_memtime();
        if (parked) continue;
        best = trs.best, tb = trs.closest, bmat = trs.mat;
      } else if (kPark) {  // no BVH, or its root is a leaf
        best = trace_flat(A.S, P.o, P.d, tmin, kInf, c, COUNT, tb, bmat);
      } else {
        best = trace<STACK, FAST, COUNT, TK>(A.S, P.o, P.d, tmin, kInf, stk, c, tb, bmat);
      }
      segs++;
      if constexpr (COUNT) {
        pseg++;
        if (!kPark || !park_ok) c.t_walk = __builtin_amdgcn_s_memtime();
        const unsigned long long sh = __ballot(1);
        if ((int)lane_id() == __ffsll((long long)sh) - 1) c.wshade++, c.lshade += (uint32_t)__popcll(sh);
      }
      __builtin_amdgcn_s_setprio(0);  // shading (and the refill after it) at the base priority
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
  if constexpr (COUNT) flush_clock(A, c);
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
// map, PK: 1 the leaf-step walk, 2 the speculative walk; the host never
// launches the PARK kernel for the scatter API, nor maps a scatter render's slots, but its
// dispatch names those builds)
#define RTX_PARK_INSTANCES(X)                                                                                    \
  X(32, false, false, 0, 1) X(32, true, false, 0, 1) X(64, false, false, 0, 1)                                  \
  X(64, true, false, 0, 1) X(32, false, true, 0, 1) X(32, true, true, 0, 1)                                     \
  X(64, false, true, 0, 1) X(64, true, true, 0, 1) X(32, false, false, 1, 1)                                    \
  X(32, true, false, 1, 1) X(64, false, false, 1, 1) X(64, true, false, 1, 1)                                   \
  X(32, false, false, 0, 2) X(32, true, false, 0, 2) X(64, false, false, 0, 2)                                  \
  X(64, true, false, 0, 2) X(32, false, false, 1, 2) X(32, true, false, 1, 2)                                   \
  X(64, false, false, 1, 2) X(64, true, false, 1, 2)
#define RTX_PARK_TRI_INSTANCES(Y) Y(32, 0, 1) Y(64, 0, 1) Y(32, 1, 1) Y(64, 1, 1) Y(32, 0, 2) Y(64, 0, 2) Y(32, 1, 2) Y(64, 1, 2)


}  // namespace rtxd
