// rtx_frame_kernels.h — the frame's kernels around the persistent / wavefront trace (included
// by rtx_capi.hip only; rtx_park.hip compiles the PARK instantiations of k_persistent alone):
//
//   k_wf_generate / k_wf_shade   the wavefront mode's primaries and shading (k_wf_extend, the
//                                closest hit, is a template in rtx_kernels.h)
//   k_accumulate                 RecordSample / IsConverged in sample order (uniform groups)
//   k_adapt_record / _floor / _expand   adaptive sampling in phases (render_adaptive)
//   k_accumulate_sum             fixed spp: the in-order sum, the last group's resolved output
//   k_accumulate_mk_adaptive     the megakernel's AdaptiveSampler
//   k_frame_init / k_slot_block_init / k_resolve
#pragma once

#include "rtx_kernels.h"

namespace rtxd {

// ---------------------------------------------------------------------------------------
// Wavefront: primary generation for every slot of active pixels
// ---------------------------------------------------------------------------------------
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

// Shading for every queued path + compacted child queue (wavefront.cc:109-217).
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

// ---------------------------------------------------------------------------------------
// One radiance record x of a pixel: RecordSample (pixel_state.h:22-39), then IsConverged
// (pixel_state.h:54-72) once the pixel has min_spp samples; the statistics come in and go out
// through r (k_adapt_record).
// ---------------------------------------------------------------------------------------
struct PixRec {
  double sum[3], mean[3], m2[3];
  int n;
  bool conv;
};
// delta / n exactly as the IEEE division rounds it, from y = RN(1 / n) and one correction
// (Markstein: q = RN(delta y) is within an ulp of delta / n, r = delta - q n is exact by fma,
// RN(q + r y) is the correctly rounded quotient; checked bit for bit against the division on
// 2e8 quotients, near-ties included, tests/test_record_division.py).  Zero, tiny (where the
// theorem's no-underflow condition could fail) and non-finite deltas take the division.
__device__ __forceinline__ double div_by_count(double delta, double n, double y) {
  double q = delta * y;
  q = fma(fma(-q, n, delta), y, q);
  if (__builtin_expect(!(fabs(delta) >= 0x1p-900 && fabs(delta) < INFINITY), 0)) q = delta / n;
  return q;
}
// RecordSample's update (pixel_state.h:22-39) of one radiance record x
__device__ __forceinline__ void record_update(PixRec& r, const double (&x)[3]) {
  r.n++;
  const double dn = (double)r.n, y = 1.0 / dn;  // (one division per sample, for the three channels)
  for (int c = 0; c < 3; c++) {
    double mu = r.mean[c];
    double delta = x[c] - mu;
    mu += div_by_count(delta, dn, y);
    double delta2 = x[c] - mu;
    r.mean[c] = mu;
    r.m2[c] += delta2 * delta;
  }
  for (int c = 0; c < 3; c++) r.sum[c] += x[c];
}
// IsConverged (pixel_state.h:54-72) of the statistics after the update, once n >= min_spp:
// err / mu > rel  <=>  m2 > rel^2 (n - 1) n mu^2 up to the few ulps the exact form rounds by,
// so the products decide where the two sides differ by more than 1e-10 relative (the usual
// case), the exact form (two divisions, two square roots) only in between; NaN fails both
// comparisons and takes the exact form too.  (All channels must pass: a conjunction, so the
// order of the reference's early exit does not matter.)
__device__ __forceinline__ bool record_converged(const PixRec& r, int min_spp, double rel) {
  if (r.n < min_spp) return false;
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const double mu = fmax(fabs(r.mean[c]), 1e-3);
    const double thr = rel * rel * ((double)(r.n - 1) * (double)r.n * (mu * mu));
    if (r.m2[c] > thr * (1.0 + 1e-10)) ok = false;
    else if (__builtin_expect(!(r.m2[c] < thr * (1.0 - 1e-10)), 0)) {
      double var = r.n > 1 ? r.m2[c] / (r.n - 1) : 0.0;
      double err = sqrt(var) / sqrt((double)r.n);
      if (err / mu > rel) ok = false;
    }
  }
  return ok;
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

// ---------------------------------------------------------------------------------------
// RecordSample in sample order (pixel_state.h:22-39) + IsConverged (pixel_state.h:54-72)
// (PixelSoA: see the tile schedule above)
// ---------------------------------------------------------------------------------------
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
  // entry i of the phase just traced: sub-pixel list[i] (nullptr: the uniform first phase, every
  // sub-pixel, q = i), its samples kcur[i] (nullptr: kuni each), their first slot off[i]
  // (nullptr: p * kuni)
  const uint32_t* list;
  const uint32_t* kcur;
  const uint32_t* off;
  uint32_t* knext;       // out: samples of entry i in the next phase (0: finished)
  int32_t kuni;
  int32_t sub_n, sub_j;  // pixel p = q * sub_n + sub_j
  int32_t min_spp, budget, phase, kcap;
  int32_t kmin;  // smallest next batch: keeps a phase with few pixels left large enough to fill the GPU
  double rel;
  double margin_step;  // the batch margin grows by this much per phase (1 + step * (phase - 1))
  double margin1;      // ... except after the first phase: this margin
  // the prediction pooled over the pixel's 3 x 3 neighbourhood (k_adapt_plan) when pool_w > 0:
  // need(p) weighted pool_w, each neighbour's 1; rv holds every pixel's need at its last record,
  // in the render's own pixel grid of `width` columns
  float* rv;
  float pool_w;
  int32_t width;
  const uint16_t* segs;           // counting renders: segments of each slot's path (else nullptr)
  unsigned long long* rec_segs;   // ... summed here over the samples the pixels record
  unsigned long long* next_active;  // the next phase's pixel count, in kSpread words kSpreadStride
                                    // apart (added here, zeroed before the launch; k_adapt_floor sums)
};
// samples at which IsConverged would hold with the current estimates
__device__ __forceinline__ double adapt_need(const double (&mean)[3], const double (&m2)[3], int n, double rel) {
  double need = 0.0;
  for (int c = 0; c < 3; c++) {
    const double var = n > 1 ? m2[c] / (n - 1) : 0.0;
    const double mu = fmax(fabs(mean[c]), 1e-3);
    need = fmax(need, var / (rel * rel * mu * mu));
  }
  return need;
}
__device__ __forceinline__ uint32_t adapt_next_batch(double need, int n, const AdaptPlan& ap) {
  const int left = ap.budget - n;
  const double margin = ap.phase == 1 ? ap.margin1 : 1.0 + ap.margin_step * (double)(ap.phase - 1);
  const double want = (need - (double)n) * margin;
  int k = (want < (double)left) ? (int)ceil(want) : left;  // NaN / inf: the whole budget
  k = max(k, min(max(4 << min(ap.phase - 1, 4), ap.kmin), left));  // at least 4, 8, ... 64 more, and kmin
  k = (k + 3) & ~3;
  return (uint32_t)min(k, min(left, ap.kcap));
}
// Counters that every wave of a launch adds to are spread over kSpread words kSpreadStride words
// apart (a device-scope atomic add to one word serialises at ~10 ns per wave)
constexpr int kSpread = 64, kSpreadStride = 16;
// A wave's continuing pixels, added to the spread word of its block (every lane takes part).
__device__ __forceinline__ void spread_add(unsigned long long* base, uint32_t kn) {
  const unsigned long long na = __popcll(__ballot(kn != 0));
  if (na && lane_id() == 0) atomicAdd(base + (blockIdx.x % kSpread) * kSpreadStride, na);
}
// One lane per sub-pixel, one wave per block: the replay of a pixel's samples is sequential
// (each step divides by the running count), so the parallelism is across pixels.  The wave's
// 64 runs of the phase's radiance records (each contiguous: pixel-major slots) come in windows
// of kRecWin samples per lane, transposed through LDS: in each load instruction, 8 lanes read 8
// consecutive 8-byte pieces of one run, so an instruction touches 8 runs (~12 cache lines)
// instead of 64; each lane then replays its own run from LDS.  The next window's loads are in
// flight while the current one is replayed.
// (8-sample windows: 16-sample windows, 186 VGPRs, measured slower after the first phase: r8e)
constexpr int kRecLpr = 8,      // lanes per run in a load instruction
    kRecRuns = 64 / kRecLpr;    // runs per load instruction
__global__ __launch_bounds__(64) void k_adapt_record(PixelSoA px, const double* __restrict__ L, int64_t n,
                                                     int64_t npix, AdaptPlan ap) {
  constexpr int kRecWin = 8, kRecPieces = 3 * kRecWin,
                kRecPitch = kRecPieces + 1,  // (odd pitch: a lane's row starts on another bank)
      kRecGroups = (kRecPieces + kRecLpr - 1) / kRecLpr;  // load instructions per run and window
  __shared__ double s_win[64 * kRecPitch];
  __shared__ int64_t s_base[64];  // the lane's first radiance word
  __shared__ int32_t s_n[64];     // its words in the window being fetched
  const int lane = (int)threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;  // entry of the phase's pixel list
  int64_t p = 0, base = 0;
  int K = 0;
  bool act = false;
  PixRec r;
  r.n = 0, r.conv = false;
  if (i < n) {
    const int64_t q = ap.list ? (int64_t)ap.list[i] : i;
    p = q * ap.sub_n + ap.sub_j;
    K = ap.kcur ? (int)ap.kcur[i] : ap.kuni;
    act = K > 0 && !px.conv[p];
    base = 3 * (ap.off ? (int64_t)ap.off[i] : p * (int64_t)ap.kuni);
    if (act) load_pixel(r, px, npix, p);
  }
  const int n0 = r.n;
  s_base[lane] = base;
  s_n[lane] = act ? 3 * min(K, kRecWin) : 0;
  __syncthreads();
  // this lane's part of the loads: runs kRecRuns * j + a, pieces kRecLpr * g + b of each
  const int a = lane / kRecLpr, b = lane % kRecLpr;
  const double* rp[kRecRuns];
#pragma unroll
  for (int j = 0; j < kRecRuns; j++) rp[j] = L + s_base[kRecRuns * j + a] + b;
  double v[kRecRuns * kRecGroups];
  uint64_t got = 0;
  static_assert(kRecRuns * kRecGroups <= 64, "got: one bit per load");
  auto fetch = [&](int t) {  // the window of samples [t, t + kRecWin) of every lane's run
    got = 0;
#pragma unroll
    for (int j = 0; j < kRecRuns; j++) {
      const int nj = s_n[kRecRuns * j + a];
#pragma unroll
      for (int g = 0; g < kRecGroups; g++)
        if (kRecLpr * g + b < nj)
          v[j * kRecGroups + g] = rp[j][3 * t + kRecLpr * g], got |= 1ull << (j * kRecGroups + g);
    }
  };
  fetch(0);
  for (int t = 0;; t += kRecWin) {
    __syncthreads();  // the previous window is replayed, s_n read
#pragma unroll
    for (int j = 0; j < kRecRuns; j++)
#pragma unroll
      for (int g = 0; g < kRecGroups; g++)
        if (got >> (j * kRecGroups + g) & 1)
          s_win[(kRecRuns * j + a) * kRecPitch + kRecLpr * g + b] = v[j * kRecGroups + g];
    const int nn = act && !r.conv ? 3 * max(0, min(K - t - kRecWin, kRecWin)) : 0;
    s_n[lane] = nn;
    __syncthreads();
    const bool more = __ballot(nn > 0) != 0ull;
    if (more) fetch(t + kRecWin);
    if (act && !r.conv) {
      // (a straight-line pass over the window, IsConverged noted rather than branched on and the
      // converging window replayed again, measured slower: 527 vs 460 us per frame, r8e / r8f)
      const double* w = s_win + lane * kRecPitch;
      const int c = min(K - t, kRecWin);
      for (int k = 0; k < c && !r.conv; k++) {
        const double x[3] = {w[3 * k], w[3 * k + 1], w[3 * k + 2]};
        record_update(r, x);
        r.conv = record_converged(r, ap.min_spp, ap.rel);
      }
    }
    if (!more) break;
  }
  uint32_t kn = 0;
  if (act) {
    if (ap.segs) {  // counting render: the segments of the samples recorded (the rest are discarded)
      const uint16_t* sg = ap.segs + base / 3;
      unsigned long long t = 0;
      for (int k = 0; k < r.n - n0; k++) t += sg[k];
      atomicAdd(ap.rec_segs, t);
    }
    store_pixel(r, px, npix, p);
    const double need = adapt_need(r.mean, r.m2, r.n, ap.rel);
    if (ap.pool_w > 0.0f) ap.rv[p] = (float)need;  // k_adapt_plan sizes the batch
    else if (!r.conv && r.n < ap.budget) kn = adapt_next_batch(need, r.n, ap);
  }
  if (ap.pool_w > 0.0f) return;
  if (i < n) ap.knext[i] = kn;
  spread_add(ap.next_active, kn);
}
// The next batches from the prediction pooled over each pixel's 3 x 3 neighbourhood (after
// k_adapt_record, when ap.pool_w > 0): a pixel's relative variance is a property of what it
// sees, shared with its neighbours, and 16 samples estimate it poorly; the pooled estimate sizes
// the batch (the result does not depend on it, only the work and the phases do).
__global__ __launch_bounds__(kBlock) void k_adapt_plan(PixelSoA px, int64_t n, int64_t npix, AdaptPlan ap) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t kn = 0;
  if (i < n) {
    const int64_t q = ap.list ? (int64_t)ap.list[i] : i, p = q * ap.sub_n + ap.sub_j;
    const int ns = px.samples[p];
    if (!px.conv[p] && ns < ap.budget) {
      const int64_t w = ap.width, x = p % w, y = p / w;
      float acc = ap.pool_w * ap.rv[p], wsum = ap.pool_w;
      for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
          const int64_t xx = x + dx, yy = y + dy, pp = yy * w + xx;
          if ((dx | dy) == 0 || xx < 0 || xx >= w || yy < 0 || pp >= npix) continue;
          const float v = ap.rv[pp];
          if (v == v) acc += v, wsum += 1.0f;
        }
      kn = adapt_next_batch((double)(acc / wsum), ns, ap);
    }
    ap.knext[i] = kn;
  }
  spread_add(ap.next_active, kn);
}
// Once the next phase's pixel count is known: every batch at least target / that count (within
// the pixel's budget and the workspace), so a phase with few pixels left is large enough to
// fill the GPU, and the pixels finish in it rather than in further phases that would be mostly
// launch drain (the last paths of a launch run with their waves nearly empty).  (Finishing every
// pixel in the next phase whenever that adds fewer than 2^22 slots measured +0.3 % on C3,
// -0.2 % on C2: not kept, profiles/r05/ab/ab_adaptive_policy_r8k.txt.)
// It also writes the next phase's pixel count for the host (*pixels).
__global__ __launch_bounds__(kBlock) void k_adapt_floor(uint32_t* __restrict__ knext, const uint32_t* __restrict__ list,
                                                        int64_t n, int32_t sub_n,
                                                        int32_t sub_j, const int32_t* __restrict__ samples,
                                                        int32_t budget, int32_t kcap, int64_t target,
                                                        const unsigned long long* __restrict__ next_active,
                                                        unsigned long long* __restrict__ pixels) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  static_assert(kSpread == 64, "one spread counter per lane");
  unsigned long long na = next_active[lane_id() * kSpreadStride];
  for (int m = 32; m >= 1; m >>= 1) na += (unsigned long long)__shfl_xor((long long)na, m);
  if (i == 0) *pixels = na;
  if (i >= n) return;
  const uint32_t k = knext[i];
  if (k == 0) return;
  const int64_t q = list ? (int64_t)list[i] : i;
  const int64_t kmin = (target + (int64_t)na - 1) / (int64_t)max(na, 1ull);
  const int left = budget - samples[q * sub_n + sub_j];
  int kn = (int)max<int64_t>((int64_t)k, min<int64_t>(kmin, (int64_t)left));
  kn = (kn + 3) & ~3;
  knext[i] = (uint32_t)min(kn, min(left, kcap));
}
// The next phase's slot map and pixel list.  Entry i of the phase just recorded (sub-pixel
// list[i]) has knext[i] samples in the next phase; pk[i] (exclusive_scan_packed) holds their
// first slot (high word) and, when knext[i] != 0, the entry's index in the next list (low
// word).  The batch occupies slots [hi, hi + knext[i]), slot hi + k being sample samples[p] + k
// of pixel p, and the next list's entry gets (sub-pixel, samples, first slot).  One block per
// kExpandPix entries; its slots are a contiguous range written by all its threads (coalesced),
// each finding its entry by a search of the block's offsets in LDS.  The last entry's thread
// writes the phase's slot count and the map's address (k_adapt_floor wrote its pixel count).
// (Few entries per block: a block over 256 of them had up to 256 x kcap slots to write.)
constexpr int kExpandPix = 32;
struct AdaptList {  // a phase's pixel list: entry i = sub-pixel q[i], k[i] samples from slot off[i]
  uint32_t *q, *k, *off;
};
__global__ __launch_bounds__(kBlock) void k_adapt_expand(const uint32_t* __restrict__ knext,
                                                         const unsigned long long* __restrict__ pk,
                                                         const uint32_t* __restrict__ list, int64_t n, int32_t sub_n,
                                                         int32_t sub_j, const int32_t* __restrict__ samples,
                                                         uint2* __restrict__ smap, AdaptList next,
                                                         unsigned long long* __restrict__ total) {
  __shared__ uint32_t s_off[kExpandPix], s_p[kExpandPix], s_s0[kExpandPix];
  __shared__ uint32_t s_end;
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * kExpandPix, i = i0 + t;
  const int nb = (int)min<int64_t>(kExpandPix, n - i0);
  if (t < nb) {
    const uint32_t k = knext[i];
    const unsigned long long v = pk[i];
    const uint32_t o = (uint32_t)(v >> 32), idx = (uint32_t)v;
    const int64_t q = list ? (int64_t)list[i] : i, p = q * sub_n + sub_j;
    s_off[t] = o, s_p[t] = (uint32_t)p, s_s0[t] = k ? (uint32_t)samples[p] : 0u;
    if (k) next.q[idx] = (uint32_t)q, next.k[idx] = k, next.off[idx] = o;
    if (t == nb - 1) {
      s_end = o + k;
      if (i == n - 1) total[0] = (unsigned long long)o + k, total[2] = (unsigned long long)smap;
    }
  }
  __syncthreads();
  const uint32_t b = s_off[0], e = s_end;
  for (uint32_t j = b + t; j < e; j += kBlock) {
    int lo = 0, hi = nb;  // the last entry with s_off <= j (a zero batch shares its successor's offset)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_off[mid] <= j) lo = mid;
      else hi = mid;
    }
    smap[j] = make_uint2(s_p[lo], s_s0[lo] + (j - s_off[lo]));
  }
}


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

// AdaptiveSampler::SamplePixel (sampler.h:44-82) replayed in sample order for the MegaKernel
// renderer.  Its quirks are kept: `pixel` is the running SUM of the samples and the mean /
// variance are taken over those running sums; luminance uses float weights (color.h:35-37);
// the loop runs while samples <= max_samples, i.e. up to max_samples + 1 samples.  State:
// px.sum = pixel, px.mean = sum, px.m2 = sum_sq, px.samples, px.conv = finished.
__device__ __forceinline__ double luminance(double x, double y, double z) {
  return (double)0.2126f * x + (double)0.7152f * y + (double)0.0722f * z;
}
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

// wavefront.cc:229-235: sum / (float)samples  (Vec3 operator/ is (1/t)*v); megakernel
// (mega_kernel.h + sampler.h:32,79): pixel /= num_samples (DefaultSampler) or /= samples
// (AdaptiveSampler).
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
// An adaptive launch's slot counter block: the 8 region counters and the next phase's spread
// pixel counts (kSpreadBase, k_adapt_record's) zeroed, the slot count and the slot map's address
// set (set: 0 keeps them, as k_adapt_expand wrote them).
constexpr int kSpreadBase = 8 * 16 + 16;  // (words; the slot block is words 8 * 16 .. + 4)
constexpr int kAdaptCtrWords = kSpreadBase + kSpread * kSpreadStride;
__global__ void k_slot_block_init(unsigned long long* __restrict__ ctr, int set, unsigned long long nslots,
                                  unsigned long long smap) {
  const int i = (int)threadIdx.x;
  if (i < 8 * 16) ctr[i] = 0ull;
  if (i < kSpread) ctr[kSpreadBase + i * kSpreadStride] = 0ull;
  if (i == 0 && set) ctr[8 * 16] = nslots, ctr[8 * 16 + 2] = smap;
}
// The pixels an adaptive frame kept sampling after its output went to the host early
// (render_device_impl): each one's final value (k_resolve's arithmetic, adaptive) written
// straight into the caller's host framebuffer (device-mapped pinned memory, the whole image,
// pixel (x, y) at y * W + x) and into the device output.
__global__ __launch_bounds__(kBlock) void k_patch_host(PixelSoA px, int64_t npix, const uint32_t* __restrict__ list,
                                                       int64_t n, PixelMap map, double* __restrict__ host_rgb,
                                                       double* __restrict__ rgb, int32_t* __restrict__ spp_out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t p = list[i];
  const int ns = px.samples[p];
  const double sc = ns > 0 ? 1.0 / (double)(float)ns : 0.0;
  int x, y;
  map.xy((uint32_t)p, x, y);
  double* h = host_rgb + 3 * ((int64_t)y * map.W + x);
  for (int c = 0; c < 3; c++) {
    const double v = ns > 0 ? sc * px.sum[c * npix + p] : 0.0;
    rgb[3 * p + c] = v, h[c] = v;
  }
  if (spp_out) spp_out[p] = ns;
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

}  // namespace rtxd
