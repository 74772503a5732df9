// rtx_bvh_build.hip — binned-SAH BVH build on the GPU (SURVEY §8f "GPU BVH build"), with
// output byte-identical to the host builder (host/src/geom.cc SahBuilder), which is itself
// pinned to the reference's Bvh::Build (bvh.h:39-68,166-367) by tests/golden.
//
// The host build is a sequential recursion; three of its details fix the output bytes and
// are reproduced exactly here:
//   * box unions fold left to right with std::min/std::max, so on equal values (±0) the
//     earlier primitive's bits win: each union is computed as an order-free key min/max
//     (±0 canonicalised) followed by the FIRST position that holds that value;
//   * libstdc++'s two-ended std::partition swaps the k-th failing element left of `mid`
//     with the k-th passing element counted from the right end: both ranks come from
//     block prefix sums, so the permutation is the same;
//   * nodes are numbered in pre-order (left subtree before right): the tree is built level
//     by level, then subtree sizes give every node its pre-order index.
// One workgroup per node of a level (the top levels are few, wide nodes; the lower levels
// are many narrow ones); the host loops over levels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "rtx.h"

extern "C" void rtx_internal_set_error(const char* msg);  // rtx_capi.hip

namespace {

constexpr int kB = 256;      // threads per node workgroup
constexpr int kWaves = kB / 64;
constexpr int kBins = 16;    // bvh.h: 16 SAH bins

struct BNode {  // BFS-order build record
  int32_t start, end;   // primitive range in idx
  int32_t left, right;  // BFS indices of the children (-1: leaf)
  int32_t size;         // nodes in the subtree (filled bottom-up)
  int32_t pre;          // pre-order index (filled top-down)
  double lo[3], hi[3];
};

struct Args {
  const double* bounds;  // n x 6: lo xyz, hi xyz (reference BoundingBox per primitive)
  int32_t* idx;          // permutation (prim_indices)
  int32_t* tmp_f;        // partition scratch (by position)
  int32_t* tmp_t;
  int32_t* rank;
  BNode* nodes;
  int32_t* n_nodes;      // allocation counter
};

// orderable key of a double, with -0 and +0 mapped to the same key
__device__ __forceinline__ uint64_t okey(double x) {
  if (x == 0.0) x = 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double okey_val(uint64_t k) {
  const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m), hi = __shfl_xor((uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
template <bool MAX>
__device__ __forceinline__ uint64_t wave_red64(uint64_t v) {
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t o = shfl_xor64(v, m);
    v = MAX ? (o > v ? o : v) : (o < v ? o : v);
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_min32(uint32_t v) {
  for (int m = 32; m >= 1; m >>= 1) {
    const uint32_t o = __shfl_xor(v, m);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// value of coordinate c (0..5 box lo/hi, 6..11 centroid as a degenerate box) of primitive p
__device__ __forceinline__ double coord(const double* __restrict__ b, int p, int c) {
  const double* q = b + 6 * (int64_t)p;
  if (c < 6) return q[c];
  const int a = (c - 6) % 3;
  return 0.5 * (q[a] + q[3 + a]);  // Aabb::center()
}

// SurfaceArea / LongestAxis as host/include/rt/geom.h (aabb.h)
__device__ __forceinline__ double area(const double lo[3], const double hi[3]) {
  const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}
__device__ __forceinline__ int bin_of(double c, double mn, double inv) {
  const int b = (int)((c - mn) * inv * 16);
  return b < 0 ? 0 : (b > 15 ? 15 : b);
}
// Interval union with std::min/std::max: first operand wins ties
__device__ __forceinline__ void unite(double lo[3], double hi[3], const double l2[3], const double h2[3]) {
  for (int a = 0; a < 3; a++) {
    lo[a] = l2[a] < lo[a] ? l2[a] : lo[a];
    hi[a] = hi[a] < h2[a] ? h2[a] : hi[a];
  }
}

__global__ __launch_bounds__(kB) void k_build_level(Args A, int32_t level_begin) {
  __shared__ uint64_t s_key[kWaves][12];
  __shared__ uint32_t s_pos[kWaves][12];
  __shared__ double s_val[12];
  __shared__ uint64_t s_bkey[kBins][6];
  __shared__ uint32_t s_bpos[kBins][6];
  __shared__ int s_bcnt[kBins];
  __shared__ int s_int[kWaves];
  __shared__ int s_dec[4];  // split (-1: leaf), axis, mid, true count
  __shared__ double s_dd[2];  // mn, inv
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  BNode* nd = A.nodes + level_begin + blockIdx.x;
  const int s = nd->start, e = nd->end, count = e - s;
  const double* __restrict__ B = A.bounds;
  int32_t* __restrict__ idx = A.idx;

  // ---- node box (coords 0..5) and centroid box (6..11): key min/max, then first position
  {
    uint64_t k[12];
    for (int c = 0; c < 12; c++) k[c] = (c % 6) < 3 ? ~0ull : 0ull;
    for (int i = s + tid; i < e; i += kB) {
      const int p = idx[i];
      for (int c = 0; c < 12; c++) {
        const uint64_t v = okey(coord(B, p, c));
        k[c] = (c % 6) < 3 ? (v < k[c] ? v : k[c]) : (v > k[c] ? v : k[c]);
      }
    }
    for (int c = 0; c < 12; c++) k[c] = (c % 6) < 3 ? wave_red64<false>(k[c]) : wave_red64<true>(k[c]);
    if (lane == 0)
      for (int c = 0; c < 12; c++) s_key[wave][c] = k[c];
    __syncthreads();
    if (tid < 12) {
      uint64_t v = s_key[0][tid];
      for (int w = 1; w < kWaves; w++) v = (tid % 6) < 3 ? min(v, s_key[w][tid]) : max(v, s_key[w][tid]);
      s_key[0][tid] = v;
    }
    __syncthreads();
    uint32_t pos[12];
    double want[12];
    for (int c = 0; c < 12; c++) pos[c] = 0xffffffffu, want[c] = okey_val(s_key[0][c]);
    for (int i = s + tid; i < e; i += kB) {
      const int p = idx[i];
      for (int c = 0; c < 12; c++)
        if (coord(B, p, c) == want[c] && (uint32_t)i < pos[c]) pos[c] = (uint32_t)i;
    }
    for (int c = 0; c < 12; c++) pos[c] = wave_min32(pos[c]);
    if (lane == 0)
      for (int c = 0; c < 12; c++) s_pos[wave][c] = pos[c];
    __syncthreads();
    if (tid < 12) {
      uint32_t v = s_pos[0][tid];
      for (int w = 1; w < kWaves; w++) v = min(v, s_pos[w][tid]);
      s_val[tid] = coord(B, idx[v], tid);
    }
    __syncthreads();
  }
  if (tid == 0) {
    for (int a = 0; a < 3; a++) nd->lo[a] = s_val[a], nd->hi[a] = s_val[3 + a];
    nd->left = nd->right = -1;
    int split = -1, axis = 0;
    if (count > 4) {
      const double* cl = s_val + 6;
      const double* ch = s_val + 9;
      const double dx = ch[0] - cl[0], dy = ch[1] - cl[1], dz = ch[2] - cl[2];
      axis = (dx >= dy && dx >= dz) ? 0 : (dy >= dz ? 1 : 2);
      const double mn = cl[axis], extent = ch[axis] - mn;
      if (extent > 0.0) {
        split = 0;  // provisional: binning follows
        s_dd[0] = mn, s_dd[1] = 1.0 / extent;
      }
    }
    s_dec[0] = split, s_dec[1] = axis;
  }
  if (tid < kBins) {
    s_bcnt[tid] = 0;
    for (int c = 0; c < 6; c++) s_bkey[tid][c] = c < 3 ? ~0ull : 0ull, s_bpos[tid][c] = 0xffffffffu;
  }
  __syncthreads();
  if (s_dec[0] < 0) return;  // leaf (count <= 4 or degenerate centroid extent)
  const int axis = s_dec[1];
  const double mn = s_dd[0], inv = s_dd[1];

  // ---- bins: counts, key min/max, then first position per bin and coordinate
  for (int i = s + tid; i < e; i += kB) {
    const int p = idx[i];
    const int b = bin_of(coord(B, p, 6 + axis), mn, inv);
    atomicAdd(&s_bcnt[b], 1);
    for (int c = 0; c < 6; c++) {
      const uint64_t v = okey(B[6 * (int64_t)p + c]);
      if (c < 3) atomicMin((unsigned long long*)&s_bkey[b][c], (unsigned long long)v);
      else atomicMax((unsigned long long*)&s_bkey[b][c], (unsigned long long)v);
    }
  }
  __syncthreads();
  for (int i = s + tid; i < e; i += kB) {
    const int p = idx[i];
    const int b = bin_of(coord(B, p, 6 + axis), mn, inv);
    for (int c = 0; c < 6; c++)
      if (B[6 * (int64_t)p + c] == okey_val(s_bkey[b][c])) atomicMin(&s_bpos[b][c], (uint32_t)i);
  }
  __syncthreads();
  if (tid == 0) {
    // SahBuilder::Emit: prefix unions from both ends, cost per split plane
    double bl[kBins][3], bh[kBins][3];
    int cnt[kBins];
    for (int b = 0; b < kBins; b++) {
      cnt[b] = s_bcnt[b];
      for (int c = 0; c < 3; c++)
        if (cnt[b]) bl[b][c] = B[6 * (int64_t)idx[s_bpos[b][c]] + c], bh[b][c] = B[6 * (int64_t)idx[s_bpos[b][3 + c]] + 3 + c];
    }
    double llo[kBins][3], lhi[kBins][3], rlo[kBins][3], rhi[kBins][3];
    int lc[kBins], rc[kBins];
    double alo[3] = {0, 0, 0}, ahi[3] = {0, 0, 0};
    int n = 0;
    for (int i = 0; i < kBins; i++) {
      if (cnt[i]) {
        if (n) unite(alo, ahi, bl[i], bh[i]);
        else for (int a = 0; a < 3; a++) alo[a] = bl[i][a], ahi[a] = bh[i][a];
        n += cnt[i];
      }
      for (int a = 0; a < 3; a++) llo[i][a] = alo[a], lhi[i][a] = ahi[a];
      lc[i] = n;
    }
    n = 0;
    for (int i = kBins - 1; i >= 0; i--) {
      if (cnt[i]) {
        if (n) unite(alo, ahi, bl[i], bh[i]);
        else for (int a = 0; a < 3; a++) alo[a] = bl[i][a], ahi[a] = bh[i][a];
        n += cnt[i];
      }
      for (int a = 0; a < 3; a++) rlo[i][a] = alo[a], rhi[i][a] = ahi[a];
      rc[i] = n;
    }
    const double A0 = area(nd->lo, nd->hi);
    double best = __builtin_inf();
    int split = -1;
    for (int i = 0; i < kBins - 1; i++) {
      if (lc[i] == 0 || rc[i + 1] == 0) continue;
      const double cost = (double)1.0f + (area(llo[i], lhi[i]) / A0) * lc[i] * (double)1.0f +
                          (area(rlo[i + 1], rhi[i + 1]) / A0) * rc[i + 1] * (double)1.0f;
      if (cost < best) best = cost, split = i;
    }
    if (split < 0 || best >= (double)((float)count * 1.0f)) split = -1;
    s_dec[0] = split;
  }
  __syncthreads();
  const int split = s_dec[0];
  if (split < 0) return;

  // ---- two-ended partition (libstdc++ __partition, bidirectional): true count first
  int tc = 0;
  for (int i = s + tid; i < e; i += kB) tc += bin_of(coord(B, idx[i], 6 + axis), mn, inv) <= split ? 1 : 0;
  tc = wave_sum(tc);
  if (lane == 0) s_int[wave] = tc;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    for (int w = 0; w < kWaves; w++) t += s_int[w];
    s_dec[3] = t;
  }
  __syncthreads();
  const int T = s_dec[3];
  const int mid = s + T;
  if (T != 0 && T != count) {
    // ranks: trues before position i (chunked block scan, in order)
    int carry = 0;
    for (int base = s; base < e; base += kB) {
      const int i = base + tid;
      const bool t = i < e && bin_of(coord(B, idx[i], 6 + axis), mn, inv) <= split;
      const unsigned long long bal = __ballot(t);
      const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) s_int[wave] = __popcll(bal);
      __syncthreads();
      int before = carry;
      for (int w = 0; w < wave; w++) before += s_int[w];
      int total = 0;
      for (int w = 0; w < kWaves; w++) total += s_int[w];
      if (i < e) {
        const int r = before + in_wave;  // trues in [s, i)
        A.rank[i] = r;
        if (i < mid && !t) A.tmp_f[s + ((i - s) - r)] = idx[i];  // k-th false left of mid
        if (i >= mid && t) A.tmp_t[s + (T - r - 1)] = idx[i];   // j-th true from the right
      }
      carry += total;
      __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    for (int i = s + tid; i < e; i += kB) {
      const int r = A.rank[i];
      const bool t = (i + 1 < e ? A.rank[i + 1] : T) != r;  // trues before i+1 > before i
      if (i < mid && !t) idx[i] = A.tmp_t[s + ((i - s) - r)];
      if (i >= mid && t) idx[i] = A.tmp_f[s + (T - r - 1)];
    }
  }
  if (tid == 0) {
    if (T == 0 || T == count) return;  // mid == start or end: leaf (no swaps happened)
    const int c = atomicAdd(A.n_nodes, 2);
    BNode* L = A.nodes + c;
    BNode* R = A.nodes + c + 1;
    L->start = s, L->end = mid, R->start = mid, R->end = e;
    nd->left = c, nd->right = c + 1;
  }
}

__global__ void k_sizes(BNode* nodes, int32_t begin, int32_t end) {
  const int i = begin + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= end) return;
  BNode& n = nodes[i];
  n.size = 1 + (n.left >= 0 ? nodes[n.left].size + nodes[n.right].size : 0);
}
__global__ void k_preorder(BNode* nodes, int32_t begin, int32_t end) {
  const int i = begin + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= end) return;
  const BNode& n = nodes[i];
  if (n.left < 0) return;
  nodes[n.left].pre = n.pre + 1;
  nodes[n.right].pre = n.pre + 1 + nodes[n.left].size;
}
__global__ void k_emit(const BNode* nodes, int32_t total, rtx_bvh_node* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const BNode& n = nodes[i];
  rtx_bvh_node o;
  for (int a = 0; a < 3; a++) o.lo[a] = n.lo[a], o.hi[a] = n.hi[a];
  if (n.left < 0) {
    o.is_leaf = 1, o.left_first = (uint32_t)n.start, o.right_count = (uint32_t)(n.end - n.start);
  } else {
    o.is_leaf = 0, o.left_first = (uint32_t)nodes[n.left].pre, o.right_count = (uint32_t)nodes[n.right].pre;
  }
  o.pad_ = 0;
  out[n.pre] = o;
}
__global__ void k_iota(int32_t* idx, int32_t n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) idx[i] = i;
}

struct Mem {
  std::vector<void*> ptrs;
  ~Mem() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <class T>
  T* get(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n * sizeof(T), 16)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return (T*)p;
  }
};

}  // namespace

extern "C" int rtx_bvh_build(int device, const double* bounds, int64_t n, rtx_bvh_node* out_nodes,
                             int64_t* out_n_nodes, uint32_t* out_prim_indices) {
  auto err = [](const std::string& m) {
    rtx_internal_set_error(m.c_str());
    return RTX_ERR_INVALID;
  };
  if (!bounds && n > 0) return err("rtx_bvh_build: bounds is NULL");
  if (!out_nodes || !out_n_nodes || !out_prim_indices) return err("rtx_bvh_build: NULL output");
  if (n < 0 || n > 0x3FFFFFFF) return err("rtx_bvh_build: primitive count out of range");
  *out_n_nodes = 0;
  if (n == 0) return RTX_OK;
  auto hip = [&](hipError_t e, const char* what) {
    if (e != hipSuccess) rtx_internal_set_error((std::string(what) + ": " + hipGetErrorString(e)).c_str());
    return e != hipSuccess;
  };
  if (hip(hipSetDevice(device), "hipSetDevice")) return RTX_ERR_HIP;
  Mem m;
  Args A;
  double* d_bounds = m.get<double>(6 * n);
  A.idx = m.get<int32_t>(n), A.tmp_f = m.get<int32_t>(n), A.tmp_t = m.get<int32_t>(n), A.rank = m.get<int32_t>(n);
  A.nodes = m.get<BNode>(2 * n);
  A.n_nodes = m.get<int32_t>(1);
  rtx_bvh_node* d_out = m.get<rtx_bvh_node>(2 * n);
  if (!d_bounds || !A.idx || !A.tmp_f || !A.tmp_t || !A.rank || !A.nodes || !A.n_nodes || !d_out)
    return err("rtx_bvh_build: device allocation failed");
  A.bounds = d_bounds;
  if (hip(hipMemcpy(d_bounds, bounds, 6 * n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy")) return RTX_ERR_HIP;
  hipLaunchKernelGGL(k_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, A.idx, (int32_t)n);
  BNode root{};
  root.start = 0, root.end = (int32_t)n, root.left = root.right = -1, root.pre = 0;
  int32_t one = 1;
  if (hip(hipMemcpy(A.nodes, &root, sizeof root, hipMemcpyHostToDevice), "hipMemcpy") ||
      hip(hipMemcpy(A.n_nodes, &one, sizeof one, hipMemcpyHostToDevice), "hipMemcpy"))
    return RTX_ERR_HIP;
  std::vector<std::pair<int32_t, int32_t>> levels;
  int32_t begin = 0, end = 1;
  while (begin < end) {
    levels.push_back({begin, end});
    hipLaunchKernelGGL(k_build_level, dim3((unsigned)(end - begin)), dim3(kB), 0, 0, A, begin);
    int32_t total = 0;
    if (hip(hipGetLastError(), "k_build_level") ||
        hip(hipMemcpy(&total, A.n_nodes, sizeof total, hipMemcpyDeviceToHost), "hipMemcpy"))
      return RTX_ERR_HIP;
    begin = end, end = total;
  }
  for (int l = (int)levels.size() - 1; l >= 0; l--) {
    const int32_t b = levels[l].first, e = levels[l].second;
    hipLaunchKernelGGL(k_sizes, dim3((unsigned)((e - b + 255) / 256)), dim3(256), 0, 0, A.nodes, b, e);
  }
  for (const auto& lv : levels)
    hipLaunchKernelGGL(k_preorder, dim3((unsigned)((lv.second - lv.first + 255) / 256)), dim3(256), 0, 0, A.nodes,
                       lv.first, lv.second);
  hipLaunchKernelGGL(k_emit, dim3((unsigned)((end + 255) / 256)), dim3(256), 0, 0, A.nodes, end, d_out);
  if (hip(hipGetLastError(), "k_emit") ||
      hip(hipMemcpy(out_nodes, d_out, (size_t)end * sizeof(rtx_bvh_node), hipMemcpyDeviceToHost), "hipMemcpy") ||
      hip(hipMemcpy(out_prim_indices, A.idx, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost), "hipMemcpy"))
    return RTX_ERR_HIP;
  *out_n_nodes = end;
  return RTX_OK;
}
