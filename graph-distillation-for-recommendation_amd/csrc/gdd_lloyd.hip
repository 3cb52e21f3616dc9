// gdd_lloyd.hip — (a6/a7/a8) grouping by label, ordered per-cluster folds, and the device-resident
// Lloyd loop of sklearn KMeans.fit.
//
// What is restated:
//   Lloyd M-step      _k_means_lloyd.pyx:111-160 with one OpenMP thread: per cluster, a sequential
//                     fp32 chain `sum + x*w` over its members in sample order; weight sums likewise
//   relocation input  _k_means_common.pyx:124-164 `((X - centers_old[labels])**2).sum(axis=1)`:
//                     numpy's pairwise sum over each contiguous row (gdd_relocate_distances)
//   average / shift   _k_means_common.pyx:215-251 `_average_centers` (empty clusters copy the FIRST
//                     heaviest cluster's row, averaged or not by loop order) and `_center_shift`
//   convergence       sklearn/cluster/_kmeans.py:717-734: strict label equality first, then
//                     `(center_shift**2).sum() <= tol` (numpy pairwise fp32 sum, compared in fp64)
//   cluster mean      clustgdd_agent_transduct.py:116-125 (`mean` of the members' rows): fp64 sum
//                     in sample order, one division, one rounding to fp32; empty -> NaN (or 0 for
//                     distill_recsys.py:623-636's clamp_min(1) means)
//
// Grouping is a stable counting sort: per wave-tile label histograms (LDS), one exclusive scan of
// the cluster-major histogram matrix, then each wave re-reads its tile and places every label at
// its cluster's running offset + its rank among equal labels of the same 64-label chunk (ballot
// match over the label bits). Sample order within a cluster is therefore preserved, which is what
// the ordered folds need.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdlib>

#include "gdd_common.hpp"

namespace gdd {
namespace {

inline unsigned blocks_of(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

// ---------------------------------------------------------------------------------------------
// stable counting sort of labels
// ---------------------------------------------------------------------------------------------
constexpr int kTileUnit = 1024;   // labels per wave per tile unit (16 per lane)
constexpr int kCountMaxK = 32768;  // LDS: (waves per block) x k int32 counters

struct GroupPlan {
  int m;           // tile = m * 1024 labels, one wave each
  int64_t ntiles;  // columns of the cluster-major histogram matrix
  int waves;       // waves per 256-lane block (each has its own k counters in LDS)
};

GroupPlan group_plan(int64_t n, int k) {
  GroupPlan p;
  p.m = (int)std::min<int64_t>(4, std::max<int64_t>(1, (n + (1 << 20) - 1) >> 20));
  p.ntiles = std::max<int64_t>(1, (n + (int64_t)p.m * kTileUnit - 1) / ((int64_t)p.m * kTileUnit));
  p.waves = k <= 4096 ? 4 : 1;
  return p;
}

template <int M>
__device__ __forceinline__ void load_tile(int64_t n, const int32_t* __restrict__ labels, int64_t base,
                                          int lane, int32_t (&lv)[M * 16]) {
#pragma unroll
  for (int q = 0; q < M * 16; ++q) {
    const int64_t i = base + (int64_t)q * 64 + lane;
    lv[q] = i < n ? labels[i] : -1;
  }
}

// per-tile histogram column: ghist[c * ntiles + t] = #{i in tile t : labels[i] == c}; labels outside
// [0, k) are not counted (they belong to no cluster, as in the reference's `labels == i` loop)
template <int M>
__global__ __launch_bounds__(256) void k_grp_hist(int64_t n, const int32_t* __restrict__ labels, int k,
                                                  int64_t ntiles, int32_t* __restrict__ ghist,
                                                  const int32_t* stop, int step_i) {
  if (stopped(stop, step_i)) return;
  extern __shared__ int32_t sh_cnt[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (t >= ntiles) return;  // whole wave; no block barriers below
  int32_t* h = sh_cnt + (size_t)wv * k;
  for (int c = lane; c < k; c += 64) h[c] = 0;
  int32_t lv[M * 16];
  load_tile<M>(n, labels, t * (M * kTileUnit), lane, lv);
#pragma unroll
  for (int q = 0; q < M * 16; ++q)
    if ((unsigned)lv[q] < (unsigned)k) atomicAdd(&h[lv[q]], 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  for (int c = lane; c < k; c += 64) ghist[(int64_t)c * ntiles + t] = h[c];
}

// gscan = exclusive scan of ghist (cluster-major): gscan[c * ntiles + t] is where tile t's first
// member of cluster c goes. Chunks of 64 labels are placed in order; within a chunk, lanes with equal
// labels (ballot match over the label bits) take consecutive slots by lane order.
template <int M>
__global__ __launch_bounds__(256) void k_grp_scatter(int64_t n, const int32_t* __restrict__ labels,
                                                     int k, int bits, int64_t ntiles,
                                                     const int32_t* __restrict__ ghist,
                                                     const int32_t* __restrict__ gscan,
                                                     int32_t* __restrict__ perm,
                                                     int32_t* __restrict__ offsets,
                                                     const int32_t* stop, int step_i) {
  if (stopped(stop, step_i)) return;
  extern __shared__ int32_t sh_off[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (t >= ntiles) return;
  int32_t* h = sh_off + (size_t)wv * k;
  for (int c = lane; c < k; c += 64) {
    const int32_t o = gscan[(int64_t)c * ntiles + t];
    h[c] = o;
    if (t == 0) offsets[c] = o;  // cluster c starts at its tile-0 offset
  }
  if (t == 0 && lane == 0) {
    const int64_t last = (int64_t)k * ntiles - 1;
    offsets[k] = gscan[last] + ghist[last];  // members with a label in [0, k)
  }
  int32_t lv[M * 16];
  const int64_t base = t * (M * kTileUnit);
  load_tile<M>(n, labels, base, lane, lv);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < M * 16; ++q) {
    const int l = lv[q];
    const bool ok = (unsigned)l < (unsigned)k;
    uint64_t peers = __ballot(ok);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (l >> b) & 1;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    if (ok) {
      const int32_t pos = h[l] + __popcll(peers & below);
      perm[pos] = (int32_t)(base + (int64_t)q * 64 + lane);
    }
    // every lane's read of h[l] above precedes the leader's update in this wave's LDS order
    if (ok && (peers & below) == 0) h[l] += __popcll(peers);
  }
}

// The same counting sort in ONE workgroup for small inputs (r04; n <= 32,768, k <= 2,048: the recsys
// KMeans shapes), instead of three dependent launches (histograms, scan, scatter: ~16 us of latency
// per Lloyd iteration there). Wave w owns tile w (M * 1024 labels, index order); its k counters sit in
// LDS. Then thread t owns clusters 2t and 2t+1: each column's exclusive prefix over the waves, the
// block's exclusive scan of the cluster totals, and the tile offsets; then the scatter of
// k_grp_scatter. Tiles, chunks and lanes are taken in index order: the same stable permutation.
constexpr int kGrpThr = 1024;
constexpr int kGrpWaves = kGrpThr / 64;
constexpr int64_t kGrpSmallMaxN = (int64_t)kGrpWaves * 2 * kTileUnit;  // M <= 2
constexpr int kGrpSmallMaxK = 2 * kGrpThr;

template <int M>
__global__ __launch_bounds__(kGrpThr) void k_grp_small(int64_t n, const int32_t* __restrict__ labels, int k,
                                                       int bits, int32_t* __restrict__ perm,
                                                       int32_t* __restrict__ offsets, const int32_t* stop,
                                                       int step_i) {
  if (stopped(stop, step_i)) return;
  extern __shared__ int32_t sh_grp[];  // [kGrpWaves][k]: counts, then each tile's running offsets
  __shared__ int32_t s_wt[kGrpWaves];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  int32_t* h = sh_grp + (size_t)wv * k;
  for (int c = lane; c < k; c += 64) h[c] = 0;
  int32_t lv[M * 16];
  const int64_t base = (int64_t)wv * (M * kTileUnit);
  load_tile<M>(n, labels, base, lane, lv);
#pragma unroll
  for (int q = 0; q < M * 16; ++q)
    if ((unsigned)lv[q] < (unsigned)k) atomicAdd(&h[lv[q]], 1);
  __syncthreads();
  // columns 2t, 2t+1: exclusive prefix over the waves (in place) and the totals
  int tot[2] = {0, 0};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = 2 * tid + u;
    if (c < k) {
      int run = 0;
      for (int w = 0; w < kGrpWaves; ++w) {
        const int v = sh_grp[(size_t)w * k + c];
        sh_grp[(size_t)w * k + c] = run;
        run += v;
      }
      tot[u] = run;
    }
  }
  // exclusive scan of the cluster totals in cluster order
  const int mine = tot[0] + tot[1];
  int inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_wt[wv] = inc;
  __syncthreads();
  int ex = inc - mine;
  for (int w = 0; w < wv; ++w) ex += s_wt[w];
  const int b0 = ex, b1 = ex + tot[0];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = 2 * tid + u;
    if (c < k) {
      const int bc = u ? b1 : b0;
      offsets[c] = bc;
      for (int w = 0; w < kGrpWaves; ++w) sh_grp[(size_t)w * k + c] += bc;
      if (c == k - 1) offsets[k] = bc + tot[u];  // members with a label in [0, k)
    }
  }
  __syncthreads();
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < M * 16; ++q) {
    const int l = lv[q];
    const bool ok = (unsigned)l < (unsigned)k;
    uint64_t peers = __ballot(ok);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (l >> b) & 1;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    if (ok) {
      const int32_t pos = h[l] + __popcll(peers & below);
      perm[pos] = (int32_t)(base + (int64_t)q * 64 + lane);
    }
    if (ok && (peers & below) == 0) h[l] += __popcll(peers);
  }
}

// radix fallback (k > kCountMaxK): stable sort of (label, index), then first-position offsets
__global__ void k_iota(int64_t n, int32_t* p) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (int32_t)i;
}

__global__ void k_offsets(int64_t n, const int32_t* __restrict__ skeys, int k,
                          int32_t* __restrict__ offsets) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const int prev = (i == 0) ? -1 : skeys[i - 1];
  const int cur = (i == n) ? k : skeys[i];
  for (int c = prev + 1; c <= cur && c <= k; ++c) offsets[c] = (int32_t)i;
}

size_t group_ws(int64_t n, int k) {
  if (k <= kCountMaxK) {
    const GroupPlan p = group_plan(n, k);
    const int64_t cells = (int64_t)k * p.ntiles;
    return 2 * align256(sizeof(int32_t) * (size_t)cells) + align256(scan_i32_ws_bytes(cells)) + 256;
  }
  return align256(sizeof(int32_t) * (size_t)n) * 2 + sort_pairs_ws_bytes(n) + 1024;
}

int group_dev(int64_t n, const int32_t* labels, int k, int32_t* perm, int32_t* offsets, void* ws,
              size_t ws_bytes, const int32_t* stop, int step_i, hipStream_t s) {
  Carver cv(ws, ws_bytes);
  if (n <= kGrpSmallMaxN && k <= kGrpSmallMaxK && !forced("group_split")) {
    int bits = 1;
    while ((1ll << bits) < (long long)k) ++bits;
    const size_t lds = sizeof(int32_t) * (size_t)kGrpWaves * k;
    auto fn = n <= (int64_t)kGrpWaves * kTileUnit ? k_grp_small<1> : k_grp_small<2>;
    if (lds > 65536)
      GDD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    fn<<<1, kGrpThr, lds, s>>>(n, labels, k, bits, perm, offsets, stop, step_i);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  if (k <= kCountMaxK) {
    const GroupPlan p = group_plan(n, k);
    const int64_t cells = (int64_t)k * p.ntiles;
    GDD_REQUIRE(cells < INT_MAX, "group_by_label: k x tiles too large");
    int32_t* ghist = cv.take<int32_t>(cells);
    int32_t* gscan = cv.take<int32_t>(cells);
    const size_t sb = scan_i32_ws_bytes(cells);
    void* sws = cv.take<char>(sb);
    if (!cv.ok()) return fail(GDD_E_WORKSPACE, "group_by_label: workspace too small");
    int bits = 1;
    while ((1ll << bits) < (long long)k) ++bits;
    const unsigned grid = (unsigned)((p.ntiles + p.waves - 1) / p.waves);
    const size_t lds = sizeof(int32_t) * (size_t)p.waves * k;
    auto go = [&](auto M_) -> int {
      constexpr int M = decltype(M_)::value;
      if (lds > 65536) {
        GDD_HIP(hipFuncSetAttribute((const void*)k_grp_hist<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        GDD_HIP(hipFuncSetAttribute((const void*)k_grp_scatter<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      }
      k_grp_hist<M><<<grid, 64 * p.waves, lds, s>>>(n, labels, k, p.ntiles, ghist, stop, step_i);
      GDD_LAUNCHED();
      int rc = exclusive_scan_i32(ghist, gscan, cells, sws, sb, s);
      if (rc) return rc;
      k_grp_scatter<M><<<grid, 64 * p.waves, lds, s>>>(n, labels, k, bits, p.ntiles, ghist, gscan, perm,
                                                       offsets, stop, step_i);
      GDD_LAUNCHED();
      return GDD_OK;
    };
    switch (p.m) {
      case 1: return go(std::integral_constant<int, 1>());
      case 2: return go(std::integral_constant<int, 2>());
      case 3: return go(std::integral_constant<int, 3>());
      default: return go(std::integral_constant<int, 4>());
    }
  }
  // the radix path does not read the stop word: after a stop it regroups the (unchanged) labels
  // into the workspace, which nothing reads any more
  int32_t* iota = cv.take<int32_t>(n);
  int32_t* skeys = cv.take<int32_t>(n);
  const size_t sb = sort_pairs_ws_bytes(n);
  void* sws = cv.take<char>(sb);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "group_by_label: workspace too small");
  int bits = 1;
  while ((1ll << bits) < (long long)k) ++bits;
  k_iota<<<blocks_of(n), 256, 0, s>>>(n, iota);
  GDD_LAUNCHED();
  int rc = sort_pairs_i32(labels, skeys, iota, perm, n, bits, sws, sb, s);
  if (rc) return rc;
  k_offsets<<<blocks_of(n + 1), 256, 0, s>>>(n, skeys, k, offsets);
  GDD_LAUNCHED();
  return GDD_OK;
}

// ---------------------------------------------------------------------------------------------
// ordered per-cluster folds: Lloyd sums (fp32 chain of x*w) and cluster means (fp64 chain of x)
// ---------------------------------------------------------------------------------------------
// Grid (feature slices, clusters), 256 threads. A block walks its cluster's members (perm[offsets[c]
// .. offsets[c+1]), sample order) in chunks of R rows x FW features staged through two LDS buffers:
// while thread f folds column f of chunk i (16 LDS reads in flight ahead of the dependent adds, two
// alternating register sets), chunk i+1's rows are in flight into registers, and chunk i+2's member
// ids (a three-slot ring) are loaded after the fold. Rows past a chunk's end are staged as +0.0,
// which leaves a sum that started at +0.0 unchanged, so the fold runs in unguarded groups of 16.
constexpr int kFoldElemsMax = 16384;  // floats per LDS chunk buffer (64 KiB)
// the cluster means use half-size chunk buffers: two workgroups fit a CU, so a launch of a few
// hundred clusters runs in one wave instead of two (each workgroup's chunk pipeline is latency-bound;
// arxiv bench shape, 454 clusters: 62.5 -> 50.4 us per cluster_mean call; quarter size 54.3)
constexpr int kFoldElemsMean = 8192;
// Lloyd sums of small clusters (r04): 8 KiB chunk buffers, so ~8 workgroups share a CU and a few
// hundred clusters of tens of members fold in one wave of workgroups instead of three (the recsys
// KMeans shapes: 6,040 x 64 with k = 604, ~10 members per cluster); dim <= 128 keeps R >= 16
constexpr int kFoldElemsSmall = 2048;
constexpr int kFoldSmallAvgRows = 64;
constexpr int kFoldMaxR = 1024;
constexpr int64_t kFoldPadMinRows = 65536;  // the M-step folds a zero-padded copy of X from here (dim % 4 != 0)

struct FoldArgs {
  int dim, fw_max, R;
  // clusters of at least big_rows members (0: none) are folded in feature slices of fw_big columns,
  // one workgroup per slice, R_big rows per chunk; Rmax = max(R, R_big) sizes the LDS id ring
  int big_rows, fw_big, R_big, Rmax;
  int c0;                  // first cluster of this launch; outputs are indexed from c0 (a slice)
  const float* X;
  const float* w;          // Lloyd sample weights (nullable: unit weights)
  const int32_t* perm;
  const int32_t* offsets;
  float* out;              // k x dim: sums (Lloyd) or means
  float* wsum;             // Lloyd weight sums
  long long* counts;       // mean: members per cluster (nullable)
  int empty_as_zero;
  const int32_t* stop;
  int step_i;
  int ld = 0;  // row stride of X (0: dim). A column range [f0, f1) folds X + f0 with dim = f1 - f0
  int64_t avg_rows = 0;  // members per cluster on average (0: unknown); small averages fold in 8 KiB chunks
  int out_dim = 0;  // output row stride and columns written (0: dim); folding a zero-padded copy of X
                    // (dim a multiple of 4) writes only its first out_dim columns
};

template <typename ACC, bool WEIGHTED>
__device__ __forceinline__ void fold_col(const float* __restrict__ col, int stride, int rp, ACC& acc,
                                         const float* __restrict__ W) {
  float A[16], B[16], WA[16], WB[16];
  auto ld = [&](float(&v)[16], float(&wv)[16], int r0) {
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = col[(r0 + u) * stride];
    if constexpr (WEIGHTED) {
#pragma unroll
      for (int u = 0; u < 16; ++u) wv[u] = W[r0 + u];
    }
  };
  auto add = [&](const float(&v)[16], const float(&wv)[16]) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (WEIGHTED) {
        const float term = v[u] * wv[u];
        acc = acc + (ACC)term;
      } else {
        acc = acc + (ACC)v[u];
      }
    }
  };
  ld(A, WA, 0);
  // opaque first group + scheduling barriers: keeps each group's reads a group of adds ahead (the
  // compiler otherwise folds the loop's phi of loads and re-issues every read next to its adds)
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    asm volatile("" : "+v"(A[u]));
    if constexpr (WEIGHTED) asm volatile("" : "+v"(WA[u]));
  }
  int r0 = 0;
  for (; r0 + 32 <= rp; r0 += 32) {
    ld(B, WB, r0 + 16);
    __builtin_amdgcn_sched_barrier(0);
    add(A, WA);
    __builtin_amdgcn_sched_barrier(0);
    if (r0 + 32 < rp) ld(A, WA, r0 + 32);
    __builtin_amdgcn_sched_barrier(0);
    add(B, WB);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (r0 < rp) add(A, WA);
}

template <typename ACC, bool VEC, bool WEIGHTED, bool MEAN, int kFoldElems = kFoldElemsMax>
__global__ __launch_bounds__(256) void k_seg_fold(const FoldArgs a) {
  if (stopped(a.stop, a.step_i)) return;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int U = VEC ? 4 : 1;            // floats per staged element
  constexpr int Q = kFoldElems / (256 * U);  // staged elements per thread per chunk
  const int dim = a.dim, tid = threadIdx.x;
  const int64_t ldx = a.ld ? a.ld : dim;
  const int c = a.c0 + (int)blockIdx.y;
  const int32_t b = a.offsets[c], e = a.offsets[c + 1];
  const int nm = e - b;
  // a large cluster's columns are split over the grid's x slices (each column's chain is its own,
  // so the order is unchanged): its CU gathers a third of each row instead of the whole row
  const bool big = a.big_rows > 0 && nm >= a.big_rows;
  const int fw = big ? a.fw_big : a.fw_max;
  const int f0 = blockIdx.x * fw;
  if (f0 >= dim) return;  // a slice only large clusters use
  const int R = big ? a.R_big : a.R;
  float* Bbuf = smem;
  int32_t* sid = reinterpret_cast<int32_t*>(smem + 2 * kFoldElems);  // 3 x Rmax
  float* Wbuf = smem + 2 * kFoldElems + 3 * a.Rmax;                    // 3 x Rmax (WEIGHTED)
  const int FW = min(fw, dim - f0);
  const int FWu = FW / U;
  ACC acc = 0;
  float wacc = 0.f;
  if (nm > 0) {
    const int nch = (nm + R - 1) / R;
    const int dr = 256 / FWu, df = 256 % FWu;
    const int r_init = tid / FWu, f_init = tid % FWu;
    float xv[Q * U];
    // member ids of a chunk: requested into registers early (fetch_ids), written to their LDS slot
    // later (put_ids), so the perm read overlaps a gather and a fold instead of ending an iteration
    constexpr int kIdsPer = kFoldMaxR / 256;
    int32_t idv[kIdsPer];
    auto fetch_ids = [&](int chunk) {
      const int m0 = chunk * R;
      const int rows = min(R, nm - m0);
#pragma unroll
      for (int q = 0; q < kIdsPer; ++q) {
        const int r = tid + 256 * q;
        if (r < R) idv[q] = a.perm[b + m0 + min(r, rows - 1)];
      }
    };
    auto put_ids = [&](int chunk) {
      const int slot = chunk % 3, m0 = chunk * R;
      const int rows = min(R, nm - m0);
#pragma unroll
      for (int q = 0; q < kIdsPer; ++q) {
        const int r = tid + 256 * q;
        if (r < R) {
          sid[slot * R + r] = idv[q];
          if constexpr (WEIGHTED) Wbuf[slot * R + r] = r < rows ? a.w[idv[q]] : 0.f;
        }
      }
    };
    auto load_ids = [&](int chunk) {
      fetch_ids(chunk);
      put_ids(chunk);
    };
    auto gather = [&](int chunk) {
      const int32_t* ids = sid + (chunk % 3) * R;
      int r = r_init, f = f_init;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int64_t id = ids[min(r, R - 1)];
        const float* src = a.X + id * ldx + f0 + f * U;
        if constexpr (VEC) {
          const float4 v = *reinterpret_cast<const float4*>(src);
          xv[4 * q] = v.x;
          xv[4 * q + 1] = v.y;
          xv[4 * q + 2] = v.z;
          xv[4 * q + 3] = v.w;
        } else {
          xv[q] = *src;
        }
        r += dr;
        f += df;
        if (f >= FWu) {
          f -= FWu;
          ++r;
        }
      }
    };
    auto store = [&](int chunk) {
      float* B = Bbuf + (chunk & 1) * kFoldElems;
      const int rows = min(R, nm - chunk * R);
      int r = r_init, f = f_init;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (r < R) {
          const bool live = r < rows;
          if constexpr (VEC) {
            float4 v = live ? make_float4(xv[4 * q], xv[4 * q + 1], xv[4 * q + 2], xv[4 * q + 3])
                            : make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(B + r * FW + 4 * f) = v;
          } else {
            B[r * FW + f] = live ? xv[q] : 0.f;
          }
        }
        r += dr;
        f += df;
        if (f >= FWu) {
          f -= FWu;
          ++r;
        }
      }
    };
    load_ids(0);
    if (nch > 1) load_ids(1);
    __syncthreads();
    gather(0);
    store(0);
    __syncthreads();
    for (int i = 0; i < nch; ++i) {
      const int rows = min(R, nm - i * R);
      if (i + 2 < nch) fetch_ids(i + 2);  // in flight through this iteration's gather and fold
      if (i + 1 < nch) gather(i + 1);  // ids of chunk i+1 were staged before the last barrier
      if (tid < FW) {
        const float* col = Bbuf + (i & 1) * kFoldElems + tid;
        fold_col<ACC, WEIGHTED>(col, FW, (rows + 15) & ~15, acc, Wbuf + (i % 3) * R);
      }
      if (WEIGHTED && tid == 255) {
        const float* W = Wbuf + (i % 3) * R;
        for (int r = 0; r < rows; ++r) wacc = wacc + W[r];
      }
      if (i + 1 < nch) {
        store(i + 1);                       // buffer (i+1)&1 was last read in iteration i-1
        if (i + 2 < nch) put_ids(i + 2);    // slot (i+2)%3 was last read in iteration i-1
      }
      __syncthreads();
    }
  }
  const int cs = c - a.c0;  // row of the output slice
  const int dout = a.out_dim ? a.out_dim : dim;
  const int64_t ob = (int64_t)cs * dout + f0;
  if constexpr (MEAN) {
    if (tid < FW) {
      float r;
      if (nm == 0)
        r = a.empty_as_zero ? 0.f : __builtin_nanf("");
      else
        r = (float)((double)acc / (double)nm);
      a.out[ob + tid] = r;
    }
    if (blockIdx.x == 0 && tid == 0 && a.counts) a.counts[cs] = nm;
  } else {
    if (tid < FW && f0 + tid < dout) a.out[ob + tid] = (float)acc;
    // unit weights: a sequential fp32 count, which sticks at 2^24
    if (blockIdx.x == 0 && tid == 255) a.wsum[cs] = WEIGHTED ? wacc : fminf((float)nm, 16777216.f);
  }
}

// The Lloyd sums over 16-byte aligned rows (r05; unit weights, FW <= 64): one wave folds, three
// gather. k_seg_fold's folding threads read one LDS float per add from row-major chunks while the same
// waves gather, and at the products shape (a 48-float padded row, 336-row chunks) the fold's dependent
// chain set the chunk time. Here the chunks are stored column-major (column f's rows contiguous,
// stride RS = R + 4 floats: RS/4 odd spreads eight consecutive columns over distinct bank groups), so
// lane f of wave 0 reads four rows per 16-byte LDS read, eight reads (32 rows) ahead of its adds, and
// waves 1..3 keep chunk i+2's rows in flight (registers) and chunk i+3's member ids (a three-slot LDS
// ring) while chunk i is folded. Same chains, same order: rows past a chunk's end are staged as +0.0.
constexpr int kCmGatherThreads = 192;

__global__ __launch_bounds__(256) void k_seg_fold_cm(const FoldArgs a) {
  if (stopped(a.stop, a.step_i)) return;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int dim = a.dim, tid = threadIdx.x;
  const int64_t ldx = a.ld ? a.ld : dim;
  const int c = a.c0 + (int)blockIdx.y;
  const int32_t b = a.offsets[c], e = a.offsets[c + 1];
  const int nm = e - b;
  const bool big = a.big_rows > 0 && nm >= a.big_rows;
  const int fw = big ? a.fw_big : a.fw_max;
  const int f0 = blockIdx.x * fw;
  if (f0 >= dim) return;
  const int R = big ? a.R_big : a.R;
  const int RS = R + 4;
  const int FW = min(fw, dim - f0);
  const int FWu = FW >> 2;
  // two column-major chunk buffers of FW x RS floats
  const int bufsz = max(a.fw_max * (a.R + 4), a.fw_big * (a.R_big + 4));
  float* Bb = smem;
  float acc = 0.f;
  if (nm > 0) {
    const int nch = (nm + R - 1) / R;
    const bool gat = tid >= 64;
    const int g = tid - 64;
    // gather slots: idx = g + 192 j over R x FWu float4 pieces (row r = idx / FWu, piece q = idx % FWu)
    const int dr = kCmGatherThreads / FWu, dq = kCmGatherThreads % FWu;
    const int r_init = gat ? g / FWu : 0, q_init = gat ? g % FWu : 0;
    // every slot loads (rows past R repeat row R-1 and are not stored): the outstanding-load counts
    // are static, so waiting for one chunk's rows never waits for the next chunk's ids
    constexpr int kMaxSlot = 22;  // R * FWu <= 16384 / 4 = 4096 pieces over 192 threads
    float4 xv[kMaxSlot];
    int32_t idr[kMaxSlot];
    auto fetch_ids = [&](int chunk) {  // each slot's member id, straight from perm
      const int m0 = chunk * R;
      const int last = min(R, nm - m0) - 1;
      int r = r_init, q = q_init;
#pragma unroll
      for (int j = 0; j < kMaxSlot; ++j) {
        idr[j] = a.perm[b + m0 + min(r, last)];
        r += dr;
        q += dq;
        if (q >= FWu) {
          q -= FWu;
          ++r;
        }
      }
    };
    auto gather = [&]() {
      int r = r_init, q = q_init;
#pragma unroll
      for (int j = 0; j < kMaxSlot; ++j) {
        (void)r;
        xv[j] = *reinterpret_cast<const float4*>(a.X + (int64_t)idr[j] * ldx + f0 + 4 * q);
        r += dr;
        q += dq;
        if (q >= FWu) {
          q -= FWu;
          ++r;
        }
      }
    };
    auto store = [&](int chunk) {
      float* B = Bb + (chunk & 1) * bufsz;
      const int rows = min(R, nm - chunk * R);
      int r = r_init, q = q_init;
#pragma unroll
      for (int j = 0; j < kMaxSlot; ++j) {
        if (r < R) {
          const bool live = r < rows;
          float* d = B + (4 * q) * RS + r;
          d[0] = live ? xv[j].x : 0.f;
          d[RS] = live ? xv[j].y : 0.f;
          d[2 * RS] = live ? xv[j].z : 0.f;
          d[3 * RS] = live ? xv[j].w : 0.f;
        }
        r += dr;
        q += dq;
        if (q >= FWu) {
          q -= FWu;
          ++r;
        }
      }
    };
    // prologue: chunk 0 staged, chunk 1's rows and chunk 2's ids in flight
    if (gat) {
      fetch_ids(0);
      gather();
      store(0);
      if (nch > 1) {
        fetch_ids(1);
        gather();
      }
      if (nch > 2) fetch_ids(2);
    }
    __syncthreads();
    for (int i = 0; i < nch; ++i) {
      if (tid < 64) {
        if (tid < FW) {  // column tid of chunk i: 16-byte reads, eight (32 rows) ahead of the adds
          const float* col = Bb + (i & 1) * bufsz + tid * RS;
          const int rows = min(R, nm - i * R);
          const int n4 = (rows + 3) >> 2;
          float4 A[8], Bv[8];
          auto ld = [&](float4(&v)[8], int g0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4*>(col)[min(g0 + u, (R >> 2) - 1)];
          };
          auto add = [&](const float4(&v)[8], int g0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              if (g0 + u < n4) {
                acc = acc + v[u].x;
                acc = acc + v[u].y;
                acc = acc + v[u].z;
                acc = acc + v[u].w;
              }
            }
          };
          ld(A, 0);
#pragma unroll
          for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(A[u].x), "+v"(A[u].y), "+v"(A[u].z), "+v"(A[u].w));
          int g0 = 0;
          for (; g0 + 16 <= n4; g0 += 16) {
            ld(Bv, g0 + 8);
            __builtin_amdgcn_sched_barrier(0);
            add(A, g0);
            __builtin_amdgcn_sched_barrier(0);
            if (g0 + 16 < n4) ld(A, g0 + 16);
            __builtin_amdgcn_sched_barrier(0);
            add(Bv, g0 + 8);
            __builtin_amdgcn_sched_barrier(0);
          }
          if (g0 < n4) {
            add(A, g0);
            if (g0 + 8 < n4) {
              ld(Bv, g0 + 8);
              add(Bv, g0 + 8);
            }
          }
        }
      } else if (gat) {
        if (i + 1 < nch) store(i + 1);  // buffer (i+1)&1 was last read in iteration i-1
        if (i + 2 < nch) {
          gather();                      // chunk i+2's rows (its ids landed an iteration ago)
          if (i + 3 < nch) fetch_ids(i + 3);
        }
      }
      __syncthreads();
    }
  }
  const int cs = c - a.c0;
  const int dout = a.out_dim ? a.out_dim : dim;
  const int64_t ob = (int64_t)cs * dout + f0;
  if (tid < FW && f0 + tid < dout) a.out[ob + tid] = acc;
  if (blockIdx.x == 0 && tid == 255) a.wsum[cs] = fminf((float)nm, 16777216.f);
}

// clusters [a0.c0, a0.c0 + count): launches of at most kFoldMaxGridY clusters (grid.y), each
// writing its slice of the outputs
constexpr int kFoldMaxGridY = 65535;
int fold_launch_one(const FoldArgs& a0, int count, bool mean, hipStream_t s);
int fold_launch(const FoldArgs& a0, int count, bool mean, hipStream_t s) {
  GDD_REQUIRE(count >= 0, "cluster fold: %d clusters", count);
  for (int off = 0; off < count; off += kFoldMaxGridY) {
    FoldArgs a = a0;
    a.c0 = a0.c0 + off;
    a.out = a0.out + (int64_t)off * (a0.out_dim ? a0.out_dim : a0.dim);
    if (a0.wsum) a.wsum = a0.wsum + off;
    if (a0.counts) a.counts = a0.counts + off;
    const int rc = fold_launch_one(a, std::min(kFoldMaxGridY, count - off), mean, s);
    if (rc) return rc;
  }
  return GDD_OK;
}

int fold_launch_one(const FoldArgs& a0, int count, bool mean, hipStream_t s) {
  FoldArgs a = a0;
  const bool weighted = a.w != nullptr;
  a.fw_max = std::min(a.dim, weighted ? 192 : 256);  // weighted: thread 255 folds the weights
  if (a.fw_max % 4 != 0 && a.fw_max < a.dim) a.fw_max &= ~3;
  const bool small = !mean && a.avg_rows > 0 && a.avg_rows <= kFoldSmallAvgRows && a.dim <= 128;
  const int elems = mean ? kFoldElemsMean : (small ? kFoldElemsSmall : kFoldElemsMax);
  int R = std::min(kFoldMaxR, elems / a.fw_max);
  R &= ~15;
  a.R = std::max(R, 16);
  const int ldx = a.ld ? a.ld : a.dim;
  const bool vec = a.dim % 4 == 0 && ldx % 4 == 0 && a.fw_max % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.X) & 15) == 0;
  unsigned nsl = (unsigned)((a.dim + a.fw_max - 1) / a.fw_max);
  constexpr int kSliceCols = 16;  // columns per slice of a large cluster (a multiple of 4)
  if (a.big_rows > 0 && !mean && a.fw_max > kSliceCols) {
    a.fw_big = kSliceCols;
    a.R_big = std::max(16, std::min(kFoldMaxR, elems / kSliceCols) & ~15);
    nsl = std::max<unsigned>(nsl, (unsigned)((a.dim + kSliceCols - 1) / kSliceCols));
  } else {
    a.big_rows = 0;
    a.fw_big = a.fw_max;
    a.R_big = a.R;
  }
  a.Rmax = std::max(a.R, a.R_big);
  if (count == 0) return GDD_OK;
  dim3 grid(nsl, (unsigned)count);
  {  // unit-weight Lloyd sums over 16-byte aligned rows: the column-major form
    if (!mean && !weighted && !small && vec && a.fw_max <= 64 && a.fw_big <= 64) {
      const size_t bufsz = std::max<size_t>((size_t)a.fw_max * (a.R + 4), (size_t)a.fw_big * (a.R_big + 4));
      const size_t lds_cm = sizeof(float) * 2 * bufsz;
      GDD_HIP(hipFuncSetAttribute((const void*)k_seg_fold_cm, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds_cm));
      k_seg_fold_cm<<<grid, 256, lds_cm, s>>>(a);
      GDD_LAUNCHED();
      return GDD_OK;
    }
  }
  const size_t lds = sizeof(float) * (2 * (size_t)elems + 3 * (size_t)a.Rmax * (weighted ? 2 : 1));
  auto go = [&](auto kern) -> int {
    GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    kern<<<grid, 256, lds, s>>>(a);
    GDD_LAUNCHED();
    return GDD_OK;
  };
  if (mean)
    return vec ? go(k_seg_fold<double, true, false, true, kFoldElemsMean>)
               : go(k_seg_fold<double, false, false, true, kFoldElemsMean>);
  if (small) {
    if (weighted)
      return vec ? go(k_seg_fold<float, true, true, false, kFoldElemsSmall>)
                 : go(k_seg_fold<float, false, true, false, kFoldElemsSmall>);
    return vec ? go(k_seg_fold<float, true, false, false, kFoldElemsSmall>)
               : go(k_seg_fold<float, false, false, false, kFoldElemsSmall>);
  }
  if (weighted)
    return vec ? go(k_seg_fold<float, true, true, false>) : go(k_seg_fold<float, false, true, false>);
  return vec ? go(k_seg_fold<float, true, false, false>) : go(k_seg_fold<float, false, false, false>);
}

// ---------------------------------------------------------------------------------------------
// numpy pairwise sum (umath loops_utils.h.src): n < 8 sequential; n <= 128 eight interleaved
// accumulators ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the n % 8 tail; otherwise split at n/2
// rounded down to a multiple of 8, left + right.
// ---------------------------------------------------------------------------------------------
template <class F>
__device__ float pw_leaf(F val, int off, int n) {
  if (n < 8) {
    float res = 0.f;
    for (int i = 0; i < n; ++i) res = res + val(off + i);
    return res;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = val(off + j);
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + val(off + i + j);
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + val(off + i);
  return res;
}

template <int D, class F>
__device__ __attribute__((noinline)) float pw_sum(F val, int off, int n) {
  if constexpr (D == 0) {
    return pw_leaf(val, off, n);
  } else {
    if (n <= 128) return pw_leaf(val, off, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_sum<D - 1>(val, off, n2) + pw_sum<D - 1>(val, off + n2, n - n2);
  }
}
constexpr int kPwDepth = 24;  // n < 128 * 2^24

// the Lloyd loop's control words
// Iteration i runs as two steps: 2i (E-step labels, grouping, sums, the empty-cluster check) and
// 2i+1 (average + shift, labels changed, convergence). stop_at = s+1 skips every later step.
struct LloydState {
  int32_t stop_at;   // offset 0
  int32_t reason;    // 0 running/max_iter, 1 strict, 2 tol, 3 needs relocation
  int32_t iter;      // iteration the reason refers to
  int32_t changed;   // labels changed in the current iteration
  int32_t done;      // iterations completed (the convergence step's count)
  int32_t pad[11];
};
static_assert(sizeof(LloydState) == 64, "LloydState is 64 bytes");

// ---------------------------------------------------------------------------------------------
// _average_centers + _center_shift
// ---------------------------------------------------------------------------------------------
// One 64-lane block per cluster. sklearn walks j = 0..k-1: a cluster with weight scales its row
// by fp32(1/w); an empty one copies the row of argmax(weight) (first maximum) as it stands at that
// moment, i.e. averaged when argmax < j. Here the heaviest cluster's block writes every empty row
// (from its raw and its averaged values) before averaging its own, so no block reads a row another
// block is rescaling; empty blocks return at once. Shifts: sqrt(_euclidean_dense_dense).
// check_st (the device loop, r04): the empty-cluster check of step 2i folded in — any empty
// cluster stops the loop at this step (reason 3, what k_lloyd_check_empty recorded one launch
// earlier) and no block writes; the host relocates and resumes without the check.
__global__ __launch_bounds__(64) void k_avg_centers(int k, int dim, float* __restrict__ C_new,
                                                    const float* __restrict__ wsum,
                                                    const float* __restrict__ C_old,
                                                    float* __restrict__ shift, const int32_t* stop,
                                                    int step_i, LloydState* check_st = nullptr,
                                                    int it = 0) {
  if (stopped(stop, step_i)) return;
  const int c = blockIdx.x, lane = threadIdx.x;
  const float wc = wsum[c];
  if (!(wc > 0.f) && !check_st) return;
  float bv = -1.f;
  int bi = INT_MAX, any_empty = 0;
  for (int j = lane; j < k; j += 64) {
    const float v = wsum[j];
    if (v > bv) {
      bv = v;
      bi = j;
    }
    any_empty |= !(v > 0.f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
    any_empty |= __shfl_xor(any_empty, o);
  }
  if (check_st && any_empty) {
    if (c == 0 && lane == 0) {
      check_st->reason = 3;
      check_st->iter = it;
      __hip_atomic_store(&check_st->stop_at, step_i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (!(wc > 0.f)) return;
  const float alpha = (float)(1.0 / (double)wc);  // `1.0 / weight` is a C double division
  const int64_t cb = (int64_t)c * dim;
  const bool donor = any_empty && bi == c;
  if (donor) {
    for (int j = 0; j < k; ++j) {
      if (wsum[j] > 0.f) continue;
      const int64_t jb = (int64_t)j * dim;
      for (int f = lane; f < dim; f += 64) {
        const float raw = C_new[cb + f];
        C_new[jb + f] = c < j ? raw * alpha : raw;
      }
    }
  }
  for (int f = lane; f < dim; f += 64) C_new[cb + f] = C_new[cb + f] * alpha;
  __syncthreads();
  if (lane == 0 && shift) {
    shift[c] = sqrtf(skl_sqdist(C_new + cb, C_old + cb, dim));
    if (donor)
      for (int j = 0; j < k; ++j)
        if (!(wsum[j] > 0.f))
          shift[j] = sqrtf(skl_sqdist(C_new + (int64_t)j * dim, C_old + (int64_t)j * dim, dim));
  }
}

// ---------------------------------------------------------------------------------------------
// the Lloyd loop's control words
// ---------------------------------------------------------------------------------------------

__global__ void k_lloyd_changed(int64_t n, const int32_t* __restrict__ labels,
                                int32_t* __restrict__ old, LloydState* st, int step_i) {
  if (stopped(&st->stop_at, step_i)) return;
  int any = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t a = labels[i];
    if (a != old[i]) {
      any = 1;
      old[i] = a;
    }
  }
  if (__any(any) && (threadIdx.x & 63) == 0) st->changed = 1;
}

__global__ __launch_bounds__(256) void k_lloyd_check_empty(int k, const float* __restrict__ wsum,
                                                           LloydState* st, int it, int step_i) {
  if (stopped(&st->stop_at, step_i)) return;
  __shared__ int s_any;
  if (threadIdx.x == 0) s_any = 0;
  __syncthreads();
  int any = 0;
  for (int j = threadIdx.x; j < k; j += blockDim.x) any |= !(wsum[j] > 0.f);
  if (any) s_any = 1;
  __syncthreads();
  if (threadIdx.x == 0 && s_any) {
    st->reason = 3;
    st->iter = it;
    __hip_atomic_store(&st->stop_at, step_i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// numpy's pairwise sum of LDS values s[0..n), its leaves evaluated by the workgroup (r04): the leaves
// of pw_sum's recursion (blocks of <= 128 values) in visit order, their eight interleaved accumulators
// one per thread, each leaf's tree and tail, then thread 0 adds the leaf values up the same recursion.
// Same operations, same order as pw_sum: the same bits. n <= kShiftLds.
constexpr int kPwLeavesMax = 256;  // leaves hold >= 57 values once n > 128: 8192 / 57 < 256
struct PwLds {
  int off[kPwLeavesMax], len[kPwLeavesMax];
  float acc[kPwLeavesMax * 8];
  float leaf[kPwLeavesMax];
  int nleaves;
};

template <int D>
__device__ void pw_leaves_rec(int off, int n, PwLds& L) {
  if constexpr (D == 0) {
    L.off[L.nleaves] = off;
    L.len[L.nleaves] = n;
    ++L.nleaves;
  } else {
    if (n <= 128) {
      L.off[L.nleaves] = off;
      L.len[L.nleaves] = n;
      ++L.nleaves;
      return;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    pw_leaves_rec<D - 1>(off, n2, L);
    pw_leaves_rec<D - 1>(off + n2, n - n2, L);
  }
}

template <int D>
__device__ float pw_combine(int n, const PwLds& L, int& li) {
  if constexpr (D == 0) {
    return L.leaf[li++];
  } else {
    if (n <= 128) return L.leaf[li++];
    int n2 = n / 2;
    n2 -= n2 % 8;
    const float a = pw_combine<D - 1>(n2, L, li);
    const float b = pw_combine<D - 1>(n - n2, L, li);
    return a + b;
  }
}

__device__ float pw_sum_block(const float* __restrict__ s, int n, PwLds& L) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    L.nleaves = 0;
    pw_leaves_rec<8>(0, n, L);
  }
  __syncthreads();
  const int nl = L.nleaves;
  for (int q = tid; q < nl * 8; q += blockDim.x) {  // leaf q / 8, accumulator q % 8
    const int off = L.off[q >> 3], len = L.len[q >> 3], j = q & 7;
    if (len >= 8) {
      float r = s[off + j];
      for (int i = 8; i < len - (len % 8); i += 8) r = r + s[off + i + j];
      L.acc[q] = r;
    }
  }
  __syncthreads();
  for (int l = tid; l < nl; l += blockDim.x) {
    const int off = L.off[l], len = L.len[l];
    float res;
    int i;
    if (len < 8) {
      res = 0.f;
      i = 0;
    } else {
      const float* r = L.acc + l * 8;
      res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      i = len - (len % 8);
    }
    for (; i < len; ++i) res = res + s[off + i];
    L.leaf[l] = res;
  }
  __syncthreads();
  int li = 0;
  return pw_combine<8>(n, L, li);  // thread 0's value is the one used
}

constexpr int kShiftLds = 8192;
__global__ __launch_bounds__(256) void k_lloyd_converge(int k, const float* __restrict__ shift,
                                                        double tol, LloydState* st, int it,
                                                        int step_i) {
  if (stopped(&st->stop_at, step_i)) return;
  __shared__ float sq[kShiftLds];
  __shared__ PwLds pl;
  const bool in_lds = k <= kShiftLds;
  if (in_lds)
    for (int j = threadIdx.x; j < k; j += blockDim.x) sq[j] = shift[j] * shift[j];
  __syncthreads();
  const int changed = st->changed;  // uniform: read by every thread before any write below
  float tot = 0.f;
  if (changed != 0 && in_lds) tot = pw_sum_block(sq, k, pl);  // every thread takes part
  __syncthreads();
  if (threadIdx.x != 0) return;
  int reason = 0;
  if (changed == 0) {
    reason = 1;  // np.array_equal(labels, labels_old)
  } else {
    if (!in_lds) tot = pw_sum<kPwDepth>([&](int j) { const float v = shift[j]; return v * v; }, 0, k);
    if ((double)tot <= tol) reason = 2;
  }
  st->changed = 0;
  st->done = it + 1;
  if (reason) {
    st->reason = reason;
    st->iter = it;
    __hip_atomic_store(&st->stop_at, step_i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ((X - C[labels])**2).sum(axis=1) in numpy's order: fp32 squares, pairwise per contiguous row
__global__ void k_relocate_distances(int64_t n, int dim, const float* __restrict__ X,
                                     const int32_t* __restrict__ labels, const float* __restrict__ C,
                                     float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* x = X + i * dim;
  const float* cr = C + (int64_t)labels[i] * dim;
  out[i] = pw_sum<kPwDepth>([&](int j) { const float d = x[j] - cr[j]; return d * d; }, 0, dim);
}


// ---------------------------------------------------------------------------------------------
// Bounded E-step (Hamerly's bounds, kept exact). Per row: ub >= ||x - C[label]|| and
// lb <= min over the other centres of ||x - c|| (true Euclidean distances, fp64). sklearn's label
// is the argmin of its computed d~(x, c) = fma(-2, <x,c>_fp32 chain, ||c||^2_fp32), and
// |d~(x, c) - (||x - c||^2 - ||x||^2)| <= E(x) = kappa (||x|| + max ||c||)^2 with
// kappa = (2 dim + 8) 2^-24 (the dot product's gamma_dim, the norm's gamma_dim and the final
// rounding). So when L = max(lb, sep[label] - ub) satisfies L^2 - ub^2 > 2 E(x), every other
// centre's computed distance exceeds the label's strictly and the label stands (sklearn's argmin,
// ties included). Rows failing the test get their full top-2 distance row (the same MFMA chains as
// the unbounded pass) and fresh bounds: ub^2 = d~1 + ||x||^2 + E, lb^2 = d~2 + ||x||^2 - E. Between
// iterations ub grows by the label's centre shift and lb shrinks by the largest shift (both
// rounded up from sklearn's fp32 shifts).
// ---------------------------------------------------------------------------------------------
constexpr double kEps32 = 5.9604644775390625e-08;  // 2^-24

// ||x|| in fp64 (upward margin); a block stages its 64 rows through LDS with coalesced loads
__global__ __launch_bounds__(256) void k_row_norm64(int64_t n, int dim, const float* __restrict__ X,
                                                   double* __restrict__ xn) {
  __shared__ float s_x[64 * 49];  // dim <= 48 (the bounded E-step's shapes)
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int rows = (int)min<int64_t>(64, n - r0);
  const float* src = X + r0 * dim;
  for (int e = threadIdx.x; e < rows * dim; e += blockDim.x) s_x[(e / dim) * (dim + 1) + e % dim] = src[e];
  __syncthreads();
  if ((int)threadIdx.x >= rows) return;
  const float* x = s_x + threadIdx.x * (dim + 1);
  double s = 0.0;
  for (int f = 0; f < dim; ++f) s = __builtin_fma((double)x[f], (double)x[f], s);
  xn[r0 + threadIdx.x] = __builtin_sqrt(s) * (1.0 + 1e-12);
}

// block c < k: sep[c] <= min over c' != c of ||C_c - C_c'||; block k: glob[0] >= max ||C_c||,
// glob[1] >= the largest centre shift (0 without shifts), and the failing-row counter cleared
__global__ __launch_bounds__(256) void k_ham_centres(int k, int dim, const float* __restrict__ C,
                                                     const float* __restrict__ shift, int have_shift,
                                                     double* __restrict__ sep, double* __restrict__ glob,
                                                     int64_t* __restrict__ count,
                                                     const int32_t* stop, int step_i) {
  if (stopped(stop, step_i)) return;
  __shared__ double red[2][256];
  const int c = blockIdx.x, tid = threadIdx.x;
  const double inf = __builtin_inf();
  if (c < k) {
    double m = inf;
    const float* cr = C + (int64_t)c * dim;
    for (int o = tid; o < k; o += blockDim.x) {
      if (o == c) continue;
      const float* orow = C + (int64_t)o * dim;
      double s2 = 0.0;
      for (int f = 0; f < dim; ++f) {
        const double d = (double)cr[f] - (double)orow[f];
        s2 = __builtin_fma(d, d, s2);
      }
      m = fmin(m, s2);
    }
    red[0][tid] = m;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
      if (tid < w) red[0][tid] = fmin(red[0][tid], red[0][tid + w]);
      __syncthreads();
    }
    if (tid == 0) sep[c] = red[0][0] == inf ? inf : __builtin_sqrt(red[0][0]) * (1.0 - 1e-12);
  } else {
    double cm = 0.0, dm = 0.0;
    for (int o = tid; o < k; o += blockDim.x) {
      const float* orow = C + (int64_t)o * dim;
      double s2 = 0.0;
      for (int f = 0; f < dim; ++f) s2 = __builtin_fma((double)orow[f], (double)orow[f], s2);
      cm = fmax(cm, s2);
      if (have_shift) dm = fmax(dm, (double)shift[o]);
    }
    red[0][tid] = cm;
    red[1][tid] = dm;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
      if (tid < w) {
        red[0][tid] = fmax(red[0][tid], red[0][tid + w]);
        red[1][tid] = fmax(red[1][tid], red[1][tid + w]);
      }
      __syncthreads();
    }
    if (tid == 0) {
      glob[0] = __builtin_sqrt(red[0][0]) * (1.0 + 1e-12);
      glob[1] = red[1][0] * (1.0 + (dim + 8) * kEps32) + 1e-18;
      *count = 0;
    }
  }
}

// the test, per row; failing rows are listed in index order inside each block's 4096-row range (one
// counter add per block: a single word takes ~90 adds per us, so one add per 256 rows cost ~0.1 ms)
constexpr int kHamRows = 16;  // rows per thread (strided by 256 inside the block's range)
__global__ __launch_bounds__(256) void k_ham_test(int64_t n, int dim, const int32_t* __restrict__ labels,
                                                  const double* __restrict__ xn, double* __restrict__ ub,
                                                  double* __restrict__ lb, const float* __restrict__ shift,
                                                  const double* __restrict__ sep,
                                                  const double* __restrict__ glob, double kappa,
                                                  int64_t* __restrict__ list, int64_t* __restrict__ count,
                                                  const int32_t* stop, int step_i) {
  if (stopped(stop, step_i)) return;
  __shared__ int s_wc[kHamRows][4];
  __shared__ int64_t s_base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 256 * kHamRows;
  const double sscale = 1.0 + (dim + 8) * kEps32;
  const double cmax = glob[0], dmax = glob[1];
  unsigned long long masks[kHamRows];
#pragma unroll
  for (int q = 0; q < kHamRows; ++q) {
    const int64_t i = r0 + q * 256 + tid;
    bool fail = false;
    if (i < n) {
      const int a = labels[i];
      const double u = ub[i] + ((double)shift[a] * sscale + 1e-18);
      const double l = lb[i] - dmax;
      const double L = fmax(l, sep[a] - u);
      const double xm = xn[i] + cmax;
      const double E = kappa * xm * xm;
      fail = !(L > u * (1.0 + 1e-12) && (L - u) * (L + u) > 2.0 * E);
      ub[i] = u;
      lb[i] = l;
    }
    masks[q] = __ballot(fail);
    if (lane == 0) s_wc[q][wave] = __popcll(masks[q]);
  }
  __syncthreads();
  if (tid == 0) {  // exclusive offsets in row order (q-major, then wave)
    int tot = 0;
    for (int q = 0; q < kHamRows; ++q)
      for (int w = 0; w < 4; ++w) {
        const int c = s_wc[q][w];
        s_wc[q][w] = tot;
        tot += c;
      }
    s_base = tot ? (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(count), (unsigned long long)tot) : 0;
  }
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < kHamRows; ++q)
    if ((masks[q] >> lane) & 1ull)
      list[s_base + s_wc[q][wave] + __popcll(masks[q] & below)] = r0 + q * 256 + tid;
}

// rows p < m (list[p], or p when list is null): label and fresh bounds from the top-2 pass
__global__ __launch_bounds__(256) void k_ham_finalize(const int64_t* __restrict__ count, int64_t n_all,
                                                      const int64_t* __restrict__ list,
                                                      const unsigned long long* __restrict__ keys,
                                                      const float* __restrict__ sec,
                                                      const double* __restrict__ xn,
                                                      const double* __restrict__ glob, double kappa,
                                                      int32_t* __restrict__ labels, double* __restrict__ ub,
                                                      double* __restrict__ lb, const int32_t* stop,
                                                      int step_i) {
  if (stopped(stop, step_i)) return;
  const int64_t m = list ? *count : n_all;
  const double cmax = glob[0];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < m;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = list ? list[p] : p;
    const unsigned long long key = keys[p];
    const unsigned hi = (unsigned)(key >> 32);
    const float d1 = __uint_as_float((hi & 0x80000000u) ? (hi & 0x7fffffffu) : ~hi);  // pack_key inverse
    const float d2 = sec[p];
    const double x = xn[i];
    const double xm = x + cmax;
    const double E = kappa * xm * xm;
    const double xlo = x / (1.0 + 3e-12);
    labels[i] = (int32_t)(unsigned)(key & 0xffffffffull);
    ub[i] = __builtin_sqrt(fmax(0.0, (double)d1 + x * x + E)) * (1.0 + 1e-12);
    lb[i] = __builtin_isinf(d2) ? __builtin_inf()
                                : __builtin_sqrt(fmax(0.0, (double)d2 + xlo * xlo - E)) * (1.0 - 1e-12);
  }
}
}  // namespace
}  // namespace gdd

using namespace gdd;

// ---- grouping and folds (C ABI) ------------------------------------------------------------------
extern "C" size_t gdd_group_ws_bytes(int64_t n, int k) { return group_ws(std::max<int64_t>(n, 1), std::max(k, 1)); }

extern "C" int gdd_group_by_label(int64_t n, const int32_t* labels, int k, int32_t* perm,
                                  int32_t* offsets, void* ws, size_t ws_bytes,
                                  gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && k > 0 && labels && perm && offsets && ws, "group_by_label: bad arguments");
  if (ws_bytes < group_ws(n, k)) return fail(GDD_E_WORKSPACE, "group_by_label: workspace too small");
  return group_dev(n, labels, k, perm, offsets, ws, ws_bytes, nullptr, 0, to_hip(stream));
}

extern "C" int gdd_segment_sum_f32(int64_t n, int dim, const float* X, const float* w,
                                   const int32_t* perm, const int32_t* offsets, int k, float* sums,
                                   float* wsum, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && k > 0 && X && perm && offsets && sums && wsum,
              "segment_sum_f32: bad arguments");
  FoldArgs a{dim, 0, 0, 0, 0, 0, 0, 0, X, w, perm, offsets, sums, wsum, nullptr, 0, nullptr, 0, 0, n / k};
  return fold_launch(a, k, false, to_hip(stream));
}

extern "C" int gdd_segment_sum_f32_part(int64_t n, int dim, const float* X, const float* w,
                                        const int32_t* perm, const int32_t* offsets, int k, int c0,
                                        int c1, float* sums_part, float* wsum_part,
                                        gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && k > 0 && 0 <= c0 && c0 <= c1 && c1 <= k && X && perm && offsets &&
                  (c0 == c1 || (sums_part && wsum_part)),
              "segment_sum_f32_part: bad arguments");
  FoldArgs a{dim, 0, 0, 0, 0, 0, 0, c0, X, w, perm, offsets, sums_part, wsum_part, nullptr, 0, nullptr, 0, 0, n / k};
  return fold_launch(a, c1 - c0, false, to_hip(stream));
}

extern "C" int gdd_cluster_mean(int64_t n, int d, const float* feat, const int32_t* perm,
                                const int32_t* offsets, int k, int empty_as_zero, float* feat_syn,
                                long long* counts, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && d > 0 && k > 0 && feat && perm && offsets && feat_syn,
              "cluster_mean: bad arguments");
  FoldArgs a{d, 0, 0, 0, 0, 0, 0, 0, feat, nullptr, perm, offsets, feat_syn, nullptr, counts, empty_as_zero, nullptr, 0};
  return fold_launch(a, k, true, to_hip(stream));
}

extern "C" int gdd_cluster_mean_part(int64_t n, int d, const float* feat, const int32_t* perm,
                                     const int32_t* offsets, int k, int c0, int c1, int empty_as_zero,
                                     float* feat_part, long long* counts_part, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && d > 0 && k > 0 && 0 <= c0 && c0 <= c1 && c1 <= k && feat && perm && offsets &&
                  (c0 == c1 || feat_part),
              "cluster_mean_part: bad arguments");
  FoldArgs a{d, 0, 0, 0, 0, 0, 0, c0, feat, nullptr, perm, offsets, feat_part, nullptr, counts_part, empty_as_zero,
             nullptr, 0};
  return fold_launch(a, c1 - c0, true, to_hip(stream));
}

extern "C" int gdd_average_centers(int k, int dim, float* C_new, const float* wsum,
                                   const float* C_old, float* center_shift, gdd_stream_t stream) {
  GDD_REQUIRE(k > 0 && dim > 0 && C_new && wsum && C_old, "average_centers: bad arguments");
  k_avg_centers<<<k, 64, 0, to_hip(stream)>>>(k, dim, C_new, wsum, C_old, center_shift, nullptr, 0);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_relocate_distances(int64_t n, int dim, const float* X, const int32_t* labels,
                                      const float* C, float* out, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && labels && C && out, "relocate_distances: bad arguments");
  k_relocate_distances<<<blocks_of(n), 256, 0, to_hip(stream)>>>(n, dim, X, labels, C, out);
  GDD_LAUNCHED();
  return GDD_OK;
}

// ---- the device-resident Lloyd loop -----------------------------------------------------------------
extern "C" size_t gdd_lloyd_state_bytes(void) { return sizeof(LloydState); }

// the bounded E-step's buffers: ||x|| (fp64), the two bounds (fp64), the failing-row list, second
// distances, a counter, the centre separations and two global bounds
static size_t prune_ws(int64_t n, int k) {
  return 4 * align256(sizeof(double) * (size_t)n) + align256(sizeof(float) * (size_t)n) +
         align256(sizeof(double) * (size_t)k) + 3 * 256;
}

// The M-step's zero-padded copy of X (r05): for dim % 4 != 0 the fold gathers its rows one float at a
// time (a 188-byte row is 16-byte aligned one time in four, and unaligned 16-byte loads measured
// slower, §4); a copy with rows of round4(dim) floats, made once per run, lets it gather 16-byte
// pieces of aligned rows. Each column's chain is unchanged and the pad columns are not written, so the
// sums are the same bits.
static int fold_pad_dim(int64_t n, int dim) {
  return (dim % 4 != 0 && n >= kFoldPadMinRows) ? (dim + 3) & ~3 : 0;
}

static size_t fold_pad_ws(int64_t n, int dim) {
  const int dp = fold_pad_dim(n, dim);
  return dp ? align256(sizeof(float) * (size_t)n * (size_t)dp) + 256 : 0;
}

__global__ void k_pad_rows(int64_t n, int dim, int dp, const float* __restrict__ X, float* __restrict__ Xp) {
  const int q4 = dp / 4;
  const int64_t total = n * q4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q4;
    const int f = (int)(i - r * q4) * 4;
    const float* src = X + r * dim;
    float4 v;
    v.x = f < dim ? src[f] : 0.f;
    v.y = f + 1 < dim ? src[f + 1] : 0.f;
    v.z = f + 2 < dim ? src[f + 2] : 0.f;
    v.w = f + 3 < dim ? src[f + 3] : 0.f;
    reinterpret_cast<float4*>(Xp)[i] = v;
  }
}

// the Lloyd loop's workspace (gdd_kmeans_lloyd_run and the phase entry points below)
struct LloydWs {
  unsigned long long* keys;
  float* cn2;
  int32_t* perm;
  int32_t* offsets;
  size_t gb;
  void* gws;
  double *xn, *ub, *lb;
  int64_t* list;
  float* sec;
  double *sep, *glob;
  int64_t* count;
};

static bool carve_lloyd(void* ws, size_t ws_bytes, int64_t n, int dim, int k, LloydWs* w) {
  Carver cv(ws, ws_bytes);
  w->keys = cv.take<unsigned long long>(n);
  w->cn2 = cv.take<float>(k);
  w->perm = cv.take<int32_t>(n);
  w->offsets = cv.take<int32_t>(k + 1);
  w->gb = group_ws(n, k);
  w->gws = cv.take<char>(w->gb);
  const int64_t pn = lloyd_prune_ok(dim, k) ? n : 0;  // the bounded E-step's per-row buffers
  const int64_t pk = lloyd_prune_ok(dim, k) ? k : 0;
  w->xn = cv.take<double>(pn);
  w->ub = cv.take<double>(pn);
  w->lb = cv.take<double>(pn);
  w->list = cv.take<int64_t>(pn);
  w->sec = cv.take<float>(pn);
  w->sep = cv.take<double>(pk);
  w->glob = cv.take<double>(2);
  w->count = cv.take<int64_t>(1);
  return cv.ok();
}

extern "C" size_t gdd_kmeans_lloyd_ws_bytes(int64_t n, int dim, int k) {
  // the bounded E-step's buffers (~36 B per row) only where it can run
  return align256(sizeof(unsigned long long) * (size_t)n) + align256(sizeof(float) * (size_t)k) +
         align256(sizeof(int32_t) * (size_t)n) + align256(sizeof(int32_t) * (size_t)(k + 1)) +
         group_ws(n, k) + (lloyd_prune_ok(dim, k) ? prune_ws(n, k) : 3 * 256) + 1024 + fold_pad_ws(n, dim);
}

extern "C" size_t gdd_kmeans_lloyd_host_ws_bytes(void) { return 4 * sizeof(LloydState); }

extern "C" int gdd_kmeans_lloyd_run(int64_t n, int dim, const float* X, int k, float* C0, float* C1,
                                    int32_t* labels, int32_t* labels_old, float* wsum, float* shift,
                                    int it0, int resume, int max_iter, double tol, void* state,
                                    int32_t* out_done, int32_t* out_reason, void* ws, size_t ws_bytes,
                                    void* host_ws, size_t host_ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && dim <= 512 && k > 0 && X && C0 && C1 && labels &&
                  labels_old && wsum && shift && state && out_done && out_reason && ws && host_ws,
              "kmeans_lloyd_run: bad arguments");
  GDD_REQUIRE(it0 >= 0 && it0 <= max_iter && max_iter < (INT_MAX / 2 - 2), "kmeans_lloyd_run: bad iteration range");
  if (ws_bytes < gdd_kmeans_lloyd_ws_bytes(n, dim, k))
    return fail(GDD_E_WORKSPACE, "kmeans_lloyd_run: workspace too small");
  if (host_ws_bytes < gdd_kmeans_lloyd_host_ws_bytes())
    return fail(GDD_E_WORKSPACE, "kmeans_lloyd_run: host workspace too small");
  hipStream_t s = to_hip(stream);
  LloydWs lw;
  if (!carve_lloyd(ws, ws_bytes, n, dim, k, &lw)) return fail(GDD_E_WORKSPACE, "kmeans_lloyd_run: workspace too small");
  auto* keys = lw.keys;
  float* cn2 = lw.cn2;
  int32_t* perm = lw.perm;
  int32_t* offsets = lw.offsets;
  const size_t gb = lw.gb;
  void* gws = lw.gws;
  double* xn = lw.xn;
  double* ub = lw.ub;
  double* lb = lw.lb;
  int64_t* list = lw.list;
  float* sec = lw.sec;
  double* sep = lw.sep;
  double* glob = lw.glob;
  int64_t* count = lw.count;
  // bounded E-steps (GDD_FORCE=lloyd_no_prune: every row every iteration), from the run's first E-step on
  const bool prune = !forced("lloyd_no_prune") && lloyd_prune_ok(dim, k);
  const int prune_first = resume ? it0 + 1 : it0;
  const double kappa = (2.0 * dim + 8.0) * kEps32;
  const unsigned fgrid = std::min<unsigned>(blocks_of(n), 2048);
  if (prune) {
    k_row_norm64<<<blocks_of(n, 64), 256, 0, s>>>(n, dim, X, xn);
    GDD_LAUNCHED();
  }
  LloydState* st = static_cast<LloydState*>(state);
  LloydState* hs = static_cast<LloydState*>(host_ws);
  // a fresh run (or a resume after the host's relocation) starts with the stop word clear; the
  // changed flag is kept on resume (the E-step that set it already ran)
  GDD_HIP(hipMemsetAsync(st, 0, offsetof(LloydState, changed), s));
  if (!resume) GDD_HIP(hipMemsetAsync(&st->changed, 0, sizeof(int32_t), s));
  FoldArgs fa{dim, 0, 0, 0, 0, 0, 0, 0, X, nullptr, perm, offsets, nullptr, wsum, nullptr, 0, &st->stop_at, 0};
  fa.avg_rows = n / k;
  const float* Xpad = nullptr;  // the padded copy for the bounded E-step's row lists (estep_no_pad: X)
  int dpad = 0;
  {  // the fold's zero-padded copy of X at the end of the workspace (fold_no_pad: gather X itself)
    const int dp = fold_pad_dim(n, dim);
    const size_t base = gdd_kmeans_lloyd_ws_bytes(n, dim, k) - fold_pad_ws(n, dim);
    const uintptr_t at = (reinterpret_cast<uintptr_t>(ws) + base + 255) & ~uintptr_t(255);
    if (dp && !forced("fold_no_pad") && ws_bytes >= base + fold_pad_ws(n, dim)) {
      float* Xp = reinterpret_cast<float*>(at);
      const int64_t total = n * (dp / 4);
      k_pad_rows<<<(unsigned)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, s>>>(n, dim, dp, X, Xp);
      GDD_LAUNCHED();
      fa.X = Xp;
      fa.dim = dp;
      fa.out_dim = dim;
      if (!forced("estep_no_pad")) {
        Xpad = Xp;
        dpad = dp;
      }
    }
  }
  {  // M-step: clusters above fold_slice x the mean size (default 1.5; 0: off) fold in slices
    const double f = forced_value("fold_slice", 1.5);
    const double rows = f * (double)n / (double)k;
    fa.big_rows = f > 0.0 ? (int)std::min<double>(std::max(rows, 4096.0), (double)INT_MAX) : 0;
  }
  const unsigned cgrid = std::min<unsigned>(blocks_of(n), 2048);
  auto enqueue = [&](int i, bool phase_a) -> int {
    float* cin = (i & 1) ? C1 : C0;
    float* cout = (i & 1) ? C0 : C1;
    const int sa = 2 * i, sb = 2 * i + 1;
    if (phase_a) {
      int rc;
      if (prune) {
        const bool first = i == prune_first;
        k_ham_centres<<<k + 1, 256, 0, s>>>(k, dim, cin, shift, first ? 0 : 1, sep, glob, count,
                                            &st->stop_at, sa);
        GDD_LAUNCHED();
        if (!first) {
          k_ham_test<<<blocks_of(n, 256 * kHamRows), 256, 0, s>>>(n, dim, labels, xn, ub, lb, shift, sep, glob, kappa,
                                                 list, count, &st->stop_at, sa);
          GDD_LAUNCHED();
          if (getenv("GDD_LLOYD_LISTLEN")) {  // diagnostics: the bounded E-step's row count (synchronises)
            int64_t cnt = 0;
            GDD_HIP(hipMemcpyAsync(&cnt, count, sizeof(cnt), hipMemcpyDeviceToHost, s));
            GDD_HIP(hipStreamSynchronize(s));
            fprintf(stderr, "lloyd iteration %d: %lld of %lld rows listed\n", i, (long long)cnt, (long long)n);
          }
        }
        rc = kmeans_assign_top2_dev(n, dim, X, first ? nullptr : list, first ? nullptr : count, k, cin,
                                    cn2, keys, sec, &st->stop_at, sa, s, Xpad, dpad);
        if (rc) return rc;
        k_ham_finalize<<<fgrid, 256, 0, s>>>(count, n, first ? nullptr : list, keys, sec, xn, glob,
                                             kappa, labels, ub, lb, &st->stop_at, sa);
        GDD_LAUNCHED();
      } else {
        rc = kmeans_assign_dev(n, dim, X, k, cin, cn2, labels, keys, &st->stop_at, sa, s);
        if (rc) return rc;
      }
      rc = group_dev(n, labels, k, perm, offsets, gws, gb, &st->stop_at, sa, s);
      if (rc) return rc;
      fa.out = cout;
      fa.step_i = sa;
      rc = fold_launch(fa, k, false, s);
      if (rc) return rc;
      // the empty-cluster check rides in the average's launch (check_st)
    }
    k_avg_centers<<<k, 64, 0, s>>>(k, dim, cout, wsum, cin, shift, &st->stop_at, sb, phase_a ? st : nullptr, i);
    GDD_LAUNCHED();
    k_lloyd_changed<<<cgrid, 256, 0, s>>>(n, labels, labels_old, st, sb);
    GDD_LAUNCHED();
    k_lloyd_converge<<<1, 256, 0, s>>>(k, shift, tol, st, i, sb);
    GDD_LAUNCHED();
    return GDD_OK;
  };
  // chunks of iterations enqueued ahead of the decision; the host reads the state of chunk c while
  // chunk c+1 runs (two pinned slots, one event each)
  struct EvPair {  // destroyed on every return, including the GDD_HIP early ones below
    hipEvent_t e[2] = {nullptr, nullptr};
    ~EvPair() {
      for (hipEvent_t x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } evs;
  hipEvent_t* ev = evs.e;
  GDD_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
  GDD_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  int rc = GDD_OK;
  int i = it0, chunk = 0, pending = -1, ch = 2;
  bool stop = false;
  int done = it0, reason = 0;
  auto poll = [&](int slot) -> int {
    GDD_HIP(hipEventSynchronize(ev[slot]));
    if (hs[slot].stop_at) {
      stop = true;
      reason = hs[slot].reason;
      done = reason == 3 ? hs[slot].iter : hs[slot].done;
    } else {
      done = hs[slot].done;
    }
    return GDD_OK;
  };
  while (i < max_iter && !stop) {
    const int m = std::min(ch, max_iter - i);
    for (int j = 0; j < m && rc == GDD_OK; ++j, ++i) rc = enqueue(i, !(resume && i == it0));
    if (rc) break;
    const int slot = chunk & 1;
    GDD_HIP(hipMemcpyAsync(&hs[slot], st, sizeof(LloydState), hipMemcpyDeviceToHost, s));
    GDD_HIP(hipEventRecord(ev[slot], s));
    if (pending >= 0) {
      rc = poll(pending);
      if (rc) break;
    }
    pending = slot;
    ++chunk;
    ch = std::min(ch * 2, 8);
  }
  if (rc == GDD_OK && pending >= 0 && !stop) rc = poll(pending);
  if (rc == GDD_OK) {
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) rc = fail((int)e, "kmeans_lloyd_run: %s", hipGetErrorString(e));
  }
  if (rc) return rc;
  if (!stop) done = max_iter;  // ran out of iterations (sklearn's loop end)
  *out_done = done;
  *out_reason = reason;
  return GDD_OK;
}

// ---- one Lloyd iteration in three phases, for a process group (gdd.sharded.ShardedKMeans) --------
// Rank r runs the bounded E-step on its rows and the M-step fold on its columns; the caller
// all-gathers the labels and the column slices of the sums in between (RCCL, stream-ordered), and
// every rank runs the same replicated update. Every kernel is gated by the stop word exactly as in
// gdd_kmeans_lloyd_run (iteration i = steps 2i and 2i+1), so the host enqueues chunks of iterations
// and reads the state once per chunk. Each value comes from the single-GPU kernels on the same
// operands: labels, sums, centres, iteration counts are bit-identical for every world size.
namespace gdd {
namespace {
// C_new[c][f] = the ranks' column slices of the sums side by side: rank r's slot (k * fw floats at
// r * k * fw) holds its k x w_r block row-major, w_r = min(fw, dim - r * fw) columns
__global__ void k_assemble_cols(int k, int dim, int fw, const float* __restrict__ parts,
                                float* __restrict__ C_new, const int32_t* stop, int step_i) {
  if (stopped(stop, step_i)) return;
  const int64_t total = (int64_t)k * dim;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e / dim), f = (int)(e - (int64_t)c * dim);
    const int r = f / fw, w = min(fw, dim - r * fw);
    C_new[e] = parts[(int64_t)r * k * fw + (int64_t)c * w + (f - r * fw)];
  }
}

// unit weights: the weight sums the fold writes (a sequential fp32 count, which sticks at 2^24), for
// a rank that folds no columns
__global__ void k_wsum_offsets(int k, const int32_t* __restrict__ offsets, float* __restrict__ wsum,
                               const int32_t* stop, int step_i) {
  if (stopped(stop, step_i)) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < k) wsum[c] = fminf((float)(offsets[c + 1] - offsets[c]), 16777216.f);
}
}  // namespace
}  // namespace gdd

extern "C" int gdd_lloyd_estep(int64_t n, int64_t r0, int64_t r1, int dim, const float* X, int k,
                               const float* C, const float* shift, int first, int32_t* labels,
                               void* state, int it, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && 0 <= r0 && r0 <= r1 && r1 <= n && dim > 0 && dim <= 512 && k > 0 && X && C &&
                  labels && state && ws && (first || shift) && it >= 0,
              "lloyd_estep: bad arguments");
  hipStream_t s = to_hip(stream);
  LloydWs lw;
  if (!carve_lloyd(ws, ws_bytes, n, dim, k, &lw)) return fail(GDD_E_WORKSPACE, "lloyd_estep: workspace too small");
  LloydState* st = static_cast<LloydState*>(state);
  const int sa = 2 * it;
  const int64_t m = r1 - r0;
  if (m == 0) return GDD_OK;
  const float* Xr = X + r0 * dim;
  const bool prune = !forced("lloyd_no_prune") && lloyd_prune_ok(dim, k);
  if (!prune) return kmeans_assign_dev(m, dim, Xr, k, C, lw.cn2, labels + r0, lw.keys, &st->stop_at, sa, s);
  const double kappa = (2.0 * dim + 8.0) * kEps32;
  if (first) {  // the rows' norms, once per fit (the bounds start at this E-step)
    k_row_norm64<<<blocks_of(m, 64), 256, 0, s>>>(m, dim, Xr, lw.xn + r0);
    GDD_LAUNCHED();
  }
  k_ham_centres<<<k + 1, 256, 0, s>>>(k, dim, C, shift, first ? 0 : 1, lw.sep, lw.glob, lw.count,
                                      &st->stop_at, sa);
  GDD_LAUNCHED();
  if (!first) {
    k_ham_test<<<blocks_of(m, 256 * kHamRows), 256, 0, s>>>(m, dim, labels + r0, lw.xn + r0, lw.ub + r0,
                                                             lw.lb + r0, shift, lw.sep, lw.glob, kappa,
                                                             lw.list, lw.count, &st->stop_at, sa);
    GDD_LAUNCHED();
  }
  int rc = kmeans_assign_top2_dev(m, dim, Xr, first ? nullptr : lw.list, first ? nullptr : lw.count, k, C,
                                  lw.cn2, lw.keys, lw.sec, &st->stop_at, sa, s);
  if (rc) return rc;
  const unsigned fgrid = std::min<unsigned>(blocks_of(m), 2048);
  k_ham_finalize<<<fgrid, 256, 0, s>>>(lw.count, m, first ? nullptr : lw.list, lw.keys, lw.sec, lw.xn + r0,
                                       lw.glob, kappa, labels + r0, lw.ub + r0, lw.lb + r0, &st->stop_at, sa);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_lloyd_mstep(int64_t n, int dim, const float* X, const int32_t* labels, int k, int f0,
                               int f1, float* sums_cols, float* wsum, void* state, int it, void* ws,
                               size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && k > 0 && 0 <= f0 && f0 <= f1 && f1 <= dim && X && labels && wsum &&
                  state && ws && (f0 == f1 || sums_cols) && it >= 0,
              "lloyd_mstep: bad arguments");
  hipStream_t s = to_hip(stream);
  LloydWs lw;
  if (!carve_lloyd(ws, ws_bytes, n, dim, k, &lw)) return fail(GDD_E_WORKSPACE, "lloyd_mstep: workspace too small");
  LloydState* st = static_cast<LloydState*>(state);
  const int sa = 2 * it;
  int rc = group_dev(n, labels, k, lw.perm, lw.offsets, lw.gws, lw.gb, &st->stop_at, sa, s);
  if (rc) return rc;
  if (f1 > f0) {
    FoldArgs fa{f1 - f0, 0, 0, 0, 0, 0, 0, 0, X + f0, nullptr, lw.perm, lw.offsets, sums_cols, wsum,
                nullptr, 0, &st->stop_at, sa, dim, n / k};
    const double fs = forced_value("fold_slice", 1.5);
    const double rows = fs * (double)n / (double)k;
    fa.big_rows = fs > 0.0 ? (int)std::min<double>(std::max(rows, 4096.0), (double)INT_MAX) : 0;
    rc = fold_launch(fa, k, false, s);
    if (rc) return rc;
  } else {
    k_wsum_offsets<<<blocks_of(k), 256, 0, s>>>(k, lw.offsets, wsum, &st->stop_at, sa);
    GDD_LAUNCHED();
  }
  k_lloyd_check_empty<<<1, 256, 0, s>>>(k, wsum, st, it, sa);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_lloyd_update(int64_t n, int dim, int k, const float* parts, int fw, float* C_new,
                                const float* wsum, const float* C_old, float* shift,
                                const int32_t* labels, int32_t* labels_old, double tol, void* state,
                                int it, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && k > 0 && fw > 0 && C_new && wsum && C_old && shift && labels &&
                  labels_old && state && it >= 0,
              "lloyd_update: bad arguments");
  hipStream_t s = to_hip(stream);
  LloydState* st = static_cast<LloydState*>(state);
  const int sb = 2 * it + 1;
  if (parts) {
    const int64_t total = (int64_t)k * dim;
    k_assemble_cols<<<(unsigned)std::min<int64_t>((total + 255) / 256, 2048), 256, 0, s>>>(
        k, dim, fw, parts, C_new, &st->stop_at, sb);
    GDD_LAUNCHED();
  }
  k_avg_centers<<<k, 64, 0, s>>>(k, dim, C_new, wsum, C_old, shift, &st->stop_at, sb);
  GDD_LAUNCHED();
  const unsigned cgrid = std::min<unsigned>(blocks_of(n), 2048);
  k_lloyd_changed<<<cgrid, 256, 0, s>>>(n, labels, labels_old, st, sb);
  GDD_LAUNCHED();
  k_lloyd_converge<<<1, 256, 0, s>>>(k, shift, tol, st, it, sb);
  GDD_LAUNCHED();
  return GDD_OK;
}
