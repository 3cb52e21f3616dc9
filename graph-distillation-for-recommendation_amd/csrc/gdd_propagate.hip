// gdd_propagate.hip — (a3) k-hop feature propagation over a normalised CSR adjacency.
//
// Restates the loop of ClustGDD/clustgdd_agent_transduct.py:59-65 (same loop three times in
// clustgdd_agent_induct.py:72-94):
//     t = 0       : p = X;                    target = fp32(1-alpha) * X
//     t = 1..T-1  : p = (fp32(alpha) * Â) @ p; target = target + fp32(1-alpha) * p
// `alpha*adj_norm` scales the stored values in fp32 (fp32(alpha) * v, rounded) before the SpMM;
// `(1-alpha)` is a Python double rounded to fp32 when it multiplies the fp32 tensor.
//
// Canonical summation order (the reference's cuSPARSE/torch-CPU order is unspecified, so parity
// with it is a tolerance; parity with oracle/ is bit-exact): the stored entries of a row, in CSR
// order, are cut into segments of GDD_PROP_SEG; a segment is an fp32 fma chain from +0; segment
// partials are added left to right.
//
// Work decomposition: one work item per row segment (short rows = one item, hub rows several), a
// group of G lanes per item, each lane owning V consecutive features (float4/float2/float loads
// of the neighbour rows of p), grid.y walking d in chunks of G*V features. Column indices and
// values are read cooperatively (one coalesced load per G entries) and broadcast with shuffles;
// neighbour-row gathers are issued kUnroll at a time ahead of the dependent fma chain. Rows that
// fit one segment write p and update target in the epilogue; split rows write partials that a
// second kernel folds in order.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "gdd_common.hpp"

namespace gdd {
namespace {

constexpr int kSeg = GDD_PROP_SEG;
constexpr int kUnroll = 8;

struct Item {
  int32_t row, begin, end, pslot;  // pslot < 0: the item is the whole row
};

template <int V>
struct VecT;
template <>
struct VecT<4> {
  using T = float4;
};
template <>
struct VecT<2> {
  using T = float2;
};
template <>
struct VecT<1> {
  using T = float;
};

template <int V>
__device__ __forceinline__ void vload(const float* p, float (&r)[V]) {
  if constexpr (V == 4) {
    float4 t = *reinterpret_cast<const float4*>(p);
    r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
  } else if constexpr (V == 2) {
    float2 t = *reinterpret_cast<const float2*>(p);
    r[0] = t.x; r[1] = t.y;
  } else {
    r[0] = *p;
  }
}
// streamed (once-touched) rows: non-temporal, so they do not push the gathered x rows out of the
// caches between their reuses
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
template <int V>
__device__ __forceinline__ void vload_nt(const float* p, float (&r)[V]) {
  if constexpr (V == 4) {
    f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
  } else if constexpr (V == 2) {
    f32x2 t = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(p));
    r[0] = t.x; r[1] = t.y;
  } else {
    r[0] = __builtin_nontemporal_load(p);
  }
}
template <int V>
__device__ __forceinline__ void vstore_nt(float* p, const float (&r)[V]) {
  if constexpr (V == 4) {
    f32x4 t = {r[0], r[1], r[2], r[3]};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
  } else if constexpr (V == 2) {
    f32x2 t = {r[0], r[1]};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x2*>(p));
  } else {
    __builtin_nontemporal_store(r[0], p);
  }
}
template <int V>
__device__ __forceinline__ void vstore(float* p, const float (&r)[V]) {
  if constexpr (V == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
  } else if constexpr (V == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(r[0], r[1]);
  } else {
    *p = r[0];
  }
}

// ---- plan: per-row segment counts -> item offsets / partial offsets -> item records ----------
// `order` (nullable): position i of the work list is row order[i] (rows scheduled longest first,
// see build_plan); counts and offsets are indexed by position
// rowwise (nullable): the locality probe's verdict (non-zero: ignore `order`, rows in row order)
__global__ void k_seg_counts(int64_t n, const int32_t* __restrict__ rowptr,
                             const int32_t* __restrict__ order, const int32_t* __restrict__ rowwise,
                             int32_t* nseg, int32_t* npart) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = (order && !(rowwise && *rowwise)) ? order[i] : i;
  int32_t len = rowptr[r + 1] - rowptr[r];
  int32_t s = len <= kSeg ? 1 : (len + kSeg - 1) / kSeg;
  nseg[i] = s;
  npart[i] = s > 1 ? s : 0;
}

__global__ void k_make_items(int64_t n, const int32_t* __restrict__ rowptr,
                             const int32_t* __restrict__ order, const int32_t* __restrict__ rowwise,
                             const int32_t* __restrict__ nseg, const int32_t* __restrict__ item_off,
                             const int32_t* __restrict__ part_off, Item* items,
                             int32_t* long_rows, int32_t* long_off, int32_t* counts) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t r = (order && !(rowwise && *rowwise)) ? order[i] : (int32_t)i;
  const int32_t b = rowptr[r], e = rowptr[r + 1], s = nseg[i], o = item_off[i];
  if (s == 1) {
    items[o] = Item{r, b, e, -1};
  } else {
    const int32_t po = part_off[i];
    for (int32_t k = 0; k < s; ++k) {
      int32_t lo = b + k * kSeg, hi = min(e, lo + kSeg);
      items[o + k] = Item{r, lo, hi, po + k};
    }
    // list of split rows for the fixup pass; list order is irrelevant (each entry is independent)
    int32_t q = atomicAdd(&counts[1], 1);
    long_rows[q] = r;
    long_off[q] = po;
  }
  if (i == n - 1) counts[0] = o + s;  // number of items
}

// the locality probe (r06): kProbeRows rows sampled at a fixed stride, up to kProbeCap entries each;
// if at least half of the sampled entries point within kProbeWindow rows of their own row, the graph's
// ids carry locality (neighbours in nearby rows: a row range's gathers share lines in one L2) and
// the hop walks the rows in order instead of longest first. One workgroup; *flag = 1 or 0.
constexpr int kProbeRows = 4096;
constexpr int kProbeCap = 64;
constexpr int kProbeWindow = 4096;
constexpr int64_t kProbeMinRows = 1000000;  // below: the longest-first schedule always (measured)
__global__ __launch_bounds__(1024) void k_locality_probe(int64_t n, const int32_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ col,
                                                         int32_t* __restrict__ flag) {
  __shared__ unsigned long long tot[2];
  if (threadIdx.x < 2) tot[threadIdx.x] = 0;
  __syncthreads();
  unsigned near = 0, all = 0;
  const int64_t stride = n / kProbeRows;
  for (int q = threadIdx.x; q < kProbeRows; q += blockDim.x) {
    const int64_t r = q * stride;
    const int32_t b = rowptr[r], e = min(rowptr[r + 1], b + kProbeCap);
    for (int32_t p = b; p < e; ++p) {
      const int64_t dlt = (int64_t)col[p] - r;
      near += (dlt <= kProbeWindow && dlt >= -kProbeWindow) ? 1u : 0u;
    }
    all += (unsigned)(e - b);
  }
  atomicAdd(&tot[0], (unsigned long long)near);
  atomicAdd(&tot[1], (unsigned long long)all);
  __syncthreads();
  if (threadIdx.x == 0) flag[0] = (tot[1] > 0 && 2 * tot[0] >= tot[1]) ? 1 : 0;
}

// sort keys for the longest-first schedule: ascending key = descending row length, rows of
// kLenKeyMax+ entries all first; ties keep row order (the radix sort is stable)
constexpr int kLenKeyBits = 10;
constexpr int32_t kLenKeyMax = (1 << kLenKeyBits) - 1;
__global__ void k_len_keys(int64_t n, const int32_t* __restrict__ rowptr, int32_t* keys,
                           int32_t* rows) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = kLenKeyMax - min(rowptr[i + 1] - rowptr[i], kLenKeyMax);
  rows[i] = (int32_t)i;
}

// ---- one hop -----------------------------------------------------------------------------------
// XCD-aware slicing (S > 0): the grid is 1-D and consecutive blocks land on consecutive XCDs, so
// block b runs on XCD b % 8. That XCD always gets feature slice (b % 8) % S of the rows, i.e. its L2
// only ever caches 1/S of every gathered row, and the 8/S XCDs sharing a slice split the items.
// S = 0: grid (items, d chunks), no XCD mapping.
template <int V, int G, int S>
__global__ __launch_bounds__(256) void k_hop(const Item* __restrict__ items,
                                             const int32_t* __restrict__ counts,
                                             const int32_t* __restrict__ col,
                                             const float* __restrict__ val, float scale, int d,
                                             const float* __restrict__ x, float* __restrict__ y,
                                             float* __restrict__ acc_out, float acc_scale,
                                             const float* __restrict__ acc_init,
                                             const float* __restrict__ acc_prev,
                                             float* __restrict__ partials,
                                             const int32_t* __restrict__ ymap,
                                             const int32_t* __restrict__ pmap, int contig) {
  const int lane = threadIdx.x & (G - 1);
  int64_t ib;  // item block
  int chunk;   // feature chunk of G*V
  if constexpr (S > 0) {
    const int xcd = blockIdx.x & 7;
    chunk = xcd % S;
    // contig (S = 1): XCD x walks the x-th eighth of the work list, so a row range's gathered rows
    // stay in one L2 (GDD_FORCE=hop_xcd_contig, the locality A/B)
    ib = contig ? (int64_t)xcd * (gridDim.x >> 3) + (blockIdx.x >> 3)
                : (int64_t)(blockIdx.x >> 3) * (8 / S) + xcd / S;
  } else {
    chunk = blockIdx.y;
    ib = blockIdx.x;
  }
  const int64_t g = (ib * blockDim.x + threadIdx.x) / G;
  if (g >= counts[0]) return;
  const Item it = items[g];
  const int f = (chunk * G + lane) * V;
  const bool fa = f < d;
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;

  for (int32_t c0 = it.begin; c0 < it.end; c0 += G) {
    const int32_t p = c0 + lane;
    const bool in = p < it.end;
    const int32_t cj = in ? __builtin_nontemporal_load(col + p) : 0;
    const float vj = in ? scale * __builtin_nontemporal_load(val + p) : 0.f;  // fp32(alpha)*v (agent :64)
    const int cnt = min(G, it.end - c0);
    for (int t = 0; t < cnt; t += kUnroll) {
      float xv[kUnroll][V];
      float vv[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int src = t + u;
        const int32_t jj = __shfl(cj, src < G ? src : 0, G);
        vv[u] = __shfl(vj, src < G ? src : 0, G);
        if (src < cnt && fa) {
          vload<V>(x + (int64_t)jj * d + f, xv[u]);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) xv[u][v] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (t + u < cnt) {
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = __builtin_fmaf(vv[u], xv[u][v], acc[v]);
        }
      }
    }
  }
  if (!fa) return;
  if (it.pslot < 0) {
    // relabelled layout (gdd_propagate_relabeled): y's row of node `row` is ymap[row] (nullptr: the
    // node's own id), acc_prev's is pmap[row]; target and acc_init keep the original ids
    const int64_t o = (int64_t)it.row * d + f;
    const int64_t oy = ymap ? (int64_t)ymap[it.row] * d + f : o;
    vstore<V>(y + oy, acc);  // gathered by the next hop: default policy
    if (acc_out) {
      float t[V];
      if (acc_init) {  // first hop: the initial target fp32(1-alpha) * X (agent :59), one rounding
        vload_nt<V>(acc_init + o, t);
#pragma unroll
        for (int v = 0; v < V; ++v) t[v] = acc_scale * t[v];
      } else {
        vload_nt<V>(acc_out + o, t);
      }
      if (acc_prev) {  // the previous hop's deferred term: its output row (this hop's input x)
        float q[V];
        vload<V>(acc_prev + (pmap ? (int64_t)pmap[it.row] * d + f : o), q);
#pragma unroll
        for (int v = 0; v < V; ++v) t[v] = t[v] + acc_scale * q[v];
      }
#pragma unroll
      for (int v = 0; v < V; ++v) t[v] = t[v] + acc_scale * acc[v];  // two roundings (agent :65)
      vstore_nt<V>(acc_out + o, t);
    }
  } else {
    vstore<V>(partials + (int64_t)it.pslot * d + f, acc);
  }
}

// fold the partials of split rows left to right, then the same epilogue. A bounded grid walks the
// split rows (their count is only known on the device; launching one block per possible split row,
// nnz/256 + 1, dispatched ~10k mostly idle blocks at the arxiv shape for 430 split rows); partials
// are requested eight at a time ahead of the ordered adds.
constexpr int kFixupBlocks = 1024;
__global__ void k_fixup(const int32_t* __restrict__ counts, const int32_t* __restrict__ long_rows,
                        const int32_t* __restrict__ long_off, const int32_t* __restrict__ rowptr,
                        int d, const float* __restrict__ partials, float* __restrict__ y,
                        float* __restrict__ acc_out, float acc_scale,
                        const float* __restrict__ acc_init, const float* __restrict__ acc_prev,
                        const int32_t* __restrict__ ymap, const int32_t* __restrict__ pmap) {
  const int nl = counts[1];
  for (int r = blockIdx.x; r < nl; r += gridDim.x) {
    const int32_t row = long_rows[r], po = long_off[r];
    const int32_t len = rowptr[row + 1] - rowptr[row];
    const int32_t s = (len + kSeg - 1) / kSeg;
    for (int f = threadIdx.x; f < d; f += blockDim.x) {
      const float* pp = partials + (int64_t)po * d + f;
      float sum = pp[0];
      int32_t k = 1;
      for (; k + 8 <= s; k += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = pp[(int64_t)(k + u) * d];
#pragma unroll
        for (int u = 0; u < 8; ++u) sum = sum + v[u];
      }
      for (; k < s; ++k) sum = sum + pp[(int64_t)k * d];
      const int64_t o = (int64_t)row * d + f;
      y[ymap ? (int64_t)ymap[row] * d + f : o] = sum;
      if (acc_out) {
        float t = acc_init ? acc_scale * acc_init[o] : acc_out[o];
        if (acc_prev) t = t + acc_scale * acc_prev[pmap ? (int64_t)pmap[row] * d + f : o];
        acc_out[o] = t + acc_scale * sum;
      }
    }
  }
}

__global__ void k_scale_copy(int64_t total, const float* __restrict__ x, float w,
                             float* __restrict__ target, float* __restrict__ copy) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    float v = x[i];
    target[i] = w * v;
    if (copy) copy[i] = v;
  }
}

// ---- dispatch ----------------------------------------------------------------------------------
struct Plan {
  Item* items;
  int32_t* counts;  // [0] items, [1] long rows
  int32_t* long_rows;
  int32_t* long_off;
  float* partials;
  int64_t max_items;
  int64_t max_long;
  void* sort_ws;
  size_t sort_bytes;
};

// work-list schedule: longest rows first (r04; row order measured slower). Items are independent (each writes its own row or partial slot), so the schedule changes only
// timing, never a result. Longest first: the long items of a power-law graph start early instead of
// trailing the grid (arxiv shape 220 -> 204 us per hop, products 9.7 -> 9.5 ms).

inline int64_t max_items_for(int64_t n, int64_t nnz) { return n + nnz / kSeg + 1; }
inline int64_t max_parts_for(int64_t nnz) { return 2 * (nnz / kSeg) + 2; }

// the schedule's stable counting sort over the length keys (gdd_group_by_label: per-wave LDS
// histograms, one scan, ranked placement; ~2.5x faster here than a radix sort of the pairs)
constexpr int kLenKeys = kLenKeyMax + 1;
size_t sched_ws_bytes(int64_t n) {
  return align256(sizeof(int32_t) * (kLenKeys + 1)) + align256(gdd_group_ws_bytes(n, kLenKeys));
}

size_t plan_ws_bytes(int64_t n, int64_t nnz, int d) {
  size_t b = 0;
  b += align256(sizeof(int32_t) * n) * 7;  // nseg, npart, item_off, part_off, sort keys/rows x3
  b += sched_ws_bytes(n);
  b += align256(sizeof(Item) * max_items_for(n, nnz));   // items
  b += align256(sizeof(int32_t) * 4);                    // counts
  b += align256(sizeof(int32_t) * (nnz / kSeg + 1)) * 2; // long rows
  b += align256(sizeof(float) * max_parts_for(nnz) * (size_t)d);
  b += scan_i32_ws_bytes(n) + 256;
  return b + 4096;
}

// carve the plan's buffers (same layout for build_plan and a later planned hop)
int carve_plan(int64_t n, int64_t nnz, int d, Carver& cv, Plan& pl, int32_t** tmp, void** scan_ws,
               size_t* scan_bytes) {
  for (int q = 0; q < 7; ++q) tmp[q] = cv.take<int32_t>(n);
  pl.max_items = max_items_for(n, nnz);
  pl.max_long = nnz / kSeg + 1;
  pl.items = cv.take<Item>(pl.max_items);
  pl.counts = cv.take<int32_t>(4);
  pl.long_rows = cv.take<int32_t>(pl.max_long);
  pl.long_off = cv.take<int32_t>(pl.max_long);
  pl.partials = cv.take<float>(max_parts_for(nnz) * (size_t)d);
  *scan_bytes = scan_i32_ws_bytes(n);
  *scan_ws = cv.take<char>(*scan_bytes);
  pl.sort_bytes = sched_ws_bytes(n);
  pl.sort_ws = cv.take<char>(pl.sort_bytes);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "propagate: workspace too small");
  return GDD_OK;
}

// given_order (nullable): the work list's row order, taken as is (the relabelled hops: rows in their
// new order, so that consecutive items gather neighbouring rows); null: longest rows first
int build_plan(int64_t n, int64_t nnz, int d, const int32_t* rowptr, const int32_t* col_for_probe,
               Carver& cv, Plan& pl, hipStream_t s, const int32_t* given_order = nullptr) {
  int32_t* tmp[7];
  void* scan_ws;
  size_t sb;
  int rc0 = carve_plan(n, nnz, d, cv, pl, tmp, &scan_ws, &sb);
  if (rc0) return rc0;
  int32_t *nseg = tmp[0], *npart = tmp[1], *item_off = tmp[2], *part_off = tmp[3];
  const unsigned gb = (unsigned)((n + 255) / 256);
  GDD_HIP(hipMemsetAsync(pl.counts, 0, sizeof(int32_t) * 4, s));
  const int32_t* order = given_order;
  // the probe's verdict in counts[2] (zeroed above): row order for graphs whose ids carry locality
  // (GDD_FORCE=hop_row_order: row order always; hop_no_probe: longest first always — A/B)
  const int32_t* rowwise = nullptr;
  if (!given_order && col_for_probe && n >= kProbeMinRows && !forced("hop_no_probe") &&
      !forced("hop_row_order")) {
    k_locality_probe<<<1, 1024, 0, s>>>(n, rowptr, col_for_probe, pl.counts + 2);
    GDD_LAUNCHED();
    rowwise = pl.counts + 2;
  }
  if (!given_order && !forced("hop_row_order")) {
    k_len_keys<<<gb, 256, 0, s>>>(n, rowptr, tmp[4], tmp[5]);
    GDD_LAUNCHED();
    // rows grouped by key, stable: the same order as a stable sort of (key, row) pairs
    Carver sc(pl.sort_ws, pl.sort_bytes);
    int32_t* key_off = sc.take<int32_t>(kLenKeys + 1);
    const size_t gws = gdd_group_ws_bytes(n, kLenKeys);
    void* gw = sc.take<char>(gws);
    if (!sc.ok()) return fail(GDD_E_WORKSPACE, "propagate: schedule workspace too small");
    int rc = gdd_group_by_label(n, tmp[4], kLenKeys, tmp[6], key_off, gw, gws,
                                reinterpret_cast<gdd_stream_t>(s));
    if (rc) return rc;
    order = tmp[6];
  }
  k_seg_counts<<<gb, 256, 0, s>>>(n, rowptr, order, rowwise, nseg, npart);
  GDD_LAUNCHED();
  int rc = exclusive_scan_i32(nseg, item_off, n, scan_ws, sb, s);
  if (rc) return rc;
  rc = exclusive_scan_i32(npart, part_off, n, scan_ws, sb, s);
  if (rc) return rc;
  k_make_items<<<gb, 256, 0, s>>>(n, rowptr, order, rowwise, nseg, item_off, part_off, pl.items,
                                  pl.long_rows, pl.long_off, pl.counts);
  GDD_LAUNCHED();
  return GDD_OK;
}

struct RowMaps {  // relabelled layouts (nullptr: original ids)
  const int32_t* y;
  const int32_t* prev;
};

template <int V, int G>
void launch_hop_vg(const Plan& pl, const int32_t* col, const float* val, float scale, int d,
                   const float* x, float* y, float* acc, float acc_scale, const float* acc_init,
                   const float* acc_prev, RowMaps rm, hipStream_t s) {
  constexpr int kGroups = 256 / G;
  const int64_t iblocks = (pl.max_items + kGroups - 1) / kGroups;
  const int chunks = (d + G * V - 1) / (G * V);
  auto xcd_launch = [&](auto S_) {
    constexpr int S = decltype(S_)::value;
    const int64_t groups = (iblocks + (8 / S) - 1) / (8 / S);
    k_hop<V, G, S><<<(unsigned)(groups * 8), 256, 0, s>>>(pl.items, pl.counts, col, val, scale, d,
                                                          x, y, acc, acc_scale, acc_init, acc_prev,
                                                          pl.partials, rm.y, rm.prev,
                                                          S == 1 && forced("hop_xcd_contig") ? 1 : 0);
  };
  if (chunks == 8)
    xcd_launch(std::integral_constant<int, 8>());
  else if (chunks == 4)
    xcd_launch(std::integral_constant<int, 4>());
  else if (chunks == 2)
    xcd_launch(std::integral_constant<int, 2>());
  else if (chunks == 1)
    xcd_launch(std::integral_constant<int, 1>());
  else
    k_hop<V, G, 0><<<dim3((unsigned)iblocks, (unsigned)chunks), 256, 0, s>>>(
        pl.items, pl.counts, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, pl.partials,
        rm.y, rm.prev, 0);
}

// lanes per item: the whole row up to 64 lanes, or narrower groups that split the row into XCD slices

template <int V>
void launch_hop_v(const Plan& pl, const int32_t* col, const float* val, float scale, int d,
                  const float* x, float* y, float* acc, float acc_scale, const float* acc_init,
                  const float* acc_prev, RowMaps rm, hipStream_t s) {
  const int lanes = (d + V - 1) / V;
  // 29..32 lanes of float4 (d in (112, 128]): two XCD slices of 16 lanes each, so an XCD's L2 caches
  // half of every gathered row (measured at the arxiv shape, d = 128: 202 vs 208 us per hop; the
  // gathers' L2 hit rate rises, the instruction overhead of the narrower groups stays small). With
  // fewer lanes the second slice idles most of its lanes while reading the whole column/value stream
  // again: products' d = 100 (25 lanes) runs 9.5 ms per hop in one 32-lane group vs 12.4 sliced.
  if (lanes <= 16 || (V == 4 && lanes > 28 && lanes <= 32))
    launch_hop_vg<V, 16>(pl, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, rm, s);
  else if (lanes <= 32)
    launch_hop_vg<V, 32>(pl, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, rm, s);
  else
    launch_hop_vg<V, 64>(pl, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, rm, s);
}

// acc_init (nullable): the accumulator's previous value is acc_scale * acc_init instead of acc (the
// first hop folds the initial target = fp32(1-alpha) * X, agent :59, into its epilogue).
// acc_prev (nullable): a term the previous hop deferred, added first: acc = (acc + acc_scale *
// acc_prev) + acc_scale * y — the same two roundings, in the same order, as two separate updates.
int run_hop(const Plan& pl, const int32_t* rowptr, const int32_t* col, const float* val,
            float scale, int d, const float* x, float* y, float* acc, float acc_scale,
            hipStream_t s, const float* acc_init = nullptr, const float* acc_prev = nullptr,
            RowMaps rm = RowMaps{nullptr, nullptr}) {
  // float4 rows need 16-byte aligned row starts: d % 4 == 0 and 16-byte aligned bases
  auto aligned = [](const void* p, int a) { return ((uintptr_t)p % a) == 0; };
  const bool a16 = aligned(x, 16) && aligned(y, 16) && (!acc || aligned(acc, 16)) &&
                   (!acc_init || aligned(acc_init, 16)) && (!acc_prev || aligned(acc_prev, 16)) &&
                   aligned(pl.partials, 16);
  const bool a8 = aligned(x, 8) && aligned(y, 8) && (!acc || aligned(acc, 8)) &&
                  (!acc_init || aligned(acc_init, 8)) && (!acc_prev || aligned(acc_prev, 8));
  if (d % 4 == 0 && a16)
    launch_hop_v<4>(pl, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, rm, s);
  else if (d % 2 == 0 && a8)
    launch_hop_v<2>(pl, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, rm, s);
  else
    launch_hop_v<1>(pl, col, val, scale, d, x, y, acc, acc_scale, acc_init, acc_prev, rm, s);
  GDD_LAUNCHED();
  const unsigned fixup_grid = (unsigned)std::min<int64_t>(pl.max_long, kFixupBlocks);
  k_fixup<<<fixup_grid, 256, 0, s>>>(pl.counts, pl.long_rows, pl.long_off, rowptr, d, pl.partials, y,
                                     acc, acc_scale, acc_init, acc_prev, rm.y, rm.prev);
  GDD_LAUNCHED();
  return GDD_OK;
}

int check_csr_args(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                   const float* val, int d) {
  GDD_REQUIRE(n > 0 && n < INT32_MAX, "propagate: n=%lld out of range", (long long)n);
  GDD_REQUIRE(nnz >= 0 && nnz < INT32_MAX, "propagate: nnz=%lld out of range", (long long)nnz);
  GDD_REQUIRE(d > 0, "propagate: d=%d must be positive", d);
  GDD_REQUIRE(rowptr && (nnz == 0 || (col && val)), "propagate: null CSR pointer");
  return GDD_OK;
}

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" size_t gdd_propagate_ws_bytes(int64_t n, int64_t nnz, int d) {
  return plan_ws_bytes(n, nnz, d);
}

extern "C" int gdd_spmm(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                        const float* val, int d, float scale, const float* x, float* y, float* acc,
                        float acc_scale, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  int rc = check_csr_args(n, nnz, rowptr, col, val, d);
  if (rc) return rc;
  GDD_REQUIRE(x && y && ws, "spmm: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  Plan pl;
  rc = build_plan(n, nnz, d, rowptr, col, cv, pl, s);
  if (rc) return rc;
  return run_hop(pl, rowptr, col, val, scale, d, x, y, acc, acc_scale, s);
}

extern "C" int gdd_spmm_plan(int64_t n, int64_t nnz, const int32_t* rowptr, int d, void* ws,
                             size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && n < INT32_MAX && nnz >= 0 && nnz < INT32_MAX && d > 0 && rowptr && ws,
              "spmm_plan: bad arguments");
  Carver cv(ws, ws_bytes);
  Plan pl;
  // no column ids here: the longest-first schedule (no locality probe)
  return build_plan(n, nnz, d, rowptr, nullptr, cv, pl, to_hip(stream));
}

extern "C" int gdd_spmm_planned(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                                const float* val, int d, float scale, const float* x, float* y,
                                float* acc, float acc_scale, const void* ws, size_t ws_bytes,
                                gdd_stream_t stream) {
  int rc = check_csr_args(n, nnz, rowptr, col, val, d);
  if (rc) return rc;
  GDD_REQUIRE(x && y && ws, "spmm_planned: null pointer");
  Carver cv(const_cast<void*>(ws), ws_bytes);
  Plan pl;
  int32_t* tmp[7];
  void* scan_ws;
  size_t sb;
  rc = carve_plan(n, nnz, d, cv, pl, tmp, &scan_ws, &sb);
  if (rc) return rc;
  return run_hop(pl, rowptr, col, val, scale, d, x, y, acc, acc_scale, to_hip(stream));
}

namespace gdd {
namespace {
__global__ void k_relabel_cols(int64_t nnz, const int32_t* __restrict__ col, const int32_t* __restrict__ rho,
                               int32_t* __restrict__ col_r) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) col_r[e] = rho[col[e]];
}

// the relabelled work order: position rho[r] holds row r
__global__ void k_invert(int64_t n, const int32_t* __restrict__ rho, int32_t* __restrict__ order) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n) order[rho[r]] = (int32_t)r;
}

// gdd_propagate; with rho the intermediate hops run in the relabelled layout (node r's row of p at
// rho[r], gathered through col_r = rho[col]): hop 1 gathers X by the original ids, target keeps the
// original ids throughout, the last hop stores p_last by the original ids
int propagate_impl(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col, const float* val,
                   const int32_t* rho, int d, const float* X, int T, float alpha, float* target,
                   float* p_last, float* p_tmp, void* ws, size_t ws_bytes, hipStream_t s) {
  int rc = 0;
  // the reference's Python doubles, rounded where they meet fp32 tensors
  const float a32 = alpha;
  const float w32 = (float)(1.0 - (double)alpha);
  const int64_t total = n * (int64_t)d;
  const unsigned eb = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
  if (T == 1) {
    k_scale_copy<<<eb, 256, 0, s>>>(total, X, w32, target, p_last);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  Carver cv(ws, ws_bytes);
  Plan pl;
  int32_t* col_r = nullptr;
  int32_t* order = nullptr;
  if (rho) {
    col_r = cv.take<int32_t>((size_t)std::max<int64_t>(nnz, 1));
    order = cv.take<int32_t>((size_t)n);
    if (!cv.ok()) return fail(GDD_E_WORKSPACE, "propagate_relabeled: workspace too small");
    if (nnz > 0) {
      k_relabel_cols<<<(unsigned)((nnz + 255) / 256), 256, 0, s>>>(nnz, col, rho, col_r);
      GDD_LAUNCHED();
    }
    k_invert<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(n, rho, order);
    GDD_LAUNCHED();
  }
  // relabelled: every hop's work list in the new order (GDD_FORCE=hop_relabel_len: longest first)
  rc = build_plan(n, nnz, d, rowptr, col, cv, pl, s, forced("hop_relabel_len") ? nullptr : order);
  if (rc) return rc;
  // ping-pong so that hop T-1 lands in p_last. The target update is paired: after the first hop,
  // hop h (odd) leaves target alone and hop h+1 adds both terms, reading p_h back as its own input
  // rows — one read-modify-write of target per two hops instead of per hop (the streamed bytes that
  // push the gathered rows out of the Infinity Cache), bit-identical (GDD_PROP_PAIR=0: every hop)
  static const bool pair = [] {
    const char* e = getenv("GDD_PROP_PAIR");
    return e == nullptr || atoi(e) != 0;
  }();
  const int hops = T - 1;
  float* bufs[2] = {(hops % 2 == 1) ? p_last : p_tmp, (hops % 2 == 1) ? p_tmp : p_last};
  const float* in = X;
  bool deferred = false;
  for (int h = 0; h < hops; ++h) {
    float* out = bufs[h % 2];
    // relabelled: hops after the first gather through col_r, every hop but the last stores its rows
    // at rho, and a deferred term (the previous hop's output) is read at rho
    const int32_t* cc = (rho && h > 0) ? col_r : col;
    const RowMaps rm{(rho && h + 1 < hops) ? rho : nullptr, (rho && h > 0) ? rho : nullptr};
    if (h == 0) {
      rc = run_hop(pl, rowptr, cc, val, a32, d, in, out, target, w32, s, X, nullptr, rm);
    } else if (deferred) {
      rc = run_hop(pl, rowptr, cc, val, a32, d, in, out, target, w32, s, nullptr, in, rm);
      deferred = false;
    } else if (pair && h + 1 < hops) {
      rc = run_hop(pl, rowptr, cc, val, a32, d, in, out, nullptr, w32, s, nullptr, nullptr, rm);
      deferred = true;
    } else {
      rc = run_hop(pl, rowptr, cc, val, a32, d, in, out, target, w32, s, nullptr, nullptr, rm);
    }
    if (rc) return rc;
    in = out;
  }
  return GDD_OK;
}
}  // namespace
}  // namespace gdd

extern "C" int gdd_propagate(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                             const float* val, int d, const float* X, int T, float alpha,
                             float* target, float* p_last, float* p_tmp, void* ws,
                             size_t ws_bytes, gdd_stream_t stream) {
  int rc = check_csr_args(n, nnz, rowptr, col, val, d);
  if (rc) return rc;
  GDD_REQUIRE(T >= 1, "propagate: T=%d must be >= 1", T);
  GDD_REQUIRE(X && target && p_last && ws && (T <= 2 || p_tmp), "propagate: null pointer");
  return propagate_impl(n, nnz, rowptr, col, val, nullptr, d, X, T, alpha, target, p_last, p_tmp, ws,
                        ws_bytes, to_hip(stream));
}

extern "C" size_t gdd_propagate_relabeled_ws_bytes(int64_t n, int64_t nnz, int d) {
  return plan_ws_bytes(n, nnz, d) + align256(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1)) +
         align256(sizeof(int32_t) * (size_t)n) + 256;
}

extern "C" int gdd_propagate_relabeled(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                                       const float* val, const int32_t* rho, int d, const float* X, int T,
                                       float alpha, float* target, float* p_last, float* p_tmp,
                                       void* ws, size_t ws_bytes, gdd_stream_t stream) {
  int rc = check_csr_args(n, nnz, rowptr, col, val, d);
  if (rc) return rc;
  GDD_REQUIRE(T >= 1, "propagate: T=%d must be >= 1", T);
  GDD_REQUIRE(rho && X && target && p_last && ws && (T <= 2 || p_tmp), "propagate_relabeled: null pointer");
  return propagate_impl(n, nnz, rowptr, col, val, rho, d, X, T, alpha, target, p_last, p_tmp, ws,
                        ws_bytes, to_hip(stream));
}
