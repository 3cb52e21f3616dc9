// gdd_subgraph.hip — induced sub-graphs on the device: adj_full[np.ix_(idx, idx)] as canonical CSR
// (utils_graphsaint.py:34-36, the train/val/test graphs of the inductive agent,
// clustgdd_agent_induct.py:38-94). Integer work: a position map, per-row counts of the entries whose
// column survives, one scan, an ordered fill. idx must be strictly increasing (GraphSAINT's role
// lists are), so the renumbered columns stay sorted within every row.
#include <climits>

#include "gdd_common.hpp"

namespace gdd {
namespace {

constexpr int kThreads = 256;

__global__ void k_pos_fill(int64_t n, int32_t* __restrict__ pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) pos[i] = -1;
}

// pos[idx[j]] = j; flags a violation of strict increase
__global__ void k_pos_set(int64_t m, const int32_t* __restrict__ idx, int64_t n, int32_t* __restrict__ pos,
                          int32_t* __restrict__ bad) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int32_t v = idx[j];
  if (v < 0 || v >= n || (j > 0 && idx[j - 1] >= v)) {
    atomicOr(bad, 1);
    return;
  }
  pos[v] = (int32_t)j;
}

// one wave per new row: count the entries whose column is in the subset
__global__ __launch_bounds__(kThreads) void k_sub_count(int64_t n, int64_t m, const int32_t* __restrict__ idx,
                                                        const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ col,
                                                        const int32_t* __restrict__ pos,
                                                        int32_t* __restrict__ cnt) {
  const int64_t j = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (j >= m) return;
  const int32_t r = idx[j];
  if (r < 0 || r >= n) {  // flagged by k_pos_set; never dereference
    if (lane == 0) cnt[j] = 0;
    return;
  }
  const int32_t b = rowptr[r], e = rowptr[r + 1];
  int c = 0;
  for (int32_t p = b + lane; p < e; p += 64) c += pos[col[p]] >= 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if (lane == 0) cnt[j] = c;
}

// one wave per new row: ordered compaction (ballot prefix) of the surviving entries
__global__ __launch_bounds__(kThreads) void k_sub_fill(int64_t n, int64_t m, const int32_t* __restrict__ idx,
                                                       const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col,
                                                       const float* __restrict__ val,
                                                       const int32_t* __restrict__ pos,
                                                       const int32_t* __restrict__ rowptr_out,
                                                       int32_t* __restrict__ col_out,
                                                       float* __restrict__ val_out) {
  const int64_t j = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (j >= m) return;
  const int32_t r = idx[j];
  if (r < 0 || r >= n) return;
  const int32_t b = rowptr[r], e = rowptr[r + 1];
  int32_t o = rowptr_out[j];
  for (int32_t p0 = b; p0 < e; p0 += 64) {
    const int32_t p = p0 + lane;
    const int32_t q = p < e ? pos[col[p]] : -1;
    const uint64_t mask = __ballot(q >= 0);
    const int before = __popcll(mask & ((1ull << lane) - 1ull));
    if (q >= 0) {
      col_out[o + before] = q;
      if (val_out) val_out[o + before] = val ? val[p] : 1.0f;
    }
    o += __popcll(mask);
  }
}

unsigned grid1(int64_t n, int t = kThreads) { return (unsigned)((n + t - 1) / t); }

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" size_t gdd_subgraph_ws_bytes(int64_t n, int64_t m) {
  return align256(sizeof(int32_t) * (size_t)n) + align256(sizeof(int32_t) * (size_t)(m + 1)) +
         align256(sizeof(int32_t)) + scan_i32_ws_bytes(m + 1) + 512;
}

extern "C" int gdd_subgraph_count(int64_t n, const int32_t* rowptr, const int32_t* col, int64_t m,
                                  const int32_t* idx, int32_t* rowptr_out, void* ws, size_t ws_bytes,
                                  gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && m > 0 && m <= n && n < INT_MAX, "subgraph: bad shape");
  GDD_REQUIRE(rowptr && col && idx && rowptr_out && ws, "subgraph: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  int32_t* pos = cv.take<int32_t>(n);
  int32_t* cnt = cv.take<int32_t>(m + 1);
  int32_t* bad = cv.take<int32_t>(1);
  const size_t sb = scan_i32_ws_bytes(m + 1);
  char* scan_ws = cv.take<char>(sb);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "subgraph: workspace too small");
  GDD_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
  GDD_HIP(hipMemsetAsync(cnt + m, 0, sizeof(int32_t), s));
  k_pos_fill<<<grid1(n), kThreads, 0, s>>>(n, pos);
  GDD_LAUNCHED();
  k_pos_set<<<grid1(m), kThreads, 0, s>>>(m, idx, n, pos, bad);
  GDD_LAUNCHED();
  k_sub_count<<<grid1(m * 64), kThreads, 0, s>>>(n, m, idx, rowptr, col, pos, cnt);
  GDD_LAUNCHED();
  return exclusive_scan_i32(cnt, rowptr_out, m + 1, scan_ws, sb, s);
}

extern "C" int gdd_subgraph_fill(int64_t n, const int32_t* rowptr, const int32_t* col, const float* val,
                                 int64_t m, const int32_t* idx, const int32_t* rowptr_out,
                                 int32_t* col_out, float* val_out, int32_t* bad_out, void* ws,
                                 size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && m > 0 && m <= n, "subgraph: bad shape");
  GDD_REQUIRE(rowptr && col && idx && rowptr_out && col_out && ws, "subgraph: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  int32_t* pos = cv.take<int32_t>(n);
  (void)cv.take<int32_t>(m + 1);
  int32_t* bad = cv.take<int32_t>(1);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "subgraph: workspace too small");
  k_sub_fill<<<grid1(m * 64), kThreads, 0, s>>>(n, m, idx, rowptr, col, val, pos, rowptr_out, col_out,
                                                val_out);
  GDD_LAUNCHED();
  if (bad_out) GDD_HIP(hipMemcpyAsync(bad_out, bad, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  return GDD_OK;
}

// ---- CSR transpose: Aᵀ as canonical CSR (the backward of the GCN evaluator's SpMM, models/gcn.py
// :36-51: d(A @ S)/dS = Aᵀ @ grad). Stable radix sort of (column, entry) pairs, so each transposed
// row lists its entries by ascending original row; counts by integer atomics, one scan.
namespace gdd {
namespace {

__global__ void k_entry_rows(int64_t n, const int32_t* __restrict__ rowptr, int32_t* __restrict__ rows,
                             int32_t* __restrict__ iota) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  for (int32_t p = rowptr[r]; p < rowptr[r + 1]; ++p) {
    rows[p] = (int32_t)r;
    iota[p] = p;
  }
}

__global__ void k_col_counts(int64_t nnz, const int32_t* __restrict__ col, int32_t* __restrict__ cnt) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < nnz) atomicAdd(cnt + col[p], 1);
}

__global__ void k_transpose_fill(int64_t nnz, const int32_t* __restrict__ perm,
                                 const int32_t* __restrict__ rows, const float* __restrict__ val,
                                 int32_t* __restrict__ col_t, float* __restrict__ val_t) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nnz) return;
  const int32_t e = perm[p];
  col_t[p] = rows[e];
  if (val_t) val_t[p] = val ? val[e] : 1.0f;
}

int bits_for(int64_t n) {
  int b = 1;
  while (b < 31 && (int64_t(1) << b) < n) ++b;
  return b;
}

}  // namespace
}  // namespace gdd

extern "C" size_t gdd_csr_transpose_ws_bytes(int64_t n, int64_t n_cols, int64_t nnz) {
  const int64_t m = n > n_cols ? n : n_cols;
  return align256(sizeof(int32_t) * (size_t)nnz) * 4 + align256(sizeof(int32_t) * (size_t)(m + 1)) +
         sort_pairs_ws_bytes(nnz) + scan_i32_ws_bytes(m + 1) + 1024;
}

extern "C" int gdd_csr_transpose(int64_t n, int64_t n_cols, int64_t nnz, const int32_t* rowptr,
                                 const int32_t* col, const float* val, int32_t* rowptr_t, int32_t* col_t,
                                 float* val_t, int32_t* perm_out, void* ws, size_t ws_bytes,
                                 gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && n < INT_MAX && n_cols > 0 && n_cols < INT_MAX && nnz >= 0 && nnz < INT_MAX,
              "csr_transpose: bad shape");
  GDD_REQUIRE(rowptr && rowptr_t && ws && (nnz == 0 || (col && col_t)), "csr_transpose: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  int32_t* rows = cv.take<int32_t>(nnz);
  int32_t* iota = cv.take<int32_t>(nnz);
  int32_t* keys = cv.take<int32_t>(nnz);
  int32_t* perm = cv.take<int32_t>(nnz);
  int32_t* cnt = cv.take<int32_t>(n_cols + 1);
  const size_t sb = sort_pairs_ws_bytes(nnz), cb = scan_i32_ws_bytes(n_cols + 1);
  char* sort_ws = cv.take<char>(sb);
  char* scan_ws = cv.take<char>(cb);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "csr_transpose: workspace too small");
  GDD_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (size_t)(n_cols + 1), s));
  if (nnz > 0) {
    k_entry_rows<<<grid1(n), kThreads, 0, s>>>(n, rowptr, rows, iota);
    GDD_LAUNCHED();
    k_col_counts<<<grid1(nnz), kThreads, 0, s>>>(nnz, col, cnt);
    GDD_LAUNCHED();
    int rc = sort_pairs_i32(col, keys, iota, perm, nnz, bits_for(n_cols), sort_ws, sb, s);
    if (rc) return rc;
    k_transpose_fill<<<grid1(nnz), kThreads, 0, s>>>(nnz, perm, rows, val, col_t, val_t);
    GDD_LAUNCHED();
    if (perm_out)
      GDD_HIP(hipMemcpyAsync(perm_out, perm, sizeof(int32_t) * (size_t)nnz, hipMemcpyDeviceToDevice, s));
  }
  return exclusive_scan_i32(cnt, rowptr_t, n_cols + 1, scan_ws, cb, s);
}
