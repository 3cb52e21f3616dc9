// gdd_recsys.hip — the recommender side of ClustGDD:
//   * build_condensed_bipartite (distill_recsys.py:184-201): interactions (u, i) -> super-node pairs
//     (u2cu[u], i2ci[i]) -> a num_cu x num_ci count matrix as canonical CSR (scipy's coo ->
//     sum_duplicates -> tocsr: rows ascending, columns ascending, values = pair counts in fp32);
//   * the per-edge dot products of the LightGCN propagation's backward (RecsysModel.propagate,
//     :322-351: d/d norm_e of index_add_(cu, it[ci] * norm) is <grad_u[cu_e], it[ci_e]>).
// Integer work by stable radix sorts (ci, then cu) and one scan; bit-exact.
#include <algorithm>
#include <climits>

#include "gdd_common.hpp"
#include "gdd_rng.hpp"

namespace gdd {
namespace {

constexpr int kThreads = 256;
unsigned grid1(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

int bits_for(int64_t n) {
  int b = 1;
  while (b < 31 && (int64_t(1) << b) < n) ++b;
  return b;
}

// super-node ids of every interaction; flags an id out of range
__global__ void k_pair_ids(int64_t E, const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                           const int32_t* __restrict__ u2cu, const int32_t* __restrict__ i2ci,
                           int64_t nu, int64_t ni, int num_cu, int num_ci, int32_t* __restrict__ cu,
                           int32_t* __restrict__ ci, int32_t* __restrict__ iota, int32_t* __restrict__ bad) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int32_t a = u[e], b = it[e];
  int32_t x = 0, y = 0;
  if (a >= 0 && a < nu && b >= 0 && b < ni) {
    x = u2cu[a];
    y = i2ci[b];
  } else {
    atomicOr(bad, 1);
  }
  if (x < 0 || x >= num_cu || y < 0 || y >= num_ci) {
    atomicOr(bad, 2);
    x = 0;
    y = 0;
  }
  cu[e] = x;
  ci[e] = y;
  iota[e] = (int32_t)e;
}

__global__ void k_gather_i32(int64_t E, const int32_t* __restrict__ src, const int32_t* __restrict__ idx,
                             int32_t* __restrict__ dst) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < E) dst[p] = src[idx[p]];
}

// run starts of the (cu, ci)-sorted pairs; each run start also counts toward its row
__global__ void k_run_flags(int64_t E, const int32_t* __restrict__ cu_s, const int32_t* __restrict__ ci_s,
                            int32_t* __restrict__ flag, int32_t* __restrict__ rowcnt) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  const bool start = p == 0 || cu_s[p] != cu_s[p - 1] || ci_s[p] != ci_s[p - 1];
  flag[p] = start ? 1 : 0;
  if (start) atomicAdd(rowcnt + cu_s[p], 1);
}

__global__ void k_run_emit(int64_t E, const int32_t* __restrict__ ci_s, const int32_t* __restrict__ flag,
                           const int32_t* __restrict__ seg, int32_t* __restrict__ starts,
                           int32_t* __restrict__ col_out, int32_t* __restrict__ nnz_out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  if (flag[p]) {
    starts[seg[p]] = (int32_t)p;
    col_out[seg[p]] = ci_s[p];
  }
  if (p == E - 1) {
    nnz_out[0] = seg[p] + flag[p];
    starts[seg[p] + flag[p]] = (int32_t)E;
  }
}

__global__ void k_run_counts(const int32_t* __restrict__ nnz, const int32_t* __restrict__ starts,
                             float* __restrict__ val_out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nnz[0]) val_out[s] = (float)(starts[s + 1] - starts[s]);
}

// out[e] = sum_f a[ra[e], f] * b[rb[e], f] (fp32, f ascending), one wave per edge-group of 64.
// Row ids outside [0, na) / [0, nb) are not read: the edge's output is NaN and *bad is set (a stale
// or foreign index buffer becomes a reported error instead of an illegal address).
__global__ __launch_bounds__(256) void k_edge_dots(int64_t E, int d, const int32_t* __restrict__ ra,
                                                   const float* __restrict__ a, int64_t na,
                                                   const int32_t* __restrict__ rb,
                                                   const float* __restrict__ b, int64_t nb,
                                                   float* __restrict__ out, int32_t* __restrict__ bad) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int32_t ia = ra[e], ib = rb[e];
  if (ia < 0 || ia >= na || ib < 0 || ib >= nb) {
    out[e] = __builtin_nanf("");
    if (bad) atomicOr(bad, 1);
    return;
  }
  const float* x = a + (int64_t)ia * d;
  const float* y = b + (int64_t)ib * d;
  float s = 0.f;
  for (int f = 0; f < d; ++f) s = __builtin_fmaf(x[f], y[f], s);
  out[e] = s;
}

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" size_t gdd_bipartite_condense_ws_bytes(int64_t E, int num_cu) {
  return align256(sizeof(int32_t) * (size_t)E) * 8 + align256(sizeof(int32_t) * (size_t)(num_cu + 1)) +
         align256(sizeof(int32_t) * 2) + sort_pairs_ws_bytes(E) + scan_i32_ws_bytes(E > num_cu ? E : num_cu + 1) +
         2048;
}

extern "C" int gdd_bipartite_condense(int64_t E, const int32_t* train_u, const int32_t* train_i,
                                      int64_t num_users, int64_t num_items, const int32_t* u2cu,
                                      const int32_t* i2ci, int num_cu, int num_ci, int32_t* rowptr_out,
                                      int32_t* col_out, float* val_out, int32_t* nnz_out,
                                      int32_t* bad_out, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(E > 0 && E < INT_MAX && num_cu > 0 && num_ci > 0 && num_users > 0 && num_items > 0,
              "bipartite_condense: bad shape");
  GDD_REQUIRE(train_u && train_i && u2cu && i2ci && rowptr_out && col_out && val_out && nnz_out && ws,
              "bipartite_condense: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  int32_t* cu = cv.take<int32_t>(E);
  int32_t* ci = cv.take<int32_t>(E);
  int32_t* iota = cv.take<int32_t>(E + 1);  // edge ids, later the run starts (+ the end)
  int32_t* k1 = cv.take<int32_t>(E);
  int32_t* p1 = cv.take<int32_t>(E);
  int32_t* k2 = cv.take<int32_t>(E);   // cu by (cu, ci)
  int32_t* p2 = cv.take<int32_t>(E);   // edge ids by (cu, ci)
  int32_t* f = cv.take<int32_t>(E);
  int32_t* rowcnt = cv.take<int32_t>(num_cu + 1);
  int32_t* bad = cv.take<int32_t>(2);
  const size_t sb = sort_pairs_ws_bytes(E), cb = scan_i32_ws_bytes(E > num_cu ? E : num_cu + 1);
  char* sort_ws = cv.take<char>(sb);
  char* scan_ws = cv.take<char>(cb);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "bipartite_condense: workspace too small");
  GDD_HIP(hipMemsetAsync(rowcnt, 0, sizeof(int32_t) * (size_t)(num_cu + 1), s));
  GDD_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t) * 2, s));
  k_pair_ids<<<grid1(E), kThreads, 0, s>>>(E, train_u, train_i, u2cu, i2ci, num_users, num_items, num_cu,
                                           num_ci, cu, ci, iota, bad);
  GDD_LAUNCHED();
  // stable LSD: by ci, then by cu
  int rc = sort_pairs_i32(ci, k1, iota, p1, E, bits_for(num_ci), sort_ws, sb, s);
  if (rc) return rc;
  k_gather_i32<<<grid1(E), kThreads, 0, s>>>(E, cu, p1, f);  // f: cu in ci order (scratch)
  GDD_LAUNCHED();
  rc = sort_pairs_i32(f, k2, p1, p2, E, bits_for(num_cu), sort_ws, sb, s);
  if (rc) return rc;
  k_gather_i32<<<grid1(E), kThreads, 0, s>>>(E, ci, p2, k1);  // k1: ci by (cu, ci)
  GDD_LAUNCHED();
  k_run_flags<<<grid1(E), kThreads, 0, s>>>(E, k2, k1, f, rowcnt);
  GDD_LAUNCHED();
  rc = exclusive_scan_i32(f, p1, E, scan_ws, cb, s);  // p1: run index of each run start
  if (rc) return rc;
  k_run_emit<<<grid1(E), kThreads, 0, s>>>(E, k1, f, p1, iota, col_out, nnz_out);  // iota: run starts
  GDD_LAUNCHED();
  k_run_counts<<<grid1(E), kThreads, 0, s>>>(nnz_out, iota, val_out);
  GDD_LAUNCHED();
  rc = exclusive_scan_i32(rowcnt, rowptr_out, num_cu + 1, scan_ws, cb, s);
  if (rc) return rc;
  if (bad_out) GDD_HIP(hipMemcpyAsync(bad_out, bad, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  return GDD_OK;
}

extern "C" int gdd_edge_dots(int64_t E, int d, const int32_t* ra, const float* a, int64_t na,
                             const int32_t* rb, const float* b, int64_t nb, float* out, int32_t* bad,
                             gdd_stream_t stream) {
  GDD_REQUIRE(E >= 0 && d > 0 && na >= 0 && nb >= 0, "edge_dots: bad shape");
  if (E == 0) return GDD_OK;
  GDD_REQUIRE(ra && a && rb && b && out, "edge_dots: null pointer");
  k_edge_dots<<<grid1(E), kThreads, 0, to_hip(stream)>>>(E, d, ra, a, na, rb, b, nb, out, bad);
  GDD_LAUNCHED();
  return GDD_OK;
}

// ---- refinement loop helpers (distill_recsys.py:217-272 sampler, :446-497 Recall@K) -------------
namespace gdd {
namespace {

// Recall@K, pass 1: the training positives of each evaluated user scored -1e9 (:479-483)
__global__ void k_recall_mask(int B, int64_t I, const int32_t* __restrict__ tr_ptr,
                              const int32_t* __restrict__ tr_col, float* __restrict__ scores) {
  const int r = blockIdx.x;
  if (r >= B) return;
  float* row = scores + (int64_t)r * I;
  for (int32_t e = tr_ptr[r] + threadIdx.x; e < tr_ptr[r + 1]; e += blockDim.x) row[tr_col[e]] = -1e9f;
}

__device__ __forceinline__ uint64_t score_key(float v, int64_t j) {
  uint32_t b = __float_as_uint(v);
  b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);  // orderable: larger float -> larger key
  return ((uint64_t)b << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)j);  // ties: lower index first
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}

// Recall@K, pass 2: one workgroup per evaluated user. The k largest scores (torch.topk; equal
// scores in ascending item order) by k rounds of a block max over the row restricted to keys below
// the previous pick, then |top-k ∩ test items| by binary search in the user's sorted, de-duplicated
// test row; integer hits summed with one atomic per user (order-free).
constexpr int kRecThreads = 256;
__global__ __launch_bounds__(kRecThreads) void k_recall_topk_hits(
    int B, int64_t I, int k, const float* __restrict__ scores, const int32_t* __restrict__ te_ptr,
    const int32_t* __restrict__ te_col, unsigned long long* __restrict__ hits) {
  __shared__ uint64_t s_w[kRecThreads / 64];
  __shared__ int32_t s_pick[256];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (r >= B) return;
  const float* row = scores + (int64_t)r * I;
  uint64_t prev = ~0ull;
  for (int q = 0; q < k; ++q) {
    uint64_t best = 0;
    for (int64_t j = tid; j < I; j += kRecThreads) {
      const uint64_t key = score_key(row[j], j);
      if (key < prev && key > best) best = key;
    }
    best = wave_max_u64(best);
    if (lane == 0) s_w[wave] = best;
    __syncthreads();
    uint64_t m = s_w[0];
#pragma unroll
    for (int w = 1; w < kRecThreads / 64; ++w) m = s_w[w] > m ? s_w[w] : m;
    if (tid == 0) s_pick[q] = (int32_t)(0xFFFFFFFFu - (uint32_t)(m & 0xFFFFFFFFu));
    prev = m;
    __syncthreads();
  }
  int found = 0;
  if (tid < k) {
    const int32_t item = s_pick[tid];
    int32_t lo = te_ptr[r], hi = te_ptr[r + 1];
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (te_col[mid] < item) lo = mid + 1; else hi = mid;
    }
    found = (lo < te_ptr[r + 1] && te_col[lo] == item) ? 1 : 0;
  }
  const unsigned long long c = __popcll(__ballot(found));
  if (lane == 0 && c) atomicAdd(hits, c);
}

}  // namespace
}  // namespace gdd

// sample_bpr_triplets_from_condensed (distill_recsys.py:217-272) on the host, drawing from the
// caller's numpy RandomState state exactly as the reference's Python loop does: randint(0, U, b)
// first, then per sample the re-draws of users without a usable positive list (up to 50), the
// positive (randint over the list), and the rejection-sampled negative (up to 50 re-draws while it
// is a positive or equals the positive). pos lists = CSR rows (indptr int64, indices int32 in the
// lists' own order: the positive is drawn by position); sorted (nullable: `indices` is sorted per
// row) is the same rows sorted, for the membership test (np.isin).
extern "C" int gdd_bpr_sample(const int64_t* indptr, const int32_t* indices, const int32_t* sorted,
                              int64_t num_users, int64_t num_items, int64_t batch, void* state,
                              int64_t* u_out, int64_t* pos_out, int64_t* neg_out) {
  GDD_REQUIRE(num_users > 0 && num_items > 0 && batch >= 0, "bpr_sample: bad sizes");
  GDD_REQUIRE(indptr && state && (batch == 0 || (u_out && pos_out && neg_out)),
              "bpr_sample: null pointer");
  LegacyRNG rng(static_cast<MTState*>(state));
  auto draw = [&](int64_t hi) {
    int64_t v;
    rng.randint(0, hi, 1, &v);
    return v;
  };
  rng.randint(0, num_users, batch, u_out);
  for (int64_t s = 0; s < batch; ++s) {
    int64_t uu = u_out[s];
    auto size_of = [&](int64_t x) { return indptr[x + 1] - indptr[x]; };
    int64_t sz = size_of(uu);
    for (int tries = 0; tries < 50 && (sz == 0 || sz >= num_items); ++tries) {
      uu = draw(num_users);
      sz = size_of(uu);
    }
    u_out[s] = uu;
    const int32_t* pl = indices + indptr[uu];
    const int32_t* ps = (sorted ? sorted : indices) + indptr[uu];
    if (sz == 0 || sz >= num_items) {  // no valid negative exists: any neg != pos
      const int64_t p = sz == 0 ? draw(num_items) : (int64_t)pl[draw(sz)];
      int64_t q = draw(num_items);
      while (q == p) q = draw(num_items);
      pos_out[s] = p;
      neg_out[s] = q;
      continue;
    }
    const int64_t p = pl[draw(sz)];
    int64_t q = draw(num_items);
    for (int tries = 0; tries < 50 && (std::binary_search(ps, ps + sz, (int32_t)q) || q == p); ++tries)
      q = draw(num_items);
    pos_out[s] = p;
    neg_out[s] = q;
  }
  return GDD_OK;
}

// Recall@K over B evaluated users: scores (B x I fp32, device, overwritten by the masking),
// tr_ptr/tr_col the users' training positives (CSR, B rows), te_ptr/te_col their de-duplicated
// sorted test items; hits (device u64) accumulates |top-k ∩ test| over the users (not zeroed here).
extern "C" int gdd_recall_at_k(int B, int64_t I, int k, float* scores, const int32_t* tr_ptr,
                               const int32_t* tr_col, const int32_t* te_ptr, const int32_t* te_col,
                               unsigned long long* hits, gdd_stream_t stream) {
  GDD_REQUIRE(B >= 0 && I > 0 && I < INT32_MAX && k >= 1 && k <= 256 && k <= I,
              "recall_at_k: B=%d I=%lld k=%d unsupported", B, (long long)I, k);
  if (B == 0) return GDD_OK;
  GDD_REQUIRE(scores && tr_ptr && te_ptr && hits, "recall_at_k: null pointer");
  hipStream_t s = to_hip(stream);
  k_recall_mask<<<B, 256, 0, s>>>(B, I, tr_ptr, tr_col, scores);
  GDD_LAUNCHED();
  k_recall_topk_hits<<<B, kRecThreads, 0, s>>>(B, I, k, scores, te_ptr, te_col, hits);
  GDD_LAUNCHED();
  return GDD_OK;
}
