// gdd_fit.hip — native host loop of MiniBatchKMeans.fit (sklearn/cluster/_kmeans.py:2046-2200).
//
// Everything the Python loop in gdd/kmeans.py did per step now runs in C++: the numpy-legacy RNG
// draws (gdd_rng.hpp), chunked H2D of the batch indices through pinned memory, two kernel launches
// per step (gdd_minibatch_step), and the host's O(k) decisions at reassignment steps. The host
// synchronises only at reassignment steps (every ceil(10k/b) steps, and while some count is zero)
// and once at the end. Draw order, reassignment rule, early-stopping and the RNG state left behind
// are sklearn's (one OpenMP thread).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gdd_common.hpp"
#include "gdd_devrng.hpp"
#include "gdd_rng.hpp"

namespace gdd {
namespace {

__global__ void k_gather_rows(int64_t m, int dim, const float* __restrict__ X,
                              const int64_t* __restrict__ idx, float* __restrict__ out) {
  const int64_t total = m * dim;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / dim;
    out[t] = X[idx[r] * dim + (t - r * dim)];
  }
}

// C[dst[j]] = X[rows[src[j]]]  (centers_new[to_reassign] = X_batch[new_centers], :1655-1662)
__global__ void k_reassign_rows(int m, int dim, const float* __restrict__ X,
                                const int64_t* __restrict__ rows, const int64_t* __restrict__ pairs,
                                float* __restrict__ C) {
  const int j = blockIdx.x;
  if (j >= m) return;
  const int64_t dst = pairs[2 * j], src = rows[pairs[2 * j + 1]];
  for (int f = threadIdx.x; f < dim; f += blockDim.x) C[dst * dim + f] = X[src * dim + f];
}

constexpr int kChunkCap = 64;

struct Pinned {
  void* p = nullptr;
};

struct FitWs {
  float* Xi;
  void* kpp_ws;
  size_t kpp_bytes;
  void* step_ws;
  size_t step_bytes;
  void* state;
  float* counts;
  float* C[2];
  int64_t* rows_d;
  int32_t* labels_b;
  int64_t* pairs;
  double* uniforms;
  int64_t* init_idx;
  int64_t* val_idx;
  int32_t* val_labels;
  float* val_sq;
  float* sq;
  float* scalar;
  void* assign_ws;
  size_t assign_bytes;
  DevMT* mtb;  // 4 device MT states: slot s % 4 (s % 3 in the two-launch loop) = after step s's draws
  float* counts2;             // one-launch loop: weight sums after odd steps (counts: even)
};

size_t fit_ws(void* base, size_t cap, int64_t n, int dim, int k, int64_t bs, int64_t isz, int T,
              FitWs* w) {
  Carver cv(base, cap);
  FitWs f;
  f.Xi = cv.take<float>((size_t)isz * dim);
  f.kpp_bytes = gdd_kmeans_plusplus_ws_bytes_k(isz, dim, T, k);
  f.kpp_ws = cv.take<char>(f.kpp_bytes);
  f.step_bytes = gdd_minibatch_step_ws_bytes(bs, k);
  f.step_ws = cv.take<char>(f.step_bytes);
  f.state = cv.take<char>(gdd_minibatch_state_bytes());
  f.counts = cv.take<float>(k);
  f.C[0] = cv.take<float>((size_t)k * dim);
  f.C[1] = cv.take<float>((size_t)k * dim);
  f.rows_d = cv.take<int64_t>((size_t)kChunkCap * bs);
  f.labels_b = cv.take<int32_t>(bs);
  f.pairs = cv.take<int64_t>(2 * (size_t)k);
  f.uniforms = cv.take<double>((size_t)std::max(k - 1, 1) * T);
  f.init_idx = cv.take<int64_t>(isz);
  f.val_idx = cv.take<int64_t>(isz);
  f.val_labels = cv.take<int32_t>(isz);
  f.val_sq = cv.take<float>(isz);
  f.sq = cv.take<float>(n);
  f.scalar = cv.take<float>(4);
  f.assign_bytes = gdd_kmeans_assign_ws_bytes(std::max(n, isz));
  f.assign_ws = cv.take<char>(f.assign_bytes);
  f.mtb = cv.take<DevMT>(4);
  f.counts2 = cv.take<float>(k);
  if (w) *w = f;
  return cv.off + 1024;
}

int local_trials(int k) { return 2 + (int)std::log((double)k); }

// The step loop with every draw and decision on the device (see the dev_loop comment in the fit).
// Per step s: the assignment launch (plus a workgroup finishing step s-1 — its batch inertia and
// convergence test — and, unless s reassigns, a workgroup drawing batch s+1), the update launch,
// and at scheduled reassignment steps the reassignment launch (which then draws batch s+1). Chunks of
// kDevChunk steps are enqueued back to back; the host reads the stop word of chunk c while chunk
// c+1 runs. Smaller chunks leave fewer no-op launches after the stop but give the host a shorter
// runway: 8, 12 and 16 measured equal within the box's noise, 4 slower.
constexpr int kDevChunk = 16;

// Steps [i0, n_steps) on the device. rr_base: the last reassignment step (the next ones every
// rr_period steps from it); norms_valid0: the workspace norms match step i0's centres. Returns the
// convergence stop in *stop_step, or in *handoff_step a step whose reassignment needs the host (more
// than b/2 centres due: np.argsort's branch) — that step's update has run, its tail and reassignment
// have not, and the generator (written back to rng) is after its batch draws.

int device_loop(int64_t n, int dim, const float* X, int k, int64_t bs, int64_t i0, int64_t rr_base,
                bool norms_valid0, int64_t n_steps, int max_no_improvement, float reassignment_ratio,
                MTState* rng, const FitWs& w, int32_t* h_flag /* pinned, >= 64 ints */,
                int64_t* stop_step, int64_t* handoff_step, hipStream_t s) {
  // the host RNG state (after the initialisation draws, or after the host's step i0 - 1) becomes
  // the device slot of step i0 - 1
  static_assert(sizeof(DevMT) == 624 * 4 + 8, "DevMT layout");
  DevMT* h_mt = reinterpret_cast<DevMT*>(h_flag + 64);  // pinned scratch after the flags
  std::memcpy(h_mt->key, rng->key, sizeof(h_mt->key));
  h_mt->pos = rng->pos;
  h_mt->pad = 0;
  GDD_HIP(hipMemcpyAsync(w.mtb + (i0 + 2) % 3, h_mt, sizeof(DevMT), hipMemcpyHostToDevice, s));
  int rc = mb_rng_launch(w.mtb + (i0 + 2) % 3, w.mtb + i0 % 3, n, bs, w.rows_d + (i0 & 1) * bs, s);
  if (rc) return rc;
  const int64_t seg0 = i0;  // the chunk lambda below has a parameter of that name
  rc = mb_loop_begin(bs, k, w.step_ws, w.step_bytes, s);
  if (rc) return rc;
  const bool reassign = reassignment_ratio > 0.f;
  // one chunk in flight before the host waits for the oldest one's stop word (two or three measured
  // equal: each extra chunk only adds a chunk of no-op launches after a stop)
  constexpr int lookahead = 1;
  hipEvent_t ev[4];
  for (int q = 0; q < 4; ++q) GDD_HIP(hipEventCreateWithFlags(&ev[q], hipEventDisableTiming));
  struct EvGuard {
    hipEvent_t* e;
    ~EvGuard() {
      for (int q = 0; q < 4; ++q) (void)hipEventDestroy(e[q]);
    }
  } guard{ev};
  int32_t* stop_word = reinterpret_cast<int32_t*>(static_cast<char*>(w.state) + 16);
  // _random_reassign (:2029-2043): n_since grows by b per step and fires (then resets) at >= 10k,
  // i.e. at steps 0, p, 2p, ... with p = ceil(10k / b)
  const int64_t rr_period = (10 * (int64_t)k + bs - 1) / bs;
  // the launches of steps [i0, i0 + m): every argument follows from the step indices and the fit's
  // buffers, so a chunk is replayed as a recorded graph keyed by them (replay_or_run)
  auto enqueue_chunk = [&](int64_t i0, int64_t m, hipStream_t cs) -> int {
    for (int64_t j = 0; j < m; ++j) {
      const int64_t st = i0 + j;
      const bool do_rr = reassign && st >= rr_base && (st - rr_base) % rr_period == 0;
      const bool has_next = st + 1 < n_steps;
      int64_t* rows_cur = w.rows_d + (st & 1) * bs;
      int64_t* rows_nxt = w.rows_d + ((st + 1) & 1) * bs;
      DevMT* mt_cur = w.mtb + st % 3;
      DevMT* mt_nxt = w.mtb + (st + 1) % 3;
      const RngNext none{nullptr, nullptr, nullptr, 0, 0};
      const RngNext next{mt_cur, mt_nxt, rows_nxt, n, bs};
      float* c_old = w.C[st % 2];
      float* c_new = w.C[(st + 1) % 2];
      // seg0 (the segment's first step), not this chunk's i0: only the segment's first step has no
      // tail (its predecessor's convergence test ran on the host)
      const int flags = GDD_STEP_CONVERGE | ((st > seg0 || norms_valid0) ? GDD_STEP_NORMS_VALID : 0) |
                        ((st == seg0 && seg0 > 0) ? kStepNoTail : 0);
      int rc2 = minibatch_step_dev(bs, dim, X, rows_cur, k, c_old, c_new, w.counts, w.labels_b, (int)st,
                                   n, max_no_improvement, flags, w.state, w.step_ws, w.step_bytes,
                                   has_next ? next : none, cs);  // at reassignment steps: speculative
      if (rc2) return rc2;
      if (do_rr) {
        rc2 = mb_reassign_launch((int)st, bs, dim, k, reassignment_ratio, X, rows_cur, c_new, w.counts,
                                 w.step_ws, w.step_bytes, mt_cur, mt_cur, has_next ? next : none,
                                 w.state, cs);
        if (rc2) return rc2;
      }
      if (!has_next) {  // the last step's inertia and convergence test (otherwise in step st+1)
        rc2 = mb_loop_end(bs, k, (int)st, n, max_no_improvement, w.state, w.step_ws, w.step_bytes, cs);
        if (rc2) return rc2;
      }
    }
    return GDD_OK;
  };
  struct {
    const void* ptr[10];  // every buffer the launches touch
    int64_t n, bs, n_steps, i0, m, dim, k, max_ni, step_bytes, seg0, rr_base;
    float ratio;
    int nv0;
  } key;
  std::memset(&key, 0, sizeof(key));
  const void* ptrs[10] = {X, w.rows_d, w.C[0], w.C[1], w.counts, w.labels_b, w.state, w.step_ws, w.mtb,
                          nullptr};
  std::memcpy(key.ptr, ptrs, sizeof(ptrs));
  key.step_bytes = (int64_t)w.step_bytes;
  key.n = n;
  key.bs = bs;
  key.n_steps = n_steps;
  key.dim = dim;
  key.k = k;
  key.max_ni = max_no_improvement;
  key.ratio = reassignment_ratio;
  key.seg0 = i0;
  key.rr_base = rr_base;
  key.nv0 = norms_valid0 ? 1 : 0;
  int64_t i = i0;
  int64_t chunk = 0;
  *stop_step = -1;
  *handoff_step = -1;
  while (i < n_steps) {
    const int64_t m = std::min<int64_t>(kDevChunk, n_steps - i);
    key.i0 = i;
    key.m = m;
    rc = replay_or_run("minibatch_chunk", &key, sizeof(key), s,
                       [&](hipStream_t cs) { return enqueue_chunk(i, m, cs); });
    if (rc) return rc;
    i += m;
    // this chunk's stop word and no-improvement count (state bytes 16..31), read back while the next
    // chunks run: slot q at h_flag[32 + 4 q]
    const int slot = (int)(chunk & 3);
    int32_t* hs = h_flag + 32 + 4 * slot;
    GDD_HIP(hipMemcpyAsync(hs, stop_word, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    GDD_HIP(hipEventRecord(ev[slot], s));
    if (chunk >= lookahead) {
      const int old = (int)((chunk - lookahead) & 3);
      GDD_HIP(hipEventSynchronize(ev[old]));
      const int32_t* ho = h_flag + 32 + 4 * old;
      if (ho[0]) break;  // the later kernels already enqueued are no-ops
    }
    ++chunk;
  }
  // the whole state word block (stop_at at byte 16, handoff at byte 32)
  GDD_HIP(hipMemcpyAsync(h_flag + 16, w.state, 48, hipMemcpyDeviceToHost, s));
  GDD_HIP(hipStreamSynchronize(s));
  const int32_t stop_at = h_flag[16 + 4], handoff = h_flag[16 + 8];
  if (handoff && handoff == stop_at)
    *handoff_step = handoff - 1;
  else if (stop_at)
    *stop_step = stop_at - 1;
  const int64_t last = *handoff_step >= 0 ? *handoff_step : (*stop_step >= 0 ? *stop_step : n_steps - 1);
  // the caller's RandomState ends where sklearn's does: after the draws of the last step (at a
  // handoff: after that step's batch draws, before its reassignment's)
  GDD_HIP(hipMemcpyAsync(h_mt, w.mtb + last % 3, sizeof(DevMT), hipMemcpyDeviceToHost, s));
  GDD_HIP(hipStreamSynchronize(s));
  std::memcpy(rng->key, h_mt->key, sizeof(h_mt->key));
  rng->pos = h_mt->pos;
  return GDD_OK;
}

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" size_t gdd_minibatch_kmeans_fit_ws_bytes(int64_t n, int dim, int k, int64_t batch_size,
                                                   int64_t init_size) {
  const int64_t bs = std::min<int64_t>(batch_size, n);
  return fit_ws(nullptr, 0, n, dim, k, bs, init_size, local_trials(k), nullptr);
}

// pinned host bytes of one fit: a chunk of batch indices, the k-means++ uniforms, read-backs
size_t fit_host_ws(int k, int64_t bs, int64_t isz, int T) {
  return sizeof(int64_t) * (size_t)kChunkCap * bs + sizeof(double) * (size_t)std::max(k - 1, 1) * T +
         sizeof(int64_t) * 2 * (size_t)isz + sizeof(float) * (size_t)k * 2 + 256 + sizeof(DevMT) +
         sizeof(int64_t) * 2 * (size_t)k;
}

extern "C" size_t gdd_minibatch_kmeans_fit_host_ws_bytes(int64_t n, int k, int64_t batch_size,
                                                         int64_t init_size) {
  const int64_t bs = std::min<int64_t>(batch_size, n);
  return fit_host_ws(k, bs, init_size, local_trials(k));
}

extern "C" int gdd_minibatch_kmeans_fit(
    int64_t n, int dim, const float* X, int k, int64_t batch_size, int max_iter,
    int max_no_improvement, float reassignment_ratio, int64_t init_size, int n_init,
    int compute_labels, void* rng_state, void (*argsort_cb)(const float*, int64_t, int64_t*),
    float* centers_out, int32_t* labels_out, float* inertia_out, int64_t* n_steps_out,
    double* ewa_out, void* ws, size_t ws_bytes, void* host_ws, size_t host_ws_bytes,
    gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && dim <= 512 && k > 0 && k <= n, "mbk_fit: bad shape");
  GDD_REQUIRE(batch_size > 0 && max_iter >= 0 && n_init >= 1 && init_size >= k && init_size <= n,
              "mbk_fit: bad parameters");
  GDD_REQUIRE(X && rng_state && centers_out && n_steps_out && ws, "mbk_fit: null pointer");
  GDD_REQUIRE(!compute_labels || (labels_out && inertia_out), "mbk_fit: labels/inertia needed");
  hipStream_t s = to_hip(stream);
  const int64_t bs = std::min<int64_t>(batch_size, n);
  const int64_t isz = init_size;
  const int T = local_trials(k);
  GDD_REQUIRE(T <= 16, "mbk_fit: k too large for the k-means++ trial count");
  FitWs w;
  if (fit_ws(ws, ws_bytes, n, dim, k, bs, isz, T, &w) > ws_bytes)
    return fail(GDD_E_WORKSPACE, "mbk_fit: workspace too small");
  LegacyRNG rng(static_cast<MTState*>(rng_state));

  // pinned staging (caller-owned): batch indices of one chunk, k-means++ uniforms, small read-backs
  const size_t pin_bytes = fit_host_ws(k, bs, isz, T);
  GDD_REQUIRE(host_ws && host_ws_bytes >= pin_bytes, "mbk_fit: pinned host workspace too small");
  Pinned pin;
  pin.p = host_ws;
  char* pp = static_cast<char*>(pin.p);
  int64_t* h_rows = reinterpret_cast<int64_t*>(pp);
  pp += sizeof(int64_t) * (size_t)kChunkCap * bs;
  double* h_u = reinterpret_cast<double*>(pp);
  pp += sizeof(double) * (size_t)std::max(k - 1, 1) * T;
  int64_t* h_idx = reinterpret_cast<int64_t*>(pp);
  pp += sizeof(int64_t) * 2 * (size_t)isz;
  float* h_counts = reinterpret_cast<float*>(pp);
  pp += sizeof(float) * (size_t)k * 2;
  int32_t* h_flag = reinterpret_cast<int32_t*>(pp);  // 64 ints of flags, then a DevMT
  pp += 256 + sizeof(DevMT);
  int64_t* h_pairs = reinterpret_cast<int64_t*>(pp);

  // ---- validation subset and initialisations (:2128-2163) ----------------------------------------
  rng.randint(0, n, isz, h_idx + isz);  // validation_indices
  GDD_HIP(hipMemcpyAsync(w.val_idx, h_idx + isz, sizeof(int64_t) * isz, hipMemcpyHostToDevice, s));
  float best_inertia = 0.f;
  bool have_best = false;
  for (int init = 0; init < n_init; ++init) {
    const float* Xi = X;
    if (isz < n) {
      rng.randint(0, n, isz, h_idx);
      GDD_HIP(hipMemcpyAsync(w.init_idx, h_idx, sizeof(int64_t) * isz, hipMemcpyHostToDevice, s));
      k_gather_rows<<<(unsigned)std::min<int64_t>((isz * dim + 255) / 256, 4096), 256, 0, s>>>(
          isz, dim, X, w.init_idx, w.Xi);
      GDD_LAUNCHED();
      Xi = w.Xi;
    }
    const int64_t first = rng.choice_uniform_weights(isz);
    for (int c = 0; c < k - 1; ++c)
      for (int t = 0; t < T; ++t) h_u[(size_t)c * T + t] = rng.next_double();
    if (k > 1)
      GDD_HIP(hipMemcpyAsync(w.uniforms, h_u, sizeof(double) * (size_t)(k - 1) * T,
                             hipMemcpyHostToDevice, s));
    float* cand = (n_init > 1 && init > 0) ? w.C[1] : w.C[0];
    int rc = gdd_kmeans_plusplus(isz, dim, Xi, nullptr, k, T, first, w.uniforms, cand, w.init_idx,
                                 w.kpp_ws, w.kpp_bytes, stream);
    if (rc) return rc;
    if (n_init > 1) {  // inertia on the validation set (_labels_inertia_threadpool_limit)
      rc = gdd_row_norms(k, dim, cand, reinterpret_cast<float*>(w.pairs), stream);
      if (rc) return rc;
      rc = gdd_kmeans_assign(isz, dim, X, w.val_idx, k, cand, reinterpret_cast<float*>(w.pairs),
                             w.val_labels, w.val_sq, w.assign_ws, w.assign_bytes, stream);
      if (rc) return rc;
      rc = gdd_inertia(isz, w.val_sq, nullptr, w.scalar, stream);
      if (rc) return rc;
      GDD_HIP(hipMemcpyAsync(h_counts, w.scalar, sizeof(float), hipMemcpyDeviceToHost, s));
      GDD_HIP(hipStreamSynchronize(s));
      const float inertia = h_counts[0];
      if (!have_best || inertia < best_inertia) {
        best_inertia = inertia;
        have_best = true;
        if (cand != w.C[0])
          GDD_HIP(hipMemcpyAsync(w.C[0], cand, sizeof(float) * (size_t)k * dim,
                                 hipMemcpyDeviceToDevice, s));
      }
    }
  }

  // ---- the step loop (:2168-2189) -----------------------------------------------------------------
  GDD_HIP(hipMemsetAsync(w.counts, 0, sizeof(float) * k, s));
  GDD_HIP(hipMemsetAsync(w.state, 0, gdd_minibatch_state_bytes(), s));
  const int64_t n_steps = ((int64_t)max_iter * n) / bs;
  bool any_zero = true;
  bool norms_valid = false;
  int64_t n_since = 0;
  int64_t i = 0, stop_step = -1;
  std::vector<float> W(k);
  std::vector<int64_t> order;
  // _mini_batch_step's reassignment branch (:1640-1667) on the host, numpy float32 semantics, after
  // the step's update (h_counts = its weight sums, read back by the caller): the argsort branch when
  // more than b/2 centres are due, the permutation draws, the row copies, the weight-sum reset
  auto host_reassign = [&](const int64_t* rows, float* c_new) -> int {
    float wmax = h_counts[0];
    for (int c = 1; c < k; ++c) wmax = std::max(wmax, h_counts[c]);
    const float thr = (float)reassignment_ratio * wmax;
    std::vector<char> to(k);
    int64_t cnt = 0;
    for (int c = 0; c < k; ++c) {
      to[c] = h_counts[c] < thr;
      cnt += to[c];
    }
    if ((double)cnt > 0.5 * (double)bs) {
      if (!argsort_cb) return fail(GDD_E_INVALID, "mbk_fit: argsort callback required (k > b/2)");
      order.assign(k, 0);
      argsort_cb(h_counts, k, order.data());  // np.argsort(weight_sums) (quicksort order)
      for (int64_t q = (int64_t)(0.5 * (double)bs); q < k; ++q) to[order[q]] = 0;
      cnt = 0;
      for (int c = 0; c < k; ++c) cnt += to[c];
    }
    if (cnt) {
      std::vector<int64_t> perm = rng.permutation(bs);  // choice(bs, replace=False, size=cnt)
      int64_t q = 0;
      for (int c = 0; c < k; ++c)
        if (to[c]) {
          h_pairs[2 * q] = c;
          h_pairs[2 * q + 1] = perm[q];
          ++q;
        }
      GDD_HIP(hipMemcpyAsync(w.pairs, h_pairs, sizeof(int64_t) * 2 * cnt, hipMemcpyHostToDevice, s));
      k_reassign_rows<<<(unsigned)cnt, 64, 0, s>>>((int)cnt, dim, X, rows, w.pairs, c_new);
      GDD_LAUNCHED();
      norms_valid = false;  // reassigned rows: the next step recomputes the norms
    }
    float mn = 0.f;
    bool first_min = true;
    for (int c = 0; c < k; ++c)
      if (!to[c] && (first_min || h_counts[c] < mn)) {
        mn = h_counts[c];
        first_min = false;
      }
    bool zero = false;
    for (int c = 0; c < k; ++c) {
      if (to[c]) h_counts[c] = mn;
      zero |= h_counts[c] == 0.f;
    }
    any_zero = zero;
    GDD_HIP(hipMemcpyAsync(w.counts, h_counts, sizeof(float) * k, hipMemcpyHostToDevice, s));
    return GDD_OK;
  };
  // Device-resident loop (any k whose reassignment swap table fits the LDS): the batch draws, the
  // scheduled reassignments and the convergence test run on the device with one host round trip
  // per chunk of steps (overlapped with the next chunk). A reassignment leaves no empty cluster
  // unless more than b/2 centres are due (then np.argsort decides which stay), so the reassignment
  // steps are periodic (every ceil(10k/b) steps from the last one) as long as that branch does not
  // fire — always when k <= b/2. When it fires (k > b/2 only), the device stops at that step and
  // hands it to the host (host_reassign); the host then runs steps while some weight sum is zero
  // (sklearn reassigns at every such step) and resumes the device loop once none is.
  const bool dev_ok = n_steps > 0 && getenv("GDD_HOST_LOOP") == nullptr && mb_reassign_ok(bs, k);
  bool use_dev = dev_ok;
  int64_t rr_base = 0;
  while (i < n_steps && stop_step < 0) {
    if (use_dev) {
      int64_t handoff = -1;
      int rc = device_loop(n, dim, X, k, bs, i, rr_base, norms_valid, n_steps, max_no_improvement,
                           reassignment_ratio, static_cast<MTState*>(rng_state), w, h_flag, &stop_step,
                           &handoff, s);
      if (rc) return rc;
      if (handoff < 0) break;  // ran to the end or stopped
      // step `handoff`: its update ran on the device; its convergence test (the tail the next
      // launch would have run) and its reassignment run here, in sklearn's order of effects
      const int64_t h = handoff;
      GDD_HIP(hipMemsetAsync(static_cast<char*>(w.state) + 16, 0, sizeof(int32_t), s));  // stop_at
      GDD_HIP(hipMemsetAsync(static_cast<char*>(w.state) + 32, 0, sizeof(int32_t), s));  // handoff
      rc = mb_loop_end(bs, k, (int)h, n, max_no_improvement, w.state, w.step_ws, w.step_bytes, s);
      if (rc) return rc;
      GDD_HIP(hipMemcpyAsync(h_flag, static_cast<char*>(w.state) + 16, sizeof(int32_t),
                             hipMemcpyDeviceToHost, s));
      GDD_HIP(hipMemcpyAsync(h_counts, w.counts, sizeof(float) * k, hipMemcpyDeviceToHost, s));
      GDD_HIP(hipStreamSynchronize(s));
      const int32_t stop_at = h_flag[0];
      norms_valid = true;  // the device update left ||C_new||^2 behind
      rc = host_reassign(w.rows_d + (h & 1) * bs, w.C[(h + 1) % 2]);
      if (rc) return rc;
      GDD_HIP(hipStreamSynchronize(s));  // the pinned staging's H2D copies are done
      if (stop_at) stop_step = stop_at - 1;  // converged at h (after its reassignment, as sklearn)
      i = h + 1;
      n_since = 0;
      rr_base = h;
      use_dev = !any_zero;
      continue;
    }
    const MTState snapshot = *static_cast<MTState*>(rng_state);
    std::vector<char> chunk_rr;
    while (i + (int64_t)chunk_rr.size() < n_steps && (int)chunk_rr.size() < kChunkCap) {
      rng.randint(0, n, bs, h_rows + chunk_rr.size() * bs);
      n_since += bs;
      const bool rr = any_zero || n_since >= 10 * (int64_t)k;  // _random_reassign (:2029-2043)
      if (rr) n_since = 0;
      chunk_rr.push_back(rr ? 1 : 0);
      if (rr) break;
    }
    const int m = (int)chunk_rr.size();
    // the previous chunk's copy has been consumed (stream order) before we overwrite h_rows: the
    // sync at the end of every chunk guarantees it
    GDD_HIP(hipMemcpyAsync(w.rows_d, h_rows, sizeof(int64_t) * (size_t)m * bs, hipMemcpyHostToDevice,
                           s));
    bool resume_dev = false;
    for (int j = 0; j < m; ++j) {
      const int64_t st = i + j;
      float* c_old = w.C[st % 2];
      float* c_new = w.C[(st + 1) % 2];
      const int64_t* rows = w.rows_d + (size_t)j * bs;
      const int flags = GDD_STEP_CONVERGE | (norms_valid ? GDD_STEP_NORMS_VALID : 0);
      int rc = gdd_minibatch_step(bs, dim, X, rows, k, c_old, c_new, w.counts, w.labels_b, (int)st, n,
                                  max_no_improvement, flags, w.state, w.step_ws, w.step_bytes,
                                  stream);
      if (rc) return rc;
      norms_valid = true;  // the step left ||c_new||^2 behind
      if (chunk_rr[j] && reassignment_ratio > 0.f) {
        GDD_HIP(hipMemcpyAsync(h_flag, static_cast<char*>(w.state) + 16, sizeof(int32_t),
                               hipMemcpyDeviceToHost, s));
        GDD_HIP(hipMemcpyAsync(h_counts, w.counts, sizeof(float) * k, hipMemcpyDeviceToHost, s));
        GDD_HIP(hipStreamSynchronize(s));
        const int32_t stop_at = h_flag[0];
        if (stop_at && stop_at - 1 < st) {  // stopped earlier in this chunk: step st never ran
          stop_step = stop_at - 1;
          break;
        }
        rc = host_reassign(rows, c_new);
        if (rc) return rc;
        if (stop_at) stop_step = stop_at - 1;
        // no weight sum left at zero: the next reassignments are periodic again (device loop)
        if (stop_at == 0 && !any_zero && dev_ok) {
          resume_dev = true;
          rr_base = st;
        }
      }
    }
    if (stop_step < 0) {
      GDD_HIP(hipMemcpyAsync(h_flag, static_cast<char*>(w.state) + 16, sizeof(int32_t),
                             hipMemcpyDeviceToHost, s));
      GDD_HIP(hipStreamSynchronize(s));
      if (h_flag[0]) stop_step = h_flag[0] - 1;
    } else {
      // also after a reassignment step's sync: its H2D copies out of the caller's pinned staging
      // (h_pairs, h_counts) are still queued, and that buffer may be reused once we return
      GDD_HIP(hipStreamSynchronize(s));
    }
    if (stop_step >= 0 && stop_step < i + m - 1) {
      // sklearn drew batch indices only up to the stopping step: rewind the generator
      *static_cast<MTState*>(rng_state) = snapshot;
      for (int64_t q = i; q <= stop_step; ++q) rng.randint(0, n, bs, h_rows);
    }
    i += m;
    use_dev = resume_dev && stop_step < 0;
  }
  const int64_t last = stop_step >= 0 ? stop_step : n_steps - 1;
  *n_steps_out = last + 1;
  const float* C = w.C[(last + 1) % 2];
  GDD_HIP(hipMemcpyAsync(centers_out, C, sizeof(float) * (size_t)k * dim, hipMemcpyDeviceToDevice, s));
  if (compute_labels) {  // final labels pass + inertia (:2191-2197)
    int rc = gdd_row_norms(k, dim, C, reinterpret_cast<float*>(w.pairs), stream);
    if (rc) return rc;
    rc = gdd_kmeans_assign(n, dim, X, nullptr, k, C, reinterpret_cast<float*>(w.pairs), labels_out,
                           w.sq, w.assign_ws, w.assign_bytes, stream);
    if (rc) return rc;
    if (compute_labels == 2) {  // per-sample squared distances for the caller's own inertia fold
      GDD_HIP(hipMemcpyAsync(inertia_out, w.sq, sizeof(float) * (size_t)n, hipMemcpyDeviceToDevice, s));
    } else {
      rc = gdd_inertia(n, w.sq, nullptr, inertia_out, stream);
      if (rc) return rc;
    }
  }
  if (ewa_out) {  // after the labels pass is enqueued, so the device never idles on this read
    GDD_HIP(hipMemcpyAsync(h_counts, w.state, sizeof(double), hipMemcpyDeviceToHost, s));
    GDD_HIP(hipStreamSynchronize(s));
    std::memcpy(ewa_out, h_counts, sizeof(double));
  }
  return GDD_OK;
}

// ---- host RNG exposure for parity tests (numpy legacy RandomState draws) ---------------------------
extern "C" int gdd_rng_randint(void* state, int64_t low, int64_t high, int64_t count, int64_t* out) {
  GDD_REQUIRE(state && out && high > low && count >= 0, "rng_randint: bad arguments");
  LegacyRNG(static_cast<MTState*>(state)).randint(low, high, count, out);
  return GDD_OK;
}

extern "C" int gdd_rng_random_sample(void* state, int64_t count, double* out) {
  GDD_REQUIRE(state && out && count >= 0, "rng_random_sample: bad arguments");
  LegacyRNG r(static_cast<MTState*>(state));
  for (int64_t i = 0; i < count; ++i) out[i] = r.next_double();
  return GDD_OK;
}

extern "C" int gdd_rng_permutation(void* state, int64_t n, int64_t* out) {
  GDD_REQUIRE(state && out && n >= 0, "rng_permutation: bad arguments");
  std::vector<int64_t> p = LegacyRNG(static_cast<MTState*>(state)).permutation(n);
  std::copy(p.begin(), p.end(), out);
  return GDD_OK;
}

extern "C" int gdd_rng_choice_unit_weights(void* state, int64_t n, int64_t* out) {
  GDD_REQUIRE(state && out && n > 0, "rng_choice: bad arguments");
  out[0] = LegacyRNG(static_cast<MTState*>(state)).choice_uniform_weights(n);
  return GDD_OK;
}
