// gdd_common.hpp — shared host/device helpers for libgdd (gfx950 only).
//
// Every kernel file is compiled with -ffp-contract=off: fp32/fp64 expressions round exactly as
// written, and every fused multiply-add in the library is an explicit fmaf()/fma(). The reference
// arithmetic being restated (OpenBLAS sgemm = fma chains; Cython loops = separate mul/add) is
// spelled out per kernel in that way, which is what makes the results bit-reproducible.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <string>

#include "gdd.h"

namespace gdd {

// ---------------------------------------------------------------------------------------------
// error reporting (thread-local message, int return codes)
// ---------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define GDD_HIP(expr)                                                                           \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess)                                                                       \
      return ::gdd::fail((int)_e, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),         \
                         __FILE__, __LINE__);                                                   \
  } while (0)

#define GDD_REQUIRE(cond, ...)                                                                  \
  do {                                                                                          \
    if (!(cond)) return ::gdd::fail(GDD_E_INVALID, __VA_ARGS__);                                \
  } while (0)

// launch check: catches bad launch configurations immediately (no host sync)
#define GDD_LAUNCHED() GDD_HIP(hipGetLastError())

inline hipStream_t to_hip(gdd_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------------------------
// workspace carving: 256-byte aligned sub-allocations out of one caller buffer
// ---------------------------------------------------------------------------------------------
struct Carver {
  char* base;
  size_t cap;
  size_t off = 0;
  Carver(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};
// size-only variant used by the *_ws_bytes queries
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ---------------------------------------------------------------------------------------------
// device-wide exclusive scans (hipcub), declared here, defined in gdd_scan.hip
// ---------------------------------------------------------------------------------------------
size_t scan_i32_ws_bytes(int64_t n);
int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes,
                       hipStream_t s);
size_t sort_pairs_ws_bytes(int64_t n);
int sort_pairs_i32(const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                   int32_t* vals_out, int64_t n, int end_bit, void* ws, size_t ws_bytes,
                   hipStream_t s);

// ---------------------------------------------------------------------------------------------
// launch-sequence replay (hipGraph). A fixed sequence of dependent launches — the k-means++ round
// chain, a chunk of MiniBatch steps — is recorded once into a graph and replayed: a graph kernel node
// starts ~1 us sooner after its predecessor than a stream launch does (tools/probe/gap_probe.hip:
// 1.6 vs 2.5-2.8 us per dependent launch). `key` (with `site`) must determine every argument of every
// launch `enqueue` issues (pointers, sizes, step indices), so a replay is the same work as the
// eager sequence. GDD_GRAPH=0 (default) runs every sequence eagerly; 1 records a key on its second
// occurrence; 2 records on the first (parity tests). Measured (r04, tools/micro_graph.py): no gain
// on the real kernels — the host enqueues far ahead of these 5-15 us kernels, so a stream launch's
// gap is already the device's own (MiniBatchKMeans fit 14.05 ms replayed vs 14.00 eager, k-means++
// 4.13 vs 4.20 ms) — and a recording costs a fit's worth of time, so it stays opt-in.
// ---------------------------------------------------------------------------------------------
// resident workgroups of a kernel on the current device (occupancy x CUs; cached)
int occupancy_blocks(const void* fn, int threads, size_t lds, int* out);
// the bf16 full labels pass's r06 kernel (gdd_bf16.hip): n >= 32, dim <= 64 and not a multiple of 16,
// 16-byte aligned X, whole rows; one launch, no workspace (c_norm2 may be null if bf16q_norms_fit)
int bf16q_launch(int64_t n, int dim, const float* X, int k, const float* C, const float* c_norm2,
                 int32_t* labels, float* sq_dist, hipStream_t s);
// whether bf16q_launch can take the centres' norms itself (c_norm2 null) at this dim and k
bool bf16q_norms_fit(int dim, int k);

// GDD_FORCE (tests and diagnostics only): a comma-separated list of tokens, each forcing a path that
// other shapes take by default (so its bits can be pinned on a small shape), e.g.
// GDD_FORCE=kpp_no_table,lloyd_no_prune or GDD_FORCE=kpp_big1_max=32768. Read on every call (host).
//   kpp_no_table      k-means++ without the n x n distance table (small and multi-block plans)
//   kpp_force_table   the multi-block table although kpp_table_pays says no (small k)
//   kpp_no_big1       the per-block table rounds instead of one workgroup per trial (n <= 16,384)
//   kpp_big1_max=N    one workgroup per trial up to N points (default 16,384, at most 32,768)
//   kpp_single_round  one table round per launch instead of the pair launches (T <= 8)
//   kpp_pair_serial   the single-block pair launch's two folds one after the other (not overlapped)
//   kpp_two_launch    the single-block rounds' distance + pick launches instead of the fused round
//   kpp_no_split      the per-(block, trial) rounds instead of the split rounds (>= 128 blocks)
//   lloyd_no_prune    every Lloyd E-step over every row (no bounds)
//   fold_no_pad       the Lloyd M-step gathers X itself instead of its zero-padded copy
//   estep_no_pad      the bounded E-step's row lists read X instead of the padded copy
//   fold_slice=F      M-step clusters above F x the mean size fold in slices (default 1.5; 0: off)
//   group_split       the multi-launch label grouping where the one-launch form fits
//   center_seq        KMeans' centring by the sequential column chains
//   bf16_v1           the r03 bf16 labels pass (gdd_kmeans.hip) instead of the r06 one (gdd_bf16.hip)
//   bf16_w4, bf16_w8  the r06 pass's 4- or 8-wave block form at any k (dims 41 .. 47)
//   hop_row_order     the propagation's work list in row order (no longest-first schedule)
//   hop_no_probe      longest first even where the locality probe would pick row order
//   hop_relabel_len   the relabelled hops' work list longest first instead of in the new order
//   hop_xcd_contig    each XCD walks a contiguous eighth of the work list (one feature slice)
bool forced(const char* token);
double forced_value(const char* token, double dflt);

int replay_or_run(const char* site, const void* key, size_t key_bytes, hipStream_t s,
                  const std::function<int(hipStream_t)>& enqueue);

// ---------------------------------------------------------------------------------------------
// internal entry points of the device-resident MiniBatchKMeans loop (gdd_kmeans.hip, used by
// gdd_fit.hip); DevMT / RngNext are defined in gdd_devrng.hpp
// ---------------------------------------------------------------------------------------------
struct DevMT;
struct RngNext;
int minibatch_step_dev(int64_t b, int dim, const float* X, const int64_t* rows, int k,
                       const float* C_old, float* C_new, float* weight_sums, int32_t* labels,
                       int step_i, int64_t n_samples, int max_no_improvement, int flags,
                       void* state, void* ws, size_t ws_bytes, const RngNext& rn, hipStream_t s);
int mb_loop_begin(int64_t b, int k, void* ws, size_t ws_bytes, hipStream_t s);
int mb_loop_end(int64_t b, int k, int last_step, int64_t n_samples, int max_no_improvement,
                void* state, void* ws, size_t ws_bytes, hipStream_t s);
int mb_rng_launch(const DevMT* in, DevMT* out, int64_t n, int64_t bs, int64_t* rows, hipStream_t s);
// the device reassignment (k_mb_reassign): any k whose swap table fits the LDS; a step with more
// than b/2 centres due (np.argsort's branch) is handed to the host through MBState.handoff
constexpr size_t kReassignLdsCap = 150 * 1024;
size_t mb_reassign_lds(int64_t bs, int k);
bool mb_reassign_ok(int64_t bs, int k);
int mb_reassign_launch(int step, int64_t bs, int dim, int k, float ratio, const float* X,
                       const int64_t* rows, float* C_new, float* counts, void* step_ws,
                       size_t step_ws_bytes, const DevMT* mt_in, DevMT* mt_mid, const RngNext& rn,
                       void* state, hipStream_t s);
// minibatch_step_dev flag: the step has no tail for step_i - 1 (the first step of a device segment
// resumed after host steps, whose convergence tests the host already ran)
constexpr int kStepNoTail = 1 << 16;

// Bound of the LDS arrival-counter spins (k_mb_reassign, k-means++ speculative prefixes and draws):
// a give-up takes the barrier redo. `make SPIN0=1` builds a twin with 0 so that every wait gives up
// and the redo paths run (tests/test_gpu_spin0.py pins them bit-for-bit against the oracle).
#ifndef GDD_SPIN_LIMIT
#define GDD_SPIN_LIMIT (1 << 16)
#endif
constexpr int kSpinLimit = GDD_SPIN_LIMIT;

// internal entry point of the k-means assignment (gdd_kmeans.hip), used by the Lloyd loop
// (gdd_lloyd.hip): ||C||² into cn2, then labels of all n rows; every kernel skips once `stop`
// says step `step_i` lies past the stopping decision (see stopped()).
int kmeans_assign_dev(int64_t n, int dim, const float* X, int k, const float* C, float* cn2,
                      int32_t* labels, unsigned long long* keys, const int32_t* stop, int step_i,
                      hipStream_t s);
// the bounded Lloyd E-step (gdd_lloyd.hip): top-2 distances of a (device-counted) row list
bool lloyd_prune_ok(int dim, int k);
int kmeans_assign_top2_dev(int64_t n_max, int dim, const float* X, const int64_t* rows,
                           const int64_t* n_dev, int k, const float* C, float* cn2,
                           unsigned long long* keys, float* sec, const int32_t* stop, int step_i,
                           hipStream_t s, const float* Xp = nullptr, int ldp = 0);

// `stop` (nullable) points at a device stop word (0 = running, s+1 = a test fired at step s; the
// MiniBatch MBState::stop_at, the Lloyd LloydState::stop_at). Kernels of a later step return at
// once, so the host can enqueue steps ahead of the stopping decision. One 32-bit word read with an
// agent-scope atomic load: the test written by a sibling block of the same launch is never seen
// torn, and step s itself always completes.
__device__ __forceinline__ bool stopped(const int32_t* stop, int step_i) {
  if (!stop) return false;
  const int v = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v != 0 && v - 1 < step_i;
}

// sklearn _euclidean_dense_dense(a, b, n_features, squared=True) (_k_means_common.pyx:26-48):
// groups of 4 summed left to right, added to the running result; remainder added one by one.
// Separate mul/add (no fma).
__device__ __forceinline__ float skl_sqdist(const float* __restrict__ a, const float* __restrict__ b,
                                            int dim) {
  float r = 0.f;
  int j = 0;
  for (; j + 4 <= dim; j += 4) {
    float d0 = a[j] - b[j], d1 = a[j + 1] - b[j + 1], d2 = a[j + 2] - b[j + 2],
          d3 = a[j + 3] - b[j + 3];
    r = r + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
  }
  for (; j < dim; ++j) {
    float d0 = a[j] - b[j];
    r = r + d0 * d0;
  }
  return r;
}

// ---------------------------------------------------------------------------------------------
// numerics shared by kernels and documented in DESIGN.md
// ---------------------------------------------------------------------------------------------
// correctly rounded fp64 x^-1/2 (numpy np.power(x, -0.5) agrees with this on ~95% of inputs, with
// the rest off by one fp64 ulp; the fp32 values derived from it agree with numpy's except w.p.~1e-8)
__host__ __device__ inline double cr_rsqrt(double x) {
  if (!(x > 0.0)) {
    if (x == 0.0) return __builtin_inf();  // caller maps inf -> 0 (deep_robust_utils.py:202)
    return __builtin_nan("");
  }
  if (__builtin_isinf(x)) return 0.0;
  double y = 1.0 / __builtin_sqrt(x);
  // residual r(y) = x*y*y - 1 evaluated with error-free products; pick the neighbour with the
  // smaller |r| (the exact value is irrational unless x is an even power of two)
  auto resid = [x](double v) {
    double hi = v * v;
    double lo = __builtin_fma(v, v, -hi);  // v*v = hi + lo exactly
    double p = x * hi;
    double pe = __builtin_fma(x, hi, -p);  // x*hi = p + pe exactly
    return (p - 1.0) + (pe + x * lo);
  };
  double r0 = resid(y);
  // y > 0: the neighbouring doubles are one unit of the bit pattern away
  union { double d; unsigned long long u; } b{y};
  b.u = r0 < 0.0 ? b.u + 1ull : b.u - 1ull;
  double y1 = b.d;
  double r1 = resid(y1);
  return (__builtin_fabs(r1) < __builtin_fabs(r0)) ? y1 : y;
}

// ---------------------------------------------------------------------------------------------
// in-kernel phase stamps (diagnostic builds only: make STAMPS=1 builds libgdd_stamps.so).
// GDD_STAMP_WHEN(table, who, slot) records s_memrealtime (100 MHz) from one thread into a per-file table
// that gdd_dbg_stamps_<file>() copies out; in the product build it expands to nothing.
// ---------------------------------------------------------------------------------------------
#ifdef GDD_STAMPS
#define GDD_STAMP_TABLE(file)                                                                   \
  __device__ unsigned long long g_stamps_##file[256];                                           \
  extern "C" int gdd_dbg_stamps_##file(unsigned long long* out) {                              \
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_##file), sizeof(g_stamps_##file)); \
  }
// stamp from the thread for which `who` holds (e.g. threadIdx.x == 0 && blockIdx.x == 0)
#define GDD_STAMP_WHEN(table, who, slot)                                                        \
  do {                                                                                          \
    if (who) table[(slot)] = __builtin_amdgcn_s_memrealtime();                                  \
  } while (0)
#else
#define GDD_STAMP_TABLE(file)
#define GDD_STAMP_WHEN(table, who, slot) \
  do {                                   \
  } while (0)
#endif

}  // namespace gdd
