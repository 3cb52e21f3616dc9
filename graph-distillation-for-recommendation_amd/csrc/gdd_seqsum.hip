// gdd_seqsum.hip — the sequential fp32 sum ((0 + t0) + t1) + ... of non-negative terms, evaluated in
// parallel with the sequential result bit for bit. This is sklearn's inertia with one OpenMP thread
// (_inertia_dense, _k_means_common.pyx:92-121: `inertia += sq_dist * sample_weight[i]` in sample
// order), which the reference reaches through MiniBatchKMeans.fit / KMeans.fit
// (clustgdd_agent_transduct.py:102-105, distill_recsys.py:172-180).
//
// Why a sequential fp32 sum can be evaluated in parallel, exactly:
// * While the running sum s lies in one binade [2^e, 2^(e+1)) (e >= -126; the subnormals share binade
//   -126's grid), s is a multiple of u = 2^(e-23). For a term t >= 0 with s + t < 2^(e+1) the fp32
//   add rounds s + t to the nearest multiple of u: fl(s + t) = s + d·u with d = round(t/u) — except
//   at an exact tie (t/u = q + 1/2), where round-to-even takes q or q+1 by the parity of s/u + q.
// * So in units of u the sum is an integer S < 2^24 that each term advances by an amount depending only
//   on S's parity: a pair (D0, D1), the advance for even and for odd S. Pairs compose associatively
//   (compose() below), so a workgroup scans them like integers.
// * The first term whose advance reaches S >= 2^24 (the sum leaves the binade) is added in hardware —
//   s is known exactly there — and the scan resumes in the new binade. Terms are non-negative, so the
//   sum only climbs: this happens at most once per binade (about log2 n times for terms of one scale).
// * A NaN, an infinity, a negative term or an infinite sum ends the parallel form: the rest is added
//   one term at a time by one thread, as before.
//
// Two forms: one workgroup walking the array in chunks (gdd_inertia, no workspace), and for long
// arrays three launches (gdd_inertia_ws): per-segment fp64 sums; per-segment advance pairs for the two
// binades the running sum most likely has there (the exact sum up to the segment ± the sequential
// sum's error); one workgroup then scans the segments' pairs binade by binade and re-walks, from the
// exact running sum, only a segment whose pairs do not apply (a binade change inside it, or a guess
// that missed).
#include <cmath>
#include <cstdlib>

#include "gdd_common.hpp"

namespace gdd {
namespace {

constexpr int kSat = 1 << 26;       // advances saturate here: anything >= 2^24 leaves the binade
constexpr int kTop = 1 << 24;       // S < 2^24 inside a binade
constexpr int kWalkThreads = 1024;  // the chunked walk's workgroup
constexpr int kWalkE = 4;           // terms per thread per chunk (chunk = 4096 terms)
constexpr int kSegThreads = 256;    // per-segment advance pairs
constexpr int kSegTerms = 2048;     // terms per segment (at most kMaxSeg segments; longer when n is large)
constexpr int kMaxSeg = 1024;       // segments per resolve window (one per thread)

struct Dp {
  int d0, d1;  // advance of S (units of u) for even / odd S
};

__device__ __forceinline__ Dp compose(Dp f, Dp g) {  // f, then g
  const int a = f.d0 + ((f.d0 & 1) ? g.d1 : g.d0);
  const int b = f.d1 + ((f.d1 & 1) ? g.d0 : g.d1);
  return {min(a, kSat), min(b, kSat)};
}

__device__ __forceinline__ int adv_at(Dp f, int S) { return (S & 1) ? f.d1 : f.d0; }

// binade of s >= 0 (finite): e with s in [2^e, 2^(e+1)), or -126 for zero and subnormals
__device__ __forceinline__ int binade_of(float s) {
  const int E = (int)((__float_as_uint(s) >> 23) & 0xff);
  return E == 0 ? -126 : E - 127;
}

__device__ __forceinline__ bool good_term(float t) { return t >= 0.f && t < __builtin_inff(); }

// the advance of one term t >= 0 (finite) in binade e
__device__ __forceinline__ Dp term_adv(float t, int e) {
  const float v = ldexpf(t, 23 - e);  // t/u: exact, or an underflow far below 1/2
  if (!(v < 33554432.f)) return {kSat, kSat};
  const float fl = floorf(v);
  const float fr = v - fl;  // exact
  const int q = (int)fl;
  if (fr < 0.5f) return {q, q};
  if (fr > 0.5f) return {q + 1, q + 1};
  return {q + (q & 1), q + ((q + 1) & 1)};  // tie: the even one of S+q, S+q+1
}

__device__ __forceinline__ float term_at(const float* __restrict__ x, const float* __restrict__ w,
                                         int64_t i) {
  return w ? x[i] * w[i] : x[i] * 1.0f;  // sq_dist * sample_weight[i]
}

// exclusive scan of one pair per thread over a workgroup of NW waves; *total = all pairs composed,
// *any = some thread's flag was set. lds: NW pairs and NW ints. Ends with a barrier (lds reusable).
template <int NW>
__device__ Dp block_excl_scan(Dp v, bool flag, Dp* lds, int* flds, Dp* total, bool* any) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Dp inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    Dp up;
    up.d0 = __shfl_up(inc.d0, o);
    up.d1 = __shfl_up(inc.d1, o);
    if (lane >= o) inc = compose(up, inc);
  }
  Dp ex;
  ex.d0 = __shfl_up(inc.d0, 1);
  ex.d1 = __shfl_up(inc.d1, 1);
  if (lane == 0) ex = {0, 0};
  const bool wflag = __ballot(flag) != 0ull;
  if (lane == 63) {
    lds[wv] = inc;
    flds[wv] = wflag;
  }
  __syncthreads();
  Dp wp = {0, 0}, tot = {0, 0};
  int fl = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const Dp t = lds[i];
    if (i < wv) wp = compose(wp, t);
    tot = compose(tot, t);
    fl |= flds[i];
  }
  *total = tot;
  *any = fl != 0;
  __syncthreads();
  return compose(wp, ex);
}

// lowest thread index with `flag` set in the workgroup (INT32_MAX if none). Ends with a barrier.
template <int NW>
__device__ int block_first(bool flag, int* lds) {
  const unsigned long long b = __ballot(flag);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) lds[wv] = b ? wv * 64 + __builtin_ctzll(b) : 0x7fffffff;
  __syncthreads();
  int m = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < NW; ++i) m = min(m, lds[i]);
  __syncthreads();
  return m;
}

struct WalkLds {
  Dp scan[kWalkThreads / 64];
  int flag[kWalkThreads / 64];
  int first[kWalkThreads / 64];
  float s_new;
  long long pos_new;
};

// The whole workgroup (kWalkThreads) continues the sequential sum s over terms [lo, hi) and returns
// it (in every thread). Chunks of kWalkThreads * kWalkE terms, each thread kWalkE consecutive ones.
__device__ __forceinline__ float walk_range(const float* __restrict__ x, const float* __restrict__ w, int64_t lo,
                            int64_t hi, float s, WalkLds& L) {
  constexpr int NW = kWalkThreads / 64;
  constexpr int64_t CH = (int64_t)kWalkThreads * kWalkE;
  const int tid = threadIdx.x;
  int64_t pos = lo;
  float t[kWalkE];
  auto load = [&](int64_t p, float* dst) {
    const int64_t b = p + (int64_t)tid * kWalkE;
#pragma unroll
    for (int j = 0; j < kWalkE; ++j) dst[j] = (b + j < hi) ? term_at(x, w, b + j) : 0.f;
  };
  if (pos < hi) load(pos, t);
  while (pos < hi) {
    if (!(s < __builtin_inff())) break;  // an infinite sum (uniform): the one-term tail below
    bool bad = false;
#pragma unroll
    for (int j = 0; j < kWalkE; ++j) bad |= !good_term(t[j]);
    const int e = binade_of(s);
    const int S0 = (int)ldexpf(s, 23 - e);
    Dp f = {0, 0};
#pragma unroll
    for (int j = 0; j < kWalkE; ++j) f = compose(f, term_adv(t[j], e));
    // the next chunk's terms in flight while this one is scanned (used unless a binade change moves pos)
    float tn[kWalkE];
    const bool more = pos + CH < hi;
    if (more) load(pos + CH, tn);
    Dp tot;
    bool any_bad;
    const Dp ex = block_excl_scan<NW>(f, bad, L.scan, L.flag, &tot, &any_bad);
    if (any_bad) break;  // NaN, infinite or negative terms in this chunk: the one-term tail below
    const int S_end = S0 + adv_at(tot, S0);
    if (S_end < kTop) {  // the whole chunk stays in the binade
      s = ldexpf((float)S_end, e - 23);
      pos += CH;
      if (more) {
#pragma unroll
        for (int j = 0; j < kWalkE; ++j) t[j] = tn[j];
      }
      continue;
    }
    const int Sb = S0 + adv_at(ex, S0);
    const int Sa = Sb + adv_at(f, Sb);
    const int c = block_first<NW>(Sa >= kTop, L.first);
    if (tid == c) {  // the first thread whose terms leave the binade finds the term and adds it
      int S = Sb;
      const int64_t b = pos + (int64_t)tid * kWalkE;
#pragma unroll
      for (int j = 0; j < kWalkE; ++j) {
        const int S2 = S + adv_at(term_adv(t[j], e), S);
        if (S2 >= kTop) {
          L.s_new = ldexpf((float)S, e - 23) + t[j];
          L.pos_new = b + j + 1;
          break;
        }
        S = S2;
      }
    }
    __syncthreads();
    s = L.s_new;
    pos = L.pos_new;
    __syncthreads();
    if (pos < hi) load(pos, t);
  }
  if (pos < hi) {  // non-finite or negative terms: one term at a time (rare)
    if (tid == 0) {
      for (int64_t i = pos; i < hi; ++i) s = s + term_at(x, w, i);
      L.s_new = s;
    }
    __syncthreads();
    s = L.s_new;
    __syncthreads();
  }
  return s;
}

__global__ __launch_bounds__(kWalkThreads) void k_seqsum_walk(int64_t n, const float* __restrict__ x,
                                                              const float* __restrict__ w,
                                                              float* __restrict__ out) {
  __shared__ WalkLds L;
  const float s = walk_range(x, w, 0, n, 0.f, L);
  if (threadIdx.x == 0) out[0] = s;
}

// ---- the segmented form ------------------------------------------------------------------------
struct SegRec {
  int e[2];   // candidate binades
  Dp f[2];    // the segment's advance pair in each
  int bad;    // a term that is NaN, infinite or negative
  int pad[3];
};

__global__ __launch_bounds__(kSegThreads) void k_seqsum_segsum(int64_t n, int64_t seg,
                                                               const float* __restrict__ x,
                                                               const float* __restrict__ w,
                                                               double* __restrict__ segsum) {
  const int64_t lo = (int64_t)blockIdx.x * seg, hi = min(n, lo + seg);
  double a = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kSegThreads) a += (double)term_at(x, w, i);
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  __shared__ double r[kSegThreads / 64];
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < kSegThreads / 64; ++i) t += r[i];
    segsum[blockIdx.x] = t;
  }
}

// binades the sequential sum most likely has at a segment starting after an exact sum P: the sequential
// fp32 sum of m terms is within (m-1)·2^-24 relative of P, usually much closer; the binade of P and
// the neighbour on the nearer side. A wrong guess only costs a re-walk of the segment.
__device__ __forceinline__ void guess_binades(double P, int* e) {
  const float p = (float)P;
  const int e0 = binade_of(p);
  e[0] = e0;
  if (e0 == -126) {
    e[1] = -125;
    return;
  }
  const float r = ldexpf(p, -e0);  // in [1, 2)
  e[1] = r >= 1.5f ? min(e0 + 1, 127) : e0 - 1;
}

__global__ __launch_bounds__(kSegThreads) void k_seqsum_segpairs(int64_t n, int64_t seg, int nseg,
                                                                 const float* __restrict__ x,
                                                                 const float* __restrict__ w,
                                                                 const double* __restrict__ segsum,
                                                                 SegRec* __restrict__ rec) {
  constexpr int NW = kSegThreads / 64;
  extern __shared__ __attribute__((aligned(16))) float stage[];  // seg terms
  __shared__ Dp scan_lds[NW];
  __shared__ int flag_lds[NW];
  __shared__ double psum[NW];
  __shared__ int bad_any;
  const int b = blockIdx.x;
  const int64_t lo = (int64_t)b * seg, hi = min(n, lo + seg);
  const int m = (int)(hi - lo);
  // exact-ish sum of every term before this segment
  double P = 0.0;
  for (int j = threadIdx.x; j < b; j += kSegThreads) P += segsum[j];
  for (int o = 32; o > 0; o >>= 1) P += __shfl_xor(P, o);
  if ((threadIdx.x & 63) == 0) psum[threadIdx.x >> 6] = P;
  if (threadIdx.x == 0) bad_any = 0;
  bool bad = false;
  for (int i = threadIdx.x; i < m; i += kSegThreads) {
    const float t = term_at(x, w, lo + i);
    bad |= !good_term(t);
    stage[i] = t;
  }
  __syncthreads();
  if (bad) bad_any = 1;
  P = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) P += psum[i];
  int e[2];
  guess_binades(P, e);
  // thread r composes terms [r*R, (r+1)*R) of the segment
  const int R = (m + kSegThreads - 1) / kSegThreads;
  const int a0 = threadIdx.x * R, a1 = min(m, a0 + R);
  Dp f0 = {0, 0}, f1 = {0, 0};
  for (int i = a0; i < a1; ++i) {
    const float t = stage[i];
    if (!good_term(t)) continue;  // the segment is re-walked anyway
    f0 = compose(f0, term_adv(t, e[0]));
    f1 = compose(f1, term_adv(t, e[1]));
  }
  Dp t0, t1;
  bool unused;
  (void)block_excl_scan<NW>(f0, false, scan_lds, flag_lds, &t0, &unused);
  (void)block_excl_scan<NW>(f1, false, scan_lds, flag_lds, &t1, &unused);
  if (threadIdx.x == 0) {
    SegRec r;
    r.e[0] = e[0];
    r.e[1] = e[1];
    r.f[0] = t0;
    r.f[1] = t1;
    r.bad = bad_any;
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    rec[b] = r;
  }
}

// One workgroup, one segment per thread (windows of kWalkThreads segments): in the current binade,
// the segments whose pairs apply are scanned together; the first one that does not is re-walked from
// the exact running sum, and the scan resumes after it.
__global__ __launch_bounds__(kWalkThreads) void k_seqsum_resolve(int64_t n, int64_t seg, int nseg,
                                                                 const float* __restrict__ x,
                                                                 const float* __restrict__ w,
                                                                 const SegRec* __restrict__ rec,
                                                                 float* __restrict__ out) {
  constexpr int NW = kWalkThreads / 64;
  __shared__ WalkLds L;
  const int tid = threadIdx.x;
  float s = 0.f;
  for (int g0 = 0; g0 < nseg; g0 += kWalkThreads) {
    const int gn = min(kWalkThreads, nseg - g0);
    SegRec my{};
    if (tid < gn) my = rec[g0 + tid];
    int b0 = 0;  // segments g0 .. g0+b0-1 are summed into s
    while (b0 < gn) {
      if (!(s < __builtin_inff())) {  // an infinite or NaN sum: the rest one term at a time
        s = walk_range(x, w, (int64_t)(g0 + b0) * seg, n, s, L);
        g0 = nseg;
        break;
      }
      const int e = binade_of(s);
      const int S0 = (int)ldexpf(s, 23 - e);
      const bool mine = tid >= b0 && tid < gn;
      Dp f = {0, 0};
      if (mine) {
        if (!my.bad && my.e[0] == e) f = my.f[0];
        else if (!my.bad && my.e[1] == e) f = my.f[1];
        else f = {kSat, kSat};  // re-walked
      }
      Dp tot;
      bool unused;
      const Dp ex = block_excl_scan<NW>(f, false, L.scan, L.flag, &tot, &unused);
      const int Sb = S0 + adv_at(ex, S0);
      const int Sa = Sb + adv_at(f, Sb);
      const int c = block_first<NW>(mine && Sa >= kTop, L.first);
      if (c == 0x7fffffff) {  // every remaining segment of the window applies
        s = ldexpf((float)(S0 + adv_at(tot, S0)), e - 23);
        break;
      }
      if (tid == c) L.s_new = ldexpf((float)Sb, e - 23);  // the exact sum before segment c
      __syncthreads();
      s = L.s_new;
      __syncthreads();
      const int64_t lo = (int64_t)(g0 + c) * seg, hi = min(n, lo + seg);
      s = walk_range(x, w, lo, hi, s, L);
      b0 = c + 1;
    }
  }
  if (tid == 0) out[0] = s;
}

// segment length: kSegTerms, doubled while there would be more than kMaxSeg segments, at most 16384
// terms (64 KB of staging); longer arrays take several resolve windows
int64_t seg_len(int64_t n) {
  int64_t seg = kSegTerms;
  while ((n + seg - 1) / seg > kMaxSeg && seg < 16384) seg *= 2;
  return seg;
}


}  // namespace


}  // namespace gdd

using namespace gdd;

extern "C" int gdd_inertia(int64_t n, const float* sq_dist, const float* w, float* out,
                           gdd_stream_t stream) {
  GDD_REQUIRE(n >= 0 && out && (n == 0 || sq_dist), "inertia: bad arguments");
  hipStream_t s = to_hip(stream);
  k_seqsum_walk<<<1, kWalkThreads, 0, s>>>(n, sq_dist, w, out);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" size_t gdd_inertia_ws_bytes(int64_t n) {
  if (n <= 0) return 256;
  const int64_t nseg = (n + seg_len(n) - 1) / seg_len(n);
  return align256(sizeof(double) * nseg) + align256(sizeof(SegRec) * nseg) + 256;
}

extern "C" int gdd_inertia_ws(int64_t n, const float* sq_dist, const float* w, float* out, void* ws,
                              size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n >= 0 && out && (n == 0 || sq_dist), "inertia_ws: bad arguments");
  hipStream_t s = to_hip(stream);
  const int64_t seg = seg_len(n);
  const int64_t nseg = (n + seg - 1) / seg;
  if (nseg <= 2) {  // short: the chunked walk alone
    k_seqsum_walk<<<1, kWalkThreads, 0, s>>>(n, sq_dist, w, out);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  GDD_REQUIRE(ws && ws_bytes >= gdd_inertia_ws_bytes(n), "inertia_ws: workspace too small");
  Carver cv(ws, ws_bytes);
  double* segsum = cv.take<double>(nseg);
  SegRec* rec = cv.take<SegRec>(nseg);
  k_seqsum_segsum<<<(unsigned)nseg, kSegThreads, 0, s>>>(n, seg, sq_dist, w, segsum);
  GDD_LAUNCHED();
  k_seqsum_segpairs<<<(unsigned)nseg, kSegThreads, sizeof(float) * seg, s>>>(n, seg, (int)nseg, sq_dist,
                                                                            w, segsum, rec);
  GDD_LAUNCHED();
  k_seqsum_resolve<<<1, kWalkThreads, 0, s>>>(n, seg, (int)nseg, sq_dist, w, rec, out);
  GDD_LAUNCHED();
  return GDD_OK;
}
