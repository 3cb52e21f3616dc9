// gdd_colsum.hip — KMeans.fit's centring at large n (sklearn/cluster/_kmeans.py:1476-1487 with
// _tolerance :279-288: X.mean(axis=0), X - mean, X.var(axis=0)) with numpy's column sums evaluated in
// parallel, bit for bit. numpy reduces axis 0 of a C-contiguous float32 matrix row by row, so each
// column is one sequential fp32 chain over all n rows (gdd_scaler.hip's k_col_stats walks those chains
// one dependent add per row: ~8.7 ms per pass at 2.45M rows).
//
// Why a sequential fp32 sum of SIGNED terms can be evaluated in parallel, exactly
// (tests/test_signed_chain_model.py is the CPU model of these kernels):
// * While the running sum s lies in one signed binade (|s| in [2^e, 2^(e+1)), one sign; e = -126
//   covers |s| < 2^-125 and zero, one grid), s = S*u with u = 2^(e-23) and S an integer. If s + t stays
//   strictly inside, fl(s + t) = (S + round(t/u))*u with ties to the even S: the advance depends only on
//   S's parity.
// * A run of terms is a two-state transducer: per start parity its advance and its least and greatest
//   partial advance (Tr). Transducers compose associatively, so a workgroup scans them.
// * A run applies from S0 when every partial sum stays strictly inside the binade: below 2^24, and
//   above 2^23 + 1/2 on the side nearer zero (under 2^e the grid halves), checked as >= 2^23 + 1.
// * Three launches per pass: per-segment fp64 column sums (k_cs_segsum); per (segment, column) the
//   transducers for the two binades the running sum most likely has there — the fp64 prefix's binade
//   and its nearer neighbour (k_cs_records); one wave per column (k_cs_resolve) scanning the
//   segments' transducers from the exact running sum and re-walking a segment where none applies
//   (k_cs_walk: 512-term passes, the first term that leaves the binade added in hardware, resume).
// * A NaN or infinite term or sum: the rest of that column is added one term at a time.
#include <cmath>
#include <cstdlib>

#include "gdd_common.hpp"

namespace gdd {
namespace {

constexpr int kCsSat = 1 << 27;
constexpr int kCsTop = 1 << 24;
constexpr int kCsLow = 1 << 23;
constexpr int kCsSeg = 512;    // rows per segment
constexpr int kCsThr = 256;
constexpr int kCsWalkE = 8;    // terms per lane per walk pass (one wave: 64 * 8 = kCsSeg)
constexpr int64_t kCsMinRows = 65536;

struct Tr {
  int a0, n0, x0;  // even start: advance, least and greatest partial advance
  int a1, n1, x1;  // odd start
};

__device__ __forceinline__ int cs_clamp(int v) { return min(max(v, -kCsSat), kCsSat); }

// the empty run: no partial sums (least +Sat, greatest -Sat)
__device__ __forceinline__ Tr tr_ident() { return {0, kCsSat, -kCsSat, 0, kCsSat, -kCsSat}; }

__device__ __forceinline__ Tr tr_compose(const Tr& f, const Tr& g) {  // f, then g
  Tr o;
  {
    const int a = f.a0;
    const bool odd = (a & 1) != 0;
    const int b = odd ? g.a1 : g.a0, bn = odd ? g.n1 : g.n0, bx = odd ? g.x1 : g.x0;
    o.a0 = cs_clamp(a + b);
    o.n0 = min(f.n0, cs_clamp(a + bn));
    o.x0 = max(f.x0, cs_clamp(a + bx));
  }
  {
    const int a = f.a1;
    const bool odd = ((a + 1) & 1) != 0;
    const int b = odd ? g.a1 : g.a0, bn = odd ? g.n1 : g.n0, bx = odd ? g.x1 : g.x0;
    o.a1 = cs_clamp(a + b);
    o.n1 = min(f.n1, cs_clamp(a + bn));
    o.x1 = max(f.x1, cs_clamp(a + bx));
  }
  return o;
}

// one term's advances in binade e (even start, odd start)
__device__ __forceinline__ void term_adv2(float t, int e, int& q0, int& q1) {
  const float v = ldexpf(t, 23 - e);  // t/u: exact, or far below 1/2, or saturated
  if (!(fabsf(v) < 67108864.f)) {
    q0 = q1 = v > 0.f ? kCsSat : -kCsSat;
    return;
  }
  const float fl = floorf(v);
  const float fr = v - fl;
  const int q = (int)fl;
  if (fr < 0.5f) {
    q0 = q1 = q;
  } else if (fr > 0.5f) {
    q0 = q1 = q + 1;
  } else {  // a tie: the even one of S+q, S+q+1
    q0 = q + (q & 1);
    q1 = q + ((q + 1) & 1);
  }
}

// f, then one term with advances (q0, q1)
__device__ __forceinline__ Tr tr_append(const Tr& f, int q0, int q1) {
  Tr o;
  {
    const int a = f.a0;
    const int v = cs_clamp(a + (((a & 1) != 0) ? q1 : q0));
    o.a0 = v;
    o.n0 = min(f.n0, v);
    o.x0 = max(f.x0, v);
  }
  {
    const int a = f.a1;
    const int v = cs_clamp(a + ((((a + 1) & 1) != 0) ? q1 : q0));
    o.a1 = v;
    o.n1 = min(f.n1, v);
    o.x1 = max(f.x1, v);
  }
  return o;
}

__device__ __forceinline__ int cs_binade(float s) {
  const int E = (int)((__float_as_uint(s) >> 23) & 0xff);
  return E == 0 ? -126 : E - 127;
}

// the run applies from S0 (in binade e): every partial sum strictly inside the binade
__device__ __forceinline__ bool tr_applies(int S0, int e, const Tr& f) {
  const bool odd = (S0 & 1) != 0;
  const long long lo = (long long)S0 + (odd ? f.n1 : f.n0);
  const long long hi = (long long)S0 + (odd ? f.x1 : f.x0);
  if (e == -126) return lo > -kCsTop && hi < kCsTop;
  if (S0 > 0) return lo > kCsLow && hi < kCsTop;
  return hi < -kCsLow && lo > -kCsTop;
}

__device__ __forceinline__ int tr_adv(const Tr& f, int S0) { return (S0 & 1) ? f.a1 : f.a0; }

// the chain's term for row r of column c: x (pass 0) or (x - m)^2 (pass 1; numpy's subtract, square)
__device__ __forceinline__ float cs_term(const float* __restrict__ X, int dim, int64_t r, int c,
                                         const float* __restrict__ m) {
  const float x = X[r * dim + c];
  if (!m) return x;
  const float d = x - m[c];
  return d * d;
}

struct CsRec {
  int e[2];   // candidate binades
  Tr f[2];    // the segment's transducer in each
  int bad;    // a NaN or infinite term in the segment
  int pad;
};

// ---- the segment passes: chunks of CR rows staged column-major in LDS -------------------------------
// A segment's rows arrive in chunks of CR rows (CR * dim <= kCsChunk floats) read as one contiguous run
// (coalesced), the next chunk's values in flight in registers while the current one is used; thread
// t < P * dim owns column t % dim and the t / dim-th of P runs of each chunk (P = 256 / dim).
constexpr int kCsChunk = 16384;
constexpr int kCsPre = kCsChunk / kCsThr;  // staged values per thread per chunk
constexpr int64_t kCsMaxDim = 256;

__host__ __device__ inline int cs_rows_per_chunk(int dim) { return max(16, (kCsChunk / dim) & ~15); }

// the chunk loop of one segment; use(col, run_lo, run_hi, colptr) per thread after each chunk lands,
// then combine() by the whole workgroup (between barriers)
template <class Use, class Combine>
__device__ __forceinline__ void cs_segment_chunks(int64_t n, int dim, const float* __restrict__ X,
                                                  const float* __restrict__ m, float* __restrict__ Xout,
                                                  int64_t lo, int64_t hi, float* buf, Use use, Combine combine) {
  const int tid = threadIdx.x;
  const int CR = cs_rows_per_chunk(dim), CS = CR + 1;
  const int P = kCsThr / dim;
  const int rl = (CR + P - 1) / P;
  const int col = tid % dim, run = tid / dim;
  const bool owner = run < P;
  float v[kCsPre];
  auto fetch = [&](int64_t r0) {
    const float* base = X + r0 * dim;
    const int last = (int)((min<int64_t>(hi, r0 + CR) - r0) * dim) - 1;
#pragma unroll
    for (int i = 0; i < kCsPre; ++i)  // unconditional (clamped) loads: static outstanding counts
      v[i] = base[min(tid + kCsThr * i, last)];
  };
  auto stage = [&](int64_t r0) {
    const int e1 = (int)((min<int64_t>(hi, r0 + CR) - r0) * dim);
    float* obase = Xout ? Xout + r0 * dim : nullptr;
    int r = tid / dim, c = tid % dim;
    const int dr = kCsThr / dim, dc = kCsThr % dim;
#pragma unroll
    for (int i = 0; i < kCsPre; ++i) {
      const int e = tid + kCsThr * i;
      if (e < e1) {
        float t = v[i];
        if (m) {
          const float d = t - m[c];
          if (obase) obase[e] = d;
          t = d * d;
        }
        buf[c * CS + r] = t;
      }
      r += dr;
      c += dc;
      if (c >= dim) {
        c -= dim;
        ++r;
      }
    }
  };
  if (lo < hi) fetch(lo);
  for (int64_t r0 = lo; r0 < hi; r0 += CR) {
    stage(r0);
    __syncthreads();
    if (r0 + CR < hi) fetch(r0 + CR);  // in flight while this chunk is used
    const int rows = (int)min<int64_t>(CR, hi - r0);
    if (owner) use(col, min(rows, run * rl), min(rows, (run + 1) * rl), buf + col * CS);
    __syncthreads();
    combine();
    __syncthreads();
  }
}

// ---- per-segment fp64 column sums (pass 1 also writes X - m) ----------------------------------------
__global__ __launch_bounds__(kCsThr) void k_cs_segsum(int64_t n, int dim, const float* __restrict__ X,
                                                      const float* __restrict__ m, float* __restrict__ Xout,
                                                      double* __restrict__ segsum) {
  extern __shared__ __attribute__((aligned(16))) float cs_buf[];
  double* part = reinterpret_cast<double*>(cs_buf + kCsChunk + kCsThr);  // P x dim partials
  const int64_t lo = (int64_t)blockIdx.x * kCsSeg, hi = min<int64_t>(n, lo + kCsSeg);
  const int tid = threadIdx.x, P = kCsThr / dim;
  double total = 0.0;
  cs_segment_chunks(
      n, dim, X, m, Xout, lo, hi, cs_buf,
      [&](int c, int a, int b, const float* colp) {
        double acc = 0.0;
        for (int r = a; r < b; ++r) acc += (double)colp[r];
        part[tid] = acc;
      },
      [&]() {
        if (tid < dim)
          for (int p = 0; p < P; ++p) total += part[p * dim + tid];
      });
  if (tid < dim) segsum[(int64_t)blockIdx.x * dim + tid] = total;
}

// exclusive fp64 prefix of the segment sums, one workgroup per column (thread t sums a contiguous
// slice, a block scan of the slice totals, then each slice's prefixes; fp64 guesses, any order)
__global__ __launch_bounds__(kCsThr) void k_cs_prefix(int nseg, int dim, const double* __restrict__ segsum,
                                                      double* __restrict__ pref) {
  __shared__ double tot[kCsThr];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int per = (nseg + kCsThr - 1) / kCsThr;
  const int b0 = min(nseg, tid * per), b1 = min(nseg, b0 + per);
  double a = 0.0;
  for (int b = b0; b < b1; ++b) a += segsum[(int64_t)b * dim + c];
  tot[tid] = a;
  __syncthreads();
  if (tid == 0) {
    double p = 0.0;
    for (int i = 0; i < kCsThr; ++i) {
      const double t = tot[i];
      tot[i] = p;
      p += t;
    }
  }
  __syncthreads();
  double p = tot[tid];
  for (int b = b0; b < b1; ++b) {
    pref[(int64_t)b * dim + c] = p;
    p += segsum[(int64_t)b * dim + c];
  }
}

// binades the sequential sum most likely has at a segment starting after an fp64 prefix P: P's binade
// and the neighbour on the nearer side (a wrong guess costs a re-walk of the segment, nothing else)
__device__ __forceinline__ bool cs_guess(double P, int* e) {
  const float p = (float)P;
  if (!(fabsf(p) < __builtin_inff())) return false;
  const int e0 = cs_binade(p);
  e[0] = e0;
  if (e0 == -126) {
    e[1] = -125;
    return true;
  }
  const float r = fabsf(ldexpf(p, -e0));  // in [1, 2)
  e[1] = r >= 1.5f ? min(e0 + 1, 127) : e0 - 1;
  return true;
}

// ---- per (segment, column) transducers in both candidate binades ---------------------------------------
__global__ __launch_bounds__(kCsThr) void k_cs_records(int64_t n, int dim, const float* __restrict__ X,
                                                       const float* __restrict__ m,
                                                       const double* __restrict__ pref,
                                                       CsRec* __restrict__ rec) {
  extern __shared__ __attribute__((aligned(16))) float cs_buf[];
  Tr* runs = reinterpret_cast<Tr*>(cs_buf + kCsChunk + kCsThr);  // P x dim x 2
  int* badv = reinterpret_cast<int*>(runs + 2 * kCsThr);
  const int b = blockIdx.x, tid = threadIdx.x, P = kCsThr / dim;
  const int64_t lo = (int64_t)b * kCsSeg, hi = min<int64_t>(n, lo + kCsSeg);
  const int col = tid % dim;
  int e[2] = {0, 0};
  const bool ok = cs_guess(pref[(int64_t)b * dim + col], e);
  Tr run0 = tr_ident(), run1 = tr_ident();
  int bad = ok ? 0 : 1;
  cs_segment_chunks(
      n, dim, X, m, nullptr, lo, hi, cs_buf,
      [&](int c, int a, int bnd, const float* colp) {
        Tr f0 = tr_ident(), f1 = tr_ident();
        int bd = 0;
        for (int r = a; r < bnd; ++r) {
          const float t = colp[r];
          bd |= !(fabsf(t) < __builtin_inff());
          int q0, q1;
          term_adv2(t, e[0], q0, q1);
          f0 = tr_append(f0, q0, q1);
          term_adv2(t, e[1], q0, q1);
          f1 = tr_append(f1, q0, q1);
        }
        runs[2 * tid] = f0;
        runs[2 * tid + 1] = f1;
        badv[tid] = bd;
      },
      [&]() {
        if (tid < dim)
          for (int p = 0; p < P; ++p) {
            run0 = tr_compose(run0, runs[2 * (p * dim + tid)]);
            run1 = tr_compose(run1, runs[2 * (p * dim + tid) + 1]);
            bad |= badv[p * dim + tid];
          }
      });
  if (tid < dim) {
    CsRec r;
    r.e[0] = e[0];
    r.e[1] = e[1];
    r.f[0] = run0;
    r.f[1] = run1;
    r.bad = bad;
    r.pad = 0;
    rec[(int64_t)b * dim + tid] = r;
  }
}

size_t cs_lds_bytes() { return sizeof(float) * (kCsChunk + kCsThr) + sizeof(Tr) * 2 * kCsThr + sizeof(int) * kCsThr; }

// ---- the resolve: one wave per column ---------------------------------------------------------------
__device__ __forceinline__ Tr tr_shfl_up(const Tr& v, int o) {
  Tr u;
  u.a0 = __shfl_up(v.a0, o); u.n0 = __shfl_up(v.n0, o); u.x0 = __shfl_up(v.x0, o);
  u.a1 = __shfl_up(v.a1, o); u.n1 = __shfl_up(v.n1, o); u.x1 = __shfl_up(v.x1, o);
  return u;
}

__device__ __forceinline__ Tr tr_shfl(const Tr& v, int l) {
  Tr u;
  u.a0 = __shfl(v.a0, l); u.n0 = __shfl(v.n0, l); u.x0 = __shfl(v.x0, l);
  u.a1 = __shfl(v.a1, l); u.n1 = __shfl(v.n1, l); u.x1 = __shfl(v.x1, l);
  return u;
}

// exclusive in-order scan of one Tr per lane of a wave; *total = all 64 composed
__device__ __forceinline__ Tr cs_wave_scan(const Tr& v, Tr* total) {
  const int lane = threadIdx.x & 63;
  Tr inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const Tr up = tr_shfl_up(inc, o);
    if (lane >= o) inc = tr_compose(up, inc);
  }
  *total = tr_shfl(inc, 63);
  Tr ex = tr_shfl_up(inc, 1);
  if (lane == 0) ex = tr_ident();
  return ex;
}

__device__ __forceinline__ int cs_wave_first(bool flag) {
  const unsigned long long b = __ballot(flag);
  return b ? __builtin_ctzll(b) : 64;
}

// the wave continues column c's sequential sum s over rows [lo, hi) and returns it (every lane): passes
// of 64 x 8 terms; where the composed path leaves the binade, the lane holding that point walks its
// terms, adds the leaving one in hardware, and the pass restarts after it
__device__ float cs_walk(const float* __restrict__ X, int dim, int c, const float* __restrict__ m,
                         int64_t lo, int64_t hi, float s) {
  const int lane = threadIdx.x & 63;
  int64_t pos = lo;
  while (pos < hi) {
    if (!(fabsf(s) < __builtin_inff())) break;
    const int64_t b = pos + (int64_t)lane * kCsWalkE;
    float t[kCsWalkE];
    bool bad = false;
#pragma unroll
    for (int j = 0; j < kCsWalkE; ++j) {
      t[j] = b + j < hi ? cs_term(X, dim, b + j, c, m) : 0.f;
      bad |= !(fabsf(t[j]) < __builtin_inff());
    }
    if (__ballot(bad) != 0ull) break;
    const int e = cs_binade(s);
    const int S0 = (int)ldexpf(s, 23 - e);
    Tr f = tr_ident();
#pragma unroll
    for (int j = 0; j < kCsWalkE; ++j) {
      if (b + j < hi) {
        int q0, q1;
        term_adv2(t[j], e, q0, q1);
        f = tr_append(f, q0, q1);
      }
    }
    Tr tot;
    const Tr ex = cs_wave_scan(f, &tot);
    const int Sb = S0 + tr_adv(ex, S0);
    const bool fail = !(tr_applies(S0, e, ex) && tr_applies(Sb, e, f));
    const int cf = cs_wave_first(fail);
    if (cf == 64) {
      s = ldexpf((float)(S0 + tr_adv(tot, S0)), e - 23);
      pos += 64 * kCsWalkE;
      continue;
    }
    // lane cf: its run's prefix applies; find the term that leaves and add it in hardware
    float s_new = 0.f;
    int j_new = kCsWalkE;
    if (lane == cf) {
      int S = Sb;
      bool left = false;
#pragma unroll
      for (int j = 0; j < kCsWalkE; ++j) {
        if (!left) {
          int q0, q1;
          term_adv2(t[j], e, q0, q1);
          const Tr g = tr_append(tr_ident(), q0, q1);
          if (tr_applies(S, e, g)) {
            S += tr_adv(g, S);
          } else {
            s_new = ldexpf((float)S, e - 23) + t[j];
            j_new = j + 1;
            left = true;
          }
        }
      }
    }
    s = __shfl(s_new, cf);
    pos = pos + (int64_t)cf * kCsWalkE + __shfl(j_new, cf);
  }
  if (pos < hi) {  // non-finite terms or sum: one term at a time (rare), lane 0, then broadcast
    float r = s;
    if (lane == 0)
      for (int64_t i = pos; i < hi; ++i) r = r + cs_term(X, dim, i, c, m);
    s = __shfl(r, 0);
  }
  return s;
}

// one wave per column: windows of 64 segments, one per lane; in the current binade the segments whose
// transducer applies are scanned together, the first that does not is walked
__global__ __launch_bounds__(64) void k_cs_resolve(int64_t n, int dim, int nseg, const float* __restrict__ X,
                                                   const float* __restrict__ m, const CsRec* __restrict__ rec,
                                                   float* __restrict__ out) {
  const int c = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  CsRec nxt{};
  if (lane < nseg) nxt = rec[(int64_t)lane * dim + c];
  for (int g0 = 0; g0 < nseg; g0 += 64) {
    const int gn = min(64, nseg - g0);
    const CsRec my = nxt;
    if (g0 + 64 + lane < nseg) nxt = rec[(int64_t)(g0 + 64 + lane) * dim + c];  // the next window in flight
    int b0 = 0;
    while (b0 < gn) {
      if (!(fabsf(s) < __builtin_inff())) {  // the rest one term at a time
        s = cs_walk(X, dim, c, m, (int64_t)(g0 + b0) * kCsSeg, n, s);
        g0 = nseg;
        break;
      }
      const int e = cs_binade(s);
      const int S0 = (int)ldexpf(s, 23 - e);
      const bool mine = lane >= b0 && lane < gn;
      Tr f = tr_ident();
      bool usable = false;
      if (mine && !my.bad) {
        if (my.e[0] == e) {
          f = my.f[0];
          usable = true;
        } else if (my.e[1] == e) {
          f = my.f[1];
          usable = true;
        }
      }
      Tr tot;
      const Tr ex = cs_wave_scan(f, &tot);
      const int Sb = S0 + tr_adv(ex, S0);
      const bool fail = mine && !(usable && tr_applies(S0, e, ex) && tr_applies(Sb, e, f));
      const int cf = cs_wave_first(fail);
      if (cf == 64) {
        s = ldexpf((float)(S0 + tr_adv(tot, S0)), e - 23);
        break;
      }
      s = ldexpf((float)__shfl(Sb, cf), e - 23);  // the exact sum before segment cf
      const int64_t lo = (int64_t)(g0 + cf) * kCsSeg, hi = min<int64_t>(n, lo + kCsSeg);
      s = cs_walk(X, dim, c, m, lo, hi, s);
      b0 = cf + 1;
    }
  }
  if (lane == 0) out[c] = (float)((double)s / (double)n);  // numpy: sum / n, rounded to fp32
}

int cs_nseg(int64_t n) { return (int)((n + kCsSeg - 1) / kCsSeg); }

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" size_t gdd_center_columns_ws_bytes(int64_t n, int dim) {
  if (n < kCsMinRows || dim < 2 || dim > kCsMaxDim) return 256;
  const size_t ns = (size_t)cs_nseg(n) * (size_t)dim;
  return 2 * align256(sizeof(double) * ns) + align256(sizeof(CsRec) * ns) + 256;
}

extern "C" int gdd_center_columns_ws(int64_t n, int dim, const float* X, float* X_out, float* mean, float* var,
                                     void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && X_out && mean && var, "center_columns_ws: bad arguments");
  // GDD_FORCE=center_seq: the sequential chains (gdd_center_columns) at any shape
  if (n < kCsMinRows || dim < 2 || dim > kCsMaxDim || forced("center_seq"))
    return gdd_center_columns(n, dim, X, X_out, mean, var, stream);
  GDD_REQUIRE(ws && ws_bytes >= gdd_center_columns_ws_bytes(n, dim), "center_columns_ws: workspace too small");
  hipStream_t s = to_hip(stream);
  const int nseg = cs_nseg(n);
  const size_t ns = (size_t)nseg * (size_t)dim;
  Carver cv(ws, ws_bytes);
  double* segsum = cv.take<double>(ns);
  double* pref = cv.take<double>(ns);
  CsRec* rec = cv.take<CsRec>(ns);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "center_columns_ws: workspace too small");
  const size_t lds = cs_lds_bytes();
  for (const void* f : {(const void*)k_cs_segsum, (const void*)k_cs_records})
    GDD_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int pass = 0; pass < 2; ++pass) {
    const float* m = pass == 0 ? nullptr : mean;
    float* o = pass == 0 ? mean : var;
    k_cs_segsum<<<(unsigned)nseg, kCsThr, lds, s>>>(n, dim, X, m, pass ? X_out : nullptr, segsum);
    GDD_LAUNCHED();
    k_cs_prefix<<<(unsigned)dim, kCsThr, 0, s>>>(nseg, dim, segsum, pref);
    GDD_LAUNCHED();
    k_cs_records<<<(unsigned)nseg, kCsThr, lds, s>>>(n, dim, X, m, pref, rec);
    GDD_LAUNCHED();
    k_cs_resolve<<<(unsigned)dim, 64, 0, s>>>(n, dim, nseg, X, m, rec, o);
    GDD_LAUNCHED();
  }
  return GDD_OK;
}
