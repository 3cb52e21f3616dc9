// gdd_kmeanspp.hip — greedy k-means++ seeding on the device (sklearn _kmeans_plusplus,
// sklearn/cluster/_kmeans.py:174-272), with the host's RNG draws passed in.
//
// Two launches per seeding round c = 1..k-1, no host round trip (the chosen trial and the current
// potential live in device memory):
//   dist(c)   grid      dist[t][i] = np.minimum(closest_i, fp32(max(0, ((-2<x_cand,x_i>) +
//                       |x_cand|^2) + |x_i|^2)))   fp64 upcast distances (pairwise.py:582-650)
//   tail(c)   1 block   pot[t] = fp32 dot(dist[t], w) in OpenBLAS SkylakeX sdot order; best =
//                       first argmin; centers[c] = X[cand[best]]; then for round c+1:
//                       cum = inclusive fp64 prefix of fp32(w * dist[best])   (stable_cumsum)
//                       cand[t] = searchsorted_left(cum, u[c][t] * (double)pot), clipped to n-1
// tail(0) seeds the loop from the first centre (random_state.choice on the host). `closest` is
// never copied: round c reads dist[(c-1)&1][best_{c-1}].
#include <algorithm>
#include <cstdlib>

#include "gdd_common.hpp"

namespace gdd {
GDD_STAMP_TABLE(kpp)
namespace {

constexpr int kMaxTrials = 16;
constexpr int kTailThreads = 1024;
constexpr int kTailLdsCum = 6144;  // cumulative potential kept in LDS up to this n (48 KiB)

struct KppState {
  float pot;   // current potential (fp32, as sklearn keeps it)
  int best;    // trial chosen in the previous round; -1 = the distances to the first centre
  int64_t cand[kMaxTrials];
};

// OpenBLAS 0.3.28/29 SkylakeX sdot (kernel/x86_64/sdot.c + sdot_microk_skylakex-2.c), emulated by
// one wave: the 64 lanes are the 4 x 16 AVX-512 accumulators of the 64-wide loop (lane u*16+l
// runs accumulator u, lane l); they fold to 4 x 8 AVX2 accumulators for the 32-wide remainder;
// lanes then combine ((a0+a1)+a2)+a3, 8 -> 4 by halves, and (h0+h1)+(h2+h3); the scalar tail is
// added in double. All 64 lanes call it; lane 0 returns the value.
// The 64 lane chains of the 64-wide loop are independent: per round, k_kpp_dist runs them in the
// blocks that produce the distances (no block ever re-reads a whole distance row), and the tail
// only combines 64 accumulators per trial (sdot_skx_finish).
// the combination after the 64-wide loop: `a` = this lane's accumulator of that loop; (rx, ry) =
// element n64 + lane of x and y (zero past n). Lane 0 returns the dot.
__device__ float sdot_skx_finish(float a, float rx, float ry, int64_t n, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int64_t n1 = n & ~31ll;
  const int64_t n64 = n1 & ~63ll;
  scratch[lane] = a;
  scratch[64 + lane] = rx;
  scratch[128 + lane] = ry;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float r = 0.f;
  if (lane == 0) {
    const float* Rx = scratch + 64;
    const float* Ry = scratch + 128;
    float acc[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int l = 0; l < 8; ++l) acc[u][l] = scratch[u * 16 + l] + scratch[u * 16 + l + 8];
    if (n64 < n1) {  // at most one 32-wide block remains
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[u][l] = __builtin_fmaf(Rx[u * 8 + l], Ry[u * 8 + l], acc[u][l]);
    }
    float s[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) s[l] = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l];
    float h[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) h[l] = s[l] + s[l + 4];
    double dot = n1 ? (double)((h[0] + h[1]) + (h[2] + h[3])) : 0.0;
    for (int64_t t = n1; t < n; ++t) {
      const float p = Ry[t - n64] * Rx[t - n64];
      dot = dot + (double)p;
    }
    r = (float)dot;
  }
  return r;
}

// sdot_skx_finish with the fold done by cross-lane shuffles instead of lane 0 over LDS (same
// operations, same order); every lane returns the dot.
__device__ float sdot_skx_finish_shfl(float a, float rx, float ry, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t n1 = n & ~31ll;
  const int64_t n64 = n1 & ~63ll;
  // acc[u][l] = a[16u + l] + a[16u + l + 8], held by lane 16u + l (l < 8)
  float acc = a + __shfl_down(a, 8);
  if (n64 < n1) {  // the 32-wide block: acc[u][l] = fma(x[n64 + 8u + l], y[n64 + 8u + l], acc[u][l])
    const int src = ((lane >> 4) << 3) + (lane & 7);
    acc = __builtin_fmaf(__shfl(rx, src), __shfl(ry, src), acc);
  }
  // s[l] = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l]  (lanes 0..7)
  const float a1 = __shfl(acc, (lane + 16) & 63), a2 = __shfl(acc, (lane + 32) & 63),
              a3 = __shfl(acc, (lane + 48) & 63);
  const float sl = ((acc + a1) + a2) + a3;
  const float h = sl + __shfl(sl, (lane + 4) & 63);  // h[l] = s[l] + s[l+4]  (lanes 0..3)
  const float h0 = __shfl(h, 0), h1 = __shfl(h, 1), h2 = __shfl(h, 2), h3 = __shfl(h, 3);
  double dot = n1 ? (double)((h0 + h1) + (h2 + h3)) : 0.0;
  for (int64_t t = n1; t < n; ++t) {
    const int L = (int)(t - n64);
    const float p = __shfl(ry, L) * __shfl(rx, L);
    dot = dot + (double)p;
  }
  return (float)dot;
}

// the whole dot by one wave (used once, for the first centre's potential)
__device__ float sdot_skx_wave(const float* __restrict__ x, const float* __restrict__ y, int64_t n,
                               float* scratch /* 192 floats of LDS owned by this wave */) {
  const int lane = threadIdx.x & 63;
  const int64_t n64 = n & ~63ll;
  const int64_t ri = n64 + lane;
  const float rx = ri < n ? x[ri] : 0.f;
  const float ry = ri < n ? (y ? y[ri] : 1.0f) : 0.f;
  // y == nullptr: unit sample weights (fma(x, 1, a) == a + x, one rounding either way)
  float a = 0.f;
  for (int64_t i0 = 0; i0 < n64; i0 += 64 * 32) {
    float xv[32], yv[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int64_t i = i0 + 64 * u + lane;
      xv[u] = i < n64 ? x[i] : 0.f;
      yv[u] = (i < n64 && y) ? y[i] : 1.0f;
    }
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (i0 + 64 * u < n64) a = __builtin_fmaf(xv[u], yv[u], a);
  }
  return sdot_skx_finish(a, rx, ry, n, scratch);
}

__device__ __forceinline__ float np_minimum(float a, float b) {
  if (a != a || b != b) return __builtin_nanf("");
  return b < a ? b : a;
}

// |x|^2 in fp64 (row_norms of the upcast chunk) and the distances to the first center
__global__ void k_kpp_init(int64_t n, int dim, const float* __restrict__ X, int64_t first_id,
                           double* __restrict__ xsq, float* __restrict__ closest) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* xi = X + i * dim;
  const float* xc = X + first_id * dim;
  double s = 0.0, sc = 0.0, dot = 0.0;
  for (int j = 0; j < dim; ++j) {
    const double v = (double)xi[j], c = (double)xc[j];
    s = __builtin_fma(v, v, s);
    sc = __builtin_fma(c, c, sc);
    dot = __builtin_fma(c, v, dot);
  }
  xsq[i] = s;
  const float f = (float)(((-2.0 * dot) + sc) + s);
  closest[i] = f < 0.f ? 0.f : f;
}

// Round c: distances of every point to trial t's candidate (fp64 upcast, pairwise.py:582-650),
// np.minimum with the current closest distances, and the 64-wide-loop chains of the potential's
// sdot. Grid (G, T): block (g, t) owns the sdot lanes l in [g*L, (g+1)*L), L = 64/G, i.e. the
// points i = l + 64 j, j < J = n64/64; it writes their distances to dist[t][i] (the tail's cumsum
// reads one row), runs its lanes' ordered fp32 chains over them and leaves acc[t][l]. Block 0 also
// writes the remainder points n64 <= i < n. The candidate row is staged in LDS as fp64.
template <bool kChainLds>
__global__ __launch_bounds__(256) void k_kpp_dist(int64_t n, int dim, const float* __restrict__ X,
                                                  const float* __restrict__ w,
                                                  const double* __restrict__ xsq,
                                                  const float* __restrict__ closest0,
                                                  const float* __restrict__ dist_prev,
                                                  const KppState* __restrict__ st,
                                                  float* __restrict__ dist, float* __restrict__ acc,
                                                  int L) {
  GDD_STAMP_WHEN(g_stamps_kpp, (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0), 20);
  extern __shared__ double s_c[];  // dim doubles, then the block's chain distances (fp32)
  const int t = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  const int64_t J = n >> 6, n64 = J << 6;
  const int64_t nloc = (int64_t)L * J;
  const int64_t ntot = nloc + (g == 0 ? n - n64 : 0);
  const int best = st->best;
  const int64_t ct = st->cand[t];
  const double cn = xsq[ct];
  const float* closest = best < 0 ? closest0 : dist_prev + (int64_t)best * n;
  for (int j = tid; j < dim; j += blockDim.x) s_c[j] = (double)X[ct * dim + j];
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0), 21);
  float* sd = reinterpret_cast<float*>(s_c + dim);
  float* drow = dist + (int64_t)t * n;
  for (int64_t q = tid; q < ntot; q += blockDim.x) {
    int64_t i;
    if (q < nloc) {
      const int64_t j = q / L;
      i = (int64_t)g * L + (q - j * L) + 64 * j;
    } else {
      i = n64 + (q - nloc);
    }
    const float* xi = X + i * dim;
    const double xs = xsq[i];
    const float cl = closest[i];
    double dot = 0.0;
    int j = 0;
    for (; j + 8 <= dim; j += 8) {  // eight loads in flight ahead of the ordered fmas
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xi[j + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) dot = __builtin_fma(s_c[j + u], (double)v[u], dot);
    }
    for (; j < dim; ++j) dot = __builtin_fma(s_c[j], (double)xi[j], dot);
    const double d = ((-2.0 * dot) + cn) + xs;
    float f = (float)d;
    f = f < 0.f ? 0.f : f;
    f = np_minimum(cl, f);
    drow[i] = f;
    if (kChainLds && q < nloc) sd[q] = f;
  }
  __syncthreads();  // also orders this block's global writes for the chain reads below
  GDD_STAMP_WHEN(g_stamps_kpp, (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0), 22);
  if (tid < L) {
    const int l = g * L + tid;
    float a = 0.f;
    int64_t j = 0;
    for (; j + 8 <= J; j += 8) {
      float xv[8], yv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t i = l + 64 * (j + u);
        xv[u] = kChainLds ? sd[(j + u) * L + tid] : drow[i];
        yv[u] = w ? w[i] : 1.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a = __builtin_fmaf(xv[u], yv[u], a);
    }
    for (; j < J; ++j) {
      const int64_t i = l + 64 * j;
      a = __builtin_fmaf(kChainLds ? sd[j * L + tid] : drow[i], w ? w[i] : 1.0f, a);
    }
    acc[t * 64 + l] = a;
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0), 23);
}

// end of round c (c = 0: the first centre) and the candidate draw of round c+1
__global__ __launch_bounds__(kTailThreads) void k_kpp_tail(
    int64_t n, int dim, const float* __restrict__ X, const float* __restrict__ w,
    const float* __restrict__ closest0, const float* __restrict__ dist,
    const float* __restrict__ acc, int T, int c, int k,
    int64_t first_id, const double* __restrict__ uniforms, const double* __restrict__ xsq,
    double* __restrict__ cum, float* __restrict__ centers, int64_t* __restrict__ indices,
    KppState* __restrict__ st) {
  __shared__ float scratch[kMaxTrials * 192];
  __shared__ float s_pot[kMaxTrials];
  __shared__ double s_part[kTailThreads / 64];
  __shared__ double s_cum[kTailLdsCum];
  __shared__ int s_best;
  __shared__ int64_t s_src;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 0 + 10 * (c & 1));
  // this round's draw for the next candidates, requested up front
  const double u_mine = (tid < T && c + 1 < k) ? uniforms[(int64_t)c * T + tid] : 0.0;
  // ---- finish round c ----
  if (c == 0) {
    if (wave == 0) {
      const float p = sdot_skx_wave(closest0, w, n, scratch);  // closest_dist_sq @ sample_weight
      if (tid == 0) s_pot[0] = p;
    }
    __syncthreads();
    if (tid == 0) {
      s_best = -1;
      s_src = first_id;
      st->best = -1;
      st->pot = s_pot[0];
      indices[0] = first_id;
    }
  } else {
    if (wave < T) {
      const int lane = tid & 63;
      const int64_t ri = (n & ~63ll) + lane;
      const float rx = ri < n ? dist[(int64_t)wave * n + ri] : 0.f;
      const float ry = ri < n ? (w ? w[ri] : 1.0f) : 0.f;
      const float p = sdot_skx_finish(acc[wave * 64 + lane], rx, ry, n, scratch + wave * 192);
      if (lane == 0) s_pot[wave] = p;
    }
    __syncthreads();
    GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 1 + 10 * (c & 1));
    if (tid == 0) {
      int b = 0;  // np.argmin: first minimum; a NaN is returned as soon as it is met
      for (int t = 1; t < T; ++t) {
        const float pb = s_pot[b], pt = s_pot[t];
        if (pb == pb && (pt < pb || pt != pt)) b = t;
      }
      s_best = b;
      s_src = st->cand[b];
      st->best = b;
      st->pot = s_pot[b];
      indices[c] = st->cand[b];
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 2 + 10 * (c & 1));
  for (int j = tid; j < dim; j += kTailThreads) centers[(int64_t)c * dim + j] = X[s_src * dim + j];
  if (c + 1 >= k) return;
  // ---- candidates of round c+1 ----
  const float* closest = s_best < 0 ? closest0 : dist + (int64_t)s_best * n;
  const int64_t chunk = (n + kTailThreads - 1) / kTailThreads;
  const int64_t lo = min<int64_t>(n, tid * chunk), hi = min<int64_t>(n, lo + chunk);
  // fp32 products w_i * closest_i of this thread's chunk (kept in registers when it is short)
  constexpr int kReg = 8;
  float pr[kReg];
#pragma unroll
  for (int u = 0; u < kReg; ++u) {
    const int64_t i = lo + u;
    pr[u] = (chunk <= kReg && i < hi) ? (w ? w[i] : 1.0f) * closest[i] : 0.f;
  }
  double run = 0.0;
  if (chunk <= kReg) {
#pragma unroll
    for (int u = 0; u < kReg; ++u)
      if (lo + u < hi) run = run + (double)pr[u];
  } else {
    for (int64_t i = lo; i < hi; ++i) run = run + (double)((w ? w[i] : 1.0f) * closest[i]);
  }
  // exclusive scan of the per-thread chunk totals: wave shuffles, then the 16 wave totals
  const int lane = tid & 63;
  double incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_part[wave] = incl;
  __syncthreads();
  if (tid == 0) {
    double a = 0.0;
    for (int q = 0; q < kTailThreads / 64; ++q) {
      const double t = s_part[q];
      s_part[q] = a;
      a += t;
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 4 + 10 * (c & 1));
  double base = s_part[wave] + (incl - run);
  // small n: the cumulative potential stays in LDS for the binary searches
  double* cs = (n <= kTailLdsCum) ? s_cum : cum;
  if (chunk <= kReg) {
#pragma unroll
    for (int u = 0; u < kReg; ++u)
      if (lo + u < hi) {
        base = base + (double)pr[u];
        cs[lo + u] = base;
      }
  } else {
    for (int64_t i = lo; i < hi; ++i) {
      base = base + (double)((w ? w[i] : 1.0f) * closest[i]);
      cs[i] = base;
    }
  }
  __threadfence_block();
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 5 + 10 * (c & 1));
  if (tid < T) {
    const double r = u_mine * (double)s_pot[s_best < 0 ? 0 : s_best];
    int64_t a = 0, b = n;  // first index with cum[idx] >= r  (np.searchsorted side='left')
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (cs[m] < r)
        a = m + 1;
      else
        b = m;
    }
    if (a > n - 1) a = n - 1;
    st->cand[tid] = a;
  }
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 6 + 10 * (c & 1));
}

// Rounds c >= 1 when every thread's share of a distance row fits in registers (chunk <= kR) and
// T <= kTT. Everything the round needs is requested up front: the lane accumulators and
// remainders for the potentials and every trial's slice of its distance row, so the cumulative
// potential of the winning trial starts as soon as the argmin is known; the binary searches are
// replaced by counts (cum is non-decreasing: searchsorted_left(cum, r) = #{i : cum[i] < r}).
template <int kTT, int kR>
__global__ __launch_bounds__(kTailThreads) void k_kpp_tail_fast(
    int64_t n, int dim, const float* __restrict__ X, const float* __restrict__ w,
    const float* __restrict__ dist, const float* __restrict__ acc, int T, int c, int k,
    const double* __restrict__ uniforms, float* __restrict__ centers,
    int64_t* __restrict__ indices, KppState* __restrict__ st) {
  __shared__ float s_pot[kMaxTrials];
  __shared__ double s_r[kMaxTrials];
  __shared__ double s_part[kTailThreads / 64];
  __shared__ int s_cnt[kMaxTrials][kTailThreads / 64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 0 + 10 * (c & 1));
  const bool more = c + 1 < k;
  const double u_mine = (tid < T && more) ? uniforms[(int64_t)c * T + tid] : 0.0;
  const int64_t chunk = (n + kTailThreads - 1) / kTailThreads;
  const int64_t lo = min<int64_t>(n, tid * chunk), hi = min<int64_t>(n, lo + chunk);
  float wv[kR];
#pragma unroll
  for (int u = 0; u < kR; ++u) wv[u] = (w && lo + u < hi) ? w[lo + u] : 1.0f;
  // potentials of the T trials
  if (wave < T) {
    const int64_t ri = (n & ~63ll) + lane;
    const float rx = ri < n ? dist[(int64_t)wave * n + ri] : 0.f;
    const float ry = ri < n ? (w ? w[ri] : 1.0f) : 0.f;
    const float p = sdot_skx_finish_shfl(acc[wave * 64 + lane], rx, ry, n);
    if (lane == 0) s_pot[wave] = p;
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 1 + 10 * (c & 1));
  int b = 0;  // np.argmin: first minimum; a NaN is returned as soon as it is met
  for (int t = 1; t < T; ++t) {
    const float pb = s_pot[b], pt = s_pot[t];
    if (pb == pb && (pt < pb || pt != pt)) b = t;
  }
  const float pot = s_pot[b];
  const int64_t src = st->cand[b];
  if (tid == 0) {
    st->best = b;
    st->pot = pot;
    indices[c] = src;
  }
  if (tid < T) s_r[tid] = u_mine * (double)pot;
  for (int j = tid; j < dim; j += kTailThreads) centers[(int64_t)c * dim + j] = X[src * dim + j];
  if (!more) return;
  // cumulative potential of the winning trial (fp64 of the fp32 products w_i * closest_i)
  float pr[kR];
  const float* row = dist + (int64_t)b * n;
#pragma unroll
  for (int u = 0; u < kR; ++u) pr[u] = (lo + u < hi) ? wv[u] * row[lo + u] : 0.f;
  double run = 0.0;
#pragma unroll
  for (int u = 0; u < kR; ++u)
    if (lo + u < hi) run = run + (double)pr[u];
  double incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_part[wave] = incl;
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 4 + 10 * (c & 1));
  double base = incl - run;
  for (int q = 0; q < wave; ++q) base += s_part[q];
  // counts of cum[i] < r_t over the wave's entries (one ballot per entry slot and trial)
  double cu[kR];
#pragma unroll
  for (int u = 0; u < kR; ++u) {
    base = base + (double)pr[u];
    cu[u] = base;
  }
#pragma unroll
  for (int t = 0; t < kTT; ++t) {
    if (t < T) {
      const double r = s_r[t];
      int cw = 0;
#pragma unroll
      for (int u = 0; u < kR; ++u) cw += __popcll(__ballot(lo + u < hi && cu[u] < r));
      if (lane == 0) s_cnt[t][wave] = cw;
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 5 + 10 * (c & 1));
  if (tid < T) {
    int64_t a = 0;
    for (int q = 0; q < kTailThreads / 64; ++q) a += s_cnt[tid][q];
    if (a > n - 1) a = n - 1;
    st->cand[tid] = a;
  }
  GDD_STAMP_WHEN(g_stamps_kpp, tid == 0, 6 + 10 * (c & 1));
}

// ---- speculative candidate draws -----------------------------------------------------------------
// Round c's tail used to be serial: potentials -> argmin -> the winning trial's cumulative potential
// -> the next candidates. But every trial t already has its own row dist[t] (the closest distances
// if t wins), so the next round's candidates can be drawn for EVERY possible winner, in parallel,
// one workgroup per trial: next[t][j] = searchsorted(cumsum(w * dist[t]), u[c][j] * pot[t]). The
// next distance launch then reads the T potentials, takes the argmin b (first minimum, NaN first as
// np.argmin) and uses next[b][*] — the argmin and its dependent row read leave the critical path.
struct KppSpec {
  float pot[2][kMaxTrials];                   // by round parity: potentials of that round's trials
  int64_t cand[2][kMaxTrials];                // by round parity: that round's candidates
  int64_t next[2][kMaxTrials][kMaxTrials];    // next[p][t][j]: round c+1's trial j if t wins round c
};

__device__ __forceinline__ int kpp_argmin(const float* pot, int T) {
  int b = 0;
  for (int t = 1; t < T; ++t) {
    const float pb = pot[b], pt = pot[t];
    if (pb == pb && (pt < pb || pt != pt)) b = t;
  }
  return b;
}

// round 0 (the tail of the first centre, from KppState) seeds round 1: one "trial" that always wins
__global__ void k_kpp_spec_seed(const KppState* __restrict__ st, int T, KppSpec* __restrict__ sp) {
  const int j = threadIdx.x;
  if (j < kMaxTrials) {
    sp->pot[0][j] = j == 0 ? st->pot : __builtin_inff();
    if (j < T) sp->next[0][0][j] = st->cand[j];
  }
}

// round c >= 1, workgroup (g, t): the winner of round c-1, this trial's candidate, then the
// distance phase (kpp_dist_phase's work) with the candidate passed in
__global__ __launch_bounds__(256) void k_kpp_dist_spec(
    int64_t n, int dim, const float* __restrict__ X, const float* __restrict__ w,
    const double* __restrict__ xsq, const float* __restrict__ closest0,
    const float* __restrict__ dist_prev, KppSpec* __restrict__ sp, float* __restrict__ dist,
    float* __restrict__ acc, int L, int T, int c, float* __restrict__ centers,
    int64_t* __restrict__ indices) {
  extern __shared__ double s_c[];
  const int t = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  const int pp = (c - 1) & 1;
  const int b = kpp_argmin(sp->pot[pp], T);
  const int64_t ct = sp->next[pp][b][t];
  if (g == 0 && tid == 0) sp->cand[c & 1][t] = ct;
  if (c >= 2 && g == 0 && t == 0) {  // round c-1's centre (round 0's is written by its tail)
    const int64_t src = sp->cand[pp][b];
    if (tid == 0) indices[c - 1] = src;
    for (int j = tid; j < dim; j += blockDim.x) centers[(int64_t)(c - 1) * dim + j] = X[src * dim + j];
  }
  const int64_t J = n >> 6, n64 = J << 6;
  const int64_t nloc = (int64_t)L * J;
  const int64_t ntot = nloc + (g == 0 ? n - n64 : 0);
  const double cn = xsq[ct];
  const float* closest = c == 1 ? closest0 : dist_prev + (int64_t)b * n;
  for (int j = tid; j < dim; j += blockDim.x) s_c[j] = (double)X[ct * dim + j];
  __syncthreads();
  float* sd = reinterpret_cast<float*>(s_c + dim);
  float* drow = dist + (int64_t)t * n;
  for (int64_t q = tid; q < ntot; q += blockDim.x) {
    int64_t i;
    if (q < nloc) {
      const int64_t j = q / L;
      i = (int64_t)g * L + (q - j * L) + 64 * j;
    } else {
      i = n64 + (q - nloc);
    }
    const float* xi = X + i * dim;
    const double xs = xsq[i];
    const float cl = closest[i];
    double dot = 0.0;
    int j = 0;
    for (; j + 8 <= dim; j += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xi[j + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) dot = __builtin_fma(s_c[j + u], (double)v[u], dot);
    }
    for (; j < dim; ++j) dot = __builtin_fma(s_c[j], (double)xi[j], dot);
    const double d = ((-2.0 * dot) + cn) + xs;
    float f = (float)d;
    f = f < 0.f ? 0.f : f;
    f = np_minimum(cl, f);
    drow[i] = f;
    if (q < nloc) sd[q] = f;
  }
  __syncthreads();
  if (tid < L) {
    const int l = g * L + tid;
    float a = 0.f;
    int64_t j = 0;
    for (; j + 8 <= J; j += 8) {
      float xv[8], yv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        xv[u] = sd[(j + u) * L + tid];
        yv[u] = w ? w[l + 64 * (j + u)] : 1.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a = __builtin_fmaf(xv[u], yv[u], a);
    }
    for (; j < J; ++j) a = __builtin_fmaf(sd[j * L + tid], w ? w[l + 64 * j] : 1.0f, a);
    acc[t * 64 + l] = a;
  }
}

// round c, workgroup t: this trial's potential and, unless c is the last round, the next round's
// candidates should t win (counts over this trial's cumulative potential, as k_kpp_tail_fast)
template <int kR>
__global__ __launch_bounds__(kTailThreads) void k_kpp_trial_tail(
    int64_t n, const float* __restrict__ w, const float* __restrict__ dist,
    const float* __restrict__ acc, int T, int c, int k, const double* __restrict__ uniforms,
    KppSpec* __restrict__ sp) {
  __shared__ float s_pot;
  __shared__ double s_r[kMaxTrials];
  __shared__ double s_part[kTailThreads / 64];
  __shared__ int s_cnt[kMaxTrials][kTailThreads / 64];
  const int t = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int p = c & 1;
  const bool more = c + 1 < k;
  const double u_mine = (tid < T && more) ? uniforms[(int64_t)c * T + tid] : 0.0;
  const int64_t chunk = (n + kTailThreads - 1) / kTailThreads;
  const int64_t lo = min<int64_t>(n, tid * chunk), hi = min<int64_t>(n, lo + chunk);
  const float* row = dist + (int64_t)t * n;
  float pr[kR];
#pragma unroll
  for (int u = 0; u < kR; ++u)
    pr[u] = (more && lo + u < hi) ? (w ? w[lo + u] : 1.0f) * row[lo + u] : 0.f;
  if (wave == 0) {
    const int64_t ri = (n & ~63ll) + lane;
    const float rx = ri < n ? row[ri] : 0.f;
    const float ry = ri < n ? (w ? w[ri] : 1.0f) : 0.f;
    const float pt = sdot_skx_finish_shfl(acc[t * 64 + lane], rx, ry, n);
    if (lane == 0) {
      s_pot = pt;
      sp->pot[p][t] = pt;
    }
  }
  if (!more) return;
  double run = 0.0;
#pragma unroll
  for (int u = 0; u < kR; ++u)
    if (lo + u < hi) run = run + (double)pr[u];
  double incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_part[wave] = incl;
  __syncthreads();  // s_pot, s_part
  if (tid < T) s_r[tid] = u_mine * (double)s_pot;
  // exclusive prefix of the wave totals: lanes 0..15 scan them, every lane takes its wave's entry
  double wp = lane < kTailThreads / 64 ? s_part[lane] : 0.0;
  double wincl = wp;
#pragma unroll
  for (int o = 1; o < kTailThreads / 64; o <<= 1) {
    const double v = __shfl_up(wincl, o);
    if (lane >= o) wincl += v;
  }
  double base = (incl - run) + (wave > 0 ? __shfl(wincl, wave - 1) : 0.0);
  double cu[kR];
#pragma unroll
  for (int u = 0; u < kR; ++u) {
    base = base + (double)pr[u];
    cu[u] = base;
  }
  __syncthreads();  // s_r
  for (int j = 0; j < T; ++j) {
    const double r = s_r[j];
    int cw = 0;
#pragma unroll
    for (int u = 0; u < kR; ++u) cw += __popcll(__ballot(lo + u < hi && cu[u] < r));
    if (lane == 0) s_cnt[j][wave] = cw;
  }
  __syncthreads();
  if (tid < T) {
    int64_t a = 0;
    for (int q = 0; q < kTailThreads / 64; ++q) a += s_cnt[tid][q];
    if (a > n - 1) a = n - 1;
    sp->next[p][t][tid] = a;
  }
}

// after the last round: its winner is the last centre
__global__ void k_kpp_spec_finish(int dim, const float* __restrict__ X, const KppSpec* __restrict__ sp,
                                  int T, int c, float* __restrict__ centers,
                                  int64_t* __restrict__ indices) {
  const int p = c & 1;
  const int b = kpp_argmin(sp->pot[p], T);
  const int64_t src = sp->cand[p][b];
  if (threadIdx.x == 0) indices[c] = src;
  for (int j = threadIdx.x; j < dim; j += blockDim.x) centers[(int64_t)c * dim + j] = X[src * dim + j];
}

// ---- one launch per round ---------------------------------------------------------------------
// Round c's launch also finishes round c-1: every workgroup folds the previous round's lane
// accumulators into the T potentials (redundantly, from 2 KB), takes the argmin b, scans the
// winner's row dist_prev[b] into the fp64 cumulative potential and draws ITS trial's candidate by
// counting (searchsorted_left), then runs the distance phase for that candidate. One launch and
// three dependent memory trips per round (accumulators, winner's row, candidate row) instead of two
// launches with a single-workgroup tail between them. Workgroup (0, 0) writes round c-1's centre.
// Needs chunk = ceil(n / 256) <= kR (each thread scans <= kR consecutive entries of the row).
template <int kR, int kPre>
__global__ __launch_bounds__(256) void k_kpp_round(
    int64_t n, int dim, const float* __restrict__ X, const float* __restrict__ w,
    const double* __restrict__ xsq, const float* __restrict__ closest0,
    const float* __restrict__ dist_prev, float* __restrict__ dist_cur,
    const float* __restrict__ acc_prev, float* __restrict__ acc_cur, int L, int T, int c,
    const double* __restrict__ uniforms, const KppState* __restrict__ st,
    const int64_t* __restrict__ cand_prev, int64_t* __restrict__ cand_cur,
    float* __restrict__ centers, int64_t* __restrict__ indices) {
  extern __shared__ double s_c[];  // dim doubles, then the chain distances (fp32)
  __shared__ float s_pot[kMaxTrials];
  __shared__ double s_part[4];
  __shared__ int s_cnt[4];
  const int t = blockIdx.y, g = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nw = blockDim.x >> 6;
  const double u = uniforms[(int64_t)(c - 1) * T + t];
  // this workgroup's points (strided lanes, see k_kpp_dist) and, with kPre, their rows requested now
  const int64_t J = n >> 6, n64 = J << 6;
  const int64_t nloc = (int64_t)L * J;
  const int64_t ntot = nloc + (g == 0 ? n - n64 : 0);
  auto point_of = [&](int64_t q) -> int64_t {
    if (q < nloc) {
      const int64_t j = q / L;
      return (int64_t)g * L + (q - j * L) + 64 * j;
    }
    return n64 + (q - nloc);
  };
  float xr[kPre > 0 ? kPre : 1];
  double xs0 = 0.0;
  const int64_t i0 = tid < ntot ? point_of(tid) : 0;
  auto prefetch_rows = [&]() {  // dim % 4 == 0 (host-checked): float4 loads
    if (kPre > 0 && tid < ntot) {
      const float4* xi = reinterpret_cast<const float4*>(X + i0 * dim);
#pragma unroll
      for (int j = 0; j < (kPre > 0 ? kPre : 4) / 4; ++j) {
        const float4 v = 4 * j < dim ? xi[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        xr[4 * j] = v.x;
        xr[4 * j + 1] = v.y;
        xr[4 * j + 2] = v.z;
        xr[4 * j + 3] = v.w;
      }
      xs0 = xsq[i0];
    }
  };
  // ---- previous round's potentials and winner (round 0: the first centre's potential)
  if (c == 1) {
    if (tid == 0) s_pot[0] = st->pot;
    prefetch_rows();
  } else {
    // the potentials' inputs are requested before the point rows, so they land first
    float a_in[kMaxTrials / 4], rx_in[kMaxTrials / 4];
    const int64_t ri = (n & ~63ll) + lane;
    const float ry = ri < n ? (w ? w[ri] : 1.0f) : 0.f;
#pragma unroll
    for (int q = 0; q < kMaxTrials / 4; ++q) {
      const int tr = wave + q * 4;
      a_in[q] = tr < T ? acc_prev[tr * 64 + lane] : 0.f;
      rx_in[q] = (tr < T && ri < n) ? dist_prev[(int64_t)tr * n + ri] : 0.f;
    }
    prefetch_rows();
#pragma unroll
    for (int q = 0; q < kMaxTrials / 4; ++q) {
      const int tr = wave + q * 4;
      if (tr < T) {
        const float p = sdot_skx_finish_shfl(a_in[q], rx_in[q], ry, n);
        if (lane == 0) s_pot[tr] = p;
      }
    }
  }
  __syncthreads();
  const int b = c == 1 ? 0 : kpp_argmin(s_pot, T);
  const double r = u * (double)s_pot[b];
  const float* row = c == 1 ? closest0 : dist_prev + (int64_t)b * n;
  const float cl0 = (kPre > 0 && tid < ntot) ? row[i0] : 0.f;
  // ---- the winner's cumulative potential, scanned in place; this trial's candidate by counting
  const int64_t chunk = (n + blockDim.x - 1) / blockDim.x;
  const int64_t lo = min<int64_t>(n, tid * chunk), hi = min<int64_t>(n, lo + chunk);
  float pr[kR];
#pragma unroll
  for (int q = 0; q < kR; ++q) pr[q] = (lo + q < hi) ? (w ? w[lo + q] : 1.0f) * row[lo + q] : 0.f;
  double run = 0.0;
#pragma unroll
  for (int q = 0; q < kR; ++q)
    if (lo + q < hi) run = run + (double)pr[q];
  double incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_part[wave] = incl;
  __syncthreads();
  double base = incl - run;
  for (int q = 0; q < wave; ++q) base += s_part[q];
  int cw = 0;
#pragma unroll
  for (int q = 0; q < kR; ++q) {
    base = base + (double)pr[q];
    cw += __popcll(__ballot(lo + q < hi && base < r));
  }
  if (lane == 0) s_cnt[wave] = cw;
  __syncthreads();
  int64_t ct = 0;
  for (int q = 0; q < nw; ++q) ct += s_cnt[q];
  if (ct > n - 1) ct = n - 1;
  if (g == 0 && tid == 0) cand_cur[t] = ct;
  if (c >= 2 && g == 0 && t == 0) {  // round c-1's centre (round 0's is written by its tail)
    const int64_t src = cand_prev[b];
    if (tid == 0) indices[c - 1] = src;
    for (int j = tid; j < dim; j += blockDim.x) centers[(int64_t)(c - 1) * dim + j] = X[src * dim + j];
  }
  // ---- distances to this trial's candidate, np.minimum with the winner's row, lane chains
  const double cn = xsq[ct];
  for (int j = tid; j < dim; j += blockDim.x) s_c[j] = (double)X[ct * dim + j];
  __syncthreads();
  float* sd = reinterpret_cast<float*>(s_c + dim);
  float* drow = dist_cur + (int64_t)t * n;
  if (kPre > 0) {  // one point per thread, row already in registers
    if (tid < ntot) {
      double dot = 0.0;
#pragma unroll
      for (int j = 0; j < (kPre > 0 ? kPre : 1); ++j)
        if (j < dim) dot = __builtin_fma(s_c[j], (double)xr[j], dot);
      const double d = ((-2.0 * dot) + cn) + xs0;
      float f = (float)d;
      f = f < 0.f ? 0.f : f;
      f = np_minimum(cl0, f);
      drow[i0] = f;
      if (tid < nloc) sd[tid] = f;
    }
  } else
  for (int64_t q = tid; q < ntot; q += blockDim.x) {
    const int64_t i = point_of(q);
    const float* xi = X + i * dim;
    const double xs = xsq[i];
    const float cl = row[i];
    double dot = 0.0;
    int j = 0;
    for (; j + 8 <= dim; j += 8) {
      float v[8];
#pragma unroll
      for (int uu = 0; uu < 8; ++uu) v[uu] = xi[j + uu];
#pragma unroll
      for (int uu = 0; uu < 8; ++uu) dot = __builtin_fma(s_c[j + uu], (double)v[uu], dot);
    }
    for (; j < dim; ++j) dot = __builtin_fma(s_c[j], (double)xi[j], dot);
    const double d = ((-2.0 * dot) + cn) + xs;
    float f = (float)d;
    f = f < 0.f ? 0.f : f;
    f = np_minimum(cl, f);
    drow[i] = f;
    if (q < nloc) sd[q] = f;
  }
  __syncthreads();
  if (tid < L) {
    const int l = g * L + tid;
    float a = 0.f;
    int64_t j = 0;
    for (; j + 8 <= J; j += 8) {
      float xv[8], yv[8];
#pragma unroll
      for (int uu = 0; uu < 8; ++uu) {
        xv[uu] = sd[(j + uu) * L + tid];
        yv[uu] = w ? w[l + 64 * (j + uu)] : 1.0f;
      }
#pragma unroll
      for (int uu = 0; uu < 8; ++uu) a = __builtin_fmaf(xv[uu], yv[uu], a);
    }
    for (; j < J; ++j) a = __builtin_fmaf(sd[j * L + tid], w ? w[l + 64 * j] : 1.0f, a);
    acc_cur[t * 64 + l] = a;
  }
}

// after the last round: its potentials, winner and centre
__global__ __launch_bounds__(256) void k_kpp_round_final(
    int64_t n, int dim, const float* __restrict__ X, const float* __restrict__ w,
    const float* __restrict__ dist, const float* __restrict__ acc, int T, int c,
    const int64_t* __restrict__ cand, float* __restrict__ centers, int64_t* __restrict__ indices) {
  __shared__ float s_pot[kMaxTrials];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  for (int tr = wave; tr < T; tr += nw) {
    const int64_t ri = (n & ~63ll) + lane;
    const float rx = ri < n ? dist[(int64_t)tr * n + ri] : 0.f;
    const float ry = ri < n ? (w ? w[ri] : 1.0f) : 0.f;
    const float p = sdot_skx_finish_shfl(acc[tr * 64 + lane], rx, ry, n);
    if (lane == 0) s_pot[tr] = p;
  }
  __syncthreads();
  const int b = kpp_argmin(s_pot, T);
  const int64_t src = cand[b];
  if (tid == 0) indices[c] = src;
  for (int j = tid; j < dim; j += blockDim.x) centers[(int64_t)c * dim + j] = X[src * dim + j];
}

// ---- all rounds in one launch ------------------------------------------------------------------
// The same two phases per round, inside one persistent launch of G*T workgroups (<= 256, one per
// CU, so all are resident): every workgroup runs its slice of the distance phase, releases its
// writes and arrives on a counter; the last arriver runs the tail (potentials, argmin, cumulative
// potential, next candidates) and publishes the next round number; the others wait for it. This
// removes two launch ramps and a dependent kernel boundary per round, but each round then pays two
// agent-scope fences per workgroup; see the launcher for the measurement. Every wait is bounded:
// a workgroup that waits too long sets `err` and leaves.
struct KppSync {
  unsigned int arrive;  // arrivals so far (NB per round)
  unsigned int round;   // candidates published for this round
  unsigned int err;
  unsigned int pad;
};

__device__ __forceinline__ bool kpp_wait_round(KppSync* sy, unsigned c) {
  unsigned long long spins = 0;
  while (__hip_atomic_load(&sy->round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < c) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1ull << 22)) return false;
  }
  return true;
}

// distance phase of workgroup (g, t): as k_kpp_dist with the chain distances in LDS
__device__ void kpp_dist_phase(int64_t n, int dim, const float* __restrict__ X,
                               const float* __restrict__ w, const double* __restrict__ xsq,
                               const float* __restrict__ closest0, const float* __restrict__ dist_prev,
                               const KppState* __restrict__ st, float* __restrict__ dist,
                               float* __restrict__ acc, int L, int t, int g, double* s_c) {
  const int tid = threadIdx.x;
  const int64_t J = n >> 6, n64 = J << 6;
  const int64_t nloc = (int64_t)L * J;
  const int64_t ntot = nloc + (g == 0 ? n - n64 : 0);
  const int best = st->best;
  const int64_t ct = st->cand[t];
  const double cn = xsq[ct];
  const float* closest = best < 0 ? closest0 : dist_prev + (int64_t)best * n;
  for (int j = tid; j < dim; j += blockDim.x) s_c[j] = (double)X[ct * dim + j];
  __syncthreads();
  float* sd = reinterpret_cast<float*>(s_c + dim);
  float* drow = dist + (int64_t)t * n;
  for (int64_t q = tid; q < ntot; q += blockDim.x) {
    int64_t i;
    if (q < nloc) {
      const int64_t j = q / L;
      i = (int64_t)g * L + (q - j * L) + 64 * j;
    } else {
      i = n64 + (q - nloc);
    }
    const float* xi = X + i * dim;
    const double xs = xsq[i];
    const float cl = closest[i];
    double dot = 0.0;
    int j = 0;
    for (; j + 8 <= dim; j += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xi[j + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) dot = __builtin_fma(s_c[j + u], (double)v[u], dot);
    }
    for (; j < dim; ++j) dot = __builtin_fma(s_c[j], (double)xi[j], dot);
    const double d = ((-2.0 * dot) + cn) + xs;
    float f = (float)d;
    f = f < 0.f ? 0.f : f;
    f = np_minimum(cl, f);
    drow[i] = f;
    if (q < nloc) sd[q] = f;
  }
  __syncthreads();
  if (tid < L) {
    const int l = g * L + tid;
    float a = 0.f;
    int64_t j = 0;
    for (; j + 8 <= J; j += 8) {
      float xv[8], yv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        xv[u] = sd[(j + u) * L + tid];
        yv[u] = w ? w[l + 64 * (j + u)] : 1.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a = __builtin_fmaf(xv[u], yv[u], a);
    }
    for (; j < J; ++j) a = __builtin_fmaf(sd[j * L + tid], w ? w[l + 64 * j] : 1.0f, a);
    acc[t * 64 + l] = a;
  }
}

// tail phase by one 256-thread workgroup (each thread owns <= kR consecutive points of a row)
template <int kR>
__device__ void kpp_tail_phase(int64_t n, int dim, const float* __restrict__ X,
                               const float* __restrict__ w, const float* __restrict__ dist,
                               const float* __restrict__ acc, int T, int c, int k,
                               const double* __restrict__ uniforms, float* __restrict__ centers,
                               int64_t* __restrict__ indices, KppState* __restrict__ st,
                               float* s_pot, double* s_r, double* s_part, int* s_cnt) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  const bool more = c + 1 < k;
  const double u_mine = (tid < T && more) ? uniforms[(int64_t)c * T + tid] : 0.0;
  for (int tr = wave; tr < T; tr += nw) {
    const int64_t ri = (n & ~63ll) + lane;
    const float rx = ri < n ? dist[(int64_t)tr * n + ri] : 0.f;
    const float ry = ri < n ? (w ? w[ri] : 1.0f) : 0.f;
    const float p = sdot_skx_finish_shfl(acc[tr * 64 + lane], rx, ry, n);
    if (lane == 0) s_pot[tr] = p;
  }
  __syncthreads();
  int b = 0;  // np.argmin: first minimum; a NaN is returned as soon as it is met
  for (int t = 1; t < T; ++t) {
    const float pb = s_pot[b], pt = s_pot[t];
    if (pb == pb && (pt < pb || pt != pt)) b = t;
  }
  const float pot = s_pot[b];
  const int64_t src = st->cand[b];
  for (int j = tid; j < dim; j += blockDim.x) centers[(int64_t)c * dim + j] = X[src * dim + j];
  if (tid == 0) indices[c] = src;
  if (!more) return;
  if (tid < T) s_r[tid] = u_mine * (double)pot;
  const int64_t chunk = (n + blockDim.x - 1) / blockDim.x;
  const int64_t lo = min<int64_t>(n, tid * chunk), hi = min<int64_t>(n, lo + chunk);
  const float* row = dist + (int64_t)b * n;
  float pr[kR];
#pragma unroll
  for (int u = 0; u < kR; ++u) pr[u] = (lo + u < hi) ? (w ? w[lo + u] : 1.0f) * row[lo + u] : 0.f;
  double run = 0.0;
#pragma unroll
  for (int u = 0; u < kR; ++u)
    if (lo + u < hi) run = run + (double)pr[u];
  double incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_part[wave] = incl;
  __syncthreads();  // s_part, s_r; also every thread has read st->cand[b]
  double base = incl - run;
  for (int q = 0; q < wave; ++q) base += s_part[q];
  double cu[kR];
#pragma unroll
  for (int u = 0; u < kR; ++u) {
    base = base + (double)pr[u];
    cu[u] = base;
  }
  for (int t = 0; t < T; ++t) {
    const double r = s_r[t];
    int cw = 0;
#pragma unroll
    for (int u = 0; u < kR; ++u) cw += __popcll(__ballot(lo + u < hi && cu[u] < r));
    if (lane == 0) s_cnt[t * 4 + wave] = cw;
  }
  __syncthreads();
  if (tid < T) {
    int64_t a = 0;
    for (int q = 0; q < nw; ++q) a += s_cnt[tid * 4 + q];
    if (a > n - 1) a = n - 1;
    st->cand[tid] = a;
  }
  if (tid == 0) {
    st->best = b;
    st->pot = pot;
  }
}

template <int kR>
__global__ __launch_bounds__(256) void k_kpp_rounds(
    int64_t n, int dim, const float* __restrict__ X, const float* __restrict__ w,
    const double* __restrict__ xsq, const float* __restrict__ closest0, float* __restrict__ dist0,
    float* __restrict__ dist1, float* __restrict__ acc, int L, int G, int T, int k,
    const double* __restrict__ uniforms, float* __restrict__ centers, int64_t* __restrict__ indices,
    KppState* __restrict__ st, KppSync* __restrict__ sy) {
  extern __shared__ double s_c[];
  __shared__ float s_pot[kMaxTrials];
  __shared__ double s_r[kMaxTrials];
  __shared__ double s_part[4];
  __shared__ int s_cnt[kMaxTrials * 4];
  __shared__ int s_flag;
  const int tid = threadIdx.x;
  const int t = blockIdx.x / G, g = blockIdx.x - t * G;
  const unsigned NB = gridDim.x;
  for (int c = 1; c < k; ++c) {
    if (c > 1) {
      if (tid == 0) s_flag = kpp_wait_round(sy, (unsigned)c) ? 1 : 0;
      __syncthreads();
      if (!s_flag) {
        if (tid == 0) atomicOr(&sy->err, 1u);
        return;
      }
      __threadfence();  // acquire: the published candidates and the previous distance rows
    }
    const float* prev = ((c - 1) & 1) ? dist1 : dist0;
    float* cur = (c & 1) ? dist1 : dist0;
    kpp_dist_phase(n, dim, X, w, xsq, closest0, prev, st, cur, acc, L, t, g, s_c);
    __threadfence();  // release this workgroup's distances and chain accumulators
    __syncthreads();
    if (tid == 0) s_flag = (atomicAdd(&sy->arrive, 1u) == (unsigned)c * NB - 1u) ? 1 : 0;
    __syncthreads();
    if (!s_flag) continue;
    __threadfence();  // acquire every workgroup's writes of this round
    kpp_tail_phase<kR>(n, dim, X, w, cur, acc, T, c, k, uniforms, centers, indices, st, s_pot, s_r,
                       s_part, s_cnt);
    __threadfence();  // release the next round's candidates
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&sy->round, (unsigned)(c + 1), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_ones(int64_t n, float* p) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 1.0f;
}

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" size_t gdd_kmeans_plusplus_ws_bytes(int64_t n, int n_trials) {
  size_t b = 0;
  b += align256(sizeof(KppState));
  b += align256(sizeof(double) * n);                                        // xsq
  b += align256(sizeof(float) * n);                                         // closest0
  b += 2 * align256(sizeof(float) * n * (size_t)std::max(n_trials, 1));     // dist ping-pong
  b += align256(sizeof(double) * n);                                        // cum
  b += 2 * align256(sizeof(float) * 64 * (size_t)std::max(n_trials, 1));   // lane accumulators
  b += 2 * align256(sizeof(int64_t) * kMaxTrials);                          // round candidates
  b += align256(sizeof(KppSync));
  b += align256(sizeof(KppSpec));
  return b + 2048;
}

extern "C" int gdd_kmeans_plusplus(int64_t n, int dim, const float* X, const float* w, int k,
                                   int n_trials, int64_t first_id, const double* uniforms,
                                   float* centers, int64_t* indices, void* ws, size_t ws_bytes,
                                   gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && k > 0 && k <= n, "kmeans++: n=%lld dim=%d k=%d invalid",
              (long long)n, dim, k);
  GDD_REQUIRE(n_trials >= 1 && n_trials <= kMaxTrials, "kmeans++: n_trials=%d unsupported",
              n_trials);
  GDD_REQUIRE(dim <= 4096, "kmeans++: dim=%d unsupported", dim);
  GDD_REQUIRE(first_id >= 0 && first_id < n, "kmeans++: first_id out of range");
  GDD_REQUIRE(X && centers && indices && ws && (k == 1 || uniforms), "kmeans++: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  KppState* st = cv.take<KppState>(1);
  double* xsq = cv.take<double>(n);
  float* closest0 = cv.take<float>(n);
  float* dist[2] = {cv.take<float>(n * (size_t)n_trials), cv.take<float>(n * (size_t)n_trials)};
  double* cum = cv.take<double>(n);
  float* acc = cv.take<float>(64 * (size_t)n_trials);
  float* acc2 = cv.take<float>(64 * (size_t)n_trials);
  int64_t* candb[2] = {cv.take<int64_t>(kMaxTrials), cv.take<int64_t>(kMaxTrials)};
  KppSync* sy = cv.take<KppSync>(1);
  KppSpec* sp = cv.take<KppSpec>(1);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "kmeans++: workspace too small");
  const unsigned nb = (unsigned)((n + 255) / 256);
  // w == nullptr: unit sample weights, handled in the kernels
  k_kpp_init<<<nb, 256, 0, s>>>(n, dim, X, first_id, xsq, closest0);
  GDD_LAUNCHED();
  k_kpp_tail<<<1, kTailThreads, 0, s>>>(n, dim, X, w, closest0, dist[1], acc, n_trials, 0, k,
                                        first_id, uniforms, xsq, cum, centers, indices, st);
  GDD_LAUNCHED();
  // lanes per distance block: about one point per thread (L * J ~ 256), L a power of two
  const int64_t J = n >> 6;
  int L = 64;
  while (L > 1 && (int64_t)L * J > 256) L >>= 1;
  const int G = 64 / L;
  // the block's chain distances stay in LDS when they fit next to the candidate row
  const size_t lds_chain = sizeof(double) * (size_t)dim + sizeof(float) * (size_t)L * J;
  const int chain_in_lds = lds_chain <= 65536 ? 1 : 0;
  const size_t lds = chain_in_lds ? lds_chain : sizeof(double) * (size_t)dim;
  if (lds > 65536)
    GDD_HIP(hipFuncSetAttribute((const void*)k_kpp_dist<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // all rounds in one persistent launch (opt-in, GDD_KPP_PERSISTENT=1): measured 31 us per round
  // at the arxiv shape against 13 us for the two launches below — the agent-scope fences each
  // workgroup needs per round (L2 write-back + invalidate on gfx950) cost more than the launch
  // boundaries they replace. Kept for the handoff work that would make it pay (sc1 granules).
  const int NB = G * n_trials;
  if (k > 1 && NB <= 256 && chain_in_lds && (n + 255) / 256 <= 16 &&
      getenv("GDD_KPP_PERSISTENT") != nullptr) {
    GDD_HIP(hipMemsetAsync(sy, 0, sizeof(KppSync), s));
    if (lds > 65536)
      GDD_HIP(hipFuncSetAttribute((const void*)k_kpp_rounds<16>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_kpp_rounds<16><<<NB, 256, lds, s>>>(n, dim, X, w, xsq, closest0, dist[0], dist[1], acc, L, G,
                                          n_trials, k, uniforms, centers, indices, st, sy);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  // one launch per round (k_kpp_round) when a 256-thread workgroup scans the winner's row in
  // <= 16 entries per thread
  if (k > 1 && chain_in_lds && (n + 255) / 256 <= 16 && getenv("GDD_KPP_SPEC") == nullptr) {
    float* accb[2] = {acc, acc2};
    // opt-in (GDD_KPP_PREFETCH=1): the point rows requested into registers at the start of the
    // round. Measured slower at the arxiv shape (13.7 vs 12.6 ms per fit): the extra in-flight
    // loads delay the critical potential/winner-row requests more than they hide.
    const bool pre = (int64_t)L * J + (n - (J << 6)) <= 256 && dim <= 64 && dim % 4 == 0 &&
                     (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
                     getenv("GDD_KPP_PREFETCH") != nullptr;
    auto kern = pre ? k_kpp_round<16, 64> : k_kpp_round<16, 0>;
    if (lds > 65536)
      GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
    for (int c = 1; c < k; ++c) {
      kern<<<dim3(G, n_trials), 256, lds, s>>>(
          n, dim, X, w, xsq, closest0, dist[(c - 1) & 1], dist[c & 1], accb[(c - 1) & 1],
          accb[c & 1], L, n_trials, c, uniforms, st, candb[(c - 1) & 1], candb[c & 1], centers,
          indices);
      GDD_LAUNCHED();
    }
    k_kpp_round_final<<<1, 256, 0, s>>>(n, dim, X, w, dist[(k - 1) & 1], accb[(k - 1) & 1],
                                        n_trials, k - 1, candb[(k - 1) & 1], centers, indices);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  // speculative draws: per round one distance launch and one per-trial tail launch (T workgroups)
  constexpr int kSpecR = 8;
  if (k > 1 && chain_in_lds && (n + kTailThreads - 1) / kTailThreads <= kSpecR) {
    k_kpp_spec_seed<<<1, 64, 0, s>>>(st, n_trials, sp);
    GDD_LAUNCHED();
    if (lds > 65536)
      GDD_HIP(hipFuncSetAttribute((const void*)k_kpp_dist_spec,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int c = 1; c < k; ++c) {
      const float* prev = dist[(c - 1) & 1];
      float* cur = dist[c & 1];
      k_kpp_dist_spec<<<dim3(G, n_trials), 256, lds, s>>>(n, dim, X, w, xsq, closest0, prev, sp, cur,
                                                          acc, L, n_trials, c, centers, indices);
      GDD_LAUNCHED();
      k_kpp_trial_tail<kSpecR><<<n_trials, kTailThreads, 0, s>>>(n, w, cur, acc, n_trials, c, k,
                                                                 uniforms, sp);
      GDD_LAUNCHED();
    }
    k_kpp_spec_finish<<<1, 256, 0, s>>>(dim, X, sp, n_trials, k - 1, centers, indices);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  constexpr int kFastT = 12, kFastR = 4;
  const bool fast_tail = n_trials <= kFastT && (n + kTailThreads - 1) / kTailThreads <= kFastR;
  for (int c = 1; c < k; ++c) {
    const float* prev = dist[(c - 1) & 1];
    float* cur = dist[c & 1];
    if (chain_in_lds)
      k_kpp_dist<true><<<dim3(G, n_trials), 256, lds, s>>>(n, dim, X, w, xsq, closest0, prev, st,
                                                           cur, acc, L);
    else
      k_kpp_dist<false><<<dim3(G, n_trials), 256, lds, s>>>(n, dim, X, w, xsq, closest0, prev, st,
                                                            cur, acc, L);
    GDD_LAUNCHED();
    if (fast_tail)
      k_kpp_tail_fast<kFastT, kFastR><<<1, kTailThreads, 0, s>>>(n, dim, X, w, cur, acc, n_trials, c,
                                                                 k, uniforms, centers, indices, st);
    else
      k_kpp_tail<<<1, kTailThreads, 0, s>>>(n, dim, X, w, closest0, cur, acc, n_trials, c, k,
                                            first_id, uniforms, xsq, cum, centers, indices, st);
    GDD_LAUNCHED();
  }
  return GDD_OK;
}
