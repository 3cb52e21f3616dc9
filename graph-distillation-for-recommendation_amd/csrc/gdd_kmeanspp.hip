// gdd_kmeanspp.hip — greedy k-means++ seeding on the device (sklearn _kmeans_plusplus,
// sklearn/cluster/_kmeans.py:174-272), with the host's RNG draws passed in.
//
// One persistent workgroup of 1024 threads runs all k-1 seeding rounds with block barriers only
// (no host round trips); the working set (closest distances, candidate distances, the fp64
// cumulative potential) stays in L2. Per round c = 1..k-1:
//   1. cum[i]  = inclusive fp64 prefix of fp32(w_i * closest_i)       (stable_cumsum, fp64)
//   2. cand[t] = searchsorted_left(cum, u[c-1][t] * (double)pot), clipped to n-1
//   3. dist[t][i] = min(closest_i, fp32(max(0, ((-2<x_cand, x_i>) + |x_cand|^2) + |x_i|^2)))
//      (fp64 upcast distances stored as fp32: sklearn/metrics/pairwise.py:582-650; np.minimum)
//   4. pot[t] = fp32 dot(dist[t], w) in the OpenBLAS SkylakeX sdot order
//   5. best = first argmin pot; pot = pot[best]; closest = dist[best]; centers[c] = X[cand[best]]
#include <algorithm>

#include "gdd_common.hpp"

namespace gdd {
namespace {

constexpr int kThreads = 1024;
constexpr int kMaxTrials = 16;

// OpenBLAS 0.3.28/29 SkylakeX sdot (kernel/x86_64/sdot.c + sdot_microk_skylakex-2.c), emulated by
// one wave: the 64 lanes are the 4 x 16 AVX-512 accumulators of the 64-wide loop; they fold to
// 4 x 8 AVX2 accumulators for the 32-wide remainder; lanes then combine ((a0+a1)+a2)+a3, 8 -> 4 by
// halves, and (h0+h1)+(h2+h3); the scalar tail is added in double. Called by all 64 lanes of a wave.
__device__ float sdot_skx_wave(const float* __restrict__ x, const float* __restrict__ y, int64_t n,
                               float* scratch /* 64 floats of LDS for this wave */) {
  const int lane = threadIdx.x & 63;
  const int64_t n1 = n & ~31ll;
  const int64_t n64 = n1 & ~63ll;
  float a = 0.f;
  for (int64_t i = lane; i < n64; i += 64) a = __builtin_fmaf(x[i], y[i], a);
  scratch[lane] = a;  // lane = u*16 + l  <->  accum_u5 lane l
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float r = 0.f;
  if (lane == 0) {
    float acc[4][8];
    for (int u = 0; u < 4; ++u)
      for (int l = 0; l < 8; ++l) acc[u][l] = scratch[u * 16 + l] + scratch[u * 16 + l + 8];
    for (int64_t i = n64; i < n1; i += 32)
      for (int u = 0; u < 4; ++u)
        for (int l = 0; l < 8; ++l) acc[u][l] = __builtin_fmaf(x[i + u * 8 + l], y[i + u * 8 + l], acc[u][l]);
    float s[8];
    for (int l = 0; l < 8; ++l) s[l] = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l];
    float h[4];
    for (int l = 0; l < 4; ++l) h[l] = s[l] + s[l + 4];
    double dot = n1 ? (double)((h[0] + h[1]) + (h[2] + h[3])) : 0.0;
    for (int64_t i = n1; i < n; ++i) {
      const float p = y[i] * x[i];
      dot = dot + (double)p;
    }
    r = (float)dot;
  }
  return r;
}

__device__ __forceinline__ float np_minimum(float a, float b) {
  if (a != a || b != b) return __builtin_nanf("");
  return b < a ? b : a;
}

__global__ __launch_bounds__(kThreads) void k_kpp(int64_t n, int dim, const float* __restrict__ X,
                                                  const float* __restrict__ w, int k, int T,
                                                  int64_t first_id,
                                                  const double* __restrict__ uniforms,
                                                  float* __restrict__ centers,
                                                  int64_t* __restrict__ indices,
                                                  double* __restrict__ xsq,
                                                  float* __restrict__ closest,
                                                  float* __restrict__ dist,
                                                  double* __restrict__ cum) {
  __shared__ double s_part[kThreads];
  __shared__ float s_scratch[kThreads];
  __shared__ int64_t s_cand[kMaxTrials];
  __shared__ float s_pot[kMaxTrials];
  __shared__ double s_cnorm[kMaxTrials];
  __shared__ float s_cur_pot;
  __shared__ int s_best;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;

  // |x_i|^2 in fp64 (row_norms of the upcast chunk)
  for (int64_t i = tid; i < n; i += kThreads) {
    double s = 0.0;
    for (int j = 0; j < dim; ++j) {
      const double v = (double)X[i * dim + j];
      s = __builtin_fma(v, v, s);
    }
    xsq[i] = s;
  }
  // first center
  for (int j = tid; j < dim; j += kThreads) centers[j] = X[first_id * dim + j];
  if (tid == 0) indices[0] = first_id;
  __syncthreads();
  // closest distances to the first center
  {
    const float* xc = X + first_id * dim;
    const double cn = xsq[first_id];
    for (int64_t i = tid; i < n; i += kThreads) {
      double dot = 0.0;
      for (int j = 0; j < dim; ++j) dot = __builtin_fma((double)xc[j], (double)X[i * dim + j], dot);
      double d = ((-2.0 * dot) + cn) + xsq[i];
      float f = (float)d;
      closest[i] = f < 0.f ? 0.f : f;
    }
  }
  __syncthreads();
  if (wave == 0) {
    float p = sdot_skx_wave(closest, w, n, s_scratch);
    if (tid == 0) s_cur_pot = p;
  }
  __syncthreads();

  const int64_t chunk = (n + kThreads - 1) / kThreads;
  for (int c = 1; c < k; ++c) {
    // 1. fp64 cumulative potential: per-thread contiguous chunks, block scan of chunk totals
    const int64_t lo = tid * chunk, hi = min<int64_t>(n, lo + chunk);
    double run = 0.0;
    for (int64_t i = lo; i < hi; ++i) run = run + (double)(w[i] * closest[i]);
    s_part[tid] = run;
    __syncthreads();
    for (int off = 1; off < kThreads; off <<= 1) {
      double v = tid >= off ? s_part[tid - off] : 0.0;
      __syncthreads();
      s_part[tid] += v;
      __syncthreads();
    }
    double base = tid ? s_part[tid - 1] : 0.0;
    for (int64_t i = lo; i < hi; ++i) {
      base = base + (double)(w[i] * closest[i]);
      cum[i] = base;
    }
    __syncthreads();
    // 2. candidates: np.searchsorted(cum, u * pot) (side='left'), clipped to n-1
    if (tid < T) {
      const double r = uniforms[(int64_t)(c - 1) * T + tid] * (double)s_cur_pot;
      int64_t a = 0, b = n;  // first index with cum[idx] >= r
      while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (cum[m] < r)
          a = m + 1;
        else
          b = m;
      }
      if (a > n - 1) a = n - 1;
      s_cand[tid] = a;
      s_cnorm[tid] = xsq[a];
    }
    __syncthreads();
    // 3. distances to every candidate, min with closest
    for (int64_t i = tid; i < n; i += kThreads) {
      const float cl = closest[i];
      for (int t = 0; t < T; ++t) {
        const float* xc = X + s_cand[t] * dim;
        double dot = 0.0;
        for (int j = 0; j < dim; ++j)
          dot = __builtin_fma((double)xc[j], (double)X[i * dim + j], dot);
        const double d = ((-2.0 * dot) + s_cnorm[t]) + xsq[i];
        float f = (float)d;
        f = f < 0.f ? 0.f : f;
        dist[(int64_t)t * n + i] = np_minimum(cl, f);
      }
    }
    __syncthreads();
    // 4. candidate potentials, one wave per candidate
    if (wave < T) {
      const float p = sdot_skx_wave(dist + (int64_t)wave * n, w, n, s_scratch + wave * 64);
      if ((tid & 63) == 0) s_pot[wave] = p;
    }
    __syncthreads();
    // 5. pick the best candidate (np.argmin: first minimum, NaN wins)
    if (tid == 0) {
      int b = 0;
      for (int t = 1; t < T; ++t) {
        const float pb = s_pot[b], pt = s_pot[t];
        if (pb == pb && (pt < pb || pt != pt)) b = t;
      }
      s_best = b;
      s_cur_pot = s_pot[b];
      indices[c] = s_cand[b];
    }
    __syncthreads();
    const int b = s_best;
    const float* src = dist + (int64_t)b * n;
    for (int64_t i = tid; i < n; i += kThreads) closest[i] = src[i];
    for (int j = tid; j < dim; j += kThreads) centers[(int64_t)c * dim + j] = X[s_cand[b] * dim + j];
    __syncthreads();
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
  b += align256(sizeof(double) * n);                          // xsq
  b += align256(sizeof(float) * n);                           // closest
  b += align256(sizeof(float) * n * (size_t)std::max(n_trials, 1));  // dist
  b += align256(sizeof(double) * n);                          // cum
  b += align256(sizeof(float) * n);                           // ones (w == NULL)
  return b + 1024;
}

extern "C" int gdd_kmeans_plusplus(int64_t n, int dim, const float* X, const float* w, int k,
                                   int n_trials, int64_t first_id, const double* uniforms,
                                   float* centers, int64_t* indices, void* ws, size_t ws_bytes,
                                   gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && k > 0 && k <= n, "kmeans++: n=%lld dim=%d k=%d invalid",
              (long long)n, dim, k);
  GDD_REQUIRE(n_trials >= 1 && n_trials <= kMaxTrials, "kmeans++: n_trials=%d unsupported",
              n_trials);
  GDD_REQUIRE(first_id >= 0 && first_id < n, "kmeans++: first_id out of range");
  GDD_REQUIRE(X && centers && indices && ws && (k == 1 || uniforms), "kmeans++: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  double* xsq = cv.take<double>(n);
  float* closest = cv.take<float>(n);
  float* dist = cv.take<float>(n * (size_t)n_trials);
  double* cum = cv.take<double>(n);
  float* ones = cv.take<float>(n);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "kmeans++: workspace too small");
  if (!w) {
    k_ones<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(n, ones);
    GDD_LAUNCHED();
    w = ones;
  }
  k_kpp<<<1, kThreads, 0, s>>>(n, dim, X, w, k, n_trials, first_id, uniforms, centers, indices, xsq,
                               closest, dist, cum);
  GDD_LAUNCHED();
  return GDD_OK;
}
