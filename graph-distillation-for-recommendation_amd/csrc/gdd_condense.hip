// gdd_condense.hip — ClustGDD's graph condensation on the device:
//
//   attaw / vanilla effective-resistance edge weights   utils_clustgdd.py:149-182
//   per-class sparsification (softmax weights, top-k)    clustgdd_agent_transduct.py:131-232
//   cluster-level graph P^T A P, diagonal removed        clustgdd_agent_transduct.py:234-250
//
// Everything is O(nnz) integer/byte or elementwise fp32 work, HBM/L2-bound; nothing here is a GEMM.
// Orders (restated bit for bit by oracle/condense.py):
//   * unit rows: sqrtf of the sequential fp32 sum of squares (correctly rounded), clamped at 1e-8;
//     cosine: sequential fp32 sum of the unit rows' products; reweighted value = val * cos;
//   * degrees: sequential fp32 row sums in CSR order (torch sparse @ ones);
//   * ER = v / deg[src] + v / deg[dst];
//   * softmax: e = fp32(exp(double(x - max))), sequential fp32 sum, e / s;
//   * top-k: orderable 32-bit keys (NaN largest, -0 == +0), 4-pass radix select of the threshold
//     per class, then the edges above it plus the lowest-index ties, written in edge order;
//   * compress: int64 fixed point llrint(v * 2^s), s = 62 - ceil(log2 max|v|) - ceil(log2(m+1)),
//     exact integer sums per (cluster, cluster) with agent-scope atomics (order-free, so
//     deterministic), then fp64 sum * 2^-s / (|a| |b|) rounded to fp32; empty clusters NaN.
#include <climits>
#include <cmath>

#include "gdd_common.hpp"

namespace gdd {
namespace {

constexpr int kThreads = 256;
constexpr int kTkBlk = 4096;  // top-k compaction block (edges)

__device__ __forceinline__ uint32_t okey(float f) {
  if (f != f) return 0xFFFFFFFFu;  // NaN: largest (torch.topk)
  if (f == 0.f) f = 0.f;           // -0 ties with +0
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void k_coo_rows(int64_t n, const int32_t* __restrict__ rowptr, int32_t* __restrict__ rows) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e) rows[e] = (int32_t)r;
}

__global__ void k_unit_rows(int64_t n, int C, const float* __restrict__ x, float* __restrict__ xu) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* xr = x + r * C;
  float s = 0.f;
  for (int j = 0; j < C; ++j) s = s + xr[j] * xr[j];
  const float nrm = fmaxf(sqrtf(s), 1e-8f);
  for (int j = 0; j < C; ++j) xu[r * C + j] = xr[j] / nrm;
}

__global__ void k_edge_cos(int64_t nnz, int C, const int32_t* __restrict__ rows,
                           const int32_t* __restrict__ col, const float* __restrict__ val,
                           const float* __restrict__ xu, float* __restrict__ rew) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const float* a = xu + (int64_t)rows[e] * C;
  const float* b = xu + (int64_t)col[e] * C;
  float s = 0.f;
  int j = 0;
  if ((C & 3) == 0) {  // rows 16-byte aligned: 8 float4 pairs in flight ahead of the ordered sum
    for (; j + 32 <= C; j += 32) {
      float4 x[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        x[u] = *reinterpret_cast<const float4*>(a + j + 4 * u);
        y[u] = *reinterpret_cast<const float4*>(b + j + 4 * u);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s = s + x[u].x * y[u].x;
        s = s + x[u].y * y[u].y;
        s = s + x[u].z * y[u].z;
        s = s + x[u].w * y[u].w;
      }
    }
    for (; j + 4 <= C; j += 4) {
      const float4 x = *reinterpret_cast<const float4*>(a + j);
      const float4 y = *reinterpret_cast<const float4*>(b + j);
      s = s + x.x * y.x;
      s = s + x.y * y.y;
      s = s + x.z * y.z;
      s = s + x.w * y.w;
    }
  }
  for (; j < C; ++j) s = s + a[j] * b[j];
  rew[e] = (val ? val[e] : 1.0f) * s;
}

constexpr int kLongRow = 512;  // rows at least this long are summed by a whole workgroup

// sequential fp32 row sums in CSR order (rows shorter than kLongRow: one thread each)
__global__ void k_row_sums(int64_t n, const int32_t* __restrict__ rowptr, const float* __restrict__ v,
                           float* __restrict__ deg) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t e1 = rowptr[r + 1];
  int32_t e = rowptr[r];
  if (e1 - e >= kLongRow) return;
  float s = 0.f;
  for (; e + 8 <= e1; e += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = v ? v[e + u] : 1.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + t[u];
  }
  for (; e < e1; ++e) s = s + (v ? v[e] : 1.0f);
  deg[r] = s;
}

// rows of kLongRow+ entries: the workgroup of 64 rows walks its long rows; per row, all threads stage
// chunks of 4096 values into LDS (coalesced) and thread 0 folds them in order (float4 LDS reads
// eight ahead of the dependent adds), double-buffered so the next chunk loads under the fold
__global__ __launch_bounds__(kThreads) void k_row_sums_long(int64_t n, const int32_t* __restrict__ rowptr,
                                                            const float* __restrict__ v,
                                                            float* __restrict__ deg) {
  __shared__ __attribute__((aligned(16))) float buf[2][4096];
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  for (int64_t r = r0; r < min<int64_t>(n, r0 + 64); ++r) {
    const int32_t b = rowptr[r], e1 = rowptr[r + 1];
    if (e1 - b < kLongRow) continue;  // uniform across the workgroup
    float acc = 0.f;
    int cur = 0;
    for (int32_t c = b; c < e1; c += 4096) {
      const int m = min(4096, e1 - c);
      for (int t = threadIdx.x; t < m; t += kThreads) buf[cur][t] = v ? v[c + t] : 1.0f;
      __syncthreads();
      if (threadIdx.x == 0) {
        const float4* b4 = reinterpret_cast<const float4*>(buf[cur]);
        int t = 0;
        for (; t + 32 <= m; t += 32) {
          float4 x[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) x[u] = b4[t / 4 + u];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            acc = acc + x[u].x;
            acc = acc + x[u].y;
            acc = acc + x[u].z;
            acc = acc + x[u].w;
          }
        }
        for (; t < m; ++t) acc = acc + buf[cur][t];
      }
      cur ^= 1;
    }
    if (threadIdx.x == 0) deg[r] = acc;
    __syncthreads();
  }
}

__global__ void k_er(int64_t nnz, const int32_t* __restrict__ rows, const int32_t* __restrict__ col,
                     const float* __restrict__ v, const float* __restrict__ deg, float* __restrict__ er) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const float x = v ? v[e] : 1.0f;
  er[e] = x / deg[rows[e]] + x / deg[col[e]];
}

__global__ void k_softmax_rows(int64_t n, int C, const float* __restrict__ x, float* __restrict__ p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* xr = x + r * C;
  float m = xr[0];
  for (int j = 1; j < C; ++j) m = fmaxf(m, xr[j]);
  float s = 0.f;
  for (int j = 0; j < C; ++j) {
    const float e = (float)exp((double)(xr[j] - m));
    p[r * C + j] = e;
    s = s + e;
  }
  for (int j = 0; j < C; ++j) p[r * C + j] = p[r * C + j] / s;
}

// w[i][e] = (p[src][i] * p[dst][i]) * er[e] for every class i (probs == nullptr: one set, w = er)
__global__ void k_class_keys(int64_t nnz, int nsets, const int32_t* __restrict__ rows,
                             const int32_t* __restrict__ col, const float* __restrict__ er,
                             const float* __restrict__ probs, uint32_t* __restrict__ keys) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const float x = er[e];
  if (!probs) {
    keys[e] = okey(x);
    return;
  }
  const float* pa = probs + (int64_t)rows[e] * nsets;
  const float* pb = probs + (int64_t)col[e] * nsets;
  int i = 0;
  if ((nsets & 3) == 0) {
    for (; i + 4 <= nsets; i += 4) {
      const float4 u = *reinterpret_cast<const float4*>(pa + i);
      const float4 v = *reinterpret_cast<const float4*>(pb + i);
      keys[(int64_t)i * nnz + e] = okey((u.x * v.x) * x);
      keys[(int64_t)(i + 1) * nnz + e] = okey((u.y * v.y) * x);
      keys[(int64_t)(i + 2) * nnz + e] = okey((u.z * v.z) * x);
      keys[(int64_t)(i + 3) * nnz + e] = okey((u.w * v.w) * x);
    }
  }
  for (; i < nsets; ++i) keys[(int64_t)i * nnz + e] = okey((pa[i] * pb[i]) * x);
}

// ---- radix select of the m-th largest key per set (4 passes of 8 bits, top byte first) ----
struct TkState {
  uint32_t prefix, mask;
  int64_t remaining;  // edges still to take at the threshold once the prefix is complete
};

__global__ void k_tk_init(int nsets, int64_t m, TkState* __restrict__ st, uint32_t* __restrict__ hist) {
  const int i = blockIdx.x;
  if (threadIdx.x == 0) st[i] = TkState{0u, 0u, m};
  hist[(int64_t)i * 256 + threadIdx.x] = 0u;
}

__global__ __launch_bounds__(kThreads) void k_tk_hist(int64_t nnz, int shift,
                                                      const uint32_t* __restrict__ keys,
                                                      const TkState* __restrict__ st,
                                                      uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int i = blockIdx.y;
  h[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t prefix = st[i].prefix, mask = st[i].mask;
  const uint32_t* k = keys + (int64_t)i * nnz;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < nnz;
       e += (int64_t)gridDim.x * kThreads) {
    const uint32_t key = k[e];
    if ((key & mask) == prefix) atomicAdd(&h[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[(int64_t)i * 256 + threadIdx.x], h[threadIdx.x]);
}

// one workgroup per set: the bin, from the top, where the running count reaches `remaining`
__global__ __launch_bounds__(256) void k_tk_pick(int shift, TkState* __restrict__ st,
                                                 uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int i = blockIdx.x, t = threadIdx.x;
  h[t] = hist[(int64_t)i * 256 + t];
  hist[(int64_t)i * 256 + t] = 0u;  // ready for the next pass
  __syncthreads();
  if (t == 0) {
    TkState s = st[i];
    int64_t above = 0;
    int b = 255;
    for (; b > 0; --b) {
      if (above + (int64_t)h[b] >= s.remaining) break;
      above += h[b];
    }
    s.prefix |= (uint32_t)b << shift;
    s.mask |= 255u << shift;
    s.remaining -= above;
    st[i] = s;
  }
}

// per block of kTkBlk edges: how many lie above the threshold and how many tie with it
__global__ __launch_bounds__(kThreads) void k_tk_count(int64_t nnz, int nblk,
                                                       const uint32_t* __restrict__ keys,
                                                       const TkState* __restrict__ st,
                                                       int2* __restrict__ cnt) {
  __shared__ int s_gt[kThreads / 64], s_eq[kThreads / 64];
  const int i = blockIdx.y, b = blockIdx.x;
  const uint32_t thr = st[i].prefix;
  const uint32_t* k = keys + (int64_t)i * nnz;
  int gt = 0, eq = 0;
  for (int q = threadIdx.x; q < kTkBlk; q += kThreads) {
    const int64_t e = (int64_t)b * kTkBlk + q;
    const uint32_t key = e < nnz ? k[e] : 0u;
    gt += e < nnz && key > thr;
    eq += e < nnz && key == thr;
  }
  for (int o = 32; o > 0; o >>= 1) {
    gt += __shfl_down(gt, o);
    eq += __shfl_down(eq, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s_gt[threadIdx.x >> 6] = gt;
    s_eq[threadIdx.x >> 6] = eq;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0, c = 0;
    for (int w = 0; w < kThreads / 64; ++w) {
      a += s_gt[w];
      c += s_eq[w];
    }
    cnt[(int64_t)i * nblk + b] = make_int2(a, c);
  }
}

// exclusive scan of the block counts (one workgroup per set, sequential over blocks by 256 lanes)
__global__ __launch_bounds__(256) void k_tk_scan(int nblk, const int2* __restrict__ cnt,
                                                 int2* __restrict__ off) {
  __shared__ int2 s_tot[256];
  const int i = blockIdx.x, t = threadIdx.x;
  const int per = (nblk + 255) / 256;
  const int lo = min(nblk, t * per), hi = min(nblk, lo + per);
  int a = 0, c = 0;
  for (int b = lo; b < hi; ++b) {
    const int2 v = cnt[(int64_t)i * nblk + b];
    a += v.x;
    c += v.y;
  }
  s_tot[t] = make_int2(a, c);
  __syncthreads();
  if (t == 0) {
    int2 run = make_int2(0, 0);
    for (int q = 0; q < 256; ++q) {
      const int2 v = s_tot[q];
      s_tot[q] = run;
      run.x += v.x;
      run.y += v.y;
    }
  }
  __syncthreads();
  int2 run = s_tot[t];
  for (int b = lo; b < hi; ++b) {
    const int2 v = cnt[(int64_t)i * nblk + b];
    off[(int64_t)i * nblk + b] = run;
    run.x += v.x;
    run.y += v.y;
  }
}

// write the selected edge ids in edge order: all above the threshold, and the first `remaining`
// ties; output position = selected edges before it
__global__ __launch_bounds__(kThreads) void k_tk_emit(int64_t nnz, int nblk, int64_t m,
                                                      const uint32_t* __restrict__ keys,
                                                      const TkState* __restrict__ st,
                                                      const int2* __restrict__ off,
                                                      int32_t* __restrict__ sel) {
  __shared__ int s_gt[kThreads / 64], s_eq[kThreads / 64];
  __shared__ int s_base_gt, s_base_eq;
  const int i = blockIdx.y, b = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t thr = st[i].prefix;
  const int64_t rem = st[i].remaining;
  const uint32_t* k = keys + (int64_t)i * nnz;
  int32_t* out = sel + (int64_t)i * m;
  const int2 o = off[(int64_t)i * nblk + b];
  if (threadIdx.x == 0) {
    s_base_gt = o.x;
    s_base_eq = o.y;
  }
  __syncthreads();
  for (int q0 = 0; q0 < kTkBlk; q0 += kThreads) {
    const int64_t e = (int64_t)b * kTkBlk + q0 + threadIdx.x;
    const uint32_t key = e < nnz ? k[e] : 0u;
    const bool gt = e < nnz && key > thr, eq = e < nnz && key == thr;
    const uint64_t bg = __ballot(gt), be = __ballot(eq);
    const uint64_t below = (lane ? (~0ull >> (64 - lane)) : 0ull);
    if (lane == 0) {
      s_gt[wave] = __popcll(bg);
      s_eq[wave] = __popcll(be);
    }
    __syncthreads();
    int pg = s_base_gt, pe = s_base_eq;
    for (int w = 0; w < wave; ++w) {
      pg += s_gt[w];
      pe += s_eq[w];
    }
    pg += __popcll(bg & below);
    pe += __popcll(be & below);
    // selected before e: every above-threshold edge plus the ties already taken (capped at rem)
    const int64_t pos = (int64_t)pg + min<int64_t>(pe, rem);
    if (gt || (eq && pe < rem)) out[pos] = (int32_t)e;
    __syncthreads();
    if (threadIdx.x == 0) {
      int a = 0, c = 0;
      for (int w = 0; w < kThreads / 64; ++w) {
        a += s_gt[w];
        c += s_eq[w];
      }
      s_base_gt += a;
      s_base_eq += c;
    }
    __syncthreads();
  }
}

// ---- graph_compress --------------------------------------------------------------------------------
struct FixState {
  uint32_t maxabs_bits;
  int shift;
};

// cluster sizes: per-workgroup LDS histograms (kk <= 16384), merged with one global add per bin
__global__ __launch_bounds__(kThreads) void k_label_sizes(int64_t n, const int32_t* __restrict__ labels,
                                                          int kk, unsigned long long* __restrict__ size) {
  extern __shared__ unsigned int h[];
  for (int b = threadIdx.x; b < kk; b += kThreads) h[b] = 0u;
  __syncthreads();
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < n; r += (int64_t)gridDim.x * kThreads) {
    const int a = labels[r];
    if (a >= 0 && a < kk) atomicAdd(&h[a], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kk; b += kThreads)
    if (h[b]) atomicAdd(&size[b], (unsigned long long)h[b]);
}

__global__ void k_fix_maxabs(int64_t m, const int32_t* __restrict__ sel, const float* __restrict__ val,
                             FixState* __restrict__ fs) {
  __shared__ uint32_t s_m[kThreads / 64];
  uint32_t mx = 0u;
  for (int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x; q < m; q += (int64_t)gridDim.x * kThreads) {
    const int64_t e = sel ? sel[q] : q;
    const float v = val ? val[e] : 1.0f;
    const uint32_t b = __float_as_uint(fabsf(v));  // non-negative floats order as integers
    mx = b > mx ? b : mx;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = __shfl_down(mx, o);
    mx = y > mx ? y : mx;
  }
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kThreads / 64; ++w) mx = s_m[w] > mx ? s_m[w] : mx;
    atomicMax(&fs->maxabs_bits, mx);
  }
}

__device__ __forceinline__ int fix_shift(uint32_t maxabs_bits, int64_t m) {
  int e1 = 0, e2 = 0;
  const float mx = __uint_as_float(maxabs_bits);
  if (mx > 0.f) (void)frexpf(mx, &e1);
  (void)frexp((double)(m + 1), &e2);
  return 62 - e1 - e2;
}

__global__ void k_compress_acc(int64_t m, const int32_t* __restrict__ sel, const int32_t* __restrict__ rows,
                               const int32_t* __restrict__ col, const float* __restrict__ val,
                               const int32_t* __restrict__ labels, int kk, const FixState* __restrict__ fs,
                               unsigned long long* __restrict__ acc) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= m) return;
  const int64_t e = sel ? sel[q] : q;
  const int a = labels[rows[e]], b = labels[col[e]];
  const int s = fix_shift(fs->maxabs_bits, m);
  const double v = (double)(val ? val[e] : 1.0f);
  const long long fx = llrint(ldexp(v, s));
  if (fx != 0) atomicAdd(&acc[(int64_t)a * kk + b], (unsigned long long)fx);
}

__global__ void k_compress_fin(int kk, int64_t m, const unsigned long long* __restrict__ acc,
                               const unsigned long long* __restrict__ size,
                               const FixState* __restrict__ fs, float* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= (int64_t)kk * kk) return;
  const int a = (int)(c / kk), b = (int)(c - (int64_t)a * kk);
  const int s = fix_shift(fs->maxabs_bits, m);
  const double sa = (double)size[a], sb = (double)size[b];
  float f;
  if (sa == 0.0 || sb == 0.0) {
    f = __builtin_nanf("");
  } else {
    const double x = ldexp((double)(long long)acc[c], -s);
    f = (float)(x / (sa * sb));
  }
  if (a == b) f = f - f;  // torch: C - diag(diag(C)) (NaN stays NaN)
  out[c] = f;
}

// selected edges -> CSR (edge order is CSR order, so only the row pointers need counting)
__global__ void k_sel_rows(int64_t m, const int32_t* __restrict__ sel, const int32_t* __restrict__ rows,
                           const int32_t* __restrict__ col, const float* __restrict__ val,
                           int32_t* __restrict__ cnt, int32_t* __restrict__ col_out,
                           float* __restrict__ val_out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= m) return;
  const int32_t e = sel[q];
  atomicAdd(&cnt[rows[e]], 1);
  col_out[q] = col[e];
  val_out[q] = val ? val[e] : 1.0f;
}

unsigned grid1(int64_t n, int t = kThreads) { return (unsigned)((n + t - 1) / t); }

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" int gdd_coo_rows(int64_t n, const int32_t* rowptr, int32_t* rows, gdd_stream_t stream) {
  GDD_REQUIRE(n >= 0 && rowptr && (n == 0 || rows), "coo_rows: bad arguments");
  if (n == 0) return GDD_OK;
  k_coo_rows<<<grid1(n), kThreads, 0, to_hip(stream)>>>(n, rowptr, rows);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" size_t gdd_er_ws_bytes(int64_t n, int C) {
  return align256(sizeof(float) * (size_t)n * (size_t)std::max(C, 1)) + align256(sizeof(float) * n) + 256;
}

extern "C" int gdd_attaw_er(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* rows,
                            const int32_t* col, const float* val, int C, const float* ebd, float* rew,
                            float* er, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && nnz >= 0 && C > 0, "attaw_er: bad shape");
  GDD_REQUIRE(rowptr && (nnz == 0 || (rows && col && rew && er)) && ebd && ws, "attaw_er: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  float* xu = cv.take<float>((size_t)n * C);
  float* deg = cv.take<float>(n);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "attaw_er: workspace too small");
  k_unit_rows<<<grid1(n), kThreads, 0, s>>>(n, C, ebd, xu);
  GDD_LAUNCHED();
  if (nnz == 0) return GDD_OK;
  k_edge_cos<<<grid1(nnz), kThreads, 0, s>>>(nnz, C, rows, col, val, xu, rew);
  GDD_LAUNCHED();
  k_row_sums<<<grid1(n), kThreads, 0, s>>>(n, rowptr, rew, deg);
  GDD_LAUNCHED();
  k_row_sums_long<<<grid1(n, 64), kThreads, 0, s>>>(n, rowptr, rew, deg);
  GDD_LAUNCHED();
  k_er<<<grid1(nnz), kThreads, 0, s>>>(nnz, rows, col, rew, deg, er);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_vanilla_er(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* rows,
                              const int32_t* col, const float* val, float* er, void* ws,
                              size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && nnz >= 0, "vanilla_er: bad shape");
  GDD_REQUIRE(rowptr && (nnz == 0 || (rows && col && er)) && ws, "vanilla_er: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  float* deg = cv.take<float>(n);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "vanilla_er: workspace too small");
  if (nnz == 0) return GDD_OK;
  k_row_sums<<<grid1(n), kThreads, 0, s>>>(n, rowptr, val, deg);
  GDD_LAUNCHED();
  k_row_sums_long<<<grid1(n, 64), kThreads, 0, s>>>(n, rowptr, val, deg);
  GDD_LAUNCHED();
  k_er<<<grid1(nnz), kThreads, 0, s>>>(nnz, rows, col, val, deg, er);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_softmax_rows(int64_t n, int C, const float* x, float* p, gdd_stream_t stream) {
  GDD_REQUIRE(n >= 0 && C > 0 && (n == 0 || (x && p)), "softmax_rows: bad arguments");
  if (n == 0) return GDD_OK;
  k_softmax_rows<<<grid1(n), kThreads, 0, to_hip(stream)>>>(n, C, x, p);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" size_t gdd_topk_ws_bytes(int64_t nnz, int nsets) {
  const size_t S = (size_t)std::max(nsets, 1);
  const size_t nblk = (size_t)((nnz + kTkBlk - 1) / kTkBlk);
  return align256(sizeof(uint32_t) * (size_t)nnz * S) + align256(sizeof(TkState) * S) +
         align256(sizeof(uint32_t) * 256 * S) + 2 * align256(sizeof(int2) * nblk * S) + 256;
}

extern "C" int gdd_class_topk(int64_t nnz, const int32_t* rows, const int32_t* col, const float* er,
                              int nsets, const float* probs, int64_t m, int32_t* sel, void* ws,
                              size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(nnz >= 0 && nnz < INT_MAX && nsets >= 1 && m >= 0 && m <= nnz, "class_topk: bad shape");
  GDD_REQUIRE(probs || nsets == 1, "class_topk: several sets need class probabilities");
  GDD_REQUIRE(ws && (nnz == 0 || (er && (!probs || (rows && col)))) && (m == 0 || sel),
              "class_topk: null pointer");
  if (m == 0) return GDD_OK;
  hipStream_t s = to_hip(stream);
  const int nblk = (int)((nnz + kTkBlk - 1) / kTkBlk);
  Carver cv(ws, ws_bytes);
  uint32_t* keys = cv.take<uint32_t>((size_t)nnz * nsets);
  TkState* st = cv.take<TkState>(nsets);
  uint32_t* hist = cv.take<uint32_t>(256 * (size_t)nsets);
  int2* cnt = cv.take<int2>((size_t)nblk * nsets);
  int2* off = cv.take<int2>((size_t)nblk * nsets);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "class_topk: workspace too small");
  k_class_keys<<<grid1(nnz), kThreads, 0, s>>>(nnz, nsets, rows, col, er, probs, keys);
  GDD_LAUNCHED();
  k_tk_init<<<nsets, 256, 0, s>>>(nsets, m, st, hist);
  GDD_LAUNCHED();
  const unsigned gx = (unsigned)std::min<int64_t>(std::max<int64_t>(nblk, 1), 1024);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    k_tk_hist<<<dim3(gx, nsets), kThreads, 0, s>>>(nnz, shift, keys, st, hist);
    GDD_LAUNCHED();
    k_tk_pick<<<nsets, 256, 0, s>>>(shift, st, hist);
    GDD_LAUNCHED();
  }
  k_tk_count<<<dim3(nblk, nsets), kThreads, 0, s>>>(nnz, nblk, keys, st, cnt);
  GDD_LAUNCHED();
  k_tk_scan<<<nsets, 256, 0, s>>>(nblk, cnt, off);
  GDD_LAUNCHED();
  k_tk_emit<<<dim3(nblk, nsets), kThreads, 0, s>>>(nnz, nblk, m, keys, st, off, sel);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" size_t gdd_compress_ws_bytes(int kk) {
  return align256(sizeof(unsigned long long) * (size_t)kk * kk) +
         align256(sizeof(unsigned long long) * (size_t)kk) + align256(sizeof(FixState)) + 256;
}

extern "C" int gdd_graph_compress(int64_t n, const int32_t* labels, int kk, int64_t m,
                                  const int32_t* rows, const int32_t* col, const float* val,
                                  const int32_t* sel, float* out, void* ws, size_t ws_bytes,
                                  gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && kk > 0 && m >= 0, "graph_compress: bad shape");
  GDD_REQUIRE(labels && out && ws && (m == 0 || (rows && col)), "graph_compress: null pointer");
  hipStream_t s = to_hip(stream);
  Carver cv(ws, ws_bytes);
  unsigned long long* acc = cv.take<unsigned long long>((size_t)kk * kk);
  unsigned long long* size = cv.take<unsigned long long>(kk);
  FixState* fs = cv.take<FixState>(1);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "graph_compress: workspace too small");
  GDD_HIP(hipMemsetAsync(acc, 0, sizeof(unsigned long long) * (size_t)kk * kk, s));
  GDD_HIP(hipMemsetAsync(size, 0, sizeof(unsigned long long) * (size_t)kk, s));
  GDD_HIP(hipMemsetAsync(fs, 0, sizeof(FixState), s));
  GDD_REQUIRE(kk <= 16384, "graph_compress: at most 16384 clusters");
  k_label_sizes<<<(unsigned)std::min<int64_t>(grid1(n), 256), kThreads, sizeof(unsigned) * kk, s>>>(
      n, labels, kk, size);
  GDD_LAUNCHED();
  if (m > 0) {
    k_fix_maxabs<<<(unsigned)std::min<int64_t>(grid1(m), 1024), kThreads, 0, s>>>(m, sel, val, fs);
    GDD_LAUNCHED();
    k_compress_acc<<<grid1(m), kThreads, 0, s>>>(m, sel, rows, col, val, labels, kk, fs, acc);
    GDD_LAUNCHED();
  }
  k_compress_fin<<<grid1((int64_t)kk * kk), kThreads, 0, s>>>(kk, m, acc, size, fs, out);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" size_t gdd_select_csr_ws_bytes(int64_t n) {
  return align256(sizeof(int32_t) * (n + 1)) + scan_i32_ws_bytes(n + 1) + 512;
}

extern "C" int gdd_select_csr(int64_t n, const int32_t* rows, const int32_t* col, const float* val,
                              int64_t m, const int32_t* sel, int32_t* rowptr_out, int32_t* col_out,
                              float* val_out, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && m >= 0 && m < INT_MAX, "select_csr: bad shape");
  GDD_REQUIRE(rowptr_out && ws && (m == 0 || (rows && col && sel && col_out && val_out)),
              "select_csr: null pointer");
  hipStream_t s = to_hip(stream);
  const size_t sb = scan_i32_ws_bytes(n + 1);
  Carver cv(ws, ws_bytes);
  int32_t* cnt = cv.take<int32_t>(n + 1);
  char* scan_ws = cv.take<char>(sb);
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "select_csr: workspace too small");
  GDD_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (n + 1), s));
  if (m > 0) {
    k_sel_rows<<<grid1(m), kThreads, 0, s>>>(m, sel, rows, col, val, cnt, col_out, val_out);
    GDD_LAUNCHED();
  }
  return exclusive_scan_i32(cnt, rowptr_out, n + 1, scan_ws, sb, s);
}
