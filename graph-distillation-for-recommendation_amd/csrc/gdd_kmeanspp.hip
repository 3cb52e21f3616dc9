// gdd_kmeanspp.hip — greedy k-means++ seeding on the device (sklearn _kmeans_plusplus,
// sklearn/cluster/_kmeans.py:174-272), with the host's RNG draws passed in.
//
// What has to match, element for element (oracle/gdd_oracle.c restates each piece and is pinned
// against scikit-learn 1.7.2 + numpy 2.2 + OpenBLAS 0.3.29 SkylakeX, 8 BLAS threads):
//   distances   _euclidean_distances(C, X, squared=True) on fp32 X: rows of X in chunks of
//               batch_size upcast to fp64, d = ((-2 C.X^T) + |c|^2) + |x|^2 with numpy's fp64 einsum
//               norms, fp32, max(., 0). The fp64 product's summation order is OpenBLAS's and depends
//               on the chunk shape (ddot, dgemv_t, the TN small-matrix dgemm, the regular dgemm and
//               its edge kernels); skl_mode() picks it per (point, trial). Almost every shape is the
//               plain k-ordered chain (the fast path); the others take skl_dot().
//   potentials  first centre: closest @ w = sdot (64 lane chains); trials (T >= 2): (T, n) @ (n, 1)
//               = sgemv_t: per trial, fp32 lane chains inside blocks of 4096 entries (NBMAX), the
//               block results added in order, the n%4 trailing entries last.
//   candidates  searchsorted_left(cumsum_fp64(w * closest), u * pot), clipped to n - 1.
//
// Layout: the points are cut into blocks of 4096 (kBlk) — the sgemv_t block and the unit of the
// cumulative potential. One launch per round c = 1..k-1, grid (blocks, T), 256 threads:
//   fold      every workgroup folds round c-1's per-block potential terms into the T potentials,
//             takes the argmin (np.argmin: first minimum, NaN first) and the winner's row;
//   draw      finds the block where the winner's cumulative potential crosses u * pot (per-block
//             fp64 totals, scanned in a fixed order) and counts inside that block: its trial's
//             candidate (cum is non-decreasing, so searchsorted_left = #{cum < r});
//   distance  its block of points against that candidate, np.minimum with the winner's row;
//   terms     the block's fp64 cumulative total and the block's sgemv_t lane chains (4 or 8 fp32
//             chains of <= 1024 entries) — round c+1's fold reads T * blocks values, never a row.
// A last single-workgroup launch folds round k-1. The cumulative potential is evaluated block-wise
// (thread-sequential, then fixed shuffle/wave combinations) instead of strictly left to right; every
// workgroup evaluates the same numbers. It can differ from numpy's by fp64 rounding only, and every
// search checks whether that rounding could decide its draw (cum_tol): if so, one thread replays
// numpy's left-to-right sum (np_cumsum_search), so every draw is numpy's.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>

#include <cstring>

#include "gdd_common.hpp"

namespace gdd {
GDD_STAMP_TABLE(kpp)
namespace {

constexpr int kMaxTrials = 16;
constexpr int kBlk = 4096;               // sgemv_t NBMAX and the cumulative-potential block
constexpr int kThr = 1024;               // 16 waves: one workgroup per (block, trial)
constexpr int kWaves = kThr / 64;
constexpr int kPer = kBlk / kThr;        // 4 entries per thread
constexpr int kBlasThreads = 8;          // OpenBLAS threads of the pinned reference run

struct KppState {
  float pot;  // the first centre's potential (sdot)
  int pad;
};

__device__ __forceinline__ float np_minimum(float a, float b) {
  if (a != a || b != b) return __builtin_nanf("");
  return b < a ? b : a;
}

// row_norms of the upcast chunk (pairwise.py _euclidean_distances_upcast): numpy's fp64 einsum
// order — 2 lanes over 8-element blocks, high pair first, zero-padded pairs for the tail, a0 + a1.
// fp32 squares are exact in fp64, so only the order matters.
__device__ __forceinline__ double npy_sumsq_f64(const float* __restrict__ x, int dim) {
  double a0 = 0.0, a1 = 0.0;
  int j = 0;
  for (; dim - j >= 8; j += 8) {
#pragma unroll
    for (int v = 3; v >= 0; --v) {
      const double e0 = x[j + 2 * v], e1 = x[j + 2 * v + 1];
      a0 = e0 * e0 + a0;
      a1 = e1 * e1 + a1;
    }
  }
  for (; j < dim; j += 2) {
    const double e0 = x[j], e1 = j + 1 < dim ? (double)x[j + 1] : 0.0;
    a0 = e0 * e0 + a0;
    a1 = e1 * e1 + a1;
  }
  return a0 + a1;
}

// ---- OpenBLAS SkylakeX sdot (kernel/x86_64/sdot.c + sdot_microk_skylakex-2.c) ---------------------
// One wave: lane u*16+l runs AVX-512 accumulator u, lane l of the 64-wide loop; they fold to 4 x 8
// AVX2 accumulators for the 32-wide remainder; then ((a0+a1)+a2)+a3, 8 -> 4 by halves,
// (h0+h1)+(h2+h3); the scalar tail is added in double. Lane 0 returns the value.
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
    if (n64 < n1) {
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

__device__ float sdot_skx_wave(const float* __restrict__ x, const float* __restrict__ y, int64_t n,
                               float* scratch /* 192 floats of LDS owned by this wave */) {
  const int lane = threadIdx.x & 63;
  const int64_t n64 = n & ~63ll;
  const int64_t ri = n64 + lane;
  const float rx = ri < n ? x[ri] : 0.f;
  const float ry = ri < n ? (y ? y[ri] : 1.0f) : 0.f;
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

// ---- scikit-learn's upcast distance: which OpenBLAS summation order element (point i, trial t)
// gets (oracle_skl_dot_mode in oracle/gdd_oracle.c states the rules and where they were pinned) ----
enum SklMode { SKL_SEQ, SKL_TREE8, SKL_HALVES8, SKL_GEMV4, SKL_GEMV2, SKL_L2E, SKL_L4E, SKL_DDOT };

struct SklPlan {
  int64_t n, B;  // points; rows per chunk of _euclidean_distances_upcast for this call
  int T, dim;    // candidate rows of the call (1: the first centre)
  int all_seq;   // every element takes the plain k-ordered chain (no K split): the fast path
  int pad;
};

__device__ __forceinline__ int skl_gemv_kind(int64_t j, int64_t w) {
  const int64_t w4 = w & ~3ll;
  return (j >= w4 && (w & 2) && j < w4 + 2) ? SKL_GEMV2 : SKL_GEMV4;
}

__device__ int skl_mode(const SklPlan& p, int64_t i, int t, int* split) {
  const int64_t s = (i / p.B) * p.B;
  const int64_t m = min(p.B, p.n - s), r = i - s;
  *split = 0;
  if (p.T == 1 && m == 1) return SKL_DDOT;
  if (p.T == 1) {  // dgemv_t; columns split over the BLAS threads when dim * m >= 460800
    int64_t a = 0, wd = m;
    if ((int64_t)p.dim * m >= 460800) {
      int64_t left = m, s0 = 0;
      for (int cpu = 0; left > 0; ++cpu) {
        const int rest = kBlasThreads - cpu;
        int64_t w = rest > 0 ? (left + rest - 1) / rest : left;
        w = max<int64_t>(w, 4);
        w = min<int64_t>(w, left);
        if (r < s0 + w) {
          a = s0;
          wd = w;
          break;
        }
        s0 += w;
        left -= w;
      }
    }
    return skl_gemv_kind(r - a, wd);
  }
  if (m == 1) return skl_gemv_kind(t, p.T);
  const double mnk = (double)m * (double)p.T * (double)p.dim;
  if (mnk <= 1e6 && m * p.T <= 1200 && p.dim >= 32)  // TN small-matrix kernel
    return (r < (m & ~3ll) || t < (p.T & ~3)) ? SKL_TREE8 : SKL_HALVES8;
  const bool threaded = kBlasThreads >= 2 && mnk >= 524288.0;
  if (p.dim > 384) *split = threaded ? (p.dim + 1) / 2 : ((p.dim / 2 + 15) / 16) * 16;
  if (!threaded && m > 192 && t < (p.T / 12) * 12) {  // single-threaded edge kernels
    const int64_t e = (m & ~15ll) + ((m & 8) ? 8 : 0);
    if (r >= e) return ((m & 4) && r < e + 4) ? SKL_L2E : SKL_L4E;
  }
  return SKL_SEQ;
}

// the k-ordered fp64 chain (fp32 products are exact in fp64: fma == mul + add)
__device__ __forceinline__ double dot_seq(const double* __restrict__ c, const float* __restrict__ x,
                                          int dim) {
  double dot = 0.0;
  int j = 0;
  for (; j + 8 <= dim; j += 8) {  // eight loads in flight ahead of the ordered fmas
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) dot = __builtin_fma(c[j + u], (double)v[u], dot);
  }
  for (; j < dim; ++j) dot = __builtin_fma(c[j], (double)x[j], dot);
  return dot;
}

__device__ double skl_dot(const double* __restrict__ c, const float* __restrict__ x, int d, int mode,
                          int sp) {
  switch (mode) {
    case SKL_SEQ: {
      if (sp <= 0) return dot_seq(c, x, d);
      double a = 0.0, b = 0.0;
      for (int k = 0; k < sp; ++k) a = __builtin_fma(c[k], (double)x[k], a);
      for (int k = sp; k < d; ++k) b = __builtin_fma(c[k], (double)x[k], b);
      return a + b;
    }
    case SKL_TREE8:
    case SKL_HALVES8: {
      double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      int k = 0;
      for (; k + 8 <= d; k += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = __builtin_fma(c[k + u], (double)x[k + u], a[u]);
      }
#pragma unroll
      for (int u = 0; u < 7; ++u)
        if (k + u < d) a[u] = __builtin_fma(c[k + u], (double)x[k + u], a[u]);
      if (mode == SKL_TREE8) return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      return ((a[0] + a[4]) + (a[2] + a[6])) + ((a[1] + a[5]) + (a[3] + a[7]));
    }
    case SKL_GEMV4:
    case SKL_GEMV2: {
      const int d4 = d & ~3;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      for (int k = 0; k < d4; k += 4) {
        if (mode == SKL_GEMV4) {
          a0 = __builtin_fma(c[k], (double)x[k], a0);
          a1 = __builtin_fma(c[k + 1], (double)x[k + 1], a1);
          a2 = __builtin_fma(c[k + 2], (double)x[k + 2], a2);
          a3 = __builtin_fma(c[k + 3], (double)x[k + 3], a3);
        } else {
          a0 = __builtin_fma(c[k], (double)x[k], a0);
          a1 = __builtin_fma(c[k + 1], (double)x[k + 1], a1);
          a0 = __builtin_fma(c[k + 2], (double)x[k + 2], a0);
          a1 = __builtin_fma(c[k + 3], (double)x[k + 3], a1);
        }
      }
      double r = 0.0 + (mode == SKL_GEMV4 ? (a0 + a2) + (a1 + a3) : a0 + a1);
      if (d > d4) {
        double s = c[d4] * (double)x[d4];
        for (int k = d4 + 1; k < d; ++k) s = __builtin_fma(c[k], (double)x[k], s);
        r = r + s;
      }
      return r;
    }
    case SKL_L2E: {
      const int db = d & ~1;
      double a0 = 0.0, a1 = 0.0;
      for (int k = 0; k < db; k += 2) {
        a0 = __builtin_fma(c[k], (double)x[k], a0);
        a1 = __builtin_fma(c[k + 1], (double)x[k + 1], a1);
      }
      double r = a0 + a1;
      for (int k = db; k < d; ++k) r = __builtin_fma(c[k], (double)x[k], r);
      return r;
    }
    case SKL_L4E: {
      const int db = d & ~3;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      for (int k = 0; k < db; k += 4) {
        a0 = __builtin_fma(c[k], (double)x[k], a0);
        a1 = __builtin_fma(c[k + 1], (double)x[k + 1], a1);
        a2 = __builtin_fma(c[k + 2], (double)x[k + 2], a2);
        a3 = __builtin_fma(c[k + 3], (double)x[k + 3], a3);
      }
      double r = (a0 + a1) + (a2 + a3);
      for (int k = db; k < d; ++k) r = __builtin_fma(c[k], (double)x[k], r);
      return r;
    }
    default: {  // SKL_DDOT: 4 x 8 lanes over 32-blocks, folded to 4 x 4, 16-blocks, tail in order
      const int n1 = d & ~15, n32 = n1 & ~31;
      double r = 0.0;
      if (n1) {
        double z[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int l = 0; l < 8; ++l) z[u][l] = 0.0;
        for (int i = 0; i < n32; i += 32)
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int l = 0; l < 8; ++l)
              z[u][l] = __builtin_fma(c[i + u * 8 + l], (double)x[i + u * 8 + l], z[u][l]);
        double q[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int l = 0; l < 4; ++l) q[u][l] = z[u][l] + z[u][l + 4];
        for (int i = n32; i < n1; i += 16)
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int l = 0; l < 4; ++l)
              q[u][l] = __builtin_fma(c[i + u * 4 + l], (double)x[i + u * 4 + l], q[u][l]);
        double h[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) h[l] = ((q[0][l] + q[1][l]) + q[2][l]) + q[3][l];
        r = (h[0] + h[2]) + (h[1] + h[3]);
      }
      for (int k = n1; k < d; ++k) r = __builtin_fma((double)x[k], c[k], r);
      return r;
    }
  }
}

// does every element of the chunk with m rows take the plain k-ordered chain? (the per-chunk form of
// the host's skl_all_seq: a call whose last chunk is small runs edge kernels there, but its other
// chunks stay plain)
__device__ __forceinline__ bool skl_chunk_seq(const SklPlan& p, int64_t m) {
  if (p.T == 1 || p.dim > 384 || m <= 1) return false;
  const double mnk = (double)m * p.T * p.dim;
  if (mnk <= 1e6 && m * p.T <= 1200 && p.dim >= 32) return false;
  const bool threaded = kBlasThreads >= 2 && mnk >= 524288.0;
  if (!threaded && m > 192 && p.T >= 12 && (m & 7) != 0) return false;
  return true;
}

__device__ __forceinline__ double skl_point_dot(const SklPlan& p, const double* __restrict__ c,
                                                const float* __restrict__ x, int64_t i, int t) {
  if (p.all_seq) return dot_seq(c, x, p.dim);
  int sp;
  const int mode = skl_mode(p, i, t, &sp);
  if (mode == SKL_SEQ && sp == 0) return dot_seq(c, x, p.dim);
  return skl_dot(c, x, p.dim, mode, sp);
}

// the plain k-ordered fp64 chains of the kPer points tid + kThr * q of the block at j0 against the
// staged candidate s_c (all_seq plans): the points' chains are interleaved and each step's loads for
// all of them are in flight together (float4 when rows are 16-byte aligned)
__device__ __forceinline__ void seq_dots(const float* __restrict__ X, int dim, int64_t n, int64_t j0,
                                         const double* __restrict__ s_c, double (&dot)[kPer]) {
  const int tid = threadIdx.x;
  const float* xr[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = j0 + tid + kThr * q;
    xr[q] = X + (i < n ? i : j0) * (int64_t)dim;
    dot[q] = 0.0;
  }
  int j = 0;
  if ((dim & 3) == 0 && ((uintptr_t)X & 15) == 0) {
    for (; j + 8 <= dim; j += 8) {
      float4 u0[kPer], u1[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        u0[q] = *reinterpret_cast<const float4*>(xr[q] + j);
        u1[q] = *reinterpret_cast<const float4*>(xr[q] + j + 4);
      }
      const double c0 = s_c[j], c1 = s_c[j + 1], c2 = s_c[j + 2], c3 = s_c[j + 3];
      const double c4 = s_c[j + 4], c5 = s_c[j + 5], c6 = s_c[j + 6], c7 = s_c[j + 7];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        double d = dot[q];
        d = __builtin_fma(c0, (double)u0[q].x, d);
        d = __builtin_fma(c1, (double)u0[q].y, d);
        d = __builtin_fma(c2, (double)u0[q].z, d);
        d = __builtin_fma(c3, (double)u0[q].w, d);
        d = __builtin_fma(c4, (double)u1[q].x, d);
        d = __builtin_fma(c5, (double)u1[q].y, d);
        d = __builtin_fma(c6, (double)u1[q].z, d);
        d = __builtin_fma(c7, (double)u1[q].w, d);
        dot[q] = d;
      }
    }
    if (j + 4 <= dim) {
      float4 u0[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) u0[q] = *reinterpret_cast<const float4*>(xr[q] + j);
      const double c0 = s_c[j], c1 = s_c[j + 1], c2 = s_c[j + 2], c3 = s_c[j + 3];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        double d = dot[q];
        d = __builtin_fma(c0, (double)u0[q].x, d);
        d = __builtin_fma(c1, (double)u0[q].y, d);
        d = __builtin_fma(c2, (double)u0[q].z, d);
        d = __builtin_fma(c3, (double)u0[q].w, d);
        dot[q] = d;
      }
      j += 4;
    }
  }
  for (; j + 4 <= dim; j += 4) {
    float u[kPer][4];
#pragma unroll
    for (int q = 0; q < kPer; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) u[q][v] = xr[q][j + v];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const double cv = s_c[j + v];
#pragma unroll
      for (int q = 0; q < kPer; ++q) dot[q] = __builtin_fma(cv, (double)u[q][v], dot[q]);
    }
  }
  for (; j < dim; ++j) {
    const double cv = s_c[j];
#pragma unroll
    for (int q = 0; q < kPer; ++q) dot[q] = __builtin_fma(cv, (double)xr[q][j], dot[q]);
  }
}

// seq_dots from the transpose XT (dim x n): lanes read consecutive points of one feature, so every
// load is coalesced (a row-major read of 4096 scattered rows refetches each line per feature group)
__device__ __forceinline__ void seq_dots_t(const float* __restrict__ XT, int dim, int64_t n, int64_t j0,
                                           const double* __restrict__ s_c, double (&dot)[kPer]) {
  const int tid = threadIdx.x;
  int64_t ix[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = j0 + tid + kThr * q;
    ix[q] = i < n ? i : j0;
    dot[q] = 0.0;
  }
  int j = 0;
  for (; j + 8 <= dim; j += 8) {
    float u[8][kPer];
#pragma unroll
    for (int v = 0; v < 8; ++v)
#pragma unroll
      for (int q = 0; q < kPer; ++q) u[v][q] = XT[(int64_t)(j + v) * n + ix[q]];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const double cv = s_c[j + v];
#pragma unroll
      for (int q = 0; q < kPer; ++q) dot[q] = __builtin_fma(cv, (double)u[v][q], dot[q]);
    }
  }
  for (; j < dim; ++j) {
    const double cv = s_c[j];
#pragma unroll
    for (int q = 0; q < kPer; ++q) dot[q] = __builtin_fma(cv, (double)XT[(int64_t)j * n + ix[q]], dot[q]);
  }
}

// ---- the block-wise fp64 cumulative potential ----------------------------------------------------
// prefix(e) of entry e = 16*tid + u of a block: thread-sequential running sum r_u, the exclusive
// shuffle scan E of the thread totals inside the wave, the wave totals added in wave order B:
// prefix = (B + E) + r_u. Both the producer of a block's total and the searches use this function,
// so a block's total equals the prefix of its last entry bit for bit.
__device__ __forceinline__ void block_prefix(const double (&v)[kPer], double (&pre)[kPer],
                                             double* s_wave /* kWaves */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double r[kPer];
  double run = 0.0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    run = run + v[u];
    r[u] = run;
  }
  double inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(inc, o);
    if (lane >= o) inc = inc + y;
  }
  double ex = __shfl_up(inc, 1);
  if (lane == 0) ex = 0.0;
  __syncthreads();  // s_wave may still be read by a previous call
  if (lane == 63) s_wave[wave] = inc;
  __syncthreads();
  double B = 0.0;
  for (int q = 0; q < wave; ++q) B = B + s_wave[q];
  const double base = B + ex;
#pragma unroll
  for (int u = 0; u < kPer; ++u) pre[u] = base + r[u];
}

// ---- numpy's left-to-right cumsum, exactly --------------------------------------------------------
// Every prefix in this file is a blocked evaluation of np.cumsum(w * closest, dtype=float64)
// (sklearn/utils/extmath.py stable_cumsum). Any summation order of m non-negative terms lies within
// gamma_{m-1} = (m-1)u / (1 - (m-1)u), u = 2^-53, relative of the exact sum S (Higham, "Accuracy and
// Stability of Numerical Algorithms", 2nd ed., eq. 4.4), so a blocked prefix c and numpy's sequential
// prefix s of the same entry differ by at most 2 gamma S. A decision `c < r` can come out differently
// from numpy's `s < r` only if c and s straddle r, which needs |c - r| <= 2 gamma S with S <= r / (1 -
// gamma): tol = 2.25 n u r bounds that for every n < 2^31. Each search below checks the prefixes
// that decide its draw against tol (the two neighbours of a binary search's answer; every counted
// entry of a ballot count; the block boundaries of the multi-block scan) and, when one is that close,
// one thread replays numpy's sum strictly left to right. For a draw the check passes, the blocked
// answer IS numpy's; the replay runs with probability ~5 n u per draw.
//   exact = 1: that rule; 0: never replay (test only: shows a case is adversarial); 2: always replay.
__device__ __forceinline__ double cum_tol(int exact, int64_t n, double r) {
  return exact == 2 ? __builtin_inf() : exact == 0 ? -1.0 : 2.25 * (double)n * 0x1p-53 * r;
}

// searchsorted_left(np.cumsum(w * row, dtype=float64), r): the products in fp32, the running sum in
// fp64, entry by entry.
// Rows in LDS (n <= 4096: the single-block paths): one thread, the plain walk.
__device__ __noinline__ int64_t np_cumsum_search(const float* row, const float* w, int64_t n, double r) {
  double run = 0.0;
  for (int64_t e = 0; e < n; ++e) {
    run = run + (double)((w ? w[e] : 1.0f) * row[e]);
    if (!(run < r)) return e;
  }
  return n;
}

// Rows in global memory (the multi-block rounds, up to millions of entries): one whole wave. Lane j
// loads entry e0 + j of the next 64-entry group (coalesced, a group ahead of the adds); every lane
// runs the same dependent chain, taking entry j from lane j (readlane, uniform), and tests the
// threshold off the chain; a group that reaches r is walked again entry by entry. Returns the same
// value in every lane.
__device__ __forceinline__ float lane_f(float x, int j) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), j));
}

__device__ __forceinline__ int64_t np_cumsum_search_wave(const float* row, const float* w, int64_t n,
                                                         double r) {
  const int lane = threadIdx.x & 63;
  auto ld = [&](int64_t b) {
    const int64_t e = min(b + lane, n - 1);  // past n: clamped, never added
    return (w ? w[e] : 1.0f) * row[e];
  };
  double run = 0.0;
  int64_t e0 = 0;
  float xa = ld(0);
  for (; e0 + 64 <= n; e0 += 64) {
    const float xb = ld(e0 + 64);
    double s = run;
    bool hit = false;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      s = s + (double)lane_f(xa, j);
      hit = hit || !(s < r);
    }
    if (hit) {
      s = run;
      for (int j = 0; j < 64; ++j) {
        s = s + (double)lane_f(xa, j);
        if (!(s < r)) return e0 + j;
      }
    }
    run = s;
    xa = xb;
  }
  for (int j = 0; e0 + j < n; ++j) {
    run = run + (double)lane_f(xa, j);
    if (!(run < r)) return e0 + j;
  }
  return n;
}

// ---- the trials' potentials from their per-block sgemv_t terms -------------------------------------
struct KppArgs {
  int64_t n, m1;      // points; m1 = n & ~3 (the entries under sgemv_t blocks)
  int dim, T, nblk, nsg;  // nblk = ceil(n / 4096); nsg = ceil(m1 / 4096)
  const float* X;
  const float* XT;    // dim x n transpose for the plain-chain distances (nullptr: read X rows)
  const float* w;     // sample weights (nullptr: ones)
  const double* xsq;
  const float* closest0;
  const double* fsum0;  // [nblk] block totals of w * closest0
  float* dist[2];     // [T][n] by round parity
  float* vblk[2];     // [T][nblk] sgemv_t block results
  double* fsum[2];    // [T][nblk] cumulative-potential block totals
  double* pfx[2];     // [T][n] the block prefixes behind fsum (nullptr: recomputed by the count)
  int64_t* cand[2];   // [kMaxTrials]
  float* pot1;        // [2] T == 1: the round's potential (sdot), by parity
  int* winq;          // [2] round c-1's winning trial, by the parity of c (the split-round path)
  const double* uniforms;
  const KppState* st;
  float* centers;
  int64_t* indices;
  SklPlan plan;
  int exact;          // cum_tol's mode
  const float* D;     // the n x n distance table (plain-chain plans, n <= kDmBigMax), or nullptr
};

__device__ __forceinline__ float wv(const float* w, int64_t i) { return w ? w[i] : 1.0f; }

// potential of trial tr of the round whose terms are at parity q: the block results in order, then
// the m3 trailing entries (their products folded as the sgemv_t scalar tail: p0, fma, fma)
__device__ float fold_pot(const KppArgs& a, int q, int tr) {
  const float* vb = a.vblk[q] + (int64_t)tr * a.nblk;
  float y = 0.f;
  int b = 0;
  for (; b + 8 <= a.nsg; b += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = vb[b + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) y = y + v[u];
  }
  for (; b < a.nsg; ++b) y = y + vb[b];
  if (a.m1 < a.n) {
    const float* row = a.dist[q] + (int64_t)tr * a.n;
    float s = row[a.m1] * wv(a.w, a.m1);
    for (int64_t o = a.m1 + 1; o < a.n; ++o) s = __builtin_fmaf(row[o], wv(a.w, o), s);
    y = y + s;
  }
  return y;
}

// the T potentials of the round at parity q into s_pot; returns the argmin (np.argmin semantics).
// The per-block sgemv_t results are staged through LDS in chunks (every thread loads, one memory
// round trip per chunk), then T threads fold their trial's chunk in block order: the same sequential
// fp32 chain as fold_pot, without one dependent global load group per 8 blocks.
constexpr int kFoldChunk = 512;
__device__ int fold_round(const KppArgs& a, int q, float* s_pot) {
  __shared__ float s_fold[kFoldChunk * kMaxTrials];
  const int tid = threadIdx.x;
  if (a.T == 1) {
    if (tid == 0) s_pot[0] = a.pot1[q];
  } else {
    float y = 0.f;
    for (int64_t b0 = 0; b0 < a.nsg; b0 += kFoldChunk) {
      const int m = (int)min<int64_t>(kFoldChunk, a.nsg - b0);
      for (int e = tid; e < m * a.T; e += blockDim.x) {
        const int tr = e / m, bb = e - tr * m;
        s_fold[tr * kFoldChunk + bb] = a.vblk[q][(int64_t)tr * a.nblk + b0 + bb];
      }
      __syncthreads();
      if (tid < a.T) {
        const float* v = s_fold + tid * kFoldChunk;
        for (int bb = 0; bb < m; ++bb) y = y + v[bb];
      }
      __syncthreads();
    }
    if (tid < a.T) {
      if (a.m1 < a.n) {
        const float* row = a.dist[q] + (int64_t)tid * a.n;
        float sx = row[a.m1] * wv(a.w, a.m1);
        for (int64_t o = a.m1 + 1; o < a.n; ++o) sx = __builtin_fmaf(row[o], wv(a.w, o), sx);
        y = y + sx;
      }
      s_pot[tid] = y;
    }
  }
  __syncthreads();
  int b = 0;
  for (int t = 1; t < a.T; ++t) {
    const float pb = s_pot[b], pt = s_pot[t];
    if (pb == pb && (pt < pb || pt != pt)) b = t;
  }
  return b;
}

// ---- first centre -----------------------------------------------------------------------------------
// One workgroup per block: |x|^2 (numpy einsum order), the distances to the first centre (T = 1
// orders: dgemv_t / ddot), and the block's cumulative-potential total.
__global__ __launch_bounds__(kThr) void k_kpp_init(KppArgs a, SklPlan p1, int64_t first_id,
                                                   double* __restrict__ xsq_out,
                                                   float* __restrict__ closest_out,
                                                   double* __restrict__ fsum_out) {
  extern __shared__ double s_c[];  // dim doubles, then the block's distances (fp32)
  __shared__ double s_wave[kWaves];
  __shared__ double s_sc;
  const int tid = threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.x * kBlk;
  const float* xc = a.X + first_id * a.dim;
  for (int j = tid; j < a.dim; j += kThr) s_c[j] = (double)xc[j];
  if (tid == 0) s_sc = npy_sumsq_f64(xc, a.dim);
  __syncthreads();
  float* s_d = reinterpret_cast<float*>(s_c + a.dim);
  const double sc = s_sc;
#pragma unroll 1
  for (int u = 0; u < kPer; ++u) {
    const int o = tid + kThr * u;
    const int64_t i = j0 + o;
    float f = 0.f;
    if (i < a.n) {
      const float* xi = a.X + i * a.dim;
      const double s = npy_sumsq_f64(xi, a.dim);
      xsq_out[i] = s;
      const double dot = skl_point_dot(p1, s_c, xi, i, 0);
      f = (float)(((-2.0 * dot) + sc) + s);
      f = f < 0.f ? 0.f : f;
      closest_out[i] = f;
    }
    s_d[o] = f;
  }
  __syncthreads();
  double v[kPer], pre[kPer];
  float xs[kPer];  // every read before the weights' branches (r04)
#pragma unroll
  for (int u = 0; u < kPer; ++u) xs[u] = s_d[kPer * tid + u];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t e = j0 + kPer * tid + u;
    v[u] = e < a.n ? (double)(wv(a.w, e) * xs[u]) : 0.0;
  }
  block_prefix(v, pre, s_wave);
  const int64_t last = min<int64_t>(a.n, j0 + kBlk) - 1 - j0;
  if (tid == (int)(last / kPer)) fsum_out[blockIdx.x] = pre[last % kPer];
}

// the first centre's potential (closest @ w: sdot), index and row
__global__ void k_kpp_first(int64_t n, int dim, const float* __restrict__ X,
                            const float* __restrict__ w, const float* __restrict__ closest0,
                            int64_t first_id, KppState* __restrict__ st,
                            float* __restrict__ centers, int64_t* __restrict__ indices) {
  __shared__ float scratch[192];
  const float p = sdot_skx_wave(closest0, w, n, scratch);
  if (threadIdx.x == 0) {
    st->pot = p;
    indices[0] = first_id;
  }
  for (int j = threadIdx.x; j < dim; j += blockDim.x) centers[j] = X[first_id * dim + j];
}

// the first centre's potential with unit weights for large n: the same 64 lane chains as
// sdot_skx_wave (lane l adds entries l, l + 64, ... in order), with waves 1..15 staging chunks of
// 256 x 64 entries (64 KB) into a two-slot LDS ring for wave 0 — one wave alone keeps only ~16 KB
// of loads in flight (2.8 ms at 2.45M entries)
constexpr int kFirstSteps = 256;  // 64-entry steps per staged chunk
__global__ __launch_bounds__(1024) void k_kpp_first_big(int64_t n, int dim, const float* __restrict__ X,
                                                        const float* __restrict__ closest0, int64_t first_id,
                                                        KppState* __restrict__ st, float* __restrict__ centers,
                                                        int64_t* __restrict__ indices) {
  extern __shared__ __attribute__((aligned(16))) float ring[];  // 2 x kFirstSteps * 64 floats
  __shared__ float scratch[192];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t n64 = n & ~63ll;
  constexpr int kChunk = kFirstSteps * 64;
  const int64_t nch = (n64 + kChunk - 1) / kChunk;
  auto stage = [&](int64_t ch) {  // waves 1..15
    float* dst = ring + (ch & 1) * kChunk;
    const int64_t base = ch * kChunk;
    for (int e = tid - 64; e < kChunk; e += 960) {
      const int64_t i = base + e;
      dst[e] = i < n64 ? closest0[i] : 0.f;
    }
  };
  if (wave > 0 && nch > 0) stage(0);
  __syncthreads();
  float a = 0.f;
  for (int64_t ch = 0; ch < nch; ++ch) {
    if (wave > 0) {
      if (ch + 1 < nch) stage(ch + 1);
    } else {
      const float* src = ring + (ch & 1) * kChunk + lane;
      const int steps = (int)min<int64_t>(kFirstSteps, (n64 - ch * kChunk) >> 6);
      for (int u = 0; u < steps; ++u) a = __builtin_fmaf(src[64 * u], 1.0f, a);
    }
    __syncthreads();
  }
  if (wave == 0) {
    const int64_t ri = n64 + lane;
    const float rx = ri < n ? closest0[ri] : 0.f;
    const float ry = ri < n ? 1.0f : 0.f;
    const float p = sdot_skx_finish(a, rx, ry, n, scratch);
    if (lane == 0) {
      st->pot = p;
      indices[0] = first_id;
    }
    for (int j = lane; j < dim; j += 64) centers[j] = X[first_id * dim + j];
  }
}

// T == 1: the single trial's potential is (1, n) @ (n, 1) -> sdot
__global__ void k_kpp_pot1(int64_t n, const float* __restrict__ row, const float* __restrict__ w,
                           float* __restrict__ out) {
  __shared__ float scratch[192];
  const float p = sdot_skx_wave(row, w, n, scratch);
  if (threadIdx.x == 0) *out = p;
}

// ---- distances of one block's points to the staged candidate s_c (|c|^2 = cn), np.minimum with
// the winner's row; written to drow (global) and s_d (LDS, block order)
template <bool SEQ>
__device__ __forceinline__ void block_dists(const KppArgs& a, int t, int64_t j0, double cn,
                                            const double* __restrict__ s_c,
                                            const float* __restrict__ wrow, float* __restrict__ drow,
                                            float* __restrict__ s_d) {
  const int tid = threadIdx.x;
  const int64_t n = a.n;
  if constexpr (SEQ) {
    double dot[kPer];
    if (a.XT)
      seq_dots_t(a.XT, a.dim, n, j0, s_c, dot);
    else
      seq_dots(a.X, a.dim, n, j0, s_c, dot);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int o = tid + kThr * q;
      const int64_t i = j0 + o;
      float f = 0.f;
      if (i < n) {
        f = (float)(((-2.0 * dot[q]) + cn) + a.xsq[i]);
        f = f < 0.f ? 0.f : f;
        f = np_minimum(wrow[i], f);
        drow[i] = f;
      }
      s_d[o] = f;
    }
  } else {
    // the block's points in chunks of _euclidean_distances_upcast that all take the plain chain:
    // the interleaved fast path of SEQ (only a call's small last chunk runs the edge kernels)
    bool bseq = true;
    {
      const int64_t B = a.plan.B;
      const int64_t s0 = j0 / B, s1 = min(n - 1, j0 + (int64_t)kBlk - 1) / B;
      for (int64_t sc = s0; sc <= s1; ++sc) bseq = bseq && skl_chunk_seq(a.plan, min(B, n - sc * B));
    }
    if (bseq) {
      double dot[kPer];
      if (a.XT)
        seq_dots_t(a.XT, a.dim, n, j0, s_c, dot);
      else
        seq_dots(a.X, a.dim, n, j0, s_c, dot);
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int o = tid + kThr * q;
        const int64_t i = j0 + o;
        float f = 0.f;
        if (i < n) {
          f = (float)(((-2.0 * dot[q]) + cn) + a.xsq[i]);
          f = f < 0.f ? 0.f : f;
          f = np_minimum(wrow[i], f);
          drow[i] = f;
        }
        s_d[o] = f;
      }
      return;
    }
#pragma unroll 1
    for (int q = 0; q < kPer; ++q) {
      const int o = tid + kThr * q;
      const int64_t i = j0 + o;
      float f = 0.f;
      if (i < n) {
        const float* xi = a.X + i * a.dim;
        const double dot = skl_point_dot(a.plan, s_c, xi, i, t);
        f = (float)(((-2.0 * dot) + cn) + a.xsq[i]);
        f = f < 0.f ? 0.f : f;
        f = np_minimum(wrow[i], f);
        drow[i] = f;
      }
      s_d[o] = f;
    }
  }
}

// x, or -0.0 (the identity of +: acc + -0.0 == acc for every acc, signed zeros and NaN included) when
// !in, by a bit mask: a masked chain entry then costs one dependent add. Written as `in ? acc + x : acc`
// the select sat on the chain after each add (v_add, s_nop, v_cndmask per entry; r05).
__device__ __forceinline__ float add_operand(float x, bool in) {
  return __int_as_float(__float_as_int(x) & (in ? 0xffffffffu : 0x80000000u));
}

// One unit-weight sgemv_t lane chain in LDS: acc + x over p[0], p[S], p[2S], ... (L entries). Two
// 16-entry register groups alternate: a group's reads (immediate offsets from one address) are
// issued a whole group of dependent adds ahead of their use (scheduling barriers keep them there, as
// in chain_add). Reads run at most 32 S entries past the chain: the row buffer is padded for them.
template <int S>
__device__ __forceinline__ float chain_unit_lds(const float* __restrict__ p, int L, float acc) {
  float A[16], B[16];
  auto ld = [&](float (&R)[16], int m) {
#pragma unroll
    for (int q = 0; q < 16; ++q) R[q] = p[S * (m + q)];
  };
  int m = 0;
  ld(A, 0);
  for (; m + 32 <= L; m += 32) {
    ld(B, m + 16);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = acc + A[q];
    __builtin_amdgcn_sched_barrier(0);
    ld(A, m + 32);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = acc + B[q];
    __builtin_amdgcn_sched_barrier(0);
  }
  ld(B, m + 16);  // A holds entries m .. m + 15; fewer than 32 remain
  auto grp = [&](const float* g, int e) {  // as chain_add's rest: groups of four
    if (e + 3 < L) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = acc + g[r];
    } else if (e < L) {
      acc = acc + g[0];
      acc = acc + add_operand(g[1], e + 1 < L);
      acc = acc + add_operand(g[2], e + 2 < L);
    }
  };
#pragma unroll
  for (int q = 0; q < 16; q += 4) grp(A + q, m + q);
#pragma unroll
  for (int q = 0; q < 16; q += 4) grp(B + q, m + 16 + q);
  return acc;
}
constexpr int kChainPad = 32 * 8 + 16;  // floats past the row that the chains' look-ahead may read

// sgemv_t block result of trial t over the NB (> 0) entries of s_d (weights wb, nullptr: ones), run by
// one wave; lane 0 returns it
__device__ float sgemv_block_wave(const float* __restrict__ s_d, const float* __restrict__ wb,
                                  int64_t NB, int t, int T) {
  const int lane = threadIdx.x & 63;
  const bool k4x2 = (T & 2) && t >= (T & ~3) && t < (T & ~3) + 2;
  float acc = 0.f;
  if (k4x2) {  // 4 lanes (o % 4), product then add
    if (lane < 4) {
      int64_t o = lane;
      for (; o + 28 < NB; o += 32) {
        float x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = s_d[o + 4 * q] * (wb ? wb[o + 4 * q] : 1.0f);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = acc + x[q];
      }
      for (; o < NB; o += 4) acc = acc + s_d[o] * (wb ? wb[o] : 1.0f);
    }
    const float a1 = __shfl(acc, 1), a2 = __shfl(acc, 2), a3 = __shfl(acc, 3);
    return (acc + a1) + (a2 + a3);
  }
  // 8 lanes: the first NB&4 entries into lanes 0..3, then lane (o - (NB&4)) % 8; fma
  const int64_t h4 = NB & 4;
  if (lane < 8) {
    if (lane < h4) acc = __builtin_fmaf(s_d[lane], wb ? wb[lane] : 1.0f, acc);
    int64_t o = h4 + lane;
    // (r05: chain_unit_lds' two 16-entry read-ahead groups measured slower here, 5.1 vs 3.8 us per
    // 4096-entry block at the Ali-Display shape)
    if (!wb) {  // unit weights: fma(x, 1, acc) == acc + x; 32 LDS reads ahead of the chain
      for (; o + 8 * 31 < NB; o += 256) {
        float x[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) x[q] = s_d[o + 8 * q];
#pragma unroll
        for (int q = 0; q < 32; ++q) acc = acc + x[q];
      }
    }
    for (; o + 56 < NB; o += 64) {
      float x[8], y[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        x[q] = s_d[o + 8 * q];
        y[q] = wb ? wb[o + 8 * q] : 1.0f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) acc = __builtin_fmaf(x[q], y[q], acc);
    }
    for (; o < NB; o += 8) acc = __builtin_fmaf(s_d[o], wb ? wb[o] : 1.0f, acc);
  }
  const float ql = acc + __shfl(acc, (lane + 4) & 63);  // q_l = a_l + a_{l+4}
  const float q1 = __shfl(ql, 1), q2 = __shfl(ql, 2), q3 = __shfl(ql, 3);
  return (ql + q1) + (q2 + q3);
}

__device__ __forceinline__ void waves_arrive(int* ctr);
__device__ __forceinline__ bool waves_wait(int* ctr, int target);

// ---- one seeding round ------------------------------------------------------------------------------
constexpr int kWaveFoldBlk = 16;  // k_kpp_round's barrier-free fold: up to this many sgemv_t blocks
template <bool SEQ, bool PICK = false>
__global__ __launch_bounds__(kThr) void k_kpp_round(KppArgs a, int c) {
  extern __shared__ double s_c[];  // dim doubles, then the block's distances (fp32)
  __shared__ float s_pot[kMaxTrials];
  __shared__ double s_wave[kWaves];
  __shared__ int s_jmin;
  __shared__ double s_P, s_tot;
  __shared__ int s_cnt[kWaves], s_amb[kWaves];
  __shared__ int64_t s_ct;
  __shared__ int s_pfxsync, s_pfxfail;
  const int t = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int pq = (c - 1) & 1, cq = c & 1;
  const int64_t n = a.n;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0), 20);
  const double u = a.uniforms[(int64_t)(c - 1) * a.T + t];
  if (tid == 0) {
    s_jmin = INT_MAX;
    s_pfxsync = 0;
    s_pfxfail = 0;
  }
  // r05: round c-1's candidates (lane q: trial q's) requested with the fold's block terms instead of
  // after the winner is known (that was a dependent trip)
  const int64_t csl = c >= 2 ? a.cand[pq][min(lane, a.T - 1)] : 0;
  // ---- fold round c-1 (round 0: the first centre)
  int bw = 0;
  float pot;
  const float* wrow;
  const double* wfs;
  if (c == 1) {
    pot = a.st->pot;
    wrow = a.closest0;
    wfs = a.fsum0;
    __syncthreads();
  } else if (a.T > 1 && a.T <= 64 && a.nsg <= kWaveFoldBlk && a.n - a.m1 <= 3) {
    // r05: every wave folds every trial (lane q: trial q's block terms in block order, then the
    // n % 4 tail: fold_round's operations) and takes the argmin by shuffles, so no barrier
    const int tq = min(lane, a.T - 1);
    float vb[kWaveFoldBlk], tx[3] = {0.f, 0.f, 0.f}, tw[3] = {1.f, 1.f, 1.f};
    const int64_t nt = a.n - a.m1;
#pragma unroll
    for (int b = 0; b < kWaveFoldBlk; ++b)
      vb[b] = b < a.nsg ? a.vblk[pq][(int64_t)tq * a.nblk + b] : 0.f;
    {
      const float* row = a.dist[pq] + (int64_t)tq * a.n;
#pragma unroll
      for (int o = 0; o < 3; ++o)
        if (o < nt) {
          tx[o] = row[a.m1 + o];
          tw[o] = wv(a.w, a.m1 + o);
        }
    }
    float y = 0.f;
#pragma unroll
    for (int b = 0; b < kWaveFoldBlk; ++b)
      if (b < a.nsg) y = y + vb[b];
    if (nt > 0) {
      float sx = tx[0] * tw[0];
#pragma unroll
      for (int o = 1; o < 3; ++o)
        if (o < nt) sx = __builtin_fmaf(tx[o], tw[o], sx);
      y = y + sx;
    }
    int b = 0;  // np.argmin: first minimum, a NaN wins at once
    float pb = __shfl(y, 0);
    for (int q = 1; q < a.T; ++q) {
      const float pt = __shfl(y, q);
      if (pb == pb && (pt < pb || pt != pt)) {
        b = q;
        pb = pt;
      }
    }
    bw = b;
    pot = pb;
    wrow = a.dist[pq] + (int64_t)bw * n;
    wfs = a.fsum[pq] + (int64_t)bw * a.nblk;
  } else {
    bw = fold_round(a, pq, s_pot);
    pot = s_pot[bw];
    wrow = a.dist[pq] + (int64_t)bw * n;
    wfs = a.fsum[pq] + (int64_t)bw * a.nblk;
  }
  const int64_t src_prev = __shfl(csl, bw);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0), 21);
  const double r = u * (double)pot;
  // ---- the block where the cumulative potential reaches r
  int jb = INT_MAX;
  double Pf_b = 0.0, tot_b = 0.0;
  if (a.nblk <= 64) {
    // r05: one block per lane and every wave the same scan — wave 0's operations in the workgroup
    // form below, where wave 0's lanes hold every block and the other waves' totals are zeros — so
    // every wave knows the block without a barrier
    const double wj = lane < a.nblk ? wfs[lane] : 0.0;
    double inc = wj;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(inc, o);
      if (lane >= o) inc = inc + y;
    }
    double ex = __shfl_up(inc, 1);
    if (lane == 0) ex = 0.0;
    const double P = 0.0 + ex;
    const double Pn = P + wj;
    const unsigned long long hit = __ballot(lane < a.nblk && Pn >= r);
    if (hit) {
      jb = __ffsll((long long)hit) - 1;
      Pf_b = __shfl(P, jb);
    }
    tot_b = 0.0 + __shfl(inc, 63);  // + the other waves' zero totals: unchanged
  } else {
    const int64_t ch = (a.nblk + kThr - 1) / kThr;
    const int64_t lo = min<int64_t>(a.nblk, tid * ch), hi = min<int64_t>(a.nblk, lo + ch);
    double run = 0.0;
    for (int64_t j = lo; j < hi; ++j) run = run + wfs[j];
    double inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(inc, o);
      if (lane >= o) inc = inc + y;
    }
    double ex = __shfl_up(inc, 1);
    if (lane == 0) ex = 0.0;
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    double B = 0.0;
    for (int q = 0; q < wave; ++q) B = B + s_wave[q];
    double P = B + ex;
    int found = INT_MAX;
    double Pf = 0.0;
    for (int64_t j = lo; j < hi; ++j) {
      const double Pn = P + wfs[j];
      if (Pn >= r) {
        found = (int)j;
        Pf = P;
        break;
      }
      P = Pn;
    }
    if (found != INT_MAX) atomicMin(&s_jmin, found);
    __syncthreads();
    if (found != INT_MAX && found == s_jmin) s_P = Pf;
    if (tid == 0) {  // the whole cumulative potential (the no-crossing case's boundary)
      double tot = 0.0;
      for (int q = 0; q < kWaves; ++q) tot = tot + s_wave[q];
      s_tot = tot;
    }
    __syncthreads();
    jb = s_jmin;
    Pf_b = s_P;
    tot_b = s_tot;
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0), 22);
  int64_t ct = n - 1;
  const double tol = cum_tol(a.exact, n, r);
  // the deciding prefixes: block jb's entries (pv) and the boundary before it (Pb), or the whole
  // total when no block crosses
  double pv[kPer];
  const int64_t e0 = (int64_t)jb * kBlk + kPer * tid;
  const double Pb = jb != INT_MAX ? Pf_b : tot_b;
  bool amb;  // a deciding prefix within tol of r (uniform across the workgroup)
  if (jb != INT_MAX) {  // count inside block jb (uniform branch)
    double v[kPer], pre[kPer];
    if (c >= 2 && a.pfx[pq]) {  // r05: the previous round stored the winner's block prefixes
      const double* pf = a.pfx[pq] + (int64_t)bw * n;
#pragma unroll
      for (int q = 0; q < kPer; ++q) pre[q] = pf[min<int64_t>(e0 + q, n - 1)];
    } else {
#pragma unroll
      for (int q = 0; q < kPer; ++q) v[q] = (double)wrow[min<int64_t>(e0 + q, n - 1)];  // reads first
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int64_t e = e0 + q;
        v[q] = e < n ? (double)(wv(a.w, e) * (float)v[q]) : 0.0;
      }
      block_prefix(v, pre, s_wave);
    }
    int cw = 0;
    bool aw = false;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      pv[q] = Pb + pre[q];
      cw += __popcll(__ballot(e0 + q < n && pv[q] < r));
      aw = aw || __ballot(e0 + q < n && fabs(pv[q] - r) <= tol) != 0ull;
    }
    if (lane == 0) {
      s_cnt[wave] = cw;
      s_amb[wave] = aw;
    }
    __syncthreads();
    int64_t cnt = 0;
    amb = fabs(Pb - r) <= tol;  // the boundary before block jb (entries of earlier blocks)
    for (int q = 0; q < kWaves; ++q) {
      cnt += s_cnt[q];
      amb = amb || s_amb[q];
    }
    ct = min<int64_t>(n - 1, (int64_t)jb * kBlk + cnt);
  } else {
    amb = fabs(Pb - r) <= tol;
  }
  if (amb && a.exact == 1) {
    // cum_tol bounds numpy's rounding by 2.25 n u r whatever the row holds. A row-specific bound
    // decides most of these draws without the replay: with g = ulp(total) (every partial sum is at
    // most the total), an entry that is a multiple of g adds to numpy's running sum exactly unless the
    // sum enters a new binade; each other ("fine") entry costs at most g / 2 and the binade entries
    // together at most g (ulps double per binade), so |numpy - exact| <= A = (F / 2 + 1) g for F fine
    // entries in the row. The blocked prefixes are trees of height <= h: |blocked - exact| <=
    // gamma_h * exact (Higham eq. 4.4). A decision can differ from numpy's only if |p - r| <= A +
    // 2 gamma_h max(p, r); only then does the replay run.
    __syncthreads();  // s_cnt / s_amb reused below
    // any g >= ulp(numpy's largest partial sum) will do: the total over-estimated by numpy's gamma_n
    const double sup = tot_b * (1.0 + (double)(n + 256) * 0x1p-52);
    const int E = sup > 0.0 ? ilogb(sup) : -1074;
    const double ginv = ldexp(1.0, 52 - E);
    int fine = 0;
    for (int64_t e = tid; e < n; e += kThr) {
      const double x = (double)(wv(a.w, e) * wrow[e]);
      const double q = x * ginv;
      fine += !(q == trunc(q)) ? 1 : 0;  // NaN / inf count as fine (the replay decides)
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) fine += __shfl_xor(fine, o);
    if (lane == 0) s_cnt[wave] = fine;
    __syncthreads();
    int64_t F = 0;
    for (int q = 0; q < kWaves; ++q) F += s_cnt[q];
    const double g = ldexp(1.0, E - 52);
    const double A = ((double)F * 0.5 + 1.0) * g;
    const int64_t ch = (a.nblk + kThr - 1) / kThr;
    const double gh = (double)(96 + ch) * 0x1p-53 * 1.01;
    const bool finite = tot_b == tot_b && tot_b < __builtin_inf();
    bool aw = !finite || fabs(Pb - r) <= A + 2.0 * gh * fmax(Pb, r);
    if (jb != INT_MAX) {
#pragma unroll
      for (int q = 0; q < kPer; ++q)
        aw = aw || (e0 + q < n && fabs(pv[q] - r) <= A + 2.0 * gh * fmax(pv[q], r));
    }
    aw = __ballot(aw) != 0ull;
    __syncthreads();
    if (lane == 0) s_amb[wave] = aw;
    __syncthreads();
    amb = false;
    for (int q = 0; q < kWaves; ++q) amb = amb || s_amb[q];
  }
  if (amb) {  // numpy's sequential cumsum decides this draw
    if (wave == 0) {
      const int64_t e = np_cumsum_search_wave(wrow, a.w, n, r);
      if (lane == 0) s_ct = min<int64_t>(n - 1, e);
    }
    __syncthreads();
    ct = s_ct;
  }
  if (blk == 0 && tid == 0) a.cand[cq][t] = ct;
  if (PICK && blk == 0 && t == 0 && tid == 0) a.winq[cq] = bw;
  // round c-1's centre: its index (the rows are gathered after the rounds, k_kpp_gather_centres)
  if (c >= 2 && blk == 0 && t == 0 && tid == 0) a.indices[c - 1] = src_prev;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0), 23);
  if constexpr (PICK) return;  // the split path: k_kpp_dists computes every trial's distances
  // ---- distances of this block's points to the candidate, np.minimum with the winner's row
  float* s_d = reinterpret_cast<float*>(s_c + a.dim);
  const int64_t j0 = (int64_t)blk * kBlk;
  float* drow = a.dist[cq] + (int64_t)t * n;
  if (SEQ && a.D) {  // the distance table holds the plain chain's value for every (candidate, point)
    const float* Drow = a.D + ct * n;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int o = tid + kThr * q;
      const int64_t i = j0 + o;
      float f = 0.f;
      if (i < n) {
        f = np_minimum(wrow[i], Drow[i]);
        drow[i] = f;
      }
      s_d[o] = f;
    }
  } else {
    const double cn = a.xsq[ct];
    for (int j = tid; j < a.dim; j += kThr) s_c[j] = (double)a.X[ct * a.dim + j];
    __syncthreads();
    block_dists<SEQ>(a, t, j0, cn, s_c, wrow, drow, s_d);
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0), 24);
  // ---- the block's terms for round c+1: cumulative total, sgemv_t lane chains
  const int64_t NB = min<int64_t>(kBlk, a.m1 - j0);
  // r05: the block prefix beside the lane chain instead of before it. Every wave posts its scan total
  // and arrives on an LDS counter; wave 0 (no waves before it: block_prefix's B = 0) stores its
  // prefixes and runs the chain, the others wait for the count and finish theirs. A wait that gave
  // up is redone with block_prefix after a closing barrier.
  const bool ovl = !PICK && NB > 0 && a.T > 1;
  {
    double v[kPer], pre[kPer];
    float xs[kPer];  // every read before the weights' branches (r04)
#pragma unroll
    for (int q = 0; q < kPer; ++q) xs[q] = s_d[kPer * tid + q];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t e = j0 + kPer * tid + q;
      v[q] = e < n ? (double)(wv(a.w, e) * xs[q]) : 0.0;
    }
    const int64_t last = min<int64_t>(n, j0 + kBlk) - 1 - j0;
    auto emit = [&]() {
      if (tid == (int)(last / kPer)) a.fsum[cq][(int64_t)t * a.nblk + blk] = pre[last % kPer];
      if (a.pfx[cq]) {  // r05: the next round's count inside the winner's block reads these back
        double* pf = a.pfx[cq] + (int64_t)t * n + j0 + kPer * tid;
#pragma unroll
        for (int q = 0; q < kPer; ++q)
          if (j0 + kPer * tid + q < n) pf[q] = pre[q];
      }
    };
    if (ovl) {
      double r[kPer];
      double run = 0.0;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        run = run + v[q];
        r[q] = run;
      }
      double inc = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(inc, o);
        if (lane >= o) inc = inc + y;
      }
      double ex = __shfl_up(inc, 1);
      if (lane == 0) ex = 0.0;
      if (lane == 63) s_wave[wave] = inc;
      waves_arrive(&s_pfxsync);
      bool ok = true;
      double B = 0.0;
      if (wave > 0) {
        ok = waves_wait(&s_pfxsync, kWaves);
        for (int q = 0; q < wave; ++q) B = B + s_wave[q];
      }
      const double base = B + ex;
#pragma unroll
      for (int q = 0; q < kPer; ++q) pre[q] = base + r[q];
      if (ok) emit();
      else if (lane == 0) s_pfxfail = 1;
    } else {
      block_prefix(v, pre, s_wave);
      emit();
    }
    if (ovl && wave == 0) {  // the chain, beside the other waves' prefixes
      const float y = sgemv_block_wave(s_d, a.w ? a.w + j0 : nullptr, NB, t, a.T);
      if (lane == 0) a.vblk[cq][(int64_t)t * a.nblk + blk] = y;
    }
    if (ovl) {
      __syncthreads();
      if (s_pfxfail) {  // a bounded wait gave up: the prefixes again, with barriers
        block_prefix(v, pre, s_wave);
        emit();
      }
    }
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0), 25);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blk == 0 && t == 0 && c < 128), 128 + c);
}

// ---- round c's distances for ALL trials of one point block (the split-round path, SEQ, T <= 8) ------
// One workgroup per 4096-point block reads its points' features once (the dim x n transpose,
// coalesced) and runs the T k-ordered fp64 chains side by side, instead of T workgroups re-reading
// the same block (T x the X traffic); then, per trial, np.minimum with the winner's row, the
// cumulative-potential block total (block_prefix) and the sgemv_t block term (wave t).
constexpr int kSplitMaxT = 8;
constexpr int kSplitMinBlocks = 128;
// T is a template argument: with a runtime trial count every (feature, trial) pair of the chain
// loop became its own branch with an LDS read waited on before its four fmas (the r03 products
// profile: ~40 G fp64 fma/s per CU, a quarter of the issue rate).
template <int T>
__global__ __launch_bounds__(kThr) void k_kpp_dists(KppArgs a, int c) {
  extern __shared__ double s_cs[];  // T * dim doubles (candidate rows), then T * kBlk floats
  __shared__ double s_cn[kSplitMaxT];
  const int blk = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int dim = a.dim;
  const int pq = (c - 1) & 1, cq = c & 1;
  const int64_t n = a.n, j0 = (int64_t)blk * kBlk;
  const float* wrow = c == 1 ? a.closest0 : a.dist[pq] + (int64_t)a.winq[cq] * n;
  // stamps (diagnostic build, tools/stamps.py kpp-dists): round 5, block 0 and the last block
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && c == 5 && (blk == 0 || blk == a.nblk - 1)), blk == 0 ? 30 : 40);
  for (int e = tid; e < T * dim; e += kThr) {
    const int t = e / dim, j = e - t * dim;
    s_cs[e] = (double)a.X[a.cand[cq][t] * dim + j];
  }
  if (tid < T) s_cn[tid] = a.xsq[a.cand[cq][tid]];
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && c == 5 && (blk == 0 || blk == a.nblk - 1)), blk == 0 ? 31 : 41);
  float* s_d = reinterpret_cast<float*>(s_cs + T * dim);
  // feature f of point j0 + off[q] is xt[f * n + off[q]]: a wave-uniform row base plus a 32-bit
  // lane offset, so each load takes one scalar base and no 64-bit vector address
  const float* __restrict__ xt = a.XT + j0;
  uint32_t off[kPer];
  double dot[kSplitMaxT][kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = j0 + tid + kThr * q;
    off[q] = i < n ? (uint32_t)(tid + kThr * q) : 0u;
#pragma unroll
    for (int t = 0; t < kSplitMaxT; ++t) dot[t][q] = 0.0;
  }
  // The chains are bound by the latency of their XT loads (one wave per SIMD slot, no room in LDS
  // to stage the block): D trips of G features each are in flight ahead of the fmas that use them.
  constexpr int G = 1;  // features per trip: 4 spilled at T = 7 under the 128-VGPR cap of 1024 threads
  constexpr int D = 3;
  const int ntrip = dim / G;
  float buf[D][G][kPer];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < ntrip) {
#pragma unroll
      for (int v = 0; v < G; ++v)
#pragma unroll
        for (int q = 0; q < kPer; ++q) buf[d][v][q] = (xt + (int64_t)(d * G + v) * n)[off[q]];
    }
  for (int tr0 = 0; tr0 < ntrip; tr0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int tr = tr0 + d;
      if (tr >= ntrip) break;
      float u[G][kPer];
#pragma unroll
      for (int v = 0; v < G; ++v)
#pragma unroll
        for (int q = 0; q < kPer; ++q) u[v][q] = buf[d][v][q];
      if (tr + D < ntrip) {
#pragma unroll
        for (int v = 0; v < G; ++v)
#pragma unroll
          for (int q = 0; q < kPer; ++q)
            buf[d][v][q] = (xt + (int64_t)((tr + D) * G + v) * n)[off[q]];
      }
      const int jj = tr * G;
#pragma unroll
      for (int v = 0; v < G; ++v)
#pragma unroll
        for (int t = 0; t < kSplitMaxT; ++t)
          if (t < T) {
            const double cv = s_cs[t * dim + jj + v];
#pragma unroll
            for (int q = 0; q < kPer; ++q) dot[t][q] = __builtin_fma(cv, (double)u[v][q], dot[t][q]);
          }
    }
  }
  int j = ntrip * G;
  for (; j < dim; ++j) {
    float u[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) u[q] = (xt + (int64_t)j * n)[off[q]];
#pragma unroll
    for (int t = 0; t < kSplitMaxT; ++t)
      if (t < T) {
        const double cv = s_cs[t * dim + j];
#pragma unroll
        for (int q = 0; q < kPer; ++q) dot[t][q] = __builtin_fma(cv, (double)u[q], dot[t][q]);
      }
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && c == 5 && (blk == 0 || blk == a.nblk - 1)), blk == 0 ? 32 : 42);
  float wv_[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = j0 + tid + kThr * q;
    wv_[q] = i < n ? wrow[i] : 0.f;
  }
#pragma unroll
  for (int t = 0; t < kSplitMaxT; ++t) {
    if (t >= T) break;
    float* drow = a.dist[cq] + (int64_t)t * n;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int o = tid + kThr * q;
      const int64_t i = j0 + o;
      float f = 0.f;
      if (i < n) {
        f = (float)(((-2.0 * dot[t][q]) + s_cn[t]) + a.xsq[i]);
        f = f < 0.f ? 0.f : f;
        f = np_minimum(wv_[q], f);
        drow[i] = f;
      }
      s_d[t * kBlk + o] = f;
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && c == 5 && (blk == 0 || blk == a.nblk - 1)), blk == 0 ? 33 : 43);
  // the block's cumulative-potential total per trial: block_prefix's operations for every trial with
  // one barrier (r05; the per-trial calls paid two barriers each), the total kept by the thread that
  // owns the block's last entry
  {
    __shared__ double s_wt[kSplitMaxT][kWaves];
    const int64_t last = min<int64_t>(n, j0 + kBlk) - 1 - j0;
    const bool owner = tid == (int)(last / kPer);
    double rl[kSplitMaxT], exl[kSplitMaxT];
#pragma unroll
    for (int t = 0; t < kSplitMaxT; ++t) {
      rl[t] = 0.0;
      exl[t] = 0.0;
      if (t < T) {
        float xs[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) xs[q] = s_d[t * kBlk + kPer * tid + q];
        double run = 0.0, r[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
          const int64_t e = j0 + kPer * tid + q;
          run = run + (e < n ? (double)(wv(a.w, e) * xs[q]) : 0.0);
          r[q] = run;
        }
        double inc = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const double y = __shfl_up(inc, o);
          if (lane >= o) inc = inc + y;
        }
        double ex = __shfl_up(inc, 1);
        if (lane == 0) ex = 0.0;
        if (lane == 63) s_wt[t][wave] = inc;
        exl[t] = ex;
#pragma unroll
        for (int q = 0; q < kPer; ++q)
          if (q == (int)(last % kPer)) rl[t] = r[q];
      }
    }
    __syncthreads();
    if (owner) {
#pragma unroll
      for (int t = 0; t < kSplitMaxT; ++t) {
        if (t < T) {
          double B = 0.0;
          for (int q = 0; q < wave; ++q) B = B + s_wt[t][q];
          a.fsum[cq][(int64_t)t * a.nblk + blk] = (B + exl[t]) + rl[t];
        }
      }
    }
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && c == 5 && (blk == 0 || blk == a.nblk - 1)), blk == 0 ? 34 : 44);
  const int64_t NB = min<int64_t>(kBlk, a.m1 - j0);
  if (NB > 0 && wave < T) {  // wave t: trial t's sgemv_t block term
    const float v = sgemv_block_wave(s_d + wave * kBlk, a.w ? a.w + j0 : nullptr, NB, wave, T);
    if (lane == 0) a.vblk[cq][(int64_t)wave * a.nblk + blk] = v;
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (lane == 0 && wave == 0 && c == 5 && (blk == 0 || blk == a.nblk - 1)),
                 blk == 0 ? 35 : 45);
#ifdef GDD_STAMPS
  if (lane == 0 && c == 5) atomicMax(&g_stamps_kpp[46], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// after the last round: its potentials, winner and centre
__global__ __launch_bounds__(kThr) void k_kpp_final(KppArgs a, int c) {
  __shared__ float s_pot[kMaxTrials];
  const int q = c & 1;
  const int b = fold_round(a, q, s_pot);
  const int64_t src = a.cand[q][b];
  if (threadIdx.x == 0) a.indices[c] = src;
  for (int j = threadIdx.x; j < a.dim; j += kThr) a.centers[(int64_t)c * a.dim + j] = a.X[src * a.dim + j];
}

// ---- single-block rounds (n <= 4096, T >= 2: MiniBatchKMeans' init subset, small KMeans) ---------
// Two launches per round, each moving little data through any one CU (a CU pulls only ~35-70 GB/s
// from L2/Infinity Cache, so staging T rows in one workgroup costs microseconds):
//   k_kpp1_dist (round c)  points x trial-groups over many workgroups: reads round c-1's T
//       potentials and the T x T table of "candidates if trial t wins", takes np.argmin, and computes
//       its 64 points' distances to this round's T candidates, np.minimum with the winner's row.
//   k_kpp1_pick (round c)  one workgroup per trial: stages the trial's row, runs its sgemv_t lane
//       chains (the exact potential), its fp64 cumulative potential, and counts the candidates every
//       trial would draw in round c+1 if this trial wins (the uniforms are known in advance).
// Round 0 (the first centre) is a pick over closest0 with the sdot potential. After round k-1,
// k_kpp1_final takes the last argmin.
constexpr int kTg = 2;       // trials per thread in the distance phase
constexpr int kPts = 64;     // points per distance workgroup (one per lane; waves = trial groups)

struct Kpp1Args {
  int64_t n, m1;
  int dim, T, k, pad;
  const float* X;
  const float* XT;     // X^T (dim x n) for plain-chain plans
  const float* w;
  const double* xsq;
  const float* closest0;
  const KppState* st;
  const double* uniforms;
  float* dist[2];      // [T][n]
  float* potv[2];      // [T]
  int64_t* candw[2];   // [T][T]
  int64_t* candself[2];  // [T]
  int64_t* candr[2];   // fused rounds: the round's T candidates (written by the previous fold)
  double* candn[2];    // fused rounds: their squared norms
  int* win;            // fused rounds: [2] the winning trial, by round parity
  unsigned* counter;   // fused rounds: [k] arrivals per round (zeroed per fit)
  float* centers;
  int64_t* indices;
  SklPlan plan;
  // two rounds per launch (k_kpp1_dm2): round c+1's trial t given round c's winner w, at w * T + t
  float* dist2[2];       // [T*T][n]
  float* potv2[2];       // [T*T]
  int64_t* candw2[2];    // [T*T][T]
  int64_t* candself2[2];  // [T*T]
  int exact;             // cum_tol's mode
};

__device__ __forceinline__ int kpp1_argmin(const float* __restrict__ pot, int T) {
  int b = 0;
  for (int q = 1; q < T; ++q) {
    const float pb = pot[b], pt = pot[q];
    if (pb == pb && (pt < pb || pt != pt)) b = q;
  }
  return b;
}

template <bool SEQ>
__global__ __launch_bounds__(256) void k_kpp1_dist(Kpp1Args a, int c) {
  extern __shared__ double s_cr[];  // T * dim candidate rows (fp64)
  __shared__ int64_t s_cw[kMaxTrials * kMaxTrials];
  __shared__ double s_cn[kMaxTrials];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pq = (c - 1) & 1, cq = c & 1, T = a.T, dim = a.dim;
  const int Tp = c == 1 ? 1 : T;  // trials of round c-1 (round 0: the first centre)
  const int n = (int)a.n;
  const int i = blockIdx.x * kPts + lane;
  const int ic = min(i, n - 1);  // clamped: every load below is unconditional (no branches
                                 // around loads, so they all stay in flight together)
  const int t0 = (blockIdx.y * 4 + wave) * kTg;
  const bool live = i < n && t0 < T;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0 && c == a.k - 2), 60);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0 && c == a.k - 1), 65);
  // round trip 1: the point's row, round c-1's potentials and its whole candidate table
  constexpr int kX = SEQ ? 48 : 1;
  float x[kX];
  if (SEQ && dim <= kX) {
#pragma unroll
    for (int v = 0; v < kX; ++v) x[v] = a.XT[(int64_t)min(v, dim - 1) * n + ic];
  }
  const double xs = a.xsq[ic];
  float pv[kMaxTrials];
#pragma unroll
  for (int q = 0; q < kMaxTrials; ++q) pv[q] = a.potv[pq][min(q, Tp - 1)];
  if (tid < Tp * T) s_cw[tid] = a.candw[pq][tid];
  int bw = 0;  // np.argmin: first minimum, a NaN wins at once
  float best = pv[0];
#pragma unroll
  for (int q = 1; q < kMaxTrials; ++q) {
    const float pt = pv[q];
    if (q < Tp && best == best && (pt < best || pt != pt)) {
      bw = q;
      best = pt;
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0 && c == a.k - 2), 61);
  // round trip 2: the winner's row, this round's candidate rows and norms
  const float wi = c == 1 ? a.closest0[ic] : a.dist[pq][(int64_t)bw * n + ic];
  const int64_t* cand = s_cw + bw * T;
  if (tid < T) s_cn[tid] = a.xsq[cand[tid]];
  // candidate rows in fp64; short rows (plain chains) padded with zeros to kX, so the chain below
  // runs a fixed trip count without branches (dot + 0 * x == dot)
  const int cs = (SEQ && dim <= kX) ? kX : dim;
  for (int e = tid; e < T * cs; e += 256) {
    const int t = e / cs, j = e - t * cs;
    s_cr[e] = j < dim ? (double)a.X[cand[t] * dim + min(j, dim - 1)] : 0.0;
  }
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    if (tid < T) a.candself[cq][tid] = cand[tid];
    if (c >= 2) {  // round c-1's centre
      const int64_t src = a.candself[pq][bw];
      if (tid == 0) a.indices[c - 1] = src;
      for (int j = tid; j < dim; j += 256) a.centers[(int64_t)(c - 1) * dim + j] = a.X[src * dim + j];
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0 && c == a.k - 2), 62);
  if (!live) return;
  double dot[kTg];
  const int t1 = min(t0 + 1, T - 1);
  if constexpr (SEQ) {
    dot[0] = 0.0;
    dot[1] = 0.0;
    const double* c0 = s_cr + (size_t)t0 * cs;
    const double* c1 = s_cr + (size_t)t1 * cs;
    if (dim <= kX) {
#pragma unroll
      for (int v = 0; v < kX; ++v) {
        const double xv = (double)x[v];
        dot[0] = __builtin_fma(c0[v], xv, dot[0]);
        dot[1] = __builtin_fma(c1[v], xv, dot[1]);
      }
    } else {
      for (int j = 0; j < dim; j += 16) {
        float y[16];
#pragma unroll
        for (int v = 0; v < 16; ++v) y[v] = a.XT[(int64_t)min(j + v, dim - 1) * n + i];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          if (j + v < dim) {
            dot[0] = __builtin_fma(c0[j + v], (double)y[v], dot[0]);
            dot[1] = __builtin_fma(c1[j + v], (double)y[v], dot[1]);
          }
        }
      }
    }
  } else {
    dot[0] = skl_point_dot(a.plan, s_cr + (size_t)t0 * dim, a.X + (int64_t)i * dim, i, t0);
    dot[1] = skl_point_dot(a.plan, s_cr + (size_t)t1 * dim, a.X + (int64_t)i * dim, i, t1);
  }
#pragma unroll
  for (int u = 0; u < kTg; ++u) {
    const int t = t0 + u;
    if (t < T) {
      float f = (float)(((-2.0 * dot[u]) + s_cn[t]) + xs);
      f = f < 0.f ? 0.f : f;
      a.dist[cq][(int64_t)t * n + i] = np_minimum(wi, f);
    }
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0 && c == a.k - 2), 63);
}

// one sgemv_t lane chain over L entries stored contiguously in LDS (chain-major layout):
// acc = acc + x in order. Two 32-entry register groups alternate, each group's 16-byte reads issued a
// whole group of dependent adds ahead of their use (scheduling barriers keep them there; the first
// group goes through an empty asm so InstCombine cannot turn the loop's phi of loads into a load of
// a phi of addresses, which would put every read right in front of its adds). Look-ahead reads run
// at most 63 entries past L, inside the lane's kChainLd-float row (L <= 1024).
__device__ __forceinline__ void chain_load32(const float* __restrict__ p, float4 (&v)[8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + 4 * u);
}

__device__ __forceinline__ void chain_add32(const float4 (&v)[8], float& acc) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    acc = acc + v[u].x;
    acc = acc + v[u].y;
    acc = acc + v[u].z;
    acc = acc + v[u].w;
  }
}

__device__ __forceinline__ float chain_add(const float* __restrict__ p, int L, float acc) {
  int m = 0;
  float4 A[8];
  chain_load32(p, A);  // past L: row padding, never added
#pragma unroll
  for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(A[u].x), "+v"(A[u].y), "+v"(A[u].z), "+v"(A[u].w));
  for (; m + 64 <= L; m += 64) {
    float4 B[8];
    chain_load32(p + m + 32, B);
    __builtin_amdgcn_sched_barrier(0);
    chain_add32(A, acc);
    __builtin_amdgcn_sched_barrier(0);
    chain_load32(p + m + 64, A);
    __builtin_amdgcn_sched_barrier(0);
    chain_add32(B, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  // A holds entries m .. m+31 (L - m < 64): the rest without single-entry LDS round trips
  float4 B[8];
  chain_load32(p + m + 32, B);
  // the rest in groups of four: whole groups plain, the group that ends the chain with its extra
  // entries masked to -0.0 (L differs by at most one between lanes, so only that group branches)
  auto grp = [&](const float4& g, int e) {
    if (e + 3 < L) {
      acc = acc + g.x;
      acc = acc + g.y;
      acc = acc + g.z;
      acc = acc + g.w;
    } else if (e < L) {
      acc = acc + g.x;
      acc = acc + add_operand(g.y, e + 1 < L);
      acc = acc + add_operand(g.z, e + 2 < L);
    }
  };
#pragma unroll
  for (int u = 0; u < 8; ++u) grp(A[u], m + 4 * u);
#pragma unroll
  for (int u = 0; u < 8; ++u) grp(B[u], m + 32 + 4 * u);
  return acc;
}

constexpr int kChainLd = kBlk / 4 + 68;  // chain-major LDS stride (floats): 4 (mod 64), >= 1024 + 4

// round c's trial t (c == 0: the first centre over closest0, potential = the sdot): potential,
// cumulative potential, and round c+1's candidates if this trial wins
__global__ __launch_bounds__(kThr) void k_kpp1_pick(Kpp1Args a, int c) {
  __shared__ float s_d[kBlk];
  __shared__ float s_ch[8 * kChainLd];  // unit weights: chain l's entries contiguous
  __shared__ double s_wave[kWaves];
  __shared__ int s_cnt[kMaxTrials][kWaves], s_amb[kMaxTrials][kWaves];
  __shared__ float s_pot;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = c & 1, T = a.T;
  const int n = (int)a.n, m1 = (int)a.m1;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 70);
  // this round's uniforms for the next round's draws: requested up front
  double u[kMaxTrials];
  const int un = c + 1 < a.k ? T : 1;
#pragma unroll
  for (int q = 0; q < kMaxTrials; ++q) u[q] = a.uniforms[(int64_t)c * T + min(q, un - 1)];
  const float* row = c == 0 ? a.closest0 : a.dist[cq] + (int64_t)t * n;
  const bool k4x2 = c > 0 && (T & 2) && t >= (T & ~3) && t < (T & ~3) + 2;
  const int nl = k4x2 ? 4 : 8;                 // chain lanes
  const int h4 = k4x2 ? 0 : (m1 & 4);          // 8-lane kernel: first m1 & 4 entries go to lanes 0..3
  const bool perm = c > 0 && a.w == nullptr;
  float r[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) r[q] = row[min(tid + kThr * q, n - 1)];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = tid + kThr * q;
    if (e < n) {
      s_d[e] = r[q];
      if (perm && e >= h4 && e < m1) {
        const int o = e - h4;
        s_ch[(o % nl) * kChainLd + o / nl] = r[q];
      }
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 71);
  double v[kPer], pre[kPer];
  float xs[kPer];  // every read before the weights' branches (r04)
#pragma unroll
  for (int q = 0; q < kPer; ++q) xs[q] = s_d[kPer * tid + q];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = kPer * tid + q;
    v[q] = e < n ? (double)(wv(a.w, e) * xs[q]) : 0.0;
  }
  block_prefix(v, pre, s_wave);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 72);
  if (wave == 0) {
    float y = 0.f;
    if (c == 0) {
      y = a.st->pot;
    } else if (m1 > 0) {  // sgemv_t: the block's lane chains, then the n % 4 trailing entries
      if (perm) {
        float acc = 0.f;
        if (lane < nl) {
          if (lane < h4) acc = acc + s_d[lane];
          const int o0 = lane;  // chain lane's entries o = h4 + lane + nl * m
          const int L = (m1 - h4 - o0 + nl - 1) / nl;
          acc = chain_add(s_ch + lane * kChainLd, max(L, 0), acc);
        }
        if (k4x2) {
          const float a1 = __shfl(acc, 1), a2 = __shfl(acc, 2), a3 = __shfl(acc, 3);
          y = (acc + a1) + (a2 + a3);
        } else {
          const float ql = acc + __shfl(acc, (lane + 4) & 63);
          const float q1 = __shfl(ql, 1), q2 = __shfl(ql, 2), q3 = __shfl(ql, 3);
          y = (ql + q1) + (q2 + q3);
        }
      } else {
        y = sgemv_block_wave(s_d, a.w, m1, t, T);
      }
    }
    if (c > 0 && m1 < n && lane == 0) {
      float sx = s_d[m1] * wv(a.w, m1);
      for (int o = m1 + 1; o < n; ++o) sx = __builtin_fmaf(s_d[o], wv(a.w, o), sx);
      y = y + sx;
    }
    if (lane == 0) {
      s_pot = y;
      a.potv[cq][t] = y;
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 73);
  if (c + 1 >= a.k) return;
  const double pot = (double)s_pot;
#pragma unroll
  for (int t2 = 0; t2 < kMaxTrials; ++t2) {
    if (t2 < T) {
      const double rr = u[t2] * pot;
      const double tol = cum_tol(a.exact, n, rr);
      int cw = 0;
      bool aw = false;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const bool live = kPer * tid + q < n;
        cw += __popcll(__ballot(live && pre[q] < rr));
        aw = aw || __ballot(live && fabs(pre[q] - rr) <= tol) != 0ull;
      }
      if (lane == 0) {
        s_cnt[t2][wave] = cw;
        s_amb[t2][wave] = aw;
      }
    }
  }
  __syncthreads();
  if (tid < T) {
    int64_t cnt = 0;
    bool amb = false;
    for (int q = 0; q < kWaves; ++q) {
      cnt += s_cnt[tid][q];
      amb = amb || s_amb[tid][q];
    }
    if (amb) cnt = np_cumsum_search(s_d, a.w, n, a.uniforms[(int64_t)c * T + tid] * pot);
    a.candw[cq][(int64_t)t * T + tid] = min<int64_t>(n - 1, cnt);
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 74);
}

constexpr int kFPW = 22;     // prefix entries per thread of waves 1..3 in the fold (192 x 22 >= 4096)

// waves 1-3 only (the fold's prefix waves): every calling wave's earlier LDS writes are visible to
// the others once the count reaches target; false if the spin gave up (bounded)
// k_kpp1_big's speculative draws: every wave arrives (its earlier LDS writes then visible to a
// waiting wave); waves_wait spins until target waves arrived, false if the spin gave up (bounded)
__device__ __forceinline__ void waves_arrive(int* ctr) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool waves_wait(int* ctr, int target) {
  for (int it = 0; it < kSpinLimit; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

__device__ __forceinline__ bool prefix_waves_sync(int* ctr, int target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int it = 0; it < kSpinLimit; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

// ---- the fold's parts (kpp1_fold_trial, kpp1_fold_pair) ----------------------------------------------
// wave 0: trial t's exact sgemv_t potential over the row in s_d (chain-major copy in s_ch for unit
// weights): the lane chains, then the n % 4 trailing entries; lane 0 returns it
__device__ __forceinline__ float fold_potential(const Kpp1Args& a, const float* __restrict__ s_d,
                                                const float* __restrict__ s_ch, int t, bool k4x2, int h4) {
  const int lane = threadIdx.x & 63;
  const int T = a.T, n = (int)a.n, m1 = (int)a.m1;
  float y = 0.f;
  if (m1 > 0) {
    if (a.w == nullptr) {
      const int nl = k4x2 ? 4 : 8;
      float acc = 0.f;
      if (lane < nl) {
        if (lane < h4) acc = acc + s_d[lane];
        const int L = (m1 - h4 - lane + nl - 1) / nl;
        acc = chain_add(s_ch + lane * kChainLd, max(L, 0), acc);
      }
      if (k4x2) {
        const float a1 = __shfl(acc, 1), a2 = __shfl(acc, 2), a3 = __shfl(acc, 3);
        y = (acc + a1) + (a2 + a3);
      } else {
        const float ql = acc + __shfl(acc, (lane + 4) & 63);
        const float q1 = __shfl(ql, 1), q2 = __shfl(ql, 2), q3 = __shfl(ql, 3);
        y = (ql + q1) + (q2 + q3);
      }
    } else {
      y = sgemv_block_wave(s_d, a.w, m1, t, T);
    }
  }
  if (m1 < n && lane == 0) {
    float sx = s_d[m1] * wv(a.w, m1);
    for (int o = m1 + 1; o < n; ++o) sx = __builtin_fmaf(s_d[o], wv(a.w, o), sx);
    y = y + sx;
  }
  return y;
}

// waves 1-3 (prefix thread jp = tid - 64): the thread's run over entries kFPW jp .. + kFPW - 1 of s_d
// (w * x in fp32, then fp64 adds), the wave's exclusive offset added; the wave total into
// s_wave[wave - 1]. Every read issued before the run (a per-entry weight branch had each read waited
// on alone: ~2 us, as long as the chains, r04 stamps); entries past n add +0.0
__device__ __forceinline__ void fold_prefix(const Kpp1Args& a, const float* __restrict__ s_d, int jp,
                                            double (&pre)[kFPW], double* __restrict__ s_wave) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = (int)a.n;
  float xv[kFPW];
#pragma unroll
  for (int q = 0; q < kFPW; ++q) xv[q] = s_d[min(kFPW * jp + q, n - 1)];
  if (a.w) {
#pragma unroll
    for (int q = 0; q < kFPW; ++q) {
      const int e = kFPW * jp + q;
      xv[q] = e < n ? a.w[min(e, n - 1)] * xv[q] : 0.f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < kFPW; ++q) xv[q] = kFPW * jp + q < n ? xv[q] : 0.f;  // 1.0f * x == x
  }
  double run = 0.0;
#pragma unroll
  for (int q = 0; q < kFPW; ++q) {
    run = run + (double)xv[q];
    pre[q] = run;
  }
  double inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(inc, o);
    if (lane >= o) inc = inc + y;
  }
  double ex = __shfl_up(inc, 1);
  if (lane == 0) ex = 0.0;
  if (lane == 63) s_wave[wave - 1] = inc;
#pragma unroll
  for (int q = 0; q < kFPW; ++q) pre[q] = ex + pre[q];
}

// the regular draws for the uniforms in `redo` (lane q of every wave holds u_q in ut) over the complete
// cumulative potential s_cum: searchsorted_left(cum, u * pot) in two ballots. Lane l of every wave
// holds the last value of block l (64 blocks of Bk = ceil(n / 64) entries); wave w takes uniforms w,
// w + 4, ...: the blocks below r counted by one ballot, then one LDS read per lane and a ballot inside
// the next block — two LDS trips instead of log2(n) dependent ones. The rounding check covers the
// block's entries and the entry before it (every deciding neighbour; a count that differs from
// numpy's needs a prefix within tol of r, non-monotone rounding steps included)
__device__ __forceinline__ void fold_search(const Kpp1Args& a, unsigned long long redo, double ut, double pot,
                                            const double* __restrict__ s_cum, const float* __restrict__ s_d,
                                            int64_t* cand_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int T = a.T, n = (int)a.n;
  const int Bk = (n + 63) >> 6;
  const int nb = (n + Bk - 1) / Bk;
  const double cl = s_cum[min((lane + 1) * Bk, n) - 1];
  for (int t2 = wave; t2 < T; t2 += (int)(blockDim.x >> 6)) {
    if (!((redo >> t2) & 1ull)) continue;
    const double rr = __shfl(ut, t2) * pot;
    const double tol = cum_tol(a.exact, n, rr);
    const int c0 = __popcll(__ballot(lane < nb && cl < rr));
    int idx;
    bool amb;
    if (c0 >= nb) {
      idx = n;
      amb = fabs(__shfl(cl, nb - 1) - rr) <= tol;
    } else {
      const int e = c0 * Bk + lane;
      const bool live = lane < Bk && e < n;
      const double v = live ? s_cum[min(e, n - 1)] : 0.0;
      idx = c0 * Bk + __popcll(__ballot(live && v < rr));
      const double prev = __shfl(cl, c0 > 0 ? c0 - 1 : 0);
      amb = __ballot(live && fabs(v - rr) <= tol) != 0ull || (c0 > 0 && fabs(prev - rr) <= tol);
    }
    if (amb) {
      int rep = 0;
      if (lane == 0) rep = (int)np_cumsum_search(s_d, a.w, n, rr);
      idx = __shfl(rep, 0);
    }
    if (lane == 0) cand_out[t2] = min(n - 1, idx);
  }
}

// a speculative draw is numpy's index when the exact threshold rr falls between the same two
// cumulative values (lo: entry idx - 1, hi: entry idx), neither within 4 cum_tol of it
__device__ __forceinline__ bool spec_draw_good(const Kpp1Args& a, int idx, double lo, double hi, double rr) {
  const int n = (int)a.n;
  const double tol = cum_tol(a.exact, n, rr);
  return tol >= 0.0 && (idx == 0 || (lo < rr && fabs(lo - rr) > 4.0 * tol)) &&
         (idx == n || (!(hi < rr) && fabs(hi - rr) > 4.0 * tol));
}

// the fold of round c's trial t by one 256-thread workgroup holding the trial's row in registers
// (r[q] = entry tid + 256 q): the exact sgemv_t potential, the fp64 cumulative potential and the
// candidates every trial would draw in round c+1 if t wins
// pot_out (nullable) receives the potential, cand_out[0..T) the candidates (global memory or LDS)
__device__ __forceinline__ void kpp1_fold_trial(const Kpp1Args& a, int c, int t, const float (&r)[16],
                                                double ut, float* __restrict__ s_d,
                                                float* __restrict__ s_ch, double* __restrict__ s_cum,
                                                double* __restrict__ s_wave, float* __restrict__ s_pot_p,
                                                float* pot_out, int64_t* cand_out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T;
  const int n = (int)a.n;
  float& s_pot = *s_pot_p;
  const int m1 = (int)a.m1;
  const bool k4x2 = (T & 2) && t >= (T & ~3) && t < (T & ~3) + 2;
  const int h4 = k4x2 ? 0 : (m1 & 4);
  const bool perm = a.w == nullptr;
  // speculative searches (r04): while wave 0 runs the lane chains (~2 us of dependent
  // adds), waves 1-3 finish the cumulative potential among themselves (an LDS arrival counter, not the
  // workgroup barrier) and search every uniform with the fp64 total standing in for the potential.
  // After the chains each result is checked against the exact potential (it is numpy's index when
  // the exact threshold falls between the same two prefixes, neither within 4 cum_tol of it); any
  // other case runs the regular search for that uniform.
  __shared__ int s_sync;
  __shared__ int s_sidx[kMaxTrials];
  __shared__ int s_sok;
  // measured (profiles/r04_kpp_spec_search.txt): T = 8 (3000 x 40, k = 454) 8.07 -> 7.44 us per round
  // once the prefix reads are batched (before that the prefix alone took as long as the chains and the
  // speculation lost); T = 7 (3706 x 64, k = 371) 11.33 -> 10.44, T = 6 (Cora) 9.97 -> 9.68
  const bool spec = c + 1 < a.k && T <= 12;
  if (tid == 0) {
    s_sync = 0;
    s_sok = 1;
  }
  {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = tid + 256 * q;
      if (e < n) {
        s_d[e] = r[q];
        if (perm && e >= h4 && e < m1) {
          const int o = e - h4;
          if (k4x2)
            s_ch[(o & 3) * kChainLd + (o >> 2)] = r[q];
          else
            s_ch[(o & 7) * kChainLd + (o >> 3)] = r[q];
        }
      }
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 63);
  const int jp = tid - 64;  // prefix thread of waves 1..3
  double pre[kFPW];
  if (wave == 0) {  // sgemv_t: the lane chains, then the n % 4 trailing entries
    const float y = fold_potential(a, s_d, s_ch, t, k4x2, h4);
    if (lane == 0) {
      s_pot = y;
      if (pot_out) *pot_out = y;
    }
    GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 76);
  } else {  // the cumulative potential: thread runs and the wave's inclusive scan
    fold_prefix(a, s_d, jp, pre, s_wave);
    GDD_STAMP_WHEN(g_stamps_kpp, (tid == 64 && t == 0 && c == a.k - 2), 75);
    if (spec) {
      bool ok = prefix_waves_sync(&s_sync, 3);
      double B = 0.0;
      for (int q = 0; q < wave - 1; ++q) B = B + s_wave[q];
#pragma unroll
      for (int q = 0; q < kFPW; ++q) {
        const int e = kFPW * jp + q;
        if (e < n) s_cum[e] = B + pre[q];
      }
      ok = prefix_waves_sync(&s_sync, 6) && ok;
      const double pot_s = (double)(float)s_cum[n - 1];
      // searchsorted_left(cum, u * pot_s) in two ballots (the regular search's form, no rounding check)
      const int Bk = (n + 63) >> 6;
      const int nb = (n + Bk - 1) / Bk;
      const double cl = s_cum[min((lane + 1) * Bk, n) - 1];
      // this wave's uniforms (wave - 1, wave + 2, ... < T <= 12): every first ballot, then every
      // second-level read issued together, then the second ballots
      double rrs[4], vv[4];
      int c0s[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t2 = wave - 1 + 3 * i;
        rrs[i] = __shfl(ut, min(t2, T - 1)) * pot_s;
        c0s[i] = __popcll(__ballot(lane < nb && cl < rrs[i]));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = c0s[i] * Bk + lane;
        vv[i] = s_cum[min(e, n - 1)];  // c0s[i] == nb: unused
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t2 = wave - 1 + 3 * i;
        if (t2 >= T) continue;
        int idx = n;
        if (c0s[i] < nb) {
          const int e = c0s[i] * Bk + lane;
          const bool live = lane < Bk && e < n;
          idx = c0s[i] * Bk + __popcll(__ballot(live && vv[i] < rrs[i]));
        }
        if (lane == 0) s_sidx[t2] = idx;
      }
      if (!ok && lane == 0) s_sok = 0;
      GDD_STAMP_WHEN(g_stamps_kpp, (tid == 64 && t == 0 && c == a.k - 2), 77);
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 70);
  unsigned long long redo = ~0ull;  // the uniforms the regular search below takes
  if (spec) {
    // the check, one lane per uniform; s_cum is complete (written before the barrier)
    bool good = false;
    if (tid < T && s_sok) {
      const int idx = s_sidx[tid];
      good = spec_draw_good(a, idx, idx > 0 ? s_cum[idx - 1] : -1.0, idx < n ? s_cum[idx] : 0.0,
                            ut * (double)s_pot);
      if (good) cand_out[tid] = min(n - 1, idx);
    }
    redo = __ballot(tid < T && !good);  // wave 0's lanes tid < T
    __shared__ unsigned long long s_redo;
    if (tid == 0) s_redo = redo;
    __syncthreads();
    redo = s_redo;
    if (redo == 0ull) {
      GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 74);
      return;
    }
  }
  if (c + 1 < a.k) {
    // the prefix again when it was not written here yet, or was written while a bounded spin gave up
    // (s_sok = 0: another wave's total may have been missing from B); s_wave is complete now
    if (wave > 0 && (!spec || !s_sok)) {
      double B = 0.0;
      for (int q = 0; q < wave - 1; ++q) B = B + s_wave[q];
      const double pot = (double)s_pot;
#pragma unroll
      for (int q = 0; q < kFPW; ++q) {
        const int e = kFPW * jp + q;
        if (e < n) s_cum[e] = B + pre[q];
      }
      (void)pot;
    }
    __syncthreads();
    fold_search(a, redo, ut, (double)s_pot, s_cum, s_d, cand_out);
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 74);
}


constexpr int kMaxDimF = 512;  // fused rounds: candidate rows up to this many features

// ---- single-block rounds in ONE launch. Grid (point blocks of 256, T trials): workgroup (b, t)
// computes trial t's distances for its 256 points; the last workgroup of trial t to finish folds
// trial t (the pick work: its exact sgemv_t potential, its cumulative potential, and the candidates
// every trial would draw in round c+1 if t wins). Hand-off without fences, in the first form of
// MI355X_MICROARCH.md's table: every distance store sc1 (write-through), every storing wave drained
// (vmcnt(0)), a workgroup barrier, one lane's agent-scope add to the trial's counter for the round;
// the workgroup whose add returns G-1 reads the row back with sc1 loads. Nothing spins.
constexpr int kFPts = 256;   // points per distance workgroup
template <bool SEQ>
__global__ __launch_bounds__(256) void k_kpp1_fused(Kpp1Args a, int c) {
  __shared__ double s_c[kMaxDimF];              // this trial's candidate row (fp64, zero-padded)
  __shared__ float s_d[kBlk];                   // fold: the row, natural order
  __shared__ float s_ch[8 * kChainLd];          // fold: chain-major copy (unit weights)
  __shared__ double s_cum[kBlk];               // fold: the winner-if row's cumulative potential
  __shared__ double s_wave[4];
  __shared__ float s_pot;
  __shared__ double s_cn;
  __shared__ int s_last;
  const int tid = threadIdx.x;
  const int t = blockIdx.y, pq = (c - 1) & 1, cq = c & 1, T = a.T, dim = a.dim;
  const int Tp = c == 1 ? 1 : T;  // trials of round c-1 (round 0: the first centre)
  const int n = (int)a.n;
  const int i = blockIdx.x * kFPts + tid;
  const int ic = min(i, n - 1);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && t == 0 && c == a.k - 2), 60);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && t == 0 && c == a.k - 1), 65);
  // round trip 1: the point's column, round c-1's potentials and this trial's column of its table
  constexpr int kX = SEQ ? 48 : 1;
  float x[kX];
  if (SEQ && dim <= kX) {
#pragma unroll
    for (int v = 0; v < kX; ++v) x[v] = a.XT[(int64_t)min(v, dim - 1) * n + ic];
  }
  const double xs = a.xsq[ic];
  float pv[kMaxTrials], dv[kMaxTrials];
  int64_t cw[kMaxTrials];
  // every trial's distance for this point too (the winner is not known yet): the winner's row
  // then costs no dependent round trip of its own
  const float* dprev = c == 1 ? a.closest0 : a.dist[pq];
#pragma unroll
  for (int q = 0; q < kMaxTrials; ++q) {
    pv[q] = a.potv[pq][min(q, Tp - 1)];
    cw[q] = a.candw[pq][(int64_t)min(q, Tp - 1) * T + t];
    dv[q] = dprev[(int64_t)min(q, Tp - 1) * n + ic];
  }
  int bw = 0;  // np.argmin: first minimum, a NaN wins at once
  float best = pv[0];
  int64_t ct = cw[0];
  float wi = dv[0];
#pragma unroll
  for (int q = 1; q < kMaxTrials; ++q) {
    const float pt = pv[q];
    if (q < Tp && best == best && (pt < best || pt != pt)) {
      bw = q;
      best = pt;
      ct = cw[q];
      wi = dv[q];
    }
  }
  // round trip 2: this trial's candidate row
  const int cs = (SEQ && dim <= kX) ? kX : dim;
  for (int j = tid; j < cs; j += 256) s_c[j] = j < dim ? (double)a.X[ct * dim + min(j, dim - 1)] : 0.0;
  if (tid == 0) s_cn = a.xsq[ct];
  if (blockIdx.x == 0 && tid == 0) {
    a.candself[cq][t] = ct;
    if (c >= 2 && t == 0) a.indices[c - 1] = a.candself[pq][bw];  // rows gathered after the rounds
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && blockIdx.x == 0 && t == 0 && c == a.k - 2), 61);
  if (i < n) {
    double dot = 0.0;
    if constexpr (SEQ) {
      if (dim <= kX) {
#pragma unroll
        for (int v = 0; v < kX; ++v) dot = __builtin_fma(s_c[v], (double)x[v], dot);
      } else {
        for (int j = 0; j < dim; j += 16) {
          float y[16];
#pragma unroll
          for (int v = 0; v < 16; ++v) y[v] = a.XT[(int64_t)min(j + v, dim - 1) * n + i];
#pragma unroll
          for (int v = 0; v < 16; ++v)
            if (j + v < dim) dot = __builtin_fma(s_c[j + v], (double)y[v], dot);
        }
      }
    } else {
      dot = skl_point_dot(a.plan, s_c, a.X + (int64_t)i * dim, i, t);
    }
    float f = (float)(((-2.0 * dot) + s_cn) + xs);
    f = f < 0.f ? 0.f : f;
    __hip_atomic_store(a.dist[cq] + (int64_t)t * n + i, np_minimum(wi, f), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);  // sc1: write-through
  }
  // hand-off: every storing wave drained, barrier, one agent-scope add per workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(a.counter + (int64_t)c * T + t, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 62);
  // ---- fold trial t (its last workgroup): the row back with sc1 loads
  const double ut = (c + 1 < a.k && (tid & 63) < T) ? a.uniforms[(int64_t)c * T + (tid & 63)] : 0.0;
  float r[16];
  {
    const float* row = a.dist[cq] + (int64_t)t * n;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      r[q] = __hip_atomic_load(row + min(tid + 256 * q, n - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  kpp1_fold_trial(a, c, t, r, ut, s_d, s_ch, s_cum, s_wave, &s_pot, a.potv[cq] + t,
                  a.candw[cq] + (int64_t)t * T);
}

// ---- single-block rounds from a distance table (plain-chain plans, dim <= 64, n <= 4096). The
// plain fp64 chain of a distance does not depend on the trial slot the candidate occupies, so every
// distance a round can ask for is one entry of D[j][i] = the clamped fp32 upcast distance between
// candidate point j and point i, computed once per fit by k_kpp_dmat in exactly the arithmetic of
// the distance phase above (zero-padded 48- or 64-term fma chain, ((-2 dot) + |c|^2) + |x|^2, clamp).
// A round is then ONE workgroup per trial: round c-1's potentials and this trial's candidate column
// (trip 1), the winner's row = the closest distances and the candidate's D row (trip 2), the fold.
// No distance phase, no write-through hand-off, no re-read of the row.
// The chain's feature slots: 48 (dim <= 48) or 64 (dim <= 64, e.g. the recsys SVD embeddings);
// slots past dim are zero, and an fma with a zero operand leaves the chain unchanged.
constexpr int kDmX = 64;   // widest table chain (dim <= kDmX)
constexpr int kDmMinK = 16;  // centres from which the table is built

template <int TI, int TJ>
__global__ __launch_bounds__(256) void k_kpp_dmat_t(int n, int dim, const float* __restrict__ XT,
                                                    const double* __restrict__ xsq,
                                                    float* __restrict__ D) {
  constexpr int BI = 16 * TI, BJ = 16 * TJ;  // block tile: BI points x BJ candidates
  extern __shared__ __attribute__((aligned(16))) double s_dm[];
  double* s_x = s_dm;             // [dim][BI] points
  double* s_c = s_dm + BI * dim;  // [dim][BJ] candidates
  const int tid = threadIdx.x, ti = tid & 15, tj = tid >> 4;
  const int i0 = blockIdx.x * BI, j0 = blockIdx.y * BJ;
  for (int e = tid; e < BI * dim; e += 256) {
    const int v = e / BI, q = e - v * BI;
    s_x[e] = (double)XT[(int64_t)v * n + min(i0 + q, n - 1)];
  }
  for (int e = tid; e < BJ * dim; e += 256) {
    const int v = e / BJ, q = e - v * BJ;
    s_c[e] = (double)XT[(int64_t)v * n + min(j0 + q, n - 1)];
  }
  double xs[TI], cn[TJ];
#pragma unroll
  for (int b = 0; b < TI; ++b) xs[b] = xsq[min(i0 + TI * ti + b, n - 1)];
#pragma unroll
  for (int a = 0; a < TJ; ++a) cn[a] = xsq[min(j0 + TJ * tj + a, n - 1)];
  __syncthreads();
  double dot[TJ][TI];
#pragma unroll
  for (int a = 0; a < TJ; ++a)
#pragma unroll
    for (int b = 0; b < TI; ++b) dot[a][b] = 0.0;
  const double* px = s_x + TI * ti;
  const double* pc = s_c + TJ * tj;
  for (int v = 0; v < dim; ++v) {
    double xv[TI], cv[TJ];
#pragma unroll
    for (int b = 0; b < TI; b += 2) {
      const double2 t = *reinterpret_cast<const double2*>(px + BI * v + b);
      xv[b] = t.x;
      xv[b + 1] = t.y;
    }
#pragma unroll
    for (int a = 0; a < TJ; a += 2) {
      const double2 t = *reinterpret_cast<const double2*>(pc + BJ * v + a);
      cv[a] = t.x;
      cv[a + 1] = t.y;
    }
#pragma unroll
    for (int a = 0; a < TJ; ++a)
#pragma unroll
      for (int b = 0; b < TI; ++b) dot[a][b] = __builtin_fma(cv[a], xv[b], dot[a][b]);
  }
  const int ib = i0 + TI * ti;
  const bool vec = (n & 3) == 0 && ib + TI - 1 < n;
#pragma unroll
  for (int a = 0; a < TJ; ++a) {
    const int j = j0 + TJ * tj + a;
    if (j >= n) break;
    float f[TI];
#pragma unroll
    for (int b = 0; b < TI; ++b) {
      f[b] = (float)(((-2.0 * dot[a][b]) + cn[a]) + xs[b]);
      f[b] = f[b] < 0.f ? 0.f : f[b];
    }
    float* out = D + (int64_t)j * n + ib;
    if (vec) {
#pragma unroll
      for (int b = 0; b < TI; b += 4)
        *reinterpret_cast<float4*>(out + b) = make_float4(f[b], f[b + 1], f[b + 2], f[b + 3]);
    } else {
#pragma unroll
      for (int b = 0; b < TI; ++b)
        if (ib + b < n) out[b] = f[b];
    }
  }
}

// the n x n distance table (k_kpp_dmat_t: 4 x 4 fp64 register tiles per thread; r05 measured the
// 8 x 4 and 8 x 8 tiles and the r04 one-row-per-thread form slower)
int launch_kpp_dmat(int64_t n, int dim, const float* X, const float* XT, const double* xsq, float* D,
                    hipStream_t s) {
  (void)X;
  constexpr int ti = 4, tj = 4;
  const size_t lds = sizeof(double) * 16 * (size_t)(ti + tj) * dim;
  if (lds > 65536)
    GDD_HIP(hipFuncSetAttribute((const void*)k_kpp_dmat_t<ti, tj>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
  const dim3 g((unsigned)((n + 16 * ti - 1) / (16 * ti)), (unsigned)((n + 16 * tj - 1) / (16 * tj)));
  k_kpp_dmat_t<ti, tj><<<g, 256, lds, s>>>((int)n, dim, XT, xsq, D);
  GDD_LAUNCHED();
  return GDD_OK;
}

__global__ __launch_bounds__(256) void k_kpp1_dm(Kpp1Args a, const float* __restrict__ D, int c) {
  __shared__ float s_d[kBlk];
  __shared__ float s_ch[8 * kChainLd];
  __shared__ double s_cum[kBlk];
  __shared__ double s_wave[4];
  __shared__ float s_pot;
  const int tid = threadIdx.x;
  const int t = blockIdx.x, pq = (c - 1) & 1, cq = c & 1, T = a.T;
  const int Tp = c == 1 ? 1 : T;  // trials of round c-1 (round 0: the first centre)
  const int n = (int)a.n;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 60);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 1), 65);
  // trip 1: round c-1's potentials and this trial's column of its candidate table
  float pv[kMaxTrials];
  int64_t cw[kMaxTrials];
#pragma unroll
  for (int q = 0; q < kMaxTrials; ++q) {
    pv[q] = a.potv[pq][min(q, Tp - 1)];
    cw[q] = a.candw[pq][(int64_t)min(q, Tp - 1) * T + t];
  }
  const double ut = (c + 1 < a.k && (tid & 63) < T) ? a.uniforms[(int64_t)c * T + (tid & 63)] : 0.0;
  // round c-1's own candidates with the potentials (not a dependent trip after the argmin)
  const int64_t csl = c >= 2 ? a.candself[pq][min(tid & 63, T - 1)] : 0;
  int bw = 0;  // np.argmin: first minimum, a NaN wins at once
  float best = pv[0];
  int64_t ct = cw[0];
#pragma unroll
  for (int q = 1; q < kMaxTrials; ++q) {
    const float pt = pv[q];
    if (q < Tp && best == best && (pt < best || pt != pt)) {
      bw = q;
      best = pt;
      ct = cw[q];
    }
  }
  const int64_t sw = __shfl(csl, bw);
  if (tid == 0) {
    a.candself[cq][t] = ct;
    if (c >= 2 && t == 0) a.indices[c - 1] = sw;  // rows gathered after the rounds
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 61);
  // trip 2: the closest distances (round c-1's winning row) and the candidate's table row
  const float* wrow = c == 1 ? a.closest0 : a.dist[pq] + (int64_t)bw * n;
  const float* drow = D + ct * n;
  float wi[16], dd[16], r[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = min(tid + 256 * q, n - 1);
    wi[q] = wrow[e];
    dd[q] = drow[e];
  }
  float* orow = a.dist[cq] + (int64_t)t * n;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    r[q] = np_minimum(wi[q], dd[q]);
    if (tid + 256 * q < n) orow[tid + 256 * q] = r[q];
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 62);
  kpp1_fold_trial(a, c, t, r, ut, s_d, s_ch, s_cum, s_wave, &s_pot, a.potv[cq] + t,
                  a.candw[cq] + (int64_t)t * T);
}

// ---- a pair launch's two folds overlapped (r06). The serial form (kpp1_fold_trial twice) runs round
// c's fold, then loads round c+1's row, then folds it: two lane-chain runs (~2 us each at 3,000
// entries) and the row's load one after another. Here wave 0 runs round c's chains while waves 1-3
// finish its cumulative potential, draw slot t2's candidate with the fp64 total standing in for the
// potential (kpp1_fold_trial's speculative search), load that candidate's table row, form round c+1's
// row and its cumulative potential and speculatively draw round c+2's candidates; wave 0 then checks
// the slot-t2 draw against round c's exact potential and runs round c+1's chains. Waves 1-3 meet on an
// LDS arrival counter and never wait for wave 0. If the check fails (the threshold within 4 cum_tol of
// a deciding prefix, or the stand-in potential moved the count), or a bounded spin gives up, the call
// returns false after its barrier and the caller redoes the pair serially — so every result is the
// serial form's. Level-1 row in r (entry tid + 256 q), trial w's lane form; level 2 trial t2's.
__device__ __forceinline__ bool kpp1_fold_pair(const Kpp1Args& a, const float* __restrict__ D, int c, int w,
                                               int t2, int lq, const float (&r)[16], double ut, double ut2,
                                               float* __restrict__ s_d, float* __restrict__ s_ch,
                                               float* __restrict__ s_d2, float* __restrict__ s_ch2,
                                               double* __restrict__ s_cum, double* __restrict__ s_wave) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T, n = (int)a.n, m1 = (int)a.m1;
  const bool perm = a.w == nullptr;
  const int j = w * T + t2;
  const bool k4x2_1 = (T & 2) && w >= (T & ~3) && w < (T & ~3) + 2;
  const bool k4x2_2 = (T & 2) && t2 >= (T & ~3) && t2 < (T & ~3) + 2;
  const int h4_1 = k4x2_1 ? 0 : (m1 & 4), h4_2 = k4x2_2 ? 0 : (m1 & 4);
  const bool spec2 = c + 2 < a.k;  // round c+1 draws round c+2's candidates
  __shared__ int s_arr;            // waves 1-3: arrivals
  __shared__ int s_fail;           // a check or a bounded spin failed: the caller redoes the pair
  __shared__ int s_idx1;           // slot t2's speculative draw and its deciding neighbours
  __shared__ double s_lo1, s_hi1;
  __shared__ int s_sidx2[kMaxTrials];
  __shared__ float s_pot2;
  if (tid == 0) {
    s_arr = 0;
    s_fail = 0;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q;
    if (e < n) {
      s_d[e] = r[q];
      if (perm && e >= h4_1 && e < m1) {
        const int o = e - h4_1;
        if (k4x2_1)
          s_ch[(o & 3) * kChainLd + (o >> 2)] = r[q];
        else
          s_ch[(o & 7) * kChainLd + (o >> 3)] = r[q];
      }
    }
  }
  __syncthreads();
  if (wave == 0) {
    float y = fold_potential(a, s_d, s_ch, w, k4x2_1, h4_1);
    y = __shfl(y, 0);
    if (lane == 0 && t2 == 0) a.potv[lq][w] = y;
    bool ok = waves_wait(&s_arr, 9);  // slot t2's draw published
    ok = ok && spec_draw_good(a, s_idx1, s_lo1, s_hi1, __shfl(ut, t2) * (double)y);
    ok = ok && waves_wait(&s_arr, 12);  // round c+1's row complete
    if (!ok) {
      if (lane == 0) s_fail = 1;
    } else {
      const float y2 = fold_potential(a, s_d2, s_ch2, t2, k4x2_2, h4_2);
      if (lane == 0) {
        s_pot2 = y2;
        a.potv2[lq][j] = y2;
      }
    }
  } else {
    const int jp = tid - 64;
    double pre[kFPW];
    fold_prefix(a, s_d, jp, pre, s_wave);
    bool ok = prefix_waves_sync(&s_arr, 3);
    double B = 0.0;
    for (int q = 0; q < wave - 1; ++q) B = B + s_wave[q];
#pragma unroll
    for (int q = 0; q < kFPW; ++q) {
      const int e = kFPW * jp + q;
      if (e < n) s_cum[e] = B + pre[q];
    }
    ok = prefix_waves_sync(&s_arr, 6) && ok;
    // slot t2's draw, by each of the three waves (same bits): searchsorted_left in two ballots
    const int Bk = (n + 63) >> 6;
    const int nb = (n + Bk - 1) / Bk;
    int idx = n;
    {
      const double cl = s_cum[min((lane + 1) * Bk, n) - 1];
      const double rr = __shfl(ut, t2) * (double)(float)s_cum[n - 1];
      const int c0 = __popcll(__ballot(lane < nb && cl < rr));
      if (c0 < nb) {
        const int e = c0 * Bk + lane;
        const bool live = lane < Bk && e < n;
        const double v = s_cum[min(e, n - 1)];
        idx = c0 * Bk + __popcll(__ballot(live && v < rr));
      }
    }
    if (wave == 1 && lane == 0) {
      s_idx1 = idx;
      s_lo1 = idx > 0 ? s_cum[idx - 1] : -1.0;
      s_hi1 = idx < n ? s_cum[idx] : 0.0;
    }
    ok = prefix_waves_sync(&s_arr, 9) && ok;  // every read of round c's s_cum and s_wave done
    // round c+1's row: entries jp + 192 q, against the speculatively drawn candidate's table row
    {
      const int64_t c1 = min(n - 1, idx);
      const float* drow = D + c1 * n;
      float* orow = a.dist2[lq] + (int64_t)j * n;
      float dd[kFPW];
#pragma unroll
      for (int q = 0; q < kFPW; ++q) dd[q] = drow[min(jp + 192 * q, n - 1)];
#pragma unroll
      for (int q = 0; q < kFPW; ++q) {
        const int e = jp + 192 * q;
        if (e < n) {
          const float f = np_minimum(s_d[e], dd[q]);
          orow[e] = f;
          s_d2[e] = f;
          if (perm && e >= h4_2 && e < m1) {
            const int o = e - h4_2;
            if (k4x2_2)
              s_ch2[(o & 3) * kChainLd + (o >> 2)] = f;
            else
              s_ch2[(o & 7) * kChainLd + (o >> 3)] = f;
          }
        }
      }
    }
    ok = prefix_waves_sync(&s_arr, 12) && ok;  // the row complete (wave 0 waits for it)
    fold_prefix(a, s_d2, jp, pre, s_wave);
    ok = prefix_waves_sync(&s_arr, 15) && ok;
    B = 0.0;
    for (int q = 0; q < wave - 1; ++q) B = B + s_wave[q];
#pragma unroll
    for (int q = 0; q < kFPW; ++q) {
      const int e = kFPW * jp + q;
      if (e < n) s_cum[e] = B + pre[q];
    }
    ok = prefix_waves_sync(&s_arr, 18) && ok;
    if (spec2) {  // round c+2's draws with the fp64 total for round c+1's potential (4 per wave)
      const double pot_s = (double)(float)s_cum[n - 1];
      const double cl = s_cum[min((lane + 1) * Bk, n) - 1];
      double rrs[4], vv[4];
      int c0s[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u2 = wave - 1 + 3 * i;
        rrs[i] = __shfl(ut2, min(u2, T - 1)) * pot_s;
        c0s[i] = __popcll(__ballot(lane < nb && cl < rrs[i]));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) vv[i] = s_cum[min(c0s[i] * Bk + lane, n - 1)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u2 = wave - 1 + 3 * i;
        if (u2 >= T) continue;
        int id2 = n;
        if (c0s[i] < nb) {
          const int e = c0s[i] * Bk + lane;
          const bool live = lane < Bk && e < n;
          id2 = c0s[i] * Bk + __popcll(__ballot(live && vv[i] < rrs[i]));
        }
        if (lane == 0) s_sidx2[u2] = id2;
      }
    }
    if (!ok && lane == 0) s_fail = 1;
  }
  __syncthreads();
  if (s_fail) return false;
  if (tid == 0) a.candself2[lq][j] = min(n - 1, s_idx1);
  if (!spec2) return true;
  // round c+1's draws: the check (lane q of wave 0 for uniform q), the regular search for the rest
  int64_t* cand_out = a.candw2[lq] + (int64_t)j * T;
  const double pot2 = (double)s_pot2;
  bool good = false;
  if (tid < T) {
    const int idx = s_sidx2[tid];
    good = spec_draw_good(a, idx, idx > 0 ? s_cum[idx - 1] : -1.0, idx < n ? s_cum[idx] : 0.0, ut2 * pot2);
    if (good) cand_out[tid] = min(n - 1, idx);
  }
  __shared__ unsigned long long s_redo;
  const unsigned long long redo = __ballot(tid < T && !good);  // wave 0's lanes tid < T
  if (tid == 0) s_redo = redo;
  __syncthreads();
  if (s_redo != 0ull) fold_search(a, s_redo, ut2, pot2, s_cum, s_d2, cand_out);
  return true;
}

// ---- two rounds per launch over the distance table (default for table plans, T <= 8). Workgroup
// w * T + t runs round c+1's trial t on the assumption that round c's trial w wins: it forms trial w's
// row and folds it (same operands, same slot, so bit-identical to what a round-c workgroup w would
// compute), takes w's round-(c+1) candidate for slot t, reads that candidate's table row (a third
// dependent trip) and folds round c+1's trial t. Workgroup w * T also publishes round c's trial w
// (potential, candidate). The next launch resolves both winners from the potentials: T + T * T
// floats and its column of the T * T x T candidate table in its first trip, one wave lane per entry.
// A trailing odd round runs alone (pair == 0: T workgroups, round c only). State slots alternate by
// launch (lq); round 1 reads the first centre's slot-0 candidates, so the first launch writes slot 1.
// Per round this halves the launches and their two leading trips (k_kpp1_dm: 9.2 us per round).
constexpr int kPairMaxT = 8;  // T * T <= 64: one wave lane per round-(c-1) candidate

__global__ __launch_bounds__(256) void k_kpp1_dm2(Kpp1Args a, const float* __restrict__ D, int c, int lq,
                                                  int pair, int overlap) {
  __shared__ float s_d[kBlk];
  __shared__ float s_ch[8 * kChainLd];
  __shared__ float s_d2[kBlk];             // the overlapped form: round c+1's row
  __shared__ float s_ch2[8 * kChainLd];
  __shared__ double s_cum[kBlk];
  __shared__ double s_wave[4];
  __shared__ float s_pot;
  __shared__ int64_t s_cand[kMaxTrials];
  const int tid = threadIdx.x, lane = tid & 63;
  const int T = a.T, pl = lq ^ 1, TT = T * T;
  const int n = (int)a.n;
  const int g = blockIdx.x;
  const int w = pair ? g / T : g;        // round c's trial this workgroup forms first
  const int t2 = pair ? g - w * T : 0;   // round c+1's trial (pair launches)
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && g == 0 && c == a.k - 3 + (a.k & 1)), 60);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && g == 0 && c == a.k - 1 + (a.k & 1)), 65);
  // trip 1: the previous launch's potentials and this slot's candidates
  const float* wrow;
  int64_t ct;
  if (c == 1) {
    wrow = a.closest0;
    ct = a.candw[0][w];  // k_kpp1_pick(.., 0): the first centre's candidates
  } else {
    float pv[kPairMaxT];
#pragma unroll
    for (int q = 0; q < kPairMaxT; ++q) pv[q] = a.potv[pl][min(q, T - 1)];
    const float p2 = a.potv2[pl][min(lane, TT - 1)];
    const int64_t c2 = a.candw2[pl][(int64_t)min(lane, TT - 1) * T + w];
    // the previous launch's own candidates, requested with the potentials (r05: read after the
    // argmin they were a second dependent trip on workgroup 0's wave 0, the launch's straggler)
    const int64_t cs1 = a.candself[pl][min(lane, T - 1)];
    const int64_t cs2 = a.candself2[pl][min(lane, TT - 1)];
    int bw = 0;  // np.argmin: first minimum, a NaN wins at once
    float best = pv[0];
#pragma unroll
    for (int q = 1; q < kPairMaxT; ++q) {
      const float pt = pv[q];
      if (q < T && best == best && (pt < best || pt != pt)) {
        bw = q;
        best = pt;
      }
    }
    int bv = 0;
    float best2 = __shfl(p2, bw * T);
    for (int q = 1; q < T; ++q) {
      const float pt = __shfl(p2, bw * T + q);
      if (best2 == best2 && (pt < best2 || pt != pt)) {
        bv = q;
        best2 = pt;
      }
    }
    const int j = bw * T + bv;
    ct = __shfl(c2, j);
    wrow = a.dist2[pl] + (int64_t)j * n;
    const int64_t i1 = __shfl(cs1, bw), i2 = __shfl(cs2, j);
    if (g == 0 && tid == 0) {  // rows gathered after the rounds
      a.indices[c - 2] = i1;
      a.indices[c - 1] = i2;
    }
  }
  const double ut = (c + 1 < a.k && (tid & 63) < T) ? a.uniforms[(int64_t)c * T + (tid & 63)] : 0.0;
  const double ut2 = (pair && c + 2 < a.k && (tid & 63) < T) ? a.uniforms[(int64_t)(c + 1) * T + (tid & 63)] : 0.0;
  if (tid == 0 && (!pair || t2 == 0)) a.candself[lq][w] = ct;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && g == 0 && c == a.k - 3 + (a.k & 1)), 61);
  // trip 2: the closest distances and the candidate's table row
  const float* drow = D + ct * n;
  float wi[16], dd[16], r[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = min(tid + 256 * q, n - 1);
    wi[q] = wrow[e];
    dd[q] = drow[e];
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) r[q] = np_minimum(wi[q], dd[q]);
  if (!pair) {  // the last round alone: as k_kpp1_dm
    kpp1_fold_trial(a, c, w, r, ut, s_d, s_ch, s_cum, s_wave, &s_pot, a.potv[lq] + w,
                    a.candw[lq] + (int64_t)w * T);
    return;
  }
  if (overlap && kpp1_fold_pair(a, D, c, w, t2, lq, r, ut, ut2, s_d, s_ch, s_d2, s_ch2, s_cum, s_wave)) return;
  __syncthreads();  // (after a failed overlapped pair: its LDS reads done before the serial form's writes)
  kpp1_fold_trial(a, c, w, r, ut, s_d, s_ch, s_cum, s_wave, &s_pot, t2 == 0 ? a.potv[lq] + w : nullptr,
                  s_cand);
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && g == 0 && c == a.k - 3 + (a.k & 1)), 62);
  // trip 3: round c+1's candidate for slot t2 if w wins, and its table row
  const int64_t c1 = s_cand[t2];
  const int j = w * T + t2;
  if (tid == 0) a.candself2[lq][j] = c1;
  const float* drow2 = D + c1 * n;
#pragma unroll
  for (int q = 0; q < 16; ++q) dd[q] = drow2[min(tid + 256 * q, n - 1)];
  float* orow = a.dist2[lq] + (int64_t)j * n;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    wi[q] = np_minimum(r[q], dd[q]);
    if (tid + 256 * q < n) orow[tid + 256 * q] = wi[q];
  }
  kpp1_fold_trial(a, c + 1, t2, wi, ut2, s_d, s_ch, s_cum, s_wave, &s_pot, a.potv2[lq] + j,
                  a.candw2[lq] + (int64_t)j * T);
}

// after the last launch of k_kpp1_dm2: its winner(s) and the last centre
__global__ __launch_bounds__(64) void k_kpp1_final2(Kpp1Args a, int c, int lq, int pair) {
  const int T = a.T;
  const int b = kpp1_argmin(a.potv[lq], T);
  int64_t src = a.candself[lq][b];
  if (pair) {
    const int v = kpp1_argmin(a.potv2[lq] + (int64_t)b * T, T);
    if (threadIdx.x == 0) a.indices[c - 1] = src;
    src = a.candself2[lq][(int64_t)b * T + v];
  }
  if (threadIdx.x == 0) a.indices[c] = src;
  for (int j = threadIdx.x; j < a.dim; j += 64) a.centers[(int64_t)c * a.dim + j] = a.X[src * a.dim + j];
}

// after round k-1: its winner and centre
__global__ __launch_bounds__(64) void k_kpp1_final(Kpp1Args a, int c) {
  const int q = c & 1;
  const int b = kpp1_argmin(a.potv[q], a.T);
  const int64_t src = a.candself[q][b];
  if (threadIdx.x == 0) a.indices[c] = src;
  for (int j = threadIdx.x; j < a.dim; j += 64) a.centers[(int64_t)c * a.dim + j] = a.X[src * a.dim + j];
}

// ---- table rounds for 4096 < n <= 32768 (r04): ONE 1024-thread workgroup per trial, as k_kpp1_dm
// (no per-block partial terms, no fold launch reading T x blocks values). The ML-1M users (6,040 x 64,
// k = 604) and Ali-Display users (17,730 x 64, k = 1,773) shapes of the recsys clustering. Per round c:
//   trip 1   lane q of every wave loads round c-1's potential q, this slot's candidate if q won and
//            q's own candidate, and round c+1's uniform q; np.argmin over lanes;
//   trip 2   the winner's row (the closest distances) and the candidate's table row, coalesced
//            (entry tid + 1024 q), np.minimum, stored for round c+1's winner read and into LDS;
//   fold     each thread's fp64 run over its segment, a wave scan and the wave totals give every
//            entry's cumulative potential; waves b < nsg run the sgemv_t lane chains of 4096-entry block
//            b (the order of sgemv_block_wave, the multi-block rounds' block term; unit weights read
//            with immediate offsets, a 16-entry group ahead of the adds), added in block
//            order, then the n % 4 tail — the same potential bits as k_kpp_round;
//   draws    searchsorted_left(cum, u * pot) for round c+1's T uniforms as a count of entries below
//            the threshold: whole segments below by ballot counts, the segment that straddles it by a
//            walk (LDS add); a prefix within cum_tol of the threshold replays numpy's left-to-right sum.
// Round 0 (c == 0, one workgroup) draws round 1's candidates from the first centre's closest0 and
// its sdot potential. LDS: the row, 4 * (1024 * EPT + kChainPad) bytes (dynamic).
constexpr int kBigThr = 1024;
constexpr int kBigWaves = kBigThr / 64;
constexpr int64_t kBig1Max = 32768;


// sgemv_block_wave over entries [j0, j0 + NB) of the LDS row: the same lanes, order and operations
// (8 lanes: first NB & 4 entries on lanes 0..3, then lane (o - h4) % 8, fma with the weight —
// fma(x, 1, acc) == acc + x; the 4-lane trials: product, then add — x * 1 == x).
__device__ __forceinline__ float sgemv_block_lds(const float* __restrict__ s, const float* __restrict__ w,
                                                 int j0, int NB, int t, int T) {
  const int lane = threadIdx.x & 63;
  const bool k4x2 = (T & 2) && t >= (T & ~3) && t < (T & ~3) + 2;
  const int nl = k4x2 ? 4 : 8;
  const int h4 = k4x2 ? 0 : (NB & 4);
  float acc = 0.f;
  if (lane < nl) {
    if (lane < h4) acc = __builtin_fmaf(s[j0 + lane], w ? w[j0 + lane] : 1.0f, acc);
    const int o0 = h4 + lane;
    const int L = o0 < NB ? (NB - o0 + nl - 1) / nl : 0;  // this lane's chain length
    if (w == nullptr) {
      acc = k4x2 ? chain_unit_lds<4>(s + j0 + o0, L, acc) : chain_unit_lds<8>(s + j0 + o0, L, acc);
    } else {
      for (int m = 0; m < L; ++m) {
        const int e = j0 + o0 + nl * m;
        acc = k4x2 ? acc + s[e] * w[e] : __builtin_fmaf(s[e], w[e], acc);
      }
    }
  }
  if (k4x2) {
    const float a1 = __shfl(acc, 1), a2 = __shfl(acc, 2), a3 = __shfl(acc, 3);
    return (acc + a1) + (a2 + a3);
  }
  const float ql = acc + __shfl(acc, (lane + 4) & 63);  // q_l = a_l + a_{l+4}
  const float q1 = __shfl(ql, 1), q2 = __shfl(ql, 2), q3 = __shfl(ql, 3);
  return (ql + q1) + (q2 + q3);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the 1024-thread table rounds' shared state besides the row (k_kpp1_big, k_kpp1_big2)
struct BigLds {
  double wt[kBigWaves];
  float vb[8];
  float pot;
  int cnt[kMaxTrials];
  int part[kMaxTrials];
  int amb[kMaxTrials];
  double off[kBigThr], first[kBigThr], last[kBigThr];
  int arr;                 // speculative draws: waves that wrote their prefix data
  int sidx[kMaxTrials];    // speculative draws: counts (-1: not usable)
  double lo[kMaxTrials], hi[kMaxTrials];  // and their deciding neighbours
  unsigned long long redo;  // the uniforms the regular draws take
};

// a fold's counters, zeroed before the barrier that publishes its row
__device__ __forceinline__ void big_fold_reset(BigLds& L) {
  const int tid = threadIdx.x;
  if (tid < kMaxTrials) {
    L.part[tid] = 0;
    L.amb[tid] = 0;
  }
  if (tid == 0) L.arr = 0;
}

// The fold of round c's trial t over the row in s_row (entries [0, n), zeros up to kBigThr * EPT):
// the potential (pot_out, nullable) and the candidates round c+1's T uniforms draw if t wins
// (cand_out[0..T), global memory or LDS). Lane q < T of every wave holds u_q = uniforms[c T + q] in ut.
// Called after a barrier that follows big_fold_reset and the row's stores.
template <int EPT>
__device__ __forceinline__ void big_fold(const Kpp1Args& a, int c, int t, double ut, const float* s_row,
                                         BigLds& L, float* pot_out, int64_t* cand_out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T;
  const int n = (int)a.n, m1 = (int)a.m1;
  const int nsg = (m1 + kBlk - 1) / kBlk;  // chain waves (4096-entry sgemv_t blocks)
  // speculative draws (r04): waves nsg .. nsg + T - 1 draw round c+1's candidates while waves < nsg
  // run the lane chains, the fp64 total standing in for the potential; checked after it (below)
  const bool spec = c >= 1 && c + 1 < a.k && nsg + T <= kBigWaves;
  // ---- this thread's segment: products (fp32) and its fp64 run
  const int e0 = EPT * tid;
  float v[EPT];
#pragma unroll
  for (int q = 0; q < EPT; q += 4) {
    const float4 x = *reinterpret_cast<const float4*>(s_row + e0 + q);
    v[q] = x.x;
    v[q + 1] = x.y;
    v[q + 2] = x.z;
    v[q + 3] = x.w;
  }
  if (a.w) {
#pragma unroll
    for (int q = 0; q < EPT; ++q) v[q] = e0 + q < n ? a.w[e0 + q] * v[q] : 0.f;
  }
  double tot = 0.0;
#pragma unroll
  for (int q = 0; q < EPT; ++q) tot = tot + (double)v[q];
  double inc = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(inc, o);
    if (lane >= o) inc = inc + y;
  }
  double ex = __shfl_up(inc, 1);
  if (lane == 0) ex = 0.0;
  if (lane == 63) L.wt[wave] = inc;
  if (spec) {  // until the barrier below L.off / L.last hold each segment's in-wave prefix and total
    L.off[tid] = ex;
    L.last[tid] = tot;
    waves_arrive(&L.arr);
  }
  // the sgemv_t block terms (rounds >= 1)
  if (c >= 1 && wave < nsg) {
    const int j0 = wave * kBlk;
    const float vb = sgemv_block_lds(s_row, a.w, j0, min(kBlk, m1 - j0), t, T);
    if (lane == 0) L.vb[wave] = vb;
  } else if (spec && wave - nsg < T) {
    // searchsorted_left(cum, u * pot_s), pot_s = fp32(fp64 total), without the rounding check (the
    // check after the potential decides): the wave totals' running sum finds the group of 64
    // segments (contiguous entries) holding the threshold, one ballot over that group's segment
    // ends counts the segments below, the segment that straddles it is walked. Offsets are the
    // group's running sum plus the in-wave prefix — within fp64 roundings of the regular ones: a
    // count they change has a value within 4 cum_tol of the threshold, which the check refuses.
    // One group per uniform keeps the LDS reads beside the chains small.
    const int t2 = wave - nsg;
    bool ok = waves_wait(&L.arr, kBigWaves);
    double tall = 0.0;
    for (int q = 0; q < kBigWaves; ++q) tall = tall + L.wt[q];
    const double rr = readlane_f64(ut, t2) * (double)(float)tall;
    int g = 0;
    double W = 0.0, Wg = 0.0;
    for (int q = 0; q < kBigWaves; ++q) {
      W = W + L.wt[q];
      if (W < rr) {
        g = q + 1;
        Wg = W;
      }
    }
    int full = 0, part = 0;
    if (g >= kBigWaves) {
      full = n;  // every entry below (idx = n)
    } else {
      const int j = lane + 64 * g, ej = EPT * j;
      const bool live = ej < n;
      const double oj = L.off[j] + Wg;
      const double tt = L.last[j];
      float x0 = s_row[ej];
      if (a.w) x0 = live ? a.w[ej] * x0 : 0.f;
      const bool below = live && ej + EPT <= n && oj + tt < rr;
      full = 64 * EPT * g + EPT * __popcll(__ballot(below));
      if (live && !below && oj + (double)x0 < rr) {  // may straddle the threshold: walk it
        float vs[EPT];
#pragma unroll
        for (int q = 0; q < EPT; q += 4) {
          const float4 x = *reinterpret_cast<const float4*>(s_row + ej + q);
          vs[q] = x.x;
          vs[q + 1] = x.y;
          vs[q + 2] = x.z;
          vs[q + 3] = x.w;
        }
        if (a.w) {
#pragma unroll
          for (int q = 0; q < EPT; ++q) vs[q] = ej + q < n ? a.w[ej + q] * vs[q] : 0.f;
        }
        double run = oj;
#pragma unroll
        for (int q = 0; q < EPT; ++q) {
          run = run + (double)vs[q];
          if (ej + q < n) part += run < rr;
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
    ok = __ballot(!ok) == 0ull;
    // the deciding neighbours for the check, independent of the potential: the walk's cumulative
    // values of entries idx - 1 (lane 0) and idx (lane 1), with the regular offsets (in-wave prefix,
    // then the wave totals in order) and each segment's reads issued before its run
    const int idx = full + part;
    double nv = lane == 0 ? -1.0 : 0.0;
    const int e = idx - 1 + lane;
    if (lane < 2 && e >= 0 && e < n) {
      const int j = e / EPT, ej = EPT * j;
      float vs[EPT];
#pragma unroll
      for (int q = 0; q < EPT; q += 4) {
        const float4 x = *reinterpret_cast<const float4*>(s_row + ej + q);
        vs[q] = x.x;
        vs[q + 1] = x.y;
        vs[q + 2] = x.z;
        vs[q + 3] = x.w;
      }
      if (a.w) {
#pragma unroll
        for (int q = 0; q < EPT; ++q) vs[q] = ej + q < n ? a.w[ej + q] * vs[q] : 0.f;
      }
      double run = L.off[j];  // ex of segment j until the barrier below
      for (int q = 0; q < (j >> 6); ++q) run = run + L.wt[q];
#pragma unroll
      for (int q = 0; q < EPT; ++q) {
        run = run + (double)vs[q];
        if (ej + q == e) nv = run;
      }
    }
    const double hi = __shfl(nv, 1);
    if (lane == 0) {
      L.sidx[t2] = ok ? idx : -1;
      L.lo[t2] = nv;
      L.hi[t2] = hi;
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 93);
  double off = ex;
  for (int q = 0; q < wave; ++q) off = off + L.wt[q];
  if (!spec) {  // speculative draws: written only if some uniform takes the regular draws
    L.off[tid] = off;
    L.first[tid] = off + (double)v[0];  // the segment's first cumulative value (as the walk's)
    L.last[tid] = off + tot;            // its last, to within EPT roundings (far inside cum_tol)
  }
  unsigned long long redo = ~0ull;  // the uniforms the regular draws take
  if (spec) {
    // wave 0: the potential (every lane the same sums), then the check, one lane per uniform — the
    // speculative count is numpy's index when the exact threshold falls between the same two
    // cumulative values, neither within 4 cum_tol of it (the fold's check); one barrier
    if (wave == 0) {
      float y = 0.f;
      for (int b = 0; b < nsg; ++b) y = y + L.vb[b];
      if (m1 < n) {
        float sx = s_row[m1] * wv(a.w, m1);
        for (int o = m1 + 1; o < n; ++o) sx = __builtin_fmaf(s_row[o], wv(a.w, o), sx);
        y = y + sx;
      }
      if (lane == 0) {
        if (pot_out) *pot_out = y;
        L.pot = y;
      }
      bool good = false;
      if (lane < T) {
        const int idx = L.sidx[lane];
        if (idx >= 0) {
          const double rr = ut * (double)y;
          const double tol = cum_tol(a.exact, n, rr);
          const double lo = L.lo[lane], hi = L.hi[lane];
          good = tol >= 0.0 && (idx == 0 || (lo < rr && fabs(lo - rr) > 4.0 * tol)) &&
                 (idx == n || (!(hi < rr) && fabs(hi - rr) > 4.0 * tol));
          if (good) cand_out[lane] = min(n - 1, idx);
        }
      }
      const unsigned long long r = __ballot(lane < T && !good);
      if (lane == 0) L.redo = r;
    }
    __syncthreads();
    GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 96);
    redo = L.redo;
    if (redo == 0ull) {
      GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 97);
      GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 94);
      return;
    }
    L.off[tid] = off;
    L.first[tid] = off + (double)v[0];
    L.last[tid] = off + tot;
    __syncthreads();
  } else {
    if (tid == 0) {
      float y;
      if (c == 0) {
        y = a.st->pot;
      } else {
        y = 0.f;
        for (int b = 0; b < nsg; ++b) y = y + L.vb[b];
        if (m1 < n) {
          float sx = s_row[m1] * wv(a.w, m1);
          for (int o = m1 + 1; o < n; ++o) sx = __builtin_fmaf(s_row[o], wv(a.w, o), sx);
          y = y + sx;
        }
        if (pot_out) *pot_out = y;
      }
      L.pot = y;
    }
    __syncthreads();
    GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 96);
    if (c + 1 >= a.k) return;
  }
  // ---- draws for round c+1 if this trial wins: wave t2 takes uniform t2 over every segment (lane l:
  // segments l, l + 64, ...): whole segments below are counted by ballot, a segment that straddles
  // the threshold is walked by its lane — the owner's run, recomputed from LDS in the same order
  if (wave < T && ((redo >> wave) & 1ull)) {
    const int t2 = wave;
    const double pot = (double)L.pot;
    const double rr = readlane_f64(ut, t2) * pot;  // wave-uniform: a scalar read of lane t2
    const double tol = cum_tol(a.exact, n, rr);
    const bool strict = !(tol < 0.0);  // tol < 0 (GDD_KPP_EXACT=0, tests): every segment walks
    int full = 0, part = 0;
    bool amb = false;
    double fj[kBigThr / 64], lj[kBigThr / 64];  // every segment's first and last value, read at once
#pragma unroll
    for (int i = 0; i < kBigThr / 64; ++i) {
      fj[i] = L.first[lane + 64 * i];
      lj[i] = L.last[lane + 64 * i];
    }
#pragma unroll
    for (int i = 0; i < kBigThr / 64; ++i) {
      const int j = lane + 64 * i;
      const int ej = EPT * j;
      const bool live = ej < n;
      // a whole segment below, none of it within tol (the run only climbs)
      const bool below = live && ej + EPT <= n && strict && lj[i] < rr - 2.0 * tol;
      full += __popcll(__ballot(below));
      if (live && !below && !(strict && fj[i] > rr + tol)) {  // not wholly above either: walk it
        const double oj = L.off[j];
        {
          float vs[EPT];  // the segment's terms, every read issued before the run
#pragma unroll
          for (int q = 0; q < EPT; q += 4) {
            const float4 x = *reinterpret_cast<const float4*>(s_row + ej + q);
            vs[q] = x.x;
            vs[q + 1] = x.y;
            vs[q + 2] = x.z;
            vs[q + 3] = x.w;
          }
          if (a.w) {
#pragma unroll
            for (int q = 0; q < EPT; ++q) vs[q] = ej + q < n ? a.w[ej + q] * vs[q] : 0.f;
          }
          double run = oj;
#pragma unroll
          for (int q = 0; q < EPT; ++q) {
            run = run + (double)vs[q];
            if (ej + q < n) {
              part += run < rr;
              amb = amb || fabs(run - rr) <= tol;
            }
          }
        }
      }
    }
    if (part) atomicAdd(&L.part[t2], part);
    if (amb) L.amb[t2] = 1;
    if (lane == 0) L.cnt[t2] = EPT * full;
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 97);
  if (tid < T && ((redo >> tid) & 1ull)) {
    int64_t cnt = (int64_t)L.cnt[tid] + L.part[tid];
    if (L.amb[tid]) cnt = np_cumsum_search(s_row, a.w, n, ut * (double)L.pot);  // lane tid holds u_tid
    cand_out[tid] = min<int64_t>(n - 1, cnt);
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 94);
}

template <int EPT>
__global__ __launch_bounds__(kBigThr) void k_kpp1_big(Kpp1Args a, const float* __restrict__ D, int c) {
  extern __shared__ __attribute__((aligned(16))) float s_row[];  // kBigThr * EPT + kChainPad floats
  __shared__ BigLds L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int T = a.T;
  const int n = (int)a.n;
  const int t = blockIdx.x;
  const int cq = c & 1, pq = (c - 1) & 1;
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 90);
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 1), 95);
  big_fold_reset(L);
  // ---- trip 1, every load at once (lane q): round c-1's potential q, this slot's candidate if q
  // won, q's own candidate, round c+1's uniform q
  const double ut = (c + 1 < a.k && lane < T) ? a.uniforms[(int64_t)c * T + lane] : 0.0;
  const float* wrow = a.closest0;
  int64_t ct = 0;
  if (c >= 1) {
    const int Tp = c >= 2 ? T : 1;  // round 0 has one "trial": the first centre
    const int ql = min(lane, Tp - 1);
    const float pvl = a.potv[pq][ql];  // round 0 writes none: unused when Tp == 1
    const int64_t cwl = a.candw[pq][(int64_t)ql * T + t];
    const int64_t csl = a.candself[pq][ql];
    int bw = 0;  // np.argmin: first minimum, a NaN wins at once
    float best = __shfl(pvl, 0);
    for (int q = 1; q < Tp; ++q) {
      const float pt = __shfl(pvl, q);
      if (best == best && (pt < best || pt != pt)) {
        bw = q;
        best = pt;
      }
    }
    ct = __shfl(cwl, bw);
    const int64_t sw = __shfl(csl, bw);
    if (c >= 2) wrow = a.dist[pq] + (int64_t)bw * n;
    if (tid == 0) {
      a.candself[cq][t] = ct;
      if (c >= 2 && t == 0) a.indices[c - 1] = sw;
    }
  }
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 91);
  // ---- trip 2: the closest distances and the candidate's table row
  {
    constexpr int QC = EPT < 16 ? EPT : 16;  // loads in flight per thread and row (registers)
    float* orow = a.dist[cq] + (int64_t)t * n;
#pragma unroll
    for (int q0 = 0; q0 < EPT; q0 += QC) {
      float wi[QC], dd[QC];
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int e = min(tid + kBigThr * (q0 + q), n - 1);
        wi[q] = wrow[e];
        dd[q] = c >= 1 ? D[ct * n + e] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int e = tid + kBigThr * (q0 + q);
        const float f = c >= 1 ? np_minimum(wi[q], dd[q]) : wi[q];
        if (e < n && c >= 1) orow[e] = f;
        s_row[e] = e < n ? f : 0.f;
      }
    }
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kpp, (tid == 0 && t == 0 && c == a.k - 2), 92);
  big_fold<EPT>(a, c, t, ut, s_row, L, c >= 1 ? a.potv[cq] + t : nullptr, a.candw[cq] + (int64_t)t * T);
}

// ---- two rounds per launch over the table (4096 < n <= kBig1Max, T <= kPairMaxT; r06): k_kpp1_dm2's
// pairing with k_kpp1_big's 1024-thread fold. Workgroup w * T + t2 forms round c's trial w (the
// candidate's row against the winner's, as a round-c workgroup w would: same operands, same bits),
// folds it, takes the candidate round c+1's slot t2 draws if w wins, forms that row and folds it
// (candidates for round c+2). Workgroup w * T publishes round c's trial w. The next launch resolves
// both winners (k_kpp1_dm2's trip 1). A trailing odd round runs alone (pair == 0, T workgroups).
template <int EPT>
__global__ __launch_bounds__(kBigThr) void k_kpp1_big2(Kpp1Args a, const float* __restrict__ D, int c,
                                                        int lq, int pair) {
  extern __shared__ __attribute__((aligned(16))) float s_row[];  // kBigThr * EPT + kChainPad floats
  __shared__ BigLds L;
  __shared__ int64_t s_cand[kMaxTrials];
  const int tid = threadIdx.x, lane = tid & 63;
  const int T = a.T, pl = lq ^ 1, TT = T * T;
  const int n = (int)a.n;
  const int g = blockIdx.x;
  const int w = pair ? g / T : g;       // round c's trial this workgroup forms first
  const int t2 = pair ? g - w * T : 0;  // round c+1's trial (pair launches)
  big_fold_reset(L);
  // trip 1: the previous launch's potentials and this slot's candidates (as k_kpp1_dm2)
  const float* wrow;
  int64_t ct;
  if (c == 1) {
    wrow = a.closest0;
    ct = a.candw[0][w];  // round 0 (k_kpp1_big, one workgroup): the first centre's candidates
  } else {
    float pv[kPairMaxT];
#pragma unroll
    for (int q = 0; q < kPairMaxT; ++q) pv[q] = a.potv[pl][min(q, T - 1)];
    const float p2 = a.potv2[pl][min(lane, TT - 1)];
    const int64_t c2 = a.candw2[pl][(int64_t)min(lane, TT - 1) * T + w];
    const int64_t cs1 = a.candself[pl][min(lane, T - 1)];
    const int64_t cs2 = a.candself2[pl][min(lane, TT - 1)];
    int bw = 0;  // np.argmin: first minimum, a NaN wins at once
    float best = pv[0];
#pragma unroll
    for (int q = 1; q < kPairMaxT; ++q) {
      const float pt = pv[q];
      if (q < T && best == best && (pt < best || pt != pt)) {
        bw = q;
        best = pt;
      }
    }
    int bv = 0;
    float best2 = __shfl(p2, bw * T);
    for (int q = 1; q < T; ++q) {
      const float pt = __shfl(p2, bw * T + q);
      if (best2 == best2 && (pt < best2 || pt != pt)) {
        bv = q;
        best2 = pt;
      }
    }
    const int j = bw * T + bv;
    ct = __shfl(c2, j);
    wrow = a.dist2[pl] + (int64_t)j * n;
    const int64_t i1 = __shfl(cs1, bw), i2 = __shfl(cs2, j);
    if (g == 0 && tid == 0) {  // rows gathered after the rounds
      a.indices[c - 2] = i1;
      a.indices[c - 1] = i2;
    }
  }
  const double ut = (c + 1 < a.k && lane < T) ? a.uniforms[(int64_t)c * T + lane] : 0.0;
  if (tid == 0 && t2 == 0) a.candself[lq][w] = ct;
  // trip 2: the closest distances and the candidate's table row
  {
    constexpr int QC = EPT < 16 ? EPT : 16;
#pragma unroll
    for (int q0 = 0; q0 < EPT; q0 += QC) {
      float wi[QC], dd[QC];
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int e = min(tid + kBigThr * (q0 + q), n - 1);
        wi[q] = wrow[e];
        dd[q] = D[ct * n + e];
      }
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int e = tid + kBigThr * (q0 + q);
        s_row[e] = e < n ? np_minimum(wi[q], dd[q]) : 0.f;
      }
    }
  }
  __syncthreads();
  if (!pair) {  // the last round alone
    big_fold<EPT>(a, c, w, ut, s_row, L, a.potv[lq] + w, a.candw[lq] + (int64_t)w * T);
    return;
  }
  big_fold<EPT>(a, c, w, ut, s_row, L, t2 == 0 ? a.potv[lq] + w : nullptr, s_cand);
  __syncthreads();
  // trip 3: round c+1's candidate for slot t2 if w wins, its table row, and round c+2's uniforms
  // (requested here, not held in registers across the first fold)
  const int64_t c1 = s_cand[t2];
  const int j = w * T + t2;
  const double ut2 = (c + 2 < a.k && lane < T) ? a.uniforms[(int64_t)(c + 1) * T + lane] : 0.0;
  if (tid == 0) a.candself2[lq][j] = c1;
  big_fold_reset(L);
  {
    constexpr int QC = EPT < 16 ? EPT : 16;
    float* orow = a.dist2[lq] + (int64_t)j * n;
#pragma unroll
    for (int q0 = 0; q0 < EPT; q0 += QC) {
      float dd[QC];
#pragma unroll
      for (int q = 0; q < QC; ++q) dd[q] = D[c1 * n + min(tid + kBigThr * (q0 + q), n - 1)];
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int e = tid + kBigThr * (q0 + q);
        if (e < n) {  // the entry this thread stored in trip 2
          const float f = np_minimum(s_row[e], dd[q]);
          orow[e] = f;
          s_row[e] = f;
        }
      }
    }
  }
  __syncthreads();
  big_fold<EPT>(a, c + 1, t2, ut2, s_row, L, a.potv2[lq] + j, a.candw2[lq] + (int64_t)j * T);
}

// centres from their indices (fused rounds record only the index of each round's winner)
__global__ void k_kpp_gather_centres(int k, int dim, const float* __restrict__ X,
                                     const int64_t* __restrict__ indices, float* __restrict__ centers) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)k * dim) return;
  const int64_t c = e / dim, j = e - c * dim;
  centers[e] = X[indices[c] * dim + j];
}

// X^T (dim x n) for the single-block distance phase: coalesced loads
// X (n x dim) -> XT (dim x n) through 64 x 64 LDS tiles: rows read along the feature axis, columns
// written along the point axis, both coalesced (the element-wise form read one line per element)
constexpr int kXtTile = 64;
__global__ __launch_bounds__(256) void k_kpp_xt(int n, int dim, const float* __restrict__ X,
                                                float* __restrict__ XT) {
  __shared__ float tile[kXtTile][kXtTile + 1];
  const int i0 = blockIdx.x * kXtTile, j0 = blockIdx.y * kXtTile;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4 threads
  for (int r = ty; r < kXtTile; r += 4) {
    const int i = i0 + r, j = j0 + tx;
    tile[r][tx] = (i < n && j < dim) ? X[(int64_t)i * dim + j] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < kXtTile; r += 4) {
    const int j = j0 + r, i = i0 + tx;
    if (j < dim && i < n) XT[(int64_t)j * n + i] = tile[tx][r];
  }
}

// _euclidean_distances(C, X, squared=True) on its own (the distance of every round, exposed for
// callers and for the element-wise parity tests of every summation-order mode)
__global__ __launch_bounds__(kThr) void k_skl_sqdist(SklPlan p, const float* __restrict__ C,
                                                     const float* __restrict__ X,
                                                     float* __restrict__ out) {
  extern __shared__ double s_c[];
  __shared__ double s_cn;
  const int t = blockIdx.y;
  const float* ct = C + (int64_t)t * p.dim;
  for (int j = threadIdx.x; j < p.dim; j += kThr) s_c[j] = (double)ct[j];
  if (threadIdx.x == 0) s_cn = npy_sumsq_f64(ct, p.dim);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kThr + threadIdx.x;
  if (i >= p.n) return;
  const float* xi = X + i * p.dim;
  const double dot = skl_point_dot(p, s_c, xi, i, t);
  float f = (float)(((-2.0 * dot) + s_cn) + npy_sumsq_f64(xi, p.dim));
  out[(int64_t)t * p.n + i] = f < 0.f ? 0.f : f;
}

// ---- host side ------------------------------------------------------------------------------------

int64_t skl_batch_size(int64_t nx, int64_t ny, int dim) {  // pairwise.py _euclidean_distances_upcast
  double maxmem = (double)((nx + ny) * (int64_t)dim + nx * ny) / 10.0;
  if (maxmem < 1310720.0) maxmem = 1310720.0;
  const double tmp = 2.0 * dim;
  const int64_t b = (int64_t)((-tmp + std::sqrt(tmp * tmp + 4.0 * maxmem)) / 2.0);
  return b < 1 ? 1 : b;
}

// true when every element of a call with T candidate rows takes the plain chain
bool skl_all_seq(int64_t n, int T, int dim, int64_t B) {
  if (T == 1 || dim > 384) return false;
  int64_t ms[2] = {std::min(n, B), n > B ? n % B : 0};
  for (int64_t m : ms) {
    if (m <= 0) continue;
    if (m == 1) return false;
    const double mnk = (double)m * T * dim;
    if (mnk <= 1e6 && m * T <= 1200 && dim >= 32) return false;
    const bool threaded = kBlasThreads >= 2 && mnk >= 524288.0;
    if (!threaded && m > 192 && T >= 12 && (m & 7) != 0) return false;
  }
  return true;
}

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" int gdd_skl_sqdist(int n_rows, const float* C, int64_t n, int dim, const float* X,
                              float* out, gdd_stream_t stream) {
  GDD_REQUIRE(n_rows >= 1 && n > 0 && dim > 0 && dim <= 4096, "skl_sqdist: invalid shape");
  GDD_REQUIRE(n <= (int64_t)INT_MAX * kThr, "skl_sqdist: n too large");
  GDD_REQUIRE(C && X && out, "skl_sqdist: null pointer");
  SklPlan p{n, skl_batch_size(n_rows, n, dim), n_rows, dim, 0, 0};
  p.all_seq = skl_all_seq(n, n_rows, dim, p.B) ? 1 : 0;
  const size_t lds = sizeof(double) * (size_t)dim;
  k_skl_sqdist<<<dim3((unsigned)((n + kThr - 1) / kThr), (unsigned)n_rows), kThr, lds,
                 to_hip(stream)>>>(p, C, X, out);
  GDD_LAUNCHED();
  return GDD_OK;
}

size_t kpp_ws_bytes(int64_t n, int dim, int n_trials, int k);

// k (centres) sizes the fused rounds' arrival counters and gates the tables. This query bounds it
// by n (an upper bound for every k); gdd_kmeans_plusplus_ws_bytes_k sizes for the caller's k
extern "C" size_t gdd_kmeans_plusplus_ws_bytes(int64_t n, int dim, int n_trials) {
  return kpp_ws_bytes(n, dim, n_trials, (int)std::min<int64_t>(n, INT_MAX));
}

extern "C" size_t gdd_kmeans_plusplus_ws_bytes_k(int64_t n, int dim, int n_trials, int k) {
  return kpp_ws_bytes(n, dim, n_trials, std::max(1, k));
}

// the multi-block rounds read their distances from an n x n table when every distance is the plain
// chain (slot-independent) and the table is affordable: n <= kDmBigMax (4 GiB), dim <= kDmX, k >=
// kDmMinK. ML-1M users (6,040 x 64, k = 604), Ali-Display users (17,730 x 64, k = 1,773)
constexpr int64_t kDmBigMax = 32768;
// largest n for k_kpp1_big (one workgroup per trial): beyond ~16K points one CU's share of the row
// traffic (two rows in, one out per round) outweighs the per-block rounds' extra launch work
// (Ali-Display users, 17,730 points: 35.2 vs 23.5 us per round); GDD_FORCE=kpp_big1_max=N overrides
int64_t kpp_big1_max() {
  const int64_t v = (int64_t)forced_value("kpp_big1_max", 16384);
  return v < kBig1Max ? v : kBig1Max;
}
// the table costs n^2 dim fp64 fmas once (~0.45 ms at 6,040 x 64, i.e. ~5e12 fma/s) and saves each
// of the k - 1 rounds its distance phase (>= ~5 us per round beyond 4096 points): build it only when
// (k - 1) x 5 us covers n^2 dim / 5e12 s, i.e. (k - 1) 2.5e7 >= n^2 dim (k = 20 at
// n = 32,768 would build a 4 GiB table for 19 rounds). ML-1M users (6,040 x 64, k = 604): 1.5e10 >=
// 2.3e9; Ali-Display users (17,730 x 64, k = 1,773): 4.4e10 >= 2.0e10
bool kpp_table_pays(int64_t n, int dim, int k) {
  return (double)(k - 1) * 2.5e7 >= (double)n * (double)n * (double)std::max(dim, 1);
}
bool kpp_big_table(int64_t n, int dim, int T, int k) {
  if (n <= kBlk || n > kDmBigMax || dim > kDmX || T < 2 || k < kDmMinK) return false;
  if (forced("kpp_no_table")) return false;
  if (!kpp_table_pays(n, dim, k) && !forced("kpp_force_table")) return false;
  return skl_all_seq(n, T, dim, skl_batch_size(T, n, dim));
}
// the single-block table (n <= 4096, at most 64 MiB): built from kDmMinK centres on
bool kpp_small_table(int64_t n, int dim, int T, int k) {
  return n <= kBlk && dim <= kDmX && T >= 2 && k >= kDmMinK;
}
// the 1024-thread table rounds two per launch (k_kpp1_big2; T <= kPairMaxT, the 8-entry segments,
// n <= 8192: at 16 and 32 entries two folds in one kernel spill): workspace for the pairs
bool kpp_big_pairs(int64_t n, int dim, int T, int k) {
  return T <= kPairMaxT && n <= (int64_t)kBigThr * 8 && kpp_big_table(n, dim, T, k);
}

size_t kpp_ws_bytes(int64_t n, int dim, int n_trials, int k) {
  const size_t T = (size_t)std::max(n_trials, 1);
  const size_t nblk = (size_t)((n + kBlk - 1) / kBlk);
  size_t b = 0;
  b += align256(sizeof(KppState));
  b += align256(sizeof(double) * n);          // xsq
  b += align256(sizeof(float) * n);           // closest0
  b += align256(sizeof(double) * nblk);       // fsum0
  b += 2 * align256(sizeof(float) * n * T);   // dist ping-pong
  b += 2 * align256(sizeof(float) * nblk * T);    // vblk
  b += 2 * align256(sizeof(double) * nblk * T);   // fsum
  b += 2 * align256(sizeof(int64_t) * kMaxTrials);
  b += align256(sizeof(float) * 2);           // pot1
  b += align256(sizeof(int) * 2);             // winq
  b += 2 * align256(sizeof(float) * T);       // potv
  b += 2 * align256(sizeof(int64_t) * T * T); // candw
  b += 2 * align256(sizeof(int64_t) * T);     // candself
  b += 2 * align256(sizeof(int64_t) * T) + 2 * align256(sizeof(double) * T);  // candr, candn
  b += align256(sizeof(int) * 2) + align256(sizeof(unsigned) * (size_t)std::max(k, 1) * T);  // counters
  if (n <= kBlk || (int64_t)n * std::max(dim, 1) < INT_MAX)
    b += align256(sizeof(float) * n * (size_t)std::max(dim, 1));  // XT
  if (kpp_big_table(n, dim, (int)T, k))
    b += align256(sizeof(float) * n * n) + 2 * align256(sizeof(double) * n * T);  // table, block prefixes
  if (kpp_small_table(n, dim, (int)T, k)) b += align256(sizeof(float) * n * n);  // distance table
  if (kpp_small_table(n, dim, (int)T, k) || kpp_big_pairs(n, dim, (int)T, k))
    b += 2 * (align256(sizeof(float) * T * T * n) + align256(sizeof(float) * T * T) +
              align256(sizeof(int64_t) * T * T * T) + align256(sizeof(int64_t) * T * T));  // pair rounds
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
  GDD_REQUIRE(dim <= 4096, "kmeans++: dim=%d unsupported", dim);
  GDD_REQUIRE(n < (int64_t)INT_MAX * kBlk, "kmeans++: n=%lld too large", (long long)n);
  GDD_REQUIRE(first_id >= 0 && first_id < n, "kmeans++: first_id out of range");
  GDD_REQUIRE(X && centers && indices && ws && (k == 1 || uniforms), "kmeans++: null pointer");
  hipStream_t s = to_hip(stream);
  const int T = n_trials;
  const int nblk = (int)((n + kBlk - 1) / kBlk);
  Carver cv(ws, ws_bytes);
  KppArgs a{};
  KppState* st = cv.take<KppState>(1);
  double* xsq = cv.take<double>(n);
  float* closest0 = cv.take<float>(n);
  double* fsum0 = cv.take<double>(nblk);
  for (int q = 0; q < 2; ++q) a.dist[q] = cv.take<float>(n * (size_t)T);
  for (int q = 0; q < 2; ++q) a.vblk[q] = cv.take<float>((size_t)nblk * T);
  for (int q = 0; q < 2; ++q) a.fsum[q] = cv.take<double>((size_t)nblk * T);
  for (int q = 0; q < 2; ++q) a.cand[q] = cv.take<int64_t>(kMaxTrials);
  a.pot1 = cv.take<float>(2);
  a.winq = cv.take<int>(2);
  Kpp1Args b1;
  std::memset(&b1, 0, sizeof(b1));  // padding too: b1 is part of the chain's replay key
  for (int q = 0; q < 2; ++q) b1.potv[q] = cv.take<float>(T);
  for (int q = 0; q < 2; ++q) b1.candw[q] = cv.take<int64_t>((size_t)T * T);
  for (int q = 0; q < 2; ++q) b1.candself[q] = cv.take<int64_t>(T);
  for (int q = 0; q < 2; ++q) b1.candr[q] = cv.take<int64_t>(T);
  for (int q = 0; q < 2; ++q) b1.candn[q] = cv.take<double>(T);
  b1.win = cv.take<int>(2);
  b1.counter = cv.take<unsigned>((size_t)std::max(k, 1) * T);  // rounds c < k, trial t
  float* XT = (n <= kBlk || n * (int64_t)dim < INT_MAX) ? cv.take<float>((size_t)n * dim) : nullptr;
  float* Dbig = kpp_big_table(n, dim, T, k) ? cv.take<float>((size_t)n * n) : nullptr;
  // the per-block table rounds keep each round's block prefixes for the next round's count (r05)
  const bool big1 = n <= kpp_big1_max() && T >= 2 && !forced("kpp_no_big1");
  for (int q = 0; q < 2; ++q) a.pfx[q] = (Dbig && !big1) ? cv.take<double>((size_t)n * T) : nullptr;
  float* Dm = kpp_small_table(n, dim, T, k) ? cv.take<float>((size_t)n * n) : nullptr;
  const bool pairs_big = Dbig && big1 && kpp_big_pairs(n, dim, T, k);
  if (Dm || pairs_big) {
    for (int q = 0; q < 2; ++q) {
      b1.dist2[q] = cv.take<float>((size_t)T * T * n);
      b1.potv2[q] = cv.take<float>((size_t)T * T);
      b1.candw2[q] = cv.take<int64_t>((size_t)T * T * T);
      b1.candself2[q] = cv.take<int64_t>((size_t)T * T);
    }
  }
  if (!cv.ok()) return fail(GDD_E_WORKSPACE, "kmeans++: workspace too small");
  a.n = n;
  a.m1 = n & ~3ll;
  a.dim = dim;
  a.T = T;
  a.nblk = nblk;
  a.nsg = (int)((a.m1 + kBlk - 1) / kBlk);
  a.X = X;
  a.XT = n > kBlk ? XT : nullptr;  // the single-block path keeps its own copy in b1
  a.w = w;
  a.xsq = xsq;
  a.closest0 = closest0;
  a.fsum0 = fsum0;
  a.uniforms = uniforms;
  a.st = st;
  a.centers = centers;
  a.indices = indices;
  a.plan = SklPlan{n, skl_batch_size(T, n, dim), T, dim, 0, 0};
  a.plan.all_seq = skl_all_seq(n, T, dim, a.plan.B) ? 1 : 0;
  {  // cum_tol's mode (diagnostic): GDD_KPP_EXACT=0 never replays (tests only), 2 always replays
    const char* ex = getenv("GDD_KPP_EXACT");
    a.exact = ex ? atoi(ex) : 1;
  }
  const SklPlan p1{n, skl_batch_size(1, n, dim), 1, dim, 0, 0};
  const size_t lds = sizeof(double) * (size_t)dim + sizeof(float) * (kBlk + kChainPad);  // + chain read-ahead
  const bool seq = a.plan.all_seq != 0;
  const bool single = nblk == 1 && T >= 2 && (!seq || XT);
  if (lds > 65536) {
    const void* fns[] = {(const void*)k_kpp_init, (const void*)k_kpp_round<true>,
                         (const void*)k_kpp_round<false>};
    for (const void* f : fns)
      GDD_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  if (a.XT) {
    k_kpp_xt<<<dim3((unsigned)((n + kXtTile - 1) / kXtTile), (unsigned)((dim + kXtTile - 1) / kXtTile)), 256, 0,
               s>>>((int)n, dim, X, XT);
    GDD_LAUNCHED();
  }
  k_kpp_init<<<nblk, kThr, lds, s>>>(a, p1, first_id, xsq, closest0, fsum0);
  GDD_LAUNCHED();
  if (w == nullptr && n >= (int64_t)kFirstSteps * 64 * 2) {  // large n, unit weights: staged chains
    const size_t fl = sizeof(float) * 2 * kFirstSteps * 64;
    GDD_HIP(hipFuncSetAttribute((const void*)k_kpp_first_big, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl));
    k_kpp_first_big<<<1, 1024, fl, s>>>(n, dim, X, closest0, first_id, st, centers, indices);
  } else {
    k_kpp_first<<<1, 64, 0, s>>>(n, dim, X, w, closest0, first_id, st, centers, indices);
  }
  GDD_LAUNCHED();
  if (k == 1) return GDD_OK;
  if (single) {
    b1.n = n;
    b1.m1 = a.m1;
    b1.dim = dim;
    b1.T = T;
    b1.k = k;
    b1.X = X;
    b1.XT = XT;
    b1.w = w;
    b1.xsq = xsq;
    b1.closest0 = closest0;
    b1.st = st;
    b1.uniforms = uniforms;
    for (int q = 0; q < 2; ++q) b1.dist[q] = a.dist[q];
    b1.centers = centers;
    b1.indices = indices;
    b1.plan = a.plan;
    b1.exact = a.exact;
    if (seq) {
      k_kpp_xt<<<dim3((unsigned)((n + kXtTile - 1) / kXtTile), (unsigned)((dim + kXtTile - 1) / kXtTile)), 256, 0,
               s>>>((int)n, dim, X, XT);
      GDD_LAUNCHED();
    }
    const size_t lds1 = sizeof(double) * (size_t)T * std::max(dim, 48);
    if (lds1 > 65536)
      for (const void* f : {(const void*)k_kpp1_dist<true>, (const void*)k_kpp1_dist<false>})
        GDD_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
    const dim3 g1((unsigned)((n + kPts - 1) / kPts), (unsigned)(((T + kTg - 1) / kTg + 3) / 4));
    k_kpp1_pick<<<1, kThr, 0, s>>>(b1, 0);
    GDD_LAUNCHED();
    // the distance table pays once the rounds it saves (~3 us each) cover its one-off build
    if (seq && Dm && k >= kDmMinK && !forced("kpp_no_table")) {
      if (const int rc = launch_kpp_dmat(n, dim, X, XT, xsq, Dm, s)) return rc;
      if (T <= kPairMaxT && !forced("kpp_single_round")) {
        // two rounds per launch (a trailing odd round alone). The chain's arguments are fixed by
        // (b1, Dm, k): it is replayed as one recorded graph (replay_or_run) — every launch then
        // starts ~1 us sooner after the previous one
        // the pair's two folds overlapped (kpp1_fold_pair); GDD_FORCE=kpp_pair_serial: one after the other
        const int overlap = forced("kpp_pair_serial") ? 0 : 1;
        auto chain = [&](hipStream_t cs) -> int {
          int lq = 1, pair = 0;
          for (int c = 1; c < k; c += 2) {
            lq = ((c - 1) / 2 + 1) & 1;
            pair = c + 1 < k ? 1 : 0;
            const unsigned grid = (unsigned)(pair ? T * T : T);
            k_kpp1_dm2<<<grid, 256, 0, cs>>>(b1, Dm, c, lq, pair, overlap);
            GDD_LAUNCHED();
          }
          k_kpp1_final2<<<1, 64, 0, cs>>>(b1, k - 1, lq, pair);
          GDD_LAUNCHED();
          if (k > 2) {
            k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, cs>>>(
                k, dim, X, indices, centers);
            GDD_LAUNCHED();
          }
          return GDD_OK;
        };
        struct {
          Kpp1Args b1;
          const float* Dm;
          int k, overlap;
        } key;
        std::memset(&key, 0, sizeof(key));
        key.b1 = b1;
        key.Dm = Dm;
        key.k = k;
        key.overlap = overlap;
        return replay_or_run("kpp_pair_chain", &key, sizeof(key), s, chain);
      }
      for (int c = 1; c < k; ++c) {
        k_kpp1_dm<<<(unsigned)T, 256, 0, s>>>(b1, Dm, c);
        GDD_LAUNCHED();
      }
      k_kpp1_final<<<1, 64, 0, s>>>(b1, k - 1);
      GDD_LAUNCHED();
      if (k > 2) {
        k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, s>>>(k, dim, X, indices,
                                                                                         centers);
        GDD_LAUNCHED();
      }
      return GDD_OK;
    }
    const dim3 gf((unsigned)((n + kFPts - 1) / kFPts), (unsigned)T);
    if (dim <= kMaxDimF && gf.x * gf.y <= 256 && !forced("kpp_two_launch")) {
      // one launch per round: distances, then each trial's last workgroup folds it (no fences)
      GDD_HIP(hipMemsetAsync(b1.counter, 0, sizeof(unsigned) * (size_t)k * T, s));
      for (int c = 1; c < k; ++c) {
        if (seq)
          k_kpp1_fused<true><<<gf, 256, 0, s>>>(b1, c);
        else
          k_kpp1_fused<false><<<gf, 256, 0, s>>>(b1, c);
        GDD_LAUNCHED();
      }
      k_kpp1_final<<<1, 64, 0, s>>>(b1, k - 1);
      GDD_LAUNCHED();
      if (k > 2) {  // rounds 1..k-2 recorded indices only (round 0's and k-1's rows are written)
        k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, s>>>(k, dim, X, indices,
                                                                                         centers);
        GDD_LAUNCHED();
      }
      return GDD_OK;
    }
    for (int c = 1; c < k; ++c) {
      if (seq)
        k_kpp1_dist<true><<<g1, 256, lds1, s>>>(b1, c);
      else
        k_kpp1_dist<false><<<g1, 256, lds1, s>>>(b1, c);
      GDD_LAUNCHED();
      k_kpp1_pick<<<T, kThr, 0, s>>>(b1, c);
      GDD_LAUNCHED();
    }
    k_kpp1_final<<<1, 64, 0, s>>>(b1, k - 1);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  const size_t lds_split = sizeof(double) * (size_t)T * dim + sizeof(float) * (size_t)T * kBlk;
  // the split path has one workgroup per 4096-point block: it pays only when there are enough
  // blocks to fill the chip (products' 2.45M points: 598 blocks). With few blocks the per-(block,
  // trial) rounds win (6,040 points: 22 vs 69 us per round; 40,000: 47 vs 84).
  const bool split = seq && a.XT && T >= 2 && T <= kSplitMaxT && lds_split <= 150 * 1024 &&
                     nblk >= kSplitMinBlocks && !forced("kpp_no_split");
  if (split) {
    void (*dists)(KppArgs, int) = nullptr;
    switch (T) {
      case 2: dists = k_kpp_dists<2>; break;
      case 3: dists = k_kpp_dists<3>; break;
      case 4: dists = k_kpp_dists<4>; break;
      case 5: dists = k_kpp_dists<5>; break;
      case 6: dists = k_kpp_dists<6>; break;
      case 7: dists = k_kpp_dists<7>; break;
      default: dists = k_kpp_dists<8>; break;
    }
    GDD_HIP(hipFuncSetAttribute((const void*)dists, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_split));
    for (int c = 1; c < k; ++c) {
      k_kpp_round<true, true><<<dim3(1, T), kThr, lds, s>>>(a, c);   // fold, winner, candidates
      GDD_LAUNCHED();
      dists<<<nblk, kThr, lds_split, s>>>(a, c);                    // every trial's distances
      GDD_LAUNCHED();
    }
    k_kpp_final<<<1, kThr, 0, s>>>(a, k - 1);
    GDD_LAUNCHED();
    k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, s>>>(k, dim, X, indices,
                                                                                     centers);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  if (Dbig && seq && a.XT) {  // the distances once per fit (~n^2 dim fp64 fmas), then table rounds
    if (const int rc = launch_kpp_dmat(n, dim, X, a.XT, xsq, Dbig, s)) return rc;
    a.D = Dbig;
    if (big1) {
      // one 1024-thread workgroup per trial (k_kpp1_big); GDD_FORCE=kpp_no_big1 keeps the per-block rounds
      b1.n = n;
      b1.m1 = a.m1;
      b1.dim = dim;
      b1.T = T;
      b1.k = k;
      b1.X = X;
      b1.w = w;
      b1.xsq = xsq;
      b1.closest0 = closest0;
      b1.st = st;
      b1.uniforms = uniforms;
      for (int q = 0; q < 2; ++q) b1.dist[q] = a.dist[q];
      b1.centers = centers;
      b1.indices = indices;
      b1.plan = a.plan;
      b1.exact = a.exact;
      void (*big)(Kpp1Args, const float*, int) = nullptr;
      int ept = 0;
      if (n <= (int64_t)kBigThr * 8) {
        big = k_kpp1_big<8>;
        ept = 8;
      } else if (n <= (int64_t)kBigThr * 16) {
        big = k_kpp1_big<16>;
        ept = 16;
      } else {
        big = k_kpp1_big<32>;
        ept = 32;
      }
      const size_t lds_big = sizeof(float) * ((size_t)kBigThr * ept + kChainPad);
      GDD_HIP(hipFuncSetAttribute((const void*)big, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_big));
      big<<<1, kBigThr, lds_big, s>>>(b1, Dbig, 0);  // round 1's candidates from the first centre
      GDD_LAUNCHED();
      if (pairs_big && !forced("kpp_single_round")) {  // two rounds per launch (r06)
        void (*big2)(Kpp1Args, const float*, int, int, int) = k_kpp1_big2<8>;  // n <= 8192: ept == 8
        GDD_HIP(hipFuncSetAttribute((const void*)big2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_big));
        int lq = 1, pair = 0;
        for (int c = 1; c < k; c += 2) {
          lq = ((c - 1) / 2 + 1) & 1;
          pair = c + 1 < k ? 1 : 0;
          big2<<<(unsigned)(pair ? T * T : T), kBigThr, lds_big, s>>>(b1, Dbig, c, lq, pair);
          GDD_LAUNCHED();
        }
        k_kpp1_final2<<<1, 64, 0, s>>>(b1, k - 1, lq, pair);
        GDD_LAUNCHED();
        if (k > 2) {
          k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, s>>>(k, dim, X, indices,
                                                                                           centers);
          GDD_LAUNCHED();
        }
        return GDD_OK;
      }
      for (int c = 1; c < k; ++c) {
        big<<<(unsigned)T, kBigThr, lds_big, s>>>(b1, Dbig, c);
        GDD_LAUNCHED();
      }
      k_kpp1_final<<<1, 64, 0, s>>>(b1, k - 1);
      GDD_LAUNCHED();
      if (k > 2) {
        k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, s>>>(k, dim, X, indices,
                                                                                         centers);
        GDD_LAUNCHED();
      }
      return GDD_OK;
    }
  }
  for (int c = 1; c < k; ++c) {
    if (seq)
      k_kpp_round<true><<<dim3(nblk, T), kThr, lds, s>>>(a, c);
    else
      k_kpp_round<false><<<dim3(nblk, T), kThr, lds, s>>>(a, c);
    GDD_LAUNCHED();
    if (T == 1) {
      k_kpp_pot1<<<1, 64, 0, s>>>(n, a.dist[c & 1], w, a.pot1 + (c & 1));
      GDD_LAUNCHED();
    }
  }
  k_kpp_final<<<1, kThr, 0, s>>>(a, k - 1);
  GDD_LAUNCHED();
  k_kpp_gather_centres<<<(unsigned)(((int64_t)k * dim + 255) / 256), 256, 0, s>>>(k, dim, X, indices,
                                                                                   centers);
  GDD_LAUNCHED();
  return GDD_OK;
}
