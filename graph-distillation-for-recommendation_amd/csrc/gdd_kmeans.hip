// gdd_kmeans.hip — (a5/a6/a8) the WCSS k-means building blocks, scikit-learn 1.7.2 semantics.
//
// What is restated (sklearn/cluster/…):
//   row norms        utils/extmath.py:76  np.einsum("ij,ij->i") — numpy SSE3 float32 kernel order
//   assignment       _k_means_lloyd.pyx:172-213 — ||C||² then sgemm(-2·X·Cᵀ, beta=1), row argmin
//                    with strict '<' (first index wins). OpenBLAS sgemm computes every element as a
//                    k-ordered fp32 fma chain finished by fma(-2, acc, ||c||²) (verified bit-exact in
//                    oracle/ tests); v_mfma_f32_32x32x2_f32 is exactly such a chain, so the MFMA
//                    distance tile reproduces it bit for bit.
//   sample distance  _k_means_common.pyx:26-48 _euclidean_dense_dense (4-term groups, no fma)
//   inertia          _k_means_common.pyx:92-121 (one OpenMP thread: sequential fp32)
//   minibatch update _k_means_minibatch.pyx:59-108
//   Lloyd M-step     _k_means_lloyd.pyx:111-160 (one OpenMP thread: sequential per cluster)
//   average / shift  _k_means_common.pyx:215-251
// Loop control, RNG draws and rare branches (reassignment, relocation) live in the host layer.
#include <algorithm>
#include <mutex>
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "gdd_common.hpp"
#include "gdd_devrng.hpp"

namespace gdd {
GDD_STAMP_TABLE(kmeans)
namespace {

using floatx16 = __attribute__((ext_vector_type(16))) float;

// ---------------------------------------------------------------------------------------------
// row norms in numpy einsum float32 SSE order (sum_of_products_contig_contig_outstride0_two):
// 4 lanes; per 16-element block acc_l = x[12+l]^2 + acc_l, then x[8+l]^2, x[4+l]^2, x[l]^2
// (separate mul and add); 4-element zero-padded tail blocks; result (a0+a1)+(a2+a3).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float npy_sumsq(const float* __restrict__ x, int dim) {
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int j = 0;
  for (; dim - j >= 16; j += 16) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      float t = x[j + 12 + l] * x[j + 12 + l] + a[l];
      t = x[j + 8 + l] * x[j + 8 + l] + t;
      t = x[j + 4 + l] * x[j + 4 + l] + t;
      a[l] = x[j + l] * x[j + l] + t;
    }
  }
  for (; j < dim; j += 4) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      float v = (j + l < dim) ? x[j + l] : 0.f;
      a[l] = v * v + a[l];
    }
  }
  return (a[0] + a[1]) + (a[2] + a[3]);
}

// accumulator l of npy_sumsq (the same per-lane arithmetic): four lanes form the norm together
__device__ __forceinline__ float npy_sumsq_acc(const float* __restrict__ x, int dim, int l) {
  float a = 0.f;
  int j = 0;
  for (; dim - j >= 16; j += 16) {
    float t = x[j + 12 + l] * x[j + 12 + l] + a;
    t = x[j + 8 + l] * x[j + 8 + l] + t;
    t = x[j + 4 + l] * x[j + 4 + l] + t;
    a = x[j + l] * x[j + l] + t;
  }
  for (; j < dim; j += 4) {
    const float v = (j + l < dim) ? x[j + l] : 0.f;
    a = v * v + a;
  }
  return a;
}

__global__ void k_row_norms(int64_t n, int dim, const float* __restrict__ X, float* __restrict__ out,
                            const int32_t* __restrict__ stop, int step_i) {
  if (stopped(stop, step_i)) return;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = npy_sumsq(X + i * dim, dim);
}

// skl_sqdist with a 16-byte-aligned global `a`, dim % 4 == 0: the row is fetched as float4, eight
// at a time ahead of the ordered group sums (same arithmetic, same order)
__device__ __forceinline__ float skl_sqdist_v4(const float* __restrict__ a, const float* __restrict__ b,
                                               int dim) {
  const float4* a4 = reinterpret_cast<const float4*>(a);
  const int q = dim >> 2;
  float r = 0.f;
  for (int j0 = 0; j0 < q; j0 += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = j0 + u < q ? a4[j0 + u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (j0 + u < q) {
        const float* bb = b + 4 * (j0 + u);
        const float d0 = v[u].x - bb[0], d1 = v[u].y - bb[1], d2 = v[u].z - bb[2], d3 = v[u].w - bb[3];
        r = r + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
      }
    }
  }
  return r;
}

// ---------------------------------------------------------------------------------------------
// assignment: MFMA distance tiles + lexicographic (distance, index) argmin
// ---------------------------------------------------------------------------------------------
// (d, c) packed so that unsigned 64-bit order == lexicographic order on (d as float, c)
__device__ __forceinline__ unsigned long long pack_key(float d, int c) {
  // -0.0 + 0.0 = +0.0: both zeros get one key, so they tie on the index as sklearn's `<` does
  unsigned u = __float_as_uint(d + 0.0f);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned)c;
}

// lexicographic (distance, index) minimum of one lane's 16 tile entries against its running best:
// lane l holds centres cb + (r&3) + 8(r>>2) + 4(l>>5), increasing with r, so a strict float `<`
// keeps the lowest index among equal distances; the result is packed once
__device__ __forceinline__ unsigned long long tile_best(const floatx16& acc, const float* Nw, int cb,
                                                       int kh, int k, unsigned long long best) {
  float nv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) nv[r] = Nw[(r & 3) + 8 * (r >> 2) + 4 * kh];
  float bd = 0.f;
  int bi = -1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ci = cb + (r & 3) + 8 * (r >> 2) + 4 * kh;
    const float d = __builtin_fmaf(-2.f, acc[r], nv[r]);
    if (ci < k && (bi < 0 || d < bd)) {
      bd = d;
      bi = ci;
    }
  }
  if (bi < 0) return best;
  const unsigned long long key = pack_key(bd, bi);
  return key < best ? key : best;
}

// tile_best plus the second-smallest distance value (any other centre), for the Lloyd loop's
// distance bounds: `bd` is the value packed in `best`, `sec` the smallest value among the rest
__device__ __forceinline__ void tile_top2(const floatx16& acc, const float* Nw, int cb, int kh, int k,
                                          unsigned long long& best, float& bd, float& sec) {
  float nv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) nv[r] = Nw[(r & 3) + 8 * (r >> 2) + 4 * kh];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ci = cb + (r & 3) + 8 * (r >> 2) + 4 * kh;
    const float d = __builtin_fmaf(-2.f, acc[r], nv[r]);
    if (ci < k) {
      const unsigned long long key = pack_key(d, ci);
      if (key < best) {
        sec = fminf(sec, bd);
        best = key;
        bd = d;
      } else {
        sec = fminf(sec, d);
      }
    }
  }
}

__global__ void k_fill_u64(int64_t n, unsigned long long* p, unsigned long long v,
                           const int32_t* __restrict__ stop, int step_i) {
  if (stopped(stop, step_i)) return;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// One block = WAVES waves x 32 points; blockIdx.y = a chunk of `cch` centers. A wave computes
// 32x32 tiles D[center][point] = sum_t C[center][t] * X[point][t] with chained
// v_mfma_f32_32x32x2_f32 (lanes 0-31 feed feature 2s, lanes 32-63 feature 2s+1 of each step, so the
// chain visits features in order 0,1,2,...). Lane l then holds point l&31 against the 16 centers
// (r&3)+8(r>>2)+4(l>>5), r = 0..15, and keeps a running lexicographic minimum; the two half-waves
// merge with one xor-shuffle and the block's result enters keys[] through a 64-bit atomicMin.
// Rows are zero-padded to dimp (a multiple of 16 features, so the step loop runs in unguarded groups
// of 8 whose LDS operands are all read before the group's MFMAs), two centre tiles advance together
// (two independent accumulator chains), and LDS rows use an odd stride (dimp+1 floats) so the 32 rows
// read by one ds_read_b32 hit 32 banks. Zero features add exact zeros to the fma chain (a -0/+0
// difference in a dot product is erased by pack_key), so the distances stay bit-exact.
template <int WAVES, bool VEC>
__global__ __launch_bounds__(64 * WAVES) void k_assign(int64_t n, int dim, int dimp,
                                                       const float* __restrict__ X,
                                                       const int64_t* __restrict__ rows, int k,
                                                       const float* __restrict__ C,
                                                       const float* __restrict__ cn2, int cch,
                                                       unsigned long long* __restrict__ keys,
                                                       const int32_t* __restrict__ stop, int step_i) {
  if (stopped(stop, step_i)) return;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kPts = 32 * WAVES;
  const int S = dimp + 1;
  const int c0 = blockIdx.y * cch;
  const int nc = min(k, c0 + cch) - c0;
  const int ncp = (nc + 31) & ~31;
  float* Cl = lds;
  float* Pl = Cl + (size_t)ncp * S;
  float* Nl = Pl + (size_t)kPts * S;
  const int tid = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kPts;
  if (VEC) {  // float4 rows (dim % 4 == 0, 16-byte aligned X and C)
    const int q = dim >> 2;
    for (int idx = tid; idx < kPts * q; idx += blockDim.x) {
      const int r = idx / q, c4 = idx - r * q;
      const int64_t pi = p0 + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pi < n) v = *reinterpret_cast<const float4*>(X + (rows ? rows[pi] : pi) * dim + 4 * c4);
      float* d = Pl + r * S + 4 * c4;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    for (int idx = tid; idx < ncp * q; idx += blockDim.x) {
      const int r = idx / q, c4 = idx - r * q;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < nc) v = *reinterpret_cast<const float4*>(C + (int64_t)(c0 + r) * dim + 4 * c4);
      float* d = Cl + r * S + 4 * c4;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
  } else {
    for (int idx = tid; idx < kPts * dim; idx += blockDim.x) {
      const int r = idx / dim, c = idx - r * dim;
      const int64_t pi = p0 + r;
      Pl[r * S + c] = pi < n ? X[(rows ? rows[pi] : pi) * dim + c] : 0.f;
    }
    for (int idx = tid; idx < ncp * dim; idx += blockDim.x) {
      const int r = idx / dim, c = idx - r * dim;
      Cl[r * S + c] = r < nc ? C[(int64_t)(c0 + r) * dim + c] : 0.f;
    }
  }
  const int pad = dimp - dim;
  if (pad > 0) {
    for (int idx = tid; idx < (ncp + kPts) * pad; idx += blockDim.x) {
      const int r = idx / pad, c = dim + (idx - r * pad);
      Cl[r * S + c] = 0.f;  // rows ncp.. are the point rows (Pl follows Cl with the same stride)
    }
  }
  for (int idx = tid; idx < ncp; idx += blockDim.x) Nl[idx] = idx < nc ? cn2[c0 + idx] : 0.f;
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63;
  const int kh = lane >> 5;
  const float* bp = Pl + (wave * 32 + (lane & 31)) * S + kh;
  const int ns = dimp >> 1;  // a multiple of 8
  unsigned long long best = ~0ull;
  for (int ct = 0; ct < ncp; ct += 64) {
    const bool two = ct + 32 < ncp;
    const float* ap0 = Cl + (ct + (lane & 31)) * S + kh;
    const float* ap1 = two ? ap0 + 32 * S : ap0;
    floatx16 acc0 = {}, acc1 = {};
    for (int s0 = 0; s0 < ns; s0 += 8) {
      float a0[8], a1[8], bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = 2 * (s0 + u);
        a0[u] = ap0[o];
        a1[u] = ap1[o];
        bv[u] = bp[o];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], bv[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], bv[u], acc1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ci = ct + (r & 3) + 8 * (r >> 2) + 4 * kh;
      if (ci < nc) {
        const float d = __builtin_fmaf(-2.f, acc0[r], Nl[ci]);
        const unsigned long long key = pack_key(d, c0 + ci);
        best = key < best ? key : best;
      }
      const int cj = ci + 32;
      if (two && cj < nc) {
        const float d = __builtin_fmaf(-2.f, acc1[r], Nl[cj]);
        const unsigned long long key = pack_key(d, c0 + cj);
        best = key < best ? key : best;
      }
    }
  }
  const unsigned long long other = __shfl_xor(best, 32);
  best = other < best ? other : best;
  if (lane < 32) {
    const int64_t pi = p0 + wave * 32 + lane;
    if (pi < n && best != ~0ull) atomicMin(keys + pi, best);
  }
}

// Persistent variant for dimp <= 96 (every config's k-means input): a block stages its centre
// chunk ONCE, then walks point tiles t = blockIdx.x, +gridDim.x, ... While a tile's MFMA tiles run,
// the next tile's rows are already in flight into registers (two threads per point row, features
// h, h+2, ... with clamped, unconditional loads), so the staging hides behind the MFMAs instead of
// preceding them in every block. Same tiles, order and key merge as k_assign (bit-exact); with a
// single centre chunk (gridDim.y == 1) the keys are stored, not atomically merged.
constexpr int kPersistMaxHalf = 48;  // ceil(96 / 2) row elements per thread
template <int NT>  // centre tiles (independent accumulator chains) per pass; 2 (the tail pass: 1)
__global__ __launch_bounds__(256) void k_assign_persist(int64_t n, int dim, int dimp,
                                                       const float* __restrict__ X,
                                                       const int64_t* __restrict__ rows, int k,
                                                       const float* __restrict__ C,
                                                       const float* __restrict__ cn2, int cch,
                                                       unsigned long long* __restrict__ keys,
                                                       const int32_t* __restrict__ stop, int step_i) {
  if (stopped(stop, step_i)) return;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kPts = 128;
  const int S = dimp + 1;
  const int c0 = blockIdx.y * cch;
  const int nc = min(k, c0 + cch) - c0;
  const int ncp = (nc + 31) & ~31;
  float* Cl = lds;
  float* Pl = Cl + (size_t)ncp * S;
  float* Nl = Pl + (size_t)kPts * S;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < ncp * dimp; idx += blockDim.x) {
    const int r = idx / dimp, c = idx - r * dimp;
    Cl[r * S + c] = (r < nc && c < dim) ? C[(int64_t)(c0 + r) * dim + c] : 0.f;
  }
  for (int idx = tid; idx < ncp; idx += blockDim.x) Nl[idx] = idx < nc ? cn2[c0 + idx] : 0.f;
  const int64_t ntiles = (n + kPts - 1) / kPts;
  const int pr = tid >> 1, ph = tid & 1;  // staging: point row pr, features ph, ph+2, ...
  const int half = (dim + 1 - ph) >> 1;   // this thread's element count
  float v[kPersistMaxHalf];
  auto fetch = [&](int64_t t) {
    const int64_t pi = t * kPts + pr;
    const bool ok = pi < n;
    const float* xr = X + (ok ? (rows ? rows[pi] : pi) : 0) * dim;
#pragma unroll
    for (int j = 0; j < kPersistMaxHalf; ++j) v[j] = xr[min(ph + 2 * j, dim - 1)];
    if (!ok) {
#pragma unroll
      for (int j = 0; j < kPersistMaxHalf; ++j) v[j] = 0.f;
    }
  };
  int64_t t = blockIdx.x;
  if (t < ntiles) fetch(t);
  const int wave = tid >> 6, lane = tid & 63;
  const int kh = lane >> 5;
  const float* bp = Pl + (wave * 32 + (lane & 31)) * S + kh;
  const int ns = dimp >> 1;
  for (; t < ntiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's MFMAs are done with Pl
#pragma unroll
    for (int j = 0; j < kPersistMaxHalf; ++j) {
      const int c = ph + 2 * j;
      if (c < dimp) Pl[pr * S + c] = (j < half) ? v[j] : 0.f;
    }
    __syncthreads();
    if (t + gridDim.x < ntiles) fetch(t + gridDim.x);  // in flight during this tile's MFMAs
    unsigned long long best = ~0ull;
    // one pass: M centre tiles from ct, M independent accumulator chains, then the per-tile scans
    auto pass = [&](auto M_, int ct) {
      constexpr int M = decltype(M_)::value;
      const float* ap[M];
#pragma unroll
      for (int q = 0; q < M; ++q) ap[q] = Cl + (ct + 32 * q + (lane & 31)) * S + kh;
      floatx16 acc[M];
#pragma unroll
      for (int q = 0; q < M; ++q) acc[q] = floatx16{};
      for (int s0 = 0; s0 < ns; s0 += 8) {
        float a[M][8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int o = 2 * (s0 + u);
#pragma unroll
          for (int q = 0; q < M; ++q) a[q][u] = ap[q][o];
          bv[u] = bp[o];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
          for (int q = 0; q < M; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][u], bv[u], acc[q], 0, 0, 0);
        }
      }
      // per tile: a strict float `<` scan (lowest index among equal distances), one packed key
#pragma unroll
      for (int q = 0; q < M; ++q)
        best = tile_best(acc[q], Nl + ct + 32 * q, c0 + ct + 32 * q, kh, c0 + nc, best);
    };
    int ct = 0;
    for (; ct + 32 * NT <= ncp; ct += 32 * NT) pass(std::integral_constant<int, NT>(), ct);
    if (ct < ncp) pass(std::integral_constant<int, 1>(), ct);  // an odd last tile runs alone
    const unsigned long long other = __shfl_xor(best, 32);
    best = other < best ? other : best;
    if (lane < 32) {
      const int64_t pi = t * kPts + wave * 32 + lane;
      if (pi < n && best != ~0ull) {
        if (gridDim.y == 1)
          keys[pi] = best;
        else
          atomicMin(keys + pi, best);
      }
    }
  }
}

// Wave-tile variant (default for dimp <= 96): the same tiles, chains, order and key merge as
// k_assign_persist (bit-exact), but every wave walks 32-point tiles of its own (t = global wave id,
// + all waves) through its own LDS slot, so the tile loop has no workgroup barrier: the waves of a
// SIMD drift apart and one wave's MFMA chain covers another's staging and argmin epilogue (the
// persistent form synchronised all its waves twice per 128-point tile). With contiguous rows (no
// row list) a tile is 32 consecutive rows = one contiguous run of 32*dim floats, fetched as float4
// (coalesced, 16-byte aligned for any dim since 32*dim*4 is a multiple of 16) and scattered into the
// zero-padded LDS rows; with a row list, two lanes per row as in k_assign_persist. The centre chunk
// is staged once per block; W waves per block share it (W = 12 at the products shape: 3 per SIMD).
// F: float4 per lane of a contiguous tile (6: dim <= 48); a row-list tile uses 4F elements per lane
// (two lanes per row). Wider rows (dim 49..96) keep k_assign_persist: their prefetched tile would
// spill at three waves per SIMD.
// TOP2 (one centre chunk, gridDim.y == 1): also sec[i] = the second-smallest distance of row i;
// n_dev (nullable): the row count is read on the device (a row list built by an earlier kernel).
// ROW4 (row lists only): X is a zero-padded copy with 16-byte aligned rows of ldx floats (the Lloyd
// run's M-step copy, r05); each lane of a row's pair reads F 16-byte pieces instead of 4F floats
template <int NT, int W, bool CONTIG, int F, bool TOP2 = false, bool ROW4 = false>
__global__ __launch_bounds__(64 * W) void k_assign_waves(int64_t n, int dim, int dimp,
                                                         const float* __restrict__ X,
                                                         const int64_t* __restrict__ rows, int k,
                                                         const float* __restrict__ C,
                                                         const float* __restrict__ cn2, int cch,
                                                         unsigned long long* __restrict__ keys,
                                                         const int32_t* __restrict__ stop, int step_i,
                                                         float* __restrict__ sec = nullptr,
                                                         const int64_t* __restrict__ n_dev = nullptr,
                                                         int ldx = 0) {
  if (stopped(stop, step_i)) return;
  if (n_dev) n = *n_dev;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int S = dimp + 1;
  const int c0 = blockIdx.y * cch;
  const int nc = min(k, c0 + cch) - c0;
  const int ncp = (nc + 31) & ~31;
  float* Cl = lds;
  float* Nl = Cl + (size_t)ncp * S;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  float* Pw = Nl + ncp + (size_t)wave * 32 * S;
  for (int idx = tid; idx < ncp * dimp; idx += blockDim.x) {
    const int r = idx / dimp, c = idx - r * dimp;
    Cl[r * S + c] = (r < nc && c < dim) ? C[(int64_t)(c0 + r) * dim + c] : 0.f;
  }
  for (int idx = tid; idx < ncp; idx += blockDim.x) Nl[idx] = idx < nc ? cn2[c0 + idx] : 0.f;
  // the padding columns of the wave's rows stay zero (the scatter below writes columns < dim only)
  for (int idx = lane; idx < 32 * S; idx += 64) Pw[idx] = 0.f;
  __syncthreads();  // the only workgroup barrier: the centre chunk is read-only from here on
  const int64_t ntiles = (n + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * W;
  int64_t t = (int64_t)blockIdx.x * W + wave;
  const int tot = 32 * dim;  // floats per full tile
  const float rdim = 1.0f / (float)dim;
  float4 v4[CONTIG ? F : 1];
  float v[CONTIG ? 1 : 4 * F];
  const int pr = lane >> 1, ph = lane & 1;
  const int half = (dim + 1 - ph) >> 1;
  auto fetch = [&](int64_t tt) {
    if constexpr (CONTIG) {
      const int64_t base = tt * 32 * (int64_t)dim;
      const int64_t lim = n * (int64_t)dim - base;  // floats left in X from the tile start
      const float* xt = X + base;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        const int e = 4 * (lane + 64 * j);
        if (e + 3 < tot && e + 3 < lim) {
          v4[j] = *reinterpret_cast<const float4*>(xt + e);
        } else {  // the tile's (or X's) ragged end
          float q[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) q[u] = (e + u < tot && e + u < lim) ? xt[e + u] : 0.f;
          v4[j] = make_float4(q[0], q[1], q[2], q[3]);
        }
      }
    } else if constexpr (ROW4) {
      const int64_t pi = tt * 32 + pr;
      const bool ok = pi < n;
      const float4* xr4 = reinterpret_cast<const float4*>(X + (ok ? (rows ? rows[pi] : pi) : 0) * (int64_t)ldx);
#pragma unroll
      for (int j = 0; j < F; ++j) {
        const int q = 2 * j + ph;
        const float4 w = (ok && 4 * q < dim) ? xr4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        v[4 * j] = w.x;
        v[4 * j + 1] = w.y;
        v[4 * j + 2] = w.z;
        v[4 * j + 3] = w.w;
      }
    } else {
      const int64_t pi = tt * 32 + pr;
      const bool ok = pi < n;
      const float* xr = X + (ok ? (rows ? rows[pi] : pi) : 0) * dim;
#pragma unroll
      for (int j = 0; j < 4 * F; ++j) v[j] = xr[min(ph + 2 * j, dim - 1)];
      if (!ok) {
#pragma unroll
        for (int j = 0; j < 4 * F; ++j) v[j] = 0.f;
      }
    }
  };
  auto stage = [&]() {
    if constexpr (CONTIG) {
#pragma unroll
      for (int j = 0; j < F; ++j) {
        const int e = 4 * (lane + 64 * j);
        const float q[4] = {v4[j].x, v4[j].y, v4[j].z, v4[j].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ee = e + u;
          if (ee < tot) {
            // ee / dim by the fp32 reciprocal (ee < 3072: exact operands), corrected by one step
            int r = (int)((float)ee * rdim);
            int c = ee - r * dim;
            if (c < 0) {
              --r;
              c += dim;
            } else if (c >= dim) {
              ++r;
              c -= dim;
            }
            Pw[r * S + c] = q[u];
          }
        }
      }
    } else if constexpr (ROW4) {
#pragma unroll
      for (int j = 0; j < F; ++j) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = 4 * (2 * j + ph) + u;
          if (c < dim) Pw[pr * S + c] = v[4 * j + u];
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4 * F; ++j) {
        const int c = ph + 2 * j;
        if (c < dim) Pw[pr * S + c] = (j < half) ? v[j] : 0.f;
      }
    }
  };
  if (t < ntiles) fetch(t);
  const int kh = lane >> 5;
  const float* bp = Pw + (lane & 31) * S + kh;
  const int ns = dimp >> 1;
  for (; t < ntiles; t += stride) {
    // this wave's previous tile is done with its slot (the wave's LDS reads return in order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    stage();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (t + stride < ntiles) fetch(t + stride);  // in flight during this tile's MFMAs
    unsigned long long best = ~0ull;
    float bd = __builtin_inff(), sd = __builtin_inff();
    auto pass = [&](auto M_, int ct) {
      constexpr int M = decltype(M_)::value;
      const float* ap[M];
#pragma unroll
      for (int q = 0; q < M; ++q) ap[q] = Cl + (ct + 32 * q + (lane & 31)) * S + kh;
      floatx16 acc[M];
#pragma unroll
      for (int q = 0; q < M; ++q) acc[q] = floatx16{};
      // groups of eight K-steps, then the rest (r05: rows padded to an even width, not to 16 —
      // the padding's zero steps only ever added +0 to the chains)
      const int nfull = ns & ~7;
      for (int s0 = 0; s0 < nfull; s0 += 8) {
        float a[M][8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int o = 2 * (s0 + u);
#pragma unroll
          for (int q = 0; q < M; ++q) a[q][u] = ap[q][o];
          bv[u] = bp[o];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
          for (int q = 0; q < M; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][u], bv[u], acc[q], 0, 0, 0);
        }
      }
      if (nfull < ns) {
        const int rem = ns - nfull;
        float a[M][8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int o = 2 * (nfull + min(u, rem - 1));
#pragma unroll
          for (int q = 0; q < M; ++q) a[q][u] = ap[q][o];
          bv[u] = bp[o];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (u < rem) {
#pragma unroll
            for (int q = 0; q < M; ++q)
              acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][u], bv[u], acc[q], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < M; ++q) {
        if constexpr (TOP2)
          tile_top2(acc[q], Nl + ct + 32 * q, c0 + ct + 32 * q, kh, c0 + nc, best, bd, sd);
        else
          best = tile_best(acc[q], Nl + ct + 32 * q, c0 + ct + 32 * q, kh, c0 + nc, best);
      }
    };
    int ct = 0;
    for (; ct + 32 * NT <= ncp; ct += 32 * NT) pass(std::integral_constant<int, NT>(), ct);
    if (ct < ncp) pass(std::integral_constant<int, 1>(), ct);
    const unsigned long long other = __shfl_xor(best, 32);
    if constexpr (TOP2) {  // merge the two half-waves' (best, second) pairs
      const float obd = __shfl_xor(bd, 32), osd = __shfl_xor(sd, 32);
      sd = fminf(fminf(sd, osd), other < best ? bd : obd);
    }
    best = other < best ? other : best;
    if (lane < 32) {
      const int64_t pi = t * 32 + lane;
      if (pi < n && best != ~0ull) {
        if (gridDim.y == 1)
          keys[pi] = best;
        else
          atomicMin(keys + pi, best);
        if constexpr (TOP2) sec[pi] = sd;
      }
    }
  }
}

// ---- bf16 distance variant (configs 2, 3 and 5 carry fp32 and bf16 distances) ----
// Same block shape and key merge as k_assign, but the X and C tiles are rounded to bf16 (nearest
// even) in LDS and each 32x32 tile is a chain of v_mfma_f32_32x32x16_bf16 (fp32 accumulate). The
// distance is fma(-2, <x, c>_bf16, ||c||^2) with the fp32 numpy-order norms, the label the first
// minimum. Not bit-compatible with sklearn (the dot products round their operands): labels agree
// except where two centres' fp32 distances lie within the bf16 rounding of the dot products.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__host__ __device__ inline size_t assign_bf16_lds(int waves, int dimp16, int cch) {
  const int SB = dimp16 + 8;  // bf16 per LDS row: 16-byte aligned rows, shifted by 16 B per row
  const int ncp = (cch + 31) & ~31;
  return sizeof(uint16_t) * ((size_t)ncp * SB + (size_t)32 * waves * SB) + sizeof(float) * ncp + 16;
}

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_assign_bf16(int64_t n, int dim, int dimp16,
                                                            const float* __restrict__ X,
                                                            const int64_t* __restrict__ rows, int k,
                                                            const float* __restrict__ C,
                                                            const float* __restrict__ cn2, int cch,
                                                            unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
  constexpr int kPts = 32 * WAVES;
  const int SB = dimp16 + 8;
  const int c0 = blockIdx.y * cch;
  const int nc = min(k, c0 + cch) - c0;
  const int ncp = (nc + 31) & ~31;
  uint16_t* Cl = lds16;
  uint16_t* Pl = Cl + (size_t)ncp * SB;
  float* Nl = reinterpret_cast<float*>(Pl + (size_t)kPts * SB);
  const int tid = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kPts;
  for (int idx = tid; idx < kPts * dimp16; idx += blockDim.x) {
    const int r = idx / dimp16, c = idx - r * dimp16;
    const int64_t pi = p0 + r;
    float v = 0.f;
    if (pi < n && c < dim) {
      const int64_t src = rows ? rows[pi] : pi;
      v = X[src * dim + c];
    }
    Pl[r * SB + c] = f32_to_bf16_rne(v);
  }
  for (int idx = tid; idx < ncp * dimp16; idx += blockDim.x) {
    const int r = idx / dimp16, c = idx - r * dimp16;
    Cl[r * SB + c] = f32_to_bf16_rne((r < nc && c < dim) ? C[(int64_t)(c0 + r) * dim + c] : 0.f);
  }
  for (int idx = tid; idx < ncp; idx += blockDim.x) Nl[idx] = idx < nc ? cn2[c0 + idx] : 0.f;
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  const int kh = lane >> 5;
  const uint16_t* bp = Pl + (wave * 32 + (lane & 31)) * SB + 8 * kh;
  unsigned long long best = ~0ull;
  for (int ct = 0; ct < ncp; ct += 32) {
    const uint16_t* ap = Cl + (ct + (lane & 31)) * SB + 8 * kh;
    floatx16 acc = {};
    for (int s16 = 0; s16 < dimp16; s16 += 16) {
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(ap + s16);
      const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(bp + s16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ci = ct + (r & 3) + 8 * (r >> 2) + 4 * kh;
      if (ci < nc) {
        const float d = __builtin_fmaf(-2.f, acc[r], Nl[ci]);
        const unsigned long long key = pack_key(d, c0 + ci);
        best = key < best ? key : best;
      }
    }
  }
  const unsigned long long other = __shfl_xor(best, 32);
  best = other < best ? other : best;
  if (lane < 32) {
    const int64_t pi = p0 + wave * 32 + lane;
    if (pi < n && best != ~0ull) atomicMin(keys + pi, best);
  }
}

__global__ void k_assign_finalize(int64_t n, int dim, const float* __restrict__ X,
                                  const int64_t* __restrict__ rows, const float* __restrict__ C,
                                  const unsigned long long* __restrict__ keys,
                                  int32_t* __restrict__ labels, float* __restrict__ sq_dist,
                                  const int32_t* __restrict__ stop, int step_i) {
  if (stopped(stop, step_i)) return;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long key = keys[i];
  const int lab = (key == ~0ull) ? 0 : (int)(unsigned)(key & 0xffffffffull);
  labels[i] = lab;
  if (sq_dist) {
    const int64_t src = rows ? rows[i] : i;
    sq_dist[i] = skl_sqdist(X + src * dim, C + (int64_t)lab * dim, dim);
  }
}


// ---- persistent bf16 full pass (predict(precision="bf16")) ------------------
// HBM-bound design (X is read once: 460 MB at products, ~77 us at the achievable 6 TB/s; the bf16
// MFMAs are ~18 us of that shape's work and the argmin epilogue ~28 us of VALU):
//   * the centres' v_mfma_f32_32x32x16_bf16 A-fragments ([centre tile][k-step][lane] x 8 bf16) and
//     their fp32 norms (+inf past k) are built ONCE by k_bf16_frags into the workspace; every block
//     copies them into LDS with coalesced 16-byte loads (building them per block from scalar loads of
//     C cost more than the tiles at small n);
//   * each wave walks 32-point tiles: a tile's rows are one contiguous span of X, read as float4 two
//     tiles ahead of the compute (two register sets, the loop unrolled by two), scattered into a
//     wave-private LDS slot with a row stride padded to a multiple of 16 floats (the pad columns stay
//     zero), so each lane's B-fragment (one point's 8 features per k-step) is two ds_read_b128;
//   * point = column of the 32x32 product, so the argmin over each centre tile is lane-local; one
//     lane^32 merge at the end. d = fma(-2, <x, c>_bf16, ||c||^2), first minimum; labels written
//     directly (no key buffer, no atomics); sq_dist (nullable) is the exact fp32
//     _euclidean_dense_dense to the chosen centre.
// The grid is the resident set (blocks per CU from the occupancy query x CUs), so no block waits for a
// second wave of the grid.
typedef float floatx4_t __attribute__((ext_vector_type(4)));

__host__ __device__ inline int bf16p_stride(int dim) { return (dim + 15) & ~15; }

__host__ __device__ inline size_t assign_bf16p_lds(int ktiles, int nsteps, int dim) {
  return (size_t)ktiles * nsteps * 64 * 16 + (size_t)ktiles * 32 * sizeof(float) +
         (size_t)4 * 32 * bf16p_stride(dim) * sizeof(float);
}

__host__ __device__ inline size_t bf16_frag_bytes(int ktiles, int nsteps) {
  return (size_t)ktiles * nsteps * 64 * 16 + (size_t)ktiles * 32 * sizeof(float);
}

// the A-fragments of every centre tile and the norms (+inf past k), once per call
__global__ void k_bf16_frags(int dim, int nsteps, int ktiles, int k, const float* __restrict__ C,
                             const float* __restrict__ cn2, bf16x8_t* __restrict__ frags,
                             float* __restrict__ cn_out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < ktiles * nsteps * 64) {
    const int l = e & 63, rest = e >> 6;
    const int st = rest % nsteps, ct = rest / nsteps;
    const int c = ct * 32 + (l & 31), f0 = 16 * st + 8 * (l >> 5);
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)((c < k && f0 + j < dim) ? C[(int64_t)c * dim + f0 + j] : 0.f);
    frags[e] = v;
  }
  if (e < ktiles * 32) cn_out[e] = e < k ? cn2[e] : __builtin_inff();
}

template <int PER>  // float4 loads per lane per 32-point tile: PER >= ceil(32 * dim / 256)
__global__ __launch_bounds__(256) void k_assign_bf16p(int64_t n, int dim, int nsteps, int ktiles,
                                                      const float* __restrict__ X, int k,
                                                      const bf16x8_t* __restrict__ frags,
                                                      const float* __restrict__ cn_in,
                                                      const float* __restrict__ C,
                                                      int32_t* __restrict__ labels,
                                                      float* __restrict__ sq_dist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16x8_t* Af = reinterpret_cast<bf16x8_t*>(smem);
  float* Cn = reinterpret_cast<float*>(smem + (size_t)ktiles * nsteps * 64 * 16);
  float* Pt = Cn + ktiles * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int SP = bf16p_stride(dim);
  {  // the prebuilt fragments and norms: coalesced 16-byte copies
    const int nfr = ktiles * nsteps * 64;
    for (int e = tid; e < nfr; e += 256) Af[e] = frags[e];
    for (int c = tid; c < ktiles * 32; c += 256) Cn[c] = cn_in[c];
  }
  float* my = Pt + wave * 32 * SP;
  for (int e = lane; e < 32 * SP; e += 64) my[e] = 0.f;  // pad columns stay zero
  __syncthreads();
  const int nf4 = 8 * dim;  // float4 per full tile (32 rows x dim floats)
  const int64_t ntiles = (n + 31) / 32, nfull = n / 32;
  const int64_t step = (int64_t)gridDim.x * 4;
  auto fetch = [&](int64_t tt, float4 (&v)[PER]) {
    if (tt >= nfull) return;  // the partial last tile is read scalar in stage()
    const float4* src = reinterpret_cast<const float4*>(X + tt * 32 * dim);
#pragma unroll
    for (int q = 0; q < PER; ++q) v[q] = src[min(lane + 64 * q, nf4 - 1)];
  };
  auto stage = [&](int64_t tt, const float4 (&v)[PER]) {
    if (tt < nfull) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int e4 = lane + 64 * q;
        if (e4 < nf4) {
          const float w4[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int e = 4 * e4 + j, row = e / dim;
            my[row * SP + (e - row * dim)] = w4[j];
          }
        }
      }
    } else {
      const int64_t rows = n - tt * 32;
      for (int e = lane; e < 32 * dim; e += 64) {
        const int row = e / dim;
        my[row * SP + (e - row * dim)] = e < rows * dim ? X[tt * 32 * dim + e] : 0.f;
      }
    }
  };
  auto compute = [&](int64_t tt) {
    bf16x8_t b[8];
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      if (st < nsteps) {
        const floatx4_t lo = *reinterpret_cast<const floatx4_t*>(my + r * SP + 16 * st + 8 * h);
        const floatx4_t hi = *reinterpret_cast<const floatx4_t*>(my + r * SP + 16 * st + 8 * h + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          b[st][j] = (__bf16)lo[j];
          b[st][4 + j] = (__bf16)hi[j];
        }
      }
    }
    float bestd = __builtin_inff();
    int bestc = 0;
    for (int ct = 0; ct < ktiles; ++ct) {
      floatx16 acc = {};
#pragma unroll
      for (int st = 0; st < 8; ++st)
        if (st < nsteps) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Af[(ct * nsteps + st) * 64 + lane], b[st], acc, 0, 0, 0);
      const floatx4_t* cp = reinterpret_cast<const floatx4_t*>(Cn + ct * 32 + 4 * h);
      floatx4_t cn[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) cn[g] = cp[2 * g];  // rows 8g + 4h .. +3
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float d = __builtin_fmaf(-2.f, acc[reg], cn[reg >> 2][reg & 3]);
        if (d < bestd) {
          bestd = d;
          bestc = ct * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        }
      }
    }
    const float od = __shfl_xor(bestd, 32);
    const int oc = __shfl_xor(bestc, 32);
    if (od < bestd || (od == bestd && oc < bestc)) {
      bestd = od;
      bestc = oc;
    }
    const int64_t p = tt * 32 + r;
    if (h == 0 && p < n) {
      labels[p] = bestc;
      if (sq_dist) sq_dist[p] = skl_sqdist(my + r * SP, C + (int64_t)bestc * dim, dim);
    }
  };
  float4 va[PER], vb[PER];
  int64_t t = (int64_t)blockIdx.x * 4 + wave;
  fetch(t, va);
  fetch(t + step, vb);
  while (t < ntiles) {
    stage(t, va);
    fetch(t + 2 * step, va);  // two tiles in flight while this one computes
    compute(t);
    t += step;
    if (t >= ntiles) break;
    stage(t, vb);
    fetch(t + 2 * step, vb);
    compute(t);
    t += step;
  }
}

// ---------------------------------------------------------------------------------------------
// small batches (minibatch steps): one block of WAVES waves per 32 points. Wave w owns centre tiles
// w, w+WAVES, ...; it stages its tile (and, without cached norms, their numpy-order norms) in LDS,
// runs the MFMA chain with all operands preloaded from LDS into registers (the chain then issues
// back to back), and the block merges the per-wave minima in LDS — no atomics, no key buffer,
// labels and sq_dist written directly. Latency plan (one launch ≈ two dependent memory trips):
// the row indices and every wave's first centre tile are requested together; the point rows
// follow once the indices land. VEC: dim % 4 == 0 and 16-byte aligned X/C (float4 loads).
// ---------------------------------------------------------------------------------------------
// LDS: points, WAVES centre tiles, their norms, the per-wave minima, the distance terms
__host__ __device__ inline size_t assign_small_lds(int waves, int dim) {
  const int dimp = (dim + 1) & ~1, S = dimp + 1;
  const int nt = (dim >> 2) + (dim & 3);
  return sizeof(float) * ((size_t)(32 + 32 * waves) * S + 32 * waves) + 16 +
         sizeof(unsigned long long) * 32 * waves + sizeof(float) * 32 * (size_t)nt;
}

// rows [0, nrows) of a 32-row tile, row r at src(r) (dim floats), into LDS rows of stride S;
// rows >= nrows and the pad column (dimp > dim) are zero. Up to 8 loads per lane are issued
// before the first LDS store.
template <bool VEC, int U = 8, class RowPtr>
__device__ __forceinline__ void stage_rows32(float* __restrict__ dst, int S, RowPtr src, int nrows,
                                             int dim, int dimp, int lane, int nlanes) {
  if (VEC) {
    const int q = dim >> 2;  // float4 per row
    const int total = 32 * q;
    for (int base = 0; base < total; base += nlanes * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = base + u * nlanes + lane;
        const int r = idx / q;
        v[u] = (idx < total && r < nrows)
                   ? *reinterpret_cast<const float4*>(src(r) + 4 * (idx - r * q))
                   : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = base + u * nlanes + lane;
        if (idx < total) {
          const int r = idx / q;
          float* d = dst + r * S + 4 * (idx - r * q);
          d[0] = v[u].x;
          d[1] = v[u].y;
          d[2] = v[u].z;
          d[3] = v[u].w;
        }
      }
    }
  } else {
    const int total = 32 * dim;
    for (int base = 0; base < total; base += nlanes * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = base + u * nlanes + lane;
        const int r = idx / dim;
        v[u] = (idx < total && r < nrows) ? src(r)[idx - r * dim] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = base + u * nlanes + lane;
        if (idx < total) {
          const int r = idx / dim;
          dst[r * S + (idx - r * dim)] = v[u];
        }
      }
    }
  }
  if (dimp > dim)
    for (int r = lane; r < 32; r += nlanes) dst[r * S + dim] = 0.f;
}

// D = C_tile · P_tileᵀ over the feature axis in order 0,1,2,... as ONE fma chain per element
// (bit-identical to the OpenBLAS sgemm element). Operands of up to P chain steps are read from
// LDS into registers first, so the MFMAs issue back to back instead of one LDS latency apart.
template <int P>
__device__ __forceinline__ floatx16 mfma_chain(const float* __restrict__ ap,
                                               const float* __restrict__ bp, int dimp) {
  floatx16 acc = {};
  for (int s0 = 0; s0 < dimp; s0 += 2 * P) {
    const int ns = min(P, (dimp - s0) >> 1);
    float av[P], bv[P];
#pragma unroll
    for (int u = 0; u < P; ++u)
      if (u < ns) {
        av[u] = ap[s0 + 2 * u];
        bv[u] = bp[s0 + 2 * u];
      }
#pragma unroll
    for (int u = 0; u < P; ++u)
      if (u < ns) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
  return acc;
}

template <int WAVES, bool VEC>
__global__ __launch_bounds__(64 * WAVES) void k_assign_small(
    int64_t n, int dim, int dimp, const float* __restrict__ X, const int64_t* __restrict__ rows,
    int k, const float* __restrict__ C, const float* __restrict__ cn2, int32_t* __restrict__ labels,
    float* __restrict__ sq_dist, const int32_t* __restrict__ stop, int step_i, RngNext rn) {
  if (stopped(stop, step_i)) return;
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 0);
  constexpr int kTileU = WAVES == 16 ? 6 : 8;  // 16 waves: 128 VGPRs per lane, fewer loads in flight
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (rn.rows && blockIdx.x == gridDim.x - 1) {
    // extra workgroup: the next step's batch indices (randint(0, n, b)) from the device MT state,
    // concurrently with this step's assignment
    mt_randint_from(rn.in, reinterpret_cast<uint32_t*>(lds), 0, rn.n, rn.bs, rn.rows, rn.out);
    return;
  }
  const int S = dimp + 1;
  float* Pl = lds;                                 // 32 points x S
  float* Cl = Pl + 32 * S;                         // WAVES x 32 centres x S (consecutive tiles)
  float* Nl = Cl + (size_t)WAVES * 32 * S;         // WAVES x 32 norms
  unsigned long long* Kl =
      reinterpret_cast<unsigned long long*>(((uintptr_t)(Nl + 32 * WAVES) + 15) & ~uintptr_t(15));
  __shared__ int64_t s_rows[32];
  __shared__ int s_lab[32];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t p0 = (int64_t)blockIdx.x * 32;
  const int np = (int)min<int64_t>(32, n - p0);
  // trip 1: the batch's row indices and this wave's first centre tile, requested together
  int64_t my_row = 0;
  if (tid < 32 && tid < np) my_row = rows ? rows[p0 + tid] : p0 + tid;
  float* Cw = Cl + (size_t)wave * 32 * S;
  float* Nw = Nl + wave * 32;
  if (wave * 32 < k) {
    const float* Cb = C + (int64_t)wave * 32 * dim;
    stage_rows32<VEC, kTileU>(Cw, S, [&](int r) { return Cb + (int64_t)r * dim; }, k - wave * 32,
                              dim, dimp, lane, 64);
    if (cn2 && lane < 32) Nw[lane] = (wave * 32 + lane < k) ? cn2[wave * 32 + lane] : 0.f;
  }
  if (tid < 32) s_rows[tid] = my_row;
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 2);
  // trip 2: the point rows
  stage_rows32<VEC, 4>(Pl, S, [&](int r) { return X + s_rows[r] * dim; }, np, dim, dimp, tid,
                       64 * WAVES);
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 3);
  const int kh = lane >> 5;
  const float* bp = Pl + (lane & 31) * S + kh;
  const float* ap = Cw + (lane & 31) * S + kh;
  unsigned long long best = ~0ull;
  for (int cb = wave * 32; cb < k; cb += 32 * WAVES) {
    if (cb != wave * 32) {  // k > 32*WAVES: later tiles of this wave (after its reads of the last)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const float* Cb = C + (int64_t)cb * dim;
      stage_rows32<VEC, kTileU>(Cw, S, [&](int r) { return Cb + (int64_t)r * dim; }, k - cb, dim,
                                dimp, lane, 64);
      if (cn2 && lane < 32) Nw[lane] = (cb + lane < k) ? cn2[cb + lane] : 0.f;
    }
    if (!cn2) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < 32) Nw[lane] = (cb + lane < k) ? npy_sumsq(Cw + lane * S, dim) : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const floatx16 acc = mfma_chain<WAVES == 16 ? 10 : 16>(ap, bp, dimp);
    GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 5);
    best = tile_best(acc, Nw, cb, kh, k, best);
  }
  const unsigned long long other = __shfl_xor(best, 32);
  best = other < best ? other : best;
  if (lane < 32) Kl[wave * 32 + lane] = best;
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 13);
  if (wave == 0 && lane < 32) {
    unsigned long long b = Kl[lane];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) {
      const unsigned long long o = Kl[w * 32 + lane];
      b = o < b ? o : b;
    }
    const int lab = (b == ~0ull) ? 0 : (int)(unsigned)(b & 0xffffffffull);
    s_lab[lane] = lab;
    if (lane < np) labels[p0 + lane] = lab;
  }
  if (!sq_dist) return;
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 14);
  // ||x - c_label||^2 in the _euclidean_dense_dense order: the terms (4-element groups, then the
  // remainder elements) are formed by the whole block, then each point's lane adds them in order.
  // With k <= 32*WAVES every centre row is still in LDS (tile c/32 row c%32 = Cl + c*S).
  const bool resident = k <= 32 * WAVES;
  const int ng = dim >> 2, nt = ng + (dim & 3);
  float* tbuf = reinterpret_cast<float*>(Kl + 32 * WAVES);
  for (int idx = tid; idx < 32 * nt; idx += blockDim.x) {
    const int p = idx / nt, t = idx - p * nt;
    if (p >= np) continue;
    const float* x = Pl + p * S;
    const float* c = resident ? Cl + (size_t)s_lab[p] * S : C + (int64_t)s_lab[p] * dim;
    float v;
    if (t < ng) {
      const int j = 4 * t;
      const float d0 = x[j] - c[j], d1 = x[j + 1] - c[j + 1], d2 = x[j + 2] - c[j + 2],
                  d3 = x[j + 3] - c[j + 3];
      v = ((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3;
    } else {
      const int j = 4 * ng + (t - ng);
      const float d0 = x[j] - c[j];
      v = d0 * d0;
    }
    tbuf[idx] = v;
  }
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 15);
  if (tid < np) {
    float r = 0.f;
    for (int t = 0; t < nt; ++t) r = r + tbuf[tid * nt + t];
    sq_dist[p0 + tid] = r;
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 16);
}

// Sequential fp32 fold acc = ((acc + b[0]) + b[1]) + ... of m LDS floats by ONE lane. The next
// eight float4 reads are issued before the current 32 dependent adds, so the add chain (not the
// LDS latency) bounds it. b must be 16-byte aligned.
__device__ __forceinline__ float fold_seq_lds(const float* __restrict__ b, int m, float acc) {
  // two register buffers of 8 float4, used alternately (no copies): each loads while the other's
  // 32 terms are added
  const float4* b4 = reinterpret_cast<const float4*>(b);
  const int g = m >> 5;
  int q = 0;
  if (g > 0) {
    float4 A[8], B[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) A[u] = b4[u];
    for (; q + 2 <= g; q += 2) {
#pragma unroll
      for (int u = 0; u < 8; ++u) B[u] = b4[(q + 1) * 8 + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc = acc + A[u].x;
        acc = acc + A[u].y;
        acc = acc + A[u].z;
        acc = acc + A[u].w;
      }
      if (q + 2 < g) {
#pragma unroll
        for (int u = 0; u < 8; ++u) A[u] = b4[(q + 2) * 8 + u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc = acc + B[u].x;
        acc = acc + B[u].y;
        acc = acc + B[u].z;
        acc = acc + B[u].w;
      }
    }
    if (q < g) {  // one group left, in A
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc = acc + A[u].x;
        acc = acc + A[u].y;
        acc = acc + A[u].z;
        acc = acc + A[u].w;
      }
    }
  }
  for (int t = g << 5; t < m; ++t) acc = acc + b[t];
  return acc;
}

// ---------------------------------------------------------------------------------------------
// MiniBatchKMeans early stopping on the device: _mini_batch_convergence (_kmeans.py:1960-2027)
// with Python-float (fp64, unfused) arithmetic, so the host need not read the inertia every step.
// ---------------------------------------------------------------------------------------------
struct MBState {
  double ewa, ewa_min;
  int32_t stop_at;       // offset 16: 0 while running, s+1 once the test fired at step s
  int32_t has_ewa, has_min, no_improvement;
  int32_t handoff;       // offset 32: s+1 once step s's reassignment needs the host (np.argsort branch)
  int32_t pad[3];
};

// one thread; st->stop_at is published with an agent-scope atomic store (read by sibling blocks).
// The state is read into registers first (MbConv) — the tail block requests it before its inertia
// fold, so the test after the fold costs no dependent memory trips; only this thread writes it.
struct MbConv {
  double ewa, ewa_min;
  int32_t stop_at, has_ewa, has_min, no_improvement;
};

__device__ __forceinline__ MbConv mb_conv_load(const MBState* __restrict__ st) {
  MbConv c;
  c.stop_at = __hip_atomic_load(&st->stop_at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  c.ewa = st->ewa;
  c.ewa_min = st->ewa_min;
  c.has_ewa = st->has_ewa;
  c.has_min = st->has_min;
  c.no_improvement = st->no_improvement;
  return c;
}

__device__ void mb_converge_from(MbConv c, int step_i, int64_t bs, int64_t n, int max_no_improvement,
                                 float inertia, MBState* __restrict__ st) {
  if (c.stop_at) return;
  const double bi = (double)inertia / (double)bs;
  if (step_i == 0) return;  // the first step's inertia is the init's
  if (!c.has_ewa) {
    c.ewa = bi;
    c.has_ewa = 1;
  } else {
    double a = (double)bs * 2.0 / (double)(n + 1);
    a = a < 1.0 ? a : 1.0;
    c.ewa = c.ewa * (1.0 - a) + bi * a;
  }
  if (!c.has_min || c.ewa < c.ewa_min) {
    c.no_improvement = 0;
    c.ewa_min = c.ewa;
    c.has_min = 1;
  } else {
    c.no_improvement += 1;
  }
  st->ewa = c.ewa;
  st->ewa_min = c.ewa_min;
  st->has_ewa = c.has_ewa;
  st->has_min = c.has_min;
  st->no_improvement = c.no_improvement;
  if (max_no_improvement >= 0 && c.no_improvement >= max_no_improvement)
    __hip_atomic_store(&st->stop_at, step_i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void mb_converge(int step_i, int64_t bs, int64_t n, int max_no_improvement, float inertia,
                            MBState* __restrict__ st) {
  mb_converge_from(mb_conv_load(st), step_i, bs, n, max_no_improvement, inertia, st);
}

// sequential fp32 inertia of one batch by one workgroup (staged in LDS 2048 at a time; lane 0
// folds them in order reading 16 bytes per LDS access)
__device__ float mb_batch_inertia(int64_t b, const float* __restrict__ sq, float* stage) {
  float acc = 0.f;
  for (int64_t base = 0; base < b; base += 2048) {
    const int m = (int)min<int64_t>(2048, b - base);
#pragma unroll 8
    for (int t = threadIdx.x; t < m; t += blockDim.x) stage[t] = sq[base + t] * 1.0f;
    __syncthreads();
    if (threadIdx.x == 0) acc = fold_seq_lds(stage, m, acc);
    __syncthreads();
  }
  return acc;
}

__global__ void k_mb_converge(int step_i, int64_t bs, int64_t n, int max_no_improvement,
                              const float* __restrict__ batch_inertia, MBState* __restrict__ st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  mb_converge(step_i, bs, n, max_no_improvement, batch_inertia[0], st);
}

// the end of a step: its batch inertia (sequential fp32 over the per-sample distances the update
// left) and, with `converge`, the early-stopping test. Runs as its own launch (public step API)
// or as an extra workgroup of the NEXT step's assignment launch (device loop), where it overlaps
// that assignment: the next update is the first kernel that must see its stop decision.
struct MbTail {
  const float* sq;
  float* inertia;
  MBState* st;
  int64_t b;
  int64_t n_samples;
  int max_ni;
  int step;
  int converge;
  int active;
};

// stp: the loop stopped before this launch's step (tested after the fold's loads, before the writes)
__device__ void mb_tail_block(const MbTail& tl, float* stage, bool stp = false) {
  MbConv c{};
  if (threadIdx.x == 0 && tl.converge) c = mb_conv_load(tl.st);  // in flight during the fold
  const float inertia = mb_batch_inertia(tl.b, tl.sq, stage);
  if (stp) return;
  if (threadIdx.x == 0) {
    tl.inertia[0] = inertia;
    if (tl.converge) mb_converge_from(c, tl.step, tl.b, tl.n_samples, tl.max_ni, inertia, tl.st);
  }
}

__global__ __launch_bounds__(256) void k_mb_tail(MbTail tl, const int32_t* __restrict__ stop) {
  if (stopped(stop, tl.step)) return;
  __shared__ __attribute__((aligned(16))) float stage[2048];
  mb_tail_block(tl, stage);
}

// ---------------------------------------------------------------------------------------------
// MiniBatchKMeans assignment spread over the chip: block (pb, g) takes batch points
// [32pb, 32pb + 32) against centre tiles g*W .. g*W + W-1 (one 32-centre tile per wave), so every
// CU runs about one MFMA chain per SIMD instead of one CU running all k/32 of them. The per-wave
// minima merge in LDS and then across the G blocks of a point group with a 64-bit atomicMin on
// the (distance, index) key (a plain store when G == 1); the update kernel reads the labels out of
// the keys. Extra workgroups past the P*G assignment blocks run, in this order: the previous
// step's tail (inertia + convergence, `tl.active`) and the next step's batch draw (`rn.rows`).
// ---------------------------------------------------------------------------------------------
__host__ __device__ inline size_t mb_assign_lds(int waves, int dim) {
  const int dimp = (dim + 1) & ~1, S = dimp + 1;
  return sizeof(float) * ((size_t)(32 + 32 * waves) * S + 32 * waves) + 16 +
         sizeof(unsigned long long) * 32 * waves;
}

template <int W, bool VEC>
__global__ __launch_bounds__(64 * W) void k_mb_assign(
    int64_t n, int dim, int dimp, const float* __restrict__ X, const int64_t* __restrict__ rows,
    int k, const float* __restrict__ C, const float* __restrict__ cn2,
    unsigned long long* __restrict__ keys, int G, int P, const int32_t* __restrict__ stop,
    int step_i, MbTail tl, RngNext rn) {
  // the stop word goes out with trip 1's loads and is tested before the first global store (r05:
  // tested first it cost each launch one more dependent round trip); a block that runs on after
  // the loop stopped only writes buffers no later step reads, as a block that started first would
  const int32_t sv = stop ? __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  const bool stp = sv != 0 && sv - 1 < step_i;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int blk = blockIdx.x;
  if (blk >= P * G) {
    const int e = blk - P * G;
    if (tl.active && e == 0) {
      GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 82);
      mb_tail_block(tl, lds, stp);
      GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 80);
    } else if (rn.rows) {
      GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 83);
      uint32_t* ring = reinterpret_cast<uint32_t*>(lds);
      for (int i = threadIdx.x; i < 624; i += blockDim.x) ring[i] = rn.in->key[i];
      const int pos = rn.in->pos;
      __syncthreads();
      if (stp) return;
      mt_randint_ring(ring, pos, 0, rn.n, rn.bs, rn.rows, rn.out);
      GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 81);
    }
    return;
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 0);
  const int pb = blk / G, g = blk - pb * G;
  const int S = dimp + 1;
  float* Pl = lds;                              // 32 points x S
  float* Cl = Pl + 32 * S;                      // W centre tiles x 32 x S
  float* Nl = Cl + (size_t)W * 32 * S;          // W x 32 norms
  unsigned long long* Kl =
      reinterpret_cast<unsigned long long*>(((uintptr_t)(Nl + 32 * W) + 15) & ~uintptr_t(15));
  __shared__ int64_t s_rows[32];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t p0 = (int64_t)pb * 32;
  const int np = (int)min<int64_t>(32, n - p0);
  const int cb = (g * W + wave) * 32;  // this wave's tile
  // trip 1: row indices and the centre tile, requested together
  int64_t my_row = 0;
  if (tid < 32 && tid < np) my_row = rows ? rows[p0 + tid] : p0 + tid;
  float* Cw = Cl + (size_t)wave * 32 * S;
  float* Nw = Nl + wave * 32;
  if (cb < k) {
    const float* Cb = C + (int64_t)cb * dim;
    stage_rows32<VEC>(Cw, S, [&](int r) { return Cb + (int64_t)r * dim; }, k - cb, dim, dimp, lane,
                      64);
    if (cn2 && lane < 32) Nw[lane] = (cb + lane < k) ? cn2[cb + lane] : 0.f;
  }
  if (tid < 32) s_rows[tid] = my_row;
  __syncthreads();
  if (stp) return;
  // trip 2: the point rows
  stage_rows32<VEC, 4>(Pl, S, [&](int r) { return X + s_rows[r] * dim; }, np, dim, dimp, tid,
                       64 * W);
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 3);
  unsigned long long best = ~0ull;
  if (cb < k) {
    const int kh = lane >> 5;
    if (!cn2 && lane < 32) Nw[lane] = (cb + lane < k) ? npy_sumsq(Cw + lane * S, dim) : 0.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 4);
    const floatx16 acc = mfma_chain<16>(Cw + (lane & 31) * S + kh, Pl + (lane & 31) * S + kh, dimp);
    GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0 && acc[0] != 12345.f), 5);
    best = tile_best(acc, Nw, cb, kh, k, best);
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0 && best != 0ull), 6);
  const unsigned long long other = __shfl_xor(best, 32);
  best = other < best ? other : best;
  if (lane < 32) Kl[wave * 32 + lane] = best;
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 13);
  if (wave == 0 && lane < np) {
    unsigned long long b = Kl[lane];
#pragma unroll
    for (int q = 1; q < W; ++q) {
      const unsigned long long o = Kl[q * 32 + lane];
      b = o < b ? o : b;
    }
    if (G == 1)
      keys[p0 + lane] = b;
    else
      atomicMin(keys + p0 + lane, b);
  }
}

// ---------------------------------------------------------------------------------------------
// MiniBatchKMeans update, one wave per cluster. Membership comes from `labels` or, in the fused
// step, from the assignment's 64-bit keys (label = low word), then:
//   * labels_out (nullable): the batch labels; sq_out (nullable): each member's distance to its
//     old centre in the _euclidean_dense_dense order (the step's inertia terms, _k_means_common.pyx
//     :26-48 / :92-121) — computed here, where the member rows are gathered anyway;
//   * keys_reset (nullable): the other key buffer is cleared for the next step's assignment.
// The member list and the members' source rows live in LDS (dynamic: 12*b bytes). cn2_out
// (nullable) receives the numpy-order norm of the new centre for the next step's assignment.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_minibatch_update(int64_t b, int dim, const float* __restrict__ X,
                                                        const int64_t* __restrict__ rows,
                                                        const float* __restrict__ w,
                                                        const int32_t* __restrict__ labels,
                                                        const unsigned long long* __restrict__ keys,
                                                        int k, const float* __restrict__ C_old,
                                                        float* __restrict__ C_new,
                                                        float* __restrict__ Wsum,
                                                        float* __restrict__ cn2_out,
                                                        const int32_t* __restrict__ stop, int step_i,
                                                        int32_t* __restrict__ labels_out,
                                                        float* __restrict__ sq_out,
                                                        unsigned long long* __restrict__ keys_reset) {
  // the stop word goes out with the label loads and is tested before the first global store (r05)
  const int32_t sv = stop ? __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 20);
  extern __shared__ __attribute__((aligned(16))) float mb_lds[];
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 21);
  if (sq_out) {  // the old centre row, for the member distances (after the new row in LDS)
    float* crow = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(reinterpret_cast<int64_t*>(mb_lds) + b) + b) + dim;
    for (int f = lane; f < dim; f += 64) crow[f] = C_old[(int64_t)c * dim + f];
  }
  int64_t* src = reinterpret_cast<int64_t*>(mb_lds);      // b source rows
  int32_t* mem = reinterpret_cast<int32_t*>(src + b);     // b member positions
  int count = 0;
  for (int64_t base = 0; base < b; base += 64 * 16) {
    // sixteen independent label loads in flight per lane (a 1024-sample batch in one trip), then
    // the ordered ballot compaction
    int32_t lab[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int64_t i = base + u * 64 + lane;
      lab[u] = i < b ? (keys ? (int32_t)(unsigned)(keys[i] & 0xffffffffull) : labels[i]) : -1;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const bool is = lab[u] == c;
      const unsigned long long m = __ballot(is);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      if (is) mem[count + before] = (int32_t)(base + u * 64 + lane);
      count += __popcll(m);
    }
  }
  __syncthreads();
  if (sv != 0 && sv - 1 < step_i) return;
  if (keys_reset)
    for (int64_t i = (int64_t)c * 64 + lane; i < b; i += (int64_t)gridDim.x * 64) keys_reset[i] = ~0ull;
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 22);
  // the members' source rows: one dependent trip for the few members only (requesting all b batch
  // rows with the labels measured slower: 454 workgroups x 8 KB more L2 reads, 6.9 -> 7.8 us)
  for (int t = lane; t < count; t += 64) src[t] = rows ? rows[mem[t]] : (int64_t)mem[t];
  __syncthreads();
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 23);
  if (labels_out || sq_out) {  // per member: its label and its distance to the old centre
    const float* crow = reinterpret_cast<float*>(mem + b) + dim;  // staged at the start
    const bool v4 = (dim & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    for (int t = lane; t < count; t += 64) {
      if (labels_out) labels_out[mem[t]] = c;
      if (sq_out)
        sq_out[mem[t]] = v4 ? skl_sqdist_v4(X + src[t] * dim, crow, dim)
                            : skl_sqdist(X + src[t] * dim, crow, dim);
    }
  }
  // wsum: sequential fp32 in batch order (update_center_dense :78-83); unit weights sum exactly
  float wsum = 0.f;
  if (w) {
    for (int t = 0; t < count; ++t) wsum = wsum + w[mem[t]];
  } else {
    wsum = (float)count;
  }
  const float W = Wsum[c];
  const int64_t cb = (int64_t)c * dim;
  // the new row goes to LDS after the member lists (12*b bytes >= 8 KiB; dim <= 512 floats)
  float* row_out = reinterpret_cast<float*>(mem + b);
  if (wsum > 0.f) {
    const float Wn = W + wsum;
    const float alpha = 1.0f / Wn;  // Cython `1 / weight_sums[c]` with float operands
    for (int f = lane; f < dim; f += 64) {
      float acc = C_old[cb + f] * W;
      // up to 16 member gathers in flight ahead of the ordered adds (r04: the tail members were
      // gathered one dependent load at a time, and most centres have fewer than four members);
      // x * 1.0f == x, so unit weights skip the product
      for (int t0 = 0; t0 < count; t0 += 16) {
        const int m = min(16, count - t0);
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = u < m ? X[src[t0 + u] * dim + f] : 0.f;
        if (w) {
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (u < m) acc = acc + v[u] * w[mem[t0 + u]];
        } else {
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (u < m) acc = acc + v[u];
        }
      }
      const float v = acc * alpha;
      C_new[cb + f] = v;
      row_out[f] = v;
    }
    __syncthreads();
    if (lane == 0) Wsum[c] = Wn;
  } else {
    for (int f = lane; f < dim; f += 64) {
      const float v = C_old[cb + f];
      C_new[cb + f] = v;
      row_out[f] = v;
    }
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 24);
  if (cn2_out) {  // the new row is also staged in LDS: npy_sumsq's four accumulators on four lanes
    __syncthreads();
    const float acc = lane < 4 ? npy_sumsq_acc(row_out, dim, lane) : 0.f;
    const float a0 = __shfl(acc, 0), a1 = __shfl(acc, 1), a2 = __shfl(acc, 2), a3 = __shfl(acc, 3);
    if (lane == 0) cn2_out[c] = (a0 + a1) + (a2 + a3);
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, (threadIdx.x == 0 && blockIdx.x == 0), 25);
}

__global__ void k_point_center_sqdist(int64_t n, int dim, const float* __restrict__ X,
                                      const int32_t* __restrict__ labels,
                                      const float* __restrict__ C, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = skl_sqdist(X + i * dim, C + (int64_t)labels[i] * dim, dim);
}

// row argmax (torch.argmax of the centres, transduct:126)
__global__ void k_argmax_rows(int k, int dim, const float* __restrict__ C, int64_t* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= k) return;
  const float* r = C + (int64_t)c * dim;
  int best = 0;
  float bv = r[0];
  for (int j = 1; j < dim; ++j) {
    const float v = r[j];
    if (v > bv || (v != v && bv == bv)) {  // torch.argmax: NaN counts as the maximum
      bv = v;
      best = j;
    }
  }
  out[c] = best;
}

inline unsigned blocks_for(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

}  // namespace
}  // namespace gdd

using namespace gdd;

// -------------------------------------------------------------------------------------------------
extern "C" int gdd_row_norms(int64_t n, int dim, const float* X, float* out, gdd_stream_t stream) {
  GDD_REQUIRE(n >= 0 && dim > 0 && (n == 0 || (X && out)), "row_norms: bad arguments");
  if (n == 0) return GDD_OK;
  k_row_norms<<<blocks_for(n), 256, 0, to_hip(stream)>>>(n, dim, X, out, nullptr, 0);
  GDD_LAUNCHED();
  return GDD_OK;
}

namespace {
// resident workgroups of a kernel on the current device (occupancy x CUs), cached per (device,
// kernel, threads, LDS): the persistent launches size their grids by it on every call
int resident_blocks(const void* fn, int threads, size_t lds, int* out) {
  struct Entry {
    int dev, threads;
    const void* fn;
    size_t lds;
    int blocks;
  };
  static std::mutex mu;
  static Entry cache[32];
  static int used = 0, next = 0;  // filled slots; round-robin slot to replace once full
  int dev = 0;
  GDD_HIP(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> g(mu);
    for (int i = 0; i < used; ++i)
      if (cache[i].dev == dev && cache[i].fn == fn && cache[i].threads == threads && cache[i].lds == lds) {
        *out = cache[i].blocks;
        return GDD_OK;
      }
  }
  int occ = 0, cus = 0;
  GDD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, lds));
  GDD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  *out = std::max(occ, 1) * std::max(cus, 1);
  std::lock_guard<std::mutex> g(mu);
  if (used < 32) {
    cache[used++] = Entry{dev, threads, fn, lds, *out};
  } else {
    cache[next] = Entry{dev, threads, fn, lds, *out};
    next = (next + 1) % 32;
  }
  return GDD_OK;
}

}  // namespace
int gdd::occupancy_blocks(const void* fn, int threads, size_t lds, int* out) {
  return resident_blocks(fn, threads, lds, out);
}
namespace {

// LDS bytes of k_assign for a given geometry
size_t assign_lds(int waves, int dimp, int cch) {
  const int S = dimp + 1;
  const int ncp = (cch + 31) & ~31;
  return sizeof(float) * ((size_t)ncp * S + (size_t)32 * waves * S + ncp);
}

constexpr size_t kLdsCap = 160 * 1024;

bool use_small_assign(int64_t n, int dim) {
  return n <= 16384 && assign_small_lds(4, dim) <= kLdsCap;
}

template <int W, bool VEC>
int launch_assign_small_t(int64_t n, int dim, const float* X, const int64_t* rows, int k,
                          const float* C, const float* cn2, int32_t* labels, float* sq_dist,
                          const int32_t* stop, int step_i, const RngNext& rn, hipStream_t s) {
  const int dimp = (dim + 1) & ~1;
  const size_t lds = std::max(assign_small_lds(W, dim), kMtRingBytes + 64);
  if (lds > 65536)
    GDD_HIP(hipFuncSetAttribute((const void*)k_assign_small<W, VEC>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const unsigned grid = (unsigned)((n + 31) / 32) + (rn.rows ? 1u : 0u);
  k_assign_small<W, VEC><<<grid, 64 * W, lds, s>>>(n, dim, dimp, X, rows, k, C, cn2, labels,
                                                   sq_dist, stop, step_i, rn);
  GDD_LAUNCHED();
  return GDD_OK;
}

template <bool VEC>
int launch_assign_small(int64_t n, int dim, const float* X, const int64_t* rows, int k,
                        const float* C, const float* cn2, int32_t* labels, float* sq_dist,
                        const int32_t* stop, int step_i, const RngNext& rn, hipStream_t s) {
  // one 32-centre tile per wave when LDS allows (k <= 512), else fewer waves looping over tiles
  const int tiles = (k + 31) / 32;
  if (tiles > 8 && assign_small_lds(16, dim) <= kLdsCap)
    return launch_assign_small_t<16, VEC>(n, dim, X, rows, k, C, cn2, labels, sq_dist, stop, step_i,
                                          rn, s);
  if (tiles > 4 && assign_small_lds(8, dim) <= kLdsCap)
    return launch_assign_small_t<8, VEC>(n, dim, X, rows, k, C, cn2, labels, sq_dist, stop, step_i,
                                         rn, s);
  return launch_assign_small_t<4, VEC>(n, dim, X, rows, k, C, cn2, labels, sq_dist, stop, step_i,
                                       rn, s);
}

// labels (+ optional per-sample sq_dist) of n samples against k centres.
// small n: fused k_assign_small; large n: centre chunks over grid.y + 64-bit atomicMin keys.
// rn.rows != nullptr (small n only): the launch also draws the next batch (see RngNext).
int launch_assign(int64_t n, int dim, const float* X, const int64_t* rows, int k, const float* C,
                  const float* c_norm2, int32_t* labels, float* sq_dist,
                  unsigned long long* keys, const int32_t* stop, int step_i, hipStream_t s,
                  const RngNext& rn = RngNext{nullptr, nullptr, nullptr, 0, 0}) {
  if (use_small_assign(n, dim)) {
    const bool vec = (dim % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(C)) & 15) == 0;
    return vec ? launch_assign_small<true>(n, dim, X, rows, k, C, c_norm2, labels, sq_dist, stop,
                                           step_i, rn, s)
               : launch_assign_small<false>(n, dim, X, rows, k, C, c_norm2, labels, sq_dist, stop,
                                            step_i, rn, s);
  }
  GDD_REQUIRE(!rn.rows, "assign: in-launch batch draws need the small-batch path");
  GDD_REQUIRE(c_norm2 && keys, "assign: large-n path needs c_norm2 and the key workspace");
  const int dimp16 = (dim + 15) & ~15;  // zero-padded rows: unguarded groups of 8 MFMA steps
  if (dimp16 <= 96) {
    // persistent blocks: all centres in one chunk when they fit 2 blocks per CU, else the fewest
    // chunks that do; about two blocks per CU walk the point tiles
    const int kt = (k + 31) / 32;
    int chunks = 1;
    while (chunks < kt && assign_lds(4, dimp16, ((kt + chunks - 1) / chunks) * 32) > 78 * 1024) ++chunks;
    const int cch = ((kt + chunks - 1) / chunks) * 32;
    const int gy = (k + cch - 1) / cch;
    const int64_t ntiles = (n + 127) / 128;
    const int64_t gx = std::min<int64_t>(ntiles, std::max<int64_t>(1, 512 / gy));
    const size_t lds = assign_lds(4, dimp16, cch);
    if (gy > 1) {
      k_fill_u64<<<blocks_for(n), 256, 0, s>>>(n, keys, ~0ull, stop, step_i);
      GDD_LAUNCHED();
    }
    auto go = [&](auto kern) -> int {
      if (lds > 65536)
        GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      kern<<<dim3((unsigned)gx, (unsigned)gy), 256, lds, s>>>(n, dim, dimp16, X, rows, k, C, c_norm2, cch,
                                                              keys, stop, step_i);
      GDD_LAUNCHED();
      return GDD_OK;
    };
    // two centre tiles per pass: four accumulator chains would need 292 registers, one wave per SIMD
    // (measured 1.38 vs 0.91 ms at the products shape)
    int rc0;
    if (dimp16 > 48) {  // wave tiles: dim <= 48 (every config's k-means input)
      rc0 = go(k_assign_persist<2>);
    } else {
      // wave tiles: as many waves per block as the LDS holds with every centre in one chunk (the
      // centre chunk is staged once per block), at least 4; else the persistent form's chunks.
      // 12 waves (768 threads) leave 170 registers per lane: two chains and the prefetched tile
      // without spills, three waves per SIMD
      const int dimpw = (dim + 1) & ~1;  // even row width: the K = 2 steps (r05; was 16-padded)
      int Wn = 0;
      for (int wv : {12, 8, 4})
        if (Wn == 0 && assign_lds(wv, dimpw, (k + 31) & ~31) <= 150 * 1024) Wn = wv;
      const int cchw = Wn ? ((k + 31) & ~31) : cch;
      if (!Wn) Wn = 4;
      const int gyw = (k + cchw - 1) / cchw;
      const size_t ldsw = assign_lds(Wn, dimpw, cchw);
      const int64_t wtiles = (n + 31) / 32;
      const bool contig = rows == nullptr && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
      if (gyw > 1 && gy == 1) {
        k_fill_u64<<<blocks_for(n), 256, 0, s>>>(n, keys, ~0ull, stop, step_i);
        GDD_LAUNCHED();
      }
      auto gow = [&](auto kern, int wv) -> int {
        if (ldsw > 65536)
          GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsw));
        int res = 0;
        const int rrc = resident_blocks((const void*)kern, 64 * wv, ldsw, &res);
        if (rrc) return rrc;
        const int64_t per = std::max<int64_t>(1, (int64_t)res / gyw);
        const int64_t gxw = std::min<int64_t>((wtiles + wv - 1) / wv, per);
        kern<<<dim3((unsigned)gxw, (unsigned)gyw), 64 * wv, ldsw, s>>>(n, dim, dimpw, X, rows, k, C,
                                                                      c_norm2, cchw, keys, stop, step_i,
                                                                      nullptr, nullptr, 0);
        GDD_LAUNCHED();
        return GDD_OK;
      };
      auto pick = [&](auto W_) -> int {
        constexpr int Wc = decltype(W_)::value;
        return contig ? gow(k_assign_waves<2, Wc, true, 6>, Wc) : gow(k_assign_waves<2, Wc, false, 6>, Wc);
      };
      if (Wn == 12)
        rc0 = pick(std::integral_constant<int, 12>());
      else if (Wn == 8)
        rc0 = pick(std::integral_constant<int, 8>());
      else
        rc0 = pick(std::integral_constant<int, 4>());
    }
    if (rc0) return rc0;
    k_assign_finalize<<<blocks_for(n), 256, 0, s>>>(n, dim, X, rows, C, keys, labels, sq_dist, stop,
                                                    step_i);
    GDD_LAUNCHED();
    return GDD_OK;
  }
  const int waves = dimp16 <= 96 ? 4 : (dimp16 <= 224 ? 2 : 1);
  const int64_t gx = (n + 32 * waves - 1) / (32 * waves);
  // centers per block: as many as fit the LDS budget (>= 32), then fewer while the grid is too
  // small to occupy 256 CUs
  const size_t budget = dimp16 <= 224 ? 65536 : 160000;
  const int kp = (k + 31) & ~31;
  int cch = 32;
  while (cch + 32 <= kp && assign_lds(waves, dimp16, cch + 32) <= budget) cch += 32;
  int64_t gy = (k + cch - 1) / cch;
  while (gx * gy < 1024 && cch > 32) {
    cch -= 32;
    gy = (k + cch - 1) / cch;
  }
  GDD_REQUIRE(gx < (1ll << 31) && gy < 65536, "assign: grid too large");
  const size_t lds = assign_lds(waves, dimp16, cch);
  k_fill_u64<<<blocks_for(n), 256, 0, s>>>(n, keys, ~0ull, stop, step_i);
  GDD_LAUNCHED();
  dim3 grid((unsigned)gx, (unsigned)gy);
  const bool vec = (dim % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(C)) & 15) == 0;
  auto go = [&](auto W_, auto V_) {
    constexpr int W = decltype(W_)::value;
    constexpr bool V = decltype(V_)::value;
    if (lds > 65536)  // gfx950 has 160 KiB of LDS per CU; opt in above the 64 KiB default
      GDD_HIP(hipFuncSetAttribute((const void*)k_assign<W, V>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
    k_assign<W, V><<<grid, 64 * W, lds, s>>>(n, dim, dimp16, X, rows, k, C, c_norm2, cch, keys, stop,
                                             step_i);
    return GDD_OK;
  };
  using T4 = std::integral_constant<int, 4>;
  using T2 = std::integral_constant<int, 2>;
  using T1 = std::integral_constant<int, 1>;
  using VT = std::true_type;
  using VF = std::false_type;
  int rc0;
  if (waves == 4)
    rc0 = vec ? go(T4(), VT()) : go(T4(), VF());
  else if (waves == 2)
    rc0 = vec ? go(T2(), VT()) : go(T2(), VF());
  else
    rc0 = vec ? go(T1(), VT()) : go(T1(), VF());
  if (rc0) return rc0;
  GDD_LAUNCHED();
  k_assign_finalize<<<blocks_for(n), 256, 0, s>>>(n, dim, X, rows, C, keys, labels, sq_dist, stop,
                                                  step_i);
  GDD_LAUNCHED();
  return GDD_OK;
}
}  // namespace

namespace gdd {
int kmeans_assign_dev(int64_t n, int dim, const float* X, int k, const float* C, float* cn2,
                      int32_t* labels, unsigned long long* keys, const int32_t* stop, int step_i,
                      hipStream_t s) {
  k_row_norms<<<blocks_for(k), 256, 0, s>>>(k, dim, C, cn2, stop, step_i);
  GDD_LAUNCHED();
  return launch_assign(n, dim, X, nullptr, k, C, cn2, labels, nullptr, keys, stop, step_i, s);
}

// the Lloyd loop's bounded E-step needs the top-2 wave-tile pass with every centre in one chunk
static int top2_waves(int dim, int k) {
  const int dimp16 = (dim + 15) & ~15;
  if (dimp16 > 48) return 0;
  const int dimpw = (dim + 1) & ~1;
  for (int wv : {12, 8, 4})
    if (assign_lds(wv, dimpw, (k + 31) & ~31) <= 150 * 1024) return wv;
  return 0;
}

bool lloyd_prune_ok(int dim, int k) { return top2_waves(dim, k) > 0; }

// ||C||^2 into cn2, then keys[p] (packed best distance + centre) and sec[p] (second-smallest
// distance) for rows p < *n_dev (rows[p] with a row list, else p); n_max bounds the grid
int kmeans_assign_top2_dev(int64_t n_max, int dim, const float* X, const int64_t* rows,
                           const int64_t* n_dev, int k, const float* C, float* cn2,
                           unsigned long long* keys, float* sec, const int32_t* stop, int step_i,
                           hipStream_t s, const float* Xp, int ldp) {
  const int Wn = top2_waves(dim, k);
  GDD_REQUIRE(Wn > 0 && n_max > 0, "assign_top2: unsupported shape");
  k_row_norms<<<blocks_for(k), 256, 0, s>>>(k, dim, C, cn2, stop, step_i);
  GDD_LAUNCHED();
  const int dimpw = (dim + 1) & ~1;
  const int cch = (k + 31) & ~31;
  const size_t lds = assign_lds(Wn, dimpw, cch);
  const int64_t wtiles = (n_max + 31) / 32;
  const bool contig = rows == nullptr && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  // a row list over the padded copy: 16-byte pieces of aligned rows (F = 6 pieces per lane cover 48)
  const bool row4 = !contig && Xp && ldp % 4 == 0 && ldp >= dim && ldp <= 48 &&
                    (reinterpret_cast<uintptr_t>(Xp) & 15) == 0;
  auto go = [&](auto kern, int wv) -> int {
    if (lds > 65536)
      GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int res = 0;
    const int rrc = resident_blocks((const void*)kern, 64 * wv, lds, &res);
    if (rrc) return rrc;
    const int64_t gx = std::max<int64_t>(1, std::min<int64_t>((wtiles + wv - 1) / wv, res));
    kern<<<dim3((unsigned)gx, 1), 64 * wv, lds, s>>>(n_max, dim, dimpw, row4 ? Xp : X, rows, k, C, cn2, cch,
                                                     keys, stop, step_i, sec, n_dev, row4 ? ldp : 0);
    GDD_LAUNCHED();
    return GDD_OK;
  };
  auto pick = [&](auto W_) -> int {
    constexpr int Wc = decltype(W_)::value;
    if (contig) return go(k_assign_waves<2, Wc, true, 6, true>, Wc);
    return row4 ? go(k_assign_waves<2, Wc, false, 6, true, true>, Wc) : go(k_assign_waves<2, Wc, false, 6, true>, Wc);
  };
  if (Wn == 12) return pick(std::integral_constant<int, 12>());
  if (Wn == 8) return pick(std::integral_constant<int, 8>());
  return pick(std::integral_constant<int, 4>());
}
}  // namespace gdd

extern "C" size_t gdd_kmeans_assign_ws_bytes(int64_t n) {
  return align256(sizeof(unsigned long long) * (size_t)std::max<int64_t>(n, 1));
}

extern "C" int gdd_kmeans_assign(int64_t n, int dim, const float* X, const int64_t* rows, int k,
                                 const float* C, const float* c_norm2, int32_t* labels,
                                 float* sq_dist, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n >= 0 && dim > 0 && dim <= 512 && k > 0, "assign: n=%lld dim=%d k=%d unsupported",
              (long long)n, dim, k);
  GDD_REQUIRE(n == 0 || (X && C && c_norm2 && labels && ws), "assign: null pointer");
  if (n == 0) return GDD_OK;
  if (ws_bytes < gdd_kmeans_assign_ws_bytes(n))
    return fail(GDD_E_WORKSPACE, "assign: workspace %zu too small", ws_bytes);
  return launch_assign(n, dim, X, rows, k, C, c_norm2, labels, sq_dist,
                       static_cast<unsigned long long*>(ws), nullptr, 0, to_hip(stream));
}

extern "C" int gdd_kmeans_assign_bf16(int64_t n, int dim, const float* X, const int64_t* rows, int k,
                                      const float* C, const float* c_norm2, int32_t* labels,
                                      float* sq_dist, void* ws, size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && dim <= 512 && k > 0, "kmeans_assign_bf16: bad shape");
  GDD_REQUIRE(X && C && labels && ws, "kmeans_assign_bf16: null pointer");
  if (ws_bytes < gdd_kmeans_assign_ws_bytes(n))
    return fail(GDD_E_WORKSPACE, "kmeans_assign_bf16: workspace too small");
  hipStream_t s = to_hip(stream);
  float* cn_tmp = nullptr;  // c_norm2 NULL: the r06 pass computes them in its fragment kernel, the
  auto own_norms = [&]() -> int {  // other forms here, into a stream-ordered temporary
    if (c_norm2) return GDD_OK;
    GDD_HIP(hipMallocAsync(reinterpret_cast<void**>(&cn_tmp), sizeof(float) * (size_t)k, s));
    k_row_norms<<<blocks_for(k), 256, 0, s>>>(k, dim, C, cn_tmp, nullptr, 0);
    GDD_LAUNCHED();
    c_norm2 = cn_tmp;
    return GDD_OK;
  };
  auto done = [&](int rc) -> int {
    if (cn_tmp) GDD_HIP(hipFreeAsync(cn_tmp, s));
    return rc;
  };
  unsigned long long* keys = static_cast<unsigned long long*>(ws);
  const int dimp16 = (dim + 15) & ~15;
  {  // the persistent kernel: whole rows (no gathered rows), dim <= 128, centre fragments fit LDS
    const int nsteps = dimp16 / 16, ktiles = (k + 31) / 32;
    const size_t lds = assign_bf16p_lds(ktiles, nsteps, dim);
    const int per_need = (8 * dim + 63) / 64;
    const bool aligned = (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    const size_t fb = bf16_frag_bytes(ktiles, nsteps);
    if (!rows && dim <= 128 && aligned && lds <= 150 * 1024 && fb <= ws_bytes) {
      // the r06 kernel (gdd_bf16.hip) where its shapes allow; GDD_FORCE=bf16_v1: the r03 kernel (A/B)
      if (!forced("bf16_v1") && n >= 32 && nsteps <= 4 && dim % 16 != 0) {
        if (!bf16q_norms_fit(dim, k))
          if (const int rc = own_norms()) return rc;
        return done(bf16q_launch(n, dim, X, k, C, c_norm2, labels, sq_dist, s));
      }
      if (const int rc = own_norms()) return rc;
      const int64_t ntiles = (n + 31) / 32;
      bf16x8_t* frags = static_cast<bf16x8_t*>(ws);  // the keys are not used on this path
      float* cn = reinterpret_cast<float*>(static_cast<char*>(ws) + (size_t)ktiles * nsteps * 64 * 16);
      const int nfr = std::max(ktiles * nsteps * 64, ktiles * 32);
      k_bf16_frags<<<(nfr + 255) / 256, 256, 0, s>>>(dim, nsteps, ktiles, k, C, c_norm2, frags, cn);
      GDD_LAUNCHED();
      auto go = [&](auto P_) -> int {
        constexpr int P = decltype(P_)::value;
        const void* fn = (const void*)k_assign_bf16p<P>;
        GDD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int res = 0;
        const int rrc = resident_blocks(fn, 256, lds, &res);
        if (rrc) return done(rrc);
        const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ntiles + 3) / 4, (int64_t)res));
        k_assign_bf16p<P><<<grid, 256, lds, s>>>(n, dim, nsteps, ktiles, X, k, frags, cn, C, labels, sq_dist);
        GDD_LAUNCHED();
        return done(GDD_OK);
      };
      if (per_need <= 1) return go(std::integral_constant<int, 1>());
      if (per_need <= 2) return go(std::integral_constant<int, 2>());
      if (per_need <= 4) return go(std::integral_constant<int, 4>());
      if (per_need <= 6) return go(std::integral_constant<int, 6>());
      if (per_need <= 8) return go(std::integral_constant<int, 8>());
      if (per_need <= 12) return go(std::integral_constant<int, 12>());
      return go(std::integral_constant<int, 16>());
    }
  }
  constexpr int kWaves = 4;
  const int64_t gx = (n + 32 * kWaves - 1) / (32 * kWaves);
  const int kp = (k + 31) & ~31;
  int cch = 32;
  while (cch + 32 <= kp && assign_bf16_lds(kWaves, dimp16, cch + 32) <= 65536) cch += 32;
  int64_t gy = (k + cch - 1) / cch;
  while (gx * gy < 1024 && cch > 32) {
    cch -= 32;
    gy = (k + cch - 1) / cch;
  }
  GDD_REQUIRE(gx < (1ll << 31) && gy < 65536, "kmeans_assign_bf16: grid too large");
  if (const int rc = own_norms()) return rc;
  const size_t lds = assign_bf16_lds(kWaves, dimp16, cch);
  k_fill_u64<<<blocks_for(n), 256, 0, s>>>(n, keys, ~0ull, nullptr, 0);
  GDD_LAUNCHED();
  k_assign_bf16<kWaves><<<dim3((unsigned)gx, (unsigned)gy), 64 * kWaves, lds, s>>>(
      n, dim, dimp16, X, rows, k, C, c_norm2, cch, keys);
  GDD_LAUNCHED();
  k_assign_finalize<<<blocks_for(n), 256, 0, s>>>(n, dim, X, rows, C, keys, labels, sq_dist, nullptr, 0);
  GDD_LAUNCHED();
  return done(GDD_OK);
}


extern "C" size_t gdd_minibatch_update_ws_bytes(int64_t b, int k) {
  (void)b;
  (void)k;
  return 256;  // member lists live in LDS; kept for ABI stability
}

namespace {
constexpr int64_t kMaxBatch = 13312;  // 12*b bytes of LDS per update block (<= 156 KiB)

size_t update_lds(int64_t b) {
  // src rows (8b) + member positions (4b) + the new and the old centre rows (<= 2 x 512 floats)
  return 12 * (size_t)b + 2 * 512 * sizeof(float);
}

int launch_update(int64_t b, int dim, const float* X, const int64_t* rows, const float* w,
                  const int32_t* labels, const unsigned long long* keys, int k, const float* C_old,
                  float* C_new, float* Wsum, float* cn2_out, const int32_t* stop, int step_i,
                  int32_t* labels_out, float* sq_out, unsigned long long* keys_reset,
                  hipStream_t s) {
  GDD_REQUIRE(b <= kMaxBatch, "minibatch: batch %lld exceeds %lld", (long long)b,
              (long long)kMaxBatch);
  const size_t lds = update_lds(b);
  if (lds > 65536)
    GDD_HIP(hipFuncSetAttribute((const void*)k_minibatch_update,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  k_minibatch_update<<<k, 64, lds, s>>>(b, dim, X, rows, w, labels, keys, k, C_old, C_new, Wsum,
                                        cn2_out, stop, step_i, labels_out, sq_out, keys_reset);
  GDD_LAUNCHED();
  return GDD_OK;
}

template <int W, bool VEC>
int launch_mb_assign_t(int64_t b, int dim, const float* X, const int64_t* rows, int k,
                       const float* C, const float* cn2, unsigned long long* keys,
                       const int32_t* stop, int step_i, const MbTail& tl, const RngNext& rn,
                       hipStream_t s) {
  const int dimp = (dim + 1) & ~1;
  const int tiles = (k + 31) / 32;
  const int G = (tiles + W - 1) / W;
  const int P = (int)((b + 31) / 32);
  const size_t lds = std::max({mb_assign_lds(W, dim), sizeof(float) * 2048 + 16,
                               kMtRingBytes + 64});
  if (lds > 65536)
    GDD_HIP(hipFuncSetAttribute((const void*)k_mb_assign<W, VEC>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const unsigned grid = (unsigned)(P * G) + (tl.active ? 1u : 0u) + (rn.rows ? 1u : 0u);
  k_mb_assign<W, VEC><<<grid, 64 * W, lds, s>>>(b, dim, dimp, X, rows, k, C, cn2, keys, G, P, stop,
                                                step_i, tl, rn);
  GDD_LAUNCHED();
  return GDD_OK;
}

template <bool VEC>
int launch_mb_assign_v(int64_t b, int dim, const float* X, const int64_t* rows, int k,
                       const float* C, const float* cn2, unsigned long long* keys,
                       const int32_t* stop, int step_i, const MbTail& tl, const RngNext& rn,
                       hipStream_t s) {
  if (mb_assign_lds(4, dim) <= 96 * 1024)
    return launch_mb_assign_t<4, VEC>(b, dim, X, rows, k, C, cn2, keys, stop, step_i, tl, rn, s);
  if (mb_assign_lds(2, dim) <= kLdsCap)
    return launch_mb_assign_t<2, VEC>(b, dim, X, rows, k, C, cn2, keys, stop, step_i, tl, rn, s);
  return launch_mb_assign_t<1, VEC>(b, dim, X, rows, k, C, cn2, keys, stop, step_i, tl, rn, s);
}

int launch_mb_assign(int64_t b, int dim, const float* X, const int64_t* rows, int k, const float* C,
                     const float* cn2, unsigned long long* keys, const int32_t* stop, int step_i,
                     const MbTail& tl, const RngNext& rn, hipStream_t s) {
  const bool vec = (dim % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(C)) & 15) == 0;
  return vec ? launch_mb_assign_v<true>(b, dim, X, rows, k, C, cn2, keys, stop, step_i, tl, rn, s)
             : launch_mb_assign_v<false>(b, dim, X, rows, k, C, cn2, keys, stop, step_i, tl, rn, s);
}
}  // namespace

extern "C" int gdd_minibatch_update(int64_t b, int dim, const float* X, const int64_t* rows,
                                    const float* w, const int32_t* labels, int k,
                                    const float* C_old, float* C_new, float* weight_sums, void* ws,
                                    size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(b > 0 && dim > 0 && k > 0, "minibatch_update: bad shape");
  GDD_REQUIRE(X && labels && C_old && C_new && weight_sums, "minibatch_update: null pointer");
  GDD_REQUIRE(C_old != C_new, "minibatch_update: C_old and C_new must differ");
  (void)ws;
  (void)ws_bytes;
  return launch_update(b, dim, X, rows, w, labels, nullptr, k, C_old, C_new, weight_sums, nullptr,
                       nullptr, 0, nullptr, nullptr, nullptr, to_hip(stream));
}

// ---- fused MiniBatchKMeans step (_mini_batch_step + _mini_batch_convergence) ------------------
// Step s uses key buffer and distance buffer s % 2: the assignment writes keys[s%2], the update
// reads them (and clears keys[(s+1)%2] for step s+1) and writes sq[s%2], the tail folds sq[s%2].
namespace {
struct StepWs {
  unsigned long long* keys[2];
  float* cn2;
  float* sq[2];
  float* inertia;
};
StepWs carve_step(void* ws, size_t ws_bytes, int64_t b, int k) {
  Carver cv(ws, ws_bytes);
  StepWs w;
  w.keys[0] = cv.take<unsigned long long>(b);
  w.keys[1] = cv.take<unsigned long long>(b);
  w.cn2 = cv.take<float>(k);
  w.sq[0] = cv.take<float>(b);
  w.sq[1] = cv.take<float>(b);
  w.inertia = cv.take<float>(1);
  return w;
}
}  // namespace

extern "C" size_t gdd_minibatch_state_bytes(void) { return sizeof(MBState); }

extern "C" size_t gdd_minibatch_step_ws_bytes(int64_t b, int k) {
  const size_t bb = (size_t)std::max<int64_t>(b, 1);
  return 2 * align256(sizeof(unsigned long long) * bb) + align256(sizeof(float) * (size_t)std::max(k, 1)) +
         2 * align256(sizeof(float) * bb) + align256(sizeof(float)) + 1024;
}

extern "C" int gdd_minibatch_step(int64_t b, int dim, const float* X, const int64_t* rows, int k,
                                  const float* C_old, float* C_new, float* weight_sums,
                                  int32_t* labels, int step_i, int64_t n_samples,
                                  int max_no_improvement, int flags, void* state, void* ws,
                                  size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(b > 0 && dim > 0 && dim <= 512 && k > 0 && n_samples > 0, "minibatch_step: bad shape");
  GDD_REQUIRE(X && rows && C_old && C_new && weight_sums && labels && state && ws,
              "minibatch_step: null pointer");
  GDD_REQUIRE(C_old != C_new, "minibatch_step: C_old and C_new must differ");
  if (ws_bytes < gdd_minibatch_step_ws_bytes(b, k))
    return fail(GDD_E_WORKSPACE, "minibatch_step: workspace too small");
  hipStream_t s = to_hip(stream);
  MBState* st = static_cast<MBState*>(state);
  const int32_t* stop = &st->stop_at;
  StepWs w = carve_step(ws, ws_bytes, b, k);
  const int cur = step_i & 1;
  k_fill_u64<<<blocks_for(b), 256, 0, s>>>(b, w.keys[cur], ~0ull, stop, step_i);
  GDD_LAUNCHED();
  const float* cn2 = (flags & GDD_STEP_NORMS_VALID) ? w.cn2 : nullptr;
  const MbTail none{nullptr, nullptr, nullptr, 0, 0, 0, 0, 0, 0};
  int rc = launch_mb_assign(b, dim, X, rows, k, C_old, cn2, w.keys[cur], stop, step_i, none,
                            RngNext{nullptr, nullptr, nullptr, 0, 0}, s);
  if (rc) return rc;
  rc = launch_update(b, dim, X, rows, nullptr, nullptr, w.keys[cur], k, C_old, C_new, weight_sums,
                     w.cn2, stop, step_i, labels, w.sq[cur], nullptr, s);
  if (rc) return rc;
  const MbTail tl{w.sq[cur], w.inertia, st, b, n_samples, max_no_improvement, step_i,
                  (flags & GDD_STEP_CONVERGE) ? 1 : 0, 1};
  k_mb_tail<<<1, 256, 0, s>>>(tl, stop);
  GDD_LAUNCHED();
  return GDD_OK;
}

// device loop, step s: the assignment launch also folds step s-1's inertia and runs its
// convergence test (tail) and, with rn, draws batch s+1; the update clears the other key buffer
int gdd::minibatch_step_dev(int64_t b, int dim, const float* X, const int64_t* rows, int k,
                            const float* C_old, float* C_new, float* weight_sums, int32_t* labels,
                            int step_i, int64_t n_samples, int max_no_improvement, int flags,
                            void* state, void* ws, size_t ws_bytes, const RngNext& rn,
                            hipStream_t s) {
  GDD_REQUIRE(b > 0 && dim > 0 && dim <= 512 && k > 0 && n_samples > 0, "minibatch_step: bad shape");
  GDD_REQUIRE(X && rows && C_old && C_new && weight_sums && labels && state && ws,
              "minibatch_step: null pointer");
  GDD_REQUIRE(C_old != C_new, "minibatch_step: C_old and C_new must differ");
  if (ws_bytes < gdd_minibatch_step_ws_bytes(b, k))
    return fail(GDD_E_WORKSPACE, "minibatch_step: workspace too small");
  MBState* st = static_cast<MBState*>(state);
  const int32_t* stop = &st->stop_at;
  StepWs w = carve_step(ws, ws_bytes, b, k);
  const int cur = step_i & 1, prev = cur ^ 1;
  const float* cn2 = (flags & GDD_STEP_NORMS_VALID) ? w.cn2 : nullptr;
  const MbTail tl{w.sq[prev], w.inertia, st, b, n_samples, max_no_improvement, step_i - 1,
                  (flags & GDD_STEP_CONVERGE) ? 1 : 0, (step_i > 0 && !(flags & kStepNoTail)) ? 1 : 0};
  int rc = launch_mb_assign(b, dim, X, rows, k, C_old, cn2, w.keys[cur], stop, step_i, tl, rn, s);
  if (rc) return rc;
  return launch_update(b, dim, X, rows, nullptr, nullptr, w.keys[cur], k, C_old, C_new,
                       weight_sums, w.cn2, stop, step_i, labels, w.sq[cur], w.keys[prev], s);
}

// device loop: clear both key buffers before step 0; after the last step, its tail
int gdd::mb_loop_begin(int64_t b, int k, void* ws, size_t ws_bytes, hipStream_t s) {
  StepWs w = carve_step(ws, ws_bytes, b, k);
  for (int q = 0; q < 2; ++q) {
    k_fill_u64<<<blocks_for(b), 256, 0, s>>>(b, w.keys[q], ~0ull, nullptr, 0);
    GDD_LAUNCHED();
  }
  return GDD_OK;
}

int gdd::mb_loop_end(int64_t b, int k, int last_step, int64_t n_samples, int max_no_improvement,
                     void* state, void* ws, size_t ws_bytes, hipStream_t s) {
  StepWs w = carve_step(ws, ws_bytes, b, k);
  MBState* st = static_cast<MBState*>(state);
  const MbTail tl{w.sq[last_step & 1], w.inertia, st, b, n_samples, max_no_improvement, last_step,
                  1, 1};
  k_mb_tail<<<1, 256, 0, s>>>(tl, &st->stop_at);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_minibatch_converge(int64_t b, int k, int step_i, int64_t n_samples,
                                      int max_no_improvement, void* state, void* ws,
                                      size_t ws_bytes, gdd_stream_t stream) {
  GDD_REQUIRE(b > 0 && k > 0 && n_samples > 0 && state && ws, "minibatch_converge: bad arguments");
  if (ws_bytes < gdd_minibatch_step_ws_bytes(b, k))
    return fail(GDD_E_WORKSPACE, "minibatch_converge: workspace too small");
  // the batch inertia of the preceding gdd_minibatch_step, at its fixed workspace offset
  StepWs w = carve_step(ws, ws_bytes, b, k);
  k_mb_converge<<<1, 64, 0, to_hip(stream)>>>(step_i, b, n_samples, max_no_improvement, w.inertia,
                                              static_cast<MBState*>(state));
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_point_center_sqdist(int64_t n, int dim, const float* X, const int32_t* labels,
                                       const float* C, float* out, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && labels && C && out, "point_center_sqdist: bad arguments");
  k_point_center_sqdist<<<blocks_for(n), 256, 0, to_hip(stream)>>>(n, dim, X, labels, C, out);
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_argmax_rows(int k, int dim, const float* centers, int64_t* out,
                               gdd_stream_t stream) {
  GDD_REQUIRE(k > 0 && dim > 0 && centers && out, "argmax_rows: bad arguments");
  k_argmax_rows<<<blocks_for(k), 256, 0, to_hip(stream)>>>(k, dim, centers, out);
  GDD_LAUNCHED();
  return GDD_OK;
}

// ---- device-side MiniBatchKMeans control: batch draws and random reassignment ------------------
namespace gdd {
namespace {

// randint(0, n, b) for one step from the device MT state (single workgroup)
__global__ __launch_bounds__(1024) void k_mb_rng(const DevMT* __restrict__ in, DevMT* __restrict__ out,
                                                 int64_t n, int64_t bs, int64_t* __restrict__ rows) {
  __shared__ uint32_t ring[kMtRingBytes / sizeof(uint32_t)];
  mt_randint_from(in, ring, 0, n, bs, rows, out);
}

constexpr int kRsParCopy = 2;  // k_mb_reassign: row copies in three block trips beside a one-wave next draw

// LDS arrival counters among some of a workgroup's waves (the others busy elsewhere): every
// arriving wave's earlier LDS and global writes are visible to a wave whose wait returned true;
// false if the bounded spin gave up
__device__ __forceinline__ void waves_arrive_rs(int* ctr) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool waves_wait_rs(int* ctr, int target) {
  for (int it = 0; it < kSpinLimit; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

// The reassignment branch of _mini_batch_step (sklearn/cluster/_kmeans.py:1640-1667) at a step
// the host scheduled (_random_reassign :2029-2043), one workgroup, after that step's update:
//   to = counts < fp32(ratio) * max(counts); with m = |to| > 0:
//   new = permutation(b)[:m]  (random_state.choice(b, replace=False, size=m), legacy draws);
//   C_new[to] = X[rows[new]] in cluster order; ||C_new[c]||^2 refreshed for those rows;
//   counts[to] = min(counts[~to]).
// `mid` receives the MT state after the permutation draws (the state sklearn leaves if this is
// the last step); with rn.rows the workgroup then draws the next step's batch.
// Wave 0 does the serial parts without block barriers (the count statistics, then the shuffle's
// draws); all waves then trace permutation(b)[r] for r < m (one wave per r) and copy the rows.
// m > b/2 (possible only when k > b/2) needs np.argsort's order of the weight sums (numpy's
// introsort: its tie order is numpy's own): the workgroup then changes nothing, records the step in
// st->handoff and stops the loop there (stop_at = step + 1, so every later launch no-ops); the host
// runs this step's convergence test and reassignment and resumes (gdd_fit.hip).
__global__ __launch_bounds__(1024) void k_mb_reassign(
    int step, int64_t bs, int dim, int k, float ratio, const float* __restrict__ X,
    const int64_t* __restrict__ rows, float* __restrict__ C_new, float* __restrict__ counts,
    float* __restrict__ cn2, const DevMT* __restrict__ mt_in, DevMT* __restrict__ mt_mid,
    RngNext rn, MBState* __restrict__ mbs, int form) {
  int32_t* stop = &mbs->stop_at;
  // the stop word alone first: here that measured faster than requesting it with the counts and the
  // key block (r05 trace A/B: 7.31 vs 8.06 us per check; the launches after a stop exit at once)
  if (stopped(stop, step)) return;
#ifdef GDD_STAMPS
  unsigned long long tl[7] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0};
#define RS_STAMP(q) tl[(q) - 40] = __builtin_amdgcn_s_memrealtime()
#else
#define RS_STAMP(q) do {} while (0)
#endif
  GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 40);
  extern __shared__ __attribute__((aligned(16))) int J[];  // bs shuffle draws, then the reassigned clusters in order (k ints)
  __shared__ MTScratch ms;
  __shared__ float s_thr, s_min;
  __shared__ int s_m;
  __shared__ int s_sync[2], s_bad;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = blockDim.x >> 6;
  int* s_list = J + ((bs + 1) & ~1ll);
  uint32_t* ring = reinterpret_cast<uint32_t*>(s_list + k);  // + 64 ints of scratch
  if (t < 2) s_sync[t] = 0;
  if (t == 0) s_bad = 0;
  // the key block's loads go out with wave 0's loads of the counts
  const uint32_t kreg = t < 624 ? mt_in->key[t] : 0u;
  const int preg = mt_in->pos;
  if (wave == 0) {
    // up to 1024 counts in registers, every load in flight at once (a loop of dependent loads
    // would pay one memory round trip per 64 clusters)
    constexpr int kReg = 16;
    float cv[kReg];
#pragma unroll
    for (int q = 0; q < kReg; ++q) cv[q] = counts[min(lane + 64 * q, k - 1)];
    float mx = -__builtin_inff();
#pragma unroll
    for (int q = 0; q < kReg; ++q)
      if (lane + 64 * q < k) mx = fmaxf(mx, cv[q]);
    for (int c = 64 * kReg + lane; c < k; c += 64) mx = fmaxf(mx, counts[c]);
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float thr = ratio * mx;  // NEP 50: fp32(ratio) * fp32 max, rounded to fp32
    float mn = __builtin_inff();
    int base = 0;
    for (int c0 = 0; c0 < k; c0 += 64) {
      const int c = c0 + lane;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < kReg; ++q)
        if (c0 == 64 * q) v = cv[q];
      if (c0 >= 64 * kReg) v = c < k ? counts[c] : 0.f;
      const bool to = c < k && v < thr;
      if (c < k && !to) mn = fminf(mn, v);
      const unsigned long long b = __ballot(to);
      if (to) s_list[base + __popcll(b & ((1ull << lane) - 1ull))] = c;
      base += __popcll(b);
    }
    for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o));
    if (lane == 0) {
      s_thr = thr;
      s_min = mn;
      s_m = base;
    }
  }
  if (t < 624) {
    ms.key[t] = kreg;
  }
  if (t == 0) ms.pos = preg;
  __syncthreads();
  const int m = s_m;
  const float thr = s_thr, cmin = s_min;
  if (2 * (int64_t)m > bs) {  // the argsort branch (_kmeans.py:1644-1648): the host's
    if (t == 0) {
      mbs->handoff = step + 1;
      __hip_atomic_store(stop, step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 41);
  RS_STAMP(41);
  GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 42);
  RS_STAMP(42);
  GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0 && m > 0, 48);
  if (m > 0) {
    if (wave == 0) {
      if (lane == 0) J[0] = 0;
      mt_shuffle_draws_wave(&ms, (int)bs, J);
    }
    __syncthreads();
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0 && m > 0, 49);
  if (m > 0 && (form & kRsParCopy)) {
    // r05: the next batch draw (one wave: mt_randint_wave) beside the row copies, and the copies in
    // three block-wide trips instead of one dependent chain per reassigned cluster: every trace
    // first, then every batch row index, then every row and norm; the copy waves meet on LDS
    // counters so the drawing wave is never waited for. A timed-out counter wait is redone after the
    // closing barrier (the copies are plain overwrites).
    GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 43);
    RS_STAMP(43);
    const bool draw = rn.rows != nullptr;
    // with a draw, the drawing wave (the last: w % 4 == 3) keeps its SIMD to itself — waves
    // w % 4 == 3 copy nothing — and raises its issue priority
    const bool copier = !draw || (wave & 3) != 3;
    const int nc = draw ? nw - (nw >> 2) : nw;  // copy waves
    const int ci = draw ? wave - (wave >> 2) : wave;  // this copy wave's index
    const size_t src_off = (sizeof(int) * (size_t)(((bs + 1) & ~1ll) + k) + kMtRingBytes + 7) & ~(size_t)7;
    int64_t* s_src = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(J) + src_off);
    int* s_pos = reinterpret_cast<int*>(s_src + (bs / 2 + 1));
    auto rows_in = [&](int tc, int stride) {
      for (int r = tc; r < m; r += stride) s_src[r] = rows[s_pos[r]];
    };
    auto rows_out = [&](int tc, int stride) {
      const int md = m * dim;
      for (int e = tc; e < md; e += stride) {
        const int r = e / dim, f = e - r * dim;
        C_new[(int64_t)s_list[r] * dim + f] = X[s_src[r] * dim + f];
      }
      for (int r = tc; r < m; r += stride) cn2[s_list[r]] = npy_sumsq(X + s_src[r] * dim, dim);
    };
    if (draw && wave == nw - 1) {
      __builtin_amdgcn_s_setprio(3);
      mt_store_wave(&ms, mt_mid);  // before the draw twists the key block in place
      GDD_STAMP_WHEN(g_stamps_kmeans, lane == 0, 64);
      mt_randint_wave(&ms, 0, rn.n, rn.bs, rn.rows);
      GDD_STAMP_WHEN(g_stamps_kmeans, lane == 0, 65);
      mt_store_wave(&ms, rn.out);
      GDD_STAMP_WHEN(g_stamps_kmeans, lane == 0, 58);
    } else if (copier) {
      if (!draw) mt_store(&ms, mt_mid);  // every wave copies here
      const int tc = 64 * ci + lane, stride = 64 * nc;
      for (int r = ci; r < m; r += nc) {
        const int q = shuffle_trace_wave4(J, (int)bs, r);
        if (lane == 0) s_pos[r] = q;
      }
      // a wave whose wait gave up copies nothing (s_pos / s_src entries of other waves may not be
      // written yet, and they are addresses): it raises s_bad before it arrives at the next counter,
      // so a wave whose second wait succeeds sees every earlier give-up and skips its copies too
      waves_arrive_rs(&s_sync[0]);
      bool ok = waves_wait_rs(&s_sync[0], nc);
      if (ok)
        rows_in(tc, stride);
      else if (lane == 0)
        __hip_atomic_store(&s_bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      waves_arrive_rs(&s_sync[1]);
      ok = waves_wait_rs(&s_sync[1], nc) && ok;
      if (ok && __hip_atomic_load(&s_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        rows_out(tc, stride);
      else if (lane == 0)
        __hip_atomic_store(&s_bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      for (int c = tc; c < k; c += stride)
        if (counts[c] < thr) counts[c] = cmin;
      GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 59);
    }
    __syncthreads();
    if (s_bad) {  // a counter wait gave up: every trace is in now, redo the copies in order
      rows_in(t, blockDim.x);
      __syncthreads();
      rows_out(t, blockDim.x);
    }
    GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 45);
    RS_STAMP(45);
  } else if (m > 0) {
    GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 43);
    RS_STAMP(43);
    mt_store(&ms, mt_mid);
    for (int r = wave; r < m; r += nw) {
      const int c = s_list[r];
      const int64_t src = rows[shuffle_trace_wave(J, (int)bs, r)];
      const float* xr = X + src * dim;
      float* cr = C_new + (int64_t)c * dim;
      for (int f = lane; f < dim; f += 64) cr[f] = xr[f];
      if (lane == 0) cn2[c] = npy_sumsq(xr, dim);
    }
    for (int c = t; c < k; c += blockDim.x)
      if (counts[c] < thr) counts[c] = cmin;
    GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 44);
    RS_STAMP(44);
    if (rn.rows) {  // the next batch after the permutation (replaces the speculative one)
      for (int i = t; i < 624; i += blockDim.x) ring[i] = ms.key[i];
      __syncthreads();
      mt_randint_ring(ring, ms.pos, 0, rn.n, rn.bs, rn.rows, rn.out);
      GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 45);
      RS_STAMP(45);
    }
  } else {
    // nothing drawn: the state stays, and the step's own launch already drew the next batch
    // from it (the host passes that speculative draw at every reassignment step)
    GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 44);
    RS_STAMP(44);
    if (mt_mid != mt_in) mt_store(&ms, mt_mid);
  }
  GDD_STAMP_WHEN(g_stamps_kmeans, threadIdx.x == 0, 46);
  RS_STAMP(46);
#ifdef GDD_STAMPS
  if (threadIdx.x == 0 && m > 0) {
    for (int q = 0; q < 7; ++q) g_stamps_kmeans[50 + q] = tl[q];
    g_stamps_kmeans[57] = (unsigned long long)m;
  }
#endif
#undef RS_STAMP
}

}  // namespace

int mb_rng_launch(const DevMT* in, DevMT* out, int64_t n, int64_t bs, int64_t* rows, hipStream_t s) {
  GDD_REQUIRE(n > 0 && n - 1 <= 0xffffffffll, "mb_rng: n out of range");
  k_mb_rng<<<1, 1024, 0, s>>>(in, out, n, bs, rows);
  GDD_LAUNCHED();
  return GDD_OK;
}

size_t mb_reassign_lds(int64_t bs, int k) {
  return sizeof(int) * (size_t)((bs + 1) & ~1ll) + sizeof(int) * (size_t)k + kMtRingBytes;
}

bool mb_reassign_ok(int64_t bs, int k) { return mb_reassign_lds(bs, k) <= kReassignLdsCap; }

int mb_reassign_launch(int step, int64_t bs, int dim, int k, float ratio, const float* X,
                       const int64_t* rows, float* C_new, float* counts, void* step_ws,
                       size_t step_ws_bytes, const DevMT* mt_in, DevMT* mt_mid, const RngNext& rn,
                       void* state, hipStream_t s) {
  StepWs w = carve_step(step_ws, step_ws_bytes, bs, k);
  size_t lds = mb_reassign_lds(bs, k);
  GDD_REQUIRE(lds <= kReassignLdsCap, "mb_reassign: batch too large for the LDS swap table");
  // the parallel copies (kRsParCopy) where their index tables (bs/2 + 1 rows: m <= bs/2 here) fit
  // after the base layout; else one dependent copy chain per reassigned cluster
  int form = kRsParCopy;
  const size_t par_lds =
      ((sizeof(int) * (size_t)(((bs + 1) & ~1ll) + k) + kMtRingBytes + 7) & ~(size_t)7) +
      12 * (size_t)(bs / 2 + 1);
  if ((form & kRsParCopy) && par_lds <= kReassignLdsCap)
    lds = std::max(lds, par_lds);
  else
    form &= ~kRsParCopy;
  if (lds > 65536)
    GDD_HIP(hipFuncSetAttribute((const void*)k_mb_reassign, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
  k_mb_reassign<<<1, 1024, lds, s>>>(step, bs, dim, k, ratio, X, rows, C_new, counts, w.cn2, mt_in,
                                     mt_mid, rn, static_cast<MBState*>(state), form);
  GDD_LAUNCHED();
  return GDD_OK;
}

}  // namespace gdd
