// gdd_scaler.hip — (a8) StandardScaler(with_mean=True, with_std=True).fit_transform on the device.
//
// distill_recsys.kmeans_cluster (ClustGDD/distill_recsys.py:172) scales the SVD embeddings before
// k-means. scikit-learn 1.7.2 (sklearn/preprocessing/_data.py partial_fit + transform, through
// sklearn/utils/extmath.py _incremental_mean_and_var with no prior samples):
//   sum_j   = np.sum(X[:, j], dtype=float64)             rows in order (an axis-0 reduction)
//   mean_j  = sum_j / n
//   t_ij    = float64(x_ij) - mean_j
//   corr_j  = sum_i t_ij ; ssq_j = sum_i t_ij*t_ij        rows in order
//   var_j   = (ssq_j - corr_j*corr_j / n) / n
//   scale_j = sqrt(var_j), or 1 when var_j <= n*eps*var_j + (n*mean_j*eps)^2 (_is_constant_feature)
//   out_ij  = fp32( fp32(float64(x_ij) - mean_j) / scale_j )   (X -= mean_; X /= scale_ on fp32 X)
// The ordered fp64 sums run as k_scaler_stats below (the centring kernel's staging: waves 1..3 stage
// row chunks in LDS, one lane of wave 0 folds each column; r06 — the r05 form, one lane per column
// with eight rows' loads in flight, took 19.9 ms at the Reddit train shape, 153,932 x 602, against
// ~1.5 ms now); the transform is elementwise.
#include <algorithm>
#include <climits>

#include "gdd_common.hpp"

namespace gdd {
namespace {

__global__ void k_scale_rows(int64_t total, int dim, const float* __restrict__ X,
                             const double* __restrict__ mean, const double* __restrict__ scale,
                             float* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % dim);
    const float c = (float)((double)X[t] - mean[j]);
    out[t] = (float)((double)c / scale[j]);
  }
}

}  // namespace
}  // namespace gdd

using namespace gdd;

extern "C" int gdd_standard_scaler_transform(int64_t n, int dim, const float* X, const double* mean,
                                             const double* scale, float* X_out, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && X_out && mean && scale, "standard_scaler_transform: bad arguments");
  hipStream_t s = to_hip(stream);
  const int64_t total = n * (int64_t)dim;
  k_scale_rows<<<(unsigned)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, s>>>(
      total, dim, X, mean, scale, X_out);
  GDD_LAUNCHED();
  return GDD_OK;
}

// ---- KMeans.fit's centring (sklearn/cluster/_kmeans.py:1476-1487 via _tolerance :279-288):
// X_mean = X.mean(axis=0); X -= X_mean; tol = mean(X.var(axis=0)) * tol, in numpy's summation order.
//  * dim > 1: numpy reduces axis 0 of a C-contiguous float32 array row by row, so each column is a
//    sequential fp32 chain; the quotient by n is rounded to fp32 (numpy divides by an intp in fp64
//    then casts: identical, a double-rounded quotient is the correctly rounded one). var: sequential
//    fp32 sum of (x - mean)^2 (subtract, square, add), over n.
//  * dim == 1: the reduced axis is contiguous, so numpy runs its pairwise sum (umath
//    loops_utils.h.src pairwise_sum: n < 8 sequential; n <= 128 eight interleaved accumulators
//    combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the n % 8 tail; otherwise split at n/2 rounded
//    down to a multiple of 8) over 8192-element buffer chunks whose results add in order to 0.
namespace gdd {
namespace {

// dim > 1. Each column's sums are sequential fp32 chains over all n rows, so the kernel is bound by
// the add chain (one dependent v_add_f32 per row) as long as rows arrive fast enough. Workgroup g
// owns columns [8g, 8g + w). Roles: waves 1..3 stage chunks of 768 rows x 8 columns into two
// column-major LDS buffers (the next chunk's loads in flight in registers meanwhile; in the second
// pass they also write x - mean from those registers); lane j of wave 0 only folds column j, its
// 16-byte reads issued a 32-row group ahead of the dependent adds. Only blocks with blockIdx % 8 == 0
// work: they share one XCD's L2 under the observed round-robin placement, so X's lines come from HBM
// once for all column groups (speed only, not correctness).
constexpr int kCW = 8;                     // columns per workgroup
constexpr int kCR = 768;                   // rows per staged chunk
constexpr int kCL = 192;                   // staging threads (waves 1..3)
constexpr int kCQ = kCR * kCW / kCL;       // staged elements per staging thread per chunk
constexpr int kCS = kCR + 8;               // column stride in LDS: (8c + r) % 64 banks, 16-B rows
constexpr int kColXcd = 8;

__device__ __forceinline__ void col_fold32(const float4 (&v)[8], float& acc) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    acc = acc + v[u].x;
    acc = acc + v[u].y;
    acc = acc + v[u].z;
    acc = acc + v[u].w;
  }
}

__device__ __forceinline__ void col_load32(const float* __restrict__ p, float4 (&v)[8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + 4 * u);
}

// rows of one staged column, in order (x in the first pass, (x - mean)^2 in the second). Two 32-row
// register groups alternate: each group's 16-byte reads are issued a whole group of dependent adds
// ahead of their use (scheduling barriers keep the compiler from sinking them next to their adds;
// the first group passes through an empty asm so InstCombine cannot fold the loop's phi of loads
// into a load of a phi of addresses). Look-ahead reads past `rows` land in the next column or the
// padding and are never folded.
__device__ __forceinline__ float col_fold(const float* __restrict__ col, int rows, float acc) {
  int r = 0;
  if (rows >= 64) {
    float4 A[8], B[8];
    col_load32(col, A);
#pragma unroll
    for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(A[u].x), "+v"(A[u].y), "+v"(A[u].z), "+v"(A[u].w));
    for (; r + 64 <= rows; r += 64) {
      col_load32(col + r + 32, B);
      __builtin_amdgcn_sched_barrier(0);
      col_fold32(A, acc);
      __builtin_amdgcn_sched_barrier(0);
      col_load32(col + r + 64, A);
      __builtin_amdgcn_sched_barrier(0);
      col_fold32(B, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (; r < rows; ++r) acc = acc + col[r];
  return acc;
}

__global__ __launch_bounds__(256) void k_col_stats(int64_t n, int dim, const float* __restrict__ X,
                                                   float* __restrict__ X_out, float* __restrict__ mean,
                                                   float* __restrict__ var) {
  if (blockIdx.x % kColXcd) return;
  // two column-major chunk buffers, plus the padding the fold's look-ahead reads may touch
  __shared__ __attribute__((aligned(16))) float buf[2 * kCW * kCS + 32];
  __shared__ float s_m[kCW];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform role branch
  const int c0 = (int)(blockIdx.x / kColXcd) * kCW, w = min(kCW, dim - c0);
  const int64_t nchunks = (n + kCR - 1) / kCR;
  for (int pass = 0; pass < 2; ++pass) {
    if (wave == 0) {  // ---- the fold wave
      float acc = 0.f;
      __syncthreads();  // chunk 0 staged
      for (int64_t i = 0; i < nchunks; ++i) {
        const int rows = (int)min((int64_t)kCR, n - i * kCR);
        if (tid < w) {
          const float* col = buf + (i & 1) * kCW * kCS + tid * kCS;
          acc = col_fold(col, rows, acc);
        }
        __syncthreads();  // slot i&1 free, chunk i+1 staged
      }
      if (tid < w) {
        const float q = (float)((double)acc / (double)n);
        if (pass == 0) {
          mean[c0 + tid] = q;
          s_m[tid] = q;
        } else {
          var[c0 + tid] = q;
        }
      }
    } else {  // ---- the staging waves
      const int lt = tid - 64;
      const int cc = lt & (kCW - 1);  // kCL is a multiple of kCW: every staged element is column cc
      const float mc = pass == 1 ? s_m[min(cc, w - 1)] : 0.f;
      float v[kCQ];
      // unconditional loads at clamped addresses; rows >= n and columns >= w are never folded or written
      auto fetch = [&](int64_t i) {
#pragma unroll
        for (int q = 0; q < kCQ; ++q) {
          const int e = lt + kCL * q;
          const int64_t row = min(i * kCR + (e >> 3), n - 1);
          const int c = min(e & (kCW - 1), w - 1);
          v[q] = X[row * dim + c0 + c];
        }
      };
      auto store = [&](int64_t i) {
        float* sb = buf + (i & 1) * kCW * kCS;
#pragma unroll
        for (int q = 0; q < kCQ; ++q) {  // second pass: the squared deviations, ready to add
          const int e = lt + kCL * q;
          const float d = v[q] - mc;
          sb[(e & (kCW - 1)) * kCS + (e >> 3)] = pass == 0 ? v[q] : d * d;
        }
        if (pass == 1 && cc < w) {  // x - mean straight from the registers (column cc throughout)
          const int64_t rows = min((int64_t)kCR, n - i * kCR);
          float* o = X_out + (i * kCR) * dim + c0 + cc;
#pragma unroll
          for (int q = 0; q < kCQ; ++q) {
            const int r = (lt + kCL * q) >> 3;
            if (r < rows) o[(int64_t)r * dim] = v[q] - mc;
          }
        }
      };
      fetch(0);
      store(0);
      if (nchunks > 1) fetch(1);
      __syncthreads();  // chunk 0 staged
      for (int64_t i = 0; i < nchunks; ++i) {
        if (i + 1 < nchunks) {
          store(i + 1);                         // waits for the chunk in flight
          if (i + 2 < nchunks) fetch(i + 2);    // and puts the next one in flight
        }
        __syncthreads();
      }
    }
    __syncthreads();  // the means in s_m before the second pass
  }
}

// StandardScaler's statistics (top of file) with k_col_stats' staging: workgroup g owns columns
// [8g, 8g + w); waves 1..3 stage 768-row chunks of x (both passes) column-major; lane j of wave 0
// folds column j: pass 0 s = s + double(x); pass 1 t = double(x) - mean, corr = corr + t,
// ssq = ssq + t*t — the oracle's (and numpy's axis-0) row order, one dependent fp64 add per row.
template <int PASS>
__device__ __forceinline__ void sc_fold32(const float4 (&v)[8], double m, double& a, double& b) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float x4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (PASS == 0) {
        a = a + (double)x4[q];
      } else {
        const double t = (double)x4[q] - m;
        a = a + t;
        b = b + t * t;
      }
    }
  }
}

template <int PASS>
__device__ __forceinline__ void sc_fold(const float* __restrict__ col, int rows, double m, double& a,
                                        double& b) {
  int r = 0;
  if (rows >= 64) {
    float4 A[8], B[8];
    col_load32(col, A);
#pragma unroll
    for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(A[u].x), "+v"(A[u].y), "+v"(A[u].z), "+v"(A[u].w));
    for (; r + 64 <= rows; r += 64) {
      col_load32(col + r + 32, B);
      __builtin_amdgcn_sched_barrier(0);
      sc_fold32<PASS>(A, m, a, b);
      __builtin_amdgcn_sched_barrier(0);
      col_load32(col + r + 64, A);
      __builtin_amdgcn_sched_barrier(0);
      sc_fold32<PASS>(B, m, a, b);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (; r < rows; ++r) {
    if constexpr (PASS == 0) {
      a = a + (double)col[r];
    } else {
      const double t = (double)col[r] - m;
      a = a + t;
      b = b + t * t;
    }
  }
}

// one_xcd: only blocks with blockIdx % 8 == 0 work (k_col_stats' placement: one XCD's L2 serves every
// column group); else block g owns group g (more groups than one XCD has CUs)
__global__ __launch_bounds__(256) void k_scaler_stats(int64_t n, int dim, const float* __restrict__ X,
                                                      double* __restrict__ mean_out,
                                                      double* __restrict__ scale_out, int one_xcd) {
  if (one_xcd && blockIdx.x % kColXcd) return;
  __shared__ __attribute__((aligned(16))) float buf[2 * kCW * kCS + 32];
  __shared__ double s_m[kCW];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = (int)(one_xcd ? blockIdx.x / kColXcd : blockIdx.x) * kCW, w = min(kCW, dim - c0);
  const int64_t nchunks = (n + kCR - 1) / kCR;
  const double dn = (double)n;
  for (int pass = 0; pass < 2; ++pass) {
    if (wave == 0) {
      double a = 0.0, b = 0.0;
      const double m = (pass == 1 && tid < w) ? s_m[tid] : 0.0;
      __syncthreads();  // chunk 0 staged
      for (int64_t i = 0; i < nchunks; ++i) {
        const int rows = (int)min((int64_t)kCR, n - i * kCR);
        if (tid < w) {
          const float* col = buf + (i & 1) * kCW * kCS + tid * kCS;
          if (pass == 0)
            sc_fold<0>(col, rows, m, a, b);
          else
            sc_fold<1>(col, rows, m, a, b);
        }
        __syncthreads();
      }
      if (tid < w) {
        if (pass == 0) {
          s_m[tid] = a / dn;
        } else {
          const double mean = m, var = (b - (a * a) / dn) / dn;
          const double eps = 2.220446049250313e-16;
          const double nme = (dn * mean) * eps;
          const bool constant = var <= (dn * eps) * var + nme * nme;  // _is_constant_feature
          mean_out[c0 + tid] = mean;
          scale_out[c0 + tid] = constant ? 1.0 : __builtin_sqrt(var);
        }
      }
    } else {
      const int lt = tid - 64;
      float v[kCQ];
      auto fetch = [&](int64_t i) {
#pragma unroll
        for (int q = 0; q < kCQ; ++q) {
          const int e = lt + kCL * q;
          const int64_t row = min(i * kCR + (e >> 3), n - 1);
          const int c = min(e & (kCW - 1), w - 1);
          v[q] = X[row * dim + c0 + c];
        }
      };
      auto store = [&](int64_t i) {
        float* sb = buf + (i & 1) * kCW * kCS;
#pragma unroll
        for (int q = 0; q < kCQ; ++q) {
          const int e = lt + kCL * q;
          sb[(e & (kCW - 1)) * kCS + (e >> 3)] = v[q];
        }
      };
      fetch(0);
      store(0);
      if (nchunks > 1) fetch(1);
      __syncthreads();
      for (int64_t i = 0; i < nchunks; ++i) {
        if (i + 1 < nchunks) {
          store(i + 1);
          if (i + 2 < nchunks) fetch(i + 2);
        }
        __syncthreads();
      }
    }
    __syncthreads();  // the means in s_m before the second pass
  }
}

// numpy's pairwise leaf (len <= 128) over x (pass 0) or over (x - m)^2 (pass 1, which also writes
// x - m).
__device__ float pw_leaf(const float* __restrict__ a, float* __restrict__ o, int len, int pass, float m) {
  auto val = [&](int i) {
    const float x = a[i];
    if (pass == 0) return x;
    const float d = x - m;
    o[i] = d;
    return d * d;
  };
  if (len < 8) {
    float res = 0.f;
    for (int i = 0; i < len; ++i) res = res + val(i);
    return res;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = val(j);
  int i = 8;
  for (; i < len - (len % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + val(i + j);
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < len; ++i) res = res + val(i);
  return res;
}

// dim == 1: one wave. Per 8192-element chunk lane 0 lists the pairwise tree's leaves (left first),
// the lanes sum the leaves, lane 0 combines them post-order (left + right at every split).
constexpr int kPwChunk = 8192, kPwMaxLeaves = 128;  // a split of > 128 leaves halves >= 64 long
__global__ __launch_bounds__(64) void k_col_stats_pw(int64_t n, const float* __restrict__ X,
                                                     float* __restrict__ X_out, float* __restrict__ mean,
                                                     float* __restrict__ var) {
  __shared__ int loff[kPwMaxLeaves], llen[kPwMaxLeaves];
  __shared__ float lsum[kPwMaxLeaves];
  __shared__ int s_nl;
  __shared__ float s_m;
  __shared__ int sm[32], ss[32];
  __shared__ float sl[32];
  const int lane = threadIdx.x;
  float m = 0.f;
  for (int pass = 0; pass < 2; ++pass) {
    float tot = 0.f;
    for (int64_t c = 0; c < n; c += kPwChunk) {
      const int len = (int)min((int64_t)kPwChunk, n - c);
      if (lane == 0) {
        int sp = 0, nl = 0, off = 0;
        sm[sp++] = len;
        while (sp > 0) {
          const int mm = sm[--sp];
          if (mm <= 128) {
            loff[nl] = off;
            llen[nl] = mm;
            ++nl;
            off += mm;
          } else {
            const int n2 = mm / 2 - (mm / 2) % 8;
            sm[sp++] = mm - n2;
            sm[sp++] = n2;
          }
        }
        s_nl = nl;
      }
      __syncthreads();
      for (int l = lane; l < s_nl; l += 64)
        lsum[l] = pw_leaf(X + c + loff[l], X_out + c + loff[l], llen[l], pass, m);
      __syncthreads();
      if (lane == 0) {
        int sp = 1, li = 0;
        float ret = 0.f;
        bool have = false;
        sm[0] = len;
        ss[0] = 0;
        while (sp > 0) {
          const int t = sp - 1;
          if (have) {
            if (ss[t] == 1) {  // left done: keep it, descend right
              sl[t] = ret;
              ss[t] = 2;
              have = false;
              const int n2 = sm[t] / 2 - (sm[t] / 2) % 8;
              sm[sp] = sm[t] - n2;
              ss[sp] = 0;
              ++sp;
            } else {  // right done
              ret = sl[t] + ret;
              --sp;
            }
            continue;
          }
          const int mm = sm[t];
          if (mm <= 128) {
            ret = lsum[li++];
            --sp;
            have = true;
            continue;
          }
          ss[t] = 1;
          sm[sp] = mm / 2 - (mm / 2) % 8;
          ss[sp] = 0;
          ++sp;
        }
        tot = tot + ret;
      }
      __syncthreads();
    }
    if (lane == 0) {
      if (pass == 0) {
        s_m = (float)((double)tot / (double)n);
        mean[0] = s_m;
      } else {
        var[0] = (float)((double)tot / (double)n);
      }
    }
    __syncthreads();
    m = s_m;
  }
}

}  // namespace
}  // namespace gdd

extern "C" int gdd_center_columns(int64_t n, int dim, const float* X, float* X_out, float* mean,
                                  float* var, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && X_out && mean && var, "center_columns: bad arguments");
  hipStream_t s = to_hip(stream);
  if (dim == 1) {
    k_col_stats_pw<<<1, 64, 0, s>>>(n, X, X_out, mean, var);
  } else {
    const unsigned groups = (unsigned)((dim + kCW - 1) / kCW);
    k_col_stats<<<groups * kColXcd, 256, 0, s>>>(n, dim, X, X_out, mean, var);
  }
  GDD_LAUNCHED();
  return GDD_OK;
}

extern "C" int gdd_standard_scaler(int64_t n, int dim, const float* X, float* X_out, double* mean,
                                   double* scale, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && X_out && mean && scale, "standard_scaler: bad arguments");
  hipStream_t s = to_hip(stream);
  const unsigned groups = (unsigned)((dim + kCW - 1) / kCW);
  // up to 32 column groups on one XCD (its CUs); more spread over all (GDD_FORCE=scaler_one_xcd /
  // scaler_spread: either, A/B)
  const bool one = forced("scaler_one_xcd") || (groups <= 32 && !forced("scaler_spread"));
  k_scaler_stats<<<one ? groups * kColXcd : groups, 256, 0, s>>>(n, dim, X, mean, scale, one ? 1 : 0);
  GDD_LAUNCHED();
  const int64_t total = n * (int64_t)dim;
  k_scale_rows<<<(unsigned)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, s>>>(
      total, dim, X, mean, scale, X_out);
  GDD_LAUNCHED();
  return GDD_OK;
}
