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
// One lane per column runs the ordered fp64 sums (eight rows' loads in flight ahead of the adds);
// the transform is elementwise.
#include <algorithm>

#include "gdd_common.hpp"

namespace gdd {
namespace {

__global__ __launch_bounds__(64) void k_col_stats(int64_t n, int dim, const float* __restrict__ X,
                                                  double* __restrict__ mean_out,
                                                  double* __restrict__ scale_out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= dim) return;
  double s = 0.0;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = X[(i + u) * dim + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + (double)v[u];
  }
  for (; i < n; ++i) s = s + (double)X[i * dim + j];
  const double dn = (double)n;
  const double mean = s / dn;
  double corr = 0.0, ssq = 0.0;
  for (i = 0; i + 8 <= n; i += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = X[(i + u) * dim + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double t = (double)v[u] - mean;
      corr = corr + t;
      ssq = ssq + t * t;
    }
  }
  for (; i < n; ++i) {
    const double t = (double)X[i * dim + j] - mean;
    corr = corr + t;
    ssq = ssq + t * t;
  }
  const double var = (ssq - (corr * corr) / dn) / dn;
  const double eps = 2.220446049250313e-16;
  const double nme = (dn * mean) * eps;
  const bool constant = var <= (dn * eps) * var + nme * nme;
  mean_out[j] = mean;
  scale_out[j] = constant ? 1.0 : __builtin_sqrt(var);
}

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

extern "C" int gdd_standard_scaler(int64_t n, int dim, const float* X, float* X_out, double* mean,
                                   double* scale, gdd_stream_t stream) {
  GDD_REQUIRE(n > 0 && dim > 0 && X && X_out && mean && scale, "standard_scaler: bad arguments");
  hipStream_t s = to_hip(stream);
  k_col_stats<<<(unsigned)((dim + 63) / 64), 64, 0, s>>>(n, dim, X, mean, scale);
  GDD_LAUNCHED();
  const int64_t total = n * (int64_t)dim;
  k_scale_rows<<<(unsigned)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, s>>>(
      total, dim, X, mean, scale, X_out);
  GDD_LAUNCHED();
  return GDD_OK;
}

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
