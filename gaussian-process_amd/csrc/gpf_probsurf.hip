// gpf_probsurf.hip — probability surface of merged GP results.
//
// Reference: calc_prob_surf.py:15-30 (sum_gaussians) and :67-81 (per-row driver). Per grid row,
// the finite entries of the row tail, compacted in order, are read as (mu, sd) pairs; rows
// with fewer than 2 or an odd number of finite entries are skipped. The row's 100-point grid is
// numpy.linspace(min(mu - 3 sd), max(mu + 3 sd), 100) and its bin probabilities are
//   p_j = (1/k) sum_i [Phi((y_j + dy/2 - mu_i) / sd_i) - Phi((y_j - dy/2 - mu_i) / sd_i)],
// dy = |max(y) - min(y)| / 100, accumulated in the reference's order (z += cdf; z -= cdf).
// Phi follows scipy's ndtr: 0.5 + 0.5 erf(x/sqrt2) for |x/sqrt2| < 1/sqrt2, else from erfc.
// One workgroup per row, one thread per grid point; HBM-bound on the 1.6 KB written per row.
#pragma once
#include "gpf_common.hip"

namespace gpf {

constexpr int PS_POINTS = 100;  // calc_prob_surf.py:70 (points per row)
constexpr int PS_NTH = 128;
constexpr int PS_EMAX = 1024;   // tail entries per row held in LDS

__device__ __forceinline__ double ndtr(double a) {
  const double x = a * 0.70710678118654752440;  // 1/sqrt(2)
  const double z = fabs(x);
  if (z < 0.70710678118654752440) return 0.5 + 0.5 * erf(x);
  const double y = 0.5 * erfc(z);
  return (x > 0.0) ? 1.0 - y : y;
}

// tails: M x E row-major (the row entries after the kinematic columns, +-inf/NaN = missing)
__global__ __launch_bounds__(PS_NTH) void k_prob_surf(const double* __restrict__ tails, int64_t M, int E,
                                                      double* __restrict__ yout, double* __restrict__ pout,
                                                      int* __restrict__ ok) {
  __shared__ double g[PS_EMAX];
  __shared__ double ybuf[PS_POINTS];
  __shared__ int kk;
  __shared__ double lo_s, hi_s;
  const int64_t row = blockIdx.x;
  const int t = threadIdx.x;
  const double* tr = tails + row * (int64_t)E;
  if (t == 0) {
    int n = 0;
    for (int c = 0; c < E; ++c) {
      const double v = tr[c];
      if (isfinite(v)) g[n++] = v;
    }
    int k = (n < 2 || (n & 1)) ? 0 : n / 2;
    double lo = 0.0, hi = 0.0;
    for (int i = 0; i < k; ++i) {  // builtin min/max over numpy arrays: first extreme wins
      const double a = g[2 * i] - 3.0 * g[2 * i + 1];
      const double b = g[2 * i] + 3.0 * g[2 * i + 1];
      if (i == 0 || a < lo) lo = a;
      if (i == 0 || b > hi) hi = b;
    }
    kk = k;
    lo_s = lo;
    hi_s = hi;
  }
  __syncthreads();
  const int k = kk;
  if (k == 0) {
    if (t == 0) ok[row] = 0;
    return;
  }
  const double lo = lo_s, hi = hi_s;
  // numpy.linspace(lo, hi, 100): y = arange * step + start (or arange / div * delta when the
  // step is zero), last point = stop
  const double delta = hi - lo, step = delta / (PS_POINTS - 1);
  double y = 0.0;
  if (t < PS_POINTS) {
    const double i = (double)t;
    y = (step == 0.0) ? (i / (PS_POINTS - 1)) * delta + lo : i * step + lo;
    if (t == PS_POINTS - 1) y = hi;
    ybuf[t] = y;
  }
  __syncthreads();
  if (t >= PS_POINTS) return;
  double ymax = ybuf[0], ymin = ybuf[0];
  for (int j = 1; j < PS_POINTS; ++j) {
    ymax = fmax(ymax, ybuf[j]);
    ymin = fmin(ymin, ybuf[j]);
  }
  const double dy = fabs(ymax - ymin) / PS_POINTS;
  const double h = dy / 2.0;
  const double yp = y + h, ym = y - h;
  double z = 0.0;
  for (int i = 0; i < k; ++i) {
    const double mu = g[2 * i], sd = g[2 * i + 1];
    z = z + ndtr((yp - mu) / sd);
    z = z - ndtr((ym - mu) / sd);
  }
  const int64_t o = row * PS_POINTS + t;
  yout[o] = y;
  pout[o] = z / (double)k;
  if (t == 0) ok[row] = 1;
}

}  // namespace gpf
