// gpf_probsurf.hip — probability surface of merged GP results.
//
// Reference: calc_prob_surf.py:15-30 (sum_gaussians) and :67-81 (per-row driver). Per grid row,
// the finite entries of the row tail, compacted in order, are read as (mu, sd) pairs; rows
// with fewer than 2 or an odd number of finite entries are skipped. The row's 100-point grid is
// numpy.linspace(min(mu - 3 sd), max(mu + 3 sd), 100) and its bin probabilities are
//   p_j = (1/k) sum_i [Phi((y_j + dy/2 - mu_i) / sd_i) - Phi((y_j - dy/2 - mu_i) / sd_i)],
// dy = |max(y) - min(y)| / 100, accumulated in the reference's order (z += cdf; z -= cdf).
// Phi follows scipy's ndtr: 0.5 + 0.5 erf(x/sqrt2) for |x/sqrt2| < 1/sqrt2, else from erfc.
// k_prob_prep (one thread per row: compaction, grid ends, bin width), then k_prob_surf (one
// thread per grid point of the flattened rows x 100 items); VALU-bound (erf/erfc, divisions).
#pragma once
#include "gpf_common.hip"

namespace gpf {

constexpr int PS_POINTS = 100;  // calc_prob_surf.py:70 (points per row)
constexpr int PS_EMAX = 1024;   // tail entries per row (argument bound of gpf_prob_surface)

__device__ __forceinline__ double ndtr(double a) {
  const double x = a * 0.70710678118654752440;  // 1/sqrt(2)
  const double z = fabs(x);
  if (z < 0.70710678118654752440) return 0.5 + 0.5 * erf(x);
  const double y = 0.5 * erfc(z);
  return (x > 0.0) ? 1.0 - y : y;
}

// Row setup, one thread per row: the finite entries of the row tail compacted in order into
// cmp (row stride E), and info = {lo, hi, dy, k}: the grid ends min(mu - 3 sd), max(mu + 3 sd)
// (builtin min/max over numpy arrays: the first extreme wins), dy = |max(y) - min(y)| / 100 over
// the row's linspace values, and k pairs (0: the row is skipped: fewer than 2 or an odd number of
// finite entries). tails: M x E row-major (the row entries after the kinematic columns, +-inf/NaN
// = missing).
__device__ __forceinline__ double ps_linspace(int t, double lo, double hi) {
  // numpy.linspace(lo, hi, 100): y = arange * step + start (or arange / div * delta when the
  // step is zero), last point = stop
  const double delta = hi - lo, step = delta / (PS_POINTS - 1);
  const double i = (double)t;
  double y = (step == 0.0) ? (i / (PS_POINTS - 1)) * delta + lo : i * step + lo;
  if (t == PS_POINTS - 1) y = hi;
  return y;
}

__global__ __launch_bounds__(NTHR) void k_prob_prep(const double* __restrict__ tails, int64_t M, int E,
                                                    double* __restrict__ cmp, double4* __restrict__ info) {
  const int64_t row = (int64_t)blockIdx.x * NTHR + threadIdx.x;
  if (row >= M) return;
  const double* tr = tails + row * (int64_t)E;
  double* g = cmp + row * (int64_t)E;
  int n = 0;
  for (int c = 0; c < E; ++c) {
    const double v = tr[c];
    if (isfinite(v)) g[n++] = v;
  }
  const int k = (n < 2 || (n & 1)) ? 0 : n / 2;
  double lo = 0.0, hi = 0.0, dy = 0.0;
  for (int i = 0; i < k; ++i) {
    const double a = g[2 * i] - 3.0 * g[2 * i + 1];
    const double b = g[2 * i] + 3.0 * g[2 * i + 1];
    if (i == 0 || a < lo) lo = a;
    if (i == 0 || b > hi) hi = b;
  }
  if (k > 0) {
    double ymax = ps_linspace(0, lo, hi), ymin = ymax;
    for (int j = 1; j < PS_POINTS; ++j) {
      const double y = ps_linspace(j, lo, hi);
      ymax = fmax(ymax, y);
      ymin = fmin(ymin, y);
    }
    dy = fabs(ymax - ymin) / PS_POINTS;
  }
  info[row] = make_double4(lo, hi, dy, (double)k);
}

// Grid values and bin probabilities, one thread per (row, grid point) over the flattened
// M x 100 items (full 64-lane waves; a wave spans at most two rows):
//   p_j = (1/k) sum_i [Phi((y_j + dy/2 - mu_i) / sd_i) - Phi((y_j - dy/2 - mu_i) / sd_i)]
// accumulated in the reference's order (z += cdf; z -= cdf). VALU-bound on the erf/erfc and
// division sequences (2 k of each per item).
__global__ __launch_bounds__(NTHR) void k_prob_surf(const double* __restrict__ cmp, const double4* __restrict__ info,
                                                    int64_t M, int E, double* __restrict__ yout,
                                                    double* __restrict__ pout, int* __restrict__ ok) {
  const int64_t item = (int64_t)blockIdx.x * NTHR + threadIdx.x;
  if (item >= M * PS_POINTS) return;
  const int64_t row = item / PS_POINTS;
  const int t = (int)(item - row * PS_POINTS);
  const double4 in = info[row];
  const int k = (int)in.w;
  if (k == 0) {
    if (t == 0) ok[row] = 0;
    return;
  }
  const double y = ps_linspace(t, in.x, in.y);
  const double h = in.z / 2.0;
  const double yp = y + h, ym = y - h;
  const double* g = cmp + row * (int64_t)E;
  double z = 0.0;
  for (int i = 0; i < k; ++i) {
    const double mu = g[2 * i], sd = g[2 * i + 1];
    z = z + ndtr((yp - mu) / sd);
    z = z - ndtr((ym - mu) / sd);
  }
  yout[item] = y;
  pout[item] = z / (double)k;
  if (t == 0) ok[row] = 1;
}

}  // namespace gpf
