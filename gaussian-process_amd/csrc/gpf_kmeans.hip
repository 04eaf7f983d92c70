// gpf_kmeans.hip — the Lloyd iterations of the KMeans subsample (find_len_scales.py:25-47,
// sklearn KMeans(n_clusters=max_points, n_init='auto', random_state=0)).
//
// One call of gpf_kmeans_step is one E-step (and M-step sums) of sklearn's lloyd_iter_chunked_dense
// (sklearn/cluster/_k_means_lloyd.pyx) over the n centred points kept on the device:
//   label_i = the first j minimising ||c_j||^2 - 2 x_i.c_j      (_update_chunk_dense: the ||x||^2 term
//                                                                 is common to a row and dropped)
//   sums_j  = sum of the x_i labelled j, count_j = their number  (unit sample weights)
//   dist_i  = ||x_i - c_{label_i}||^2                             (what _relocate_empty_clusters_dense
//                                                                 ranks when a cluster is empty)
// The host (gpfit.kmeans) runs sklearn's loop around it: relocation, averaging, centre shift,
// strict / tolerance convergence, the final E-step. The work per iteration is n x k x d — the part
// that grows with the data; everything per cluster is O(k d) on the host.
#pragma once
#include "gpf_common.hip"

namespace gpf {

constexpr int KM_MAXKD = 8192;  // k x (d + 1) doubles staged in LDS (centres and their norms: 64 KiB)

// one thread per point; the centres and their squared norms staged in LDS (dynamic: k*d + k doubles).
// D > 0: the point's coordinates in registers (a compile-time d); D = 0: any d, the coordinates read
// from memory per centre (a run-time-sized private array would live in scratch). The same operations
// in the same order either way.
template <int D>
__global__ __launch_bounds__(NTHR) void k_km_assign(int64_t n, int d, int k, const double* __restrict__ X,
                                                    const double* __restrict__ C, int* __restrict__ labels,
                                                    double* __restrict__ dist) {
  extern __shared__ double km_lds[];
  double* sc = km_lds;           // [k][d]
  double* cn = km_lds + k * d;   // [k]
  if (D > 0) d = D;
  for (int t = threadIdx.x; t < k * d; t += NTHR) sc[t] = C[t];
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += NTHR) {
    double s = 0.0;
    for (int f = 0; f < d; ++f) s = s + sc[j * d + f] * sc[j * d + f];  // row_norms(centers, squared=True)
    cn[j] = s;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * NTHR + threadIdx.x;
  if (i >= n) return;
  double x[D > 0 ? D : 1];
  const double* xi = X + i * d;
  if (D > 0) {
#pragma unroll
    for (int f = 0; f < D; ++f) x[f] = xi[f];
  }
  auto coord = [&](int f) { return D > 0 ? x[f] : xi[f]; };
  int best = 0;
  double bv = 0.0;
  for (int j = 0; j < k; ++j) {
    double dot = 0.0;
    if (D > 0) {
#pragma unroll
      for (int f = 0; f < D; ++f) dot = dot + x[f] * sc[j * D + f];
    } else {
      for (int f = 0; f < d; ++f) dot = dot + xi[f] * sc[j * d + f];
    }
    const double v = cn[j] + (-2.0 * dot);
    if (j == 0 || v < bv) {  // strict: the first minimum, as the reference's loop
      bv = v;
      best = j;
    }
  }
  double dd = 0.0;
  for (int f = 0; f < d; ++f) {
    const double t = coord(f) - sc[best * d + f];
    dd = dd + t * t;
  }
  labels[i] = best;
  dist[i] = dd;
}

inline void launch_km_assign(hipStream_t st, int64_t n, int d, int k, const double* X, const double* C, int* labels,
                             double* dist) {
  const dim3 grid((unsigned)((n + NTHR - 1) / NTHR)), block(NTHR);
  const size_t lds = (size_t)(k * d + k) * 8;
  switch (d) {
    case 1: hipLaunchKernelGGL(k_km_assign<1>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    case 2: hipLaunchKernelGGL(k_km_assign<2>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    case 3: hipLaunchKernelGGL(k_km_assign<3>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    case 4: hipLaunchKernelGGL(k_km_assign<4>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    case 5: hipLaunchKernelGGL(k_km_assign<5>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    case 6: hipLaunchKernelGGL(k_km_assign<6>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    case 8: hipLaunchKernelGGL(k_km_assign<8>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
    default: hipLaunchKernelGGL(k_km_assign<0>, grid, block, lds, st, n, d, k, X, C, labels, dist); break;
  }
}

// one workgroup per cluster: the members' coordinate sums and count, in a fixed order (each thread
// its strided points in index order, then a fixed LDS tree): deterministic for given labels
__global__ __launch_bounds__(NTHR) void k_km_sums(int64_t n, int d, const double* __restrict__ X,
                                                  const int* __restrict__ labels, double* __restrict__ sums,
                                                  double* __restrict__ counts) {
  __shared__ double red[NTHR];
  __shared__ double cnt[NTHR];
  const int j = blockIdx.x, tid = threadIdx.x;
  for (int f = 0; f < d; ++f) {
    double s = 0.0, c = 0.0;
    for (int64_t i = tid; i < n; i += NTHR)
      if (labels[i] == j) {
        s = s + X[i * d + f];
        c = c + 1.0;
      }
    red[tid] = s;
    cnt[tid] = c;
    __syncthreads();
    for (int h = NTHR / 2; h > 0; h >>= 1) {
      if (tid < h) {
        red[tid] = red[tid] + red[tid + h];
        cnt[tid] = cnt[tid] + cnt[tid + h];
      }
      __syncthreads();
    }
    if (tid == 0) {
      sums[j * d + f] = red[0];
      if (f == 0) counts[j] = cnt[0];
    }
    __syncthreads();
  }
}

}  // namespace gpf
