// gpf_covariance.hip — squared-exponential covariance builders (HBM-bound writes).
//
// kernel_func (GP_func.py:49-65): a = x / l per dimension (:56-57), squared norms
// summed over dimensions in order (:59-60), (|a_i|^2 + |a_j|^2) - 2 a_i.a_j (:62),
// clamp at 0 (:63), exp(-0.5 r2) (:65); K adds diag(e^2) (:21). One 64x64 output
// tile per workgroup: the scaled coordinates of its 64 rows and 64 columns are
// staged in LDS once, then every lane writes 16 outputs, consecutive lanes on
// consecutive columns (512 contiguous bytes per row per wave).
#pragma once
#include "gpf_common.hip"

namespace gpf {

constexpr int BT = 64;  // covariance build tile

// ----------------------------------------------------------------------------
// K build: lower tiles of K = SE(x,x;l) + diag(e^2) for every particle, padded
// to Npad with an identity block (so padded rows factor to L = I, z = 0).
// Op order mirrors kernel_func (GP_func.py:56-65): a = x / l, |a|^2 summed over
// dims in order, (|a_i|^2 + |a_j|^2) - 2 a_i.a_j, clamp >= 0, exp(-0.5 r2).
// Also seeds the per-particle RHS workspace with y (padded with zeros).
// grid: (nb*(nb+1)/2, P) for every lower 64x64 tile, or (3*nt, P) with diag_only: the lower
// tiles of the 128-wide diagonal blocks only (k_step computes the others itself).
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(NTHR) void k_build_cov(int N, int Npad, int d, const double* __restrict__ x,
                                                    const double* __restrict__ y, const double* __restrict__ e,
                                                    const double* __restrict__ ls, double* __restrict__ Lb,
                                                    double* __restrict__ yb, int* __restrict__ info, int diag_only,
                                                    int* __restrict__ dflag, int* __restrict__ cflag,
                                                    int* __restrict__ pst, long long pstride, int pnt) {
  __shared__ double ai[DMAX][BT];
  __shared__ double aj[DMAX][BT];
  __shared__ double ni[BT], nj[BT];
  const int tid = threadIdx.x;
  const int p = blockIdx.y;
  // lower-triangular tile index -> (bi, bj), bi >= bj
  const int idx = blockIdx.x;
  int bi, bj;
  if (diag_only) {  // the three lower 64x64 tiles of 128-wide diagonal block idx / 3
    const int b = idx / 3, m = idx % 3;
    bi = 2 * b + (m > 0);
    bj = 2 * b + (m == 2);
  } else {
    bi = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
    while ((bi + 1) * (bi + 2) / 2 <= idx) ++bi;
    while (bi * (bi + 1) / 2 > idx) --bi;
    bj = idx - bi * (bi + 1) / 2;
  }
  const double* lp = ls + (size_t)p * d;
  if (idx == 0 && tid == 0) {
    info[p] = 0;  // the factorisation kernels only ever set it
    dflag[p] = -1;  // no diagonal block published yet (early diagonal factor, k_step)
    cflag[p] = -1;  // no critical tile published yet (quadrant finish, k_step)
  }
  // the persistent factorisation's counters (gpf_persist.hip PState: lcol | ucol | sdone, each
  // [P][nt], then the queue heads and the abort word): block column I of particle p starts with
  // nothing finished, except U block 0, which k_diag factors before k_factor runs
  if (pst && diag_only && (idx % 3) == 0 && tid == 0) {
    const int I = idx / 3;
    pst[(size_t)p * pnt + I] = 0;
    pst[pstride + (size_t)p * pnt + I] = (I == 0) ? 1 : 0;
    pst[2 * pstride + (size_t)p * pnt + I] = 0;
  }
  if (pst && idx == 0 && p == 0 && tid < 16) pst[3 * pstride + tid] = 0;

  if (tid < 128) {
    const int t = tid & 63;
    const int g = (tid < 64 ? bi : bj) * BT + t;
    double(*a)[BT] = (tid < 64) ? ai : aj;
    double nrm = 0.0;
    if (g < N) {
      for (int k = 0; k < d; ++k) {
        const double v = x[(size_t)k * N + g] / lp[k];
        a[k][t] = v;
        nrm = nrm + v * v;
      }
    }
    if (tid < 64) ni[t] = nrm; else nj[t] = nrm;
  }
  __syncthreads();

  double* Lp = Lb + (size_t)p * Npad * Npad;
#pragma unroll 4
  for (int u = 0; u < (BT * BT) / NTHR; ++u) {
    const int q = tid + NTHR * u;
    const int r = q >> 6, c = q & 63;
    const int gi = bi * BT + r, gj = bj * BT + c;
    double v;
    if (gi < N && gj < N) {
      double dot = ai[0][r] * aj[0][c];
      for (int k = 1; k < d; ++k) dot = fma(ai[k][r], aj[k][c], dot);
      double r2 = (ni[r] + nj[c]) - 2.0 * dot;
      r2 = r2 > 0.0 ? r2 : 0.0;  // np.maximum(sq_dist, 0)
      v = exp(-0.5 * r2);
      if (gi == gj) v = v + e[gi] * e[gi];
    } else {
      v = (gi == gj) ? 1.0 : 0.0;
    }
    Lp[(size_t)gi * Npad + gj] = v;
  }
  if (bi == bj && tid < BT) {
    const int g = bi * BT + tid;
    yb[(size_t)p * Npad + g] = (g < N) ? y[g] : 0.0;
  }
}

// Rectangular cross-covariance kernel_func(x1, x2, l) (no noise) into
// out[i*ldo + j] for i < R, j < C; entries with i >= N1 or j >= N2 are 0.
// One workgroup per CC_R x 256 output block: the scaled coordinates and squared norms of its
// rows and 256 columns are staged once in LDS (dynamic: d x (CC_R + 256) + CC_R + 256 doubles),
// then every lane keeps its column's coordinates in registers and writes CC_R outputs, a wave
// covering 64 consecutive columns of one row (512 contiguous bytes; 4 waves = one 2 KiB row
// segment). Write-bound (8 B per output) once the exponential per output is spread over enough
// resident waves. D: the dimension as a template constant (1..4; 0 = any d <= DMAX at run time).
// grid: (ceil(C/256), ceil(R/CC_R)), dynamic LDS cross_cov_lds(d) bytes
// 32 rows x 256 columns per workgroup; non-temporal stores (A/B, profiles/r3/ab_cross_cov.txt:
// 4.7 -> 4.9 TB/s)
constexpr int CC_R = 32, CC_C = 256;
__host__ __device__ constexpr size_t cross_cov_lds(int d) { return (size_t)(d + 1) * (CC_R + CC_C) * 8; }
template <int D>
__global__ __launch_bounds__(NTHR) void k_cross_cov(int N1, int N2, int R, int C, int dd,
                                                    const double* __restrict__ x1, int ld1,
                                                    const double* __restrict__ x2, int ld2,
                                                    const double* __restrict__ l, double* __restrict__ out,
                                                    int64_t ldo) {
  const int d = D > 0 ? D : dd;
  extern __shared__ double cc_lds[];
  double* ai = cc_lds;                  // [d][CC_R]
  double* aj = ai + (size_t)d * CC_R;   // [d][256]
  double* ni = aj + (size_t)d * CC_C;   // [CC_R]
  double* nj = ni + CC_R;               // [256]
  const int tid = threadIdx.x;
  const int bi = blockIdx.y, bj = blockIdx.x;
  for (int t = tid; t < CC_R + CC_C; t += NTHR) {
    const bool first = t < CC_R;
    const int tt = first ? t : t - CC_R;
    const int g = first ? bi * CC_R + tt : bj * CC_C + tt;
    const int lim = first ? N1 : N2;
    const double* xs = first ? x1 : x2;
    const int ldx = first ? ld1 : ld2;
    double* a = first ? ai : aj;
    const int lda = first ? CC_R : CC_C;
    double nrm = 0.0;
    if (g < lim) {
      for (int k = 0; k < d; ++k) {
        const double v = xs[(size_t)k * ldx + g] / l[k];
        a[k * lda + tt] = v;
        nrm = nrm + v * v;
      }
    }
    (first ? ni : nj)[tt] = nrm;
  }
  __syncthreads();
  const int c = tid & (CC_C - 1);  // this lane's column (the 4 waves cover 256 consecutive ones)
  const int gj = bj * CC_C + c;
  if (gj >= C) return;
  constexpr int DR = D > 0 ? D : DMAX;
  double bc[DR];  // the column's scaled coordinates
#pragma unroll
  for (int k = 0; k < DR; ++k) bc[k] = (k < d) ? aj[k * CC_C + c] : 0.0;
  const double nc = nj[c];
  const bool colok = gj < N2;
  double* op = out + gj;
  const int r0 = bi * CC_R;
  const int rmax = min(CC_R, R - r0);
#pragma unroll 4
  for (int r = 0; r < rmax; ++r) {
    const int gi = r0 + r;
    double v = 0.0;
    if (gi < N1 && colok) {
      double dot = ai[r] * bc[0];
#pragma unroll
      for (int k = 1; k < DR; ++k)
        if (k < d) dot = fma(ai[k * CC_R + r], bc[k], dot);
      double r2 = (ni[r] + nc) - 2.0 * dot;
      r2 = r2 > 0.0 ? r2 : 0.0;
      v = exp(-0.5 * r2);
    }
    __builtin_nontemporal_store(v, op + (size_t)gi * ldo);
  }
}

// k_cross_cov for dimension d on `stream` (grid and LDS as above). (r4: a form with two columns per
// lane, 16-B non-temporal stores and row blocks strided over a resident grid was bitwise equal and
// 3-5% slower on the prediction's 331 MB K_s — the kernel is bound by its exp() issue, not by the
// store path; and an exp with the libm's algorithm and constants but one v_fma_f64 per Horner step
// (28 instead of ~45 VALU instructions per output, bitwise the libm's) was 10-20% slower, its loop
// no longer unrolled; profiles/r4/ab_cross_cov_pair.txt.)
inline void launch_cross_cov(hipStream_t stream, int N1, int N2, int R, int C, int d, const double* x1, int ld1,
                             const double* x2, int ld2, const double* l, double* out, int64_t ldo) {
  const dim3 grid((unsigned)((C + CC_C - 1) / CC_C), (unsigned)((R + CC_R - 1) / CC_R));
  const size_t lds = cross_cov_lds(d);
  switch (d) {
    case 1: hipLaunchKernelGGL(k_cross_cov<1>, grid, dim3(NTHR), lds, stream, N1, N2, R, C, d, x1, ld1, x2, ld2, l, out, ldo); break;
    case 2: hipLaunchKernelGGL(k_cross_cov<2>, grid, dim3(NTHR), lds, stream, N1, N2, R, C, d, x1, ld1, x2, ld2, l, out, ldo); break;
    case 3: hipLaunchKernelGGL(k_cross_cov<3>, grid, dim3(NTHR), lds, stream, N1, N2, R, C, d, x1, ld1, x2, ld2, l, out, ldo); break;
    case 4: hipLaunchKernelGGL(k_cross_cov<4>, grid, dim3(NTHR), lds, stream, N1, N2, R, C, d, x1, ld1, x2, ld2, l, out, ldo); break;
    default: hipLaunchKernelGGL(k_cross_cov<0>, grid, dim3(NTHR), lds, stream, N1, N2, R, C, d, x1, ld1, x2, ld2, l, out, ldo); break;
  }
}

}  // namespace gpf
