// gpf_predict.hip — GP prediction at arbitrary query points (GP_func.py:26-45).
//
// With U = L^-1 from the factorisation, the reference's v = solve(L, K_s) (:38)
// is V = U K_s; only its column sums of squares are needed (:39), so every
// 128x128 tile of V is reduced in registers and never stored.
#pragma once
#include "gpf_common.hip"

#ifndef GPF_VSQ_BNT
#define GPF_VSQ_BNT 0  // (K_s column tiles are re-read by every row tile: default cache policy)
#endif
namespace gpf {

// Row tile t of V = U K_s (GP_func.py:38: v = solve(L, K_s), with U = L^-1), reduced per column
// in registers and never stored:
//   vsq[t][q*128 + c] = sum over the 128 rows of tile t of V(r, c)^2        (GP_func.py:39)
//   vz [t][q*128 + c] = sum over the same rows of V(r, c) z_t(r)
// where z = U y: sum_t vz[t] = (U K_s)^T U y = K_s^T alpha = mu (GP_func.py:36), so the mean needs
// neither alpha nor a second pass over K_s. Each wave holds all 128 rows of its 16 columns: the
// sums run per lane over the rows of each row half, then over the 4 lane groups, then upper half
// + lower half (fixed order). Row tiles t0 .. t0 + gridDim.y - 1, the deepest first (t = nt-1
// streams (t+1) x 128 deep: the dispatch order is x fastest, so the longest workgroups start in the
// first rounds instead of forming the launch's tail).
// grid: (nqt, rows)
__global__ __launch_bounds__(Geo<T>::NTH, 4) void k_predict_vsq(int Npad, const double* __restrict__ U,
                                                         const double* __restrict__ Ks, int ldks,
                                                         double* __restrict__ vsq, const double* __restrict__ z,
                                                         double* __restrict__ vz, int t0) {
  __shared__ __attribute__((aligned(16))) double smem[DL_STAGE];
  // (r6: XCD-owned column tiles — every row tile of a column tile on one XCD — measured 2.55-2.59
  // vs 2.50 ms and were removed; profiles/r6/ab_vsq_xcd.txt)
  const int q = blockIdx.x, t = t0 + (int)gridDim.y - 1 - (int)blockIdx.y;
  const Quad<T> qd;
  Acc<T> acc;
  acc.zero();
  // U is lower triangular: row tile t needs columns [0, (t+1) * 128), and in the last 128 of them
  // row block mi only the chunks c <= mi add non-zeros (TRI_A_LAST skips the chunks c >= 4 for the
  // row blocks mi < 4: 16 of the diagonal block's 64 chunk x row block MFMA groups, exact zeros; r5)
  gemm_stream_dl<true, false, TRI_A_LAST, 2, GPF_VSQ_BNT != 0>(acc, U + (size_t)t * T * Npad, Npad, Ks + (size_t)q * T, ldks, (t + 1) * T,
                                          smem, qd);
  constexpr int MBR = Geo<T>::MBR;
  const double* zt = z + (size_t)t * T + (qd.lane >> 4);
  double half[2], zh[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double a2 = 0.0, az = 0.0;
#pragma unroll
    for (int mi = h * MBR / 2; mi < (h + 1) * MBR / 2; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a2 = fma(acc.v[mi][0][r], acc.v[mi][0][r], a2);
        az = fma(acc.v[mi][0][r], zt[mi * 16 + 4 * r], az);
      }
    half[h] = sum_lane_groups(a2);
    zh[h] = sum_lane_groups(az);
  }
  if ((qd.lane >> 4) == 0) {
    const size_t o = (size_t)t * ldks + (size_t)q * T + qd.col(0);
    vsq[o] = half[0] + half[1];
    vz[o] = zh[0] + zh[1];
  }
}

// mu_q = sum_t vz[t][q] = K_s[:, q]^T alpha (GP_func.py:36; k_predict_vsq: V^T z, the row tiles in
// order; the reference's GEMV re-read all of K_s, 331 MB per 10k queries at N=4096);
// var = clip(1 - sum v^2, 1e-12) (:39-40)
// grid: (ceil(M/256))
__global__ __launch_bounds__(NTHR) void k_predict_out(int nt, int M, const double* __restrict__ vz, int ldks,
                                                      const double* __restrict__ vsq, double* __restrict__ mu,
                                                      double* __restrict__ sd) {
  const int q = blockIdx.x * NTHR + threadIdx.x;
  if (q >= M) return;
  double m = 0.0;
  for (int t = 0; t < nt; ++t) m = m + vz[(size_t)t * ldks + q];
  double s = 0.0;
  for (int t = 0; t < nt; ++t) s = s + vsq[(size_t)t * ldks + q];
  double var = 1.0 - s;
  var = (var < 1e-12) ? 1e-12 : var;
  mu[q] = m;
  sd[q] = sqrt(var);
}

// alpha_c = sum_t szp[t][c] over row tiles t >= c/128 (particle slot 0). grid: ceil(N/256)
__global__ __launch_bounds__(NTHR) void k_alpha(int N, int Npad, int nt, const double* __restrict__ szp,
                                                double* __restrict__ alpha) {
  const int c = blockIdx.x * NTHR + threadIdx.x;
  if (c >= N) return;
  double a = 0.0;
  for (int t = c / T; t < nt; ++t) a = a + szp[(size_t)t * Npad + c];
  alpha[c] = a;
}

// f64 MFMA layout self-test: one wave, C = A(16x4) * B(4x16)
__global__ void k_selftest_mfma(const double* a, const double* b, double* c) {
  const int l = threadIdx.x;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = mfma(a[(l & 15) * 4 + (l >> 4)], b[(l >> 4) * 16 + (l & 15)], acc);
  for (int r = 0; r < 4; ++r) c[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// FP64 MFMA issue-rate probe: every wave runs `iters` rounds of 8 independent
// v_mfma_f64_16x16x4_f64 chains (2048 flops each); out[block] keeps the result live.
__global__ __launch_bounds__(NTHR) void k_mfma_rate(int iters, double seed, double* out, unsigned long long* clk) {
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  d4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  const double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = mfma(a, b, acc[i]);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[blockIdx.x] = s;  // practically never taken; keeps the chains live
  span.stop(clk);
}

}  // namespace gpf
