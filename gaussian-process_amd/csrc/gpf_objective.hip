// gpf_objective.hip — the calibration loss of find_len_scales.py:161-177.
#pragma once
#include "gpf_common.hip"

namespace gpf {

// ----------------------------------------------------------------------------
// Per training point (x_fit = x_known, find_len_scales.py:159):
//   alpha_c  = sum_t szp[t][c],  dinv_c = sum_t s2p[t][c]   (t = c/64 .. nt-1)
//   mu = y - e^2 alpha ; var = clip(e^2 - e^4 dinv, 1e-12) ; sd = sqrt(var)
//   pulls (mu - y) / max(sd * s_k, 1e-12), |pull| <= 1 (find_len_scales.py:161-163)
// |pull_k| <= 1 is monotone in k (sd*s_k non-decreasing), so the literal test is
// bisected for the first k that passes and the point is histogrammed there;
// the coverage counts are the prefix sums (k_score). Same comparisons, same
// IEEE division, 10 per point instead of 1000.
// grid: (ceil(N/256), P)
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(NTHR) void k_points(int N, int Npad, int nt, int K, const double* __restrict__ y,
                                                 const double* __restrict__ e, const double* __restrict__ sig,
                                                 const double* __restrict__ s2p, const double* __restrict__ szp,
                                                 double* __restrict__ mu_out, double* __restrict__ sd_out,
                                                 int* __restrict__ hist) {
  const int p = blockIdx.y;
  const int jj = blockIdx.x * NTHR + threadIdx.x;
  if (jj >= N) return;
  const int t0 = jj / T;  // first 128-row tile holding a nonzero of column jj
  const double* a2 = s2p + (size_t)p * nt * Npad;
  const double* az = szp + (size_t)p * nt * Npad;
  double dinv = 0.0, al = 0.0;
  for (int t = t0; t < nt; ++t) {
    dinv = dinv + a2[(size_t)t * Npad + jj];
    al = al + az[(size_t)t * Npad + jj];
  }
  const double e2 = e[jj] * e[jj];
  const double yv = y[jj];
  const double mu = yv - e2 * al;
  double var = e2 - (e2 * e2) * dinv;
  var = (var < 1e-12) ? 1e-12 : var;  // np.clip(., 1e-12, None), NaN passes through
  const double sd = sqrt(var);
  mu_out[(size_t)p * Npad + jj] = mu;
  sd_out[(size_t)p * Npad + jj] = sd;
  const double num = mu - yv;
  int lo = 0, hi = K;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    double den = sd * sig[mid];
    den = (den < 1e-12) ? 1e-12 : den;  // np.maximum(scaled_e, 1e-12)
    const double pull = num / den;
    if (fabs(pull) <= 1.0) hi = mid; else lo = mid + 1;
  }
  atomicAdd(&hist[(size_t)p * (K + 1) + lo], 1);
}

// numpy float64 pairwise summation (np.add.reduce order; oracle/pairwise.py).
__device__ double pairwise_leaf(const double* a, int len) {
  if (len < 8) {
    double r = 0.0;
    for (int i = 0; i < len; ++i) r = r + a[i];
    return r;
  }
  double q[8];
  for (int u = 0; u < 8; ++u) q[u] = a[u];
  int i = 8;
  const int stop = len - (len % 8);
  for (; i < stop; i += 8)
    for (int u = 0; u < 8; ++u) q[u] = q[u] + a[i + u];
  double r = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  for (; i < len; ++i) r = r + a[i];
  return r;
}

// numpy's recursion: n <= 128 is a leaf, else split at (n/2) rounded down to a multiple
// of 8 and return left + right. Explicit stack, same order; `leaf(off, len)` supplies
// the value of each leaf, visited left to right. The stack (run by one thread) lives in LDS:
// as a dynamically indexed private array it went to scratch.
struct PwStack {
  int off[32], len[32], stage[32];
  double left[32];
};
template <typename Leaf>
__device__ double pairwise_tree(int n, Leaf leaf, PwStack& st) {
  int* off = st.off;
  int* len = st.len;
  int* stage = st.stage;
  double* left = st.left;
  int sp = 0;
  off[0] = 0; len[0] = n; stage[0] = 0;
  for (;;) {
    while (len[sp] > 128) {
      int half = len[sp] / 2;
      half -= half % 8;
      stage[sp] = 1;
      off[sp + 1] = off[sp]; len[sp + 1] = half; stage[sp + 1] = 0;
      ++sp;
    }
    double v = leaf(off[sp], len[sp]);
    for (;;) {
      if (sp == 0) return v;
      --sp;
      if (stage[sp] == 1) {
        left[sp] = v;
        stage[sp] = 2;
        int half = len[sp] / 2;
        half -= half % 8;
        off[sp + 1] = off[sp] + half; len[sp + 1] = len[sp] - half; stage[sp + 1] = 0;
        ++sp;
        break;
      }
      v = left[sp] + v;
    }
  }
}

// Same sum, leaves in parallel: thread 0 lists the leaves, one thread per leaf sums it,
// thread 0 combines them in the tree's order. Block-wide (all threads call); the result
// is returned in thread 0. Scratch: leaf tables of PW_LEAVES entries.
constexpr int PW_LEAVES = 64;  // K <= KGRID_MAX = 4096 -> at most 64 leaves of >= 64
__device__ double pairwise_sum_block(const double* a, int n, int* loff, int* llen, double* lsum, int* nleaf) {
  const int tid = threadIdx.x;
  __shared__ PwStack st;
  if (tid == 0) {
    int cnt = 0;
    pairwise_tree(n, [&](int off, int len) {
      loff[cnt] = off;
      llen[cnt] = len;
      ++cnt;
      return 0.0;
    }, st);
    *nleaf = cnt;
  }
  __syncthreads();
  if (tid < *nleaf) lsum[tid] = pairwise_leaf(a + loff[tid], llen[tid]);
  __syncthreads();
  double r = 0.0;
  if (tid == 0) {
    int idx = 0;
    r = pairwise_tree(n, [&](int, int) { return lsum[idx++]; }, st);
  }
  return r;
}

// ----------------------------------------------------------------------------
// Per particle score (find_len_scales.py:163-177, negated like evaluate_loss :182):
//   coverage_k = count_k / N, W = trapz(|coverage - expected|, s) with numpy's
//   pairwise summation order, proximity = clip(1 - 2 d_min, 0, 1),
//   loss = -(-W - 0.01 proximity).
// grid: (P)
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(NTHR) void k_score(int N, int K, int d, const double* __restrict__ sig,
                                                const double* __restrict__ expct, int* __restrict__ hist,
                                                const double* __restrict__ ls, const double* __restrict__ lo,
                                                const double* __restrict__ hi, double* __restrict__ loss) {
  __shared__ int cnt[KGRID_MAX + 1];
  __shared__ double gap[KGRID_MAX];
  __shared__ double term[KGRID_MAX];
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
  int* h = hist + (size_t)p * (K + 1);
  // coverage counts = inclusive prefix sums of the histogram (exact integers: a block scan)
  __shared__ int seg[NTHR];
  {
    const int per = (K + NTHR - 1) / NTHR, k0 = tid * per, k1 = min(K, k0 + per);
    int run = 0;
    for (int k = k0; k < k1; ++k) { run += h[k]; cnt[k] = run; }
    seg[tid] = run;
    __syncthreads();
    for (int o = 1; o < NTHR; o <<= 1) {  // Hillis-Steele inclusive scan of the segment totals
      const int v = (tid >= o) ? seg[tid - o] : 0;
      __syncthreads();
      seg[tid] += v;
      __syncthreads();
    }
    const int base = (tid > 0) ? seg[tid - 1] : 0;
    for (int k = k0; k < k1; ++k) cnt[k] += base;
  }
  __syncthreads();
  for (int k = tid; k <= K; k += NTHR) h[k] = 0;  // leave the histogram zeroed for the next batch
  for (int k = tid; k < K; k += NTHR) {
    const double cov = (double)cnt[k] / (double)N;
    gap[k] = fabs(cov - expct[k]);
  }
  __syncthreads();
  // trapezoid terms (np.trapezoid): (s[k+1]-s[k]) * (gap[k+1]+gap[k]) / 2
  for (int k = tid; k < K - 1; k += NTHR) term[k] = ((sig[k + 1] - sig[k]) * (gap[k + 1] + gap[k])) / 2.0;
  __syncthreads();
  __shared__ int loff[PW_LEAVES], llen[PW_LEAVES], nleaf;
  __shared__ double lsum[PW_LEAVES];
  const double Wsum = pairwise_sum_block(term, K - 1, loff, llen, lsum, &nleaf);
  if (tid == 0) {
    const double W = Wsum;
    const double* l = ls + (size_t)p * d;
    double dmin = 0.0;
    for (int k = 0; k < d; ++k) {
      const double span = hi[k] - lo[k];
      const double a = (l[k] - lo[k]) / span;
      const double b = (hi[k] - l[k]) / span;
      const double m = (b < a) ? b : a;  // np.minimum (no NaN here: sentinels never reach the GPU)
      if (k == 0 || m < dmin) dmin = m;   // builtin min(): first minimum wins
    }
    double prox = 1.0 - 2.0 * dmin;
    prox = prox < 0.0 ? 0.0 : (prox > 1.0 ? 1.0 : prox);
    const double neg = -W - (0.01 * prox);
    loss[p] = -neg;
  }
}

}  // namespace gpf
