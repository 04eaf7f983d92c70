// gpf_hull.hip — the grid fill of the convex-hull rasteriser.
//
// Reference: convex_hull.py:203-224 (fill_convex_hull) and :122-155 (scanfill). After the
// hull facets are rasterised (host), the grid is filled d times: sort the points
// lexicographically with the fill axis as the last key (the reference's column rotation),
// and between every two consecutive points that differ only along that axis step
// cur = round_to_res(cur + res) for every coordinate while cur[axis] < b[axis] (so the last
// step may pass b); the union of all points is the next grid. round_to_res is
// convex_hull.py:13-24: rint(v / res) * res, then numpy.around to the decimals of str(res)
// when res < 1. Here each gap is one thread (count pass, scan, emit pass); the sort is an
// LSD sequence of stable 64-bit radix sorts (rocPRIM via hipCUB), one per column, and the
// de-duplication compares whole rows (IEEE ==, so -0.0 == 0.0 as in Python's set).
#pragma once
#include <hipcub/hipcub.hpp>

#include "gpf_common.hip"

namespace gpf {

struct HullDims {
  int d, axis;
  double res[DMAX];
  double p10[DMAX];  // 10^decimals, or 0 when res >= 1 (no numpy.around)
};

constexpr int64_t HULL_MAX_STEPS = (int64_t)1 << 26;  // per gap; a guard against res = 0

__device__ __forceinline__ double round_to_res(double v, double res, double p10) {
  double s = rint(v / res) * res;  // Python round() on a float64: half to even
  if (p10 > 0.0) s = rint(s * p10) / p10;  // numpy.around(s, decimals)
  return s;
}

// Stepped points of gap k = (G[k], G[k+1]) (0 when they do not share a line). Every coordinate
// evolves on its own (cur[j] = round_to_res(cur[j] + stride_j) per step) and only the fill axis
// decides the step count, so the axis is stepped first (count pass: that alone) and the emit pass
// then replays each other coordinate for the same count: the same arithmetic per coordinate in
// the same order, with no per-lane coordinate array (r6: the DMAX-double array lived in scratch,
// 272 B per lane; VERDICT r5 hygiene).
template <bool EMIT>
__device__ __forceinline__ int64_t hull_gap(const double* __restrict__ G, int64_t k, const HullDims& hd,
                                            double* __restrict__ out) {
  const int d = hd.d, ax = hd.axis;
  const double* a = G + k * d;
  const double* b = a + d;
  for (int j = 0; j < d; ++j)
    if (j != ax && !(a[j] == b[j])) return 0;
  double c = a[ax];
  const double end = b[ax], rax = hd.res[ax], pax = hd.p10[ax];
  int64_t s = 0;
  while (c < end && s < HULL_MAX_STEPS) {
    c = round_to_res(c + rax, rax, pax);
    if (EMIT) out[s * d + ax] = c;
    ++s;
  }
  if (EMIT)
    for (int j = 0; j < d; ++j) {
      if (j == ax) continue;
      double v = a[j];
      const double r = hd.res[j], q = hd.p10[j];
      for (int64_t t = 0; t < s; ++t) {
        v = round_to_res(v + 0.0, r, q);
        out[t * d + j] = v;
      }
    }
  return s;
}

__global__ void k_hull_count(const double* __restrict__ G, int64_t m, HullDims hd, int64_t* __restrict__ cnt) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  cnt[k] = (k + 1 < m) ? hull_gap<false>(G, k, hd, nullptr) : 0;
}

__global__ void k_hull_emit(const double* __restrict__ G, int64_t m, HullDims hd, const int64_t* __restrict__ off,
                            double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k + 1 >= m) return;
  hull_gap<true>(G, k, hd, out + off[k] * hd.d);
}

// order-preserving 64-bit key of column c of row perm[i] (-0.0 keyed as +0.0: they compare equal)
__global__ void k_hull_key(const double* __restrict__ rows, const int64_t* __restrict__ perm, int64_t n, int d,
                           int c, uint64_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = rows[perm[i] * d + c];
  if (v == 0.0) v = 0.0;
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  key[i] = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ void k_hull_iota(int64_t* __restrict__ perm, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) perm[i] = i;
}

// flag[i] = row perm[i] differs from row perm[i-1] (first row always kept)
__global__ void k_hull_flag(const double* __restrict__ rows, const int64_t* __restrict__ perm, int64_t n, int d,
                            int64_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t f = 1;
  if (i > 0) {
    const double* a = rows + perm[i] * d;
    const double* b = rows + perm[i - 1] * d;
    bool same = true;
    for (int j = 0; j < d; ++j) same = same && (a[j] == b[j]);
    f = same ? 0 : 1;
  }
  flag[i] = f;
}

__global__ void k_hull_compact(const double* __restrict__ rows, const int64_t* __restrict__ perm,
                               const int64_t* __restrict__ flag, const int64_t* __restrict__ pos, int64_t n, int d,
                               double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !flag[i]) return;
  for (int j = 0; j < d; ++j) out[pos[i] * d + j] = rows[perm[i] * d + j];
}

}  // namespace gpf
