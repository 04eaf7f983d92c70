// gpf_diag.hip — the 128x128 diagonal-block factor of the blocked factorisation, blocked by 16
// over the whole block (r5).
//
// Reference op (per particle, one diagonal block of GP_func.py:22,24,38): L = chol(A) (dpotrf),
// U = L^-1 (what the identity formulation needs of solve(L, K_s)), z = U y (solve(L, y)), and the
// column partials of colsum(U o U) and U^T z over the block's 128 rows. Replaces round 4's
// factor128 (two 64x64 factors around 64-level GEMM phases, ~97-113k cycles on the chain of every
// latency-bound launch, ~48 us).
//
// The block is an 8 x 8 grid of 16 x 16 blocks, right-looking, one 16-wide block column ("panel")
// per step k, the 36 lower blocks LDS-resident (stride 17: 76.5 KiB) or in registers:
//   P_k  wave 0 factors the diagonal block A_kk on its own (db_panel): L_kk, X_kk = L_kk^-1 and
//        z_k in one [A | I | y] elimination, lane = row / column;
//   Q_k  (one barrier later) the rows below it by MFMA, L(i,k)^T = X_kk A(i,k)^T, their y update
//        y_i -= L(i,k) z_k, and on the chain the next diagonal block A(k+1,k+1) -= L(k+1,k)
//        L(k+1,k)^T;
//   and, beside wave 0's next panel (P_{k+1}), on waves 1-3 and 5-7 (not wave 4: FP64 MFMAs and
//   VALU share a SIMD's FP64 units, and wave 4 shares wave 0's SIMD):
//        the rest of step k's trailing update A(i,j) -= L(i,k) L(j,k)^T (k+1 <= j <= i);
//        step k of the inverse, right-looking by block columns: the owner wave of column j of
//        X = L^-1 (its blocks in registers, the accumulator layout) finalises X_kj = -X_kk S_kj
//        (j < k) and adds S_ij += L(i,k) X_kj for i > k, stores X_kj (U_JJ) and adds its share
//        of the column partials.
// Two barriers per panel. Every product is a 16x16x16 MFMA product (4 v_mfma_f64_16x16x4) with
// operands from LDS or from the owner's accumulators (register e of a 16x16 accumulator is the
// B operand of k-step e: X_kj and L(i,k)^T never move). Fixed assignment of work to waves and a
// fixed summation order: deterministic (not bitwise round 4's factor128; test_factor128 checks it
// against LAPACK and the reference fixtures pin every schedule that uses it).
#pragma once
#include "gpf_common.hip"

namespace gpf {

#ifdef GPF_DB_STAMPS
// Probe builds only (scripts/probes/f128_probe.hip): s_memtime of wave W's lane 0 in workgroup 0 at
// phase ends, [W][slot]: slot 2k: after panel k / step k-1's work, 2k+1: after Q_k; 16: end.
__device__ unsigned long long g_db_stamps[8][20];
#define DB_STAMP(W, i)                                                              \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) {                               \
      unsigned long long t_;                                                        \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");    \
      g_db_stamps[W][i] = t_;                                                       \
    }                                                                               \
  } while (0)
#else
#define DB_STAMP(W, i) \
  do {                \
  } while (0)
#endif

// The diagonal-block routines run on all DNTH (= 512) threads of the factorisation workgroups
// (k_diag, and fused or as the early diagonal workgroup in k_step / k_factor).
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long i = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)i, lane);
  const int hi = __builtin_amdgcn_readlane((int)(i >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Barrier for LDS-only hand-offs between the waves of the diagonal factor: every wave's LDS
// operations retired, then s_barrier (the asm's memory clobber keeps the compiler from moving
// memory operations across it). Unlike __syncthreads() (a workgroup-scope release fence) it does
// not wait for the wave's outstanding global stores, so the L/U tile stores of the factor drain
// behind its LDS phases instead of stalling every barrier.
__device__ __forceinline__ void lsync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 1/sqrt(p) for the pivots of the diagonal factor: v_rsq_f64 and two Newton steps
// (y += y (1/2 - p/2 y^2)), a short dependent chain instead of the ~25 ops of a correctly
// rounded sqrt followed by a division; within a few ulp of 1/sqrt(p).
__device__ __forceinline__ double rsqrt_nr(double p) {
  double y = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double t = fma(-(h * y), y, 0.5);
    y = fma(y, t, y);
  }
  return y;
}

constexpr int DB_LD = 17;                   // row stride of a 16x16 block in LDS (doubles)
constexpr int DB_BLK = 16 * DB_LD;          // doubles per block
constexpr int DB_NB = 36;                   // lower blocks (i >= j) of the 8 x 8 grid
constexpr int DB_Y = DB_NB * DB_BLK;        // y -> z, 128 doubles
constexpr int DB_UNIT = DB_Y + T;           // 31 doubles: 15 zeros, 1, 15 zeros (the X lanes' identity rows)
constexpr int DB_LDS = DB_UNIT + 32;        // doubles of LDS the factor uses (78 KiB)

__host__ __device__ constexpr int db_bid(int i, int j) { return i * (i + 1) / 2 + j; }
// element (r, c) of a block: row-major, stride 17: the 16 rows x 2 depths of an MFMA operand read
// per 32 lanes land on 32 distinct bank pairs, and every access is one per-lane base (the lane's
// row or column) plus immediate offsets (an XOR swizzle kept ~16 per-lane offsets live per access
// pattern across the whole factor)
__device__ __forceinline__ int db_off(int r, int c) { return r * DB_LD + c; }

// ---- one-wave 16x16 block helpers (lane l: g = l >> 4, c = l & 15) ----
// A operand of k-step s from block M: A(r, k) = M(r, k), r = l & 15, k = 4 s + g. Also the B
// operand of M^T: B(k, c) = M^T(k, c) = M(c, k).
__device__ __forceinline__ void db_opa(const double* M, double (&a)[4]) {
  const int l = threadIdx.x & 63, r = l & 15, g = l >> 4;
#pragma unroll
  for (int s = 0; s < 4; ++s) a[s] = M[db_off(r, 4 * s + g)];
}
// accumulator layout: register e = element (4 e + g, c) (= the B operand of k-step e)
__device__ __forceinline__ d4 db_ld(const double* M) {
  const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
  d4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = M[db_off(4 * e + g, c)];
  return v;
}
__device__ __forceinline__ void db_st(double* M, const d4& v) {
  const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) M[db_off(4 * e + g, c)] = v[e];
}
// transposed: register e = element (c, 4 e + g) of M, i.e. (4 e + g, c) of M^T
__device__ __forceinline__ d4 db_ld_t(const double* M) {
  const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
  d4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = M[db_off(c, 4 * e + g)];
  return v;
}
__device__ __forceinline__ void db_st_t(double* M, const d4& v) {
  const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) M[db_off(c, 4 * e + g)] = v[e];
}
// C -= A B^T, A and B blocks in LDS (rows as A operands)
__device__ __forceinline__ d4 db_sub_abt(d4 acc, const double* A, const double* B) {
  double a[4], b[4];
  db_opa(A, a);
  db_opa(B, b);
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = mfma_neg_a(a[s], b[s], acc);
  return acc;
}
// acc (+/-)= A X with A in LDS and X in the accumulator layout (its registers are the B operands)
template <bool NEG>
__device__ __forceinline__ d4 db_mul_ax(d4 acc, const double* A, const d4& X) {
  double a[4];
  db_opa(A, a);
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = NEG ? mfma_neg_a(a[s], X[s], acc) : mfma(a[s], X[s], acc);
  return acc;
}

// ---- static work assignment (compile-time k, block indices, waves) ----
// owner wave of column j of X (SIMD s holds waves s and s + 4): columns 0, 3, 6 on SIMD 1, 1, 4, 7
// on SIMD 2, 2, 5 on SIMD 3, so that each step's active columns spread over the three SIMDs
__host__ __device__ constexpr int db_col_wave(int j) {
  return j == 0 ? 1 : j == 1 ? 2 : j == 2 ? 3 : j == 3 ? 5 : j == 4 ? 6 : j == 5 ? 7 : j == 6 ? 5 : 6;
}
// products the owner of column j does in step t of the inverse (finalise + contributions)
__host__ __device__ constexpr int db_x_work(int t, int j) { return j > t ? 0 : (j < t ? 1 : 0) + (7 - t); }
// the trailing-update blocks of step k beside panel k+1: every (i, j), k+1 <= j <= i, but the next
// diagonal block (k+1, k+1), which Q_k updates on the chain
__host__ __device__ constexpr bool db_in_bulk(int k, int i, int j) {
  return j >= k + 1 && i >= j && i < 8 && !(i == k + 1 && j == k + 1);
}
// owner wave of the trailing-update block (i, j) of step k: greedy in a fixed block order onto the
// least-loaded SIMD (1-3) counting step k's inverse work, then its less-loaded wave
__host__ __device__ constexpr int db_bulk_wave(int k, int bi, int bj) {
  int wl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j <= k && j < 8; ++j) wl[db_col_wave(j)] += db_x_work(k, j);
  for (int i = k + 1; i < 8; ++i)
    for (int j = k + 1; j <= i; ++j) {
      if (!db_in_bulk(k, i, j)) continue;
      int best = 1;
      for (int s = 2; s <= 3; ++s)
        if (wl[s] + wl[s + 4] < wl[best] + wl[best + 4]) best = s;
      const int w = wl[best + 4] < wl[best] ? best + 4 : best;
      if (i == bi && j == bj) return w;
      wl[w] += 1;
    }
  return -1;
}
// Q_k: the block rows i = k+1 .. 7 below the panel, one TRSM each; row k+1 (which also updates the
// next diagonal block: the chain) on wave 4, alone on its SIMD while wave 0 waits, the others on
// waves 1-3, 5-7
__host__ __device__ constexpr int db_q_wave(int k, int i) {
  return i == k + 1 ? 4 : (i - k - 2 == 0 ? 1 : i - k - 2 == 1 ? 2 : i - k - 2 == 2 ? 3 : i - k - 2 == 3 ? 5 : i - k - 2 == 4 ? 6 : 7);
}

// m of lanes 0..15 copied to lanes 16..31, 32..47, 48..63 (v_permlane32_swap: lanes 32..63 take
// lanes 0..31; v_permlane16_swap: rows 1 and 3 take rows 0 and 2), per 32-bit half.
__device__ __forceinline__ unsigned row0_to_rows_u32(unsigned v) {
  const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(a[0], a[0], false, false);
  return b[0];
}
__device__ __forceinline__ double row0_to_rows(double m) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, m);
  const unsigned lo = row0_to_rows_u32((unsigned)u), hi = row0_to_rows_u32((unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// x -= L(S, q) * m with L(S, q) = lane S of the lane's row of mc (v_fmac_f64 with row_newbcast:S;
// fma(-m, L, x) and fma(-L, m, x) are the same rounding)
// (volatile: the column's DPP operations stay in order, and the first one carries the 2 wait states
// a DPP read of a VGPR just written by a VALU operation needs — the compiler's hazard recognizer
// does not look into inline asm)
template <int S, bool FIRST>
__device__ __forceinline__ void db_fmac_bcast(double& x, double mc, double m) {
  if (FIRST)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(x) : "v"(mc), "v"(m), "i"(S));
  else
    asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(mc), "v"(m), "i"(S));
}
// the entries s = q + D .. 15 of column q (q runtime-constant after unrolling: a switch on s)
template <int D>
__device__ __forceinline__ void db_fmac_bcast_from(int q, double (&x)[16], double mc, double m) {
#pragma unroll
  for (int s = 0; s < 16; ++s)
    if (s == q + D) {
      switch (s) {
        case 2: db_fmac_bcast<2, true>(x[s], mc, m); break;
        case 3: db_fmac_bcast<3, true>(x[s], mc, m); break;
        case 4: db_fmac_bcast<4, true>(x[s], mc, m); break;
        case 5: db_fmac_bcast<5, true>(x[s], mc, m); break;
        case 6: db_fmac_bcast<6, true>(x[s], mc, m); break;
        case 7: db_fmac_bcast<7, true>(x[s], mc, m); break;
        case 8: db_fmac_bcast<8, true>(x[s], mc, m); break;
        case 9: db_fmac_bcast<9, true>(x[s], mc, m); break;
        case 10: db_fmac_bcast<10, true>(x[s], mc, m); break;
        case 11: db_fmac_bcast<11, true>(x[s], mc, m); break;
        case 12: db_fmac_bcast<12, true>(x[s], mc, m); break;
        case 13: db_fmac_bcast<13, true>(x[s], mc, m); break;
        case 14: db_fmac_bcast<14, true>(x[s], mc, m); break;
        default: db_fmac_bcast<15, true>(x[s], mc, m); break;
      }
    } else if (s > q + D) {
      switch (s) {
        case 0: db_fmac_bcast<0, false>(x[s], mc, m); break;
        case 1: db_fmac_bcast<1, false>(x[s], mc, m); break;
        case 2: db_fmac_bcast<2, false>(x[s], mc, m); break;
        case 3: db_fmac_bcast<3, false>(x[s], mc, m); break;
        case 4: db_fmac_bcast<4, false>(x[s], mc, m); break;
        case 5: db_fmac_bcast<5, false>(x[s], mc, m); break;
        case 6: db_fmac_bcast<6, false>(x[s], mc, m); break;
        case 7: db_fmac_bcast<7, false>(x[s], mc, m); break;
        case 8: db_fmac_bcast<8, false>(x[s], mc, m); break;
        case 9: db_fmac_bcast<9, false>(x[s], mc, m); break;
        case 10: db_fmac_bcast<10, false>(x[s], mc, m); break;
        case 11: db_fmac_bcast<11, false>(x[s], mc, m); break;
        case 12: db_fmac_bcast<12, false>(x[s], mc, m); break;
        case 13: db_fmac_bcast<13, false>(x[s], mc, m); break;
        case 14: db_fmac_bcast<14, false>(x[s], mc, m); break;
        default: db_fmac_bcast<15, false>(x[s], mc, m); break;
      }
    }
}

// ---- the panel: wave 0 ----
#ifndef GPF_PANEL_GST_LATE  // 0: the panel's global stores ahead of the barrier into Q_k (round 5)
#define GPF_PANEL_GST_LATE 1
#endif
#ifndef GPF_DB_PANEL_GST  // probe builds only: 0 drops the panel's global stores (L 1, U 2) to time them
#define GPF_DB_PANEL_GST 3
#endif
// The 16 x 16 diagonal block A_kk, as an [A | I | y] elimination on one wave: lane r < 16 holds row r
// of A (columns <= r), lane 16 + c column c of X_kk = L_kk^-1 (the identity to start), lane 32 the
// block's 16 entries of y. Every role takes the same update, x[s] -= m * L(s, q), with its
// multiplier m (A: L(r, q); X: X(q, c); y: z_q) — one fma per entry and column for the whole wave.
// Leaves L_kk (lanes 0..15) and X_kk (lanes 16..31) in x for db_panel_gst, writes X_kk to the LDS
// diagonal slot and z_k to the LDS y. Returns whether a pivot was not > 0.
__device__ __forceinline__ bool db_panel_core(double* lds, int k, double (&x)[16]) {
  const int r = threadIdx.x & 63;
  double* blk = lds + db_bid(k, k) * DB_BLK;  // A_kk; then X_kk
  const bool arow = r < 16, xcol = r >= 16 && r < 32, ylane = r == 32;
  int ro = r;
  asm volatile("" : "+v"(ro));  // (an opaque lane index: the initial values are not kept live across panels)
  // Every lane loads its 16 entries from a row of its own — A rows from the block (the entries
  // right of the diagonal are A's symmetric values: finite, updated, never stored or read), the X
  // lanes from the unit vector (lane 16 + c: e_c), the y lane from y, the others anything — with
  // no per-entry select: the role selects cost ~100 VALU instructions per panel (r5 probe).
  const int row_off = arow ? db_bid(k, k) * DB_BLK + ro * DB_LD
                           : (xcol ? DB_UNIT + 15 - (ro - 16) : (ylane ? DB_Y + 16 * k : DB_UNIT));
  const double* src = lds + row_off;
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = src[c];
  bool bad = false;
  // Column q: pivot from lane q, 1/sqrt by v_rsq + Newton, scale, then the rank-1 update of every
  // later entry s of the lane's row with L(s, q), in column order (each entry takes its updates
  // q = 0, 1, .. in sequence, as a right-looking potrf does: an exactly singular block then ends
  // with the same pivot rounding as LAPACK's column order, tests/test_gpu.py::
  // test_not_positive_definite_raises_like_numpy). The entry q+1 (the next pivot's, on the chain)
  // takes L(q+1, q) by v_readlane; the entries s >= q+2 by DPP: m of lanes 0..15 is copied to the
  // other three rows of 16 lanes (two permlane swaps per 32-bit half), and each entry is one
  // v_fmac_f64 whose first operand is row_newbcast:s of that copy — lane s of the lane's own row,
  // i.e. L(s, q) in every row — in place of two v_readlane, the SGPR hazard wait and a v_fma.
  // Measured per column on wave 0 alone (probe, profiles/r5/f128_*.txt): 299 cycles with the
  // selects gone and the loads batched; the register-only column loop is 187, its pivot chain alone
  // 124. Rejected: the pivot chain's 1/sqrt interleaved with the updates by scheduling barriers
  // (465 vs 426 at the time), one column deferred through an LDS broadcast buffer (439-441), the
  // chain on uniform values one step ahead (456-460; with one Newton step 439-443).
  double inv;
  {
    const double p0 = readlane_f64(x[0], 0);
    bad = !(p0 > 0.0);
    inv = rsqrt_nr(p0);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const double m = (arow && r < q) ? 0.0 : x[q] * inv;
    x[q] = m;
    if (q == 15) break;
    x[q + 1] = fma(-m, readlane_f64(m, q + 1), x[q + 1]);
    const double pn = readlane_f64(x[q + 1], q + 1);
    bad = bad | !(pn > 0.0);
    inv = rsqrt_nr(pn);
    if (q + 2 < 16) {
      db_fmac_bcast_from<2>(q, x, row0_to_rows(m), m);
    }
  }
  if (xcol) {  // X_kk: lane 16 + c holds column c
    const int c = r - 16;
#pragma unroll
    for (int s = 0; s < 16; ++s) blk[db_off(s, c)] = x[s];
  }
  if (ylane) {
#pragma unroll
    for (int s = 0; s < 16; ++s) lds[DB_Y + 16 * k + s] = x[s];
  }
  return bad;
}
// The panel's global stores: L_kk (zeros above the diagonal) and X_kk (U_kk). Issued after the
// barrier that hands X_kk to Q_k (db_path_panel), so they drain while wave 4 runs Q_k's chain row
// instead of ahead of the barrier (-4.4% cycles per factor on the f128 probe,
// profiles/r6/f128_q_chain_late_stores.txt; X_kk stored by its column's owner wave instead, on
// another SIMD, measured no better and was dropped).
template <bool WT>
__device__ __forceinline__ void db_panel_gst(int k, const double (&x)[16], double* __restrict__ Lt, double* __restrict__ Ut,
                                             size_t ld) {
  const int r = threadIdx.x & 63;
  // (the diagonal row's own entries right of its pivot took updates with m = L(q, q): not stored)
  if (r < 16 && (GPF_DB_PANEL_GST & 1)) {
    double* gl = Lt + (size_t)(16 * k + r) * ld + 16 * k;
#pragma unroll
    for (int c = 0; c < 16; c += 2) *reinterpret_cast<d2*>(gl + c) = d2{c <= r ? x[c] : 0.0, c + 1 <= r ? x[c + 1] : 0.0};
  }
  if (r >= 16 && r < 32 && (GPF_DB_PANEL_GST & 2)) {
    double* gu = Ut + (size_t)(16 * k) * ld + 16 * k + (r - 16);
#pragma unroll
    for (int s = 0; s < 16; ++s) gst<WT>(gu + (size_t)s * ld, x[s]);
  }
}
// the panel with its stores in line (the probes)
template <bool WT>
__device__ __forceinline__ bool db_panel(double* lds, int k, double* __restrict__ Lt, double* __restrict__ Ut, size_t ld) {
  double x[16];
  const bool bad = db_panel_core(lds, k, x);
  db_panel_gst<WT>(k, x, Lt, Ut, ld);
  return bad;
}

#ifndef GPF_Q_CHAIN_FIRST  // 0: Q_k's row k+1 forms the y update before the next diagonal block
#define GPF_Q_CHAIN_FIRST 1
#endif
// Q_k, block row i > k: L(i,k)^T = X_kk A(i,k)^T (the B operand A(i,k)^T is the A-operand read of
// A(i,k)), y_i -= L(i,k) z_k, L(i,k) to LDS and L; row k+1 then updates the next diagonal block
// A(k+1,k+1) -= L(k+1,k) L(k+1,k)^T (its A operand: the rows just stored, read back by this wave).
template <bool WT>
__device__ __forceinline__ void db_q_item(double* lds, int k, int i, double* __restrict__ Lt, size_t ld) {
  const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
  auto B = [&](int ii, int jj) { return lds + db_bid(ii, jj) * DB_BLK; };
  double* Aik = B(i, k);
  double xa[4], ab[4];
  db_opa(B(k, k), xa);
  db_opa(Aik, ab);
  d4 cnext = {0.0, 0.0, 0.0, 0.0};
  if (i == k + 1) cnext = db_ld(B(i, i));  // (read with the operands: off the chain below)
  d4 lt = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) lt = mfma(xa[s], ab[s], lt);
#if GPF_Q_CHAIN_FIRST
  // Row k+1 (the chain into panel k+1): the next diagonal block's MFMAs issue first, so that the
  // y update's VALU work and lane sums below run while they execute instead of ahead of them.
  d4 acc = cnext;
  if (i == k + 1) {
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma_neg_a(lt[s], lt[s], acc);
  }
#endif
  // y_i -= L(i,k) z_k: lane (g, c) holds L(i,k)(c, 4e + g)
  double yp = 0.0;
#pragma unroll
  for (int e = 0; e < 4; ++e) yp = fma(lt[e], lds[DB_Y + 16 * k + 4 * e + g], yp);
  yp = sum_lane_groups(yp);
#if GPF_Q_CHAIN_FIRST
  if (i == k + 1) db_st(B(i, i), acc);
  if (g == 0) lds[DB_Y + 16 * i + c] = lds[DB_Y + 16 * i + c] - yp;
  db_st_t(Aik, lt);  // L(i,k) for the trailing updates and the inverse
#else
  db_st_t(Aik, lt);  // L(i,k) for the trailing updates and the inverse
  if (g == 0) lds[DB_Y + 16 * i + c] = lds[DB_Y + 16 * i + c] - yp;
  if (i == k + 1) {
    // (the A operand of k-step s, L(r, 4 s + g) at lane (g, r), is lt[s] itself — the same lane
    // mapping as the B operand: no LDS round trip through the rows just stored, on the chain)
    d4 acc = cnext;
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma_neg_a(lt[s], lt[s], acc);
    db_st(B(i, i), acc);
  }
#endif
  double* gl = Lt + (size_t)(16 * i + c) * ld + 16 * k + g;
#pragma unroll
  for (int e = 0; e < 4; ++e) gl[4 * e] = lt[e];
}

// Column j of X = L^-1 on its owner wave: S_ij (i > t) and the current X_tj in registers
// (accumulator layout), the column partials (colsum(X o X), X^T z) per lane.
struct DbCol {
  d4 x[8];        // block i of column j: S_ij until step i finalises it, then X_ij
  double s2, sz;  // lane (g, c): partial sums over the rows 4 e + g of column c's finalised blocks
};

// Step t of the inverse for column j (compile-time t, j; j <= t): finalise X_tj, store it, add its
// partials, and the contributions S_ij += L(i,t) X_tj (i > t)
template <bool WT, int t, int j>
__device__ __forceinline__ void db_x_step(DbCol& col, double* lds, double* __restrict__ Ut, size_t ld) {
  const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
  auto B = [&](int i, int jj) { return lds + db_bid(i, jj) * DB_BLK; };
  if constexpr (j == t) {  // the column's first step: X_tt from the panel, empty sums
    col.x[t] = db_ld(B(t, t));
#pragma unroll
    for (int i = t + 1; i < 8; ++i) col.x[i] = d4{0.0, 0.0, 0.0, 0.0};
    col.s2 = 0.0;
    col.sz = 0.0;
  } else {
    col.x[t] = db_mul_ax<true>(d4{0.0, 0.0, 0.0, 0.0}, B(t, t), col.x[t]);  // X_tj = -X_tt S_tj
    double* gu = Ut + (size_t)(16 * t + g) * ld + 16 * j + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) gst<WT>(gu + (size_t)(4 * e) * ld, col.x[t][e]);
  }
  // (one product at a time: the scheduler would otherwise hoist every product's operand reads
  // ahead of the MFMAs and spill the column's accumulators; the SIMD's other wave fills the gaps)
#pragma unroll
  for (int i = t + 1; i < 8; ++i) {
    col.x[i] = db_mul_ax<false>(col.x[i], B(i, t), col.x[t]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the column partials of X_tj (after the contributions: fewer registers live)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const double v = col.x[t][e];
    col.s2 = fma(v, v, col.s2);
    col.sz = fma(v, lds[DB_Y + 16 * t + 4 * e + g], col.sz);
  }
  // (formed here: sunk to the end, the sums kept every finalised block of the column live)
  asm volatile("" : "+v"(col.s2), "+v"(col.sz));
}

// the columns of X wave W owns: at most two (db_col_wave)
__host__ __device__ constexpr int db_col_of(int W, int n) {
  int m = 0;
  for (int j = 0; j < 8; ++j)
    if (db_col_wave(j) == W) {
      if (m == n) return j;
      ++m;
    }
  return -1;
}

// the trailing update of step k beside panel k+1 (db_in_bulk): the blocks wave W owns
template <int k, int W>
__device__ __forceinline__ void db_bulk(double* lds) {
  auto B = [&](int i, int j) { return lds + db_bid(i, j) * DB_BLK; };
#pragma unroll
  for (int i = k + 1; i < 8; ++i)
#pragma unroll
    for (int j = k + 1; j <= i; ++j)
      if constexpr (true) {
        if (db_in_bulk(k, i, j) && db_bulk_wave(k, i, j) == W) {
          double* C = B(i, j);
          db_st(C, db_sub_abt(db_ld(C), B(i, k), B(j, k)));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
}

template <bool WT, int k, int W>
__device__ __forceinline__ void db_q(double* lds, double* __restrict__ Lt, size_t ld) {
#pragma unroll
  for (int i = k + 1; i < 8; ++i)
    if constexpr (true) {
      if (db_q_wave(k, i) == W) db_q_item<WT>(lds, k, i, Lt, ld);
    }
}

// Each wave runs its own path (a compile-time wave: every ownership decision is static, so no
// column's registers are merged across other waves' branches); all paths pass the same barriers:
// one after the load, two per step (one after the last panel), and the publish's.
template <bool WT>
__device__ __forceinline__ void db_publish(double* __restrict__ yseg, const double* lds, int* pub, int pub_val) {
  if (threadIdx.x < T) gst<WT>(&yseg[threadIdx.x], lds[DB_Y + threadIdx.x]);  // z (final since the last panel)
  if (pub) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's U and z stores drained
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(pub, pub_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wave 0's path: the 8 panels as a runtime loop over one copy of the panel code (no Q items are
// wave 0's: db_q_wave). Unrolled per k (r5 first version) the path was ~8 x 8 KiB of straight-line
// code, every panel fetched cold: in situ a panel cost ~60% more than the same code looping alone
// (profiles/r5/f128_*.txt).
template <bool WT>
__device__ __forceinline__ void db_path_panel(double* lds, double* __restrict__ Lt, double* __restrict__ Ut, size_t ld,
                                              double* __restrict__ yseg, int* __restrict__ info, int* pub, int pub_val) {
  bool bad = false;
#pragma unroll 1
  for (int k = 0; k < 8; ++k) {
#if GPF_PANEL_GST_LATE
    double x[16];
    bad = db_panel_core(lds, k, x) | bad;
    DB_STAMP(0, 2 * k);
    lsync();
    db_panel_gst<WT>(k, x, Lt, Ut, ld);
#else
    bad = db_panel<WT>(lds, k, Lt, Ut, ld) | bad;
    DB_STAMP(0, 2 * k);
    lsync();
#endif
    if (k < 7) {
      DB_STAMP(0, 2 * k + 1);
      lsync();
    }
  }
  db_publish<WT>(yseg, lds, pub, pub_val);
  DB_STAMP(0, 16);
  // (the pivots are wave-uniform) an atomic OR: other workgroups of the launch may set the timeout
  // bit of the same word concurrently (a plain read-modify-write could erase it)
  if (bad && threadIdx.x == 0) __hip_atomic_fetch_or(info, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool WT, int k, int W>
__device__ __forceinline__ void db_step_other(double* lds, DbCol& c0, DbCol& c1, double* __restrict__ Lt,
                                              double* __restrict__ Ut, size_t ld) {
  constexpr int J0 = db_col_of(W, 0), J1 = db_col_of(W, 1);
  if constexpr (k >= 1 && W != 4) {
    db_bulk<k - 1, W>(lds);
    if constexpr (J0 >= 0 && J0 <= k - 1) db_x_step<WT, k - 1, J0>(c0, lds, Ut, ld);
    if constexpr (J1 >= 0 && J1 <= k - 1) db_x_step<WT, k - 1, J1>(c1, lds, Ut, ld);
  }
  DB_STAMP(W, 2 * k);
  lsync();
  if constexpr (k < 7) {
    db_q<WT, k, W>(lds, Lt, ld);
    DB_STAMP(W, 2 * k + 1);
    lsync();
  }
}

template <bool WT, int W>
__device__ __forceinline__ void db_path_other(double* lds, double* __restrict__ Lt, double* __restrict__ Ut, size_t ld,
                                              double* __restrict__ yseg, double* __restrict__ s2o,
                                              double* __restrict__ szo, int* pub, int pub_val) {
  constexpr int J0 = db_col_of(W, 0), J1 = db_col_of(W, 1);
  DbCol c0, c1;
  db_step_other<WT, 0, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 1, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 2, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 3, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 4, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 5, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 6, W>(lds, c0, c1, Lt, Ut, ld);
  db_step_other<WT, 7, W>(lds, c0, c1, Lt, Ut, ld);
  // the last inverse step (X_7j = -X_77 S_7j)
  if constexpr (J0 >= 0) db_x_step<WT, 7, J0>(c0, lds, Ut, ld);
  if constexpr (J1 >= 0) db_x_step<WT, 7, J1>(c1, lds, Ut, ld);
  DB_STAMP(W, 16);
  db_publish<WT>(yseg, lds, pub, pub_val);
  // column partials (after the publish: the launch's tiles do not read them): lane (g, c) holds
  // rows 4 e + g of every block of the column
  const int lane = threadIdx.x & 63;
  if constexpr (J0 >= 0) {
    const double a2 = sum_lane_groups(c0.s2), az = sum_lane_groups(c0.sz);
    if (lane < 16) {
      s2o[16 * J0 + lane] = a2;
      szo[16 * J0 + lane] = az;
    }
  }
  if constexpr (J1 >= 0) {
    const double a2 = sum_lane_groups(c1.s2), az = sum_lane_groups(c1.sz);
    if (lane < 16) {
      s2o[16 * J1 + lane] = a2;
      szo[16 * J1 + lane] = az;
    }
  }
}

// The diagonal block at Lt / Ut (row stride ld): in: Lt's lower 128 x 128 (A, fully reduced),
// yseg (y, fully reduced); out: Lt = L (zeros above the diagonal), Ut = L^-1 (likewise), yseg = z,
// s2o / szo = the column partials. lds: DB_LDS doubles. WT: write-through U and z (read by other
// workgroups of the launch after pub). pub (nullable): set to pub_val once U and z are stored and
// drained, before the partials. info gets 1 on a pivot that is not > 0.
template <bool WT = false>
__device__ __forceinline__ void factor128(double* __restrict__ Lt, double* __restrict__ Ut, size_t ld,
                                          double* __restrict__ yseg, double* __restrict__ s2o, double* __restrict__ szo,
                                          int* __restrict__ info, double* lds, int* pub = nullptr, int pub_val = 0) {
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // A's 36 lower blocks -> LDS (16 B per lane from memory), y -> LDS
  {
    const double* A = launder(Lt);
    int to = tid;
    asm volatile("" : "+v"(to));  // (the thread's load decode is formed here, not hoisted into the caller and spilled)
#pragma unroll
    for (int u = 0; u < (DB_NB * 16 * 8) / DNTH; ++u) {
      const int q = to + DNTH * u, row = q >> 3, cp = q & 7;  // block row `row` (0..575), pair cp
      int bi = 0, rem = row;
#pragma unroll
      for (int t = 1; t < 8; ++t)
        if (rem >= 16 * t) {
          rem -= 16 * t;
          bi = t;
        }
      const int bj = rem >> 4, rr = rem & 15;
      const d2 v = *reinterpret_cast<const d2*>(A + (size_t)(16 * bi + rr) * ld + 16 * bj + 2 * cp);
      double* s = lds + db_bid(bi, bj) * DB_BLK + db_off(rr, 2 * cp);
      s[0] = v.x;
      s[1] = v.y;
    }
    if (tid < T) lds[DB_Y + tid] = yseg[tid];
    if (tid < 32) lds[DB_UNIT + tid] = tid == 15 ? 1.0 : 0.0;
  }
  // zeros above the diagonal blocks of L and U (wave 4: idle otherwise; nothing reads them here)
  if (wave == 4) {
    const int lane = tid & 63;
    for (int t = 0; t < 7; ++t)
      for (int q = lane; q < 16 * 8 * (7 - t); q += 64) {  // rows 16t.., columns 16(t+1)..127, pairs
        const int rr = q / (8 * (7 - t)), cp = q % (8 * (7 - t));
        const size_t o = (size_t)(16 * t + rr) * ld + 16 * (t + 1) + 2 * cp;
        *reinterpret_cast<d2*>(Lt + o) = d2{0.0, 0.0};
        gst<WT>(Ut + o, 0.0);
        gst<WT>(Ut + o + 1, 0.0);
      }
  }
  DB_STAMP(0, 17);
  lsync();
  switch (wave) {
    case 0: db_path_panel<WT>(lds, Lt, Ut, ld, yseg, info, pub, pub_val); break;
    case 1: db_path_other<WT, 1>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
    case 2: db_path_other<WT, 2>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
    case 3: db_path_other<WT, 3>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
    case 4: db_path_other<WT, 4>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
    case 5: db_path_other<WT, 5>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
    case 6: db_path_other<WT, 6>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
    default: db_path_other<WT, 7>(lds, Lt, Ut, ld, yseg, s2o, szo, pub, pub_val); break;
  }
}

}  // namespace gpf
