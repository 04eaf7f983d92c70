// gpf_factor.hip — batched left-looking Cholesky + triangular inverse on gfx950.
//
// Reference op replaced (per particle, GP_func.py:21-24,38 via find_len_scales.py:159):
//   L = cholesky(K)            LAPACK dpotrf
//   solve(L.T, solve(L, y))    2x LAPACK dgesv on triangular factors
//   solve(L, K_s)              LAPACK dgesv with N right-hand sides
// Here: L = chol(K), U = L^-1 and z = U y, plus the column partials of
// diag(K^-1) = colsum(U o U) and alpha = U^T z, in 2/3 N^3 flops (potrf + trtri)
// instead of the reference's ~4.3 N^3.
//
// Blocking: 128-wide block columns J (T = 128). Launch J (k_step) advances every
// particle of the chunk by one block column:
//   L tiles (I > J):  L_IJ = (A_IJ - L_I,<J L_J,<J^T) U_JJ^T       streamed MFMA GEMM, depth 128 J,
//                     computed transposed and finished from the registers (step_item)
//                     A_II -= L_IJ L_IJ^T ; y_I -= L_IJ z_J         look-ahead (keeps A_II and y current)
//   U tiles (K < J):  U_JK = -U_JJ (L_J,[K,J) U_[K,J),K)           streamed MFMA GEMM, depth 128 (J-K)
// and the workgroup that finishes A_{J+1,J+1} factors it in the same launch (factor128:
// L, U = L^-1 and z of the diagonal block); k_diag does block 0 before the first launch.
// A left-looking step streams each factored panel once per 128 output columns,
// so the GEMMs run at ~32 flop per HBM byte (64-wide columns: ~16, HBM-bound).
// GEMM operands go global -> LDS by direct-to-LDS loads (gemm_stream_dl), and MFMAs on
// known-zero triangles are skipped (Tri in gpf_common.hip).

#pragma once
#include "gpf_common.hip"

namespace gpf {

#ifdef GPF_DIAG_STAMPS
// Diagnostic build only (-DGPF_DIAG_STAMPS): thread 0 of workgroup 0 records s_memtime at
// phase boundaries of factor128 into a buffer nothing else reads.
// [0, 32): factor128 phases and the k = 4 details; [32, 32 + 16 * 16): per panel k of the last
// factor64 call, slot 16 k + s: s < 8 wave s arriving at the panel barrier, 8 wave 0 leaving it,
// 9 wave 0 after its strip update, 10 wave 0 after its panel factor, 11-13 update wave
// DIAG_UW after its block slot j, 14 wave DIAG_UW leaving the barrier
#ifndef DIAG_UW
#define DIAG_UW 4
#endif
constexpr int DIAG_NSTAMPS = 32 + 16 * 16;
__device__ unsigned long long g_diag_stamps[DIAG_NSTAMPS];
#define DIAG_STAMP(i) DIAG_STAMP_T(i, 0)
#define DIAG_STAMP_T(i, thr)                                                                       \
  do {                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    if (threadIdx.x == (thr) && blockIdx.x == 0 && blockIdx.y == 0) {  /* WG (p 0, w 0) */                                \
      unsigned long long t_;                                                                     \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                  \
      g_diag_stamps[i] = t_;                                                                     \
    }                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                           \
  } while (0)
#else
#define DIAG_STAMP(i) \
  do {               \
  } while (0)
#define DIAG_STAMP_T(i, thr) \
  do {                      \
  } while (0)
#endif

// The diagonal-block routines below run on all DNTH (= 512) threads of the
// factorisation workgroups (k_diag and, fused, k_step).

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

constexpr int F64_BUF = 1024;  // LDS scratch of the diagonal factor (>= the 512-double reduction scratch)

// ----------------------------------------------------------------------------
// Blocked 64x64 factor: 16-wide block columns, right-looking.
// Round 2's 4-wide panels passed 17 barriers and put the 4x4 pivot chain, the strip hand-off and
// the update waves' serialised operand loads on every 4 columns (~3.4k cycles per panel,
// profiles/r3/factor64_panel_stamps.txt). Here one wave factors a whole 16-column block column
// (all rows below the diagonal at once, lane = row, registers only), and everything else is
// 16x16x16 MFMA products between LDS blocks on the other waves, two barriers per block column:
//   P1(k): wave 0 factors block column k (rows 16k..63) -> L_{.,k};   other waves, off the
//          chain: the trailing updates of columns >= k+1 by block column k-1, X_{k-1,k-1} =
//          L_{k-1,k-1}^-1 (one lane per column, forward substitution) and the inverse's products
//   P2(k): the chain: A_{i,k+1} -= L_ik L_{k+1,k}^T (i > k, one wave per block); inverse products
// then three short phases finish the last block row of X = L^-1:
//   X_ij = -X_ii sum_{t=j}^{i-1} L_it X_tj   (block back-substitution, accumulated in X's blocks)
// Deterministic (a fixed assignment of blocks to waves); not bitwise the 4-wide panels' result.
// Waves w and w+4 share a SIMD: while wave 0 factors a block column, wave 4 stays idle and the
// longest side job (the 16x16 inversion) runs on wave 6.
// ----------------------------------------------------------------------------

// D (+)= (NEG ? -1 : 1) A B for 16x16 blocks in LDS: A row-major [r][k] at pa; B as [k][c] at pb
// (BT = false) or given transposed, Bt[c][k] at pb (BT = true); D row-major at pc (ACC: D is
// also the addend). One wave.
template <bool BT, bool NEG, bool ACC>
__device__ __forceinline__ void mm16(double* pc, int ldc, const double* pa, int lda, const double* pb, int ldb) {
  const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
  double a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a[s] = pa[lr * lda + 4 * s + lk];
    b[s] = BT ? pb[lr * ldb + 4 * s + lk] : pb[(4 * s + lk) * ldb + lr];
  }
  d4 acc;
#pragma unroll
  for (int e = 0; e < 4; ++e) acc[e] = ACC ? pc[(lk + 4 * e) * ldc + lr] : 0.0;
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = NEG ? mfma_neg_a(a[s], b[s], acc) : mfma(a[s], b[s], acc);
#pragma unroll
  for (int e = 0; e < 4; ++e) pc[(lk + 4 * e) * ldc + lr] = acc[e];
}

// Block column k (rows 16k..63, columns 16k..16k+15, fully updated by the earlier columns) on one
// wave: lane r holds row 16k + r. Column by column: pivot from lane q (readlane), 1/sqrt by
// v_rsq + Newton, scale the column, rank-1 update of the lane's row (one fma per entry) with the
// column's other diagonal-block entries (readlanes, a few per scheduling region: the scheduler
// would otherwise hoist a column's readlanes together and spill the scalar registers; an LDS
// column buffer instead measured more vector spills inside k_step). Writes L (zeros above the
// diagonal of block (k,k)) and the pivots' reciprocal square roots dinv[16k + q]. Returns whether
// a pivot was not > 0.
__device__ __forceinline__ bool f64b_column(double* sA, int la, int k, double* dinv) {
  const int r = threadIdx.x & 63;
  const int R = 16 * k + r;
  const bool live = R < 64;
  double* row = sA + (live ? R : 0) * la + 16 * k;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = (live && (r >= 16 || c <= r)) ? row[c] : 0.0;
  bool bad = false;
  double myinv = 0.0;  // lane q: the reciprocal square root of pivot q
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const double p = readlane_f64(a[q], q);
    bad = bad | !(p > 0.0);
    const double inv = rsqrt_nr(p);
    const double l = (r > q) ? a[q] * inv : ((r == q) ? p * inv : 0.0);
    a[q] = l;
    myinv = (r == q) ? inv : myinv;
#pragma unroll
    for (int s = q + 1; s < 16; ++s) {
      a[s] = fma(-l, readlane_f64(l, s), a[s]);
      if (((s - q) & 3) == 0) __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (r < 16) dinv[16 * k + r] = myinv;
  if (live) {
#pragma unroll
    for (int c = 0; c < 16; ++c) row[c] = (r < 16 && c > r) ? 0.0 : a[c];
  }
  return bad;
}

// X_kk = L_kk^-1 of a 16x16 lower-triangular block (zeros above its diagonal in LDS): lane c
// (c < 16) forward-substitutes column c, x_i = -(sum_{j<i} L_ij x_j) * dinv_i, x_c = dinv_c (the
// [A | I] elimination's X_qq); the L entries are uniform LDS reads. One wave; writes zeros above
// the diagonal of X_kk. (A column-oriented variant, every later row taking x_j's term at once,
// spilled inside k_step.)
__device__ __forceinline__ void f64b_inv(const double* sL, int la, double* sXo, int lx, const double* dv) {
  const int lane = threadIdx.x & 63, c = lane & 15;
  double x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double dot = 0.0;
#pragma unroll
    for (int j = 0; j < i; ++j) dot = fma(sL[i * la + j], x[j], dot);
    x[i] = (i < c) ? 0.0 : ((i == c) ? dv[i] : -dot * dv[i]);
    __builtin_amdgcn_sched_barrier(0);  // a row of uniform L reads per region (register budget)
  }
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) sXo[i * lx + c] = x[i];
  }
}

__device__ __forceinline__ bool factor64_blocked(double* sA, int la, double* sX, int lx, double* buf) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* dinv = buf;  // [64]
  auto Ab = [&](int i, int j) { return sA + 16 * i * la + 16 * j; };
  auto Xb = [&](int i, int j) { return sX + 16 * i * lx + 16 * j; };
  bool bad = false;
  DIAG_STAMP_T(31, 0);
  // P1(0) / P2(0)
  if (wave == 0) {
    bad = f64b_column(sA, la, 0, dinv);
    DIAG_STAMP_T(41, 0);
  }
  lsync();
  DIAG_STAMP_T(32, 0);  // (diagnostic build) thread 0 leaves barrier 0
  if (wave >= 1 && wave <= 3) mm16<true, true, true>(Ab(wave, 1), la, Ab(wave, 0), la, Ab(1, 0), la);  // A_i1 -= L_i0 L_10^T
  lsync();
  DIAG_STAMP_T(33, 0);  // (diagnostic build) thread 0 leaves barrier 1
  // P1(1): column 1 | X_00, A_22 / A_32 / A_33 -= (column 0 terms)
  if (wave == 0) {
    bad = f64b_column(sA, la, 1, dinv) | bad;
    DIAG_STAMP_T(42, 0);
  }
  else if (wave == 1) mm16<true, true, true>(Ab(2, 2), la, Ab(2, 0), la, Ab(2, 0), la);
  else if (wave == 2) mm16<true, true, true>(Ab(3, 2), la, Ab(3, 0), la, Ab(2, 0), la);
  else if (wave == 3) mm16<true, true, true>(Ab(3, 3), la, Ab(3, 0), la, Ab(3, 0), la);
  else if (wave == 6) f64b_inv(Ab(0, 0), la, Xb(0, 0), lx, dinv);
  lsync();
  DIAG_STAMP_T(34, 0);  // (diagnostic build) thread 0 leaves barrier 2
  // P2(1): A_i2 -= L_i1 L_21^T | Xcur_i0 = L_i0 X_00
  if (wave == 1 || wave == 2) mm16<true, true, true>(Ab(wave + 1, 2), la, Ab(wave + 1, 1), la, Ab(2, 1), la);
  else if (wave >= 4 && wave <= 6) mm16<false, false, false>(Xb(wave - 3, 0), lx, Ab(wave - 3, 0), la, Xb(0, 0), lx);
  lsync();
  DIAG_STAMP_T(35, 0);  // (diagnostic build) thread 0 leaves barrier 3
  // P1(2): column 2 | X_11, A_33 -= L_31 L_31^T
  if (wave == 0) {
    bad = f64b_column(sA, la, 2, dinv) | bad;
    DIAG_STAMP_T(43, 0);
  }
  else if (wave == 3) mm16<true, true, true>(Ab(3, 3), la, Ab(3, 1), la, Ab(3, 1), la);
  else if (wave == 6) f64b_inv(Ab(1, 1), la, Xb(1, 1), lx, dinv + 16);
  lsync();
  DIAG_STAMP_T(36, 0);  // (diagnostic build) thread 0 leaves barrier 4
  // P2(2): A_33 -= L_32 L_32^T | X_10 = -X_11 Xcur_10, Xcur_21 = L_21 X_11, Xcur_31 = L_31 X_11
  if (wave == 1) mm16<true, true, true>(Ab(3, 3), la, Ab(3, 2), la, Ab(3, 2), la);
  else if (wave == 4) mm16<false, true, false>(Xb(1, 0), lx, Xb(1, 1), lx, Xb(1, 0), lx);
  else if (wave == 5) mm16<false, false, false>(Xb(2, 1), lx, Ab(2, 1), la, Xb(1, 1), lx);
  else if (wave == 6) mm16<false, false, false>(Xb(3, 1), lx, Ab(3, 1), la, Xb(1, 1), lx);
  lsync();
  DIAG_STAMP_T(37, 0);  // (diagnostic build) thread 0 leaves barrier 5
  // P1(3): column 3 | X_22, Xcur_20 += L_21 X_10, Xcur_30 += L_31 X_10
  if (wave == 0) {
    bad = f64b_column(sA, la, 3, dinv) | bad;
    DIAG_STAMP_T(44, 0);
  }
  else if (wave == 6) f64b_inv(Ab(2, 2), la, Xb(2, 2), lx, dinv + 32);
  else if (wave == 5) mm16<false, false, true>(Xb(2, 0), lx, Ab(2, 1), la, Xb(1, 0), lx);
  else if (wave == 7) mm16<false, false, true>(Xb(3, 0), lx, Ab(3, 1), la, Xb(1, 0), lx);
  lsync();
  DIAG_STAMP_T(38, 0);  // (diagnostic build) thread 0 leaves barrier 6
  // T1: X_33 | X_20 = -X_22 Xcur_20, X_21 = -X_22 Xcur_21, Xcur_32 = L_32 X_22
  if (wave == 4) f64b_inv(Ab(3, 3), la, Xb(3, 3), lx, dinv + 48);
  else if (wave == 5) mm16<false, true, false>(Xb(2, 0), lx, Xb(2, 2), lx, Xb(2, 0), lx);
  else if (wave == 6) mm16<false, true, false>(Xb(2, 1), lx, Xb(2, 2), lx, Xb(2, 1), lx);
  else if (wave == 7) mm16<false, false, false>(Xb(3, 2), lx, Ab(3, 2), la, Xb(2, 2), lx);
  lsync();
  DIAG_STAMP_T(39, 0);  // (diagnostic build) thread 0 leaves barrier 7
  // T2: Xcur_30 += L_32 X_20, Xcur_31 += L_32 X_21
  if (wave == 5 || wave == 6) mm16<false, false, true>(Xb(3, wave - 5), lx, Ab(3, 2), la, Xb(2, wave - 5), lx);
  lsync();
  DIAG_STAMP_T(40, 0);  // (diagnostic build) thread 0 leaves barrier 8
  // T3: X_3j = -X_33 Xcur_3j; zeros above the diagonal blocks of L and X
  if (wave >= 5) mm16<false, true, false>(Xb(3, wave - 5), lx, Xb(3, 3), lx, Xb(3, wave - 5), lx);
#pragma unroll
  for (int u = 0; u < 6 * 256 / DNTH; ++u) {
    const int i = threadIdx.x + DNTH * u;
    const int t = i >> 8, e = i & 255;  // upper blocks (0,1) (0,2) (0,3) (1,2) (1,3) (2,3)
    const int bi = (t < 3) ? 0 : (t < 5) ? 1 : 2;
    const int bj = (t < 3) ? t + 1 : (t < 5) ? t - 1 : 3;
    const int rr = 16 * bi + (e >> 4), cc = 16 * bj + (e & 15);
    sA[rr * la + cc] = 0.0;
    sX[rr * lx + cc] = 0.0;
  }
  return bad;
}

__device__ __forceinline__ bool factor64(double* sA, int la, double* sX, int lx, double* buf) {
  return factor64_blocked(sA, la, sX, lx, buf);
}

// Fixed-order sum of the 8 partials scratch[q*64 + i], q = 0..7.
__device__ __forceinline__ double sum8(const double* scratch, int i) {
  return (((scratch[i] + scratch[64 + i]) + (scratch[128 + i] + scratch[192 + i])) +
          ((scratch[256 + i] + scratch[320 + i]) + (scratch[384 + i] + scratch[448 + i])));
}

// out[r] = (sum_c s1[r][c] v1[c]) for r < 64 (or out[r] -= that); 8 partial sums
// per row combined in fixed order. Ends with a barrier.
__device__ __forceinline__ void rows_dot64(double* out, const double* s1, int l1, const double* v1, double* scratch,
                                           bool accumulate) {
  const int tid = threadIdx.x;
  const int r = tid & 63, q = tid >> 6;
  double acc = 0.0;
  for (int c = q * 8; c < q * 8 + 8; ++c) acc = fma(s1[r * l1 + c], v1[c], acc);
  scratch[q * 64 + r] = acc;
  lsync();
  if (tid < 64) {
    const double s = sum8(scratch, tid);
    out[tid] = accumulate ? out[tid] - s : s;
  }
  lsync();
}

// Column partials of a 64x64 LDS tile s (rows r, cols c): s2[c] += sum_r s^2,
// sz[c] += sum_r s * z[r]. Fixed order. Ends with a barrier. scratch: 512 doubles.
__device__ __forceinline__ void cols_partial64(double* s2, double* sz, const double* s, int ls, const double* z,
                                               double* scratch) {
  const int tid = threadIdx.x;
  const int c = tid & 63, q = tid >> 6;
  double a2 = 0.0, az = 0.0;
  for (int r = q * 8; r < q * 8 + 8; ++r) {
    const double v = s[r * ls + c];
    a2 = fma(v, v, a2);
    az = fma(v, z[r], az);
  }
  scratch[q * 64 + c] = a2;
  lsync();
  if (tid < 64) s2[tid] = s2[tid] + sum8(scratch, tid);
  lsync();
  scratch[q * 64 + c] = az;
  lsync();
  if (tid < 64) sz[tid] = sz[tid] + sum8(scratch, tid);
  lsync();
}

struct DiagSmem {
  double* t0;       // 64 x LDH
  double* t1;       // 64 x LDH
  double* y;        // 128
  double* z;        // 128
  double* ps2;      // 128
  double* psz;      // 128
  double* scratch;  // DIAG_SMALL (>= 512)
};

// ----------------------------------------------------------------------------
// Factor one fully reduced 128x128 diagonal block in place (2x2 blocks of 64):
//   L11,U11 = factor64(A11) ; L21 = A21 U11^T ; A22 -= L21 L21^T ; L22,U22 = factor64(A22)
//   U21 = -U22 (L21 U11) ; z = L^-1 y by forward substitution ; partials of colsum(U^2),
//   U^T z for the 128 columns.
// Lt/Ut: top-left of the block in the particle's L / U buffers (row stride ld);
// yseg: the block's 128 RHS entries (replaced by z); s2o/szo: 128 partial outputs.
// ----------------------------------------------------------------------------
// pub (the early diagonal factor, WT = true): the per-particle flag to set to pub_val once U_JJ
// and z_J — all a tile of the launch reads — are stored (write-through) and drained; the column
// partials of the block (read only after the launch) are formed after the flag ("early publish").
template <bool WT = false>
__device__ __forceinline__ void factor128(double* __restrict__ Lt, double* __restrict__ Ut, size_t ld,
                                          double* __restrict__ yseg, double* __restrict__ s2o,
                                          double* __restrict__ szo, int* __restrict__ info, const DiagSmem& sm,
                                          bool pad2, int* pub = nullptr, int pub_val = 0) {
  const int tid = threadIdx.x;
  const Quad<64> qd;
  double* const t0 = sm.t0;
  double* const t1 = sm.t1;

  DIAG_STAMP(0);
  // (a) L11, U11, z1
  tile64_to_lds(t0, LDH, Lt, ld);
  if (tid < T) {
    sm.y[tid] = yseg[tid];
    sm.ps2[tid] = 0.0;
    sm.psz[tid] = 0.0;
  }
  lsync();
  bool bad = factor64(t0, LDH, t1, LDH, sm.scratch);
  lsync();
  DIAG_STAMP(1);
  lds_to_tile64(Lt, ld, t0, LDH, true);
  zero_tile64(Lt + H, ld);
  lds_to_tile64<WT>(Ut, ld, t1, LDH, false);
  zero_tile64<WT>(Ut + H, ld);
  rows_dot64(sm.z, t1, LDH, sm.y, sm.scratch, false);          // z1 = U11 y1
  cols_partial64(sm.ps2, sm.psz, t1, LDH, sm.z, sm.scratch);   // U11 columns

  if (pad2) {
    // rows/columns 64..127 of this block are all padding (A21 = 0, A22 = I from the K build and
    // no earlier column touches them): L21 = U21 = 0, L22 = U22 = I, z2 = 0 — exactly what the
    // general path computes, without the second 64x64 factor
    zero_tile64(Lt + (size_t)H * ld, ld);
    zero_tile64<WT>(Ut + (size_t)H * ld, ld);
    for (int i = tid; i < H * H; i += DNTH) {
      const int r = i >> 6, c = i & 63;
      Lt[(size_t)(H + r) * ld + H + c] = (r == c) ? 1.0 : 0.0;
      gst<WT>(&Ut[(size_t)(H + r) * ld + H + c], (r == c) ? 1.0 : 0.0);
    }
    if (tid < T) {
      s2o[tid] = (tid < H) ? sm.ps2[tid] : 1.0;
      szo[tid] = (tid < H) ? sm.psz[tid] : 0.0;
      gst<WT>(&yseg[tid], (tid < H) ? sm.z[tid] : 0.0);
    }
    if (bad && tid == 0 && *info == 0) *info = 1;
    if (pub) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(pub, pub_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  DIAG_STAMP(2);
  // (b) L21 = A21 U11^T; A22 is read into registers now, so its load runs behind (b) and (c)
  double* U21 = Ut + (size_t)H * ld;
  const double* A22 = Lt + (size_t)H * ld + H;
  Acc<64> a22;
  a22.load(qd, A22, ld);
  tile64_to_lds(t0, LDH, Lt + (size_t)H * ld, ld);
  lsync();
  Acc<64> acc;
  acc.zero();
  gemm_lds64<false, TRI_B_KLEC>(acc, t0, LDH, t1, LDH, qd);  // U11^T is upper triangular
  lsync();
  acc.foreach(qd, [&](int r, int c, double v) {
      t0[r * LDH + c] = v;
      Lt[(size_t)(H + r) * ld + c] = v;
    });
  lsync();

  DIAG_STAMP(3);
  // (c) A22 -= L21 L21^T ; y2 -= L21 z1 ; T = L21 U11 (to the U21 slot as scratch)
  acc.zero();
  gemm_lds64<false, TRI_C_LOWER>(acc, t0, LDH, t0, LDH, qd);  // factor64 reads the lower triangle only
  rows_dot64(sm.y + H, t0, LDH, sm.z, sm.scratch, true);
  Acc<64> tt;
  tt.zero();
  gemm_lds64<true, TRI_B_KGEC>(tt, t0, LDH, t1, LDH, qd);  // U11 is lower triangular
  lsync();
  tt.foreach(qd, [&](int r, int c, double v) { gst<WT>(&U21[(size_t)r * ld + c], v); });
#pragma unroll
  for (int mi = 0; mi < Acc<64>::MBR; ++mi)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc.v[mi][0][e] = a22.v[mi][0][e] - acc.v[mi][0][e];
  acc.foreach(qd, [&](int r, int c, double v) { t0[r * LDH + c] = v; });
  lsync();

  DIAG_STAMP(4);
  // (d) L22, U22
  bad = factor64(t0, LDH, t1, LDH, sm.scratch) | bad;
  lsync();
  DIAG_STAMP(5);
  // T (stored to the U21 slot in (c), long drained: the factor ran since) read back into
  // registers first, so the loads run behind the stores of L22 and U22
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  d2 tv[2048 / DNTH];
#pragma unroll
  for (int u = 0; u < 2048 / DNTH; ++u) {
    const int q = tid + DNTH * u, row = q >> 5, c2 = q & 31;
    tv[u] = *reinterpret_cast<const d2*>(U21 + (size_t)row * ld + 2 * c2);
  }
  lds_to_tile64(Lt + (size_t)H * ld + H, ld, t0, LDH, true);
  lds_to_tile64<WT>(Ut + (size_t)H * ld + H, ld, t1, LDH, false);
  lsync();

  DIAG_STAMP(6);
  // (e) U21 = -U22 T
#pragma unroll
  for (int u = 0; u < 2048 / DNTH; ++u) {
    const int q = tid + DNTH * u, row = q >> 5, c2 = q & 31;
    t0[row * LDH + 2 * c2] = tv[u].x;
    t0[row * LDH + 2 * c2 + 1] = tv[u].y;
  }
  lsync();
  acc.zero();
  gemm_lds64<true, TRI_A_KLER>(acc, t1, LDH, t0, LDH, qd);  // U22 is lower triangular
  lsync();
  acc.foreach(qd, [&](int r, int c, double v) {
      t0[r * LDH + c] = -v;
      gst<WT>(&U21[(size_t)r * ld + c], -v);
    });
  lsync();

  DIAG_STAMP(7);
  // (f) forward substitution: z2 = U22 (y2 - L21 z1) (y2 already reduced in (c))
  rows_dot64(sm.z + H, t1, LDH, sm.y + H, sm.scratch, false);
  if (pub) {  // early publish: U_JJ (stored write-through above) and z_J are complete
    if (tid < T) gst<WT>(&yseg[tid], sm.z[tid]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's U_JJ and z_J stores drained
    __syncthreads();
    if (tid == 0) __hip_atomic_store(pub, pub_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  DIAG_STAMP(8);
  // (g) partials: columns 0..63 get the U21 rows, columns 64..127 the U22 rows
  cols_partial64(sm.ps2, sm.psz, t0, LDH, sm.z + H, sm.scratch);
  cols_partial64(sm.ps2 + H, sm.psz + H, t1, LDH, sm.z + H, sm.scratch);
  if (tid < T) {
    s2o[tid] = sm.ps2[tid];
    szo[tid] = sm.psz[tid];
    if (!pub) gst<WT>(&yseg[tid], sm.z[tid]);
  }
  if (bad && tid == 0 && *info == 0) *info = 1;
  DIAG_STAMP(9);
}

// Shared-memory carve-up for the diagonal factor: two 64x64 tiles and the small
// vectors live in `base` (the GEMM staging area, DIAG_BASE doubles), the
// 512-double reduction scratch in `small`.
constexpr int DIAG_BASE = 2 * H * LDH + 4 * T;
constexpr int DIAG_SMALL = F64_BUF;  // factor64's buffers (also >= the 512-double reduction scratch)
__device__ __forceinline__ DiagSmem carve_diag(double* base, double* small) {
  DiagSmem s;
  s.t0 = base;
  s.t1 = base + H * LDH;
  s.y = base + 2 * H * LDH;
  s.z = s.y + T;
  s.ps2 = s.z + T;
  s.psz = s.ps2 + T;
  s.scratch = small;
  return s;
}

// Diagonal block J of every particle (A_JJ already reduced by the look-ahead of
// all earlier block columns). Launched for J = 0 only; every later diagonal
// block is factored inside k_step by the workgroup that finishes reducing it.
// grid: (P)
__global__ __launch_bounds__(DNTH) void k_diag(int J, int nt, int N, int Npad, double* __restrict__ Lb,
                                                  double* __restrict__ Ub, double* __restrict__ yb,
                                                  double* __restrict__ s2p, double* __restrict__ szp,
                                                  int* __restrict__ info, int* __restrict__ dflag) {
  if (threadIdx.x == 0) dflag[blockIdx.x] = J;  // a new factorisation: block J published (launches follow in order)
  __shared__ __attribute__((aligned(16))) double tiles[DIAG_BASE];
  __shared__ __attribute__((aligned(16))) double small[DIAG_SMALL];
  const int p = blockIdx.x;
  const size_t ld = (size_t)Npad;
  const size_t off = (size_t)p * ld * ld + (size_t)J * T * ld + (size_t)J * T;
  const DiagSmem sm = carve_diag(tiles, small);
  const size_t poff = ((size_t)p * nt + J) * Npad + (size_t)J * T;
  factor128(Lb + off, Ub + off, ld, yb + (size_t)p * Npad + J * T, s2p + poff, szp + poff, info + p, sm,
            J * T + H >= N);
}

// ----------------------------------------------------------------------------
// Block column J for every particle. 1-D grid of P*(nt-1) workgroups; a
// workgroup's (particle p, tile w) comes from its linear id (step_tile):
//   w <  nt-1-J : L tile I = J+1+w; the workgroup with I = J+1 (w = 0) then
//                 factors the now fully reduced diagonal block J+1
//   w >= nt-1-J : U tile K = w-(nt-1-J)
// Work per tile falls with w (L tiles and U_0 have depth J, U_K depth J-K).
// The dispatcher deals linear ids round-robin over the 8 XCDs, so with P a
// multiple of 8 every workgroup of particle p lands on XCD p mod 8 (its shared
// B panel is fetched into one L2 only). Within an XCD the ids run in groups of
// `grp` particles, w-major inside a group (longest tile first): grp = P/8 is
// longest-first over the whole launch; smaller groups keep fewer particles'
// B panels live in the 4 MB L2 at a time.
// ----------------------------------------------------------------------------
__host__ __device__ __forceinline__ void step_tile(int b, int P, int ntl, int grp, int& p, int& w) {
  if ((P & 7) != 0 || grp <= 0) {  // particle fastest
    p = b % P;
    w = b / P;
    return;
  }
  const int xcd = b & 7, s = b >> 3, pq = P >> 3;
  const int per = grp * ntl;
  const int gi = s / per, r = s - gi * per;
  const int gs = grp < pq - gi * grp ? grp : pq - gi * grp;  // the last group may be smaller
  w = r / gs;
  p = (gi * grp + (r - w * gs)) * 8 + xcd;
}

enum { SPLIT_NONE = 0, SPLIT_ALL = 1, SPLIT_CRIT = 2 };
enum { ROLE_IDLE = 0, ROLE_WHOLE = 1, ROLE_PIECE = 2, ROLE_DIAG = 3, ROLE_SYRK = 4, ROLE_LA = 5 };

// Early diagonal factor (k_step<SPLIT, ED = 1>; the host chooses it for launches that leave
// workgroup slots idle): launch J starts with P extra workgroups that factor diagonal
// block J (factor128: L_JJ, U_JJ, z_J, the column partials) and publish it through a
// per-particle flag, while every tile of the launch runs the GEMM part of its work; a tile waits
// for the flag only before its first use of U_JJ / z_J. The diagonal factor (~55 us on one
// workgroup) then overlaps the launch's GEMMs instead of closing the previous launch's critical
// tile (I = J+1) in series. Launch 0 factors block 0 the same way (k_build_cov resets the flags
// to -1). With ED = 0 the critical tile factors block J+1 itself (fused) and k_diag block 0.

// Deferred diagonal update (defer = 1; the factorisations without the all-tile split): instead of
// every L tile applying its rank-128 look-ahead A_II -= L_IJ L_IJ^T in every launch (a
// read-modify-write of a 128 KiB tile per tile and launch, each a short triangular GEMM), launch J
// starts with one SYRK workgroup per particle (1 <= J <= nt-2) that applies all the earlier terms
// to the next diagonal block in one deep GEMM, S = A_{J+1,J+1} - L_{J+1,<J} L_{J+1,<J}^T (its
// inputs are all from earlier launches), and publishes S (write-through, then a per-particle
// flag); the critical tile I = J+1 adds the last term L_{J+1,J} L_{J+1,J}^T once its TRMM is done
// (at J = 0 it is the whole update). The SYRK workgroup runs beside the critical tile's GEMM
// (depth 128 J, ~9/16 of its MFMAs) and is done long before the tile needs S. The other L tiles
// touch no diagonal block. Same MFMAs in the same order per element of A_II: bitwise the
// per-launch look-ahead's values.

// Balanced all-tile split (SPLIT_ALL): tile w of launch J is cut into pieces of about `tgt` 16-deep
// chunks each (the host picks tgt per launch so that the launch fills the CUs once), so every
// piece — the critical tile's included — does about the same work, instead of a fixed number of
// pieces per tile (which gave the deepest tiles the longest pieces: the critical tile's GEMM, not
// the diagonal factor, ended the launch). At most SPLIT_MAXS pieces (the reduction tree's bound).
constexpr int SPLIT_MAXS = 32;
__host__ __device__ __forceinline__ int split_all_chunks(int J, int w, int nt) {
  const int nL = nt - 1 - J;
  return (w < nL ? J : J - (w - nL)) * (T / DL_KC);  // L tile: depth 128J; U tile K: 128(J-K)
}
__host__ __device__ __forceinline__ int split_all_pieces(int J, int w, int nt, int tgt) {
  const int ch = split_all_chunks(J, w, nt);
  const int s = ch <= 0 ? 1 : (ch + tgt - 1) / tgt;
  return s > SPLIT_MAXS ? SPLIT_MAXS : s;
}

// Workgroup b of a k_step<SPLIT> launch (grid: [P diagonal workgroups if ed] + [P SYRK workgroups
// if sy] + P * sum_w split_all_pieces(J, w, nt, S) for SPLIT_ALL (tiles in order w = 0, 1, ..:
// the critical tile first, then the L tiles, then the U tiles deepest first; pieces particle-
// fastest), P*(nt-1) + P*(S-1) for SPLIT_CRIT, P*(nt-1) otherwise): its
// particle p, tile w, split index sidx, and whether it factors the diagonal block (ROLE_DIAG,
// w = -1), reduces the next diagonal block (ROLE_SYRK, w = -1), runs the whole tile, one depth
// range (piece sidx of S) of it, or nothing. The kernel and the host-side plan check
// (gpf_plan_check) both decode through this function.
// ro (r4, "reordered"; launches with diagonal and SYRK workgroups, no split, particle-fastest
// tiles): the dispatcher deals a launch's workgroups over the CUs in block order, so with more
// workgroups than CUs the last ones land on the CUs of the first — the diagonal workgroups, in the
// order above: every diagonal factor of config B's launches 1..nt-2 shared its CU, 56-61 us instead
// of 46 alone (profiles/r4/diag_coresidence_B.txt). Reordered: first the lightest tile of each
// particle (the U tile K = J-1, one 128-deep block, that then waits for the diagonal block), then
// the SYRK and the diagonal workgroups, then the other tiles, the lightest last, so the CUs that
// take two workgroups pair two light tiles and both chains (the diagonal factor; the SYRK update
// and the look-ahead) run alone. (SYRK workgroups last, paired with the light U tiles, ran the
// diagonal factor alone too but cost B 2%: profiles/r4/diag_coresidence_B_reorder1.txt.)
template <int SPLIT>
__host__ __device__ __forceinline__ int step_decode(int b, int J, int P, int nt, int grp, int S, int ed, int sy, int la,
                                                    int& p, int& w, int& sidx, int ro = 0) {
  const int tiles = P * (nt - 1);
  sidx = 0;
  if (SPLIT == SPLIT_NONE && ro) {  // (ed, sy, J >= 1, grp == 0: gpf_plan_check)
    p = b % P;
    if (b < P) {
      w = nt - 2;  // U tile K = J - 1
      return ROLE_WHOLE;
    }
    if (b < 3 * P) {
      w = -1;
      return b < 2 * P ? ROLE_SYRK : ROLE_DIAG;
    }
    w = (b - 3 * P) / P;  // tiles w = 0 .. nt-3, particle fastest
    return ROLE_WHOLE;
  }
  if (ed) {
    if (b < P) {
      p = b;
      w = -1;
      return ROLE_DIAG;
    }
    b -= P;
  }
  if (sy) {
    if (b < P) {
      p = b;
      w = -1;
      return ROLE_SYRK;
    }
    b -= P;
  }
  if (la) {
    if (b < P) {
      p = b;
      w = -1;
      return ROLE_LA;
    }
    b -= P;
  }
  if (SPLIT == SPLIT_ALL) {  // S: chunks per piece
    int np = 1;
    for (w = 0; w < nt - 2; ++w) {
      np = split_all_pieces(J, w, nt, S);
      if (b < P * np) break;
      b -= P * np;
    }
    if (w == nt - 2) np = split_all_pieces(J, w, nt, S);
    p = b % P;
    sidx = b / P;  // (< np for every dispatched workgroup: gpf_plan_check)
    return np > 1 ? ROLE_PIECE : ROLE_WHOLE;
  } else if (SPLIT == SPLIT_CRIT && b < P * S) {  // the S pieces of the critical tiles
    p = b % P;
    w = 0;
    sidx = b / P;
  } else {  // particle-fastest order (grp = 0) puts the critical tiles w = 0 at b < P
    step_tile(b - (SPLIT == SPLIT_CRIT ? P * (S - 1) : 0), P, nt - 1, grp, p, w);
  }
  const bool ltile = w < nt - 1 - J;
  if (ltile) {
    // L tiles split their depth-128J GEMM (only with the K tiles fused into k_step)
    if (SPLIT == SPLIT_CRIT && w == 0 && J > 0) return ROLE_PIECE;
    return (SPLIT != SPLIT_NONE && sidx > 0) ? ROLE_IDLE : ROLE_WHOLE;  // nothing to split at J = 0
  }
  return (SPLIT == SPLIT_CRIT && sidx > 0) ? ROLE_IDLE : ROLE_WHOLE;  // U tiles never split in CRIT
}

// LDS of a k_step workgroup (doubles): the GEMM stages (DL_STAGE), the diagonal factor
// (DIAG_BASE + DIAG_SMALL), the staged U_JJ of the triangular finishes (TRI_LDS) with z_J behind
// it, or the coordinates of a covariance tile. ~77 KiB: two workgroups per CU.
constexpr int STEP_ZJ = TRI_LDS;  // z_J (128 doubles) beside the staged U_JJ
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int STEP_LDS = cmax(cmax(DL_STAGE, DIAG_BASE + DIAG_SMALL), cmax(STEP_ZJ + T, 2 * DMAX * T + 2 * T));
static_assert(STEP_LDS * 8 <= 80 * 1024, "two k_step workgroups per CU (160 KiB of LDS)");
constexpr int STEP_NTH = Geo<T>::NTH;     // 512 threads: 8 waves, 128x16 per wave
static_assert(STEP_NTH == DNTH, "the fused diagonal runs on the step workgroup");

constexpr int STEP_WAVES_PER_SIMD = 4;  // 2 workgroups of 8 waves per CU
#ifdef GPF_WG_TRACE
// Diagnostic build only (-DGPF_WG_TRACE): per-workgroup start/end (s_memrealtime, 100 MHz)
// and hardware placement of every k_step workgroup, per block column J.
constexpr int WG_TRACE_J = 64, WG_TRACE_N = 4096;
__device__ unsigned long long g_wg_trace[WG_TRACE_J][WG_TRACE_N][3];
__device__ unsigned long long g_wg_phase[WG_TRACE_J][WG_TRACE_N][4];  // wave-0 phase ends (see step_item; [3]: split piece's GEMM before its tree)
__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define GPF_PHASE(k) \
  if (tid == 0 && J < WG_TRACE_J && blockIdx.x < WG_TRACE_N) g_wg_phase[J][blockIdx.x][k] = realtime()
#else
#define GPF_PHASE(k)
#endif

// K(R, C) block of one particle (R != C: no diagonal entries, so no noise term) straight into the
// accumulator layout (rows from block R, columns from block C), with k_build_cov's op order
// (bitwise the same values, kernel_func GP_func.py:56-65; the two blocks enter symmetrically —
// commuting products and sums — so K(J, I) = K(I, J)^T bitwise): the scaled coordinates and
// squared norms of the tile's 128 rows and 128 columns are staged in LDS first. Replaces the
// write of the K tile in the K build and its read back; only the diagonal blocks are still built
// (k_build_cov, diag_only).
__device__ __forceinline__ void cov_tile_acc(Acc<T>& acc, const Quad<T>& qd, const double* __restrict__ x,
                                             const double* __restrict__ lp, int d, int N, int R, int C,
                                             double* smem) {
  const int tid = threadIdx.x;
  double* sa = smem;              // [d][T] scaled coordinates of rows (block R)
  double* sb = smem + d * T;      // [d][T] ... of columns (block C)
  double* na = smem + 2 * d * T;  // [T] squared norms of rows
  double* nb = na + T;            // [T] ... of columns
  if (tid < 2 * T) {
    const int t = tid & (T - 1);
    const bool rows = tid < T;
    const int g = (rows ? R : C) * T + t;
    double* a = rows ? sa : sb;
    double nrm = 0.0;
    if (g < N) {
      for (int k = 0; k < d; ++k) {
        const double v = x[(size_t)k * N + g] / lp[k];
        a[k * T + t] = v;
        nrm = nrm + v * v;
      }
    }
    (rows ? na : nb)[t] = nrm;
  }
  __syncthreads();
#pragma unroll
  for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
    for (int ni = 0; ni < Acc<T>::MBC; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = qd.row(mi, r), col = qd.col(ni);
        double v = 0.0;
        if (R * T + row < N && C * T + col < N) {
          double dot = sa[row] * sb[col];
          for (int k = 1; k < d; ++k) dot = fma(sa[k * T + row], sb[k * T + col], dot);
          double r2 = (na[row] + nb[col]) - 2.0 * dot;
          r2 = r2 > 0.0 ? r2 : 0.0;  // np.maximum(sq_dist, 0)
          v = exp(-0.5 * r2);
        }
        acc.v[mi][ni][r] = v;
      }
  __syncthreads();
}

// ----------------------------------------------------------------------------
// Split-K for launches with few tiles (a single particle: the prediction path, or small
// swarms): the streamed GEMM of a tile is cut into S depth ranges, one workgroup ("piece")
// each, and the S partial products are summed by a binary tree of hand-offs: at level l the
// pieces pair up by node (c = s >> l, sibling c ^ 1); each takes a ticket on the pair's counter;
// the first to arrive stores its node sum to the node's slot, raises the pair's ready flag and
// leaves; the second waits for that flag (the first is running: it took its ticket), adds the
// sibling's slot and carries the pair up; the last one standing holds the whole sum in its
// accumulators and finishes the tile. Per level the chain (the second arriver) pays a ticket and
// a 128 KiB read, not also a store and its drain (round 3: the tree sits on the prediction's
// critical path once the pieces are balanced). IEEE addition commutes, so a node's sum does not
// depend on which sibling arrived last: results are deterministic.
// Hand-off (the memory-model argument): node sums are stored write-through (agent-scope relaxed
// atomic stores, `sc1`: the line goes to memory, no L2 write-back fence, which on gfx950 would
// write back every dirty line of the XCD's L2 — ~10-100 us here), every wave drains them
// (s_waitcnt vmcnt(0)) before the barrier that precedes the ready flag, and the second arriver
// does an agent-scope acquire (L1/L2 invalidate) after seeing the flag, before reading the
// sibling's slot, which may have been written from another XCD. The second arriver resets the
// pair's ticket and flag for the next launch. The wait is bounded like wait_diag (`spins`; on
// timeout info gets bit 2 and the piece gives up, so the host reports the error).
// seed(acc) (SEEDED: piece 0 only) starts piece 0's accumulator instead of zero: the L tiles seed
// it with their covariance tile A_IJ, so the finisher does not compute it after the pieces, on
// the critical path; piece 0 takes SEED_CH fewer chunks for it (r4: the seed cost it ~11 us,
// and as the carrier of every level it reached, the whole tree waited for it).
// (r4) Node sums are kept in the accumulators' own layout (wave, register pair, lane: 16-B
// accesses, 1 KiB per wave instruction) instead of the row-major tile (8-B accesses): nothing but
// the tree reads the slots. Prediction factor 2.99 -> 2.78-2.83 ms with both
// (profiles/r4/ab_split_tree.txt).
// ----------------------------------------------------------------------------
// (A radix-4 tree — groups of up to 4 nodes, the last arriver forming ((n0 + n1) + (n2 + n3)),
// bitwise these sums with half the levels — measured slower: factor 3.45 -> 3.73 ms, the
// carrier's three 128 KiB reads per level cost more than the saved hand-offs;
// profiles/r3s2/ab_split_tree_radix.txt.)
// (sc1 loads of the sibling's node sum in place of the acquire: within noise; 4 or 8 row blocks of
// it read per scheduling group instead of 2: slower; profiles/r4/ab_split_tree.txt.)
constexpr int SEED_CH = 4;     // split_part: chunks of GEMM piece 0's covariance seed stands for
constexpr int TREE_BATCH = 2;  // row blocks of the sibling's node sum read per scheduling group
constexpr int SPLIT_TREE = 80;              // tickets per split tile: pair (level l < 5, pair k < 16) at l * 16 + k
constexpr int SPLIT_CNT = 2 * SPLIT_TREE;   // + the pairs' ready flags at SPLIT_TREE + l * 16 + k

template <bool NN, bool NEG, bool SEEDED = false, typename Seed>
__device__ __forceinline__ bool split_part(Acc<T>& acc, const double* Ap, int lda, const double* Bp, int ldb, int nch, int S,
                           int s, double* __restrict__ pt, unsigned* __restrict__ ct, double* smem,
                           const Quad<T>& qd, int* flag, int* info, int spins, Seed seed, int J) {
  // piece boundaries over nch + e chunks, the first e of them standing for piece 0's seed (its
  // covariance tile costs about SEED_CH chunks of GEMM), so that the seeded piece — the carrier
  // of every tree level it reaches — ends its GEMM with the others
  const int e = SEEDED ? SEED_CH : 0;
  const int c0 = s == 0 ? 0 : max(0, s * (nch + e) / S - e), c1 = max(0, (s + 1) * (nch + e) / S - e);
  if (SEEDED && s == 0)
    seed(acc);
  else
    acc.zero();
  if (c1 > c0)
    gemm_stream_dl<NN, NEG>(acc, Ap + (size_t)c0 * DL_KC, lda,
                            NN ? Bp + (size_t)c0 * DL_KC * ldb : Bp + (size_t)c0 * DL_KC, ldb, (c1 - c0) * DL_KC,
                            smem, qd);
#ifdef GPF_WG_TRACE
  {
    const int tid = threadIdx.x;
    GPF_PHASE(3);  // (trace build) this piece's GEMM done, before the reduction tree
  }
#else
  (void)J;
#endif
  for (int l = 0; (1 << l) < S; ++l) {
    const int c = s >> l, sib = c ^ 1;
    if ((sib << l) >= S) continue;  // no sibling range at this level: go up alone
    unsigned* tk = ct + l * 16 + (c >> 1);
    unsigned* rdy = ct + SPLIT_TREE + l * 16 + (c >> 1);
    __syncthreads();  // (the previous level's reads of *flag are done)
    if (threadIdx.x == 0) *flag = (int)__hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag == 0) {  // first: publish the node sum, then the sibling carries the pair on
      {  // register-native slot layout: 16-B write-through stores, 1 KiB per wave instruction
        const auto ws = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(pt + (size_t)(c << l) * T * T), 0,
                                                          T * T * 8, 0x00020000);
        const int wb = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (Acc<T>::MBR * Acc<T>::MBC * 2048);
#pragma unroll
        for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
          for (int ni = 0; ni < Acc<T>::MBC; ++ni)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const double a0 = acc.v[mi][ni][2 * h], a1 = acc.v[mi][ni][2 * h + 1];
              const unsigned long long u0 = __builtin_bit_cast(unsigned long long, a0),
                                       u1 = __builtin_bit_cast(unsigned long long, a1);
              const __attribute__((ext_vector_type(4))) unsigned q4 = {(unsigned)u0, (unsigned)(u0 >> 32),
                                                                        (unsigned)u1, (unsigned)(u1 >> 32)};
              __builtin_amdgcn_raw_buffer_store_b128(q4, ws, qd.lane * 16, wb + ((mi * Acc<T>::MBC + ni) * 2 + h) * 1024,
                                                     16);  // sc1: write-through
            }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave drains its part of the node sum
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(rdy, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __syncthreads();  // (every wave has read *flag)
    if (threadIdx.x == 0) {
      int n = 0, late = 0;
      while (__hip_atomic_load(rdy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        if (n++ >= spins) {
          __hip_atomic_fetch_or(info, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          late = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (!late) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(rdy, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      *flag = late;
    }
    __syncthreads();
    if (*flag) return false;  // timed out: the host reports it
    // the sibling's node sum through a buffer descriptor: one 32-bit per-lane offset and the
    // element displacements in soffset (64-bit per-element addresses were hoisted out of the tree
    // loop and spilled)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(pt + (size_t)(sib << l) * T * T), 0, T * T * 8,
                                                      0x00020000);
    const int wb = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (Acc<T>::MBR * Acc<T>::MBC * 2048);
#pragma unroll
    for (int mi = 0; mi < Acc<T>::MBR; ++mi) {
#pragma unroll
      for (int ni = 0; ni < Acc<T>::MBC; ++ni)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto q4 = __builtin_amdgcn_raw_buffer_load_b128(rs, qd.lane * 16, wb + ((mi * Acc<T>::MBC + ni) * 2 + h) * 1024, 0);
          const unsigned long long u0 = (unsigned long long)q4[0] | ((unsigned long long)q4[1] << 32),
                                   u1 = (unsigned long long)q4[2] | ((unsigned long long)q4[3] << 32);
          acc.v[mi][ni][2 * h] = acc.v[mi][ni][2 * h] + __builtin_bit_cast(double, u0);
          acc.v[mi][ni][2 * h + 1] = acc.v[mi][ni][2 * h + 1] + __builtin_bit_cast(double, u1);
        }
      if ((mi % TREE_BATCH) == TREE_BATCH - 1) __builtin_amdgcn_sched_barrier(0);
    }
  }
  return true;
}

// Consumer side of the early diagonal factor: wait until the launch's diagonal workgroup of this
// particle has published block J (flag >= J), then an agent-scope acquire (its stores are
// write-through, factor128<true>, so no L2 write-back fence was needed on its side). The spin is
// bounded (`spins` polls of ~1 us; the host passes ~2M, i.e. ~2 s, or a debug bound): on timeout
// info gets bit 2, the host reports an error, and the caller skips everything that would read the
// unpublished block (returns true) so the launch still drains.
__device__ __forceinline__ bool wait_diag(const int* flag, int J, int* info, int spins, int* sflag) {
  if (threadIdx.x == 0) {
    int n = 0, late = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < J) {
      if (n++ >= spins) {
        __hip_atomic_fetch_or(info, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        late = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(16);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *sflag = late;
  }
  __syncthreads();
  return *sflag != 0;
}

// SYRK workgroup of launch J (deferred diagonal update, see step_decode): A_{J+1,J+1} -=
// L_{J+1,<J} L_{J+1,<J}^T in one depth-128 J GEMM, published write-through with a per-particle flag.
__device__ __forceinline__ void syrk_item(int J, int p, int Npad, double* __restrict__ Lb, int* __restrict__ yflag,
                                          double* lds) {
  const size_t ld = (size_t)Npad;
  const int I = J + 1;
  double* Lp = Lb + (size_t)p * ld * ld;
  double* Aii = Lp + (size_t)I * T * ld + (size_t)I * T;
  const Quad<T> qd;
  syrk_tile<true>(Aii, ld, Lp + (size_t)I * T * ld, Npad, J * T, lds, qd);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's part drained
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(yflag + p, J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Look-ahead of launch J (launches with the early diagonal factor and no split, 1 <= J <= nt-3),
// run by the launch's SYRK workgroup after it has published its block (both GEMMs stream the same
// row panel L_{J+1,<J}; a workgroup of its own, ROLE_LA, only without the deferred update — an
// extra workgroup per particle pushed the diagonal factor onto shared CUs): the next launch's critical tile (I = J+2 of block column J+1) over the columns
// < J — its covariance seed and a depth-128J GEMM, everything except block column J, which this
// launch is computing — to lab (plain stores, read after the launch boundary). Launch J+1's
// critical tile then runs a single 128-deep block after loading it instead of the whole
// depth-128(J+1) GEMM, so its chain is the diagonal factor, not its GEMM (config B: the chain of
// J >= 4 was that GEMM, profiles/r3s2/crit_B_*.txt). Bitwise the same accumulation.
// How far the look-ahead of launch J goes: the first la_chunks(J) 16-deep chunks (of the 8J the
// columns < J hold). The SYRK workgroup that runs it spends ~9/16 of a depth-128J GEMM on its own
// lower-triangular update first, so it takes ~7/16 of the depth and the critical tile of launch
// J+1 continues from there: both then end near the launch's other deep L tiles (a look-ahead
// over the whole depth made that workgroup the launch's last, profiles/r3s2/ab_lookahead_B.txt).
__host__ __device__ __forceinline__ int la_chunks(int J) { return 7 * 8 * J / 16; }

// The partial of launch J goes to slot J & 1 of its particle (two slots per particle): the
// critical tile of launch J + 1 reads slot J & 1 while launch J + 1's own look-ahead writes slot
// (J + 1) & 1, so a critical tile dispatched late (concurrent groups over-subscribing the slots,
// another process on the GPU) can never seed from the next tile's partial.
__host__ __device__ __forceinline__ size_t la_slot(int p, int J) { return (size_t)(2 * p + (J & 1)) * T * T; }

__device__ __forceinline__ void la_item(int J, int p, int Npad, const double* __restrict__ Lb, int N,
                                        const double* __restrict__ x, const double* __restrict__ ls, int d,
                                        double* __restrict__ lab, double* lds) {
  const size_t ld = (size_t)Npad;
  const double* Lp = Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  Acc<T> acc;
  cov_tile_acc(acc, qd, x, ls + (size_t)p * d, d, N, J + 1, J + 2, lds);
  gemm_stream_dl<false, true>(acc, Lp + (size_t)(J + 1) * T * ld, Npad, Lp + (size_t)(J + 2) * T * ld, Npad,
                              la_chunks(J) * DL_KC, lds, qd);
  acc.store(qd, lab + la_slot(p, J), T);
}

// Tile w of block column J of particle p (the unit of work of k_step); role from step_decode.
//   L tile (I = J+1+w):  D = A_IJ^T - L_J,<J L_I,<J^T  (the transposed panel C^T, so that each
//                        wave holds all 128 k of the triangular multiply for its 16 rows of C)
//                        L_IJ^T = U_JJ D               (trmm_acc, U_JJ staged in LDS)
//                        A_II -= L_IJ L_IJ^T ; y_I -= L_IJ z_J
//   U tile (K = w-nL):   W = L_J,[K,J) U_[K,J),K ; U_JK = -U_JJ W (trmm_acc); column partials
// The products the finishes need never leave the registers: no C or W round trip through
// memory, no streamed second operand, no barrier inside the triangular multiplies.
template <int SPLIT, int ED>
__device__ __forceinline__ void step_item(int role, int J, int w, int p, int nt, int Npad, double* __restrict__ Lb,
                                          double* __restrict__ Ub, double* __restrict__ yb,
                                          double* __restrict__ s2p, double* __restrict__ szp,
                                          int* __restrict__ info, int N, const double* __restrict__ x,
                                          const double* __restrict__ ls, int d, int S, int S2, int sidx,
                                          double* __restrict__ part, unsigned* __restrict__ cnt, int* sflag,
                                          const int* __restrict__ dflag, const int* __restrict__ yflag, int defer,
                                          int spins, int la, const double* __restrict__ lab, double* lds) {
  const int tid = threadIdx.x;
  const int nL = nt - 1 - J;
  const size_t ld = (size_t)Npad;
  if (SPLIT != SPLIT_NONE && role == ROLE_IDLE) return;
  double* Lp = Lb + (size_t)p * ld * ld;
  double* Up = Ub + (size_t)p * ld * ld;
  double* yp = yb + (size_t)p * Npad;
  const Quad<T> qd;
  const int g = qd.lane >> 4, cl = qd.lane & 15;
  const double* Ujj = Up + (size_t)J * T * ld + (size_t)J * T;
  double* zj = lds + STEP_ZJ;  // z_J (128), written by the diagonal factor of block J

  if (w < nL) {
    const int I = J + 1 + w;
    double* Aij = Lp + (size_t)I * T * ld + (size_t)J * T;
    double* Aii = Lp + (size_t)I * T * ld + (size_t)I * T;
    const double* lp = ls + (size_t)p * d;
    Acc<T> acc;
    // D = C^T = A_JI - L_J,<J L_I,<J^T (accumulator seeded with the covariance tile, A operand
    // negated through the MFMA modifier)
    if (SPLIT != SPLIT_NONE && role == ROLE_PIECE) {
      // split-K: partial GEMMs, the last workgroup to arrive finishes the tile; piece 0 seeds
      // its partial with the covariance tile (the unsplit path's accumulator seed)
      // (S2 partial slots per tile; the all-tile split's pieces per tile from the chunk target S)
      double* pt = part + (size_t)(p * (nt - 1) + w) * S2 * T * T;
      const int Sx = SPLIT == SPLIT_ALL ? split_all_pieces(J, w, nt, S) : S;
      if (!split_part<false, true, true>(acc, Lp + (size_t)J * T * ld, Npad, Lp + (size_t)I * T * ld, Npad,
                                         J * T / DL_KC, Sx, sidx, pt, cnt + (size_t)(p * (nt - 1) + w) * SPLIT_CNT, lds,
                                         qd, sflag, info + p, spins,
                                         [&](Acc<T>& a) { cov_tile_acc(a, qd, x, lp, d, N, J, I, lds); }, J))
        return;  // (the finisher's accumulators hold D)
    } else if (SPLIT == SPLIT_NONE && ED && (la & 2) && I == J + 1) {
      // look-ahead seed: launch J-1 left this tile's GEMM over its first la_chunks(J-1) chunks (cov
      // seed included); the rest follows — the same MFMAs in the same order
      const int k0 = la_chunks(J - 1) * DL_KC;  // where launch J-1's look-ahead stopped
      if (la & 4) {  // test hook (GPF_LA_DELAY_TEST): dispatched "late", after this launch's look-ahead wrote
        for (int i = 0; i < 96; ++i) __builtin_amdgcn_s_sleep(127);  // ~0.3 ms
        __syncthreads();
      }
      acc.load(qd, lab + la_slot(p, J - 1), T);
      gemm_stream_dl<false, true>(acc, Lp + (size_t)J * T * ld + k0, Npad, Lp + (size_t)I * T * ld + k0, Npad, J * T - k0,
                                  lds, qd);
    } else {
      cov_tile_acc(acc, qd, x, lp, d, N, J, I, lds);
      if (J > 0)
        gemm_stream_dl<false, true>(acc, Lp + (size_t)J * T * ld, Npad, Lp + (size_t)I * T * ld, Npad, J * T, lds, qd);
    }
    GPF_PHASE(0);
    if (ED && wait_diag(dflag + p, J, info + p, spins, sflag)) return;  // U_JJ, z_J (launch 0 too)
    if (tid < T) zj[tid] = yp[J * T + tid];
    tri_to_lds(Ujj, ld, lds);  // (its barrier also publishes z_J)
    // L_IJ^T = U_JJ D by row halves of L_IJ^T (= column halves of L_IJ): lane (g, c) of the wave
    // with slab cb gets L(cb + c, 16 jb + 4 e + g), stores it and adds its share of row cb + c of
    // L_IJ z_J (k ascending per lane, then the 4 lane groups)
    double* lrow = launder(Aij + (size_t)(qd.cb + cl) * ld + g);
    double yr = 0.0;
#pragma unroll
    for (int P = 0; P < 4; ++P) {
      d4 o[2];
      switch (P) {
        case 0: trmm_acc<0, false>(o, acc, lds); break;
        case 1: trmm_acc<1, false>(o, acc, lds); break;
        case 2: trmm_acc<2, false>(o, acc, lds); break;
        default: trmm_acc<3, false>(o, acc, lds); break;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lrow[16 * (2 * P + j) + 4 * e] = o[j][e];
          yr = fma(o[j][e], zj[16 * (2 * P + j) + 4 * e + g], yr);
        }
    }
    yr = sum_lane_groups(yr);
    if (g == 0) yp[I * T + qd.cb + cl] = yp[I * T + qd.cb + cl] - yr;  // y_I -= L_IJ z_J
    GPF_PHASE(1);
    __syncthreads();  // L_IJ stored (workgroup release) and the staged U_JJ read: LDS free
    // look-ahead: A_II -= L_IJ L_IJ^T (the full tile; only its lower half is ever read). Deferred
    // (SPLIT_ALL never defers): only the critical tile, on top of the launch's SYRK workgroup's S.
    const bool defer_on = SPLIT != SPLIT_ALL && defer;
    if (!defer_on || I == J + 1) {
      if (defer_on && J > 0 && wait_diag(yflag + p, J, info + p, spins, sflag)) return;  // S published
      syrk_tile<false>(Aii, ld, Aij, Npad, T, lds, qd);
    }
    GPF_PHASE(2);
    if (!ED && I == J + 1) {  // fused diagonal factor of block J+1 (A_II, y_I fully reduced)
      __syncthreads();
      const size_t poff = ((size_t)p * nt + I) * Npad + (size_t)I * T;
      __builtin_amdgcn_s_setprio(3);  // latency-critical: the next launch waits for this block
      factor128(Aii, Up + (size_t)I * T * ld + (size_t)I * T, ld, yp + I * T, s2p + poff, szp + poff, info + p,
                carve_diag(lds, lds + DIAG_BASE), I * T + H >= N);
    }
  } else {
    const int K = w - nL;
    double* Ujk = Up + (size_t)J * T * ld + (size_t)K * T;
    Acc<T> acc;
    // W = L_J,[K,J) U_[K,J),K (U_KK is lower triangular: the wave's first chunks add zeros)
    if (SPLIT == SPLIT_ALL && role == ROLE_PIECE) {  // split-K (the triangular first block runs dense: its upper part holds zeros)
      double* pt = part + (size_t)(p * (nt - 1) + w) * S2 * T * T;
      const int Sx = split_all_pieces(J, w, nt, S);
      if (!split_part<true, false, false>(acc, Lp + (size_t)J * T * ld + (size_t)K * T, Npad,
                                          Up + (size_t)K * T * ld + (size_t)K * T, Npad, (J - K) * T / DL_KC, Sx, sidx,
                                          pt, cnt + (size_t)(p * (nt - 1) + w) * SPLIT_CNT, lds, qd, sflag, info + p,
                                          spins, [](Acc<T>&) {}, J))
        return;
    } else {
      acc.zero();
      gemm_stream_dl<true, false, TRI_B_KGEC>(acc, Lp + (size_t)J * T * ld + (size_t)K * T, Npad,
                                              Up + (size_t)K * T * ld + (size_t)K * T, Npad, (J - K) * T, lds, qd);
    }
    GPF_PHASE(0);
    if (ED && wait_diag(dflag + p, J, info + p, spins, sflag)) return;  // U_JJ, z_J (U tiles exist for J > 0 only)
    if (tid < T) zj[tid] = yp[J * T + tid];
    tri_to_lds(Ujj, ld, lds);
    // U_JK = -U_JJ W by row halves; the column partials of colsum(U^2) and U^T z summed per half
    // (rows ascending per lane, then the 4 lane groups), then upper half + lower half
    double* ucol = launder(Ujk + (size_t)g * ld + qd.cb + cl);
    double a2[2] = {0.0, 0.0}, az[2] = {0.0, 0.0};
#pragma unroll
    for (int P = 0; P < 4; ++P) {
      d4 o[2];
      switch (P) {
        case 0: trmm_acc<0, true>(o, acc, lds); break;
        case 1: trmm_acc<1, true>(o, acc, lds); break;
        case 2: trmm_acc<2, true>(o, acc, lds); break;
        default: trmm_acc<3, true>(o, acc, lds); break;
      }
      const int h = P >> 1;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = 16 * (2 * P + j) + 4 * e;  // + g
          const double v = o[j][e];
          ucol[(size_t)row * ld] = v;
          a2[h] = fma(v, v, a2[h]);
          az[h] = fma(v, zj[row + g], az[h]);
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a2[h] = sum_lane_groups(a2[h]);
      az[h] = sum_lane_groups(az[h]);
    }
    GPF_PHASE(1);
    if (g == 0) {
      const size_t poff = ((size_t)p * nt + J) * Npad + (size_t)K * T + qd.cb + cl;
      s2p[poff] = a2[0] + a2[1];
      szp[poff] = az[0] + az[1];
    }
  }
}

// SPLIT: SPLIT_ALL cuts every tile (launches with few tiles), SPLIT_CRIT only the critical-path
// tile I = J+1 of each particle (launches that leave slots idle: its S pieces are dispatched
// first, ahead of the unsplit tiles); SPLIT_NONE carries no split code at all, so its register
// allocation is that of the plain schedule.
template <int SPLIT, int ED>
__global__ __launch_bounds__(STEP_NTH, STEP_WAVES_PER_SIMD) void k_step(int J, int nt, int Npad, double* __restrict__ Lb,
                                                  double* __restrict__ Ub, double* __restrict__ yb,
                                                  double* __restrict__ s2p, double* __restrict__ szp,
                                                  int* __restrict__ info, int P, int grp, int N,
                                                  const double* __restrict__ x, const double* __restrict__ ls,
                                                  int d, int S, int S2, double* __restrict__ part,
                                                  unsigned* __restrict__ cnt, int* __restrict__ dflag, int ed,
                                                  int* __restrict__ yflag, int defer, int sy, int spins, int la,
                                                  double* __restrict__ lab, unsigned long long* __restrict__ clk) {
  const int tid = threadIdx.x;
  __shared__ unsigned long long sclk[2];
  const ClockSpan span(sclk);
  span.start(clk);
#ifdef GPF_WG_TRACE
  if (tid == 0 && J < WG_TRACE_J && blockIdx.x < WG_TRACE_N) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_wg_trace[J][blockIdx.x][0] = realtime();
    g_wg_trace[J][blockIdx.x][2] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
  __shared__ __attribute__((aligned(16))) double lds[STEP_LDS];
  __shared__ int sflag;
  int p, w, sidx;
  const int role = step_decode<SPLIT>((int)blockIdx.x, J, P, nt, grp, S, ED && ed, SPLIT != SPLIT_ALL && sy,
                                      SPLIT == SPLIT_NONE && ED && (la & 1) && !sy, p, w, sidx,
                                      SPLIT == SPLIT_NONE && ED && (la & 32) != 0);
#ifdef GPF_CHECK
  // diagnostic build (-DGPF_CHECK): every index the workgroup derives its addresses from, checked
  // against the launch's extents before any access (an out-of-range role prints and does nothing)
  {
    bool ok = p >= 0 && p < P && J >= 0 && J < nt && Npad == nt * T && S >= 1 && S2 >= 1 && S2 <= SPLIT_MAXS;
    if (role == ROLE_SYRK) ok = ok && w == -1 && J >= 1 && J <= nt - 2 && yflag != nullptr;
    else if (role == ROLE_LA) ok = ok && w == -1 && J >= 1 && J + 2 < nt && lab != nullptr;
    else if (role == ROLE_DIAG) ok = ok && w == -1 && ED && dflag != nullptr;
    else if (role != ROLE_IDLE) ok = ok && w >= 0 && w < nt - 1 && sidx >= 0 &&
                                     sidx < (SPLIT == SPLIT_ALL ? split_all_pieces(J, w, nt, S) : S) && sidx < S2 &&
                                     (role != ROLE_PIECE || (part != nullptr && cnt != nullptr && S > 1)) &&
                                     (w >= nt - 1 - J || J + 1 + w < nt) && (w < nt - 1 - J || w - (nt - 1 - J) < J);
    if (!ok) {
      if (tid == 0)
        printf("k_step check: J=%d block %d role %d p=%d w=%d sidx=%d (P=%d nt=%d S=%d)\n", J, (int)blockIdx.x, role,
               p, w, sidx, P, nt, S);
      return;
    }
  }
#endif
  if (SPLIT != SPLIT_ALL && role == ROLE_SYRK) {
    syrk_item(J, p, Npad, Lb, yflag, lds);
    if (SPLIT == SPLIT_NONE && ED && (la & 1)) {  // the look-ahead rides on the SYRK workgroup (after its flag)
      __syncthreads();
      la_item(J, p, Npad, Lb, N, x, ls, d, lab, lds);
    }
  } else if (SPLIT == SPLIT_NONE && ED && role == ROLE_LA) {
    la_item(J, p, Npad, Lb, N, x, ls, d, lab, lds);
  } else if (ED && role == ROLE_DIAG) {
    // diagonal block J of particle p (fully reduced by the previous launches' look-ahead): factor,
    // then publish to this launch's tiles (write-through stores drained, then the flag)
    const size_t ld = (size_t)Npad;
    const size_t off = (size_t)p * ld * ld + (size_t)J * T * ld + (size_t)J * T;
    const size_t poff = ((size_t)p * nt + J) * Npad + (size_t)J * T;
    __builtin_amdgcn_s_setprio(3);  // the launch's tiles wait for this block
    // publishes block J (dflag[p] = J) as soon as U_JJ and z_J are stored, before its partials
    factor128<true>(Lb + off, Ub + off, ld, yb + (size_t)p * Npad + J * T, s2p + poff, szp + poff, info + p,
                    carve_diag(lds, lds + DIAG_BASE), J * T + H >= N, dflag + p, J);
  } else {
    step_item<SPLIT, ED>(role, J, w, p, nt, Npad, Lb, Ub, yb, s2p, szp, info, N, x, ls, d, S, S2, sidx, part, cnt, &sflag,
                         dflag, yflag, defer, spins, la, lab, lds);
  }
  span.stop(clk);
#ifdef GPF_WG_TRACE
  __syncthreads();
  if (tid == 0 && J < WG_TRACE_J && blockIdx.x < WG_TRACE_N) g_wg_trace[J][blockIdx.x][1] = realtime();
#endif
}


// Debug hook (gpf_debug_factor64): factor64 on two host-given 64x64 matrices in a row
// (in: 2 x 64 x 64 row-major; out: L then X for each).
__global__ __launch_bounds__(DNTH) void k_debug_factor64(const double* __restrict__ in, double* __restrict__ out,
                                                         int* __restrict__ bad) {
  __shared__ __attribute__((aligned(16))) double t[2 * H * LDH];
  __shared__ __attribute__((aligned(16))) double scratch[F64_BUF];
  const int tid = threadIdx.x;
  for (int k = 0; k < 2; ++k) {
    for (int i = tid; i < H * H; i += DNTH) t[(i / H) * LDH + i % H] = in[k * H * H + i];
    __syncthreads();
    const bool b = factor64(t, LDH, t + H * LDH, LDH, scratch);
    __syncthreads();
    for (int i = tid; i < H * H; i += DNTH) {
      out[(2 * k) * H * H + i] = t[(i / H) * LDH + i % H];
      out[(2 * k + 1) * H * H + i] = t[H * LDH + (i / H) * LDH + i % H];
    }
    if (tid == 0) bad[k] = b;
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// Measurement hook (gpf_gemm_bench): the L-tile GEMM of k_step in isolation.
// Workgroup b: particle p = b % P, tile w = b / P; D_w -= L_p[rows J, :D] L_p[rows I, :D]^T
// with I = J+1+w, J = D/T (mode 0), or every workgroup on the same operands (mode 1:
// L2-resident, isolates the core from HBM); +4: the U-tile shape (B given as a [k][c] row panel).
// The tile goes to C + b*T*T.
// ----------------------------------------------------------------------------
// Operand fill of the GEMM-core measurement: values in [-1, 1) from a hash of the index (the MFMA's
// power, and so the clock the chip holds, depends on its operand bits: zero operands ran the core at
// ~2.39 GHz where k_step's real data holds ~2.18 GHz).
__global__ __launch_bounds__(NTHR) void k_fill_hash(double* __restrict__ p, long long n) {
  for (long long i = blockIdx.x * (long long)NTHR + threadIdx.x; i < n; i += (long long)gridDim.x * NTHR) {
    unsigned long long h = (unsigned long long)i * 0x9e3779b97f4a7c15ull;
    h ^= h >> 31;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 29;
    p[i] = (double)(h >> 11) * 0x1.0p-52 - 1.0;
  }
}

__global__ __launch_bounds__(STEP_NTH, STEP_WAVES_PER_SIMD) void k_gemm_bench(int mode, int D, int Npad, int P,
                                                                                   const double* __restrict__ Lb,
                                                                                   double* __restrict__ C,
                                                                                   unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[DL_STAGE];
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  const int b = blockIdx.x;
  const bool shared = (mode & 1) != 0;
  const int p = shared ? 0 : b % P, w = shared ? 0 : b / P;
  const size_t ld = (size_t)Npad;
  const int J = D / T, I = J + 1 + w;
  const double* Lp = Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  Acc<T> acc;
  acc.zero();
  if (mode & 4)
    gemm_stream_dl<true, false>(acc, Lp + (size_t)I * T * ld, Npad, Lp + (size_t)w * T, Npad, D, smem, qd);
  else
    gemm_stream_dl<false, true>(acc, Lp + (size_t)J * T * ld, Npad, Lp + (size_t)I * T * ld, Npad, D, smem, qd);
  acc.store(qd, C + (size_t)b * T * T, T);
  span.stop(clk);
}

}  // namespace gpf
