// gpf_persist.hip — persistent, dependency-driven block-column factorisation (the slot-bound
// schedules: config C, D's and E's per-GPU shares).
//
// Reference op replaced: the same as k_step's (GP_func.py:21-24,38 via find_len_scales.py:159 —
// chol(K), its inverse, z = L^-1 y and the column partials), for every particle of a batch.
//
// Why: with one k_step launch per 128-wide block column, every launch drains before the next one
// starts. Its last tiles hold a few slots while the others idle, 32 times per group at N=4096
// (~17% of the matrix pipe's cycles idle at config C with two concurrent group streams filling
// part of the gaps). Here one launch of resident workgroups (two per CU) takes the
// tiles of every block column from per-XCD work queues in dependency order, and a tile waits only
// for the tiles it reads — particle p's block column J+1 starts while other particles' column J
// tails are still running.
//
// Items (one 128x128 tile of one particle; the arithmetic of step_item's unsplit path with the
// deferred diagonal update and the fused diagonal factor, so the factor is bitwise k_step's):
//   SYRK  (J, p), 1 <= J <= nt-2:  S = A_{J+1,J+1} - L_{J+1,<J} L_{J+1,<J}^T
//   L tile (J, I), I > J:          D = A_JI - L_J,<J L_I,<J^T ; L_IJ^T = U_JJ D ; y_I -= L_IJ z_J;
//                                  I = J+1 (the critical tile) then adds L_IJ L_IJ^T to S and
//                                  factors diagonal block I (factor128: L_II, U_II, z_I, partials)
//   U tile (J, K), K < J:          U_JK = -U_JJ (L_J,[K,J) U_[K,J),K) ; column partials
// Block 0 is factored by k_diag before the launch.
//
// Dependencies, tracked per particle by monotone counters (PState):
//   lcol[I] = number of block columns of L finished in block row I   (L tile (J, I) stores J+1)
//   ucol[K] = number of block rows of U finished in block column K   (diagonal K stores K+1 once
//             U_KK and z_K are out, U tile (J, K) stores J+1)
//   sdone[I] = 1 once the SYRK item has published S for diagonal block I
// so L tile (J, I) waits for lcol[I] >= J-1 and lcol[J] >= J-1 before the GEMM over the columns
// < J-1 (r4 look-ahead), for lcol[I] >= J and lcol[J] >= J before the last block column, and for
// ucol[J] >= J+1 before its finish; U tile (J, K) for lcol[J] >= J and ucol[K] >= J, then
// ucol[J] >= J+1; SYRK
// (J) for lcol[J+1] >= J; the critical tile also for sdone[J+1]. Each counter is written in
// increasing order because each of its writers depends on the previous one.
//
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility): everything another item
// reads is stored write-through (sc1), every storing wave drains (s_waitcnt vmcnt(0)) before the
// workgroup barrier that precedes the counter store (an agent-scope relaxed atomic store); the
// consumer polls with relaxed agent loads, then one agent-scope acquire (L1 invalidate) before it
// reads. Nothing depends on which XCD runs which item: the queues only bias placement.
//
// Scheduling: queue q holds the items of the particles p = q (mod nq), nq = min(8, P), block
// column by block column; within a column the SYRK items first, then the critical tiles, then the
// other L tiles, then the U tiles deepest first (particles interleaved at each position). A
// workgroup serves the queue of its own XCD (HW_REG_XCC_ID), so a particle's tiles share one L2,
// and steals from the others once it is empty. Deadlock freedom: an item only ever waits for
// items earlier in its queue; items are taken only by running workgroups, so the earliest
// unfinished item is always running with its inputs complete (whatever the residency).
// Every wait is bounded: a timeout sets info bit 2 and a global abort word that every other wait
// and the queue loop check, so the launch drains promptly and the host reports the error.
#pragma once
#include "gpf_factor.hip"

namespace gpf {


struct PState {
  int* lcol;       // [P][nt]
  int* ucol;       // [P][nt]
  int* sdone;      // [P][nt]
  unsigned* head;  // [PQ_MAX] queue tickets
  int* abort;      // [1]
};

constexpr int PQ_MAX = 8;

__host__ __device__ __forceinline__ int p_nq(int P) { return P < PQ_MAX ? P : PQ_MAX; }
__host__ __device__ __forceinline__ int p_npq(int P, int q) {
  const int nq = p_nq(P);
  return (P - q + nq - 1) / nq;
}
__host__ __device__ __forceinline__ int p_sy(int J, int nt) { return (J >= 1 && J <= nt - 2) ? 1 : 0; }
__host__ __device__ __forceinline__ long long p_col_items(int P, int nt, int q, int J) {
  return (long long)p_npq(P, q) * (nt - 1 + p_sy(J, nt));
}
__host__ __device__ __forceinline__ long long p_queue_items(int P, int nt, int q) {
  long long n = 0;
  for (int J = 0; J < nt; ++J) n += p_col_items(P, nt, q, J);
  return n;
}

enum { PK_SYRK = 0, PK_LTILE = 1, PK_UTILE = 2 };

// Ticket t of queue q -> (kind, J, p, w), w as in step_item (w < nt-1-J: L tile I = J+1+w, else U
// tile K = w-(nt-1-J)). (Jc, bc): a column and the first ticket of that column, at or before t
// (tickets of one queue only grow, so the scan resumes where the last one stopped); updated.
// The host-side plan check (gpf_plan_check) decodes through this function too.
__host__ __device__ __forceinline__ int p_decode(long long t, int P, int nt, int q, int& Jc, long long& bc, int& p,
                                                 int& w) {
  for (;;) {
    const long long c = p_col_items(P, nt, q, Jc);
    if (t < bc + c || Jc == nt - 1) break;
    bc += c;
    ++Jc;
  }
  const int npq = p_npq(P, q), nq = p_nq(P);
  const long long r = t - bc;
  const int s = (int)(r / npq), pi = (int)(r - (long long)s * npq);
  p = q + pi * nq;
  const int sy = p_sy(Jc, nt);
  if (sy && s == 0) {
    w = -1;
    return PK_SYRK;
  }
  w = s - sy;
  return w < nt - 1 - Jc ? PK_LTILE : PK_UTILE;
}

// Wait until *f1 >= v1 and *f2 >= v2 (relaxed agent polls by one lane: sc1 loads, both issued
// before either is tested). Returns true (and the item skips its dependent work) on a timeout or
// once another item has timed out (the abort word).
// No acquire (L1 invalidate) follows: what an item reads behind a counter is either written once
// per factorisation (the L and U tiles, U_JJ, S: no CU reads those bytes in this launch before
// their producer's counter is up, and the launch starts with invalidated caches, so no stale copy
// can exist; the producer's sc1 stores reached memory before its counter) or is re-written
// within the launch (y, z) and then read with sc1 loads, which bypass the L1 (p_ld).
__device__ __forceinline__ bool p_wait(const int* f1, int v1, const int* f2, int v2, int* info, int* abort, int spins,
                                       int* sflag) {
  if (threadIdx.x == 0) {
    int n = 0, late = 0;
    for (;;) {
      const int a = __hip_atomic_load(f1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int b = __hip_atomic_load(f2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a >= v1 && b >= v2) break;
      if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || n++ >= spins) {
        late = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (late) {
      __hip_atomic_fetch_or(info, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *sflag = late;
  }
  __syncthreads();
  return *sflag != 0;
}

// A double re-written within the launch (y_I, z_J), read past the L1 (sc1).
__device__ __forceinline__ double p_ld(const double* q) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(q),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Publish: every wave's stores drained, then one lane raises the counter.
__device__ __forceinline__ void p_publish(int* f, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct PItem {
  int nt, Npad, N, d, spins;
  double* Lb;
  double* Ub;
  double* yb;
  double* s2p;
  double* szp;
  int* info;
  const double* x;
  const double* ls;
};

// SYRK item of block column J (deferred diagonal update): S = A_{J+1,J+1} - L_{J+1,<J} L_{J+1,<J}^T.
__device__ __forceinline__ void p_syrk(const PItem& a, const PState& st, int J, int p, int* sflag, double* lds) {
  const int nt = a.nt;
  const int* lc = st.lcol + (size_t)p * nt;
  if (p_wait(lc + J + 1, J, lc + J + 1, J, a.info + p, st.abort, a.spins, sflag)) return;
  const size_t ld = (size_t)a.Npad;
  double* Lp = a.Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  syrk_tile<true>(Lp + (size_t)(J + 1) * T * ld + (size_t)(J + 1) * T, ld, Lp + (size_t)(J + 1) * T * ld, a.Npad, J * T,
                  lds, qd);
  p_publish(st.sdone + (size_t)p * nt + J + 1, 1);
}

// L tile (J, I) (see the file comment); I = J+1 also reduces and factors diagonal block I.
__device__ __forceinline__ void p_ltile(const PItem& a, const PState& st, int J, int I, int p, int* sflag, double* lds) {
  const int tid = threadIdx.x, nt = a.nt;
  const size_t ld = (size_t)a.Npad;
  const int* lc = st.lcol + (size_t)p * nt;
  const int* uc = st.ucol + (size_t)p * nt;
  int* info = a.info + p;
  double* Lp = a.Lb + (size_t)p * ld * ld;
  double* Up = a.Ub + (size_t)p * ld * ld;
  double* yp = a.yb + (size_t)p * a.Npad;
  const Quad<T> qd;
  const int g = qd.lane >> 4, cl = qd.lane & 15;
  double* zj = lds + STEP_ZJ;
  double* Aij = Lp + (size_t)I * T * ld + (size_t)J * T;
  // D = C^T = A_JI - L_J,<J L_I,<J^T (rows I and J through column J-1). Look-ahead (r4): the GEMM
  // over the columns < J-1 needs rows I and J only through column J-2, so it starts as soon as
  // block column J-2 has them — while column J-1's chain (its critical tile, which produces
  // L_{J,J-1}, and diagonal factor) still runs; the last block column J-1 follows once rows I and
  // J have it. The same chunks in the same order: bitwise the one-piece GEMM.
  Acc<T> acc;
  if (J > 1 && p_wait(lc + I, J - 1, lc + J, J - 1, info, st.abort, a.spins, sflag)) return;
  cov_tile_acc(acc, qd, a.x, a.ls + (size_t)p * a.d, a.d, a.N, J, I, lds);
  if (J > 0 && !gemm_stream_dl_wait<false, true, TRI_NONE>(acc, Lp + (size_t)J * T * ld, a.Npad, Lp + (size_t)I * T * ld,
                                                           a.Npad, J * T, (J - 1) * T, lds, qd, [&] {
                                                             return p_wait(lc + I, J, lc + J, J, info, st.abort, a.spins,
                                                                           sflag);
                                                           }))
    return;
  // U_JJ and z_J (diagonal block J)
  if (p_wait(uc + J, J + 1, uc + J, J + 1, info, st.abort, a.spins, sflag)) return;
  if (tid < T) zj[tid] = p_ld(yp + J * T + tid);
  tri_to_lds(Up + (size_t)J * T * ld + (size_t)J * T, ld, lds);
  // L_IJ^T = U_JJ D by row halves (step_item), stored write-through
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
        gst<true>(&lrow[16 * (2 * P + j) + 4 * e], o[j][e]);
        yr = fma(o[j][e], zj[16 * (2 * P + j) + 4 * e + g], yr);
      }
  }
  yr = sum_lane_groups(yr);
  if (g == 0) gst<true>(&yp[I * T + qd.cb + cl], p_ld(yp + I * T + qd.cb + cl) - yr);  // y_I -= L_IJ z_J
  p_publish(st.lcol + (size_t)p * nt + I, J + 1);  // (its barrier also frees the staged U_JJ)
  if (I != J + 1) return;
  // the critical tile: A_II = S - L_IJ L_IJ^T (at J = 0 the whole update), then factor block I
  if (J > 0 && p_wait(st.sdone + (size_t)p * nt + I, 1, st.sdone + (size_t)p * nt + I, 1, info, st.abort, a.spins, sflag))
    return;
  double* Aii = Lp + (size_t)I * T * ld + (size_t)I * T;
  syrk_tile<false>(Aii, ld, Aij, a.Npad, T, lds, qd);
  __syncthreads();
  const size_t poff = ((size_t)p * nt + I) * a.Npad + (size_t)I * T;
  __builtin_amdgcn_s_setprio(3);  // latency-critical: every tile of column I waits for this block
  // U_II and z_I are stored write-through and published (ucol[I] = I+1) before the partials
  factor128<true>(Aii, Up + (size_t)I * T * ld + (size_t)I * T, ld, yp + I * T, a.s2p + poff, a.szp + poff, info,
                  lds, st.ucol + (size_t)p * nt + I, I + 1);
  __builtin_amdgcn_s_setprio(0);
}

// U tile (J, K), K < J (see the file comment).
__device__ __forceinline__ void p_utile(const PItem& a, const PState& st, int J, int K, int p, int* sflag, double* lds) {
  const int tid = threadIdx.x, nt = a.nt;
  const size_t ld = (size_t)a.Npad;
  const int* lc = st.lcol + (size_t)p * nt;
  const int* uc = st.ucol + (size_t)p * nt;
  int* info = a.info + p;
  double* Lp = a.Lb + (size_t)p * ld * ld;
  double* Up = a.Ub + (size_t)p * ld * ld;
  double* yp = a.yb + (size_t)p * a.Npad;
  const Quad<T> qd;
  const int g = qd.lane >> 4, cl = qd.lane & 15;
  double* zj = lds + STEP_ZJ;
  // W = L_J,[K,J) U_[K,J),K: row J through column J-1, column K of U through row J-1
  if (p_wait(lc + J, J, uc + K, J, info, st.abort, a.spins, sflag)) return;
  Acc<T> acc;
  acc.zero();
  gemm_stream_dl<true, false, TRI_B_KGEC>(acc, Lp + (size_t)J * T * ld + (size_t)K * T, a.Npad,
                                          Up + (size_t)K * T * ld + (size_t)K * T, a.Npad, (J - K) * T, lds, qd);
  if (p_wait(uc + J, J + 1, uc + J, J + 1, info, st.abort, a.spins, sflag)) return;
  if (tid < T) zj[tid] = p_ld(yp + J * T + tid);
  tri_to_lds(Up + (size_t)J * T * ld + (size_t)J * T, ld, lds);
  double* ucol = launder(Up + (size_t)J * T * ld + (size_t)K * T + (size_t)g * ld + qd.cb + cl);
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
        gst<true>(&ucol[(size_t)row * ld], v);
        a2[h] = fma(v, v, a2[h]);
        az[h] = fma(v, zj[row + g], az[h]);
      }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    a2[h] = sum_lane_groups(a2[h]);
    az[h] = sum_lane_groups(az[h]);
  }
  if (g == 0) {
    const size_t poff = ((size_t)p * nt + J) * a.Npad + (size_t)K * T + qd.cb + cl;
    a.s2p[poff] = a2[0] + a2[1];
    a.szp[poff] = az[0] + az[1];
  }
  p_publish(st.ucol + (size_t)p * nt + K, J + 1);
}

// The dependency-ordered factorisation: one workgroup per item (grid = every item of every queue),
// but a workgroup does not run the item its block index names: it takes the next ticket of its
// XCD's queue when it starts (or of another queue once that one is empty). Tickets are therefore
// handed out in the order the dispatcher starts workgroups, to running workgroups only, which is
// what the deadlock-freedom argument needs; and as one item per workgroup the register allocation
// is k_step's (a loop over items kept the decode and addressing state live across the tile bodies
// and spilled). The grid equals the number of items, so every workgroup finds a ticket.
__global__ __launch_bounds__(STEP_NTH, STEP_WAVES_PER_SIMD) void k_factor(PItem a, PState st, int P,
                                                                                unsigned long long* __restrict__ clk) {
  __shared__ unsigned long long sclk[2];
  const ClockSpan span(sclk);
  span.start(clk);
  __shared__ __attribute__((aligned(16))) double lds[STEP_LDS];
  __shared__ int sflag;
  __shared__ long long sticket;
  __shared__ int squeue;
  const int nt = a.nt, nq = p_nq(P);
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const int q0 = (int)(xcc & 7u) % nq;
    long long tk = -1;
    int q = q0;
    for (int qi = 0; qi < nq && tk < 0; ++qi) {
      q = (q0 + qi) % nq;
      const unsigned t = __hip_atomic_fetch_add(st.head + q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((long long)t < p_queue_items(P, nt, q)) tk = t;
    }
    if (__hip_atomic_load(st.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) tk = -1;  // drain
    sticket = tk;
    squeue = q;
  }
  __syncthreads();
  // (the ticket and queue come through LDS: readfirstlane makes them — and the particle, column
  // and tile decoded from them, and every counter address — scalar, so they do not occupy vector
  // registers across the tile's GEMM)
  const long long tk0 = sticket;
  const long long tk = (long long)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)tk0 >> 32))
                                    << 32) |
                                   (unsigned)__builtin_amdgcn_readfirstlane((unsigned)tk0));
  if (tk < 0) return;
  const int q = __builtin_amdgcn_readfirstlane(squeue);
  // column of ticket tk: items before column J = npq (J (nt-1) + #SYRK columns < J), monotone in J
  const long long npq = p_npq(P, q);
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    const long long before = npq * ((long long)mid * (nt - 1) + (mid >= 2 ? (mid - 1 < nt - 2 ? mid - 1 : nt - 2) : 0));
    if (before <= tk) lo = mid;
    else hi = mid - 1;
  }
  int Jc = lo;
  long long bc = npq * ((long long)lo * (nt - 1) + (lo >= 2 ? (lo - 1 < nt - 2 ? lo - 1 : nt - 2) : 0));
  int p, w;
  const int kind = p_decode(tk, P, nt, q, Jc, bc, p, w);
  const int J = Jc;
  if (kind == PK_SYRK) p_syrk(a, st, J, p, &sflag, lds);
  else if (kind == PK_LTILE) p_ltile(a, st, J, J + 1 + w, p, &sflag, lds);
  else p_utile(a, st, J, w - (nt - 1 - J), p, &sflag, lds);
  span.stop(clk);
}

// Workgroups of one k_factor launch: every item of every queue.
__host__ __device__ __forceinline__ long long p_total_items(int P, int nt) {
  long long n = 0;
  for (int q = 0; q < p_nq(P); ++q) n += p_queue_items(P, nt, q);
  return n;
}

}  // namespace gpf
