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
#include "gpf_diag.hip"

namespace gpf {

// Diagonal block J of every particle (A_JJ already reduced by the look-ahead of
// all earlier block columns). Launched for J = 0 only; every later diagonal
// block is factored inside k_step by the workgroup that finishes reducing it.
// grid: (P)
__global__ __launch_bounds__(DNTH) void k_diag(int J, int nt, int N, int Npad, double* __restrict__ Lb,
                                                  double* __restrict__ Ub, double* __restrict__ yb,
                                                  double* __restrict__ s2p, double* __restrict__ szp,
                                                  int* __restrict__ info, int* __restrict__ dflag) {
  if (threadIdx.x == 0) dflag[blockIdx.x] = J;  // a new factorisation: block J published (launches follow in order)
  __shared__ __attribute__((aligned(16))) double lds[DB_LDS];
  const int p = blockIdx.x;
  const size_t ld = (size_t)Npad;
  const size_t off = (size_t)p * ld * ld + (size_t)J * T * ld + (size_t)J * T;
  const size_t poff = ((size_t)p * nt + J) * Npad + (size_t)J * T;
  factor128(Lb + off, Ub + off, ld, yb + (size_t)p * Npad + J * T, s2p + poff, szp + poff, info + p, lds);
  (void)N;
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

// (r5: the critical-tile split SPLIT_CRIT = 2 of rounds 1-4 — off by default since round 2 and
// slower again on B in r5, profiles/r5/ab_split_crit_B.txt — and its reduction tree were removed.)
enum { SPLIT_NONE = 0, SPLIT_ALL = 1 };
enum { ROLE_IDLE = 0, ROLE_WHOLE = 1, ROLE_PIECE = 2, ROLE_DIAG = 3, ROLE_SYRK = 4, ROLE_LA = 5, ROLE_PLA = 6, ROLE_SYRKP = 7,
       ROLE_LPIECE = 8 };

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
// (r5) At least SPLIT_MINP pieces per tile: the flat finish (flat_piece) spreads a tile's
// triangular multiply and diagonal-block update over its pieces' CUs, so the shallow tiles of the
// first launches (J = 0: no GEMM at all) no longer finish on one CU each (launch 0: ~77 us, the
// diagonal factor ~40 of it). Pieces past the depth add zero partials.
constexpr int SPLIT_MAXS = 32;
constexpr int SPLIT_MINP = 4;
__host__ __device__ __forceinline__ int split_all_chunks(int J, int w, int nt) {
  const int nL = nt - 1 - J;
  return (w < nL ? J : J - (w - nL)) * (T / DL_KC);  // L tile: depth 128J; U tile K: 128(J-K)
}
__host__ __device__ __forceinline__ int split_all_pieces(int J, int w, int nt, int tgt) {
  const int ch = split_all_chunks(J, w, nt);
  int s = ch <= 0 ? 1 : (ch + tgt - 1) / tgt;
  s = s < SPLIT_MINP ? SPLIT_MINP : s;
  return s > SPLIT_MAXS ? SPLIT_MAXS : s;
}

// Workgroup b of a k_step<SPLIT> launch (grid: [P diagonal workgroups if ed] + [P SYRK workgroups
// if sy] + P * sum_w split_all_pieces(J, w, nt, S) for SPLIT_ALL (tiles in order w = 0, 1, ..:
// the critical tile first, then the L tiles, then the U tiles deepest first; pieces particle-
// fastest), P*(nt-1) otherwise): its
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
  } else {  // particle-fastest order (grp = 0) puts the critical tiles w = 0 at b < P
    step_tile(b, P, nt - 1, grp, p, w);
  }
  return ROLE_WHOLE;
}

// ----------------------------------------------------------------------------
// Paired block columns (r6; k_step<SPLIT_NONE, 0>, the slot-bound launches of configs C/D; VERDICT r5
// item 1). A left-looking launch streams every tile's B panel (row panel I of L for an L tile, column
// panel K of U for a U tile) from HBM once per block column: ~2.4 GB per group launch at C, 16x the
// compulsory stores, and the HBM stream costs the chip its clock (profiles/r5/gemm_ablate.txt: the
// same GEMM loop holds 2.2 GHz streaming from HBM, 2.38 GHz on L2-resident panels). Block column J+1
// needs the same panels over the same depth [0, J) plus one more 128-block, so the launches go in
// pairs:
//   lead J (pair = 1):    every tile of column J as before, and beside each tile of column J+1 that
//                         exists already (L tiles I >= J+2, U tiles K < J) its GEMM over the columns
//                         < J (ROLE_PLA: the covariance seed included), stored to a partial slot; the
//                         SYRK workgroup of block J+1 as before, and a partial SYRK of block J+2 over
//                         the same depth (ROLE_SYRKP, in place);
//   follow J+1 (pair = 2): every tile loads its partial and runs the one remaining 128-deep block (the
//                         columns of block J) before its finish; the critical tile applies blocks J
//                         and J+1 to its diagonal block (the rest was ROLE_SYRKP's); no SYRK workgroups.
// A tile's workgroup and its partner stream the same panel at the same time from one XCD (pair_decode),
// so the panel is fetched into that XCD's L2 once: the probe (scripts/probes/gemm_ablate.hip,
// profiles/r6/pair_*.txt) ran such pairs at 72.5-73.3 TF/s and 2.33-2.34 GHz against 68.6-68.7 TF/s
// and 2.21-2.23 GHz for the single-output loop, at the same 0.95 per clock and with two ordinary
// 8-wave workgroups per CU (the 16-wave two-output workgroup of round 5 held the clock too but lost
// per clock, 0.93, and leaves its finishes without a co-resident workgroup). Every element sees the
// same MFMAs in the same order as in the unpaired launches (a chain split at a chunk boundary with
// an exact store and reload), so the factor is bitwise unchanged (test_paired_block_columns_bitwise).
// ----------------------------------------------------------------------------
// workgroups per particle of tile w's unit in a lead launch: the tile, its partner (w = 0: the SYRK
// workgroup of block J+1; else the look-ahead partial), and for w = 1 when it is the L tile I = J+2
// the partial SYRK of block J+2 (all three stream row panel J+2)
__host__ __device__ __forceinline__ int pair_unit(int J, int w, int nt) { return (w == 1 && J + 2 <= nt - 1) ? 3 : 2; }
__host__ __device__ __forceinline__ int pair_grid_per_particle(int J, int nt) {
  int n = 0;
  for (int w = 0; w < nt - 1; ++w) n += pair_unit(J, w, nt);
  return n;
}
// Workgroup b of a lead launch (P a multiple of 8, w-major as step_tile's particle-fastest order):
// per tile w, groups of 8 particles (one per XCD: b & 7 = p & 7), first the tile's own workgroups
// (ROLE_WHOLE), then the partners of the same 8 particles — so a partner sits 8 (or 16) ids behind
// its tile, on the same XCD, dispatched together with it (w = 0: the SYRK workgroups 8 ids ahead of
// their critical tiles).
__host__ __device__ __forceinline__ int pair_decode(int b, int J, int P, int nt, int& p, int& w, int* hout = nullptr) {
  int base = 0;
  for (w = 0; w < nt - 2; ++w) {
    const int n = pair_unit(J, w, nt) * P;
    if (b < base + n) break;
    base += n;
  }
  const int u = pair_unit(J, w, nt), r = b - base, c = r / (8 * u), h = (r % (8 * u)) / 8;
  p = 8 * c + (r & 7);
  if (hout) *hout = h;
  if (w == 0) {  // the SYRK workgroups ahead of their critical tiles, which wait for them (no wait can
                 // then depend on a workgroup not yet dispatched)
    if (h == 1) return ROLE_WHOLE;
    w = -1;  // (as step_decode's SYRK workgroups)
    return ROLE_SYRK;
  }
  if (h == 0) return ROLE_WHOLE;
  return h == 1 ? ROLE_PLA : ROLE_SYRKP;
}
// Start synchronisation of a lead launch's partners (a performance hint, never a data dependency):
// a tile's workgroup and its partner share their panel through the XCD's L2 only while they stream
// it together, and the dispatcher starts a partner whenever a slot of its XCD frees — after the first
// round of a launch partners drift apart by a finish phase or more. So every member h of a unit
// stores the launch's tag (unique per factorisation and launch) into its word on arrival, and the
// earlier-dispatched members wait until every later member of the unit has arrived. A waiting
// workgroup waits only for the ids right behind it in its XCD's dispatch order, which are next for
// that XCD's next free slot: the wait always ends. Bounded (~50 us); on timeout it just proceeds.
constexpr int PAIR_HMAX = 3;
__device__ __forceinline__ void pair_start_sync(int J, int u, int h, int p, int nt, int* pstart, int ptag) {
  int* f = pstart + ((size_t)p * (nt - 1) + u) * PAIR_HMAX;
  const int n = pair_unit(J, u, nt);
  if (threadIdx.x == 0) {
    __hip_atomic_store(f + h, ptag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < 20000; ++k) {
      bool all = true;
      for (int j = h + 1; j < n; ++j) all = all && __hip_atomic_load(f + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ptag;
      if (all) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// the partial slot of tile w' (follow-launch numbering; the lead's tile w + 1) of particle p
__host__ __device__ __forceinline__ size_t pair_slot(int p, int wf, int nt) { return ((size_t)p * (nt - 1) + wf) * T * T; }

// ----------------------------------------------------------------------------
// All-tile look-ahead in pieces (r6; k_step<SPLIT_NONE, 1>: the early-diagonal launches of config B,
// fewer tiles than workgroup slots). There a launch lasts as long as its longest
// item: from J = 3 the deep non-critical tiles, one depth-128J GEMM on one CU each (~95 us at J = 5,
// against ~60 us of work per CU; profiles/r5/crit_B_r5.txt). Here launch J (J >= 1) also runs, in
// pieces of at most LALL_PB 128-blocks each (ROLE_LPIECE), every GEMM of launch J+1 over the columns
// that are final before launch J — column J+1's L tiles I >= J+2 over [0, J) (covariance seed in
// piece 0), its U tiles K < J over [K, J), and the diagonal update of block J+2 over [0, J) — to
// partial slots; launch J+1's tiles and SYRK workgroup then sum their item's partials in piece
// order, run the one remaining 128-block (the columns of block J) and finish as before. Every item
// of a launch is then at most LALL_PB blocks of GEMM (or one block plus a finish), and the launch's
// chain is the diagonal factor and the critical tile's finish. The partials of launch J go to parity
// J & 1 of the buffer, so launch J+1 reads one half while it writes the other. Deterministic; the sum
// of partials rounds differently from one MFMA chain (within 1e-12 of the unsplit factor,
// test_all_tile_lookahead_pieces).
// (the look-ahead launches pass P, the piece size in blocks and the slots per particle packed in
// k_step's ptag)
__host__ __device__ __forceinline__ int lall_tag(int P, int pb, int smax) { return (pb << 28) | (P << 16) | smax; }
__host__ __device__ __forceinline__ int P_of(int tag) { return (tag >> 16) & 0xfff; }
__host__ __device__ __forceinline__ int pb_of(int tag) { return tag >> 28; }
__host__ __device__ __forceinline__ int smax_of(int tag) { return tag & 0xffff; }
__host__ __device__ __forceinline__ int lall_items(int J, int nt) {  // items launch J produces, per particle
  return J < 1 || J + 1 > nt - 1 ? 0 : (nt - 2 - J) + J + (J + 2 <= nt - 1 ? 1 : 0);
}
__host__ __device__ __forceinline__ int lall_depth(int J, int it, int nt) {  // in 128-blocks
  const int nLc = nt - 2 - J;
  return it < nLc ? J : it < nLc + J ? J - (it - nLc) : J;
}
__host__ __device__ __forceinline__ int lall_np(int J, int it, int nt, int pb) { return (lall_depth(J, it, nt) + pb - 1) / pb; }
__host__ __device__ __forceinline__ int lall_off(int J, int it, int nt, int pb) {
  int o = 0;
  for (int i = 0; i < it; ++i) o += lall_np(J, i, nt, pb);
  return o;
}
__host__ __device__ __forceinline__ int lall_total(int J, int nt, int pb) { return lall_off(J, lall_items(J, nt), nt, pb); }
// slot of piece s of item it produced by launch J for particle p (P particles in the group, smax slots
// per particle and parity)
__host__ __device__ __forceinline__ size_t lall_slot(int J, int it, int s, int p, int P, int nt, int smax, int pb) {
  return ((size_t)((J & 1) * P + p) * smax + lall_off(J, it, nt, pb) + s) * T * T;
}
// Workgroup b of a look-ahead launch past its diagonal, SYRK and tile workgroups (r = b - those): piece
// s of item it of particle p (items in order, their pieces in order, particles fastest)
__host__ __device__ __forceinline__ void lall_decode(int r, int J, int P, int nt, int pb, int& p, int& it, int& s) {
  p = r % P;
  int q = r / P;
  const int ni = lall_items(J, nt);
  for (it = 0; it < ni - 1; ++it) {
    const int n = lall_np(J, it, nt, pb);
    if (q < n) break;
    q -= n;
  }
  s = q;
}

// LDS of a k_step workgroup (doubles): the GEMM stages (DL_STAGE), the diagonal factor
// (DB_LDS), the staged U_JJ of the triangular finishes (TRI_LDS) with z_J behind
// it, or the coordinates of a covariance tile. ~77 KiB: two workgroups per CU.
constexpr int STEP_ZJ = TRI_LDS;      // z_J (128 doubles) beside the staged U_JJ
constexpr int STEP_XS = STEP_ZJ + T;  // flat finish: the U-tile column sums one wave hands the other (64)
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int STEP_LDS = cmax(cmax(DL_STAGE, DB_LDS), cmax(STEP_XS + 64, 2 * DMAX * T + 2 * T));
static_assert(STEP_LDS * 8 <= 80 * 1024, "two k_step workgroups per CU (160 KiB of LDS)");
// k_step<SPLIT_ALL> (one workgroup per CU: the launch budget is the CU count): the flat finish's
// reduction gets its own area behind the staged U_JJ, so U_JJ can be staged before the reduction
// (flat_piece)
constexpr int FLAT_RB = STEP_XS + 64;                 // 2 regions x 16 units x 128 doubles
constexpr int STEP_LDS_FLAT = FLAT_RB + 2 * 2048;
static_assert(STEP_LDS_FLAT >= STEP_LDS && STEP_LDS_FLAT * 8 <= 160 * 1024 && (FLAT_RB * 8) % 16 == 0, "flat LDS");
constexpr int STEP_NTH = Geo<T>::NTH;     // 512 threads: 8 waves, 128x16 per wave
static_assert(STEP_NTH == DNTH, "the fused diagonal runs on the step workgroup");

constexpr int STEP_WAVES_PER_SIMD = 4;  // 2 workgroups of 8 waves per CU
#ifdef GPF_WG_TRACE
// Diagnostic build only (-DGPF_WG_TRACE): per-workgroup start/end (s_memrealtime, 100 MHz)
// and hardware placement of every k_step workgroup, per block column J.
constexpr int WG_TRACE_J = 64, WG_TRACE_N = 4096;
__device__ unsigned long long g_wg_trace[WG_TRACE_J][WG_TRACE_N][3];
__device__ unsigned long long g_wg_phase[WG_TRACE_J][WG_TRACE_N][4];  // wave-0 phase ends (see step_item; [3]: a split piece's GEMM before its tree, a whole tile's U_JJ staged)
__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
// (r5: the latest wave's end of the phase: lane 0 of every wave that reaches it, atomic max)
#define GPF_PHASE(k)                                                                                   \
  if ((tid & 63) == 0 && J < WG_TRACE_J && blockIdx.x < WG_TRACE_N)                                  \
  __hip_atomic_fetch_max(&g_wg_phase[J][blockIdx.x][k], realtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define GPF_PHASE(k)
#endif

#ifndef GPF_FLAT_KOUTER  // 0: the all-tile split's seed element by element
#define GPF_FLAT_KOUTER 1
#endif
#ifndef GPF_COV_KOUTER  // 0: the covariance seed element by element (round 5)
#define GPF_COV_KOUTER 1
#endif
// K(R, C) block of one particle (R != C: no diagonal entries, so no noise term) straight into the
// accumulator layout (rows from block R, columns from block C), with k_build_cov's op order
// (bitwise the same values, kernel_func GP_func.py:56-65; the two blocks enter symmetrically —
// commuting products and sums — so K(J, I) = K(I, J)^T bitwise): the scaled coordinates and
// squared norms of the tile's 128 rows and 128 columns are staged in LDS first. Replaces the
// write of the K tile in the K build and its read back; only the diagonal blocks are still built
// (k_build_cov, diag_only).
template <bool KOUTER = (GPF_COV_KOUTER != 0)>
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
    } else {
      for (int k = 0; k < d; ++k) a[k * T + t] = 0.0;  // (padding: finite, replaced by 0 below)
    }
    (rows ? na : nb)[t] = nrm;
  }
  __syncthreads();
  // (r6) coordinate k outermost: the dot products accumulate in the accumulators themselves, the
  // lane's one column value per k is read once, and the runtime-d loop runs d times per tile instead
  // of per element — the seed's VALU work shrinks (it runs beside the co-resident workgroup's
  // MFMAs, where VALU issue is slow). Per element the same operations in the same order.
  if constexpr (KOUTER) {
    static_assert(Acc<T>::MBC == 1, "one column per lane");
    const int col = qd.col(0);
    const double b0 = sb[col];
#pragma unroll
    for (int mi = 0; mi < Acc<T>::MBR; ++mi) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc.v[mi][0][r] = sa[qd.row(mi, r)] * b0;
      __builtin_amdgcn_sched_barrier(0);  // (the row reads in groups of 4: not all 32 in flight)
    }
    for (int k = 1; k < d; ++k) {
      const double bk = sb[k * T + col];
#pragma unroll
      for (int mi = 0; mi < Acc<T>::MBR; ++mi) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc.v[mi][0][r] = fma(sa[k * T + qd.row(mi, r)], bk, acc.v[mi][0][r]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const double nc = nb[col];
    const bool cin = C * T + col < N;
#pragma unroll
    for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = qd.row(mi, r);
        double r2 = (na[row] + nc) - 2.0 * acc.v[mi][0][r];
        r2 = r2 > 0.0 ? r2 : 0.0;  // np.maximum(sq_dist, 0)
        acc.v[mi][0][r] = (cin && R * T + row < N) ? exp(-0.5 * r2) : 0.0;
        __builtin_amdgcn_sched_barrier(0);  // (one exp at a time: the 32 interleaved spilled)
      }
    __syncthreads();
    return;
  }
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
// Split-K pieces (SPLIT_ALL): piece 0 of an L tile seeds its partial with the covariance tile A_IJ
// (the unsplit path's accumulator seed) and takes SEED_CH fewer chunks for it, so that it ends its
// GEMM with the others (r4: the seed cost it ~11 us).
constexpr int SEED_CH = 4;  // chunks of GEMM piece 0's covariance seed stands for
// One piece's partial GEMM: piece boundaries over nch + e chunks, the first e of them standing
// for piece 0's seed (its covariance tile costs about SEED_CH chunks of GEMM), so that the seeded
// piece ends its GEMM with the others.
template <bool NN, bool NEG, bool SEEDED, typename Seed>
__device__ __forceinline__ void split_gemm(Acc<T>& acc, const double* Ap, int lda, const double* Bp, int ldb, int nch,
                                           int S, int s, double* smem, const Quad<T>& qd, Seed seed) {
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
}

// A partial (or node sum) to its 128 KiB slot in the accumulators' own layout: wave w's
// registers at bytes [16 KiB w, 16 KiB (w+1)), register pair (mi, h) of every lane as one 1 KiB
// block (16-B write-through stores, 1 KiB per wave instruction). Nothing but the split-K
// reductions reads the slots.
constexpr int NODE_WAVE = Acc<T>::MBR * Acc<T>::MBC * 2048;  // bytes per wave region
__device__ __forceinline__ void store_node(const Acc<T>& acc, double* slot, const Quad<T>& qd) {
  const auto ws = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(slot), 0, T * T * 8, 0x00020000);
  const int wb = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * NODE_WAVE;
#pragma unroll
  for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
    for (int ni = 0; ni < Acc<T>::MBC; ++ni)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double a0 = acc.v[mi][ni][2 * h], a1 = acc.v[mi][ni][2 * h + 1];
        const unsigned long long u0 = __builtin_bit_cast(unsigned long long, a0),
                                 u1 = __builtin_bit_cast(unsigned long long, a1);
        const __attribute__((ext_vector_type(4))) unsigned q4 = {(unsigned)u0, (unsigned)(u0 >> 32), (unsigned)u1,
                                                                  (unsigned)(u1 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(q4, ws, qd.lane * 16, wb + ((mi * Acc<T>::MBC + ni) * 2 + h) * 1024,
                                               16);  // sc1: write-through
      }
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

// ----------------------------------------------------------------------------
// Flat split-K finish (SPLIT_ALL; r5). The reduction tree above hands every tile's sum to one
// workgroup, which then also runs the whole finish (the triangular multiply of the 8 column
// slabs and, for an L tile, the 36-block diagonal update A_II -= L_IJ L_IJ^T) alone: for the
// single-particle prediction that was ~30 us of tree plus ~20 us of one-CU finish per launch, on
// every launch's chain. Here the np pieces of a tile share all of it:
//   A  every piece stores its partial to its slot (write-through, drained) and counts in (c[0]);
//   R  piece s < min(np, 8) owns the regions r = s + np k < 8 (at most 2: np >= SPLIT_MINP);
//      once all np partials are in, its 8 waves sum those regions' 1-KiB units over the slots
//      (slot order, so results are deterministic; 16 slots per round trip) into its LDS;
//   T  the region's two waves take the sum from LDS, wait for the diagonal block (U_JJ, z_J),
//      stage U_JJ and finish it: the triangular multiply (output row blocks split between the
//      two), the stores and the column partials (U tiles), or, for an L tile, its rows of L_IJ
//      also to slot 1 in the MFMA operand layout, then count in (c[1 + r], 2 per region);
//   C  (L tiles) the 8 np waves take the 36 lower 16x16 blocks of A_II -= L_IJ L_IJ^T, block
//      (ib, jb) as soon as the regions of slabs ib and jb are in: 32 MFMAs over k ascending with
//      A_II as the seed — the per-element MFMA sequence of syrk_rows; the diagonal blocks also
//      y_I -= L_IJ z_J for their rows.
// The hand-off reads bypass the caches (FLAT_LD, below). r5 (profiles/r5/predict_trace_*.txt):
// prediction N=4096, per launch 46-67 us of which the finish after the pieces' GEMMs ~20 us.
// Every wait is bounded (`spins`; timeout: info bit 2, the wave or piece leaves). No wait can hold
// the slots an awaited workgroup needs: the diagonal workgroups come first in the launch and wait
// for nothing; the np <= SPLIT_MAXS pieces of a tile have consecutive workgroup ids, which the
// dispatcher deals round-robin over the 8 XCDs and in order within each, so an XCD holds at most
// 4 pieces of a tile — a stalled XCD (64 slots) would need all its slots taken by pieces of the
// lowest incomplete tile. Counters: FLAT_CNT words per (particle, launch, tile), zeroed by the
// factorisation's memset, never reused within it.
constexpr int FLAT_CNT = 16;  // [0] partials stored; [1 + r]: the waves that finished region r of an L tile
                              // (its phase-C operands stored)
__host__ __device__ __forceinline__ int split_cnt_stride(int nt) {  // counter words per split tile and particle
  return FLAT_CNT * nt;
}
// Quad<128>::cb / 16 of wave r: the column slab held in wave region r of a slot (an involution, so
// also the region of slab s)
__device__ __forceinline__ int region_slab(int r) { return r < 4 ? r : 11 - r; }

// The flat finish's hand-offs read what other workgroups stored write-through (sc1) with loads
// that bypass L1 and L2 (sc0 sc1: from memory), after a relaxed poll of the counter, instead of an
// agent-scope acquire: that acquire invalidates the XCD's L2, and ~1000 waiting waves per launch
// issuing it thrashed the L2s of every XCD — the diagonal-update phase alone took ~25 us in the
// first launches (same box, prediction factorisation 2.44-2.57 -> 2.15-2.25 ms; profiles/r5/
// ab_flat_bypass.txt, predict_trace_bypass.txt). The data each reader needs was drained to memory
// before the counter moved (s_waitcnt vmcnt(0) after the write-through stores).
constexpr int FLAT_LD = 17;  // buffer-load cache policy of the flat finish's hand-off reads: sc0 | sc1
// Bounded wave-level wait for *c >= n (the reads after it use FLAT_LD); true: timed out (info bit 2).
__device__ __forceinline__ bool wave_wait(const unsigned* c, unsigned n, int* info, int spins) {
  int k = 0;
  while ((unsigned)__builtin_amdgcn_readfirstlane(
             (int)__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < n) {
    if (k++ >= spins) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(info, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  asm volatile("" ::: "memory");  // (no acquire: the reads that follow bypass the caches, FLAT_LD)
  return false;
}

// The same for the whole workgroup (thread 0 polls; ends with a barrier).
__device__ __forceinline__ bool group_wait(const unsigned* c, unsigned n, int* info, int spins, int* sflag) {
  if (threadIdx.x == 0) {
    int k = 0, late = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
      if (k++ >= spins) {
        __hip_atomic_fetch_or(info, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        late = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    asm volatile("" ::: "memory");  // (no acquire: FLAT_LD reads)
    *sflag = late;
  }
  __syncthreads();
  return *sflag != 0;
}

typedef unsigned u4v __attribute__((ext_vector_type(4)));

// Unit u summed over the np slots in slot order (phase R, local): 16 slots per round trip.
__device__ __forceinline__ d2 flat_sum_unit(const double* pt, int np, int u) {
  const int lane = threadIdx.x & 63;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(pt), 0, np * T * T * 8, 0x00020000);
  d2 sum = {0.0, 0.0};
  for (int i0 = 0; i0 < np; i0 += 16) {
    u4v q[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i0 + i < np) q[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (i0 + i) * (T * T * 8) + u * 1024, FLAT_LD);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i0 + i < np) {
        const d2 v = __builtin_bit_cast(d2, q[i]);
        sum = (i0 + i == 0) ? v : sum + v;
      }
  }
  return sum;
}
// A region's 16 summed units from LDS (1 KiB each, 16 B per lane) into the accumulator layout.
__device__ __forceinline__ void flat_lds_region(Acc<T>& acc, const double* s) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const d2 v = *reinterpret_cast<const d2*>(s + (2 * mi + h) * 128 + lane * 2);
      acc.v[mi][0][2 * h] = v.x;
      acc.v[mi][0][2 * h + 1] = v.y;
    }
}

// Phase T leaves each finished L region's rows of L_IJ in slot 1 in the MFMA operand layout: the
// triangular multiply's output lane (g, c) holds L(cb + c, 4 t + g) for t = 0..31 — exactly the
// A/B operand of k-step t of a 16x16 block product — stored as 16 pairs (t, t+1), 1 KiB per wave
// instruction. Phase C's operands are then 16 coalesced 16-B loads per slab, not 32 strided 8-B
// row reads.
__device__ __forceinline__ void flat_store_operand(const d4 (&o)[2], double* slot1, int r, int P) {
  const int lane = threadIdx.x & 63;
  const auto ws = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(slot1), 0, T * T * 8, 0x00020000);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; e += 2)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, d2{o[j][e], o[j][e + 1]}), ws, lane * 16,
                                             r * NODE_WAVE + (2 * (2 * P + j) + e / 2) * 1024, 16);  // write-through
}
// 8 k-steps (t0 .. t0+7) of a slab's operands: 4 coalesced 16-B loads
__device__ __forceinline__ void flat_load_operand8(double (&a)[8], const double* slot1, int r, int t0) {
  const int lane = threadIdx.x & 63;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(slot1), 0, T * T * 8, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const d2 v = __builtin_bit_cast(
        d2, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, r * NODE_WAVE + (t0 / 2 + i) * 1024, FLAT_LD));
    a[2 * i] = v.x;
    a[2 * i + 1] = v.y;
  }
}

// Phase C: block (ib, jb) (ib >= jb) of A_II -= L_IJ L_IJ^T: 32 MFMAs, k = 4 t + (lane >> 4)
// ascending, seeded with A_II (syrk_rows' operands and order per element); the diagonal blocks
// also y_I -= L_IJ z_J for their 16 rows (t ascending per lane, then the lane groups). The
// operands stream in 4 batches of 8 k-steps, two in flight (32 k-steps of both operands at once
// are 128 VGPRs: the compiler serialised their loads into several round trips).
// wait(): the block's regions are in (true: timed out — the block is abandoned); A_II's block,
// which nothing else in the launch touches, is read before it, beside the wait.
template <typename W>
__device__ __forceinline__ bool flat_syrk_block(double* Aii, size_t ld, const double* slot1, int ib, int jb, double* yi,
                                                const double* zj, W wait) {
  const int lane = threadIdx.x & 63, g = lane >> 4, cl = lane & 15;
  double* cp = launder(Aii + (size_t)(16 * ib + g) * ld + 16 * jb + cl);
  const int ra = region_slab(ib), rb = region_slab(jb);
  const bool diag = ib == jb;
  d4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = cp[(size_t)(4 * r) * ld];
  if (wait()) return true;
  const auto zs = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(zj), 0, T * 8, 0x00020000);
  double yr = 0.0;
  double a[2][8], b[2][8];
  flat_load_operand8(a[0], slot1, ra, 0);
  if (!diag) flat_load_operand8(b[0], slot1, rb, 0);
  flat_load_operand8(a[1], slot1, ra, 8);
  if (!diag) flat_load_operand8(b[1], slot1, rb, 8);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = q & 1;
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = mfma_neg_a(a[u][t], diag ? a[u][t] : b[u][t], acc);
    if (diag) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        yr = fma(a[u][t], __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zs, (4 * (8 * q + t) + g) * 8, 0, FLAT_LD)),
                 yr);
    }
    if (q + 2 < 4) {
      flat_load_operand8(a[u], slot1, ra, 8 * (q + 2));
      if (!diag) flat_load_operand8(b[u], slot1, rb, 8 * (q + 2));
    }
  }
  if (diag) {
    yr = sum_lane_groups(yr);
    if (g == 0) yi[16 * ib + cl] = yi[16 * ib + cl] - yr;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) cp[(size_t)(4 * r) * ld] = acc[r];
  return false;
}

// One piece (sidx of np) of tile w of launch J under the flat finish (see above); LT: an L tile.
template <bool LT>
__device__ __forceinline__ void flat_piece(int J, int w, int p, int nt, int Npad, double* __restrict__ Lp,
                                        double* __restrict__ Up, double* __restrict__ yp, double* __restrict__ s2p,
                                        double* __restrict__ szp, int* __restrict__ info, int N,
                                        const double* __restrict__ x, const double* __restrict__ lp, int d, int np,
                                        int sidx, int S2, double* __restrict__ part, unsigned* __restrict__ cnt,
                                        int* sflag, const int* __restrict__ dflag, int spins, double* lds) {
  const int tid = threadIdx.x;
  const size_t ld = (size_t)Npad;
  const int nL = nt - 1 - J;
  const int I = J + 1 + w, K = w - nL;
  const Quad<T> qd;
  const int g = qd.lane >> 4, cl = qd.lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* pt = part + (size_t)(p * (nt - 1) + w) * S2 * T * T;
  unsigned* ca = cnt + (size_t)p * (nt - 1) * split_cnt_stride(nt) + (size_t)(J * (nt - 1) + w) * FLAT_CNT;
  // A: the partial (piece 0 of an L tile seeded with the covariance tile A_IJ^T)
  Acc<T> acc;
  if (LT)
    split_gemm<false, true, true>(acc, Lp + (size_t)J * T * ld, Npad, Lp + (size_t)I * T * ld, Npad, J * T / DL_KC,
                                  np, sidx, lds, qd, [&](Acc<T>& a) {
                                    // (k outer here too: prediction factor -1.8% despite a 20 B private segment, ab_cov_seed_kouter.txt)
                                    cov_tile_acc<GPF_FLAT_KOUTER != 0>(a, qd, x, lp, d, N, J, I, lds);
                                  });
  else  // (the triangular first block runs dense: its upper part holds zeros)
    split_gemm<true, false, false>(acc, Lp + (size_t)J * T * ld + (size_t)K * T, Npad,
                                   Up + (size_t)K * T * ld + (size_t)K * T, Npad, (J - K) * T / DL_KC, np, sidx, lds, qd,
                                   [](Acc<T>&) {});
  store_node(acc, pt + (size_t)sidx * T * T, qd);
  acc.zero();  // (dead until phase T reloads it: a constant, not 64 registers held across phase R)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's part of the partial drained
  __syncthreads();
  if (tid == 0) __hip_atomic_fetch_add(ca, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  GPF_PHASE(3);
  // T (with R): piece s < min(np, 8) finishes regions r = s + np k < 8 (nr of them). With np >= 4
  // (always: SPLIT_MINP) two waves share a region (on different SIMDs): the triangular multiply's
  // output row blocks {0,1, 6,7} (P = 0, 3) and {2,3, 4,5} (P = 1, 2), 72 of its 144 MFMAs each.
  static_assert(SPLIT_MINP >= 4, "flat_piece: two waves per region, at most 2 regions per piece");
  const int half = wave & 1;
  const int r = sidx + np * (wave >> 1);  // the region this wave finishes (if < 8)
  double* slot1 = pt + (size_t)T * T;
  if (sidx < 8) {
    double* zj = lds + STEP_ZJ;
    // (r5) if the diagonal block is already published once this piece's partial is in (the deep
    // launches: the diagonal factor ends before the GEMMs), U_JJ and z_J are staged while the other
    // pieces' partials arrive, and the reduction goes to its own area (FLAT_RB); otherwise the
    // reduction runs first, as it can before the diagonal block exists
    if (threadIdx.x == 0) *sflag = __hip_atomic_load(dflag + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= J;
    __syncthreads();
    const bool early = *sflag != 0;
    __syncthreads();  // (sflag is the waits' broadcast word)
    double* rb = early ? lds + FLAT_RB : lds;
    if (early) {
      if (wait_diag(dflag + p, J, info, spins, sflag)) return;  // (published: one poll and the acquire)
      if (!LT && tid < T) zj[tid] = yp[J * T + tid];
      tri_to_lds(Up + (size_t)J * T * ld + (size_t)J * T, ld, lds);  // (its barrier also publishes z_J)
    }
    if (group_wait(ca, (unsigned)np, info, spins, sflag)) return;
    // R, local: the piece's 8 waves sum its regions' 16 1-KiB units each over the np slots (slot
    // order) into LDS, where the region's two waves pick their operand up — no store, drain,
    // counter and reload through memory between the reduction and the triangular multiply
    const int nr = (8 - sidx + np - 1) / np;
    for (int i = wave; i < 16 * nr; i += 8) {
      const int k = i >> 4, j = i & 15;
      const d2 sum = flat_sum_unit(pt, np, (sidx + np * k) * 16 + j);
      *reinterpret_cast<d2*>(rb + k * 2048 + j * 128 + qd.lane * 2) = sum;
    }
    __syncthreads();
    GPF_PHASE(0);
    if (r < 8) flat_lds_region(acc, rb + ((r - sidx) / np) * 2048);
    if (!early) {
      if (wait_diag(dflag + p, J, info, spins, sflag)) return;  // U_JJ, z_J (its barrier: the region reads done)
      if (!LT && tid < T) zj[tid] = yp[J * T + tid];
      tri_to_lds(Up + (size_t)J * T * ld + (size_t)J * T, ld, lds);  // (its barrier also publishes z_J)
    }
    const bool outer = half == 0;  // this wave's output row blocks: P = 0, 3 (outer) or 1, 2
    const int cb = 16 * region_slab(r < 8 ? r : 0);
    if (LT) {
      if (r < 8) {
        // L_IJ^T = U_JJ D for the slab's 16 columns of D (rows cb.. of L_IJ); the rows also to slot 1
        // in the operand layout (y_I -= L_IJ z_J follows in phase C, from those operands)
        double* lrow = launder(Lp + (size_t)(I * T + cb + cl) * ld + (size_t)J * T + g);
#pragma unroll
        for (int P = 0; P < 4; ++P) {
          if (outer != (P == 0 || P == 3)) continue;
          d4 o[2];
          switch (P) {
            case 0: trmm_acc<0, false>(o, acc, lds); break;
            case 1: trmm_acc<1, false>(o, acc, lds); break;
            case 2: trmm_acc<2, false>(o, acc, lds); break;
            default: trmm_acc<3, false>(o, acc, lds); break;
          }
          flat_store_operand(o, slot1, r, P);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) lrow[16 * (2 * P + j) + 4 * e] = o[j][e];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the region's operands drained
        if (qd.lane == 0) __hip_atomic_fetch_add(ca + 1 + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      // U_JK = -U_JJ W; the column partials of colsum(U^2) and U^T z: each wave's rows in P order,
      // the 4 lane groups, then the two waves' sums, half 0's first
      double a2 = 0.0, az = 0.0;
      if (r < 8) {
        double* ucol = launder(Up + (size_t)(J * T + g) * ld + (size_t)K * T + cb + cl);
#pragma unroll
        for (int P = 0; P < 4; ++P) {
          if (outer != (P == 0 || P == 3)) continue;
          d4 o[2];
          switch (P) {
            case 0: trmm_acc<0, true>(o, acc, lds); break;
            case 1: trmm_acc<1, true>(o, acc, lds); break;
            case 2: trmm_acc<2, true>(o, acc, lds); break;
            default: trmm_acc<3, true>(o, acc, lds); break;
          }
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int row = 16 * (2 * P + j) + 4 * e;  // + g
              const double v = o[j][e];
              ucol[(size_t)row * ld] = v;
              a2 = fma(v, v, a2);
              az = fma(v, zj[row + g], az);
            }
        }
        a2 = sum_lane_groups(a2);
        az = sum_lane_groups(az);
      }
      // half 1's sums for half 0: only the waves that finish a region (r < 8: pairs wave >> 1 <= 1,
      // since np >= SPLIT_MINP >= 4) hand sums over, 32 doubles per pair inside the 64 of STEP_XS;
      // the waves with r >= 8 must not store (pairs 2 and 3 wrote zeros into FLAT_RB,
      // the early path's reduction area, racing with its reads)
      static_assert(STEP_XS + 32 * ((8 + SPLIT_MINP - 1) / SPLIT_MINP) <= FLAT_RB, "flat finish: XS hand-over area");
      double* xs = lds + STEP_XS + 32 * (wave >> 1);
      if (r < 8 && half == 1 && g == 0) {
        xs[2 * cl] = a2;
        xs[2 * cl + 1] = az;
      }
      __syncthreads();  // (every wave of the piece: none has left since the diagonal wait)
      if (r < 8 && half == 0 && g == 0) {
        const size_t poff = ((size_t)p * nt + J) * Npad + (size_t)K * T + cb + cl;
        s2p[poff] = a2 + xs[2 * cl];
        szp[poff] = az + xs[2 * cl + 1];
      }
    }
  }
  GPF_PHASE(1);
  if (!LT) return;
  // C (block b = ib (ib + 1) / 2 + jb waits for the regions of slabs ib and jb only; the diagonal
  // blocks also apply y_I -= L_IJ z_J for their slab's rows, from the same operands)
  const unsigned ready = 2u;  // the region's two waves
  double* Aii = Lp + (size_t)I * T * ld + (size_t)I * T;
  for (int b = sidx * 8 + wave; b < 36; b += 8 * np) {
    int ib = 0;
    while ((ib + 1) * (ib + 2) / 2 <= b) ++ib;
    const int jb = b - ib * (ib + 1) / 2;
    if (flat_syrk_block(Aii, ld, slot1, ib, jb, ib == jb ? yp + (size_t)I * T : nullptr, yp + (size_t)J * T, [&] {
          return wave_wait(ca + 1 + region_slab(ib), ready, info, spins) ||
                 wave_wait(ca + 1 + region_slab(jb), ready, info, spins);
        }))
      return;
  }
  GPF_PHASE(2);
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

// A partial from its slot in the accumulators' own layout (store_node's: wave w's 16 KiB, one 1 KiB
// block per register pair and 16 B per lane), read back by the same wave layout: 16-B loads.
__device__ __forceinline__ void load_node(Acc<T>& acc, const double* slot) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(slot), 0, T * T * 8, 0x00020000);
  const int wb = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * NODE_WAVE, lane = threadIdx.x & 63;
#pragma unroll
  for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const d2 v = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, wb + (mi * 2 + h) * 1024, 0));
      acc.v[mi][0][2 * h] = v.x;
      acc.v[mi][0][2 * h + 1] = v.y;
    }
}

// Lead launch J, ROLE_PLA: block column J+1's tile (the lead's tile w = w' + 1) over the columns < J,
// the GEMM the follow launch would otherwise stream again — L tile I = J+1+w: the covariance seed
// A_{J+1,I}^T (cov_tile_acc) minus L_{J+1,<J} L_{I,<J}^T; U tile K: L_{J+1,[K,J)} U_{[K,J),K} (its first
// block triangular) — to the particle's slot w' (plain stores: the follow launch reads it after the
// launch boundary).
__device__ __forceinline__ void pla_item(int J, int w, int p, int nt, int Npad, const double* __restrict__ Lb,
                                         const double* __restrict__ Ub, int N, const double* __restrict__ x,
                                         const double* __restrict__ ls, int d, double* __restrict__ pb, double* lds) {
  const size_t ld = (size_t)Npad;
  const int nL = nt - 1 - J;
  const double* Lp = Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  Acc<T> acc;
  if (w < nL) {
    const int I = J + 1 + w;
    cov_tile_acc(acc, qd, x, ls + (size_t)p * d, d, N, J + 1, I, lds);
    gemm_stream_dl<false, true>(acc, Lp + (size_t)(J + 1) * T * ld, Npad, Lp + (size_t)I * T * ld, Npad, J * T, lds, qd);
  } else {
    const int K = w - nL;
    const double* Up = Ub + (size_t)p * ld * ld;
    acc.zero();
    gemm_stream_dl<true, false, TRI_B_KGEC>(acc, Lp + (size_t)(J + 1) * T * ld + (size_t)K * T, Npad,
                                            Up + (size_t)K * T * ld + (size_t)K * T, Npad, (J - K) * T, lds, qd);
  }
  store_node(acc, pb + pair_slot(p, w - 1, nt), qd);
}

// Lead launch J, ROLE_SYRKP: A_{J+2,J+2} -= L_{J+2,<J} L_{J+2,<J}^T in place (plain stores; the follow
// launch's critical tile continues with blocks J and J+1).
__device__ __forceinline__ void syrkp_item(int J, int p, int Npad, double* __restrict__ Lb, double* lds) {
  const size_t ld = (size_t)Npad;
  const int I = J + 2;
  double* Lp = Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  syrk_tile<false>(Lp + (size_t)I * T * ld + (size_t)I * T, ld, Lp + (size_t)I * T * ld, Npad, J * T, lds, qd);
}

// Block layout of a look-ahead launch: [diagonal P][SYRK P] then the tiles and the pieces — tiles
// first (pair bit 2 clear) or the pieces first (bit 2 set: the pieces wait for nothing, the tiles
// for the diagonal block anyway). nstd = the diagonal, SYRK and tile workgroups.
__host__ __device__ __forceinline__ int lall_head(int P, int nt, int nstd) { return nstd - P * (nt - 1); }
__host__ __device__ __forceinline__ bool lall_is_piece(int b, int J, int P, int nt, int nstd, int bits, int tag) {
  if (!(bits & 4)) return b >= nstd;
  const int h = lall_head(P, nt, nstd);
  return b >= h && b < h + P * lall_total(J, nt, pb_of(tag));
}
__host__ __device__ __forceinline__ int lall_piece_index(int b, int P, int nt, int nstd, int bits) {
  return (bits & 4) ? b - lall_head(P, nt, nstd) : b - nstd;
}
// (pieces first: the block index step_decode sees for a diagonal, SYRK or tile workgroup)
__host__ __device__ __forceinline__ int lall_tile_block(int b, int J, int P, int nt, int nstd, int tag) {
  return b < lall_head(P, nt, nstd) ? b : b - P * lall_total(J, nt, pb_of(tag));
}
// acc += a partial in store_node's layout (its 16-B units added as they arrive: no second accumulator set)
__device__ __forceinline__ void add_node(Acc<T>& acc, const double* slot) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(slot), 0, T * T * 8, 0x00020000);
  const int wb = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * NODE_WAVE, lane = threadIdx.x & 63;
#pragma unroll
  for (int mi = 0; mi < Acc<T>::MBR; ++mi)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const d2 v = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, wb + (mi * 2 + h) * 1024, 0));
      acc.v[mi][0][2 * h] = acc.v[mi][0][2 * h] + v.x;
      acc.v[mi][0][2 * h + 1] = acc.v[mi][0][2 * h + 1] + v.y;
    }
}
// the summed partials of item it (launch J-1's pieces, in piece order)
__device__ __forceinline__ void lall_seed(Acc<T>& acc, const double* lb, int J, int it, int p, int tag, int nt) {
  const int P = P_of(tag), smax = smax_of(tag), pb = pb_of(tag);
  const int np = lall_np(J - 1, it, nt, pb);
  const double* s0 = lb + lall_slot(J - 1, it, 0, p, P, nt, smax, pb);
  load_node(acc, s0);
  for (int s = 1; s < np; ++s) add_node(acc, s0 + (size_t)s * T * T);
}

// ROLE_LPIECE: piece s of item it of launch J (see lall_items)
__device__ __forceinline__ void lall_piece(int J, int it, int s, int p, int nt, int Npad, const double* __restrict__ Lb,
                                           const double* __restrict__ Ub, int N, const double* __restrict__ x,
                                           const double* __restrict__ ls, int d, double* __restrict__ lb, int tag,
                                           double* lds) {
  const size_t ld = (size_t)Npad;
  const int pb = pb_of(tag);
  const int nLc = nt - 2 - J, depth = lall_depth(J, it, nt);
  const int b0 = s * pb, nb = min(pb, depth - b0);
  const double* Lp = Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  Acc<T> acc;
  if (it < nLc) {  // L tile I of column J+1: (A_{J+1,I} seed) - L_{J+1,[b0,b0+nb)} L_{I,[b0,b0+nb)}^T
    const int I = J + 2 + it;
    if (s == 0) cov_tile_acc(acc, qd, x, ls + (size_t)p * d, d, N, J + 1, I, lds);
    else acc.zero();
    gemm_stream_dl<false, true>(acc, Lp + (size_t)(J + 1) * T * ld + (size_t)b0 * T, Npad,
                                Lp + (size_t)I * T * ld + (size_t)b0 * T, Npad, nb * T, lds, qd);
  } else if (it < nLc + J) {  // U tile K: L_{J+1,K+[b0,b0+nb)} U_{K+[b0,b0+nb),K} (U_KK lower triangular)
    const int K = it - nLc;
    const double* Up = Ub + (size_t)p * ld * ld;
    const double* A = Lp + (size_t)(J + 1) * T * ld + (size_t)(K + b0) * T;
    const double* B = Up + (size_t)(K + b0) * T * ld + (size_t)K * T;
    acc.zero();
    if (s == 0) gemm_stream_dl<true, false, TRI_B_KGEC>(acc, A, Npad, B, Npad, nb * T, lds, qd);
    else gemm_stream_dl<true, false>(acc, A, Npad, B, Npad, nb * T, lds, qd);
  } else {  // the diagonal update of block J+2 (lower part; piece 0 seeded with A_{J+2,J+2})
    const double* Ar = Lp + (size_t)(J + 2) * T * ld + (size_t)b0 * T;
    if (s == 0) acc.load(qd, Lp + (size_t)(J + 2) * T * ld + (size_t)(J + 2) * T, ld);
    else acc.zero();
    // (dense: the lower-only pattern with the whole accumulator live spilled k_step<0,1> — 802 VGPRs,
    // 312 B/lane; the upper blocks only ever hold A's mirror, never read)
    gemm_stream_dl<false, true>(acc, Ar, Npad, Ar, Npad, nb * T, lds, qd);
  }
  store_node(acc, lb + lall_slot(J, it, s, p, P_of(tag), nt, smax_of(tag), pb), qd);
}

// SYRK workgroup of a look-ahead launch J >= 2: S = A_{J+1,J+1} - L_{J+1,<J} L_{J+1,<J}^T from launch
// J-1's pieces over [0, J-1) (item nt-2) plus block column J-1, published like syrk_item's.
__device__ __forceinline__ void lall_syrk_item(int J, int p, int nt, int Npad, double* __restrict__ Lb,
                                               int* __restrict__ yflag, const double* __restrict__ lb, int tag,
                                               double* lds) {
  const size_t ld = (size_t)Npad;
  const int I = J + 1;
  double* Lp = Lb + (size_t)p * ld * ld;
  const Quad<T> qd;
  Acc<T> acc;
  lall_seed(acc, lb, J, nt - 2, p, tag, nt);
  const double* Ar = Lp + (size_t)I * T * ld + (size_t)(J - 1) * T;
  gemm_stream_dl<false, true>(acc, Ar, Npad, Ar, Npad, T, lds, qd);  // (dense, as lall_piece's)
  acc.store_wt(qd, Lp + (size_t)I * T * ld + (size_t)I * T, ld);  // (the upper half: A's mirror, never read)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(yflag + p, J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The finished L and U tiles' stores in step_item (r6: non-temporal stores measured 1362-1365 vs
// 1372-1376 evals/s on C, same box; profiles/r6/ab_store_nt_groups.txt)
__device__ __forceinline__ void tile_st(double* p, double v) { *p = v; }

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
                                          int spins, int la, const double* __restrict__ lab, int pair,
                                          const double* __restrict__ pb, int ptag, double* lds) {
  const int tid = threadIdx.x;
  const int nL = nt - 1 - J;
  // (paired block columns exist only in the fused-diagonal schedule: the other instantiations keep
  // their register allocation)
  constexpr bool PAIRS = SPLIT == SPLIT_NONE && !ED;
  const bool follow = PAIRS && pair == 2;
  // all-tile look-ahead (early-diagonal launches): this launch's tiles seed from launch J-1's pieces
  constexpr bool LALL = SPLIT == SPLIT_NONE && ED;
  const bool lseed = LALL && (pair & 2) && J >= 2;
  const size_t ld = (size_t)Npad;
  if (SPLIT != SPLIT_NONE && role == ROLE_IDLE) return;
  double* Lp = Lb + (size_t)p * ld * ld;
  double* Up = Ub + (size_t)p * ld * ld;
  double* yp = yb + (size_t)p * Npad;
  if constexpr (SPLIT == SPLIT_ALL) {
    static_assert(ED, "the all-tile split runs with the early diagonal factor (host: early_diag)");
    // (every tile of the launch: the single-piece ones, ROLE_WHOLE, finish the same way)
    const int np = split_all_pieces(J, w, nt, S);
if (w < nL)
      flat_piece<true>(J, w, p, nt, Npad, Lp, Up, yp, s2p, szp, info + p, N, x, ls + (size_t)p * d, d, np, sidx, S2, part,
                       cnt, sflag, dflag, spins, lds);
    else
      flat_piece<false>(J, w, p, nt, Npad, Lp, Up, yp, s2p, szp, info + p, N, x, ls + (size_t)p * d, d, np, sidx, S2, part,
                        cnt, sflag, dflag, spins, lds);
    return;
  }
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
    if (SPLIT == SPLIT_NONE && ED && (la & 2) && I == J + 1) {
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
    } else if (lseed) {
      // the pieces of launch J-1 (seed and the columns < J-1), then block column J-1
      lall_seed(acc, pb, J, w, p, ptag, nt);
      gemm_stream_dl<false, true>(acc, Lp + (size_t)J * T * ld + (size_t)(J - 1) * T, Npad,
                                  Lp + (size_t)I * T * ld + (size_t)(J - 1) * T, Npad, T, lds, qd);
    } else if (follow) {
      // follow launch: the lead's partial (seed and the columns < J-1), then block column J-1
      load_node(acc, pb + pair_slot(p, w, nt));
      gemm_stream_dl<false, true>(acc, Lp + (size_t)J * T * ld + (size_t)(J - 1) * T, Npad,
                                  Lp + (size_t)I * T * ld + (size_t)(J - 1) * T, Npad, T, lds, qd);
    } else {
      cov_tile_acc(acc, qd, x, lp, d, N, J, I, lds);
      if (J > 0)
        gemm_stream_dl<false, true>(acc, Lp + (size_t)J * T * ld, Npad, Lp + (size_t)I * T * ld, Npad, J * T, lds, qd);
    }
    GPF_PHASE(0);
    if (ED && wait_diag(dflag + p, J, info + p, spins, sflag)) return;  // U_JJ, z_J (launch 0 too)
    if (tid < T) zj[tid] = yp[J * T + tid];
    tri_to_lds(Ujj, ld, lds);  // (its barrier also publishes z_J)
    GPF_PHASE(3);
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
          tile_st(&lrow[16 * (2 * P + j) + 4 * e], o[j][e]);
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
    if (follow && I == J + 1) {
      // the lead's ROLE_SYRKP left A_II reduced over the columns < J-1: blocks J-1 and J remain (one
      // 256-deep update, the chunks in the order the SYRK workgroup and this tile would run them)
      syrk_tile<false>(Aii, ld, Aij - T, Npad, 2 * T, lds, qd);
    } else if (!defer_on || I == J + 1) {
      if (defer_on && J > 0 && wait_diag(yflag + p, J, info + p, spins, sflag)) return;  // S published
      syrk_tile<false>(Aii, ld, Aij, Npad, T, lds, qd);
    }
    GPF_PHASE(2);
    if (!ED && I == J + 1) {  // fused diagonal factor of block J+1 (A_II, y_I fully reduced)
      __syncthreads();
      const size_t poff = ((size_t)p * nt + I) * Npad + (size_t)I * T;
      __builtin_amdgcn_s_setprio(3);  // latency-critical: the next launch waits for this block
      factor128(Aii, Up + (size_t)I * T * ld + (size_t)I * T, ld, yp + I * T, s2p + poff, szp + poff, info + p, lds);
    }
  } else {
    const int K = w - nL;
    double* Ujk = Up + (size_t)J * T * ld + (size_t)K * T;
    Acc<T> acc;
    // W = L_J,[K,J) U_[K,J),K (U_KK is lower triangular: the wave's first chunks add zeros)
    if (lseed && K < J - 1) {
      lall_seed(acc, pb, J, w, p, ptag, nt);
      gemm_stream_dl<true, false>(acc, Lp + (size_t)J * T * ld + (size_t)(J - 1) * T, Npad,
                                  Up + (size_t)(J - 1) * T * ld + (size_t)K * T, Npad, T, lds, qd);
    } else if (follow && K < J - 1) {
      // follow launch: the lead's partial over [K, J-1), then block row J-1 of U's column panel K
      load_node(acc, pb + pair_slot(p, w, nt));
      gemm_stream_dl<true, false>(acc, Lp + (size_t)J * T * ld + (size_t)(J - 1) * T, Npad,
                                  Up + (size_t)(J - 1) * T * ld + (size_t)K * T, Npad, T, lds, qd);
    } else {
      acc.zero();
      gemm_stream_dl<true, false, TRI_B_KGEC>(acc, Lp + (size_t)J * T * ld + (size_t)K * T, Npad,
                                              Up + (size_t)K * T * ld + (size_t)K * T, Npad, (J - K) * T, lds, qd);
    }
    GPF_PHASE(0);
    if (ED && wait_diag(dflag + p, J, info + p, spins, sflag)) return;  // U_JJ, z_J (U tiles exist for J > 0 only)
    if (tid < T) zj[tid] = yp[J * T + tid];
#ifdef GPF_WG_TRACE
    tri_to_lds(Ujj, ld, lds, [&] { GPF_PHASE(2); });  // (U tiles: slot 2 = the staging's loads arrived)
#else
    tri_to_lds(Ujj, ld, lds);
#endif
    GPF_PHASE(3);
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
          tile_st(&ucol[(size_t)row * ld], v);
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

// SPLIT: SPLIT_ALL cuts every tile (launches with few tiles; always with the early diagonal
// factor, ED = 1); SPLIT_NONE carries no split code at all, so its register allocation is that of
// the plain schedule.
// (SPLIT_ALL's flat finish takes ~110 KiB of LDS: one workgroup per CU, 2 waves per SIMD — the
// occupancy its register allocation is asked for, instead of an unreachable 4)
template <int SPLIT, int ED>
__global__ __launch_bounds__(STEP_NTH, SPLIT == SPLIT_ALL ? 2 : STEP_WAVES_PER_SIMD) void k_step(int J, int nt, int Npad, double* __restrict__ Lb,
                                                  double* __restrict__ Ub, double* __restrict__ yb,
                                                  double* __restrict__ s2p, double* __restrict__ szp,
                                                  int* __restrict__ info, int P, int grp, int N,
                                                  const double* __restrict__ x, const double* __restrict__ ls,
                                                  int d, int S, int S2, double* __restrict__ part,
                                                  unsigned* __restrict__ cnt, int* __restrict__ dflag, int ed,
                                                  int* __restrict__ yflag, int defer, int sy, int spins, int la,
                                                  double* __restrict__ lab, int pair, double* __restrict__ pb,
                                                  int* __restrict__ pstart, int ptag,
                                                  unsigned long long* __restrict__ clk) {
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
  __shared__ __attribute__((aligned(16))) double lds[SPLIT == SPLIT_ALL ? STEP_LDS_FLAT : STEP_LDS];
  __shared__ int sflag;
  int p, w, sidx = 0;
  constexpr bool PAIRS = SPLIT == SPLIT_NONE && !ED;
  int uh = 0, lit = -1;
  constexpr bool LALL = SPLIT == SPLIT_NONE && ED;
  // look-ahead launches: the pieces follow the diagonal, SYRK and tile workgroups (lall_decode)
  const int nstd = (ED && ed ? P : 0) + (SPLIT != SPLIT_ALL && sy ? P : 0) + P * (nt - 1);
  int role;
  if (PAIRS && pair == 1) {
    role = pair_decode((int)blockIdx.x, J, P, nt, p, w, &uh);
  } else if (LALL && (pair & 1) && lall_is_piece((int)blockIdx.x, J, P, nt, nstd, pair, ptag)) {
    lall_decode(lall_piece_index((int)blockIdx.x, P, nt, nstd, pair), J, P, nt, pb_of(ptag), p, lit, sidx);
    w = -1;
    role = ROLE_LPIECE;
  } else {
    role = step_decode<SPLIT>(LALL && (pair & 5) == 5 ? lall_tile_block((int)blockIdx.x, J, P, nt, nstd, ptag) : (int)blockIdx.x, J,
                              P, nt, grp, S, ED && ed, SPLIT != SPLIT_ALL && sy,
                              SPLIT == SPLIT_NONE && ED && (la & 1) && !sy, p, w, sidx,
                              SPLIT == SPLIT_NONE && ED && (la & 32) != 0);
  }
#ifdef GPF_CHECK
  // diagnostic build (-DGPF_CHECK): every index the workgroup derives its addresses from, checked
  // against the launch's extents before any access (an out-of-range role prints and does nothing)
  {
    bool ok = p >= 0 && p < P && J >= 0 && J < nt && Npad == nt * T && S >= 1 && S2 >= 1 && S2 <= SPLIT_MAXS;
    if (role == ROLE_SYRK) ok = ok && w == -1 && J >= 1 && J <= nt - 2 && yflag != nullptr;
    else if (role == ROLE_LA) ok = ok && w == -1 && J >= 1 && J + 2 < nt && lab != nullptr;
    else if (role == ROLE_DIAG) ok = ok && w == -1 && ED && dflag != nullptr;
    else if (role == ROLE_PLA) ok = ok && PAIRS && pair == 1 && pb != nullptr && w >= 1 && w < nt - 1 && J >= 1 &&
                                     (w >= nt - 1 - J || J + 1 + w < nt);
    else if (role == ROLE_SYRKP) ok = ok && PAIRS && pair == 1 && w == 1 && J >= 1 && J + 2 <= nt - 1;
    else if (role == ROLE_LPIECE) ok = ok && LALL && pb != nullptr && lit >= 0 && lit < lall_items(J, nt) && sidx >= 0 &&
                                       sidx < lall_np(J, lit, nt, pb_of(ptag)) && P_of(ptag) == P &&
                                       lall_off(J, lit, nt, pb_of(ptag)) + sidx < smax_of(ptag);
    else if (role != ROLE_IDLE) ok = ok && w >= 0 && w < nt - 1 && sidx >= 0 && (pair != 2 || pb != nullptr) &&
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
  if (PAIRS && pair == 1 && pstart) pair_start_sync(J, role == ROLE_SYRK ? 0 : w, uh, p, nt, pstart, ptag);
  if (LALL && role == ROLE_LPIECE) {
    lall_piece(J, lit, sidx, p, nt, Npad, Lb, Ub, N, x, ls, d, pb, ptag, lds);
  } else if (LALL && role == ROLE_SYRK && (pair & 2) && J >= 2) {
    lall_syrk_item(J, p, nt, Npad, Lb, yflag, pb, ptag, lds);
  } else if (PAIRS && role == ROLE_PLA) {
    pla_item(J, w, p, nt, Npad, Lb, Ub, N, x, ls, d, pb, lds);
  } else if (PAIRS && role == ROLE_SYRKP) {
    syrkp_item(J, p, Npad, Lb, lds);
  } else if (SPLIT != SPLIT_ALL && role == ROLE_SYRK) {
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
    factor128<true>(Lb + off, Ub + off, ld, yb + (size_t)p * Npad + J * T, s2p + poff, szp + poff, info + p, lds,
                    dflag + p, J);
  } else {
    step_item<SPLIT, ED>(role, J, w, p, nt, Npad, Lb, Ub, yb, s2p, szp, info, N, x, ls, d, S, S2, sidx, part, cnt, &sflag,
                         dflag, yflag, defer, spins, la, lab, pair, pb, ptag, lds);
  }
  span.stop(clk);
#ifdef GPF_WG_TRACE
  __syncthreads();
  if (tid == 0 && J < WG_TRACE_J && blockIdx.x < WG_TRACE_N) g_wg_trace[J][blockIdx.x][1] = realtime();
#endif
}


// Debug / measurement hook (gpf_debug_factor128): factor128 on n host-given 128x128 blocks, one
// workgroup each (in place: A -> L, the U blocks, y -> z, the partials); cyc[b] = the workgroup's
// s_memtime cycles from the first load to the last store (nullable).
__global__ __launch_bounds__(DNTH) void k_debug_factor128(double* __restrict__ L, double* __restrict__ U,
                                                          double* __restrict__ y, double* __restrict__ s2,
                                                          double* __restrict__ sz, int* __restrict__ bad,
                                                          unsigned long long* __restrict__ cyc) {
  __shared__ __attribute__((aligned(16))) double lds[DB_LDS];
  const int b = blockIdx.x;
  unsigned long long t0 = 0, t1 = 0;
  __syncthreads();
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  factor128(L + (size_t)b * T * T, U + (size_t)b * T * T, T, y + (size_t)b * T, s2 + (size_t)b * T, sz + (size_t)b * T,
            bad + b, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (cyc && threadIdx.x == 0) cyc[b] = t1 - t0;
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

template <int NS>
__global__ __launch_bounds__(STEP_NTH, NS >= 3 ? 2 : STEP_WAVES_PER_SIMD) void k_gemm_bench(int mode, int D, int Npad, int P,
                                                                                   const double* __restrict__ Lb,
                                                                                   double* __restrict__ C,
                                                                                   unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[NS * DL_BUF];
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
    gemm_stream_dl<true, false, TRI_NONE, NS>(acc, Lp + (size_t)I * T * ld, Npad, Lp + (size_t)w * T, Npad, D, smem, qd);
  else
    gemm_stream_dl<false, true, TRI_NONE, NS>(acc, Lp + (size_t)J * T * ld, Npad, Lp + (size_t)I * T * ld, Npad, D, smem, qd);
  acc.store(qd, C + (size_t)b * T * T, T);
  span.stop(clk);
}

}  // namespace gpf
