// gpf_common.hip — shared device machinery for the gfx950 GP-fit kernels:
// FP64 MFMA tile GEMMs (streamed through LDS or fully LDS-resident), the
// accumulator ownership map and small reduction helpers.
//
// All arithmetic is IEEE fp64 (an fp32 factor misses the 1e-6
// tolerance by orders of magnitude). The file is compiled with -ffp-contract=off;
// the only fused multiply-adds are the MFMA contractions and explicit fma().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace gpf {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));  // plain vector type: SROA-friendly (HIP's double2 is a class)

constexpr int NTHR = 256;   // 4 waves of 64 lanes per workgroup (covariance / objective kernels)
constexpr int DNTH = 512;   // 8 waves: the factorisation kernels (k_step, k_diag)
constexpr int T = 128;      // factorisation block (block column width, padding granule)
constexpr int DMAX = 32;    // max input dimensionality of the covariance builders
constexpr int KGRID_MAX = 4096;

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  // v_mfma_f64_16x16x4_f64: A 16x4 (lane l: row l&15, k l>>4), B 4x16 (k l>>4, col l&15),
  // C/D 16x16: col = lane&15, row = (lane>>4) + 4*reg.
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Per-tile-size geometry. A TM x TM output tile is owned by NW waves arranged
// WR x WC; each wave holds a (TM/WR) x (TM/WC) sub-tile as MBR x MBC MFMA blocks
// of 16x16 (accumulators: 4 doubles per lane per block).
template <int TM> struct TileCfg;
template <> struct TileCfg<128> {  // the factorisation / prediction GEMMs: 8 waves, 128x16 per wave
  static constexpr int KC = 16, NW = 8, WR = 1, WC = 8;
};

template <int TM> struct Geo {
  static constexpr int KC = TileCfg<TM>::KC;
  static constexpr int NW = TileCfg<TM>::NW;
  static constexpr int WR = TileCfg<TM>::WR;
  static constexpr int WC = TileCfg<TM>::WC;
  static constexpr int NTH = 64 * NW;
  static constexpr int MBR = TM / WR / 16;
  static constexpr int MBC = TM / WC / 16;
  static_assert(WR * WC == NW, "wave grid");
};

// Wave -> sub-tile map. The 8 waves of a workgroup sit two to a SIMD: waves w and w + 4 share
// one (the dispatcher deals them cyclically over the CU's 4 SIMDs). Under a triangular
// operand or a lower-only output (Tri) the live MFMAs of a sub-tile depend on where it sits,
// so the map pairs a light sub-tile with a heavy one on every SIMD:
//   128-tiles (WR = 1, WC = 8): wave w owns all 128 rows of the 16-column slab w (w < 4) or
//     11 - w (w >= 4), so SIMD s holds slabs s and 7 - s (a lower-only SYRK: 9 live 16x16
//     blocks per SIMD for every s);
//   64-tiles (WR = 2, WC = 4): the column slabs of the second row half are mirrored.
// Any map is a permutation of the same per-element work: results are bitwise unchanged.
template <int TM> struct Quad {
  int lane, rb, cb;
  __device__ Quad() {
    const int tid = threadIdx.x;
    lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar) tile origin
    if constexpr (Geo<TM>::WR == 1) {
      rb = 0;
      cb = (w >= 4 ? 11 - w : w) * (TM / Geo<TM>::WC);
    } else {
      const int wr = w / Geo<TM>::WC, wc = w % Geo<TM>::WC;
      rb = wr * (TM / Geo<TM>::WR);
      cb = ((wr & 1) ? (Geo<TM>::WC - 1 - wc) : wc) * (TM / Geo<TM>::WC);
    }
  }
  __device__ __forceinline__ int row(int mi, int r) const { return rb + mi * 16 + (lane >> 4) + 4 * r; }
  __device__ __forceinline__ int col(int ni) const { return cb + ni * 16 + (lane & 15); }
};

// Hide a global pointer's value from the optimiser so addresses derived from it
// are recomputed per use instead of being kept live (and spilled) across GEMMs.
// The pointer goes through the asm in the global address space, so accesses
// through the result stay global_load/store: a generic (flat) access would also
// count against lgkmcnt, and every LDS wait would then wait for HBM as well.
template <typename P>
__device__ __forceinline__ P* launder(P* p) {
  using G = __attribute__((address_space(1))) P*;
  G g = (G)p;
  asm volatile("" : "+v"(g));
  return (P*)g;
}

template <int TM> struct Acc {
  static constexpr int MBR = Geo<TM>::MBR, MBC = Geo<TM>::MBC;
  d4 v[MBR][MBC];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < MBR; ++i)
#pragma unroll
      for (int j = 0; j < MBC; ++j) v[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  }
  template <typename F>
  __device__ __forceinline__ void foreach(const Quad<TM>& q, F f) const {
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi)
#pragma unroll
      for (int ni = 0; ni < MBC; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) f(q.row(mi, r), q.col(ni), v[mi][ni][r]);
  }
  // Load / store the owned elements of a row-major global tile.
  __device__ __forceinline__ void load(const Quad<TM>& q, const double* base, size_t ld) {
    const double* p0 = launder(base + (size_t)(q.rb + (q.lane >> 4)) * ld + q.cb + (q.lane & 15));
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi)
#pragma unroll
      for (int ni = 0; ni < MBC; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[mi][ni][r] = p0[(size_t)(mi * 16 + 4 * r) * ld + ni * 16];
  }
  __device__ __forceinline__ void store(const Quad<TM>& q, double* base, size_t ld) const {
    double* p0 = launder(base + (size_t)(q.rb + (q.lane >> 4)) * ld + q.cb + (q.lane & 15));
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi)
#pragma unroll
      for (int ni = 0; ni < MBC; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) p0[(size_t)(mi * 16 + 4 * r) * ld + ni * 16] = v[mi][ni][r];
  }
  // store() with write-through (sc1) stores: the tile reaches memory without an L2
  // write-back fence, for a hand-off to another workgroup inside the launch (split-K)
  __device__ __forceinline__ void store_wt(const Quad<TM>& q, double* base, size_t ld) const {
    using G = __attribute__((address_space(1))) unsigned long long*;
    G p0 = (G)launder(base + (size_t)(q.rb + (q.lane >> 4)) * ld + q.cb + (q.lane & 15));
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi)
#pragma unroll
      for (int ni = 0; ni < MBC; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __hip_atomic_store(p0 + (size_t)(mi * 16 + 4 * r) * ld + ni * 16,
                             (unsigned long long)__double_as_longlong(v[mi][ni][r]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  // Visit each owned element together with its slot in a row-major global tile.
  // The per-lane base is formed once; the per-element offsets are wave-uniform
  // (scalar registers), so no per-element 64-bit address stays live.
  template <typename F>
  __device__ __forceinline__ void visit(const Quad<TM>& q, double* base, size_t ld, F f) const {
    double* p0 = launder(base + (size_t)(q.rb + (q.lane >> 4)) * ld + q.cb + (q.lane & 15));
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi)
#pragma unroll
      for (int ni = 0; ni < MBC; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) f(p0[(size_t)(mi * 16 + 4 * r) * ld + ni * 16], v[mi][ni][r]);
  }
};

// Known-zero structure of a GEMM's operands or unneeded output: MFMAs whose
// 16x16x4 block is entirely zero (or whose output block is never read) are
// skipped by a wave-uniform branch. Skipping adds of exact zeros leaves every
// result bit unchanged (up to the sign of a zero).
enum Tri : int {
  TRI_NONE = 0,
  TRI_B_KLEC,   // B(k,c) = 0 for k > c   (B = U^T with U lower triangular)
  TRI_B_KGEC,   // B(k,c) = 0 for k < c   (B = U with U lower triangular in its first T rows)
  TRI_A_KLER,   // A(r,k) = 0 for k > r   (A = U lower triangular)
  TRI_C_LOWER,  // only C(r,c) with c <= r is ever read (symmetric rank-k update)
  TRI_A_LAST,   // A's last 128 columns lower triangular by rows: A(r, K-128+c) = 0 for c > r
                // (A = a row tile of U = L^-1 over columns [0, 128(t+1)): k_predict_vsq)
};

// does the 16x16x4 MFMA block (rows R0.., cols C0.., depth k..k+3) contribute?
template <int TRI>
__device__ __forceinline__ bool tri_live(int R0, int C0, int k) {
  if (TRI == TRI_B_KLEC) return k <= C0 + 15;
  if (TRI == TRI_B_KGEC) return k + 3 >= C0;
  if (TRI == TRI_A_KLER) return k <= R0 + 15;
  if (TRI == TRI_C_LOWER) return C0 <= R0 + 15;
  return true;
}

// ----------------------------------------------------------------------------
// Direct-to-LDS streaming GEMM, TM = 128: acc (+/-)= A(128 x K) B(K x 128) with
//   A (r,k) at Ap[r*lda + k]                 (row panel, k contiguous)
//   B (k,c) at Bp[c*ldb + k]   (!NN: B^T given as a row panel, stored like A)
//           at Bp[k*ldb + c]   ( NN: B given as a row panel)
// Chunks of KC = 16 go global -> LDS by global_load_lds_dwordx4 (no VGPR staging, no
// ds_write; the loads of chunk t+1 stay in flight across the chunk-t MFMAs); one barrier per
// chunk. Each wave instruction fills one 1 KiB block with 16 B per lane in lane order, so the
// bank-conflict-free layout is made by choosing which global pair each lane fetches (XOR
// swizzles):
//   [r][k] panels: 8 rows x 8 k-pairs per block; pair kp of row r sits in slot kp ^ dl_sw(r),
//                  so the 16 rows of an MFMA operand read spread over the banks;
//   [k][c] panels: one k-row per block; column pair cp of row k sits in slot cp ^ 8 (k % 4),
//                  so the 4 k-rows of an operand read land 128 B apart.
// NEG negates through the MFMA's own A-negate modifier. LDS: 2 x 2 x 128 x 16 doubles = 64 KiB.
// ----------------------------------------------------------------------------
constexpr int DL_KC = 16;
constexpr int DL_BUF = 2 * 128 * DL_KC;  // one stage (A + B), doubles
constexpr int DL_STAGE = 2 * DL_BUF;     // double-buffered

__device__ __forceinline__ d4 mfma_neg_a(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);  // blgp bit 0 = negate A (f64)
}

// One wave-wide 16 B/lane global -> LDS transfer into the 1 KiB block at l (wave-uniform).
// Issued from inline asm: the compiler does not track the LDS write of the asm, so it no longer
// places an s_waitcnt vmcnt(0) in front of the next LDS read (which it must do for the builtin,
// since it cannot tell which LDS bytes the transfer writes). That wait drained the next chunk's
// prefetch before the current chunk's MFMAs could start. Every pipeline that uses dl_load waits
// for its own transfers itself (s_waitcnt vmcnt before the barrier that publishes a chunk).
__device__ __forceinline__ void dl_load(const double* g, double* l) {
  const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)l;
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m) : "memory");
}
// The same transfer in the saddr form: a wave-uniform 64-bit base in SGPRs plus a 32-bit per-lane
// byte offset, so the streamed GEMMs keep one VGPR per transfer stream instead of forming a 64-bit
// address per lane and transfer.
template <bool NT = false>
__device__ __forceinline__ void dl_load_s(const void* base, uint32_t off, double* l) {
  const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)l;
  if constexpr (NT)  // non-temporal: a panel streamed once per launch does not evict the shared ones from L2
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" ::"v"(off), "s"(base), "{m0}"(m) : "memory");
  else
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(base), "{m0}"(m) : "memory");
}
// B panels streamed once per launch (the k_step tiles' row / column panels) load non-temporal, so
// they stop evicting the launch's shared A panels (row panel J) from the XCD's L2: r6, same box,
// config C 1360 -> 1387 evals/s, the clock 2136 -> 2177 MHz, FETCH 2.25 -> 2.01 GB per group launch
// (profiles/r6/ab_b_nt.txt). -DGPF_B_NT=0 builds the default policy everywhere (A/B).
#ifndef GPF_SUM_SHFL  // 1: the lane-group sums by ds_bpermute (__shfl_xor), as up to round 6
#define GPF_SUM_SHFL 0
#endif
#ifndef GPF_B_NT
#define GPF_B_NT 1
#endif

// Slot swizzle of the [r][k] panels: k-pair kp of row r sits in slot kp ^ dl_sw(r). An MFMA
// operand read takes 16 consecutive rows at one k per half-wave; rows r and r+8 share a bank
// with sw = r & 7, while sw = (r >> 1) & 7 gives the 16 rows 16 distinct bank pairs (even and
// odd rows sit 16 banks apart). Row offsets of operand blocks are multiples of 16, so the
// swizzle of a read depends on the lane only and block displacements stay immediates.
__device__ __forceinline__ int dl_sw(int r) { return (r >> 1) & 7; }

// A wave-uniform pointer forced into SGPRs (v_readfirstlane of each half): the saddr transfers
// need their base there, and the divergence analysis cannot always prove a base uniform (e.g.
// behind a branch on a value read from LDS), in which case the "s" operand would get a VGPR pair.
template <typename P>
__device__ __forceinline__ P* uniform_ptr(P* p) {
  const unsigned long long v = (unsigned long long)(uintptr_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (P*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
}

// Per-lane LDS byte offsets of an MFMA A-operand read from a [r][k] panel in the dl_sw layout
// (rows r0 + (lane & 15), r0 a multiple of 16; depth 4 s + (lane >> 4) of a 16-deep chunk), for
// the k-steps s = 0..3 of a chunk. Row-block and chunk displacements are added as immediates.
__device__ __forceinline__ void dl_row_offsets(int lane, uint32_t (&o)[4]) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int s = 0; s < 4; ++s) o[s] = 8u * (uint32_t)(lr * DL_KC + 2 * ((2 * s + (lk >> 1)) ^ dl_sw(lr)) + (lk & 1));
}

// Dense chunks [t0, t1) with no VALU address work inside the loop: VALU ops do not overlap the
// FP64 MFMAs of their SIMD, so each one costs issue time. The per-lane LDS byte offsets are formed
// once per call; the buffer parity is unrolled, so buffer, k-step and row-block displacements are
// ds_read immediates; the global sources are a scalar chunk base plus a fixed 32-bit per-lane
// byte offset (the saddr form of global_load_lds). Wave layout of the 128-tiles: all 128 rows
// (8 row blocks) x one 16-column slab, so a k-step is 8 A reads, 1 B read and 8 MFMAs.
// NS: LDS stages (2: double-buffered, the default; 3-4 for one-workgroup-per-CU launches, where
// the next chunk's transfer has less time behind one chunk of MFMAs than two workgroups give it)
template <bool NN, bool NEG, int NS = 2, bool BNT = true>
struct DenseRun {
  static_assert(NS >= 2 && NS <= 4, "DenseRun stages");
  static constexpr int MBR = Geo<128>::MBR;  // 8
  static_assert(Geo<128>::MBC == 1 && Geo<128>::WR == 1, "128-tile wave layout: all rows x one column slab");
  uint32_t la[4], lb[4];  // LDS read offsets (bytes) per k-step: A rows, B^T rows (!NN) / B (NN, [0] only)
  uint32_t ga[2], gb[2];  // global byte offsets of the two 1 KiB blocks per operand this wave fills
  int blk0;               // first block index of this wave

  __device__ __forceinline__ DenseRun(const Quad<128>& qd, int lda, int ldb, int wave) {
    const int lane = qd.lane, lr = lane & 15, lk = lane >> 4;
    dl_row_offsets(lane, la);
    if (!NN) {
#pragma unroll
      for (int s = 0; s < 4; ++s) lb[s] = la[s] + 8u * (uint32_t)(128 * DL_KC + qd.cb * DL_KC);  // dl_sw(cb + lr) = dl_sw(lr)
    } else {
      const int col = qd.cb + lr;
      lb[0] = 8u * (uint32_t)(128 * DL_KC + lk * 128 + 2 * ((col >> 1) ^ (8 * (lk & 3))) + (col & 1));
      lb[1] = lb[2] = lb[3] = lb[0];
    }
    blk0 = 2 * wave;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int blk = blk0 + u, row = 8 * blk + (lane >> 3), kp = (lane & 7) ^ dl_sw(row);
      ga[u] = 8u * (uint32_t)(row * lda + 2 * kp);
      gb[u] = NN ? 8u * (uint32_t)(blk * ldb + 2 * (lane ^ (8 * (blk & 3)))) : 8u * (uint32_t)(row * ldb + 2 * kp);
    }
  }

  template <int BUF>
  __device__ __forceinline__ void issue(const double* Ap, const double* Bp, int ldb, int c, double* smem) const {
    // (uniform_ptr: a no-op where the chunk base is already scalar, as in every dense loop)
    const char* Ac = uniform_ptr((const char*)(Ap + c * DL_KC));
    const char* Bc = uniform_ptr(NN ? (const char*)(Bp + (size_t)c * DL_KC * ldb) : (const char*)(Bp + c * DL_KC));
    double* sbuf = smem + BUF * DL_BUF;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int blk = blk0 + u;
      dl_load_s(Ac, ga[u], sbuf + blk * 8 * DL_KC);
      dl_load_s<BNT && GPF_B_NT != 0>(Bc, gb[u], sbuf + 128 * DL_KC + (NN ? blk * 128 : blk * 8 * DL_KC));
    }
  }

  // operand reads of k-step s for the row blocks mi >= M0
  template <int M0>
  __device__ __forceinline__ void reads(const char* sb, int s, double (&a)[MBR], double& b) const {
#pragma unroll
    for (int mi = M0; mi < MBR; ++mi) a[mi] = *(const double*)(sb + la[s] + mi * 16 * DL_KC * 8);
    b = NN ? *(const double*)(sb + lb[0] + s * 512 * 8) : *(const double*)(sb + lb[s]);
  }

  // the MFMAs of one chunk for the row blocks mi >= M0 (M0 = MBR: none); one operand register set
  // (the 8 x 1 wave layout needs 9 operands per k-step, and a second set, read a k-step ahead,
  // would push the accumulator-resident finishes over the 128-register budget of 4 waves per SIMD)
  template <int BUF, int M0>
  __device__ __forceinline__ void mma(Acc<128>& acc, const double* smem) const {
    if constexpr (M0 >= MBR) return;
    const char* sb = (const char*)smem + BUF * DL_BUF * 8;
    double a[MBR], b;
    reads<M0>(sb, 0, a, b);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int mi = M0; mi < MBR; ++mi) acc.v[mi][0] = NEG ? mfma_neg_a(a[mi], b, acc.v[mi][0]) : mfma(a[mi], b, acc.v[mi][0]);
      if (s < 3) reads<M0>(sb, s + 1, a, b);
    }
  }

  template <int BUF, int M0>
  __device__ __forceinline__ void chunk(Acc<128>& acc, const double* Ap, const double* Bp, int ldb, int t, int nch,
                                        double* smem) const {
    // chunk t's transfers done; chunks t+1 .. t+NS-2 (4 transfers each per wave) may be in flight
    if constexpr (NS == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (t + NS - 2 < nch) {
        if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (t + NS - 1 < nch) issue<(BUF + NS - 1) % NS>(Ap, Bp, ldb, t + NS - 1, smem);
    mma<BUF, M0>(acc, smem);
  }
  template <int M0>
  __device__ __forceinline__ void chunk_rt(int b, Acc<128>& acc, const double* Ap, const double* Bp, int ldb, int t,
                                           int nch, double* smem) const {
    switch (b) {
      case 0: chunk<0, M0>(acc, Ap, Bp, ldb, t, nch, smem); break;
      case 1: chunk<1 % NS, M0>(acc, Ap, Bp, ldb, t, nch, smem); break;
      case 2: chunk<2 % NS, M0>(acc, Ap, Bp, ldb, t, nch, smem); break;
      default: chunk<3 % NS, M0>(acc, Ap, Bp, ldb, t, nch, smem); break;
    }
  }

  // chunks [t0, t1) with one MFMA pattern (row blocks mi >= M0; M0 = MBR keeps only the
  // transfers and barriers)
  template <int M0>
  __device__ __forceinline__ void run(Acc<128>& acc, const double* Ap, const double* Bp, int ldb, int t0, int t1,
                                      int nch, double* smem) const {
    int t = t0;
    if constexpr (NS == 2) {
      if (t < t1 && (t & 1)) chunk<1, M0>(acc, Ap, Bp, ldb, t++, nch, smem);
#pragma unroll 1
      for (; t + 1 < t1; t += 2) {
        chunk<0, M0>(acc, Ap, Bp, ldb, t, nch, smem);
        chunk<1, M0>(acc, Ap, Bp, ldb, t + 1, nch, smem);
      }
      if (t < t1) chunk<0, M0>(acc, Ap, Bp, ldb, t, nch, smem);
    } else {
#pragma unroll 1
      for (; t < t1 && t % NS != 0; ++t) chunk_rt<M0>(t % NS, acc, Ap, Bp, ldb, t, nch, smem);
#pragma unroll 1
      for (; t + NS - 1 < t1; t += NS) {
        chunk<0, M0>(acc, Ap, Bp, ldb, t, nch, smem);
        chunk<1, M0>(acc, Ap, Bp, ldb, t + 1, nch, smem);
        chunk<2 % NS, M0>(acc, Ap, Bp, ldb, t + 2, nch, smem);
        if constexpr (NS == 4) chunk<3, M0>(acc, Ap, Bp, ldb, t + 3, nch, smem);
      }
#pragma unroll 1
      for (; t < t1; ++t) chunk_rt<M0>(t % NS, acc, Ap, Bp, ldb, t, nch, smem);
    }
  }
};

// Known-zero skipping (Tri) at chunk granularity: every Tri boundary sits on a multiple of 16
// in k, rows and columns, so whether an MFMA block contributes (tri_live) is the same for the
// 4 k-steps of a 16-deep chunk, and per wave the chunks fall into a few contiguous runs with one
// pattern each. Each run is its own straight-line loop (one pattern per loop keeps the register
// allocation of the dense loop); exactly the MFMAs tri_live admits are issued, so results are
// bitwise those of per-block skipping. Every wave still passes one barrier per chunk.
// BNT: the B panel loads non-temporal (a panel read once per launch; GPF_B_NT)
template <bool NN, bool NEG = false, int TRI = TRI_NONE, int NS = 2, bool BNT = true>
__device__ __forceinline__ void gemm_stream_dl(Acc<128>& acc, const double* __restrict__ Ap, int lda, const double* __restrict__ Bp,
                               int ldb, int K, double* smem, const Quad<128>& qd) {
  const int nch = K / DL_KC;
  if (nch <= 0) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double* Ar = uniform_ptr(Ap);  // scalar bases
  const double* Br = uniform_ptr(Bp);
  const DenseRun<NN, NEG, NS, BNT> dr(qd, lda, ldb, wave);
  dr.template issue<0>(Ar, Br, ldb, 0, smem);
  if constexpr (NS >= 3) {  // the first NS-1 chunks in flight
    if (nch > 1) dr.template issue<1>(Ar, Br, ldb, 1, smem);
    if constexpr (NS >= 4)
      if (nch > 2) dr.template issue<2>(Ar, Br, ldb, 2, smem);
  }
  // Drain every outstanding vector-memory op here (the chunk-0 transfers, which the first chunk
  // waits for anyway, and e.g. an accumulator seed loaded just before) through the builtin, so
  // that the compiler's wait bookkeeping sees them done: otherwise it keeps an s_waitcnt for the
  // seed inside the K loop, where it also drains the asm-issued prefetch of the next chunk.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  // every run of this GEMM uses the one set of per-lane offsets formed above: no VALU address
  // work in any of the loops
#define GPF_RUN(m0, a, b) dr.template run<m0>(acc, Ar, Br, ldb, (a), (b), nch, smem)
  const int slab = qd.cb / 16;  // wave-uniform
  if constexpr (TRI == TRI_NONE) {
    GPF_RUN(0, 0, nch);
  } else if constexpr (TRI == TRI_B_KGEC) {  // the slab's columns c >= 16 slab: chunks t < slab add zeros
    const int t1 = min(nch, slab);
    GPF_RUN(8, 0, t1);
    GPF_RUN(0, t1, nch);
  } else if constexpr (TRI == TRI_A_LAST) {  // chunk c of the last 128 columns adds zeros to row blocks mi < c
    // (at half-block granularity: the chunks c >= 4 run for mi >= 4 only; one run per chunk and M0
    // spilled 12 VGPRs of the accumulators)
    const int t0 = nch - 8;  // (K >= 128: at least one full block)
    GPF_RUN(0, 0, t0 + 4);
    GPF_RUN(4, t0 + 4, nch);
  } else {  // TRI_C_LOWER: only the row blocks mi >= slab of the output are ever read
    static_assert(TRI == TRI_C_LOWER, "known-zero pattern");
    switch (slab) {
      case 0: GPF_RUN(0, 0, nch); break;
      case 1: GPF_RUN(1, 0, nch); break;
      case 2: GPF_RUN(2, 0, nch); break;
      case 3: GPF_RUN(3, 0, nch); break;
      case 4: GPF_RUN(4, 0, nch); break;
      case 5: GPF_RUN(5, 0, nch); break;
      case 6: GPF_RUN(6, 0, nch); break;
      default: GPF_RUN(7, 0, nch); break;
    }
  }
#undef GPF_RUN
  __syncthreads();
}

// gemm_stream_dl over [0, K) that stops after the first K1 (a multiple of 16, 0 <= K1 < K) for
// wait(): the chunks [0, K1/16) run (the last of them prefetches nothing), then wait() — a
// workgroup-uniform hand-off that returns true to abandon the GEMM (the result is then not used) —
// then chunk K1/16 is issued and the rest runs. One DenseRun and one set of per-lane offsets for both
// parts (two gemm_stream_dl calls around a wait kept both sets and the accumulators live across it
// and spilled); the same chunks and MFMAs in the same order: bitwise the one-piece GEMM.
// TRI: TRI_NONE, or TRI_B_KGEC with K1 at or past the triangular first 128 rows.
template <bool NN, bool NEG, int TRI, typename W>
__device__ __forceinline__ bool gemm_stream_dl_wait(Acc<128>& acc, const double* __restrict__ Ap, int lda,
                                                    const double* __restrict__ Bp, int ldb, int K, int K1, double* smem,
                                                    const Quad<128>& qd, W wait) {
  static_assert(TRI == TRI_NONE || TRI == TRI_B_KGEC, "gemm_stream_dl_wait: known-zero pattern");
  const int nch = K / DL_KC, n1 = K1 / DL_KC;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double* Ar = uniform_ptr(Ap);
  const double* Br = uniform_ptr(Bp);
  const DenseRun<NN, NEG> dr(qd, lda, ldb, wave);
  if (n1 > 0) {
    dr.template issue<0>(Ar, Br, ldb, 0, smem);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // (as in gemm_stream_dl)
    if constexpr (TRI == TRI_B_KGEC) {
      const int t1 = min(n1, qd.cb / 16);
      dr.template run<8>(acc, Ar, Br, ldb, 0, t1, n1, smem);
      dr.template run<0>(acc, Ar, Br, ldb, t1, n1, n1, smem);
    } else {
      dr.template run<0>(acc, Ar, Br, ldb, 0, n1, n1, smem);
    }
    __syncthreads();  // every wave's reads of the last buffer are done
  }
  if (wait()) return false;
  if (n1 & 1)
    dr.template issue<1>(Ar, Br, ldb, n1, smem);
  else
    dr.template issue<0>(Ar, Br, ldb, n1, smem);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  dr.template run<0>(acc, Ar, Br, ldb, n1, nch, nch, smem);
  __syncthreads();
  return true;
}

// Symmetric rank-K update of a 128x128 tile: C -= A A^T for its lower triangle only, A (128 x K)
// a [r][k] row panel streamed through the direct-to-LDS pipeline. The wave with column slab s
// owns the row blocks mi >= s of its slab (the others lie above the diagonal and are never read):
// it loads, updates and stores just those, so per pattern only its live accumulators are live.
// WT: write-through stores (the result is handed to another workgroup of the launch).
template <bool WT, int M0>
__device__ __forceinline__ void syrk_rows(double* __restrict__ C, size_t ldc, const double* __restrict__ A, int lda,
                                          int K, double* smem, const Quad<128>& qd) {
  Acc<128> acc;
  double* p0 = launder(C + (size_t)(qd.lane >> 4) * ldc + qd.cb + (qd.lane & 15));
#pragma unroll
  for (int mi = M0; mi < 8; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc.v[mi][0][r] = p0[(size_t)(mi * 16 + 4 * r) * ldc];
  const int nch = K / DL_KC;
  if (nch > 0) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const DenseRun<false, true> dr(qd, lda, lda, wave);
    A = uniform_ptr(A);
    dr.template issue<0>(A, A, lda, 0, smem);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the seed loads retired outside the loop (gemm_stream_dl)
    dr.template run<M0>(acc, A, A, lda, 0, nch, nch, smem);
    __syncthreads();
  }
  // the stores go through a freshly laundered base: with the seed loads' 64-bit addresses reused
  // here, the compiler kept up to 32 of them live across the GEMM and spilled them
  double* p1 = launder(C + (size_t)(qd.lane >> 4) * ldc + qd.cb + (qd.lane & 15));
#pragma unroll
  for (int mi = M0; mi < 8; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double* q = p1 + (size_t)(mi * 16 + 4 * r) * ldc;
      if (WT)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(q),
                           (unsigned long long)__double_as_longlong(acc.v[mi][0][r]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      else
        *q = acc.v[mi][0][r];
    }
}

template <bool WT>
__device__ __forceinline__ void syrk_tile(double* __restrict__ C, size_t ldc, const double* __restrict__ A, int lda,
                                          int K, double* smem, const Quad<128>& qd) {
  switch (qd.cb / 16) {  // wave-uniform
    case 0: syrk_rows<WT, 0>(C, ldc, A, lda, K, smem, qd); break;
    case 1: syrk_rows<WT, 1>(C, ldc, A, lda, K, smem, qd); break;
    case 2: syrk_rows<WT, 2>(C, ldc, A, lda, K, smem, qd); break;
    case 3: syrk_rows<WT, 3>(C, ldc, A, lda, K, smem, qd); break;
    case 4: syrk_rows<WT, 4>(C, ldc, A, lda, K, smem, qd); break;
    case 5: syrk_rows<WT, 5>(C, ldc, A, lda, K, smem, qd); break;
    case 6: syrk_rows<WT, 6>(C, ldc, A, lda, K, smem, qd); break;
    default: syrk_rows<WT, 7>(C, ldc, A, lda, K, smem, qd); break;
  }
}

// ----------------------------------------------------------------------------
// Triangular multiplies with the second operand in the accumulators (the L- and U-tile
// finishes of k_step). A lower-triangular 128x128 U (the diagonal block U_JJ = L_JJ^-1) is
// staged once in LDS as 8 column chunks of 16: chunk m holds rows [16 m, 128), row stride 17
// doubles (the pad spreads an A-operand read — 16 rows x 4 consecutive k per half-wave — over
// the banks: one 2-way pair). With the stride the read offsets of the 4 k-steps of a block are
// immediates off one per-lane base. 36 blocks of 16 x 17 = 9792 doubles (76.5 KiB).
// ----------------------------------------------------------------------------
constexpr int TRI_LD = 17;
constexpr int TRI_LDS = 36 * 16 * TRI_LD;  // doubles
__host__ __device__ constexpr int tri_chunk(int m) { return 16 * TRI_LD * (8 * m - m * (m - 1) / 2); }  // chunk m's first double

// U (row-major, leading dimension ld, lower triangle read) -> LDS: 576 chunk rows of 16 doubles,
// 8 pairs each, 9 pairs per thread through registers (the odd stride rules out direct-to-LDS
// transfers). Ends with a barrier.
__device__ __forceinline__ int tri_row_chunk(int ri, int& rr) {  // chunk row ri (0..575) -> chunk m, row rr in it
  int m = 0, base = 0;
#pragma unroll
  for (int mm = 0; mm < 7; ++mm)
    if (ri >= base + 16 * (8 - m)) {
      base += 16 * (8 - m);
      ++m;
    }
  rr = ri - base;
  return m;
}
struct NoHook {
  __device__ void operator()() const {}
};
#ifndef GPF_TRI_STAGE_SCALAR  // 0: round 5's per-lane chunk-row decode (tri_row_chunk per pair)
#define GPF_TRI_STAGE_SCALAR 1
#endif
// Block b (0..35, chunk-major: chunk m holds blocks rb = m .. 7) -> chunk m, block row rb
__host__ __device__ __forceinline__ void tri_block(int b, int& m, int& rb) {
  m = 0;
  int base = 0;
#pragma unroll
  for (int mm = 0; mm < 7; ++mm)
    if (b >= base + (8 - m)) {
      base += 8 - m;
      ++m;
    }
  rb = m + (b - base);
}
// (Hook: trace builds only — called once the wave's loads have arrived)
// r6 (GPF_TRI_STAGE_SCALAR): each thread keeps one (row, pair) slot of a 16 x 16 block — lane
// offsets formed once — and walks the blocks b = group + 4u, group = tid / 128 wave-uniform, so the
// block decode and its offsets are scalar work. The per-pair chunk-row decode of the round-5 form
// was ~25 VALU instructions per pair, and VALU issue crawls on a SIMD whose matrix pipe the
// co-resident workgroup's GEMM keeps busy: the staging's writes and barrier took ~12 us of its
// ~20 us per finish (profiles/r6/phase_C_finish_split*.txt). Same LDS image.
template <typename Hook = NoHook>
__device__ __forceinline__ void tri_to_lds(const double* __restrict__ U, size_t ld, double* s, Hook hook = Hook()) {
#if GPF_TRI_STAGE_SCALAR
  {
    const int tid = threadIdx.x;
    const int grp = __builtin_amdgcn_readfirstlane(tid >> 7);  // 2 waves per group: uniform
    const int r = (tid >> 3) & 15, kp = tid & 7;
    const double* ul = U + (size_t)r * ld + 2 * kp;
    d2 v[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      int m, rb;
      tri_block(grp + 4 * u, m, rb);
      v[u] = *reinterpret_cast<const d2*>(ul + (size_t)(16 * rb) * ld + 16 * m);
    }
    if constexpr (!__is_same(Hook, NoHook)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      hook();
    }
    double* sl = s + r * TRI_LD + 2 * kp;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      int m, rb;
      tri_block(grp + 4 * u, m, rb);
      const int off = tri_chunk(m) + 16 * (rb - m) * TRI_LD;  // block (rb, m) in chunk m
      sl[off] = v[u].x;
      sl[off + 1] = v[u].y;
    }
    __syncthreads();
    return;
  }
#endif
  int tid = threadIdx.x;
  d2 v[9];
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    const int i = tid + DNTH * u, ri = i >> 3, kp = i & 7;  // chunk row ri (0..575), pair kp
    int rr;
    const int m = tri_row_chunk(ri, rr);  // row 16 m + rr of U
    v[u] = *reinterpret_cast<const d2*>(U + (size_t)(16 * m + rr) * ld + 16 * m + 2 * kp);
  }
  if constexpr (!__is_same(Hook, NoHook)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    hook();
  }
  asm volatile("" : "+v"(tid));  // (the destinations are recomputed: not 9 more registers held across the loads)
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    const int i = tid + DNTH * u, ri = i >> 3, kp = i & 7;
    int rr;
    const int m = tri_row_chunk(ri, rr);
    const int dst = tri_chunk(m) + rr * TRI_LD + 2 * kp;
    s[dst] = v[u].x;
    s[dst + 1] = v[u].y;
  }
  __syncthreads();
}

// out[j] (+)= sum_{k <= i} U(i, k) X(k, n) for the row blocks ib = 2 P + j (i in [16 ib, 16 ib + 16))
// and the wave's 16 columns n, NEG: -= (the MFMA's A-negate). X in the accumulator layout: the
// register e of block mi of a lane (g = lane >> 4, c = lane & 15) holds X(16 mi + 4 e + g, cb + c),
// which is exactly the B operand of k-step 16 mi + 4 e. Per output block the k-steps run in
// ascending order (the two blocks' chains interleaved). Software-pipelined by one k-step: the A
// operands of step q+1 are read before the MFMAs of step q; scheduling barriers keep the compiler
// from hoisting more reads (their registers would spill X). Two output blocks per call keep the
// finish within the 128-register budget of 4 waves per SIMD.
template <int P, bool NEG>
__device__ __forceinline__ void trmm_acc(d4 (&out)[2], const Acc<128>& X, const double* sU) {
  constexpr int NQ = 4 * (2 * P + 2);  // k-steps (mi, e)
  const int lane = threadIdx.x & 63;
  // per-lane byte bases: row (lane & 15), k (lane >> 4); offsets past 32 KiB go through the
  // second base (ds_read offsets are 16-bit), which is hidden from the optimiser so that it
  // stays one register
  const uint32_t b0 = 8u * (uint32_t)((lane & 15) * TRI_LD + (lane >> 4));
  uint32_t b1 = b0 + 32768u;
  asm volatile("" : "+v"(b1));
  const char* u = (const char*)sU;
  out[0] = d4{0.0, 0.0, 0.0, 0.0};
  out[1] = d4{0.0, 0.0, 0.0, 0.0};
  double a[2][2];
  auto reads = [&](int q, double (&r)[2]) {
    const int mi = q >> 2, e = q & 3;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (2 * P + j >= mi) {
        const int off = 8 * (tri_chunk(mi) + (2 * P + j - mi) * 16 * TRI_LD + 4 * e);
        r[j] = off < 32768 ? *(const double*)(u + b0 + off) : *(const double*)(u + b1 + (off - 32768));
      }
  };
  reads(0, a[0]);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q + 1 < NQ) reads(q + 1, a[(q + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    const int mi = q >> 2, e = q & 3;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (2 * P + j >= mi)
        out[j] = NEG ? mfma_neg_a(a[q & 1][j], X.v[mi][0][e], out[j]) : mfma(a[q & 1][j], X.v[mi][0][e], out[j]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Global store of one double; WT: write-through (agent-scope relaxed atomic store: the line is
// written to memory without an L2 write-back fence), for data another workgroup of the same
// launch reads after a flag hand-off (the early diagonal factor, k_step).
template <bool WT = false>
__device__ __forceinline__ void gst(double* p, double v) {
  if (WT)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

// Shader-clock probe of the factorisation kernels (profiling passes only; clk == nullptr
// otherwise): thread 0 of every workgroup adds its own span in shader clocks (s_memtime) and in
// the 100 MHz reference clock (s_memrealtime) to clk[0] / clk[1], so the host gets the clock the
// chip actually held while the kernel ran: clk[0] / clk[1] x 100 MHz. Times the FP64 MFMA rate
// per clock (128 flop per CU) it is the box's FP64 matrix ceiling during that kernel.
struct ClockSpan {  // the two start stamps wait in LDS (kept in registers they spilled in k_step)
  unsigned long long* s;
  __device__ __forceinline__ explicit ClockSpan(unsigned long long* lds2) : s(lds2) {}
  __device__ __forceinline__ void start(const unsigned long long* clk) const {
    if (clk && threadIdx.x == 0) {
      unsigned long long t0, r0;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
      s[0] = t0;
      s[1] = r0;
    }
  }
  __device__ __forceinline__ void stop(unsigned long long* clk) const {
    if (clk && threadIdx.x == 0) {
      unsigned long long t1, r1;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
      __hip_atomic_fetch_add(clk, t1 - s[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(clk + 1, r1 - s[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
};

// v + (v of lane l ^ 16) (ROWS = 16) or l ^ 32 (ROWS = 32) by the gfx950 permlane swaps (VALU, no
// LDS crossbar round trip as ds_bpermute): swap(v, v) returns {v with the upper rows of each pair
// replaced by the lower, v with the lower replaced by the upper}, so every lane finds its own value in
// one result and its partner's in the other; their sum is v + partner (addition commutes: bitwise the
// same as v + __shfl_xor(v, ROWS)).
template <int ROWS>
__device__ __forceinline__ double add_swapped(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  unsigned a0, a1, b0, b1;
  if constexpr (ROWS == 16) {
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  } else {
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  }
  const double x = __builtin_bit_cast(double, ((unsigned long long)b0 << 32) | a0);
  const double y = __builtin_bit_cast(double, ((unsigned long long)b1 << 32) | a1);
  return x + y;
}

// Sum over the 4 lane groups {l, l^16, l^32, l^48} of a wave; the result is
// bitwise identical in all four lanes ((g0+g1)+(g2+g3), addition commutes).
__device__ __forceinline__ double sum_lane_groups(double v) {
#if GPF_SUM_SHFL
  v = v + __shfl_xor(v, 16);
  v = v + __shfl_xor(v, 32);
  return v;
#else
  return add_swapped<32>(add_swapped<16>(v));
#endif
}

}  // namespace gpf
