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
constexpr int H = 64;       // half block: the unblocked diagonal factor works on 64x64
constexpr int LDH = H + 1;  // [row][k] stride of an LDS-resident 64x64 tile (odd: conflict-free b64 / read2_b64)
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
#ifndef GPF_STEP_KC
#define GPF_STEP_KC 16  // K depth per LDS stage of the 128-tile GEMMs (build-time tuning knob)
#endif
template <> struct TileCfg<128> {  // the factorisation / prediction GEMMs: 8 waves, 64x32 per wave
  static constexpr int KC = GPF_STEP_KC, NW = 8, WR = 2, WC = 4;
};
template <> struct TileCfg<64> {   // LDS-resident 64x64 products inside the diagonal factor: 8 waves, 32x16 each
  static constexpr int KC = 32, NW = 8, WR = 2, WC = 4;
};

template <int TM> struct Geo {
  static constexpr int KC = TileCfg<TM>::KC;
  static constexpr int NW = TileCfg<TM>::NW;
  static constexpr int WR = TileCfg<TM>::WR;
  static constexpr int WC = TileCfg<TM>::WC;
  static constexpr int NTH = 64 * NW;
  static constexpr int MBR = TM / WR / 16;
  static constexpr int MBC = TM / WC / 16;
  // [row][k] staging stride: odd, so 16 consecutive rows hit 16 distinct bank pairs both for
  // ds_read_b64 (banks mod 64) and for the ds_read2_b64 the compiler pairs them into (mod 32)
  static constexpr int RK = KC + 1;
  static constexpr int KN = TM + 16;  // [k][col] staging stride (2*ld == 32 mod 64 dwords)
  static constexpr int SA = TM * RK;
  static constexpr int SB = (TM * RK > KC * KN) ? TM * RK : KC * KN;
  static constexpr int STAGE = 2 * (SA + SB);  // double-buffered A + B chunks (doubles)
  static constexpr int NLD = TM * KC / 2 / NTH;  // 16-byte loads per thread per operand per chunk
  static_assert(NLD * 2 * NTH == TM * KC, "staging map");
  static_assert(WR * WC == NW, "wave grid");
};

// Wave -> sub-tile map. The waves of a workgroup are dealt round-robin over the CU's 4
// SIMDs (wave w on SIMD w % 4), so with WC = 4 the two waves sharing a SIMD own the
// same column slab in the two row halves. Under a triangular operand (TRI_B_*) or a
// lower-only output (TRI_C_LOWER) the skipped MFMAs then pile onto the same SIMDs:
// in the 128-wide TRMM one SIMD issues all of its blocks while another issues an
// eighth. GPF_BAL mirrors the column slabs of the second row half (wc -> WC-1-wc), so
// each SIMD pairs a light slab with a heavy one. Any map is a permutation of the same
// per-element work: results are bitwise unchanged.
#ifndef GPF_BAL
#define GPF_BAL 1
#endif
template <int TM> struct Quad {
  int lane, rb, cb;
  __device__ Quad() {
    const int tid = threadIdx.x;
    lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar) tile origin
    const int wr = w / Geo<TM>::WC, wc = w % Geo<TM>::WC;
    rb = wr * (TM / Geo<TM>::WR);
    cb = ((GPF_BAL && (wr & 1)) ? (Geo<TM>::WC - 1 - wc) : wc) * (TM / Geo<TM>::WC);
  }
  __device__ __forceinline__ int wrow() const { return (threadIdx.x >> 6) / Geo<TM>::WC; }
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

// ----------------------------------------------------------------------------
// Streaming tile GEMM: acc(TM x TM) += A(TM x K) * B(K x TM)
//   A (r,k) at Ap[r*lda + k]                      (row panel, k contiguous)
//   B (k,c) at Bp[c*ldb + k]   (!NN: B^T given as a row panel)
//           at Bp[k*ldb + c]   ( NN: B given as a row panel)
// K is a multiple of KC. Chunks are double-buffered through LDS: the global loads
// of chunk t+1 are in flight while chunk t feeds the MFMAs; one barrier per chunk.
// NEG stages A negated, i.e. acc -= A B (sign flips are exact: acc = C - A B
// rounds exactly like a subtraction). Ends with a barrier, so the staging area
// may be reused right after.
// ----------------------------------------------------------------------------
template <int TM, bool NN>
__device__ __forceinline__ void stage_load(d2 (&ra)[Geo<TM>::NLD], d2 (&rb)[Geo<TM>::NLD],
                                           const double* __restrict__ Ap, int lda, const double* __restrict__ Bp,
                                           int ldb, int k0, int tid) {
  constexpr int KC = Geo<TM>::KC;
#pragma unroll
  for (int u = 0; u < Geo<TM>::NLD; ++u) {
    const int q = tid + Geo<TM>::NTH * u;
    const int row = q / (KC / 2), c2 = q % (KC / 2);
    ra[u] = *reinterpret_cast<const d2*>(Ap + (size_t)row * lda + k0 + 2 * c2);
    if (!NN) {
      rb[u] = *reinterpret_cast<const d2*>(Bp + (size_t)row * ldb + k0 + 2 * c2);
    } else {
      const int kr = q / (TM / 2), cc = q % (TM / 2);
      rb[u] = *reinterpret_cast<const d2*>(Bp + (size_t)(k0 + kr) * ldb + 2 * cc);
    }
  }
}

template <int TM, bool NN, bool NEG>
__device__ __forceinline__ void stage_store(double* sA, double* sB, const d2 (&ra)[Geo<TM>::NLD],
                                            const d2 (&rb)[Geo<TM>::NLD], int tid) {
  constexpr int KC = Geo<TM>::KC, RK = Geo<TM>::RK, KN = Geo<TM>::KN;
#pragma unroll
  for (int u = 0; u < Geo<TM>::NLD; ++u) {
    const int q = tid + Geo<TM>::NTH * u;
    const int row = q / (KC / 2), c2 = q % (KC / 2);
    const d2 va = NEG ? -ra[u] : ra[u];
    sA[row * RK + 2 * c2] = va.x;  // odd stride: 8-byte aligned rows, two b64 stores
    sA[row * RK + 2 * c2 + 1] = va.y;
    if (!NN) {
      sB[row * RK + 2 * c2] = rb[u].x;
      sB[row * RK + 2 * c2 + 1] = rb[u].y;
    } else {
      const int kr = q / (TM / 2), cc = q % (TM / 2);
      *reinterpret_cast<d2*>(sB + kr * KN + 2 * cc) = rb[u];
    }
  }
}

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

template <int TM, bool NN, int TRI = TRI_NONE>
__device__ __forceinline__ void stage_mma(Acc<TM>& acc, const double* sA, const double* sB, const Quad<TM>& qd,
                                          int k0 = 0) {
  constexpr int KC = Geo<TM>::KC, RK = Geo<TM>::RK, KN = Geo<TM>::KN;
  constexpr int MBR = Geo<TM>::MBR, MBC = Geo<TM>::MBC;
  const int lr = qd.lane & 15, lk = qd.lane >> 4;
#pragma unroll
  for (int ks = 0; ks < KC; ks += 4) {
    double a[MBR], b[MBC];
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi) a[mi] = sA[(qd.rb + mi * 16 + lr) * RK + ks + lk];
#pragma unroll
    for (int ni = 0; ni < MBC; ++ni) {
      if (!NN)
        b[ni] = sB[(qd.cb + ni * 16 + lr) * RK + ks + lk];
      else
        b[ni] = sB[(ks + lk) * KN + qd.cb + ni * 16 + lr];
    }
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi)
#pragma unroll
      for (int ni = 0; ni < MBC; ++ni)
        if (tri_live<TRI>(qd.rb + mi * 16, qd.cb + ni * 16, k0 + ks)) acc.v[mi][ni] = mfma(a[mi], b[ni], acc.v[mi][ni]);
  }
}

template <int TM, bool NN, bool NEG = false, int TRI = TRI_NONE>
__device__ void gemm_stream(Acc<TM>& acc, const double* __restrict__ Ap, int lda, const double* __restrict__ Bp,
                            int ldb, int K, double* smem, const Quad<TM>& qd) {
  constexpr int KC = Geo<TM>::KC, SA = Geo<TM>::SA, SB = Geo<TM>::SB, NLD = Geo<TM>::NLD;
  const int tid = threadIdx.x;
  const int nch = K / KC;
  if (nch <= 0) return;
  Ap = launder(Ap);
  Bp = launder(Bp);
  d2 ra[NLD], rb[NLD];
  stage_load<TM, NN>(ra, rb, Ap, lda, Bp, ldb, 0, tid);
  stage_store<TM, NN, NEG>(smem, smem + SA, ra, rb, tid);
  __syncthreads();
#pragma unroll 1
  for (int t = 0; t < nch; ++t) {
    const bool more = (t + 1) < nch;
    if (more) stage_load<TM, NN>(ra, rb, Ap, lda, Bp, ldb, (t + 1) * KC, tid);
    const double* cur = smem + (t & 1) * (SA + SB);
    stage_mma<TM, NN, TRI>(acc, cur, cur + SA, qd, t * KC);
    if (more) {
      double* nxt = smem + ((t + 1) & 1) * (SA + SB);
      stage_store<TM, NN, NEG>(nxt, nxt + SA, ra, rb, tid);
    }
    __syncthreads();
  }
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
#ifndef GPF_DL_ASM
#define GPF_DL_ASM 1  // build-time A/B knob
#endif
__device__ __forceinline__ void dl_load(const double* g, double* l) {
#if GPF_DL_ASM
  const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)l;
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m) : "memory");
#else
  __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
#endif
}

// Slot swizzle of the [r][k] panels: k-pair kp of row r sits in slot kp ^ dl_sw(r). An MFMA
// operand read takes 16 consecutive rows at one k per half-wave; rows r and r+8 share a bank
// with sw = r & 7, while sw = (r >> 1) & 7 gives the 16 rows 16 distinct bank pairs (even and
// odd rows sit 16 banks apart). Row offsets of operand blocks are multiples of 16, so the
// swizzle of a read depends on the lane only and block displacements stay immediates.
#ifndef GPF_DL_SW
#define GPF_DL_SW 1
#endif
__device__ __forceinline__ int dl_sw(int r) { return GPF_DL_SW ? ((r >> 1) & 7) : (r & 7); }

// Dense chunks [t0, t1) (every MFMA block live) with no VALU address work inside the loop:
// VALU ops do not overlap the FP64 MFMAs of their SIMD, so each one costs issue time. The per-lane
// LDS byte offsets are formed once per call; the buffer parity is unrolled, so buffer, k-step and
// row/column-block displacements are ds_read immediates; the global sources are a scalar chunk
// base plus a fixed 32-bit per-lane byte offset (the saddr form of global_load_lds).
template <bool NN, bool NEG>
struct DenseRun {
  uint32_t la[4], lb[4];  // LDS read offsets (bytes) per k-step: A rows, B^T rows (!NN) / B (NN, [0..1] per ni)
  uint32_t ga[2], gb[2];  // global byte offsets of the two 1 KiB blocks per operand this wave fills
  int blk0;               // first block index of this wave

  __device__ __forceinline__ DenseRun(const Quad<128>& qd, int lda, int ldb, int wave) {
    const int lane = qd.lane, lr = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kp = 2 * s + (lk >> 1);
      la[s] = 8u * (uint32_t)((qd.rb + lr) * DL_KC + 2 * (kp ^ dl_sw(lr)) + (lk & 1));
      if (!NN) lb[s] = 8u * (uint32_t)(128 * DL_KC + (qd.cb + lr) * DL_KC + 2 * (kp ^ dl_sw(lr)) + (lk & 1));
    }
    if (NN) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = qd.cb + ni * 16 + lr;
        lb[ni] = 8u * (uint32_t)(128 * DL_KC + lk * 128 + 2 * ((col >> 1) ^ (8 * (lk & 3))) + (col & 1));
      }
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
    const char* Ac = (const char*)(Ap + c * DL_KC);
    const char* Bc = NN ? (const char*)(Bp + (size_t)c * DL_KC * ldb) : (const char*)(Bp + c * DL_KC);
    double* sbuf = smem + BUF * DL_BUF;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int blk = blk0 + u;
      dl_load((const double*)(Ac + ga[u]), sbuf + blk * 8 * DL_KC);
      dl_load((const double*)(Bc + gb[u]), sbuf + 128 * DL_KC + (NN ? blk * 128 : blk * 8 * DL_KC));
    }
  }

  // operand reads of k-step s; only rows mi >= MLO and the live columns (patterns as in dl_mma_live)
  template <int M0 = 0, int M1 = 0>
  __device__ __forceinline__ void reads(const char* sb, int s, double (&a)[4], double (&b)[2]) const {
    constexpr int MLO = M0 < M1 ? M0 : M1;
#pragma unroll
    for (int mi = MLO; mi < 4; ++mi) a[mi] = *(const double*)(sb + la[s] + mi * 16 * DL_KC * 8);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      if ((ni == 0 ? M0 : M1) >= 4) continue;
      b[ni] = NN ? *(const double*)(sb + lb[ni] + s * 512 * 8) : *(const double*)(sb + lb[s] + ni * 16 * DL_KC * 8);
    }
  }

  template <int BUF, int M0 = 0, int M1 = 0>
  __device__ __forceinline__ void mma(Acc<128>& acc, const double* smem) const {
    if constexpr (M0 >= 4 && M1 >= 4) return;
    constexpr int MLO = M0 < M1 ? M0 : M1;
    const char* sb = (const char*)smem + BUF * DL_BUF * 8;
    // operands of k-step s+1 are read into the other register set before the MFMAs of step s
    double a[2][4], b[2][2];
    reads<M0, M1>(sb, 0, a[0], b[0]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s < 3) reads<M0, M1>(sb, s + 1, a[(s + 1) & 1], b[(s + 1) & 1]);
#pragma unroll
      for (int mi = MLO; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          if (mi >= (ni == 0 ? M0 : M1))
            acc.v[mi][ni] = NEG ? mfma_neg_a(a[s & 1][mi], b[s & 1][ni], acc.v[mi][ni])
                                : mfma(a[s & 1][mi], b[s & 1][ni], acc.v[mi][ni]);
    }
  }

  template <int BUF, int M0 = 0, int M1 = 0>
  __device__ __forceinline__ void chunk(Acc<128>& acc, const double* Ap, const double* Bp, int ldb, int t, int nch,
                                        double* smem) const {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < nch) issue<1 - BUF>(Ap, Bp, ldb, t + 1, smem);
    mma<BUF, M0, M1>(acc, smem);
  }

  // chunks [t0, t1) with one MFMA pattern (M0, M1 as in dl_mma_live; <4, 4> keeps only the
  // transfers and barriers)
  template <int M0 = 0, int M1 = 0>
  __device__ __forceinline__ void run(Acc<128>& acc, const double* Ap, const double* Bp, int ldb, int t0, int t1,
                                      int nch, double* smem) const {
    int t = t0;
    if (t < t1 && (t & 1)) chunk<1, M0, M1>(acc, Ap, Bp, ldb, t++, nch, smem);
#pragma unroll 1
    for (; t + 1 < t1; t += 2) {
      chunk<0, M0, M1>(acc, Ap, Bp, ldb, t, nch, smem);
      chunk<1, M0, M1>(acc, Ap, Bp, ldb, t + 1, nch, smem);
    }
    if (t < t1) chunk<0, M0, M1>(acc, Ap, Bp, ldb, t, nch, smem);
  }
};

// Known-zero skipping (Tri) at chunk granularity: every Tri boundary sits on a multiple of 16
// in k, rows and columns, so whether an MFMA block contributes (tri_live) is the same for the
// 4 k-steps of a 16-deep chunk, and per wave the chunks fall into a few contiguous runs with one
// pattern each. Each run is its own straight-line loop (one pattern per loop keeps the register
// allocation of the dense loop); exactly the MFMAs tri_live admits are issued, so results are
// bitwise those of per-block skipping. Every wave still passes one barrier per chunk.
template <bool NN, bool NEG = false, int TRI = TRI_NONE>
__device__ void gemm_stream_dl(Acc<128>& acc, const double* __restrict__ Ap, int lda, const double* __restrict__ Bp,
                               int ldb, int K, double* smem, const Quad<128>& qd) {
  const int nch = K / DL_KC;
  if (nch <= 0) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double* Ar = Ap;  // scalar bases
  const double* Br = Bp;
  const DenseRun<NN, NEG> dr(qd, lda, ldb, wave);
  dr.template issue<0>(Ar, Br, ldb, 0, smem);
  // Drain every outstanding vector-memory op here (the chunk-0 transfers, which the first chunk
  // waits for anyway, and e.g. an accumulator seed loaded just before) through the builtin, so
  // that the compiler's wait bookkeeping sees them done: otherwise it keeps an s_waitcnt for the
  // seed inside the K loop, where it also drains the asm-issued prefetch of the next chunk.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  // every run of this GEMM uses the one set of per-lane offsets formed above: no VALU address
  // work in any of the loops, and no per-pattern copies of hoisted offsets competing for VGPRs
#define GPF_RUN(m0, m1, a, b) dr.template run<m0, m1>(acc, Ar, Br, ldb, (a), (b), nch, smem)
  if constexpr (TRI == TRI_NONE) {
    GPF_RUN(0, 0, 0, nch);
  } else if constexpr (TRI == TRI_B_KLEC) {  // column ni live iff 16 t <= cb + 16 ni
    const int t1 = min(nch, qd.cb / 16 + 1), t2 = min(nch, t1 + 1);
    GPF_RUN(0, 0, 0, t1);
    GPF_RUN(4, 0, t1, t2);
    GPF_RUN(4, 4, t2, nch);
  } else if constexpr (TRI == TRI_B_KGEC) {  // column ni live iff 16 t >= cb + 16 ni
    const int t1 = min(nch, qd.cb / 16), t2 = min(nch, t1 + 1);
    GPF_RUN(4, 4, 0, t1);
    GPF_RUN(0, 4, t1, t2);
    GPF_RUN(0, 0, t2, nch);
  } else if constexpr (TRI == TRI_A_KLER) {  // row block mi live iff 16 t <= rb + 16 mi
    const int t1 = min(nch, qd.rb / 16 + 1);
    const int t2 = min(nch, t1 + 1), t3 = min(nch, t1 + 2), t4 = min(nch, t1 + 3);
    GPF_RUN(0, 0, 0, t1);
    GPF_RUN(1, 1, t1, t2);
    GPF_RUN(2, 2, t2, t3);
    GPF_RUN(3, 3, t3, t4);
    GPF_RUN(4, 4, t4, nch);
  } else {  // TRI_C_LOWER: block live iff cb + 16 ni <= rb + 16 mi, for every chunk
    static_assert(TRI == TRI_C_LOWER, "known-zero pattern");
    // coarse patterns: the one dead block of the (0,1) and (2,3) sub-tiles is computed as well
    // (upper-triangle output, never read; the live blocks see the same MFMA sequence), so the
    // SYRK needs no pattern of its own (per-pattern and per-block variants measured slower,
    // profiles/r1/gemm_loop_ab.txt)
    const int dc = qd.cb - qd.rb;  // in {-64, -32, 0, 32, 64, 96}
    if (dc <= 0) GPF_RUN(0, 0, 0, nch);
    else if (dc <= 32) GPF_RUN(2, 2, 0, nch);
    else GPF_RUN(4, 4, 0, nch);
  }
#undef GPF_RUN
  __syncthreads();
}

// 64x64x64 GEMM with both operands resident in LDS (8 waves, 32x16 each):
//   A (r,k) at sA[r*la + k];  B (k,c) at sB[c*lb + k] (!NN) or sB[k*lb + c] (NN).
// TRI: known-zero structure (as in the streamed GEMMs): each wave runs only the k-steps whose
// 16x16x4 blocks can be non-zero (wave-uniform bounds; 16-aligned blocks, so every skipped
// MFMA would add exact zeros: results are bitwise those of the dense loop).
template <bool NN, int TRI = TRI_NONE>
__device__ __forceinline__ void gemm_lds64(Acc<64>& acc, const double* sA, int la, const double* sB, int lb,
                                           const Quad<64>& qd) {
  constexpr int MBR = Geo<64>::MBR, MBC = Geo<64>::MBC;
  static_assert(MBR == 2 && MBC == 1, "wave sub-tile of the 64-tile GEMM");
  const int lr = qd.lane & 15, lk = qd.lane >> 4;
  int k0 = 0, k1 = H;
  if (TRI == TRI_B_KLEC) k1 = qd.cb + 16;           // B(k,c) = 0 for k > c
  if (TRI == TRI_B_KGEC) k0 = qd.cb;                // B(k,c) = 0 for k < c
  if (TRI == TRI_A_KLER) k1 = qd.rb + 32;           // A(r,k) = 0 for k > r (row block 0 stops at rb + 16)
  const bool live0 = TRI != TRI_C_LOWER || qd.cb < qd.rb + 16;  // lower-only output: row block 0
  const bool live1 = TRI != TRI_C_LOWER || qd.cb < qd.rb + 32;  // ... row block 1
#pragma unroll 4
  for (int ks = k0; ks < k1; ks += 4) {
    double a[MBR], b[MBC];
#pragma unroll
    for (int mi = 0; mi < MBR; ++mi) a[mi] = sA[(qd.rb + mi * 16 + lr) * la + ks + lk];
#pragma unroll
    for (int ni = 0; ni < MBC; ++ni) {
      if (!NN)
        b[ni] = sB[(qd.cb + ni * 16 + lr) * lb + ks + lk];
      else
        b[ni] = sB[(ks + lk) * lb + qd.cb + ni * 16 + lr];
    }
    const bool m0 = TRI == TRI_A_KLER ? ks < qd.rb + 16 : live0;
    if (m0) acc.v[0][0] = mfma(a[0], b[0], acc.v[0][0]);
    if (live1) acc.v[1][0] = mfma(a[1], b[0], acc.v[1][0]);
  }
}

// Coalesced 64x64 global tile -> LDS [row][col] with stride ld, 16 B per lane (DNTH threads).
__device__ __forceinline__ void tile64_to_lds(double* s, int ld, const double* __restrict__ g, size_t gld) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2048 / DNTH; ++u) {
    const int q = tid + DNTH * u;
    const int row = q >> 5, c2 = q & 31;
    const d2 v = *reinterpret_cast<const d2*>(g + (size_t)row * gld + 2 * c2);
    s[row * ld + 2 * c2] = v.x;
    s[row * ld + 2 * c2 + 1] = v.y;
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

// LDS 64x64 -> global, optionally zeroing the strict upper triangle.
template <bool WT = false>
__device__ __forceinline__ void lds_to_tile64(double* __restrict__ g, size_t gld, const double* s, int ld,
                                              bool lower_only) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2048 / DNTH; ++u) {
    const int q = tid + DNTH * u;
    const int row = q >> 5, c2 = q & 31;
    d2 v;
    v.x = (lower_only && 2 * c2 > row) ? 0.0 : s[row * ld + 2 * c2];
    v.y = (lower_only && 2 * c2 + 1 > row) ? 0.0 : s[row * ld + 2 * c2 + 1];
    double* gp = g + (size_t)row * gld + 2 * c2;
    if (WT) {
      gst<true>(gp, v.x);
      gst<true>(gp + 1, v.y);
    } else {
      *reinterpret_cast<d2*>(gp) = v;
    }
  }
}

template <bool WT = false>
__device__ __forceinline__ void zero_tile64(double* __restrict__ g, size_t gld) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2048 / DNTH; ++u) {
    const int q = tid + DNTH * u;
    const int row = q >> 5, c2 = q & 31;
    double* gp = g + (size_t)row * gld + 2 * c2;
    if (WT) {
      gst<true>(gp, 0.0);
      gst<true>(gp + 1, 0.0);
    } else {
      *reinterpret_cast<d2*>(gp) = d2{0.0, 0.0};
    }
  }
}

// One butterfly step of acc_row_dot over the live list v[0 .. 2H): lanes with bit H of their
// column index keep the upper half. Every index is a compile-time constant (pack expansion, no
// loop): a loop over j left the selects to the optimiser, which turned them into a
// lane-dependent index into v and lowered that as chains of 16 v_cndmask per element.
template <int H, int... J>
__device__ __forceinline__ void row_dot_step(double (&v)[16], bool up, std::integer_sequence<int, J...>) {
  ((v[J] = (up ? v[J + H] : v[J]) + __shfl_xor(up ? v[J] : v[J + H], H)), ...);
}

// Row sums of the 128-tile accumulator times a column vector z (LDS, 128 entries) over this
// wave's 32 columns: the two column blocks are combined in each lane, then the 16 lanes of a
// lane group (same rows, different columns) by a butterfly reduce-scatter (15 shuffles instead
// of 4 x 16). Returns, in lane (g = lane >> 4, c = lane & 15), the sum of row
// rb + 16 (c >> 2) + g + 4 (c & 3) (accumulator index mi = c >> 2, r = c & 3). Fixed order.
__device__ __forceinline__ double acc_row_dot(const Acc<128>& acc, const Quad<128>& qd, const double* z) {
  static_assert(Acc<128>::MBR == 4 && Acc<128>::MBC == 2, "layout of the 128-tile accumulator");
  const double z0 = z[qd.col(0)], z1 = z[qd.col(1)];
  double v[16];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[mi * 4 + r] = fma(acc.v[mi][1][r], z1, acc.v[mi][0][r] * z0);
  const int c = qd.lane & 15;
  row_dot_step<8>(v, (c & 8) != 0, std::make_integer_sequence<int, 8>{});
  row_dot_step<4>(v, (c & 4) != 0, std::make_integer_sequence<int, 4>{});
  row_dot_step<2>(v, (c & 2) != 0, std::make_integer_sequence<int, 2>{});
  row_dot_step<1>(v, (c & 1) != 0, std::make_integer_sequence<int, 1>{});
  return v[0];
}

// Sum over the 4 lane groups {l, l^16, l^32, l^48} of a wave; the result is
// bitwise identical in all four lanes ((g0+g1)+(g2+g3), addition commutes).
__device__ __forceinline__ double sum_lane_groups(double v) {
  v = v + __shfl_xor(v, 16);
  v = v + __shfl_xor(v, 32);
  return v;
}

}  // namespace gpf
