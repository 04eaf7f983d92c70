// Feasibility probe (not product code): fp64-accurate GEMM emulated on the int8 matrix cores
// (Ozaki-style fixed-point slicing), the "next" item of DESIGN.md §8.
//
//   C = A B^T, A [M][K], B [N][K] fp64 with entries bounded by 2^ea, 2^eb (the factor's L and
//   U = L^-1 are: |L_ij| <= sqrt(1 + e_i^2), ||U||_2 <= 1 / min e). Each matrix is cut into S
//   int8 digit planes, a = 2^(ea+1) sum_s d_s 2^(-7(s+1)), |d_s| <= 64 (round-to-nearest digits),
//   and C = 2^(ea+eb+2) sum_{s+t<S} 2^(-7(s+t+2)) (D^A_s D^B_t^T): every digit product is exact in
//   the int32 accumulators; products of equal weight (s + t = g) share one accumulator, S of them.
//
// Parts: (1) the v_mfma_i32_32x32x32_i8 operand map, checked with exact integers; (2) GEMM
// throughput (fp64-equivalent TF/s) with digit planes streamed from HBM; (3) accuracy against a
// long-double reference next to a plain fp64 GEMM of the same data.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/ozaki_core.hip -o /tmp/ozaki_core
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));    // 16 int8 operands
typedef int v16i __attribute__((ext_vector_type(16)));  // 32x32 int32 accumulator fragment

#ifndef NS
#define NS 7  // digit planes per operand
#endif

// ---- (1) operand map -------------------------------------------------------------------
// hypothesis: lane l holds A[r = l & 31][k = 16 (l >> 5) + j] and B[k = 16 (l >> 5) + j][c = l & 31]
// in byte j = 0..15; C/D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (l >> 5).
__global__ void k_map(const int8_t* A, const int8_t* B, int* C) {  // A [32][32] (r, k), B [32][32] (c, k)
  const int l = threadIdx.x;
  v4i a, b;
  int8_t* pa = (int8_t*)&a;
  int8_t* pb = (int8_t*)&b;
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[(l & 31) * 32 + 16 * (l >> 5) + j];
    pb[j] = B[(l & 31) * 32 + 16 * (l >> 5) + j];
  }
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[r];
}

// ---- (2)/(3) GEMM ----------------------------------------------------------------------
// Planes: A [NS][M][K], B [NS][N][K] int8, K contiguous. Workgroup tile 128 x 64, four waves
// (one per SIMD), wave w: rows 32w..32w+31, two 32x32 column blocks. NS (NS+1)/2 digit
// products per pair of fragments, NS int32 accumulators per output element.
__global__ __launch_bounds__(256, 1) void k_ozaki(const int8_t* __restrict__ Ap, const int8_t* __restrict__ Bp,
                                                 int M, int N, int K, double* __restrict__ C, int ea, int eb) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int mt = M / 128;
  const int tm = blockIdx.x % mt, tn = blockIdx.x / mt;
  const int kh = 16 * (l >> 5);
  const int8_t* pa = Ap + (size_t)(tm * 128 + 32 * w + (l & 31)) * K + kh;
  const int8_t* pb = Bp + (size_t)(tn * 64 + (l & 31)) * K + kh;
  const size_t sa = (size_t)M * K, sb = (size_t)N * K;
  v16i acc[NS][2];
#pragma unroll
  for (int g = 0; g < NS; ++g) acc[g][0] = acc[g][1] = v16i{};
  v4i a[NS], b[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    a[s] = *(const v4i*)(pa + s * sa);
    b[s][0] = *(const v4i*)(pb + s * sb);
    b[s][1] = *(const v4i*)(pb + s * sb + (size_t)32 * K);
  }
  for (int k0 = 0; k0 < K; k0 += 32) {
    v4i an[NS], bn[NS][2];
    const int kn = (k0 + 32 < K) ? k0 + 32 : k0;  // prefetch the next k-step (the last reloads)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      an[s] = *(const v4i*)(pa + s * sa + kn);
      bn[s][0] = *(const v4i*)(pb + s * sb + kn);
      bn[s][1] = *(const v4i*)(pb + s * sb + (size_t)32 * K + kn);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int t = 0; t < NS - s; ++t) {
        acc[s + t][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[t][0], acc[s + t][0], 0, 0, 0);
        acc[s + t][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[t][1], acc[s + t][1], 0, 0, 0);
      }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      a[s] = an[s];
      b[s][0] = bn[s][0];
      b[s][1] = bn[s][1];
    }
  }
  // C = 2^(ea+eb+2) sum_g 2^(-7(g+2)) acc[g], smallest weight first
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      double v = 0.0;
#pragma unroll
      for (int g = NS - 1; g >= 0; --g) v = v + ldexp((double)acc[g][nb][r], -7 * (g + 2));
      const int row = tm * 128 + 32 * w + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int col = tn * 64 + nb * 32 + (l & 31);
      C[(size_t)row * N + col] = ldexp(v, ea + eb + 2);
    }
}

// LDS-staged version: each 32-deep k-step the workgroup stages its NS planes of A (128 rows) and
// B (64 rows) in LDS (double-buffered, 48 KB per buffer at NS = 8; layout [plane][k half][row][16 B]
// so that a fragment read is 64 consecutive 16-byte words: no bank conflicts), the global loads
// of the next step are issued before the MFMAs of this one. swz: XCD-aware tile order (the
// workgroups of one XCD take a contiguous range of tiles, 4 tile rows x 8 tile columns at a time).
template <int R>
__device__ __forceinline__ int lds_off(int s, int kh, int row) { return ((s * 2 + kh) * R + row) * 16; }

template <int WN, bool PF2 = false>  // 32 x (32 WN) per wave; 4 (2 / WN) waves: WN = 2 one wave per SIMD, WN = 1 two
__global__ __launch_bounds__(128 * (2 / WN) * 2, 1) void k_ozaki_lds(const int8_t* __restrict__ Ap,
                                                                    const int8_t* __restrict__ Bp, int M, int N, int K,
                                                                    double* __restrict__ C, int ea, int eb, int swz) {
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  constexpr int NTH = 256 * (2 / WN);
  constexpr int BUF = NS * 2 * (128 + 64) * 16;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w & 3, wn = w >> 2;  // 32-row block, 32-column block (WN = 1)
  const int mt = M / 128, ntn = N / 64;
  int tm, tn;
  if (swz) {
    const int per = (mt * ntn) / 8;
    const int t = (blockIdx.x % 8) * per + blockIdx.x / 8;
    tm = (t / (4 * ntn)) * 4 + (t % 4);
    tn = (t / 4) % ntn;
  } else {
    tm = blockIdx.x % mt;
    tn = blockIdx.x / mt;
  }
  const size_t sa = (size_t)M * K, sb = (size_t)N * K;
  // staging map: chunk c = (plane, row, k half), k half fastest; A: NS*256 chunks, B: NS*128
  constexpr int NA = (NS * 256 + NTH - 1) / NTH, NB = (NS * 128 + NTH - 1) / NTH;
  const int8_t* ga[NA];
  int la[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int c = min(tid + NTH * j, NS * 256 - 1), sp = c / 256, row = (c % 256) / 2, kh = c & 1;
    ga[j] = Ap + sp * sa + (size_t)(tm * 128 + row) * K + 16 * kh;
    la[j] = lds_off<128>(sp, kh, row);
  }
  const int8_t* gb[NB];
  int lb[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int c = min(tid + NTH * j, NS * 128 - 1), sp = c / 128, row = (c % 128) / 2, kh = c & 1;
    gb[j] = Bp + sp * sb + (size_t)(tn * 64 + row) * K + 16 * kh;
    lb[j] = NS * 2 * 128 * 16 + lds_off<64>(sp, kh, row);
  }
  v4i ra[NA], rb[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) ra[j] = *(const v4i*)ga[j];
#pragma unroll
  for (int j = 0; j < NB; ++j) rb[j] = *(const v4i*)gb[j];
#pragma unroll
  for (int j = 0; j < NA; ++j) *(v4i*)(lds + la[j]) = ra[j];  // (clamped duplicates store the same bytes)
#pragma unroll
  for (int j = 0; j < NB; ++j) *(v4i*)(lds + lb[j]) = rb[j];
  __syncthreads();
  v16i acc[NS][WN];
#pragma unroll
  for (int g = 0; g < NS; ++g)
#pragma unroll
    for (int nb = 0; nb < WN; ++nb) acc[g][nb] = v16i{};
  const int fa = lds_off<128>(0, l >> 5, 32 * wm + (l & 31));
  const int fb = NS * 2 * 128 * 16 + lds_off<64>(0, l >> 5, 32 * wn + (l & 31));
  const int nsteps = K / 32;
  // PF2: global loads issued two k-steps ahead into a second register set (written to LDS at
  // the end of the following step), so that two steps of MFMAs cover their latency
  v4i qa[NA], qb[NB];
  if (PF2 && nsteps > 1) {
#pragma unroll
    for (int j = 0; j < NA; ++j) qa[j] = *(const v4i*)(ga[j] + 32);
#pragma unroll
    for (int j = 0; j < NB; ++j) qb[j] = *(const v4i*)(gb[j] + 32);
  }
  for (int i = 0; i < nsteps; ++i) {
    const int8_t* cur = lds + (i & 1) * BUF;
    int8_t* nxt = lds + ((i + 1) & 1) * BUF;
    const bool more = i + 1 < nsteps;
    if (PF2) {
      // ra <- step i+1 (already in qa), qa <- step i+2
#pragma unroll
      for (int j = 0; j < NA; ++j) ra[j] = qa[j];
#pragma unroll
      for (int j = 0; j < NB; ++j) rb[j] = qb[j];
      if (i + 2 < nsteps) {
#pragma unroll
        for (int j = 0; j < NA; ++j) qa[j] = *(const v4i*)(ga[j] + 32 * (i + 2));
#pragma unroll
        for (int j = 0; j < NB; ++j) qb[j] = *(const v4i*)(gb[j] + 32 * (i + 2));
      }
    } else if (more) {
#pragma unroll
      for (int j = 0; j < NA; ++j) ra[j] = *(const v4i*)(ga[j] + 32 * (i + 1));
#pragma unroll
      for (int j = 0; j < NB; ++j) rb[j] = *(const v4i*)(gb[j] + 32 * (i + 1));
    }
    v4i a[NS], b[NS][WN];
#pragma unroll
    for (int sp = 0; sp < NS; ++sp) {
      a[sp] = *(const v4i*)(cur + fa + sp * 2 * 128 * 16);
#pragma unroll
      for (int nb = 0; nb < WN; ++nb) b[sp][nb] = *(const v4i*)(cur + fb + sp * 2 * 64 * 16 + nb * 32 * 16);
    }
    // products in order of the later plane they need (max(s, t)), so the first MFMAs wait only
    // for the first planes' LDS reads (LDS returns in order: partial lgkmcnt waits)
#pragma unroll
    for (int m = 0; m < NS; ++m)
#pragma unroll
      for (int sp = 0; sp <= m; ++sp) {
        const int t = (sp == m) ? 0 : m;  // pairs (m, t <= m) and (sp < m, m)
#pragma unroll
        for (int u = 0; u <= (sp == m ? m : 0); ++u) {
          const int s1 = sp, t1 = (sp == m) ? u : t;
          if (s1 + t1 < NS)
#pragma unroll
            for (int nb = 0; nb < WN; ++nb)
              acc[s1 + t1][nb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s1], b[t1][nb], acc[s1 + t1][nb], 0, 0, 0);
        }
      }
    if (more) {
#pragma unroll
      for (int j = 0; j < NA; ++j) *(v4i*)(nxt + la[j]) = ra[j];
#pragma unroll
      for (int j = 0; j < NB; ++j) *(v4i*)(nxt + lb[j]) = rb[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int nb = 0; nb < WN; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      double v = 0.0;
#pragma unroll
      for (int g = NS - 1; g >= 0; --g) v = v + ldexp((double)acc[g][nb][r], -7 * (g + 2));
      const int row = tm * 128 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int col = tn * 64 + (WN == 2 ? nb : wn) * 32 + (l & 31);
      C[(size_t)row * N + col] = ldexp(v, ea + eb + 2);
    }
}
constexpr int OZ_LDS = 2 * NS * 2 * (128 + 64) * 16;

// MFMA ceiling of the same digit-product sequence: operands loaded once, K/32 k-steps of MFMAs
// (no operand traffic), same epilogue
__global__ __launch_bounds__(256, 1) void k_ozaki_regs(const int8_t* __restrict__ Ap, const int8_t* __restrict__ Bp,
                                                      int M, int N, int K, double* __restrict__ C) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int mt = M / 128;
  const int tm = blockIdx.x % mt, tn = blockIdx.x / mt;
  const int8_t* pa = Ap + (size_t)(tm * 128 + 32 * w + (l & 31)) * 32 + 16 * (l >> 5);
  const int8_t* pb = Bp + (size_t)(tn * 64 + (l & 31)) * 32 + 16 * (l >> 5);
  v16i acc[NS][2];
#pragma unroll
  for (int g = 0; g < NS; ++g) acc[g][0] = acc[g][1] = v16i{};
  v4i a[NS], b[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    a[s] = *(const v4i*)(pa + (size_t)s * M * 32);
    b[s][0] = *(const v4i*)(pb + (size_t)s * N * 32);
    b[s][1] = *(const v4i*)(pb + (size_t)s * N * 32 + 32 * 32);
  }
  for (int k0 = 0; k0 < K; k0 += 32) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int t = 0; t < NS - s; ++t) {
        acc[s + t][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[t][0], acc[s + t][0], 0, 0, 0);
        acc[s + t][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[t][1], acc[s + t][1], 0, 0, 0);
      }
  }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      double v = 0.0;
#pragma unroll
      for (int g = NS - 1; g >= 0; --g) v = v + ldexp((double)acc[g][nb][r], -7 * (g + 2));
      const int row = tm * 128 + 32 * w + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int col = tn * 64 + nb * 32 + (l & 31);
      C[(size_t)row * N + col] = v;
    }
}

// plain fp64 GEMM C = A B^T on the FP64 MFMA (v_mfma_f64_16x16x4), operands from global: the
// accuracy comparison's fp64 arm (same data, same sums), not a tuned kernel
__global__ void k_f64(const double* A, const double* B, int M, int N, int K, double* C) {
  const int l = threadIdx.x & 63;
  const int row0 = blockIdx.x * 16, col0 = blockIdx.y * 16;
  typedef double v4d __attribute__((ext_vector_type(4)));
  v4d acc = {};
  for (int k = 0; k < K; k += 4) {
    const double a = A[(size_t)(row0 + (l & 15)) * K + k + (l >> 4)];
    const double b = B[(size_t)(col0 + (l & 15)) * K + k + (l >> 4)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) C[(size_t)(row0 + (l >> 4) + 4 * r) * N + col0 + (l & 15)] = acc[r];
}

static int exp_bound(const std::vector<double>& a) {
  double m = 0;
  for (double v : a) m = std::max(m, std::fabs(v));
  int e;
  std::frexp(m, &e);  // m < 2^e
  return e;
}

// digits of a / 2^(e+1) (|.| <= 1/2): NS planes, round to nearest, |d| <= 64
static void slice(const std::vector<double>& a, int e, int rows, int K, std::vector<int8_t>& planes) {
  planes.assign((size_t)NS * rows * K, 0);
  for (size_t i = 0; i < (size_t)rows * K; ++i) {
    double r = std::ldexp(a[i], -(e + 1));
    for (int s = 0; s < NS; ++s) {
      r = r * 128.0;
      const double d = std::nearbyint(r);
      r -= d;
      planes[(size_t)s * rows * K + i] = (int8_t)d;
    }
  }
}

// lower-triangular factor-like data: Cholesky of an SE covariance of sorted points + noise
static std::vector<double> factor_like(int n, double ell, double noise, std::mt19937_64& g) {
  std::uniform_real_distribution<double> u(0, 1);
  std::vector<double> t(n), A((size_t)n * n), L((size_t)n * n, 0.0);
  for (auto& v : t) v = u(g);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[(size_t)i * n + j] = std::exp(-0.5 * (t[i] - t[j]) * (t[i] - t[j]) / (ell * ell)) + (i == j ? noise * noise : 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) d -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
    d = std::sqrt(d);
    L[(size_t)j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = A[(size_t)i * n + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
      L[(size_t)i * n + j] = s / d;
    }
  }
  return L;
}

int main(int argc, char** argv) {
  CK(hipFuncSetAttribute((const void*)k_ozaki_lds<2>, hipFuncAttributeMaxDynamicSharedMemorySize, OZ_LDS));
  CK(hipFuncSetAttribute((const void*)k_ozaki_lds<1>, hipFuncAttributeMaxDynamicSharedMemorySize, OZ_LDS));
  CK(hipFuncSetAttribute((const void*)k_ozaki_lds<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, OZ_LDS));
  // ---- (1) map
  {
    std::mt19937_64 g(1);
    std::uniform_int_distribution<int> u(-100, 100);
    std::vector<int8_t> A(1024), B(1024);
    for (auto& v : A) v = (int8_t)u(g);
    for (auto& v : B) v = (int8_t)u(g);
    int8_t *dA, *dB;
    int* dC;
    CK(hipMalloc(&dA, 1024));
    CK(hipMalloc(&dB, 1024));
    CK(hipMalloc(&dC, 4096));
    CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    std::vector<int> C(1024);
    CK(hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int r = 0; r < 32; ++r)
      for (int c = 0; c < 32; ++c) {
        int s = 0;
        for (int k = 0; k < 32; ++k) s += A[r * 32 + k] * B[c * 32 + k];
        bad += s != C[r * 32 + c];
      }
    printf("map: %d of 1024 entries differ from A B^T (0 = operand map confirmed)\n", bad);
    if (bad) return 2;
  }
  // ---- (3) accuracy: L-like operands, C = L1 L2^T over K
  {
    const int M = 256, N = 128, K = 1024;
    std::mt19937_64 g(7);
    const std::vector<double> L1 = factor_like(K, 0.3, 0.1, g);
    const std::vector<double> L2 = factor_like(K, 0.5, 0.1, g);
    std::vector<double> A((size_t)M * K), B((size_t)N * K);
    for (int i = 0; i < M; ++i)
      for (int k = 0; k < K; ++k) A[(size_t)i * K + k] = L1[(size_t)(K - M + i) * K + k];
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < K; ++k) B[(size_t)i * K + k] = L2[(size_t)(K - N - 64 + i) * K + k];
    const int ea = exp_bound(A), eb = exp_bound(B);
    std::vector<int8_t> pA, pB;
    slice(A, ea, M, K, pA);
    slice(B, eb, N, K, pB);
    int8_t *dA, *dB;
    double *dC, *dF, *dAd, *dBd;
    CK(hipMalloc(&dA, pA.size()));
    CK(hipMalloc(&dB, pB.size()));
    CK(hipMalloc(&dC, (size_t)M * N * 8));
    CK(hipMalloc(&dF, (size_t)M * N * 8));
    CK(hipMalloc(&dAd, A.size() * 8));
    CK(hipMalloc(&dBd, B.size() * 8));
    CK(hipMemcpy(dA, pA.data(), pA.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, pB.data(), pB.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dAd, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dBd, B.data(), B.size() * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_ozaki, dim3((M / 128) * (N / 64)), dim3(256), 0, 0, dA, dB, M, N, K, dC, ea, eb);
    hipLaunchKernelGGL(k_f64, dim3(M / 16, N / 16), dim3(64), 0, 0, dAd, dBd, M, N, K, dF);
    CK(hipDeviceSynchronize());
    std::vector<double> Co((size_t)M * N), Cf((size_t)M * N), Cl((size_t)M * N);
    CK(hipMemcpy(Co.data(), dC, Co.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemset(dC, 0, (size_t)M * N * 8));
    for (int wn = 0; wn <= 2; ++wn) {
      CK(hipMemset(dC, 0, (size_t)M * N * 8));
      if (wn == 0)
        hipLaunchKernelGGL((k_ozaki_lds<1, true>), dim3((M / 128) * (N / 64)), dim3(512), OZ_LDS, 0, dA, dB, M, N, K, dC, ea, eb, 0);
      else if (wn == 2)
        hipLaunchKernelGGL(k_ozaki_lds<2>, dim3((M / 128) * (N / 64)), dim3(256), OZ_LDS, 0, dA, dB, M, N, K, dC, ea, eb, 0);
      else
        hipLaunchKernelGGL(k_ozaki_lds<1>, dim3((M / 128) * (N / 64)), dim3(512), OZ_LDS, 0, dA, dB, M, N, K, dC, ea, eb, 0);
      CK(hipDeviceSynchronize());
      CK(hipGetLastError());
      CK(hipMemcpy(Cl.data(), dC, Cl.size() * 8, hipMemcpyDeviceToHost));
      printf("LDS-staged kernel (%d waves%s) vs register-streamed kernel: %s\n", wn ? 8 / wn : 8, wn ? "" : ", loads two steps ahead",
             memcmp(Cl.data(), Co.data(), Cl.size() * 8) == 0 ? "bitwise equal" : "DIFFERENT");
    }
    CK(hipMemcpy(Cf.data(), dF, Cf.size() * 8, hipMemcpyDeviceToHost));
    double eo = 0, ef = 0, cmax = 0, rowabs = 0;
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < N; ++j) {
        long double s = 0, sa = 0;
        for (int k = 0; k < K; ++k) {
          s += (long double)A[(size_t)i * K + k] * B[(size_t)j * K + k];
          sa += std::fabs((long double)A[(size_t)i * K + k] * B[(size_t)j * K + k]);
        }
        eo = std::max(eo, (double)std::fabs((long double)Co[(size_t)i * N + j] - s));
        ef = std::max(ef, (double)std::fabs((long double)Cf[(size_t)i * N + j] - s));
        cmax = std::max(cmax, (double)std::fabs(s));
        rowabs = std::max(rowabs, (double)sa);
      }
    printf("accuracy (M=%d N=%d K=%d, factor-like operands, NS=%d digit planes): max|C-C_exact| ozaki %.3e  fp64 MFMA %.3e"
           "  (max|C| %.3e, max sum|a b| %.3e)\n", M, N, K, NS, eo, ef, cmax, rowabs);
    CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(dC)); CK(hipFree(dF)); CK(hipFree(dAd)); CK(hipFree(dBd));
  }
  // ---- (2) throughput
  {
    const int M = 8192, N = 4096, K = argc > 1 ? atoi(argv[1]) : 2048;
    int8_t *dA, *dB;
    double* dC;
    CK(hipMalloc(&dA, (size_t)NS * M * K));
    CK(hipMalloc(&dB, (size_t)NS * N * K));
    CK(hipMalloc(&dC, (size_t)M * N * 8));
    CK(hipMemset(dA, 3, (size_t)NS * M * K));
    CK(hipMemset(dB, 5, (size_t)NS * N * K));
    const int grid = (M / 128) * (N / 64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_ozaki, dim3(grid), dim3(256), 0, 0, dA, dB, M, N, K, dC, 0, 0);
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_ozaki, dim3(grid), dim3(256), 0, 0, dA, dB, M, N, K, dC, 0, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double fl = 2.0 * M * N * K;
    const double prods = NS * (NS + 1) / 2;
    printf("throughput (M=%d N=%d K=%d, %d workgroups, %g digit products): %.3f ms  fp64-equivalent %.1f TF/s  int8 %.0f TOP/s"
           "  planes streamed %.2f TB/s\n", M, N, K, grid, prods, ms, fl / ms * 1e-9, fl * prods / ms * 1e-9,
           (double)NS * K * (128 + 64) * grid / ms * 1e-9);
    for (int v = 0; v < 5; ++v) {
      const int swz = v == 4 ? 1 : v & 1, wn = (v >> 1) ? 1 : 2;
      auto go = [&] {
        if (v == 4)
          hipLaunchKernelGGL((k_ozaki_lds<1, true>), dim3(grid), dim3(512), OZ_LDS, 0, dA, dB, M, N, K, dC, 0, 0, swz);
        else if (wn == 2)
          hipLaunchKernelGGL(k_ozaki_lds<2>, dim3(grid), dim3(256), OZ_LDS, 0, dA, dB, M, N, K, dC, 0, 0, swz);
        else
          hipLaunchKernelGGL(k_ozaki_lds<1>, dim3(grid), dim3(512), OZ_LDS, 0, dA, dB, M, N, K, dC, 0, 0, swz);
      };
      go();
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      printf("LDS-staged (%d waves, %s tile order%s): %.3f ms  fp64-equivalent %.1f TF/s  int8 %.0f TOP/s\n", 8 / wn,
             swz ? "XCD-aware" : "plain", v == 4 ? ", loads two steps ahead" : "", ms, fl / ms * 1e-9,
             fl * prods / ms * 1e-9);
    }
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_ozaki_regs, dim3(grid), dim3(256), 0, 0, dA, dB, M, N, K, dC);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("MFMA ceiling (operands in registers, same products and epilogue): %.3f ms  fp64-equivalent %.1f TF/s  int8 %.0f TOP/s\n",
           ms, fl / ms * 1e-9, fl * prods / ms * 1e-9);
  }
  return 0;
}
