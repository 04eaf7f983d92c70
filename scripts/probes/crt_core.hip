// Feasibility probe (not product code): fp64-accurate GEMM on the int8 matrix cores through the
// Chinese remainder theorem (Ozaki scheme II form), the follow-up of ozaki_core.hip.
//
//   A [M][K], B [N][K] fp64, |a| < 2^ea, |b| < 2^eb. a_int = round(a 2^(BITS-ea)) (|a_int| < 2^BITS),
//   likewise b_int; C_int = A_int B_int^T is an exact integer with |C_int| < K 2^(2 BITS). With NM
//   pairwise coprime moduli m_i <= 256 (product > 2 K 2^(2 BITS)), each pass i multiplies the int8
//   residues (a_int mod m_i, centred) on v_mfma_i32_32x32x32_i8 with ONE int32 accumulator per
//   output element (|sum| <= K 128^2 < 2^31), reduces it mod m_i and stores the residue byte;
//   an epilogue rebuilds C_int by Garner's mixed-radix algorithm in 128-bit integers and scales.
//   One accumulator set per pass (instead of one per digit weight) lets a workgroup hold a
//   256x256 tile: half the operand bytes per flop of the digit form's 128x64.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/probes/crt_core.hip -o scripts/probes/crt_core
// (-ffp-contract=off: the reconstruction's error-free sums must not be fused into FMAs)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int NM = 16;     // moduli
constexpr int BITS = 52;   // operand integer bits
__constant__ int c_mod[NM];
static const int h_mod[NM] = {256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193};
// compile-time copies for the reconstruction (modular reductions by constants become multiplies)
struct Mods {
  int m[NM];
  int inv[NM][NM];  // inv[i][j] = m_j^-1 mod m_i (j < i)
};
constexpr Mods make_mods() {
  Mods r{{256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193}, {}};
  for (int i = 0; i < NM; ++i)
    for (int j = 0; j < i; ++j)
      for (int x = 1; x < r.m[i]; ++x)
        if ((r.m[j] % r.m[i]) * x % r.m[i] == 1) {
          r.inv[i][j] = x;
          break;
        }
  return r;
}
constexpr Mods kM = make_mods();

// ---- GEMM of one modulus' residue planes: R_i = (A_i B_i^T) mod m_i as bytes ------------------
// Workgroup tile 256 x 256, 8 waves (4 x 2), wave tile 64 x 128 (2 x 4 blocks of 32x32), k-steps of
// 64 (two MFMA k-steps per barrier), double-buffered LDS [k half][row][16 B] per 32-deep sub-step.
constexpr int TM = 256, TN = 256, KS = 64;
constexpr int LDS_STAGE = (TM + TN) * KS;  // bytes
__device__ __forceinline__ int loff(int sub, int kh, int row, int rows) { return ((sub * 2 + kh) * rows + row) * 16; }

__global__ __launch_bounds__(512, 1) void k_crt_pass(const int8_t* __restrict__ Ap, const int8_t* __restrict__ Bp,
                                                    int M, int N, int K, int mi, uint8_t* __restrict__ R) {
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * LDS_STAGE];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w & 3, wn = w >> 2;
  const int mt = M / TM, ntn = N / TN;
  // XCD-aware order: the workgroups of one XCD take a contiguous range of tiles
  const int per = (mt * ntn + 7) / 8;
  int t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (per * 8 != mt * ntn) t = blockIdx.x;
  const int tm = t % mt, tn = t / mt;
  const int8_t* Ai = Ap + (size_t)mi * M * K;
  const int8_t* Bi = Bp + (size_t)mi * N * K;
  // staging: per stage (TM + TN) rows x 64 bytes = 4 16-byte chunks per row: 2048 chunks, 4 per thread
  const int8_t* g[4];
  int so[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = tid + 512 * j;             // chunk: (row, q) with q = 16-byte quarter of the 64-byte k-step
    const int row = c >> 2, q = c & 3;       // rows 0..511: A rows then B rows
    const int sub = q >> 1, kh = q & 1;
    if (row < TM) {
      g[j] = Ai + (size_t)(tm * TM + row) * K + 16 * q;
      so[j] = loff(sub, kh, row, TM);
    } else {
      g[j] = Bi + (size_t)(tn * TN + row - TM) * K + 16 * q;
      so[j] = 2 * 2 * TM * 16 + loff(sub, kh, row - TM, TN);
    }
  }
  v4i st[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) st[j] = *(const v4i*)g[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) *(v4i*)(lds + so[j]) = st[j];
  __syncthreads();
  v16i acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = v16i{};
  const int nsteps = K / KS;
  for (int s = 0; s < nsteps; ++s) {
    const int8_t* cur = lds + (s & 1) * LDS_STAGE;
    int8_t* nxt = lds + ((s + 1) & 1) * LDS_STAGE;
    const bool more = s + 1 < nsteps;
    if (more) {
#pragma unroll
      for (int j = 0; j < 4; ++j) st[j] = *(const v4i*)(g[j] + KS * (s + 1));
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      v4i fa[2], fb[4];
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[a] = *(const v4i*)(cur + loff(sub, l >> 5, 64 * wm + 32 * a + (l & 31), TM));
#pragma unroll
      for (int b = 0; b < 4; ++b)
        fb[b] = *(const v4i*)(cur + 2 * 2 * TM * 16 + loff(sub, l >> 5, 128 * wn + 32 * b + (l & 31), TN));
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < 4; ++j) *(v4i*)(nxt + so[j]) = st[j];
    }
    __syncthreads();
  }
  const int m = c_mod[mi];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int v = acc[a][b][r] % m;
        v += v < 0 ? m : 0;
        const int row = tm * TM + 64 * wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        const int col = tn * TN + 128 * wn + 32 * b + (l & 31);
        R[((size_t)mi * M + row) * N + col] = (uint8_t)v;
      }
}

// ---- Garner reconstruction: residues -> C = C_int 2^(-scale) -------------------------------
__constant__ int c_inv[NM][NM];  // c_inv[i][j] = m_j^-1 mod m_i (j < i)
__global__ void k_crt_garner(const uint8_t* __restrict__ R, size_t MN, double* __restrict__ C, int scale) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= MN) return;
  unsigned v[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const unsigned mi = (unsigned)kM.m[i];
    unsigned x = R[(size_t)i * MN + e];
    // v_i = (((x - v_0) m_0^-1 - v_1) m_1^-1 - ...) mod m_i, unsigned: x + m_i - (v_j mod m_i) >= 0
#pragma unroll
    for (int j = 0; j < i; ++j) x = ((x + mi - v[j] % mi) * (unsigned)kM.inv[i][j]) % mi;
    v[i] = x;
  }
  // C_int = v_0 + m_0 (v_1 + m_1 (v_2 + ...)), Horner from the top, 128-bit
  __int128 acc = 0, P = 1;
#pragma unroll
  for (int i = NM - 1; i >= 0; --i) acc = acc * kM.m[i] + v[i];
#pragma unroll
  for (int i = 0; i < NM; ++i) P *= kM.m[i];
  if (acc > P / 2) acc -= P;  // centred
  const bool neg = acc < 0;
  unsigned __int128 u = neg ? (unsigned __int128)(-acc) : (unsigned __int128)acc;
  const double d = ldexp((double)(uint64_t)(u >> 64), 64) + (double)(uint64_t)u;
  C[e] = ldexp(neg ? -d : d, -scale);
}

// Floating-point CRT reconstruction: X = sum_i c_i W_i mod M with W_i = M_i (M_i^-1 mod m_i);
// X / M = frac(sum_i c_i q_i), q_i = W_i / M in [0, 1) as double-double constants; the sum
// (< 2^12) in double-double keeps X / M to ~2^-94, then C = (X / M) M 2^-scale.
__constant__ double c_qhi[NM], c_qlo[NM];
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}
__global__ void k_crt_fp(const uint8_t* __restrict__ R, size_t MN, double* __restrict__ C, double Mscaled) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= MN) return;
  double sh = 0.0, sl = 0.0;
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const double c = (double)R[(size_t)i * MN + e];
    const double ph = c * c_qhi[i];
    const double pe = fma(c, c_qhi[i], -ph);  // exact product error
    double t, te;
    two_sum(sh, ph, t, te);
    sh = t;
    sl += te + pe + c * c_qlo[i];
  }
  // frac, centred: subtract the nearest integer (exact), renormalise
  const double n = rint(sh);
  double h = sh - n, l = sl;
  const double r = rint(h + l);  // the low part may carry past +-1/2
  h -= r;
  C[e] = (h + l) * Mscaled;
}

// plain fp64 GEMM on the FP64 MFMA: the accuracy comparison's fp64 arm
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
  std::frexp(m, &e);
  return e;
}

static void residues(const std::vector<double>& a, int e, size_t n, std::vector<int8_t>& planes) {
  planes.assign((size_t)NM * n, 0);
  for (size_t i = 0; i < n; ++i) {
    const long long v = std::llround(std::ldexp(a[i], BITS - e));
    for (int k = 0; k < NM; ++k) {
      long long r = v % h_mod[k];
      if (r < 0) r += h_mod[k];
      if (r > (h_mod[k] - 1) / 2) r -= h_mod[k];  // centred: [-128, 127] for 256, [-(m-1)/2, (m-1)/2] else
      planes[(size_t)k * n + i] = (int8_t)r;
    }
  }
}

static std::vector<double> factor_like(int n, double ell, double noise, std::mt19937_64& g) {
  std::uniform_real_distribution<double> u(0, 1);
  std::vector<double> t(n), A((size_t)n * n), L((size_t)n * n, 0.0);
  for (auto& v : t) v = u(g);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      A[(size_t)i * n + j] = std::exp(-0.5 * (t[i] - t[j]) * (t[i] - t[j]) / (ell * ell)) + (i == j ? noise * noise : 0.0);
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

static double g_M = 0;  // product of the moduli as a double
static void run_crt(const int8_t* dA, const int8_t* dB, int M, int N, int K, uint8_t* dR, double* dC, int scale,
                    bool fp = false) {
  const int grid = (M / TM) * (N / TN);
  for (int i = 0; i < NM; ++i) hipLaunchKernelGGL(k_crt_pass, dim3(grid), dim3(512), 0, 0, dA, dB, M, N, K, i, dR);
  const size_t MN = (size_t)M * N;
  if (fp)
    hipLaunchKernelGGL(k_crt_fp, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, 0, dR, MN, dC, std::ldexp(g_M, -scale));
  else
    hipLaunchKernelGGL(k_crt_garner, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, 0, dR, MN, dC, scale);
}

int main(int argc, char** argv) {
  {  // moduli constants
    int inv[NM][NM] = {};
    for (int i = 0; i < NM; ++i)
      for (int j = 0; j < i; ++j)
        for (int x = 1; x < h_mod[i]; ++x)
          if ((long long)(h_mod[j] % h_mod[i]) * x % h_mod[i] == 1) {
            inv[i][j] = x;
            break;
          }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_mod), h_mod, sizeof(h_mod)));
    {  // q_i = W_i / M as double-double, by binary long division in 128-bit integers
      typedef unsigned __int128 u128;
      u128 Mb = 1;
      for (int i = 0; i < NM; ++i) Mb *= (u128)h_mod[i];
      double qh[NM], ql[NM];
      for (int i = 0; i < NM; ++i) {
        const u128 Mi = Mb / (u128)h_mod[i];
        const int mi = h_mod[i];
        const int r = (int)(Mi % (u128)mi);
        int inv = 0;
        for (int x = 1; x < mi; ++x)
          if (r * x % mi == 1) { inv = x; break; }
        u128 W = Mi * (u128)inv % Mb;  // < M
        unsigned long long c1 = 0, c2 = 0;
        for (int b = 0; b < 100; ++b) {  // 100 fraction bits of W / M
          W <<= 1;  // W < M < 2^126: no overflow
          const int bit = W >= Mb;
          if (bit) W -= Mb;
          if (b < 50) c1 = (c1 << 1) | bit; else c2 = (c2 << 1) | bit;
        }
        const double d1 = std::ldexp((double)c1, -50), d2 = std::ldexp((double)c2, -100);
        qh[i] = d1 + d2;
        ql[i] = d2 - (qh[i] - d1);
      }
      CK(hipMemcpyToSymbol(HIP_SYMBOL(c_qhi), qh, sizeof(qh)));
      CK(hipMemcpyToSymbol(HIP_SYMBOL(c_qlo), ql, sizeof(ql)));
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_inv), inv, sizeof(inv)));
    double lg = 0;
    for (int i = 0; i < NM; ++i) lg += std::log2((double)h_mod[i]);
    g_M = 1.0;
    for (int i = 0; i < NM; ++i) g_M *= (double)h_mod[i];
    printf("moduli: %d, product 2^%.1f (needs > 2^%d at K = 4096, %d-bit operands)\n", NM, lg, 1 + 12 + 2 * BITS, BITS);
  }
  // ---- accuracy
  {
    const int M = 256, N = 256, K = 1024;
    std::mt19937_64 g(7);
    const std::vector<double> L1 = factor_like(K, 0.3, 0.1, g);
    const std::vector<double> L2 = factor_like(K, 0.5, 0.1, g);
    std::vector<double> A((size_t)M * K), B((size_t)N * K);
    for (int i = 0; i < M; ++i)
      for (int k = 0; k < K; ++k) A[(size_t)i * K + k] = L1[(size_t)(K - M + i) * K + k];
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < K; ++k) B[(size_t)i * K + k] = L2[(size_t)(K - N + i) * K + k];
    const int ea = exp_bound(A), eb = exp_bound(B);
    std::vector<int8_t> pA, pB;
    residues(A, ea, A.size(), pA);
    residues(B, eb, B.size(), pB);
    int8_t *dA, *dB;
    uint8_t* dR;
    double *dC, *dF, *dAd, *dBd;
    CK(hipMalloc(&dA, pA.size()));
    CK(hipMalloc(&dB, pB.size()));
    CK(hipMalloc(&dR, (size_t)NM * M * N));
    CK(hipMalloc(&dC, (size_t)M * N * 8));
    CK(hipMalloc(&dF, (size_t)M * N * 8));
    CK(hipMalloc(&dAd, A.size() * 8));
    CK(hipMalloc(&dBd, B.size() * 8));
    CK(hipMemcpy(dA, pA.data(), pA.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, pB.data(), pB.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dAd, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dBd, B.data(), B.size() * 8, hipMemcpyHostToDevice));
    run_crt(dA, dB, M, N, K, dR, dC, 2 * BITS - ea - eb);
    hipLaunchKernelGGL(k_f64, dim3(M / 16, N / 16), dim3(64), 0, 0, dAd, dBd, M, N, K, dF);
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    std::vector<double> Cc((size_t)M * N), Cf((size_t)M * N), Cp((size_t)M * N);
    CK(hipMemcpy(Cc.data(), dC, Cc.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(Cf.data(), dF, Cf.size() * 8, hipMemcpyDeviceToHost));
    run_crt(dA, dB, M, N, K, dR, dC, 2 * BITS - ea - eb, true);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(Cp.data(), dC, Cp.size() * 8, hipMemcpyDeviceToHost));
    double ep = 0;
    double ec = 0, ef = 0, cmax = 0;
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < N; ++j) {
        long double s = 0;
        for (int k = 0; k < K; ++k) s += (long double)A[(size_t)i * K + k] * B[(size_t)j * K + k];
        ec = std::max(ec, (double)std::fabs((long double)Cc[(size_t)i * N + j] - s));
        ef = std::max(ef, (double)std::fabs((long double)Cf[(size_t)i * N + j] - s));
        ep = std::max(ep, (double)std::fabs((long double)Cp[(size_t)i * N + j] - s));
        cmax = std::max(cmax, (double)std::fabs(s));
      }
    printf("accuracy (M=%d N=%d K=%d, factor-like operands, %d moduli, %d-bit operands): max|C-C_exact| crt %.3e  "
           "fp64 MFMA %.3e  (max|C| %.3e); floating-point reconstruction %.3e\n", M, N, K, NM, BITS, ec, ef, cmax, ep);
    CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(dR)); CK(hipFree(dC)); CK(hipFree(dF)); CK(hipFree(dAd)); CK(hipFree(dBd));
  }
  // ---- throughput
  {
    const int M = 8192, N = 4096, K = argc > 1 ? atoi(argv[1]) : 2048;
    int8_t *dA, *dB;
    uint8_t* dR;
    double* dC;
    CK(hipMalloc(&dA, (size_t)NM * M * K));
    CK(hipMalloc(&dB, (size_t)NM * N * K));
    CK(hipMalloc(&dR, (size_t)NM * M * N));
    CK(hipMalloc(&dC, (size_t)M * N * 8));
    CK(hipMemset(dA, 3, (size_t)NM * M * K));
    CK(hipMemset(dB, 5, (size_t)NM * N * K));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    run_crt(dA, dB, M, N, K, dR, dC, 0);
    const int reps = 5;
    const int grid = (M / TM) * (N / TN);
    const size_t MN = (size_t)M * N;
    float ms_p = 0, ms_g = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < NM; ++i) hipLaunchKernelGGL(k_crt_pass, dim3(grid), dim3(512), 0, 0, dA, dB, M, N, K, i, dR);
      CK(hipEventRecord(e1));
      hipLaunchKernelGGL(k_crt_fp, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, 0, dR, MN, dC, 1.0);
      CK(hipEventRecord(e2));
      CK(hipEventSynchronize(e2));
      float a, b;
      CK(hipEventElapsedTime(&a, e0, e1));
      CK(hipEventElapsedTime(&b, e1, e2));
      ms_p += a;
      ms_g += b;
    }
    ms_p /= reps;
    ms_g /= reps;
    const double fl = 2.0 * M * N * K;
    printf("throughput (M=%d N=%d K=%d, %d workgroups of 256x256, %d passes): passes %.3f ms + reconstruction %.3f ms  "
           "fp64-equivalent %.1f TF/s (passes alone %.1f)  int8 %.0f TOP/s  residues streamed %.2f TB/s\n",
           M, N, K, grid, NM, ms_p, ms_g, fl / (ms_p + ms_g) * 1e-9, fl / ms_p * 1e-9, fl * NM / ms_p * 1e-9,
           (double)NM * K * (TM + TN) * grid / ms_p * 1e-9);
  }
  return 0;
}
