// f128_probe.hip — standalone probe of the diagonal-block factor (r5: the 16-blocked factor128 of
// gpf_diag.hip; round 4's two-64x64 factor measured 115-116k cycles here, profiles/r5/f128_probe_*), on P random GP covariance blocks
// (SE kernel of 128 points in [0,1]^3 + noise), one workgroup per block. Prints the per-workgroup
// cycles (s_memtime) and the agreement of L, U, z and the partials between the two, and the
// residuals |L L^T - A| and |U L - I| of the new one. Also the dense register-only MFMA loop at
// several chain counts and waves per SIMD (the roofline ceiling).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/probes/f128_probe.hip -o f128_probe
#include <hip/hip_runtime.h>
#define GPF_DB_STAMPS 1

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../gaussian-process_amd/csrc/gpf_common.hip"
#include "../../gaussian-process_amd/csrc/gpf_factor.hip"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using namespace gpf;
constexpr int NB = 128;

__device__ __forceinline__ unsigned long long memtime() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ __launch_bounds__(DNTH) void k_new(double* L, double* U, double* y, double* s2, double* sz, int* info,
                                              unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double lds[DB_LDS];
  const int p = blockIdx.x;
  __syncthreads();
  const unsigned long long t0 = memtime();
  factor128<true>(L + (size_t)p * NB * NB, U + (size_t)p * NB * NB, NB, y + p * NB, s2 + p * NB, sz + p * NB,
                      info + p, lds);
  __syncthreads();
  const unsigned long long t1 = memtime();
  if (threadIdx.x == 0) cyc[p] = t1 - t0;
}

// the panel alone: wave 0 runs the 8 diagonal-block panels on block data in LDS (the other waves
// exit after the load); cyc[p] = s_memtime cycles of the 8 panels
__global__ __launch_bounds__(DNTH) void k_panels(double* L, double* U, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double lds[DB_LDS];
  const int p = blockIdx.x;
  const double* A = L + (size_t)p * NB * NB;
  for (int i = threadIdx.x; i < NB * NB; i += DNTH) {
    const int r = i / NB, c = i % NB;
    if (c <= r) lds[db_bid(r / 16, c / 16) * DB_BLK + db_off(r % 16, c % 16)] = A[i];
  }
  for (int i = threadIdx.x; i < NB; i += DNTH) lds[DB_Y + i] = 1.0;
  if (threadIdx.x < 32) lds[DB_UNIT + threadIdx.x] = threadIdx.x == 15 ? 1.0 : 0.0;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const unsigned long long t0 = memtime();
  bool bad = false;
#pragma unroll 1
  for (int k = 0; k < 8; ++k) bad = db_panel<true>(lds, k, L + (size_t)p * NB * NB, U + (size_t)p * NB * NB, NB) | bad;
  const unsigned long long t1 = memtime();
  if (threadIdx.x == 0) cyc[p] = t1 - t0 + (bad ? 1 : 0);
}

// wave 0 runs the 8 panels (as k_panels) while waves 1..7 run MODE: 0 nothing, 1 an FP64 MFMA
// chain loop (registers only), 2 FP64 v_fma loop, 3 LDS read loop; wave 0's cycles are reported
template <int MODE>
__global__ __launch_bounds__(DNTH) void k_contend(double* L, double* U, unsigned long long* cyc, double* sink) {
  __shared__ __attribute__((aligned(16))) double lds[DB_LDS];
  __shared__ int done;
  const int p = blockIdx.x;
  const double* A = L + (size_t)p * NB * NB;
  for (int i = threadIdx.x; i < NB * NB; i += DNTH) {
    const int r = i / NB, c = i % NB;
    if (c <= r) lds[db_bid(r / 16, c / 16) * DB_BLK + db_off(r % 16, c % 16)] = A[i];
  }
  for (int i = threadIdx.x; i < NB; i += DNTH) lds[DB_Y + i] = 1.0;
  if (threadIdx.x < 32) lds[DB_UNIT + threadIdx.x] = threadIdx.x == 15 ? 1.0 : 0.0;
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave == 0) {
    const unsigned long long t0 = memtime();
    bool bad = false;
#pragma unroll 1
    for (int k = 0; k < 8; ++k) bad = db_panel<true>(lds, k, L + (size_t)p * NB * NB, U + (size_t)p * NB * NB, NB) | bad;
    const unsigned long long t1 = memtime();
    if (threadIdx.x == 0) {
      cyc[p] = t1 - t0 + (bad ? 1 : 0);
      __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return;
  }
  if (MODE == 0) return;
  if (MODE == 4 && wave == 4) return;  // MFMA on the other SIMDs only
  if (MODE == 5 && wave != 4) return;  // MFMA on wave 0's SIMD only
  double a = threadIdx.x * 1e-3, b = 0.999;
  d4 acc[4] = {};
  double v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = a + u;
  const double* lp = lds + (threadIdx.x & 63) * 2;
  double ls = 0.0;
  for (int it = 0; it < 100000; ++it) {
    if (__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
#pragma unroll
    for (int rep = 0; rep < 8; ++rep) {
      if (MODE == 1 || MODE >= 4)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
      if (MODE == 2)
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = fma(v[u], b, 0.25);
      if (MODE == 3)
#pragma unroll
        for (int u = 0; u < 8; ++u) ls += lp[(u * 128 + rep * 16) & 4095];
    }
  }
  double t = ls;
#pragma unroll
  for (int c = 0; c < 4; ++c) t += acc[c][0] + acc[c][1];
#pragma unroll
  for (int u = 0; u < 8; ++u) t += v[u];
  sink[threadIdx.x + blockIdx.x * DNTH] = t;
}
template <int MODE>
static void contend_case(double* dL, double* dU, unsigned long long* dcyc, double* sink, int P, const char* name) {
  hipLaunchKernelGGL(k_contend<MODE>, dim3(P), dim3(DNTH), 0, 0, dL, dU, dcyc, sink);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> c(P);
  CK(hipMemcpy(c.data(), dcyc, P * 8, hipMemcpyDeviceToHost));
  double m = 0;
  for (int i = 0; i < P; ++i) m += (double)c[i];
  printf("panel with waves 1..7 running %-22s %.0f cycles (%.0f per column)\n", name, m / P, m / P / 128);
}

static void panel_case(double* dL, double* dU, unsigned long long* dcyc, int P) {
  hipLaunchKernelGGL(k_panels, dim3(P), dim3(DNTH), 0, 0, dL, dU, dcyc);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> c(P);
  CK(hipMemcpy(c.data(), dcyc, P * 8, hipMemcpyDeviceToHost));
  double m = 0;
  for (int i = 0; i < P; ++i) m += (double)c[i];
  printf("panel: 8 panels on wave 0 alone, %.0f cycles (%.0f per column)\n", m / P, m / P / 128);
}

// dependent-chain latency of single FP64 VALU ops on one wave (cycles per op, s_memtime)
template <int OP>
__global__ __launch_bounds__(64) void k_lat(double a, double b, int n, double* out, unsigned long long* cyc) {
  double x = a + threadIdx.x * 1e-9;
  const unsigned long long t0 = memtime();
#pragma unroll 1
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (OP == 0) x = fma(x, b, 0.25);
      if (OP == 1) x = __builtin_amdgcn_rsq(x) + 0.5;
      if (OP == 2) x = readlane_f64(x, 5) * b;
      if (OP == 3) x = x * b;
    }
    if (OP >= 4) {  // throughput: 8 independent chains
      double y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) y[u] = x + u;
#pragma unroll
      for (int rep = 0; rep < 4; ++rep)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (OP == 4) y[u] = fma(y[u], b, 0.25);
          if (OP == 5) db_fmac_bcast<5, false>(y[u], x, b);
          if (OP == 6) y[u] = y[u] * readlane_f64(x + u, 5);
          if (OP == 7) y[u] = __builtin_amdgcn_rsq(y[u]);
        }
      double t = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) t += y[u];
      x = t * 1e-3;
    }
  }
  const unsigned long long t1 = memtime();
  if (threadIdx.x == 0) {
    out[0] = x;
    cyc[0] = t1 - t0;
  }
}
// the panel's column loop alone on register data (no LDS, no stores), 8 panels' worth of columns;
// MODE 0: as db_panel; 1: no updates s >= q+2; 2: no 1/sqrt chain (inv fixed); 3: 1 + 2
template <int MODE>
__global__ __launch_bounds__(64) void k_col(const double* in, double* out, unsigned long long* cyc) {
  const int r = threadIdx.x;
  const bool arow = r < 16;
  double x[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = in[r * 16 + c];
  bool bad = false;
  const unsigned long long t0 = memtime();
#pragma unroll 1
  for (int k = 0; k < 8; ++k) {
    double inv = MODE >= 2 ? 0.5 : rsqrt_nr(readlane_f64(x[0], 0));
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const double m = (arow && r < q) ? 0.0 : x[q] * inv;
      x[q] = m;
      if (q == 15) break;
      x[q + 1] = fma(-m, readlane_f64(m, q + 1), x[q + 1]);
      const double pn = readlane_f64(x[q + 1], q + 1);
      bad = bad | !(pn > 0.0);
      if (MODE < 2) inv = rsqrt_nr(pn);
      if ((MODE & 1) == 0 && q + 2 < 16) db_fmac_bcast_from<2>(q, x, row0_to_rows(m), m);
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = x[c] * 1.0001 + 1.0;  // (keeps the values positive definite-ish)
  }
  const unsigned long long t1 = memtime();
  double t = bad ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) t += x[c];
  out[r] = t;
  if (r == 0) cyc[0] = t1 - t0;
}
template <int MODE>
static void col_case(const char* name) {
  double *in, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&in, 64 * 16 * 8));
  CK(hipMalloc(&out, 64 * 8));
  CK(hipMalloc(&cyc, 8));
  std::vector<double> h(64 * 16);
  for (int i = 0; i < 64 * 16; ++i) h[i] = (i % 17 == 0) ? 4.0 : 0.01 * ((i * 7) % 13);
  CK(hipMemcpy(in, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  unsigned long long best = ~0ull;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_col<MODE>, dim3(1), dim3(64), 0, 0, in, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    best = c < best ? c : best;
  }
  printf("column loop %-30s %.0f cycles per column\n", name, (double)best / 128.0);
  hipFree(in);
  hipFree(out);
  hipFree(cyc);
}

template <int OP>
static void lat_case(const char* name) {
  double* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, 8));
  CK(hipMalloc(&cyc, 8));
  const int n = 4096;
  hipLaunchKernelGGL(k_lat<OP>, dim3(1), dim3(64), 0, 0, 0.7, 0.999, n, out, cyc);
  CK(hipDeviceSynchronize());
  unsigned long long c;
  CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
  if (OP >= 4)
    printf("throughput %-31s %.1f cycles per op (8 independent chains)\n", name, (double)c / (32.0 * n));
  else
    printf("latency %-34s %.1f cycles per dependent op\n", name, (double)c / (8.0 * n));
  hipFree(out);
  hipFree(cyc);
}

template <int CH>
__global__ __launch_bounds__(256) void k_mfma(int iters, double seed, double* out, unsigned long long* clk) {
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  d4 acc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  const double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = mfma(a, b, acc[i]);
#pragma unroll
    for (int i = 0; i < CH; ++i) asm volatile("" : "+v"(acc[i]));  // (accumulators stay in VGPRs: no AGPR copies)
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < CH; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[blockIdx.x] = s;
  span.stop(clk);
}

template <int CH>
static void mfma_case(int wps) {
  const int blocks = 256 * wps, iters = 32768 / CH;
  double* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, blocks * 8));
  CK(hipMalloc(&clk, 16));
  CK(hipMemset(clk, 0, 16));
  hipLaunchKernelGGL(k_mfma<CH>, dim3(blocks), dim3(256), 0, 0, iters, 1.0, out, nullptr);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_mfma<CH>, dim3(blocks), dim3(256), 0, 0, iters, 1.0, out, clk);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  const double mhz = 100.0 * (double)h[0] / (double)h[1];
  const double tf = (double)blocks * 4.0 * iters * CH * 2048.0 / (ms * 1e-3) / 1e12;
  const double ceil = 128.0 * 256 * mhz * 1e6 / 1e12;
  printf("mfma chains %2d waves/SIMD %d: %.1f TF/s at %.0f MHz = %.3f of 128 flop/CU/clk\n", CH, wps, tf, mhz, tf / ceil);
  hipFree(out);
  hipFree(clk);
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 512;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  std::vector<double> A((size_t)P * NB * NB), Y((size_t)P * NB);
  for (int p = 0; p < P; ++p) {
    double x[3][NB];
    for (int d = 0; d < 3; ++d)
      for (int i = 0; i < NB; ++i) x[d][i] = U01(rng);
    const double ls = 0.15 + 0.5 * U01(rng), e2 = 0.01;
    for (int i = 0; i < NB; ++i) {
      for (int j = 0; j < NB; ++j) {
        double r2 = 0.0;
        for (int d = 0; d < 3; ++d) r2 += (x[d][i] - x[d][j]) * (x[d][i] - x[d][j]) / (ls * ls);
        A[(size_t)p * NB * NB + i * NB + j] = std::exp(-0.5 * r2) + (i == j ? e2 : 0.0);
      }
      Y[(size_t)p * NB + i] = std::sin(6.0 * x[0][i]) + 0.1 * (U01(rng) - 0.5);
    }
  }
  const size_t nm = (size_t)P * NB * NB;
  double *dA, *dL[2], *dU[2], *dy[2], *ds2[2], *dsz[2];
  int* dinfo[2];
  unsigned long long* dcyc;
  CK(hipMalloc(&dA, nm * 8));
  CK(hipMemcpy(dA, A.data(), nm * 8, hipMemcpyHostToDevice));
  for (int v = 0; v < 2; ++v) {
    CK(hipMalloc(&dL[v], nm * 8));
    CK(hipMalloc(&dU[v], nm * 8));
    CK(hipMalloc(&dy[v], (size_t)P * NB * 8));
    CK(hipMalloc(&ds2[v], (size_t)P * NB * 8));
    CK(hipMalloc(&dsz[v], (size_t)P * NB * 8));
    CK(hipMalloc(&dinfo[v], P * 4));
  }
  CK(hipMalloc(&dcyc, P * 8));
  std::vector<unsigned long long> cyc(P);
  const char* name[2] = {"old factor128 (2 x factor64)", "new factor128 (16-blocked)"};
  for (int v = 1; v < 2; ++v) {
    for (int pass = 0; pass < 2; ++pass) {  // P and P/2 workgroups (2 and 1 per CU at P = 512)
      const int Pw = pass == 0 ? P / 2 : P;
      double best = 1e30, sum = 0;
      double mean_cyc = 0;
      for (int r = 0; r < reps; ++r) {
        CK(hipMemcpy(dL[v], dA, nm * 8, hipMemcpyDeviceToDevice));
        CK(hipMemset(dU[v], 0x7f, nm * 8));
        CK(hipMemcpy(dy[v], Y.data(), (size_t)P * NB * 8, hipMemcpyHostToDevice));
        CK(hipMemset(dinfo[v], 0, P * 4));
        CK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_new, dim3(Pw), dim3(DNTH), 0, 0, dL[v], dU[v], dy[v], ds2[v], dsz[v], dinfo[v], dcyc);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = std::min(best, (double)ms);
        sum += ms;
        CK(hipMemcpy(cyc.data(), dcyc, Pw * 8, hipMemcpyDeviceToHost));
        double m = 0;
        for (int p = 0; p < Pw; ++p) m += (double)cyc[p];
        mean_cyc += m / Pw;
      }
      printf("%s, %d workgroups: kernel %.1f us (best of %d), mean %.1f us, %.0f cycles per workgroup (s_memtime)\n",
             name[v], Pw, best * 1e3, reps, sum / reps * 1e3, mean_cyc / reps);
    }
  }
  // agreement and residuals (the last run of each, all P blocks)
  std::vector<double> L[2], Uh[2], z[2], s2[2], sz[2];
  std::vector<int> info[2];
  for (int v = 1; v < 2; ++v) {
    L[v].resize(nm);
    Uh[v].resize(nm);
    z[v].resize((size_t)P * NB);
    s2[v].resize((size_t)P * NB);
    sz[v].resize((size_t)P * NB);
    info[v].resize(P);
    CK(hipMemcpy(L[v].data(), dL[v], nm * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(Uh[v].data(), dU[v], nm * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(z[v].data(), dy[v], (size_t)P * NB * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s2[v].data(), ds2[v], (size_t)P * NB * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sz[v].data(), dsz[v], (size_t)P * NB * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(info[v].data(), dinfo[v], P * 4, hipMemcpyDeviceToHost));
  }
  auto maxrel = [&](const std::vector<double>& a, const std::vector<double>& b, double floor) {
    double m = 0;
    for (size_t i = 0; i < a.size(); ++i) m = std::max(m, std::fabs(a[i] - b[i]) / std::max(std::fabs(b[i]), floor));
    return m;
  };
  int bad1 = 0;
  for (int p = 0; p < P; ++p) bad1 += info[1][p] != 0;
  printf("info != 0: new %d (round 4's factor128 measured 115-116k cycles per workgroup on this probe)\n", bad1);
  // residuals of the new factor on a few blocks (upper triangles must be exact zeros)
  double rl = 0, ru = 0, up = 0, rz = 0;
  for (int p = 0; p < std::min(P, 16); ++p) {
    const double* l = &L[1][(size_t)p * NB * NB];
    const double* u = &Uh[1][(size_t)p * NB * NB];
    const double* a = &A[(size_t)p * NB * NB];
    for (int i = 0; i < NB; ++i)
      for (int j = 0; j < NB; ++j) {
        if (j > i) {
          up = std::max(up, std::fabs(l[i * NB + j]) + std::fabs(u[i * NB + j]));
          continue;
        }
        long double s = 0, t = 0;
        for (int k = 0; k <= j; ++k) s += (long double)l[i * NB + k] * l[j * NB + k];
        for (int k = j; k <= i; ++k) t += (long double)u[i * NB + k] * l[k * NB + j];
        rl = std::max(rl, (double)std::fabs(s - (long double)a[i * NB + j]));
        ru = std::max(ru, (double)std::fabs(t - (i == j ? 1.0L : 0.0L)));
      }
    for (int i = 0; i < NB; ++i) {  // z = U y
      long double s = 0;
      for (int k = 0; k <= i; ++k) s += (long double)u[i * NB + k] * Y[(size_t)p * NB + k];
      rz = std::max(rz, (double)std::fabs((s - z[1][(size_t)p * NB + i]) / (std::fabs(s) + 1e-3)));
    }
  }
  printf("new: max |L L^T - A| %.3e  max |U L - I| %.3e  upper-triangle |L|+|U| %.3e  z = U y rel %.3e\n", rl, ru, up,
         rz);
  // first mismatches of block 0 against a host Cholesky / inverse (long double)
  {
    const double* a = &A[0];
    std::vector<long double> Lr(NB * NB, 0.0L), Xr(NB * NB, 0.0L), zr(NB, 0.0L);
    for (int j = 0; j < NB; ++j) {
      long double d = a[j * NB + j];
      for (int k = 0; k < j; ++k) d -= Lr[j * NB + k] * Lr[j * NB + k];
      Lr[j * NB + j] = std::sqrt(d);
      for (int i = j + 1; i < NB; ++i) {
        long double s = a[i * NB + j];
        for (int k = 0; k < j; ++k) s -= Lr[i * NB + k] * Lr[j * NB + k];
        Lr[i * NB + j] = s / Lr[j * NB + j];
      }
    }
    for (int c = 0; c < NB; ++c)
      for (int i = c; i < NB; ++i) {
        long double s = (i == c) ? 1.0L : 0.0L;
        for (int k = c; k < i; ++k) s -= Lr[i * NB + k] * Xr[k * NB + c];
        Xr[i * NB + c] = s / Lr[i * NB + i];
      }
    for (int i = 0; i < NB; ++i) {
      long double s = 0;
      for (int k = 0; k <= i; ++k) s += Xr[i * NB + k] * Y[k];
      zr[i] = s;
    }
    int shown = 0;
    for (int i = 0; i < NB && shown < 12; ++i)
      for (int j = 0; j < NB && shown < 12; ++j) {
        const double l = L[1][i * NB + j], u = Uh[1][i * NB + j];
        const double el = (double)Lr[i * NB + j], eu = (double)Xr[i * NB + j];
        if (std::fabs(l - el) > 1e-9 * (1 + std::fabs(el)) || std::fabs(u - eu) > 1e-7 * (1 + std::fabs(eu))) {
          printf("  block0 (%3d,%3d): L %.6e want %.6e | U %.6e want %.6e\n", i, j, l, el, u, eu);
          ++shown;
        }
      }
    int zs = 0;
    for (int i = 0; i < NB && zs < 8; ++i)
      if (std::fabs(z[1][i] - (double)zr[i]) > 1e-9 * (1 + std::fabs((double)zr[i]))) {
        printf("  block0 z[%d] = %.6e want %.6e\n", i, z[1][i], (double)zr[i]);
        ++zs;
      }
    unsigned long long st[8][20];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_db_stamps), sizeof(st)));
    const unsigned long long t0 = st[0][17];
    printf("stamps (cycles from the load barrier), wave 0: panel k end / Q_k end; wave 1, 2: step end / Q end\n");
    for (int w : {0, 1, 2, 3, 4, 5, 6, 7}) {
      printf("  w%d:", w);
      for (int i = 0; i < 17; ++i) printf(" %lld", (long long)(st[w][i] - t0));
      printf("\n");
    }
  }
  const bool ok = bad1 == 0 && rl < 1e-12 && ru < 1e-8 && up == 0.0 && rz < 1e-10;
  printf("%s\n", ok ? "PROBE OK" : "PROBE MISMATCH");
  CK(hipMemcpy(dL[1], dA, nm * 8, hipMemcpyDeviceToDevice));
  lat_case<0>("v_fma_f64");
  lat_case<1>("v_rsq_f64 + v_add_f64");
  lat_case<2>("v_readlane_b32 x2 + v_mul_f64");
  lat_case<3>("v_mul_f64");
  lat_case<4>("v_fma_f64");
  lat_case<5>("v_fmac_f64_dpp row_newbcast");
  lat_case<6>("v_readlane_b32 x2 + v_mul_f64");
  lat_case<7>("v_rsq_f64");
  col_case<0>("as db_panel");
  col_case<1>("without updates s >= q+2");
  col_case<2>("without the 1/sqrt chain");
  col_case<3>("neither");
  panel_case(dL[1], dU[1], dcyc, 256);
  {
    double* sink;
    CK(hipMalloc(&sink, 256 * DNTH * 8));
    for (int rep = 0; rep < 2; ++rep) {
      contend_case<0>(dL[1], dU[1], dcyc, sink, 256, "nothing");
      contend_case<1>(dL[1], dU[1], dcyc, sink, 256, "FP64 MFMA chains");
      contend_case<2>(dL[1], dU[1], dcyc, sink, 256, "FP64 v_fma chains");
      contend_case<3>(dL[1], dU[1], dcyc, sink, 256, "LDS reads");
      contend_case<4>(dL[1], dU[1], dcyc, sink, 256, "MFMA, not wave 4");
      contend_case<5>(dL[1], dU[1], dcyc, sink, 256, "MFMA, wave 4 only");
    }
    hipFree(sink);
  }
  mfma_case<8>(1);
  mfma_case<8>(2);
  mfma_case<8>(4);
  mfma_case<16>(2);
  mfma_case<4>(4);
  mfma_case<16>(4);
  return ok ? 0 : 2;
}
