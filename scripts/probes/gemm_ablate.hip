// gemm_ablate.hip — where the streamed GEMM core (gpf_common.hip DenseRun, the k_step L-tile shape:
// 128x128 output per 512-thread workgroup, 2 workgroups per CU, 16-deep chunks) loses its ~11% per
// clock against the register-only MFMA loop. Each variant removes one part of the chunk loop:
//   0  gemm_stream_dl itself
//   1  the same loop written out here (sanity: must match 0)
//   2  no global->LDS transfers (LDS holds the first two chunks; barrier and operand reads kept)
//   3  no transfers, no barrier (operand reads + MFMAs only)
//   4  transfers + barrier, no operand reads (operands read once before the loop)
//   5  MFMAs only
//   6  as 1 with the k-step's operands read one k-step ahead (two register sets)
//   7  two outputs per workgroup sharing the streamed B panel, one workgroup per CU (k_dual)
//   8  the same on a 16-wave workgroup: one output per 8 waves, 4 waves per SIMD (k_dual16)
//   9  r6: single-output 8-wave workgroups, 2 per CU, in pairs that share the B panel through the
//      XCD's L2 (workgroups b and b + 8: the dispatcher deals ids round-robin over the 8 XCDs, so
//      both sit on one XCD and start together), against A panels J and J+1 (k_pair2)
//  10  the same pairs placed on different XCDs (b and b + 1): no L2 sharing (control)
// Per variant: TF/s, the shader clock held (s_memtime over s_memrealtime) and the fraction of
// 128 flop/CU/clk at that clock. Operands are hashed values in [-1, 1) (the clock depends on them).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm --amdgpu-mfma-vgpr-form \
//     scripts/probes/gemm_ablate.hip -o gemm_ablate && ./gemm_ablate [tiles] [depth] [shared]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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
using DR = DenseRun<false, true, 2>;

// variant 6's chunk: operands of k-step s+1 read before the MFMAs of k-step s
template <int BUF>
__device__ __forceinline__ void mma_ahead(const DR& dr, Acc<128>& acc, const double* smem) {
  const char* sb = (const char*)smem + BUF * DL_BUF * 8;
  double a0[8], b0, a1[8], b1;
  dr.reads<0>(sb, 0, a0, b0);
  dr.reads<0>(sb, 1, a1, b1);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) acc.v[mi][0] = mfma_neg_a(a0[mi], b0, acc.v[mi][0]);
  dr.reads<0>(sb, 2, a0, b0);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) acc.v[mi][0] = mfma_neg_a(a1[mi], b1, acc.v[mi][0]);
  dr.reads<0>(sb, 3, a1, b1);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) acc.v[mi][0] = mfma_neg_a(a0[mi], b0, acc.v[mi][0]);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) acc.v[mi][0] = mfma_neg_a(a1[mi], b1, acc.v[mi][0]);
}

template <int V, int BUF>
__device__ __forceinline__ void body(const DR& dr, Acc<128>& acc, const double* A, const double* B, int ld, int t,
                                     int nch, double* smem, const double (&ra)[8], double rb) {
  constexpr bool LOADS = V == 1 || V == 4 || V == 6, BAR = V == 1 || V == 2 || V == 4 || V == 6;
  if (LOADS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (BAR) __syncthreads();
  else asm volatile("" ::: "memory");  // (keeps the operand reads of a chunk in their chunk: no spills)
  if (LOADS && t + 1 < nch) dr.issue<BUF ^ 1>(A, B, ld, t + 1, smem);
  if constexpr (V == 4 || V == 5) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) acc.v[mi][0] = mfma_neg_a(ra[mi], rb, acc.v[mi][0]);
  } else if constexpr (V == 6) {
    mma_ahead<BUF>(dr, acc, smem);
  } else {
    dr.mma<BUF, 0>(acc, smem);
  }
}

template <int V>
__global__ __launch_bounds__(STEP_NTH, STEP_WAVES_PER_SIMD) void k_abl(const double* __restrict__ L, int ld, int D,
                                                                       int shared, double* __restrict__ C,
                                                                       unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[2 * DL_BUF];
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  const int b = blockIdx.x;
  const double* A = uniform_ptr(L);
  const double* B = uniform_ptr(L + (size_t)(shared ? 1 : 1 + b) * T * ld);
  const Quad<T> qd;
  Acc<T> acc;
  acc.zero();
  if constexpr (V == 0) {
    gemm_stream_dl<false, true>(acc, A, ld, B, ld, D, smem, qd);
  } else {
    const int nch = D / DL_KC, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const DR dr(qd, ld, ld, wave);
    dr.issue<0>(A, B, ld, 0, smem);
    dr.issue<1>(A, B, ld, 1, smem);  // both buffers hold real operands (variants without transfers)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    double ra[8], rb;
    dr.reads<0>((const char*)smem, 0, ra, rb);
#pragma unroll 1
    for (int t = 0; t + 1 < nch; t += 2) {
      body<V, 0>(dr, acc, A, B, ld, t, nch, smem, ra, rb);
      body<V, 1>(dr, acc, A, B, ld, t + 1, nch, smem, ra, rb);
    }
    __syncthreads();
  }
  acc.store(qd, C + (size_t)b * T * T, T);
  span.stop(clk);
}

// variant 7: the 256-wide block column's core: one 8-wave workgroup per CU (256 VGPRs)
// computes two 128x128 outputs that share the streamed B panel (row panel I, distinct per
// workgroup) against two A panels (row panels J and J+1, shared by every workgroup): per k-step
// a wave reads 8 + 8 A values and one B value and issues 16 MFMAs; 48 KiB of LDS per stage.
constexpr int DUAL_BUF = 3 * 128 * DL_KC;
template <int BUF>
__device__ __forceinline__ void dual_issue(const DR& dr, const double* A0, const double* A1, const double* B, int c,
                                           double* smem) {
  const char* a0 = uniform_ptr((const char*)(A0 + c * DL_KC));
  const char* a1 = uniform_ptr((const char*)(A1 + c * DL_KC));
  const char* bb = uniform_ptr((const char*)(B + c * DL_KC));
  double* sbuf = smem + BUF * DUAL_BUF;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int blk = dr.blk0 + u;
    dl_load_s(a0, dr.ga[u], sbuf + blk * 8 * DL_KC);
    dl_load_s(a1, dr.ga[u], sbuf + 128 * DL_KC + blk * 8 * DL_KC);
    dl_load_s(bb, dr.gb[u], sbuf + 256 * DL_KC + blk * 8 * DL_KC);
  }
}
template <int BUF>
__device__ __forceinline__ void dual_mma(const DR& dr, Acc<128>& c0, Acc<128>& c1, const double* smem) {
  const char* sb = (const char*)smem + BUF * DUAL_BUF * 8;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    double a0[8], a1[8], b;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) a0[mi] = *(const double*)(sb + dr.la[s] + mi * 16 * DL_KC * 8);
    dr.reads<0>(sb + 128 * DL_KC * 8, s, a1, b);  // (its B read lands in the B region: lb = la + 128 KC)
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) c0.v[mi][0] = mfma_neg_a(a0[mi], b, c0.v[mi][0]);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) c1.v[mi][0] = mfma_neg_a(a1[mi], b, c1.v[mi][0]);
  }
}
template <int BUF>
__device__ __forceinline__ void dual_body(const DR& dr, Acc<128>& c0, Acc<128>& c1, const double* A0, const double* A1,
                                          const double* B, int t, int nch, double* smem) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t + 1 < nch) dual_issue<BUF ^ 1>(dr, A0, A1, B, t + 1, smem);
  dual_mma<BUF>(dr, c0, c1, smem);
}
// (NS = 3: chunk t+2 in flight while chunk t runs; 144 KiB of LDS)
template <int BUF>
__device__ __forceinline__ void dual_body3(const DR& dr, Acc<128>& c0, Acc<128>& c1, const double* A0, const double* A1,
                                           const double* B, int t, int nch, double* smem) {
  if (t + 1 < nch) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // chunk t done, t+1 may be in flight
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t + 2 < nch) dual_issue<(BUF + 2) % 3>(dr, A0, A1, B, t + 2, smem);
  dual_mma<BUF>(dr, c0, c1, smem);
}
__global__ __launch_bounds__(STEP_NTH, 2) void k_dual3(const double* __restrict__ L, int ld, int D, int shared,
                                                       double* __restrict__ C, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[3 * DUAL_BUF];
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  const int b = blockIdx.x;
  const double* A0 = uniform_ptr(L);
  const double* A1 = uniform_ptr(L + (size_t)T * ld);
  const double* B = uniform_ptr(L + (size_t)(shared ? 2 : 2 + b) * T * ld);
  const Quad<T> qd;
  Acc<T> c0, c1;
  c0.zero();
  c1.zero();
  const int nch = D / DL_KC, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const DR dr(qd, ld, ld, wave);
  dual_issue<0>(dr, A0, A1, B, 0, smem);
  dual_issue<1>(dr, A0, A1, B, 1, smem);
  __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll 1
  for (int t = 0; t + 2 < nch; t += 3) {  // (nch % 3 == 0: main checks)
    dual_body3<0>(dr, c0, c1, A0, A1, B, t, nch, smem);
    dual_body3<1>(dr, c0, c1, A0, A1, B, t + 1, nch, smem);
    dual_body3<2>(dr, c0, c1, A0, A1, B, t + 2, nch, smem);
  }
  __syncthreads();
  c0.store(qd, C + (size_t)(2 * b) * T * T, T);
  c1.store(qd, C + (size_t)(2 * b + 1) * T * T, T);
  span.stop(clk);
}

// variant 8: the same two outputs on a 16-wave workgroup (1024 threads, 4 waves per SIMD, 128
// VGPRs): waves 0-7 own output 0, waves 8-15 output 1, both read the one B chunk in LDS.
template <int BUF>
__device__ __forceinline__ void dual16_issue(const DR& dr, int o, const double* A0, const double* A1, const double* B,
                                             int c, double* smem) {
  double* sbuf = smem + BUF * DUAL_BUF;
  if (o == 0) {
    const char* a0 = uniform_ptr((const char*)(A0 + c * DL_KC));
    const char* bb = uniform_ptr((const char*)(B + c * DL_KC));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int blk = dr.blk0 + u;
      dl_load_s(a0, dr.ga[u], sbuf + blk * 8 * DL_KC);
      dl_load_s(bb, dr.gb[u], sbuf + 256 * DL_KC + blk * 8 * DL_KC);
    }
  } else {
    const char* a1 = uniform_ptr((const char*)(A1 + c * DL_KC));
#pragma unroll
    for (int u = 0; u < 2; ++u) dl_load_s(a1, dr.ga[u], sbuf + 128 * DL_KC + (dr.blk0 + u) * 8 * DL_KC);
  }
}
template <int BUF>
__device__ __forceinline__ void dual16_body(const DR& dr, int o, Acc<128>& acc, const double* A0, const double* A1,
                                            const double* B, int t, int nch, double* smem) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t + 1 < nch) dual16_issue<BUF ^ 1>(dr, o, A0, A1, B, t + 1, smem);
  const char* sb = (const char*)smem + BUF * DUAL_BUF * 8;
  const char* sa = sb + o * 128 * DL_KC * 8;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    double a[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) a[mi] = *(const double*)(sa + dr.la[st] + mi * 16 * DL_KC * 8);
    const double b = *(const double*)(sb + 128 * DL_KC * 8 + dr.lb[st]);  // (the B region: lb = la + 128 KC + cb)
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) acc.v[mi][0] = mfma_neg_a(a[mi], b, acc.v[mi][0]);
  }
}
__global__ __launch_bounds__(1024, 1) void k_dual16(const double* __restrict__ L, int ld, int D, int shared,
                                                    double* __restrict__ C, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[2 * DUAL_BUF];
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  const int b = blockIdx.x;
  const double* A0 = uniform_ptr(L);
  const double* A1 = uniform_ptr(L + (size_t)T * ld);
  const double* B = uniform_ptr(L + (size_t)(shared ? 2 : 2 + b) * T * ld);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), o = w >> 3, wl = w & 7;
  Quad<T> qd;
  qd.cb = (wl >= 4 ? 11 - wl : wl) * 16;
  const DR dr(qd, ld, ld, wl);
  Acc<T> acc;
  acc.zero();
  const int nch = D / DL_KC;
  dual16_issue<0>(dr, o, A0, A1, B, 0, smem);
  __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll 1
  for (int t = 0; t + 1 < nch; t += 2) {
    dual16_body<0>(dr, o, acc, A0, A1, B, t, nch, smem);
    dual16_body<1>(dr, o, acc, A0, A1, B, t + 1, nch, smem);
  }
  __syncthreads();
  acc.store(qd, C + (size_t)(2 * b + o) * T * T, T);
  span.stop(clk);
}

__global__ __launch_bounds__(STEP_NTH, 2) void k_dual(const double* __restrict__ L, int ld, int D, int shared,
                                                      double* __restrict__ C, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[2 * DUAL_BUF];
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  const int b = blockIdx.x;
  const double* A0 = uniform_ptr(L);
  const double* A1 = uniform_ptr(L + (size_t)T * ld);
  const double* B = uniform_ptr(L + (size_t)(shared ? 2 : 2 + b) * T * ld);
  const Quad<T> qd;
  Acc<T> c0, c1;
  c0.zero();
  c1.zero();
  const int nch = D / DL_KC, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const DR dr(qd, ld, ld, wave);
  dual_issue<0>(dr, A0, A1, B, 0, smem);
  __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll 1
  for (int t = 0; t + 1 < nch; t += 2) {
    dual_body<0>(dr, c0, c1, A0, A1, B, t, nch, smem);
    dual_body<1>(dr, c0, c1, A0, A1, B, t + 1, nch, smem);
  }
  __syncthreads();
  c0.store(qd, C + (size_t)(2 * b) * T * T, T);
  c1.store(qd, C + (size_t)(2 * b + 1) * T * T, T);
  span.stop(clk);
}

// variants 9/10: workgroup b computes output o of pair q against A panel o (row panel 0 or 1), B panel
// 2 + q; XCD-local pairs (9: b, b + 8) or split pairs (10: b, b + 1)
template <int XL>
__global__ __launch_bounds__(STEP_NTH, STEP_WAVES_PER_SIMD) void k_pair2(const double* __restrict__ L, int ld, int D,
                                                                         double* __restrict__ C,
                                                                         unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) double smem[2 * DL_BUF];
  __shared__ unsigned long long cs[2];
  const ClockSpan span(cs);
  span.start(clk);
  const int b = blockIdx.x;
  const int o = XL ? (b >> 3) & 1 : b & 1, q = XL ? (b >> 4) * 8 + (b & 7) : b >> 1;
  const Quad<T> qd;
  Acc<T> acc;
  acc.zero();
  gemm_stream_dl<false, true>(acc, L + (size_t)o * T * ld, ld, L + (size_t)(2 + q) * T * ld, ld, D, smem, qd);
  acc.store(qd, C + (size_t)b * T * T, T);
  span.stop(clk);
}

template <int XL>
void run_pair2(int W, int D, const double* L, int ld, double* C, unsigned long long* clk, double mhz_ref) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_pair2<XL>, dim3(W), dim3(STEP_NTH), 0, 0, L, ld, D, C, nullptr);
  CK(hipMemset(clk, 0, 16));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_pair2<XL>, dim3(W), dim3(STEP_NTH), 0, 0, L, ld, D, C, clk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  const double mhz = (double)h[0] / (double)h[1] * mhz_ref;
  const double tf = 2.0 * T * T * (double)D * W * iters / (ms * 1e-3) / 1e12;
  printf("%d %-44s %6.1f TF/s at %5.0f MHz = %.3f of 128 flop/CU/clk\n", XL ? 9 : 10,
         XL ? "pairs sharing B through the XCD's L2" : "pairs split over two XCDs (control)", tf, mhz,
         tf * 1e12 / (128.0 * 256 * mhz * 1e6));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int V>
void run(const char* name, int W, int D, int shared, const double* L, int ld, double* C, unsigned long long* clk,
         double mhz_ref) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_abl<V>, dim3(W), dim3(STEP_NTH), 0, 0, L, ld, D, shared, C, nullptr);
  CK(hipMemset(clk, 0, 16));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_abl<V>, dim3(W), dim3(STEP_NTH), 0, 0, L, ld, D, shared, C, clk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  const double mhz = (double)h[0] / (double)h[1] * mhz_ref;
  const double tf = 2.0 * T * T * (double)D * W * iters / (ms * 1e-3) / 1e12;
  const double frac = tf * 1e12 / (128.0 * 256 * mhz * 1e6);
  printf("%d %-44s %6.1f TF/s at %5.0f MHz = %.3f of 128 flop/CU/clk\n", V, name, tf, mhz, frac);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

// variant 7 over W/2 workgroups (the same outputs and flops as W single-output workgroups)
void run_dual(int W, int D, int shared, const double* L, int ld, double* C, unsigned long long* clk, double mhz_ref,
              int ns = 2) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int Wd = W / 2;
  const auto kern = ns == 16 ? k_dual16 : ns == 3 ? k_dual3 : k_dual;
  const int nth = ns == 16 ? 1024 : STEP_NTH;
  hipLaunchKernelGGL(kern, dim3(Wd), dim3(nth), 0, 0, L, ld, D, shared, C, nullptr);
  CK(hipMemset(clk, 0, 16));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(kern, dim3(Wd), dim3(nth), 0, 0, L, ld, D, shared, C, clk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  const double mhz = (double)h[0] / (double)h[1] * mhz_ref;
  const double tf = 2.0 * 2.0 * T * T * (double)D * Wd * iters / (ms * 1e-3) / 1e12;
  printf("7 %-44s %6.1f TF/s at %5.0f MHz = %.3f of 128 flop/CU/clk\n",
         ns == 16 ? "two outputs, 16-wave workgroup, one per CU"
         : ns == 3 ? "two outputs per workgroup, one per CU, 3 stages" : "two outputs per workgroup, one per CU", tf, mhz,
         tf * 1e12 / (128.0 * 256 * mhz * 1e6));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 1024, D = argc > 2 ? atoi(argv[2]) : 2048, shared = argc > 3 ? atoi(argv[3]) : 0;
  if (D % 256 || D < 256 || W < 1 || W > 4096) {
    fprintf(stderr, "bad args\n");
    return 1;
  }
  if (W % 16) {
    fprintf(stderr, "tiles: a multiple of 16\n");
    return 1;
  }
  const int ld = D, rows = (shared ? 3 : W + 2) * T;
  double *L, *C;
  unsigned long long* clk;
  CK(hipMalloc(&L, (size_t)rows * ld * 8));
  CK(hipMalloc(&C, (size_t)W * T * T * 8));
  CK(hipMalloc(&clk, 16));
  hipLaunchKernelGGL(k_fill_hash, dim3(4096), dim3(NTHR), 0, 0, L, (long long)rows * ld);
  CK(hipDeviceSynchronize());
  printf("tiles %d depth %d %s B panels\n", W, D, shared ? "one shared (L2-resident)" : "distinct (HBM)");
  const double ref = 100.0;  // s_memrealtime: 100 MHz
  if (getenv("ABL_PMC")) {  // (a short run for rocprofv3 --pmc: the single-output loop and the 16-wave pair only)
    run<1>("same loop here", W, D, shared, L, ld, C, clk, ref);
    run_dual(W, D, shared, L, ld, C, clk, ref, 16);
    if (W % 16 == 0) run_pair2<1>(W, D, L, ld, C, clk, ref);
    printf("PROBE OK\n");
    return 0;
  }
  if (getenv("ABL_PAIR")) {  // (r6: the L2-shared pairs against the single-output loop and the 16-wave pair)
    for (int rep = 0; rep < 2; ++rep) {
      run<1>("same loop here", W, D, shared, L, ld, C, clk, ref);
      run_dual(W, D, shared, L, ld, C, clk, ref, 16);
      run_pair2<1>(W, D, L, ld, C, clk, ref);
      run_pair2<0>(W, D, L, ld, C, clk, ref);
    }
    printf("PROBE OK\n");
    return 0;
  }
  run<0>("gemm_stream_dl", W, D, shared, L, ld, C, clk, ref);
  run<1>("same loop here", W, D, shared, L, ld, C, clk, ref);
  run<2>("no transfers", W, D, shared, L, ld, C, clk, ref);
  run<3>("no transfers, no barrier", W, D, shared, L, ld, C, clk, ref);
  run<4>("transfers + barrier, no operand reads", W, D, shared, L, ld, C, clk, ref);
  run<5>("MFMAs only", W, D, shared, L, ld, C, clk, ref);
  run<6>("as 1, operands read a k-step ahead", W, D, shared, L, ld, C, clk, ref);
  run<0>("gemm_stream_dl again (the first run starts cold)", W, D, shared, L, ld, C, clk, ref);
  run_dual(W, D, shared, L, ld, C, clk, ref);
  run<1>("same loop here, again", W, D, shared, L, ld, C, clk, ref);
  run_dual(W, D, shared, L, ld, C, clk, ref);
  run_dual(W, D, shared, L, ld, C, clk, ref, 16);
  run<1>("same loop here, again", W, D, shared, L, ld, C, clk, ref);
  run_dual(W, D, shared, L, ld, C, clk, ref, 16);
  if ((D / DL_KC) % 3 == 0) {
    run_dual(W, D, shared, L, ld, C, clk, ref, 3);
    run<1>("same loop here, again", W, D, shared, L, ld, C, clk, ref);
    run_dual(W, D, shared, L, ld, C, clk, ref, 3);
  }
  CK(hipFree(L));
  CK(hipFree(C));
  CK(hipFree(clk));
  printf("PROBE OK\n");
  return 0;
}
