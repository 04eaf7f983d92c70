// Probe: does FP64 VALU FMA work overlap FP64 MFMA on gfx950 (separate pipes)?
// Workgroups of 8 waves: waves 0-3 (one per SIMD) run independent v_mfma_f64_16x16x4 chains,
// waves 4-7 run independent v_fma_f64 chains. Modes: 1 = MFMA waves only, 2 = VALU waves only,
// 3 = both. If mode 3 takes ~max(mode 1, mode 2), the pipes co-issue.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k(int mode, int iters, int vreps, double* out) {
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  double r = 0.0;
  if (w < 4) {
    if (!(mode & 1)) return;
    d4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;
    double x = 1.0 + lane * 1e-3, y = 1.0 - lane * 1e-3;
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
      a4 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a4, 0, 0, 0);
      a5 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a5, 0, 0, 0);
      a6 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a6, 0, 0, 0);
      a7 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a7, 0, 0, 0);
    }
    d4 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    r = s[0] + s[1] + s[2] + s[3];
  } else {
    if (!(mode & 2)) return;
    double c[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) c[j] = lane * 1e-3 + j;
    const double x = 1.0000001, y = 0.9999999;
    for (int i = 0; i < iters * vreps / 2; ++i) {
#pragma unroll
      for (int rep = 0; rep < 2; ++rep)
#pragma unroll
        for (int j = 0; j < 16; ++j) c[j] = __builtin_fma(c[j], x, y);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) r += c[j];
  }
  if (r == 12345.678) out[0] = r;  // keep the chains live
}

int main() {
  double* out;
  hipMalloc(&out, 8);
  const int blocks = 256 * 4, iters = 20000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int vreps : {2, 6, 8, 10})
  for (int mode = 1; mode <= 3; ++mode) {
    if (mode == 1 && vreps != 2) continue;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, mode, 100, vreps, out);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, mode, iters, vreps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // per wave-iteration: MFMA 8 x 2048 flop; VALU 32 x 64 lanes x 2 flop
    const double mf = (mode & 1) ? 4.0 * blocks * iters * 8 * 2048.0 : 0.0;
    const double vf = (mode & 2) ? 4.0 * blocks * (double)(iters * vreps / 2) * 32 * 64 * 2.0 : 0.0;
    printf("vreps %d mode %d: %.3f ms  MFMA %.1f TF  VALU %.1f TF  total %.1f TF\n", vreps, mode, ms, mf / ms / 1e9, vf / ms / 1e9,
           (mf + vf) / ms / 1e9);
  }
  return 0;
}
