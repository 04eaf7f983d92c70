"""The k_step GEMM core (gpf_gemm_bench, hashed operands) at one and at two workgroups per CU and
at piece-like (short) and long depths: how much of the FP64 MFMA rate a split-K piece's GEMM can
reach when the all-tile split runs one piece per CU (the prediction factorisation)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402

ctx = gpfit.Context(0)
print("mfma peak probe:", round(ctx.mfma_peak(), 1), "TF/s")
for depth in (256, 512, 2048):
    for P, tiles in ((32, 8), (64, 8)):
        for ns, mode in ((2, 0), (3, 16), (4, 32)):
            if P * tiles > 256 and ns > 2:
                continue  # (3-4 stages take one workgroup per CU)
            tf = max(ctx.gemm_bench(mode=mode, npad=4096, particles=P, tiles=tiles, depth=depth, iters=5)
                     for _ in range(3))
            print(f"depth {depth:5d}  workgroups {P * tiles:4d} ({P * tiles // 256} per CU)  {ns} stages: "
                  f"{tf:6.1f} TF/s at {ctx.bench_clock():.0f} MHz")
