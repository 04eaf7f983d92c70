"""GEMM-core microbenchmark (gpf_gemm_bench): TF/s of the k_step L-tile GEMM alone."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gaussian-process_amd"))
import torch  # noqa: F401,E402  (initialise the HIP runtime first)
from gpfit import Context  # noqa: E402

ctx = Context()
print("mfma_peak(k_mfma_rate)", round(ctx.mfma_peak(blocks=2048, iters=4096), 1), "TF")
for mode, npad, P, tiles, D in [(0, 4096, 64, 15, 2048), (2, 4096, 64, 15, 2048), (1, 4096, 64, 15, 2048),
                                (3, 4096, 64, 15, 2048), (0, 8192, 32, 31, 4096), (2, 8192, 32, 31, 4096),
                                (0, 4096, 64, 27, 512), (2, 4096, 64, 27, 512),
                                (6, 4096, 64, 15, 2048), (7, 4096, 64, 15, 2048), (6, 4096, 64, 27, 512),
                                (10, 4096, 64, 15, 2048), (11, 4096, 64, 15, 2048), (14, 4096, 64, 15, 2048), (10, 4096, 64, 27, 512)]:
    tf = ctx.gemm_bench(mode=mode, npad=npad, particles=P, tiles=tiles, depth=D, iters=5)
    print(f"mode {mode} Npad {npad} P {P} tiles {tiles} depth {D}: {tf:.1f} TF/s", flush=True)
ctx.close()
