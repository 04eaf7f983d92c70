"""GEMM-core latency probe: the ring GEMM (gemm_stream_ring, 8-deep chunks, 64 KiB ring) at
prefetch distances of 1, 2 and 3 chunks vs the default direct-to-LDS path (mode 2)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gaussian-process_amd"))
import torch  # noqa: F401,E402
from gpfit import Context  # noqa: E402

ctx = Context()
for rep in range(2):
    for mode, label in [(2, "dl (KC16, dist 1 chunk = 16 deep)"), (8 + 48, "ring dist 1 (8 deep)"),
                        (8 + 32, "ring dist 2 (16 deep)"), (8 + 16, "ring dist 3 (24 deep)"),
                        (8, "ring dist 2 staggered (d8)"), (8 + 4 + 16, "ring dist 3 NN")]:
        tf = ctx.gemm_bench(mode=mode, npad=4096, particles=64, tiles=15, depth=2048, iters=5)
        print(f"mode {mode:3d} {label:36s}: {tf:.1f} TF/s", flush=True)
ctx.close()
