"""One GEMM-core configuration (for PMC passes): mode, npad, P, tiles, depth from argv."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gaussian-process_amd"))
import torch  # noqa: F401,E402
from gpfit import Context  # noqa: E402

mode, npad, P, tiles, D = (int(v) for v in sys.argv[1:6])
ctx = Context()
print(f"mode {mode}: {ctx.gemm_bench(mode=mode, npad=npad, particles=P, tiles=tiles, depth=D, iters=3):.1f} TF/s")
ctx.close()
