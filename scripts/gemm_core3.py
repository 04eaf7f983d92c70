"""GEMM-core microbenchmark (gpf_gemm_bench) of a given library (GPFIT_LIB): the k_step L-tile
GEMM alone, L2-resident shared operands and per-particle operands. MODES: 'old' (round-2 bit
layout: 2 = direct, 1 = shared, 4 = NN) or 'new' (round 3: direct always, 1 = shared, 4 = NN)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gaussian-process_amd"))
from gpfit import Context  # noqa: E402

old = os.environ.get("MODES", "new") == "old"
ctx = Context()
for name, mode, npad, P, tiles, D in [("shared LLt", 1, 4096, 64, 15, 2048), ("per-particle LLt", 0, 4096, 64, 15, 2048),
                                      ("shared NN", 5, 4096, 64, 15, 2048), ("per-particle LLt deep", 0, 8192, 32, 31, 4096)]:
    m = (mode | 2) if old else mode
    tf = ctx.gemm_bench(mode=m, npad=npad, particles=P, tiles=tiles, depth=D, iters=5)
    print(f"{name:24s} Npad {npad} P {P} tiles {tiles} depth {D}: {tf:.1f} TF/s", flush=True)
ctx.close()
