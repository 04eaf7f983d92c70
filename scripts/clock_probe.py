"""Shader clock vs load (round-4 diagnostic): the GEMM core alone (gpf_gemm_bench, the k_step
stream on L-tile-shaped operands) for short and sustained runs, and the dense MFMA loop
(gpf_mfma_peak), each with the clock its launches held (gpf_bench_clock). Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gaussian-process_amd"))
import gpfit  # noqa: E402

ctx = gpfit.Context(0)
FP64_SPEC, SPEC_MHZ = 78.6, 2400.0
out = {}
for name, mode, iters in (("core_zero_3", 10, 3), ("core_zero_1500", 10, 1500), ("core_3", 2, 3), ("core_300", 2, 300),
                          ("core_1500", 2, 1500), ("core_shared_1500", 1, 1500)):
    t = time.time()
    tf = ctx.gemm_bench(mode=mode, npad=4096, particles=64, tiles=15, depth=2048, iters=iters)
    mhz = ctx.bench_clock()
    out[name] = {"tflops": tf, "sclk_mhz": mhz, "frac_of_clock_ceiling": tf / (FP64_SPEC * mhz / SPEC_MHZ),
                 "wall_s": time.time() - t}
for name, iters in (("mfma_loop", 8192), ("mfma_loop_long", 65536)):
    tf = ctx.mfma_peak(blocks=1024, iters=iters)
    mhz = ctx.bench_clock()
    out[name] = {"tflops": tf, "sclk_mhz": mhz, "frac_of_clock_ceiling": tf / (FP64_SPEC * mhz / SPEC_MHZ)}
print(json.dumps(out))
