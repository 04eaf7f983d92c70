"""The GEMM-core ceiling (gpf_gemm_bench) against its grid geometry: 960 workgroups fill the
512 slots (256 CUs x 2) 1.875 times, so the last round runs 448 of 512 and the core reads ~6%
low; 1024 and 512 workgroups are whole rounds. Prints TF/s, the clock held and the fraction of
128 flop/CU/clk at that clock per geometry."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gaussian-process_amd")]
import gpfit  # noqa: E402

ctx = gpfit.Context(0)
ctx.gemm_bench(mode=2, npad=4096, particles=64, tiles=8, depth=2048, iters=100)  # clock settle
for tiles, depth in ((15, 2048), (16, 1920), (8, 2048), (15, 2048), (16, 1920)):
    tf = ctx.gemm_bench(mode=2, npad=4096, particles=64, tiles=tiles, depth=depth, iters=300)
    mhz = ctx.bench_clock()
    print(f"tiles {tiles:2d} x 64 particles = {64 * tiles:4d} workgroups, depth {depth}: {tf:5.1f} TF/s at "
          f"{mhz:5.0f} MHz = {tf * 1e12 / (128 * 256 * mhz * 1e6):.3f} of 128 flop/CU/clk", flush=True)
