"""Where a kernel spills: compile gpfit_api.hip for gfx950 (device only, build() flags,
-gline-tables-only) and list each scratch_* instruction of the kernels whose symbol contains the
given substring with the source lines (file:line) of the instructions just before it.
Usage: python scripts/spill_sites.py k_factor [k_stepILi0ELi1E ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gaussian-process_amd", "csrc", "gpfit_api.hip")


def main():
    pats = sys.argv[1:] or ["k_step"]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "dev.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                        "-Wno-unused-value", "-Wno-unused-result", "-mllvm", "--amdgpu-mfma-vgpr-form", "--cuda-device-only", "-gline-tables-only", "-S", SRC,
                        "-o", out], check=True, capture_output=True)
        lines = open(out).read().splitlines()
    files, fn, hist = {}, None, []
    for line in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s*"([^"]*)"', line)
        if m:
            files[m.group(1)] = m.group(3).split("/")[-1]
    for line in lines:
        m = re.match(r"^(_Z\S+):", line)
        if m:
            fn, hist = m.group(1), []
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            hist.append(f"{files.get(m.group(1), m.group(1))}:{m.group(2)}")
            hist = hist[-60:]
        if fn and any(p in fn for p in pats) and "scratch_" in line:
            seen = []
            for h in reversed(hist):
                if h not in seen:
                    seen.append(h)
            print(f"{fn[:40]}  {line.strip()[:60]}\n    {' '.join(seen[:8])}")


if __name__ == "__main__":
    main()
