"""Compile gpfit_api.hip for gfx950 (device only, build() flags) with the compiler's
kernel-resource-usage remarks and print one row per kernel: VGPRs, AGPRs, SGPRs, VGPR spill,
SGPR spill (to VGPR lanes), scratch bytes/lane, occupancy, LDS bytes.
Usage: python scripts/resource_usage.py [extra hipcc flags...] [> profiles/rN/kernel_resource_usage.txt]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gaussian-process_amd", "csrc", "gpfit_api.hip")
KEYS = ["VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
        "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]


def main():
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-Wno-unused-value", "-Wno-unused-result", "-mllvm", "--amdgpu-mfma-vgpr-form", "--cuda-device-only", "-c",
               "-Rpass-analysis=kernel-resource-usage", SRC, "-o", os.path.join(td, "dev.o")] + sys.argv[1:]
        r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr[-4000:])
        sys.exit(r.returncode)
    ver = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True, text=True).stdout
    m = re.search(r"HIP version: (\S+)", ver)
    rows, cur = {}, None
    for line in r.stderr.splitlines():
        f = re.search(r"Function Name: (\S+)", line)
        if f:
            cur = f.group(1)
            rows[cur] = {}
            continue
        k = re.search(r"remark: \s*(" + "|".join(re.escape(k) for k in KEYS) + r"): (\d+)", line)
        if k and cur:
            rows[cur][k.group(1)] = k.group(2)
    print(f"# hipcc {m.group(1) if m else '?'}, build() flags + -Rpass-analysis=kernel-resource-usage "
          f"{' '.join(sys.argv[1:])}, device code of gpfit_api.hip")
    print("# kernel | VGPRs | AGPRs | SGPRs | VGPR spill | SGPR spill (to VGPR lanes, no memory) | scratch B/lane | waves/SIMD | LDS B")
    for name, v in rows.items():
        short = re.sub(r"^_ZN3gpf\d+", "", name)[:60]
        print(f"{short:60s} | " + " | ".join(v.get(k, "?") for k in KEYS))


if __name__ == "__main__":
    main()
