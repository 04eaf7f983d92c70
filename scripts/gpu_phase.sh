#!/bin/bash
# Per-phase k_step workgroup times (diagnostic trace build) at config C and B.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-phase}; mkdir -p $O
timeout -k 10 120 python scripts/wg_phase.py > $O/phase_C.txt 2>&1 || exit $?
N=1024 P=32 timeout -k 10 120 python scripts/wg_phase.py > $O/phase_B.txt 2>&1 || exit $?
tail -3 $O/phase_C.txt
