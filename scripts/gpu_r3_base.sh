#!/bin/bash
# Round-3 baseline on the box: GPU parity suite, default bench, per-phase k_step trace at C and B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3base}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 120 python scripts/wg_phase.py > $O/phase_C.txt 2>&1 || exit $?
N=1024 P=32 timeout -k 10 120 python scripts/wg_phase.py > $O/phase_B.txt 2>&1 || exit $?
tail -3 $O/phase_C.txt
