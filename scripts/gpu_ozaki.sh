#!/bin/bash
# Int8-emulated fp64 GEMM feasibility probe (scripts/probes/ozaki_core.hip), plus the parity
# test of the fused/early/deep/quadrant schedules.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-oz}; mkdir -p $O
timeout -k 10 120 ./scripts/probes/ozaki_core 2048 > $O/ozaki.txt 2>&1; rc=$?; cat $O/ozaki.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 120 ./scripts/probes/ozaki_core 4096 | tail -2 >> $O/ozaki.txt || exit $?
[ -x scripts/probes/ozaki_core8 ] && { timeout -k 10 120 ./scripts/probes/ozaki_core8 2048 >> $O/ozaki.txt 2>&1 || exit $?; }
tail -1 $O/ozaki.txt
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "early_diagonal" > $O/unit.log 2>&1; rc=$?; tail -2 $O/unit.log; exit $rc
fi
