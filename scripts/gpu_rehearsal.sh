#!/bin/bash
# Rehearsal of the driver's round-end GPU tiers on a fresh box: pytest -m gpu, smoke() (which
# rebuilds the library on a GPU box), then the default bench line.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-rehearsal}; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
s0=$(date +%s); timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?; echo "smoke wall $(( $(date +%s) - s0 )) s"
grep -E "smoke|build" $O/smoke.log | cut -c1-160
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
