#!/bin/bash
# One iteration: GPU parity suite (unless SKIP_TESTS), benches C and B, phase traces at C and B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3it}; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
BQ="--no-cpu --predict-points 0 --no-hull --psurf-rows 0"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 $BQ > $O/bench_C.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 40 --warmup 4 $BQ > $O/bench_B.log 2>&1 || exit $?
for f in C B; do python -c "import json; d=json.loads(open('$O/bench_$f.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(d['value'],1), 'frac', round(r['frac'],3))"; done
if [ -z "$SKIP_PHASE" ]; then
  timeout -k 10 120 python scripts/wg_phase3.py > $O/phase_C.txt 2>&1 || exit $?
  N=1024 D=2 P=32 timeout -k 10 120 python scripts/wg_phase3.py > $O/phase_B.txt 2>&1 || exit $?
  tail -1 $O/phase_C.txt; tail -1 $O/phase_B.txt
fi
