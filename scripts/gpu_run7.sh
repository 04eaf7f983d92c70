#!/bin/bash
# Env A/B: particle groups and stagger at config C (64 particles), plus a parity spot check.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${TAG:-r2n}; mkdir -p gpurun_out/$O
BQ="--no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 --n 4096 --d 3 --steps 6 --warmup 1"
GPF_GROUPS=2 GPF_GROUP_STAGGER=4 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k "headline or configD" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$O/pytest_stagger.log 2>&1 || { tail -5 gpurun_out/$O/pytest_stagger.log; exit 1; }
tail -1 gpurun_out/$O/pytest_stagger.log
for r in 1 2; do
  for v in "1 0" "2 0" "2 2" "2 4" "2 8" "4 4"; do
    set -- $v
    GPF_GROUPS=$1 GPF_GROUP_STAGGER=$2 timeout -k 10 300 python bench.py --swarm-per-gpu 64 $BQ > gpurun_out/$O/g$1_s$2_$r.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/$O/g$1_s$2_$r.log').read().strip().splitlines()[-1]); print('groups $1 stagger $2 #$r', round(d['value'],1))"
  done
done
