#!/bin/bash
# GPU tests first (the early diagonal hand-off), then A/B prev vs new and critical-tile traces.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${TAG:-r2h}; mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$O/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TAG=$O VARIANTS="prev new" CFGS="C B" REPS=2 bash scripts/gpu_abx.sh || exit $?
for v in prev new; do GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --pso-steps 0 --psurf-rows 0 --no-hull > gpurun_out/$O/pred_$v.log 2>&1 || exit $?; python -c "import json; d=json.loads(open('gpurun_out/$O/pred_$v.log').read().strip().splitlines()[-1]); print('$v predict', d['predict']['ms'], 'ms factor', d['predict']['factor_ms'])"; done
MODE=predict timeout -k 10 200 python scripts/crit_trace.py > gpurun_out/$O/crit_predict.txt 2>&1 || exit $?
MODE=eval timeout -k 10 200 python scripts/crit_trace.py > gpurun_out/$O/crit_B.txt 2>&1 || exit $?
tail -8 gpurun_out/$O/crit_predict.txt; cat gpurun_out/$O/crit_B.txt
