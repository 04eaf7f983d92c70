#!/bin/bash
# GPU tests, lib A/B (prev vs new) on B / N2048 / C / D and the prediction, critical-tile traces.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${TAG:-r2j}; mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$O/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
BQ="--no-cpu --pso-steps 0 --no-hull --psurf-rows 0"
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32 --steps 30 --predict-points 0" [C]="--n 4096 --d 3 --swarm-per-gpu 64 --steps 6 --predict-points 0"
                 [D]="--n 4096 --d 3 --swarm-per-gpu 32 --steps 8 --predict-points 0" [N2048]="--n 2048 --d 3 --swarm-per-gpu 32 --steps 15 --predict-points 0"
                 [PRED]="--n 4096 --d 3 --swarm-per-gpu 8 --steps 1" )
for r in 1 2; do
  for c in ${CFGS:-B N2048 PRED C D}; do
    for v in prev new; do
      GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 300 python bench.py ${CFG[$c]} --warmup 1 $BQ > gpurun_out/$O/${v}_${c}_$r.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('gpurun_out/$O/${v}_${c}_$r.log').read().strip().splitlines()[-1]); p=d.get('predict') or {}; print('$v $c #$r', round(d['value'],1), 'evals/s', ('predict %.2f ms factor %.2f ms' % (p['ms'], p['factor_ms'])) if p else '')"
    done
  done
done
MODE=predict timeout -k 10 200 python scripts/crit_trace.py > gpurun_out/$O/crit_predict.txt 2>&1 || exit $?
MODE=eval timeout -k 10 200 python scripts/crit_trace.py > gpurun_out/$O/crit_B.txt 2>&1 || exit $?
tail -6 gpurun_out/$O/crit_predict.txt; cat gpurun_out/$O/crit_B.txt
