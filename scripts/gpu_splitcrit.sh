#!/bin/bash
# Critical-tile split (GPF_SPLIT_CRIT): its GPU tests, then config B (and a mid-size case)
# with S = 1 (off) vs forced factors, interleaved on one box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-splitcrit}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "split" > $O/pytest_split.log 2>&1
rc=$?; tail -2 $O/pytest_split.log; [ $rc -ne 0 ] && exit $rc
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32 --steps 20 --warmup 2" [M]="--n 2048 --d 3 --swarm-per-gpu 32 --steps 10 --warmup 1" )
for r in 1 2; do
  for c in ${CFGS:-B M}; do
    for S in ${SS:-1 2 4 8}; do
      GPF_SPLIT_CRIT=$S timeout -k 10 200 python bench.py ${CFG[$c]} --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/${c}_S${S}_$r.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/${c}_S${S}_$r.log').read().strip().splitlines()[-1]); print('$c S=$S #$r', round(d['value'],1), 'evals/s', round(d['ms_per_step'],3), 'ms/step')"
    done
  done
done
if [ -n "$PRED" ]; then  # the all-tile split (single-particle prediction) on the same box
  for r in 1 2; do
    timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --pso-steps 0 --no-hull --psurf-rows 0 > $O/pred_$r.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/pred_$r.log').read().strip().splitlines()[-1]); p=d['predict']; print('predict #$r', round(p['ms'],2), 'ms (factor', round(p['factor_ms'],2), 'ms)  C', round(d['value'],1))"
  done
fi
