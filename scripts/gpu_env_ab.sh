#!/bin/bash
# A/B of environment knobs on bench configs (same box, back to back).
#   ENV_LIST="GPF_STEP_GROUP=0 GPF_STEP_GROUP=1"  CFGS="C B"
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/envab
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32" [C]="--n 4096 --d 3 --swarm-per-gpu 64"
                 [D]="--n 4096 --d 3 --swarm-per-gpu 32" [E]="--n 16384 --d 4 --swarm-per-gpu 16 --hetero"
                 [F]="--n 2048 --d 3 --swarm-per-gpu 32" [G]="--n 1536 --d 2 --swarm-per-gpu 32" [H]="--n 3072 --d 3 --swarm-per-gpu 16" )
for e in $ENV_LIST; do
  for c in ${CFGS:-C}; do
    tag=${e//[^A-Za-z0-9]/_}_${c}_$RANDOM
    env $e timeout -k 10 300 python bench.py ${CFG[$c]} --steps ${STEPS:-5} --warmup 1 --no-cpu --pso-steps 0 ${EXTRA} > gpurun_out/envab/$tag.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/envab/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$e $c', round(d['value'],1), 'evals/s  step', round(r['achieved'],1), 'TF  factor-wall', round(r['factor_phase_tflops'],1), 'TF  predict factor', round((d.get('predict') or {}).get('factor_ms',0),2), 'ms')"
  done
done
