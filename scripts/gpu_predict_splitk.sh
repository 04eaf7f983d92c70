#!/bin/bash
# A/B of the single-particle split-K factor (GPF_SPLIT_K) on the prediction's factorisation
# (bench predict.factor_ms at N=4096, d=3), interleaved, two rounds.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/predk
for r in 1 2; do for s in ${SLIST:-16 8 12 20}; do
  f=gpurun_out/predk/n${N:-4096}_s${s}_$r.log
  GPF_SPLIT_K=$s timeout -k 10 120 python bench.py --n ${N:-4096} --d 3 --swarm-per-gpu 8 --steps 1 --warmup 1 --no-cpu --pso-steps 0 --no-hull --psurf-rows 0 > $f 2>&1 || { tail -3 $f; exit 1; }
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); p=d['predict']; print('N=${N:-4096} GPF_SPLIT_K=$s', round(p['ms'],2), 'ms  factor', round(p['factor_ms'],3), 'ms')"
done; done
