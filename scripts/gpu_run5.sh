#!/bin/bash
# GPU tests; env A/B of GPF_EARLY_DIAG=0/1 on configs C, D share, E share, N=2048 P=32, B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${TAG:-r2i}; mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$O/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
BQ="--no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0"
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32 --steps 30" [C]="--n 4096 --d 3 --swarm-per-gpu 64 --steps 6"
                 [D]="--n 4096 --d 3 --swarm-per-gpu 32 --steps 8" [N2048]="--n 2048 --d 3 --swarm-per-gpu 32 --steps 15"
                 [E]="--n 16384 --d 4 --swarm-per-gpu 16 --hetero --steps 2" )
for r in 1 2; do
  for c in ${CFGS:-C D N2048 B E}; do
    for ed in 0 1; do
      GPF_EARLY_DIAG=$ed timeout -k 10 300 python bench.py ${CFG[$c]} --warmup 1 $BQ > gpurun_out/$O/ed${ed}_${c}_$r.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('gpurun_out/$O/ed${ed}_${c}_$r.log').read().strip().splitlines()[-1]); print('ED=$ed $c #$r', round(d['value'],1), 'evals/s')"
    done
  done
done
