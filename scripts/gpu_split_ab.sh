#!/bin/bash
# Split L/U schedule (GPF_SPLIT) A/B on one build: bitwise check, then configs C and B, 2 rounds.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-split}; mkdir -p $O
GPF_SPLIT=0 timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit.so /tmp/s0.npz > $O/cmp.log 2>&1 || exit $?
GPF_SPLIT=1 timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit.so /tmp/s1.npz >> $O/cmp.log 2>&1 || exit $?
python scripts/compare_libs.py diff /tmp/s0.npz /tmp/s1.npz >> $O/cmp.log 2>&1; tail -1 $O/cmp.log
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32" [C]="--n 4096 --d 3 --swarm-per-gpu 64" [E]="--n 16384 --d 4 --swarm-per-gpu 16 --hetero" )
for r in 1 2; do
  for c in ${CFGS:-C B}; do
    for v in 0 1; do
      GPF_SPLIT=$v timeout -k 10 300 python bench.py ${CFG[$c]} --steps ${STEPS:-5} --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/s${v}_${c}_$r.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/s${v}_${c}_$r.log').read().strip().splitlines()[-1]); r=d['roofline']; print('split $v $c #$r', round(d['value'],1), 'evals/s  per-launch', round(r['achieved'],1), 'TF  factor-wall', round(r['factor_phase_tflops'],1), 'TF')"
    done
  done
done
