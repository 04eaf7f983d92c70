#!/bin/bash
# Interleaved A/B of environment settings (ENVS, ';'-separated, e.g. "GPF_PERSIST=0;GPF_FLOW=1")
# on configs CFGS, REPS rounds; one bitwise dump per setting against the first.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-envx}; mkdir -p $O
IFS=';' read -ra EL <<< "$ENVS"
i=0
for e in "${EL[@]}"; do
  env $e timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit.so /tmp/gpf_$i.npz > $O/cmp_$i.log 2>&1 || exit $?
  [ $i -gt 0 ] && { python scripts/compare_libs.py diff /tmp/gpf_0.npz /tmp/gpf_$i.npz > $O/diff_$i.log 2>&1; echo "[$e] $(tail -1 $O/diff_$i.log)"; }
  i=$((i+1))
done
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32" [C]="--n 4096 --d 3 --swarm-per-gpu 64"
                 [D]="--n 4096 --d 3 --swarm-per-gpu 32" [E]="--n 16384 --d 4 --swarm-per-gpu 16 --hetero" )
for r in $(seq ${REPS:-1}); do
  for c in ${CFGS:-C}; do
    i=0
    for e in "${EL[@]}"; do
      tag=e${i}_${c}_$r
      env $e timeout -k 10 300 python bench.py ${CFG[$c]} --steps ${STEPS:-5} --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/$tag.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('[$e] $c #$r', round(d['value'],1), 'evals/s  k', round(r['achieved'],1), 'TF')"
      i=$((i+1))
    done
  done
done
