#!/bin/bash
# Does per-launch HIP-event profiling cost throughput? bench at B and C with and without it.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-profab}; mkdir -p $O
for r in 1 2; do
  for c in "B:--n 1024 --d 2 --swarm-per-gpu 32" "C:--n 4096 --d 3 --swarm-per-gpu 64"; do
    n=${c%%:*}; a=${c#*:}
    for f in "" "--no-profile"; do
      timeout -k 10 300 python bench.py $a --steps ${STEPS:-20} --warmup 2 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 $f > $O/${n}_${r}${f}.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/${n}_${r}${f}.log').read().strip().splitlines()[-1]); print('$n #$r ${f:-profile}', round(d['value'],1), 'evals/s', round(d['ms_per_step'],4), 'ms')"
    done
  done
done
