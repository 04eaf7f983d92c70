#!/bin/bash
# particle-group stream count A/B on configs C and B (same box, back to back)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/groups
for g in ${GROUPS_LIST:-1 2 4}; do
  for cfg in "--n 4096 --d 3 --swarm-per-gpu 64" "--n 1024 --d 2 --swarm-per-gpu 32"; do
    tag=g${g}_$(echo $cfg | awk '{print $2}')
    GPF_GROUPS=$g timeout -k 10 200 python bench.py $cfg --steps 5 --warmup 1 --no-cpu --pso-steps 0 > gpurun_out/groups/$tag.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/groups/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['value'],1), 'evals/s  step-avg', round(r['achieved'],1), 'TF  factor-wall', round(r['factor_phase_tflops'],1), 'TF')"
  done
done
