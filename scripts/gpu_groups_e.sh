#!/bin/bash
# GPU tests on the current build, particle groups on concurrent streams (GPF_GROUPS) at C and
# D's per-GPU share, and the config-E shape on one GPU.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ge}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for g in 1 2; do
    for cfg in "C:--n 4096 --d 3 --swarm-per-gpu 64" "D:--n 4096 --d 3 --swarm-per-gpu 32"; do
      n=${cfg%%:*}; a=${cfg#*:}
      GPF_GROUPS=$g timeout -k 10 300 python bench.py $a --steps 5 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/g${g}_${n}_$r.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/g${g}_${n}_$r.log').read().strip().splitlines()[-1]); print('groups $g $n #$r', round(d['value'],1), 'evals/s')"
    done
  done
done
timeout -k 10 400 python bench.py --n 16384 --d 4 --swarm-per-gpu 16 --hetero --steps 2 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/configE.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/configE.log').read().strip().splitlines()[-1]); print('E 1 GPU', round(d['value'],2), 'evals/s', round(d['roofline']['achieved'],1), 'TF')"
