#!/bin/bash
# Split-K check: GPU tests, then the prediction line and config B with GPF_SPLIT_K=1 (off) vs default.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-splitk}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for k in 1 0; do
    if [ $k = 1 ]; then E="GPF_SPLIT_K=1"; else E="GPF_SPLIT_K_DEFAULT=1"; fi
    env $E timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --pso-steps 0 --no-hull --psurf-rows 0 > $O/pred_k${k}_$r.log 2>&1 || exit $?
    env $E timeout -k 10 300 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 10 --warmup 2 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/B_k${k}_$r.log 2>&1 || exit $?
    python -c "
import json
d=json.loads(open('$O/pred_k${k}_$r.log').read().strip().splitlines()[-1]); p=d['predict']
b=json.loads(open('$O/B_k${k}_$r.log').read().strip().splitlines()[-1])
print('$E #$r predict', round(p['ms'],2), 'ms (factor', round(p['factor_ms'],2), 'ms)  C', round(d['value'],1), ' B', round(b['value'],1))"
  done
done
