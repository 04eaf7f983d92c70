#!/bin/bash
# Secondary-kernel parity (prob surface, cross covariance, prediction), their bench lines, then
# an A/B of the latency knobs (critical-tile priority, critical-tile split) on B and the prediction.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-sec2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "prob_surface or kernel_func or predict" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --pso-steps 0 --no-hull > $O/bench_sec.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench_sec.log').read().strip().splitlines()[-1]); p=d['predict']; s=d['prob_surface']; print('predict', round(p['ms'],3), 'factor', round(p['factor_ms'],3), 'cross_cov GB/s', round(p['k_cross_cov_GBps'])); print('psurf kernel ms', round(s['kernel_ms'],3), 'rows/s', round(s['rows_per_s_kernel']))"
[ -n "$VARIANTS" ] && bash scripts/gpu_ab.sh
exit 0
