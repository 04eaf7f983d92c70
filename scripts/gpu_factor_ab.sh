#!/bin/bash
# Diagonal-factor A/B: unit tests, then B/C throughput of libgpfit_prev vs libgpfit_new, then
# the B bench with prediction for both.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r2fab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "factor64 or early_diag" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/unit.log 2>&1; rc=$?; tail -3 $O/unit.log; [ $rc = 0 ] || exit $rc
TAG=${TAG:-r2fab} VARIANTS="prev new" CFGS="${CFGS:-B C}" REPS=2 NOPHASE=1 NOTEST=1 bash scripts/gpu_run1.sh || exit $?
for v in prev new; do
  GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 300 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 5 --warmup 1 --no-cpu > $O/pred_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/pred_$v.log').read().strip().splitlines()[-1]); print('$v', {k: d[k] for k in d if 'predict' in k or k=='value'}, d.get('phases', {}).get('predict', ''))"
done
STAMPS_LIB=libgpfit_stamps.so timeout -k 10 300 python scripts/diag_stamps.py > $O/stamps.log 2>&1 || exit $?; grep -v amdgpu.ids $O/stamps.log | head -3
