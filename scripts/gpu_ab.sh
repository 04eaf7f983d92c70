#!/bin/bash
# A/B of library variants on the headline bench (same box, back to back)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for v in $VARIANTS; do
  GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --pso-steps 0 > gpurun_out/ab/$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value'],1), 'evals/s', round(d['roofline']['achieved'],1), 'TF')"
done
