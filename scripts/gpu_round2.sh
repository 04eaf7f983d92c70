#!/bin/bash
# bitwise A/B vs libgpfit_ref.so, GPU tests, then back-to-back bench of VARIANTS (libgpfit_<v>.so)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-round2}; mkdir -p $O
timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit_ref.so /tmp/gpf_ref.npz > $O/cmp.log 2>&1 || exit $?
timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit.so /tmp/gpf_new.npz >> $O/cmp.log 2>&1 || exit $?
python scripts/compare_libs.py diff /tmp/gpf_ref.npz /tmp/gpf_new.npz >> $O/cmp.log 2>&1; tail -1 $O/cmp.log
timeout -k 10 500 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in $VARIANTS; do
  for c in "--n 4096 --d 3 --swarm-per-gpu 64" "--n 1024 --d 2 --swarm-per-gpu 32"; do
    GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 200 python bench.py $c --steps 5 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --psurf-rows 0 > $O/b.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('$v', d['config']['N'], round(d['value'],1), 'evals/s', round(d['roofline']['achieved'],1), 'TF')"
  done
done
for v in $VARIANTS; do
  GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 200 python bench.py --n 4096 --d 3 --swarm-per-gpu 32 --steps 5 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --psurf-rows 0 --no-hull > $O/b.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('$v', d['config']['N'], 'P32', round(d['value'],1), 'evals/s', round(d['roofline']['achieved'],1), 'TF')"
done
