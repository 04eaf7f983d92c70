#!/bin/bash
# Groups A/B (GPF_GROUPS=1 vs the default) at C, 128 particles, N=2048 P=64; rocprof union check.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${TAG:-r2o}; mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$O/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/$O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
BQ="--no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 --warmup 1"
declare -A CFG=( [C]="--n 4096 --d 3 --swarm-per-gpu 64 --steps 6" [C128]="--n 4096 --d 3 --swarm-per-gpu 128 --steps 3"
                 [N2048P64]="--n 2048 --d 3 --swarm-per-gpu 64 --steps 10" )
for r in 1 2; do
  for c in C C128 N2048P64; do
    for g in 1 default; do
      if [ $g = 1 ]; then export GPF_GROUPS=1; else unset GPF_GROUPS; fi
      timeout -k 10 300 python bench.py ${CFG[$c]} $BQ > gpurun_out/$O/g${g}_${c}_$r.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('gpurun_out/$O/g${g}_${c}_$r.log').read().strip().splitlines()[-1]); r=d['roofline']; print('groups=$g $c #$r', round(d['value'],1), 'frac', round(r['frac'],3))"
    done
  done
done
unset GPF_GROUPS
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$O/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 $BQ > gpurun_out/$O/prof.log 2>&1 || exit $?
tail -1 gpurun_out/$O/prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench under rocprof:', round(d['value'],1), 'achieved', round(r['achieved'],2), r['timing'][:60])"
f=$(find gpurun_out/$O/prof -name "*kernel_trace.csv" | head -1); python scripts/kernel_union.py $f 4096 64 3
