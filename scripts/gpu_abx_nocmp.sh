#!/bin/bash
# Bitwise check of libgpfit.so against libgpfit_ref.so, then an interleaved A/B of library
# variants (VARIANTS, each gaussian-process_amd/libgpfit_<v>.so) on configs CFGS, REPS times.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-abx}; mkdir -p $O
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32" [C]="--n 4096 --d 3 --swarm-per-gpu 64"
                 [D]="--n 4096 --d 3 --swarm-per-gpu 32" [E]="--n 16384 --d 4 --swarm-per-gpu 16 --hetero" )
for r in $(seq ${REPS:-2}); do
  for c in ${CFGS:-C}; do
    for v in $VARIANTS; do
      tag=${v}_${c}_$r
      GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 300 python bench.py ${CFG[$c]} --steps ${STEPS:-5} --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/$tag.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$v $c #$r', round(d['value'],1), 'evals/s  step', round(r['achieved'],1), 'TF')"
    done
  done
done
if [ -n "$TIMELINE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > $O/prof.log 2>&1 || exit $?
  f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python scripts/step_timeline.py $f 4096 > $O/timeline.txt; head -12 $O/timeline.txt; tail -1 $O/timeline.txt
fi
