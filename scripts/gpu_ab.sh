#!/bin/bash
# Interleaved A/B of library variants (VARIANTS, each gaussian-process_amd/libgpfit_<v>.so, or
# <v>@VAR=val[,VAR=val]: that library under those environment knobs) on configs CFGS, REPS
# rounds, one box (boxes of the pool differ by a few %).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
declare -A CFG=( [B]="--n 1024 --d 2 --swarm-per-gpu 32" [C]="--n 4096 --d 3 --swarm-per-gpu 64"
                 [D]="--n 4096 --d 3 --swarm-per-gpu 32" [E]="--n 16384 --d 4 --swarm-per-gpu 16 --hetero"
                 [P]="--n 4096 --d 3 --swarm-per-gpu 1" )
for r in $(seq ${REPS:-2}); do
  for c in ${CFGS:-C}; do
    for spec in $VARIANTS; do
      v=${spec%%@*}
      envs=""
      [ "$spec" != "$v" ] && envs=${spec#*@}
      envs=${envs//,/ }
      tag=${spec//[^A-Za-z0-9_]/_}_${c}_$r
      if [ "$c" = PRED ]; then  # the prediction line: GP at 10k query points, N=4096 (median of 3 calls)
        env $envs GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --pso-steps 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary > $O/$tag.log 2>&1 || exit $?
        python -c "import json; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])['predict']; print('$spec $c #$r', round(d['ms'],3), 'ms (profiled', round(d.get('ms_profiled_pass',0),3), ') factor', round(d['factor_ms'],3), 'ms  cross_cov', round(d['k_cross_cov_GBps']), 'GB/s  vsq', round(d['k_predict_vsq_ms'],3), 'ms', round(d['k_predict_vsq_tflops'],1), 'TF')"
        continue
      fi
      env $envs GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 300 python bench.py ${CFG[$c]} --steps ${STEPS:-8} --warmup 2 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary > $O/$tag.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$spec $c #$r', round(d['value'],1), 'evals/s  ', round(r['achieved'],2), 'TF', r['kernel'], 'sclk', r.get('box_sclk_mhz'), 'of ceiling', r.get('frac_of_box_ceiling'))"
    done
  done
done
