#!/bin/bash
# A/B (prev vs new; bitwise check vs ref), diag stamps, kernel traces of config B and predict.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${TAG:-r2f}; mkdir -p gpurun_out/$O
TAG=$O VARIANTS="${VARIANTS:-prev new}" CFGS="${CFGS:-C B}" REPS=${REPS:-2} bash scripts/gpu_abx.sh || exit $?
timeout -k 10 200 python scripts/diag_stamps.py > gpurun_out/$O/diag_stamps.log 2>&1 || exit $?
tail -4 gpurun_out/$O/diag_stamps.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$O/profB -o b --output-format csv -- python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 3 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --psurf-rows 0 > gpurun_out/$O/profB.log 2>&1 || exit $?
f=$(find gpurun_out/$O/profB -name "*kernel_trace.csv" | head -1); python scripts/launch_list.py $f 24 > gpurun_out/$O/launches_B.txt; tail -14 gpurun_out/$O/launches_B.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$O/profP -o p --output-format csv -- python scripts/predict_probe.py > gpurun_out/$O/profP.log 2>&1 || exit $?
f=$(find gpurun_out/$O/profP -name "*kernel_trace.csv" | head -1); python scripts/launch_list.py $f 40 > gpurun_out/$O/launches_P.txt; tail -12 gpurun_out/$O/launches_P.txt
