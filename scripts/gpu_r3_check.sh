#!/bin/bash
# Round-3 check on the box: GPU parity suite, default bench (config C), config B, the prediction.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3chk}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
BQ="--no-cpu --predict-points 0 --no-hull --psurf-rows 0"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench_C.log 2>&1 || exit $?
tail -1 $O/bench_C.log | cut -c1-300
timeout -k 10 300 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 40 --warmup 4 $BQ > $O/bench_B.log 2>&1 || exit $?
tail -1 $O/bench_B.log | cut -c1-200
