#!/bin/bash
# r6: the look-ahead piece tests, then a same-box A/B of config B over piece sizes and orders.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r6lall}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -k "${PYTEST_K:-all_tile_lookahead or configB}" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
LIBS=${LIBS:-"libgpfit.so libgpfit.so:GPF_LA_ALL=1,GPF_LA_ALL_PB=1 libgpfit.so:GPF_LA_ALL=1,GPF_LA_ALL_PB=1,GPF_LA_ALL_FIRST=0 libgpfit.so:GPF_LA_ALL=1,GPF_LA_ALL_PB=2"} BENCH_ARGS="--n 1024 --d 2 --swarm-per-gpu 32 --seed 0" STEPS=200 TAG=$(basename $O) bash scripts/gpu_lib_ab.sh
