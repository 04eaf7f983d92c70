cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -k "all_tile_lookahead or configB or early_diagonal or not_pd_past_block3_on_timed_schedules" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
LIBS="libgpfit.so libgpfit.so:GPF_LA_ALL=1 libgpfit.so:GPF_LA_ALL=1,GPF_STEP_1PERCU=1" BENCH_ARGS="--n 1024 --d 2 --swarm-per-gpu 32 --seed 0" STEPS=200 TAG=r6j bash scripts/gpu_lib_ab.sh
