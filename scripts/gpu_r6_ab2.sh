cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -k "all_tile_lookahead or predict" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
GPF_VSQ_XCD=1 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "predict" > $O/pytest_vsqxcd.log 2>&1 || { tail -20 $O/pytest_vsqxcd.log; exit 5; }
tail -1 $O/pytest_vsqxcd.log
LIBS="libgpfit.so libgpfit.so:GPF_LA_ALL=1 libgpfit.so:GPF_LA_ALL=1,GPF_LA_ALL_FROM=-3" BENCH_ARGS="--n 1024 --d 2 --swarm-per-gpu 32 --seed 0" STEPS=200 TAG=r6o bash scripts/gpu_lib_ab.sh
LIBS="libgpfit.so libgpfit.so:GPF_VSQ_XCD=1" SEC=1 REPS=2 STEPS=20 TAG=r6o2 bash scripts/gpu_lib_ab.sh
