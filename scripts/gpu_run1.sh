cd "$GRAFT_REPO_ROOT"
TAG=r2c VARIANTS="prev new" CFGS="C B" REPS=2 bash scripts/gpu_abx.sh || exit $?
TAG=r2c bash scripts/gpu_phase.sh || exit $?
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2c/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r2c/pytest_gpu.log; exit $rc
