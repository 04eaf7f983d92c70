#!/bin/bash
# A/B of libgpfit_prev vs libgpfit_new (configs C, B), phase trace of the trace build, GPU tests.
cd "$GRAFT_REPO_ROOT"
O=${TAG:-r2ab}
TAG=$O VARIANTS="${VARIANTS:-prev new}" CFGS="${CFGS:-C B}" REPS=${REPS:-2} bash scripts/gpu_abx.sh || exit $?
if [ -z "$NOPHASE" ]; then TAG=$O bash scripts/gpu_phase.sh || exit $?; fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$O/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/$O/pytest_gpu.log; exit $rc
fi
