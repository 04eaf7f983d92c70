#!/bin/bash
# (1) bounds-checked build on the tests that cover the early-diagonal / split paths (the r2
# early-publish fault configuration), (2) the GPU parity suite on the default library,
# (3) interleaved A/B of variants on C and B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-combo}; mkdir -p $O
GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_check.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "split or early_diagonal or handoff or configB" > $O/pytest_check.log 2>&1
rc=$?; echo "check-build pytest rc=$rc"; tail -2 $O/pytest_check.log; grep -c "k_step check" $O/pytest_check.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
TAG=${TAG:-combo}_ab VARIANTS="${VARIANTS:-base pub wprio ob2}" CFGS="${CFGS:-C B}" REPS=${REPS:-2} bash scripts/gpu_ab.sh
