#!/bin/bash
# Diagonal-factor variants: GPU suite on the default build, factor64/early-diagonal/configB tests on
# the one-Newton-step build, factor128 stamps, A/B at B and the prediction.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fac}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_nr1.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "factor64 or early_diagonal or configB or configC or headline or random or predict" > $O/pytest_nr1.log 2>&1
echo "nr1 pytest rc=$?"; tail -2 $O/pytest_nr1.log
CFGS="1024x32,4096x1" timeout -k 10 200 python scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids > $O/stamps.log; cat $O/stamps.log
TAG=${TAG:-fac}_ab VARIANTS="${VARIANTS:-pub f2 nr1 nolsync}" CFGS="${CFGS:-B PRED}" REPS=${REPS:-2} bash scripts/gpu_ab.sh
