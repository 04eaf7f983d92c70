#!/bin/bash
# Deep diagonal update (GPF_DEEP_SYRK): parity tests that cover the fused path, then an A/B of
# the knob on the slot-bound configs.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-deep}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "early_diagonal or reference or headline or split" > $O/unit.log 2>&1; rc=$?; tail -3 $O/unit.log; [ $rc = 0 ] || exit $rc
EXTRA="--predict-points 0 --no-hull --psurf-rows 0" ENV_LIST="GPF_DEEP_SYRK=0 GPF_DEEP_SYRK=1 GPF_DEEP_SYRK=0 GPF_DEEP_SYRK=1" CFGS="${CFGS:-C D E}" bash scripts/gpu_env_ab.sh
