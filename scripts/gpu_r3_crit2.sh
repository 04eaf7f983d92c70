#!/bin/bash
# Deeper split of the critical tile under the all-tile split: split-K parity tests, the
# prediction's critical-tile timeline, the diagonal factor's per-panel stamps, then an A/B.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-crit2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "split or predict or early_diag or handoff or configB" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MODE=predict timeout -k 10 200 python scripts/crit_trace.py > $O/crit_pred.txt 2>&1 || exit $?
tail -12 $O/crit_pred.txt
CFGS=4096x1,1024x32 timeout -k 10 200 python scripts/diag_stamps.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt | grep -v amdgpu
[ -n "$VARIANTS" ] && bash scripts/gpu_ab.sh
exit 0
