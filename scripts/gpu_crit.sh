#!/bin/bash
# Critical-tile timelines (trace build) of config B and the prediction under ENV_LIST settings.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-crit}; mkdir -p $O
for e in ${ENV_LIST:-GPF_NONE=0}; do
  tag=${e//[^A-Za-z0-9]/_}
  env $e MODE=eval timeout -k 10 200 python scripts/crit_trace.py > $O/crit_B_$tag.txt 2>&1 || exit $?
  env $e MODE=predict timeout -k 10 200 python scripts/crit_trace.py > $O/crit_pred_$tag.txt 2>&1 || exit $?
  echo "== $e"; grep -v amdgpu.ids $O/crit_B_$tag.txt; tail -4 $O/crit_pred_$tag.txt
done
