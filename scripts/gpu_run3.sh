#!/bin/bash
# Critical-tile timelines (trace build): predict at N=4096 and config B.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r2g}; mkdir -p $O
MODE=predict timeout -k 10 200 python scripts/crit_trace.py > $O/crit_predict.txt 2>&1 || exit $?
MODE=eval timeout -k 10 200 python scripts/crit_trace.py > $O/crit_B.txt 2>&1 || exit $?
cat $O/crit_predict.txt | tail -34; cat $O/crit_B.txt
