#!/bin/bash
# Whole GPU suite on the default build, then an optional A/B.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
[ -n "$VARIANTS" ] && bash scripts/gpu_ab.sh
exit 0
