#!/bin/bash
# Round-4 A/B: selected GPU tests, then library variants x environment knobs on configs (gpu_ab.sh).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4ab}; mkdir -p $O
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "$PYTEST_K" > $O/pytest.log 2>&1
  rc=$?
  grep -E "passed|failed|error" $O/pytest.log | tail -3
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
fi
TAG=${TAG:-r4ab}/ab bash scripts/gpu_ab.sh
