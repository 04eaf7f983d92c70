#!/bin/bash
# The GPU test suite (one process, per-test timeout) and, with BENCH=1, a short default bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-tests}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-60} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
  python - "$O/bench.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("C", round(d["value"], 1), d["unit"], "frac", round(r["frac"], 3), r["kernel"], "sclk", r.get("box_sclk_mhz"),
      "ceiling", r.get("box_fp64_ceiling_tflops"), "of ceiling", r.get("frac_of_box_ceiling"))
for c in d.get("configs") or []:
    print(c["config"], round(c["value"], 1), "evals/s frac", round(c["frac"], 3), "ms/step", round(c["ms_per_step"], 2))
p = d.get("predict") or {}
print("predict ms", round(p.get("ms", 0), 3), "profiled", round(p.get("ms_profiled_pass", 0), 3), "factor", round(p.get("factor_ms", 0), 3),
      "vsq", round(p.get("k_predict_vsq_ms", 0), 3), "other", round(p.get("other_ms_profiled", 0), 3))
PY
fi
