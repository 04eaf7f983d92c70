#!/bin/bash
# Round-6: the whole GPU suite (one process, per-test timeout), then the default bench line
# (python bench.py: 200 timed steps, every secondary line, the CPU baseline).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6suite}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("C", round(d["value"], 1), d["unit"], "frac", round(r["frac"], 3), "sclk", r.get("box_sclk_mhz"), "of ceiling", r.get("frac_of_box_ceiling"))
for c in d.get("configs") or []:
    print(c["config"], round(c["value"], 1), "frac", round(c["frac"], 3))
p = d.get("predict") or {}
print("predict ms", p.get("ms"), "factor", p.get("factor_ms"), "vsq", p.get("k_predict_vsq_ms"))
print("cpu", d.get("cpu_baseline"))
PY
