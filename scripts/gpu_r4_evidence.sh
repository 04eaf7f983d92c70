#!/bin/bash
# Round-4 evidence, part 1 (PART=1): the whole GPU suite and the default bench line (config C plus
# the B / D-share / E-share secondary lines, prediction, CPU baselines). Part 2 (PART=2): rocprofv3
# kernel stats + trace of the config-C bench and the PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA
# busy) of its dominant kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4ev}; mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  grep -E "passed|failed|error" $O/pytest.log | tail -2
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
  timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
  python - "$O/bench.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("C", round(d["value"], 1), "frac", round(r["frac"], 3), r["kernel"], "sclk", r.get("box_sclk_mhz"), "of ceiling", r.get("frac_of_box_ceiling"))
for c in d.get("configs") or []:
    print(c["config"], round(c["value"], 1), "frac", round(c["frac"], 3), "of ceiling", c.get("frac_of_box_ceiling"))
p = d["predict"]
print("predict", round(p["ms"], 3), "factor", round(p["factor_ms"], 3), "vsq", round(p["k_predict_vsq_ms"], 3))
PY
else
  B="python bench.py --steps 3 --warmup 1 --pso-steps 0 --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- $B > $O/prof.log 2>&1 || exit 4
  f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
  python scripts/kernel_union.py $f 4096 64 3 > $O/kernel_union.txt 2>&1 || true
  python scripts/step_timeline.py $f 4096 > $O/timeline.txt 2>&1 || true
  B2="python bench.py --steps 2 --warmup 1 --pso-steps 0 --no-profile --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o f --output-format csv -- $B2 > $O/pmc_fetch.log 2>&1 || exit 5
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o w --output-format csv -- $B2 > $O/pmc_write.log 2>&1 || exit 5
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o m --output-format csv -- $B2 > $O/pmc_mfma.log 2>&1 || exit 5
  python scripts/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/k_step_traffic.json 4096 3 64
  python scripts/pmc_counters.py $O/k_step_counters.json "per k_step dispatch averages, N=4096 d=3 swarm 64 (rocprofv3 --pmc, separate passes)" $O/pmc_mfma $O/pmc_fetch $O/pmc_write
  cat $O/kernel_union.txt | tail -5
fi
