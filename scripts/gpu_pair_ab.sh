#!/bin/bash
# r6: paired block columns — the bitwise GPU test, then a same-box interleaved A/B of the config-C
# headline: unpaired (GPF_PAIR=0), paired without / with the partners' start sync.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-pair}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "${PYTEST_K:-paired_block}" > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
B="python bench.py --steps ${STEPS:-40} --warmup 2 --pso-steps 0 --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
for rep in 1 2; do
  for m in "0 1" "1 0" "1 1"; do
    set -- $m
    GPF_PAIR=$1 GPF_PAIR_SYNC=$2 timeout -k 10 300 $B > $O/bench_p$1s$2.$rep.json 2> $O/bench_p$1s$2.$rep.err || { tail -5 $O/bench_p$1s$2.$rep.err; exit 3; }
    python - $O/bench_p$1s$2.$rep.json "pair $1 sync $2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "C", round(d["value"], 1), "frac", round(r["frac"], 3), "sclk", round(r.get("box_sclk_mhz") or 0),
      "of ceiling", round(r.get("frac_of_box_ceiling") or 0, 3))
PY
  done
done
