#!/bin/bash
# FETCH/WRITE per k_step launch and the bench clock under schedule knobs (VARIANTS: env specs
# like "GPF_STEP_GROUP=1,GPF_X=2" or "base"), config C, one box (round-4 traffic-vs-clock probe).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4t}; mkdir -p $O
B2="python bench.py --steps 2 --warmup 1 --pso-steps 0 --no-profile --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
for spec in $VARIANTS; do
  envs=""; [ "$spec" != base ] && envs=${spec//,/ }
  t=${spec//[^A-Za-z0-9_]/_}
  env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 2 --no-cpu --pso-steps 0 --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary > $O/$t.bench 2>&1 || exit 3
  env $envs timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/$t.f -o f --output-format csv -- $B2 > $O/$t.f.log 2>&1 || exit 5
  env $envs timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/$t.w -o w --output-format csv -- $B2 > $O/$t.w.log 2>&1 || exit 5
  python scripts/pmc_traffic.py $O/$t.f $O/$t.w $O/$t.traffic.json 4096 3 64 > /dev/null 2>&1
  python - "$O/$t.bench" "$O/$t.traffic.json" "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
t = json.load(open(sys.argv[2]))
print(sys.argv[3], round(d["value"], 1), "evals/s", round(r["achieved"], 2), "TF sclk", round(r.get("box_sclk_mhz") or 0),
      "per-clock", round(r.get("frac_of_box_ceiling") or 0, 3), "FETCHx2+WRITE GB/launch", round(t["bytes_per_launch"] / 1e9, 3))
PY
done
