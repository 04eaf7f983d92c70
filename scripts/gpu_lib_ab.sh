#!/bin/bash
# Same-box interleaved A/B of library variants (scripts/build_variant.sh): the config-C bench line
# (and, with SEC=1, B / D-share / E-share and the prediction), then one FETCH_SIZE pass per variant
# over one factorisation (PMC=1). LIBS: space-separated library file names under gaussian-process_amd/.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-libab}; mkdir -p $O
LIBS=${LIBS:-"libgpfit.so"}
if [ "${SEC:-0}" = 1 ]; then EXTRA="--pso-steps 0 --no-cpu --predict-points 10000 --no-hull --no-kmeans --psurf-rows 0";
else EXTRA="--pso-steps 0 --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"; fi
B="python bench.py --steps ${STEPS:-40} --warmup 2 $EXTRA ${BENCH_ARGS:-}"
for rep in $(seq ${REPS:-2}); do
  for V in $LIBS; do
    L=${V%%:*}; E=""; [ "$V" != "$L" ] && E=$(echo ${V#*:} | tr ',' ' ')
    L_=$(echo $V | tr ':,=' '___')
    env $E GPFIT_LIB=$PWD/gaussian-process_amd/$L timeout -k 10 400 $B > $O/bench_$L_.$rep.json 2> $O/bench_$L_.$rep.err || { tail -5 $O/bench_$L_.$rep.err; exit 3; }
    python - $O/bench_$L_.$rep.json $V <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
line = f"{sys.argv[2]:34s} C {d['value']:.1f} frac {r['frac']:.3f} sclk {round(r.get('box_sclk_mhz') or 0)} of-ceiling {r.get('frac_of_box_ceiling') or 0:.3f}"
for c in d.get("configs") or []:
    line += f" | {c['config']} {c['value']:.1f}"
p = d.get("predict") or {}
if p: line += f" | predict {p.get('ms', 0):.3f} ms factor {p.get('factor_ms', 0):.3f} vsq {p.get('k_predict_vsq_ms', 0):.3f}"
print(line)
PY
  done
done
if [ "${PMC:-0}" = 1 ]; then
  B1="python bench.py --steps 1 --warmup 0 --pso-steps 0 --no-cpu --no-profile --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
  for V in $LIBS; do
    L=${V%%:*}; E=""; [ "$V" != "$L" ] && E=$(echo ${V#*:} | tr ',' ' ')
    L_=$(echo $V | tr ':,=' '___')
    [ -n "$E" ] && export $E
    GPFIT_LIB=$PWD/gaussian-process_amd/$L timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f_$L_ -o x --output-format csv -- $B1 > $O/f_$L_.log 2>&1 || exit 5
    [ -n "$E" ] && unset $(echo $E | sed 's/=[^ ]*//g')
    python - $O/f_$L_ $V <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_step" in r["Kernel_Name"]]
byd = {}
for r in rows:
    byd.setdefault(r.get("Dispatch_Id") or r.get("Correlation_Id"), []).append(float(r["Counter_Value"]))
vals = [sum(v) * 1024 * 2 / 1e9 for v in byd.values()][-64:]  # one factorisation: 2 groups x 32 launches
print(f"{sys.argv[2]:34s} FETCH_SIZE x2 over the last {len(vals)} k_step launches: {sum(vals):.1f} GB ({sum(vals)/len(vals):.2f} GB per launch)")
PY
  done
fi
