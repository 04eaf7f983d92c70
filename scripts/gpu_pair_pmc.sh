#!/bin/bash
# r6: HBM traffic of the factorisation, paired vs unpaired block columns (one particle group, config C):
# FETCH_SIZE and WRITE_SIZE summed over every k_step launch of one factorisation (separate passes).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-pairpmc}; mkdir -p $O
B="python bench.py --steps 1 --warmup 0 --pso-steps 0 --no-cpu --no-profile --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
for m in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GPF_GROUPS=1 GPF_PAIR=$m timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $O/p$m$c -o x --output-format csv -- $B > $O/p$m$c.log 2>&1 || exit 5
  done
done
python - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for m in (0, 1):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{O}/p{m}{c}/**/*counter_collection.csv", recursive=True)[0]
        rows = [r for r in csv.DictReader(open(f)) if "k_step" in r["Kernel_Name"]]
        # the bench runs warm-up factorisations first: keep the last 32 launches (one factorisation)
        byd = collections.OrderedDict()
        for r in rows:
            byd.setdefault(r.get("Dispatch_Id") or r.get("Correlation_Id"), []).append(float(r["Counter_Value"]))
        vals = [sum(v) for v in byd.values()][-32:]
        tot[c] = sum(vals) * 1024 / 1e9 * (2 if c == "FETCH_SIZE" else 1)  # KB -> GB; gfx950 FETCH x2
        print(f"pair={m} {c}: {tot[c]:.2f} GB over {len(vals)} k_step launches; per launch:", " ".join(f"{v*1024/1e9*(2 if c=='FETCH_SIZE' else 1):.2f}" for v in vals))
PY
