#!/bin/bash
# Per-launch spans of one factorisation (rocprofv3 kernel trace + scripts/launch_spans.py) for each
# variant in VARIANTS ("name:VAR=VAL,VAR2=VAL ..."), bench arguments in BENCH_ARGS.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-spans}; mkdir -p $O
B="python bench.py --steps 2 --warmup 1 --pso-steps 0 --no-cpu --no-profile --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary ${BENCH_ARGS:-}"
for V in ${VARIANTS:-base}; do
  n=${V%%:*}; E=""; [ "$V" != "$n" ] && E=$(echo ${V#*:} | tr ',' ' ')
  ( [ -n "$E" ] && export $E; timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$n -o t --output-format csv -- $B > $O/tr_$n.log 2>&1 ) || exit 4
  python scripts/launch_spans.py $(find $O/tr_$n -name "*kernel_trace.csv" | head -1) > $O/spans_$n.txt
  echo "$n: $(tail -1 $O/spans_$n.txt)"
done
