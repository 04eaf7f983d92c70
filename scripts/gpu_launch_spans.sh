cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r6d; mkdir -p $O
B="python bench.py --steps 2 --warmup 1 --pso-steps 0 --no-cpu --no-profile --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
for m in 0 1; do
  GPF_GROUPS=1 GPF_PAIR=$m timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr$m -o t --output-format csv -- $B > $O/tr$m.log 2>&1 || exit 4
  python scripts/launch_spans.py $(find $O/tr$m -name "*kernel_trace.csv" | head -1) > $O/spans$m.txt
  tail -1 $O/spans$m.txt
done
