#!/bin/bash
# Round-2 evidence run: build on the box (forced: proves the .so compiles from this tree), GPU
# tests, default bench, rocprofv3 kernel stats of the bench's timed region. TAG names the
# output directory; STEPS lists what to run (default: all).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2}; mkdir -p $O
STEPS=${STEPS:-"build probe test bench prof"}
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has build; then
  GPF_FORCE_BUILD=1 timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || exit 3
  tail -1 $O/build.log
fi
if has probe; then
  { echo "nproc=$(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null;
    python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))";
    free -g | head -2; } > $O/host_probe.txt 2>&1
  cat $O/host_probe.txt
fi
if has test; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
if has bench; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1 || exit $?
  tail -1 $O/bench.log | cut -c1-400
fi
if has prof; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --psurf-rows 0 --no-hull > $O/prof.log 2>&1 || exit $?
  find $O/prof -name "*stats*"
fi
exit 0
