#!/bin/bash
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r1}
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 3
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/$TAG/pytest_gpu.log; tail -4 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$TAG/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --pso-steps 0 > gpurun_out/$TAG/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/$TAG/prof -name "*stats*" | head
exit $rc
