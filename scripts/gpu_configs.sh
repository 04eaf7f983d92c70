#!/bin/bash
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r1}
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 3
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 20 --warmup 2 --cpu-sample 16 > gpurun_out/$TAG/bench_B.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/bench_B.log
timeout -k 10 400 python bench.py --n 16384 --d 4 --hetero --swarm-per-gpu 16 --steps 2 --warmup 1 --pso-steps 0 --no-cpu > gpurun_out/$TAG/bench_E.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/bench_E.log
