#!/bin/bash
# round-1 first GPU pass: parity tests, short bench, kernel-trace profile
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench1.log
exit $rc
