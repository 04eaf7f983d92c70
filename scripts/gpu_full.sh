#!/bin/bash
# Round evidence: GPU tests, default bench (CPU baseline + prediction line), torchrun world-1
# sanity of the RCCL path, config B/D-per-GPU lines, rocprofv3 kernel stats of the bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-full}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || exit 3
timeout -k 10 500 python -m pytest tests -q -m gpu -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu --pso-steps 2 --predict-points 0 > $O/bench_torchrun1.log 2>&1 || exit $?
tail -1 $O/bench_torchrun1.log | cut -c1-200
timeout -k 10 200 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 20 --warmup 2 --no-cpu --predict-points 0 > $O/bench_configB.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --n 4096 --d 3 --swarm-per-gpu 32 --steps 5 --warmup 1 --no-cpu --predict-points 0 > $O/bench_configD_pergpu.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python scripts/step_timeline.py $f 4096 > $O/timeline.txt; tail -1 $O/timeline.txt
if [ -f gaussian-process_amd/libgpfit_trace.so ]; then
  timeout -k 10 200 python scripts/wg_trace.py > $O/wg_trace.txt 2>&1 || exit $?
  tail -1 $O/wg_trace.txt
fi
