#!/bin/bash
# Round evidence: forced build, default bench (config C + CPU baselines + secondary lines),
# configs B / D-share / E-share, torchrun world 1, rocprofv3 kernel stats + timeline of the
# config-C bench, PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) for the HBM traffic of k_step.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ev}; mkdir -p $O
GPF_FORCE_BUILD=1 timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || exit 3
tail -1 $O/build.log
timeout -k 10 600 python bench.py > $O/bench_C.log 2>&1 || exit $?
tail -1 $O/bench_C.log | cut -c1-300
BQ="--no-cpu --predict-points 0 --no-hull --psurf-rows 0"
timeout -k 10 300 python bench.py --n 1024 --d 2 --swarm-per-gpu 32 --steps 40 --warmup 4 $BQ > $O/bench_B.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --n 4096 --d 3 --swarm-per-gpu 32 --steps 10 --warmup 2 $BQ > $O/bench_D_share.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --n 16384 --d 4 --hetero --swarm-per-gpu 16 --steps 3 --warmup 1 --pso-steps 0 $BQ > $O/bench_E_share.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 1 $BQ > $O/bench_torchrun1.log 2>&1 || exit $?
for f in B D_share E_share torchrun1; do python -c "import json,sys; d=json.loads(open('$O/bench_$f.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(d['value'],1), d['unit'], 'frac', round(r['frac'],3), r['timing'][:40])"; done
B="python bench.py --steps 3 --warmup 1 --pso-steps 0 $BQ"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- $B > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python scripts/step_timeline.py $f 4096 > $O/timeline.txt
python scripts/kernel_union.py $f 4096 64 3 | tee $O/kernel_union.txt
tail -1 $O/prof.log | cut -c1-120 > /dev/null
B2="python bench.py --steps 2 --warmup 1 --pso-steps 0 --no-profile $BQ"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o f --output-format csv -- $B2 > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o w --output-format csv -- $B2 > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o m --output-format csv -- $B2 > $O/pmc_mfma.log 2>&1 || exit $?
python scripts/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/k_step_traffic.json 4096 3 64
python scripts/pmc_counters.py $O/k_step_counters.json "per k_step dispatch averages, N=4096 d=3 swarm 64 (rocprofv3 --pmc, separate passes)" $O/pmc_mfma $O/pmc_fetch $O/pmc_write
TAG=${TAG:-ev}_sec bash scripts/gpu_secondary.sh
