#!/bin/bash
# Round-6 evidence: rocprofv3 kernel stats + trace of the config-C bench and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, MFMA busy) of its dominant kernel; then the same for the
# single-particle prediction (scripts/predict_probe.py: k_step<SPLIT_ALL, 1>, the flat finish).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6ev}; mkdir -p $O
B="python bench.py --steps 3 --warmup 1 --pso-steps 0 --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- $B > $O/prof.log 2>&1 || exit 4
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python scripts/kernel_union.py $f 4096 64 3 > $O/kernel_union.txt 2>&1 || true
B2="python bench.py --steps 2 --warmup 1 --pso-steps 0 --no-profile --no-cpu --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o f --output-format csv -- $B2 > $O/pmc_fetch.log 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o w --output-format csv -- $B2 > $O/pmc_write.log 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o m --output-format csv -- $B2 > $O/pmc_mfma.log 2>&1 || exit 5
python scripts/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/k_step_traffic.json 4096 3 64
python scripts/pmc_counters.py $O/k_step_counters.json "per k_step dispatch averages, N=4096 d=3 swarm 64 (rocprofv3 --pmc, separate passes)" $O/pmc_mfma $O/pmc_fetch $O/pmc_write
# the prediction (3 calls of GP at 10k points, N=4096)
P="python scripts/predict_probe.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pprof -o pred --output-format csv -- $P > $O/pprof.log 2>&1 || exit 6
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/ppmc_fetch -o f --output-format csv -- $P > $O/ppmc_fetch.log 2>&1 || exit 7
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/ppmc_write -o w --output-format csv -- $P > $O/ppmc_write.log 2>&1 || exit 7
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/ppmc_mfma -o m --output-format csv -- $P > $O/ppmc_mfma.log 2>&1 || exit 7
KNAME=k_step python scripts/pmc_counters.py $O/predict_k_step_counters.json "per k_step<SPLIT_ALL,1> dispatch averages, prediction N=4096 d=3 (3 factorisations x 32 launches; rocprofv3 --pmc, separate passes)" $O/ppmc_mfma $O/ppmc_fetch $O/ppmc_write
tail -3 $O/kernel_union.txt
