#!/bin/bash
# PMC passes for the dominant kernel (separate runs: FETCH_SIZE / WRITE_SIZE / MFMA busy)
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r1}
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 3
mkdir -p gpurun_out/$TAG
B="python bench.py --steps 2 --warmup 1 --no-cpu --pso-steps 0 --no-profile --predict-points 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d gpurun_out/$TAG/pmc_fetch -o f --output-format csv -- $B > gpurun_out/$TAG/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -d gpurun_out/$TAG/pmc_write -o w --output-format csv -- $B > gpurun_out/$TAG/pmc_write.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -T -d gpurun_out/$TAG/pmc_mfma -o m --output-format csv -- $B > gpurun_out/$TAG/pmc_mfma.log 2>&1
echo "mfma pass rc=$?"
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -T -d gpurun_out/$TAG/pmc_l2 -o l --output-format csv -- $B > gpurun_out/$TAG/pmc_l2.log 2>&1
echo "l2 pass rc=$?"
python scripts/pmc_traffic.py gpurun_out/$TAG/pmc_fetch gpurun_out/$TAG/pmc_write gpurun_out/$TAG/k_step_traffic.json 4096 3 64
ls -R gpurun_out/$TAG | head -30
python scripts/pmc_counters.py gpurun_out/$TAG/k_step_counters.json "per k_step dispatch averages, N=4096 d=3 swarm 64 (rocprofv3 --pmc, separate passes)" gpurun_out/$TAG/pmc_mfma gpurun_out/$TAG/pmc_l2 gpurun_out/$TAG/pmc_fetch gpurun_out/$TAG/pmc_write
