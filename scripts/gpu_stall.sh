#!/bin/bash
# stall / cache counters for k_step (each pass its own run), plus a kernel-trace pass
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r1}
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 3
mkdir -p gpurun_out/$TAG
B="python bench.py --steps 2 --warmup 1 --no-cpu --pso-steps 0 --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$TAG/trace -o t --output-format csv -- $B > gpurun_out/$TAG/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -T -d gpurun_out/$TAG/sq -o s --output-format csv -- $B > gpurun_out/$TAG/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -T -d gpurun_out/$TAG/tcc -o c --output-format csv -- $B > gpurun_out/$TAG/tcc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d gpurun_out/$TAG/pmc_fetch -o f --output-format csv -- $B > gpurun_out/$TAG/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -d gpurun_out/$TAG/pmc_write -o w --output-format csv -- $B > gpurun_out/$TAG/pmc_write.log 2>&1 || exit $?
python scripts/pmc_traffic.py gpurun_out/$TAG/pmc_fetch gpurun_out/$TAG/pmc_write gpurun_out/$TAG/k_step_traffic.json 4096 3 64
cat gpurun_out/$TAG/trace/t_kernel_stats.csv
