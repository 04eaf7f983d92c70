#!/bin/bash
# PMC passes for the secondary kernels (probability surface: FP64 VALU flops and busy; cross
# covariance / V = U K_s: HBM bytes) on the bench's secondary lines only.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sec}; mkdir -p $O
B="python bench.py --steps 1 --warmup 1 --no-cpu --pso-steps 0 --no-hull --no-profile"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o v --output-format csv -- $B > $O/pmc_valu.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o w --output-format csv -- $B > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o f --output-format csv -- $B > $O/pmc_fetch.log 2>&1 || exit $?
python scripts/pmc_secondary.py $O/secondary_pmc.json $O/pmc_valu $O/pmc_write $O/pmc_fetch
