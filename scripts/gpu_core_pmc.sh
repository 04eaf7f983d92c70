#!/bin/bash
# PMC passes on the GEMM core alone (k_gemm_bench), one counter group per pass
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/corepmc; mkdir -p $O
ARGS=${ARGS:-"2 4096 64 15 2048"}
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_LDS SQ_WAIT_ANY" "SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-trace -d $PWD/$O/p$i -o p --output-format csv -- python scripts/gemm_core_one.py $ARGS > $O/p$i.log 2>&1 || exit $?
done
python scripts/pmc_counters_k.py k_gemm_bench $O/p1 $O/p2 $O/p3 $O/p4 $O/p5
