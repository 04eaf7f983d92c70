#!/bin/bash
# Which SQ counters this gfx950 exposes, then stall-type counters on the GEMM core (k_gemm_bench).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/corestall; mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/sq_counters.txt; wc -l $O/sq_counters.txt
ARGS=${ARGS:-"2 4096 64 15 2048"}
i=0
for grp in "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INST_CYCLES_VMEM" "SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $PWD/$O/p$i -o p --output-format csv -- python scripts/gemm_core_one.py $ARGS > $O/p$i.log 2>&1 || echo "pass $i ($grp) failed: $(tail -1 $O/p$i.log)"
done
python scripts/pmc_counters_k.py k_gemm_bench $O/p1 $O/p2 $O/p3 $O/p4 $O/p5 $O/p6
