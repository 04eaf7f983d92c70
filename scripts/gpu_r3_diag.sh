#!/bin/bash
# GEMM core old vs new library; per-phase k_step trace of the new schedule at C and B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3diag}; mkdir -p $O
MODES=old GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_ref.so timeout -k 10 120 python scripts/gemm_core3.py > $O/core_old.txt 2>&1 || exit $?
timeout -k 10 120 python scripts/gemm_core3.py > $O/core_new.txt 2>&1 || exit $?
paste $O/core_old.txt $O/core_new.txt | cut -c1-200
timeout -k 10 120 python scripts/wg_phase3.py > $O/phase_C.txt 2>&1 || exit $?
N=1024 D=2 P=32 timeout -k 10 120 python scripts/wg_phase3.py > $O/phase_B.txt 2>&1 || exit $?
tail -3 $O/phase_C.txt; tail -3 $O/phase_B.txt
