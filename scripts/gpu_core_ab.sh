#!/bin/bash
# GEMM-core rate (gpf_gemm_bench) of library variants VARIANTS, same box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-coreab}; mkdir -p $O
for v in $VARIANTS; do
  GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 120 python scripts/gemm_core_one.py 2 4096 64 15 2048 > $O/core_$v.log 2>&1 || exit $?
  GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -k 10 120 python scripts/gemm_core_one.py 6 4096 64 15 2048 >> $O/core_$v.log 2>&1 || exit $?
  echo "$v: $(grep mode $O/core_$v.log | tr '\n' ' ')"
done
