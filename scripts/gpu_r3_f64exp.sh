#!/bin/bash
# factor64 bound experiment: diagonal-factor stamps with the update waves' work removed (stnoupd)
# and with the panel wave's factor removed (stnopan), against the real build (stamps).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-f64exp}; mkdir -p $O
for v in ${STLIBS:-stamps stnoupd stnopan}; do
  STAMPS_LIB=libgpfit_$v.so CFGS=128x1,4096x1 timeout -k 10 200 python scripts/diag_stamps.py > $O/$v.txt 2>&1 || exit $?
  echo "== $v"; grep -E "^N=" $O/$v.txt
done
[ -n "$VARIANTS" ] && bash scripts/gpu_ab.sh
exit 0
