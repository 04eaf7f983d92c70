#!/bin/bash
# factor64 update-wave passes: bitwise check against the previous build, stamps, A/B.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-f64}; mkdir -p $O
timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit_prev.so /tmp/gpf_a.npz > $O/cmp.log 2>&1 || exit $?
timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit_new.so /tmp/gpf_b.npz >> $O/cmp.log 2>&1 || exit $?
python scripts/compare_libs.py diff /tmp/gpf_a.npz /tmp/gpf_b.npz >> $O/cmp.log 2>&1; tail -3 $O/cmp.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "split or predict or early_diag or handoff or configB or factor64" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
CFGS=128x1,4096x1,1024x32 timeout -k 10 200 python scripts/diag_stamps.py > $O/stamps.txt 2>&1 || exit $?
grep -v amdgpu $O/stamps.txt
[ -n "$VARIANTS" ] && bash scripts/gpu_ab.sh
exit 0
