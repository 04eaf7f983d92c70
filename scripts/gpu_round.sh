#!/bin/bash
# One GPU call: bitwise A/B vs a reference build (if present), GPU tests, diag stamps, benches C and B.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-round}; mkdir -p $O
if [ -f gaussian-process_amd/libgpfit_ref.so ]; then
  timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit_ref.so /tmp/gpf_ref.npz > $O/cmp.log 2>&1 || exit $?
  timeout -k 10 200 python scripts/compare_libs.py dump gaussian-process_amd/libgpfit.so /tmp/gpf_new.npz >> $O/cmp.log 2>&1 || exit $?
  python scripts/compare_libs.py diff /tmp/gpf_ref.npz /tmp/gpf_new.npz >> $O/cmp.log 2>&1; tail -1 $O/cmp.log
fi
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
if [ -f gaussian-process_amd/libgpfit_stamps.so ]; then
  timeout -k 10 200 python scripts/diag_stamps.py > $O/stamps.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/stamps.log
fi
ENV_LIST="GPF_GROUPS=1" CFGS="${CFGS:-C B}" ./scripts/gpu_env_ab.sh
