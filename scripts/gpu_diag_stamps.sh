#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stamps
timeout -k 10 300 python scripts/diag_stamps.py > gpurun_out/stamps/stamps.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/stamps/stamps.log; exit $rc
