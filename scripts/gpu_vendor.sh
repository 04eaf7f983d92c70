#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vendor
timeout -k 10 300 python scripts/vendor_ref.py > gpurun_out/vendor/vendor.log 2>&1; rc=$?
cat gpurun_out/vendor/vendor.log | grep -v amdgpu.ids; exit $rc
