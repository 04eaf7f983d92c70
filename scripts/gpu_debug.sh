#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
timeout -k 10 300 python scripts/debug_factor.py > gpurun_out/dbg/debug.log 2>&1
rc=$?; cat gpurun_out/dbg/debug.log | tail -60; exit $rc
