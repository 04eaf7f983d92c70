#!/bin/bash
# factor128 phase stamps (diagnostic build) at config B's last launch and the prediction's; the
# default bench (secondary lines included, no CPU baseline).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stamps}; mkdir -p $O
CFGS="1024x32,4096x1" timeout -k 10 200 python scripts/diag_stamps.py > $O/stamps.log 2>&1 || exit $?
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['predict'])[:600]); print(json.dumps(d['prob_surface'])[:400])"
