#!/bin/bash
# rocprofv3 kernel trace of a short bench run + per-block-column timeline (scripts/step_timeline.py)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tl}; mkdir -p $O
N=${N:-4096}; D=${D:-3}; P=${P:-64}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o tl --output-format csv -- python bench.py --n $N --d $D --swarm-per-gpu $P --steps 2 --warmup 1 --no-cpu --pso-steps 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python scripts/step_timeline.py $f $N
