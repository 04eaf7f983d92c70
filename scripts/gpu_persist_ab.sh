#!/bin/bash
# Persistent factorisation: its GPU tests, then an interleaved A/B against the per-block-column
# launches (GPF_PERSIST=0) on configs C, D's and E's shares.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-pab}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "${PYTEST_K:-persistent or configC or configD or configE}" > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
Q="--no-cpu --pso-steps 0 --predict-points 0 --no-hull --no-kmeans --psurf-rows 0 --no-secondary"
for r in 1 2; do
  for v in 1 0; do
    GPF_PERSIST=$v timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 2 $Q > $O/C_${v}_${r}.log 2>&1 || exit 4
    python -c "import json; d=json.loads(open('$O/C_${v}_${r}.log').read().strip().splitlines()[-1]); r=d['roofline']; print('C persist=$v #$r', round(d['value'],1), 'evals/s', round(r['achieved'],2), 'TF', r['kernel'], round(r['avg_launch_ms'],3), 'ms/launch sclk', r.get('box_sclk_mhz'), 'ceil', r.get('box_fp64_ceiling_tflops'))"
    GPF_PERSIST=$v timeout -k 10 300 python bench.py --steps 20 --warmup 2 --swarm-per-gpu 32 $Q > $O/D_${v}_${r}.log 2>&1 || exit 4
    python -c "import json; d=json.loads(open('$O/D_${v}_${r}.log').read().strip().splitlines()[-1]); r=d['roofline']; print('D persist=$v #$r', round(d['value'],1), 'evals/s', round(r['achieved'],2), 'TF')"
  done
done
for v in 1 0; do
  GPF_PERSIST=$v timeout -k 10 300 python bench.py --n 16384 --d 4 --hetero --swarm-per-gpu 16 --steps 3 --warmup 1 $Q > $O/E_$v.log 2>&1 || exit 4
  python -c "import json; d=json.loads(open('$O/E_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('E persist=$v', round(d['value'],2), 'evals/s', round(r['achieved'],2), 'TF')"
done
