cd "$GRAFT_REPO_ROOT"
for g in 1 2 1 2; do
  GPF_GROUPS=$g timeout -k 10 200 python bench.py --n 4096 --d 3 --swarm-per-gpu 32 --steps 5 --warmup 1 --no-cpu --pso-steps 0 --predict-points 0 --psurf-rows 0 --no-hull > /tmp/d.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('/tmp/d.log').read().strip().splitlines()[-1]); print('groups $g', round(d['value'],1))"
done
