#!/bin/bash
# Bench spread over workload-draw seeds at the driver's shape (20 steps) and one 300-step run
# (sustained rate + amd-smi activity over a long window).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/seeds
for s in 0 1 2 3 4; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --seed $s > gpurun_out/seeds/s$s.log 2>&1 || exit $?
  echo "seed=$s $(grep '^{' gpurun_out/seeds/s$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline_floor_ms_per_step"], d["sol_pct"], d["smi"]["gfx_activity_pct_mean"])')"
done
timeout -k 10 300 python bench.py --steps 300 --warmup 5 > gpurun_out/seeds/long300.log 2>&1 || exit $?
echo "steps=300 $(grep '^{' gpurun_out/seeds/long300.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline_floor_ms_per_step"], d["sol_pct"], d["gpu_util_pct"], d["smi"])')"
