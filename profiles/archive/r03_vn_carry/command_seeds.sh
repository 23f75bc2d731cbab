#!/bin/bash
# Virtual 8-GPU node on one MI355X, two more arrival seeds (48 epochs each): greedy, the planner
# without and with the backlog carry, random.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/virtual_node_bench.py --gpus 8 --epochs 48 --warmup 3 --seed 1 \
  --policies greedy corun_plan_t30_s05 corun_plan_t30_s05_c100 random \
  --out gpurun_out/vn8_seed1.json > gpurun_out/vn8_seed1.log 2>&1 &&
timeout -k 10 400 python -u tools/virtual_node_bench.py --gpus 8 --epochs 48 --warmup 3 --seed 2 \
  --policies greedy corun_plan_t30_s05 corun_plan_t30_s05_c100 random \
  --out gpurun_out/vn8_seed2.json > gpurun_out/vn8_seed2.log 2>&1
rc=$?
tail -1 gpurun_out/vn8_seed2.log | cut -c1-200
exit $rc
