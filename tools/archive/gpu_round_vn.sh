#!/bin/bash
# GPU round (tools/gpu_round.sh) followed by the virtual-node policy comparison at 8 GPUs
# (old planner default, backlog-carry planner, greedy, random; same arrivals, 48 epochs).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu_round.sh &&
timeout -k 10 900 python -u tools/virtual_node_bench.py --gpus 8 --epochs 48 --warmup 3 \
  --policies greedy corun_plan_t30_s05 corun_plan_t30_s05_c100 random \
  --out gpurun_out/vn8_carry.json > gpurun_out/vn8_carry.log 2>&1
rc=$?
tail -2 gpurun_out/vn8_carry.log | cut -c1-400
exit $rc
