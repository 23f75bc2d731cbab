#!/bin/bash
# Virtual-node placement A/B on one MI355X: 8, 4 and 2 virtual GPUs, 48 epochs each, policies
# interleaved per epoch on the same arrivals.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u tools/virtual_node_bench.py --gpus 8 --epochs 48 --warmup 3 \
  --policies greedy corun_plan_t30_s05 corun_plan_t30_s05_c100 corun_plan_t30_s05_c100_nofb \
  --out gpurun_out/vn8_fb.json > gpurun_out/vn8_fb.log 2>&1 &&
timeout -k 10 300 python -u tools/virtual_node_bench.py --gpus 4 --epochs 48 --warmup 3 \
  --policies greedy corun_plan_t30_s05 corun_plan_t30_s05_c100 random \
  --out gpurun_out/vn4_fb.json > gpurun_out/vn4_fb.log 2>&1 &&
timeout -k 10 300 python -u tools/virtual_node_bench.py --gpus 2 --epochs 48 --warmup 3 \
  --policies greedy corun_plan_t30_s05 corun_plan_t30_s05_c100 random \
  --out gpurun_out/vn2_fb.json > gpurun_out/vn2_fb.log 2>&1
rc=$?
for f in gpurun_out/vn8_fb.log gpurun_out/vn4_fb.log gpurun_out/vn2_fb.log; do tail -1 "$f" | cut -c1-200; done
exit $rc
