#!/bin/bash
# Round-4 GPU call: the pipelined virtual node (8 GPUs, 48 epochs, 2 seeds, 3 gating passes) for
# greedy and the planner at corun sigma 0.05 (default) / 0.1 / 0.2.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_pvn_sigma
mkdir -p $OUT
timeout -k 10 900 python -u tools/pipelined_vn.py --gpus 8 --epochs 48 --warmup 5 --seeds 0 1 --passes 3 \
  --policies greedy planner planner-sig10 planner-sig20 --out $OUT/pipelined_vn.json > $OUT/pipelined_vn.log 2>&1
rc=$?
tail -1 $OUT/pipelined_vn.log | cut -c1-1500
exit $rc
