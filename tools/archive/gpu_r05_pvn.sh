#!/bin/bash
# Round-5 pipelined virtual node (8 GPUs, 48 epochs, 2 seeds, 3 broadcast-gating passes): greedy,
# the full planner and the planner at effort levels 1 and 2 -- the round-5 planner (measured
# speeds instead of the backlog integrator, no-empty-GPU rule, fast-forwarded slot plans).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_NAME:-r05_pvn}
mkdir -p $OUT
timeout -k 10 1100 python -u tools/pipelined_vn.py --gpus 8 --epochs 48 --warmup 5 --seeds ${SEEDS:-0 1} --passes 3 \
  --policies ${POLICIES:-greedy planner planner-e1 planner-e2} --out $OUT/pipelined_vn.json > $OUT/pipelined_vn.log 2>&1
rc=$?
tail -1 $OUT/pipelined_vn.log | cut -c1-1500
exit $rc
