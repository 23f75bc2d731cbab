#!/bin/bash
# Round-4 GPU call: the GPU test suite at HEAD, then the pipelined virtual node (8 GPUs, 48
# epochs, 2 seeds, 3 broadcast-gating passes) for greedy, the full planner and the planner at the
# cheaper effort levels the adaptive control plane uses at 8 GPUs (box CPU: 8.1 / 6.3 / 4.5 /
# 4.1 ms per epoch for levels 0-3 against a ~6.7 ms epoch).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_pvn_effort
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 900 python -u tools/pipelined_vn.py --gpus 8 --epochs 48 --warmup 5 --seeds 0 1 --passes 3 \
  --policies greedy planner planner-e1 planner-e2 planner-e3 --out $OUT/pipelined_vn.json > $OUT/pipelined_vn.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/pipelined_vn.log | cut -c1-1500
exit $rc
