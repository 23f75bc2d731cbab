#!/bin/bash
# Round-4 GPU call: where the N=1 SLO misses are -- the bench's one-GPU placement stream (48
# epochs, 3 seeds) replayed through the launch-ahead slot pipeline, SLOs met per workload.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_n1_wl
mkdir -p $OUT
timeout -k 10 600 python -u tools/pipelined_vn.py --gpus 1 --epochs 48 --warmup 5 --seeds 0 1 2 --passes 1 \
  --policies planner --out $OUT/pvn_n1.json > $OUT/pvn_n1.log 2>&1
rc=$?
tail -1 $OUT/pvn_n1.log | cut -c1-600
exit $rc
