#!/bin/bash
# Short bench sweep on the GPU box: each GPU step has its own time limit and the chain
# stops at the first failure (no GPU work after a fault/timeout).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --out gpurun_out/b_default.json > gpurun_out/b_default.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cu-mask --out gpurun_out/b_nomask.json > gpurun_out/b_nomask.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --policy random --out gpurun_out/b_random.json > gpurun_out/b_random.log 2>&1
rc=$?
for f in gpurun_out/b_*.log; do echo "== $f"; grep '^{' $f | cut -c1-400; tail -2 $f | grep -v '^{'; done
exit $rc
