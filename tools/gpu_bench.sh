#!/bin/bash
# Short bench sweep on the GPU box: each GPU step has its own time limit and the chain
# stops at the first failure (no GPU work after a fault/timeout).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --out gpurun_out/b_default.json > gpurun_out/b_default.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --qos guaranteed --out gpurun_out/b_guaranteed.json > gpurun_out/b_guaranteed.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --policy random --out gpurun_out/b_random.json > gpurun_out/b_random.log 2>&1
rc=$?
for f in gpurun_out/b_*.json; do echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print({k:d.get(k) for k in ['value','ms_per_step','gpu_util_pct','cu_share_occupancy_pct','mfma_util_pct','achieved_tflops','slo_attainment_pct','host_ms_per_step_rank0']})"; done
exit $rc
