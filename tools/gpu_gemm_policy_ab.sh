#!/bin/bash
# Bench A/B of the GEMM tile policy (0 = default picker, 1 = 8-phase 256x256 also for pods
# whose CU share it fills), interleaved runs on one box.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2; do
  for p in 0 1; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --gemm-policy $p > gpurun_out/ab_${p}_${i}.log 2>&1 || exit $?
    echo "policy=$p run=$i $(grep '^{' gpurun_out/ab_${p}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"])')"
  done
done
