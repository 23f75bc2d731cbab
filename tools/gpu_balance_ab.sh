#!/bin/bash
# 1-GPU A/B of the balance term (--balance 1 default vs 0), interleaved, plus the GPU tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
: > gpurun_out/balance_ab.txt
for run in 1 2; do
  for b in 1 0; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --balance $b --out gpurun_out/bal_$b.json > gpurun_out/bal_$b.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/bal_$b.json'));print('balance=$b run=$run', d['value'], d['ms_per_step'], d['gpu_util_pct'], d['slo_attainment_pct'])" >> gpurun_out/balance_ab.txt
  done
done
tail -2 gpurun_out/pytest_gpu.log; cat gpurun_out/balance_ab.txt
