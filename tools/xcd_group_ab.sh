#!/bin/bash
# Rows per group inside an XCD block (--xcd-group 2/4/8; 4 = default), bench interleaved at the
# driver's shape (20 steps) and 60 steps.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/xg
timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/xg/gemm_test.log 2>&1 || exit $?
tail -1 gpurun_out/xg/gemm_test.log
for steps in 20 60; do
  for i in 1 2; do
    for g in 2 4 8 1; do
      timeout -k 10 200 python bench.py --steps $steps --warmup 5 --xcd-group $g > gpurun_out/xg/b${steps}_${g}_${i}.log 2>&1 || exit $?
      echo "steps=$steps group=$g run=$i $(grep '^{' gpurun_out/xg/b${steps}_${g}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"], d.get("slo_attainment_pct"))')"
    done
  done
done
