#!/bin/bash
# XCD-block GEMM tile order A/B (set_xcd_blocks 0/1): GEMM tests, the catalog GEMM tiles lone
# and as the 4-stream co-run mix (+ lone big shapes), the bench interleaved at the driver's
# shape (20 steps) and at 60 steps (--xcd-blocks 0/1).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/xcd
timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/xcd/gemm_test.log 2>&1 || exit $?
tail -1 gpurun_out/xcd/gemm_test.log
timeout -k 10 400 python -u tools/gemm_knob_mix.py set_xcd_blocks big > gpurun_out/xcd/mix.log 2>&1 || exit $?
cat gpurun_out/xcd/mix.log
for steps in 20 60; do
  for i in 1 2 3; do
    for x in 0 1; do
      timeout -k 10 200 python bench.py --steps $steps --warmup 5 --xcd-blocks $x > gpurun_out/xcd/b${steps}_${x}_${i}.log 2>&1 || exit $?
      echo "steps=$steps xcd=$x run=$i $(grep '^{' gpurun_out/xcd/b${steps}_${x}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"], d.get("slo_attainment_pct"))')"
    done
  done
done
