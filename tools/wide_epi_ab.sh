#!/bin/bash
# GEMM wide-epilogue A/B: GEMM tests (all tiles + 8-phase race screen), the catalog GEMM
# tiles lone and as the 4-stream co-run mix, and the bench interleaved (--wide-epilogue 0/1).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/gemm_test.log 2>&1 || exit $?
tail -1 gpurun_out/gemm_test.log
timeout -k 10 300 python -u tools/gemm_knob_mix.py > gpurun_out/wide_epi_mix.log 2>&1 || exit $?
cat gpurun_out/wide_epi_mix.log
for i in 1 2 3; do
  for w in 0 1; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --wide-epilogue $w > gpurun_out/wab_${w}_${i}.log 2>&1 || exit $?
    echo "wide=$w run=$i $(grep '^{' gpurun_out/wab_${w}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"])')"
  done
done
