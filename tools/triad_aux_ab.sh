#!/bin/bash
# Stream-kernel cache-policy study: variant 5 (buffer instructions) with sc0/sc1/nt policies vs the
# default (variant 6 -> non-temporal global loads): triad tests, lone HBM rate per policy, the
# bench interleaved at the driver's shape.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/aux
timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "triad" > gpurun_out/aux/test.log 2>&1 || exit $?
tail -1 gpurun_out/aux/test.log
timeout -k 10 120 python -u tools/triad_aux_rate.py > gpurun_out/aux/rate.log 2>&1 || exit $?
cat gpurun_out/aux/rate.log
for i in 1 2; do
  for arm in "6 2" "5 2" "5 18" "5 19" "5 3" "5 0"; do
    set -- $arm
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --triad-variant $1 --triad-aux $2 > gpurun_out/aux/b_${1}_${2}_${i}.log 2>&1 || exit $?
    echo "variant=$1 aux=$2 run=$i $(grep '^{' gpurun_out/aux/b_${1}_${2}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"], d["achieved_hbm_tbps_per_gpu"], d.get("slo_attainment_pct"))')"
  done
done
