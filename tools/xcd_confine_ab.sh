#!/bin/bash
# XCD-confinement study: the probe (dispatch check, bit-exact numerics, stream rates, 2 GEMM + 2
# stream pods), then the bench interleaved at the driver's shape with --xcd-confine 0/1.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/xc
timeout -k 10 300 python -u tools/xcd_confine_probe.py > gpurun_out/xc/probe.log 2>&1 || { cat gpurun_out/xc/probe.log; exit 1; }
cat gpurun_out/xc/probe.log
for i in 1 2 3; do
  for x in 0 1; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --xcd-confine $x > gpurun_out/xc/b_${x}_${i}.log 2>&1 || exit $?
    echo "confine=$x run=$i $(grep '^{' gpurun_out/xc/b_${x}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"], d["achieved_hbm_tbps_per_gpu"], d.get("slo_attainment_pct"))')"
  done
done
