#!/bin/bash
# Round-4 GPU call: lone 8-phase GEMMs in the plain GROUP_M tile order -- the tile-order and
# 8-phase GPU tests, the lone-GEMM sweep against hipBLASLt (7 interleaved rounds), and the bench
# at the driver's shape (co-running pods keep the XCD-block order).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_lone_order
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "tile_orders or 8phase or gemm" > $OUT/pytest_gemm.log 2>&1 &&
XCD_SWEEP_ARMS=torch,g4,plain XCD_SWEEP_ROUNDS=7 XCD_SWEEP_OUT=$OUT/gemm_xcd.json timeout -k 10 400 python tools/gemm_xcd_sweep.py > $OUT/gemm_xcd.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench20.json > $OUT/bench20.log 2>&1
rc=$?
tail -2 $OUT/pytest_gemm.log; cat $OUT/gemm_xcd.log
python -c "
import json; d=json.load(open('$OUT/bench20.json')); print('bench20', d['value'], d['slo_attainment_pct'])"
exit $rc
