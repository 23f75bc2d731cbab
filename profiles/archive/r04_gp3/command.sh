#!/bin/bash
# Round-4 GPU call: GEMM policy 3 (co-running pods take the 8-phase 256x256 tile already when it
# gives half of their CU share a workgroup) against the default policy 1, N=1 interleaved A/B.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_gp3
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "8phase or gemm" > $OUT/pytest_gemm.log 2>&1 &&
timeout -k 10 900 python tools/ab.py --rounds 4 --steps 20 --warmup 5 --timeout 150 --out $OUT \
  --arm base="" --arm gp3="--gemm-policy 3" > $OUT/ab.log 2>&1
rc=$?
tail -2 $OUT/pytest_gemm.log; tail -1 $OUT/ab.log | cut -c1-1500
exit $rc
