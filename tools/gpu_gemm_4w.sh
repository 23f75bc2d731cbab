#!/bin/bash
# 4-wave 256x256 GEMM (tiles 11/12): race-screen numerics first, then the big-GEMM table.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "8phase_numerics" > gpurun_out/gemm4w_test.log 2>&1 &&
GEMM_BIG_ARMS=${ARMS:-10,11,12} timeout -k 10 400 python -u tools/gemm_big.py > gpurun_out/gemm4w_big.log 2>&1
rc=$?
tail -8 gpurun_out/gemm4w_test.log; cat gpurun_out/gemm4w_big.log
exit $rc
