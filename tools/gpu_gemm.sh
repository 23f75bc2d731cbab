#!/bin/bash
# GEMM kernel round: numerics of every tile variant, the tile study, then the 1-GPU bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_native.py -x -q -k "gemm" > gpurun_out/pytest_gemm.log 2>&1 &&
timeout -k 10 500 python tools/gemm_tiles.py > gpurun_out/gemm_tiles.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gemm.log; grep concurrent -A0 gpurun_out/gemm_tiles.log; grep "'tile'" gpurun_out/gemm_tiles.log | tail -8; grep '^{' gpurun_out/bench.log | cut -c1-900
exit $rc
