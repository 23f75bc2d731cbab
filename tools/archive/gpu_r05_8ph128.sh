#!/bin/bash
# Round 5: the 256x128 8-phase tile (13) -- numerics / race screen, kernel study, bench A/B
# against the 128x128 co-run default (policy 7 vs 1).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "every_tile_variant or race_screen or matches_fp32" > gpurun_out/tiles_pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/small_gemm_study.py > gpurun_out/small_gemm_study.log 2>&1 &&
timeout -k 10 900 python tools/ab.py --rounds 4 --steps 20 --warmup 5 --out gpurun_out/r05_8ph128_ab \
  --arm p1="--gemm-policy 1" --arm p7="--gemm-policy 7"
rc=$?
tail -3 gpurun_out/tiles_pytest.log; tail -14 gpurun_out/small_gemm_study.log | cut -c1-400
exit $rc
