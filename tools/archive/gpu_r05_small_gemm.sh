#!/bin/bash
# Round 5: the co-run small-GEMM path -- numerics / race screen of the multi-stage 128x128 tiles,
# the per-setting kernel study (tools/small_gemm_study.py), then an interleaved bench A/B of the
# co-run small-GEMM policies (1 = 128x128 2-stage, 5 / 6 = 3 / 4 stages).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "every_tile_variant or race_screen" > gpurun_out/tiles_pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/small_gemm_study.py > gpurun_out/small_gemm_study.log 2>&1 &&
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --out gpurun_out/r05_small_ab \
  --arm p1="--gemm-policy 1" --arm p5="--gemm-policy 5" --arm p6="--gemm-policy 6"
rc=$?
tail -3 gpurun_out/tiles_pytest.log; tail -12 gpurun_out/small_gemm_study.log
exit $rc
