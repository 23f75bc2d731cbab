#!/bin/bash
# Round 5: timed-region PMC record of the bench kernels (default policy), then an interleaved
# 20-step bench A/B of the co-run small-GEMM tile policy (1 = 128x128, 3 = 256x128 2-stage,
# 4 = 256x128 3-stage).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
PMC_OUT=r05_pmc bash tools/gpu_pmc_bench.sh > gpurun_out/r05_pmc.log 2>&1 &&
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --out gpurun_out/r05_gemm_ab \
  --arm p1="--gemm-policy 1" --arm p3="--gemm-policy 3" --arm p4="--gemm-policy 4"
