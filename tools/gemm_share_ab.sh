#!/bin/bash
# Interleaved A/B of the co-run GEMM tile policy and HIP-graph replay in the 1-GPU bench (8 HW
# queues, bench.py's default): share-sized tiles vs whole-chip tiles, 128x128 vs the 8-phase
# 256x256 for co-running pods, graphs on/off.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gshare8
for r in 1 2; do
  for cfg in "1 1 1" "1 0 1" "0 1 1" "0 0 1" "1 1 0"; do
    set -- $cfg
    tag=s$1_p$2_g$3_r$r
    timeout -k 10 120 python bench.py --steps 60 --warmup 5 --gemm-share $1 --gemm-policy $2 --graphs $3 --out gpurun_out/gshare8/$tag.json > gpurun_out/gshare8/$tag.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/gshare8/$tag.json')); print('share=$1 policy=$2 graphs=$3 r=$r', d['value'], d['ms_per_step'], d['sol_pct']['peak'], d['mfma_util_pct'], d['slo_attainment_pct'])"
  done
done
