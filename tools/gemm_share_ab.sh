#!/bin/bash
# Interleaved A/B of the co-run GEMM tile policy in the 1-GPU bench: share-sized tiles
# (default) vs whole-chip tiles vs the 8-phase 256x256 for co-running pods.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gshare
for r in 1 2; do
  for cfg in "1 0" "0 0" "1 1" "0 1"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps 60 --warmup 5 --gemm-share $1 --gemm-policy $2 --out gpurun_out/gshare/s$1_p$2_r$r.json > gpurun_out/gshare/s$1_p$2_r$r.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/gshare/s$1_p$2_r$r.json')); print('share=$1 policy=$2 r=$r', d['value'], d['ms_per_step'], d['sol_pct']['peak'], d['mfma_util_pct'])"
  done
done
