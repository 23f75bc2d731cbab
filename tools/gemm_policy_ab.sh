#!/bin/bash
# Interleaved A/B of the co-run GEMM tile policy in the 1-GPU bench: 1 = 8-phase 256x256 when its
# tiles fill the pod's CU share (default), 3 / 4 = also when they fill half / a quarter of it.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gpol
STEPS=${STEPS:-60}
for r in 1 2 3; do
  for p in ${POLICIES:-1 3 4}; do
    timeout -k 10 120 python bench.py --steps $STEPS --warmup 5 --gemm-policy $p --out gpurun_out/gpol/p${p}_s${STEPS}_r$r.json > gpurun_out/gpol/p${p}_r$r.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/gpol/p${p}_s${STEPS}_r$r.json')); print('steps=$STEPS policy=$p r=$r', d['value'], d['ms_per_step'], d['sol_pct']['peak'], d['mfma_util_pct'], d['slo_attainment_pct'])"
  done
done
