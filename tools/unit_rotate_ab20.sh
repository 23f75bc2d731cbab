#!/bin/bash
# Interleaved A/B of the CU-slot rotation at the driver's bench shape (20 steps, 5 warmup).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/urot20
for r in 1 2 3; do
  for u in 0 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --unit-rotate $u --out gpurun_out/urot20/u${u}_r$r.json > gpurun_out/urot20/u${u}_r$r.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/urot20/u${u}_r$r.json')); print('rotate=$u r=$r', d['value'], d['ms_per_step'], d['slo_attainment_pct'])"
  done
done
