#!/bin/bash
# Interleaved A/B: executor-side slot balancing (LPT onto the least-backlogged CU slot) at 20 and 60 steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sbal
for r in 1 2 3; do
  for k in 20 60; do
    for b in 0 1; do
      timeout -k 10 120 python bench.py --steps $k --warmup 5 --slot-balance $b --out gpurun_out/sbal/b${b}_k${k}_r$r.json > gpurun_out/sbal/b${b}_k${k}_r$r.log 2>&1 || exit $?
      python -c "import json; d=json.load(open('gpurun_out/sbal/b${b}_k${k}_r$r.json')); print('balance=$b K=$k r=$r', d['value'], d['ms_per_step'], d['slo_attainment_pct'])"
    done
  done
done
