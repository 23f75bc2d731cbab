#!/bin/bash
# Fixed per-run cost of the timed region: bench at K = 10 / 20 / 40 / 80 timed steps (5 warm-up);
# a linear fit of K x ms_per_step = K x s + c separates the steady epoch s from the fill/drain c.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/steps
for k in 10 20 40 80 20 80; do
  timeout -k 10 120 python bench.py --steps $k --warmup 5 --out gpurun_out/steps/k$k.json > gpurun_out/steps/k$k.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/steps/k$k.json')); print('K=$k', d['value'], d['ms_per_step'])"
done
