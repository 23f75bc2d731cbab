#!/bin/bash
# Pod kernel sequences replayed as HIP graphs (--graphs 1, default) vs launched eagerly (0),
# bench interleaved at the driver's shape (20 steps) and at 60 steps.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/gr
for steps in 20 60; do
  for i in 1 2 3; do
    for g in 0 1; do
      timeout -k 10 200 python bench.py --steps $steps --warmup 5 --graphs $g > gpurun_out/gr/b${steps}_${g}_${i}.log 2>&1 || exit $?
      echo "steps=$steps graphs=$g run=$i $(grep '^{' gpurun_out/gr/b${steps}_${g}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_ms_per_step_rank0"], d.get("slo_attainment_pct"))')"
    done
  done
done
