#!/bin/bash
# Interleaved A/B on one MI355X: online interference learning with and without the learned prior
# scale (--online-scale), at the driver's shape (20 steps) and over 60 steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/oscale
for rep in ${REPS:-1 2}; do
  for s in 0 1; do
    for n in ${STEPS:-20 60}; do
      timeout -k 10 200 python bench.py --steps $n --warmup 5 --online-scale $s > gpurun_out/oscale/r${rep}_s${s}_n${n}.log 2>&1 || exit $?
      echo "rep $rep scale $s steps $n: $(grep -o '"value": [0-9.]*\|"slo_attainment_pct": [0-9.]*\|"interference_mae": {[^}]*}' gpurun_out/oscale/r${rep}_s${s}_n${n}.log | tr '\n' ' ')"
    done
  done
done
