#!/bin/bash
# Control-plane cost per 8-GPU epoch on the box CPU for alternative effort-level tables
# (GPUSCHED_EFFORT_LEVELS, plugins.gpu.planner.BurstPlanner.EFFORT_LEVELS), interleaved with the
# default table: tools/cp_timing.py, 8 GPUs x 4 pods, 60 timed epochs.
#   TABLES="name=levels;..." rows "sweep divisor,phantoms,pipeline eval,model slots" per level
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUT_NAME:-cp_levels}
mkdir -p $OUT
: > $OUT/summary.txt
for r in ${ROUNDS:-1 2 3}; do
  CP_TIMING_GPUS=8 CP_TIMING_CONFIGS=bench-defaults,bench-effort1,bench-effort2 \
    timeout -k 10 300 python tools/cp_timing.py > $OUT/default_r$r.txt 2>&1 || exit $?
  sed "s/^/default r$r /" $OUT/default_r$r.txt >> $OUT/summary.txt
  for t in $TABLES; do
    name=${t%%=*}; lv=${t#*=}
    GPUSCHED_EFFORT_LEVELS="$lv" CP_TIMING_GPUS=8 CP_TIMING_CONFIGS=${LEVEL_CONFIGS:-bench-effort1} \
      timeout -k 10 300 python tools/cp_timing.py > $OUT/${name}_r$r.txt 2>&1 || exit $?
    sed "s/^/$name r$r /" $OUT/${name}_r$r.txt >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
