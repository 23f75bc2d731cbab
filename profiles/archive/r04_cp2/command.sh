#!/bin/bash
# Round-4 GPU call: control-plane cost on the box CPU with the burst planner and slot timelines
# compiled (Cython, _native/cyaccel.py) against the same modules from their .py sources
# (GPUSCHED_CY_SKIP), interleaved twice; the effort ladder at 8 GPUs; the bench at the driver's
# shape twice; the 8-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp CP_TIMING_GPUS=8
OUT=gpurun_out/r04_cp2
mkdir -p $OUT
SKIP=plugins.gpu.planner,plugins.gpu.timeline
timeout -k 10 300 python tools/cp_timing.py > $OUT/cp_compiled_1.txt 2>&1 &&
GPUSCHED_CY_SKIP=$SKIP timeout -k 10 300 python tools/cp_timing.py > $OUT/cp_pyplanner_1.txt 2>&1 &&
timeout -k 10 300 python tools/cp_timing.py > $OUT/cp_compiled_2.txt 2>&1 &&
GPUSCHED_CY_SKIP=$SKIP timeout -k 10 300 python tools/cp_timing.py > $OUT/cp_pyplanner_2.txt 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench20a.json > $OUT/bench20a.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench20b.json > $OUT/bench20b.log 2>&1 &&
timeout -k 10 420 bash tools/rehearsal_8rank.sh > $OUT/rehearsal.txt 2>&1 &&
cp gpurun_out/rehearsal_8rank.json $OUT/
rc=$?
for f in cp_compiled_1 cp_pyplanner_1 cp_compiled_2 cp_pyplanner_2; do echo "== $f"; cat $OUT/$f.txt; done
for f in bench20a bench20b; do python -c "
import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['slo_attainment_pct'], d['sol_pct'], d['control_plane_ms_per_epoch'])"; done
cat $OUT/rehearsal.txt
exit $rc
