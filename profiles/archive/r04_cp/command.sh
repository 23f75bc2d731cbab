#!/bin/bash
# Round-4 GPU call 2: control-plane cost on the box CPU (bench defaults incl. slot planning),
# the 8-rank rehearsal, and an interleaved N=1 A/B of the slot planner's spread tolerance
# against the executor's LPT re-slotting.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_cp
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "planner_feedback_moves_work" > gpurun_out/r04_cp/pytest_direction.log 2>&1 &&
timeout -k 10 400 python tools/cp_timing.py > gpurun_out/r04_cp/cp_timing_box.txt 2>&1 &&
timeout -k 10 420 bash tools/rehearsal_8rank.sh > gpurun_out/r04_cp/rehearsal.txt 2>&1 &&
cp gpurun_out/rehearsal_8rank.json gpurun_out/r04_cp/ &&
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --timeout 150 --out gpurun_out/r04_cp/ab20 \
  --arm sp0="--slot-spread-ms 0" --arm sp1="--slot-spread-ms 1" --arm balanced="--slot-balance 1 --plan-slots 0" \
  --arm sp2="--slot-spread-ms 2" > gpurun_out/r04_cp/ab20.log 2>&1
rc=$?
grep -E "measured feedback|passed|failed|Error" gpurun_out/r04_cp/pytest_direction.log | cut -c1-600; cat gpurun_out/r04_cp/cp_timing_box.txt; cat gpurun_out/r04_cp/rehearsal.txt; tail -1 gpurun_out/r04_cp/ab20.log | cut -c1-900
exit $rc
