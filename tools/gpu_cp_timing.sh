#!/bin/bash
# Control-plane cost per 8-GPU epoch on the box CPU (tools/cp_timing.py, interleaved rounds).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
CP_TIMING_GPUS=8 CP_TIMING_ROUNDS=${ROUNDS:-3} CP_GC_SETTLE=${GC_SETTLE:-1} CP_TIMING_CONFIGS=${CONFIGS:-plain,bench-defaults,bench-effort1,bench-effort2} \
  timeout -k 10 600 python tools/cp_timing.py > gpurun_out/cp_timing_box.txt 2>&1
rc=$?
cat gpurun_out/cp_timing_box.txt
exit $rc
