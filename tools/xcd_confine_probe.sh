#!/bin/bash
# XCD-confinement probe (tools/xcd_confine_probe.py) under its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/xcd_confine_probe.py > gpurun_out/xcd_confine.log 2>&1
rc=$?
cat gpurun_out/xcd_confine.log
exit $rc
