#!/bin/bash
# Round 6: the hardware direction tests (40 % and 15 % slower GPU 1) with the rank-test speed gate.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_dir; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 180 --timeout-method thread tests/test_gpu_native.py \
  -k "direction or slower_gpu or 15pct" > $O/direction.log 2>&1 || exit $?
echo done
