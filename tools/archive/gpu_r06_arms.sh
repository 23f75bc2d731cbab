#!/bin/bash
# Round 6: the busy-ms hardware test, then the --gemm-policy arms 5-7 re-measured after the
# picker fix, interleaved with the default arm 1, 20-step bench each.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_arms; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 180 --timeout-method thread tests/test_gpu_telemetry.py \
  -k busy_ms > $O/busy_ms.log 2>&1 || exit $?
for r in 1 2 3; do
  for p in 1 5 6 7; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/p${p}_r$r.json 2> $O/p${p}_r$r.err || exit $?
  done
done
echo done
