#!/bin/bash
# Round 6 batch: busy-ms hardware test, triad variants (kernel level), hardware-queue count
# experiment, triad-variant bench A/B, GEMM policy arms 5-7 vs 1.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_arms; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 180 --timeout-method thread tests/test_gpu_telemetry.py \
  -k busy_ms > $O/busy_ms.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/triad_variants.py > $O/triad_variants.log 2>&1 || exit $?
bash tools/gpu_r06_queues.sh || exit $?
for r in 1 2 3; do
  for v in 6 5 7; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --triad-variant $v > $O/tv${v}_r$r.json 2> $O/tv${v}_r$r.err || exit $?
  done
done
for r in 1 2; do
  for p in 1 5 6 7; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/p${p}_r$r.json 2> $O/p${p}_r$r.err || exit $?
  done
done
echo done
