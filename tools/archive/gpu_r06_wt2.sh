#!/bin/bash
# Round 6: write-through stores only for the largest streams (variants 9 / 10) vs the default.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_wt2; mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "triad_variants" > $O/numerics.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in 6 9 10; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --triad-variant $v > $O/b_v${v}_r$r.json 2> $O/b_v${v}_r$r.err || exit $?
  done
done
echo done
