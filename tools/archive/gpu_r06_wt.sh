#!/bin/bash
# Round 6: write-through (sc1) triad stores, variant 8 -- numerics, kernel-level co-run beside an
# 8-phase GEMM, replay of the driver's timed pods, bench A/B against the default (auto = 3).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_wt; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "triad_variants" > $O/numerics.log 2>&1 || exit $?
TRIAD_VARIANTS=3,8 timeout -k 10 120 python3 -u tools/triad_variants.py > $O/triad_variants.log 2>&1 || exit $?
for v in 6 8; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --only replay,replay_triad --bench-args "--triad-variant $v" --out $O/replay_v$v.json > $O/replay_v$v.log 2>&1 || exit $?
done
for r in 1 2 3; do
  for v in 6 8; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --triad-variant $v > $O/b_v${v}_r$r.json 2> $O/b_v${v}_r$r.err || exit $?
  done
done
echo done
