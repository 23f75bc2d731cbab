#!/bin/bash
# Round 6: share-capped 8-phase GEMM launches (--gemm-policy 9) -- numerics, replay, bench A/B.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_cap; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "policy9" > $O/numerics.log 2>&1 || exit $?
for p in 1 9; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --only replay,replay_gemm --bench-args "--gemm-policy $p" --out $O/replay_p$p.json > $O/replay_p$p.log 2>&1 || exit $?
done
for r in 1 2 3; do
  for p in 1 9; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/b_p${p}_r$r.json 2> $O/b_p${p}_r$r.err || exit $?
  done
done
echo done
