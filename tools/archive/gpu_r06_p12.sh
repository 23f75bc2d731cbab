#!/bin/bash
# Round 6: arm 12 (every co-running GEMM 256x256 divides on the 4-wave kernel, even under-filling
# its share) against arm 10 (the default): replay and 4 interleaved bench rounds.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_p12; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
for p in 10 12; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --only replay,replay_gemm --bench-args "--gemm-policy $p" --out $O/replay_p$p.json > $O/replay_p$p.log 2>&1 || exit $?
done
for r in 1 2 3 4; do
  for p in 12 10; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/b_p${p}_r$r.json 2> $O/b_p${p}_r$r.err || exit $?
  done
done
echo done
