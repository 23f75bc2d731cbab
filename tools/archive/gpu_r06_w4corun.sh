#!/bin/bash
# Round 6: the 4-wave GEMM (tile 14) for co-running pods (--gemm-policy 10) -- one wave per SIMD
# leaves room for the other pods' stream waves on its CUs.  Numerics under arm 10, GEMM-only /
# full replay of the driver's timed pods, bench A/B against arm 1 (triad variant 6 = default;
# 7 = the 30-VGPR triad).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_w4corun; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
for p in 1 10; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --only replay,replay_gemm --bench-args "--gemm-policy $p" --out $O/replay_p$p.json > $O/replay_p$p.log 2>&1 || exit $?
done
for r in 1 2 3; do
  for arm in "1 6" "10 6" "10 7"; do
    set -- $arm
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $1 --triad-variant $2 > $O/b_p$1_v$2_r$r.json 2> $O/b_p$1_v$2_r$r.err || exit $?
  done
done
echo done
