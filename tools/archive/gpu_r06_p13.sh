#!/bin/bash
# Round 6: arm 13 (arm 10 + the 4-wave kernel on 128x128 blocks for the small co-run GEMMs) --
# numerics (race screen, arm test), GEMM-only / full replay, 4 interleaved bench rounds vs arm 10.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_p13; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "policy11_13 or (8phase_numerics_and_race_screen and 16)" -p no:cacheprovider > $O/numerics.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/gemm_w4_check.py 10 > $O/check.log 2>&1 || exit $?
for p in 10 13; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --only replay,replay_gemm --bench-args "--gemm-policy $p" --out $O/replay_p$p.json > $O/replay_p$p.log 2>&1 || exit $?
done
for r in 1 2 3 4; do
  for p in 13 10; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/b_p${p}_r$r.json 2> $O/b_p${p}_r$r.err || exit $?
  done
done
echo done
