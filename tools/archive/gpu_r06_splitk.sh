#!/bin/bash
# Round 6: co-run split-K on the 8-phase kernel (--gemm-policy 8) --
# numerics, GEMM-only / full replay of the driver's timed pods, bench A/B against arm 1.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_splitk; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "split_k" > $O/numerics.log 2>&1 || exit $?
for p in 1 8; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --only replay,replay_gemm --bench-args "--gemm-policy $p" --out $O/replay_p$p.json > $O/replay_p$p.log 2>&1 || exit $?
done
for r in 1 2 3; do
  for p in 1 8; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/b_p${p}_r$r.json 2> $O/b_p${p}_r$r.err || exit $?
  done
done
echo done
