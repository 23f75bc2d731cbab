#!/bin/bash
# Round 6: 3,000-step benches (seeds 0-2) at the round-6 default (arm 10) and arm 1 (the round-5
# GEMM policy), interleaved -- steady-state evidence next to profiles/r05_final/longrun/.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_longrun; mkdir -p $O
for seed in 0 1 2; do
  for p in 10 1; do
    timeout -k 10 240 python3 bench.py --steps 3000 --warmup 5 --seed $seed --gemm-policy $p > $O/b_p${p}_s$seed.json 2> $O/b_p${p}_s$seed.err || exit $?
  done
done
echo done
