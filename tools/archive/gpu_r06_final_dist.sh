#!/bin/bash
# Round 6: the final tree's headline spread -- ten back-to-back runs of the driver's bench command
# (N=1, 20 steps after 5 warm-up) and one 3,000-step run (seed 0).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_final_dist; mkdir -p $O
for r in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r$r.json 2> $O/bench_r$r.err || exit $?
done
timeout -k 10 240 python3 bench.py --steps 3000 --warmup 5 --seed 0 > $O/bench3000_s0.json 2> $O/bench3000_s0.err || exit $?
echo done
