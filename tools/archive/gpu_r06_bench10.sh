#!/bin/bash
# Round 6: ten back-to-back runs of the driver's bench command at the final tree (N=1, 20 steps
# after 5 warm-up) -- the spread of the headline number on one box.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_bench10; mkdir -p $O
for r in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r$r.json 2> $O/bench_r$r.err || exit $?
done
echo done
