#!/bin/bash
# Round 6: launch-ahead depth under the 4-wave co-run GEMM -- 2 (default) vs 3 vs 1, 4 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_lookahead; mkdir -p $O
for r in 1 2 3 4; do
  for la in 3 2 1; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --lookahead $la > $O/b_la${la}_r$r.json 2> $O/b_la${la}_r$r.err || exit $?
  done
done
echo done
