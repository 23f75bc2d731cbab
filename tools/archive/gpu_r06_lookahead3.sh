#!/bin/bash
# Round 6: launch-ahead depth 3 (default) vs 2, third box, 5 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_lookahead3; mkdir -p $O
for r in 1 2 3 4 5; do
  for la in 2 3; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --lookahead $la > $O/b_la${la}_r$r.json 2> $O/b_la${la}_r$r.err || exit $?
  done
done
echo done
