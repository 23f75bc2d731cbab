#!/bin/bash
# Round 6: co-run replay vs the number of hardware queues created BEFORE the 4 slot streams,
# then the core regimes again in the fast layout (4 queues first).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_queues2; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
G="python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2"
for k in 0 1 2 3 5 6 8; do
  timeout -k 10 200 $G --only replay,replay_la2 --extra-streams $k:before --out $O/k$k.json > $O/k$k.log 2>&1 || exit $?
done
timeout -k 10 400 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 4 --extra-streams 4:before --out $O/core_fast.json > $O/core_fast.log 2>&1 || exit $?
echo done
