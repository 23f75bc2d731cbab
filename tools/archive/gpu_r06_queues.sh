#!/bin/bash
# Round 6: does the number of hardware queues in a process change the co-run replay?
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_queues; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
G="python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2"
timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 $G --only replay,replay_la2 --out $O/a_base.json > $O/a_base.log 2>&1 || exit $?
timeout -k 10 200 $G --only replay,replay_la2,split_share --out $O/b_split.json > $O/b_split.log 2>&1 || exit $?
timeout -k 10 200 $G --only replay,replay_la2 --extra-streams 1:after --out $O/c_x1after.json > $O/c_x1after.log 2>&1 || exit $?
timeout -k 10 200 $G --only replay,replay_la2 --extra-streams 4:after --out $O/d_x4after.json > $O/d_x4after.log 2>&1 || exit $?
timeout -k 10 200 $G --only replay,replay_la2 --extra-streams 4:before --out $O/e_x4before.json > $O/e_x4before.log 2>&1 || exit $?
timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 > $O/bench2.json 2> $O/bench2.err || exit $?
echo done
