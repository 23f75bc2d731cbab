#!/bin/bash
# Round 6 gap decomposition, second pass: every regime family in its own process with only the
# streams it uses, at the bench's hardware-queue limit (16).  Inputs: the driver-config bench
# run's timed placements (tools/inputs/r06_place_seed0.json, seed 0, 20 steps after 5 warm-up).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_gap3; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
timeout -k 10 300 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 4 --out $O/core.json > $O/core.log 2>&1 || exit $?
for u in 3 4 5; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --mask-units $u --out $O/mask$u.json > $O/mask$u.log 2>&1 || exit $?
done
timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --triad-units --umc-cal --out $O/cal.json > $O/cal.log 2>&1 || exit $?
echo done
