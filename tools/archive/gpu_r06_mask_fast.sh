#!/bin/bash
# Round 6: the CU-partitioned kind split (triads masked to u units, GEMMs on the rest) in the fast
# hardware-queue layout, next to the replay in the same layout.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_mask_fast; mkdir -p $O
P=tools/inputs/r06_place_seed0.json
timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
  --only replay --out $O/replay.json > $O/replay.log 2>&1 || exit $?
for u in 3 4 5; do
  timeout -k 10 200 python3 -u tools/gap_decomp.py --placements $P --reps 3 --passes 2 --extra-streams 4:before \
    --mask-units $u --out $O/mask$u.json > $O/mask$u.log 2>&1 || exit $?
done
echo done
