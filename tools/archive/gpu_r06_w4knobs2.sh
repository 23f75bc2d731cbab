#!/bin/bash
# Round 6: XCD tile-group rows under arm 10, second pass with the arm order rotated (g8 first).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_w4knobs2; mkdir -p $O
for r in 1 2 3 4; do
  for arm in "g8:--xcd-group 8" "base:" "g16:--xcd-group 16" "g2:--xcd-group 2"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 $flags > $O/b_${name}_r$r.json 2> $O/b_${name}_r$r.err || exit $?
  done
done
echo done
