#!/bin/bash
# Round 6: knobs around arm 10 (the default) -- XCD tile-group rows, the plain GROUP_M order and
# the 22-VGPR stream kernel -- 3 interleaved bench rounds each at the driver's shape.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_w4knobs; mkdir -p $O
for r in 1 2 3; do
  for arm in "base:" "g2:--xcd-group 2" "g8:--xcd-group 8" "plain:--xcd-blocks 0" "v5:--triad-variant 5"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 $flags > $O/b_${name}_r$r.json 2> $O/b_${name}_r$r.err || exit $?
  done
done
echo done
