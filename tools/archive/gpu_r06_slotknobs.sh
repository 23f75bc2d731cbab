#!/bin/bash
# Round 6: slot-planning knobs under the 4-wave co-run GEMM -- 4 interleaved bench rounds.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_slotknobs; mkdir -p $O
for r in 1 2 3 4; do
  for arm in "base:" "spread1:--slot-spread-ms 1" "spread4:--slot-spread-ms 4" "model:--plan-slots model"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 $flags > $O/b_${name}_r$r.json 2> $O/b_${name}_r$r.err || exit $?
  done
done
echo done
