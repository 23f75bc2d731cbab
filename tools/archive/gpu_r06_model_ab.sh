#!/bin/bash
# Round 6: the co-run model refitted under the 4-wave co-run GEMM (data/corun_mi355x_r06.json)
# against the shipped one -- 5 interleaved bench rounds at the driver's shape.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_model_ab; mkdir -p $O
for r in 1 2 3 4 5; do
  for arm in "new:--corun-model k8s_gpu_scheduler_amd/data/corun_mi355x_r06.json" "old:"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 $flags > $O/b_${name}_r$r.json 2> $O/b_${name}_r$r.err || exit $?
  done
done
echo done
