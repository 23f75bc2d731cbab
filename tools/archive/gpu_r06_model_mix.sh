#!/bin/bash
# Round 6: which half of the refitted co-run model plans worse -- new alone times with the shipped
# coupling (B) and the shipped alone times with the new coupling (C) against the shipped model.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_model_mix; mkdir -p $O
for r in 1 2 3 4; do
  for arm in "B:--corun-model k8s_gpu_scheduler_amd/data/corun_mix_B.json" "C:--corun-model k8s_gpu_scheduler_amd/data/corun_mix_C.json" "old:"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 $flags > $O/b_${name}_r$r.json 2> $O/b_${name}_r$r.err || exit $?
  done
done
echo done
