#!/bin/bash
# Interleaved A/B of the HIP hardware-queue budget for the 1-GPU bench: with 4 queues (the
# box's exported default) the 4 pod streams + the control stream + the null stream share
# queues, and pods whose streams land on one queue run back to back instead of side by side.
# GPUSCHED_HW_QUEUES is what bench.py raises GPU_MAX_HW_QUEUES to.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/hwq
for r in 1 2; do
  for q in ${HWQ_LIST:-4 8 6}; do
    GPUSCHED_HW_QUEUES=$q GPU_MAX_HW_QUEUES=4 timeout -k 10 120 python bench.py --steps 60 --warmup 5 --out gpurun_out/hwq/q${q}_r${r}.json > gpurun_out/hwq/q${q}_r${r}.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/hwq/q${q}_r${r}.json')); print('q=$q r=$r', d['value'], d['ms_per_step'], d['gpu_util_pct'], d['sol_pct'])"
  done
done
