#!/bin/bash
# Round 6: co-run model data under the 4-wave co-run GEMM (arm 10, the default): 2,400 isolated
# 1-4 pod groups (models.corun collect) and 150-step bench pipeline traces for seeds 0-2
# (GPUSCHED_BENCH_TRACE), as the shipped model's training data was collected in rounds 3-4.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06_corun; mkdir -p $O
timeout -k 10 400 python3 -u -m k8s_gpu_scheduler_amd.models.corun collect --groups 2400 --out $O/groups.json > $O/collect.log 2>&1 || exit $?
for seed in 0 1 2; do
  GPUSCHED_BENCH_TRACE=$O/trace_s$seed.json timeout -k 10 200 python3 bench.py --steps 150 --warmup 5 --seed $seed \
    --out $O/trace_s${seed}_result.json > $O/trace_s$seed.log 2>&1 || exit $?
done
echo done
