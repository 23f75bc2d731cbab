#!/bin/bash
# Per-pod pipeline traces of the bench (GPUSCHED_BENCH_TRACE) over several slot policies and
# seeds: training / validation data for the co-run model in the pipelined setting.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_traces
for seed in 0 1 2; do
  for arm in "balanced:--slot-balance 1" "slots:--slot-balance 0 --plan-slots 1 --slot-spread-ms 2" "fixed:--slot-balance 0"; do
    name=${arm%%:*}; flags=${arm#*:}
    GPUSCHED_BENCH_TRACE=gpurun_out/r04_traces/${name}_s${seed}.json timeout -k 10 150 python bench.py --steps 150 --warmup 5 \
      --seed $seed $flags --out gpurun_out/r04_traces/${name}_s${seed}_result.json > gpurun_out/r04_traces/${name}_s${seed}.log 2>&1 || exit 1
    echo "$name seed $seed done"
  done
done
