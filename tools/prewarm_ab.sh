#!/bin/bash
# Does a device warm-up before the warm-up epochs change the driver-shape (20-step) bench?
# (hypothesis: the GPU runs the first timed epochs' GEMMs below its steady clock)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prewarm
for r in 1 2; do
  for p in 0 300 1000; do
    GPUSCHED_BENCH_TRACE=gpurun_out/prewarm/trace_p${p}_r$r.json timeout -k 10 120 python bench.py --steps 20 --warmup 5 --prewarm-ms $p --out gpurun_out/prewarm/p${p}_r$r.json > gpurun_out/prewarm/p${p}_r$r.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/prewarm/p${p}_r$r.json')); print('prewarm=$p r=$r', d['value'], d['ms_per_step'], d['smi'])"
  done
done
