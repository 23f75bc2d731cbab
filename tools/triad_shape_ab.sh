#!/bin/bash
# Interleaved A/B of the HBM-stream kernel launch shape in the 1-GPU bench (bench.py raises the
# HW queues to 8), then a rocprofv3 kernel trace of the default for the GEMM/stream overlap
# timeline (GPU_MAX_HW_QUEUES exported: the profiler initialises HIP before bench.py runs).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/tshape8
mkdir -p $out
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 > $out/prof.log 2>&1 || exit $?
for r in 1 2; do
  for cfg in "6 0" "3 256" "3 1024" "4 512" "3 2048" "3 4096"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps 60 --warmup 5 --triad-variant $1 --triad-blocks $2 --out $out/v$1_b$2_r$r.json > $out/v$1_b$2_r$r.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('$out/v$1_b$2_r$r.json')); print('v=$1 b=$2 r=$r', d['value'], d['ms_per_step'], d['sol_pct']['peak'])"
  done
done
