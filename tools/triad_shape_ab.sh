#!/bin/bash
# Interleaved A/B of the HBM-stream kernel launch shape in the 1-GPU bench (8 HW queues),
# then a rocprofv3 kernel trace of the default for the GEMM/stream overlap timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tshape
for r in 1 2; do
  for cfg in "6 0" "3 256" "3 512" "3 1024" "4 256" "4 512" "3 2048"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps 60 --warmup 5 --triad-variant $1 --triad-blocks $2 --out gpurun_out/tshape/v$1_b$2_r$r.json > gpurun_out/tshape/v$1_b$2_r$r.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/tshape/v$1_b$2_r$r.json')); print('v=$1 b=$2 r=$r', d['value'], d['ms_per_step'], d['sol_pct']['peak'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tshape/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 > gpurun_out/tshape/prof.log 2>&1
