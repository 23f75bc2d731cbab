#!/bin/bash
# Round-4 evidence at the final head: smoke(), the GPU test suite, the bench at the driver's shape
# twice and at 60 steps, a rocprofv3 kernel-statistics profile of a bench run WITHOUT the
# pre-warm loop (so the statistics are the pods' kernels only), and the 8-rank rehearsal on one
# GPU.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_final
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench20a.json > $OUT/bench20a.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench20b.json > $OUT/bench20b.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --out $OUT/bench60.json > $OUT/bench60.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --prewarm-ms 0 > $OUT/bench_prof.log 2>&1 &&
timeout -k 10 420 bash tools/rehearsal_8rank.sh > $OUT/rehearsal.txt 2>&1 &&
cp gpurun_out/rehearsal_8rank.json $OUT/
rc=$?
tail -1 $OUT/smoke.log; tail -2 $OUT/pytest_gpu.log
for f in bench20a bench20b bench60; do python -c "
import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['slo_attainment_pct'], d['sol_pct'], d['planner'].get('slot_policy'), d['control_plane_ms_per_epoch'])"; done
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/bench_kernel_stats.csv && cut -c1-160 $OUT/bench_kernel_stats.csv | head -6
cat $OUT/rehearsal.txt
exit $rc
