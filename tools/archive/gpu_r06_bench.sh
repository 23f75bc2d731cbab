#!/bin/bash
# Round 6: the bench at the driver's shape three times and its rocprofv3 kernel statistics (csv).
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/gpurun_out/${BENCH_OUT:-r06_bench}; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r$r.json 2> $O/bench_r$r.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 > $O/rocprof_bench.log 2>&1 || exit $?
echo done
