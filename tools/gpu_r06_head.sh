#!/bin/bash
# Round-6 head check: pytest -m gpu, smoke(), the bench at the driver's shape three times, and a
# rocprofv3 kernel-trace profile of the bench (kernel statistics) -- outputs in gpurun_out/r06_head.
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/gpurun_out/r06_head; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r$r.json 2> $O/bench_r$r.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 > $O/rocprof_bench.log 2>&1 || exit $?
echo done
