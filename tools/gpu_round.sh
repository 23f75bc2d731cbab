#!/bin/bash
# GPU test round: pytest -m gpu, smoke, the bench at the driver's shape (20 steps) and at 60 steps,
# a rocprofv3 kernel-trace profile of the bench.
# Steps are chained with && so nothing else touches the GPU after a failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 > gpurun_out/bench60.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/bench_prof.log 2>&1
rc=$?
grep -h '^{' gpurun_out/bench20.log gpurun_out/bench60.log 2>/dev/null | cut -c1-300
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log 2>/dev/null; grep '^{' gpurun_out/bench_prof.log 2>/dev/null | cut -c1-300
exit $rc
