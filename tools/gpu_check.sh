#!/bin/bash
# Quick GPU check after a change: pytest -m gpu, smoke, a 1-GPU bench, and the scheduler-only
# throughput on the box CPU with the cycle cache on and off.  Steps chained with &&.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python tools/sched_throughput.py --out gpurun_out/sched_fast.json > gpurun_out/sched_fast.log 2>&1 &&
timeout -k 10 300 python tools/sched_throughput.py --no-fast-path --out gpurun_out/sched_slow.json > gpurun_out/sched_slow.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log 2>/dev/null; grep '^{' gpurun_out/bench.log 2>/dev/null | cut -c1-400
exit $rc
