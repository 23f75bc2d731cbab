#!/bin/bash
# GPU check: pytest -m gpu (verbose), the planner direction test twice more with its state
# printed, smoke, and the bench at the driver's shape (20 steps).  Steps are chained with &&
# so nothing else touches the GPU after a failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -m gpu -x -s -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    -k test_planner_feedback_moves_work_off_a_really_slower_gpu > gpurun_out/direction_$i.log 2>&1 || exit 1
done &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1
rc=$?
grep -h '^{' gpurun_out/bench20.log 2>/dev/null | cut -c1-400
tail -3 gpurun_out/pytest_gpu.log; grep -h "measured\|epoch 12\|passed\|failed" gpurun_out/direction_*.log | cut -c1-600
tail -2 gpurun_out/smoke.log 2>/dev/null
exit $rc
