#!/bin/bash
# hipGraph A/B: graph-replay test, then the 1-GPU bench eager vs graphs (Burstable and Guaranteed).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gr
timeout -k 10 300 python -m pytest tests/test_gpu_native.py -x -q -k "graph_replay or executor_epoch" > gpurun_out/gr/pytest.log 2>&1 &&
for q in burstable guaranteed; do for g in 0 1; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --qos $q --graphs $g --out gpurun_out/gr/${q}_g$g.json > gpurun_out/gr/${q}_g$g.log 2>&1 || exit $?
done; done
rc=$?
tail -2 gpurun_out/gr/pytest.log
for f in gpurun_out/gr/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', {k:d.get(k) for k in ['value','ms_per_step','gpu_util_pct','host_ms_per_step_rank0']})"; done
exit $rc
