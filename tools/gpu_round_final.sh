#!/bin/bash
# End-of-round GPU check: the GPU round (tools/gpu_round.sh) and a 2-rank rehearsal on the one
# GPU (gloo, both ranks on device 0): two GPU groups, so the co-run planner with backlog carry and
# measured feedback runs on real pipelined timelines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu_round.sh &&
GPUSCHED_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --backend gloo --steps 40 --warmup 5 \
  --out gpurun_out/rehearsal_2rank.json > gpurun_out/rehearsal_2rank.log 2>&1
rc=$?
python -c "
import json
d=json.load(open('gpurun_out/rehearsal_2rank.json'))
print({k: d.get(k) for k in ('value','ms_per_step','slo_attainment_pct','control_plane_ms_per_epoch')}, {k: d['config'].get(k) for k in ('plan_carry','plan_feedback')})
" 2>/dev/null
exit $rc
