#!/bin/bash
# 8 real rank processes on a 1-GPU box (gloo; every rank maps onto device 0 with shared operand
# buffers): samplers, HIP launches, the control-plane process and the planner at the bench
# defaults.  A host-side rehearsal of the driver's 8-GPU run; the GPU itself is shared 8 ways.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp GPUSCHED_FORCE_DEVICE=0 GPUSCHED_SHARED_BUFFERS=1
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 "$@" \
  --out gpurun_out/rehearsal_8rank.json > gpurun_out/rehearsal_8rank.log 2>&1
rc=$?
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/rehearsal_8rank.json"))
except Exception as e:
    print("no result", e); raise SystemExit(0)
print({k: d.get(k) for k in ("value", "ms_per_step", "control_plane_ms_per_epoch", "slo_attainment_pct")})
print("rank0", d.get("host_ms_per_step_rank0"), "cfg", {k: d["config"].get(k) for k in ("plan_carry", "plan_feedback")})
PY
exit $rc
