#!/bin/bash
# 1-GPU bench (control plane in its own process) + a 2-rank rehearsal of the distributed
# path on the same GPU (gloo; RCCL refuses two ranks on one device).  Chained with &&.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --out gpurun_out/b_proc.json > gpurun_out/b_proc.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --control-plane inline --out gpurun_out/b_inline.json > gpurun_out/b_inline.log 2>&1 &&
GPUSCHED_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo \
  --out gpurun_out/b_2rank.json > gpurun_out/b_2rank.log 2>&1
rc=$?
for f in gpurun_out/b_proc.json gpurun_out/b_inline.json gpurun_out/b_2rank.json; do
  [ -f $f ] && python -c "import json; d=json.load(open('$f')); print('$f', {k:d.get(k) for k in ['value','n_gpus','ms_per_step','gpu_util_pct','mfma_util_pct','slo_attainment_pct','sched_ms_per_pod','host_ms_per_step_rank0']})"
done
[ $rc -ne 0 ] && tail -20 gpurun_out/b_2rank.log
exit $rc
