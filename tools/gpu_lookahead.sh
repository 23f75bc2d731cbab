#!/bin/bash
# Epoch lookahead study: 1-GPU bench at lookahead 1/2/3, then 2- and 4-rank rehearsals on
# the one GPU (gloo) at lookahead 1 and 2.  Steps chained with &&.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/la
run1() { timeout -k 10 240 python bench.py --steps 30 --warmup 5 --lookahead $1 --out gpurun_out/la/g1_l$1.json > gpurun_out/la/g1_l$1.log 2>&1; }
runn() { GPUSCHED_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$1 \
  --master-addr 127.0.0.1 --master-port $((29540 + $1 * 10 + $2)) bench.py --gpus $1 --steps 20 --warmup 3 --backend gloo \
  --lookahead $2 --out gpurun_out/la/r$1_l$2.json > gpurun_out/la/r$1_l$2.log 2>&1; }
run1 1 && run1 2 && run1 3 && runn 2 1 && runn 2 2 && runn 4 1 && runn 4 2
rc=$?
for f in gpurun_out/la/*.json; do
  python -c "import json; d=json.load(open('$f')); print('$f', {k:d.get(k) for k in ['value','n_gpus','ms_per_step','gpu_util_pct','slo_attainment_pct','host_ms_per_step_rank0']})"
done
exit $rc
