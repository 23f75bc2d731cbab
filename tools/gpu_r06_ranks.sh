#!/bin/bash
# Round 6: the multi-rank code path on the one-GPU box -- 2 ranks and 8 ranks (gloo, every rank on
# device 0) through bench.py, the driver's N>1 launch shape (torch.distributed.run).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_ranks
GPUSCHED_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --backend gloo --steps 40 --warmup 5 \
  --out gpurun_out/r06_ranks/rehearsal_2rank.json > gpurun_out/r06_ranks/rehearsal_2rank.log 2>&1 || exit $?
bash tools/rehearsal_8rank.sh || exit $?
cp gpurun_out/rehearsal_8rank.json gpurun_out/rehearsal_8rank.log gpurun_out/r06_ranks/
echo done
