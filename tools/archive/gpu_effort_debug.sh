cd "${GRAFT_REPO_ROOT:-.}"
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= TMPDIR=/tmp GPUSCHED_EFFORT_DEBUG=1
mkdir -p gpurun_out/effdbg
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29901 bench.py --gpus 8 --sim-timed --sim-scale 0.8 --steps 40 --warmup 5 \
    --out gpurun_out/effdbg/a.json > gpurun_out/effdbg/a.log 2>&1
rc=$?
grep "\[effort\]" gpurun_out/effdbg/a.log | head -60
exit $rc
