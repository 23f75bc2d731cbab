cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
GPUSCHED_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo \
  --out gpurun_out/b_2rank.json > gpurun_out/b_2rank.log 2>&1 &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
python -c "import json; d=json.load(open('gpurun_out/b_2rank.json')); print({k:d.get(k) for k in ['value','n_gpus','ms_per_step','gpu_util_pct','config']})"
tail -3 gpurun_out/pytest_gpu.log
exit $rc
