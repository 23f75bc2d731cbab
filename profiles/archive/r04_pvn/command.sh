#!/bin/bash
# Round-4 GPU call: RCCL set-check GPU test, the pipelined virtual node on the MI355X (3 seeds),
# and an interleaved N=1 bench A/B of the CU-slot policy at the new defaults.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_pvn
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "rccl_set_check or fabric_probe" > gpurun_out/r04_pvn/pytest_probe.log 2>&1 &&
timeout -k 10 900 python -u tools/pipelined_vn.py --gpus 8 --epochs 48 --warmup 5 --seeds 0 1 2 \
  --out gpurun_out/r04_pvn/pipelined_vn.json > gpurun_out/r04_pvn/pipelined_vn.log 2>&1 &&
timeout -k 10 600 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --timeout 150 --out gpurun_out/r04_pvn/ab20 \
  --arm slots="" --arm balanced="--slot-balance 1 --plan-slots 0" --arm fixed="--plan-slots 0" > gpurun_out/r04_pvn/ab20.log 2>&1
rc=$?
tail -2 gpurun_out/r04_pvn/pytest_probe.log; tail -2 gpurun_out/r04_pvn/pipelined_vn.log | cut -c1-600; tail -1 gpurun_out/r04_pvn/ab20.log | cut -c1-600
exit $rc
