#!/bin/bash
# Round-4 GPU call 3: the GPU test suite at HEAD, then an interleaved N=1 A/B of who picks the
# CU slot: the scheduler's LPT (default), the executor's LPT re-slotting (round 3), the co-run
# model's slot plan and the ledger's first fit.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_slots
timeout -k 10 300 python tools/cp_timing.py > gpurun_out/r04_slots/cp_timing_box.txt 2>&1 &&
GPUSCHED_PLAN_THREADS=1 timeout -k 10 300 python tools/cp_timing.py > gpurun_out/r04_slots/cp_timing_box_1thread.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04_slots/pytest_gpu.log 2>&1 &&
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --timeout 150 --out gpurun_out/r04_slots/ab20 \
  --arm auto="" --arm executor="--slot-balance 1 --plan-slots off" --arm model="--plan-slots model" \
  --arm off="--plan-slots off" > gpurun_out/r04_slots/ab20.log 2>&1 &&
timeout -k 10 900 python -u tools/pipelined_vn.py --gpus 8 --epochs 48 --warmup 5 --seeds 0 1 2 --passes 4 \
  --policies greedy planner --out gpurun_out/r04_slots/pipelined_vn.json > gpurun_out/r04_slots/pipelined_vn.log 2>&1
rc=$?
tail -4 gpurun_out/r04_slots/cp_timing_box.txt gpurun_out/r04_slots/cp_timing_box_1thread.txt; tail -3 gpurun_out/r04_slots/pytest_gpu.log; tail -1 gpurun_out/r04_slots/ab20.log | cut -c1-1200; tail -1 gpurun_out/r04_slots/pipelined_vn.log | cut -c1-900
exit $rc
