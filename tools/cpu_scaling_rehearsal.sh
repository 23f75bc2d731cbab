#!/bin/bash
# CPU-only rehearsal of the N-GPU bench on the box's CPUs: gloo ranks, simulated executor
# that sleeps out a modelled device time per epoch (co-run rates measured on MI355X), so
# the control-plane process and the per-epoch placement broadcast are exercised at the
# 8-GPU epoch rate.  No GPU is touched.  Usage: tools/cpu_scaling_rehearsal.sh [balance]
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
B=${1:-1}
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
: > gpurun_out/cpu_rehearsal.txt
for n in 1 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --sim-timed --sim-scale ${SIM_SCALE:-1.0} --steps 40 --warmup 5 --balance $B \
    --out gpurun_out/cpu_rehearsal_$n.json > gpurun_out/cpu_rehearsal_$n.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/cpu_rehearsal_$n.json'));print($n, d['value'], d['ms_per_step'], d['sched_ms_per_pod'], d['control_plane_ms_per_epoch'], (d.get('planner') or {}).get('effort_epochs'), d['host_ms_per_step_rank0'])" >> gpurun_out/cpu_rehearsal.txt
done
cat gpurun_out/cpu_rehearsal.txt
