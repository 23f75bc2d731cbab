#!/bin/bash
# A/B of the burst planner in the 8-rank CPU rehearsal (gloo ranks, timed simulated
# executor; no GPU): plan off, plan with load tolerance 0.05 and 0.0.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
N=${1:-8}
: > gpurun_out/plan_ab.txt
for cfg in "0 0.05" "1 0.05" "1 0.0"; do
  set -- $cfg
  tag=p$1_t$2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29755 bench.py --gpus $N --sim-timed --steps 40 --warmup 5 --plan-bursts $1 --plan-tolerance $2 \
    --out gpurun_out/plan_ab_$tag.json > gpurun_out/plan_ab_$tag.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/plan_ab_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['sched_ms_per_pod'], d['host_ms_per_step_rank0'])" >> gpurun_out/plan_ab.txt
done
cat gpurun_out/plan_ab.txt
