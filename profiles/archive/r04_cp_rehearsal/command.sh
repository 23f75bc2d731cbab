#!/bin/bash
# Round-4 box-CPU rehearsal of the 8-GPU bench's control plane (no GPU touched): 8 gloo ranks with
# the timed simulated executor (an epoch occupies a modelled device for its pods' co-run cost,
# x0.8 = ~6.7 ms, the MI355X epoch), the control-plane process on the box CPU at the bench defaults.
# Arms: adaptive effort (down at 85 % of the period, the default; and at 95 %), and each effort
# level pinned (--cp-adaptive 0). Two interleaved rounds. ARMS=jump: the jump-to-fit rule.
cd "${GRAFT_REPO_ROOT:-.}"
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= TMPDIR=/tmp
OUT=gpurun_out/r04_cp_rehearsal
mkdir -p $OUT
run() {  # name port flags...
  local name=$1 port=$2; shift 2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 8 --sim-timed --sim-scale 0.8 --steps 60 --warmup 5 "$@" \
    --out $OUT/$name.json > $OUT/$name.log 2>&1 || return $?
  python -c "
import json; d=json.load(open('$OUT/$name.json'))
print('$name', d['value'], d['ms_per_step'], d['control_plane_ms_per_epoch'], d['planner'].get('effort_epochs'), d['slo_attainment_pct'])" >> $OUT/summary.txt
}
: > $OUT/summary.txt
ARMS=${ARMS:-full}
if [ "$ARMS" = full ]; then
for r in 1 2; do
  run adapt85_r$r $((29800 + r)) &&
  run adapt95_r$r $((29810 + r)) --cp-effort-down 0.95 &&
  run e0_r$r $((29820 + r)) --cp-adaptive 0 &&
  run e1_r$r $((29830 + r)) --cp-adaptive 0 --plan-effort 1 &&
  run e2_r$r $((29840 + r)) --cp-adaptive 0 --plan-effort 2 || exit $?
done
else
# the jump-to-fit adaptive rule against pinned levels, at the driver's shape (20 steps) and 60 steps
for r in 1 2; do
  run adapt_s20_r$r $((29850 + r)) --steps 20 &&
  run e2_s20_r$r $((29860 + r)) --steps 20 --cp-adaptive 0 --plan-effort 2 &&
  run adapt_s60_r$r $((29870 + r)) &&
  run e1_s60_r$r $((29880 + r)) --cp-adaptive 0 --plan-effort 1 &&
  run e2_s60_r$r $((29890 + r)) --cp-adaptive 0 --plan-effort 2 || exit $?
done
fi
cat $OUT/summary.txt
