#!/bin/bash
# Box-CPU rehearsal of the 8-GPU bench's control plane (no GPU touched): 8 gloo ranks with the
# timed simulated executor (an epoch occupies a modelled device for its pods' co-run cost, x0.8 =
# ~6.7 ms, the MI355X epoch), the control-plane process on the box CPU at the bench defaults.
# Arms: adaptive effort (the default), with OLD_RULE=1 the round-5-first thresholds (up 0.6 /
# target 0.7), and levels 0 / 1 pinned (--cp-adaptive 0), interleaved.
cd "${GRAFT_REPO_ROOT:-.}"
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= TMPDIR=/tmp
OUT=gpurun_out/${OUT_NAME:-cp_rehearsal}
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
for r in ${ROUNDS:-1 2}; do
  run adapt_r$r $((29800 + r)) &&
  if [ -n "$OLD_RULE" ]; then run adapt06_r$r $((29810 + r)) --cp-effort-up 0.6 --cp-effort-target 0.7; fi &&
  run e0_r$r $((29820 + r)) --cp-adaptive 0 &&
  run e1_r$r $((29830 + r)) --cp-adaptive 0 --plan-effort 1 || exit $?
done
cat $OUT/summary.txt
