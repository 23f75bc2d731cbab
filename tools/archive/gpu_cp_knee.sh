#!/bin/bash
# Where the control plane starts pacing the GPUs (box CPU, no GPU touched): the 8-rank rehearsal
# of tools/gpu_cp_rehearsal.sh with the planner pinned at one level and a busy wait of X ms added
# to every epoch's schedule (GPUSCHED_CP_EXTRA_MS) -- the same placements, only a costlier
# control plane.  ms / step stays flat while the control plane keeps up and rises once its
# epoch cost passes what the pipeline hides; the knee sets the effort rule's thresholds.
cd "${GRAFT_REPO_ROOT:-.}"
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= TMPDIR=/tmp
OUT=gpurun_out/${OUT_NAME:-cp_knee}
mkdir -p $OUT
run() {  # name port extra_ms flags...
  local name=$1 port=$2 extra=$3; shift 3
  GPUSCHED_CP_EXTRA_MS=$extra timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --sim-timed --sim-scale 0.8 --steps 60 \
    --warmup 5 "$@" --out $OUT/$name.json > $OUT/$name.log 2>&1 || return $?
  python -c "
import json; d=json.load(open('$OUT/$name.json'))
print('$name', 'extra_ms', $extra, d['value'], d['ms_per_step'], d['control_plane_ms_per_epoch'],
      d.get('control_plane_side_ms_per_epoch'), d['planner'].get('effort_epochs'))" >> $OUT/summary.txt
}
: > $OUT/summary.txt
LEVEL=${LEVEL:-1}
EXTRAS=${EXTRAS:-0 0.8 1.6 2.4}
port=29850
for r in ${ROUNDS:-1 2}; do
  for x in $EXTRAS; do
    port=$((port + 1))
    run l${LEVEL}_x${x}_r$r $port $x --cp-adaptive 0 --plan-effort $LEVEL || exit $?
  done
done
cat $OUT/summary.txt
