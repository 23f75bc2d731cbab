#!/bin/bash
# Interleaved A/B of the CU-slot policy at N=1: executor LPT balancing (round-3 default), the
# scheduler's slot plan on the pipeline (plan_slots), and the scheduler's first-fit slots.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_slots_ab}
timeout -k 10 700 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --timeout 150 --out ${OUT}20 \
  --arm balanced="--slot-balance 1" --arm slots2="--slot-balance 0 --plan-slots 1 --slot-spread-ms 2" \
  --arm slots4="--slot-balance 0 --plan-slots 1 --slot-spread-ms 4" --arm fixed="--slot-balance 0" > ${OUT}20.log 2>&1 &&
timeout -k 10 500 python tools/ab.py --rounds 1 --steps 60 --warmup 5 --timeout 150 --out ${OUT}60 \
  --arm balanced="--slot-balance 1" --arm slots2="--slot-balance 0 --plan-slots 1 --slot-spread-ms 2" \
  --arm slots4="--slot-balance 0 --plan-slots 1 --slot-spread-ms 4" --arm fixed="--slot-balance 0" > ${OUT}60.log 2>&1
