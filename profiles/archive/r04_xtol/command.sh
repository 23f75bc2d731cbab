#!/bin/bash
# Round-4 GPU call: interference-aware slot levelling at N=1 (GPUSCHED_LPT_XTOL: among the slots
# within xtol x the pod's predicted work of the least loaded stream, the one with the least
# predicted coupling to the other slots' overlapping pods) against plain levelling, 4 rounds.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_xtol
mkdir -p $OUT
timeout -k 10 1000 python tools/ab.py --rounds 4 --steps 20 --warmup 5 --timeout 150 --out $OUT \
  --arm base="" --arm x06="GPUSCHED_LPT_XTOL=0.6" --arm x10="GPUSCHED_LPT_XTOL=1.0" > $OUT/ab.log 2>&1
rc=$?
tail -1 $OUT/ab.log | cut -c1-1500
exit $rc
