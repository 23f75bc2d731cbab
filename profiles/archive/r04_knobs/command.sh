#!/bin/bash
# Round-4 GPU call: kernel-side knobs re-checked under the round-4 defaults (scheduler slot
# levelling), for SLOs met as well as pods/s -- earlier rounds chose them on pods/s alone:
# 128x128 tiles for co-running pods (--gemm-policy 0), the 8x-unrolled stream kernel
# (--triad-variant 4), 2 tile rows per XCD group (--xcd-group 2). Interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_knobs
mkdir -p $OUT
timeout -k 10 1000 python tools/ab.py --rounds 3 --steps 20 --warmup 5 --timeout 150 --out $OUT \
  --arm base="" --arm gp0="--gemm-policy 0" --arm tv4="--triad-variant 4" --arm xg2="--xcd-group 2" \
  > $OUT/ab.log 2>&1
rc=$?
tail -8 $OUT/ab.log | cut -c1-1500
exit $rc
