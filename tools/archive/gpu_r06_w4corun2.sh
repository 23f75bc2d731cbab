#!/bin/bash
# Round 6: arm 10 (co-running 256x256 GEMMs on the 4-wave kernel) confirmation -- GPU numerics of
# the arm, then 5 interleaved bench rounds of arm 1, arm 10 and arm 10 with whole-kernel priority.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_w4corun2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "policy10 or (8phase_numerics_and_race_screen and 14)" -p no:cacheprovider > $O/numerics.log 2>&1 || exit $?
for r in 1 2 3 4 5; do
  for arm in "1 0" "10 0" "10 1"; do
    set -- $arm
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $1 --w4-prio $2 > $O/b_p$1_prio$2_r$r.json 2> $O/b_p$1_prio$2_r$r.err || exit $?
  done
done
echo done
