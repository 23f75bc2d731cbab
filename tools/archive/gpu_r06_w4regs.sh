#!/bin/bash
# Round 6: tile 14 at 385 registers (one A fragment set, bias folded into the accumulator start):
# numerics, lone timing, and 4 interleaved bench rounds of arm 10 against arm 1 (unchanged).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_w4regs; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "policy10 or policy11 or (8phase_numerics_and_race_screen and (14 or 15))" -p no:cacheprovider > $O/numerics.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/gemm_w4_check.py 20 > $O/check.log 2>&1 || exit $?
for r in 1 2 3 4; do
  for p in 10 1; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --gemm-policy $p > $O/b_p${p}_r$r.json 2> $O/b_p${p}_r$r.err || exit $?
  done
done
echo done
