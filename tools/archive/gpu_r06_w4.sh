#!/bin/bash
# Round-6 lone-GEMM study on one MI355X: tile 14 (4-wave 256x256, AGPR-tied MFMAs, 5-slot ring)
# numerics race screen, numerics + wall TF/s next to tile 10 and hipBLASLt on the lone shapes,
# the timing probes, and the two counter passes of profiles/r05_lone_gemm_pmc/ on tile 14.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/w4final
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "8phase_numerics_and_race_screen" -p no:cacheprovider > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/gemm_w4_check.py 30 > $OUT/check.log 2>&1 &&
timeout -k 10 200 python -u tools/gemm_w4_probe.py 8192 8192 8192 30 > $OUT/probe.log 2>&1 &&
cd /tmp &&
GEMM_TILE=14 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_pmc_probe.py 8192 8192 8192 5 > $GRAFT_REPO_ROOT/$OUT/p1.log 2>&1 &&
GEMM_TILE=14 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM \
  --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_pmc_probe.py 8192 8192 8192 5 > $GRAFT_REPO_ROOT/$OUT/p2.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -3 $OUT/pytest.log
grep -v amdgpu.ids $OUT/probe.log | grep "round 2"
exit $rc
