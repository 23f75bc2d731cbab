#!/bin/bash
# Lone-GEMM counters: this framework's 8-phase kernel vs hipBLASLt on one shape (default
# 8192^3): wall-clock TF/s, a kernel trace (per-dispatch time), and two counter passes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_NAME:-gemm_pmc}
mkdir -p $OUT
SHAPE=${SHAPE:-8192 8192 8192}
for t in ${WALL_TILES:-0 9 10}; do
  GEMM_TILE=$t timeout -k 10 120 python tools/gemm_pmc_probe.py $SHAPE 50 >> $OUT/wall.txt 2>&1 || exit $?
done &&
cd /tmp &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_pmc_probe.py $SHAPE 10 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_pmc_probe.py $SHAPE 5 > $GRAFT_REPO_ROOT/$OUT/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM \
  --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_pmc_probe.py $SHAPE 5 > $GRAFT_REPO_ROOT/$OUT/p2.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
cat $OUT/wall.txt
find $OUT -name "*.csv" | head -20
exit $rc
