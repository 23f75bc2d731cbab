#!/bin/bash
# Per-dispatch clock and MFMA busy of the own 8192^3 kernel vs hipBLASLt (own --pmc runs with
# --kernel-trace only, one counter group per pass).
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/clk
cd /tmp && export TMPDIR=/tmp
S="${1:-8192 8192 8192}"
TILE="${TILE:-10}"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/clk/a -o run -- python3 $R/tools/gemm_clock_one.py $S $TILE 10 > $R/gpurun_out/clk/a.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/clk/b -o run -- python3 $R/tools/gemm_clock_one.py $S $TILE 10 > $R/gpurun_out/clk/b.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/clk/t -o run -- python3 $R/tools/gemm_clock_one.py $S $TILE 10 > $R/gpurun_out/clk/t.log 2>&1
rc=$?
ls -R $R/gpurun_out/clk | head -30
exit $rc
