#!/bin/bash
# PMC counters of the GEMM tiles (own runs: --pmc only, no trace domains).
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for t in 1 4; do
  timeout -k 10 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/pmc/a_t$t -o run -- python3 $R/tools/gemm_one.py 8192 8192 8192 $t 5 > $R/gpurun_out/pmc/a_t$t.log 2>&1 || exit $?
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc/b_t$t -o run -- python3 $R/tools/gemm_one.py 8192 8192 8192 $t 5 > $R/gpurun_out/pmc/b_t$t.log 2>&1 || exit $?
done
ls -R $R/gpurun_out/pmc | head -30
