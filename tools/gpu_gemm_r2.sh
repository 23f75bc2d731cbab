#!/bin/bash
# GEMM round 2: tile tests + race screen, lone-GEMM table (tiles 1/4/9/10 vs hipBLASLt), PMC
# passes (own runs, --pmc only) of the 8-phase kernels at 8192^3.
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
timeout -k 10 200 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/gemm_test.log 2>&1 || exit $?
GEMM_BIG_ARMS=1,4,9,10 timeout -k 10 300 python -u tools/gemm_big.py > gpurun_out/gemm_big.log 2>&1 || exit $?
cd /tmp
for t in 9 10; do
  timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc2/a_t$t -o run -- python3 $R/tools/gemm_one.py 8192 8192 8192 $t 5 > $R/gpurun_out/pmc2/a_t$t.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmc2/b_t$t -o run -- python3 $R/tools/gemm_one.py 8192 8192 8192 $t 5 > $R/gpurun_out/pmc2/b_t$t.log 2>&1 || exit $?
done
cat $R/gpurun_out/gemm_big.log
