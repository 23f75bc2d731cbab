#!/bin/bash
# Hardware counters of the bench's kernels (rocprofv3 --pmc, one pass per counter group, each in
# its own run; kernels are serialised under --pmc, so these are per-kernel totals, not co-run).
# Summary: tools/pmc_bench_summary.py -> gpurun_out/pmc_bench/summary.json
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_bench
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 4 --warmup 1 --control-plane inline --graphs 0 --prewarm-ms 0"
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_bench/p$i -o run -- $B > $R/gpurun_out/pmc_bench/p$i.log 2>&1 || exit $?
done
timeout -k 10 60 python3 $R/tools/pmc_bench_summary.py $R/gpurun_out/pmc_bench
