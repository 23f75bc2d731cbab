#!/bin/bash
# Hardware counters of the bench's kernels over the TIMED region (rocprofv3 --pmc, one pass per
# counter group, each in its own run; kernels are serialised under --pmc, so these are per-kernel
# totals, not co-run).  The bench brackets its timed epochs with marker kernels
# (GPUSCHED_PROFILE_MARKERS) and lists the timed pods for the compulsory-bytes column.
# Summary: tools/pmc_bench_summary.py -> gpurun_out/pmc_bench/summary.json
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PMC_OUT:-pmc_bench}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPUSCHED_PROFILE_MARKERS=$O/timed_pods.json
B="python3 $R/bench.py --steps ${PMC_STEPS:-6} --warmup 1 --control-plane inline --graphs 0 --prewarm-ms 0 ${PMC_ARGS:-}"
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 || exit $?
done
timeout -k 10 60 python3 $R/tools/pmc_bench_summary.py $O
