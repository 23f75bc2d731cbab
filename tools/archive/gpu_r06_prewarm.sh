#!/bin/bash
# Round 6: pre-warm load A/B (GEMM + stream mix vs GEMM only), interleaved, and a rocprofv3
# kernel trace of the bench with the timed-region markers (tools/trace_kernel_summary.py).
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/gpurun_out/r06_prewarm; mkdir -p $O
for r in 1 2 3; do
  for k in mix gemm; do
    timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --prewarm-kind $k > $O/${k}_r$r.json 2> $O/${k}_r$r.err || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
export GPUSCHED_PROFILE_MARKERS=$O/timed_pods.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 > $O/rocprof_bench.log 2>&1 || exit $?
echo done
