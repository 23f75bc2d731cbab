#!/bin/bash
# Round-5 cold-start broadening + the timed-region PMC pass (item 7).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05_coldstart
mkdir -p $O
timeout -k 10 600 python3 -u tools/corun_extra_groups.py --out $O/groups.json > $O/collect.log 2>&1 &&
timeout -k 10 120 python3 tools/corun_extra_eval.py $O/groups.json --out $O/extra.json > $O/eval.log 2>&1 &&
PMC_OUT=r05_pmc bash tools/gpu_pmc_bench.sh
