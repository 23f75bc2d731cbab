#!/bin/bash
# Measure the MI355X configuration/interference tables, then bench with them.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/data
timeout -k 10 500 python -m k8s_gpu_scheduler_amd.models.profile --out gpurun_out/data > gpurun_out/profile.log 2>&1 &&
cp gpurun_out/data/*.tsv k8s_gpu_scheduler_amd/data/ &&
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --out gpurun_out/b_measured.json > gpurun_out/b_measured.log 2>&1
rc=$?
tail -2 gpurun_out/profile.log
python -c "import json; d=json.load(open('gpurun_out/b_measured.json')); print({k:d.get(k) for k in ['value','ms_per_step','gpu_util_pct','mfma_util_pct','achieved_tflops','slo_attainment_pct','host_ms_per_step_rank0']})"
exit $rc
