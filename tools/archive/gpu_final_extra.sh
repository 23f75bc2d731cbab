cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out/r05_final_extra
OUT_NAME=cp_rehearsal_r05e bash tools/gpu_cp_rehearsal.sh > gpurun_out/r05_final_extra/rehearsal.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 60 --warmup 5 > gpurun_out/r05_final_extra/bench60.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_final_extra/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --prewarm-ms 0 > $R/gpurun_out/r05_final_extra/prof.log 2>&1
