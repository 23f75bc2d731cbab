#!/bin/bash
# Round 5: extra workloads through the executor (GPU test), the CU fill from a real rocprofv3
# kernel trace vs the tile picker's (models.workloads.cu_fill), and the timed-region PMC pass.
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
O=$R/gpurun_out/r05_fill
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native.py \
  -k "extra_workloads or graph_replay" > $O/pytest.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && export PYTHONPATH=$R
for w in fp8_llm_2048 onnx_resnet50_2048 tensorflow_resnet50_4096 onnx_ssd_mobilenet_2048; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$w -o run -- \
    python3 -m k8s_gpu_scheduler_amd.ops.podrun --workload $w --iters 5 --cu-budget 64 > $O/$w.log 2>&1 || exit $?
done
O_DIR=$O timeout -k 10 60 python3 - > $O/fill.txt 2>&1 <<'PY' || exit $?
import glob, os
from k8s_gpu_scheduler_amd.agent.pod_profiler import summarize_kernel_trace
from k8s_gpu_scheduler_amd.models import workloads as W
O = os.environ.get("O_DIR", "")
for w in ("fp8_llm_2048", "onnx_resnet50_2048", "tensorflow_resnet50_4096", "onnx_ssd_mobilenet_2048"):
    f = glob.glob(f"{O}/{w}/**/*kernel_trace.csv", recursive=True)
    s = summarize_kernel_trace(f[0]) if f else {}
    print(w, "trace cu_fill", s.get("cu_fill"), "picker (roofline-weighted)", round(W.cu_fill(W.get(w)), 4), flush=True)
PY
cd $R && PMC_OUT=r05_pmc bash tools/gpu_pmc_bench.sh
