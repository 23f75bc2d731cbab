"""Container entrypoint of a synthetic pod: run one catalog (or extra) workload on the GPU the pod got.

    python -m k8s_gpu_scheduler_amd.ops.podrun --workload onnx_resnet50_1024 [--iters N]

The device comes from the container env the scheduler wrote (ROCR_VISIBLE_DEVICES /
HIP_VISIBLE_DEVICES, and HSA_CU_MASK for a Guaranteed share -- the ROCm runtime applies
them, so the process simply uses device 0); iterations default to the pod's ITERATIONS env.
The workload is the same kernel mix the bench's executor runs (models.workloads: native
MFMA GEMMs and HBM stream triads), and the GEMM tiles are sized for the pod's CU share
(`GPU_SCHED_CU` when set).  Prints one JSON line: workload, iterations, wall ms, throughput.
This is what the e2e tests and the profiling webhook's GPU test launch as a "container".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--workload", required=True)
    ap.add_argument("--iters", type=int, default=0, help="default: the ITERATIONS env, else 20")
    ap.add_argument("--cu-budget", type=int, default=0, help="GEMM tile sizing: the pod's CU share (0 = whole GPU)")
    a = ap.parse_args(argv)
    import torch
    from ..models import workloads as W
    from ..parallel.executor import _Buffers, enqueue_ops
    try:
        w = W.get(a.workload)
    except KeyError:
        print(f"unknown workload {a.workload!r}", file=sys.stderr)
        return 2
    iters = a.iters or int(float(os.environ.get("ITERATIONS", "0") or 0)) or 20
    budget = a.cu_budget or int(os.environ.get("GPU_SCHED_CU", "0") or 0)
    torch.cuda.set_device(0)
    bufs = _Buffers(w, torch.device("cuda", 0))
    st = torch.cuda.current_stream()

    def run(n: int) -> None:
        enqueue_ops(bufs, n, st, budget)

    run(1)                                   # first launch: code objects, allocations
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(iters)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"workload": a.workload, "iters": iters, "ms": round(ms, 3),
                      "throughput": round(iters / (ms / 1e3), 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
