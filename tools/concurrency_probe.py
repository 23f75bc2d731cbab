"""Do the 4 pods of an epoch really run side by side?  Launches epochs of 4 Burstable pods
(slots 0/2/4/6) through the real DeviceExecutor, with and without HIP-graph replay, and
prints each pod's start/end (HIP events, relative to the epoch's first start).  Writes
gpurun_out/concurrency.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402

WL = ["onnx_mobilenet_2048", "onnx_resnet50_2048", "tensorflow_ssd_mobilenet_2048", "tensorflow_resnet50_1024"]


def epoch(ex, tag, n_epochs=3):
    eps = [[PodRun(4 * e + i, WL[(i + e) % 4], 2 * i, 2, 20, masked=False) for i in range(4)] for e in range(n_epochs)]
    torch.cuda.synchronize()
    for ep in eps:
        ex.launch_epoch(ep)
    torch.cuda.synchronize()
    t0 = eps[0][0].start
    rows = []
    for e, ep in enumerate(eps):
        for r in ep:
            rows.append({"epoch": e, "slot": r.first_unit // 2, "wl": r.workload,
                         "start_ms": round(t0.elapsed_time(r.start), 3), "end_ms": round(t0.elapsed_time(r.end), 3)})
    print(tag, flush=True)
    for x in rows:
        print("  ", x, flush=True)
    return rows


def main():
    out = {}
    for graphs in (True, False):
        ex = DeviceExecutor(0)
        ex.use_graphs = graphs
        ex.warm([PodRun(0, wl, u, 2, 20, masked=False) for wl in WL for u in (0, 2, 4, 6)])
        epoch(ex, "warm")
        out[f"graphs={graphs}"] = epoch(ex, f"graphs={graphs}")
        ex.close()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/concurrency.json", "w"), indent=1)


if __name__ == "__main__":
    main()
