"""Do co-running pod streams get equal service?  (co-run model residuals, profiles/r03_corun/)

The co-run model fitted on 2558 measured groups is unbiased for the first three pods of a
4-pod group but predicts the FOURTH-launched pod 24 % too fast.  This probe separates the
candidate causes by running 4 identical pods (one workload) co-located, many times:

  order     slots 0, 2, 4, 6 launched in that order
  reverse   the same slots launched 6, 4, 2, 0 (does the slow one follow the slot's stream
            or the launch position?)
  rotate    launch order rotated every repetition

and reports per slot and per launch position the median pod time.

    python tools/queue_fairness_probe.py [--workload onnx_resnet50_2048] [--reps 12]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
_q = int(os.environ.get("GPUSCHED_HW_QUEUES", "16"))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _q <= 32:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_q)

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402

SLOTS = (0, 2, 4, 6)


def run(ex: DeviceExecutor, wls, order):
    runs = [PodRun(i, wls[i], SLOTS[i], 2, 20, masked=False) for i in range(4)]
    launch = [runs[i] for i in order]
    torch.cuda.synchronize()
    ex.launch_epoch(launch)
    ex.join_current()
    torch.cuda.synchronize()
    return [r.start.elapsed_time(r.end) for r in runs]        # per slot index


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", nargs="+", default=["onnx_resnet50_2048", "tensorflow_mobilenet_2048",
                                                       "onnx_ssd_mobilenet_2048"])
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--out", default="gpurun_out/queue_fairness.json")
    a = ap.parse_args()
    ex = DeviceExecutor(0, use_cu_masks=True)
    ex.use_graphs = True
    ex.warm([PodRun(0, wl, u, 2, 20, masked=False) for wl in W.NAMES for u in SLOTS])
    out = {}
    for wl in a.workloads:
        wls = [wl] * 4
        res = {}
        for mode in ("order", "reverse", "rotate"):
            per_slot = {s: [] for s in range(4)}
            per_pos = {p: [] for p in range(4)}
            for rep in range(a.reps):
                if mode == "order":
                    order = [0, 1, 2, 3]
                elif mode == "reverse":
                    order = [3, 2, 1, 0]
                else:
                    order = [(rep + i) % 4 for i in range(4)]
                ms = run(ex, wls, order)
                for pos, s in enumerate(order):
                    per_slot[s].append(ms[s])
                    per_pos[pos].append(ms[s])
            res[mode] = {"slot_ms": [round(statistics.median(per_slot[s]), 3) for s in range(4)],
                         "launch_pos_ms": [round(statistics.median(per_pos[p]), 3) for p in range(4)]}
            print(wl, mode, res[mode], flush=True)
        out[wl] = res
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    ex.close()


if __name__ == "__main__":
    main()
