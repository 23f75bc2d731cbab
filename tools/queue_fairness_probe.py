"""Do co-running pod streams get equal service from the hardware?

The co-run model fitted on 2558 measured groups was unbiased for the first three pods of a
4-pod group but predicted the fourth 24 % too fast, and in the virtual-node runs the pod on
the fourth stream met its SLO 10 % of the time against 60-98 % for the others.  This probe
found why (profiles/archive/r03_queue_fairness/README.md): the tools waited for a group by making
the DEFAULT stream wait on the pods' end events.  That stream-wait sits as a pending barrier
packet on the default stream's hardware queue while the pods run.  The pod stream whose
queue shares a hardware pipe with it -- the 4th pod stream to get its first graph captured
-- is then served at about half rate.  Waiting from the host (executor.wait_all) makes the
4 streams equal and the 4-pod group 40 % shorter.

Runs P identical pods co-located, each on its own stream, many times; prints per-stream
median ms and the group makespan:

  --join          wait with a default-stream barrier (the old way) instead of from the host
  --sac-before N  warm one extra, never-run pod right before pod N (it takes N's pipe slot)
  --warm-reverse  create streams / buffers / graphs in reverse pod order
  --rotate        rotate the launch order every repetition
  --masked        Guaranteed pods (disjoint CU masks)
  --alone         also time one pod alone

    GPU_MAX_HW_QUEUES=16 python tools/queue_fairness_probe.py --pods 4 [--join]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", nargs="+", default=["onnx_resnet50_2048", "onnx_ssd_mobilenet_2048"])
    ap.add_argument("--pods", type=int, default=4)
    ap.add_argument("--join", action="store_true")
    ap.add_argument("--sac-before", type=int, default=-1)
    ap.add_argument("--warm-reverse", action="store_true")
    ap.add_argument("--rotate", action="store_true")
    ap.add_argument("--masked", action="store_true")
    ap.add_argument("--alone", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ex = DeviceExecutor(0, use_cu_masks=a.masked, units_per_gpu=max(8, a.pods + 1))
    wd = max(1, 8 // a.pods) if a.masked else 1

    def pod(i: int, wl: str) -> PodRun:
        return PodRun(i, wl, i * wd, wd, 20, masked=a.masked)

    ex.use_graphs = True
    order_w = list(range(a.pods - 1, -1, -1) if a.warm_reverse else range(a.pods))
    if a.sac_before >= 0:
        i = order_w.index(a.sac_before)
        order_w = order_w[:i] + [a.pods] + order_w[i:]
    ex.warm([pod(u, wl) for wl in a.workloads for u in order_w])
    res = {"hw_queues_env": os.environ.get("GPU_MAX_HW_QUEUES"), "pods": a.pods, "join": a.join,
           "sac_before": a.sac_before, "warm_reverse": a.warm_reverse, "rotate": a.rotate, "masked": a.masked,
           "tag": a.tag, "workloads": {}}
    for wl in a.workloads:
        per = {u: [] for u in range(a.pods)}
        span = []
        for rep in range(a.reps):
            runs = [pod(u, wl) for u in range(a.pods)]
            order = [(rep + i) % a.pods for i in range(a.pods)] if a.rotate else list(range(a.pods))
            torch.cuda.synchronize()
            ex.launch_epoch([runs[i] for i in order])
            if a.join:
                cur = torch.cuda.current_stream()
                for r in runs:
                    cur.wait_event(r.end)
            else:
                ex.wait_all()
            torch.cuda.synchronize()
            for r in runs:
                per[r.pod_id].append(r.start.elapsed_time(r.end))
            t0 = runs[order[0]].start
            span.append(max(t0.elapsed_time(r.end) for r in runs) - min(t0.elapsed_time(r.start) for r in runs))
        med = [round(statistics.median(per[u]), 3) for u in range(a.pods)]
        rec = {"stream_ms": med, "max_over_min": round(max(med) / min(med), 3),
               "group_makespan_ms": round(statistics.median(span), 3)}
        if a.alone:
            al = []
            for rep in range(a.reps):
                r = pod(0, wl)
                torch.cuda.synchronize()
                ex.launch_epoch([r])
                ex.wait_all()
                al.append(r.start.elapsed_time(r.end))
            rec["alone_ms"] = round(statistics.median(al), 3)
        res["workloads"][wl] = rec
        print(a.tag, wl, rec, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)
    ex.close()


if __name__ == "__main__":
    main()
