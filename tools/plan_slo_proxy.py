"""Predicted-SLO proxy for the burst planner (CPU only, no GPU).

Runs the bench's control plane (parallel.podbench.ControlPlane: apiserver + scheduler +
Poisson workload arrivals at 4 quarter-GPU pods per GPU per epoch) with and without
`planBursts`, and after each epoch counts the pods predicted to meet their SLO under the
interference table: pod `a` on a device meets it when `SLO <= pred(a) - sum intf[a][b]`
over its co-residents `b` (the reference's test, gpu_plugins.go:589-612).  Also reports
the predicted load imbalance (max / mean of the per-GPU alone work) the plan accepts.

    python tools/plan_slo_proxy.py [--gpus 4 8] [--epochs 40]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from k8s_gpu_scheduler_amd.parallel.podbench import NODE, ControlPlane  # noqa: E402


def epoch_stats(cp: ControlPlane):
    pl = cp.plugin
    ok = n = 0
    load = {}
    for st in cp.ledger.devices(NODE):
        uses = list(st.pods.values())
        load[st.device.gpu] = load.get(st.device.gpu, 0.0) + st.work
        for a in uses:
            conf, intf = pl._pod_predictions(a.name)
            pred = conf.get(pl._col(a.units[1], st.device.units), -1.0) if conf else -1.0
            loss = 0.0
            for b in uses:
                if b is not a and intf:
                    c = pl._workload_col(b.name, intf)
                    loss += intf.get(c, 0.0) if c else 0.0
            n += 1
            ok += a.slo <= 0 or not (a.slo > pred - loss)
    vals = list(load.values()) or [0.0]
    mean = sum(vals) / len(vals)
    return ok, n, (max(vals) / mean if mean > 0 else 1.0)


def run(gpus: int, plan: bool, epochs: int, seed: int):
    cp = ControlPlane(n_gpus=gpus, pods_per_gpu=4, iters=20, seed=seed, plan_bursts=plan,
                      learn_interference=False)
    ok = n = 0
    imb = []
    t = 0.0
    for _ in range(epochs):
        cp.finish_live()
        t0 = time.perf_counter()
        cp.schedule_epoch()
        t += time.perf_counter() - t0
        o, k, r = epoch_stats(cp)
        ok, n = ok + o, n + k
        imb.append(r)
    return {"gpus": gpus, "plan": plan, "pred_slo_ok_pct": round(100.0 * ok / max(n, 1), 2), "pods": n,
            "mean_max_over_mean_load": round(sum(imb) / len(imb), 4),
            "sched_ms_per_epoch": round(1e3 * t / epochs, 2), "unscheduled": cp.unscheduled}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, nargs="+", default=[4, 8])
    ap.add_argument("--epochs", type=int, default=40)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    for g in a.gpus:
        for plan in (False, True):
            print(json.dumps(run(g, plan, a.epochs, a.seed)), flush=True)


if __name__ == "__main__":
    main()
