"""How late does the host see a pod epoch finish?  (profiles/archive/r03_window/)

The 1-rank plain bench path collected every epoch ~6 ms after its last pod kernel ended
(pod timelines, GPUSCHED_BENCH_TRACE), the 1-rank RCCL path within 0.1 ms.  This probe runs
the bench's executor (graphs, per-pod streams, 2-deep launch-ahead) with different host wait
strategies and reports, per strategy, the lag between an epoch's last pod end (HIP event
timestamp) and the host noticing it:

  sync        r.end.synchronize()                  (blocking hipEventSynchronize)
  poll        r.end.query() + 20 us sleeps
  spin        r.end.query() busy loop
  side_sync   poll, and every poll a synchronize of an empty side stream
  side_query  poll, and every poll a query of an empty side stream's event
  bcast       a 1-rank RCCL group; per epoch a broadcast + D2H on the side stream (what the
              RCCL bench path does), then sync

    python tools/event_lag_probe.py [--epochs 40] [--out gpurun_out/event_lag.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
_q = int(os.environ.get("GPUSCHED_HW_QUEUES", "16"))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _q <= 32:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_q)

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402


def run(ex: DeviceExecutor, side, mode: str, epochs: int, rng: random.Random, dist=None, cp=None):
    lags = []
    torch.cuda.synchronize()
    ref = torch.cuda.Event(enable_timing=True)
    ref.record(side)
    ref.synchronize()
    t_ref = time.perf_counter()
    pending = []
    buf = torch.zeros(64, dtype=torch.int32, device="cuda") if dist is not None else None
    ev_side = torch.cuda.Event()

    def wait(runs):
        for r in runs:
            ev = r.end
            if mode == "sync":
                ev.synchronize()
            elif mode == "spin":
                while not ev.query():
                    pass
            else:
                while not ev.query():
                    if mode == "side_sync":
                        side.synchronize()
                    elif mode == "side_query":
                        ev_side.record(side)
                        ev_side.query()
                    time.sleep(20e-6)
        t = time.perf_counter()
        end = max(ref.elapsed_time(r.end) for r in runs)
        lags.append((t - t_ref) * 1e3 - end)

    for e in range(epochs):
        runs = [PodRun(i, rng.choice(W.NAMES), 2 * i, 2, 20, masked=False) for i in range(4)]
        if dist is not None:
            with torch.cuda.stream(side):
                buf.copy_(torch.arange(64, dtype=torch.int32))
                dist.broadcast(buf, 0)
                buf.cpu()
        if cp is not None:
            cp.request_schedule()          # the bench's order: ask, launch, collect, receive
        ex.launch_epoch(runs)
        pending.append(runs)
        while len(pending) > 2:
            wait(pending.pop(0))
        if cp is not None:
            cp.get_schedule()
    while pending:
        wait(pending.pop(0))
    return lags


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=40)
    ap.add_argument("--modes", nargs="+", default=["sync", "poll", "spin", "side_sync", "side_query", "bcast"])
    ap.add_argument("--out", default="gpurun_out/event_lag.json")
    ap.add_argument("--smi-period-ms", type=float, default=0.0,
                    help="run the bench's amd-smi activity sampler thread meanwhile (0 = off)")
    ap.add_argument("--control-plane", action="store_true",
                    help="also run the bench's control-plane process, asked for a schedule every epoch")
    a = ap.parse_args()
    cp = None
    if a.control_plane:        # spawned before anything touches the GPU, as in the bench
        from k8s_gpu_scheduler_amd.parallel.controlplane_proc import ControlPlaneProc
        cp = ControlPlaneProc(n_gpus=1, pods_per_gpu=4, iters=20, seed=0)
        cp.schedule_epoch()
    smi = None
    if a.smi_period_ms > 0:
        from k8s_gpu_scheduler_amd.telemetry.smi_sampler import ActivitySampler
        smi = ActivitySampler([0], a.smi_period_ms / 1e3)
        print("smi sampler", smi.start(), flush=True)
    ex = DeviceExecutor(0, use_cu_masks=True)
    ex.use_graphs = True
    ex.warm([PodRun(0, wl, u, 2, 20, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])
    side = torch.cuda.Stream()
    out = {}
    rng = random.Random(0)
    for mode in a.modes:
        dist = None
        if mode == "bcast":
            import torch.distributed as td
            from k8s_gpu_scheduler_amd.parallel.launch import free_port
            td.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", world_size=1, rank=0,
                                  device_id=torch.device("cuda", 0))
            dist = td
        lags = run(ex, side, "sync" if mode == "bcast" else mode, a.epochs, rng, dist, cp)
        body = lags[3:]
        out[mode] = {"median_ms": round(statistics.median(body), 3), "max_ms": round(max(body), 3),
                     "min_ms": round(min(body), 3), "last_epoch_ms": round(lags[-1], 3)}
        print(mode, out[mode], flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    if smi is not None:
        smi.stop()
    if cp is not None:
        cp.close()
    ex.close()


if __name__ == "__main__":
    main()
