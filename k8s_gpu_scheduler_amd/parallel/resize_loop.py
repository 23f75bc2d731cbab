"""BASELINE config 5: the recommender resize loop under Poisson pod arrivals.

Users over-request: every arriving pod asks for `--request-cu` CUs (default 128 = half an
MI355X) and twice the HBM its workload uses, with an SLO drawn like the main bench's.  Each
epoch:

  1. Poisson(`--rate` x GPUs) new pods are CREATED; with `--resize` the mutating admission
     (recommender.admission.ResizeAdmission) rewrites their requests from the workload's
     measured history -- the smallest CU share that still meets the SLO, HBM p95 + headroom;
  2. the scheduler places what fits (pods that do not fit stay pending and are retried the
     next epoch -- the backlog);
  3. the executor runs the placed pods (Guaranteed QoS: hard CU masks, so a pod's measured
     throughput belongs to its share) on the GPU -- or the roofline model with --sim;
  4. each finished pod is reported the way a node sees it -- a GPU process with its VRAM,
     CU occupancy and (executor-known) throughput -- and the real node agent
     (agent.NodeAgent.pod_usage / record_history: process -> pod attribution through the
     apiserver, history keyed by workload) appends it to Redis, where the admission reads
     it; then the pod is deleted.
     `--history rocprof` (GPU): the pods are real containers-as-processes instead
     (ops.podrun through the kubelet-style launcher), wrapped in rocprofv3 by the profiling
     webhook chained behind the resize admission, and the history comes from the node
     agent's ProfileIngestor reading their rocprofv3 output (agent.profile_webhook) --
     the deployed path, with kernel-level samples (throughput = iterations / kernel span).

Reported per run: pods completed/s, mean CU request at admission, SLO attainment, backlog,
GPU CU-share occupancy -- with and without the loop.

  python -m k8s_gpu_scheduler_amd.parallel.resize_loop [--sim] [--gpus 8] [--epochs 40] [--no-resize]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import random
import time
from typing import Any, Dict, List, Optional

import numpy as np

from ..api import constants as C
from ..api import objects as O
from ..framework.config import default_gpu_config
from ..framework.scheduler import Scheduler
from ..kube.client import FakeCluster
from ..models import workloads as W
from ..plugins import full_registry
from ..plugins.gpu.devices import CUS_PER_XCD, DeviceLedger
from ..recommender.admission import RedisHistory, ResizeAdmission, workload_key
from ..store.fake_redis import FakeRedisBackend, FakeRedisEngine
from ..store.resp import Redis
from .podbench import SimExecutor, analytic_predictions, measured_predictions

NODE = "mi355x-0"


class ExecutorProcessSource:
    """The executor's finished pods as the agent's device source would list them: one
    "process" per pod on its device (pid -> pod uid through `uid_of`, like a cgroup)."""

    def __init__(self, ledger: DeviceLedger, node: str):
        self.ledger, self.node = ledger, node
        self.procs: Dict[str, List[Dict[str, Any]]] = {}
        self._uid: Dict[int, str] = {}
        self._pid = 1000

    def devices(self) -> List[Dict[str, Any]]:
        return [d.device.to_json() for d in self.ledger.devices(self.node)]

    def processes(self, index: int) -> List[Dict[str, Any]]:
        devs = self.devices()
        return list(self.procs.get(devs[index]["uuid"], [])) if 0 <= index < len(devs) else []

    def report(self, uuid: str, pod_uid: str, vram_gib: float, cus: int, throughput: float) -> None:
        self._pid += 1
        self._uid[self._pid] = pod_uid
        self.procs.setdefault(uuid, []).append({"pid": self._pid, "vram_bytes": int(vram_gib * 2**30),
                                                "cu_occupancy": cus, "throughput": throughput})

    def uid_of(self, pid: int) -> Optional[str]:
        return self._uid.get(pid)

    def clear(self) -> None:
        self.procs.clear()
        self._uid.clear()


def _poisson(rng: random.Random, lam: float) -> int:
    # Knuth; lam is small (a few pods per GPU per epoch)
    L, k, p = math.exp(-lam), 0, 1.0
    while True:
        p *= rng.random()
        if p <= L:
            return k
        k += 1


def run(n_gpus: int = 1, epochs: int = 40, rate: float = 3.0, request_cu: int = 128, iters: int = 20,
        resize: bool = True, sim: bool = False, seed: int = 0, device: int = 0,
        history: str = "executor", workdir: str = "") -> Dict[str, Any]:
    if n_gpus > 1 and not sim:
        raise ValueError("one process drives one GPU: multi-GPU resize loops run with sim=True")
    if history == "rocprof":
        if sim:
            raise ValueError("--history rocprof runs real pod processes under rocprofv3 (GPU)")
        return _run_rocprof(epochs, rate, request_cu, iters, resize, seed, workdir)
    rng = random.Random(seed)
    preds = measured_predictions() or analytic_predictions()
    conf = preds._conf
    quarter = {n: conf.by_label[n][f"4P_{C.MI355X}"] for n in W.NAMES}
    fc = FakeCluster(sync_watch=True, auto_run=True)
    fc.create("nodes", O.make_node(NODE, gpus=n_gpus))
    hist = RedisHistory(Redis(FakeRedisBackend(FakeRedisEngine())))
    adm = ResizeAdmission(hist.read, preds.configurations) if resize else None
    if adm is not None:
        fc.add_admission("pods", adm)
    cfg = default_gpu_config({"w_slo": 1.0, "w_pack": 0.25, "w_telemetry": 0.0, "compat_env": False},
                             disable_defaults=True)
    cfg.pod_initial_backoff_s = 0.0
    ledger = DeviceLedger()
    sched = Scheduler(fc, cfg, full_registry(), bind_async=False, record_events=False, seed=seed,
                      extras={"ledger": ledger, "predictions": preds})
    sched.keep_results = False
    sched.start_informers()
    sched.queue.initial_backoff_s = 0.0
    from ..agent.agent import NodeAgent
    procs = ExecutorProcessSource(ledger, NODE)
    agent = NodeAgent(NODE, hist.redis, procs, client=fc, pod_resolver=procs.uid_of)    # type: ignore[arg-type]
    from .executor import PodRun
    if sim:
        ex: Any = SimExecutor()
    else:
        from .executor import DeviceExecutor
        ex = DeviceExecutor(device, use_cu_masks=True)
        ex.warm([PodRun(0, wl, u, n, 1, masked=True) for wl in W.NAMES for n in (1, 2, 4) for u in range(0, 8, n)])
    weights = [1.0 / (1 + (i % 6)) for i in range(len(W.NAMES))]
    stats = {"created": 0, "completed": 0, "slo_ok": 0, "req_cu": [], "busy_unit_ms": 0.0, "backlog": []}
    wall_ms = 0.0
    serial = 0
    for e in range(epochs):
        for _ in range(_poisson(rng, rate * n_gpus)):
            wl = rng.choices(W.NAMES, weights)[0]
            w = W.CATALOG[wl]
            slo = quarter[wl] * rng.uniform(0.5, 0.95)
            pod = O.make_pod(f"{wl.replace('_', '-')}-{serial}", gpu_cu=request_cu,
                             gpu_mem_gib=round(2 * w.hbm_gib, 1), slo=round(slo, 3))
            serial += 1
            fc.create("pods", pod, owned=True)
            stats["created"] += 1
        sched.queue.move_all_to_active_or_backoff("epoch")
        results = sched.schedule_pending()
        runs: List[PodRun] = []
        placed: List[str] = []
        devs_of: List[str] = []
        for r in results:
            if not r.node:
                continue
            pl = ledger.placement(r.pod_key)
            if pl is None:
                continue
            st = next(s for s in ledger.devices(NODE) if s.device.uuid == pl[1][0])
            u0, n = st.pods[r.pod_key].units
            ns, name = r.pod_key.split("/", 1)
            pod = fc.get("pods", name, ns)
            stats["req_cu"].append(O.gpu_request(pod)[1])
            runs.append(PodRun(len(runs), workload_key(pod), u0, n, iters, O.pod_slo(pod), masked=True))
            placed.append(r.pod_key)
            devs_of.append(pl[1][0])
        t0 = time.perf_counter()
        ex.launch_epoch(runs)
        if not sim:
            ex.wait_epoch(runs)
        st_ep = ex.collect(runs)
        wall_ms += (time.perf_counter() - t0) * 1e3 if not sim else max(st_ep["span_ms"], 0.0)
        stats["busy_unit_ms"] += st_ep["busy_unit_ms"]
        procs.clear()
        for r, key, uuid in zip(runs, placed, devs_of):
            ns, name = key.split("/", 1)
            procs.report(uuid, O.uid(fc.get("pods", name, ns)), W.CATALOG[r.workload].hbm_gib,
                         r.n_units * CUS_PER_XCD, round(r.throughput, 3))
        stats["history_samples"] = stats.get("history_samples", 0) + agent.record_history()   # agent -> Redis
        for r, key in zip(runs, placed):
            stats["completed"] += 1
            stats["slo_ok"] += int(r.slo <= 0 or r.throughput >= r.slo)
            ns, name = key.split("/", 1)
            fc.delete("pods", name, ns)
        stats["backlog"].append(sum(sched.queue.pending().values()))
    if not sim:
        ex.close()
    secs = max(wall_ms, 1e-6) / 1e3
    return {"resize": resize, "sim": sim, "n_gpus": n_gpus, "epochs": epochs, "rate_per_gpu": rate,
            "request_cu": request_cu, "created": stats["created"], "completed": stats["completed"],
            "pods_per_s": round(stats["completed"] / secs, 2),
            "mean_cu_request_placed": round(float(np.mean(stats["req_cu"])) if stats["req_cu"] else 0.0, 1),
            "slo_attainment_pct": round(100.0 * stats["slo_ok"] / max(stats["completed"], 1), 2),
            "cu_share_occupancy_pct": round(100.0 * stats["busy_unit_ms"] / (8 * n_gpus * max(wall_ms, 1e-6)), 2),
            "final_backlog": stats["backlog"][-1] if stats["backlog"] else 0,
            "mean_backlog": round(float(np.mean(stats["backlog"])) if stats["backlog"] else 0.0, 2),
            "admission": adm.stats if adm is not None else None,
            "history": {"source": "node agent (process list -> pod -> workload key)",
                        "samples": stats.get("history_samples", 0)}}


def _run_rocprof(epochs: int, rate: float, request_cu: int, iters: int, resize: bool, seed: int,
                 workdir: str, profile_samples: int = 3) -> Dict[str, Any]:
    """The resize loop fed by the deployable profiler: pods run as processes; the first
    `profile_samples` pods of each workload opt in to the profiling webhook (label), so they
    run under the injected rocprofv3 and the agent's ingestor turns their output into the
    history the resize admission reads -- a sampling profiler, as a cluster would run it.
    Throughput and SLOs are accounted from every pod's own report (unprofiled pods carry no
    profiler overhead)."""
    import sys
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    from ..agent import profile_webhook as PW
    from ..agent.launcher import PodLauncher
    from ..agent.pod_profiler import ROCPROF, ProfileIngestor
    rng = random.Random(seed)
    preds = measured_predictions() or analytic_predictions()
    conf = preds._conf
    quarter = {n: conf.by_label[n][f"4P_{C.MI355X}"] for n in W.NAMES}
    work = workdir or tempfile.mkdtemp(prefix="resize-rocprof-", dir=os.environ.get("TMPDIR") or None)
    fc = FakeCluster(sync_watch=True, auto_run=True)
    fc.create("nodes", O.make_node(NODE, gpus=1))
    hist = RedisHistory(Redis(FakeRedisBackend(FakeRedisEngine())))
    adm = ResizeAdmission(hist.read, preds.configurations) if resize else None
    fc.add_admission("pods", PW.ChainAdmission(adm, PW.ProfileInjector(rocprof=ROCPROF)))
    cfg = default_gpu_config({"w_slo": 1.0, "w_pack": 0.25, "w_telemetry": 0.0, "compat_env": False},
                             disable_defaults=True)
    cfg.pod_initial_backoff_s = 0.0
    ledger = DeviceLedger()
    sched = Scheduler(fc, cfg, full_registry(), bind_async=False, record_events=False, seed=seed,
                      extras={"ledger": ledger, "predictions": preds})
    sched.keep_results = False
    sched.start_informers()
    sched.queue.initial_backoff_s = 0.0
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    la = PodLauncher(fc, NODE, timeout_s=240)
    la.host_root = work
    la.cwd = work
    la.extra_env = {"TMPDIR": work, "PYTHONPATH": root}
    base_env_for = la.env_for

    def env_for(pod):           # the fake node's UUIDs are not this box's: keep the share, run unfiltered
        env = {k: v for k, v in base_env_for(pod).items()
               if k not in (C.ENV_ROCR_VISIBLE, C.ENV_HIP_VISIBLE, C.ENV_CU_MASK)}
        env["GPU_SCHED_CU"] = str(O.gpu_request(pod)[1])
        return env
    la.env_for = env_for
    ing = ProfileIngestor(work + PW.HOST_DIR, hist)
    weights = [1.0 / (1 + (i % 6)) for i in range(len(W.NAMES))]
    stats = {"created": 0, "completed": 0, "slo_ok": 0, "req_cu": [], "backlog": [], "samples": 0, "failed": 0,
             "profiled": 0}
    profiled_by_wl: Dict[str, int] = {}
    serial = 0
    t_all = time.perf_counter()
    for e in range(epochs):
        for _ in range(_poisson(rng, rate)):
            wl = rng.choices(W.NAMES, weights)[0]
            w = W.CATALOG[wl]
            prof = profiled_by_wl.get(wl, 0) < profile_samples
            if prof:
                profiled_by_wl[wl] = profiled_by_wl.get(wl, 0) + 1
            pod = O.make_pod(f"{wl.replace('_', '-')}-{serial}", gpu_cu=request_cu,
                             gpu_mem_gib=round(2 * w.hbm_gib, 1), slo=round(quarter[wl] * rng.uniform(0.5, 0.95), 3),
                             env={C.ENV_ITERATIONS: str(iters)}, labels_={PW.LABEL_PROFILE: "trace"} if prof else None)
            pod["spec"]["containers"][0]["command"] = [sys.executable, "-m", "k8s_gpu_scheduler_amd.ops.podrun"]
            pod["spec"]["containers"][0]["args"] = ["--workload", wl]
            serial += 1
            fc.create("pods", pod, owned=True)
            stats["created"] += 1
        sched.queue.move_all_to_active_or_backoff("epoch")
        results = sched.schedule_pending()
        pods = []
        for r in results:
            if r.node:
                ns, name = r.pod_key.split("/", 1)
                pods.append(fc.get("pods", name, ns))
                stats["req_cu"].append(O.gpu_request(pods[-1])[1])
        stats["profiled"] += sum(1 for p in pods if O.labels(p).get(PW.LABEL_PROFILE))
        with ThreadPoolExecutor(max_workers=max(1, len(pods))) as tp:
            res = list(tp.map(la.run, pods))
        stats["failed"] += sum(1 for x in res if x.rc != 0)
        stats["samples"] += ing.step()
        for pod, x in zip(pods, res):
            rep = x.json() if x.rc == 0 else None
            if rep and rep.get("throughput"):
                stats["completed"] += 1
                stats["slo_ok"] += int(O.pod_slo(pod) <= 0 or rep["throughput"] >= O.pod_slo(pod))
            fc.delete("pods", O.name(pod), O.namespace(pod))
        stats["backlog"].append(sum(sched.queue.pending().values()))
        print(f"[resize-rocprof] resize={resize} epoch {e + 1}/{epochs}: ran {len(pods)}, completed "
              f"{stats['completed']}, backlog {stats['backlog'][-1]}, samples {stats['samples']}",
              file=sys.stderr, flush=True)
    return {"resize": resize, "history": {"source": "rocprofv3 via the profiling webhook -> node agent ingestor",
                                          "samples": stats["samples"], "profiled_pods": stats["profiled"],
                                          "profile_samples_per_workload": profile_samples},
            "epochs": epochs, "rate_per_gpu": rate, "request_cu": request_cu, "created": stats["created"],
            "completed": stats["completed"], "failed_pods": stats["failed"],
            "mean_cu_request_placed": round(float(np.mean(stats["req_cu"])) if stats["req_cu"] else 0.0, 1),
            "slo_attainment_pct": round(100.0 * stats["slo_ok"] / max(stats["completed"], 1), 2),
            "final_backlog": stats["backlog"][-1] if stats["backlog"] else 0,
            "mean_backlog": round(float(np.mean(stats["backlog"])) if stats["backlog"] else 0.0, 2),
            "admission": adm.stats if adm is not None else None,
            "wall_s": round(time.perf_counter() - t_all, 1)}


def main(argv: Optional[List[str]] = None) -> Dict[str, Any]:
    ap = argparse.ArgumentParser(description="recommender resize loop under Poisson arrivals (config 5)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=40)
    ap.add_argument("--rate", type=float, default=3.0, help="mean arrivals per GPU per epoch")
    ap.add_argument("--request-cu", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sim", action="store_true")
    ap.add_argument("--no-resize", action="store_true")
    ap.add_argument("--both", action="store_true", help="run with and without the loop")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--history", default="executor", choices=["executor", "rocprof"],
                    help="where the workload history comes from: the executor's accounting reported as a "
                         "process list (default), or rocprofv3 output of real pod processes (GPU)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    modes = [True, False] if a.both else [not a.no_resize]
    out = {"runs": [run(a.gpus, a.epochs, a.rate, a.request_cu, a.iters, m, a.sim, a.seed, history=a.history)
                    for m in modes]}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return out


if __name__ == "__main__":
    main()
