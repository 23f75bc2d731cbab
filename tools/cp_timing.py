"""Control-plane throughput at N GPUs (CPU only): ms to schedule one epoch of N x 4 pods
(median over the timed epochs; `mean` includes the occasional garbage-collector pause).

Two configurations: the plain GPU plugin (no burst planner) and the bench defaults (co-run
planner with backlog carry and measured feedback; each epoch's telemetry is fed back from the
co-run model, as `tools/virtual_node_bench.py --simulate` does), so the planner's full
per-epoch cost is in the figure.  The online co-run learner is off, as in the bench since round 5
(`--corun-learn 0`: its refits never landed inside a driver-length run).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from k8s_gpu_scheduler_amd.parallel.podbench import ControlPlane  # noqa: E402

BENCH = dict(balance=1.0, plan_bursts=True, plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05,
             plan_carry=1.0, plan_feedback=True, plan_slots="auto", learn_corun=False)


def run(n: int, kwargs: dict, epochs: int = 60, warm: int = 10) -> float:
    import virtual_node_bench as V
    V.N_GPUS = n
    V.SIM.update(on=True, sigma=0.05, rng=np.random.default_rng(0), speed=[])
    cp = ControlPlane(n, 4, 20, 0, gc_settle=os.environ.get("CP_GC_SETTLE", "1") == "1", **kwargs)
    ts = []
    for e in range(warm + epochs):
        if e == warm:
            cp.reset_stats()                 # the bench's warmup -> timed transition
        cp.finish_live()
        t = time.perf_counter()
        arr = cp.schedule_epoch()
        if e >= warm:
            ts.append(time.perf_counter() - t)
        if kwargs:
            V.epoch(cp, None, arr, "t")      # telemetry back into the control plane (not timed)
    return float(np.median(ts)), float(np.mean(ts))


CONFIGS = [("plain", {}), ("bench-defaults", BENCH)]
# the adaptive control plane's cheaper levels (planner.set_effort; bench --plan-effort)
CONFIGS += [(f"bench-effort{k}", dict(BENCH, effort=k)) for k in (1, 2, 3)]
only = os.environ.get("CP_TIMING_GPUS")
pick = os.environ.get("CP_TIMING_CONFIGS")          # comma-separated config names (default: all)
rounds = int(os.environ.get("CP_TIMING_ROUNDS", "1"))  # interleaved rounds: the median is printed
if pick:
    CONFIGS = [c for c in CONFIGS if c[0] in pick.split(",")]
res = {}
for r in range(rounds):
    for name, kw in CONFIGS:
        for n in ((int(only),) if only else (1, 2, 4, 8)):
            res.setdefault((name, n), []).append(run(n, kw))
for (name, n), v in res.items():
    dt = float(np.median([x[0] for x in v]))
    mean = float(np.median([x[1] for x in v]))
    print(f"{name} gpus={n} pods/epoch={4 * n} ms/epoch={dt * 1e3:.2f} mean={mean * 1e3:.2f} ms/pod={dt * 1e3 / (4 * n):.3f}"
          + (f" rounds={[round(x[0] * 1e3, 2) for x in v]}" if rounds > 1 else ""), flush=True)
