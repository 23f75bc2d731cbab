"""Where an 8-GPU control-plane epoch's planning time goes (CPU only): tools/cp_timing.py's
bench configuration per effort level, with the burst planner's stages and native calls timed
(wall ms per epoch).  Run on the box CPU for judged numbers (tools/gpu_cp_timing.sh's host).

    python tools/cp_breakdown.py [levels=0,1,2]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from k8s_gpu_scheduler_amd._native import _core  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.podbench import ControlPlane  # noqa: E402
from k8s_gpu_scheduler_amd.plugins.gpu import planner as P  # noqa: E402
from k8s_gpu_scheduler_amd.plugins.gpu import timeline as TL  # noqa: E402

BENCH = dict(balance=1.0, plan_bursts=True, plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05,
             plan_carry=1.0, plan_feedback=True, plan_slots="auto", learn_corun=False)
acc = {}


def _wrap(owner, name, label):
    f = getattr(owner, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[label] = acc.get(label, 0.0) + time.perf_counter() - t
    setattr(owner, name, g)


for n in ("_plan_corun", "_plan_slots", "_pipe_context", "_burst", "_carry", "placed", "realign"):
    if hasattr(P.BurstPlanner, n):
        _wrap(P.BurstPlanner, n, n)
_wrap(TL.SlotTimeline, "_context", "timeline._context")
_wrap(ControlPlane, "update_telemetry", "cp.update_telemetry(outside the epoch)")
_wrap(ControlPlane, "finish_live", "cp.finish_live(outside the epoch)")
_wrap(TL.SlotTimeline, "pipeline", "timeline.pipeline")
_wrap(_core, "plan_corun", "native.plan_corun")
_wrap(_core, "plan_slots", "native.plan_slots(sum over threads)")


def main() -> None:
    import virtual_node_bench as V
    levels = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2").split(",")]
    for lvl in levels:
        V.N_GPUS = 8
        V.SIM.update(on=True, sigma=0.05, rng=np.random.default_rng(0), speed=[])
        kw = {} if lvl < 0 else (dict(BENCH, effort=lvl) if lvl else BENCH)     # -1: plain plugin
        cp = ControlPlane(8, 4, 20, 0, **kw)
        for _ in range(10):
            cp.finish_live()
            V.epoch(cp, None, cp.schedule_epoch(), "t")
        import gc
        mode = os.environ.get("CP_GC", "")
        if mode == "off":
            gc.disable()
        elif mode == "freeze":
            gc.collect()
            gc.freeze()
        elif mode == "settle":
            from k8s_gpu_scheduler_amd.utils.gctune import settle
            settle()
        acc.clear()
        fw = cp.sched.frameworks[next(iter(cp.sched.frameworks))]
        fw.metrics.ext_ns.clear()
        fw.metrics.ext_calls.clear()
        ts = []
        for _ in range(60):
            cp.finish_live()
            t = time.perf_counter()
            arr = cp.schedule_epoch()
            ts.append(time.perf_counter() - t)
            if kw:
                V.epoch(cp, None, arr, "t")
        if mode == "off":
            gc.enable()
        parts = " ".join(f"{k}={v / 60 * 1e3:.3f}" for k, v in sorted(acc.items(), key=lambda x: -x[1]))
        ext = " ".join(f"{k}={v / 60 / 1e6:.3f}" for k, v in sorted(fw.metrics.ext_ns.items(), key=lambda x: -x[1]))
        print(f"gc={mode or 'default'} level {lvl}: epoch {np.median(ts) * 1e3:.2f} ms (median) "
              f"{np.mean(ts) * 1e3:.2f} (mean) | {parts} || extension points ms/epoch: {ext}", flush=True)


if __name__ == "__main__":
    main()
