"""Measured backlog feedback in the deployed scheduler (plugins.gpu.feedback): pod completions
(container startedAt / finishedAt) corrected by the node-wide median measured / predicted
ratio move the burst planner's backlog -- one GPU 10 % slower than its sibling sheds planned
work within a few bursts, a uniform 10 % slowdown of every GPU changes nothing."""
import datetime as dt

import numpy as np
import pytest

from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.models import workloads as W
from k8s_gpu_scheduler_amd.models.corun import CorunModel
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger
from k8s_gpu_scheduler_amd.plugins.gpu.feedback import measured_ms
from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions
from k8s_gpu_scheduler_amd.telemetry.cache import TelemetryCache

has_core = _native.core() is not None
T0 = dt.datetime(2026, 1, 1, tzinfo=dt.timezone.utc)


def _iso(t: float) -> str:
    return (T0 + dt.timedelta(seconds=t)).isoformat().replace("+00:00", "Z")


def test_measured_ms_from_container_statuses_and_annotation():
    pod = O.make_pod("p", gpu_cu=64)
    pod["status"] = {"phase": "Succeeded", "containerStatuses": [
        {"state": {"terminated": {"startedAt": _iso(1.0), "finishedAt": _iso(3.5)}}},
        {"state": {"terminated": {"startedAt": _iso(0.5), "finishedAt": _iso(2.0)}}}]}
    assert abs(measured_ms(pod) - 3000.0) < 1e-6
    pod["metadata"].setdefault("annotations", {})["gpu-scheduler.amd.com/busy-ms"] = "12.5"
    assert measured_ms(pod) == 12.5


def _run(slow: tuple, bursts: int = 24, seed: int = 0, overhead: float = 3.0):
    """bursts of 8 pods onto a 2-GPU node; each burst's pods then finish after their true
    co-run duration (the model's, x `slow[gpu]`, x a container overhead common to all)."""
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n0", gpus=2))
    ledger = DeviceLedger()
    model = CorunModel.load()
    args = {"w_slo": 1.0, "w_pack": 0.25, "w_telemetry": 0.0, "w_balance": 1.0, "slo_objective": "corun",
            "plan_bursts": True, "plan_tolerance": 0.3, "plan_carry": 1.0}
    s = Scheduler(fc, default_gpu_config(args, disable_defaults=True), full_registry(), bind_async=False, seed=0,
                  extras={"ledger": ledger, "telemetry": TelemetryCache(stale_s=0),
                          "predictions": CachedPredictions(corun=model)})
    s.start_informers()
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    rng = np.random.default_rng(seed)
    gpu_of = {d.device.uuid: d.device.gpu for d in ledger.devices("n0")}
    t = 0.0
    share, placements = [], []
    for b in range(bursts):
        names = []
        for i in range(8):
            wl = W.NAMES[int(rng.integers(len(W.NAMES)))]
            nm = f"{wl.replace('_', '-')}-b{b}-{i}"
            fc.create("pods", O.make_pod(nm, gpu_cu=64, env={C.ENV_ITERATIONS: "20000"}))
            names.append((nm, wl))
        assert all(r.node for r in s.schedule_pending())
        groups = {0: [], 1: []}
        for nm, wl in names:
            pod = fc.get("pods", nm, "default")
            groups[gpu_of[O.annotations(pod)[C.ANNOT_DEVICES]]].append((nm, wl))
        work = {g: sum(model.alone_ms[model.wid(wl)] for _, wl in m) for g, m in groups.items()}
        if b >= bursts // 3:
            share.append(work[1] / (work[0] + work[1]))
        placements.append(sorted((g, nm) for g, m in groups.items() for nm, _ in m))
        for g, m in groups.items():
            d = model.group_durations([model.wid(wl) for _, wl in m], [20000] * len(m))
            for (nm, _), ms in zip(m, d):
                fin = t + ms / 1e3 * slow[g] * overhead
                fc.patch("pods", nm, {"status": {"phase": "Succeeded", "containerStatuses": [
                    {"name": "main", "state": {"terminated": {"startedAt": _iso(t), "finishedAt": _iso(fin)}}}]}},
                    "merge", "default")
        for nm, _ in names:
            fc.delete("pods", nm, "default")
        t += 100.0
    pl = plugin.planner
    return float(np.mean(share)), dict(pl.backlog), pl.feedback, placements


@pytest.mark.skipif(not has_core, reason="_core not built")
def test_slow_gpu_sheds_planned_work_uniform_slowdown_changes_nothing():
    base_share, base_bl, fb0, pl0 = _run((1.0, 1.0))
    assert fb0.applied > 0
    uni_share, uni_bl, _, pl1 = _run((1.1, 1.1))
    assert pl1 == pl0                                      # uniform: the median absorbs it
    assert uni_bl == pytest.approx(base_bl, rel=1e-5, abs=1e-2)     # (timestamps carry microseconds)
    slow_share, slow_bl, fb, _ = _run((1.0, 1.1))
    pl = fb.planner
    g0, g1 = ("n0", 0), ("n0", 1)
    assert fb.corrections[g1] > fb.corrections[g0]
    assert pl.speed(g1) > pl.speed(g0)
    # the share that levels the MEASURED work is 1 / 2.1 = 0.476 for a GPU 10 % slower: the
    # planner moves toward it and no further (round 4's unbounded integrator overshot to 0.44;
    # each GPU is full every burst here, so only long / short swaps can move work)
    assert 0.46 < slow_share < base_share - 0.005, (slow_share, base_share)
