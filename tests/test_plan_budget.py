"""The deployed scheduler's planning budget (GPU plugin arg planBudgetMs): every burst plan's
wall time is measured by the planner and its effort level follows the budget -- a burst of 64
pods over budget drops the planner to a cheaper level, later small bursts bring it back -- and
the level is exported as gpusched_plan_effort_level (before, only the bench
adapted its effort).  Plan costs are scripted (the planner's clock) so the test is exact."""
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
from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions
from k8s_gpu_scheduler_amd.telemetry.cache import TelemetryCache
from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter, observe_planner

pytestmark = pytest.mark.skipif(_native.core() is None, reason="_core not built")


class ScriptedClock:
    """Alternating start / end reads: the end read advances by the scripted plan cost."""

    def __init__(self, cost_of):
        self.t, self.calls, self.cost_of = 100.0, 0, cost_of

    def __call__(self):
        self.calls += 1
        if self.calls % 2 == 0:
            self.t += self.cost_of()
        return self.t


def test_burst_over_budget_drops_effort_and_recovers_with_the_level_exported():
    fc = FakeCluster()
    for n in ("n0", "n1"):
        fc.create("nodes", O.make_node(n, gpus=8))
    args = {"w_slo": 1.0, "w_pack": 0.25, "w_telemetry": 0.0, "w_balance": 1.0, "slo_objective": "corun",
            "plan_bursts": True, "plan_tolerance": 0.3, "plan_carry": 1.0, "planBudgetMs": 10.0}
    s = Scheduler(fc, default_gpu_config(args, disable_defaults=True), full_registry(), bind_async=False, seed=0,
                  extras={"ledger": DeviceLedger(), "telemetry": TelemetryCache(stale_s=0),
                          "predictions": CachedPredictions(corun=CorunModel.load())})
    s.start_informers()
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    pl = plugin.planner
    assert pl.budget is not None and pl.budget_ms == 10.0
    burst = {"n": 0}
    # a plan costs 0.5 ms per pod of its burst at full effort, scaled by the level's measured cost
    pl.clock = ScriptedClock(lambda: 0.5e-3 * burst["n"] * pl.budget.LEVEL_COST[pl.effort])
    rng = np.random.default_rng(0)
    exp = GpuExporter("sched")
    levels = []

    def run_burst(b, n):
        burst["n"] = n
        names = []
        for i in range(n):
            wl = W.NAMES[int(rng.integers(len(W.NAMES)))]
            nm = f"{wl.replace('_', '-')}-b{b}-{i}"
            fc.create("pods", O.make_pod(nm, gpu_cu=64, env={C.ENV_ITERATIONS: "20"}))
            names.append(nm)
        res = s.schedule_pending()
        assert all(r.node for r in res), [r.status for r in res if not r.node]
        for nm in names:
            fc.delete("pods", nm, "default")
        observe_planner(exp, C.SCHEDULER_NAME, s.frameworks[C.SCHEDULER_NAME])
        levels.append(pl.effort)

    for b in range(3):                  # 64-pod bursts: 32 ms at level 0 against a 10 ms budget
        run_burst(b, 64)
    assert levels[0] == 0 and max(levels) == pl.MAX_EFFORT, levels
    text = exp.render().decode()
    assert f'gpusched_plan_effort_level{{profile="{C.SCHEDULER_NAME}"}} {float(pl.MAX_EFFORT)}' in text
    for b in range(3, 16):              # small bursts: back to full effort
        run_burst(b, 8)
    assert levels[-1] == 0, levels
    assert pl.budget.changes >= 2 and pl.stats["plans_timed"] == 16
    assert f'gpusched_plan_effort_level{{profile="{C.SCHEDULER_NAME}"}} 0.0' in exp.render().decode()


def _place_bursts(plan_hints: bool, disable_defaults: bool):
    fc = FakeCluster()
    for n in ("n0", "n1", "n2"):
        fc.create("nodes", O.make_node(n, gpus=8))
    # (one LPT arrival window: the queue's 1 s wall-clock windows could split a burst differently
    # in the two runs -- a different scheduling order, not a different plan)
    args = {"w_slo": 1.0, "w_pack": 0.25, "w_telemetry": 0.0, "w_balance": 1.0, "slo_objective": "corun",
            "plan_bursts": True, "plan_tolerance": 0.3, "plan_carry": 1.0, "lpt_window_s": 1e9}
    s = Scheduler(fc, default_gpu_config(args, disable_defaults=disable_defaults), full_registry(),
                  bind_async=False, seed=0,
                  extras={"ledger": DeviceLedger(), "telemetry": TelemetryCache(stale_s=0),
                          "predictions": CachedPredictions(corun=CorunModel.load())})
    s.plan_hints = plan_hints
    s.start_informers()
    rng = np.random.default_rng(3)
    out = []
    for b in range(4):
        names = []
        for i in range(24):
            wl = W.NAMES[int(rng.integers(len(W.NAMES)))]
            nm = f"{wl.replace('_', '-')}-b{b}-{i}"
            fc.create("pods", O.make_pod(nm, gpu_cu=64, env={C.ENV_ITERATIONS: "20"}))
            names.append(nm)
        assert all(r.node for r in s.schedule_pending())
        for nm in names:
            p = fc.get("pods", nm, "default")
            out.append((nm, O.node_name_of(p), O.annotations(p)[C.ANNOT_DEVICE_INDICES]))
        if b % 2:                      # half the bursts finish: residents for the next plans
            for nm in names:
                fc.delete("pods", nm, "default")
    return out, s.plan_hint_hits


@pytest.mark.parametrize("disable_defaults", [True, False])
def test_planned_pods_skip_score_with_identical_placements(disable_defaults):
    """Framework.plan_hint: a pod the GPU plugin's burst plan has already placed is filtered on
    its planned node only and skips Score when the GPU weight (10100) decides Score anyway -- the
    placements, node AND CU slot, are exactly those of the full cycle.  With the in-tree score
    plugins enabled beside it the hint stays off: NodePreferAvoidPods (weight 10000) can outvote
    one GPU point, so Score must run."""
    fast, hits = _place_bursts(True, disable_defaults)
    full, hits0 = _place_bursts(False, disable_defaults)
    assert hits0 == 0
    if disable_defaults:
        assert hits >= 4 * 23 - 4                   # every pod after the first of each burst
    else:
        assert hits == 0
    assert fast == full
