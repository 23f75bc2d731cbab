"""Cross-cycle node-result cache (framework.fastpath) and its native host selection
(`_core.select_nodes`): identical placements to the node-at-a-time path, O(changed nodes)
work per pod, correct invalidation on every kind of node-local change."""
import random

import numpy as np
import pytest

from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.changes import ChangeLog
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.fastpath import select_nodes_py
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.models import workloads as W
from k8s_gpu_scheduler_amd.parallel.podbench import analytic_predictions
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger
from k8s_gpu_scheduler_amd.telemetry.cache import DeviceSample, TelemetryCache


def _cluster(n_nodes, fast, seed=3, args=None, nodes_fn=None):
    fc = FakeCluster()
    for i in range(n_nodes):
        node = nodes_fn(i) if nodes_fn else O.make_node(f"mi355x-{i:03d}", gpus=8)
        fc.create("nodes", node)
    tele = TelemetryCache(stale_s=0)
    extras = {"ledger": DeviceLedger(), "telemetry": tele, "predictions": analytic_predictions()}
    s = Scheduler(fc, default_gpu_config(dict({"weightBalance": 1.0}, **(args or {}))), full_registry(),
                  bind_async=False, record_events=False, seed=seed, extras=extras)
    s.fast_path = fast
    s.fast_min_nodes = 0
    s.start_informers()
    return fc, s, tele


def _placements(fc):
    out = {}
    for p in fc.list("pods")[0]:
        ann = O.annotations(p)
        out[O.name(p)] = (O.node_name_of(p), ann.get(C.ANNOT_DEVICE_INDICES, ""))
    return out


def _pods(rng, n, start=0, templates=0):
    """Random fractional pods; with `templates` > 0 they are replicas of that many
    deployments (equal requests, SLO and workload -> equal cycle signatures)."""
    tpl = [(rng.choice(W.NAMES).replace("_", "-"), rng.choice([32, 64, 64, 128]), rng.choice([2, 4, 8]),
            rng.uniform(5, 50), rng.choice(["100m", "2", "8"])) for _ in range(templates)]
    pods = []
    for i in range(start, start + n):
        if tpl:
            wl, cu, mem, slo, cpu = rng.choice(tpl)
        else:
            wl, cu, mem, slo, cpu = (rng.choice(W.NAMES).replace("_", "-"), rng.choice([32, 64, 64, 128]),
                                     rng.choice([2, 4, 8]), rng.uniform(5, 50), rng.choice(["100m", "2", "8"]))
        pods.append(O.make_pod(f"{wl}-{i}", gpu_cu=cu, gpu_mem_gib=mem, slo=slo, cpu=cpu))
    return pods


def _run_both(n_nodes, script, args=None, nodes_fn=None):
    """Run the same event script on a fast-path and an ordinary scheduler; return both
    clusters' final placements and the fast scheduler."""
    res = []
    for fast in (False, True):
        fc, s, tele = _cluster(n_nodes, fast, args=args, nodes_fn=nodes_fn)
        script(fc, s, tele)
        res.append((_placements(fc), s))
    return res


def test_select_nodes_native_matches_python():
    core = _native.core()
    if core is None:
        pytest.skip("native core not built")
    rng = np.random.default_rng(0)
    for trial in range(200):
        n = int(rng.integers(1, 60))
        feas = (rng.random(n) < 0.6).astype(np.int8)
        if trial % 3 == 0:
            feas[rng.random(n) < 0.2] = -1      # not evaluated yet: returned for evaluation
        raw = rng.integers(0, 101, size=(3, n)).astype(np.int64)
        if trial % 5 == 0:
            raw[:, :] = 50                       # all tied
        norm = np.asarray([0, 1, int(trial % 2)], np.int8)
        w = np.asarray([1, 10100, 2], np.int64)
        start, limit = int(rng.integers(0, n)), int(rng.integers(0, n + 1))
        a = core.select_nodes(feas, raw, norm, w, start, limit)
        b = select_nodes_py(feas, raw, norm, w, start, limit)
        assert a[4] == b[4]
        assert list(np.asarray(a[5])) == list(np.asarray(b[5]))
        if len(a[5]) == 0:
            assert a[0] == b[0]
        for x, y in zip(a[1:4], b[1:4]):
            assert list(np.asarray(x)) == list(np.asarray(y))
    # a score out of range is reported with the plugin index
    bad = core.select_nodes(np.ones(2, np.int8), np.asarray([[0, 150]], np.int64), np.zeros(1, np.int8),
                            np.ones(1, np.int64), 0, 0)
    assert bad[4] == 0


def test_identical_placements_large_cluster_with_sampling():
    """120 nodes: adaptive sampling (limit < nodes) and the rotating start index are
    exercised; fractional pods of mixed sizes with SLOs and interference predictions."""
    def script(fc, s, tele):
        rng = random.Random(7)
        for p in _pods(rng, 100) + _pods(rng, 150, start=100, templates=3):
            fc.create("pods", p)
        s.schedule_pending()
    (slow, _), (fast, sf) = _run_both(120, script)
    assert slow == fast
    st = sf._fast[C.SCHEDULER_NAME].stats
    assert st["fallback"] == 0 and st["cycles"] == 250
    # unique pods re-evaluate every node; replicas of a deployment only the nodes touched
    # since that deployment's previous pod
    assert st["rescored"] < 100 * 120 + 3 * 120 + 150 * 8


def test_identical_under_churn_taints_telemetry_and_deletes():
    """Node updates (taint, unschedulable, label), pod deletions (ledger release), telemetry
    samples and a node added mid-run: each must invalidate exactly what it affects."""
    def script(fc, s, tele):
        rng = random.Random(11)
        pods = _pods(rng, 60, templates=4)
        for p in pods[:30]:
            fc.create("pods", p)
        s.schedule_pending()
        n5 = fc.get("nodes", "mi355x-005")
        n5 = dict(n5, spec=dict(n5.get("spec") or {}, taints=[{"key": "k", "value": "v", "effect": "NoSchedule"}]))
        fc.update("nodes", n5)
        n7 = fc.get("nodes", "mi355x-007")
        fc.update("nodes", dict(n7, spec=dict(n7.get("spec") or {}, unschedulable=True)))
        for i in range(0, 30, 3):
            fc.delete("pods", O.name(pods[i]))
        for g in range(8):
            uuid = s.frameworks[C.SCHEDULER_NAME].plugin("GPU").ledger.devices("mi355x-002")[g].device.uuid
            tele.update("mi355x-002", uuid, DeviceSample(gfx_activity=0.97, vram_used_mb=200 * 1024))
        fc.create("nodes", O.make_node("mi355x-999", gpus=8))
        for p in pods[30:]:
            fc.create("pods", p)
        s.schedule_pending()
    (slow, _), (fast, sf) = _run_both(110, script)
    assert slow == fast
    assert not any(v[0] in ("mi355x-005", "mi355x-007") for k, v in fast.items() if int(k.rsplit("-", 1)[1]) >= 30)
    assert sf._fast[C.SCHEDULER_NAME].stats["fallback"] == 0


def test_uncacheable_pod_falls_back_and_stays_identical():
    """A pod with a hard topology-spread constraint depends on other nodes' pods: the cycle
    takes the ordinary path for it (and the cache stays consistent for the next pods)."""
    def zoned(i):
        return O.make_node(f"mi355x-{i:03d}", gpus=8, labels_={"topology.kubernetes.io/zone": f"z{i % 3}"})

    def script(fc, s, tele):
        rng = random.Random(5)
        pods = _pods(rng, 20)
        spread = O.make_pod("spread-0", gpu_cu=64, slo=10, labels_={"app": "s"})
        spread["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone",
                                                         "whenUnsatisfiable": "DoNotSchedule",
                                                         "labelSelector": {"matchLabels": {"app": "s"}}}]
        for p in pods[:10] + [spread] + pods[10:]:
            fc.create("pods", p)
            s.schedule_pending()
    (slow, _), (fast, sf) = _run_both(30, script, nodes_fn=zoned)
    assert slow == fast
    assert sf._fast[C.SCHEDULER_NAME].stats["fallback"] >= 1


def test_unschedulable_pod_reports_reasons_through_ordinary_path():
    fc, s, _ = _cluster(3, True)
    fc.create("pods", O.make_pod("huge-0", gpu_cu=64, gpu_mem_gib=10_000, slo=10))
    res = s.schedule_pending()
    assert not res[0].status.ok and "nodes are available" in res[0].status.message()


def test_change_log_cursor_and_compaction():
    log = ChangeLog(cap=8)
    c0 = log.seq
    log.touch("a")
    log.touch("b")
    assert log.since(c0) == {"a", "b"}
    c1 = log.seq
    assert log.since(c1) == set()
    for i in range(20):
        log.touch(f"n{i}")
    assert log.since(c0) is None            # compacted away: the caller rebuilds
    e = log.epoch
    log.touch_all()
    assert log.epoch == e + 1
