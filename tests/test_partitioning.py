"""Scheduler-driven MI355X compute partitioning, end to end on a fake cluster.

Reference: Score picks a MIG layout from the pod's predictions, relabels the node, restarts
the profiler and polls Redis for the new UUIDs (pkg/plugins/gpu_plugin/gpu_plugins.go:357-453,
478-496).  Here: pending isolated pods -> partition controller (idle nodes only) -> node
label -> agent (capability probe, idleness check, taint, amd-smi apply, republish, untaint)
-> scheduler re-reads the inventory -> the pods bind to partitions.
"""
import json
import time

from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
from k8s_gpu_scheduler_amd.agent.devices import StaticSource, partition_capabilities, synthetic_node
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.kube.resources import Resources
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.partitioner import size_from_predictions
from k8s_gpu_scheduler_amd.store import schema
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
from k8s_gpu_scheduler_amd.store.resp import Redis

ISO = {C.ANNOT_ISOLATION: "partition"}


def rds():
    return Redis(FakeRedisBackend(FakeRedisEngine()))


def _cluster(nodes=("n1",)):
    fc = FakeCluster()
    r = rds()
    agents = {}
    for n in nodes:
        fc.create("nodes", O.make_node(n, gpus=8))
        ag = NodeAgent(n, r, synthetic_node(8, node=n), client=fc)
        ag.step()                       # publish devices + partition capabilities
        agents[n] = ag
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, record_events=False,
                  extras={"redis": r})
    s.start_informers()
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    return fc, r, agents, s, plugin


def _drain(s, fc, names, timeout=15.0):
    t = time.time()
    while time.time() - t < timeout:
        s.schedule_pending(timeout_s=0.2)
        if all(O.node_name_of(fc.get("pods", n, "default")) for n in names):
            return True
    return False


def test_size_from_predictions_most_partitions_meeting_slo():
    conf = {"1P_MI355X": 100.0, "2P_MI355X": 80.0, "4P_MI355X": 60.0, "8P_MI355X": 30.0}
    assert size_from_predictions(conf, 50.0) == 64          # QPX: 60 >= 50, CPX 30 < 50
    assert size_from_predictions(conf, 20.0) == 32          # CPX meets it
    assert size_from_predictions(conf, 500.0) == 256        # nothing meets it: best predicted
    assert size_from_predictions({}, 50.0) is None


def test_agent_publishes_probed_capabilities():
    fc, r, agents, s, plugin = _cluster()
    caps = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_CAPS])
    assert caps["compute_modes"] == ["SPX", "DPX", "QPX", "CPX"] and caps["probed"]
    assert json.loads(r.get(schema.partition_caps_key("n1"))) == caps


def test_burst_of_eighth_gpu_pods_triggers_cpx_and_binds(monkeypatch):
    fc, r, agents, s, plugin = _cluster()
    taints = []
    orig = Resources.taint_node

    def spy(self, node, key, value="true", effect="NoSchedule"):
        taints.append((node, key, value))
        return orig(self, node, key, value, effect)
    monkeypatch.setattr(Resources, "taint_node", spy)
    names = [f"iso-{i}" for i in range(16)]
    for n in names:
        fc.create("pods", O.make_pod(n, gpu_cu=32, gpu_mem_gib=8, annotations_=ISO))
    res = s.schedule_pending()
    assert len(res) == 16 and not any(x.node for x in res)
    assert "no free CPX partition" in res[0].status.message()
    # the controller (never Score) asks for CPX on the idle node
    dec = plugin.partitioner.step()
    assert [(d.node, d.mode) for d in dec] == [("n1", "CPX")]
    assert O.labels(fc.get("nodes", "n1"))[C.LABEL_COMPUTE_PARTITION] == "CPX"
    assert plugin.partitioner.step() == []                  # already requested: no second request
    # the agent: taint -> apply -> republish 64 UUIDs -> untaint
    assert agents["n1"].reconcile_partitions()
    assert taints == [("n1", C.TAINT_PARTITIONING, "CPX")]
    assert not O.node_taints(fc.get("nodes", "n1"))
    assert len(schema.read_uuids(r, "n1")) == 64
    assert json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_STATE])["state"] == "applied"
    # the scheduler re-reads the inventory on the node update; the pods bind to partitions
    assert _drain(s, fc, names)
    devs = {d.device.uuid: d.device for d in plugin.ledger.devices("n1")}
    got = [O.annotations(fc.get("pods", n, "default"))[C.ANNOT_DEVICES] for n in names]
    assert len(set(got)) == 16 and all(devs[u].cus == 32 and devs[u].partitions == 8 for u in got)


def test_controller_never_picks_a_busy_node():
    fc, r, agents, s, plugin = _cluster(("n1", "n2"))
    fc.create("pods", O.make_pod("resident", gpu_cu=64, gpu_mem_gib=4,
                                 node_selector={"kubernetes.io/hostname": "n1"}))
    (res,) = s.schedule_pending()
    assert res.node == "n1"
    for i in range(8):
        fc.create("pods", O.make_pod(f"iso-{i}", gpu_cu=64, annotations_=ISO))
    s.schedule_pending()
    dec = plugin.partitioner.step()
    assert [(d.node, d.mode) for d in dec] == [("n2", "QPX")]
    assert O.labels(fc.get("nodes", "n1"))[C.LABEL_COMPUTE_PARTITION] == "SPX"


def test_slo_only_isolated_pod_is_sized_from_predictions():
    from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions, _Tab
    fc, r, agents, s, plugin = _cluster()
    cp = CachedPredictions()
    cols = ["1P_MI355X", "2P_MI355X", "4P_MI355X", "8P_MI355X"]
    cp._conf = _Tab(["onnx_resnet50_1024"], cols, [[400.0, 300.0, 200.0, 90.0]], "t")
    cp._intf = _Tab(["onnx_resnet50_1024_MI355X"], ["onnx_resnet50_1024"], [[0.0]], "t")
    plugin.predictions = cp
    fc.create("pods", O.make_pod("onnx-resnet50-1024-a", slo=150, annotations_=ISO))
    s.schedule_pending()
    dec = plugin.partitioner.step()
    pod = fc.get("pods", "onnx-resnet50-1024-a", "default")
    assert O.annotations(pod)[C.ANNOT_PARTITION_CUS] == "64"        # 4P meets 150, 8P does not
    assert [d.mode for d in dec] == ["QPX"]
    assert agents["n1"].reconcile_partitions()
    assert _drain(s, fc, ["onnx-resnet50-1024-a"])
    u = O.annotations(fc.get("pods", "onnx-resnet50-1024-a", "default"))[C.ANNOT_DEVICES]
    assert {d.device.uuid: d.device.cus for d in plugin.ledger.devices("n1")}[u] == 64


def test_agent_refuses_busy_gpu_then_gives_up():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=8))
    src = synthetic_node(8, node="n1")
    src.procs = {3: [{"pid": 4242, "name": "train.py", "vram_bytes": 2**30}]}
    ag = NodeAgent("n1", rds(), src, client=fc, drain_timeout_s=3600)
    ag.step()
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "CPX"}}}, "merge")
    assert not ag.reconcile_partitions()
    assert src.partition_calls == []                         # a busy GPU is never repartitioned
    st = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_STATE])
    assert st["state"] == "waiting-idle" and "pid 4242" in st["busy"][0]
    assert O.node_taints(fc.get("nodes", "n1"))[0]["key"] == C.TAINT_PARTITIONING    # draining
    ag.drain_timeout_s = 0.0
    time.sleep(0.01)
    assert not ag.reconcile_partitions()
    st = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_STATE])
    assert st["state"] == "refused" and not O.node_taints(fc.get("nodes", "n1"))
    assert O.labels(fc.get("nodes", "n1"))[C.LABEL_COMPUTE_PARTITION] == "SPX"      # request reverted
    assert src.partition_calls == []


def test_agent_refuses_unsupported_mode_and_unprobed_gpu():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=2))
    src = StaticSource(synthetic_node(2, node="n1").devices(), profiles=[
        {"mode": "SPX", "partitions": 1, "memory_caps": ["NPS1"]},
        {"mode": "CPX", "partitions": 8, "memory_caps": ["NPS1"]}])
    ag = NodeAgent("n1", rds(), src, client=fc)
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "QPX"}}}, "merge")
    assert not ag.reconcile_partitions() and src.partition_calls == []
    st = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_STATE])
    assert st["state"] == "refused" and "not supported" in st["reason"]
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "CPX",
                                                     C.LABEL_MEMORY_PARTITION: "NPS2"}}}, "merge")
    assert not ag.reconcile_partitions() and src.partition_calls == []       # NPS2 not allowed with CPX
    # no readable profiles (amd-smi without privileges): nothing is assumed, nothing applied
    src.profiles = []
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "CPX"}}}, "merge")
    assert not ag.reconcile_partitions() and src.partition_calls == []
    assert "unknown" in json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_STATE])["reason"]


def test_memory_partition_applied_before_compute():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=2))
    src = synthetic_node(2, node="n1")
    ag = NodeAgent("n1", rds(), src, client=fc)
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "DPX",
                                                     C.LABEL_MEMORY_PARTITION: "NPS2"}}}, "merge")
    assert ag.reconcile_partitions()
    assert src.partition_calls[:2] == [(0, "NPS2"), (1, "NPS2")]
    assert [m for _, m in src.partition_calls[2:]] == ["DPX", "DPX"]
    caps = partition_capabilities(src.partition_info(0))
    assert caps.current_memory == "NPS2" and caps.current_compute == "DPX"


def test_unledgered_busy_node_is_requested_once_then_backed_off():
    """A node busy with GPU work the ledger cannot see (a process of another scheduler):
    the controller asks once, the agent drains, times out and refuses, and while the
    isolated pod stays pending the controller does not re-taint that node for that mode
    until the backoff expires (advisor round 2: the request/refuse loop)."""
    fc, r, agents, s, plugin = _cluster()
    agents["n1"].source.procs = {2: [{"pid": 999, "name": "other-scheduler-job", "vram_bytes": 2**30}]}
    agents["n1"].drain_timeout_s = 0.0
    for i in range(8):
        fc.create("pods", O.make_pod(f"iso-{i}", gpu_cu=32, annotations_=ISO))
    s.schedule_pending()
    pc = plugin.partitioner
    assert [(d.node, d.mode) for d in pc.step()] == [("n1", "CPX")]
    assert not agents["n1"].reconcile_partitions()          # busy: starts draining (taint)
    time.sleep(0.01)
    assert not agents["n1"].reconcile_partitions()          # drain timed out: refused + reverted
    node = fc.get("nodes", "n1")
    assert json.loads(O.annotations(node)[C.ANNOT_PARTITION_STATE])["state"] == "refused"
    assert O.labels(node)[C.LABEL_COMPUTE_PARTITION] == "SPX" and not O.node_taints(node)
    for _ in range(3):                                      # pods still pending: no new request
        s.schedule_pending(timeout_s=0.05)
        assert pc.step() == []
    assert O.labels(fc.get("nodes", "n1"))[C.LABEL_COMPUTE_PARTITION] == "SPX"
    assert pc.backed_off("n1", "CPX") and not pc.backed_off("n1", "QPX")
    # once the backoff has expired the node is eligible again
    pc._backoff[("n1", "CPX")] = 0.0
    fc.patch("nodes", "n1", {"metadata": {"annotations": {C.ANNOT_PARTITION_STATE: json.dumps(
        {"state": "refused", "mode": "CPX", "ts": time.time() - 2 * pc.backoff_s})}}}, "merge")
    assert [(d.node, d.mode) for d in pc.step()] == [("n1", "CPX")]


def test_request_reverted_without_state_annotation_backs_off():
    """If the agent could not write partition-state, a request of ours whose label came back
    reverted without the mode being applied still counts as refused."""
    fc, r, agents, s, plugin = _cluster()
    for i in range(8):
        fc.create("pods", O.make_pod(f"iso-{i}", gpu_cu=32, annotations_=ISO))
    s.schedule_pending()
    pc = plugin.partitioner
    assert [d.mode for d in pc.step()] == ["CPX"]
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "SPX"}}}, "merge")
    assert pc.step() == [] and pc.backed_off("n1", "CPX")


def _preds_plugin(plugin, conf_row):
    from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions, _Tab
    cp = CachedPredictions()
    cols = ["1P_MI355X", "2P_MI355X", "4P_MI355X", "8P_MI355X"]
    cp._conf = _Tab(["onnx_resnet50_1024"], cols, [conf_row], "t")
    cp._intf = _Tab(["onnx_resnet50_1024_MI355X"], ["onnx_resnet50_1024"], [[0.0]], "t")
    plugin.predictions = cp


def test_slo_only_pod_no_share_can_satisfy_triggers_partition_and_binds():
    """An SLO-only pod (no amd.com/* request) whose SLO the default 64-CU share cannot meet
    (predicted 200 < SLO 250) but a DPX half-GPU can (300): Filter keeps it off shared
    GPUs, the controller sizes it from its predictions (128 CUs) and asks for DPX on the
    IDLE node only -- the busy one keeps its mode -- and after the agent applies and
    republishes, the pod binds to a 128-CU partition."""
    fc, r, agents, s, plugin = _cluster(("n1", "n2"))
    _preds_plugin(plugin, [400.0, 300.0, 200.0, 90.0])
    fc.create("pods", O.make_pod("resident", gpu_cu=64, gpu_mem_gib=4,
                                 node_selector={"kubernetes.io/hostname": "n1"}))
    (res,) = s.schedule_pending()
    assert res.node == "n1"
    fc.create("pods", O.make_pod("onnx-resnet50-1024-slo", slo=250))
    (res,) = s.schedule_pending()
    assert not res.node and "DPX partition" in res.status.message()     # never onto a shared GPU
    dec = plugin.partitioner.step()
    assert [(d.node, d.mode) for d in dec] == [("n2", "DPX")]
    assert O.labels(fc.get("nodes", "n1"))[C.LABEL_COMPUTE_PARTITION] == "SPX"
    pod = fc.get("pods", "onnx-resnet50-1024-slo", "default")
    assert O.annotations(pod)[C.ANNOT_PARTITION_CUS] == "128"
    assert agents["n2"].reconcile_partitions()
    assert _drain(s, fc, ["onnx-resnet50-1024-slo"])
    u = O.annotations(fc.get("pods", "onnx-resnet50-1024-slo", "default"))[C.ANNOT_DEVICES]
    assert {d.device.uuid: d.device.cus for d in plugin.ledger.devices("n2")}[u] == 128


def test_slo_only_pod_a_share_can_satisfy_stays_fractional():
    fc, r, agents, s, plugin = _cluster()
    _preds_plugin(plugin, [400.0, 300.0, 200.0, 90.0])
    fc.create("pods", O.make_pod("onnx-resnet50-1024-ok", slo=150))      # 200 at 64 CUs meets 150
    (res,) = s.schedule_pending()
    assert res.node == "n1" and plugin.partitioner.step() == []
    plugin.args.slo_partitioning = False                                   # opt-out: reference behaviour
    fc.create("pods", O.make_pod("onnx-resnet50-1024-hard", slo=250))
    (res,) = s.schedule_pending()
    assert res.node == "n1"


def test_agent_partition_dry_run_records_amd_smi_calls():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=2))
    src = synthetic_node(2, node="n1")
    ag = NodeAgent("n1", rds(), src, client=fc, partition_dry_run=True)
    ag.step()
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "QPX",
                                                     C.LABEL_MEMORY_PARTITION: "NPS2"}}}, "merge")
    assert not ag.reconcile_partitions()
    assert src.partition_calls == [] and not O.node_taints(fc.get("nodes", "n1"))
    st = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_PARTITION_STATE])
    assert st["state"] == "dry-run"
    assert st["calls"] == [
        {"gpu": 0, "device_index": 0, "call": "amdsmi_set_gpu_memory_partition", "mode": "NPS2"},
        {"gpu": 1, "device_index": 1, "call": "amdsmi_set_gpu_memory_partition", "mode": "NPS2"},
        {"gpu": 0, "device_index": 0, "call": "amdsmi_set_gpu_compute_partition", "mode": "QPX"},
        {"gpu": 1, "device_index": 1, "call": "amdsmi_set_gpu_compute_partition", "mode": "QPX"}]


def test_measured_fabric_steers_quad_away_from_degraded_link():
    """Scripted fabric probe: pair (1, 2) copies at a third of the other pairs' rate.  The
    agent publishes the matrix with the topology (only while idle), and a 4-GPU pod takes
    a quad without that pair although GPUs 0-3 are the first same-NUMA quad."""
    from k8s_gpu_scheduler_amd.agent.fabric import FabricProber, degraded_pairs
    from k8s_gpu_scheduler_amd.plugins.gpu.topology import Topology, select_gpu_set
    bw = [[0.0 if i == j else 120.0 for j in range(8)] for i in range(8)]
    bw[1][2] = bw[2][1] = 40.0
    calls = []

    def probe():
        calls.append(1)
        return {"n": 8, "bw_gbps": bw}
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=8))
    r = rds()
    src = synthetic_node(8, node="n1")
    src.procs = {0: [{"pid": 77, "name": "busy"}]}
    ag = NodeAgent("n1", r, src, client=fc, fabric=FabricProber(probe))
    ag.step()                                                 # publish + probe attempt
    assert calls == []                                        # busy GPUs: deferred
    src.procs = {}
    assert ag.probe_fabric() and not ag.probe_fabric()
    assert calls == [1]                                       # once, when idle
    topo = Topology.from_json(json.loads(r.get(schema.topology_key("n1"))))
    assert topo.pair_bw(1, 2) == 40.0 and degraded_pairs(bw) == [(1, 2), (2, 1)]
    gpus, q = select_gpu_set(topo, list(range(8)), 4)
    assert not {1, 2} <= set(gpus) and q == 1.0
    assert select_gpu_set(Topology.fully_connected(8), list(range(8)), 4)[0] == [0, 1, 2, 3]
    # end to end through the scheduler: the plugin reads the published topology
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, record_events=False,
                  extras={"redis": r})
    s.start_informers()
    fc.create("pods", O.make_pod("ring-4", gpus=4))
    (res,) = s.schedule_pending()
    assert res.node == "n1"
    idx = json.loads(O.annotations(fc.get("pods", "ring-4", "default"))[C.ANNOT_DEVICE_INDICES])
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    gpu_of = {d.device.uuid: d.device.gpu for d in plugin.ledger.devices("n1")}
    assert not {1, 2} <= {gpu_of[a[0]] for a in idx}
    # a partition change makes the probe due again
    ag.fabric.invalidate()
    assert not ag.probe_fabric() and calls == [1]             # the 4-GPU pod runs: not now
    fc.delete("pods", "ring-4", "default")
    assert ag.probe_fabric() and calls == [1, 1]


def test_slo_sized_pod_takes_a_larger_gpu_when_no_node_can_be_cut():
    """Liveness on a busy SPX cluster: the SLO-sized pod needs a 128-CU partition, every node
    has a resident pod (the controller never re-partitions a busy node), so after one
    controller step finds no candidate the pod takes a free whole 256-CU GPU instead of
    staying Pending; an idle node, by contrast, is cut to DPX first (test above)."""
    fc, r, agents, s, plugin = _cluster(("n1", "n2"))
    _preds_plugin(plugin, [400.0, 300.0, 200.0, 90.0])
    for n in ("n1", "n2"):
        fc.create("pods", O.make_pod(f"resident-{n}", gpu_cu=64, gpu_mem_gib=4,
                                     node_selector={"kubernetes.io/hostname": n}))
    assert all(res.node for res in s.schedule_pending())
    fc.create("pods", O.make_pod("onnx-resnet50-1024-slo", slo=250))
    (res,) = s.schedule_pending()
    assert not res.node                                   # a cut might still come: wait for it
    assert plugin.partitioner.step() == [] and plugin.partitioner.stuck == {128}
    assert _drain(s, fc, ["onnx-resnet50-1024-slo"])
    pod = fc.get("pods", "onnx-resnet50-1024-slo", "default")
    u = O.annotations(pod)[C.ANNOT_DEVICES]
    devs = {d.device.uuid: d for n in ("n1", "n2") for d in plugin.ledger.devices(n)}
    assert devs[u].device.cus == 256 and list(devs[u].pods) == ["default/onnx-resnet50-1024-slo"]


def test_background_probes_taint_discard_when_busy_and_publish_bad_sets():
    """agent.probes: the fabric probe runs off the agent's step with the node tainted, a
    result measured while a pod appeared is thrown away, and the RCCL check of a multi-GPU
    pod's GPU set (scripted) reaches the topology key: the degraded set steers the next
    4-GPU pod elsewhere (the probe blocked the agent loop and ran un-tainted)."""
    from k8s_gpu_scheduler_amd.agent.fabric import FabricProber
    from k8s_gpu_scheduler_amd.agent.probes import SetChecker
    from k8s_gpu_scheduler_amd.plugins.gpu.topology import Topology, select_gpu_set
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=8))
    r = rds()
    src = synthetic_node(8, node="n1")
    seen_taints = []

    def fabric_probe():
        seen_taints.append([t["key"] for t in O.node_taints(fc.get("nodes", "n1"))])
        if len(seen_taints) == 1:           # a pod sneaks onto the node mid-probe
            p = O.make_pod("sneaky", gpu_cu=64)
            p["spec"]["nodeName"] = "n1"
            fc.create("pods", p)
        return {"n": 8, "bw_gbps": [[0.0 if i == j else 120.0 for j in range(8)] for i in range(8)]}
    bw = {(0, 1, 2, 3): 80.0, (4, 5, 6, 7): 300.0, (0, 1, 4, 5): 310.0}
    set_calls = []

    def set_probe(gpus):
        set_calls.append(tuple(gpus))
        return {"world": len(gpus), "results": [{"op": "all_reduce", "busbw_gbps": bw[tuple(gpus)]}]}
    sets = SetChecker(set_probe)
    ag = NodeAgent("n1", r, src, client=fc, fabric=FabricProber(fabric_probe), set_checks=sets)
    ag.step()                                   # the step never probes itself
    assert seen_taints == []
    w = ag.probes
    assert w.tick() == "fabric" and w.discarded == 1 and ag.fabric.due      # busy afterwards: discarded
    assert seen_taints == [[C.TAINT_PROBING]]
    assert not O.node_taints(fc.get("nodes", "n1"))                       # untainted again
    assert w.tick() is None                                                # still busy: deferred
    fc.delete("pods", "sneaky", "default")
    assert w.tick() == "fabric" and not ag.fabric.due
    topo = Topology.from_json(json.loads(r.get(schema.topology_key("n1"))))
    assert topo.pair_bw(0, 1) == 120.0
    # three multi-GPU pods ran on these sets (annotated with their devices, now finished)
    uu = [d["uuid"] for d in src.devices()]
    for i, s_ in enumerate(bw):
        p = O.make_pod(f"ring-{i}", gpus=4, phase="Succeeded")
        p["spec"]["nodeName"] = "n1"
        p["metadata"].setdefault("annotations", {})[C.ANNOT_DEVICES] = ",".join(uu[g] for g in s_)
        fc.create("pods", p)
    ag.step()
    assert sorted(sets.pending()) == sorted(bw)
    while w.tick():
        pass
    assert sorted(set_calls) == sorted(bw) and sets.pending() == []
    topo = Topology.from_json(json.loads(r.get(schema.topology_key("n1"))))
    assert topo.bad_sets == [[0, 1, 2, 3]]                     # 80 < 0.6 x median 300
    gpus, q = select_gpu_set(topo, list(range(8)), 4)
    assert gpus != [0, 1, 2, 3] and q < 1.0 or gpus != [0, 1, 2, 3]
    assert select_gpu_set(topo, [0, 1, 2, 3], 4)[1] == 0.5      # only the bad set left: degraded
    ag.step()
    assert sets.pending() == []                                # checked recently: not again


def test_failed_probes_back_off_and_a_failing_set_is_published_bad():
    """a probe that ran on idle GPUs and produced nothing (child crash, RCCL
    timeout, no JSON) stayed due, so the worker re-tainted the node and re-ran it every
    period forever, and a set that hangs RCCL was never marked bad."""
    from k8s_gpu_scheduler_amd.agent.fabric import FabricProber
    from k8s_gpu_scheduler_amd.agent.probes import SetChecker
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=8))
    r = rds()
    src = synthetic_node(8, node="n1")
    calls = {"fabric": 0, "set": 0}

    def fabric_probe():
        calls["fabric"] += 1
        return None

    def set_probe(gpus):
        calls["set"] += 1
        return None
    now = [1000.0]
    sets = SetChecker(set_probe, clock=lambda: now[0], retry_s=300.0, max_failures=2)
    ag = NodeAgent("n1", r, src, client=fc, fabric=FabricProber(fabric_probe), set_checks=sets)
    w = ag.probes
    assert w.tick() == "fabric" and calls["fabric"] == 1 and w.failed == ["fabric"]
    assert not O.node_taints(fc.get("nodes", "n1"))            # untainted after the failed run
    assert w.tick() is None and calls["fabric"] == 1           # backing off: not re-run at once
    # a 4-GPU pod ran on GPUs 0-3; its set check fails twice -> published as a bad set
    uu = [d["uuid"] for d in src.devices()]
    p = O.make_pod("ring", gpus=4, phase="Succeeded")
    p["spec"]["nodeName"] = "n1"
    p["metadata"].setdefault("annotations", {})[C.ANNOT_DEVICES] = ",".join(uu[:4])
    fc.create("pods", p)
    ag.step()
    assert sets.pending() == [(0, 1, 2, 3)]
    assert w.tick() == "set 0,1,2,3" and calls["set"] == 1 and sets.pending() == []
    assert w.tick() is None and calls["set"] == 1              # out of the queue
    ag.step()
    assert sets.pending() == []                                # re-noted only after the back-off
    now[0] += 301.0
    ag.step()
    assert sets.pending() == [(0, 1, 2, 3)]
    assert w.tick() == "set 0,1,2,3" and calls["set"] == 2
    assert sets.bad_sets() == [[0, 1, 2, 3]]
    topo = json.loads(r.get(schema.topology_key("n1")))
    assert [0, 1, 2, 3] in topo["bad_sets"]
    assert not O.node_taints(fc.get("nodes", "n1"))
