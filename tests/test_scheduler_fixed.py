"""Scheduler framework + GPU plugin (fixed mode) on a FakeCluster.

Covers BASELINE.json configs on CPU:
  1. busybox pods, no GPU request, 2-node cluster (plugin plumbing)
  3. fractional pods bin-packed onto 8 MI355X by CU units + HBM (+ telemetry)
  4. a 4-GPU pod on an xGMI-connected NUMA-local quad
plus framework semantics: NormalizeScore, weights, Reserve/Unreserve on bind failure,
PreBind env written before bind, restart recovery from annotations, unschedulable
handling, config loading.
"""
import json

import pytest

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config, load_config, parse_config
from k8s_gpu_scheduler_amd.framework.interface import NodeScore, min_max_normalize
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import Conflict, FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger
from k8s_gpu_scheduler_amd.plugins.gpu.topology import Topology, select_gpu_set
from k8s_gpu_scheduler_amd.telemetry.cache import DeviceSample, TelemetryCache


def world(nodes=("node-a",), gpus=8, args=None, **kw):
    fc = FakeCluster()
    for n in nodes:
        fc.create("nodes", O.make_node(n, gpus=gpus))
    ledger, tele = DeviceLedger(), TelemetryCache(stale_s=0)
    s = Scheduler(fc, default_gpu_config(args or {}), full_registry(), bind_async=False, seed=0,
                  extras={"ledger": ledger, "telemetry": tele}, **kw)
    s.start_informers()
    return fc, s, ledger, tele


def test_normalize_score_reference_semantics():
    s = [NodeScore("a", 10), NodeScore("b", 35), NodeScore("c", 60)]
    min_max_normalize(s)
    assert [x.score for x in s] == [0, 50, 100]
    s = [NodeScore("a", 7), NodeScore("b", 7)]
    min_max_normalize(s)
    assert [x.score for x in s] == [0, 0]


def test_config_loader_reference_manifest():
    import os
    p = "/root/reference/deploy/scheduler.yaml"
    text = open(p).read() if os.path.exists(p) else None
    if text is None:
        pytest.skip("reference deploy not mounted")
    cfg = load_config(text)
    prof = cfg.profile("gpu-scheduler")
    assert cfg.leader_election.leader_elect and cfg.leader_election.resource_name == "gpu-scheduler"
    assert [(r.name, r.weight) for r in prof.enabled("score") if r.name == "GPU"] == [("GPU", 10100)]
    assert [r.name for r in prof.enabled("postBind")] == ["GPU"]
    assert "DefaultBinder" in [r.name for r in prof.enabled("bind")]
    # our own deploy manifest parses too
    ours = os.path.join(os.path.dirname(os.path.dirname(__file__)), "deploy", "scheduler.yaml")
    if os.path.exists(ours):
        assert load_config(open(ours).read()).profile("gpu-scheduler") is not None


def test_config_disable_all_and_unknown_api():
    cfg = parse_config({"apiVersion": "kubescheduler.config.k8s.io/v1", "kind": "KubeSchedulerConfiguration",
                        "profiles": [{"schedulerName": "x", "plugins": {"score": {"disabled": [{"name": "*"}],
                                                                                  "enabled": [{"name": "GPU"}]}}}]})
    assert [r.name for r in cfg.profile("x").enabled("score")] == ["GPU"]
    with pytest.raises(ValueError):
        parse_config({"apiVersion": "v0", "kind": "KubeSchedulerConfiguration"})


def test_config1_busybox_two_nodes():
    """busybox pods, no GPU request, 2 nodes: default plugins schedule them, GPU plugin skips."""
    fc, s, _, _ = world(nodes=("node-a", "node-b"), gpus=0)
    fc.create("configmaps", O.make_config_map("game-demo"))
    for i in range(4):
        fc.create("pods", O.make_pod(f"busybox-{i}", config_maps=["game-demo"]))
    res = s.schedule_pending()
    assert all(r.status.ok and r.node in ("node-a", "node-b") for r in res) and len(res) == 4
    assert len(fc.bindings) == 4
    # least-allocated default scoring spreads them
    assert {r.node for r in res} == {"node-a", "node-b"}


def test_slo_only_pod_prefers_gpu_but_does_not_require_one():
    """The reference's busybox fixture carries an SLO env and no GPU request: it must still
    schedule on a CPU-only cluster, and gets a default GPU share where one exists."""
    fc, s, ledger, _ = world(nodes=("node-a", "node-b"), gpus=0)
    fc.create("pods", O.make_pod("busybox-slo", slo=10))
    (r,) = s.schedule_pending()
    assert r.status.ok and ledger.placement("default/busybox-slo") is None
    fc2, s2, ledger2, _ = world()
    fc2.create("pods", O.make_pod("busybox-slo", slo=10))
    (r2,) = s2.schedule_pending()
    assert r2.status.ok and ledger2.placement("default/busybox-slo") is not None
    # an explicit amd.com/gpu-cu request stays a hard requirement
    fc.create("pods", O.make_pod("needs-gpu", gpu_cu=32))
    (r3,) = s.schedule_pending()
    assert not r3.status.ok


def test_config3_fractional_binpack_and_env():
    fc, s, ledger, tele = world()
    fc.create("configmaps", O.make_config_map("env-p0"))
    pods = [O.make_pod(f"p{i}", gpu_cu=64, gpu_mem_gib=16, config_maps=[f"env-p{i}"] if i == 0 else [])
            for i in range(32)]
    for p in pods:
        fc.create("pods", p)
    res = s.schedule_pending()
    assert all(r.status.ok for r in res), [r.status.message() for r in res if not r.status.ok]
    # 32 quarter-GPU pods fill all 8 GPUs exactly: every unit used, 4 pods per GPU
    per_gpu = {}
    for st in ledger.devices("node-a"):
        assert st.free_units == 0
        per_gpu[st.device.gpu] = len(st.pods)
    assert set(per_gpu.values()) == {4}
    # 33rd pod does not fit
    fc.create("pods", O.make_pod("extra", gpu_cu=64))
    (r,) = s.schedule_pending()
    assert not r.status.ok and "GPU" in r.status.message() or "Insufficient" in r.status.message()
    # PreBind wrote the device env before bind
    d = fc.get("configmaps", "env-p0", "default")["data"]
    ann = O.annotations(fc.get("pods", "p0", "default"))
    assert d[C.ENV_ROCR_VISIBLE] == ann[C.ANNOT_DEVICES]
    u0 = json.loads(ann[C.ANNOT_DEVICE_INDICES])[0][1]
    # ROCr syntax, GPU index relative to ROCR_VISIBLE_DEVICES: "0:<cu ranges>"
    assert d[C.ENV_CU_MASK] == f"0:{32 * u0}-{32 * u0 + 63}"
    assert d[C.ENV_HIP_VISIBLE] == "0" and ann[C.ANNOT_CU_MASK] == d[C.ENV_CU_MASK]
    assert d[C.ENV_CUDA_VISIBLE] == d[C.ENV_ROCR_VISIBLE]          # compat keys
    assert d[C.ENV_MPS_THREADS] == "25"


def test_binpack_fills_one_gpu_first_and_spread_policy():
    fc, s, ledger, _ = world()
    for i in range(4):
        fc.create("pods", O.make_pod(f"p{i}", gpu_cu=64))
    s.schedule_pending()
    used = {st.device.gpu for st in ledger.devices("node-a") if st.pods}
    assert len(used) == 1
    fc2, s2, ledger2, _ = world(args={"pack": "spread"})
    for i in range(4):
        fc2.create("pods", O.make_pod(f"p{i}", gpu_cu=64))
    s2.schedule_pending()
    assert len({st.device.gpu for st in ledger2.devices("node-a") if st.pods}) == 4


def test_telemetry_steers_away_from_busy_gpu():
    fc, s, ledger, tele = world(args={"pack": "spread", "w_pack": 0.0, "w_telemetry": 1.0})
    devs = ledger.devices("node-a")
    for st in devs:
        tele.update("node-a", st.device.uuid, DeviceSample(gfx_activity=0.9 if st.device.gpu != 5 else 0.05))
    fc.create("pods", O.make_pod("p", gpu_cu=64))
    s.schedule_pending()
    assert [st.device.gpu for st in ledger.devices("node-a") if st.pods] == [5]


def test_config4_quad_on_numa_local_clique():
    fc, s, ledger, _ = world()
    fc.create("pods", O.make_pod("frac", gpu_cu=32))          # lands on GPU 0 (binpack)
    fc.create("pods", O.make_pod("quad", gpus=4))
    res = s.schedule_pending()
    assert all(r.status.ok for r in res)
    quad = sorted(st.device.gpu for st in ledger.devices("node-a") if "default/quad" in st.pods)
    assert quad == [4, 5, 6, 7]                                   # the only whole free NUMA domain
    env = O.annotations(fc.get("pods", "quad", "default"))[C.ANNOT_DEVICES].split(",")
    assert len(env) == 4
    fc.create("pods", O.make_pod("quad2", gpus=4))
    (r,) = s.schedule_pending()
    assert not r.status.ok                                        # GPU 0 has a fractional resident


def test_topology_selection_rules():
    t = Topology.fully_connected(8)
    assert select_gpu_set(t, range(8), 4)[0] == [0, 1, 2, 3]
    assert select_gpu_set(t, [1, 2, 4, 5, 6, 7], 2)[0] == [1, 2]  # best fit: smaller domain
    t.link_type[0][1] = t.link_type[1][0] = "PCIE"
    assert 1 not in select_gpu_set(t, [0, 1, 2, 3], 3)[0] or 0 not in select_gpu_set(t, [0, 1, 2, 3], 3)[0]
    assert select_gpu_set(t, [0, 1], 2) is None


def test_quad_avoids_busy_xgmi_links():
    """Two equally good NUMA-local quads: live xGMI traffic on one GPU of the first steers
    the 4-GPU pod to the other (telemetry-aware topology Filter/Score, BASELINE config 4)."""
    t = Topology.fully_connected(8)
    assert select_gpu_set(t, range(8), 4, {1: 0.8})[0] == [4, 5, 6, 7]
    assert select_gpu_set(t, range(8), 4, {1: 0.04})[0] == [0, 1, 2, 3]     # below the 10 % quantum
    fc, s, ledger, tele = world()
    for st in ledger.devices("node-a"):
        tele.update("node-a", st.device.uuid,
                    DeviceSample(xgmi_tx_bps=600e9 if st.device.gpu == 2 else 0.0))
    fc.create("pods", O.make_pod("quad", gpus=4))
    (r,) = s.schedule_pending()
    assert r.status.ok
    assert sorted(st.device.gpu for st in ledger.devices("node-a") if st.pods) == [4, 5, 6, 7]


def test_bind_failure_unreserves_and_requeues():
    fc, s, ledger, _ = world()
    fc.fail_next("bind", "pods", Conflict("apiserver says no"))
    fc.create("pods", O.make_pod("p", gpu_cu=128))
    (r,) = s.schedule_pending()
    assert not r.status.ok and s.stats["bind_failures"] == 1
    assert all(not st.pods for st in ledger.devices("node-a"))   # unreserved
    assert ledger.placement("default/p") is None
    s.queue.initial_backoff_s = 0
    s.queue.move_all_to_active_or_backoff()
    res = s.schedule_pending()
    assert res and res[0].status.ok


def test_restart_recovers_reservations_from_annotations():
    fc, s, ledger, _ = world()
    for i in range(3):
        fc.create("pods", O.make_pod(f"p{i}", gpu_cu=64, gpu_mem_gib=8))
    s.schedule_pending()
    before = json.loads(ledger.snapshot_json())
    # a fresh scheduler (process restart) rebuilds the ledger from pod annotations
    ledger2 = DeviceLedger()
    s2 = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False,
                   extras={"ledger": ledger2, "telemetry": TelemetryCache()})
    s2.start_informers()
    assert json.loads(ledger2.snapshot_json()) == before
    # finished pods release capacity
    fc.set_pod_phase("default", "p0", "Succeeded")
    assert ledger2.placement("default/p0") is None


def test_slo_objective_prefers_tight_fit():
    """With predictions, a pod goes where its predicted throughput just exceeds its SLO
    (the reference objective) -- here: the device whose resident interferes
    least."""
    from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions, _Tab
    cp = CachedPredictions()
    cp._conf = _Tab(["wl_a", "wl_b"], ["4P_MI355X"], [[100.0], [100.0]], "t")
    cp._intf = _Tab(["wl_a", "wl_b"], ["wl_a", "wl_b"], [[30.0, 1.0], [1.0, 30.0]], "t")
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n", gpus=2))
    s = Scheduler(fc, default_gpu_config({"w_pack": 0.0, "w_telemetry": 0.0}), full_registry(),
                  bind_async=False, extras={"predictions": cp})
    s.start_informers()
    fc.create("pods", O.make_pod("wl-a-1", gpu_cu=64, slo=60))
    fc.create("pods", O.make_pod("wl-b-1", gpu_cu=64, slo=60))
    s.schedule_pending()
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    g = {k: plugin.ledger.placement(k)[1][0] for k in ("default/wl-a-1", "default/wl-b-1")}
    # second pod of type a should join the device of b (cross interference 1 vs 30)
    fc.create("pods", O.make_pod("wl-a-2", gpu_cu=64, slo=60))
    s.schedule_pending()
    assert plugin.ledger.placement("default/wl-a-2")[1][0] == g["default/wl-b-1"] != g["default/wl-a-1"] \
        or g["default/wl-a-1"] == g["default/wl-b-1"]


def test_adaptive_node_sampling_large_cluster():
    """kube-scheduler's numFeasibleNodesToFind: with 1000 nodes only 42 % are filtered to
    feasibility per cycle (50 - 1000/125), starting where the previous cycle stopped, so
    consecutive pods spread over the cluster; percentageOfNodesToScore=100 scores all."""
    fc, s, ledger, _ = world(nodes=[f"n{i:04d}" for i in range(1000)], gpus=8)
    assert s.num_feasible_nodes_to_find(1000) == 420 and s.num_feasible_nodes_to_find(50) == 50
    assert s.num_feasible_nodes_to_find(100000) == 5000          # 5 % floor
    s.keep_results = True
    for i in range(3):
        fc.create("pods", O.make_pod(f"p{i}", gpu_cu=64))
    res = s.schedule_pending()
    assert all(r.status.ok for r in res) and all(r.evaluated == 420 for r in res)
    s.config.percentage_of_nodes_to_score = 100
    fc.create("pods", O.make_pod("q", gpu_cu=64))
    (r,) = s.schedule_pending()
    assert r.status.ok and r.evaluated == 1000


def test_gpu_aware_preemption():
    """DefaultPreemption (PostFilter, on by default as in kube-scheduler): a high-priority
    pod that finds no free CU units evicts the minimal set of lower-priority pods on the best
    node -- judged by the GPU plugin's what-if ledger -- is nominated there, and lands once
    the victims are gone.  Equal/higher priority pods are never victims."""
    cfg = default_gpu_config({})
    cfg.pod_initial_backoff_s = 0.0
    fc = FakeCluster()
    fc.create("nodes", O.make_node("node-a", gpus=1))
    ledger = DeviceLedger()
    s = Scheduler(fc, cfg, full_registry(), bind_async=False, seed=0, extras={"ledger": ledger})
    s.start_informers()
    s.queue.initial_backoff_s = 0.0
    fc.create("pods", O.make_pod("low-a", gpu_cu=128, priority=1))
    fc.create("pods", O.make_pod("low-b", gpu_cu=64, priority=2))
    fc.create("pods", O.make_pod("same", gpu_cu=64, priority=10))
    assert all(r.status.ok for r in s.schedule_pending())            # GPU full: 128 + 64 + 64
    fc.create("pods", O.make_pod("high", gpu_cu=128, priority=10))
    # cycle 1 fails and preempts; the victim's delete requeues the preemptor at once (the
    # move request arrived during its own cycle), cycle 2 binds it
    r, r2 = s.schedule_pending()
    assert not r.status.ok and "preempt" in r.status.message() and r.nominated == "node-a"
    names = {O.name(p) for p in fc.list("pods")[0]}
    assert names == {"low-b", "same", "high"}                          # one victim: the 128-CU low-a
    assert fc.get("pods", "high", "default")["status"]["nominatedNodeName"] == "node-a"
    assert r2.pod_key == "default/high" and r2.status.ok and r2.node == "node-a"
    # a pod that cannot preempt anything (no lower priority left to evict) stays pending
    fc.create("pods", O.make_pod("never", gpu_cu=128, priority=10))
    (r3,) = s.schedule_pending()
    assert not r3.status.ok and {O.name(p) for p in fc.list("pods")[0]} >= {"low-b", "same", "high"}


def test_default_placement_filters_ports_affinity_spread():
    """kube-scheduler default filters the reference inherited: hostPort conflicts (NodePorts),
    required pod anti-affinity / affinity (InterPodAffinity, incl. symmetry) and
    DoNotSchedule topology spreading (PodTopologySpread)."""
    fc = FakeCluster()
    for n, zone in (("n1", "z1"), ("n2", "z1"), ("n3", "z2")):
        fc.create("nodes", O.make_node(n, gpus=0, labels_={"topology.kubernetes.io/zone": zone}))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, seed=0)
    s.start_informers()

    def pod(name, **spec):
        p = O.make_pod(name, labels_=spec.pop("labels", {}))
        p["spec"].update(spec)
        return p
    # NodePorts: three pods on hostPort 8080 fill three nodes, the fourth cannot fit
    for i in range(4):
        p = pod(f"web-{i}")
        p["spec"]["containers"][0]["ports"] = [{"containerPort": 80, "hostPort": 8080}]
        fc.create("pods", p)
    res = s.schedule_pending()
    assert [r.status.ok for r in res] == [True, True, True, False]
    assert len({r.node for r in res if r.status.ok}) == 3
    assert "free ports" in res[3].status.message()
    for i in range(4):
        fc.delete("pods", f"web-{i}", "default")
    # anti-affinity across zones: one per zone, the third has nowhere to go
    anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "kv"}}, "topologyKey": "topology.kubernetes.io/zone"}]}}
    for i in range(3):
        fc.create("pods", pod(f"kv-{i}", labels={"app": "kv"}, affinity=anti))
    res = s.schedule_pending()
    assert [r.status.ok for r in res] == [True, True, False]
    zones = {O.labels(fc.get("nodes", r.node))["topology.kubernetes.io/zone"] for r in res if r.status.ok}
    assert zones == {"z1", "z2"}
    # symmetry: a plain pod labelled app=kv is repelled by the existing pods' anti-affinity
    fc.delete("pods", "kv-2", "default")
    fc.create("pods", pod("kv-plain", labels={"app": "kv"}))
    (r,) = s.schedule_pending()
    assert not r.status.ok and "anti-affinity" in r.status.message()
    fc.delete("pods", "kv-plain", "default")
    # affinity: co-locate with the db pod's node
    fc.create("pods", pod("db", labels={"app": "db"}, nodeName="n2"))
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "kubernetes.io/hostname"}]}}
    fc.create("pods", pod("cache", affinity=aff))
    (r,) = s.schedule_pending()
    assert r.status.ok and r.node == "n2"
    # topology spread over zones, maxSkew 1
    spread = [{"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "sp"}}}]
    for i in range(4):
        fc.create("pods", pod(f"sp-{i}", labels={"app": "sp"}, topologySpreadConstraints=spread))
    res = s.schedule_pending()
    assert all(r.status.ok for r in res)
    per_zone = {}
    for r in res:
        z = O.labels(fc.get("nodes", r.node))["topology.kubernetes.io/zone"]
        per_zone[z] = per_zone.get(z, 0) + 1
    assert per_zone == {"z1": 2, "z2": 2}


def test_replicas_sharing_a_config_map_keep_their_own_device():
    """replicas referencing one envFrom ConfigMap would overwrite each
    other's device env.  Fixed mode never writes device identity into a shared ConfigMap
    (and removes a stale one); each replica's assignment lives in its own annotations (the
    device plugin's Allocate env), while a pod with a private ConfigMap still gets the env."""
    fc, s, ledger, tele = world()
    fc.create("configmaps", O.make_config_map("game-demo", {C.ENV_ROCR_VISIBLE: "GPU-stale", "OTHER": "x"}))
    fc.create("configmaps", O.make_config_map("private"))
    for i in range(2):
        fc.create("pods", O.make_pod(f"busybox-{i}", gpu_cu=64, gpu_mem_gib=4, config_maps=["game-demo"]))
    fc.create("pods", O.make_pod("solo", gpu_cu=64, gpu_mem_gib=4, config_maps=["private"]))
    res = s.schedule_pending()
    assert all(r.status.ok for r in res)
    shared = fc.get("configmaps", "game-demo", "default")["data"]
    assert shared == {"OTHER": "x"}                 # no device identity, stale key removed
    a0 = O.annotations(fc.get("pods", "busybox-0", "default"))
    a1 = O.annotations(fc.get("pods", "busybox-1", "default"))
    assert (a0[C.ANNOT_DEVICES], a0[C.ANNOT_DEVICE_INDICES]) != (a1[C.ANNOT_DEVICES], a1[C.ANNOT_DEVICE_INDICES])
    priv = fc.get("configmaps", "private", "default")["data"]
    assert priv[C.ENV_ROCR_VISIBLE] == O.annotations(fc.get("pods", "solo", "default"))[C.ANNOT_DEVICES]


@pytest.mark.parametrize("mode,parts", [("CPX", 8), ("QPX", 4)])
def test_multi_device_pods_on_partitions_spread_over_distinct_gpus(mode, parts):
    """a multi-device pod on a partitioned node gets partitions of
    DISTINCT physical GPUs forming an xGMI clique (same NUMA domain first), and two
    multi-device pods never share a physical GPU (its partitions share its xGMI links);
    single-device pods may still use any free partition."""
    fc = FakeCluster()
    fc.create("nodes", O.make_node("node-a", gpus=8, partition=mode))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, seed=0)
    s.start_informers()
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    gpu_of = {st.device.uuid: st.device.gpu for st in plugin.ledger.devices("node-a")}
    assert len(gpu_of) == 8 * parts

    def gpus(name):
        ann = O.annotations(fc.get("pods", name, "default"))[C.ANNOT_DEVICES].split(",")
        return [gpu_of[u] for u in ann]
    fc.create("pods", O.make_pod("ring-a", gpus=4))
    fc.create("pods", O.make_pod("ring-b", gpus=4))
    r = s.schedule_pending()
    assert all(x.status.ok for x in r), [x.status.message() for x in r]
    ga, gb = gpus("ring-a"), gpus("ring-b")
    assert len(set(ga)) == 4 and len(set(gb)) == 4 and not set(ga) & set(gb)
    topo = plugin.topologies["node-a"]
    assert len({topo.numa[g] for g in ga}) == 1 and len({topo.numa[g] for g in gb}) == 1
    fc.create("pods", O.make_pod("ring-c", gpus=2))         # every GPU already carries a ring
    (rc,) = s.schedule_pending()
    assert not rc.node
    fc.create("pods", O.make_pod("single", gpus=1))
    (rs,) = s.schedule_pending()
    assert rs.status.ok and rs.node == "node-a"
