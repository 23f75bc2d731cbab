"""The rest of kube-scheduler v1.21's in-tree registry (the reference's scheduler is that
release, reference go.mod k8s.io/kubernetes v1.21.0): resource scorers with non-zero
request defaults and weights (LeastAllocated, MostAllocated, BalancedAllocation,
RequestedToCapacityRatio), SelectorSpread, ServiceAffinity, NodeLabel, PodTopologySpread's
system default constraints and the in-tree attach limits.  Expected scores are worked out
by hand from the upstream formulas (integer milli-CPU / bytes, Go integer division)."""
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import parse_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry

ZONE = "topology.kubernetes.io/zone"


def _sched(fc, plugin, weight=1, args=None, filter_=False, prefilter=False):
    pre = [{"name": plugin}] if plugin in ("SelectorSpread", "PodTopologySpread") else []
    plugins = {"preScore": {"disabled": [{"name": "*"}], "enabled": pre},
               "score": {"disabled": [{"name": "*"}], "enabled": [{"name": plugin, "weight": weight}]}}
    if filter_:
        plugins["filter"] = {"enabled": [{"name": plugin}]}
    if prefilter:
        plugins["preFilter"] = {"enabled": [{"name": plugin}]}
    prof = {"schedulerName": C.SCHEDULER_NAME, "plugins": plugins}
    if args is not None:
        prof["pluginConfig"] = [{"name": plugin, "args": args}]
    doc = {"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
           "profiles": [prof]}
    s = Scheduler(fc, parse_config(doc), full_registry(), bind_async=False, seed=0)
    s.fast_path = False
    s.start_informers()
    return s


def _node(name, labels=None, **kw):
    return O.make_node(name, gpus=0, labels_=labels or {}, **kw)


def _bare_pod(name, labels=None, **spec):
    p = O.make_pod(name, labels_=labels or {})
    p["spec"]["containers"][0]["resources"] = {}
    p["spec"].update(spec)
    return p


def _run(s, fc, pod):
    fc.create("pods", pod)
    (r,) = s.schedule_pending()
    return r


def _resource_cluster():
    fc = FakeCluster()
    for n in ("n1", "n2"):
        fc.create("nodes", _node(n, cpu="4", memory="8Gi"))
    busy = O.make_pod("busy", cpu="2", memory="2Gi", node_name="n2")
    fc.create("pods", busy)
    return fc


def test_nonzero_requests():
    p = _bare_pod("x")
    assert O.pod_nonzero_requests(p) == (O.DEFAULT_MILLI_CPU_REQUEST, O.DEFAULT_MEMORY_REQUEST)
    q = O.make_pod("y", cpu="250m", memory="0")
    q["spec"]["initContainers"] = [{"name": "init", "resources": {"requests": {"cpu": "1", "memory": "1Gi"}}}]
    q["spec"]["overhead"] = {"cpu": "50m"}
    assert O.pod_nonzero_requests(q) == (1050, 2 ** 30)     # init max, explicit 0 memory kept, overhead


def test_least_allocated_counts_default_requests():
    fc = _resource_cluster()
    r = _run(_sched(fc, "NodeResourcesLeastAllocated"), fc, _bare_pod("p"))
    # n1: cpu (4000-100)*100//4000 = 97, mem 97 -> 97; n2: cpu 1900 -> 47, mem 72 -> (47+72)//2
    assert r.node == "n1" and r.scores == {"n1": 97, "n2": 59}


def test_most_allocated_bin_packs():
    fc = _resource_cluster()
    r = _run(_sched(fc, "NodeResourcesMostAllocated"), fc, _bare_pod("p"))
    assert r.node == "n2" and r.scores == {"n1": 2, "n2": 39}
    # resource weights: memory only
    fc2 = _resource_cluster()
    r = _run(_sched(fc2, "NodeResourcesMostAllocated", args={"resources": [{"name": "memory", "weight": 1}]}),
             fc2, _bare_pod("q"))
    assert r.scores == {"n1": 2, "n2": 27}


def test_balanced_allocation_is_one_minus_the_fraction_gap():
    fc = _resource_cluster()
    r = _run(_sched(fc, "NodeResourcesBalancedAllocation"), fc, _bare_pod("p"))
    assert r.node == "n1" and r.scores == {"n1": 99, "n2": 74}


def test_requested_to_capacity_ratio_broken_linear_shape():
    fc = _resource_cluster()
    args = {"shape": [{"utilization": 0, "score": 0}, {"utilization": 100, "score": 10}],
            "resources": [{"name": "cpu", "weight": 3}, {"name": "memory", "weight": 1}]}
    r = _run(_sched(fc, "RequestedToCapacityRatio", args=args), fc, _bare_pod("p"))
    # n2: cpu utilisation 53, memory 28 -> round((53*3 + 28) / 4) = 47
    assert r.node == "n2" and r.scores == {"n1": 3, "n2": 47}
    import pytest
    with pytest.raises(ValueError):
        _sched(FakeCluster(), "RequestedToCapacityRatio", args={"shape": [{"utilization": 50, "score": 1},
                                                                          {"utilization": 40, "score": 2}]})


def test_selector_spread_blends_node_and_zone_counts():
    fc = FakeCluster()
    for n, z in (("n1", "z1"), ("n2", "z1"), ("n3", "z2")):
        fc.create("nodes", _node(n, {ZONE: z}))
    fc.create("services", {"metadata": {"name": "web", "namespace": "default"}, "spec": {"selector": {"app": "web"}}})
    s = _sched(fc, "SelectorSpread")
    for i, n in enumerate(("n1", "n1", "n3")):
        fc.create("pods", _bare_pod(f"w{i}", {"app": "web"}, nodeName=n))
    r = _run(s, fc, _bare_pod("w9", {"app": "web"}))
    # counts 2/0/1, zones z1=2 z2=1: n2 = 100/3 (empty node, full zone), n3 = 50/3 + 2/3*50
    assert r.node == "n3" and r.scores == {"n1": 0, "n2": 33, "n3": 50}
    r = _run(s, fc, _bare_pod("loner", {"app": "other"}))     # nothing selects it: no preference
    assert r.scores["n1"] == r.scores["n2"] == r.scores["n3"]


def test_service_affinity_filter_and_anti_affinity_score():
    def cluster():
        fc = FakeCluster()
        for n, z in (("n1", "z1"), ("n2", "z1"), ("n3", "z2"), ("n4", "z2")):
            fc.create("nodes", _node(n, {"zone": z}))
        fc.create("services", {"metadata": {"name": "db", "namespace": "default"}, "spec": {"selector": {"app": "db"}}})
        return fc
    fc = cluster()
    s = _sched(fc, "ServiceAffinity", args={"affinityLabels": ["zone"]}, filter_=True, prefilter=True)
    fc.create("pods", _bare_pod("db-0", {"app": "db"}, nodeName="n3"))
    for i in range(3):
        r = _run(s, fc, _bare_pod(f"db-{i + 1}", {"app": "db"}))
        assert r.status.ok and r.node in ("n3", "n4")        # the service's first pod pinned zone z2
    fc = cluster()
    s = _sched(fc, "ServiceAffinity", args={"antiAffinityLabelsPreference": ["zone"]})
    fc.create("pods", _bare_pod("db-0", {"app": "db"}, nodeName="n3"))
    r = _run(s, fc, _bare_pod("db-1", {"app": "db"}))
    assert r.node in ("n1", "n2") and r.scores == {"n1": 100, "n2": 100, "n3": 0, "n4": 0}


def test_node_label_filter_and_preference():
    fc = FakeCluster()
    for n, lab in (("n1", {"gpu": ""}), ("n2", {"gpu": "", "fast": ""}), ("n3", {"gpu": "", "fast": "", "maintenance": ""}),
                   ("n4", {})):
        fc.create("nodes", _node(n, lab))
    s = _sched(fc, "NodeLabel", filter_=True,
               args={"presentLabels": ["gpu"], "absentLabels": ["maintenance"], "presentLabelsPreference": ["fast"]})
    r = _run(s, fc, _bare_pod("p"))
    assert r.node == "n2" and r.scores == {"n1": 0, "n2": 100}


def test_pod_topology_spread_system_defaults_spread_a_replicaset():
    fc = FakeCluster()
    for n in ("n1", "n2", "n3"):
        fc.create("nodes", _node(n))
    fc.create("replicasets", {"metadata": {"name": "api-rs", "namespace": "default"},
                              "spec": {"selector": {"matchLabels": {"app": "api"}}}})
    owner = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "api-rs", "uid": "rs1", "controller": True}]

    def api_pod(name, **spec):
        p = _bare_pod(name, {"app": "api"}, **spec)
        p["metadata"]["ownerReferences"] = owner
        return p
    s = _sched(fc, "PodTopologySpread", weight=2)
    for i, n in enumerate(("n1", "n1", "n2")):
        fc.create("pods", api_pod(f"a{i}", nodeName=n))
    r = _run(s, fc, api_pod("a9"))
    # hostname maxSkew 3: raw round(c x ln 5 + 2) = 5 / 4 / 2 -> 100 x (5 + 2 - s) // 5, weight 2;
    # the zone default adds nothing (no zone labels)
    assert r.node == "n3" and r.scores == {"n1": 80, "n2": 120, "n3": 200}
    r = _run(s, fc, _bare_pod("free"))                        # no owner: no default constraints
    assert len(set(r.scores.values())) == 1
    import pytest
    from k8s_gpu_scheduler_amd.framework.placement_plugins import PodTopologySpread
    with pytest.raises(ValueError):
        PodTopologySpread({"defaultConstraints": [{"maxSkew": 1, "topologyKey": ZONE,
                                                   "whenUnsatisfiable": "DoNotSchedule"}]})
    pts = PodTopologySpread({"defaultingType": "List", "defaultConstraints": []})
    assert pts.spread_constraints(api_pod("z"), "ScheduleAnyway") == ([], False)


def test_in_tree_attach_limits():
    from k8s_gpu_scheduler_amd.framework.volume_plugins import EBSLimits
    fc = FakeCluster()
    n1 = _node("n1")
    n1["status"]["allocatable"]["attachable-volumes-gce-pd"] = "1"
    fc.create("nodes", n1)
    fc.create("nodes", _node("n2"))
    s = _sched(fc, "NodeResourcesLeastAllocated")       # default filters (incl. GCEPDLimits) stay on

    def disk(pd):
        return [{"name": "d", "gcePersistentDisk": {"pdName": pd, "readOnly": True}}]
    fc.create("pods", _bare_pod("a", volumes=disk("pd-a"), nodeName="n1"))
    r = _run(s, fc, _bare_pod("b", volumes=disk("pd-b")))
    assert r.status.ok and r.node == "n2"                 # n1's single GCE PD slot is taken
    r = _run(s, fc, _bare_pod("c", volumes=disk("pd-a"), nodeSelector={"kubernetes.io/hostname": "n1"}))
    assert r.status.ok and r.node == "n1"                 # the same disk needs no new attachment
    r = _run(s, fc, _bare_pod("d", volumes=disk("pd-d"), nodeSelector={"kubernetes.io/hostname": "n1"}))
    assert not r.status.ok and "exceed max volume count" in r.status.message()
    ebs = EBSLimits()
    assert ebs._max(_node("m", {"node.kubernetes.io/instance-type": "m5.large"})) == 25
    assert ebs._max(_node("x", {"node.kubernetes.io/instance-type": "m4.large"})) == 39


def test_workload_resources_over_http():
    from k8s_gpu_scheduler_amd.kube.fake_apiserver import FakeApiServer
    from k8s_gpu_scheduler_amd.kube.rest import RestClient, RestConfig
    srv = FakeApiServer(FakeCluster()).start()
    try:
        rc = RestClient(RestConfig(srv.url))
        rc.create("services", {"metadata": {"name": "web", "namespace": "default"}, "spec": {"selector": {"a": "b"}}})
        rc.create("replicasets", {"metadata": {"name": "rs", "namespace": "default"},
                                  "spec": {"selector": {"matchLabels": {"a": "b"}}}})
        rc.create("statefulsets", {"metadata": {"name": "ss", "namespace": "default"}, "spec": {}})
        assert [O.name(x) for x in rc.list("services", "default")[0]] == ["web"]
        assert rc.get("replicasets", "rs", "default")["kind"] == "ReplicaSet"
        assert rc.get("statefulsets", "ss", "default")["apiVersion"] == "apps/v1"
    finally:
        srv.stop()


def test_fit_ignored_resource_groups():
    from k8s_gpu_scheduler_amd.framework.default_plugins import NodeResourcesFit
    fit = NodeResourcesFit({"ignoredResourceGroups": ["example.com"], "ignoredResources": ["foo.io/bar"]})
    assert fit._ignored("example.com/widget") and fit._ignored("foo.io/bar")
    assert not fit._ignored("amd.com/gpu") and not fit._ignored("cpu")
