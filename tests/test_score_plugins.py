"""kube-scheduler's default Score plugins (framework/score_plugins.py): each plugin alone in a
profile, on a small fake cluster, against the upstream formulas and normalisations."""
import json

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import parse_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.framework.score_plugins import node_selector_term_matches, normalized_image_name
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry


def _cluster(nodes):
    fc = FakeCluster()
    for name, mutate in nodes:
        n = O.make_node(name, gpus=0)
        mutate(n)
        fc.create("nodes", n)
    return fc


def _sched(fc, plugin, weight=1):
    doc = {"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": C.SCHEDULER_NAME, "plugins": {
               "preScore": {"disabled": [{"name": "*"}], "enabled": [{"name": plugin}]},
               "score": {"disabled": [{"name": "*"}], "enabled": [{"name": plugin, "weight": weight}]}}}]}
    s = Scheduler(fc, parse_config(doc), full_registry(), bind_async=False, seed=0)
    s.fast_path = False
    s.start_informers()
    return s


def _pod(name, **spec):
    p = O.make_pod(name, labels_=spec.pop("labels", {}))
    p["spec"].update(spec)
    return p


def _scores(s, fc, pod):
    fc.create("pods", pod)
    (r,) = s.schedule_pending()
    assert r.status.ok, r.status.message()
    return r.node, r.scores


def _label(**kv):
    return lambda n: O.labels(n).update(kv) or n["metadata"].setdefault("labels", {}).update(kv)


def test_taint_toleration_prefers_fewer_intolerable_prefer_no_schedule_taints():
    def taints(*keys):
        return lambda n: n["spec"].__setitem__("taints", [{"key": k, "effect": "PreferNoSchedule"} for k in keys])
    fc = _cluster([("n1", taints()), ("n2", taints("k1")), ("n3", taints("k1", "k2"))])
    s = _sched(fc, "TaintToleration")
    node, sc = _scores(s, fc, _pod("p"))
    assert node == "n1" and sc == {"n1": 100, "n2": 50, "n3": 0}
    node, sc = _scores(s, fc, _pod("q", tolerations=[{"key": "k1", "operator": "Exists", "effect": "PreferNoSchedule"}]))
    assert sc == {"n1": 100, "n2": 100, "n3": 0}


def test_node_affinity_preferred_terms_weighted_and_normalised():
    fc = _cluster([("n1", _label(disk="ssd")), ("n2", _label(disk="hdd", gen="5")), ("n3", _label())])
    s = _sched(fc, "NodeAffinity")
    aff = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 80, "preference": {"matchExpressions": [{"key": "disk", "operator": "In", "values": ["ssd"]}]}},
        {"weight": 20, "preference": {"matchExpressions": [{"key": "gen", "operator": "Gt", "values": ["3"]}]}}]}}
    node, sc = _scores(s, fc, _pod("p", affinity=aff))
    assert node == "n1" and sc == {"n1": 100, "n2": 25, "n3": 0}
    by_name = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 5, "preference": {"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["n3"]}]}}]}}
    node, _ = _scores(s, fc, _pod("q", affinity=by_name))
    assert node == "n3"


def test_node_selector_terms_operators():
    node = O.make_node("n7", gpus=0, labels_={"a": "1", "gen": "5"})
    assert node_selector_term_matches(node, {"matchExpressions": [{"key": "a", "operator": "Exists"}]})
    assert node_selector_term_matches(node, {"matchExpressions": [{"key": "b", "operator": "DoesNotExist"}]})
    assert not node_selector_term_matches(node, {"matchExpressions": [{"key": "gen", "operator": "Lt", "values": ["5"]}]})
    assert node_selector_term_matches(node, {"matchExpressions": [{"key": "a", "operator": "NotIn", "values": ["2"]}],
                                             "matchFields": [{"key": "metadata.name", "operator": "In", "values": ["n7"]}]})
    assert not node_selector_term_matches(node, {})          # an empty term matches nothing


def test_inter_pod_affinity_preferred_terms_and_symmetry():
    zone = "topology.kubernetes.io/zone"
    fc = _cluster([("n1", _label(**{zone: "z1"})), ("n2", _label(**{zone: "z1"})), ("n3", _label(**{zone: "z2"}))])
    s = _sched(fc, "InterPodAffinity")
    fc.create("pods", _pod("db", labels={"app": "db"}, nodeName="n2"))
    term = {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": zone}
    pref = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [{"weight": 10, "podAffinityTerm": term}]}}
    node, sc = _scores(s, fc, _pod("web", affinity=pref))
    assert sc == {"n1": 100, "n2": 100, "n3": 0} and node in ("n1", "n2")
    anti = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [{"weight": 10, "podAffinityTerm": term}]}}
    node, sc = _scores(s, fc, _pod("batch", affinity=anti))
    assert node == "n3" and sc["n3"] == 100 and sc["n1"] == sc["n2"] == 0
    # symmetry: an existing pod's preferred affinity pulls a matching incoming pod to its host
    fc.create("pods", _pod("cache", nodeName="n1", affinity={"podAffinity": {
        "preferredDuringSchedulingIgnoredDuringExecution": [{"weight": 7, "podAffinityTerm": {
            "labelSelector": {"matchLabels": {"app": "api"}}, "topologyKey": "kubernetes.io/hostname"}}]}}))
    node, _ = _scores(s, fc, _pod("api", labels={"app": "api"}))
    assert node == "n1"


def test_pod_topology_spread_schedule_anyway_prefers_the_emptier_domain():
    zone = "topology.kubernetes.io/zone"
    fc = _cluster([("n1", _label(**{zone: "z1"})), ("n2", _label(**{zone: "z1"})), ("n3", _label(**{zone: "z2"}))])
    s = _sched(fc, "PodTopologySpread", weight=2)
    for i, n in enumerate(("n1", "n2")):
        fc.create("pods", _pod(f"x{i}", labels={"app": "x"}, nodeName=n))
    cons = [{"maxSkew": 1, "topologyKey": zone, "whenUnsatisfiable": "ScheduleAnyway",
             "labelSelector": {"matchLabels": {"app": "x"}}}]
    node, sc = _scores(s, fc, _pod("x2", labels={"app": "x"}, topologySpreadConstraints=cons))
    # raw: z1 = round(2 x log(4)) = 3, z2 = 0 -> 100 x (3 + 0 - s) / 3, weight 2
    assert node == "n3" and sc == {"n1": 0, "n2": 0, "n3": 200}


def test_image_locality_scales_by_size_and_spread():
    def images(*names_sizes):
        return lambda n: n.setdefault("status", {}).__setitem__(
            "images", [{"names": [nm], "sizeBytes": sz} for nm, sz in names_sizes])
    fc = _cluster([("n1", images(("registry.local:5000/ml/infer:1.0", 500 * 2**20))), ("n2", images())])
    s = _sched(fc, "ImageLocality")
    p = _pod("p")
    p["spec"]["containers"][0]["image"] = "registry.local:5000/ml/infer:1.0"
    node, sc = _scores(s, fc, p)
    # 500 MB x (1 of 2 nodes) = 250 MB -> 100 x (250 - 23) / (1000 - 23) = 23
    assert node == "n1" and sc == {"n1": 23, "n2": 0}
    assert normalized_image_name("nginx") == "nginx:latest"
    assert normalized_image_name("registry.local:5000/img") == "registry.local:5000/img:latest"
    assert normalized_image_name("img:2") == "img:2"


def test_node_prefer_avoid_pods_annotation():
    avoid = json.dumps({"preferAvoidPods": [{"podSignature": {"podController": {
        "kind": "ReplicaSet", "name": "web-rs", "uid": "rs-1", "controller": True}}, "reason": "maintenance"}]})
    fc = _cluster([("n1", lambda n: n["metadata"].setdefault("annotations", {}).__setitem__(
        C.ANNOT_PREFER_AVOID_PODS, avoid)), ("n2", _label())])
    s = _sched(fc, "NodePreferAvoidPods", weight=10000)
    p = _pod("web-1")
    p["metadata"]["ownerReferences"] = [{"kind": "ReplicaSet", "name": "web-rs", "uid": "rs-1", "controller": True}]
    node, sc = _scores(s, fc, p)
    assert node == "n2" and sc == {"n1": 0, "n2": 1000000}
    node, sc = _scores(s, fc, _pod("standalone"))      # no controller: the plugin skips itself
    assert sc["n1"] == sc["n2"]


def test_default_profile_has_the_upstream_score_plugins_and_weights():
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    prof = default_gpu_config({}).profiles[0]
    weights = {r.name: r.weight for r in prof.enabled("score")}
    assert weights == {"NodeResourcesBalancedAllocation": 1, "ImageLocality": 1, "InterPodAffinity": 1,
                       "NodeResourcesLeastAllocated": 1, "NodeAffinity": 1, "NodePreferAvoidPods": 10000,
                       "PodTopologySpread": 2, "TaintToleration": 1, C.PLUGIN_NAME: C.DEFAULT_SCORE_WEIGHT}
