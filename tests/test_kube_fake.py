"""FakeCluster apiserver, patches, selectors, informers, resources helpers.

The reference tests these paths only against a live cluster
(reference pkg/resources/pods_test.go, nodes_test.go); here they run hermetically.
"""
import threading
import time

import pytest

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.kube.client import AlreadyExists, Conflict, FakeCluster, Gone, NotFound
from k8s_gpu_scheduler_amd.kube.informer import SharedInformerFactory
from k8s_gpu_scheduler_amd.kube.patch import (PatchError, apply_json_patch, apply_merge_patch,
                                               match_field_selector, match_label_selector)
from k8s_gpu_scheduler_amd.kube.resources import Resources


def test_json_patch_ops():
    doc = {"metadata": {"labels": {"a": "1"}}, "spec": {"l": [1, 2]}}
    out = apply_json_patch(doc, [
        {"op": "replace", "path": "/metadata/labels", "value": {"b": "2"}},
        {"op": "add", "path": "/spec/l/-", "value": 3},
        {"op": "add", "path": "/spec/l/0", "value": 0},
        {"op": "remove", "path": "/spec/l/1"},
        {"op": "copy", "from": "/spec/l", "path": "/spec/m"},
        {"op": "test", "path": "/metadata/labels/b", "value": "2"},
        {"op": "add", "path": "/metadata/annotations", "value": {"x~y": "z"}},
        {"op": "replace", "path": "/metadata/annotations/x~0y", "value": "w"},
    ])
    assert out["metadata"]["labels"] == {"b": "2"}
    assert out["spec"]["l"] == [0, 2, 3] and out["spec"]["m"] == [0, 2, 3]
    assert out["metadata"]["annotations"] == {"x~y": "w"}
    assert doc["spec"]["l"] == [1, 2]                     # input untouched
    with pytest.raises(PatchError):
        apply_json_patch(doc, [{"op": "test", "path": "/spec/l/0", "value": 9}])


def test_merge_patch():
    assert apply_merge_patch({"a": {"b": 1, "c": 2}, "d": 1}, {"a": {"b": None, "e": 3}, "d": [1]}) == \
        {"a": {"c": 2, "e": 3}, "d": [1]}


def test_selectors():
    pod = O.make_pod("p", node_name="n1", phase="Running")
    assert match_field_selector(pod, "spec.nodeName=n1")
    assert match_field_selector(pod, "spec.nodeName==n1,status.phase=Running")
    assert not match_field_selector(pod, "spec.nodeName!=n1")
    lab = {"app": "x", "tier": "gpu"}
    assert match_label_selector(lab, "app=x,tier in (gpu,cpu),!missing")
    assert not match_label_selector(lab, "tier notin (gpu)")
    assert match_label_selector(lab, {"matchLabels": {"app": "x"},
                                      "matchExpressions": [{"key": "tier", "operator": "Exists"}]})


def test_crud_conflict_bind():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1"))
    p = fc.create("pods", O.make_pod("p1"))
    with pytest.raises(AlreadyExists):
        fc.create("pods", O.make_pod("p1"))
    stale = dict(p)
    p2 = fc.patch("pods", "p1", {"metadata": {"labels": {"x": "1"}}}, "merge", "default")
    assert O.labels(p2) == {"x": "1"}
    with pytest.raises(Conflict):
        fc.update("pods", stale)                       # old resourceVersion
    fc.bind("default", "p1", "n1")
    got = fc.get("pods", "p1", "default")
    assert O.node_name_of(got) == "n1" and O.phase(got) == "Running"
    with pytest.raises(Conflict):
        fc.bind("default", "p1", "n1")
    with pytest.raises(NotFound):
        fc.bind("default", "nope", "n1")
    fc.delete("pods", "p1", "default")
    with pytest.raises(NotFound):
        fc.get("pods", "p1", "default")


def test_fault_injection():
    fc = FakeCluster()
    fc.fail_next("create", "pods", Conflict("boom"))
    with pytest.raises(Conflict):
        fc.create("pods", O.make_pod("a"))
    fc.create("pods", O.make_pod("a"))


def test_watch_resume_and_gone():
    fc = FakeCluster(history=5)
    fc.create("configmaps", O.make_config_map("a"))
    rv = fc.resource_version
    fc.create("configmaps", O.make_config_map("b"))
    evs = list(fc.watch("configmaps", resource_version=rv, timeout_s=0.05))
    assert [O.name(e["object"]) for e in evs] == ["b"]
    for i in range(10):
        fc.create("configmaps", O.make_config_map(f"c{i}"))
    with pytest.raises(Gone):
        list(fc.watch("configmaps", resource_version="1", timeout_s=0.05))


def test_informer_sync_and_threaded():
    fc = FakeCluster()
    fc.create("pods", O.make_pod("a"))
    inf = SharedInformerFactory(fc)
    seen = []
    inf.pods().add_event_handler(lambda o: seen.append(("add", O.name(o))),
                                 lambda o, n: seen.append(("upd", O.name(n))),
                                 lambda o: seen.append(("del", O.name(o))))
    inf.start()
    assert inf.wait_for_cache_sync(1)
    fc.create("pods", O.make_pod("b"))
    fc.patch("pods", "b", {"metadata": {"labels": {"k": "v"}}}, "merge", "default")
    fc.delete("pods", "a", "default")
    assert seen == [("add", "a"), ("add", "b"), ("upd", "b"), ("del", "a")]
    assert inf.pods().lister.get("b", "default") is not None
    # queue-backed (threaded) informer on a non-sync cluster
    fc2 = FakeCluster(sync_watch=False)
    fc2.create("nodes", O.make_node("n1"))
    inf2 = SharedInformerFactory(fc2)
    names = []
    inf2.nodes().add_event_handler(lambda o: names.append(O.name(o)))
    inf2.start()
    assert inf2.wait_for_cache_sync(5)
    fc2.create("nodes", O.make_node("n2"))
    deadline = time.time() + 5
    while "n2" not in names and time.time() < deadline:
        time.sleep(0.01)
    assert names == ["n1", "n2"]
    inf2.stop()
    fc2.close_watches()


def test_resources_helpers_reference_semantics():
    """AppendToExistingConfigMapsInPod / UpdateConfigMap overwrite flag / LabelNode
    (reference pkg/resources/pods.go:98-174, nodes.go:39-68)."""
    fc = FakeCluster()
    fc.create("nodes", O.make_node("k8s-aferik-master", labels_={"role": "master"}))
    fc.create("nodes", O.make_node("k8s-aferik-gpu-a30"))
    fc.create("configmaps", O.make_config_map("game-demo", {"keep": "1"}))
    fc.create("configmaps", O.make_config_map("other"))
    fc.create("pods", O.make_pod("mlperf-gpu-onnx-mobilenet-1024", config_maps=["game-demo", "other"]))
    r = Resources(fc, "default")
    assert r.append_to_existing_config_maps_in_pod("mlperf-gpu-onnx-mobilenet-1024",
                                                   {"CUDA_VISIBLE_DEVICES": "test"}) == 2
    assert fc.get("configmaps", "other", "default")["data"] == {"CUDA_VISIBLE_DEVICES": "test"}
    r.update_config_map("game-demo", {"keep": "2", "new": "x"}, overwrite=False)
    assert fc.get("configmaps", "game-demo", "default")["data"] == {"keep": "1", "CUDA_VISIBLE_DEVICES": "test",
                                                                     "new": "x"}
    r.create_config_map("woohoo", {"1": "2"})
    assert r.get_config_map("woohoo")["data"] == {"1": "2"}
    n = r.label_node("k8s-aferik-gpu-a30", {C.LABEL_MIG_CONFIG: "all-1g.6gb"})
    assert O.labels(n)[C.LABEL_MIG_CONFIG] == "all-1g.6gb"
    # parity: labels copied from the hard-coded master node (reference nodes.go:29,43-50)
    n = r.label_node("k8s-aferik-gpu-a30", {C.LABEL_MIG_CONFIG: "all-2g.12gb"},
                     parity_master="k8s-aferik-master")
    assert O.labels(n)["role"] == "master"
    sel = Resources(fc, "default", "spec.nodeName=nowhere")
    assert sel.list_pods() == []                        # field selector honoured (fixed)


def test_concurrent_configmap_updates_retry():
    fc = FakeCluster()
    fc.create("configmaps", O.make_config_map("cm"))
    r = Resources(fc, "default")
    errs = []

    def worker(i):
        try:
            for j in range(20):
                r.update_config_map("cm", {f"k{i}-{j}": "v"})
        except Exception as e:
            errs.append(e)
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs
    assert len(fc.get("configmaps", "cm", "default")["data"]) == 80


def test_shared_configmap_writers_over_http_never_give_up():
    """16 concurrent binding-cycle-like writers over the REST client (HTTP fake apiserver)
    on one shared ConfigMap -- the reference's busybox replicas sharing `game-demo` -- plus
    an out-of-process-style writer bypassing the in-process lock: every update lands."""
    from k8s_gpu_scheduler_amd.kube.fake_apiserver import FakeApiServer
    from k8s_gpu_scheduler_amd.kube.rest import RestClient, RestConfig
    fc = FakeCluster()
    fc.create("configmaps", O.make_config_map("game-demo"))
    srv = FakeApiServer(fc).start()
    try:
        rc = RestClient(RestConfig(srv.url))
        r = Resources(rc, "default")
        errs = []

        def worker(i):
            try:
                for j in range(5):
                    r.update_config_map("game-demo", {f"pod{i}-{j}": "GPU-x"})
            except Exception as e:
                errs.append(e)

        def rogue():                        # another process's writer: optimistic retries only
            try:
                for j in range(10):
                    r._update_config_map("game-demo", {f"rogue-{j}": "1"}, True, 10)
            except Exception as e:
                errs.append(e)
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(16)] + [threading.Thread(target=rogue)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert not errs, errs[:3]
        assert len(fc.get("configmaps", "game-demo", "default")["data"]) == 16 * 5 + 10
    finally:
        srv.stop()
