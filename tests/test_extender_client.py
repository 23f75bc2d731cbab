"""HTTP scheduler extenders called by the scheduler (config `extenders:`,
framework/extender_client.py): filter narrowing with failure reasons, weighted prioritize,
extender bind, managedResources interest + ignoredByScheduler, ignorable failures."""
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import parse_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry


class _Ext:
    """A scripted extender: rejects `reject`, gives `favour` 10 points, binds through `fc`."""

    def __init__(self, fc, reject=(), favour="", node_cache=False):
        self.fc, self.reject, self.favour, self.node_cache = fc, set(reject), favour, node_cache
        self.calls = []
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
                verb = self.path.strip("/")
                outer.calls.append(verb)
                names = body.get("NodeNames") if "NodeNames" in body else \
                    [n["metadata"]["name"] for n in body["Nodes"]["items"]] if "Nodes" in body else []
                if verb == "filter":
                    keep = [n for n in names if n not in outer.reject]
                    out = {"FailedNodes": {n: "licence server says no" for n in names if n in outer.reject}}
                    if outer.node_cache:
                        out["NodeNames"] = keep
                    else:
                        out["Nodes"] = {"items": [n for n in body["Nodes"]["items"] if n["metadata"]["name"] in keep]}
                elif verb == "prioritize":
                    out = [{"Host": n, "Score": 10 if n == outer.favour else 0} for n in names]
                elif verb == "bind":
                    outer.fc.bind(body["PodNamespace"], body["PodName"], body["Node"], body["PodUID"])
                    out = {"Error": ""}
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                data = json.dumps(out).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)
        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"

    def stop(self):
        self.srv.shutdown()
        self.srv.server_close()


def _cluster(n=3):
    fc = FakeCluster()
    for i in range(1, n + 1):
        fc.create("nodes", O.make_node(f"n{i}", gpus=0))
    return fc


def _sched(fc, extenders):
    doc = {"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": C.SCHEDULER_NAME}], "extenders": extenders}
    s = Scheduler(fc, parse_config(doc), full_registry(), bind_async=False, seed=0)
    s.start_informers()
    return s


def test_filter_prioritize_bind_through_an_extender():
    fc = _cluster()
    ext = _Ext(fc, reject=("n1",), favour="n3")
    try:
        s = _sched(fc, [{"urlPrefix": ext.url, "filterVerb": "filter", "prioritizeVerb": "prioritize",
                         "bindVerb": "bind", "weight": 5}])
        assert not s.fast_path
        fc.create("pods", O.make_pod("p"))
        (r,) = s.schedule_pending()
        assert r.status.ok and r.node == "n3" and r.bound
        assert set(r.scores) == {"n2", "n3"} and r.scores["n3"] - r.scores["n2"] >= 10 * 5 * 10 - 100
        assert fc.get("pods", "p", "default")["spec"]["nodeName"] == "n3"
        assert ext.calls == ["filter", "prioritize", "bind"]
        assert fc.bindings[-1][2] == "n3"
    finally:
        ext.stop()


def test_extender_rejecting_everything_reports_its_reason():
    fc = _cluster(2)
    ext = _Ext(fc, reject=("n1", "n2"), node_cache=True)
    try:
        s = _sched(fc, [{"urlPrefix": ext.url, "filterVerb": "filter", "nodeCacheCapable": True}])
        fc.create("pods", O.make_pod("p"))
        (r,) = s.schedule_pending()
        assert not r.status.ok and "licence server says no" in r.status.message()
    finally:
        ext.stop()


def test_managed_resources_interest_and_ignored_by_scheduler():
    fc = _cluster()
    ext = _Ext(fc, reject=("n1", "n2"))
    try:
        cfg = [{"urlPrefix": ext.url, "filterVerb": "filter",
                "managedResources": [{"name": "example.com/licence", "ignoredByScheduler": True}]}]
        s = _sched(fc, cfg)
        fc.create("pods", O.make_pod("plain"))                  # not interested: no extender call
        (r,) = s.schedule_pending()
        assert r.status.ok and ext.calls == []
        p = O.make_pod("licensed")
        p["spec"]["containers"][0]["resources"]["limits"]["example.com/licence"] = "1"
        fc.create("pods", p)
        (r,) = s.schedule_pending()
        # the nodes have no example.com/licence at all: NodeResourcesFit ignores it, the extender decides
        assert r.status.ok and r.node == "n3" and ext.calls == ["filter"]
        assert "example.com/licence" in parse_config({"extenders": cfg, "profiles": [{}]}).profiles[0] \
            .args("NodeResourcesFit")["ignoredResources"]
    finally:
        ext.stop()


def test_unreachable_extender_fails_unless_ignorable():
    fc = _cluster()
    s = _sched(fc, [{"urlPrefix": "http://127.0.0.1:9", "filterVerb": "filter", "httpTimeout": "1s"}])
    fc.create("pods", O.make_pod("p"))
    (r,) = s.schedule_pending()
    assert not r.status.ok and "extender" in r.status.message()
    fc2 = _cluster()
    s2 = _sched(fc2, [{"urlPrefix": "http://127.0.0.1:9", "filterVerb": "filter", "ignorable": True,
                       "httpTimeout": 1000000000}])
    assert s2.extenders[0].cfg.http_timeout_s == 1.0
    fc2.create("pods", O.make_pod("p"))
    (r,) = s2.schedule_pending()
    assert r.status.ok


def test_config_validation():
    with pytest.raises(ValueError):
        parse_config({"extenders": [{"filterVerb": "filter"}]})
    with pytest.raises(ValueError):
        parse_config({"extenders": [{"urlPrefix": "a", "bindVerb": "b"}, {"urlPrefix": "c", "bindVerb": "b"}]})
