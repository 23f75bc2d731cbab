"""Extender HTTP protocol, Lease leader election, CLI entry points."""
import json
import os
import subprocess
import sys
import time
import urllib.request


from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.extender import Extender, ExtenderServer
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.kube.leader import LeaderElector
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisEngine, FakeRedisServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _post(url, body):
    rq = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(rq, timeout=10) as r:
        return json.loads(r.read())


def test_extender_filter_prioritize_bind():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("gpu-node", gpus=8))
    fc.create("nodes", O.make_node("cpu-node", gpus=0))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False)
    s.start_informers()
    srv = ExtenderServer(Extender(s), "127.0.0.1", 0).start()
    try:
        pod = fc.create("pods", O.make_pod("p", gpu_cu=64, gpu_mem_gib=8, scheduler="default-scheduler"))
        nodes = {"items": [fc.get("nodes", "gpu-node"), fc.get("nodes", "cpu-node")]}
        f = _post(srv.url + "/filter", {"Pod": pod, "Nodes": nodes})
        assert f["NodeNames"] == ["gpu-node"] and "cpu-node" in f["FailedNodes"]
        assert [O.name(n) for n in f["Nodes"]["items"]] == ["gpu-node"]
        pr = _post(srv.url + "/prioritize", {"Pod": pod, "NodeNames": ["gpu-node"]})
        assert pr[0]["Host"] == "gpu-node" and 0 <= pr[0]["Score"] <= 10
        b = _post(srv.url + "/bind", {"PodName": "p", "PodNamespace": "default", "PodUID": O.uid(pod),
                                     "Node": "gpu-node"})
        assert b["Error"] == ""
        got = fc.get("pods", "p", "default")
        assert O.node_name_of(got) == "gpu-node" and C.ANNOT_DEVICES in O.annotations(got)
    finally:
        srv.stop()


def test_leader_election_single_holder_and_failover():
    fc = FakeCluster()
    events = []
    a = LeaderElector(fc, "gpu-scheduler", "kube-system", "a", lease_duration_s=1.0, renew_deadline_s=0.2,
                      retry_period_s=0.05, on_started_leading=lambda: events.append("a+"),
                      on_stopped_leading=lambda: events.append("a-"))
    b = LeaderElector(fc, "gpu-scheduler", "kube-system", "b", lease_duration_s=1.0, renew_deadline_s=0.2,
                      retry_period_s=0.05, on_started_leading=lambda: events.append("b+"))
    assert a.step() and not b.step()
    assert fc.get("leases", "gpu-scheduler", "kube-system")["spec"]["holderIdentity"] == "a"
    time.sleep(1.1)                      # a stops renewing -> lease expires
    assert b.step()
    assert fc.get("leases", "gpu-scheduler", "kube-system")["spec"]["leaseTransitions"] == 1
    assert not a.step() and events == ["a+", "b+", "a-"]
    b.stop(release=True)
    assert fc.get("leases", "gpu-scheduler", "kube-system")["spec"]["holderIdentity"] == ""


def test_cli_redisctl_list_and_flush():
    srv = FakeRedisServer(FakeRedisEngine(password=C.REDIS_PASSWORD)).start()
    try:
        from k8s_gpu_scheduler_amd.store.resp import Redis
        r = Redis.connect(srv.addr, C.REDIS_PASSWORD)
        r.set("node-a", '["GPU-1"]')
        env = dict(os.environ, PYTHONPATH=ROOT)
        p = subprocess.run([sys.executable, "-m", "k8s_gpu_scheduler_amd", "redisctl", "-l", "--redis", srv.addr],
                           capture_output=True, text=True, env=env, timeout=60)
        assert p.returncode == 0 and 'node-a: ["GPU-1"]' in p.stdout
        p = subprocess.run([sys.executable, "-m", "k8s_gpu_scheduler_amd", "redisctl", "-f", "--redis", srv.addr],
                           capture_output=True, text=True, env=env, timeout=60)
        assert p.returncode == 0 and r.get_keys() == []
    finally:
        srv.stop()


def test_cli_agent_once_publishes_synthetic_node():
    srv = FakeRedisServer(FakeRedisEngine(password=C.REDIS_PASSWORD)).start()
    try:
        env = dict(os.environ, PYTHONPATH=ROOT, KUBECONFIG="/nonexistent")
        p = subprocess.run([sys.executable, "-m", "k8s_gpu_scheduler_amd", "agent", "--node", "n7", "--synthetic", "8",
                            "--redis", srv.addr, "--once", "--metrics-port", "0", "--no-discovery"],
                           capture_output=True, text=True, env=env, timeout=60)
        assert p.returncode == 0, p.stderr[-2000:]
        from k8s_gpu_scheduler_amd.store.resp import Redis
        assert len(json.loads(Redis.connect(srv.addr, C.REDIS_PASSWORD).get("n7"))) == 8
    finally:
        srv.stop()


def test_cli_devquery_runs():
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-m", "k8s_gpu_scheduler_amd", "devquery"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert p.returncode == 0 and "hip" in json.loads(p.stdout)
