"""System test of the shipped entry points as separate processes (CPU): the HTTP fake
apiserver (`fake-cluster`), the node agent (`agent --synthetic`) publishing to a Redis
server, and the scheduler (`scheduler` with our deploy/scheduler.yaml config, leader
election on a Lease) -- pods created over REST get bound with their device assignment, and
the scheduler's /metrics counts them."""
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.kube.rest import RestClient, RestConfig
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisEngine, FakeRedisServer
from k8s_gpu_scheduler_amd.store.resp import Redis

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(args, **kw):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.Popen([sys.executable, "-m", "k8s_gpu_scheduler_amd", *args], cwd=ROOT, env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, **kw)


def _wait(pred, timeout=60.0, every=0.2):
    t = time.time()
    while time.time() - t < timeout:
        v = pred()
        if v:
            return v
        time.sleep(every)
    return None


@pytest.mark.timeout(240)
def test_scheduler_agent_apiserver_as_processes(tmp_path):
    procs = []
    redis = FakeRedisServer(FakeRedisEngine(password=C.REDIS_PASSWORD)).start()
    try:
        api_port = _free_port()
        fc = _spawn(["fake-cluster", "--port", str(api_port), "--nodes", "1", "--gpus", "8"])
        procs.append(fc)
        url = fc.stdout.readline().strip()
        assert url.startswith("http"), url
        client = RestClient(RestConfig(url))
        node = O.name(client.list("nodes")[0][0])
        raddr = redis.addr
        ag = _spawn(["agent", "--fake-apiserver", url, "--redis", raddr, "--node", node, "--synthetic", "8",
                     "--once", "--no-discovery", "--metrics-port", "0"])
        assert ag.wait(120) == 0, ag.stdout.read()
        mport = _free_port()
        sc = _spawn(["scheduler", "--fake-apiserver", url, "--redis", raddr, "--no-discovery",
                     "--config", os.path.join(ROOT, "deploy", "scheduler.yaml"), "--metrics-port", str(mport)])
        procs.append(sc)
        client.create("configmaps", O.make_config_map("env-a"))
        for i in range(4):
            client.create("pods", O.make_pod(f"onnx-resnet50-1024-{i}", gpu_cu=64, gpu_mem_gib=8, slo=100,
                                             config_maps=["env-a"] if i == 0 else []))
        client.create("pods", O.make_pod("whole", gpus=2))

        def all_bound():
            pods = client.list("pods", "default")[0]
            return pods if len(pods) == 5 and all(O.node_name_of(p) for p in pods) else None
        pods = _wait(all_bound, 120)
        assert pods, [(O.name(p), O.node_name_of(p)) for p in client.list("pods", "default")[0]]
        by = {O.name(p): p for p in pods}
        uuids = json.loads(Redis.connect(raddr, C.REDIS_PASSWORD).get(node) or "[]")
        ann = O.annotations(by["onnx-resnet50-1024-0"])
        assert ann[C.ANNOT_DEVICES].startswith("GPU-") and ann[C.ANNOT_CU_MASK].startswith("0:")
        if uuids:
            assert ann[C.ANNOT_DEVICES] in uuids
        assert len(O.annotations(by["whole"])[C.ANNOT_DEVICES].split(",")) == 2
        env = client.get("configmaps", "env-a", "default")["data"]
        assert env[C.ENV_ROCR_VISIBLE] == ann[C.ANNOT_DEVICES]
        # the leader holds the Lease named in the config
        lease = client.get("leases", "gpu-scheduler", "kube-system")
        assert lease["spec"]["holderIdentity"]
        txt = _wait(lambda: (lambda t: t if 'result="scheduled"} 5.0' in t else None)(
            urllib.request.urlopen(f"http://127.0.0.1:{mport}/metrics", timeout=5).read().decode()), 30)
        assert txt, "scheduler metrics missing"
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        redis.stop()


@pytest.mark.timeout(240)
def test_agent_serves_device_plugin_to_kubelet_as_process(tmp_path):
    """The DaemonSet's command line (`agent --device-plugin`) as a process: it registers the
    three resources with a (fake) kubelet and answers Allocate for a pod the scheduler
    placed -- over Unix sockets, across processes."""
    from concurrent import futures

    import grpc

    from k8s_gpu_scheduler_amd.agent import deviceplugin as dp
    procs = []
    redis = FakeRedisServer(FakeRedisEngine(password=C.REDIS_PASSWORD)).start()
    regs = []
    kubelet = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
    kubelet.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(dp.REG_SERVICE, {
        "Register": grpc.unary_unary_rpc_method_handler(
            lambda req, ctx: (regs.append(req.resource_name), dp.Empty())[1],
            request_deserializer=dp.RegisterRequest.FromString, response_serializer=dp.Empty.SerializeToString)}),))
    kubelet.add_insecure_port(f"unix://{tmp_path}/kubelet.sock")
    kubelet.start()
    try:
        api_port = _free_port()
        fc = _spawn(["fake-cluster", "--port", str(api_port), "--nodes", "1", "--gpus", "8"])
        procs.append(fc)
        url = fc.stdout.readline().strip()
        client = RestClient(RestConfig(url))
        node = O.name(client.list("nodes")[0][0])
        ag = _spawn(["agent", "--fake-apiserver", url, "--redis", redis.addr, "--node", node, "--synthetic", "8",
                     "--no-discovery", "--metrics-port", "0", "--poll", "0.5",
                     "--device-plugin", "--device-plugin-dir", str(tmp_path)])
        procs.append(ag)
        assert _wait(lambda: len(regs) >= 3, 60), regs
        assert sorted(regs) == sorted(dp.RESOURCES)
        sc = _spawn(["scheduler", "--fake-apiserver", url, "--redis", redis.addr, "--no-discovery",
                     "--config", os.path.join(ROOT, "deploy", "scheduler.yaml"), "--metrics-port", "0"])
        procs.append(sc)
        client.create("pods", O.make_pod("frac-0", gpu_cu=64, gpu_mem_gib=8, gpu_limits=True))
        pod = _wait(lambda: (lambda p: p if O.node_name_of(p) else None)(client.get("pods", "frac-0", "default")), 90)
        if not pod:
            for p in procs:
                p.terminate()
            logs = "\n".join(f"--- {p.args[3:5]}\n" + (p.communicate(timeout=10)[0] or "")[-3000:] for p in procs)
            raise AssertionError("pod not bound; process output:\n" + logs)
        ch = grpc.insecure_channel(f"unix://{tmp_path}/{dp.socket_name(C.RESOURCE_GPU_CU)}")
        alloc = ch.unary_unary(f"/{dp.PLUGIN_SERVICE}/Allocate", request_serializer=dp.AllocateRequest.SerializeToString,
                               response_deserializer=dp.AllocateResponse.FromString)
        req = dp.AllocateRequest()
        req.container_requests.add(devices_ids=[f"tok{k}" for k in range(64)])
        resp = alloc(req, timeout=10).container_responses[0]
        ann = O.annotations(pod)
        assert resp.envs[C.ENV_ROCR_VISIBLE] == ann[C.ANNOT_DEVICES]
        assert resp.envs[C.ENV_CU_MASK] == ann[C.ANNOT_CU_MASK]
        ch.close()
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        kubelet.stop(0)
        redis.stop()


@pytest.mark.timeout(240)
def test_live_telemetry_reaches_deployed_scheduler_as_processes():
    """fake apiserver, node agent (scripted amd-smi samples: GPU 0 at 95 %, GPU 1 idle,
    exported on /metrics) and scheduler (`--telemetry-scrape` poller) as three processes:
    the busy GPU loses Score, so the pod lands on the idle one."""
    procs = []
    redis = FakeRedisServer(FakeRedisEngine(password=C.REDIS_PASSWORD)).start()
    try:
        fc = _spawn(["fake-cluster", "--port", str(_free_port()), "--nodes", "1", "--gpus", "2"])
        procs.append(fc)
        url = fc.stdout.readline().strip()
        client = RestClient(RestConfig(url))
        node = O.name(client.list("nodes")[0][0])
        mport = _free_port()
        samples = [{"index": 0, "gfx_activity": 95.0, "vram_used_mb": 2048.0, "vram_total_mb": 294912.0},
                   {"index": 1, "gfx_activity": 0.0, "vram_used_mb": 16.0, "vram_total_mb": 294912.0}]
        ag = _spawn(["agent", "--fake-apiserver", url, "--redis", redis.addr, "--node", node, "--synthetic", "2",
                     "--synthetic-samples", json.dumps(samples), "--no-discovery", "--metrics-port", str(mport),
                     "--poll", "0.3"])
        procs.append(ag)
        murl = f"http://127.0.0.1:{mport}/metrics"

        def exported():
            try:
                return "amd_gpu_gfx_activity" in urllib.request.urlopen(murl, timeout=2).read().decode()
            except Exception:
                return False
        assert _wait(exported, 90), "agent exporter not serving"
        sc = _spawn(["scheduler", "--fake-apiserver", url, "--redis", redis.addr, "--no-discovery",
                     "--config", os.path.join(ROOT, "deploy", "scheduler.yaml"), "--metrics-port", "0",
                     "--telemetry-scrape", murl, "--telemetry-period", "0.3"])
        procs.append(sc)
        r = Redis.connect(redis.addr, C.REDIS_PASSWORD)
        devs = _wait(lambda: json.loads(r.get_or("gpusched:devices:" + node) or "null"), 30)
        assert devs, "agent did not publish descriptors"
        by_gpu = {d["gpu"]: d["uuid"] for d in devs}
        time.sleep(4.0)        # leader election + informer sync + a few telemetry polls
        client.create("pods", O.make_pod("tele-0", gpu_cu=64, gpu_mem_gib=4))
        pod = _wait(lambda: (lambda p: p if O.node_name_of(p) else None)(client.get("pods", "tele-0", "default")), 90)
        assert pod, "pod not bound"
        assert O.annotations(pod)[C.ANNOT_DEVICES] == by_gpu[1], (O.annotations(pod), by_gpu)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        redis.stop()
