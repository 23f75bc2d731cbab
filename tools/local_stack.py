"""Run the whole stack locally, each component as its own process, against the HTTP fake
apiserver -- the reference's install (redis, profiler DaemonSet, recommender, scheduler,
busybox fixtures) without a cluster:

  python tools/local_stack.py [--nodes 2] [--gpus 8] [--pods 8] [--real-gpus]

Starts: fake apiserver, Redis (RESP server), recommender (gRPC, reference training data when
mounted, else the measured MI355X tables), one node agent per node (synthetic devices, or the
real ones with --real-gpus), the scheduler (deploy/scheduler.yaml profile, leader election),
then creates the reference's busybox-style pods (SLO env + envFrom ConfigMap) plus fractional
and whole-GPU pods, waits for the bindings and prints each pod's node, devices and CU mask.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from k8s_gpu_scheduler_amd.api import constants as C  # noqa: E402
from k8s_gpu_scheduler_amd.api import objects as O  # noqa: E402
from k8s_gpu_scheduler_amd.kube.rest import RestClient, RestConfig  # noqa: E402
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisEngine, FakeRedisServer  # noqa: E402

REF_DATA = "/root/reference/pkg/recommender/recommender"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


LOGDIR = os.path.join(ROOT, "gpurun_out", "local_stack")


def spawn(args, env=None, log=None):
    """Start one component; its output goes to gpurun_out/local_stack/<log>.log (a pipe nobody
    reads would block a chatty component once the pipe buffer fills)."""
    e = dict(os.environ, PYTHONPATH=ROOT, **(env or {}))
    out = subprocess.PIPE
    if log:
        os.makedirs(LOGDIR, exist_ok=True)
        out = open(os.path.join(LOGDIR, log + ".log"), "w")
    return subprocess.Popen([sys.executable, "-m", "k8s_gpu_scheduler_amd", "--v", "2", *args], cwd=ROOT, env=e,
                            stdout=out, stderr=subprocess.STDOUT, text=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=2)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--real-gpus", action="store_true")
    a = ap.parse_args()
    procs = []
    redis = FakeRedisServer(FakeRedisEngine(password=C.REDIS_PASSWORD)).start()
    try:
        api_port = free_port()
        fc = spawn(["fake-cluster", "--port", str(api_port), "--nodes", str(a.nodes), "--gpus", str(a.gpus)])
        procs.append(fc)
        url = fc.stdout.readline().strip()
        client = RestClient(RestConfig(url))
        nodes = [O.name(n) for n in client.list("nodes")[0]]
        rec_port = free_port()
        data = {}
        if os.path.isdir(REF_DATA):
            data = {"CONFIGURATIONS_DATA_PATH": os.path.join(REF_DATA, "configurations_train.ods"),
                    "INTERFERENCE_DATA_PATH": os.path.join(REF_DATA, "interference_train.ods")}
        else:
            d = os.path.join(ROOT, "k8s_gpu_scheduler_amd", "data")
            data = {"CONFIGURATIONS_DATA_PATH": os.path.join(d, "configurations_mi355x.tsv"),
                    "INTERFERENCE_DATA_PATH": os.path.join(d, "interference_mi355x.tsv")}
        procs.append(spawn(["recommender", "--port", str(rec_port), "--redis", redis.addr], env=data, log="recommender"))
        for n in nodes:
            args = ["agent", "--fake-apiserver", url, "--redis", redis.addr, "--node", n, "--once",
                    "--no-discovery", "--metrics-port", "0"]
            if not a.real_gpus:
                args += ["--synthetic", str(a.gpus)]
            ag = spawn(args, log=f"agent-{n}")
            if ag.wait(120) != 0:
                raise SystemExit(f"agent on {n} failed, see {LOGDIR}")
        procs.append(spawn(["scheduler", "--fake-apiserver", url, "--redis", redis.addr, "--no-discovery",
                            "--recommender", f"127.0.0.1:{rec_port}",
                            "--config", os.path.join(ROOT, "deploy", "scheduler.yaml"), "--metrics-port", "0"], log="scheduler"))
        client.create("configmaps", O.make_config_map("game-demo"))
        names = []
        for i in range(a.pods):          # the reference's busybox fixture: SLO env + envFrom game-demo
            names.append(f"busybox-{i}")
            client.create("pods", O.make_pod(names[-1], slo=10, config_maps=["game-demo"]))
        for i in range(a.pods):
            names.append(f"mlperf-gpu-onnx-resnet50-1024-{i}")
            client.create("pods", O.make_pod(names[-1], gpu_cu=64, gpu_mem_gib=8, slo=150))
        names.append("trainer-4gpu")
        client.create("pods", O.make_pod("trainer-4gpu", gpus=4))
        t0 = time.time()
        while time.time() - t0 < 60:
            pods = {O.name(p): p for p in client.list("pods", "default")[0]}
            if all(O.node_name_of(pods.get(n, {})) for n in names):
                break
            time.sleep(0.2)
        print(f"{'pod':40s} {'node':18s} devices / cu-mask")
        for n in names:
            p = pods.get(n, {})
            ann = O.annotations(p)
            print(f"{n:40s} {O.node_name_of(p) or '-':18s} {ann.get(C.ANNOT_DEVICES, '')[:60]} {ann.get(C.ANNOT_CU_MASK, '')}")
        unbound = [n for n in names if not O.node_name_of(pods.get(n, {}))]
        if unbound:                      # why: the scheduler's FailedScheduling events
            try:
                for ev in client.list("events", "default")[0]:
                    if ev.get("involvedObject", {}).get("name") in unbound:
                        print(f"event {ev['involvedObject']['name']}: {ev.get('reason')}: {ev.get('message')}")
            except Exception as e:
                print(f"(events unavailable: {e})")
        print(json.dumps({"bound": sum(1 for n in names if O.node_name_of(pods.get(n, {}))), "pods": len(names),
                          "seconds": round(time.time() - t0, 2)}))
        print(f"component logs: {LOGDIR}")
        return 0
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        redis.stop()


if __name__ == "__main__":
    sys.exit(main())
