"""Scheduler-only throughput (CPU): pods scheduled/s through the full framework cycle on a
FakeCluster, for the BASELINE configs that do not need a GPU, and the reference's own
algorithm (parity mode: one recommender RPC per lookup, ConfigMap writes in Score) as the
comparison point.  Writes profiles/sched_throughput.json when --out is given.

  python tools/sched_throughput.py [--pods 400] [--out profiles/sched_throughput.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_scheduler_amd.api import objects as O  # noqa: E402
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config, load_config  # noqa: E402
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler  # noqa: E402
from k8s_gpu_scheduler_amd.kube.client import FakeCluster  # noqa: E402
from k8s_gpu_scheduler_amd.plugins import full_registry  # noqa: E402

REF = "/root/reference/pkg/recommender/recommender"
PARITY_PROFILE = """
apiVersion: kubescheduler.config.k8s.io/v1beta1
kind: KubeSchedulerConfiguration
profiles:
- schedulerName: gpu-scheduler
  plugins:
    score: {enabled: [{name: GPU, weight: 10100}]}
    postBind: {enabled: [{name: GPU}]}
  pluginConfig:
  - name: GPU
    args: {mode: parity, seed: 1}
"""


FAST = True      # framework.fastpath cross-cycle node-result cache (--no-fast-path: off)


def run(fc, sched, pods, batch=None):
    sched.fast_path = FAST
    for p in pods:
        fc.create("pods", p)
    t = time.perf_counter()
    res = sched.schedule_pending()
    dt = time.perf_counter() - t
    ok = sum(1 for r in res if r.status.ok)
    return {"pods": len(res), "scheduled": ok, "seconds": round(dt, 4), "pods_per_s": round(ok / dt, 1),
            "ms_per_pod": round(dt / max(len(res), 1) * 1e3, 4)}


def busybox(n):
    fc = FakeCluster()
    for i in range(2):
        fc.create("nodes", O.make_node(f"node-{i}", gpus=0, cpu="1000"))
    fc.create("configmaps", O.make_config_map("game-demo"))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, record_events=False)
    s.keep_results = True
    s.start_informers()
    return run(fc, s, [O.make_pod(f"busybox-{i}", config_maps=["game-demo"], slo=10) for i in range(n)])


def fractional(n, nodes=4):
    fc = FakeCluster()
    for i in range(nodes):
        fc.create("nodes", O.make_node(f"mi355x-{i}", gpus=8))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, record_events=False)
    s.start_informers()
    return run(fc, s, [O.make_pod(f"onnx-resnet50-1024-{i}", gpu_cu=32, gpu_mem_gib=4, slo=100)
                       for i in range(min(n, nodes * 64))])


def parity_rpc(n):
    """The reference's algorithm on a 2-node V100-style cluster with residents, every
    prediction over gRPC (new channel per call, like client_call.go:13)."""
    if not os.path.isdir(REF):
        return {"skipped": "reference data not mounted"}
    import json as _j
    from k8s_gpu_scheduler_amd.recommender.client import RecommenderClient, RpcPredictions
    from k8s_gpu_scheduler_amd.recommender.service import RecommenderService
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    svc = RecommenderService(os.path.join(REF, "configurations_train.ods"), os.path.join(REF, "interference_train.ods"))
    svc.train()
    srv, port = svc.make_server(0, 10, "127.0.0.1")
    try:
        fc = FakeCluster()
        redis = Redis(FakeRedisBackend(FakeRedisEngine()))
        for nn in ("k8s-gpu-1", "k8s-gpu-2"):              # "gpu" in the name -> V100 (parity naming)
            fc.create("nodes", O.make_node(nn, gpus=0, cpu="1000"))
            uuid = f"GPU-{nn}-0"
            redis.set(nn, _j.dumps([uuid]))
            cm = f"cm-{nn}"
            fc.create("configmaps", O.make_config_map(cm, {"CUDA_VISIBLE_DEVICES": uuid}))
            fc.create("pods", O.make_pod("mlperf-gpu-onnx-resnet50-1024", ns=nn, slo=200, config_maps=[cm],
                                         node_name=nn, phase="Running"))
        cfg = load_config(PARITY_PROFILE)
        preds = RpcPredictions(RecommenderClient(f"127.0.0.1:{port}", new_channel_per_call=True))
        s = Scheduler(fc, cfg, full_registry(), bind_async=False, record_events=False,
                      extras={"redis": redis, "predictions": preds})
        s.start_informers()
        pods = []
        for i in range(n):
            fc.create("configmaps", O.make_config_map(f"cm-in-{i}"))
            pods.append(O.make_pod(f"mlperf-gpu-onnx-mobilenet-1024-{i}", slo=300, config_maps=[f"cm-in-{i}"]))
        out = run(fc, s, pods)
        out["rpcs"] = preds.calls
        return out
    finally:
        srv.stop(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=400)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-fast-path", action="store_true")
    a = ap.parse_args()
    global FAST
    FAST = not a.no_fast_path
    res = {"busybox_2nodes": busybox(a.pods), "fractional_4x8gpu": fractional(a.pods),
           "fractional_1000x8gpu_adaptive_sampling": fractional(a.pods, nodes=1000),
           "reference_algorithm_parity_rpc": parity_rpc(min(a.pods, 40)),
           "fast_path": FAST}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
