"""Recommender: proto wire format, imputers, gRPC server parity, hot reload, resize.

Parity vectors from SURVEY.md §2.7.4: unknown pod -> result=[0], columns=[];
`…resnet50-1024_A30` interference imputes the NaN diagonal -> 44.37.
"""
import os
import shutil
import time

import numpy as np
import pytest

from k8s_gpu_scheduler_amd.models.imputers import make_imputer
from k8s_gpu_scheduler_amd.recommender import proto as P
from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions, RecommenderClient, RpcPredictions, reply_to_map
from k8s_gpu_scheduler_amd.recommender.resize import recommend
from k8s_gpu_scheduler_amd.recommender.service import RecommenderService
from k8s_gpu_scheduler_amd.recommender.tables import Table, file_version, find_index_for_request


def test_proto_wire_compat():
    # field numbers/types of recom.proto: Request.index=1 (string), Reply.result=1 (packed float),
    # Reply.columns=2 (string)
    assert P.Request(index="ab").SerializeToString() == b"\n\x02ab"
    r = P.set_protobuf_reply([1.0], ["c"], P.Reply())
    assert r.SerializeToString() == b"\n\x04\x00\x00\x80?\x12\x01c"
    assert set(P.POOL.FindServiceByName("recommender.recommender").methods_by_name.keys()) >= \
        {"ImputeConfigurations", "ImputeInterference"}


def test_find_index():
    idx = ["onnx_mobilenet_1024", "onnx_resnet50_1024"]
    assert find_index_for_request("mlperf_gpu_onnx_resnet50_1024_A30", idx) == "onnx_resnet50_1024"
    assert find_index_for_request("busybox_abc", idx) == ""


@pytest.mark.parametrize("kind", ["iterative", "svd", "als"])
def test_imputers_recover_low_rank(kind):
    rng = np.random.default_rng(0)
    U, V = rng.normal(size=(30, 2)), rng.normal(size=(2, 8))
    X = U @ V + 10
    M = X.copy()
    hide = rng.random(X.shape) < 0.15
    M[hide] = np.nan
    m = make_imputer(kind, **({} if kind == "iterative" else {"k": 2})).fit(M)
    out = m.predict(M)
    assert np.allclose(out[~hide], X[~hide])                      # observed entries kept
    err = np.abs(out[hide] - X[hide]).mean()
    assert err < (0.6 if kind != "iterative" else 1.0), err


@pytest.fixture()
def server(ref_data, tmp_path):
    conf, intf = ref_data
    c, i = tmp_path / "c.tsv", tmp_path / "i.tsv"
    shutil.copy(conf, c)
    shutil.copy(intf, i)
    svc = RecommenderService(str(c), str(i), job_delay_s=0.2)
    svc.train()
    srv, port = svc.make_server(0, 4, "127.0.0.1")
    yield svc, f"127.0.0.1:{port}", (c, i)
    svc.stop()
    srv.stop(0)


def test_server_parity_vectors(server):
    svc, addr, _ = server
    cl = RecommenderClient(addr)
    r = cl.impute_configurations("busybox-abc")
    assert list(r.result) == [0.0] and list(r.columns) == []
    m = reply_to_map(cl.impute_interference("mlperf-gpu-onnx-resnet50-1024_A30"))
    assert m["onnx_resnet50_1024"] == pytest.approx(44.37, abs=0.01)
    conf = reply_to_map(cl.impute_configurations("mlperf-gpu-onnx-mobilenet-1024"))
    assert conf["1P_A30"] == pytest.approx(624.9) and conf["4P_V100"] == pytest.approx(474.595)
    # per-call channel (reference client_call.go:13) gives identical answers
    cl2 = RecommenderClient(addr, new_channel_per_call=True)
    assert reply_to_map(cl2.impute_configurations("mlperf-gpu-onnx-mobilenet-1024")) == conf
    cl.close()


def test_cached_predictions_match_rpc(server):
    svc, addr, _ = server
    cl = RecommenderClient(addr)
    rpc, cache = RpcPredictions(cl), CachedPredictions(cl)
    for name in ["mlperf-gpu-onnx-resnet50-2048", "tf-tensorflow-ssd-mobilenet-4096-x"]:
        a, b = rpc.configurations(name), cache.configurations(name)
        assert a.keys() == b.keys() and all(abs(a[k] - b[k]) < 1e-3 for k in a)
    a = rpc.interference("mlperf-gpu-onnx-resnet50-1024_A30")
    b = cache.interference("mlperf-gpu-onnx-resnet50-1024_A30")
    assert all(abs(a[k] - b[k]) < 1e-3 for k in a)
    assert cache.configurations("busybox") == {}


def test_hot_reload_on_md5_change(server):
    svc, addr, (c, _) = server
    cl = RecommenderClient(addr)
    v0 = cl.version().configurations
    t = Table.read_tsv(str(c))
    t.set("new_workload_1", "1P_A30", 123.0)
    t.write_tsv(str(c))
    svc.start_retrain_loop()
    deadline = time.time() + 10
    while cl.version().configurations == v0 and time.time() < deadline:
        time.sleep(0.1)
    assert cl.version().configurations == file_version(str(c)) != v0
    assert reply_to_map(cl.impute_configurations("new-workload-1"))["1P_A30"] == pytest.approx(123.0)
    # a missing file does not kill the retrain loop (reference quirk §2.9 #12)
    os.remove(str(c))
    time.sleep(0.5)
    assert svc._thread.is_alive()


def test_resize_policy():
    hist = [{"hbm_gib": 10 + i % 3, "cu": 64, "throughput": 100.0} for i in range(20)]
    a = recommend(hist, 64, 32, slo=90)
    assert a.hbm_gib == 14 and a.cu == 64                    # p95=12 GiB * 1.15 -> ceil 14
    a = recommend(hist, 64, 32, slo=40)
    assert a.cu == 32                                         # extrapolated 100*(0.5^0.85) >= 42
    a = recommend(hist, 64, 32, slo=500)
    assert a.cu == 256
    a = recommend(hist[:2], 64, 32, slo=90)
    assert a.reason == "insufficient history" and a.cu == 64
    a = recommend(hist, 64, 32, slo=50, conf_predictions={"8P_MI355X": 60.0})
    assert a.cu == 32
    busy = [{"hbm_gib": 4, "cu_busy": 0.3} for _ in range(10)]
    assert recommend(busy, 128, 8).cu == 64


def test_resize_rpc(server):
    svc, addr, _ = server
    svc.history_source = lambda pod: [{"hbm_gib": 20.0, "cu": 128, "throughput": 300.0}] * 5
    cl = RecommenderClient(addr)
    r = cl.recommend_resources("mlperf-gpu-onnx-resnet50-1024", 128, 64.0, 150.0)
    assert r.samples == 5 and r.recommended_hbm_gib == 23.0 and r.recommended_cu == 64


def test_resize_admission_loop_on_fake_cluster():
    """Config 5 loop: measured history per workload -> admission rewrites a NEW pod's GPU
    request (QoS class kept), the scheduler packs the smaller pods; the webhook form emits
    the same change as an AdmissionReview JSONPatch."""
    import base64
    import json as _json
    from k8s_gpu_scheduler_amd.api import constants as C
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.kube.patch import apply_json_patch
    from k8s_gpu_scheduler_amd.plugins import full_registry
    from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger
    from k8s_gpu_scheduler_amd.recommender.admission import (RedisHistory, ResizeAdmission, webhook_handler,
                                                             workload_key)
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    hist = RedisHistory(Redis(FakeRedisBackend(FakeRedisEngine())))
    adm = ResizeAdmission(hist.read)
    fc = FakeCluster()
    fc.add_admission("pods", adm)
    fc.create("nodes", O.make_node("n", gpus=1))
    ledger = DeviceLedger()
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, extras={"ledger": ledger})
    s.start_informers()
    # no history yet: requests untouched, only 2 of 4 128-CU pods fit one GPU
    for i in range(4):
        fc.create("pods", O.make_pod(f"onnx-resnet50-1024-a{i}", gpu_cu=128, gpu_mem_gib=20, slo=100))
    assert sum(r.status.ok for r in s.schedule_pending()) == 2
    assert workload_key(fc.get("pods", "onnx-resnet50-1024-a0", "default")) == "onnx_resnet50_1024"
    # the executor / agent measured this workload: 64 CUs already give 150 q/s, 8 GiB used
    for _ in range(8):
        hist.append("onnx_resnet50_1024", {"cu": 64, "throughput": 150.0, "hbm_gib": 8.0})
    for i in range(4):
        fc.delete("pods", f"onnx-resnet50-1024-a{i}", "default")
    for i in range(4):
        fc.create("pods", O.make_pod(f"onnx-resnet50-1024-b{i}", gpu_cu=128, gpu_mem_gib=20, slo=100))
    p = fc.get("pods", "onnx-resnet50-1024-b0", "default")
    assert O.gpu_request(p) == (0, 64, 10.0)                       # 64 CUs, p95 8 GiB * 1.15 -> 10
    assert O.gpu_qos(p) == "Guaranteed"                             # limits rewritten with requests
    assert _json.loads(O.annotations(p)[C.ANNOT_RESIZED])["from"]["cu"] == 128
    assert sum(r.status.ok for r in s.schedule_pending()) == 4      # all four now fit
    # webhook front-end: same decision as a JSONPatch
    pod = O.make_pod("onnx-resnet50-1024-c", gpu_cu=128, gpu_mem_gib=20, slo=100, gpu_limits=False)
    out = webhook_handler(adm, {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                                "request": {"uid": "u1", "kind": {"kind": "Pod"}, "operation": "CREATE",
                                            "object": pod}})
    r = out["response"]
    assert r["uid"] == "u1" and r["allowed"] and r["patchType"] == "JSONPatch"
    patched = apply_json_patch(pod, _json.loads(base64.b64decode(r["patch"])))
    assert O.gpu_request(patched, cached=False)[1] == 64 and O.gpu_qos(patched) == "Burstable"


def test_resize_webhook_http_server():
    import json as _json
    import urllib.request
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.recommender.admission import AdmissionServer, ResizeAdmission
    hist = {"onnx_mobilenet_1024": [{"cu": 32, "throughput": 400.0, "hbm_gib": 2.0}] * 5}
    srv = AdmissionServer(ResizeAdmission(lambda k: hist.get(k, [])), "127.0.0.1", 0).start()
    try:
        pod = O.make_pod("mlperf-gpu-onnx-mobilenet-1024", gpu_cu=128, gpu_mem_gib=16, slo=300)
        body = _json.dumps({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                            "request": {"uid": "x", "kind": {"kind": "Pod"}, "operation": "CREATE",
                                        "object": pod}}).encode()
        req = urllib.request.Request(srv.url + "/mutate", data=body, headers={"Content-Type": "application/json"})
        out = _json.loads(urllib.request.urlopen(req, timeout=5).read())
        assert out["response"]["allowed"] and out["response"]["patchType"] == "JSONPatch"
        assert urllib.request.urlopen(srv.url + "/healthz", timeout=5).read() == b"ok"
    finally:
        srv.stop()


def test_model_versions_persist_in_redis(tmp_path, ref_data):
    """A trained version is persisted to Redis; a restarted recommender whose training file
    is gone serves the persisted version."""
    import shutil
    from k8s_gpu_scheduler_amd.recommender.service import RecommenderService
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    conf_p, intf_p = ref_data
    c, i = tmp_path / "c.tsv", tmp_path / "i.tsv"
    shutil.copy(conf_p, c)
    shutil.copy(intf_p, i)
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    a = RecommenderService(str(c), str(i))
    a.store = r
    a.train()
    want = a.conf.get().lookup("mlperf-gpu-onnx-mobilenet-1024")
    c.unlink()
    i.unlink()
    b = RecommenderService(str(c), str(i))
    b.store = r
    b.train()
    assert b.conf.version == a.conf.version and b.intf.version == a.intf.version
    assert b.conf.get().lookup("mlperf-gpu-onnx-mobilenet-1024") == pytest.approx(want)


def test_cached_predictions_survive_late_recommender_and_follow_new_versions(ref_data, tmp_path):
    """The scheduler may start before the recommender: the cache comes up empty instead of
    failing, fills once the server answers, and a retrained version reaches it without a
    restart (the reference sees new versions because it calls per prediction)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cl = RecommenderClient(f"127.0.0.1:{port}", timeout_s=0.5)
    cache = CachedPredictions(cl, refresh_s=0.3, retry_s=0.1)
    assert cache.configurations("mlperf-gpu-onnx-mobilenet-1024") == {}
    conf, intf = ref_data
    c, i = tmp_path / "c.tsv", tmp_path / "i.tsv"
    shutil.copy(conf, c)
    shutil.copy(intf, i)
    svc = RecommenderService(str(c), str(i), job_delay_s=0.2)
    svc.train()
    srv, _ = svc.make_server(port, 2, "127.0.0.1")
    try:
        deadline = time.time() + 15
        while not cache.configurations("mlperf-gpu-onnx-mobilenet-1024") and time.time() < deadline:
            time.sleep(0.1)
        assert cache.configurations("mlperf-gpu-onnx-mobilenet-1024")["1P_A30"] == pytest.approx(624.9)
        t = Table.read_tsv(str(c))
        t.set("new_workload_1", "1P_A30", 77.0)
        t.write_tsv(str(c))
        svc.start_retrain_loop()
        deadline = time.time() + 15
        while not cache.configurations("new-workload-1") and time.time() < deadline:
            time.sleep(0.1)
        assert cache.configurations("new-workload-1")["1P_A30"] == pytest.approx(77.0)
    finally:
        cache.close()
        svc.stop()
        srv.stop(0)
        cl.close()


def test_online_interference_learns_additive_model():
    """recommender.online: ridge toward the prior, converging to the true additive matrix
    from co-run observations; prequential error of the online model beats the prior."""
    import numpy as np
    from k8s_gpu_scheduler_amd.recommender.online import OnlineInterference
    rng = np.random.default_rng(0)
    w = 6
    true = rng.uniform(0, 100, (w, w))
    prior = true + rng.normal(0, 40, (w, w))
    prior[0, 0] = np.nan                                  # unmeasured entry: filled, not fatal
    m = OnlineInterference([f"w{i}" for i in range(w)], [f"w{i}" for i in range(w)], prior, lam=2.0, refit_every=16,
                           scale=True)
    assert np.isfinite(m.matrix).all()
    # few observations: row stays near the prior
    m.observe(1, [2, 3, 4], float(true[1, [2, 3, 4]].sum()))
    m.refit()
    # column never seen -> the prior entry, scaled by the row's learned prior scale
    assert abs(m.matrix[1, 5] - m.prior[1, 5] * m.row_scale[1]) < 1e-9
    for _ in range(3000):
        a = int(rng.integers(w))
        others = [int(x) for x in rng.integers(0, w, 3)]
        m.observe(a, others, float(true[a, others].sum() + rng.normal(0, 2)))
    m.refit()
    assert np.abs(m.matrix - true).max() < 5.0
    e = m.mae()
    assert e["n"] == 3001 and e["online"] < 0.5 * e["prior"]
    plain = OnlineInterference([f"w{i}" for i in range(w)], [f"w{i}" for i in range(w)], prior, scale=False)
    plain.observe(1, [2, 3, 4], float(true[1, [2, 3, 4]].sum()))
    plain.refit()
    assert abs(plain.matrix[1, 5] - plain.prior[1, 5]) < 1e-9     # scale=False: prior kept


def test_online_interference_learns_a_systematic_prior_bias_fast():
    """A pairwise table that under-predicts 4-way co-run loss by a common factor: the prior
    scale (global, then per row) is learned from every row's observations, so 100 observations
    over 18 rows (~5 per row) already beat the plain ridge-to-prior by a wide margin."""
    import numpy as np
    from k8s_gpu_scheduler_amd.recommender.online import OnlineInterference
    rng = np.random.default_rng(0)
    w = 18
    prior = rng.uniform(50, 500, (w, w))
    true = prior * 1.6 + rng.normal(0, 20, (w, w))
    maes = {}
    for scale in (False, True):
        r = np.random.default_rng(1)
        m = OnlineInterference([str(i) for i in range(w)], [str(i) for i in range(w)], prior, scale=scale)
        for _ in range(100):
            a = int(r.integers(w))
            others = [int(x) for x in r.integers(0, w, 3)]
            m.observe(a, others, float(true[a, others].sum() + r.normal(0, 50)))
        maes[scale] = m.mae()["online"]
        if scale:
            assert 1.4 < m.global_scale < 1.8
    assert maes[True] < 0.6 * maes[False]


def test_plugin_forgets_memoised_predictions_on_new_table():
    from k8s_gpu_scheduler_amd.plugins.gpu.plugin import GPUPlugin
    from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions, _Tab
    cp = CachedPredictions()
    cp._conf = _Tab(["wl_a"], ["1P_MI355X"], [[10.0]], "v1")
    cp._intf = _Tab(["wl_a"], ["wl_a"], [[1.0]], "v1")
    p = GPUPlugin({}, None, predictions=cp)
    assert p._pod_predictions("wl-a-0")[1] == {"wl_a": 1.0}
    cp.install_interference(["wl_a"], ["wl_a"], [[5.0]], "online-1")
    assert p._pod_predictions("wl-a-0")[1] == {"wl_a": 5.0}


def test_observe_interference_rpc_serves_learned_table(server):
    """Extended.ObserveInterference: co-run observations refit the interference row and the
    learned table is served (version online-N) until the training file changes."""
    svc, addr, (c, i) = server
    cl = RecommenderClient(addr)
    before = reply_to_map(cl.impute_interference("mlperf-gpu-onnx-resnet50-1024_A30"))
    col = "onnx_mobilenet_1024"
    target = before[col] + 50.0
    obs = [("mlperf-gpu-onnx-resnet50-1024_A30", ["pod-onnx-mobilenet-1024-7"], target)] * 40
    rep = cl.observe_interference(obs + [("busybox-abc", ["x"], 1.0)])
    assert rep.accepted == 40 and rep.interference.startswith("online-") and rep.observations == 40
    assert cl.version().interference == rep.interference
    after = reply_to_map(cl.impute_interference("mlperf-gpu-onnx-resnet50-1024_A30"))
    assert abs(after[col] - target) < abs(before[col] - target) * 0.25     # moved to the observations
    assert after["onnx_resnet50_1024"] == pytest.approx(before["onnx_resnet50_1024"], rel=1e-6)  # unseen column
    # a new training file wins again (and restarts the learner from it)
    with open(i, "a") as f:
        f.write("\n")
    svc.train()
    assert not cl.version().interference.startswith("online-")


def test_online_table_survives_recommender_restart(ref_data, tmp_path):
    import shutil as _sh
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    from k8s_gpu_scheduler_amd.recommender import proto as P
    conf, intf = ref_data
    c, i = tmp_path / "c.tsv", tmp_path / "i.tsv"
    _sh.copy(conf, c)
    _sh.copy(intf, i)
    store = Redis(FakeRedisBackend(FakeRedisEngine()))
    a = RecommenderService(str(c), str(i))
    a.store = store
    a.train()
    req = P.ObserveRequest()
    for _ in range(40):
        req.observations.add(pod="mlperf-gpu-onnx-resnet50-1024_A30", co_runners=["x-onnx-mobilenet-1024"], loss=500.0)
    rep = a.ObserveInterference(req, None)
    assert rep.interference.startswith("online-")
    b = RecommenderService(str(c), str(i))        # restart with the same training file
    b.store = store
    b.train()
    assert b.intf.version == rep.interference
    learned = b.intf.get().lookup("mlperf-gpu-onnx-resnet50-1024_A30")["onnx_mobilenet_1024"]
    assert learned == pytest.approx(a.intf.get().lookup("mlperf-gpu-onnx-resnet50-1024_A30")["onnx_mobilenet_1024"])
    with open(i, "a") as f:                       # a new training file: the online table is stale
        f.write("\n")
    c2 = RecommenderService(str(c), str(i))
    c2.store = store
    c2.train()
    assert not c2.intf.version.startswith("online-")


def test_recommender_serves_the_corun_model_and_hot_reloads_it(ref_data, tmp_path):
    """ExportTable("corun") serves the multi-way co-run model (models.corun) the GPU plugin's
    co-run objective uses; a changed model file reaches a CachedPredictions without restarts."""
    import numpy as np
    from k8s_gpu_scheduler_amd.models.corun import DATA, CorunModel
    conf, intf = ref_data
    cm = tmp_path / "corun.json"
    shutil.copy(DATA, cm)
    svc = RecommenderService(str(conf), str(intf), job_delay_s=0.2, corun_path=str(cm))
    svc.train()
    srv, port = svc.make_server(0, 2, "127.0.0.1")
    try:
        cache = CachedPredictions(RecommenderClient(f"127.0.0.1:{port}"), background=False)
        cache.refresh(force=True)
        m, ref = cache.corun(), CorunModel.load(str(cm))
        assert m is not None and m.names == ref.names
        assert np.allclose(m.coupling(), ref.coupling(), rtol=1e-6) and np.allclose(m.alone_ms, ref.alone_ms)
        v0 = m.version
        ref2 = CorunModel(ref.names, ref.alone_ms * 1.1, ref.u, ref.v, dict(ref.meta, version="refit-x"))
        ref2.save(str(cm))
        svc.train()
        cache.refresh(force=True)
        assert cache.corun().version != v0 and np.allclose(cache.corun().alone_ms, ref.alone_ms * 1.1)
    finally:
        svc.stop()
        srv.stop(0)


def test_observe_corun_rpc_serves_a_refined_model(ref_data, tmp_path):
    """Extended.ObserveCorun: co-run groups measured on the cluster refine the co-run model
    (models.corun.OnlineCorun) and ExportTable("corun") serves the refined version."""
    import numpy as np
    from k8s_gpu_scheduler_amd.models.corun import DATA, CorunModel
    conf, intf = ref_data
    cm = tmp_path / "corun.json"
    shutil.copy(DATA, cm)
    svc = RecommenderService(str(conf), str(intf), corun_path=str(cm))
    svc._corun_refit_mode = False                      # refit synchronously in the test
    svc.train()
    srv, port = svc.make_server(0, 2, "127.0.0.1")
    try:
        cl = RecommenderClient(f"127.0.0.1:{port}", timeout_s=30.0)   # synchronous refits in the RPC
        base = CorunModel.load(str(cm))
        slow = CorunModel(base.names, base.alone_ms * 1.25, base.u, base.v)      # the cluster runs 25 % slower
        rng = np.random.default_rng(5)
        v0 = cl.version().corun
        for _ in range(6):
            groups = []
            for _ in range(60):
                ws = [int(x) for x in rng.integers(0, len(base.names), 4)]
                groups.append({"workloads": [base.names[w] for w in ws], "iters": [20] * 4,
                               "ms": list(slow.group_durations(ws, [20] * 4))})
            rep = cl.observe_corun(groups)
            assert rep.accepted == 60
        assert rep.corun != v0 and "+online-" in rep.corun and cl.version().corun == rep.corun
        cache = CachedPredictions(cl, background=False)
        cache.refresh(force=True)
        m = cache.corun()
        assert m.version == rep.corun
        assert np.allclose(m.alone_ms / base.alone_ms, 1.25, rtol=0.05)
    finally:
        svc.stop()
        srv.stop(0)
