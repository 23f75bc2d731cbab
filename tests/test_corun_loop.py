"""The deployed co-run learning loop: profiled pods that overlapped on one GPU -> the node
agent's co-run observer -> the recommender's ObserveCorun (online refit) -> a new served
ExportTable("corun") version -> the scheduler's GPU plugin scoring on it.

Reference analog superseded: the recommender retrains only when its training files change
(reference pkg/recommender/recom_server.py:74-134); nothing in a cluster produces data."""
import os
import shutil

import numpy as np

from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
from k8s_gpu_scheduler_amd.agent.corun_observer import CorunObserver
from k8s_gpu_scheduler_amd.agent.devices import synthetic_node
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.models.corun import DATA, CorunModel
from k8s_gpu_scheduler_amd.recommender.client import CachedPredictions, RecommenderClient
from k8s_gpu_scheduler_amd.recommender.service import RecommenderService
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
from k8s_gpu_scheduler_amd.store.resp import Redis

UUID = "GPU-aaaaaaaa-0000-0000-0000-000000000001"


def _trace_dir(root, pod, tag, t0_ns, t1_ns, n_kernels=8):
    d = os.path.join(root, O.namespace(pod), O.name(pod), O.uid(pod), "main", tag)
    os.makedirs(d)
    with open(os.path.join(d, "run_kernel_stats.csv"), "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n"k",8,1000,125,100.0\n')
    step = (t1_ns - t0_ns) // n_kernels
    with open(os.path.join(d, "run_kernel_trace.csv"), "w") as f:
        f.write('"Kernel_Name","Start_Timestamp","End_Timestamp"\n')
        for i in range(n_kernels):
            a = t0_ns + i * step
            f.write(f'"k",{a},{t1_ns if i == n_kernels - 1 else a + step - 1000}\n')
    return d


def _pod(fc, name, uuid=UUID, phase="Succeeded"):
    p = O.make_pod(name, gpu_cu=64, gpu_mem_gib=4, env={C.ENV_ITERATIONS: "20"}, node_name="n1", phase=phase)
    p["metadata"].setdefault("annotations", {})[C.ANNOT_DEVICES] = uuid
    fc.create("pods", p)
    return fc.get("pods", name, "default")


def test_observer_groups_overlapping_pods_and_waits_for_running_corunners():
    sent = []
    running = {"default/b"}
    ob = CorunObserver(sent.append, running_on=lambda u: set(running) if u == UUID else set(), settle_s=0.0)
    a = {"metadata": {"name": "a", "namespace": "default", "annotations": {C.ANNOT_DEVICES: UUID}}}
    b = {"metadata": {"name": "b", "namespace": "default", "annotations": {C.ANNOT_DEVICES: UUID}}}
    c = {"metadata": {"name": "c", "namespace": "default", "annotations": {C.ANNOT_DEVICES: "GPU-other"}}}
    assert ob.add(a, "onnx_resnet50_1024", 20, 0, 10_000_000)
    assert ob.add(c, "onnx_mobilenet_1024", 20, 0, 10_000_000)        # another GPU: its own group
    assert ob.step() == 1 and ob.pending() == 1          # a waits: b ran next to it and is still running
    running.clear()
    assert ob.add(b, "onnx_mobilenet_2048", 20, 4_000_000, 16_000_000)
    assert ob.step() == 2
    groups = [g for batch in sent for g in batch]
    ga = next(g for g in groups if "onnx_resnet50_1024" in g["workloads"]
              and g["target"][g["workloads"].index("onnx_resnet50_1024")])
    assert sorted(ga["workloads"]) == ["onnx_mobilenet_2048", "onnx_resnet50_1024"]
    i = ga["workloads"].index("onnx_mobilenet_2048")
    assert ga["start_ms"][i] == 4.0 and ga["ms"][i] == 12.0 and ga["target"] == [x == "onnx_resnet50_1024"
                                                                                for x in ga["workloads"]]


def test_observer_drops_a_target_whose_corunner_left_no_trace():
    running = {"default/unprofiled"}
    ob = CorunObserver(lambda g: None, running_on=lambda u: set(running), settle_s=0.0)
    a = {"metadata": {"name": "a", "namespace": "default", "annotations": {C.ANNOT_DEVICES: UUID}}}
    ob.add(a, "onnx_resnet50_1024", 20, 0, 10_000_000)
    running.clear()                                       # finished, never traced
    assert ob.step() == 0 and ob.dropped == 1


def test_profiled_pods_on_one_gpu_refine_the_served_model_and_the_scheduler_scores_on_it(tmp_path):
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=1))
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    cm = tmp_path / "corun.json"
    shutil.copy(DATA, cm)
    svc = RecommenderService("", "", corun_path=str(cm))
    svc._corun_refit_mode = False                       # refit synchronously in the test
    svc.corun_online_kw = {"min_obs": 8, "min_calib": 8, "refit_every": 8}
    svc.train()
    srv, port = svc.make_server(0, 2, "127.0.0.1")
    try:
        cl = RecommenderClient(f"127.0.0.1:{port}", timeout_s=30.0)   # synchronous refits in the RPC
        v0 = cl.version().corun
        base = CorunModel.load(str(cm))
        slow = CorunModel(base.names, base.alone_ms * 1.3, base.u, base.v)      # this node runs 30 % slower
        root = str(tmp_path / "prof")
        ag = NodeAgent("n1", r, synthetic_node(1, node="n1"), client=fc, profile_dir=root,
                       corun_send=cl.observe_corun)
        ag.corun.settle_s = 0.0
        pairs = [("onnx_resnet50_1024", "onnx_mobilenet_2048"), ("tensorflow_resnet50_1024", "onnx_ssd_mobilenet_1024"),
                 ("onnx_mobilenet_1024", "tensorflow_mobilenet_2048")] * 4
        t = 1_000_000_000
        for k, (wa, wb) in enumerate(pairs):
            ia, ib = base.wid(wa), base.wid(wb)
            fin = slow.group_times([ia, ib], [20, 20], [0.0, 1.0])          # b starts 1 ms after a
            pa = _pod(fc, f"{wa.replace('_', '-')}-{k}")
            pb = _pod(fc, f"{wb.replace('_', '-')}-{k}")
            _trace_dir(root, pa, "cu64-hbm4-it20", t, t + int(fin[0] * 1e6))
            _trace_dir(root, pb, "cu64-hbm4-it20", t + 1_000_000, t + int(fin[1] * 1e6))
            t += int(max(fin) * 1e6) + 5_000_000                             # groups do not overlap
        ag.step()
        assert ag.corun.sent == 2 * len(pairs) and ag.corun.dropped == 0
        v1 = cl.version().corun
        assert v1 != v0 and "+online-" in v1
        cache = CachedPredictions(cl, background=False)
        cache.refresh(force=True)
        m = cache.corun()
        assert m.version == v1
        assert float(np.median(m.alone_ms / base.alone_ms)) > 1.15        # learned: the node is slower
        # the scheduler's GPU plugin scores with the served refined model
        from k8s_gpu_scheduler_amd.plugins.gpu.plugin import GPUPlugin
        plugin = GPUPlugin({"sloObjective": "corun"}, predictions=cache)
        assert plugin.corun_model().version == v1
    finally:
        svc.stop()
        srv.stop(0)


def test_cold_start_leave_one_workload_out_on_measured_groups():
    """models.coldstart: each catalog workload in turn is dropped from the shipped model and
    re-imputed from its alone profile (alone ms per iteration, MFMA share) and the other 17
    rows; on its measured MI355X co-run groups (profiles/archive/r03_corun_v2) the imputed row's
    throughput error stays within 2x the fitted model's held-out error, and
    far below the roofline prior row's."""
    import json
    from k8s_gpu_scheduler_amd.models.coldstart import impute_row, mfma_share
    from k8s_gpu_scheduler_amd.models.corun import pack_groups
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = json.load(open(os.path.join(root, "profiles", "archive", "r03_corun_v2", "groups_2558_hostwait.json")))
    groups = [g for g in d["groups"] if len(g["w"]) >= 2]
    m = CorunModel.load()
    held_out = m.meta["report"]["test"]["mae_pct_of_mean"]
    prior = CorunModel.prior(m.names)

    def err(model, i):
        gs = [g for g in groups if m.names[i] in g["w"]]
        wids, iters, mask, ms, st = pack_groups(gs, m.names, 4)
        t = model.batch_times(wids, iters, mask, st) - st
        sel = mask & (wids == i)
        tp, tm = iters / np.maximum(t, 1e-9) * 1e3, iters / np.maximum(ms, 1e-9) * 1e3
        return 100 * np.abs(tp - tm)[sel].mean() / tm[sel].mean()
    imp, pri = [], []
    for i, n in enumerate(m.names):
        u, v, nn = impute_row(m, float(m.alone_ms[i]), mfma_share(n), exclude=[i])
        assert n not in nn
        U, V = m.u.copy(), m.v.copy()
        U[i], V[i] = u, v
        imp.append(err(CorunModel(m.names, m.alone_ms, U, V), i))
        U[i], V[i] = prior.u[i], prior.v[i]
        pri.append(err(CorunModel(m.names, m.alone_ms, U, V), i))
    assert np.mean(imp) <= 2 * held_out, (np.mean(imp), held_out)
    assert np.median(imp) <= 2 * held_out and np.mean(imp) < 0.5 * np.mean(pri), (imp, pri)


def test_unseen_workload_cold_starts_through_observe_corun_and_plans(tmp_path):
    """An unseen workload profiled alone on its GPU (a 1-pod co-run observation from the node
    agent) gets a served co-run row: `wid` is no longer -1 and the GPU plugin's model has it;
    its later co-run groups are then accepted as observations."""
    cm = tmp_path / "corun.json"
    shutil.copy(DATA, cm)
    svc = RecommenderService("", "", corun_path=str(cm))
    svc._corun_refit_mode = False
    svc.train()
    srv, port = svc.make_server(0, 2, "127.0.0.1")
    try:
        cl = RecommenderClient(f"127.0.0.1:{port}", timeout_s=30.0)   # synchronous refits in the RPC
        base = CorunModel.load(str(cm))
        assert base.wid("llama-prefill-7b-xyz") == -1
        rep = cl.observe_corun([{"workloads": ["llama_prefill_7b"], "iters": [20], "ms": [3.0],
                                 "start_ms": [0.0], "target": [True], "mfma_share": [0.9]}])
        assert rep.accepted == 1 and "+cold-1" in rep.corun
        cache = CachedPredictions(cl, background=False)
        cache.refresh(force=True)
        m = cache.corun()
        i = m.wid("llama-prefill-7b-xyz")
        assert i >= 0 and abs(m.alone_ms[i] - 0.15) < 1e-6
        # a GEMM-heavy newcomer is imputed from the GEMM-heavy catalog rows
        assert np.allclose(m.u[i], np.exp(np.mean(np.log(m.u[[m.wid(n) for n in svc._corun_online.base.meta[
            "cold_start"]["llama_prefill_7b"]["neighbours"]]]), axis=0)), rtol=0.5)
        rep = cl.observe_corun([{"workloads": ["llama_prefill_7b", "onnx_mobilenet_1024"], "iters": [20, 20],
                                 "ms": [4.0, 2.5], "start_ms": [0.0, 0.0], "target": [True, True]}])
        assert rep.accepted == 1
        from k8s_gpu_scheduler_amd.plugins.gpu.plugin import GPUPlugin
        plugin = GPUPlugin({"sloObjective": "corun"}, predictions=cache)
        assert plugin.corun_model().wid("llama-prefill-7b-abc") >= 0
    finally:
        svc.stop()
        srv.stop(0)


def test_cold_start_rows_keep_their_state_when_a_later_name_sorts_first(tmp_path):
    """rebuilding the learner with cold rows in sorted order shifted an earlier cold
    row's refit parameter and stored observations onto another workload when a later
    newcomer's name sorted before it.  Rows now append in arrival order and state moves by name."""
    cm = tmp_path / "corun.json"
    shutil.copy(DATA, cm)
    svc = RecommenderService("", "", corun_path=str(cm))
    svc._corun_refit_mode = False
    svc.train()
    srv, port = svc.make_server(0, 2, "127.0.0.1")
    try:
        cl = RecommenderClient(f"127.0.0.1:{port}", timeout_s=30.0)
        cl.observe_corun([{"workloads": ["zz_newcomer_b"], "iters": [20], "ms": [3.0], "start_ms": [0.0],
                           "target": [True], "mfma_share": [0.9]}])
        cl.observe_corun([{"workloads": ["zz_newcomer_b", "onnx_mobilenet_1024"], "iters": [20, 20],
                           "ms": [4.0, 2.5], "start_ms": [0.0, 0.0], "target": [True, True]}])
        on = svc._corun_online
        ib = on.base.wid("zz_newcomer_b")
        on._x[ib] = 0.25                                   # a refit parameter of the cold row
        cl.observe_corun([{"workloads": ["aa_newcomer_a"], "iters": [20], "ms": [1.0], "start_ms": [0.0],
                           "target": [True], "mfma_share": [0.1]}])
        on2 = svc._corun_online
        ib2, ia2 = on2.base.wid("zz_newcomer_b"), on2.base.wid("aa_newcomer_a")
        assert ia2 > ib2 >= 0                              # arrival order
        assert on2._x[ib2] == 0.25 and on2._x[ia2] == 0.0
        names = [[on2.base.names[w] for w in o[0]] for o in on2._obs]
        assert ["zz_newcomer_b", "onnx_mobilenet_1024"] in names
    finally:
        svc.stop()
        srv.stop(0)


def test_observer_drops_a_target_whose_finished_corunner_left_no_trace():
    """an unprofiled pod that overlapped the target on its device and had ALREADY
    finished when the target's trace was ingested was neither waited for nor detected.  Its
    container span (startedAt .. finishedAt) overlapping the target's now drops the target; a
    traced one or one that ran at another time does not."""
    def term(name, t0, t1):
        return {"metadata": {"name": name, "namespace": "default", "annotations": {C.ANNOT_DEVICES: UUID}},
                "status": {"phase": "Succeeded", "containerStatuses": [{"state": {"terminated": {
                    "startedAt": f"2026-01-01T00:00:{t0:02d}Z", "finishedAt": f"2026-01-01T00:00:{t1:02d}Z"}}}]}}
    pods = {"default/ghost": term("ghost", 1, 4), "default/late": term("late", 30, 40),
            "default/b": term("b", 2, 6)}

    def finished_on(uuid, span):
        from k8s_gpu_scheduler_amd.plugins.gpu.feedback import container_span
        return {k for k, p in pods.items() if (s := container_span(p)) and s[1] > span[0] and s[0] < span[1]}
    ob = CorunObserver(lambda g: None, running_on=lambda u: set(), settle_s=0.0, finished_on=finished_on)
    ob.add(term("a", 0, 5), "onnx_resnet50_1024", 20, 0, 10_000_000)     # ghost (untraced) overlapped
    assert ob.step() == 0 and ob.dropped == 1
    del pods["default/ghost"]
    sent = []
    ob2 = CorunObserver(sent.append, running_on=lambda u: set(), settle_s=0.0, finished_on=finished_on)
    ob2.add(term("b", 2, 6), "onnx_mobilenet_1024", 20, 2_000_000, 6_000_000)
    ob2.add(term("a", 0, 5), "onnx_resnet50_1024", 20, 0, 10_000_000)    # b overlapped and is traced
    assert ob2.step() == 2 and ob2.dropped == 0


def test_cold_start_transfers_to_other_kernel_mixes_with_cu_fill():
    """two workloads outside the catalog's kernel mix (models.workloads.EXTRA:
    fp8-GEMM LLM-like, triad-only), measured in co-run groups with catalog pods on MI355X
    (profiles/r05_coldstart/groups.json, tools/corun_extra_groups.py), cold-started from their
    alone groups only.  With the CU-fill scaling (betas fitted on the catalog rows alone) both
    stay within 2x the fitted model's held-out MAE; without it the chip-filling fp8 workload is
    ~3x off -- the catalog has no GEMM row that fills the chip at a pod's tile budget."""
    import json
    from k8s_gpu_scheduler_amd.models.coldstart import cu_fill, fill_betas, mfma_share, with_workload
    from k8s_gpu_scheduler_amd.models.corun import pack_groups
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = json.load(open(os.path.join(root, "profiles", "r05_coldstart", "groups.json")))
    groups = d["groups"]
    base = CorunModel.load()
    held_out = base.meta["report"]["test"]["mae_pct_of_mean"]
    bs, bp = fill_betas(base)
    assert 0.0 < bs < bp < 1.5                       # pressure scales with footprint more than sensitivity

    def alone(n):
        return float(np.median([g["ms"][0] / g["iters"] for g in groups if g["w"] == [n]]))

    def err(use_fill):
        m = base
        for x in d["extra"]:
            m = with_workload(m, x, alone(x), mfma_share(x), fill=cu_fill(x) if use_fill else None)
        out = {}
        for x in d["extra"]:
            gs = [g for g in groups if x in g["w"] and len(g["w"]) >= 2]
            wids, iters, mask, ms, st = pack_groups(gs, m.names, 4)
            t = m.batch_times(wids, iters, mask, st) - st
            sel = mask & (wids == m.index[x])
            tp, tm = iters / np.maximum(t, 1e-9) * 1e3, iters / np.maximum(ms, 1e-9) * 1e3
            out[x] = 100 * np.abs(tp - tm)[sel].mean() / tm[sel].mean()
        return out
    with_fill, without = err(True), err(False)
    assert all(v <= 2 * held_out for v in with_fill.values()), (with_fill, held_out)
    assert without["fp8_llm_2048"] > 2 * held_out > with_fill["fp8_llm_2048"], (without, with_fill)
    assert cu_fill("fp8_llm_2048") == 1.0 and cu_fill("onnx_resnet50_2048") == 0.25


def test_kernel_trace_cu_fill_reaches_the_cold_row(tmp_path):
    """The pod profiler's kernel trace gives a pod's CU fill (time-weighted workgroups / CUs);
    the co-run observer sends it with the alone group and the recommender's cold row uses it."""
    from k8s_gpu_scheduler_amd.agent.pod_profiler import summarize_kernel_trace
    tr = tmp_path / "kernel_trace.csv"
    tr.write_text("Kernel_Name,Start_Timestamp,End_Timestamp,Workgroup_Size_X,Workgroup_Size_Y,Workgroup_Size_Z,"
                  "Grid_Size_X,Grid_Size_Y,Grid_Size_Z\n"
                  "gemm_fp8,0,300,256,1,1,131072,1,1\n"            # 512 workgroups: fills 256 CUs
                  "small,300,400,256,1,1,16384,1,1\n")             # 64 workgroups: a quarter
    s = summarize_kernel_trace(str(tr))
    assert abs(s["cu_fill"] - (300 * 1.0 + 100 * 0.25) / 400) < 1e-4
    cm = tmp_path / "corun.json"
    shutil.copy(DATA, cm)
    svc = RecommenderService("", "", corun_path=str(cm))
    svc._corun_refit_mode = False
    svc.train()
    srv, port = svc.make_server(0, 2, "127.0.0.1")
    try:
        cl = RecommenderClient(f"127.0.0.1:{port}", timeout_s=30.0)
        rep = cl.observe_corun([{"workloads": ["llm_fp8_serving"], "iters": [20], "ms": [2.2], "start_ms": [0.0],
                                 "target": [True], "mfma_share": [1.0], "cu_fill": [1.0]}])
        assert rep.accepted == 1
        on = svc._corun_online
        assert on.base.meta["cold_start"]["llm_fp8_serving"]["cu_fill"] == 1.0
        i = on.base.wid("llm_fp8_serving")
        nn = [on.base.wid(n) for n in on.base.meta["cold_start"]["llm_fp8_serving"]["neighbours"]]
        # a chip-filling newcomer presses harder than the (partly idle) GEMM rows it was imputed from
        assert (on.base.u @ on.base.v[i]).mean() > max((on.base.u @ on.base.v[j]).mean() for j in nn)
    finally:
        svc.stop()
        srv.stop(0)
