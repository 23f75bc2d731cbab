"""Node agent (profiler) + REST client against the HTTP fake apiserver.

Agent parity: publishes `<node>` -> JSON UUID list only when it changes (reference
pkg/profiler/profile_gpu.sh:3-13), MIG/partition filtering, stdin protocol
(reference pkg/profiler/test.sh); new: device descriptors/topology keys, async partition
reconcile with taint/untaint, per-pod usage history.
"""
import json
import time

import pytest

from k8s_gpu_scheduler_amd.agent.agent import NodeAgent, pod_of_pid, publish_from_stdin
from k8s_gpu_scheduler_amd.agent.devices import StaticSource, parse_smi_list, synthetic_node
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster, NotFound
from k8s_gpu_scheduler_amd.kube.fake_apiserver import FakeApiServer
from k8s_gpu_scheduler_amd.kube.informer import SharedInformerFactory
from k8s_gpu_scheduler_amd.kube.rest import RestClient, RestConfig
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.store import schema
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
from k8s_gpu_scheduler_amd.store.resp import Redis


def rds():
    return Redis(FakeRedisBackend(FakeRedisEngine()))


def test_parse_smi_listing():
    txt = ("GPU 0: NVIDIA A30 (UUID: GPU-ac0112df-7098-6c59-5c4f-a57fa666f808)\n"
           "  MIG 2g.12gb Device 0: (UUID: MIG-7a700938-2114-5d88-a93c-167c2a498910)\n")
    assert parse_smi_list(txt) == ["GPU-ac0112df-7098-6c59-5c4f-a57fa666f808",
                                   "MIG-7a700938-2114-5d88-a93c-167c2a498910"]


def test_stdin_protocol_reference_fixture():
    r = rds()
    lines = ["1", "2", "3", "['GPU-ac0112df-7098-6c59-5c4f-a57fa666f808', 'MIG-7a700938-2114-5d88-a93c-167c2a498910',"
                            " 'MIG-c8956631-ac65-59d3-9065-c8764799febf']"]
    publish_from_stdin(lines, r)
    assert json.loads(r.get("1")) == ["MIG-7a700938-2114-5d88-a93c-167c2a498910",
                                      "MIG-c8956631-ac65-59d3-9065-c8764799febf"]


def test_agent_publishes_on_change_only():
    r = rds()
    src = synthetic_node(8, node="n1")
    ag = NodeAgent("n1", r, src)
    assert ag.publish() and not ag.publish()
    assert len(schema.read_uuids(r, "n1")) == 8
    assert len(schema.read_devices(r, "n1")) == 8
    assert json.loads(r.get(schema.topology_key("n1")))["n"] == 8
    src.desc = src.desc[:7]                        # a GPU disappeared (reset / UUID change)
    assert ag.publish() and len(schema.read_uuids(r, "n1")) == 7


def test_agent_partition_reconcile_end_to_end():
    """Label asks for CPX -> agent taints, applies, republishes 64 partition UUIDs,
    untaints; the scheduler then sees 64 devices of 32 CUs."""
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=8))
    r = rds()
    src = synthetic_node(8, node="n1")
    ag = NodeAgent("n1", r, src, client=fc)
    ag.publish()
    fc.patch("nodes", "n1", {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: "CPX"}}}, "merge")
    assert ag.reconcile_partitions()
    assert len(src.partition_calls) == 8 and ag.current_partition() == "CPX"
    assert len(schema.read_uuids(r, "n1")) == 64
    assert not O.node_taints(fc.get("nodes", "n1"))
    assert json.loads(r.get(schema.partition_key("n1")))["state"] == "applied"
    assert not ag.reconcile_partitions()           # idempotent
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, extras={"redis": r})
    s.start_informers()
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    devs = plugin.ledger.devices("n1")
    assert len(devs) == 64 and all(d.device.cus == 32 for d in devs)
    fc.create("pods", O.make_pod("p", gpus=1))
    (res,) = s.schedule_pending()
    assert res.status.ok


def test_tainted_node_is_filtered():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=8, taints=[{"key": C.TAINT_PARTITIONING, "value": "CPX",
                                                         "effect": "NoSchedule"}]))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False)
    s.start_informers()
    fc.create("pods", O.make_pod("p", gpu_cu=64))
    (res,) = s.schedule_pending()
    assert not res.status.ok


def test_history_and_cgroup_attribution(tmp_path):
    proc = tmp_path / "proc" / "4242"
    proc.mkdir(parents=True)
    (proc / "cgroup").write_text("0::/kubepods.slice/kubepods-burstable-pod1234abcd_5678_90ab_cdef_1234567890ab.slice/x\n")
    assert pod_of_pid(4242, str(tmp_path / "proc")) == "1234abcd-5678-90ab-cdef-1234567890ab"

    class Src(StaticSource):
        def processes(self, index):
            return [{"pid": 4242, "vram_bytes": 8 * 2**30, "cu_occupancy": 64}] if index == 0 else []
    r = rds()
    src = Src(synthetic_node(2).devices())
    ag = NodeAgent("n1", r, src, pod_resolver=lambda pid: pod_of_pid(pid, str(tmp_path / "proc")))
    n = ag.record_history({"1234abcd-5678-90ab-cdef-1234567890ab": "default/wl-pod"})
    assert n == 1
    h = schema.read_history(r, "default/wl-pod")
    assert h[0]["hbm_gib"] == 8 and h[0]["cu_busy"] == 0.25


@pytest.fixture()
def api():
    srv = FakeApiServer(token="t0k").start()
    yield srv
    srv.stop()


def test_rest_client_crud_patch_bind_watch(api, tmp_path):
    kc = api.kubeconfig(str(tmp_path / "kubeconfig"))
    cl = RestClient(RestConfig.from_kubeconfig(kc))
    cl.create("nodes", O.make_node("n1"))
    cl.create("pods", O.make_pod("p1"), "default")
    cl.create("configmaps", O.make_config_map("cm", {"a": "1"}), "default")
    items, rv = cl.list("pods", "default")
    assert [O.name(p) for p in items] == ["p1"] and rv
    cl.patch("pods", "p1", [{"op": "add", "path": "/metadata/labels/x", "value": "y"}], "json", "default")
    cl.patch("configmaps", "cm", {"data": {"b": "2"}}, "merge", "default")
    assert cl.get("configmaps", "cm", "default")["data"] == {"a": "1", "b": "2"}
    assert cl.list("pods", "default", label_selector="x=y")[0]
    cl.bind("default", "p1", "n1")
    assert O.node_name_of(cl.get("pods", "p1", "default")) == "n1"
    assert cl.list("pods", None, field_selector="spec.nodeName=n1")[0]
    with pytest.raises(NotFound):
        cl.get("pods", "nope", "default")
    evs = []
    for ev in cl.watch("configmaps", "default", rv, timeout_s=1):
        evs.append(ev["type"])
        if len(evs) >= 1:
            break
    assert evs == ["MODIFIED"]
    cl.delete("pods", "p1", "default", 0)
    with pytest.raises(Exception):
        RestClient(RestConfig(api.url, token="wrong")).list("pods", "default")


def test_scheduler_over_rest_with_threaded_informers(api, tmp_path):
    cl = RestClient(RestConfig(api.url, token="t0k"))
    api.cluster.create("nodes", O.make_node("n1", gpus=8))
    inf = SharedInformerFactory(cl)
    s = Scheduler(cl, default_gpu_config({}), full_registry(), bind_async=True, informers=inf)
    s.start()
    try:
        for i in range(6):
            cl.create("pods", O.make_pod(f"p{i}", gpu_cu=64), "default")
        deadline = time.time() + 20
        while time.time() < deadline and len(api.cluster.bindings) < 6:
            time.sleep(0.05)
        assert len(api.cluster.bindings) == 6
        ann = O.annotations(api.cluster.get("pods", "p0", "default"))
        assert ann[C.ANNOT_DEVICES].startswith("GPU-")
    finally:
        s.stop()


def _sched_with_agent(src, node="mi355x-0"):
    fc = FakeCluster()
    r = rds()
    NodeAgent(node, r, src).publish()
    fc.create("nodes", O.make_node(node, gpus=len(src.devices())))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, seed=0, extras={"redis": r})
    s.start_informers()
    return fc, s


def test_launcher_builds_kubelet_env_from_assignment():
    """Mini-kubelet: container env = env + envFrom ConfigMaps + the device allocation from the
    scheduler's annotations (ROCR_VISIBLE_DEVICES / HSA_CU_MASK), launched as a child."""
    import sys
    from k8s_gpu_scheduler_amd.agent.launcher import PodLauncher
    fc, s = _sched_with_agent(synthetic_node(8, node="mi355x-0"))
    fc.create("configmaps", O.make_config_map("cm-g", {"FROM_CM": "1"}))
    fc.create("pods", O.make_pod("guar", gpu_cu=64, gpu_mem_gib=8, slo=50, config_maps=["cm-g"]))
    fc.create("pods", O.make_pod("burst", gpu_cu=64, gpu_limits=False))
    fc.create("pods", O.make_pod("whole", gpus=1))
    assert all(r.status.ok for r in s.schedule_pending())
    keys = ["ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "HSA_CU_MASK", "SLO", "FROM_CM", "LOCAL_RANK"]
    cmd = [sys.executable, "-c", f"import os, json; print(json.dumps({{k: os.environ.get(k) for k in {keys!r}}}))"]
    la = PodLauncher(fc, "mi355x-0", command=cmd, base_env={"PATH": "/usr/bin:/bin", "LOCAL_RANK": "3"})
    res = {r.pod_key: r for r in la.run_bound()}
    assert set(res) == {"default/guar", "default/burst", "default/whole"}
    g, b, w = (res[f"default/{n}"].json() for n in ("guar", "burst", "whole"))
    ann = O.annotations(fc.get("pods", "guar", "default"))
    assert g["ROCR_VISIBLE_DEVICES"] == ann[C.ANNOT_DEVICES] and g["HIP_VISIBLE_DEVICES"] == "0"
    assert g["HSA_CU_MASK"].startswith("0:") and g["SLO"] == "50" and g["FROM_CM"] == "1"
    assert g["LOCAL_RANK"] is None                       # launcher-side rank env is scrubbed
    assert b["HSA_CU_MASK"] is None and b["ROCR_VISIBLE_DEVICES"]       # Burstable: no hard mask
    assert w["HSA_CU_MASK"] is None and w["ROCR_VISIBLE_DEVICES"].startswith("GPU-")
    assert O.phase(fc.get("pods", "whole", "default")) == "Succeeded"
    # kubelet-style container status: whole-second RFC 3339 times (what the completion feedback's
    # quantisation bound is about), the exit code, and no container left in the pid map
    term = fc.get("pods", "whole", "default")["status"]["containerStatuses"][0]["state"]["terminated"]
    assert term["exitCode"] == 0 and term["startedAt"].endswith("Z") and "." not in term["finishedAt"]
    assert la.running == {}


def test_profiled_launcher_records_history(tmp_path, monkeypatch):
    """The rocprof sidecar wraps the container command (program right after `--`) and turns
    the kernel statistics into a history sample for the pod's workload (CPU: a stand-in
    profiler script writes a kernel_stats.csv)."""
    import os
    import stat
    import sys
    from k8s_gpu_scheduler_amd.agent import pod_profiler
    from k8s_gpu_scheduler_amd.agent.pod_profiler import ProfiledLauncher
    from k8s_gpu_scheduler_amd.recommender.admission import RedisHistory
    fake = tmp_path / "rocprofv3"
    fake.write_text(
        "#!" + sys.executable + "\n"
        "import os, subprocess, sys\n"
        "a = sys.argv[1:]; d = a[a.index('-d') + 1]; cmd = a[a.index('--') + 1:]\n"
        "os.makedirs(d, exist_ok=True)\n"
        "open(os.path.join(d, 'run_kernel_stats.csv'), 'w').write(\n"
        "  'Name,Calls,TotalDurationNs,AverageNs,Percentage\\n'\n"
        "  'gemm_bf16_nt_kernel,40,2000000,50000,80\\nstream_triad,40,500000,12500,20\\n')\n"
        "sys.exit(subprocess.call(cmd))\n")
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setattr(pod_profiler, "ROCPROF", str(fake))
    fc, s = _sched_with_agent(synthetic_node(8, node="mi355x-0"))
    fc.create("pods", O.make_pod("onnx-resnet50-1024-x", gpu_cu=64, gpu_mem_gib=8))
    assert all(r.status.ok for r in s.schedule_pending())
    hist = RedisHistory(rds())
    la = ProfiledLauncher(fc, "mi355x-0", command=[sys.executable, "-c", "print('{}')"], history=hist)
    (res,) = la.run_bound()
    assert res.rc == 0
    (h,) = hist.read("onnx_resnet50_1024")
    assert h["gpu_busy_ms"] == 2.5 and h["kernels"] == 80 and h["cu"] == 64 and h["hbm_gib"] == 8
    assert h["top"][0]["name"].startswith("gemm_bf16")


def _bound_pod(fc, name, mem_gib, node="n1"):
    pod = O.make_pod(name, gpu_cu=64, gpu_mem_gib=mem_gib, node_name=node, phase="Running")
    fc.create("pods", pod)
    return fc.get("pods", name, "default")


def test_agent_flags_hbm_overuse_and_records_workload_history():
    """Scripted amd-smi process list: pod A's process holds 6 GiB against a 4 GiB share
    (flagged: node annotation, exporter gauge, event), pod B stays inside its share; both
    get a history sample under their WORKLOAD key (what the resize admission reads)."""
    from k8s_gpu_scheduler_amd.recommender.admission import RedisHistory, workload_key
    from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=2))
    a = _bound_pod(fc, "onnx-resnet50-1024-a", 4)
    b = _bound_pod(fc, "tensorflow-mobilenet-1024-b", 8)
    src = synthetic_node(2, node="n1")
    src.procs = {0: [{"pid": 101, "vram_bytes": 6 * 2**30, "cu_occupancy": 64}],
                 1: [{"pid": 202, "vram_bytes": 5 * 2**30, "cu_occupancy": 32}]}
    pids = {101: O.uid(a), 202: O.uid(b)}
    r = rds()
    exp = GpuExporter("n1")
    ag = NodeAgent("n1", r, src, client=fc, exporter=exp, pod_resolver=pids.get)
    ag.step()
    over = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_HBM_OVERUSE])
    assert list(over) == ["default/onnx-resnet50-1024-a"] and over["default/onnx-resnet50-1024-a"]["cap_gib"] == 4
    txt = exp.render().decode()
    assert 'amd_gpu_pod_hbm_overuse{node="n1",pod="default/onnx-resnet50-1024-a"} 1.0' in txt
    assert 'amd_gpu_pod_hbm_overuse{node="n1",pod="default/tensorflow-mobilenet-1024-b"} 0.0' in txt
    evs = [e for e in fc.list("events", "default")[0] if e.get("reason") == "GPUMemoryOveruse"]
    assert len(evs) == 1
    hist = RedisHistory(r)
    ha = hist.read(workload_key(a))
    assert ha and ha[-1]["hbm_gib"] == 6.0 and ha[-1]["cu"] == 64 and ha[-1]["source"] == "agent"
    assert hist.read(workload_key(b))[-1]["hbm_gib"] == 5.0
    ag.step()                                                    # same verdict: no second event
    assert len([e for e in fc.list("events", "default")[0] if e.get("reason") == "GPUMemoryOveruse"]) == 1
    src.procs[0][0]["vram_bytes"] = 3 * 2**30                    # back inside its share
    ag.step()
    assert json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_HBM_OVERUSE]) == {}


def test_agent_evicts_hbm_overuse_when_asked():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=1))
    a = _bound_pod(fc, "greedy", 2)
    src = synthetic_node(1, node="n1")
    src.procs = {0: [{"pid": 7, "vram_bytes": 40 * 2**30}]}
    ag = NodeAgent("n1", rds(), src, client=fc, pod_resolver={7: O.uid(a)}.get, evict_hbm_overuse=True)
    ag.step()
    assert ag.evicted == ["default/greedy"]
    with pytest.raises(NotFound):
        fc.get("pods", "greedy", "default")


def test_hbm_overuse_eviction_honours_pdb_and_retries():
    """Eviction goes through the Eviction API: a PodDisruptionBudget with no disruptions
    allowed refuses it (429); the pod is NOT marked handled, so the next step retries and
    succeeds once the budget allows one disruption."""
    from k8s_gpu_scheduler_amd.kube.client import TooManyRequests
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=1))
    pod = O.make_pod("greedy", gpu_cu=64, gpu_mem_gib=2, node_name="n1", phase="Running",
                     labels_={"app": "greedy"})
    fc.create("pods", pod)
    a = fc.get("pods", "greedy", "default")
    fc.create("poddisruptionbudgets", {"metadata": {"name": "greedy-pdb", "namespace": "default"},
                                       "spec": {"selector": {"matchLabels": {"app": "greedy"}}},
                                       "status": {"disruptionsAllowed": 0}})
    with pytest.raises(TooManyRequests):
        fc.evict("default", "greedy")
    src = synthetic_node(1, node="n1")
    src.procs = {0: [{"pid": 7, "vram_bytes": 40 * 2**30}]}
    ag = NodeAgent("n1", rds(), src, client=fc, pod_resolver={7: O.uid(a)}.get, evict_hbm_overuse=True)
    ag.step()
    assert ag.evicted == [] and fc.get("pods", "greedy", "default")
    assert "default/greedy" not in ag._overuse_flagged
    fc.patch("poddisruptionbudgets", "greedy-pdb", {"status": {"disruptionsAllowed": 1}}, "merge", "default")
    ag.step()
    assert ag.evicted == ["default/greedy"] and fc.evictions == [("default", "greedy")]
    with pytest.raises(NotFound):
        fc.get("pods", "greedy", "default")


def test_hbm_tolerance_is_configurable():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=1))
    a = _bound_pod(fc, "p", 4)
    src = synthetic_node(1, node="n1")
    src.procs = {0: [{"pid": 7, "vram_bytes": int(4.4 * 2**30)}]}     # 0.4 GiB of runtime overhead
    ag = NodeAgent("n1", rds(), src, client=fc, pod_resolver={7: O.uid(a)}.get)
    assert ag.check_hbm() == {}                                       # default 0.5 GiB covers it
    ag.hbm_tolerance_gib = 0.25
    assert list(ag.check_hbm()) == ["default/p"]


def test_agent_recognises_its_own_host_pid_by_cgroup(tmp_path):
    """amd-smi reports host PIDs; the agent's container PID namespace hides its host PID,
    so its own GPU context is recognised through the host /proc cgroup instead."""
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=1))
    mine = open("/proc/self/cgroup").read()
    (tmp_path / "31337").mkdir()
    (tmp_path / "31337" / "cgroup").write_text(mine)
    (tmp_path / "4242").mkdir()
    (tmp_path / "4242" / "cgroup").write_text("0::/kubepods/other-pod\n")
    src = synthetic_node(1, node="n1")
    src.procs = {0: [{"pid": 31337, "name": "agent"}, {"pid": 4242, "name": "train.py"}]}
    ag = NodeAgent("n1", rds(), src, client=fc, host_proc=str(tmp_path))
    reasons = ag.busy_reasons()
    assert len(reasons) == 1 and "4242" in reasons[0]
