"""Per-pod rocprofv3 profiling for kubelet-started pods (agent.profile_webhook +
agent.pod_profiler.ProfileIngestor): the admission mutation on a fake apiserver and over the
webhook's HTTP endpoint, kubelet-style env / $(VAR) / hostPath handling in the launcher, and
the agent turning finished profile directories into workload history.

Reference analog superseded: the profiler DaemonSet that only publishes device UUIDs
(reference pkg/profiler/profile_gpu.sh:3-13, deploy/profiler/client-daemonset.yaml:1-38)."""
import base64
import json
import os
import urllib.request

from k8s_gpu_scheduler_amd.agent import profile_webhook as PW
from k8s_gpu_scheduler_amd.agent.launcher import PodLauncher, _expand
from k8s_gpu_scheduler_amd.agent.pod_profiler import ProfileIngestor, summarize_kernel_trace
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.kube.patch import apply_json_patch
from k8s_gpu_scheduler_amd.recommender.admission import (AdmissionServer, RedisHistory, ResizeAdmission,
                                                         webhook_handler)
from k8s_gpu_scheduler_amd.recommender.resize import recommend
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
from k8s_gpu_scheduler_amd.store.resp import Redis

ARGV = ["python3", "-m", "k8s_gpu_scheduler_amd.ops.podrun", "--workload", "onnx_resnet50_1024"]


def _pod(name="onnx-resnet50-1024-a", label=True, command=True, **kw):
    pod = O.make_pod(name, gpu_cu=64, gpu_mem_gib=8, env={C.ENV_ITERATIONS: "20"},
                     labels_={PW.LABEL_PROFILE: "trace"} if label else None, **kw)
    ctr = pod["spec"]["containers"][0]
    if command:
        ctr["command"] = list(ARGV[:3])
        ctr["args"] = list(ARGV[3:])
    return pod


def test_injector_wraps_opted_in_container_program_after_double_dash():
    inj = PW.ProfileInjector(rocprof="/opt/rocm/bin/rocprofv3")
    fc = FakeCluster()
    fc.add_admission("pods", inj)
    fc.create("pods", _pod())
    fc.create("pods", _pod("tensorflow-mobilenet-1024-b", label=False))
    got = fc.get("pods", "onnx-resnet50-1024-a", "default")
    ctr = got["spec"]["containers"][0]
    cmd = ctr["command"]
    assert cmd[0] == "/opt/rocm/bin/rocprofv3" and "--kernel-trace" in cmd and "--stats" in cmd
    i = cmd.index("--")
    assert cmd[i + 1:] == ARGV[:3] and ctr["args"] == ARGV[3:]       # program right after --
    d = cmd[cmd.index("-d") + 1]
    assert d == "/gpusched-prof/cu64-hbm8-it20"
    envs = {e["name"]: e for e in ctr["env"]}
    assert envs[PW.UID_ENV]["valueFrom"]["fieldRef"]["fieldPath"] == "metadata.uid"
    assert envs[C.ENV_ITERATIONS]["value"] == "20"                  # the pod's own env kept
    # the container sees only its own <ns>/<pod>/<uid>/<container> directory of the hostPath
    assert {"name": PW.VOLUME, "mountPath": PW.MOUNT,
            "subPathExpr": "$(GPUSCHED_POD_NAMESPACE)/$(GPUSCHED_POD_NAME)/$(GPUSCHED_POD_UID)/main"} \
        in ctr["volumeMounts"]
    vol = next(v for v in got["spec"]["volumes"] if v["name"] == PW.VOLUME)
    assert vol["hostPath"] == {"path": PW.HOST_DIR, "type": "DirectoryOrCreate"}
    assert O.annotations(got)[PW.ANNOT_PROFILED] == "main"
    # not opted in: untouched; already wrapped: never wrapped twice
    plain = fc.get("pods", "tensorflow-mobilenet-1024-b", "default")
    assert plain["spec"]["containers"][0]["command"] == ARGV[:3]
    assert inj.patch_ops(got) == ([], None)


def test_injector_entrypoint_container_needs_argv_annotation_and_pmc_mode():
    inj = PW.ProfileInjector()
    pod = _pod(command=False)
    assert inj.patch_ops(pod) == ([], None) and inj.stats["skipped_no_command"] == 1
    pod["metadata"]["annotations"] = {PW.ANNOT_PROFILE_ARGV: json.dumps(ARGV),
                                      PW.ANNOT_PROFILE_COUNTERS: "SQ_WAVES,SQ_BUSY_CYCLES"}
    pod["metadata"]["labels"][PW.LABEL_PROFILE] = "pmc"
    pod["spec"]["containers"][0]["args"] = ["--ignored"]
    out = apply_json_patch(pod, inj.patch_ops(pod)[0])
    ctr = out["spec"]["containers"][0]
    cmd = ctr["command"]
    assert cmd[cmd.index("--pmc") + 1:cmd.index("--pmc") + 3] == ["SQ_WAVES", "SQ_BUSY_CYCLES"]
    assert "--kernel-trace" not in cmd                   # counters never with trace domains
    assert cmd[cmd.index("--") + 1:] == ARGV and "args" not in ctr


def test_webhook_endpoint_chains_resize_and_profile():
    """One AdmissionReview to /mutate: the resize shrinks the request from history, then the
    profiler wraps the pod -- with the RESIZED request in its path tag; /profile alone only
    wraps."""
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    hist = RedisHistory(r)
    for _ in range(4):
        hist.append("onnx_resnet50_1024", {"cu": 32, "throughput": 900.0, "hbm_gib": 3.0})
    resize = ResizeAdmission(hist.read)
    inj = PW.ProfileInjector()
    srv = AdmissionServer(PW.ChainAdmission(resize, inj), "127.0.0.1", 0, routes={"/profile": inj}).start()
    try:
        pod = _pod()
        pod["spec"]["containers"][0]["env"] = []
        pod["spec"]["containers"][0]["env"].append({"name": "SLO", "value": "500"})
        pod["spec"]["containers"][0]["env"].append({"name": C.ENV_ITERATIONS, "value": "20"})
        for path, resized in (("/mutate", True), ("/profile", False)):
            review = {"request": {"uid": "u1", "kind": {"kind": "Pod"}, "operation": "CREATE", "object": pod}}
            req = urllib.request.Request(srv.url + path, json.dumps(review).encode(),
                                         {"Content-Type": "application/json"})
            resp = json.loads(urllib.request.urlopen(req, timeout=5).read())["response"]
            assert resp["allowed"] and resp["patchType"] == "JSONPatch"
            out = apply_json_patch(pod, json.loads(base64.b64decode(resp["patch"])))
            cmd = out["spec"]["containers"][0]["command"]
            tag = cmd[cmd.index("-d") + 1].rsplit("/", 1)[1]
            assert tag.startswith("cu32-") if resized else tag.startswith("cu64-"), (path, tag)
            assert out["spec"]["containers"][0]["resources"]["requests"][C.RESOURCE_GPU_CU] == \
                ("32" if resized else "64")
    finally:
        srv.stop()


def test_launcher_expands_downward_api_vars_and_maps_host_paths(tmp_path):
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=1))
    inj = PW.ProfileInjector(rocprof="echo")
    pod = apply_json_patch(_pod(), inj.patch_ops(_pod())[0])
    fc.create("pods", pod)
    pod = fc.get("pods", O.name(pod), "default")
    la = PodLauncher(fc, "n1")
    la.host_root = str(tmp_path)
    res = la.run(pod)
    assert res.rc == 0, res.stderr
    out = res.stdout.split()
    d = out[out.index("-d") + 1]
    assert d == f"{tmp_path}{PW.HOST_DIR}/default/{O.name(pod)}/{O.uid(pod)}/main/cu64-hbm8-it20"
    assert os.path.isdir(f"{tmp_path}{PW.HOST_DIR}")
    assert _expand("$(A)-$$(A)-$(MISSING)", {"A": "x"}) == "x-$(A)-$(MISSING)"


def _write_profile(root, ns, name, uid, container, tag, kernels):
    d = os.path.join(root, ns, name, uid, container, tag)
    os.makedirs(d)
    with open(os.path.join(d, "run_kernel_stats.csv"), "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n')
        for n, calls, ns_ in kernels:
            f.write(f'"{n}",{calls},{ns_},{ns_ // calls},10.0\n')
    with open(os.path.join(d, "run_kernel_trace.csv"), "w") as f:
        f.write('"Kernel_Name","Start_Timestamp","End_Timestamp"\n')
        t = 1_000_000
        for i in range(10):        # 10 kernels of 1 ms with 0.25 ms gaps: span 12.25 ms, busy 10 ms
            f.write(f'"k",{t},{t + 1_000_000}\n')
            t += 1_250_000
    return d


def test_agent_ingests_finished_profiles_into_workload_history(tmp_path):
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    root = str(tmp_path / "prof")
    d = _write_profile(root, "default", "onnx-resnet50-1024-x7", "uid-1", "main", "cu64-hbm8-it20",
                       [("gs::gemm_bf16_nt_256_8ph<true, true, true, true, false>", 60, 8_000_000),
                        ("gs::stream_triad_u<4, true>", 20, 2_000_000)])
    os.makedirs(os.path.join(root, "default", "other", "uid-2", "main", "cu64-hbm4-it0"))   # still running
    ing = ProfileIngestor(root, RedisHistory(r))
    assert ing.step() == 1
    h = RedisHistory(r).read("onnx_resnet50_1024")
    assert len(h) == 1
    s = h[0]
    assert s["source"] == "rocprof" and s["cu"] == 64 and s["hbm_gib"] == 8.0
    assert s["kernels"] == 80 and abs(s["gpu_busy_ms"] - 10.0) < 1e-9
    assert s["top"][0]["name"].startswith("gs::gemm_bf16_nt_256_8ph")
    assert abs(s["span_ms"] - 12.25) < 1e-9 and abs(s["busy_frac"] - 10.0 / 12.25) < 1e-9
    assert abs(s["throughput"] - 20 / 10e-3) < 1e-6          # iterations per GPU-busy second
    assert not os.path.exists(d)                            # ingested once, then removed
    assert ing.step() == 0                                  # the unfinished one stays
    assert os.path.isdir(os.path.join(root, "default", "other", "uid-2", "main", "cu64-hbm4-it0"))
    # the resize recommendation reads the rocprof samples like any other history
    adv = recommend(h * 3, 128, 16.0, slo=1500.0)
    assert adv.cu == 64 and "smallest share" in adv.reason


def test_node_agent_step_runs_the_ingestor(tmp_path):
    from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
    from k8s_gpu_scheduler_amd.agent.devices import synthetic_node
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    root = str(tmp_path / "prof")
    _write_profile(root, "default", "tensorflow-mobilenet-2048-q", "u9", "main", "cu32-hbm4-it10",
                   [("gs::stream_triad_u<4, true>", 30, 3_000_000)])
    ag = NodeAgent("n1", r, synthetic_node(1, node="n1"), profile_dir=root)
    ag.step()
    h = RedisHistory(r).read("tensorflow_mobilenet_2048")
    assert h and h[-1]["cu"] == 32 and h[-1]["source"] == "rocprof"


def test_kernel_trace_summary_merges_overlaps(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text('"Start_Timestamp","End_Timestamp"\n0,4000000\n1000000,2000000\n5000000,6000000\n')
    s = summarize_kernel_trace(str(p))
    assert s == {"span_ms": 6.0, "busy_union_ms": 5.0, "first_ns": 0, "last_ns": 6000000}


def test_webhook_handler_fails_open():
    class Boom:
        def patch_ops(self, pod):
            raise RuntimeError("redis down")
    out = webhook_handler(Boom(), {"request": {"uid": "x", "kind": {"kind": "Pod"}, "object": {}}})
    assert out["response"]["allowed"] and "patch" not in out["response"]


def test_ingestor_keeps_runs_of_deleted_pods_within_the_grace_and_rejects_foreign_uids(tmp_path):
    """a Job pod deleted before the agent's pass lost its profile.  Its directory is
    authentic by construction (only its own container could write under <ns>/<pod>/<uid>), so it
    is ingested under the name's workload while younger than the orphan grace; a pod of the same
    name with ANOTHER uid still rejects it, and stale orphans are dropped."""
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    root = str(tmp_path / "prof")
    kern = [("gs::stream_triad_u<4, true>", 20, 2_000_000)]
    gone = _write_profile(root, "default", "onnx-mobilenet-1024-job1", "uid-a", "main", "cu64-hbm4-it20", kern)
    other = _write_profile(root, "default", "onnx-resnet50-2048-j", "uid-b", "main", "cu64-hbm8-it20", kern)
    old = _write_profile(root, "default", "onnx-ssd-mobilenet-1024-z", "uid-c", "main", "cu64-hbm4-it20", kern)
    os.utime(old, (1.0, 1.0))                                             # an orphan from long ago
    live = {("default", "onnx-resnet50-2048-j"): {"metadata": {"name": "onnx-resnet50-2048-j",
                                                               "namespace": "default", "uid": "uid-NEW"}}}
    forged = _write_profile(root, "default", "onnx-resnet50-4096-x", "uid-d", "main", "cu64-hbm8-it20", kern)
    ing = ProfileIngestor(root, RedisHistory(r), pod_lookup=lambda ns, n: live.get((ns, n)), orphan_grace_s=600.0)
    # the agent saw the deleted pod (and the stale one) bound to its node before they went;
    # uid-d was never seen here: a directory nobody can vouch for is dropped
    ing.note_pods([{"metadata": {"name": "onnx-mobilenet-1024-job1", "namespace": "default", "uid": "uid-a"}},
                   {"metadata": {"name": "onnx-ssd-mobilenet-1024-z", "namespace": "default", "uid": "uid-c"}}])
    assert ing.step() == 1
    assert not RedisHistory(r).read("onnx_resnet50_4096") and not os.path.exists(forged)
    assert RedisHistory(r).read("onnx_mobilenet_1024")                    # the deleted pod's run kept
    assert not RedisHistory(r).read("onnx_resnet50_2048")                 # uid mismatch: rejected
    assert not RedisHistory(r).read("onnx_ssd_mobilenet_1024")            # stale orphan: dropped
    assert not os.path.exists(gone) and not os.path.exists(other) and not os.path.exists(old)
