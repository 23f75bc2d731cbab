"""Deploy manifests keep the reference's names, namespaces, ports and RBAC surface
("same ... deploy manifests"; reference deploy/*.yaml), with the MI355X
changes (ROCm device access, no NVIDIA runtime) and a loadable scheduler profile."""
import glob
import os
import subprocess

import pytest

import yaml

from k8s_gpu_scheduler_amd.framework.config import load_config
from k8s_gpu_scheduler_amd.framework.runtime import Framework
from k8s_gpu_scheduler_amd.plugins import full_registry

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")


def _docs():
    out = []
    for f in sorted(glob.glob(os.path.join(DEPLOY, "**", "*.yaml"), recursive=True)):
        with open(f) as fh:
            for d in yaml.safe_load_all(fh):
                if d:
                    out.append((os.path.relpath(f, DEPLOY), d))
    return out


def _find(kind, name, ns=None):
    for f, d in _docs():
        md = d.get("metadata", {})
        if d.get("kind") == kind and md.get("name") == name and (ns is None or md.get("namespace") == ns):
            return d
    raise AssertionError(f"{kind} {ns}/{name} not in deploy/")


def test_every_manifest_parses_and_has_kind():
    docs = _docs()
    assert len(docs) >= 15
    for f, d in docs:
        assert d.get("apiVersion") and d.get("kind"), f


def test_reference_service_ports_and_namespaces():
    redis = _find("Service", "redis", "redis")
    assert any(p.get("nodePort") == 32767 and p.get("port") == 6379 for p in redis["spec"]["ports"])
    rec = _find("Service", "recommender", "recommender") if any(
        d.get("kind") == "Service" and d["metadata"].get("name") == "recommender" for _, d in _docs()) else None
    if rec is None:
        rec = next(d for _, d in _docs() if d.get("kind") == "Service"
                   and d["metadata"].get("namespace") == "recommender")
    assert any(p.get("nodePort") == 32700 and p.get("targetPort") in (50051, "50051") for p in rec["spec"]["ports"])
    _find("StatefulSet", "redis", "redis")


def test_scheduler_profile_loads_and_instantiates():
    cfg = load_config(os.path.join(DEPLOY, "scheduler.yaml"))
    prof = cfg.profile("gpu-scheduler")
    assert prof is not None and cfg.leader_election.leader_elect
    assert cfg.leader_election.resource_name == "gpu-scheduler"
    assert {r.name: r.weight for r in prof.enabled("score")}["GPU"] == 10100
    assert prof.args("GPU")["mode"] == "fixed"
    fw = Framework(prof, full_registry(), handle=None)
    gpu = fw.plugin("GPU")
    assert gpu.args.w_balance == 0.5 and gpu.args.model == "MI355X"
    # the deployed burst planner: co-run model, 30 % tolerance, backlog carried between bursts
    assert gpu.args.plan_bursts and gpu.args.plan_tolerance == 0.3 and gpu.args.plan_carry == 1.0
    assert gpu.args.plan_budget_ms == 20 and gpu.planner.budget is not None
    assert gpu.planner is not None and gpu.planner.carry == 1.0
    dep = _find("Deployment", "gpu-scheduler", "kube-system")
    spec = dep["spec"]["template"]["spec"]
    assert (spec.get("serviceAccountName") or spec.get("serviceAccount")) == "sample-sa"   # reference SA name


def test_rbac_covers_what_the_scheduler_does():
    rules = [r for _, d in _docs() if d.get("kind") == "ClusterRole" for r in d.get("rules", [])]

    def allowed(resource, verb):
        return any(resource in r.get("resources", []) and (verb in r.get("verbs", []) or "*" in r.get("verbs", []))
                   for r in rules)
    for res, verb in [("pods", "list"), ("pods", "watch"), ("pods", "delete"), ("pods/binding", "create"),
                      ("bindings", "create"), ("configmaps", "update"), ("configmaps", "create"),
                      ("nodes", "patch"), ("leases", "update"), ("events", "create")]:
        assert allowed(res, verb) or (res == "pods/binding" and allowed("bindings", verb)), (res, verb)


def test_node_agent_daemonset_uses_rocm_devices_not_nvidia():
    ds = next(d for _, d in _docs() if d.get("kind") == "DaemonSet")
    text = yaml.safe_dump(ds)
    assert "/dev/kfd" in text and "/dev/dri" in text
    assert "nvidia" not in text.lower()
    env = {e["name"] for c in ds["spec"]["template"]["spec"]["containers"] for e in c.get("env", [])}
    assert {"NODE_NAME", "POD_NAME", "POD_NAMESPACE"} <= env     # downward API, as the reference


def test_busybox_fixture_matches_reference_shape():
    dep = next(d for f, d in _docs() if f.startswith("busybox") and d.get("kind") == "Deployment")
    spec = dep["spec"]["template"]["spec"]
    assert spec["schedulerName"] == "gpu-scheduler"
    c = spec["containers"][0]
    assert any(e["name"] == "SLO" for e in c.get("env", []))
    assert any("configMapRef" in ef for ef in c.get("envFrom", []))


def test_agent_daemonset_serves_the_device_plugin():
    ds = next(d for _, d in _docs() if d.get("kind") == "DaemonSet")
    c = ds["spec"]["template"]["spec"]["containers"][0]
    assert "--device-plugin" in c["args"]
    assert any(m["mountPath"] == "/var/lib/kubelet/device-plugins" for m in c["volumeMounts"])
    rules = [r for f, d in _docs() if f.startswith("profiler") and d.get("kind") == "ClusterRole"
             for r in d["rules"]]
    pod_verbs = {v for r in rules if "pods" in r["resources"] for v in r["verbs"]}
    assert {"patch", "delete", "list"} <= pod_verbs


def test_agent_role_covers_what_the_agent_does():
    """The node agent creates GPUMemoryOveruse Warning events and evicts through the
    Eviction API: its ClusterRole must allow both (create_event swallows a 403)."""
    rules = [r for f, d in _docs() if f.startswith("profiler") and d.get("kind") == "ClusterRole"
             for r in d["rules"]]

    def allowed(resource, verb, group=""):
        return any(resource in r.get("resources", []) and group in r.get("apiGroups", [""])
                   and (verb in r.get("verbs", []) or "*" in r.get("verbs", [])) for r in rules)
    assert allowed("events", "create")
    assert allowed("events", "create", "events.k8s.io")
    assert allowed("pods/eviction", "create")
    assert allowed("nodes", "patch")


def _replication_script():
    import yaml
    docs = list(yaml.safe_load_all(open(os.path.join(ROOT, "deploy/redis/redis-statefulset.yaml"))))
    sts = next(d for d in docs if d and d.get("kind") == "StatefulSet")
    init = sts["spec"]["template"]["spec"]["initContainers"][0]
    return init["args"][0], {e["name"]: e["value"] for e in init["env"]}


@pytest.mark.parametrize("host,sentinel,expect", [
    ("redis-0", "", None),                                   # no sentinel: redis-0 is the master
    ("redis-2", "", "redis-0.redis.redis.svc.cluster.local"),  # no sentinel: replicas follow redis-0
    ("redis-0", "10.0.0.7", "10.0.0.7"),                     # sentinel failed over to another pod
    ("redis-1", "10.0.0.9", None),                           # this pod IS the sentinel's master
])
def test_redis_replication_bootstrap(tmp_path, host, sentinel, expect):
    """The init container's replicaof decision (reference deploy/redis/redis-statefulset.yaml:37-56),
    run under sh with stub redis-cli / hostname."""
    script, env = _replication_script()
    conf, etc, bin_ = tmp_path / "conf", tmp_path / "etc", tmp_path / "bin"
    for d in (conf, etc, bin_):
        d.mkdir()
    (conf / "redis.conf").write_text("appendonly yes\n")
    ip = {"redis-0": "10.0.0.5", "redis-1": "10.0.0.9", "redis-2": "10.0.0.11"}[host]
    (bin_ / "redis-cli").write_text(
        "#!/bin/sh\ncase \"$*\" in *ping*) [ -n \"$SENT\" ] && echo PONG || exit 1;; "
        "*get-master-addr-by-name*) echo \"$SENT\"; echo 6379;; esac\n")
    (bin_ / "hostname").write_text(
        f"#!/bin/sh\ncase \"$1\" in -f) echo {host}.redis.redis.svc.cluster.local;; -i) echo {ip};; *) echo {host};; esac\n")
    for f in bin_.iterdir():
        f.chmod(0o755)
    script = script.replace("/conf/", f"{conf}/").replace("/etc/redis/", f"{etc}/")
    e = dict(os.environ, PATH=f"{bin_}:{os.environ['PATH']}", HOSTNAME=host, SENT=sentinel, **env)
    subprocess.run(["sh", "-ec", script], env=e, check=True, capture_output=True)
    out = (etc / "redis.conf").read_text()
    assert out.startswith("appendonly yes")
    if expect is None:
        assert "replicaof" not in out
    else:
        assert f"replicaof {expect} 6379" in out
