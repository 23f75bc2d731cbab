"""Kubernetes object model.

Objects are kept in their wire form (plain JSON dicts, exactly what the apiserver sends),
so the same structures flow through the REST client, the in-memory FakeCluster, the
extender and the scheduler without conversion.  This module holds the accessors the
rest of the framework uses on them.

Reference equivalents: `utils.GetEnv` (reference utils/utils.go:124-132), the envFrom
ConfigMap walk of `GetSLOs` / `AppendToExistingConfigMapsInPod`
(reference pkg/plugins/gpu_plugin/gpu_plugins.go:111-130, pkg/resources/pods.go:156-174).
"""
from __future__ import annotations

import copy
import json
import re
import time
import uuid as _uuid
from typing import Any, Dict, Iterable, List, Optional, Tuple

from . import constants as C

Obj = Dict[str, Any]

# --------------------------------------------------------------------------- quantities
_BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DEC = {"n": 1e-9, "u": 1e-6, "m": 1e-3, "": 1.0, "k": 1e3, "K": 1e3, "M": 1e6, "G": 1e9,
        "T": 1e12, "P": 1e15, "E": 1e18}
_QRE = re.compile(r"^([+-]?[0-9.]+(?:[eE][+-]?[0-9]+)?)([a-zA-Z]*)$")


def parse_quantity(q: Any) -> float:
    """Parse a Kubernetes resource quantity ("500m", "1Gi", "2", 3) into a float."""
    if q is None:
        return 0.0
    if isinstance(q, (int, float)):
        return float(q)
    s = str(q).strip()
    m = _QRE.match(s)
    if not m:
        raise ValueError(f"invalid quantity {q!r}")
    num, suf = m.groups()
    if suf in _BIN:
        return float(num) * _BIN[suf]
    if suf in _DEC:
        return float(num) * _DEC[suf]
    raise ValueError(f"invalid quantity suffix {suf!r} in {q!r}")


def format_quantity(v: float) -> str:
    if float(v).is_integer():
        return str(int(v))
    return f"{int(round(v * 1000))}m"


# --------------------------------------------------------------------------- metadata
def meta(obj: Obj) -> Obj:
    return obj.setdefault("metadata", {})


def name(obj: Obj) -> str:
    return obj.get("metadata", {}).get("name", "")


def namespace(obj: Obj) -> str:
    return obj.get("metadata", {}).get("namespace", "") or "default"


def key(obj: Obj) -> str:
    """namespace/name key as used by client-go indexers (cluster-scoped: name)."""
    md = obj.get("metadata", {})
    ns = md.get("namespace")
    return f"{ns}/{md.get('name', '')}" if ns else md.get("name", "")


def labels(obj: Obj) -> Dict[str, str]:
    return obj.get("metadata", {}).get("labels") or {}


def annotations(obj: Obj) -> Dict[str, str]:
    return obj.get("metadata", {}).get("annotations") or {}


def uid(obj: Obj) -> str:
    return obj.get("metadata", {}).get("uid", "")


def resource_version(obj: Obj) -> str:
    return obj.get("metadata", {}).get("resourceVersion", "")


def deepcopy(obj: Any) -> Any:
    """Deep copy of a JSON-shaped object (dict/list/scalars) -- ~5x faster than
    copy.deepcopy, which matters on the apiserver/informer hot path."""
    t = type(obj)
    if t is dict:
        return {k: (v if type(v) in _SCALARS else deepcopy(v)) for k, v in obj.items()}
    if t is list:
        return [v if type(v) in _SCALARS else deepcopy(v) for v in obj]
    if t in _SCALARS:
        return obj
    return copy.deepcopy(obj)


_SCALARS = (str, int, float, bool, type(None))


# --------------------------------------------------------------------------- constructors
def make_node(node_name: str, *, gpus: int = 8, product: str = C.MI355X, cpu: str = "192",
              memory: str = "1536Gi", address: Optional[str] = None,
              labels_: Optional[Dict[str, str]] = None, partition: str = "SPX",
              taints: Optional[List[Obj]] = None) -> Obj:
    """Build a Node object describing an MI355X host (8 GPUs by default)."""
    lab = {"kubernetes.io/hostname": node_name}
    if gpus:
        lab.update({C.LABEL_GPU_PRODUCT: product, C.LABEL_GPU_COUNT: str(gpus),
                    C.LABEL_COMPUTE_PARTITION: partition,
                    C.LABEL_MEMORY_PARTITION: "NPS1"})
    if labels_:
        lab.update(labels_)
    parts = C.COMPUTE_PARTITIONS.get(partition, 1)
    alloc = {C.RESOURCE_CPU: cpu, C.RESOURCE_MEMORY: memory, C.RESOURCE_PODS: "250"}
    if gpus:
        alloc[C.RESOURCE_GPU] = str(gpus * parts)
        alloc[C.RESOURCE_GPU_CU] = str(gpus * C.MI355X_CUS)
        alloc[C.RESOURCE_GPU_MEM] = str(gpus * C.MI355X_HBM_GIB)
    return {
        "apiVersion": "v1", "kind": "Node",
        "metadata": {"name": node_name, "labels": lab},
        "spec": {"taints": list(taints or [])},
        "status": {
            "capacity": dict(alloc), "allocatable": dict(alloc),
            "addresses": [{"type": "InternalIP", "address": address or "10.0.0.1"}],
            "conditions": [{"type": "Ready", "status": "True"}],
        },
    }


def make_pod(pod_name: str, *, ns: str = "default", scheduler: str = C.SCHEDULER_NAME,
             slo: Optional[float] = None, gpus: int = 0, gpu_cu: int = 0, gpu_mem_gib: float = 0,
             cpu: str = "100m", memory: str = "64Mi", config_maps: Iterable[str] = (),
             env: Optional[Dict[str, str]] = None, annotations_: Optional[Dict[str, str]] = None,
             labels_: Optional[Dict[str, str]] = None, image: str = "busybox:latest",
             node_name: Optional[str] = None, phase: str = "Pending", priority: int = 0,
             tolerations: Optional[List[Obj]] = None, node_selector: Optional[Dict[str, str]] = None,
             gpu_limits: bool = True) -> Obj:
    """Build a Pod in the shape the reference's e2e fixtures use
    (reference deploy/busybox/busybox.yaml:15-28: schedulerName, envFrom configMapRef, env SLO)."""
    envs = []
    if slo is not None:
        envs.append({"name": C.ENV_SLO, "value": str(slo)})
    for k, v in (env or {}).items():
        envs.append({"name": k, "value": str(v)})
    req = {C.RESOURCE_CPU: cpu, C.RESOURCE_MEMORY: memory}
    if gpus:
        req[C.RESOURCE_GPU] = str(gpus)
    if gpu_cu:
        req[C.RESOURCE_GPU_CU] = str(gpu_cu)
    if gpu_mem_gib:
        req[C.RESOURCE_GPU_MEM] = format_quantity(gpu_mem_gib)
    container = {"name": "main", "image": image, "env": envs,
                 "envFrom": [{"configMapRef": {"name": cm}} for cm in config_maps],
                 "resources": {"requests": req, "limits": {k: v for k, v in req.items()
                                                           if k.startswith("amd.com/") and gpu_limits}}}
    spec = {"schedulerName": scheduler, "containers": [container], "priority": priority}
    if node_name:
        spec["nodeName"] = node_name
    if tolerations:
        spec["tolerations"] = tolerations
    if node_selector:
        spec["nodeSelector"] = node_selector
    return {
        "apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": pod_name, "namespace": ns, "uid": str(_uuid.uuid4()),
                     "labels": dict(labels_ or {}), "annotations": dict(annotations_ or {}),
                     "creationTimestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())},
        "spec": spec,
        "status": {"phase": phase},
    }


def make_config_map(cm_name: str, data: Optional[Dict[str, str]] = None, ns: str = "default") -> Obj:
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": cm_name, "namespace": ns}, "data": dict(data or {})}


# --------------------------------------------------------------------------- pod accessors
def containers(pod: Obj) -> List[Obj]:
    return pod.get("spec", {}).get("containers") or []


def get_env(pod: Obj, env_name: str) -> str:
    """Value of env var `env_name` on Containers[0] ("" when absent).
    Same contract as reference utils/utils.go:124-132."""
    cs = containers(pod)
    if not cs:
        return ""
    for e in cs[0].get("env") or []:
        if e.get("name") == env_name:
            return str(e.get("value", ""))
    return ""


def pod_slo(pod: Obj) -> float:
    """SLO (minimum throughput) of a pod: env SLO on Containers[0], else the annotation.
    Parse failure / absence -> 0 (reference gpu_plugins.go:460-469)."""
    raw = get_env(pod, C.ENV_SLO) or annotations(pod).get(C.ANNOT_SLO, "")
    try:
        return float(raw) if raw != "" else 0.0
    except ValueError:
        return 0.0


def node_unhealthy_devices(node: Obj) -> Dict[str, str]:
    """{uuid: reason} from the agent's unhealthy-devices node annotation ({} if none / bad)."""
    raw = annotations(node).get(C.ANNOT_UNHEALTHY, "")
    if not raw:
        return {}
    try:
        v = json.loads(raw)
    except ValueError:
        return {}
    return {str(k): str(r) for k, r in v.items()} if isinstance(v, dict) else {}


def pod_iterations(pod: Obj) -> float:
    """Declared iteration count of a batch pod (env ITERATIONS on Containers[0]); 0 = a
    long-running service (its load is its SLO rate instead)."""
    raw = get_env(pod, C.ENV_ITERATIONS)
    try:
        return max(0.0, float(raw)) if raw != "" else 0.0
    except ValueError:
        return 0.0


def env_from_config_maps(pod: Obj, first_container_only: bool = False) -> List[str]:
    """ConfigMap names referenced by envFrom (all containers, like
    reference pkg/resources/pods.go:162-171; or just Containers[0])."""
    out: List[str] = []
    cs = containers(pod)
    if first_container_only:
        cs = cs[:1]
    for c in cs:
        for ef in c.get("envFrom") or []:
            ref = ef.get("configMapRef")
            if ref and ref.get("name"):
                out.append(ref["name"])
    return out


def scheduler_name(pod: Obj) -> str:
    return pod.get("spec", {}).get("schedulerName") or "default-scheduler"


def node_name_of(pod: Obj) -> str:
    return pod.get("spec", {}).get("nodeName") or ""


def phase(pod: Obj) -> str:
    return pod.get("status", {}).get("phase", "")


def is_terminal(pod: Obj) -> bool:
    return phase(pod) in ("Succeeded", "Failed")


def priority(pod: Obj) -> int:
    return int(pod.get("spec", {}).get("priority") or 0)


_REQ_CACHE: Dict[str, Dict[str, float]] = {}


def pod_requests(pod: Obj) -> Dict[str, float]:
    """Sum of container requests (limits used when a request is missing, as for extended
    resources) -- the NodeResourcesFit view of a pod.  Container resources are immutable
    after creation, so the parse is memoised per pod UID (treat the result as read-only)."""
    u = pod.get("metadata", {}).get("uid")
    if u:
        hit = _REQ_CACHE.get(u)
        if hit is not None:
            return hit
        if len(_REQ_CACHE) > 200000:
            _REQ_CACHE.clear()
        tot = _pod_requests(pod)
        _REQ_CACHE[u] = tot
        return tot
    return _pod_requests(pod)


# kube-scheduler's scoring view of a container without a cpu / memory request
# (upstream schedutil.DefaultMilliCPURequest / DefaultMemoryRequest)
DEFAULT_MILLI_CPU_REQUEST = 100
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024
_NZ_CACHE: Dict[str, Tuple[int, int]] = {}


def pod_nonzero_requests(pod: Obj) -> Tuple[int, int]:
    """(milli-CPU, memory bytes) the resource Score plugins charge for a pod: each container's
    request, with an unset cpu / memory request counted as 100m / 200 MiB (an explicit 0
    stays 0), init containers as a max, plus the pod overhead (upstream
    calculatePodResourceRequest + GetNonzeroRequests).  Memoised per pod UID."""
    u = pod.get("metadata", {}).get("uid")
    if u:
        hit = _NZ_CACHE.get(u)
        if hit is not None:
            return hit
    spec = pod.get("spec") or {}

    def one(c: Obj) -> Tuple[int, int]:
        res = c.get("resources") or {}
        reqs = dict(res.get("limits") or {})       # the apiserver defaults requests from limits
        reqs.update(res.get("requests") or {})
        cpu = int(round(parse_quantity(reqs["cpu"]) * 1000)) if "cpu" in reqs else DEFAULT_MILLI_CPU_REQUEST
        mem = int(parse_quantity(reqs["memory"])) if "memory" in reqs else DEFAULT_MEMORY_REQUEST
        return cpu, mem

    cpu = mem = 0
    for c in spec.get("containers") or []:
        a, b = one(c)
        cpu, mem = cpu + a, mem + b
    for c in spec.get("initContainers") or []:
        a, b = one(c)
        cpu, mem = max(cpu, a), max(mem, b)
    ov = spec.get("overhead") or {}
    if "cpu" in ov:
        cpu += int(round(parse_quantity(ov["cpu"]) * 1000))
    if "memory" in ov:
        mem += int(parse_quantity(ov["memory"]))
    out = (cpu, mem)
    if u:
        if len(_NZ_CACHE) > 200000:
            _NZ_CACHE.clear()
        _NZ_CACHE[u] = out
    return out


def _pod_requests(pod: Obj) -> Dict[str, float]:
    tot: Dict[str, float] = {}
    for c in containers(pod):
        res = c.get("resources") or {}
        reqs = dict(res.get("limits") or {})
        reqs.update(res.get("requests") or {})
        for k, v in reqs.items():
            tot[k] = tot.get(k, 0.0) + parse_quantity(v)
    for ic in pod.get("spec", {}).get("initContainers") or []:
        res = ic.get("resources") or {}
        for k, v in (res.get("requests") or {}).items():
            tot[k] = max(tot.get(k, 0.0), parse_quantity(v))
    return tot


def forget_requests(pod: Obj) -> None:
    """Drop the memoised request parse of a pod (admission mutated its resources before
    the object was persisted)."""
    u = pod.get("metadata", {}).get("uid")
    if u:
        _REQ_CACHE.pop(u, None)


def gpu_request(pod: Obj, cached: bool = True) -> Tuple[int, int, float]:
    """(whole GPUs, CUs, HBM GiB) requested by a pod."""
    r = pod_requests(pod) if cached else _pod_requests(pod)
    return (int(r.get(C.RESOURCE_GPU, 0)), int(r.get(C.RESOURCE_GPU_CU, 0)),
            float(r.get(C.RESOURCE_GPU_MEM, 0.0)))


def gpu_qos(pod: Obj) -> str:
    """"Guaranteed" when the fractional CU request is also its limit (hard CU mask),
    "Burstable" when only requested (accounted share, may use idle CUs) -- the
    Kubernetes QoS rule applied to amd.com/gpu-cu."""
    for c in containers(pod):
        res = c.get("resources") or {}
        if C.RESOURCE_GPU_CU in (res.get("requests") or {}) and C.RESOURCE_GPU_CU not in (res.get("limits") or {}):
            return "Burstable"
    return "Guaranteed"


def wants_gpu(pod: Obj) -> bool:
    g, cu, mem = gpu_request(pod)
    return g > 0 or cu > 0 or mem > 0


# --------------------------------------------------------------------------- node accessors
def node_allocatable(node: Obj) -> Dict[str, float]:
    alloc = node.get("status", {}).get("allocatable") or node.get("status", {}).get("capacity") or {}
    return {k: parse_quantity(v) for k, v in alloc.items()}


def node_address(node: Obj) -> str:
    """First address of a node (reference utils/utils.go:66 `Status.Addresses[0].Address`)."""
    addrs = node.get("status", {}).get("addresses") or []
    return addrs[0].get("address", "") if addrs else ""


def node_taints(node: Obj) -> List[Obj]:
    return node.get("spec", {}).get("taints") or []


def node_ready(node: Obj) -> bool:
    for c in node.get("status", {}).get("conditions") or []:
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return True


def node_unschedulable(node: Obj) -> bool:
    return bool(node.get("spec", {}).get("unschedulable"))


def node_gpu_count(node: Obj) -> int:
    lab = labels(node)
    if C.LABEL_GPU_COUNT in lab:
        try:
            return int(lab[C.LABEL_GPU_COUNT])
        except ValueError:
            pass
    alloc = node_allocatable(node)
    parts = node_partitions_per_gpu(node)
    return int(alloc.get(C.RESOURCE_GPU, 0)) // max(parts, 1)


def node_partitions_per_gpu(node: Obj) -> int:
    mode = labels(node).get(C.LABEL_COMPUTE_PARTITION, "SPX")
    return C.COMPUTE_PARTITIONS.get(mode.upper(), 1)


def node_gpu_model(node: Obj, parity_names: bool = False) -> str:
    """GPU model of a node.  Fixed mode: from the node label.  Parity mode:
    from the node *name* like the reference (gpu_plugins.go:478-499: "a30" -> A30,
    "gpu" -> V100, else "")."""
    nm = name(node)
    if parity_names:
        if "a30" in nm:
            return "A30"
        if "gpu" in nm:
            return "V100"
        return ""
    lab = labels(node).get(C.LABEL_GPU_PRODUCT, "")
    if lab:
        return "MI355X" if "355" in lab else lab
    if "a30" in nm:
        return "A30"
    if "gpu" in nm:
        return "V100"
    return ""


def tolerates(pod: Obj, taint: Obj) -> bool:
    for t in pod.get("spec", {}).get("tolerations") or []:
        op = t.get("operator", "Equal")
        if t.get("effect") and t.get("effect") != taint.get("effect"):
            continue
        if op == "Exists":
            if not t.get("key") or t.get("key") == taint.get("key"):
                return True
        elif t.get("key") == taint.get("key") and t.get("value", "") == taint.get("value", ""):
            return True
    return False
