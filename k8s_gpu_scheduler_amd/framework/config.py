"""KubeSchedulerConfiguration loader.

Parses the same YAML shape the reference deploys (reference deploy/scheduler.yaml:7-23:
`kubescheduler.config.k8s.io/v1beta1`, leaderElection, profiles[].plugins.<point>
.enabled/disabled with weights) plus typed `pluginConfig[].args`, which is where every
constant the reference hard-codes becomes configurable.
Accepts v1beta1/v1beta2/v1beta3/v1 -- the plugin-set semantics are identical for what
this framework implements (enabled lists are appended to the defaults, `disabled: '*'`
clears them).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

from ..api import constants as C

DEFAULT_PLUGINS: Dict[str, List[Dict[str, Any]]] = {
    "queueSort": [{"name": "PrioritySort"}],
    "preFilter": [{"name": "NodeResourcesFit"}, {"name": "NodePorts"}, {"name": "InterPodAffinity"},
                  {"name": "PodTopologySpread"}, {"name": "VolumeBinding"}, {"name": "VolumeRestrictions"},
                  {"name": "VolumeZone"}, {"name": "EBSLimits"}, {"name": "GCEPDLimits"},
                  {"name": "NodeVolumeLimits"}, {"name": "AzureDiskLimits"}],
    "filter": [{"name": "NodeUnschedulable"}, {"name": "NodeName"}, {"name": "TaintToleration"},
               {"name": "NodeAffinity"}, {"name": "NodePorts"}, {"name": "NodeResourcesFit"},
               {"name": "VolumeRestrictions"}, {"name": "EBSLimits"}, {"name": "GCEPDLimits"},
               {"name": "NodeVolumeLimits"}, {"name": "AzureDiskLimits"}, {"name": "VolumeBinding"},
               {"name": "VolumeZone"}, {"name": "InterPodAffinity"}, {"name": "PodTopologySpread"}],
    "postFilter": [{"name": "DefaultPreemption"}],
    # upstream v1.21 defaults (pkg/scheduler/algorithmprovider/registry.go); NodeAffinity,
    # ImageLocality and NodePreferAvoidPods also PreScore here, only to skip themselves
    # when they cannot change the ranking
    "preScore": [{"name": "InterPodAffinity"}, {"name": "PodTopologySpread"}, {"name": "TaintToleration"},
                 {"name": "NodeAffinity"}, {"name": "ImageLocality"}, {"name": "NodePreferAvoidPods"}],
    "score": [{"name": "NodeResourcesBalancedAllocation", "weight": 1}, {"name": "ImageLocality", "weight": 1},
              {"name": "InterPodAffinity", "weight": 1}, {"name": "NodeResourcesLeastAllocated", "weight": 1},
              {"name": "NodeAffinity", "weight": 1}, {"name": "NodePreferAvoidPods", "weight": 10000},
              {"name": "PodTopologySpread", "weight": 2}, {"name": "TaintToleration", "weight": 1}],
    "reserve": [{"name": "VolumeBinding"}],
    "permit": [],
    "preBind": [{"name": "VolumeBinding"}],
    "bind": [{"name": "DefaultBinder"}],
    "postBind": [],
}
POINTS = list(DEFAULT_PLUGINS)
SUPPORTED_API = {"kubescheduler.config.k8s.io/v1beta1", "kubescheduler.config.k8s.io/v1beta2",
                 "kubescheduler.config.k8s.io/v1beta3", "kubescheduler.config.k8s.io/v1"}


@dataclass
class PluginRef:
    name: str
    weight: int = 1


@dataclass
class Profile:
    scheduler_name: str = "default-scheduler"
    plugins: Dict[str, List[PluginRef]] = field(default_factory=dict)
    plugin_config: Dict[str, Dict[str, Any]] = field(default_factory=dict)

    def enabled(self, point: str) -> List[PluginRef]:
        return self.plugins.get(point, [])

    def args(self, plugin: str) -> Dict[str, Any]:
        return self.plugin_config.get(plugin, {})


@dataclass
class LeaderElection:
    leader_elect: bool = False
    resource_name: str = "kube-scheduler"
    resource_namespace: str = "kube-system"
    lease_duration_s: float = 15.0
    renew_deadline_s: float = 10.0
    retry_period_s: float = 2.0


@dataclass
class ExtenderConfig:
    """One `extenders[]` entry (kube-scheduler's HTTP scheduler extenders, called by this
    scheduler -- framework.extender_client)."""
    url_prefix: str
    filter_verb: str = ""
    prioritize_verb: str = ""
    bind_verb: str = ""
    preempt_verb: str = ""
    weight: int = 1
    enable_https: bool = False
    tls_insecure: bool = False
    tls_ca_file: str = ""
    http_timeout_s: float = 30.0
    node_cache_capable: bool = False
    managed_resources: List[Dict[str, Any]] = field(default_factory=list)
    ignorable: bool = False


@dataclass
class SchedulerConfig:
    profiles: List[Profile] = field(default_factory=list)
    leader_election: LeaderElection = field(default_factory=LeaderElection)
    parallelism: int = 16
    percentage_of_nodes_to_score: int = 0
    pod_initial_backoff_s: float = 1.0
    pod_max_backoff_s: float = 10.0
    extenders: List[ExtenderConfig] = field(default_factory=list)

    def profile(self, scheduler_name: str) -> Optional[Profile]:
        for p in self.profiles:
            if p.scheduler_name == scheduler_name:
                return p
        return None


def _merge_point(point: str, spec: Optional[Dict[str, Any]]) -> List[PluginRef]:
    base = copy.deepcopy(DEFAULT_PLUGINS[point])
    spec = spec or {}
    disabled = {d.get("name") for d in spec.get("disabled") or []}
    if "*" in disabled:
        base = []
    else:
        base = [b for b in base if b["name"] not in disabled]
    out = [PluginRef(b["name"], int(b.get("weight", 1) or 1)) for b in base]
    for e in spec.get("enabled") or []:
        nm = e.get("name")
        w = int(e.get("weight", 1) or 1)
        existing = [r for r in out if r.name == nm]
        if existing:
            existing[0].weight = w
        else:
            out.append(PluginRef(nm, w))
    if point == "queueSort" and len(out) > 1:
        out = out[-1:]
    if point == "bind" and len(out) > 1:
        # a custom binder listed in enabled runs before DefaultBinder; keep both (first
        # non-Skip wins) like upstream.
        pass
    return out


def parse_config(doc: Dict[str, Any]) -> SchedulerConfig:
    api = doc.get("apiVersion", "kubescheduler.config.k8s.io/v1beta1")
    if api not in SUPPORTED_API:
        raise ValueError(f"unsupported apiVersion {api}")
    if doc.get("kind", "KubeSchedulerConfiguration") != "KubeSchedulerConfiguration":
        raise ValueError("kind must be KubeSchedulerConfiguration")
    le = doc.get("leaderElection") or {}

    def dur(v: Any, d: float) -> float:
        if v is None:
            return d
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return float(v) / 1e9              # a bare metav1.Duration number is nanoseconds
        s = str(v)
        if s.endswith("ms"):
            return float(s[:-2]) / 1000
        if s.endswith("s"):
            return float(s[:-1])
        if s.endswith("m"):
            return float(s[:-1]) * 60
        return float(s)

    cfg = SchedulerConfig(
        leader_election=LeaderElection(
            leader_elect=bool(le.get("leaderElect", False)),
            resource_name=le.get("resourceName", "kube-scheduler"),
            resource_namespace=le.get("resourceNamespace", "kube-system"),
            lease_duration_s=dur(le.get("leaseDuration"), 15.0),
            renew_deadline_s=dur(le.get("renewDeadline"), 10.0),
            retry_period_s=dur(le.get("retryPeriod"), 2.0)),
        parallelism=int(doc.get("parallelism", 16)),
        percentage_of_nodes_to_score=int(doc.get("percentageOfNodesToScore", 0) or 0),
        pod_initial_backoff_s=float(doc.get("podInitialBackoffSeconds", 1)),
        pod_max_backoff_s=float(doc.get("podMaxBackoffSeconds", 10)),
    )
    profs = doc.get("profiles") or [{"schedulerName": "default-scheduler"}]
    for p in profs:
        plugins = p.get("plugins") or {}
        prof = Profile(scheduler_name=p.get("schedulerName", "default-scheduler"))
        multi = plugins.get("multiPoint")
        for point in POINTS:
            spec = plugins.get(point)
            if multi:
                spec = copy.deepcopy(spec or {})
                spec.setdefault("enabled", [])
                spec["enabled"] = list(multi.get("enabled") or []) + spec["enabled"]
            prof.plugins[point] = _merge_point(point, spec)
        for pc in p.get("pluginConfig") or []:
            prof.plugin_config[pc["name"]] = dict(pc.get("args") or {})
        cfg.profiles.append(prof)
    ignored_ext: List[str] = []
    for e in doc.get("extenders") or []:
        if not e.get("urlPrefix"):
            raise ValueError("extenders[].urlPrefix is required")
        w = int(e.get("weight", 1) if e.get("weight") is not None else 1)
        if e.get("prioritizeVerb") and w <= 0:
            raise ValueError("extenders[].weight must be positive with a prioritizeVerb")
        tls = e.get("tlsConfig") or {}
        managed = list(e.get("managedResources") or [])
        ignored_ext += [m["name"] for m in managed if m.get("ignoredByScheduler")]
        cfg.extenders.append(ExtenderConfig(
            url_prefix=e["urlPrefix"], filter_verb=e.get("filterVerb", ""), prioritize_verb=e.get("prioritizeVerb", ""),
            bind_verb=e.get("bindVerb", ""), preempt_verb=e.get("preemptVerb", ""), weight=w,
            enable_https=bool(e.get("enableHTTPS", False)), tls_insecure=bool(tls.get("insecure", False)),
            tls_ca_file=tls.get("caFile", ""), http_timeout_s=dur(e.get("httpTimeout"), 30.0),
            node_cache_capable=bool(e.get("nodeCacheCapable", False)), managed_resources=managed,
            ignorable=bool(e.get("ignorable", False))))
    if sum(1 for x in cfg.extenders if x.bind_verb) > 1:
        raise ValueError("only one extender can implement bind")
    if ignored_ext:         # resources an extender manages are not NodeResourcesFit's to check
        for prof in cfg.profiles:
            fit = prof.plugin_config.setdefault("NodeResourcesFit", {})
            fit["ignoredResources"] = sorted(set(fit.get("ignoredResources") or []) | set(ignored_ext))
    return cfg


def load_config(path_or_text: str) -> SchedulerConfig:
    """Load from a file path, a YAML string, or a ConfigMap manifest that embeds the
    config under data["scheduler-config.yaml"] (reference deploy/scheduler.yaml:1-23)."""
    text = path_or_text
    if "\n" not in path_or_text:
        with open(path_or_text) as f:
            text = f.read()
    for doc in yaml.safe_load_all(text):
        if not doc:
            continue
        if doc.get("kind") == "ConfigMap":
            for v in (doc.get("data") or {}).values():
                inner = yaml.safe_load(v)
                if isinstance(inner, dict) and inner.get("kind") == "KubeSchedulerConfiguration":
                    return parse_config(inner)
            continue
        if doc.get("kind") == "KubeSchedulerConfiguration":
            return parse_config(doc)
    raise ValueError("no KubeSchedulerConfiguration found")


def default_gpu_config(gpu_args: Optional[Dict[str, Any]] = None, disable_defaults: bool = False,
                       queue_sort: bool = False) -> SchedulerConfig:
    """The deployed profile: GPU at score (weight 10100) + every extension point the
    fixed-mode plugin implements (filter/reserve/preBind/postBind); `queue_sort` also makes
    GPU the queueSort plugin (longest predicted work first within an arrival window)."""
    score: Dict[str, Any] = {"enabled": [{"name": C.PLUGIN_NAME, "weight": C.DEFAULT_SCORE_WEIGHT}]}
    pre_score: Dict[str, Any] = {"enabled": [{"name": C.PLUGIN_NAME}]}
    if disable_defaults:
        score["disabled"] = [{"name": "*"}]
        pre_score["disabled"] = [{"name": "*"}]      # their Score halves are off too
    doc = {
        "apiVersion": "kubescheduler.config.k8s.io/v1beta1",
        "kind": "KubeSchedulerConfiguration",
        "leaderElection": {"leaderElect": False},
        "profiles": [{
            "schedulerName": C.SCHEDULER_NAME,
            "plugins": {
                **({"queueSort": {"enabled": [{"name": C.PLUGIN_NAME}]}} if queue_sort else {}),
                "preFilter": {"enabled": [{"name": C.PLUGIN_NAME}]},
                "filter": {"enabled": [{"name": C.PLUGIN_NAME}]},
                "preScore": pre_score,
                "score": score,
                "reserve": {"enabled": [{"name": C.PLUGIN_NAME}]},
                "preBind": {"enabled": [{"name": C.PLUGIN_NAME}]},
                "postBind": {"enabled": [{"name": C.PLUGIN_NAME}]},
            },
            "pluginConfig": [{"name": C.PLUGIN_NAME, "args": dict(gpu_args or {})}],
        }],
    }
    return parse_config(doc)
