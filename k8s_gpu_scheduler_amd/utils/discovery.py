"""Service discovery helpers.

The reference resolves every service (Redis, recommender, Prometheus) by finding a pod
whose *name contains* a substring in a namespace and taking its node's first address
(reference utils/utils.go:24-70); all lookups go to a fixed NodePort
(SURVEY.md §1 "Service discovery").  The same functions exist here, plus an explicit
`Endpoints` config that skips discovery entirely (env / plugin args), which is what the
fixed mode uses by default.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from ..api import constants as C
from ..api import objects as O
from ..kube.client import KubeClient
from ..kube.resources import Resources

Obj = Dict[str, Any]


def check(err: Optional[BaseException]) -> None:
    """reference utils/utils.go:18-22 (panic on error) -- here: raise."""
    if err is not None:
        raise err


def exists(items: List[str], s: str) -> int:
    """Index of the first element that CONTAINS `s` (substring, as the reference,
    utils/utils.go:101-108), -1 if none."""
    for i, el in enumerate(items):
        if s in el:
            return i
    return -1


def remove(items: List[str], index: int) -> List[str]:
    return items[:index] + items[index + 1:]


def get_env(pod: Obj, env_name: str) -> str:
    return O.get_env(pod, env_name)


def find_node_from_pod(res: Resources, pod_name_contains: str,
                       pod_list: Optional[List[Obj]] = None,
                       parity_master: Optional[str] = None) -> List[Obj]:
    if pod_list is None:
        pod_list = res.list_pods()
    nodes = []
    for pod in pod_list:
        if pod_name_contains in O.name(pod):
            n = res.get_node(O.node_name_of(pod), parity_master)
            if n is not None:
                nodes.append(n)
    return nodes


def find_nodes_ip_from_pod(res: Resources, pod_name_contains: str,
                           pod_list: Optional[List[Obj]] = None,
                           parity_master: Optional[str] = None) -> List[Dict[str, str]]:
    """[{nodeName: firstAddress}] for nodes hosting pods whose name contains the substring."""
    return [{O.name(n): O.node_address(n)} for n in
            find_node_from_pod(res, pod_name_contains, pod_list, parity_master)]


def get_nodes_exporter_pod(res: Resources, node_name: str, pod_list: Optional[List[Obj]] = None,
                           substr: str = C.EXPORTER_POD_SUBSTR) -> str:
    """First pod on the node whose name contains `substr` (reference utils/utils.go:72-99
    looks for "dcgm"; ours is the AMD exporter)."""
    if pod_list is None:
        pod_list = [p for p in res.list_pods(all_namespaces=True) if O.node_name_of(p) == node_name]
    for p in pod_list:
        if substr in O.name(p):
            return O.name(p)
    return ""


@dataclass
class Endpoints:
    """Resolved service addresses.  `from_env()` reads GPU_SCHED_{REDIS,RECOMMENDER,PROMETHEUS}_ADDR."""
    redis: str = ""
    recommender: str = ""
    prometheus: str = ""
    redis_password: str = C.REDIS_PASSWORD
    extra: Dict[str, str] = field(default_factory=dict)

    @classmethod
    def from_env(cls) -> "Endpoints":
        return cls(redis=os.getenv("GPU_SCHED_REDIS_ADDR", ""),
                   recommender=os.getenv("GPU_SCHED_RECOMMENDER_ADDR", ""),
                   prometheus=os.getenv("GPU_SCHED_PROMETHEUS_ADDR", ""),
                   redis_password=os.getenv("GPU_SCHED_REDIS_PASSWORD", C.REDIS_PASSWORD))

    def discover(self, client: KubeClient, parity_master: Optional[str] = None) -> "Endpoints":
        """Fill unset addresses by the reference's pod-substring discovery."""
        def first_ip(ns: str, substr: str) -> str:
            res = Resources(client, ns)
            ips = find_nodes_ip_from_pod(res, substr, parity_master=parity_master)
            return next(iter(ips[0].values())) if ips else ""
        if not self.redis:
            ip = first_ip(C.REDIS_NAMESPACE, C.REDIS_POD_SUBSTR)
            self.redis = f"{ip}:{C.REDIS_NODEPORT}" if ip else ""
        if not self.recommender:
            ip = first_ip(C.RECOMMENDER_NAMESPACE, C.RECOMMENDER_POD_SUBSTR)
            self.recommender = f"{ip}:{C.RECOMMENDER_NODEPORT}" if ip else ""
        if not self.prometheus:
            ip = first_ip(C.PROMETHEUS_NAMESPACE, C.PROMETHEUS_POD_SUBSTR)
            self.prometheus = f"http://{ip}:{C.PROMETHEUS_NODEPORT}/" if ip else ""
        return self
