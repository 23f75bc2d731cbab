"""HTTP scheduler extenders called BY this scheduler (kube-scheduler's `extenders:` config).

framework.extender serves the extender protocol so a stock kube-scheduler can drive this
framework; this module is the other direction: a cluster that already runs extenders
(device-sharing, licence or quota extenders next to kube-scheduler v1.21, the reference's
scheduler) keeps them when it switches to this scheduler.  Semantics follow upstream
core/extender.go + generic_scheduler.go:

  * an extender is interested in a pod when it manages none of the pod's resources list
    (`managedResources` empty) or the pod requests / limits one of them;
  * Filter (after the filter plugins, in config order): the feasible nodes go out as
    ExtenderArgs{Pod, Nodes{items}} or {Pod, NodeNames} (`nodeCacheCapable`); the nodes
    that come back stay feasible, FailedNodes / FailedAndUnresolvableNodes add their reason
    to the pod's failure message;
  * Prioritize: HostPriority scores 0..10 (MaxExtenderPriority) are added to the plugin
    total as score x weight x 10; a failing prioritize call is skipped (upstream logs it);
  * Bind: the (single) extender with a bindVerb that is interested binds the pod instead
    of the bind plugins (PreBind still runs first);
  * a failing extender fails the cycle unless `ignorable`, in which case it is skipped.
  The preemption verb is not called (preemption runs the framework's own victim search).
"""
from __future__ import annotations

import json
import ssl
import urllib.error
import urllib.request
from typing import Any, Dict, List, Optional, Tuple

from ..api import objects as O
from .config import ExtenderConfig

Obj = Dict[str, Any]
MAX_EXTENDER_PRIORITY = 10


class ExtenderError(RuntimeError):
    pass


class HTTPExtender:
    def __init__(self, cfg: ExtenderConfig):
        self.cfg = cfg
        prefix = cfg.url_prefix.rstrip("/")
        if cfg.enable_https and prefix.startswith("http://"):
            prefix = "https://" + prefix[len("http://"):]
        elif "://" not in prefix:
            prefix = ("https://" if cfg.enable_https else "http://") + prefix
        self.prefix = prefix
        self._ctx: Optional[ssl.SSLContext] = None
        if prefix.startswith("https://"):
            ctx = ssl.create_default_context(cafile=cfg.tls_ca_file or None)
            if cfg.tls_insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            self._ctx = ctx
        self._managed = {m.get("name") for m in cfg.managed_resources if m.get("name")}

    @property
    def name(self) -> str:
        return self.prefix

    @property
    def is_ignorable(self) -> bool:
        return self.cfg.ignorable

    @property
    def is_binder(self) -> bool:
        return bool(self.cfg.bind_verb)

    def is_interested(self, pod: Obj) -> bool:
        if not self._managed:
            return True
        spec = pod.get("spec") or {}
        for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
            res = c.get("resources") or {}
            for kind in ("requests", "limits"):
                if self._managed & set((res.get(kind) or {}).keys()):
                    return True
        return False

    def _post(self, verb: str, body: Obj) -> Any:
        req = urllib.request.Request(f"{self.prefix}/{verb}", data=json.dumps(body).encode(), method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.cfg.http_timeout_s, context=self._ctx) as r:
                return json.loads(r.read() or b"null")
        except (urllib.error.URLError, OSError, ValueError) as e:
            raise ExtenderError(f"extender {self.prefix}/{verb}: {e}") from e

    def _args(self, pod: Obj, nodes: List[Any]) -> Obj:
        if self.cfg.node_cache_capable:
            return {"Pod": pod, "NodeNames": [ni.name for ni in nodes]}
        return {"Pod": pod, "Nodes": {"items": [ni.node for ni in nodes]}}

    def filter(self, pod: Obj, nodes: List[Any]) -> Tuple[List[Any], Dict[str, str], Dict[str, str]]:
        """(nodes kept, failed {node: reason}, failed-and-unresolvable {node: reason})."""
        if not self.cfg.filter_verb:
            return nodes, {}, {}
        out = self._post(self.cfg.filter_verb, self._args(pod, nodes)) or {}
        if out.get("Error"):
            raise ExtenderError(f"extender {self.prefix}: {out['Error']}")
        if self.cfg.node_cache_capable and out.get("NodeNames") is not None:
            keep = set(out.get("NodeNames") or [])
        else:
            keep = {O.name(n) for n in ((out.get("Nodes") or {}).get("items") or [])}
        return ([ni for ni in nodes if ni.name in keep], dict(out.get("FailedNodes") or {}),
                dict(out.get("FailedAndUnresolvableNodes") or {}))

    def prioritize(self, pod: Obj, nodes: List[Any]) -> Dict[str, int]:
        if not self.cfg.prioritize_verb:
            return {}
        out = self._post(self.cfg.prioritize_verb, self._args(pod, nodes)) or []
        return {h.get("Host", ""): int(h.get("Score", 0)) for h in out}

    def bind(self, pod: Obj, node: str) -> None:
        out = self._post(self.cfg.bind_verb, {"PodName": O.name(pod), "PodNamespace": O.namespace(pod),
                                              "PodUID": O.uid(pod), "Node": node}) or {}
        if out.get("Error"):
            raise ExtenderError(f"extender {self.prefix} bind: {out['Error']}")
