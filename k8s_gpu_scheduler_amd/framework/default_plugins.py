"""In-tree default plugins the reference profile keeps enabled.

The reference's profile only *adds* GPU at score/postBind (reference
deploy/scheduler.yaml:16-23), so upstream defaults (queue sort, node filters,
resource fit, default binder) stay on.  These are the subset that matters for GPU pods.
"""
from __future__ import annotations

import json
from typing import Any, Dict

from ..api import constants as C
from ..api import objects as O
from .score_plugins import NodeAffinityScore, TaintTolerationScore, node_selector_term_matches
from .interface import BindPlugin, FilterPlugin, PreFilterPlugin, QueueSortPlugin, ScorePlugin, Status
from .runtime import Registry

Obj = Dict[str, Any]


def _canon(x: Any) -> str:
    """Hashable canonical form of a pod-spec fragment (cycle-cache signatures)."""
    return json.dumps(x, sort_keys=True, separators=(",", ":")) if x else ""


# Every filter/score plugin below implements cache_signature(state, pod, phase): what its
# per-node verdict depends on besides the node's own NodeInfo (framework.fastpath).


class PrioritySort(QueueSortPlugin):
    NAME = "PrioritySort"

    def __init__(self, args=None, handle=None):
        pass

    def less(self, a, b) -> bool:
        pa, pb = O.priority(a.pod), O.priority(b.pod)
        if pa != pb:
            return pa > pb
        return a.timestamp < b.timestamp

    def sort_key(self, pi) -> tuple:
        """Total-order key of `less` (priority is immutable; a requeue re-pushes)."""
        return -O.priority(pi.pod), pi.timestamp


class NodeUnschedulable(FilterPlugin):
    NAME = "NodeUnschedulable"

    def __init__(self, args=None, handle=None):
        # node name -> node object last seen schedulable and ready (objects are replaced,
        # never mutated, on update, so identity means "unchanged")
        self._plain: Dict[str, Any] = {}

    def filter(self, state, pod, node_info):
        node = node_info.node
        if O.node_unschedulable(node):
            t = {"key": "node.kubernetes.io/unschedulable", "effect": "NoSchedule"}
            if not O.tolerates(pod, t):
                return Status.unschedulable("node(s) were unschedulable", self.NAME, True)
        if not O.node_ready(node):
            return Status.unschedulable("node(s) were not ready", self.NAME, True)
        return None

    def cache_signature(self, state, pod, phase):
        return O.tolerates(pod, {"key": "node.kubernetes.io/unschedulable", "effect": "NoSchedule"})

    def filter_nodes(self, state, pod, node_infos):
        tol = None
        out = []
        plain = self._plain
        for ni in node_infos:
            node = ni.node
            if plain.get(ni.name) is node:          # schedulable and ready, node unchanged
                out.append(None)
                continue
            if not O.node_unschedulable(node) and O.node_ready(node):
                plain[ni.name] = node
                out.append(None)
                continue
            plain.pop(ni.name, None)
            if O.node_unschedulable(node):
                if tol is None:
                    tol = O.tolerates(pod, {"key": "node.kubernetes.io/unschedulable", "effect": "NoSchedule"})
                if not tol:
                    out.append(Status.unschedulable("node(s) were unschedulable", self.NAME, True))
                    continue
            out.append(None if O.node_ready(node) else
                       Status.unschedulable("node(s) were not ready", self.NAME, True))
        return out


class NodeName(FilterPlugin):
    NAME = "NodeName"

    def __init__(self, args=None, handle=None):
        pass

    def filter(self, state, pod, node_info):
        want = pod.get("spec", {}).get("nodeName")
        if want and want != node_info.name:
            return Status.unschedulable("node(s) didn't match the requested node name", self.NAME, True)
        return None

    def cache_signature(self, state, pod, phase):
        return pod.get("spec", {}).get("nodeName") or ""

    def filter_nodes(self, state, pod, node_infos):
        want = pod.get("spec", {}).get("nodeName")
        if not want:
            return [None] * len(node_infos)
        return [None if ni.name == want else self.filter(state, pod, ni) for ni in node_infos]


class TaintToleration(FilterPlugin, TaintTolerationScore):
    """Filter: NoSchedule / NoExecute taints must be tolerated.  Score (score_plugins): fewer
    intolerable PreferNoSchedule taints rank higher."""
    NAME = "TaintToleration"

    def __init__(self, args=None, handle=None):
        self._tt_init(handle)

    def filter(self, state, pod, node_info):
        for t in O.node_taints(node_info.node):
            if t.get("effect") not in ("NoSchedule", "NoExecute"):
                continue
            if not O.tolerates(pod, t):
                return Status.unschedulable(f"node(s) had untolerated taint {{{t.get('key')}: {t.get('value', '')}}}",
                                            self.NAME, True)
        return None

    def cache_signature(self, state, pod, phase):
        return _canon(pod.get("spec", {}).get("tolerations"))

    def filter_nodes(self, state, pod, node_infos):
        # untainted nodes (the common case) need no per-node work
        return [self.filter(state, pod, ni) if O.node_taints(ni.node) else None for ni in node_infos]


class NodeAffinity(FilterPlugin, NodeAffinityScore):
    """Filter: nodeSelector and required node-selector terms (matchExpressions incl. Gt/Lt,
    matchFields on metadata.name; terms ORed).  Score (score_plugins): preferred terms."""
    NAME = "NodeAffinity"

    def __init__(self, args=None, handle=None):
        self._na_init(handle)

    def filter(self, state, pod, node_info):
        sel = pod.get("spec", {}).get("nodeSelector") or {}
        lab = O.labels(node_info.node)
        for k, v in sel.items():
            if lab.get(k) != v:
                return Status.unschedulable("node(s) didn't match Pod's node affinity/selector", self.NAME, True)
        aff = (pod.get("spec", {}).get("affinity") or {}).get("nodeAffinity") or {}
        req = aff.get("requiredDuringSchedulingIgnoredDuringExecution") or {}
        terms = req.get("nodeSelectorTerms") or []
        if terms and not any(node_selector_term_matches(node_info.node, t) for t in terms):
            return Status.unschedulable("node(s) didn't match Pod's node affinity/selector", self.NAME, True)
        return None

    def cache_signature(self, state, pod, phase):
        spec = pod.get("spec", {})
        return (_canon(spec.get("nodeSelector")), _canon((spec.get("affinity") or {}).get("nodeAffinity")))

    def filter_nodes(self, state, pod, node_infos):
        spec = pod.get("spec", {})
        if not spec.get("nodeSelector") and not ((spec.get("affinity") or {}).get("nodeAffinity")):
            return [None] * len(node_infos)
        return [self.filter(state, pod, ni) for ni in node_infos]


_FIT_KEY = "NodeResourcesFit/req"


class NodeResourcesFit(PreFilterPlugin, FilterPlugin):
    NAME = "NodeResourcesFit"

    def __init__(self, args=None, handle=None):
        self.ignored = set((args or {}).get("ignoredResources", []))
        self._memo: Dict[str, tuple] = {}      # node -> (generation, node object, request sig, status)

    def pre_filter(self, state, pod):
        state.write(_FIT_KEY, O.pod_requests(pod))
        return None

    def filter(self, state, pod, node_info):
        req = state.read(_FIT_KEY)
        if req is None:
            req = O.pod_requests(pod)
        if node_info.free(C.RESOURCE_PODS) < 1 and C.RESOURCE_PODS in node_info.allocatable:
            return Status.unschedulable("Too many pods", self.NAME)
        for r, v in req.items():
            if v <= 0 or r in self.ignored:
                continue
            if r not in node_info.allocatable and r.startswith(("amd.com/", "nvidia.com/")):
                return Status.unschedulable(f"Insufficient {r}", self.NAME)
            if r in node_info.allocatable and node_info.free(r) < v - 1e-9:
                return Status.unschedulable(f"Insufficient {r}", self.NAME)
        return None

    def cache_signature(self, state, pod, phase):
        req = state.read(_FIT_KEY)
        if req is None:
            req = O.pod_requests(pod)
        return tuple(sorted((r, v) for r, v in req.items() if v > 0 and r not in self.ignored))

    def filter_nodes(self, state, pod, node_infos):
        req = state.read(_FIT_KEY)
        if req is None:
            req = O.pod_requests(pod)
        want = [(r, v - 1e-9, r.startswith(("amd.com/", "nvidia.com/"))) for r, v in req.items()
                if v > 0 and r not in self.ignored]
        sig = tuple(want)
        pods_key = C.RESOURCE_PODS
        memo = self._memo
        out = []
        for ni in node_infos:
            # a node's verdict only changes with its NodeInfo generation / object and the
            # request; preemption what-if clones (pods removed, own generation count) bypass it
            whatif = getattr(ni, "removed", None) is not None
            hit = None if whatif else memo.get(ni.name)
            if hit is not None and hit[0] == ni.generation and hit[1] is ni.node and hit[2] == sig:
                out.append(hit[3])
                continue
            alloc, used = ni.allocatable, ni.requested
            st = None
            if pods_key in alloc and alloc[pods_key] - used.get(pods_key, 0.0) < 1:
                st = Status.unschedulable("Too many pods", self.NAME)
            else:
                for r, v, ext in want:
                    a = alloc.get(r)
                    if a is None:
                        if ext:
                            st = Status.unschedulable(f"Insufficient {r}", self.NAME)
                            break
                    elif a - used.get(r, 0.0) < v:
                        st = Status.unschedulable(f"Insufficient {r}", self.NAME)
                        break
            if not whatif:
                memo[ni.name] = (ni.generation, ni.node, sig, st)
            out.append(st)
        return out


class _ResourceScore(ScorePlugin):
    RES = (C.RESOURCE_CPU, C.RESOURCE_MEMORY)

    def __init__(self, args=None, handle=None):
        self.handle = handle
        self._memo = {}

    def score(self, state, pod, node_name):
        # a node's score only changes with its NodeInfo generation and the request
        ni = self.handle.snapshot().get(node_name)
        req = O.pod_requests(pod)
        key = (ni.generation if ni else -1, id(ni.node) if ni else 0) + tuple(req.get(r, 0.0) for r in self.RES)
        hit = self._memo.get(node_name)
        if hit is not None and hit[0] == key:
            return hit[1], None
        v = self._score(self._fractions(pod, node_name, ni, req))
        if len(self._memo) > 100000:
            self._memo.clear()
        self._memo[node_name] = (key, v)
        return v, None

    def cache_signature(self, state, pod, phase):
        req = O.pod_requests(pod)
        return tuple(req.get(r, 0.0) for r in self.RES)

    def score_nodes(self, state, pod, names):
        snap = self.handle.snapshot()
        req = O.pod_requests(pod)
        rq = tuple(req.get(r, 0.0) for r in self.RES)
        memo = self._memo
        if len(memo) > 100000:
            memo.clear()
        out = []
        for nn in names:
            ni = snap.get(nn)
            key = (ni.generation if ni else -1, id(ni.node) if ni else 0) + rq
            hit = memo.get(nn)
            if hit is not None and hit[0] == key:
                out.append(hit[1])
                continue
            v = self._score(self._fractions(pod, nn, ni, req))
            memo[nn] = (key, v)
            out.append(v)
        return out, None

    def _fractions(self, pod, node_name, ni=None, req=None):
        if ni is None:
            ni = self.handle.snapshot().get(node_name)
        if req is None:
            req = O.pod_requests(pod)
        fr = []
        for r in self.RES:
            alloc = ni.allocatable.get(r, 0.0) if ni else 0.0
            if alloc <= 0:
                continue
            fr.append(min(1.0, (ni.requested.get(r, 0.0) + req.get(r, 0.0)) / alloc))
        return fr


class NodeResourcesLeastAllocated(_ResourceScore):
    NAME = "NodeResourcesLeastAllocated"

    def _score(self, fr):
        if not fr:
            return 0
        return int(sum((1 - f) * C.MAX_NODE_SCORE for f in fr) / len(fr))


class NodeResourcesBalancedAllocation(_ResourceScore):
    NAME = "NodeResourcesBalancedAllocation"

    def _score(self, fr):
        if len(fr) < 2:
            return C.MAX_NODE_SCORE
        mean = sum(fr) / len(fr)
        var = sum((f - mean) ** 2 for f in fr) / len(fr)
        return int((1 - var ** 0.5) * C.MAX_NODE_SCORE)


class DefaultBinder(BindPlugin):
    NAME = "DefaultBinder"

    def __init__(self, args=None, handle=None):
        self.handle = handle

    def bind(self, state, pod, node_name):
        try:
            ann = state.read("bind/annotations")
            self.handle.client.bind(O.namespace(pod), O.name(pod), node_name, O.uid(pod), annotations=ann)
        except Exception as e:
            return Status.error(f"binding rejected: {e}", self.NAME)
        return None


def default_registry() -> Registry:
    from .placement_plugins import InterPodAffinity, NodePorts, PodTopologySpread
    from .coscheduling import Coscheduling
    from .preemption import DefaultPreemption
    from .score_plugins import ImageLocality, NodePreferAvoidPods
    from .volume_plugins import NodeVolumeLimits, VolumeBinding, VolumeRestrictions, VolumeZone
    r = Registry()
    for cls in (PrioritySort, NodeUnschedulable, NodeName, TaintToleration, NodeAffinity, NodeResourcesFit,
                NodeResourcesLeastAllocated, NodeResourcesBalancedAllocation, DefaultBinder, DefaultPreemption,
                NodePorts, InterPodAffinity, PodTopologySpread, Coscheduling, ImageLocality, NodePreferAvoidPods,
                VolumeBinding, VolumeRestrictions, VolumeZone, NodeVolumeLimits):
        r.register(cls.NAME, lambda args, handle, cls=cls: cls(args, handle))
    return r
