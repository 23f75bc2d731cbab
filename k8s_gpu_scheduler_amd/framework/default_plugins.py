"""In-tree plugins of kube-scheduler v1.21 (the reference's scheduler binary, reference
cmd/scheduler/main.go:15-28, go.mod k8s.io/kubernetes v1.21.0).

The reference's profile only *adds* GPU at score/postBind (reference
deploy/scheduler.yaml:16-23), so the upstream defaults stay on; `default_registry` holds
every in-tree plugin of that release so a KubeSchedulerConfiguration written for it (e.g.
NodeResourcesMostAllocated or RequestedToCapacityRatio for bin-packing) loads unchanged.
This module has the node filters, resource fit and the resource-allocation scorers; the rest
live in placement_plugins, score_plugins, volume_plugins, spread_plugins, preemption and
coscheduling.
"""
from __future__ import annotations

import json
import math
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
        args = args or {}
        self.ignored = set(args.get("ignoredResources", []))
        # ignoredResourceGroups: every extended resource of these prefixes ("example.com" of
        # "example.com/foo") is left to other plugins
        self.ignored_groups = set(args.get("ignoredResourceGroups", []))
        self._memo: Dict[str, tuple] = {}      # node -> (generation, node object, request sig, status)

    def _ignored(self, r: str) -> bool:
        return r in self.ignored or (bool(self.ignored_groups) and "/" in r and r.split("/", 1)[0] in self.ignored_groups)

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
            if v <= 0 or self._ignored(r):
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
        return tuple(sorted((r, v) for r, v in req.items() if v > 0 and not self._ignored(r)))

    def filter_nodes(self, state, pod, node_infos):
        req = state.read(_FIT_KEY)
        if req is None:
            req = O.pod_requests(pod)
        want = [(r, v - 1e-9, r.startswith(("amd.com/", "nvidia.com/"))) for r, v in req.items()
                if v > 0 and not self._ignored(r)]
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
    """Shared body of the resource-allocation Score plugins (upstream noderesources
    resource_allocation.go, v1.21): per configured resource an (allocatable, requested) pair --
    cpu and memory charge every pod's non-zero request (O.pod_nonzero_requests: an unset
    request counts as 100m / 200 MiB), other resources their plain requests, an extended
    resource the node lacks (0, 0) -- in integer units (milli-CPU, bytes), then the plugin's
    scorer.  `resources` args: [{name, weight}] (default cpu 1, memory 1)."""
    DEFAULT_RES = ((C.RESOURCE_CPU, 1), (C.RESOURCE_MEMORY, 1))

    def __init__(self, args=None, handle=None):
        self.handle = handle
        self._memo = {}
        res = (args or {}).get("resources")
        self.res = tuple((r["name"], int(r.get("weight") or 1)) for r in res) if res else self.DEFAULT_RES
        if any(w <= 0 for _, w in self.res):
            raise ValueError(f"{self.NAME}: resource weights must be positive")
        self._other = tuple(r for r, _ in self.res if r not in (C.RESOURCE_CPU, C.RESOURCE_MEMORY))

    def _request_sig(self, pod) -> tuple:
        nz = O.pod_nonzero_requests(pod)
        if not self._other:
            return nz
        req = O.pod_requests(pod)
        return nz + tuple(req.get(r, 0.0) for r in self._other)

    def _pairs(self, ni, rq: tuple):
        """[(allocatable, requested)] per configured resource, node + incoming pod."""
        out = []
        if ni is None or ni.node is None:
            return [(0, 0)] * len(self.res)
        alloc = ni.allocatable
        k = 2
        for r, _ in self.res:
            if r == C.RESOURCE_CPU:
                out.append((int(round(alloc.get(r, 0.0) * 1000)), ni.non_zero[0] + rq[0]))
            elif r == C.RESOURCE_MEMORY:
                out.append((int(alloc.get(r, 0.0)), ni.non_zero[1] + rq[1]))
            else:
                v = rq[k]
                k += 1
                if r in alloc or r == C.RESOURCE_EPHEMERAL_STORAGE:
                    out.append((int(alloc.get(r, 0.0)), int(ni.requested.get(r, 0.0) + v)))
                else:
                    out.append((0, 0))
        return out

    def score(self, state, pod, node_name):
        v, _ = self.score_nodes(state, pod, [node_name])
        return v[0], None

    def cache_signature(self, state, pod, phase):
        return self._request_sig(pod)

    def score_nodes(self, state, pod, names):
        # a node's score only changes with its NodeInfo generation and the request
        snap = self.handle.snapshot()
        rq = self._request_sig(pod)
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
            v = self._score(self._pairs(ni, rq))
            memo[nn] = (key, v)
            out.append(v)
        return out, None

    def _weighted(self, pairs, per) -> int:
        tot = wsum = 0
        for (cap, req), (_, w) in zip(pairs, self.res):
            tot += per(req, cap) * w
            wsum += w
        return tot // wsum if wsum else 0


def _least_requested(req: int, cap: int) -> int:
    if cap == 0 or req > cap:
        return 0
    return (cap - req) * C.MAX_NODE_SCORE // cap


def _most_requested(req: int, cap: int) -> int:
    if cap == 0 or req > cap:
        return 0
    return req * C.MAX_NODE_SCORE // cap


class NodeResourcesLeastAllocated(_ResourceScore):
    """(capacity - requested) / capacity per resource, weighted mean: spreads load."""
    NAME = "NodeResourcesLeastAllocated"

    def _score(self, pairs):
        return self._weighted(pairs, _least_requested)


class NodeResourcesMostAllocated(_ResourceScore):
    """requested / capacity per resource, weighted mean: bin-packs (upstream v1.21
    most_allocated.go)."""
    NAME = "NodeResourcesMostAllocated"

    def _score(self, pairs):
        return self._weighted(pairs, _most_requested)


class NodeResourcesBalancedAllocation(_ResourceScore):
    """100 x (1 - |cpu fraction - memory fraction|) (upstream v1.21 balanced_allocation.go;
    fractions of a zero capacity count as 1 and are capped at 1)."""
    NAME = "NodeResourcesBalancedAllocation"

    def __init__(self, args=None, handle=None):
        super().__init__(None, handle)          # always cpu + memory

    def _score(self, pairs):
        fr = [1.0 if cap == 0 else min(1.0, req / cap) for cap, req in pairs]
        return int((1 - abs(fr[0] - fr[1])) * C.MAX_NODE_SCORE)


class RequestedToCapacityRatio(_ResourceScore):
    """A broken-linear function of each resource's utilisation (args `shape`:
    [{utilization 0..100, score 0..10}], strictly increasing utilisation), weighted over the
    resources whose score is positive, rounded (upstream v1.21 requested_to_capacity_ratio.go)."""
    NAME = "RequestedToCapacityRatio"
    MAX_UTILIZATION = 100
    MAX_CUSTOM_SCORE = 10

    def __init__(self, args=None, handle=None):
        super().__init__(args, handle)
        shape = (args or {}).get("shape") or []
        if not shape:
            raise ValueError("RequestedToCapacityRatio: shape must not be empty")
        pts = []
        for p in shape:
            u, sc = int(p.get("utilization", 0)), int(p.get("score", 0))
            if not 0 <= u <= self.MAX_UTILIZATION:
                raise ValueError(f"RequestedToCapacityRatio: utilization {u} outside 0..100")
            if not 0 <= sc <= self.MAX_CUSTOM_SCORE:
                raise ValueError(f"RequestedToCapacityRatio: score {sc} outside 0..10")
            if pts and u <= pts[-1][0]:
                raise ValueError("RequestedToCapacityRatio: utilization values must be strictly increasing")
            pts.append((u, sc * (C.MAX_NODE_SCORE // self.MAX_CUSTOM_SCORE)))
        self.shape = tuple(pts)

    def _raw(self, p: int) -> int:
        s = self.shape
        for i, (u, sc) in enumerate(s):
            if p <= u:
                if i == 0:
                    return s[0][1]
                u0, s0 = s[i - 1]
                return s0 + _go_div((sc - s0) * (p - u0), u - u0)
        return s[-1][1]

    def _resource(self, req: int, cap: int) -> int:
        m = self.MAX_UTILIZATION
        if cap == 0 or req > cap:
            return self._raw(m)
        return self._raw(m - (cap - req) * m // cap)

    def _score(self, pairs):
        tot = wsum = 0
        for (cap, req), (_, w) in zip(pairs, self.res):
            v = self._resource(req, cap)
            if v > 0:
                tot += v * w
                wsum += w
        return int(round_half_away(tot / wsum)) if wsum else 0


def _go_div(a: int, b: int) -> int:
    """Go's integer division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def round_half_away(x: float) -> float:
    """Go's math.Round (half away from zero)."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


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
    from .spread_plugins import NodeLabel, SelectorSpread, ServiceAffinity
    from .volume_plugins import (AzureDiskLimits, CinderLimits, EBSLimits, GCEPDLimits, NodeVolumeLimits, VolumeBinding,
                                 VolumeRestrictions, VolumeZone)
    r = Registry()
    for cls in (PrioritySort, NodeUnschedulable, NodeName, TaintToleration, NodeAffinity, NodeResourcesFit,
                NodeResourcesLeastAllocated, NodeResourcesMostAllocated, NodeResourcesBalancedAllocation,
                RequestedToCapacityRatio, DefaultBinder, DefaultPreemption,
                NodePorts, InterPodAffinity, PodTopologySpread, Coscheduling, ImageLocality, NodePreferAvoidPods,
                VolumeBinding, VolumeRestrictions, VolumeZone, NodeVolumeLimits,
                EBSLimits, GCEPDLimits, AzureDiskLimits, CinderLimits, SelectorSpread, ServiceAffinity, NodeLabel):
        r.register(cls.NAME, lambda args, handle, cls=cls: cls(args, handle))
    return r
