"""kube-scheduler default filters beyond resources: NodePorts, InterPodAffinity (required
terms) and PodTopologySpread (DoNotSchedule constraints).

The reference inherits these from upstream kube-scheduler (its binary is the stock scheduler
plus the GPU plugin, reference cmd/scheduler/main.go:15-28), so a user switching over keeps
hostPort conflicts, pod (anti-)affinity and topology spreading working.  Semantics follow
upstream for the required/hard forms; the soft (preferred / ScheduleAnyway) forms are
accepted and ignored by Filter, as upstream also treats them only at Score.

Topology domains are node-label values (`topologyKey`); "existing pods" are the pods the
scheduler's cache has placed or assumed (the same view upstream uses).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

from ..api import objects as O
from ..kube.patch import match_label_selector
from .interface import FilterPlugin, PreFilterPlugin, Status
from .score_plugins import InterPodAffinityScore, PodTopologySpreadScore, _has_affinity

Obj = Dict[str, Any]


def _host_ports(pod: Obj) -> List[Tuple[str, str, int]]:
    out = []
    for c in O.containers(pod):
        for p in c.get("ports") or []:
            hp = int(p.get("hostPort") or 0)
            if hp:
                out.append((p.get("hostIP") or "0.0.0.0", (p.get("protocol") or "TCP").upper(), hp))
    return out


class NodePorts(PreFilterPlugin, FilterPlugin):
    NAME = "NodePorts"
    _KEY = "NodePorts/wanted"

    def __init__(self, args=None, handle=None):
        pass

    def pre_filter(self, state, pod):
        ports = _host_ports(pod)
        if not ports:
            return Status.skip()
        state.write(self._KEY, ports)
        return None

    def cache_signature(self, state, pod, phase):
        # the verdict depends on the node's own pods only (framework.fastpath)
        return tuple(sorted(state.read(self._KEY) or _host_ports(pod)))

    def filter(self, state, pod, node_info):
        wanted = state.read(self._KEY) or _host_ports(pod)
        if not wanted:
            return None
        used = [hp for p in node_info.pods.values() for hp in _host_ports(p)]
        for ip, proto, port in wanted:
            for uip, uproto, uport in used:
                if port == uport and proto == uproto and (ip == uip or "0.0.0.0" in (ip, uip)):
                    return Status.unschedulable("node(s) didn't have free ports for the requested pod ports",
                                                self.NAME)
        return None


def _domain(node: Optional[Obj], key: str) -> Optional[str]:
    return O.labels(node).get(key) if node is not None else None


def _term_matches(term: Obj, pod: Obj, other: Obj) -> bool:
    nss = term.get("namespaces") or [O.namespace(pod)]
    return O.namespace(other) in nss and match_label_selector(O.labels(other), term.get("labelSelector") or {})


class InterPodAffinity(PreFilterPlugin, FilterPlugin, InterPodAffinityScore):
    """Required pod affinity / anti-affinity (requiredDuringSchedulingIgnoredDuringExecution),
    including existing pods' anti-affinity against the incoming pod (symmetry).  PreFilter
    turns every term into the set of topology domains it allows or forbids, once per cycle;
    pods that carry anti-affinity terms are indexed from the informer, so a cluster where no
    pod uses (anti-)affinity pays nothing (Filter is skipped)."""
    NAME = "InterPodAffinity"
    _KEY = "InterPodAffinity/state"

    def __init__(self, args=None, handle=None):
        self.handle = handle
        self._anti: Dict[str, Obj] = {}         # assigned pods with required anti-affinity
        self._with_aff: Dict[str, Obj] = {}     # assigned pods with any pod (anti-)affinity (Score)
        if handle is not None:
            try:
                inf = handle.informer_factory.pods()
                inf.add_event_handler(self._on_pod, lambda o, n: self._on_pod(n), self._on_delete)
            except AttributeError:
                pass

    def _on_pod(self, pod: Obj) -> None:
        live = bool(O.node_name_of(pod)) and not O.is_terminal(pod)
        if live and self._terms(pod, "podAntiAffinity"):
            self._anti[O.key(pod)] = pod
        else:
            self._anti.pop(O.key(pod), None)
        if live and _has_affinity(pod):
            self._with_aff[O.key(pod)] = pod
        else:
            self._with_aff.pop(O.key(pod), None)

    def _on_delete(self, pod: Obj) -> None:
        self._anti.pop(O.key(pod), None)
        self._with_aff.pop(O.key(pod), None)

    @staticmethod
    def _terms(pod: Obj, kind: str) -> List[Obj]:
        aff = ((pod.get("spec") or {}).get("affinity") or {}).get(kind) or {}
        return list(aff.get("requiredDuringSchedulingIgnoredDuringExecution") or [])

    def pre_filter(self, state, pod):
        aff, anti = self._terms(pod, "podAffinity"), self._terms(pod, "podAntiAffinity")
        if not aff and not anti and not self._anti:
            return Status.skip()
        snap = self.handle.snapshot()
        node_of = {ni.name: ni.node for ni in snap.list()}
        forbidden: List[Tuple[str, str]] = []       # (topologyKey, value) the pod may not join
        for other in self._anti.values():
            for t in self._terms(other, "podAntiAffinity"):
                key = t.get("topologyKey", "")
                dom = _domain(node_of.get(O.node_name_of(other)), key)
                if dom is not None and _term_matches(t, other, pod):
                    forbidden.append((key, dom))
        placed = [(ni.node, o) for ni in snap.list() for o in ni.pods.values()] if (aff or anti) else []
        for t in anti:
            key = t.get("topologyKey", "")
            for node, o in placed:
                dom = _domain(node, key)
                if dom is not None and _term_matches(t, pod, o):
                    forbidden.append((key, dom))
        required: List[Tuple[str, Optional[set]]] = []   # per affinity term: allowed domains (None = any)
        for t in aff:
            key = t.get("topologyKey", "")
            doms = {_domain(node, key) for node, o in placed if _term_matches(t, pod, o)}
            doms.discard(None)
            if not doms and _term_matches(t, pod, pod):
                required.append((key, None))     # first pod of its own group: anywhere
            else:
                required.append((key, doms))
        if not forbidden and not required:
            return Status.skip()
        state.write(self._KEY, (set(forbidden), required))
        return None

    def filter(self, state, pod, node_info):
        st = state.read(self._KEY)
        if st is None:
            return None
        forbidden, required = st
        lab = O.labels(node_info.node)
        for key, dom in forbidden:
            if lab.get(key) == dom:
                return Status.unschedulable("node(s) didn't match pod anti-affinity rules", self.NAME)
        for key, doms in required:
            if key not in lab or (doms is not None and lab[key] not in doms):
                return Status.unschedulable("node(s) didn't match pod affinity rules", self.NAME)
        return None


class PodTopologySpread(PreFilterPlugin, FilterPlugin, PodTopologySpreadScore):
    """topologySpreadConstraints with whenUnsatisfiable: DoNotSchedule -- placing the pod in
    this node's domain must keep (count in domain + 1) - (min over domains) <= maxSkew.
    Domain counts are built once per cycle in PreFilter.  ScheduleAnyway constraints are
    scored (score_plugins.PodTopologySpreadScore).  Pods without constraints get the
    default constraints (args defaultingType System | List, defaultConstraints) over the
    selectors of their Services and controller (spread_plugins.default_selector)."""
    NAME = "PodTopologySpread"
    _KEY = "PodTopologySpread/counts"

    # upstream v1.21 system defaults (defaultingType: System), applied to pods without
    # constraints that a Service / ReplicationController / ReplicaSet / StatefulSet selects
    SYSTEM_DEFAULT_CONSTRAINTS = (
        {"maxSkew": 3, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "ScheduleAnyway"},
        {"maxSkew": 5, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "ScheduleAnyway"})

    def __init__(self, args=None, handle=None):
        from .spread_plugins import Owners
        args = args or {}
        self.handle = handle
        dt = args.get("defaultingType", "System")
        given = list(args.get("defaultConstraints") or [])
        if dt == "System":
            if given:
                raise ValueError("PodTopologySpread: defaultConstraints need defaultingType: List")
            self.default_constraints = list(self.SYSTEM_DEFAULT_CONSTRAINTS)
        elif dt == "List":
            if any(c.get("labelSelector") for c in given):
                raise ValueError("PodTopologySpread: defaultConstraints must not set labelSelector")
            self.default_constraints = given
        else:
            raise ValueError(f"PodTopologySpread: unknown defaultingType {dt!r}")
        self._owners = Owners(handle) if self.default_constraints else None

    def spread_constraints(self, pod, mode: str):
        """([(topologyKey, maxSkew, [label selectors])], explicit) of the pod's constraints with
        whenUnsatisfiable == mode -- or, when the pod declares none, the default constraints
        with the selectors of its Services / controller (none when nothing selects it)."""
        spec_cons = (pod.get("spec") or {}).get("topologySpreadConstraints") or []
        if spec_cons:
            return [(c.get("topologyKey", ""), int(c.get("maxSkew", 1)), [c.get("labelSelector") or {}])
                    for c in spec_cons if c.get("whenUnsatisfiable", "DoNotSchedule") == mode], True
        defs = [c for c in self.default_constraints if c.get("whenUnsatisfiable", "DoNotSchedule") == mode]
        if not defs or self._owners is None:
            return [], False
        from .spread_plugins import default_selector
        sels = default_selector(pod, self._owners)
        if not sels:
            return [], False
        return [(c.get("topologyKey", ""), int(c.get("maxSkew", 1)), sels) for c in defs], False

    def pre_filter(self, state, pod):
        cons, _ = self.spread_constraints(pod, "DoNotSchedule")
        if not cons:
            return Status.skip()
        snap = self.handle.snapshot()
        out = []
        ns = O.namespace(pod)
        for key, max_skew, sels in cons:
            counts: Dict[str, int] = {}
            for ni in snap.list():
                d = _domain(ni.node, key)
                if d is None:
                    continue
                counts[d] = counts.get(d, 0) + sum(
                    1 for o in ni.pods.values()
                    if O.namespace(o) == ns and all(match_label_selector(O.labels(o), sl) for sl in sels))
            out.append((key, max_skew, counts, min(counts.values()) if counts else 0))
        state.write(self._KEY, out)
        return None

    def filter(self, state, pod, node_info):
        for key, max_skew, counts, lowest in state.read(self._KEY) or []:
            dom = _domain(node_info.node, key)
            if dom is None:
                return Status.unschedulable("node(s) didn't match pod topology spread constraints (missing required label)",
                                            self.NAME, True)
            if counts.get(dom, 0) + 1 - lowest > max_skew:
                return Status.unschedulable("node(s) didn't match pod topology spread constraints", self.NAME)
        return None
