"""kube-scheduler v1.21 plugins that read a pod's workload owners -- the Services selecting it
and its controlling ReplicationController / ReplicaSet / StatefulSet:

  SelectorSpread   Score: pods of the same Services / controller already on the node;
                   normalised so the emptiest node scores 100, blended 2:1 with the same
                   count per zone (region + zone labels) when nodes carry zones (upstream
                   selectorspread/selector_spread.go; not in the v1.21 default profile, where
                   PodTopologySpread's system defaults cover it, but registered and
                   configurable).  Pods with topologySpreadConstraints are left alone.
  ServiceAffinity  Filter (`affinityLabels`): a pod joins the label values of the node its
                   Service's first scheduled pod landed on (unless its nodeSelector already
                   fixes them).  Score (`antiAffinityLabelsPreference`): spread a Service's
                   pods over the values of each label (upstream serviceaffinity).
  NodeLabel        Filter: `presentLabels` must all exist on the node, `absentLabels` none.
                   Score: share of `presentLabelsPreference` present and
                   `absentLabelsPreference` absent (upstream nodelabel).

`default_selector` (upstream helper.DefaultSelector) also gives PodTopologySpread its system
default constraints (score_plugins.PodTopologySpreadScore).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from ..api import objects as O
from ..kube.patch import match_label_selector
from .interface import (MAX_NODE_SCORE, FilterPlugin, NodeScore, PreFilterPlugin, PreScorePlugin, ScoreExtensions,
                        ScorePlugin, Status)

Obj = Dict[str, Any]
ZONE_WEIGHTING = 2.0 / 3.0
_REGION = ("topology.kubernetes.io/region", "failure-domain.beta.kubernetes.io/region")
_ZONE = ("topology.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/zone")


def zone_key(node: Optional[Obj]) -> str:
    """upstream utilnode.GetZoneKey: "region:\\x00:zone", "" when the node has neither."""
    lab = O.labels(node) if node else {}
    region = next((lab[k] for k in _REGION if lab.get(k)), "")
    zone = next((lab[k] for k in _ZONE if lab.get(k)), "")
    if not region and not zone:
        return ""
    return f"{region}:\x00:{zone}"


class Owners:
    """Listers of the workload objects (informers when the scheduler has a factory, else
    direct client lists)."""

    def __init__(self, handle: Any):
        self.handle = handle
        self._inf: Dict[str, Any] = {}
        f = getattr(handle, "informer_factory", None) if handle is not None else None
        if f is not None:
            try:
                self._inf = {"services": f.services(), "replicationcontrollers": f.replication_controllers(),
                             "replicasets": f.replica_sets(), "statefulsets": f.stateful_sets()}
            except AttributeError:
                self._inf = {}

    def list(self, resource: str, namespace: str) -> List[Obj]:
        inf = self._inf.get(resource)
        if inf is not None:
            return [o for o in inf.lister.list() if O.namespace(o) == namespace]
        try:
            return self.handle.client.list(resource, namespace)[0]
        except Exception:
            return []

    def get(self, resource: str, name: str, namespace: str) -> Optional[Obj]:
        inf = self._inf.get(resource)
        if inf is not None:
            return inf.lister.get(name, namespace)
        try:
            return self.handle.client.get(resource, name, namespace)
        except Exception:
            return None

    def pod_services(self, pod: Obj) -> List[Obj]:
        """Services in the pod's namespace whose (non-empty) selector selects it."""
        lab = O.labels(pod)
        out = []
        for svc in self.list("services", O.namespace(pod)):
            sel = (svc.get("spec") or {}).get("selector") or {}
            if sel and all(lab.get(k) == v for k, v in sel.items()):
                out.append(svc)
        return out


def _controller(pod: Obj) -> Optional[Obj]:
    for ref in O.meta(pod).get("ownerReferences") or []:
        if ref.get("controller"):
            return ref
    return None


def default_selector(pod: Obj, owners: Owners) -> List[Obj]:
    """The label selectors (all must match) of the pod's Services and controller: the
    Services' and a ReplicationController's selectors merged into one matchLabels, a
    ReplicaSet's / StatefulSet's LabelSelector added as is.  [] = empty selector."""
    merged: Dict[str, str] = {}
    for svc in owners.pod_services(pod):
        merged.update((svc.get("spec") or {}).get("selector") or {})
    extra: List[Obj] = []
    ref = _controller(pod)
    if ref is not None:
        kind, api = ref.get("kind"), ref.get("apiVersion", "")
        ns = O.namespace(pod)
        if kind == "ReplicationController" and api in ("v1", ""):
            rc = owners.get("replicationcontrollers", ref.get("name", ""), ns)
            if rc is not None:
                merged.update((rc.get("spec") or {}).get("selector") or {})
        elif kind in ("ReplicaSet", "StatefulSet") and api.startswith("apps/"):
            obj = owners.get("replicasets" if kind == "ReplicaSet" else "statefulsets", ref.get("name", ""), ns)
            sel = ((obj or {}).get("spec") or {}).get("selector")
            if sel and (sel.get("matchLabels") or sel.get("matchExpressions")):
                extra.append(sel)
    out = [{"matchLabels": merged}] if merged else []
    return out + extra


def selector_matches(selectors: List[Obj], labels: Dict[str, str]) -> bool:
    return bool(selectors) and all(match_label_selector(labels, s) for s in selectors)


def count_matching(pod_ns: str, selectors: List[Obj], node_pods) -> int:
    if not selectors:
        return 0
    return sum(1 for o in node_pods if O.namespace(o) == pod_ns and not O.meta(o).get("deletionTimestamp")
               and selector_matches(selectors, O.labels(o)))


# ---------------------------------------------------------------------------- SelectorSpread
class _SelectorSpreadNormalize(ScoreExtensions):
    NORMALIZE = "selector_spread"

    def __init__(self, plugin: "SelectorSpread"):
        self.plugin = plugin

    def normalize_score(self, state, pod, scores: List[NodeScore]) -> Optional[Status]:
        snap = self.plugin.handle.snapshot()
        by_zone: Dict[str, int] = {}
        zones: Dict[str, str] = {}
        max_node = 0
        for s in scores:
            max_node = max(max_node, s.score)
            ni = snap.get(s.name)
            z = zone_key(ni.node if ni else None)
            zones[s.name] = z
            if z:
                by_zone[z] = by_zone.get(z, 0) + s.score
        max_zone = max(by_zone.values(), default=0)
        for s in scores:
            f = float(MAX_NODE_SCORE)
            if max_node > 0:
                f = MAX_NODE_SCORE * ((max_node - s.score) / max_node)
            z = zones[s.name]
            if by_zone and z:
                zs = float(MAX_NODE_SCORE)
                if max_zone > 0:
                    zs = MAX_NODE_SCORE * ((max_zone - by_zone[z]) / max_zone)
                f = f * (1.0 - ZONE_WEIGHTING) + ZONE_WEIGHTING * zs
            s.score = int(f)
        return None


class SelectorSpread(PreScorePlugin, ScorePlugin):
    NAME = "SelectorSpread"
    _KEY = "SelectorSpread/selector"

    def __init__(self, args=None, handle=None):
        self.handle = handle
        self.owners = Owners(handle)
        self._norm = _SelectorSpreadNormalize(self)

    def pre_score(self, state, pod, nodes):
        if (pod.get("spec") or {}).get("topologySpreadConstraints"):
            return Status.skip()
        sel = default_selector(pod, self.owners)
        if not sel:                 # nothing to spread against: every node would score 100
            return Status.skip()
        state.write(self._KEY, sel)
        return None

    def score(self, state, pod, node_name):
        sel = state.read(self._KEY)
        ni = self.handle.snapshot().get(node_name)
        if not sel or ni is None:
            return 0, None
        return count_matching(O.namespace(pod), sel, ni.pods.values()), None

    def score_extensions(self):
        return self._norm


# ---------------------------------------------------------------------------- ServiceAffinity
class _ServiceAntiAffinityNormalize(ScoreExtensions):
    NORMALIZE = "service_anti_affinity"

    def __init__(self, plugin: "ServiceAffinity"):
        self.plugin = plugin

    def normalize_score(self, state, pod, scores: List[NodeScore]) -> Optional[Status]:
        labels = self.plugin.anti_labels
        if not labels:
            return None
        snap = self.plugin.handle.snapshot()
        out = [0.0] * len(scores)
        for label in labels:
            total = 0
            counts: Dict[str, int] = {}
            value_of: Dict[str, str] = {}
            for s in scores:
                total += s.score
                ni = snap.get(s.name)
                lab = O.labels(ni.node) if ni and ni.node else {}
                if label not in lab:
                    continue
                value_of[s.name] = lab[label]
                counts[lab[label]] = counts.get(lab[label], 0) + s.score
            for i, s in enumerate(scores):
                v = value_of.get(s.name)
                if v is None:
                    continue
                f = float(MAX_NODE_SCORE)
                if total > 0:
                    f = MAX_NODE_SCORE * ((total - counts[v]) / total)
                out[i] += f / len(labels)
        for i, s in enumerate(scores):
            s.score = int(out[i])
        return None


class ServiceAffinity(PreFilterPlugin, FilterPlugin, ScorePlugin):
    NAME = "ServiceAffinity"
    _KEY = "ServiceAffinity/state"

    def __init__(self, args=None, handle=None):
        args = args or {}
        self.handle = handle
        self.owners = Owners(handle)
        self.affinity_labels: List[str] = list(args.get("affinityLabels") or [])
        self.anti_labels: List[str] = list(args.get("antiAffinityLabelsPreference") or [])
        self._norm = _ServiceAntiAffinityNormalize(self)

    def pre_filter(self, state, pod):
        if not self.affinity_labels:
            return Status.skip()
        services = self.owners.pod_services(pod)
        lab = O.labels(pod)
        ns = O.namespace(pod)
        matching: List[Obj] = []    # scheduled pods carrying all of the pod's labels (no labels: all)
        for ni in self.handle.snapshot().list():
            for o in ni.pods.values():
                olab = O.labels(o)
                if O.namespace(o) == ns and all(olab.get(k) == v for k, v in lab.items()):
                    matching.append(o)
        state.write(self._KEY, (services, matching))
        return None

    def filter(self, state, pod, node_info):
        st = state.read(self._KEY)
        if st is None:
            return None
        services, matching = st
        want = {k: v for k, v in ((pod.get("spec") or {}).get("nodeSelector") or {}).items()
                if k in self.affinity_labels}
        if len(want) < len(self.affinity_labels) and services:
            # NodeInfo.FilterOutPods: a pod on this node counts only while this NodeInfo still
            # holds it (preemption what-ifs remove victims)
            others = [o for o in matching
                      if (o.get("spec") or {}).get("nodeName") != node_info.name or O.key(o) in node_info.pods]
            first = next((o for o in others if (o.get("spec") or {}).get("nodeName")), None)
            if first is not None:
                ni = self.handle.snapshot().get(first["spec"]["nodeName"])
                nlab = O.labels(ni.node) if ni and ni.node else {}
                for k in self.affinity_labels:
                    if k not in want and k in nlab:
                        want[k] = nlab[k]
        nlab = O.labels(node_info.node)
        if all(nlab.get(k) == v for k, v in want.items()):
            return None
        return Status.unschedulable("node(s) didn't match service affinity", self.NAME)

    def score(self, state, pod, node_name):
        if not self.anti_labels:
            return 0, None
        services = self.owners.pod_services(pod)
        ni = self.handle.snapshot().get(node_name)
        if not services or ni is None:
            return 0, None
        sel = [{"matchLabels": (services[0].get("spec") or {}).get("selector") or {}}]
        return count_matching(O.namespace(pod), sel, ni.pods.values()), None

    def score_extensions(self):
        return self._norm


# ---------------------------------------------------------------------------- NodeLabel
class NodeLabel(FilterPlugin, ScorePlugin):
    NAME = "NodeLabel"

    def __init__(self, args=None, handle=None):
        args = args or {}
        self.present: List[str] = list(args.get("presentLabels") or [])
        self.absent: List[str] = list(args.get("absentLabels") or [])
        self.present_pref: List[str] = list(args.get("presentLabelsPreference") or [])
        self.absent_pref: List[str] = list(args.get("absentLabelsPreference") or [])
        for a, b, what in ((self.present, self.absent, "presentLabels/absentLabels"),
                           (self.present_pref, self.absent_pref, "presentLabelsPreference/absentLabelsPreference")):
            if set(a) & set(b):
                raise ValueError(f"NodeLabel: {what} share labels {sorted(set(a) & set(b))}")
        self.handle = handle

    def filter(self, state, pod, node_info):
        lab = O.labels(node_info.node)
        if all(k in lab for k in self.present) and not any(k in lab for k in self.absent):
            return None
        return Status.unschedulable("node(s) didn't have the requested labels", self.NAME, True)

    def cache_signature(self, state, pod, phase):
        return ()                   # node-local, pod-independent

    def score(self, state, pod, node_name):
        n = len(self.present_pref) + len(self.absent_pref)
        if n == 0:
            return 0, None
        ni = self.handle.snapshot().get(node_name)
        lab = O.labels(ni.node) if ni and ni.node else {}
        s = sum(MAX_NODE_SCORE for k in self.present_pref if k in lab) + \
            sum(MAX_NODE_SCORE for k in self.absent_pref if k not in lab)
        return s // n, None
