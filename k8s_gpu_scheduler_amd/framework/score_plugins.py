"""kube-scheduler's default Score plugins beyond resource balance.

The reference's scheduler binary is the stock kube-scheduler v1.21 with the GPU plugin added
(reference cmd/scheduler/main.go:15-28, deploy/scheduler.yaml:15-23 keeps the default
plugins on), so a profile there also ranks nodes by: ImageLocality (weight 1),
InterPodAffinity (1), NodeAffinity (1, preferred terms), NodePreferAvoidPods (10000),
PodTopologySpread (2, ScheduleAnyway constraints) and TaintToleration (1, PreferNoSchedule).
This module holds the score halves of those plugins (the filter halves live in
default_plugins / placement_plugins) with the upstream formulas and normalisations:

  * TaintToleration  -- count of intolerable PreferNoSchedule taints, normalised reversed
                        (DefaultNormalizeScore(100, reverse=true));
  * NodeAffinity     -- sum of the weights of matching preferred node-selector terms,
                        DefaultNormalizeScore(100, reverse=false);
  * InterPodAffinity -- per topology domain: + weight of each preferred affinity term of the
                        incoming pod matching an existing pod there, - for anti-affinity, and
                        the symmetric terms of existing pods (their required affinity at
                        hardPodAffinityWeight = 1); min-max normalised;
  * PodTopologySpread -- per ScheduleAnyway constraint: matching pods in the node's domain x
                        log(#domains + 2) + maxSkew - 1, normalised so the emptiest domain
                        scores 100;
  * ImageLocality    -- sum over the pod's container images present on the node of
                        size x (nodes having it / all nodes), clamped to [23 MB, 1000 MB x
                        containers] and scaled to 0..100 (no normalisation);
  * NodePreferAvoidPods -- 0 on nodes whose scheduler.alpha.kubernetes.io/preferAvoidPods
                        annotation names the pod's ReplicaSet/ReplicationController, else 100.

Each plugin returns Skip at PreScore when it cannot change the ranking (no preferred terms,
no PreferNoSchedule taint anywhere, ...), so ordinary pods keep the cross-cycle node-result
cache (framework.fastpath); the node-local ones (ImageLocality, NodePreferAvoidPods) take
part in that cache through their signature.
"""
from __future__ import annotations

import json
import math
from typing import Any, Dict, List, Optional, Tuple

from ..api import constants as C
from ..api import objects as O
from ..kube.patch import match_label_selector
from .interface import MAX_NODE_SCORE, NodeScore, PreScorePlugin, ScoreExtensions, ScorePlugin, Status

Obj = Dict[str, Any]


# ---------------------------------------------------------------------------- node selectors
def _num(v: str) -> Optional[int]:
    try:
        return int(v)
    except (TypeError, ValueError):
        return None


def _requirement_matches(values: Dict[str, str], req: Obj) -> bool:
    key, op = req.get("key", ""), req.get("operator", "In")
    vals = [str(v) for v in req.get("values") or []]
    has = key in values
    v = values.get(key)
    if op == "In":
        return has and v in vals
    if op == "NotIn":
        return not has or v not in vals
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    if op in ("Gt", "Lt"):
        a, b = _num(v) if has else None, _num(vals[0]) if len(vals) == 1 else None
        if a is None or b is None:
            return False
        return a > b if op == "Gt" else a < b
    return False


def node_selector_term_matches(node: Optional[Obj], term: Obj) -> bool:
    """A NodeSelectorTerm (matchExpressions on labels AND matchFields on metadata.name); an
    empty term matches nothing (upstream nodeaffinity semantics)."""
    if node is None:
        return False
    exprs, fields = term.get("matchExpressions") or [], term.get("matchFields") or []
    if not exprs and not fields:
        return False
    lab = O.labels(node)
    if not all(_requirement_matches(lab, r) for r in exprs):
        return False
    fv = {"metadata.name": O.name(node)}
    return all(_requirement_matches(fv, r) for r in fields)


# ---------------------------------------------------------------------------- normalisers
class _DefaultNormalize(ScoreExtensions):
    """helper.DefaultNormalizeScore(MaxNodeScore, reverse, scores)."""

    def __init__(self, reverse: bool):
        self.reverse = reverse
        self.NORMALIZE = "default_reverse" if reverse else "default"

    def normalize_score(self, state, pod, scores: List[NodeScore]) -> Optional[Status]:
        hi = max((s.score for s in scores), default=0)
        if hi == 0:
            if self.reverse:
                for s in scores:
                    s.score = MAX_NODE_SCORE
            return None
        for s in scores:
            v = MAX_NODE_SCORE * s.score // hi
            s.score = MAX_NODE_SCORE - v if self.reverse else v
        return None


class _MinMaxNormalize(ScoreExtensions):
    """InterPodAffinity's normalisation: 100 * (s - min) / (max - min), all-equal -> 0."""
    NORMALIZE = "minmax"

    def normalize_score(self, state, pod, scores: List[NodeScore]) -> Optional[Status]:
        if not scores:
            return None
        lo, hi = min(s.score for s in scores), max(s.score for s in scores)
        for s in scores:
            s.score = (s.score - lo) * MAX_NODE_SCORE // (hi - lo) if hi > lo else 0
        return None


# ---------------------------------------------------------------------------- TaintToleration
class TaintTolerationScore(PreScorePlugin, ScorePlugin):
    """Mixin for default_plugins.TaintToleration (node-local: cacheable when active)."""
    _TT_KEY = "TaintToleration/preferNoSchedule"
    _tt_norm = _DefaultNormalize(reverse=True)

    def _tt_init(self, handle) -> None:
        """Tracks the nodes carrying a PreferNoSchedule taint from the node informer, so
        PreScore can skip in O(1) when there are none."""
        self._tt_handle = handle
        self._pns: set = set()
        if handle is not None:
            try:
                handle.informer_factory.nodes().add_event_handler(
                    self._tt_on_node, lambda o, n: self._tt_on_node(n), lambda n: self._pns.discard(O.name(n)))
            except AttributeError:
                pass

    def _tt_on_node(self, node: Obj) -> None:
        if any(t.get("effect") == "PreferNoSchedule" for t in O.node_taints(node)):
            self._pns.add(O.name(node))
        else:
            self._pns.discard(O.name(node))

    @staticmethod
    def _tt_tolerations(pod: Obj) -> List[Obj]:
        return [t for t in (pod.get("spec") or {}).get("tolerations") or []
                if t.get("effect") in (None, "", "PreferNoSchedule")]

    def pre_score(self, state, pod, nodes):
        if not self._pns:
            return Status.skip()            # every raw score 0 -> every node 100: ranking unchanged
        state.write(self._TT_KEY, self._tt_tolerations(pod))
        return None

    def score(self, state, pod, node_name):
        ni = self._tt_handle.snapshot().get(node_name)
        tols = state.read(self._TT_KEY)
        probe = {"spec": {"tolerations": self._tt_tolerations(pod) if tols is None else tols}}
        n = sum(1 for t in (O.node_taints(ni.node) if ni else [])
                if t.get("effect") == "PreferNoSchedule" and not O.tolerates(probe, t))
        return n, None

    def score_extensions(self):
        return self._tt_norm


# ---------------------------------------------------------------------------- NodeAffinity
class NodeAffinityScore(PreScorePlugin, ScorePlugin):
    """Mixin for default_plugins.NodeAffinity: preferredDuringSchedulingIgnoredDuringExecution."""
    _NA_KEY = "NodeAffinity/preferred"
    _na_norm = _DefaultNormalize(reverse=False)

    def _na_init(self, handle) -> None:
        self._na_handle = handle

    @staticmethod
    def _na_terms(pod: Obj) -> List[Obj]:
        aff = ((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}
        return [t for t in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []
                if int(t.get("weight", 0) or 0)]

    def pre_score(self, state, pod, nodes):
        terms = self._na_terms(pod)
        if not terms:
            return Status.skip()
        state.write(self._NA_KEY, terms)
        return None

    def score(self, state, pod, node_name):
        ni = self._na_handle.snapshot().get(node_name)
        node = ni.node if ni else None
        terms = state.read(self._NA_KEY)
        return sum(int(t.get("weight", 0)) for t in (self._na_terms(pod) if terms is None else terms)
                   if node_selector_term_matches(node, t.get("preference") or {})), None

    def score_extensions(self):
        return self._na_norm


# ---------------------------------------------------------------------------- InterPodAffinity
HARD_POD_AFFINITY_WEIGHT = 1


def _pref_terms(pod: Obj, kind: str) -> List[Tuple[int, Obj]]:
    aff = ((pod.get("spec") or {}).get("affinity") or {}).get(kind) or {}
    return [(int(w.get("weight", 0) or 0), w.get("podAffinityTerm") or {})
            for w in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []]


def _req_terms(pod: Obj, kind: str) -> List[Obj]:
    aff = ((pod.get("spec") or {}).get("affinity") or {}).get(kind) or {}
    return list(aff.get("requiredDuringSchedulingIgnoredDuringExecution") or [])


def _term_matches(term: Obj, owner: Obj, other: Obj) -> bool:
    nss = term.get("namespaces") or [O.namespace(owner)]
    return O.namespace(other) in nss and match_label_selector(O.labels(other), term.get("labelSelector") or {})


def _has_affinity(pod: Obj) -> bool:
    return bool(((pod.get("spec") or {}).get("affinity") or {}).get("podAffinity")
                or ((pod.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity"))


class InterPodAffinityScore(PreScorePlugin, ScorePlugin):
    """Mixin for placement_plugins.InterPodAffinity (scores depend on other nodes' pods:
    no cross-cycle cache while active)."""
    _IPA_KEY = "InterPodAffinity/topologyScore"
    _ipa_norm = _MinMaxNormalize()

    def pre_score(self, state, pod, nodes):
        pa, pn = _pref_terms(pod, "podAffinity"), _pref_terms(pod, "podAntiAffinity")
        indexed = getattr(self, "_with_aff", None)
        if not pa and not pn and not indexed:
            return Status.skip()
        snap = self.handle.snapshot()
        with_aff = []
        for o in (indexed or {}).values():
            ni = snap.get(O.node_name_of(o))
            if ni is not None:
                with_aff.append((ni.node, o))
        scores: Dict[Tuple[str, str], int] = {}

        def add(node, term, w):
            key = term.get("topologyKey", "")
            dom = O.labels(node).get(key) if node is not None else None
            if dom is not None and w:
                scores[(key, dom)] = scores.get((key, dom), 0) + w

        if pa or pn:
            for ni in snap.list():
                for o in ni.pods.values():
                    for w, t in pa:
                        if _term_matches(t, pod, o):
                            add(ni.node, t, w)
                    for w, t in pn:
                        if _term_matches(t, pod, o):
                            add(ni.node, t, -w)
        for node, o in with_aff:               # symmetry: existing pods' terms about the incoming pod
            for t in _req_terms(o, "podAffinity"):
                if _term_matches(t, o, pod):
                    add(node, t, HARD_POD_AFFINITY_WEIGHT)
            for w, t in _pref_terms(o, "podAffinity"):
                if _term_matches(t, o, pod):
                    add(node, t, w)
            for w, t in _pref_terms(o, "podAntiAffinity"):
                if _term_matches(t, o, pod):
                    add(node, t, -w)
        if not scores:
            return Status.skip()
        state.write(self._IPA_KEY, scores)
        return None

    def score(self, state, pod, node_name):
        scores = state.read(self._IPA_KEY) or {}
        ni = self.handle.snapshot().get(node_name)
        lab = O.labels(ni.node) if ni else {}
        return sum(v for (k, d), v in scores.items() if lab.get(k) == d), None

    def score_extensions(self):
        return self._ipa_norm


# ---------------------------------------------------------------------------- PodTopologySpread
class _SpreadNormalize(ScoreExtensions):
    NORMALIZE = "topology_spread"

    def normalize_score(self, state, pod, scores: List[NodeScore]) -> Optional[Status]:
        st = state.read(PodTopologySpreadScore._PTS_KEY)
        ignored = st[1] if st else set()
        vals = [s.score for s in scores if s.name not in ignored]
        lo, hi = (min(vals), max(vals)) if vals else (0, 0)
        for s in scores:
            if s.name in ignored:
                s.score = 0
            elif hi == 0:
                s.score = MAX_NODE_SCORE
            else:
                s.score = MAX_NODE_SCORE * (hi + lo - s.score) // hi
        return None


class PodTopologySpreadScore(PreScorePlugin, ScorePlugin):
    """Mixin for placement_plugins.PodTopologySpread: whenUnsatisfiable: ScheduleAnyway."""
    _PTS_KEY = "PodTopologySpread/scoreState"
    _pts_norm = _SpreadNormalize()

    def pre_score(self, state, pod, nodes):
        cons, require_all = self.spread_constraints(pod, "ScheduleAnyway")
        if not cons:
            return Status.skip()
        snap = self.handle.snapshot()
        infos = snap.list()
        cand = nodes if nodes else infos
        # explicit constraints: nodes lacking a topology key are ignored (score 0); the
        # defaulted ones (Service / controller spreading) just skip the missing keys
        ignored = {ni.name for ni in cand if any(key not in O.labels(ni.node) for key, _, _ in cons)} \
            if require_all else set()
        out = []
        ns = O.namespace(pod)
        for key, max_skew, sels in cons:
            domains = {O.labels(ni.node)[key] for ni in cand if ni.name not in ignored and key in O.labels(ni.node)}
            counts: Dict[str, int] = {}
            for ni in infos:
                d = O.labels(ni.node).get(key)
                if d is None or d not in domains:
                    continue
                counts[d] = counts.get(d, 0) + sum(1 for o in ni.pods.values()
                                                   if O.namespace(o) == ns
                                                   and all(match_label_selector(O.labels(o), sl) for sl in sels))
            weight = math.log(len(domains) + 2)
            out.append((key, max_skew, counts, weight))
        state.write(self._PTS_KEY, (out, ignored))
        return None

    def score(self, state, pod, node_name):
        st = state.read(self._PTS_KEY)
        if not st or node_name in st[1]:
            return 0, None
        ni = self.handle.snapshot().get(node_name)
        lab = O.labels(ni.node) if ni else {}
        s = 0.0
        for key, max_skew, counts, weight in st[0]:
            if key in lab:
                s += counts.get(lab[key], 0) * weight + (max_skew - 1)
        return int(round(s)), None

    def score_extensions(self):
        return self._pts_norm


# ---------------------------------------------------------------------------- ImageLocality
MB = 1024 * 1024
MIN_THRESHOLD = 23 * MB
MAX_CONTAINER_THRESHOLD = 1000 * MB


def normalized_image_name(name: str) -> str:
    """Append ':latest' when the image has no tag (upstream normalizedImageName)."""
    return name if name.rfind(":") > name.rfind("/") else name + ":latest"


class ImageLocality(PreScorePlugin, ScorePlugin):
    """Favours nodes that already hold the pod's container images (node.status.images),
    scaled by how widely each image is spread so one node does not attract every pod."""
    NAME = "ImageLocality"
    _KEY = "ImageLocality/images"

    def __init__(self, args=None, handle=None):
        self.handle = handle
        self._version = 0
        self._nodes: Dict[str, Tuple[Obj, Dict[str, int]]] = {}     # node -> (obj, image -> size)
        self._num_nodes: Dict[str, int] = {}
        if handle is not None:
            try:
                handle.informer_factory.nodes().add_event_handler(self._on_node, lambda o, n: self._on_node(n),
                                                                  self._on_node_delete)
            except AttributeError:
                pass

    def _images_of(self, node: Obj) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for im in ((node.get("status") or {}).get("images") or []):
            size = int(im.get("sizeBytes") or 0)
            for n in im.get("names") or []:
                out[normalized_image_name(n)] = size
        return out

    def _on_node(self, node: Obj) -> None:
        name = O.name(node)
        imgs = self._images_of(node)
        old = self._nodes.get(name)
        if old is not None and old[1] == imgs:
            self._nodes[name] = (node, imgs)
            return
        if old is not None:
            for n in old[1]:
                self._num_nodes[n] -= 1
        for n in imgs:
            self._num_nodes[n] = self._num_nodes.get(n, 0) + 1
        self._nodes[name] = (node, imgs)
        self._version += 1

    def _on_node_delete(self, node: Obj) -> None:
        old = self._nodes.pop(O.name(node), None)
        if old is not None:
            for n in old[1]:
                self._num_nodes[n] -= 1
            self._version += 1

    def _pod_images(self, pod: Obj) -> Tuple[str, ...]:
        return tuple(normalized_image_name(c.get("image") or "") for c in O.containers(pod) if c.get("image"))

    def pre_score(self, state, pod, nodes):
        imgs = self._pod_images(pod)
        if not imgs or not any(self._num_nodes.get(i) for i in imgs):
            return Status.skip()            # no node holds any of them: 0 everywhere
        state.write(self._KEY, imgs)
        return None

    def cache_signature(self, state, pod, phase):
        # node-local except the cluster-wide spread of each image: the version bumps when any
        # node's image list changes
        return self._pod_images(pod), self._version

    def score(self, state, pod, node_name):
        imgs = state.read(self._KEY) or self._pod_images(pod)
        ent = self._nodes.get(node_name)
        total = max(len(self._nodes), 1)
        s = 0
        if ent is not None:
            for i in imgs:
                size = ent[1].get(i)
                if size is not None:
                    s += int(size * (self._num_nodes.get(i, 0) / total))
        n_cont = max(len(O.containers(pod)), 1)
        hi = MAX_CONTAINER_THRESHOLD * n_cont
        s = min(max(s, MIN_THRESHOLD), hi)
        return MAX_NODE_SCORE * (s - MIN_THRESHOLD) // (hi - MIN_THRESHOLD), None


# ---------------------------------------------------------------------------- NodePreferAvoidPods
def _controller_ref(pod: Obj) -> Optional[Obj]:
    for ref in (pod.get("metadata") or {}).get("ownerReferences") or []:
        if ref.get("controller"):
            return ref
    return None


class NodePreferAvoidPods(PreScorePlugin, ScorePlugin):
    """0 on nodes whose preferAvoidPods annotation lists the pod's ReplicaSet /
    ReplicationController (by kind and uid), MaxNodeScore elsewhere (upstream weight 10000)."""
    NAME = "NodePreferAvoidPods"
    _KEY = "NodePreferAvoidPods/controller"

    def __init__(self, args=None, handle=None):
        self.handle = handle

    @staticmethod
    def _ref(pod: Obj) -> Optional[Tuple[str, str]]:
        ref = _controller_ref(pod)
        if ref is None or ref.get("kind") not in ("ReplicationController", "ReplicaSet"):
            return None
        return ref.get("kind"), ref.get("uid", "")

    def pre_score(self, state, pod, nodes):
        ref = self._ref(pod)
        if ref is None:
            return Status.skip()            # MaxNodeScore on every node
        state.write(self._KEY, ref)
        return None

    def cache_signature(self, state, pod, phase):
        return self._ref(pod)

    def score(self, state, pod, node_name):
        ref = state.read(self._KEY) or self._ref(pod)
        if ref is None:
            return MAX_NODE_SCORE, None
        ni = self.handle.snapshot().get(node_name)
        raw = O.annotations(ni.node if ni else {}).get(C.ANNOT_PREFER_AVOID_PODS)
        if not raw:
            return MAX_NODE_SCORE, None
        try:
            avoids = json.loads(raw).get("preferAvoidPods") or []
        except (ValueError, AttributeError):
            return MAX_NODE_SCORE, None
        for a in avoids:
            pc = ((a.get("podSignature") or {}).get("podController")) or {}
            if (pc.get("kind"), pc.get("uid", "")) == ref:
                return 0, None
        return MAX_NODE_SCORE, None
