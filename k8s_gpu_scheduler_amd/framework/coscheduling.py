"""Coscheduling (gang scheduling) for multi-pod GPU jobs.

A data- or tensor-parallel job spread over several pods (e.g. 2 pods x 8 MI355X, one RCCL
communicator across them) is useless until every rank runs, and a partial placement
holds GPUs that another job could use.  This is the scheduler-plugins `Coscheduling`
plugin on this framework's Permit/waiting-pod API (framework.scheduler.WaitingPod):

* pods of a group carry the label `scheduling.x-k8s.io/pod-group: <name>` (or the older
  `pod-group.scheduling.sigs.k8s.io/name`) and the group size in
  `pod-group.scheduling.sigs.k8s.io/min-available` (label or annotation; default: 1);
* PreFilter: a member is not even tried until `min-available` members exist;
* Permit: a member that is reserved while fewer than `min-available` members are
  reserved/bound waits (timeout `permitWaitingTimeSeconds`, default 60 s); the member
  that completes the quorum allows every waiting sibling, so the whole gang binds;
* PostFilter / Unreserve: when a member cannot be placed, or is unreserved, the waiting
  siblings are rejected so their GPUs are released at once (no partial gang holds).

The reference has no gang scheduling (its pods are single-device); it is
here because multi-GPU pods placed on xGMI cliques are exactly the jobs that span pods.
"""
from __future__ import annotations

import threading
from typing import Any, Dict, Optional, Set, Tuple

from ..api import objects as O
from .interface import PermitPlugin, PostFilterPlugin, PreFilterPlugin, ReservePlugin, Status

Obj = Dict[str, Any]

GROUP_LABELS = ("scheduling.x-k8s.io/pod-group", "pod-group.scheduling.sigs.k8s.io/name")
MIN_KEYS = ("pod-group.scheduling.sigs.k8s.io/min-available", "scheduling.x-k8s.io/min-available")


def pod_group(pod: Obj) -> Optional[Tuple[str, str]]:
    lab = O.labels(pod)
    for k in GROUP_LABELS:
        if lab.get(k):
            return O.namespace(pod), lab[k]
    return None


def min_available(pod: Obj) -> int:
    for src in (O.labels(pod), O.annotations(pod)):
        for k in MIN_KEYS:
            if src.get(k):
                try:
                    return max(1, int(src[k]))
                except ValueError:
                    pass
    return 1


class Coscheduling(PreFilterPlugin, PostFilterPlugin, ReservePlugin, PermitPlugin):
    NAME = "Coscheduling"

    def __init__(self, args: Optional[Dict[str, Any]] = None, handle: Any = None):
        args = args or {}
        self.handle = handle
        self.timeout_s = float(args.get("permitWaitingTimeSeconds", args.get("permit_timeout_s", 60.0)))
        self._lock = threading.Lock()
        self._members: Dict[Tuple[str, str], Set[str]] = {}     # group -> live member keys
        self._bound: Dict[Tuple[str, str], Set[str]] = {}       # group -> members with a node
        if handle is not None:
            try:
                inf = handle.informer_factory.pods()
                inf.add_event_handler(self._on_pod, lambda o, n: self._on_pod(n), self._on_delete)
            except AttributeError:
                pass

    # ---------------------------------------------------------------- membership
    def _on_pod(self, pod: Obj) -> None:
        g = pod_group(pod)
        if g is None:
            return
        k = O.key(pod)
        with self._lock:
            if O.is_terminal(pod):
                self._members.get(g, set()).discard(k)
                self._bound.get(g, set()).discard(k)
                return
            self._members.setdefault(g, set()).add(k)
            if O.node_name_of(pod):
                self._bound.setdefault(g, set()).add(k)

    def _on_delete(self, pod: Obj) -> None:
        g = pod_group(pod)
        if g is None:
            return
        with self._lock:
            self._members.get(g, set()).discard(O.key(pod))
            self._bound.get(g, set()).discard(O.key(pod))

    def _waiting_siblings(self, g: Tuple[str, str], me: str):
        return [wp for wp in self.handle.iterate_over_waiting_pods() if wp.key != me and pod_group(wp.pod) == g]

    # ---------------------------------------------------------------- extension points
    def pre_filter(self, state, pod):
        g = pod_group(pod)
        if g is None:
            return Status.skip()
        need = min_available(pod)
        with self._lock:
            have = len(self._members.get(g, set()) | {O.key(pod)})
        if have < need:
            return Status.unschedulable(f"pod group {g[1]}: {have} of {need} members exist", self.NAME)
        return None

    def post_filter(self, state, pod, filtered):
        g = pod_group(pod)
        if g is not None and self.handle is not None:
            for wp in self._waiting_siblings(g, O.key(pod)):
                self.handle.reject(wp.key, self.NAME, f"member {O.name(pod)} of pod group {g[1]} is unschedulable")
        return None, Status.unschedulable("pod group member unschedulable", self.NAME)

    def reserve(self, state, pod, node_name):
        return None

    def unreserve(self, state, pod, node_name):
        g = pod_group(pod)
        if g is None or self.handle is None:
            return
        for wp in self._waiting_siblings(g, O.key(pod)):
            self.handle.reject(wp.key, self.NAME, f"member {O.name(pod)} of pod group {g[1]} was unreserved")

    def permit(self, state, pod, node_name):
        g = pod_group(pod)
        if g is None or self.handle is None:
            return None, 0.0
        need = min_available(pod)
        me = O.key(pod)
        waiting = self._waiting_siblings(g, me)
        with self._lock:
            bound = set(self._bound.get(g, set()))
        ready = len(bound | {wp.key for wp in waiting} | {me})
        if ready < need:
            return Status.wait(), self.timeout_s
        for wp in waiting:                      # quorum reached: release the whole gang
            self.handle.allow(wp.key, self.NAME)
        return None, 0.0
