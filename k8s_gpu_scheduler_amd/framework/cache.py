"""Scheduler cache: NodeInfo aggregation, assumed pods, snapshots.

Upstream kube-scheduler keeps this inside the binary the reference links
(reference cmd/scheduler/main.go:20-22); the reference plugin reads it only through
`handle.SnapshotSharedLister().NodeInfos().Get` (gpu_plugins.go:798).  Re-created here:
pods are accounted on their node as soon as they are *assumed* (after Reserve) so the
next cycle sees the capacity as taken, and are confirmed / expired by informer events.
"""
from __future__ import annotations

import threading
import time
from typing import Any, Dict, List, Optional

from ..api import objects as O
from .changes import ChangeFanout

Obj = Dict[str, Any]


class NodeInfo:
    __slots__ = ("node", "pods", "requested", "allocatable", "generation", "_name", "non_zero")

    def __init__(self, node: Optional[Obj] = None):
        self.node: Optional[Obj] = None
        self.pods: Dict[str, Obj] = {}
        self.requested: Dict[str, float] = {}
        self.allocatable: Dict[str, float] = {}
        self.generation = 0
        self._name = ""
        self.non_zero = [0, 0]      # milli-CPU, memory bytes with scoring defaults (O.pod_nonzero_requests)
        if node is not None:
            self.set_node(node)

    @property
    def name(self) -> str:
        return self._name

    def set_node(self, node: Obj) -> None:
        self.node = node
        self._name = O.name(node)
        self.allocatable = O.node_allocatable(node)
        self.generation += 1

    def add_pod(self, pod: Obj) -> None:
        k = O.key(pod)
        if k in self.pods:
            self.remove_pod(self.pods[k])
        self.pods[k] = pod
        for r, v in O.pod_requests(pod).items():
            self.requested[r] = self.requested.get(r, 0.0) + v
        self.requested["pods"] = self.requested.get("pods", 0.0) + 1
        nz = O.pod_nonzero_requests(pod)
        self.non_zero = [self.non_zero[0] + nz[0], self.non_zero[1] + nz[1]]
        self.generation += 1

    def remove_pod(self, pod: Obj) -> bool:
        k = O.key(pod)
        old = self.pods.pop(k, None)
        if old is None:
            return False
        for r, v in O.pod_requests(old).items():
            self.requested[r] = self.requested.get(r, 0.0) - v
        self.requested["pods"] = self.requested.get("pods", 0.0) - 1
        nz = O.pod_nonzero_requests(old)
        self.non_zero = [self.non_zero[0] - nz[0], self.non_zero[1] - nz[1]]
        self.generation += 1
        return True

    def free(self, resource: str) -> float:
        return self.allocatable.get(resource, 0.0) - self.requested.get(resource, 0.0)

    def clone(self) -> "NodeInfo":
        n = NodeInfo()
        n.node = self.node
        n._name = self._name
        n.pods = dict(self.pods)
        n.requested = dict(self.requested)
        n.allocatable = dict(self.allocatable)
        n.non_zero = list(self.non_zero)
        n.generation = self.generation
        return n


class Snapshot:
    """Immutable per-cycle view of all NodeInfos (ordered by name for determinism)."""

    def __init__(self, infos: Dict[str, NodeInfo], ordered: Optional[List[NodeInfo]] = None,
                 index: Optional[Dict[str, int]] = None):
        self._infos = infos
        self._list = ordered if ordered is not None else [infos[k] for k in sorted(infos)]
        self._index = index

    def index(self) -> Dict[str, int]:
        """node name -> position in list() (shared between snapshots of one node set)."""
        if self._index is None:
            self._index = {ni.name: i for i, ni in enumerate(self._list)}
        return self._index

    def get(self, node_name: str) -> Optional[NodeInfo]:
        return self._infos.get(node_name)

    def list(self) -> List[NodeInfo]:
        return self._list

    def __len__(self) -> int:
        return len(self._list)


class SchedulerCache:
    def __init__(self, assume_ttl_s: float = 30.0):
        self._lock = threading.RLock()
        self._nodes: Dict[str, NodeInfo] = {}
        self._pod_node: Dict[str, str] = {}
        self._assumed: Dict[str, float] = {}      # pod key -> deadline (0 while binding)
        self._snap_gen: Dict[str, int] = {}
        self._snap: Dict[str, NodeInfo] = {}
        self.assume_ttl_s = assume_ttl_s
        # incremental snapshots: nodes touched since the last one, and whether the set of
        # nodes changed (then the name-ordered list is rebuilt)
        self._dirty: set = set()
        self._members_changed = True
        self._last: Optional[Snapshot] = None
        self._index: Dict[str, int] = {}
        self.changes = ChangeFanout()       # framework.changes logs of the scheduling cycle

    def _touch(self, name: str) -> None:
        self._dirty.add(name)
        self.changes.touch(name)

    def _membership(self) -> None:
        self._members_changed = True
        self.changes.touch_all()

    # ---------------------------------------------------------------- nodes
    def add_node(self, node: Obj) -> None:
        with self._lock:
            name = O.name(node)
            ni = self._nodes.get(name)
            if ni is None:
                ni = NodeInfo(node)
                self._nodes[name] = ni
                self._membership()
            else:
                if ni.node is None:
                    self._membership()
                ni.set_node(node)
            self._touch(name)

    update_node = add_node

    def remove_node(self, node: Obj) -> None:
        with self._lock:
            self._nodes.pop(O.name(node), None)
            self._snap.pop(O.name(node), None)
            self._snap_gen.pop(O.name(node), None)
            self._membership()
            self._touch(O.name(node))

    # ---------------------------------------------------------------- pods
    def _place(self, pod: Obj, node_name: str) -> None:
        ni = self._nodes.get(node_name)
        if ni is None:
            ni = NodeInfo()
            ni._name = node_name
            self._nodes[node_name] = ni
        ni.add_pod(pod)
        self._pod_node[O.key(pod)] = node_name
        self._touch(node_name)

    def _unplace(self, pod: Obj) -> None:
        k = O.key(pod)
        nn = self._pod_node.pop(k, None)
        if nn and nn in self._nodes:
            self._nodes[nn].remove_pod(pod)
            self._touch(nn)

    def assume_pod(self, pod: Obj, node_name: str) -> None:
        with self._lock:
            k = O.key(pod)
            if k in self._pod_node:
                self._unplace(pod)
            p = dict(pod)        # path copy: watched objects are read-only (COW store)
            p["spec"] = dict(pod.get("spec") or {}, nodeName=node_name)
            self._place(p, node_name)
            self._assumed[k] = 0.0

    def finish_binding(self, pod: Obj) -> None:
        with self._lock:
            k = O.key(pod)
            if k in self._assumed:
                self._assumed[k] = time.monotonic() + self.assume_ttl_s

    def forget_pod(self, pod: Obj) -> None:
        with self._lock:
            k = O.key(pod)
            if k in self._assumed:
                self._assumed.pop(k, None)
                self._unplace(pod)

    def is_assumed(self, pod: Obj) -> bool:
        return O.key(pod) in self._assumed

    def add_pod(self, pod: Obj) -> None:
        """Informer add/update of an assigned pod: confirms an assumed pod."""
        nn = O.node_name_of(pod)
        if not nn:
            return
        with self._lock:
            k = O.key(pod)
            self._assumed.pop(k, None)
            if k in self._pod_node:
                self._unplace(pod)
            if O.is_terminal(pod):
                return
            self._place(pod, nn)

    update_pod = add_pod

    def remove_pod(self, pod: Obj) -> None:
        with self._lock:
            self._assumed.pop(O.key(pod), None)
            self._unplace(pod)

    def cleanup_expired(self) -> int:
        now = time.monotonic()
        n = 0
        with self._lock:
            for k, dl in list(self._assumed.items()):
                if dl and dl < now:
                    nn = self._pod_node.get(k)
                    if nn and nn in self._nodes:
                        pod = self._nodes[nn].pods.get(k)
                        if pod is not None:
                            self._unplace(pod)
                    self._assumed.pop(k, None)
                    n += 1
        return n

    # ---------------------------------------------------------------- snapshot
    def snapshot(self) -> Snapshot:
        """Incremental: only NodeInfos touched since the last snapshot are re-cloned (and only
        if their generation moved); an unchanged cluster returns the previous snapshot."""
        with self._lock:
            if self._last is not None and not self._dirty and not self._members_changed:
                return self._last
            infos = dict(self._snap)          # snapshots are immutable: copy on write
            if self._members_changed or self._last is None:
                for name, ni in self._nodes.items():
                    if ni.node is None:
                        continue
                    if self._snap_gen.get(name) != ni.generation or name not in infos:
                        infos[name] = ni.clone()
                        self._snap_gen[name] = ni.generation
                for name in list(infos):
                    if name not in self._nodes or self._nodes[name].node is None:
                        infos.pop(name, None)
                        self._snap_gen.pop(name, None)
                names = sorted(infos)
                self._index = {n: i for i, n in enumerate(names)}
                ordered = [infos[n] for n in names]
            else:
                ordered = list(self._last.list())
                for name in self._dirty:
                    ni = self._nodes.get(name)
                    i = self._index.get(name)
                    if ni is None or ni.node is None or i is None:
                        continue
                    if self._snap_gen.get(name) != ni.generation:
                        c = ni.clone()
                        infos[name] = c
                        ordered[i] = c
                        self._snap_gen[name] = ni.generation
            self._snap = infos
            self._dirty.clear()
            self._members_changed = False
            self._last = Snapshot(infos, ordered, self._index)
            return self._last

    def node_index(self) -> Dict[str, int]:
        """Position of every node in the last snapshot's name-ordered list."""
        with self._lock:
            return self._index

    def node_names(self) -> List[str]:
        with self._lock:
            return [n for n, ni in self._nodes.items() if ni.node is not None]

    def pod_count(self) -> int:
        with self._lock:
            return len(self._pod_node)
