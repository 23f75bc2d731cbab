"""Per-node change log: which nodes may score or filter differently since a point in time.

Every source of node-local scheduling state appends the node's name when it changes:
the scheduler cache (a NodeInfo's pods / allocatable / node object), the GPU device ledger
(reservations, inventory), the telemetry cache (a new sample).  Changes that can affect
every node at once (node added or removed, a new prediction-table version) bump `epoch`.
The scheduling cycle's node-result cache (framework.fastpath) then re-evaluates only the
nodes touched since its last cycle -- O(changes) instead of O(nodes) Python work per pod.

kube-scheduler reaches the same end with its incremental snapshot
(pkg/scheduler/internal/cache: generation-ordered node list) plus per-plugin
PreFilter/PreScore state; the reference inherits that machinery unchanged
(reference cmd/scheduler/main.go:15-28).
"""
from __future__ import annotations

import threading
from typing import List, Optional, Set


class ChangeLog:
    def __init__(self, cap: int = 1 << 16):
        self._lock = threading.Lock()
        self._log: List[str] = []
        self._base = 0            # sequence number of _log[0]
        self.epoch = 0
        self.cap = cap

    @property
    def seq(self) -> int:
        """Sequence number the next touch gets (a cursor for `since`)."""
        return self._base + len(self._log)

    def touch(self, node: str) -> None:
        with self._lock:
            self._log.append(node)
            if len(self._log) > self.cap:
                drop = len(self._log) // 2
                del self._log[:drop]
                self._base += drop

    def touch_all(self) -> None:
        with self._lock:
            self.epoch += 1

    def since(self, seq: int) -> Optional[Set[str]]:
        """Nodes touched at or after cursor `seq`; None if that history was compacted away
        (the caller must treat every node as changed)."""
        with self._lock:
            if seq < self._base:
                return None
            return set(self._log[seq - self._base:])


class ChangeFanout:
    """The change logs a state source reports to (a ledger or telemetry cache may be shared
    by several scheduler profiles)."""

    def __init__(self) -> None:
        self.logs: List[ChangeLog] = []

    def attach(self, log: ChangeLog) -> None:
        if all(x is not log for x in self.logs):
            self.logs.append(log)

    def touch(self, node: str) -> None:
        for x in self.logs:
            x.touch(node)

    def touch_all(self) -> None:
        for x in self.logs:
            x.touch_all()
